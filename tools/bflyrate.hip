// bflyrate.hip -- SIMD cycles per 31-bit CT butterfly on gfx950, for the
// butterfly forms of the whole-plane kernel: the C++ ct_bfly of
// rnt_modarith.hpp and the 4-way interleaved inline asm of rnt_bfly4.hpp,
// at 4 waves per SIMD (one 1024-thread workgroup per CU, as k_plane_fused)
// and at 8 (two).  Each thread runs stages over 64 register words; every
// wave stamps s_memtime (shader clock) around its loop, and the report is
// the mean over waves of cycles x waves-per-SIMD / butterflies-per-wave.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I toy-heaan-ckks_amd/csrc \
//       tools/bflyrate.hip -o tools/bin/bflyrate && tools/bin/bflyrate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "rnt_bfly4.hpp"
#include "rnt_modarith.hpp"

using namespace rnt;

constexpr int ITERS = 64;

// MODE 0: C++ ct_bfly, 1: asm 4-way, 2: asm 4-way lazy
template <int MODE, int D>
__device__ __forceinline__ void stage_d(uint32_t (&x)[64], uint32_t w, uint32_t wp, const Mod<uint32_t>& mo) {
  if constexpr (MODE == 0) {
#pragma unroll
    for (int i = 0; i < 64; ++i)
      if (!(i & D)) ct_bfly(x[i], x[i | D], w, wp, mo);
  } else {
    int il[32];
    int n = 0;
#pragma unroll
    for (int i = 0; i < 64; ++i)
      if (!(i & D)) il[n++] = i;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const uint32_t ww[4] = {w, w, w, w}, wwp[4] = {wp, wp, wp, wp};
      uint64_t P[4];
      b4::shoup_prod4<true>(P, x[il[4 * g] | D], x[il[4 * g + 1] | D], x[il[4 * g + 2] | D], x[il[4 * g + 3] | D],
                            ww, wwp, mo.nq);
      uint32_t pl[4] = {(uint32_t)P[0], (uint32_t)P[1], (uint32_t)P[2], (uint32_t)P[3]};
      if constexpr (MODE == 1)
        b4::ct_reduce4(x[il[4 * g]], x[il[4 * g + 1]], x[il[4 * g + 2]], x[il[4 * g + 3]], x[il[4 * g] | D],
                       x[il[4 * g + 1] | D], x[il[4 * g + 2] | D], x[il[4 * g + 3] | D], pl, mo.q);
      else
        b4::ct_reduce4_lazy(x[il[4 * g]], x[il[4 * g + 1]], x[il[4 * g + 2]], x[il[4 * g + 3]],
                            x[il[4 * g] | D], x[il[4 * g + 1] | D], x[il[4 * g + 2] | D], x[il[4 * g + 3] | D], pl,
                            mo.q);
    }
  }
}

template <int MODE, int T>
__global__ void __launch_bounds__(T, 1) k_bfly(uint32_t* out, uint64_t* cyc, uint32_t q, uint32_t w, uint32_t wp) {
  uint32_t x[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) x[i] = (threadIdx.x * 2654435761u + i * 40503u) % q;
  const Mod<uint32_t> mo{q, 0u - q};
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
    stage_d<MODE, 32>(x, w, wp, mo);
    stage_d<MODE, 16>(x, w, wp, mo);
    stage_d<MODE, 8>(x, w, wp, mo);
    stage_d<MODE, 4>(x, w, wp, mo);
    stage_d<MODE, 2>(x, w, wp, mo);
    stage_d<MODE, 1>(x, w, wp, mo);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 64; ++i) acc ^= x[i];
  out[blockIdx.x * T + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * T + threadIdx.x) >> 6] = t1 - t0;
}

template <int MODE, int T>
static void run(const char* name, int blocks_per_cu) {
  const int cus = 256, blocks = cus * blocks_per_cu;
  uint32_t* out;
  uint64_t* cyc;
  const int waves = blocks * T / 64;
  hipMalloc(&out, (size_t)blocks * T * 4);
  hipMalloc(&cyc, (size_t)waves * 8);
  const uint32_t q = 2147352577u, w = 123456789u;
  const uint32_t wp = (uint32_t)(((uint64_t)w << 32) / q);
  hipLaunchKernelGGL((k_bfly<MODE, T>), dim3(blocks), dim3(T), 0, 0, out, cyc, q, w, wp);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k_bfly<MODE, T>), dim3(blocks), dim3(T), 0, 0, out, cyc, q, w, wp);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<uint64_t> c(waves);
  hipMemcpy(c.data(), cyc, waves * 8, hipMemcpyDeviceToHost);
  double mean = 0;
  for (auto v : c) mean += (double)v;
  mean /= waves;
  const int wps = T / 64 * blocks_per_cu / 4;  // waves per SIMD
  const double bfly_per_wave = 32.0 * 6 * ITERS;
  const double cyc_per_bfly = mean * wps / bfly_per_wave;
  const double bfly_total = bfly_per_wave * waves * 64;
  printf("%-22s waves/SIMD %d: %.1f SIMD cycles per butterfly (wave64), %.3f ms, %.3e butterflies/s\n", name, wps,
         cyc_per_bfly, ms, bfly_total / (ms * 1e-3));
  hipFree(out);
  hipFree(cyc);
}

int main() {
  run<0, 1024>("C++ ct_bfly", 1);
  run<1, 1024>("asm 4-way ct", 1);
  run<2, 1024>("asm 4-way ct lazy", 1);
  run<0, 512>("C++ ct_bfly", 1);
  run<1, 512>("asm 4-way ct", 1);
  run<0, 256>("C++ ct_bfly", 1);
  run<1, 256>("asm 4-way ct", 1);
  return 0;
}
