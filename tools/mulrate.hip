// mulrate.hip -- measures gfx950 VALU throughput of the integer ops the
// modular butterflies are built from (informs DESIGN.md's compute roofline).
// Each kernel runs independent chains per lane so the numbers are
// throughput, not latency.  Build: hipcc --offload-arch=gfx950 -O3 mulrate.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define ITERS 4096
#define CHAINS 8

template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint32_t seed) {
  uint32_t x[CHAINS];
  uint32_t y = seed * 2654435761u + threadIdx.x;
  for (int c = 0; c < CHAINS; ++c) x[c] = y + c * 7919u;
  const uint32_t q = 2147352577u, wp = 123456789u, w = 987654321u;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      if (OP == 0) x[c] = x[c] * w + c;                 // v_mul_lo_u32 (+add)
      if (OP == 1) x[c] = __umulhi(x[c], wp) + c;       // v_mul_hi_u32 (+add)
      if (OP == 2) x[c] = x[c] + w;                     // v_add_u32 baseline
      if (OP == 3) {                                     // Shoup mul + csub
        uint32_t qh = __umulhi(x[c], wp);
        uint32_t r = x[c] * w - qh * q;
        uint32_t s = r - q;
        x[c] = s < r ? s : r;
      }
      if (OP == 4) {                                     // 64-bit product
        uint64_t t = (uint64_t)x[c] * w;
        x[c] = (uint32_t)t ^ (uint32_t)(t >> 32);
      }
      if (OP == 5) x[c] = __mul24(x[c], w) + c;         // v_mul_u32_u24
    }
  }
  uint32_t acc = 0;
  for (int c = 0; c < CHAINS; ++c) acc ^= x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int OP>
double run(uint32_t* d, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u);
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, (uint32_t)r);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double ops = 5.0 * blocks * 256.0 * ITERS * CHAINS;
  return ops / (ms * 1e-3) / 1e12;  // Tera lane-ops/s
}

int main() {
  const int blocks = 256 * 8 * 4;
  uint32_t* d;
  hipMalloc(&d, blocks * 256 * sizeof(uint32_t));
  const char* names[] = {"mul_lo(+add)", "mul_hi(+add)", "add", "shoup_mul+csub", "u64 product", "mul24(+add)"};
  double r[6];
  r[0] = run<0>(d, blocks);
  r[1] = run<1>(d, blocks);
  r[2] = run<2>(d, blocks);
  r[3] = run<3>(d, blocks);
  r[4] = run<4>(d, blocks);
  r[5] = run<5>(d, blocks);
  for (int i = 0; i < 6; ++i) printf("%-16s %8.2f T lane-ops/s\n", names[i], r[i]);
  hipFree(d);
  return 0;
}
