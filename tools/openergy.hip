// openergy.hip -- power draw of back-to-back i8 MFMAs and of 32/64-bit
// integer VALU ops on random operands (dev tool for the energy model,
// DESIGN.md §4).  Each mode runs for the given seconds; the driver
// (tools/gpu_openergy.sh) samples rocm-smi meanwhile.
//   openergy <mode> <seconds>   mode: mfma | mad64 | add32 | idle
// Prints ops/s (MFMA instructions or VALU wave-instructions per second).
// Build: hipcc --offload-arch=gfx950 -O3 tools/openergy.hip -o tools/bin/openergy
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <chrono>

typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int ITER = 4096;

__global__ void __launch_bounds__(256) k_mfma(int* out, uint32_t seed) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  uint32_t s = seed ^ (t * 2654435761u);
  v4i A[4], B[2];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      s = s * 1664525u + 1013904223u;
      A[i][j] = (int)s;
    }
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 4; ++j) {
      s = s * 1664525u + 1013904223u;
      B[i][j] = (int)s;
    }
  v4i c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int it = 0; it < ITER; ++it) {
    // every MFMA takes a different operand pair than the one before it
    c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0], B[0], c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[1], B[1], c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[2], B[0], c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[3], B[1], c3, 0, 0, 0);
    asm volatile("" : "+v"(A[0]), "+v"(A[1]), "+v"(A[2]), "+v"(A[3]), "+v"(B[0]), "+v"(B[1]));
  }
  const v4i r = c0 + c1 + c2 + c3;
  if (r[0] == 0x12345678 && r[1] == 7) out[t] = r[2];
}

__global__ void __launch_bounds__(256) k_mad64(int* out, uint32_t seed) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  int32_t a[8];
  int64_t x[8];
  uint32_t s = seed ^ (t * 2654435761u);
  for (int i = 0; i < 8; ++i) {
    s = s * 1664525u + 1013904223u;
    a[i] = (int32_t)s;
    x[i] = (int64_t)s << 13;
  }
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint64_t cc;
      asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(x[i]), "=s"(cc) : "v"(a[i]), "v"(a[(i + 3) & 7]));
    }
  }
  int64_t r = 0;
  for (int i = 0; i < 8; ++i) r ^= x[i];
  if (r == 0x12345678) out[t] = (int)r;
}

__global__ void __launch_bounds__(256) k_add32(int* out, uint32_t seed) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  uint32_t x[8], y[8];
  uint32_t s = seed ^ (t * 2654435761u);
  for (int i = 0; i < 8; ++i) {
    s = s * 1664525u + 1013904223u;
    x[i] = s;
    y[i] = s * 747796405u;
  }
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y[i]));
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(y[i]) : "v"(x[(i + 1) & 7]));
  }
  uint32_t r = 0;
  for (int i = 0; i < 8; ++i) r ^= x[i] ^ y[i];
  if (r == 0x12345678) out[t] = (int)r;
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const char* mode = argv[1];
  const double secs = atof(argv[2]);
  int* out;
  if (hipMalloc(&out, 4 << 20)) return 3;
  const int blocks = 256 * 8;  // 8 waves per CU (2 per SIMD)
  double ops_per_launch = 0;
  auto launch = [&](uint32_t seed) {
    if (!strcmp(mode, "mfma")) {
      hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(256), 0, 0, out, seed);
      ops_per_launch = (double)blocks * 4 * ITER * 4;  // MFMA wave-instructions
    } else if (!strcmp(mode, "mad64")) {
      hipLaunchKernelGGL(k_mad64, dim3(blocks), dim3(256), 0, 0, out, seed);
      ops_per_launch = (double)blocks * 4 * ITER * 8;
    } else if (!strcmp(mode, "add32")) {
      hipLaunchKernelGGL(k_add32, dim3(blocks), dim3(256), 0, 0, out, seed);
      ops_per_launch = (double)blocks * 4 * ITER * 16;
    }
  };
  if (!strcmp(mode, "idle")) {
    const auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < secs) {
    }
    printf("idle\n");
    return 0;
  }
  launch(1);
  (void)hipDeviceSynchronize();
  const auto t0 = std::chrono::steady_clock::now();
  long n = 0;
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < secs) {
    for (int i = 0; i < 8; ++i) launch((uint32_t)(++n));
    (void)hipDeviceSynchronize();
  }
  const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("%s: %.4e wave-instructions/s (%ld launches in %.2f s)\n", mode, ops_per_launch * n / el, n, el);
  return 0;
}
