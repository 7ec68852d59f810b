// oprate.hip -- per-opcode VALU throughput on gfx950 via inline asm (the
// compiler cannot fold or strength-reduce the chains).  8 independent
// chains per lane, full occupancy; reports cycles per wave-instruction per
// SIMD assuming `clock_ghz` (pass it as argv[1], default 2.4).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define ITERS 2048

#define BODY(OPSTR)                                                                    \
  for (int it = 0; it < ITERS; ++it) {                                                 \
    asm volatile(OPSTR " %0, %0, %8\n\t" OPSTR " %1, %1, %8\n\t" OPSTR " %2, %2, %8\n\t" \
                 OPSTR " %3, %3, %8\n\t" OPSTR " %4, %4, %8\n\t" OPSTR " %5, %5, %8\n\t" \
                 OPSTR " %6, %6, %8\n\t" OPSTR " %7, %7, %8"                           \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), \
                   "+v"(a7)                                                            \
                 : "v"(y));                                                            \
  }

#define BODYVCC(OPSTR)                                                                    \
  for (int it = 0; it < ITERS; ++it) {                                                   \
    asm volatile(OPSTR " %0, vcc, %0, %8\n\t" OPSTR " %1, vcc, %1, %8\n\t"             \
                 OPSTR " %2, vcc, %2, %8\n\t" OPSTR " %3, vcc, %3, %8\n\t"             \
                 OPSTR " %4, vcc, %4, %8\n\t" OPSTR " %5, vcc, %5, %8\n\t"             \
                 OPSTR " %6, vcc, %6, %8\n\t" OPSTR " %7, vcc, %7, %8"                  \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),  \
                   "+v"(a7)                                                              \
                 : "v"(y) : "vcc");                                                      \
  }

#define BODYMAD()                                                                          \
  for (int it = 0; it < ITERS; ++it) {                                                     \
    asm volatile("v_mad_u64_u32 %0, s[0:1], %4, %5, %0\n\t"                              \
                 "v_mad_u64_u32 %1, s[0:1], %4, %5, %1\n\t"                              \
                 "v_mad_u64_u32 %2, s[0:1], %4, %5, %2\n\t"                              \
                 "v_mad_u64_u32 %3, s[0:1], %4, %5, %3"                                   \
                 : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3)                                \
                 : "v"(y), "v"(z) : "s0", "s1");                                           \
  }

#define BODYCND()                                                                          \
  for (int it = 0; it < ITERS; ++it) {                                                     \
    asm volatile("v_cndmask_b32_e32 %0, %0, %8, vcc\n\t v_cndmask_b32_e32 %1, %1, %8, vcc\n\t" \
                 "v_cndmask_b32_e32 %2, %2, %8, vcc\n\t v_cndmask_b32_e32 %3, %3, %8, vcc\n\t" \
                 "v_cndmask_b32_e32 %4, %4, %8, vcc\n\t v_cndmask_b32_e32 %5, %5, %8, vcc\n\t" \
                 "v_cndmask_b32_e32 %6, %6, %8, vcc\n\t v_cndmask_b32_e32 %7, %7, %8, vcc"     \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),    \
                   "+v"(a7)                                                                 \
                 : "v"(y) : "vcc");                                                         \
  }

#define BODY3(OPSTR)                                                                        \
  for (int it = 0; it < ITERS; ++it) {                                                      \
    asm volatile(OPSTR " %0, %0, %8, %9\n\t" OPSTR " %1, %1, %8, %9\n\t" OPSTR " %2, %2, %8, %9\n\t" \
                 OPSTR " %3, %3, %8, %9\n\t" OPSTR " %4, %4, %8, %9\n\t" OPSTR " %5, %5, %8, %9\n\t" \
                 OPSTR " %6, %6, %8, %9\n\t" OPSTR " %7, %7, %8, %9"                        \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),     \
                   "+v"(a7)                                                                 \
                 : "v"(y), "v"(z));                                                         \
  }

template <int OP>
__global__ void __launch_bounds__(256) k(unsigned* out, unsigned seed) {
  unsigned a0 = threadIdx.x + seed, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11,
           a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;
  unsigned y = 2654435761u ^ seed, z = 12345u;
  if (OP == 0) BODY("v_add_u32")
  if (OP == 1) BODY("v_min_u32")
  if (OP == 2) BODY("v_mul_lo_u32")
  if (OP == 3) BODY("v_mul_hi_u32")
  if (OP == 4) BODY("v_mul_u32_u24")
  if (OP == 5) BODY3("v_lshl_add_u32")
  if (OP == 6) BODY3("v_add3_u32")
  if (OP == 7) BODY("v_sub_u32")
  if (OP == 8) BODY("v_mul_hi_u32_u24")
  if (OP == 9) BODY("v_xor_b32")
  if (OP == 10) BODYCND()
  if (OP == 16) BODYVCC("v_sub_co_u32")
  if (OP == 17) BODYVCC("v_add_co_u32")
  if (OP == 18) {
    unsigned long long b0 = a0, b1 = a1, b2 = a2, b3 = a3;
    BODYMAD()
    a0 ^= (unsigned)b0; a1 ^= (unsigned)(b1 >> 7); a2 ^= (unsigned)b2; a3 ^= (unsigned)(b3 >> 3);
  }
  if (OP == 11) BODY("v_max_u32")
  if (OP == 12) BODY("v_and_b32")
  if (OP == 13) BODY("v_ashrrev_i32")
  if (OP == 14) BODY("v_min_i32")
  if (OP == 15) BODY("v_lshlrev_b32")
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int OP>
float run(unsigned* d, int blocks) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u);
  (void)hipEventRecord(a);
  for (int r = 0; r < 4; ++r) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, (unsigned)r);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 4;
}

int main(int argc, char** argv) {
  const double ghz = argc > 1 ? atof(argv[1]) : 2.4;
  const int blocks = 256 * 8 * 4;  // 8 waves per SIMD-ish, 4 rounds
  unsigned* d;
  (void)hipMalloc(&d, (size_t)blocks * 256 * sizeof(unsigned));
  const char* names[] = {"v_add_u32", "v_min_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mul_u32_u24",
                         "v_lshl_add_u32", "v_add3_u32", "v_sub_u32", "v_mul_hi_u32_u24", "v_xor_b32",
                         "v_cndmask_b32_e32", "v_max_u32", "v_and_b32", "v_ashrrev_i32", "v_min_i32",
                         "v_lshlrev_b32", "v_sub_co_u32", "v_add_co_u32", "v_mad_u64_u32(x4/iter)"};
  const int NOPS = 19;
  float ms[19];
  ms[0] = run<0>(d, blocks);
  ms[1] = run<1>(d, blocks);
  ms[2] = run<2>(d, blocks);
  ms[3] = run<3>(d, blocks);
  ms[4] = run<4>(d, blocks);
  ms[5] = run<5>(d, blocks);
  ms[6] = run<6>(d, blocks);
  ms[7] = run<7>(d, blocks);
  ms[8] = run<8>(d, blocks);
  ms[9] = run<9>(d, blocks);
  ms[10] = run<10>(d, blocks);
  ms[11] = run<11>(d, blocks);
  ms[12] = run<12>(d, blocks);
  ms[13] = run<13>(d, blocks);
  ms[14] = run<14>(d, blocks);
  ms[15] = run<15>(d, blocks);
  ms[16] = run<16>(d, blocks);
  ms[17] = run<17>(d, blocks);
  ms[18] = run<18>(d, blocks);
  const double waves = (double)blocks * 256 / 64;
  const double wave_instr = waves * ITERS * 8;
  const double simds = 256 * 4;
  for (int i = 0; i < NOPS; ++i) {
    const double per = i == 18 ? 0.5 : 1.0;  // 4 instrs per iteration instead of 8
    const double cyc = ms[i] * 1e-3 * ghz * 1e9 * simds / (wave_instr * per);
    printf("%-18s %8.3f ms  %6.2f cycles/wave-instr/SIMD @%.1fGHz\n", names[i], ms[i], cyc, ghz);
  }
  (void)hipFree(d);
  return 0;
}
