// oprate2.hip -- per-opcode VALU issue cost on gfx950, table-driven, with
// the shader clock measured inside each launch (s_memtime / s_memrealtime,
// MI355X_MICROARCH.md DVFS note) instead of assumed.  8 independent
// chains per lane, 8 waves per SIMD.  Prints cycles per wave-instruction.
#include <hip/hip_runtime.h>

#include <cstdio>

#define ITERS 1024

#define CH8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

// two-operand form: op dst, dst, y
#define OP2(NAME)                                                                             \
  __device__ __forceinline__ void body_##NAME(unsigned (&a)[8], unsigned y, unsigned z) {    \
    for (int it = 0; it < ITERS; ++it) {                                                      \
      asm volatile(#NAME " %0, %0, %8\n\t" #NAME " %1, %1, %8\n\t" #NAME " %2, %2, %8\n\t"    \
                   #NAME " %3, %3, %8\n\t" #NAME " %4, %4, %8\n\t" #NAME " %5, %5, %8\n\t"    \
                   #NAME " %6, %6, %8\n\t" #NAME " %7, %7, %8"                                \
                   : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),  \
                     "+v"(a[6]), "+v"(a[7])                                                   \
                   : "v"(y));                                                                 \
    }                                                                                         \
    (void)z;                                                                                  \
  }
#define OP3(NAME)                                                                             \
  __device__ __forceinline__ void body_##NAME(unsigned (&a)[8], unsigned y, unsigned z) {    \
    for (int it = 0; it < ITERS; ++it) {                                                      \
      asm volatile(#NAME " %0, %0, %8, %9\n\t" #NAME " %1, %1, %8, %9\n\t"                    \
                   #NAME " %2, %2, %8, %9\n\t" #NAME " %3, %3, %8, %9\n\t"                    \
                   #NAME " %4, %4, %8, %9\n\t" #NAME " %5, %5, %8, %9\n\t"                    \
                   #NAME " %6, %6, %8, %9\n\t" #NAME " %7, %7, %8, %9"                        \
                   : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),  \
                     "+v"(a[6]), "+v"(a[7])                                                   \
                   : "v"(y), "v"(z));                                                         \
    }                                                                                         \
  }
// raw string body (for modifiers / vcc forms); %0..%7 chains, %8 y, %9 z
#define OPS(NAME, S)                                                                          \
  __device__ __forceinline__ void body_##NAME(unsigned (&a)[8], unsigned y, unsigned z) {    \
    for (int it = 0; it < ITERS; ++it) {                                                      \
      asm volatile(S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)                                   \
                   : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),  \
                     "+v"(a[6]), "+v"(a[7])                                                   \
                   : "v"(y), "v"(z)                                                           \
                   : "vcc", "v40");                                                                \
    }                                                                                         \
  }

OP2(v_add_u32)
OP2(v_sub_u32)
OP2(v_min_u32)
OP2(v_max_u32)
OP2(v_min_i32)
OP2(v_mul_lo_u32)
OP2(v_mul_hi_u32)
OP2(v_mul_u32_u24)
OP2(v_xor_b32)
OP2(v_and_b32)
OP2(v_lshlrev_b32)
OP2(v_subrev_u32)
OP3(v_add3_u32)
OP3(v_med3_u32)
OP3(v_min3_u32)
OP3(v_sad_u32)
OP3(v_lshl_add_u32)
OP3(v_bfi_b32)
OP3(v_mad_u32_u24)
OP3(v_alignbit_b32)
OP3(v_perm_b32)
OP3(v_xad_u32)
OP3(v_add_lshl_u32)
#define S_SUBCLAMP(i) "v_sub_u32 %" #i ", %" #i ", %8 clamp\n\t"
OPS(sub_clamp, S_SUBCLAMP)
#define S_SUBCO32(i) "v_sub_co_u32_e32 %" #i ", vcc, %" #i ", %8\n\t"
OPS(v_sub_co_u32_e32, S_SUBCO32)
#define S_CND(i) "v_cndmask_b32_e32 %" #i ", %" #i ", %8, vcc\n\t"
OPS(v_cndmask_b32_e32, S_CND)
#define S_CMP(i) "v_cmp_gt_u32_e32 vcc, %" #i ", %8\n\t"
OPS(v_cmp_gt_u32_e32, S_CMP)
#define S_SUBB(i) "v_subb_co_u32_e32 %" #i ", vcc, %" #i ", %8, vcc\n\t"
OPS(v_subb_co_u32_e32, S_SUBB)
#define S_PKADD16(i) "v_pk_add_u16 %" #i ", %" #i ", %8\n\t"
OPS(v_pk_add_u16, S_PKADD16)
#define S_PKFMA(i) "v_pk_fma_f32 v[40:41], v[40:41], v[42:43], v[40:41]\n\t"
#define S_CSUB(i) "v_sub_u32 v40, %" #i ", %8\n\t v_min_u32 %" #i ", %" #i ", v40\n\t"
OPS(csub_sub_min, S_CSUB)
#define S_CSUBCND(i) "v_sub_co_u32_e32 v40, vcc, %" #i ", %8\n\t v_cndmask_b32_e32 %" #i ", v40, %" #i ", vcc\n\t"
OPS(csub_subco_cnd, S_CSUBCND)

// 64-bit chains
#define OP64(NAME, S)                                                                         \
  __device__ __forceinline__ void body_##NAME(unsigned (&a)[8], unsigned y, unsigned z) {    \
    unsigned long long b0 = a[0], b1 = a[1], b2 = a[2], b3 = a[3];                            \
    for (int it = 0; it < ITERS; ++it) {                                                      \
      asm volatile(S(0) S(1) S(2) S(3) S(0) S(1) S(2) S(3)                                   \
                   : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3)                                   \
                   : "v"(y), "v"(z)                                                           \
                   : "s0", "s1");                                                             \
    }                                                                                         \
    a[0] ^= (unsigned)b0; a[1] ^= (unsigned)(b1 >> 7); a[2] ^= (unsigned)b2;                  \
    a[3] ^= (unsigned)(b3 >> 3);                                                              \
  }
#define S_MAD64(i) "v_mad_u64_u32 %" #i ", s[0:1], %4, %5, %" #i "\n\t"
OP64(v_mad_u64_u32, S_MAD64)
#define S_LSHLADD64(i) "v_lshl_add_u64 %" #i ", %" #i ", 0, %" #i "\n\t"
OP64(v_lshl_add_u64, S_LSHLADD64)
#define S_FMA64(i) "v_fma_f64 %" #i ", %" #i ", %" #i ", %" #i "\n\t"
OP64(v_fma_f64, S_FMA64)
#define S_PKFMA32(i) "v_pk_fma_f32 %" #i ", %" #i ", %" #i ", %" #i "\n\t"
OP64(v_pk_fma_f32, S_PKFMA32)
#define S_PKADD32(i) "v_pk_add_f32 %" #i ", %" #i ", %" #i "\n\t"
OP64(v_pk_add_f32, S_PKADD32)
#define S_ADDCO(i) "v_add_co_u32_e64 %" #i ", s[0:1], %" #i ", %4\n\t"

struct Clk {
  unsigned long long t0, t1, r0, r1;
};

#define KERNEL(NAME)                                                                          \
  __global__ void __launch_bounds__(256) k_##NAME(unsigned* out, Clk* clk, unsigned seed) {   \
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime(); \
    unsigned a[8];                                                                            \
    for (int i = 0; i < 8; ++i) a[i] = (threadIdx.x + seed) * (2 * i + 3);                    \
    unsigned y = 2654435761u ^ seed, z = 12345u + seed;                                       \
    body_##NAME(a, y, z);                                                                     \
    unsigned s = 0;                                                                           \
    for (int i = 0; i < 8; ++i) s ^= a[i];                                                    \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                           \
    if (threadIdx.x == 0) {                                                                   \
      unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
      clk[blockIdx.x] = Clk{t0, t1, r0, r1};                                                  \
    }                                                                                         \
  }

#define LIST(X)                                                                               \
  X(v_add_u32) X(v_sub_u32) X(v_subrev_u32) X(v_min_u32) X(v_max_u32) X(v_min_i32)            \
  X(v_mul_lo_u32) X(v_mul_hi_u32) X(v_mul_u32_u24) X(v_xor_b32) X(v_and_b32) X(v_lshlrev_b32) \
  X(v_add3_u32) X(v_med3_u32) X(v_min3_u32) X(v_sad_u32) X(v_lshl_add_u32) X(v_bfi_b32)       \
  X(v_mad_u32_u24) X(v_alignbit_b32) X(v_perm_b32) X(v_xad_u32) X(v_add_lshl_u32)             \
  X(sub_clamp) X(v_sub_co_u32_e32) X(v_cndmask_b32_e32) X(v_cmp_gt_u32_e32)                   \
  X(v_subb_co_u32_e32) X(v_pk_add_u16) X(csub_sub_min) X(csub_subco_cnd)                      \
  X(v_mad_u64_u32) X(v_lshl_add_u64) X(v_fma_f64) X(v_pk_fma_f32) X(v_pk_add_f32)

LIST(KERNEL)

typedef void (*KFn)(unsigned*, Clk*, unsigned);

static void run(const char* name, KFn f, unsigned* d, Clk* c, Clk* hc, int blocks, double per_iter) {
  hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, c, 1u);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  const int R = 4;
  for (int r = 0; r < R; ++r) hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, c, (unsigned)r);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  ms /= R;
  (void)hipMemcpy(hc, c, blocks * sizeof(Clk), hipMemcpyDeviceToHost);
  // median-ish clock: average over blocks of dt/dr (realtime at 100 MHz)
  double ghz = 0;
  int n = 0;
  for (int i = 0; i < blocks; ++i) {
    double dr = (double)(hc[i].r1 - hc[i].r0);
    if (dr > 100) {
      ghz += (double)(hc[i].t1 - hc[i].t0) / dr * 0.1;
      ++n;
    }
  }
  ghz = n ? ghz / n : 2.4;
  const double waves = (double)blocks * 256 / 64;
  const double wave_instr = waves * ITERS * per_iter;
  const double cyc = ms * 1e-3 * ghz * 1e9 * 1024 / wave_instr;
  printf("%-22s %8.3f ms  clk %.2f GHz  %6.2f cycles/wave-instr/SIMD\n", name, ms, ghz, cyc);
}

int main() {
  const int blocks = 256 * 4 * 8;  // 8 waves per SIMD
  unsigned* d;
  Clk* c;
  (void)hipMalloc(&d, (size_t)blocks * 256 * sizeof(unsigned));
  (void)hipMalloc(&c, (size_t)blocks * sizeof(Clk));
  Clk* hc = new Clk[blocks];
#define RUN(NAME) run(#NAME, k_##NAME, d, c, hc, blocks, \
                      (sizeof(#NAME) > 5 && (__builtin_strncmp(#NAME, "csub", 4) == 0)) ? 16.0 : 8.0);
  LIST(RUN)
  (void)hipFree(d);
  (void)hipFree(c);
  return 0;
}
