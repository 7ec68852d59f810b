// rnt_plane.hip -- whole-plane kernels for N = 2^16, 31-bit primes (u32).
//
// Replaces, for the BASELINE metric shape, the three-launch column/row/
// column product of rnt_kernels.hip (same semantics: MulAssign on two
// coefficient-domain polys, poly.rs:307-329; transforms poly.rs:574-625).
//
// One workgroup of 1024 threads holds one (limb, poly) plane of 2^16 u32
// residues in VGPRs, 64 per thread (256 KiB: half of a CU's register file),
// and runs all 16 stages of the merged negacyclic CT network (and the 16 GS
// stages of the inverse) on it.  So a plane is read from HBM once and
// written once per launch; the three-launch path moves 9 planes per product,
// this one 5 (k_plane_fwd: b -> b^ in private order, k_plane_mul: a, b^ ->
// c).
//
// Index bits of a position j in [0, 2^16) and where they live (thread
// t in [0,1024), register i in [0,64)):
//   D1  j = t | i << 10                        registers = bits [10,16)
//   D2  j = (t & 31) | i << 5 | (t >> 5) << 11  registers = bits [5,11)
//   D3  j = i | t << 6                          registers = bits [0,6)
// Forward: load D1 (coalesced), stages 15..11 in D1, LDS exchange to D2,
// stages 10..5, exchange to D3, stages 4..0.  The inverse mirrors it.
// Consecutive distributions share one register bit (10, then 5), which
// splits each exchange into two rounds of half a plane (LDS is 160 KB, a
// plane 256 KiB): in round r every thread writes its outer registers with
// that bit = r and reads back its inner registers with that bit = r, so the
// registers it frees are the ones it refills (64 live values, no spill).
//
// LDS layout of a round: outer register slot s (the 5 other register bits)
// and outer thread t at s * 1025 + t.  Outer writes are 64 consecutive
// words per instruction; inner reads are base(t) + const(i) with lanes
// either consecutive (D2) or 1025 words apart (D3, 1025 = 1 mod 32 banks):
// conflict-free both ways.
//
// Twiddles are single words in Montgomery form (psi^{+-brv(g)} * 2^32 mod q,
// heap order g), so a lazy twiddle product is v_mad_u64_u32, v_mul_lo_u32,
// v_mad_u64_u32 -- the cost of a Shoup product at half the table bytes.  In
// D1 every twiddle a wave needs is wave-uniform (scalar loads).
#include <hip/hip_runtime.h>

#include "rnt_internal.hpp"
#include "rnt_modarith.hpp"

namespace rnt {

#if defined(__HIP_DEVICE_COMPILE__)
#define RNT_PL_CONST_AS __attribute__((address_space(4)))
#else
#define RNT_PL_CONST_AS
#endif

namespace {

constexpr int kPlLogN = 16;
constexpr uint32_t kPlN = 1u << kPlLogN;
constexpr int kPlE = 64;
constexpr int kPlT = 1024;
constexpr uint32_t kPlStride = 1025;
constexpr uint32_t kPlLdsWords = 32 * kPlStride;
// Timing experiments only (wrong results): bit 0 no data loads, bit 1 no
// vector twiddle loads, bit 2 no exchanges.
#ifndef RNT_PL_EXPT
#define RNT_PL_EXPT 0
#endif

struct PConst {
  uint32_t q, qneg;
};

// y * w * 2^-32 mod q, in [0, 2q), for any y < 2^32 and w < q:
// (y w + m q) / 2^32 < (2^32 q + 2^32 q) / 2^32.
// Plain C: hipcc emits v_mad_u64_u32, v_mul_lo_u32, v_mad_u64_u32 for it
// and, unlike rnt_modarith.hpp's keep64 forms, is free to interleave
// independent butterflies (a wave here has 32 per stage to overlap).
__device__ __forceinline__ uint32_t mmul_lazy(uint32_t y, uint32_t w, const PConst& c) {
  const uint64_t t = (uint64_t)y * w;
  const uint32_t m = (uint32_t)t * c.qneg;
  return (uint32_t)(((uint64_t)m * c.q + t) >> 32);
}
__device__ __forceinline__ uint32_t mmul(uint32_t y, uint32_t w, const PConst& c) {
  return csub<uint32_t>(mmul_lazy(y, w, c), c.q);
}

// Twiddle sources.  get<CNT>(w, k): the CNT twiddles of CT/GS stage on
// index bit k for this thread, m = 0..CNT-1 (node = base(k) + m).
struct TwUniform {  // D1: node = 2^(15-k) + m for every thread
  const RNT_PL_CONST_AS uint32_t* p;
  template <int CNT>
  __device__ __forceinline__ void get(uint32_t (&w)[CNT], int k) const {
#pragma unroll
    for (int m = 0; m < CNT; ++m) w[m] = p[(1u << (15 - k)) + m];
  }
};
struct TwVector {  // per-lane node base (D2, D3)
  const uint32_t* p;
  uint32_t hi;  // thread bits above the register field, see base()
  int sh;       // base(k) = 2^(15-k) + (hi << (sh - k))
  template <int CNT>
  __device__ __forceinline__ void get(uint32_t (&w)[CNT], int k) const {
    const uint32_t* b = p + (1u << (15 - k)) + (hi << (sh - k));
    if constexpr (RNT_PL_EXPT & 2) {
#pragma unroll
      for (int m = 0; m < CNT; ++m) w[m] = hi * 7 + m;
    } else if constexpr (CNT >= 4) {
#pragma unroll
      for (int g = 0; g < CNT / 4; ++g) {
        const uint4 v = *reinterpret_cast<const uint4*>(b + 4 * g);
        w[4 * g] = v.x;
        w[4 * g + 1] = v.y;
        w[4 * g + 2] = v.z;
        w[4 * g + 3] = v.w;
      }
    } else if constexpr (CNT == 2) {
      const uint2 v = *reinterpret_cast<const uint2*>(b);
      w[0] = v.x;
      w[1] = v.y;
    } else {
      w[0] = b[0];
    }
  }
};

// CT stage on register bit KB (index bit K = KB + RB).  MODE 0: all outputs
// reduced; 1: outputs that the next stage (bit KB-1) only multiplies stay
// in [0, 2q); 2: every output may stay in [0, 2q).  x inputs (bit KB clear)
// must be reduced.
template <int KB, int RB, int MODE, class TS>
__device__ __forceinline__ void ct_stage(uint32_t (&x)[kPlE], const TS& ts, const PConst& c) {
  constexpr int D = 1 << KB;
  constexpr int CNT = kPlE >> (KB + 1);
  uint32_t w[CNT];
  ts.template get<CNT>(w, KB + RB);
#pragma unroll
  for (int i = 0; i < kPlE; ++i) {
    if (i & D) continue;
    const int m = i >> (KB + 1);
    const bool lazy = MODE == 2 || (MODE == 1 && KB > 0 && (i & (D >> 1)));
    const uint32_t tt = mmul(x[i | D], w[m], c);
    const uint32_t u = x[i];
    if (lazy) {
      x[i] = u + tt;
      x[i | D] = u + (c.q - tt);
    } else {
      x[i] = add_mod<uint32_t>(u, tt, c.q);
      x[i | D] = sub_mod<uint32_t>(u, tt, c.q);
    }
  }
}

// GS stage on register bit KB: (u, v) -> (u + v, (u - v) w), all reduced.
template <int KB, int RB, class TS>
__device__ __forceinline__ void gs_stage(uint32_t (&x)[kPlE], const TS& ts, const PConst& c) {
  constexpr int D = 1 << KB;
  constexpr int CNT = kPlE >> (KB + 1);
  uint32_t w[CNT];
  ts.template get<CNT>(w, KB + RB);
#pragma unroll
  for (int i = 0; i < kPlE; ++i) {
    if (i & D) continue;
    const int m = i >> (KB + 1);
    const uint32_t u = x[i], v = x[i | D];
    x[i] = add_mod<uint32_t>(u, v, c.q);
    x[i | D] = mmul(u - v + c.q, w[m], c);
  }
}

// Last inverse stage (index bit 15 = D1 register bit 5) with the n^-1 (and
// Montgomery) factors folded: (u, v) -> ((u + v) f1, (u - v) f2).
__device__ __forceinline__ void gs_fold(uint32_t (&x)[kPlE], uint32_t f1, uint32_t f2,
                                        const PConst& c) {
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const uint32_t u = x[i], v = x[i + 32];
    x[i] = mmul(u + v, f1, c);
    x[i + 32] = mmul(u - v + c.q, f2, c);
  }
}

// ---- LDS exchanges (see the header comment) ------------------------------
// Inner-thread base and register offsets.  INNER = 2: D2 (outer D1),
// INNER = 3: D3 (outer D2).  Inner register i = 32 r + s lives in round r.
template <int INNER>
__device__ __forceinline__ uint32_t inner_base(uint32_t t) {
  return INNER == 2 ? (t >> 5) * kPlStride + (t & 31) : (t & 31) * kPlStride + ((t >> 5) << 5);
}
template <int INNER>
__device__ __forceinline__ constexpr uint32_t inner_off(int s) {
  return INNER == 2 ? (uint32_t)s << 5 : (uint32_t)s;
}

// outer -> inner (forward).  Outer register 2 s + r goes out in round r.
template <int INNER>
__device__ __forceinline__ void xchg_in(uint32_t (&x)[kPlE], uint32_t* lds, uint32_t t) {
  if constexpr (RNT_PL_EXPT & 4) return;
  const uint32_t rb = inner_base<INNER>(t);
  uint32_t y[kPlE];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
#pragma unroll
    for (int s = 0; s < 32; ++s) lds[(uint32_t)s * kPlStride + t] = x[2 * s + r];
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 32; ++s) y[32 * r + s] = lds[rb + inner_off<INNER>(s)];
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < kPlE; ++i) x[i] = y[i];
}

// inner -> outer (inverse).
template <int INNER>
__device__ __forceinline__ void xchg_out(uint32_t (&x)[kPlE], uint32_t* lds, uint32_t t) {
  if constexpr (RNT_PL_EXPT & 4) return;
  const uint32_t wb = inner_base<INNER>(t);
  uint32_t y[kPlE];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
#pragma unroll
    for (int s = 0; s < 32; ++s) lds[wb + inner_off<INNER>(s)] = x[32 * r + s];
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 32; ++s) y[2 * s + r] = lds[(uint32_t)s * kPlStride + t];
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < kPlE; ++i) x[i] = y[i];
}

// ---- transforms ------------------------------------------------------------
struct PlaneTw {
  TwUniform u;
  TwVector v2, v3;
};

__device__ __forceinline__ PlaneTw plane_tw(const uint32_t* tab, uint32_t t) {
  PlaneTw p;
  p.u.p = (const RNT_PL_CONST_AS uint32_t*)tab;
  p.v2.p = tab;  // D2: base(k) = 2^(15-k) + (t >> 5) << (10 - k)
  p.v2.hi = t >> 5;
  p.v2.sh = 10;
  p.v3.p = tab;  // D3: base(k) = 2^(15-k) + t << (5 - k)
  p.v3.hi = t;
  p.v3.sh = 5;
  return p;
}

// Forward: D1 in (reduced), D3 out.  LAST_LAZY: final stage outputs in
// [0, 2q) (they only feed the Montgomery pointwise product).
template <bool LAST_LAZY>
__device__ __forceinline__ void plane_fwd(uint32_t (&x)[kPlE], uint32_t* lds, uint32_t t,
                                          const PlaneTw& tw, const PConst& c) {
  ct_stage<5, 10, 1>(x, tw.u, c);
  ct_stage<4, 10, 1>(x, tw.u, c);
  ct_stage<3, 10, 1>(x, tw.u, c);
  ct_stage<2, 10, 1>(x, tw.u, c);
  ct_stage<1, 10, 0>(x, tw.u, c);
  xchg_in<2>(x, lds, t);
  ct_stage<5, 5, 1>(x, tw.v2, c);
  ct_stage<4, 5, 1>(x, tw.v2, c);
  ct_stage<3, 5, 1>(x, tw.v2, c);
  ct_stage<2, 5, 1>(x, tw.v2, c);
  ct_stage<1, 5, 1>(x, tw.v2, c);
  ct_stage<0, 5, 0>(x, tw.v2, c);
  xchg_in<3>(x, lds, t);
  ct_stage<4, 0, 1>(x, tw.v3, c);
  ct_stage<3, 0, 1>(x, tw.v3, c);
  ct_stage<2, 0, 1>(x, tw.v3, c);
  ct_stage<1, 0, 1>(x, tw.v3, c);
  ct_stage<0, 0, LAST_LAZY ? 2 : 0>(x, tw.v3, c);
}

// Inverse: D3 in (reduced), D1 out, last stage scaled by (f1, f2).
__device__ __forceinline__ void plane_inv(uint32_t (&x)[kPlE], uint32_t* lds, uint32_t t,
                                          const PlaneTw& tw, const PConst& c, uint32_t f1,
                                          uint32_t f2) {
  gs_stage<0, 0>(x, tw.v3, c);
  gs_stage<1, 0>(x, tw.v3, c);
  gs_stage<2, 0>(x, tw.v3, c);
  gs_stage<3, 0>(x, tw.v3, c);
  gs_stage<4, 0>(x, tw.v3, c);
  xchg_out<3>(x, lds, t);
  gs_stage<0, 5>(x, tw.v2, c);
  gs_stage<1, 5>(x, tw.v2, c);
  gs_stage<2, 5>(x, tw.v2, c);
  gs_stage<3, 5>(x, tw.v2, c);
  gs_stage<4, 5>(x, tw.v2, c);
  gs_stage<5, 5>(x, tw.v2, c);
  xchg_out<2>(x, lds, t);
  gs_stage<1, 10>(x, tw.u, c);
  gs_stage<2, 10>(x, tw.u, c);
  gs_stage<3, 10>(x, tw.u, c);
  gs_stage<4, 10>(x, tw.u, c);
  gs_fold(x, f1, f2, c);
}

struct PlaneArgs {
  const uint32_t* mtw;    // [Lroot][N] Montgomery forward twiddles
  const uint32_t* mitw;   // [Lroot][N] Montgomery inverse twiddles
  const LimbConst<uint32_t>* lc;
  uint32_t B;             // polys per limb in this launch
};

// b -> b^ (forward transform, private D3 order: word i * 1024 + t).
__global__ void __launch_bounds__(kPlT, 1)
k_plane_fwd(uint32_t* __restrict__ out, const uint32_t* __restrict__ in, PlaneArgs pa,
            uint64_t in_ls, uint64_t out_ls) {
  extern __shared__ uint32_t lds[];
  const uint32_t t = threadIdx.x;
  const uint32_t l = blockIdx.x / pa.B, p = blockIdx.x - l * pa.B;
  const LimbConst<uint32_t>& lc = pa.lc[l];
  const PConst c{lc.q, lc.qneg};
  const uint32_t* src = in + (uint64_t)l * in_ls + (uint64_t)p * kPlN + t;
  uint32_t x[kPlE];
#pragma unroll
  for (int i = 0; i < kPlE; ++i) x[i] = (RNT_PL_EXPT & 1) ? (t * 13 + i) % c.q : src[(uint32_t)i << 10];
  const PlaneTw tw = plane_tw(pa.mtw + (uint64_t)l * kPlN, t);
  plane_fwd<false>(x, lds, t, tw, c);
  uint32_t* dst = out + (uint64_t)l * out_ls + (uint64_t)p * kPlN + t;
#pragma unroll
  for (int i = 0; i < kPlE; ++i) dst[(uint32_t)i << 10] = x[i];
}

// c = INTT(NTT(a) (.) b^): a coefficient-domain, b^ from k_plane_fwd.
__global__ void __launch_bounds__(kPlT, 1)
k_plane_mul(uint32_t* __restrict__ out, const uint32_t* __restrict__ a,
            const uint32_t* __restrict__ bhat, PlaneArgs pa, uint64_t a_ls, uint64_t b_ls,
            uint64_t out_ls) {
  extern __shared__ uint32_t lds[];
  const uint32_t t = threadIdx.x;
  const uint32_t l = blockIdx.x / pa.B, p = blockIdx.x - l * pa.B;
  const LimbConst<uint32_t>& lc = pa.lc[l];
  const PConst c{lc.q, lc.qneg};
  const uint32_t* src = a + (uint64_t)l * a_ls + (uint64_t)p * kPlN + t;
  uint32_t x[kPlE];
#pragma unroll
  for (int i = 0; i < kPlE; ++i) x[i] = (RNT_PL_EXPT & 1) ? (t * 13 + i) % c.q : src[(uint32_t)i << 10];
  plane_fwd<true>(x, lds, t, plane_tw(pa.mtw + (uint64_t)l * kPlN, t), c);
  const uint32_t* bh = bhat + (uint64_t)l * b_ls + (uint64_t)p * kPlN + t;
  // in groups of 16 so the b^ loads do not all land in registers at once
#pragma unroll
  for (int g = 0; g < kPlE; g += 16) {
#pragma unroll
    for (int i = g; i < g + 16; ++i)
      x[i] = mmul(x[i], (RNT_PL_EXPT & 1) ? t + i : bh[(uint32_t)i << 10], c);
    __builtin_amdgcn_sched_barrier(0);
  }
  plane_inv(x, lds, t, plane_tw(pa.mitw + (uint64_t)l * kPlN, t), c, lc.mc1, lc.mc2);
  uint32_t* dst = out + (uint64_t)l * out_ls + (uint64_t)p * kPlN + t;
#pragma unroll
  for (int i = 0; i < kPlE; ++i) dst[(uint32_t)i << 10] = x[i];
}

}  // namespace

bool plane_supported(const Tables* t) { return !t->wide && t->log_n == kPlLogN && t->mtw_fwd; }

static hipError_t plane_lds(const void* f) {
  return hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)(kPlLdsWords * sizeof(uint32_t)));
}
static PlaneArgs plane_args(const Launch& k) {
  PlaneArgs pa;
  pa.mtw = (const uint32_t*)k.t->mtw_fwd;
  pa.mitw = (const uint32_t*)k.t->mtw_inv;
  pa.lc = (const LimbConst<uint32_t>*)k.t->lconst;
  pa.B = (uint32_t)k.B;
  return pa;
}

hipError_t launch_plane_fwd(const Launch& k, void* bhat, uint64_t bhat_ls, const void* b,
                            uint64_t b_ls) {
  const uint64_t planes = (uint64_t)k.L * k.B;
  if (planes == 0) return hipSuccess;
  if (planes > 0x7fffffffull) return hipErrorInvalidConfiguration;
  hipError_t e = plane_lds((const void*)k_plane_fwd);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_plane_fwd, dim3((unsigned)planes), dim3(kPlT),
                     kPlLdsWords * sizeof(uint32_t), k.s, (uint32_t*)bhat, (const uint32_t*)b,
                     plane_args(k), b_ls, bhat_ls);
  return hipGetLastError();
}

hipError_t launch_plane_mul(const Launch& k, void* out, uint64_t out_ls, const void* a,
                            uint64_t a_ls, const void* bhat, uint64_t bhat_ls) {
  const uint64_t planes = (uint64_t)k.L * k.B;
  if (planes == 0) return hipSuccess;
  if (planes > 0x7fffffffull) return hipErrorInvalidConfiguration;
  hipError_t e = plane_lds((const void*)k_plane_mul);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_plane_mul, dim3((unsigned)planes), dim3(kPlT),
                     kPlLdsWords * sizeof(uint32_t), k.s, (uint32_t*)out, (const uint32_t*)a,
                     (const uint32_t*)bhat, plane_args(k), a_ls, bhat_ls, out_ls);
  return hipGetLastError();
}

}  // namespace rnt
