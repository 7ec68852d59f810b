// rnt_plane.hip -- the whole-plane poly-mul (rnt_mul at N = 2^16, u32 bases).
//
// Reference unit: one coefficient-domain `a *= &b`
// (src/rings/backends/rns_ntt/poly.rs:307-329: to_ntt_domain of both
// operands, the pointwise mul_mod, to_coeff_domain), computed for a batch of
// (poly, limb) planes with the same merged negacyclic CT / GS network as the
// four-step kernels in rnt_kernels.hip, so the result is word-for-word the
// same (and the reference's).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "rnt_internal.hpp"
#include "rnt_modarith.hpp"
#include "rnt_device.hpp"
#include "rnt_bfly4.hpp"

namespace rnt {

// ---- whole-plane product (rnt_mul at N = 2^16, u32 canonical bases) ------
// 5 planes of HBM traffic per (poly, limb) instead of the four-step path's
// 9, in one launch, k_plane_fused: a workgroup transforms
// a, writes a^ to a scratch plane in a private layout, transforms b, reads a^
// back (pipelined 4 blocks ahead), forms the degree-3 block products and runs
// the inverse, storing c.  The butterflies run as 4-way interleaved inline
// asm (rnt_bfly4.hpp; the kernel is bound by VALU issue), pass C's twiddles
// are loaded ahead of X2, and X1 runs in its two rounds with pass B (gs B) of
// one register half between them.  (The standalone transforms at this size
// are rnt_mfma.hip's.)
// A workgroup = 1024 threads holds one 2^16-word plane, 64 words a thread.
// Thread t = (w << 6) | lam (wave w, lane lam); the 16-bit index i is split
// three ways:
//   L0  i = (r << 10) | (w << 6) | lam     registers: bits 15..10, coalesced
//   L1  i = (w << 12) | (r << 6) | lam     registers: bits 11..6
//   L2  i = (w << 12) | (lam << 6) | r     registers: bits 5..0
// and the network is the same merged negacyclic CT / GS heap as the
// four-step kernels (node = (2^16 + i) >> (b + 1) at bit b), so a^ and the
// product equal theirs word for word.  Pass A runs bits 15..10 in L0, pass
// B bits 9..6 in L1 (both with wave-uniform twiddle nodes: scalar loads),
// pass C bits 5..2 in L2 (bits 1..0 are the truncated stages).
//   X1 (L0 <-> L1) keeps the lanes and moves words between waves: 128 KiB
//      of LDS in two rounds, split on index bit 10 (a register bit on both
//      sides, so a round reads back exactly the registers it wrote).
//   X2 (L1 <-> L2) stays inside each wave: lane bits 5, 4 trade places with
//      register bits 5, 4 through v_permlane32_swap / v_permlane16_swap,
//      and the remaining 16 x 16 transposes go through a wave-private LDS
//      buffer in four rounds, with no workgroup barrier.
// The physical register of a logical one is a compile-time permutation
// (slot1, shared by L1 and L2).
namespace plane {
constexpr int T = 1024;
constexpr int XS = 17;                  // X2 buffer row stride (words): conflict-free both ways
constexpr int XW = 64 * XS;             // words of one X2 buffer (one per wave)
constexpr int X1_WORDS = 1 << 15;       // an X1 round; the X2 buffers share it
static_assert(16 * XW <= X1_WORDS, "X2 buffers inside the X1 region");
// The first HAT_LDS blocks of a^ (of 16 per thread) stay in the LDS beside
// the exchange region instead of going to the scratch plane and back.
constexpr int HAT_LDS = 2;
constexpr int LDS_WORDS = X1_WORDS + HAT_LDS * T * 4;
static_assert(LDS_WORDS * 4 <= 160 * 1024, "LDS of a CU");
__host__ __device__ constexpr int slot0(int r) { return r; }
__host__ __device__ constexpr int slot1(int r) { return 2 * (((r >> 5) << 4) | (r & 15)) + ((r >> 4) & 1); }
__host__ __device__ constexpr int slot2(int r) { return slot1(r); }
template <int L>
__host__ __device__ constexpr int slot(int r) {
  return L == 0 ? slot0(r) : slot1(r);
}
}  // namespace plane

// Tuning constants (each measured against its alternatives):
// twiddles per scalar-load chunk in pass A (64 SGPRs) and pass B, per
// per-lane chunk in pass C; a^ blocks in flight ahead of the block products.
constexpr int kPlaneChA = 32, kPlaneChB = 16, kPlaneChC = 8, kPlaneAhd = 4;

// Pass C's per-thread twiddles (stages at index bits 5..2: 1, 2, 4 and 8 of
// them), the stages in MASK (bit SL - 2) loaded ahead: before the X2
// exchange in the forward transforms, during the last block products in the
// inverse, so the loads are in flight while other work runs instead of
// stalling the stage that needs them.  Other stages fetch at the stage.
template <int MASK>
struct TwPre {
  const Tw<uint32_t>* b;
  Tw<uint32_t> s5[1], s4[2], s3[4], s2[8];
};
template <int MASK>
__device__ __forceinline__ TwPre<MASK> plane_pre(const Tw<uint32_t>* b, uint32_t node0) {
  TwPre<MASK> p;
  p.b = b;
  if constexpr (MASK & 8) p.s5[0] = tw_get<uint32_t>(b, node0 >> 6, 0u);
  if constexpr (MASK & 4) {
#pragma unroll
    for (int m = 0; m < 2; ++m) p.s4[m] = tw_get<uint32_t>(b, node0 >> 5, (uint32_t)m);
  }
  if constexpr (MASK & 2) {
#pragma unroll
    for (int m = 0; m < 4; ++m) p.s3[m] = tw_get<uint32_t>(b, node0 >> 4, (uint32_t)m);
  }
  if constexpr (MASK & 1) {
#pragma unroll
    for (int m = 0; m < 8; ++m) p.s2[m] = tw_get<uint32_t>(b, node0 >> 3, (uint32_t)m);
  }
  return p;
}
// Forward: the first three stages (5, 4, 3); inverse: none (preloading its
// first stage measured flat).
constexpr int kPreFwd = 0xE;
constexpr int kPreInv = 0;
// Twiddle m of a stage chunk at index bit SL (+ BB): from the source, or
// from the preloaded set.
template <int SL, class TS>
__device__ __forceinline__ Tw<uint32_t> tw_fetch(const TS& ts, uint32_t nb, uint32_t m) {
  return tw_get<uint32_t>(ts, nb, m);
}
template <int SL, int MASK>
__device__ __forceinline__ Tw<uint32_t> tw_fetch(const TwPre<MASK>& p, uint32_t nb, uint32_t m) {
  static_assert(SL >= 0 && SL <= 5, "pass C stages");
  if constexpr (SL < 2) return tw_get<uint32_t>(p.b, nb, m);  // the full transform's last two stages
  else if constexpr (!(MASK & (1 << (SL - 2)))) return tw_get<uint32_t>(p.b, nb, m);
  else if constexpr (SL == 5) return p.s5[0];
  else if constexpr (SL == 4) return p.s4[m];
  else if constexpr (SL == 3) return p.s3[m];
  else return p.s2[m];
}

template <class TS>
constexpr bool tw_uniform() {
  return std::is_same<TS, TwScalar<uint32_t>>::value;
}

// The n * 2^SL butterflies of a CT stage chunk in groups of four.  With
// SPLIT (a stage inside the pass) the butterflies whose upper half of e is
// set (i & (d >> 1)) are the lazy ones (both outputs only multiplied next);
// each class is grouped on its own.  Butterfly m of class CLS: twiddle j =
// m / HALF, e = CLS * HALF + m % HALF.
template <int LY, int SL, int M0, int HALF, bool LAZY, bool SW, int HM, int n>
__device__ __forceinline__ void plane_ct_groups(uint32_t (&x)[64], const Tw<uint32_t> (&t)[n], const Mod<uint32_t>& mo) {
  constexpr int d = 1 << SL, per = n * HALF, e0 = LAZY ? HALF : 0;
  // HM >= 0: only the butterflies of logical registers with bit 4 == HM
  // (one half of the L1 registers, which X1 delivers in two rounds)
  int jl[per], il[per];
  int cnt = 0;
#pragma unroll
  for (int m = 0; m < per; ++m) {
    const int j = m / HALF, i = ((M0 + j) << (SL + 1)) | (e0 + m % HALF);
    if (HM < 0 || ((i >> 4) & 1) == HM) {
      jl[cnt] = j;
      il[cnt] = i;
      ++cnt;
    }
  }
#pragma unroll
  for (int g = 0; g < per / 4; ++g) {
    if (4 * g + 3 >= cnt) break;
    const int* ii = il + 4 * g;
    const int* jj = jl + 4 * g;
    const uint32_t w[4] = {t[jj[0]].w, t[jj[1]].w, t[jj[2]].w, t[jj[3]].w};
    const uint32_t wp[4] = {t[jj[0]].p, t[jj[1]].p, t[jj[2]].p, t[jj[3]].p};
    uint64_t P[4];
    b4::shoup_prod4<SW>(P, x[plane::slot<LY>(ii[0] | d)], x[plane::slot<LY>(ii[1] | d)],
                        x[plane::slot<LY>(ii[2] | d)], x[plane::slot<LY>(ii[3] | d)], w, wp, mo.nq);
    uint32_t pl[4] = {(uint32_t)P[0], (uint32_t)P[1], (uint32_t)P[2], (uint32_t)P[3]};
    if constexpr (LAZY)
      b4::ct_reduce4_lazy(x[plane::slot<LY>(ii[0])], x[plane::slot<LY>(ii[1])], x[plane::slot<LY>(ii[2])],
                          x[plane::slot<LY>(ii[3])], x[plane::slot<LY>(ii[0] | d)], x[plane::slot<LY>(ii[1] | d)],
                          x[plane::slot<LY>(ii[2] | d)], x[plane::slot<LY>(ii[3] | d)], pl, mo.q);
    else
      b4::ct_reduce4(x[plane::slot<LY>(ii[0])], x[plane::slot<LY>(ii[1])], x[plane::slot<LY>(ii[2])],
                     x[plane::slot<LY>(ii[3])], x[plane::slot<LY>(ii[0] | d)], x[plane::slot<LY>(ii[1] | d)],
                     x[plane::slot<LY>(ii[2] | d)], x[plane::slot<LY>(ii[3] | d)], pl, mo.q);
  }
}

// GS butterflies of a stage chunk in groups of four: (u, v) <- (u + v,
// (u - v) w), every output canonical.
template <int LY, int SL, int M0, bool SW, int HM, int n>
__device__ __forceinline__ void plane_gs_groups(uint32_t (&x)[64], const Tw<uint32_t> (&t)[n], const Mod<uint32_t>& mo) {
  constexpr int d = 1 << SL, per = n * d;
  int jl[per], il[per];
  int cnt = 0;
#pragma unroll
  for (int m = 0; m < per; ++m) {
    const int j = m / d, i = ((M0 + j) << (SL + 1)) | (m % d);
    if (HM < 0 || ((i >> 4) & 1) == HM) {
      jl[cnt] = j;
      il[cnt] = i;
      ++cnt;
    }
  }
#pragma unroll
  for (int g = 0; g < per / 4; ++g) {
    if (4 * g + 3 >= cnt) break;
    const int* ii = il + 4 * g;
    const int* jj = jl + 4 * g;
    const uint32_t w[4] = {t[jj[0]].w, t[jj[1]].w, t[jj[2]].w, t[jj[3]].w};
    const uint32_t wp[4] = {t[jj[0]].p, t[jj[1]].p, t[jj[2]].p, t[jj[3]].p};
    uint32_t dd[4];
    b4::gs_pre4(x[plane::slot<LY>(ii[0])], x[plane::slot<LY>(ii[1])], x[plane::slot<LY>(ii[2])],
                x[plane::slot<LY>(ii[3])], x[plane::slot<LY>(ii[0] | d)], x[plane::slot<LY>(ii[1] | d)],
                x[plane::slot<LY>(ii[2] | d)], x[plane::slot<LY>(ii[3] | d)], dd, mo.q);
    uint64_t P[4];
    b4::shoup_prod4<SW>(P, dd[0], dd[1], dd[2], dd[3], w, wp, mo.nq);
    const uint32_t pl[4] = {(uint32_t)P[0], (uint32_t)P[1], (uint32_t)P[2], (uint32_t)P[3]};
    b4::csub4(x[plane::slot<LY>(ii[0] | d)], x[plane::slot<LY>(ii[1] | d)], x[plane::slot<LY>(ii[2] | d)],
              x[plane::slot<LY>(ii[3] | d)], pl, mo.q);
  }
}

// One chunk of a stage's twiddles.  In pass C (per-lane twiddles, LY = 2)
// the next chunk of a stage is loaded before the current chunk's
// butterflies run, so only a stage's first chunk waits for memory.
template <int n>
struct TwChunk {
  Tw<uint32_t> t[n];
};
template <int SLB, int M0, int n, class TS>
__device__ __forceinline__ TwChunk<n> plane_chunk(const TS& tw, uint32_t nb) {
  TwChunk<n> c;
#pragma unroll
  for (int j = 0; j < n; ++j)
    c.t[j] = tw_fetch<SLB>(tw, nb, (uint32_t)(M0 + j));
  return c;
}
template <int LY, int SL, int M0, int CH>
constexpr bool chunk_pipe() {
  return LY == 2 && M0 + CH < (32 >> SL);
}

// CT stages on logical register bits SLHI .. SLLO of layout LY (index bits
// [BB, BB + 6)); node0 = 2^16 + the thread's index with register bits 0.
// Twiddles in chunks of CH per stage (bounded registers beside the plane).
// As in pass_ct, outputs the next stage of the pass only multiplies stay
// in [0, 2q); the last stage leaves everything canonical.  Stages and
// chunks are template recursions, so every register index is a
// compile-time constant (a loop the unroller gave up on would put the
// plane in scratch memory).
template <int LY, int BB, int SL, int SLLO, int M0, int CH, int HM = -1, class TS, int NP = 1>
__device__ __forceinline__ void plane_ct_chunks(uint32_t (&x)[64], uint32_t nb, const TS& tw,
                                                const Mod<uint32_t>& mo, const TwChunk<NP>* pre = nullptr) {
  constexpr int d = 1 << SL, cnt = 32 >> SL, n = (cnt - M0) < CH ? (cnt - M0) : CH;
  Tw<uint32_t> t[n];
  if constexpr (NP == n && M0 > 0) {
#pragma unroll
    for (int j = 0; j < n; ++j) t[j] = pre->t[j];  // loaded during the previous chunk
  } else {
#pragma unroll
    for (int j = 0; j < n; ++j)
      t[j] = tw_fetch<BB + SL>(tw, nb, (uint32_t)(M0 + j));
  }
  constexpr bool SW = tw_uniform<TS>();
  constexpr int n2 = (cnt - M0 - CH) < CH ? (cnt - M0 - CH) : CH;
  TwChunk<(n2 > 0 ? n2 : 1)> nxt;
  if constexpr (chunk_pipe<LY, SL, M0, CH>()) nxt = plane_chunk<BB + SL, M0 + CH, (n2 > 0 ? n2 : 1)>(tw, nb);
  if constexpr (SL > SLLO) {
    plane_ct_groups<LY, SL, M0, d / 2, false, SW, HM>(x, t, mo);
    plane_ct_groups<LY, SL, M0, d / 2, true, SW, HM>(x, t, mo);
  } else {
    plane_ct_groups<LY, SL, M0, d, false, SW, HM>(x, t, mo);
  }
  if constexpr (M0 + CH < cnt) {
    if constexpr (chunk_pipe<LY, SL, M0, CH>())
      plane_ct_chunks<LY, BB, SL, SLLO, M0 + CH, CH, HM, TS, (n2 > 0 ? n2 : 1)>(x, nb, tw, mo, &nxt);
    else
      plane_ct_chunks<LY, BB, SL, SLLO, M0 + CH, CH, HM>(x, nb, tw, mo);
  }
}
template <int LY, int BB, int SL, int SLLO, int CH, int HM = -1, class TS>
__device__ __forceinline__ void plane_ct(uint32_t (&x)[64], uint32_t node0, const TS& tw,
                                         const Mod<uint32_t>& mo) {
  plane_ct_chunks<LY, BB, SL, SLLO, 0, CH, HM>(x, node0 >> (BB + SL + 1), tw, mo);
  if constexpr (SL > SLLO) plane_ct<LY, BB, SL - 1, SLLO, CH, HM>(x, node0, tw, mo);
}

// GS stages on logical register bits SLLO .. SLHI; FOLD: the stage at
// index bit 15 applies the folded constants (4/N with the Montgomery
// factor, LimbConst c1t/c2t) instead of its twiddle.
template <int LY, int BB, int SL, int M0, int CH, int HM = -1, class TS, int NP = 1>
__device__ __forceinline__ void plane_gs_chunks(uint32_t (&x)[64], uint32_t nb, const TS& itw,
                                                const Mod<uint32_t>& mo, const TwChunk<NP>* pre = nullptr) {
  constexpr int cnt = 32 >> SL, n = (cnt - M0) < CH ? (cnt - M0) : CH;
  Tw<uint32_t> t[n];
  if constexpr (NP == n && M0 > 0) {
#pragma unroll
    for (int j = 0; j < n; ++j) t[j] = pre->t[j];
  } else {
#pragma unroll
    for (int j = 0; j < n; ++j)
      t[j] = tw_fetch<BB + SL>(itw, nb, (uint32_t)(M0 + j));
  }
  constexpr int n2 = (cnt - M0 - CH) < CH ? (cnt - M0 - CH) : CH;
  TwChunk<(n2 > 0 ? n2 : 1)> nxt;
  if constexpr (chunk_pipe<LY, SL, M0, CH>()) nxt = plane_chunk<BB + SL, M0 + CH, (n2 > 0 ? n2 : 1)>(itw, nb);
  plane_gs_groups<LY, SL, M0, tw_uniform<TS>(), HM>(x, t, mo);
  if constexpr (M0 + CH < cnt) {
    if constexpr (chunk_pipe<LY, SL, M0, CH>())
      plane_gs_chunks<LY, BB, SL, M0 + CH, CH, HM, TS, (n2 > 0 ? n2 : 1)>(x, nb, itw, mo, &nxt);
    else
      plane_gs_chunks<LY, BB, SL, M0 + CH, CH, HM>(x, nb, itw, mo);
  }
}
template <int LY, int BB, int SL, int SLHI, int CH, bool FOLD, int HM = -1, class TS>
__device__ __forceinline__ void plane_gs(uint32_t (&x)[64], uint32_t node0, const TS& itw,
                                         const Mod<uint32_t>& mo, const Fold<uint32_t>& f) {
  constexpr int d = 1 << SL;
  if constexpr (FOLD && BB + SL + 1 == 16) {
#pragma unroll
    for (int e = 0; e < d; ++e) {  // the top stage: d = 32, one group
      const uint32_t u = x[plane::slot<LY>(e)], v = x[plane::slot<LY>(e | d)];
      x[plane::slot<LY>(e)] = shoup_mul(u + v, f.c1, f.c1p, mo);
      x[plane::slot<LY>(e | d)] = shoup_mul(u - v + mo.q, f.c2, f.c2p, mo);
    }
  } else {
    plane_gs_chunks<LY, BB, SL, 0, CH, HM>(x, node0 >> (BB + SL + 1), itw, mo);
  }
  if constexpr (SL < SLHI) plane_gs<LY, BB, SL + 1, SLHI, CH, FOLD, HM>(x, node0, itw, mo, f);
}

// X1, L0 <-> L1 through LDS, in two rounds: round h carries the words with
// index bit 10 == h: L0 registers 2k + h, L1 logical registers r1 =
// ((k >> 4) << 5) | (h << 4) | (k & 15), both in physical register 2k + h.
// LDS word = the 15 other index bits; every access is 64 consecutive words
// per wave.  (8-byte LDS words measured flat, profiles/r03/ab_plane_x1wide_preg.txt.)
// WRITE puts round H's registers into LDS, !WRITE takes them out; plane_fwd
// / plane_inv_tail run pass B (gs B) of the half already delivered (still to
// be sent) while the other round's LDS traffic drains.
template <bool TO_L1, int H, bool WRITE>
__device__ __forceinline__ void plane_x1_round(uint32_t (&x)[64], uint32_t* lds, uint32_t t) {
  const uint32_t w = t >> 6, lam = t & 63u;
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    const uint32_t j0 = ((uint32_t)k << 10) | t;
    const uint32_t j1 = ((((w << 1) | ((uint32_t)k >> 4))) << 10) | (((uint32_t)k & 15u) << 6) | lam;
    if constexpr (WRITE)
      lds[TO_L1 ? j0 : j1] = x[2 * k + H];
    else
      x[2 * k + H] = lds[TO_L1 ? j1 : j0];
  }
}
__device__ __forceinline__ void plane_sync() { __syncthreads(); }

// Progress priority (RNT_PLANE_PRIO) over the product's two long
// barrier-free stretches (a's pass C, the a^ store, b's load and pass A;
// then b's pass C, the block products, the inverse's gs C and X2): a wave
// lowers its priority 3 -> 0 as it advances through a stretch, so a wave
// that fell behind outranks those ahead of it and the sixteen reach the
// next barrier together instead of in age order (as k_mf_ntt's passes,
// profiles/r05/ab_mf_ntt_prio.txt).
#ifndef RNT_PLANE_PRIO
#define RNT_PLANE_PRIO 2
#endif
template <int P>
__device__ __forceinline__ void plane_prio() {
  if constexpr (RNT_PLANE_PRIO) __builtin_amdgcn_s_setprio(P);
}
// Level at each step point of the stretches, per RNT_PLANE_PRIO_VAR (A/B
// of where the steps fall): F4 after X1, F5 before pass C, F6 after it,
// H after the a^ store, A1 after b's pass A, P7 after the products (P8: at
// their middle), G8 after gs C, G9 after the inverse X2.
#ifndef RNT_PLANE_PRIO_VAR
#define RNT_PLANE_PRIO_VAR 2
#endif
enum PrioPt { F4, F5, F6, H, A1, P8, P7, G8, G9, B0, NPT };
template <int PT>
__device__ __forceinline__ void plane_prio_pt() {
  constexpr int tab[6][NPT] = {
      {3, -1, 2, 1, 0, -1, 1, -1, 0, -1},   // 0: the first steps (r05 run 1)
      {3, 2, 1, 0, 0, -1, 0, -1, 0, -1},    // 1: early
      {3, -1, -1, 2, 0, -1, 2, 1, 0, -1},   // 2: late (adopted)
      {3, -1, 2, 1, 0, 1, -1, 0, 0, -1},    // 3: the products split
      {3, -1, -1, 2, 0, -1, -1, 2, 1, 0},   // 4: later in b's stretch
      {3, -1, -1, -1, 1, -1, 2, 1, 0, -1},  // 5: later in a's stretch
  };
  constexpr int v = tab[RNT_PLANE_PRIO_VAR][PT];
  if constexpr (RNT_PLANE_PRIO && v >= 0) __builtin_amdgcn_s_setprio(v);
}
// RNT_PLANE_PRIO >= 2: also over the tail (gs A at 3, the stores at 0)
template <int P>
__device__ __forceinline__ void plane_prio_tail() {
  if constexpr (RNT_PLANE_PRIO >= 2) __builtin_amdgcn_s_setprio(P);
}

// Lane bit 5 <-> L1 register bit 5 and lane bit 4 <-> register bit 4
// (self-inverse; the two commute).
__device__ __forceinline__ void plane_swap54(uint32_t (&x)[64]) {
#pragma unroll
  for (int m = 0; m < 64; ++m) {
    if (m & 32) continue;
    const auto r = __builtin_amdgcn_permlane32_swap(x[plane::slot1(m)], x[plane::slot1(m | 32)], false, false);
    x[plane::slot1(m)] = r[0];
    x[plane::slot1(m | 32)] = r[1];
  }
#pragma unroll
  for (int m = 0; m < 64; ++m) {
    if (m & 16) continue;
    const auto r = __builtin_amdgcn_permlane16_swap(x[plane::slot1(m)], x[plane::slot1(m | 16)], false, false);
    x[plane::slot1(m)] = r[0];
    x[plane::slot1(m | 16)] = r[1];
  }
}

// X2, L1 <-> L2 inside each wave.  After plane_swap54 a lane holds index
// bits 11, 10 (lane bits 5, 4) and 3..0, a register m holds bits 5, 4
// (m >> 4) and 9..6 (m & 15); per group g = m >> 4 the 16 x 16 blocks of
// (m & 15) x (lane & 15) transpose through the wave's LDS buffer: word
// (lane, m & 15) at lane * 17 + (m & 15), read back by lane' as register
// (g << 4) | c from lane (lane' & 48) | c, column lane' & 15 (both
// directions 64 distinct banks).  LDS instructions of one wave execute in
// order, so the reads see the same wave's writes (and the next round's
// writes come after them): one buffer per wave.
template <bool TO_L2>
__device__ __forceinline__ void plane_x2(uint32_t (&x)[64], uint32_t* lds, uint32_t t) {
  const uint32_t w = t >> 6, lam = t & 63u;
  if constexpr (TO_L2) plane_swap54(x);
  const uint32_t a15 = lam * plane::XS;                          // + (m & 15)
  const uint32_t a2 = (lam & 48u) * plane::XS + (lam & 15u);     // + c * XS
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    uint32_t* buf = lds + w * plane::XW;
#pragma unroll
    for (int j = 0; j < 16; ++j) buf[TO_L2 ? a15 + j : a2 + j * plane::XS] = x[plane::slot1((g << 4) | j)];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int c = 0; c < 16; ++c) x[plane::slot1((g << 4) | c)] = buf[TO_L2 ? a2 + c * plane::XS : a15 + c];
    __builtin_amdgcn_wave_barrier();
  }
  if constexpr (!TO_L2) plane_swap54(x);
}

// Phase timeline of the plane kernels (measurement build only:
// tools/build_variant.sh trace -DRNT_PLANE_TRACE; tools/plane_trace.py).
// Lane 0 of every wave of the first 4096 workgroups waits for the wave's
// own memory operations and stamps the 100 MHz real-time counter at each
// phase boundary.
#ifdef RNT_PLANE_TRACE
constexpr int kTraceWg = 4096, kTraceStamps = 16;
__device__ uint64_t g_plane_trace[2 * kTraceWg * 16 * kTraceStamps];
#define PLANE_STAMP(K, S)                                                                       \
  do {                                                                                          \
    const uint32_t wg_ = trace_id;                                                              \
    if ((threadIdx.x & 63u) == 0 && wg_ < (uint32_t)kTraceWg) {                                 \
      __builtin_amdgcn_s_waitcnt(0);                                                            \
      g_plane_trace[(((K) * kTraceWg + wg_) * 16 + (threadIdx.x >> 6)) * kTraceStamps + (S)] =  \
          __builtin_amdgcn_s_memrealtime();                                                     \
    }                                                                                           \
  } while (0)
#else
#define PLANE_STAMP(K, S) \
  do {                    \
  } while (0)
#endif

// Register of the q-th plane load.
__host__ __device__ constexpr int plane_load_reg(int q) {
  return (((q >> 3) << 2) | (q & 3)) + ((q & 4) ? 32 : 0);
}

// Load the L0 plane at src (64 coalesced dword loads a thread).
__device__ __forceinline__ void plane_load(uint32_t (&x)[64], const uint32_t* src, uint32_t t) {
  const __amdgpu_buffer_rsrc_t g = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, (int)(4u << 16), 0x00020000);
  // in the order pass A's first stage consumes them (groups of four pairs
  // r, r + 32), so its butterflies start while the rest of the plane is
  // still arriving (loads return in order; each use waits only for its own)
#pragma unroll
  for (int q = 0; q < 64; ++q) {
    const int r = plane_load_reg(q);
    x[r] = __builtin_amdgcn_raw_buffer_load_b32(g, t * 4u, (uint32_t)r << 12, 0);
  }
}

// The truncated forward transform of the plane in x (L0 in, L2 out).
// SYNC1: other waves may still be using the LDS (their X2 buffers of an
// earlier transform) when X1 starts.
// a^ in the private layout through a buffer descriptor: block kk (4 words)
// of thread t at byte (kk * 1024 + t) * 16 -- a per-lane offset and a
// uniform one in the instruction, so no 64-bit addresses live in VGPRs.
struct HatBuf {
  __amdgpu_buffer_rsrc_t r;
  __device__ explicit HatBuf(const void* base)
      : r(__builtin_amdgcn_make_buffer_rsrc((void*)base, 0, 1 << 18, 0x00020000)) {}
  __device__ __forceinline__ void st(uint32_t t, int kk, uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) const {
    using V4 = decltype(__builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, 0));
    V4 v;
    v[0] = a0;
    v[1] = a1;
    v[2] = a2;
    v[3] = a3;
    __builtin_amdgcn_raw_buffer_store_b128(v, r, t * 16u, (uint32_t)kk << 14, 0);
  }
  __device__ __forceinline__ uint4 ld(uint32_t t, int kk) const {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, t * 16u, (uint32_t)kk << 14, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
};

struct NoHook {
  __device__ void operator()() const {}
};
// AFTER_X1 / AFTER_X2 run right after the exchanges (prefetches of the next
// operand: issued there, they are in flight during the passes that follow).
template <int K, bool SYNC1, class H1 = NoHook, class H2 = NoHook>
__device__ __forceinline__ void plane_fwd(uint32_t (&x)[64], uint32_t* lds, uint32_t t,
                                          const Tw<uint32_t>* tw, const Mod<uint32_t>& mo, uint32_t trace_id,
                                          const H1& after_x1 = H1{}, const H2& after_x2 = H2{}) {
  (void)trace_id;
  const uint32_t N = 1u << 16;
  const TwScalar<uint32_t> tws{(const RNT_CONST_AS Tw<uint32_t>*)tw};
  // pass A's twiddle nodes ((2^16 + i) >> (b + 1), b >= 10) depend on
  // register bits only, pass B's (b >= 6) on register and wave bits: both
  // wave-uniform (scalar loads)
  plane_ct<0, 10, 5, 0, kPlaneChA>(x, N, tws, mo);
  if constexpr (SYNC1) plane_prio_pt<A1>();  // b's pass A ends the first stretch
  PLANE_STAMP(K, 2);
  const uint32_t wu = __builtin_amdgcn_readfirstlane(t >> 6);
  // X1 in its two rounds, pass B of round 0's half while round 1 drains
  if constexpr (SYNC1) plane_sync();
  plane_x1_round<true, 0, true>(x, lds, t);
  plane_sync();
  plane_x1_round<true, 0, false>(x, lds, t);
  plane_sync();
  plane_x1_round<true, 1, true>(x, lds, t);
  PLANE_STAMP(K, 3);
  after_x1();
  plane_ct<1, 6, 3, 0, kPlaneChB, 0>(x, N + (wu << 12), tws, mo);
  plane_sync();
  plane_x1_round<true, 1, false>(x, lds, t);
  plane_ct<1, 6, 3, 0, kPlaneChB, 1>(x, N + (wu << 12), tws, mo);
  plane_sync();  // X2's buffers overlap the X1 region
  plane_prio_pt<F4>();
  PLANE_STAMP(K, 4);
  const auto pc = plane_pre<kPreFwd>(tw, N + (t << 6));
  plane_x2<true>(x, lds, t);
  PLANE_STAMP(K, 5);
  after_x2();
  plane_prio_pt<F5>();
  // pass C: bits 5..2 (bits 1..0 are the product's truncated stages)
  plane_ct<2, 0, 5, 2, kPlaneChC>(x, N + (t << 6), pc, mo);
  plane_prio_pt<F6>();
  PLANE_STAMP(K, 6);
}

// The inverse transform from pass C's layout (L2) to the store of c in L0:
// gs C on bits 2..5, X2, gs B, X1 (split as the forward one), gs A with the
// folded last-stage constants F (4/N with the Montgomery factor).
template <int K, class TSC>
__device__ __forceinline__ void plane_inv_tail(uint32_t (&x)[64], uint32_t* lds, uint32_t t, uint32_t* c,
                                               const Tw<uint32_t>* itw, const TSC& gsrc, const Mod<uint32_t>& mo,
                                               const Fold<uint32_t>& F, uint32_t trace_id) {
  (void)trace_id;
  const uint32_t n0 = 1u << 16;
  const TwScalar<uint32_t> itws{(const RNT_CONST_AS Tw<uint32_t>*)itw};
  plane_gs<2, 0, 2, 5, kPlaneChC, false>(x, n0 + (t << 6), gsrc, mo, Fold<uint32_t>{});
  plane_prio_pt<G8>();
  PLANE_STAMP(K, 8);
  plane_x2<false>(x, lds, t);
  plane_prio_pt<G9>();
  PLANE_STAMP(K, 9);
  const uint32_t wu = __builtin_amdgcn_readfirstlane(t >> 6);
  // gs B of round 0's half, X1 round 0 written while gs B of the other half runs
  plane_gs<1, 6, 0, 3, kPlaneChB, false, 0>(x, n0 + (wu << 12), itws, mo, Fold<uint32_t>{});
  plane_prio_pt<B0>();
  plane_sync();  // other waves may still be in their X2
  plane_x1_round<false, 0, true>(x, lds, t);
  plane_gs<1, 6, 0, 3, kPlaneChB, false, 1>(x, n0 + (wu << 12), itws, mo, Fold<uint32_t>{});
  PLANE_STAMP(K, 10);
  plane_sync();
  plane_x1_round<false, 0, false>(x, lds, t);
  plane_sync();
  plane_x1_round<false, 1, true>(x, lds, t);
  plane_sync();
  plane_x1_round<false, 1, false>(x, lds, t);
  plane_sync();
  PLANE_STAMP(K, 11);
  plane_prio_tail<3>();
  plane_gs<0, 10, 0, 5, kPlaneChA, true>(x, n0, itws, mo, F);
  plane_prio_tail<0>();
  PLANE_STAMP(K, 12);
  const __amdgpu_buffer_rsrc_t dst = __builtin_amdgcn_make_buffer_rsrc((void*)c, 0, (int)(4u << 16), 0x00020000);
#pragma unroll
  for (int r = 0; r < 64; ++r) __builtin_amdgcn_raw_buffer_store_b32(x[r], dst, t * 4u, (uint32_t)r << 12, 0);
  PLANE_STAMP(K, 13);
}

// The rest of the product once b^ is in x (L2): the degree-3 block
// products with a^ (ah: the private layout, block kk of thread t at
// ah[kk * 1024 + t]), the whole truncated inverse, c stored in L0.
// AH(kk) gives block kk of a^ (from memory, or a register prefetch).
template <int K, class AH>
__device__ __forceinline__ void plane_mul_tail(uint32_t (&x)[64], uint32_t* lds, uint32_t t, const AH& ah,
                                               uint32_t* c, const Tw<uint32_t>* tw, const Tw<uint32_t>* itw,
                                               const LimbConst<uint32_t>& lc, const Mod<uint32_t>& mo,
                                               uint32_t trace_id) {
  (void)trace_id;
  const uint32_t n0 = 1u << 16;
  // degree-3 block products: block (t << 4) | kk, zeta = (-1)^kk psi_rev[N/8 + (t << 3) + kk/2]
  const uint32_t zb = (n0 >> 3) + (t << 3);
  // a^ blocks and zeta twiddles are loaded AHD blocks ahead of their use
  // (pinned by scheduling barriers: left to itself hipcc issues each load
  // just before its product, so every block waits out a memory latency)
  constexpr int D = kPlaneAhd, Z = (D + 1) / 2 + 1;  // zeta j serves blocks 2j, 2j + 1
  uint4 abuf[D];
  Tw<uint32_t> zbuf[Z];
  TwPre<kPreInv> gpre;  // the inverse pass C's first stages, loaded during the last products
#pragma unroll
  for (int d = 0; d < D; ++d) abuf[d] = ah(d);
#pragma unroll
  for (int j = 0; j < Z; ++j) zbuf[j] = tw[zb + j];
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    const uint4 av = abuf[kk % D];
    const Tw<uint32_t> w = zbuf[(kk >> 1) % Z];
    if (kk + D < 16) abuf[kk % D] = ah(kk + D);
    if (kk == 16 - D) gpre = plane_pre<kPreInv>(itw, n0 + (t << 6));
    if ((kk & 1) && (kk >> 1) + Z < 8) zbuf[(kk >> 1) % Z] = tw[zb + (kk >> 1) + Z];
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t aa[4] = {av.x, av.y, av.z, av.w};
    const uint32_t bb[4] = {x[plane::slot2(4 * kk)], x[plane::slot2(4 * kk + 1)], x[plane::slot2(4 * kk + 2)],
                            x[plane::slot2(4 * kk + 3)]};
    if (kk == 8) plane_prio_pt<P8>();
    const uint32_t zeta = (kk & 1) ? lc.q - w.w : w.w;
    const uint32_t zeta_p = (kk & 1) ? ~w.p : w.p;
    uint32_t cc[4];
    mul_mod_x4(cc, aa, bb, zeta, zeta_p, lc.q, lc.qinv);
#pragma unroll
    for (int e = 0; e < 4; ++e) x[plane::slot2(4 * kk + e)] = cc[e];
  }
  plane_prio_pt<P7>();
  PLANE_STAMP(K, 7);
  plane_inv_tail<K>(x, lds, t, c, itw, gpre, mo, Fold<uint32_t>{lc.c1t, lc.c1t_p, lc.c2t, lc.c2t_p}, trace_id);
}

// a^ in the private layout: block kk (4 words) of thread t at (kk * 1024 + t) * 4
// of the scratch plane, the first HAT_LDS blocks at the same place in the
// LDS past the exchange region (each thread reads back only its own).
__device__ __forceinline__ uint4* hat_lds(uint32_t* lds) { return (uint4*)(lds + plane::X1_WORDS); }
__device__ __forceinline__ void plane_store_hat(const HatBuf& dst, const uint32_t (&x)[64], uint32_t t,
                                                uint32_t* lds) {
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    if (kk < plane::HAT_LDS)
      hat_lds(lds)[kk * plane::T + t] = make_uint4(x[plane::slot2(4 * kk)], x[plane::slot2(4 * kk + 1)],
                                                   x[plane::slot2(4 * kk + 2)], x[plane::slot2(4 * kk + 3)]);
    else
      dst.st(t, kk, x[plane::slot2(4 * kk)], x[plane::slot2(4 * kk + 1)], x[plane::slot2(4 * kk + 2)],
             x[plane::slot2(4 * kk + 3)]);
  }
}

// The product of one (poly, limb) plane pair: a -> a^ through the scratch
// plane ah, which the same threads read back ~40 us later (so the read is
// served by the Infinity Cache or L2 rather than HBM), then b -> b^, the
// block products and the inverse to c.  The store of a^ and the load of b
// are back to back and overlap.
__device__ __forceinline__ void plane_fused_one(uint32_t* __restrict__ c, const uint32_t* a, const uint32_t* b,
                                                uint32_t* ah, const TabPtrs<uint32_t>& tp, uint64_t ls, uint32_t poly,
                                                uint32_t l, uint32_t* lds, uint32_t t, uint32_t trace_id) {
  const uint64_t N = 1ull << 16;
  const uint64_t off = (uint64_t)l * ls + (uint64_t)poly * N;
  const LimbConst<uint32_t> lc = tp.lc[l];
  const Mod<uint32_t> mo = mod_of(lc);
  const Tw<uint32_t>* tw = tp.tw + (uint64_t)l * N;
  uint32_t x[64];
  PLANE_STAMP(0, 0);
  plane_load(x, a + off, t);
  PLANE_STAMP(0, 1);
  plane_fwd<0, false>(x, lds, t, tw, mo, trace_id);
  plane_store_hat(HatBuf(ah), x, t, lds);
  plane_prio_pt<H>();
  PLANE_STAMP(0, 7);
  PLANE_STAMP(1, 0);
  plane_load(x, b + off, t);
  PLANE_STAMP(1, 1);
  plane_fwd<1, true>(x, lds, t, tw, mo, trace_id);
  // a^ comes back from this thread's own stores above (the descriptor is
  // rebuilt from an opaque copy of the base, so nothing of the stores'
  // addressing stays live across b's transform)
  uint32_t* ah2 = ah;
  asm volatile("" : "+s"(ah2));
  const HatBuf hb(ah2);
  plane_mul_tail<1>(x, lds, t,
                    [hb, t, lds](int kk) { return kk < plane::HAT_LDS ? hat_lds(lds)[kk * plane::T + t] : hb.ld(t, kk); },
                    c + off, tw, tp.itw + (uint64_t)l * N, lc,
                    mo, trace_id);
}

// One workgroup per (poly, limb) plane pair, grid (B, L).  The a^ scratch
// plane of (poly, limb) is at limb stride sls, or (sls = 0) packed [L][B].
// (The form of this address is register allocation's business: the
// runtime choice keeps it apart from the operands' offsets, which measured
// 70 fewer SGPR spills than either form alone.)
__global__ void __launch_bounds__(plane::T, 1)
k_plane_fused(uint32_t* __restrict__ c, const uint32_t* a, const uint32_t* b, uint32_t* __restrict__ scratch,
              TabPtrs<uint32_t> tp, uint64_t ls, uint64_t sls) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const uint32_t poly = blockIdx.x, l = blockIdx.y;
  uint32_t* ah = scratch + (sls ? (uint64_t)l * sls + ((uint64_t)poly << 16) : (uint64_t)(poly + l * gridDim.x) << 16);
  plane_fused_one(c, a, b, ah, tp, ls, poly, l, (uint32_t*)smem_raw, threadIdx.x, poly + l * gridDim.x);
}

// The same product with the a^ scratch indexed by the CU the workgroup runs
// on instead of by its plane.  A workgroup takes the whole LDS (160 KiB), so
// a CU runs one at a time and no two resident workgroups share a slot; the
// slot's lines are rewritten by every plane the CU takes (256 slots in use,
// 64 MiB, instead of B L planes of scratch) and can stay in the Infinity
// Cache instead of being written back to HBM.  Slot = XCC_ID (4 bits) and
// HW_ID bits 15..8 (SE, SH, CU), kPlaneSlots in all; the caller's scratch
// holds at least that many planes (plane_scratch_planes).  sls is 0: the
// select keeps k_plane_fused's address form (its SGPR allocation).
// Same-box A/B at the metric: 140.1k against 138.6k poly-muls/s, every word
// of the 1024 x 16 output equal (profiles/r04/ab_plane_slots.txt).
static_assert(plane::LDS_WORDS * 4 > 80 * 1024, "one workgroup per CU");
__global__ void __launch_bounds__(plane::T, 1)
k_plane_fused_slots(uint32_t* __restrict__ c, const uint32_t* a, const uint32_t* b, uint32_t* __restrict__ scratch,
                    TabPtrs<uint32_t> tp, uint64_t ls, uint64_t sls) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const uint32_t poly = blockIdx.x, l = blockIdx.y;
  const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u;   // hwreg(HW_REG_XCC_ID)
  const uint32_t cu = (__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 8) & 0xffu;  // hwreg(HW_REG_HW_ID)[15:8]
  uint32_t* ah = scratch + (sls ? 0 : ((uint64_t)((xcc << 8) | cu) << 16));
  plane_fused_one(c, a, b, ah, tp, ls, poly, l, (uint32_t*)smem_raw, threadIdx.x, poly + l * gridDim.x);
}

#ifdef RNT_PLANE_TRACE
extern "C" __attribute__((visibility("default"))) int rnt_debug_plane_trace(uint64_t* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_plane_trace), sizeof(g_plane_trace));
}
#endif

// Planes of a^ scratch a launch over `planes` (poly, limb) pairs needs: one
// per pair, or one per CU slot from kPlaneSlots pairs on (512 MiB at most,
// against 4 GiB of per-pair scratch at the metric's 1024 x 16).
uint64_t plane_scratch_planes(uint64_t planes) { return planes < kPlaneSlots ? planes : kPlaneSlots; }

// The whole-plane product serves rnt_mul for u32 bases at N = 2^16 unless
// RNT_PLANE=0 (Tables::plane): its canonical arithmetic holds for any q <
// 2^31, so 30-bit bases too (131k against the lazy four-step kernels' 114k
// products/s).
bool plane_ok(const Tables* t) {
  return t->plane != 0 && !t->wide && t->log_n == 16;
}

hipError_t launch_plane_fused(const Launch& k, void* out, const void* a, const void* b, void* scratch, uint64_t ls) {
  if (k.B == 0 || k.L == 0) return hipSuccess;
  if (k.B > 0x7fffffffull || k.L > 65535) return hipErrorInvalidConfiguration;
  const size_t lds = (size_t)plane::LDS_WORDS * 4;
  if (k.B * k.L >= kPlaneSlots) {  // plane_scratch_planes: the scratch holds every slot
    hipError_t e = allow_lds(k_plane_fused_slots, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_plane_fused_slots, dim3((unsigned)k.B, (unsigned)k.L), dim3(plane::T), lds, k.s,
                       (uint32_t*)out, (const uint32_t*)a, (const uint32_t*)b, (uint32_t*)scratch,
                       tab_ptrs<uint32_t>(k.t), ls, (uint64_t)0);
    return hipGetLastError();
  }
  hipError_t e = allow_lds(k_plane_fused, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_plane_fused, dim3((unsigned)k.B, (unsigned)k.L), dim3(plane::T), lds, k.s, (uint32_t*)out,
                     (const uint32_t*)a, (const uint32_t*)b, (uint32_t*)scratch, tab_ptrs<uint32_t>(k.t), ls, ls);
  return hipGetLastError();
}

}  // namespace rnt
