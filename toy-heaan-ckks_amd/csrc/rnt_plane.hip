// rnt_plane.hip -- the whole-plane poly-mul (rnt_mul at N = 2^16, u32 bases).
//
// Reference unit: one coefficient-domain `a *= &b`
// (src/rings/backends/rns_ntt/poly.rs:307-329: to_ntt_domain of both
// operands, the pointwise mul_mod, to_coeff_domain), computed for a batch of
// (poly, limb) planes with the same merged negacyclic CT / GS network as the
// four-step kernels in rnt_kernels.hip, so the result is word-for-word the
// same (and the reference's).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "rnt_internal.hpp"
#include "rnt_modarith.hpp"
#include "rnt_device.hpp"
#include "rnt_bfly4.hpp"

namespace rnt {

// ---- whole-plane product (rnt_mul at N = 2^16, u32 canonical bases) ------
// 5 planes of HBM traffic per (poly, limb) instead of the four-step path's
// 9.  The shipped form is one launch, k_plane_fused: a
// workgroup transforms a, writes a^ to a scratch plane in a private layout,
// transforms b, reads a^ back (pipelined 4 blocks ahead), forms the degree-3
// block products and runs the inverse, storing c.  k_plane_fwd + k_plane_mul
// split the same work over two launches (RNT_PLANE=1), k_plane_fused_p is the
// persistent form (RNT_PLANE=4).  The butterflies run as 4-way interleaved
// inline asm (rnt_bfly4.hpp; the kernel is bound by VALU issue), pass C's
// twiddles are loaded ahead of X2, and X1 runs in its two rounds with pass B
// (gs B) of one register half between them.
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
#ifndef RNT_PLANE_EXP
#define RNT_PLANE_EXP 0
#endif
namespace plane {
constexpr int T = 1024;
constexpr int XS = 17;                  // X2 buffer row stride (words): conflict-free both ways
constexpr int XW = 64 * XS;             // words of one X2 buffer
constexpr int LDS_WORDS = 16 * 2 * XW;  // two X2 buffers per wave; >= 2^15 (an X1 round)
static_assert(LDS_WORDS >= (1 << 15), "X1 round");
__host__ __device__ constexpr int slot0(int r) { return r; }
__host__ __device__ constexpr int slot1(int r) { return 2 * (((r >> 5) << 4) | (r & 15)) + ((r >> 4) & 1); }
__host__ __device__ constexpr int slot2(int r) { return slot1(r); }
template <int L>
__host__ __device__ constexpr int slot(int r) {
  return L == 0 ? slot0(r) : slot1(r);
}
}  // namespace plane

// Butterflies as interleaved groups of four in inline asm (rnt_bfly4.hpp):
// 1 (default) or 0 (the C++ butterflies of rnt_modarith.hpp, A/B).
#ifndef RNT_PLANE_ASM
#define RNT_PLANE_ASM 1
#endif
// Cache policy (buffer aux bits) of the streamed operand loads and the
// product store: 0 default, 2 non-temporal (A/B knob, -DRNT_PLANE_AUX=2).
#ifndef RNT_PLANE_AUX
#define RNT_PLANE_AUX 0
#endif
constexpr int kPlaneAux = RNT_PLANE_AUX;
// plane loads in pass A's first-stage order (1) or register order (0)
#ifndef RNT_PLANE_LOAD_ORDER
#define RNT_PLANE_LOAD_ORDER 1
#endif
constexpr bool kPlaneLoadOrder = RNT_PLANE_LOAD_ORDER != 0;
// b's loads issued ahead of a^'s stores (0: none)
#ifndef RNT_PLANE_BEARLY
#define RNT_PLANE_BEARLY 0
#endif
constexpr int kPlaneBEarly = RNT_PLANE_BEARLY;
// Twiddles per scalar-load chunk in pass A (64 SGPRs at 32)
#ifndef RNT_PLANE_CHA
#define RNT_PLANE_CHA 32
#endif
constexpr int kPlaneChA = RNT_PLANE_CHA;
// a^ blocks in flight ahead of the degree-3 block products (0: loaded at use)
#ifndef RNT_PLANE_AHD
#define RNT_PLANE_AHD 4
#endif
constexpr int kPlaneAhd = RNT_PLANE_AHD;
// X1 through 8-byte LDS words (1) or 4-byte ones (0, default: the 8-byte
// form measured flat, profiles/r03/ab_plane_x1wide_preg.txt)
#ifndef RNT_PLANE_X1W
#define RNT_PLANE_X1W 0
#endif
constexpr bool kPlaneX1Wide = RNT_PLANE_X1W != 0;
// X1 in two rounds with pass B (gs B) of one half between them (1, needs
// the asm butterflies, which can run one half of the L1 registers) or as
// one exchange (0)
#ifndef RNT_PLANE_X1SPLIT
#define RNT_PLANE_X1SPLIT 1
#endif
constexpr bool kPlaneX1Split = RNT_PLANE_X1SPLIT != 0 && RNT_PLANE_ASM != 0;

// Pass C's per-thread twiddles (stages at index bits 5..2: 1, 2, 4 and 8
// of them), loaded ahead of the X2 exchange so the loads are in flight
// during it instead of stalling each stage of the pass.
#ifndef RNT_PLANE_PREC
#define RNT_PLANE_PREC 3  // forward pass C stages whose twiddles are preloaded (0..4)
#endif
#ifndef RNT_PLANE_PREG
#define RNT_PLANE_PREG 0  // inverse pass C stages preloaded (0..4; 1 measured flat)
#endif
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
// Forward: the first PREC stages (5, 4, ...); inverse: the first PREG (2, 3, ...).
constexpr int kPreFwd = (0xF0 >> RNT_PLANE_PREC) & 0xF;
constexpr int kPreInv = (1 << RNT_PLANE_PREG) - 1;
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
    c.t[j] = (RNT_PLANE_EXP & 8) ? Tw<uint32_t>{12345u + (uint32_t)j, 54321u} : tw_fetch<SLB>(tw, nb, (uint32_t)(M0 + j));
  return c;
}
#ifndef RNT_PLANE_TPIPE
#define RNT_PLANE_TPIPE 1
#endif
template <int LY, int SL, int M0, int CH>
constexpr bool chunk_pipe() {
  return RNT_PLANE_TPIPE != 0 && LY == 2 && M0 + CH < (32 >> SL);
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
      t[j] = (RNT_PLANE_EXP & 8) ? Tw<uint32_t>{12345u + (uint32_t)j, 54321u} : tw_fetch<BB + SL>(tw, nb, (uint32_t)(M0 + j));
  }
  if constexpr (RNT_PLANE_ASM != 0) {
    constexpr bool SW = tw_uniform<TS>() || (RNT_PLANE_EXP & 8) != 0;
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
    return;
  }
#pragma unroll
  for (int j = 0; j < n; ++j) {
#pragma unroll
    for (int e = 0; e < d; ++e) {
      const int i = ((M0 + j) << (SL + 1)) | e;
      if (SL > SLLO && (i & (d >> 1)))
        ct_bfly_lazy(x[plane::slot<LY>(i)], x[plane::slot<LY>(i | d)], t[j].w, t[j].p, mo);
      else
        ct_bfly(x[plane::slot<LY>(i)], x[plane::slot<LY>(i | d)], t[j].w, t[j].p, mo);
    }
  }
  if constexpr (M0 + CH < cnt) plane_ct_chunks<LY, BB, SL, SLLO, M0 + CH, CH>(x, nb, tw, mo);
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
  constexpr int d = 1 << SL, cnt = 32 >> SL, n = (cnt - M0) < CH ? (cnt - M0) : CH;
  Tw<uint32_t> t[n];
  if constexpr (NP == n && M0 > 0) {
#pragma unroll
    for (int j = 0; j < n; ++j) t[j] = pre->t[j];
  } else {
#pragma unroll
    for (int j = 0; j < n; ++j)
      t[j] = (RNT_PLANE_EXP & 8) ? Tw<uint32_t>{12345u + (uint32_t)j, 54321u} : tw_fetch<BB + SL>(itw, nb, (uint32_t)(M0 + j));
  }
  if constexpr (RNT_PLANE_ASM != 0) {
    constexpr int n2 = (cnt - M0 - CH) < CH ? (cnt - M0 - CH) : CH;
    TwChunk<(n2 > 0 ? n2 : 1)> nxt;
    if constexpr (chunk_pipe<LY, SL, M0, CH>()) nxt = plane_chunk<BB + SL, M0 + CH, (n2 > 0 ? n2 : 1)>(itw, nb);
    plane_gs_groups<LY, SL, M0, tw_uniform<TS>() || (RNT_PLANE_EXP & 8) != 0, HM>(x, t, mo);
    if constexpr (M0 + CH < cnt) {
      if constexpr (chunk_pipe<LY, SL, M0, CH>())
        plane_gs_chunks<LY, BB, SL, M0 + CH, CH, HM, TS, (n2 > 0 ? n2 : 1)>(x, nb, itw, mo, &nxt);
      else
        plane_gs_chunks<LY, BB, SL, M0 + CH, CH, HM>(x, nb, itw, mo);
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < n; ++j) {
#pragma unroll
    for (int e = 0; e < d; ++e) {
      const int i = ((M0 + j) << (SL + 1)) | e;
      gs_bfly(x[plane::slot<LY>(i)], x[plane::slot<LY>(i | d)], t[j].w, t[j].p, mo);
    }
  }
  if constexpr (M0 + CH < cnt) plane_gs_chunks<LY, BB, SL, M0 + CH, CH>(x, nb, itw, mo);
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

// X1, L0 <-> L1 through LDS.  Round h carries the words with index bit
// 10 == h: L0 registers 2k + h, L1 logical registers r1 = ((k >> 4) << 5) |
// (h << 4) | (k & 15), both in physical register 2k + h.  LDS word = the 15
// other index bits; every access is 64 consecutive words per wave.
// SYNC_FIRST: other waves may still be reading their X2 buffers.
template <bool TO_L1, bool SYNC_FIRST>
__device__ __forceinline__ void plane_x1(uint32_t (&x)[64], uint32_t* lds, uint32_t t) {
  const uint32_t w = t >> 6, lam = t & 63u;
  if constexpr ((RNT_PLANE_EXP & 16) != 0) return;
  if constexpr (SYNC_FIRST) __syncthreads();
  if constexpr (kPlaneX1Wide) {
    // 8-byte LDS words: pairs differing in index bit 11, a register bit on
    // both sides (L0 registers 4m + h, 4m + 2 + h; L1 registers 2k + h,
    // 2k + 32 + h); pair address = the index without bits 10 and 11.
    // ds_write_b64 / ds_read_b64 move 85 / 256 B per clock against 64 / 128
    // for the 4-byte forms, and every access stays 16 (32) consecutive pairs
    // per lane group: conflict-free.
    uint2* lp = (uint2*)lds;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        if constexpr (TO_L1)
          lp[((uint32_t)m << 10) | t] = make_uint2(x[4 * m + h], x[4 * m + 2 + h]);
        else
          lp[(w << 10) | ((uint32_t)m << 6) | lam] = make_uint2(x[2 * m + h], x[2 * m + 32 + h]);
      }
      __syncthreads();
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        if constexpr (TO_L1) {
          const uint2 v = lp[(w << 10) | ((uint32_t)m << 6) | lam];
          x[2 * m + h] = v.x;
          x[2 * m + 32 + h] = v.y;
        } else {
          const uint2 v = lp[((uint32_t)m << 10) | t];
          x[4 * m + h] = v.x;
          x[4 * m + 2 + h] = v.y;
        }
      }
      __syncthreads();
    }
    return;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const uint32_t j0 = ((uint32_t)k << 10) | t;
      const uint32_t j1 = ((((w << 1) | ((uint32_t)k >> 4))) << 10) | (((uint32_t)k & 15u) << 6) | lam;
      lds[TO_L1 ? j0 : j1] = x[2 * k + h];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const uint32_t j0 = ((uint32_t)k << 10) | t;
      const uint32_t j1 = ((((w << 1) | ((uint32_t)k >> 4))) << 10) | (((uint32_t)k & 15u) << 6) | lam;
      x[2 * k + h] = lds[TO_L1 ? j1 : j0];
    }
    __syncthreads();
  }
}

// One round of X1 (4-byte words), as plane_x1: WRITE puts round H's
// registers into LDS, !WRITE takes them out.  plane_fwd / plane_mul_tail
// split X1 into these so that pass B (gs B) of the half already delivered
// (still to be sent) runs while the other round's LDS traffic drains.
template <bool TO_L1, int H, bool WRITE>
__device__ __forceinline__ void plane_x1_round(uint32_t (&x)[64], uint32_t* lds, uint32_t t) {
  if constexpr ((RNT_PLANE_EXP & 16) != 0) return;
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
__device__ __forceinline__ void plane_sync() {
  if constexpr ((RNT_PLANE_EXP & 16) == 0) __syncthreads();
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
// order, so the reads see the same wave's writes; two buffers alternate.
template <bool TO_L2>
__device__ __forceinline__ void plane_x2(uint32_t (&x)[64], uint32_t* lds, uint32_t t) {
  const uint32_t w = t >> 6, lam = t & 63u;
  if constexpr ((RNT_PLANE_EXP & 16) != 0) return;
  if constexpr (TO_L2) plane_swap54(x);
  const uint32_t a15 = lam * plane::XS;                          // + (m & 15)
  const uint32_t a2 = (lam & 48u) * plane::XS + (lam & 15u);     // + c * XS
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    uint32_t* buf = lds + (w * 2u + (uint32_t)(g & 1)) * plane::XW;
#pragma unroll
    for (int j = 0; j < 16; ++j) buf[TO_L2 ? a15 + j : a2 + j * plane::XS] = x[plane::slot1((g << 4) | j)];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int c = 0; c < 16; ++c) x[plane::slot1((g << 4) | c)] = buf[TO_L2 ? a2 + c * plane::XS : a15 + c];
    __builtin_amdgcn_wave_barrier();
  }
  if constexpr (!TO_L2) plane_swap54(x);
}

// One workgroup per CU and equal work per workgroup keep every CU's load,
// compute and store phases in step across the chip, so the loads of all
// CUs meet at the HBM together while the VALUs idle, and then the other
// way round.  Delaying the first workgroup of every other CU by `ticks`
// of the 100 MHz real-time counter once shifts that CU's phase for the
// rest of the launch (its next workgroups start when the previous one
// ends), so half the CUs load while the other half compute.
__device__ __forceinline__ void plane_stagger(uint32_t ticks) {
  if (ticks == 0) return;
  const uint32_t id = blockIdx.x + blockIdx.y * gridDim.x;
  if (id >= 256u || !((id >> 3) & 1u)) return;  // first wave, every other CU of each XCD
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
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

// Measurement builds (tools/build_variant.sh, wrong results by design):
// RNT_PLANE_EXP bit 0: pass C / inverse pass C twiddles wave-uniform;
// bit 1: no plane loads (synthetic words); bit 2: no plane stores;
// bit 3: no twiddle loads in the passes (one constant); bit 4: no X1 / X2;
// bit 5: no product store; bit 6: no a^ store (the a^ loads stay).

// ... and in pass B (wave-uniform too)
#ifndef RNT_PLANE_CHB
#define RNT_PLANE_CHB 16
#endif
constexpr int kPlaneChB = RNT_PLANE_CHB;
// twiddles per chunk in pass C (per-lane twiddles)
#ifndef RNT_PLANE_CHC
#define RNT_PLANE_CHC 8
#endif
constexpr int kPlaneChC = RNT_PLANE_CHC;

// Register of the q-th plane load.
__host__ __device__ constexpr int plane_load_reg(int q) {
  return kPlaneLoadOrder ? (((q >> 3) << 2) | (q & 3)) + ((q & 4) ? 32 : 0) : q;
}

// Load the L0 plane at src (64 coalesced dword loads a thread).
__device__ __forceinline__ void plane_load(uint32_t (&x)[64], const uint32_t* src, uint32_t t) {
  if constexpr ((RNT_PLANE_EXP & 2) != 0) {
#pragma unroll
    for (int r = 0; r < 64; ++r) x[r] = (t * 2654435761u + (uint32_t)r * 40503u) >> 2;
    return;
  }
  const __amdgpu_buffer_rsrc_t g = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, (int)(4u << 16), 0x00020000);
  // in the order pass A's first stage consumes them (groups of four pairs
  // r, r + 32), so its butterflies start while the rest of the plane is
  // still arriving (loads return in order; each use waits only for its own)
#pragma unroll
  for (int q = 0; q < 64; ++q) {
    const int r = plane_load_reg(q);
    x[r] = __builtin_amdgcn_raw_buffer_load_b32(g, t * 4u, (uint32_t)r << 12, kPlaneAux);
  }
}

// The CU this workgroup runs on, as a dense id below kPlaneSlots: XCC_ID
// (hwreg 20, bits 3:0) and HW_ID's SE_ID (15:13), SH_ID (12), CU_ID (11:8).
// The plane kernels use 139 KiB of LDS and the whole register file, so a CU
// runs one of their workgroups at a time: while it runs, the id names a
// scratch slot no other workgroup of the launch uses.
constexpr uint32_t kPlaneSlots = 1u << 12;
__device__ __forceinline__ uint32_t plane_cu_slot() {
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
  const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
  return ((xcc & 15u) << 8) | (((hw >> 13) & 7u) << 5) | (((hw >> 12) & 1u) << 4) | ((hw >> 8) & 15u);
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
template <int K, bool SYNC1, class H1 = NoHook, class H2 = NoHook, bool FULL = false>
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
  PLANE_STAMP(K, 2);
  const uint32_t wu = __builtin_amdgcn_readfirstlane(t >> 6);
  if constexpr (kPlaneX1Split) {
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
  } else {
    plane_x1<true, SYNC1>(x, lds, t);
    PLANE_STAMP(K, 3);
    after_x1();
    plane_ct<1, 6, 3, 0, kPlaneChB>(x, N + (wu << 12), tws, mo);
  }
  PLANE_STAMP(K, 4);
  const auto pc = plane_pre<kPreFwd>(tw, N + (t << 6));
  plane_x2<true>(x, lds, t);
  PLANE_STAMP(K, 5);
  after_x2();
  // pass C: bits 5..2 for the product (bits 1..0 are its truncated
  // stages), bits 5..0 for a standalone transform (FULL)
  constexpr int SLLO_C = FULL ? 0 : 2;
  if constexpr ((RNT_PLANE_EXP & 1) != 0)
    plane_ct<2, 0, 5, SLLO_C, kPlaneChC>(x, N, tws, mo);
  else
    plane_ct<2, 0, 5, SLLO_C, kPlaneChC>(x, N + (t << 6), pc, mo);
  PLANE_STAMP(K, 6);
}

// The inverse transform from pass C's layout (L2) to the store of c in L0:
// gs C on bits SLLO_C..5 (2 after a truncated product, 0 for a standalone
// transform), X2, gs B, X1 (split as the forward one), gs A with the folded
// last-stage constants F (4/N with the Montgomery factor after a product,
// 1/N for a standalone transform).
template <int K, int SLLO_C, class TSC>
__device__ __forceinline__ void plane_inv_tail(uint32_t (&x)[64], uint32_t* lds, uint32_t t, uint32_t* c,
                                               const Tw<uint32_t>* itw, const TSC& gsrc, const Mod<uint32_t>& mo,
                                               const Fold<uint32_t>& F, uint32_t trace_id) {
  (void)trace_id;
  const uint32_t n0 = 1u << 16;
  const TwScalar<uint32_t> itws{(const RNT_CONST_AS Tw<uint32_t>*)itw};
  if constexpr ((RNT_PLANE_EXP & 1) != 0)
    plane_gs<2, 0, SLLO_C, 5, kPlaneChC, false>(x, n0, itws, mo, Fold<uint32_t>{});
  else
    plane_gs<2, 0, SLLO_C, 5, kPlaneChC, false>(x, n0 + (t << 6), gsrc, mo, Fold<uint32_t>{});
  PLANE_STAMP(K, 8);
  plane_x2<false>(x, lds, t);
  PLANE_STAMP(K, 9);
  const uint32_t wu = __builtin_amdgcn_readfirstlane(t >> 6);
  if constexpr (kPlaneX1Split) {
    // gs B of round 0's half, X1 round 0 written while gs B of the other half runs
    plane_gs<1, 6, 0, 3, kPlaneChB, false, 0>(x, n0 + (wu << 12), itws, mo, Fold<uint32_t>{});
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
  } else {
    plane_gs<1, 6, 0, 3, kPlaneChB, false>(x, n0 + (wu << 12), itws, mo, Fold<uint32_t>{});
    PLANE_STAMP(K, 10);
    plane_x1<false, true>(x, lds, t);  // other waves may still be in their X2
  }
  PLANE_STAMP(K, 11);
  plane_gs<0, 10, 0, 5, kPlaneChA, true>(x, n0, itws, mo, F);
  PLANE_STAMP(K, 12);
  if ((RNT_PLANE_EXP & (4 | 32)) != 0 && x[0] != 0xffffffffu) return;
  const __amdgpu_buffer_rsrc_t dst = __builtin_amdgcn_make_buffer_rsrc((void*)c, 0, (int)(4u << 16), 0x00020000);
#pragma unroll
  for (int r = 0; r < 64; ++r) __builtin_amdgcn_raw_buffer_store_b32(x[r], dst, t * 4u, (uint32_t)r << 12, kPlaneAux);
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
  constexpr int D = kPlaneAhd, Z = D > 0 ? (D + 1) / 2 + 1 : 1;  // zeta j serves blocks 2j, 2j + 1
  uint4 abuf[D > 0 ? D : 1];
  Tw<uint32_t> zbuf[Z];
  TwPre<kPreInv> gpre;  // the inverse pass C's first stages, loaded during the last products
  if constexpr (D == 0) gpre = plane_pre<kPreInv>(itw, n0 + (t << 6));
  if constexpr (D > 0) {
#pragma unroll
    for (int d = 0; d < D; ++d) abuf[d] = ah(d);
#pragma unroll
    for (int j = 0; j < Z; ++j) zbuf[j] = tw[zb + j];
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    uint4 av;
    Tw<uint32_t> w;
    if constexpr ((RNT_PLANE_EXP & 2) != 0) {
      av = make_uint4(t * 7u + kk, t * 11u, t + 3u * kk, t ^ 0x55u);
      w = tw[zb + (kk >> 1)];
    } else if constexpr (D > 0) {
      av = abuf[kk % D];
      w = zbuf[(kk >> 1) % Z];
      if (kk + D < 16) abuf[kk % D] = ah(kk + D);
      if (kk == 16 - D) gpre = plane_pre<kPreInv>(itw, n0 + (t << 6));
      if ((kk & 1) && (kk >> 1) + Z < 8) zbuf[(kk >> 1) % Z] = tw[zb + (kk >> 1) + Z];
      __builtin_amdgcn_sched_barrier(0);
    } else {
      av = ah(kk);
      w = tw[zb + (kk >> 1)];
    }
    const uint32_t aa[4] = {av.x, av.y, av.z, av.w};
    const uint32_t bb[4] = {x[plane::slot2(4 * kk)], x[plane::slot2(4 * kk + 1)], x[plane::slot2(4 * kk + 2)],
                            x[plane::slot2(4 * kk + 3)]};
    const uint32_t zeta = (kk & 1) ? lc.q - w.w : w.w;
    const uint32_t zeta_p = (kk & 1) ? ~w.p : w.p;
    uint32_t cc[4];
    mul_mod_x4(cc, aa, bb, zeta, zeta_p, lc.q, lc.qinv);
#pragma unroll
    for (int e = 0; e < 4; ++e) x[plane::slot2(4 * kk + e)] = cc[e];
  }
  PLANE_STAMP(K, 7);
  plane_inv_tail<K, 2>(x, lds, t, c, itw, gpre, mo, Fold<uint32_t>{lc.c1t, lc.c1t_p, lc.c2t, lc.c2t_p}, trace_id);
}

// a^ in the private layout: block kk (4 words) of thread t at (kk * 1024 + t) * 4
__device__ __forceinline__ void plane_store_hat(const HatBuf& dst, const uint32_t (&x)[64], uint32_t t) {
  if ((RNT_PLANE_EXP & (4 | 64)) != 0 && x[0] != 0xffffffffu) return;
#pragma unroll
  for (int kk = 0; kk < 16; ++kk)
    dst.st(t, kk, x[plane::slot2(4 * kk)], x[plane::slot2(4 * kk + 1)], x[plane::slot2(4 * kk + 2)],
           x[plane::slot2(4 * kk + 3)]);
}

// One workgroup per plane, grid (B, L).
__global__ void __launch_bounds__(plane::T, 1)
k_plane_fwd(uint32_t* __restrict__ ahat, const uint32_t* __restrict__ a, TabPtrs<uint32_t> tp, uint64_t ls,
            uint32_t stagger) {
  plane_stagger(stagger);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  uint32_t* lds = (uint32_t*)smem_raw;
  const uint32_t t = threadIdx.x, poly = blockIdx.x, l = blockIdx.y;
  const uint32_t trace_id = poly + l * gridDim.x;
  PLANE_STAMP(0, 0);
  const uint64_t N = 1ull << 16;
  const uint64_t off = (uint64_t)l * ls + (uint64_t)poly * N;
  uint32_t x[64];
  plane_load(x, a + off, t);
  PLANE_STAMP(0, 1);
  plane_fwd<0, false>(x, lds, t, tp.tw + (uint64_t)l * N, mod_of(tp.lc[l]), trace_id);
  plane_store_hat(HatBuf(ahat + off), x, t);
  PLANE_STAMP(0, 7);
}

__global__ void __launch_bounds__(plane::T, 1)
k_plane_mul(uint32_t* __restrict__ c, const uint32_t* __restrict__ b, const uint32_t* __restrict__ ahat,
            TabPtrs<uint32_t> tp, uint64_t ls, uint32_t stagger) {
  plane_stagger(stagger);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  uint32_t* lds = (uint32_t*)smem_raw;
  const uint32_t t = threadIdx.x, poly = blockIdx.x, l = blockIdx.y;
  const uint32_t trace_id = poly + l * gridDim.x;
  PLANE_STAMP(1, 0);
  const uint64_t N = 1ull << 16;
  const uint64_t off = (uint64_t)l * ls + (uint64_t)poly * N;
  const LimbConst<uint32_t> lc = tp.lc[l];
  const Mod<uint32_t> mo = mod_of(lc);
  const Tw<uint32_t>* tw = tp.tw + (uint64_t)l * N;
  uint32_t x[64];
  plane_load(x, b + off, t);
  PLANE_STAMP(1, 1);
  plane_fwd<1, false>(x, lds, t, tw, mo, trace_id);
  const uint4* ah = (const uint4*)(ahat + off);
  const HatBuf hb(ah);
  plane_mul_tail<1>(x, lds, t, [hb, t](int kk) { return hb.ld(t, kk); }, c + off, tw, tp.itw + (uint64_t)l * N,
                    lc, mo, trace_id);
}

// Both halves in one workgroup (RNT_PLANE=3): a -> a^ through the scratch
// plane, which the same threads read back ~40 us later (so the read is
// served by the Infinity Cache or L2 rather than HBM), then b -> c as
// k_plane_mul.  One launch per batch; the store of a^ and the load of b
// are back to back and overlap.
// The product of one (poly, limb) plane pair; the body of both fused kernels.
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
  if constexpr (kPlaneBEarly > 0) {
    // b's first KB loads (in plane_load's order) go out before a^'s stores,
    // so waiting for them does not wait for the stores (one in-order vmcnt
    // counter): pass A of b starts on them while the stores drain
    constexpr int KB = kPlaneBEarly;
    const uint32_t* bp = b + off;
    asm volatile("" : "+s"(bp));
    const __amdgpu_buffer_rsrc_t gb = __builtin_amdgcn_make_buffer_rsrc((void*)bp, 0, (int)(4u << 16), 0x00020000);
    uint32_t y[KB > 0 ? KB : 1];
#pragma unroll
    for (int q = 0; q < KB; ++q) {
      const int r = plane_load_reg(q);
      y[q] = __builtin_amdgcn_raw_buffer_load_b32(gb, t * 4u, (uint32_t)r << 12, kPlaneAux);
    }
    __builtin_amdgcn_sched_barrier(0);
    plane_store_hat(HatBuf(ah), x, t);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 64; ++q) {
      const int r = plane_load_reg(q);
      x[r] = q < KB ? y[q < KB ? q : 0] : __builtin_amdgcn_raw_buffer_load_b32(gb, t * 4u, (uint32_t)r << 12, kPlaneAux);
    }
  } else {
    plane_store_hat(HatBuf(ah), x, t);
    PLANE_STAMP(0, 7);
    PLANE_STAMP(1, 0);
    plane_load(x, b + off, t);
  }
  PLANE_STAMP(1, 1);
  plane_fwd<1, true>(x, lds, t, tw, mo, trace_id);
  // a^ comes back from this thread's own stores above (the descriptor is
  // rebuilt from an opaque copy of the base, so nothing of the stores'
  // addressing stays live across b's transform)
  uint32_t* ah2 = ah;
  asm volatile("" : "+s"(ah2));
  const HatBuf hb(ah2);
  plane_mul_tail<1>(x, lds, t, [hb, t](int kk) { return hb.ld(t, kk); }, c + off, tw, tp.itw + (uint64_t)l * N, lc,
                    mo, trace_id);
}


__global__ void __launch_bounds__(plane::T, 1)
k_plane_fused(uint32_t* __restrict__ c, const uint32_t* a, const uint32_t* b, uint32_t* __restrict__ scratch,
              TabPtrs<uint32_t> tp, uint64_t ls, uint32_t cu_slots) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const uint64_t N = 1ull << 16;
  const uint32_t poly = blockIdx.x, l = blockIdx.y;
  // a^ goes to a scratch plane: per (poly, limb), or (cu_slots) per CU, so
  // the launch's scratch footprint is 256 KiB per CU (64 MiB on 256 CUs),
  // rewritten by the CU's next workgroup while it may still sit in the
  // Infinity Cache
  uint32_t* ah = scratch + (cu_slots ? (uint64_t)plane_cu_slot() * N : (uint64_t)l * ls + (uint64_t)poly * N);
  plane_fused_one(c, a, b, ah, tp, ls, poly, l, (uint32_t*)smem_raw, threadIdx.x, poly + l * gridDim.x);
}

// Persistent form (RNT_PLANE=4): one workgroup per CU walks the planes p =
// blockIdx.x, + gridDim.x, ... (poly p % B, limb p / B, so the chip works on
// one limb's twiddles at a time), with its own a^ scratch plane: a plane's
// product stores and the next plane's loads meet in one wave's queue instead
// of a workgroup ending and the next one starting.
__global__ void __launch_bounds__(plane::T, 1)
k_plane_fused_p(uint32_t* __restrict__ c, const uint32_t* a, const uint32_t* b, uint32_t* __restrict__ scratch,
                TabPtrs<uint32_t> tp, uint64_t ls, uint32_t B, uint32_t planes) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  uint32_t* ah = scratch + (uint64_t)blockIdx.x * (1ull << 16);
  for (uint32_t p = blockIdx.x; p < planes; p += gridDim.x) {
    const uint32_t l = p / B, poly = p - l * B;
    // opaque per-iteration copies of the bases: nothing derived from them is
    // hoisted out of the loop and held (in spilled registers) across a body
    uint32_t* c1 = c;
    const uint32_t *a1 = a, *b1 = b;
    uint32_t* ah1 = ah;
    TabPtrs<uint32_t> tp1 = tp;
    asm volatile("" : "+s"(c1), "+s"(a1), "+s"(b1), "+s"(ah1));
    asm volatile("" : "+s"(tp1.tw), "+s"(tp1.itw), "+s"(tp1.lc));
    plane_fused_one(c1, a1, b1, ah1, tp1, ls, poly, l, (uint32_t*)smem_raw, threadIdx.x, p);
  }
}

// Standalone transforms at N = 2^16, u32 bases (rnt_ntt_fwd / rnt_ntt_inv,
// to_ntt_domain / to_coeff_domain, poly.rs:136-166): one workgroup per
// (poly, limb) plane, in place.  Forward: the L0 load, all 16 stages (pass C
// runs bits 5..0), and the L2 layout stored as it stands -- thread t holds
// the 64 consecutive device-order words (t << 6) .. (t << 6) + 63, the same
// bit-reversed order the four-step kernels write.  Inverse: those words in,
// gs C from bit 0, then as after a product with the plain 1/N fold.  2
// planes of HBM traffic per transform against the four-step kernels' 4.
template <bool INV>
__global__ void __launch_bounds__(plane::T, 1)
k_plane_ntt(uint32_t* __restrict__ data, TabPtrs<uint32_t> tp, uint64_t ls) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  uint32_t* lds = (uint32_t*)smem_raw;
  const uint32_t t = threadIdx.x, poly = blockIdx.x, l = blockIdx.y;
  const uint64_t N = 1ull << 16;
  const uint64_t off = (uint64_t)l * ls + (uint64_t)poly * N;
  const LimbConst<uint32_t> lc = tp.lc[l];
  const Mod<uint32_t> mo = mod_of(lc);
  uint32_t x[64];
  if constexpr (!INV) {
    plane_load(x, data + off, t);
    plane_fwd<0, false, NoHook, NoHook, true>(x, lds, t, tp.tw + (uint64_t)l * N, mo, poly + l * gridDim.x);
    uint32_t* dp = data + off;
    asm volatile("" : "+s"(dp));
    const __amdgpu_buffer_rsrc_t g = __builtin_amdgcn_make_buffer_rsrc((void*)dp, 0, (int)(4u << 16), 0x00020000);
    using V4 = decltype(__builtin_amdgcn_raw_buffer_load_b128(g, 0, 0, 0));
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      V4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = x[plane::slot2(4 * kk + e)];
      __builtin_amdgcn_raw_buffer_store_b128(v, g, t * 256u, (uint32_t)kk * 16u, kPlaneAux);
    }
  } else {
    const __amdgpu_buffer_rsrc_t g =
        __builtin_amdgcn_make_buffer_rsrc((void*)(data + off), 0, (int)(4u << 16), 0x00020000);
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(g, t * 256u, (uint32_t)kk * 16u, kPlaneAux);
#pragma unroll
      for (int e = 0; e < 4; ++e) x[plane::slot2(4 * kk + e)] = v[e];
    }
    const Tw<uint32_t>* itw = tp.itw + (uint64_t)l * N;
    TwPre<0> gsrc;
    gsrc.b = itw;
    plane_inv_tail<1, 0>(x, lds, t, data + off, itw, gsrc, mo, Fold<uint32_t>{lc.c1, lc.c1_p, lc.c2, lc.c2_p},
                         poly + l * gridDim.x);
  }
}

#ifdef RNT_PLANE_TRACE
extern "C" __attribute__((visibility("default"))) int rnt_debug_plane_trace(uint64_t* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_plane_trace), sizeof(g_plane_trace));
}
#endif

// The whole-plane product (k_plane_fwd + k_plane_mul) serves rnt_mul for
// u32 canonical bases at N = 2^16 when Tables::plane is set (RNT_PLANE).
// The whole-plane kernels take every u32 basis at N = 2^16 (their
// canonical arithmetic holds for any q < 2^31, so 30-bit bases too: 131k
// against the lazy four-step kernels' 114k products/s).
bool plane_ok(const Tables* t) {
  return t->plane != 0 && !t->wide && t->log_n == 16;
}

hipError_t launch_plane(const Launch& k, int which, void* out, const void* in, const void* ahat,
                        uint64_t ls) {
  if (k.B == 0 || k.L == 0) return hipSuccess;
  if (k.B > 0x7fffffffull || k.L > 65535) return hipErrorInvalidConfiguration;
  const size_t lds = (size_t)plane::LDS_WORDS * 4;
  const dim3 grid((unsigned)k.B, (unsigned)k.L);
  const uint32_t st = k.t->plane_stagger;
  if (which == 0) {
    hipError_t e = allow_lds(k_plane_fwd, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_plane_fwd, grid, dim3(plane::T), lds, k.s, (uint32_t*)out, (const uint32_t*)in,
                       tab_ptrs<uint32_t>(k.t), ls, st);
  } else {
    hipError_t e = allow_lds(k_plane_mul, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_plane_mul, grid, dim3(plane::T), lds, k.s, (uint32_t*)out, (const uint32_t*)in,
                       (const uint32_t*)ahat, tab_ptrs<uint32_t>(k.t), ls, st);
  }
  return hipGetLastError();
}

#ifndef RNT_PLANE_SLOTS
#define RNT_PLANE_SLOTS 0
#endif
// Per-CU scratch slots once the batch has at least as many planes as slots
// (the workspace, one plane per (poly, limb), then holds every slot).
bool plane_fused_slots(const Launch& k) {
  return RNT_PLANE_SLOTS && (uint64_t)k.B * k.L >= kPlaneSlots;
}

hipError_t launch_plane_ntt(const Launch& k, int inverse, void* data, uint64_t ls) {
  if (k.B == 0 || k.L == 0) return hipSuccess;
  if (k.B > 0x7fffffffull || k.L > 65535) return hipErrorInvalidConfiguration;
  const size_t lds = (size_t)plane::LDS_WORDS * 4;
  const dim3 grid((unsigned)k.B, (unsigned)k.L);
  if (inverse) {
    hipError_t e = allow_lds(k_plane_ntt<true>, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_plane_ntt<true>, grid, dim3(plane::T), lds, k.s, (uint32_t*)data, tab_ptrs<uint32_t>(k.t), ls);
  } else {
    hipError_t e = allow_lds(k_plane_ntt<false>, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_plane_ntt<false>, grid, dim3(plane::T), lds, k.s, (uint32_t*)data, tab_ptrs<uint32_t>(k.t), ls);
  }
  return hipGetLastError();
}

static int plane_cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      n = v > 0 ? v : 256;
    else
      n = 256;
  }
  return n;
}

hipError_t launch_plane_fused(const Launch& k, void* out, const void* a, const void* b, void* scratch, uint64_t ls) {
  if (k.B == 0 || k.L == 0) return hipSuccess;
  if (k.B > 0x7fffffffull || k.L > 65535) return hipErrorInvalidConfiguration;
  const size_t lds = (size_t)plane::LDS_WORDS * 4;
  const uint64_t planes = (uint64_t)k.B * k.L;
  if (k.t->plane == 4 && planes < 0xffffffffull) {
    // one workgroup per CU, each with one a^ scratch plane (planes >= grid)
    const unsigned grid = (unsigned)std::min<uint64_t>(planes, (uint64_t)plane_cu_count());
    hipError_t e = allow_lds(k_plane_fused_p, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_plane_fused_p, dim3(grid), dim3(plane::T), lds, k.s, (uint32_t*)out, (const uint32_t*)a,
                       (const uint32_t*)b, (uint32_t*)scratch, tab_ptrs<uint32_t>(k.t), ls, (uint32_t)k.B,
                       (uint32_t)planes);
    return hipGetLastError();
  }
  hipError_t e = allow_lds(k_plane_fused, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_plane_fused, dim3((unsigned)k.B, (unsigned)k.L), dim3(plane::T), lds, k.s, (uint32_t*)out,
                     (const uint32_t*)a, (const uint32_t*)b, (uint32_t*)scratch, tab_ptrs<uint32_t>(k.t), ls,
                     plane_fused_slots(k) ? 1u : 0u);
  return hipGetLastError();
}

}  // namespace rnt
