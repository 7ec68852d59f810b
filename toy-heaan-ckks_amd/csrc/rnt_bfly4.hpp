// rnt_bfly4.hpp -- four interleaved 31-bit NTT butterflies in inline asm
// (gfx950), for the whole-plane poly-mul kernels (rnt_plane.hip).
//
// Why: written in C++, every butterfly's borrow-selects (v_sub_co_u32 ->
// v_cndmask_b32) go through VCC, so hipcc schedules the butterflies one
// after another, each a single dependency chain padded with s_nop hazard
// waits (about a quarter of the instructions of k_plane_fused were s_nop).
// With four waves per SIMD (one 1024-thread workgroup per CU) that left the
// VALU at ~4.4 cycles per instruction; the measurement builds showed the
// kernel bound by that issue rate, not by memory
// (profiles/r03/ab_plane_meas_builds.txt).  Here four independent
// butterflies advance in lock step, each with its own carry pair and
// temporaries, so every producer is at least three instructions ahead of
// its consumer (the VALU->carry->v_cndmask and v_mad_u64_u32->use wait
// states hipcc pads with s_nop) and the blocks need no padding.
//
// The arithmetic is exactly that of rnt_modarith.hpp's ct_bfly /
// ct_bfly_lazy / gs_bfly (Shoup products, borrow-select reductions), so the
// results are bit-identical: canonical residues, q < 2^31, nq = 2^32 - q.
// A butterfly's Shoup product is split in two statements (the 64-bit
// product, then the reduction of its low word), because inline asm has no
// way to name one half of a 64-bit register pair.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rnt {
namespace b4 {

// P[k] = y[k] * w[k] + floor(y[k] * wp[k] / 2^32) * nq (only the low word is
// used: y w mod q in [0, 2q)).  SW: twiddles wave-uniform (SGPRs).
template <bool SW>
__device__ __forceinline__ void shoup_prod4(uint64_t (&P)[4], uint32_t y0, uint32_t y1, uint32_t y2, uint32_t y3,
                                            const uint32_t (&w)[4], const uint32_t (&wp)[4], uint32_t nq) {
  uint32_t h0, h1, h2, h3;
  uint64_t cc;
#define RNT_B4_PROD_ASM                                          \
  "v_mul_hi_u32 %[h0], %[wp0], %[y0]\n\t"                        \
  "v_mul_hi_u32 %[h1], %[wp1], %[y1]\n\t"                        \
  "v_mul_hi_u32 %[h2], %[wp2], %[y2]\n\t"                        \
  "v_mul_hi_u32 %[h3], %[wp3], %[y3]\n\t"                        \
  "v_mad_u64_u32 %[P0], %[cc], %[w0], %[y0], 0\n\t"              \
  "v_mad_u64_u32 %[P1], %[cc], %[w1], %[y1], 0\n\t"              \
  "v_mad_u64_u32 %[P2], %[cc], %[w2], %[y2], 0\n\t"              \
  "v_mad_u64_u32 %[P3], %[cc], %[w3], %[y3], 0\n\t"              \
  "v_mad_u64_u32 %[P0], %[cc], %[h0], %[nq], %[P0]\n\t"          \
  "v_mad_u64_u32 %[P1], %[cc], %[h1], %[nq], %[P1]\n\t"          \
  "v_mad_u64_u32 %[P2], %[cc], %[h2], %[nq], %[P2]\n\t"          \
  "v_mad_u64_u32 %[P3], %[cc], %[h3], %[nq], %[P3]"
#define RNT_B4_PROD_OUT                                                                       \
  [P0] "=&v"(P[0]), [P1] "=&v"(P[1]), [P2] "=&v"(P[2]), [P3] "=&v"(P[3]), [h0] "=&v"(h0), \
      [h1] "=&v"(h1), [h2] "=&v"(h2), [h3] "=&v"(h3), [cc] "=&s"(cc)
  if constexpr (SW) {
    asm volatile(RNT_B4_PROD_ASM
                 : RNT_B4_PROD_OUT
                 : [y0] "v"(y0), [y1] "v"(y1), [y2] "v"(y2), [y3] "v"(y3), [w0] "s"(w[0]), [w1] "s"(w[1]),
                   [w2] "s"(w[2]), [w3] "s"(w[3]), [wp0] "s"(wp[0]), [wp1] "s"(wp[1]), [wp2] "s"(wp[2]),
                   [wp3] "s"(wp[3]), [nq] "s"(nq));
  } else {
    asm volatile(RNT_B4_PROD_ASM
                 : RNT_B4_PROD_OUT
                 : [y0] "v"(y0), [y1] "v"(y1), [y2] "v"(y2), [y3] "v"(y3), [w0] "v"(w[0]), [w1] "v"(w[1]),
                   [w2] "v"(w[2]), [w3] "v"(w[3]), [wp0] "v"(wp[0]), [wp1] "v"(wp[1]), [wp2] "v"(wp[2]),
                   [wp3] "v"(wp[3]), [nq] "s"(nq));
  }
#undef RNT_B4_PROD_ASM
#undef RNT_B4_PROD_OUT
}

// CT butterflies, canonical outputs: t = csub(p) = y w mod q,
// (x, y) <- (x + t mod q, x - t mod q).  p[k] is clobbered.
__device__ __forceinline__ void ct_reduce4(uint32_t& x0, uint32_t& x1, uint32_t& x2, uint32_t& x3, uint32_t& y0,
                                           uint32_t& y1, uint32_t& y2, uint32_t& y3, uint32_t (&p)[4], uint32_t q) {
  uint32_t a0, a1, a2, a3, b0, b1, b2, b3;
  uint64_t c0, c1, c2, c3;
  asm volatile(
      // t' = p - q; t = borrow ? p : t'
      "v_sub_co_u32 %[a0], %[c0], %[p0], %[q]\n\t"
      "v_sub_co_u32 %[a1], %[c1], %[p1], %[q]\n\t"
      "v_sub_co_u32 %[a2], %[c2], %[p2], %[q]\n\t"
      "v_sub_co_u32 %[a3], %[c3], %[p3], %[q]\n\t"
      "v_cndmask_b32 %[a0], %[a0], %[p0], %[c0]\n\t"
      "v_cndmask_b32 %[a1], %[a1], %[p1], %[c1]\n\t"
      "v_cndmask_b32 %[a2], %[a2], %[p2], %[c2]\n\t"
      "v_cndmask_b32 %[a3], %[a3], %[p3], %[c3]\n\t"
      // d = x - t; y = borrow ? d + q : d
      "v_sub_co_u32 %[b0], %[c0], %[x0], %[a0]\n\t"
      "v_sub_co_u32 %[b1], %[c1], %[x1], %[a1]\n\t"
      "v_sub_co_u32 %[b2], %[c2], %[x2], %[a2]\n\t"
      "v_sub_co_u32 %[b3], %[c3], %[x3], %[a3]\n\t"
      "v_add_u32 %[p0], %[q], %[b0]\n\t"
      "v_add_u32 %[p1], %[q], %[b1]\n\t"
      "v_add_u32 %[p2], %[q], %[b2]\n\t"
      "v_add_u32 %[p3], %[q], %[b3]\n\t"
      "v_cndmask_b32 %[y0], %[b0], %[p0], %[c0]\n\t"
      "v_cndmask_b32 %[y1], %[b1], %[p1], %[c1]\n\t"
      "v_cndmask_b32 %[y2], %[b2], %[p2], %[c2]\n\t"
      "v_cndmask_b32 %[y3], %[b3], %[p3], %[c3]\n\t"
      // s = x + t; x = s >= q ? s - q : s
      "v_add_u32 %[b0], %[x0], %[a0]\n\t"
      "v_add_u32 %[b1], %[x1], %[a1]\n\t"
      "v_add_u32 %[b2], %[x2], %[a2]\n\t"
      "v_add_u32 %[b3], %[x3], %[a3]\n\t"
      "v_sub_co_u32 %[p0], %[c0], %[b0], %[q]\n\t"
      "v_sub_co_u32 %[p1], %[c1], %[b1], %[q]\n\t"
      "v_sub_co_u32 %[p2], %[c2], %[b2], %[q]\n\t"
      "v_sub_co_u32 %[p3], %[c3], %[b3], %[q]\n\t"
      "v_cndmask_b32 %[x0], %[p0], %[b0], %[c0]\n\t"
      "v_cndmask_b32 %[x1], %[p1], %[b1], %[c1]\n\t"
      "v_cndmask_b32 %[x2], %[p2], %[b2], %[c2]\n\t"
      "v_cndmask_b32 %[x3], %[p3], %[b3], %[c3]"
      : [x0] "+v"(x0), [x1] "+v"(x1), [x2] "+v"(x2), [x3] "+v"(x3), [y0] "+v"(y0), [y1] "+v"(y1), [y2] "+v"(y2),
        [y3] "+v"(y3), [p0] "+v"(p[0]), [p1] "+v"(p[1]), [p2] "+v"(p[2]), [p3] "+v"(p[3]), [a0] "=&v"(a0),
        [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3), [b0] "=&v"(b0), [b1] "=&v"(b1), [b2] "=&v"(b2),
        [b3] "=&v"(b3), [c0] "=&s"(c0), [c1] "=&s"(c1), [c2] "=&s"(c2), [c3] "=&s"(c3)
      : [q] "s"(q));
}

// CT butterflies with lazy outputs (both in [0, 2q], as ct_bfly_lazy):
// t = csub(p), (x, y) <- (x + t, x + q - t).
__device__ __forceinline__ void ct_reduce4_lazy(uint32_t& x0, uint32_t& x1, uint32_t& x2, uint32_t& x3,
                                                uint32_t& y0, uint32_t& y1, uint32_t& y2, uint32_t& y3,
                                                uint32_t (&p)[4], uint32_t q) {
  uint32_t a0, a1, a2, a3;
  uint64_t c0, c1, c2, c3;
  asm volatile(
      "v_sub_co_u32 %[a0], %[c0], %[p0], %[q]\n\t"
      "v_sub_co_u32 %[a1], %[c1], %[p1], %[q]\n\t"
      "v_sub_co_u32 %[a2], %[c2], %[p2], %[q]\n\t"
      "v_sub_co_u32 %[a3], %[c3], %[p3], %[q]\n\t"
      "v_cndmask_b32 %[a0], %[a0], %[p0], %[c0]\n\t"
      "v_cndmask_b32 %[a1], %[a1], %[p1], %[c1]\n\t"
      "v_cndmask_b32 %[a2], %[a2], %[p2], %[c2]\n\t"
      "v_cndmask_b32 %[a3], %[a3], %[p3], %[c3]\n\t"
      "v_sub_u32 %[y0], %[q], %[a0]\n\t"
      "v_sub_u32 %[y1], %[q], %[a1]\n\t"
      "v_sub_u32 %[y2], %[q], %[a2]\n\t"
      "v_sub_u32 %[y3], %[q], %[a3]\n\t"
      "v_add_u32 %[y0], %[x0], %[y0]\n\t"
      "v_add_u32 %[y1], %[x1], %[y1]\n\t"
      "v_add_u32 %[y2], %[x2], %[y2]\n\t"
      "v_add_u32 %[y3], %[x3], %[y3]\n\t"
      "v_add_u32 %[x0], %[x0], %[a0]\n\t"
      "v_add_u32 %[x1], %[x1], %[a1]\n\t"
      "v_add_u32 %[x2], %[x2], %[a2]\n\t"
      "v_add_u32 %[x3], %[x3], %[a3]"
      : [x0] "+v"(x0), [x1] "+v"(x1), [x2] "+v"(x2), [x3] "+v"(x3), [y0] "+v"(y0), [y1] "+v"(y1), [y2] "+v"(y2),
        [y3] "+v"(y3), [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3), [c0] "=&s"(c0),
        [c1] "=&s"(c1), [c2] "=&s"(c2), [c3] "=&s"(c3)
      : [p0] "v"(p[0]), [p1] "v"(p[1]), [p2] "v"(p[2]), [p3] "v"(p[3]), [q] "s"(q));
}

// GS butterflies, first half: x <- u + v mod q (canonical), dd = u - v + q
// in (0, 2q) (the multiplicand of y's Shoup product).  v[k] is clobbered.
__device__ __forceinline__ void gs_pre4(uint32_t& u0, uint32_t& u1, uint32_t& u2, uint32_t& u3, uint32_t& v0,
                                        uint32_t& v1, uint32_t& v2, uint32_t& v3, uint32_t (&dd)[4], uint32_t q) {
  uint32_t s0, s1, s2, s3;
  uint64_t c0, c1, c2, c3;
  asm volatile(
      "v_sub_u32 %[d0], %[u0], %[v0]\n\t"
      "v_sub_u32 %[d1], %[u1], %[v1]\n\t"
      "v_sub_u32 %[d2], %[u2], %[v2]\n\t"
      "v_sub_u32 %[d3], %[u3], %[v3]\n\t"
      "v_add_u32 %[s0], %[u0], %[v0]\n\t"
      "v_add_u32 %[s1], %[u1], %[v1]\n\t"
      "v_add_u32 %[s2], %[u2], %[v2]\n\t"
      "v_add_u32 %[s3], %[u3], %[v3]\n\t"
      "v_add_u32 %[d0], %[q], %[d0]\n\t"
      "v_add_u32 %[d1], %[q], %[d1]\n\t"
      "v_add_u32 %[d2], %[q], %[d2]\n\t"
      "v_add_u32 %[d3], %[q], %[d3]\n\t"
      "v_sub_co_u32 %[v0], %[c0], %[s0], %[q]\n\t"
      "v_sub_co_u32 %[v1], %[c1], %[s1], %[q]\n\t"
      "v_sub_co_u32 %[v2], %[c2], %[s2], %[q]\n\t"
      "v_sub_co_u32 %[v3], %[c3], %[s3], %[q]\n\t"
      "v_cndmask_b32 %[u0], %[v0], %[s0], %[c0]\n\t"
      "v_cndmask_b32 %[u1], %[v1], %[s1], %[c1]\n\t"
      "v_cndmask_b32 %[u2], %[v2], %[s2], %[c2]\n\t"
      "v_cndmask_b32 %[u3], %[v3], %[s3], %[c3]"
      : [u0] "+v"(u0), [u1] "+v"(u1), [u2] "+v"(u2), [u3] "+v"(u3), [v0] "+v"(v0), [v1] "+v"(v1), [v2] "+v"(v2),
        [v3] "+v"(v3), [d0] "=&v"(dd[0]), [d1] "=&v"(dd[1]), [d2] "=&v"(dd[2]), [d3] "=&v"(dd[3]),
        [s0] "=&v"(s0), [s1] "=&v"(s1), [s2] "=&v"(s2), [s3] "=&v"(s3), [c0] "=&s"(c0), [c1] "=&s"(c1),
        [c2] "=&s"(c2), [c3] "=&s"(c3)
      : [q] "s"(q));
}

// y[k] <- csub(p[k]) (the Shoup product's final reduction into [0, q)).
__device__ __forceinline__ void csub4(uint32_t& y0, uint32_t& y1, uint32_t& y2, uint32_t& y3, const uint32_t (&p)[4],
                                      uint32_t q) {
  uint32_t a0, a1, a2, a3;
  uint64_t c0, c1, c2, c3;
  asm volatile(
      "v_sub_co_u32 %[a0], %[c0], %[p0], %[q]\n\t"
      "v_sub_co_u32 %[a1], %[c1], %[p1], %[q]\n\t"
      "v_sub_co_u32 %[a2], %[c2], %[p2], %[q]\n\t"
      "v_sub_co_u32 %[a3], %[c3], %[p3], %[q]\n\t"
      "v_cndmask_b32 %[y0], %[a0], %[p0], %[c0]\n\t"
      "v_cndmask_b32 %[y1], %[a1], %[p1], %[c1]\n\t"
      "v_cndmask_b32 %[y2], %[a2], %[p2], %[c2]\n\t"
      "v_cndmask_b32 %[y3], %[a3], %[p3], %[c3]"
      : [y0] "+v"(y0), [y1] "+v"(y1), [y2] "+v"(y2), [y3] "+v"(y3), [a0] "=&v"(a0), [a1] "=&v"(a1),
        [a2] "=&v"(a2), [a3] "=&v"(a3), [c0] "=&s"(c0), [c1] "=&s"(c1), [c2] "=&s"(c2), [c3] "=&s"(c3)
      : [p0] "v"(p[0]), [p1] "v"(p[1]), [p2] "v"(p[2]), [p3] "v"(p[3]), [q] "s"(q));
}

}  // namespace b4
}  // namespace rnt
