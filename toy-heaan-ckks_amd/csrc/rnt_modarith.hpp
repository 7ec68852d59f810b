// rnt_modarith.hpp -- exact modular arithmetic for the RNS-NTT kernels.
//
// Two word widths share one code path:
//   W = uint32_t for primes q < 2^31 (every BASELINE config: 31-bit primes),
//   W = uint64_t for primes q < 2^63 (the reference's 40/61/62-bit tests).
// All helpers return the canonical residue in [0, q), so every result is
// bit-identical to the reference's `(a as u128 * b as u128) % q`
// (poly.rs:651-653) regardless of the reduction algorithm.
//
// The q < 2^(w-1) bound is what makes the branch-free min() reductions valid:
// a + b < 2q < 2^w never wraps, and for x < q, x - q wraps to >= 2^w - q > x.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rnt_internal.hpp"

namespace rnt {

__host__ __device__ __forceinline__ uint32_t mulhi(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umulhi(a, b);
#else
  return (uint32_t)(((uint64_t)a * b) >> 32);
#endif
}
__host__ __device__ __forceinline__ uint64_t mulhi(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

// x in [0, 2q) -> [0, q)
//
// On the device the 32-bit form is a borrow-select: v_sub_co_u32 (borrow
// into VCC / an SGPR pair) + v_cndmask_b32, two full-rate instructions
// (tools/oprate2.hip: 2.1 cycles each per wave64 on one SIMD), where the
// min(x, x - q) form costs v_sub (2.2) + v_min_u32 (4.1, half rate).
template <class W>
__host__ __device__ __forceinline__ W csub(W x, W q) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (sizeof(W) == 4) {
    W y;
    const bool borrow = __builtin_sub_overflow(x, q, &y);
    return borrow ? x : y;
  }
#endif
  W y = x - q;
  return y < x ? y : x;  // min(x, x - q) as unsigned
}

template <class W>
__host__ __device__ __forceinline__ W add_mod(W a, W b, W q) {
  return csub<W>(a + b, q);
}

// a, b in [0, q) -> a - b mod q
template <class W>
__host__ __device__ __forceinline__ W sub_mod(W a, W b, W q) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (sizeof(W) == 4) {
    W d;
    const bool borrow = __builtin_sub_overflow(a, b, &d);
    return borrow ? d + q : d;
  }
#endif
  W d = a - b;
  W e = d + q;
  return e < d ? e : d;  // min(d, d + q)
}

// Shoup multiplication by a constant w with wp = floor(w * 2^w / q):
// x * w mod q for any x < 2^w.  (Shoup 2009; Harvey 2014, Alg. 2)
template <class W>
__host__ __device__ __forceinline__ W shoup_mul(W x, W w, W wp, W q) {
  W qh = mulhi(x, wp);
  W r = x * w - qh * q;  // in [0, 2q), computed mod 2^w
  return csub<W>(r, q);
}

// Modulus bundle passed to the butterflies.  nq = 2^w - q (so q-multiples
// can be subtracted by a multiply-add).
template <class W>
struct Mod {
  W q;
  W nq;
};

// gfx950 VALU rates measured by tools/oprate.hip (cycles per wave64
// instruction per SIMD): add/sub/xor/and ~2; min/max, v_mul_lo/hi_u32,
// v_mul_u32_u24, VOP3 shifts-adds and v_mad_u64_u32 ~4.  v_mad_u64_u32
// yields a full 64-bit a*b+c for the price of one 32-bit multiply, so the
// 32-bit path builds its products from it.  The instruction is left to the
// compiler (it writes an SGPR carry, whose wait states hipcc only inserts
// for its own instructions); an empty asm on the 64-bit value keeps the
// compiler from narrowing it to mul_lo + add.
__device__ __forceinline__ uint64_t keep64(uint64_t x) {
  asm("" : "+v"(x));
  return x;
}
__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
  return keep64((uint64_t)a * b + c);
}
__device__ __forceinline__ uint64_t mul64(uint32_t a, uint32_t b) {
  return keep64((uint64_t)a * b);
}

// Shoup product, result in [0, 2q) (not reduced):
//   r = x*w - floor(x*w'/2^w)*q  (mod 2^w)
__device__ __forceinline__ uint32_t shoup_lazy(uint32_t x, uint32_t w, uint32_t wp,
                                               const Mod<uint32_t>& m) {
  const uint32_t qh = mulhi(x, wp);
  return (uint32_t)mad64(qh, m.nq, mul64(x, w));  // low word of x*w + qh*(2^32 - q)
}
__device__ __forceinline__ uint64_t shoup_lazy(uint64_t x, uint64_t w, uint64_t wp,
                                               const Mod<uint64_t>& m) {
  const uint64_t qh = mulhi(x, wp);
  return x * w - qh * m.q;
}
template <class W>
__device__ __forceinline__ W shoup_mul(W x, W w, W wp, const Mod<W>& m) {
  return csub<W>(shoup_lazy(x, w, wp, m), m.q);
}

// Montgomery product a*b*2^-w mod q (a, b in [0, q)); qinv = q^-1 mod 2^w.
template <class W>
__host__ __device__ __forceinline__ W mont_mul(W a, W b, W q, W qinv);

template <>
__host__ __device__ __forceinline__ uint32_t mont_mul<uint32_t>(uint32_t a, uint32_t b, uint32_t q,
                                                                 uint32_t qinv) {
#if defined(__HIP_DEVICE_COMPILE__)
  // m = -t q^-1 mod 2^32, so t + m q is a multiple of 2^32 and
  // (t + m q) / 2^32 < q^2/2^32 + q < 2q; 3 half-rate ops + csub.
  const uint64_t t = mul64(a, b);
  const uint32_t m = (uint32_t)t * (0u - qinv);
  return csub<uint32_t>((uint32_t)(mad64(m, q, t) >> 32), q);
#else
  uint64_t t = (uint64_t)a * b;
  uint32_t m = (uint32_t)t * qinv;
  uint32_t hi = (uint32_t)(t >> 32);
  uint32_t mh = mulhi(m, q);
  return sub_mod<uint32_t>(hi, mh, q);  // (t - m q) / 2^32, exact; hi, mh < q
#endif
}

// The same product with nqinv = -q^-1 mod 2^32 supplied by the caller.
// hipcc rewrites t * (0 - qinv) as 0 - t * qinv, a v_sub per product; a
// caller that hoists nqinv out of its loop behind an opaque copy keeps the
// single multiply.
__device__ __forceinline__ uint32_t mont_mul_nq(uint32_t a, uint32_t b, uint32_t q, uint32_t nqinv) {
  const uint64_t t = mul64(a, b);
  const uint32_t m = (uint32_t)t * nqinv;
  return csub<uint32_t>((uint32_t)(mad64(m, q, t) >> 32), q);
}

template <>
__host__ __device__ __forceinline__ uint64_t mont_mul<uint64_t>(uint64_t a, uint64_t b, uint64_t q,
                                                                 uint64_t qinv) {
  uint64_t lo = a * b;
  uint64_t hi = mulhi(a, b);
  uint64_t m = lo * qinv;
  uint64_t mh = mulhi(m, q);
  return sub_mod<uint64_t>(hi, mh, q);
}

// CT butterfly (forward, merged twist): (x, y) -> (x + w y, x - w y).
// x must be reduced; y may be anything < 2^w (it only feeds Shoup).
template <class W>
__device__ __forceinline__ void ct_bfly(W& x, W& y, W w, W wp, const Mod<W>& m) {
  const W t = shoup_mul<W>(y, w, wp, m);
  const W u = x;
  x = add_mod<W>(u, t, m.q);
  y = sub_mod<W>(u, t, m.q);
}

// Same butterfly with outputs left in [0, 2q]: used when both outputs next
// feed Shoup as multiplicands (the "y" of the following stage), so their
// reductions are dead work.
template <class W>
__device__ __forceinline__ void ct_bfly_lazy(W& x, W& y, W w, W wp, const Mod<W>& m) {
  const W t = shoup_mul<W>(y, w, wp, m);
  const W u = x;
  x = u + t;
  y = u + (m.q - t);
}

// GS butterfly (inverse): (x, y) -> (x + y, (x - y) w)
template <class W>
__device__ __forceinline__ void gs_bfly(W& x, W& y, W w, W wp, const Mod<W>& m) {
  const W u = x, v = y;
  x = add_mod<W>(u, v, m.q);
  y = shoup_mul<W>(u - v + m.q, w, wp, m);  // u - v + q in (0, 2q): any x < 2^w is fine
}

// ---- 30-bit moduli: Harvey's lazy butterflies -----------------------------
// With q < 2^30, 4q < 2^32 leaves two bits of headroom (31-bit primes leave
// one), so the product path keeps values unreduced (Harvey 2014, Alg. 4/5):
// forward CT values live in [0, 4q), inverse GS values in [0, 2q), and only
// the one reduction that keeps a sum below 4q remains per butterfly.  The
// reference's own examples use 30-bit bases (rotation_demo.rs,
// rotation_stress.rs).  Outputs at the product's end are canonical again.
struct Mod30 {
  uint32_t q;   // modulus, < 2^30
  uint32_t nq;  // 2^32 - q
  uint32_t q2;  // 2q
};

// CT: x in [0, 4q), any y < 2^32 -> both outputs in [0, 4q).
__device__ __forceinline__ void ct_bfly(uint32_t& x, uint32_t& y, uint32_t w, uint32_t wp,
                                        const Mod30& m) {
  const uint32_t t = shoup_lazy(y, w, wp, Mod<uint32_t>{m.q, m.nq});  // [0, 2q)
  const uint32_t u = csub<uint32_t>(x, m.q2);                          // [0, 2q)
  x = u + t;
  y = u + (m.q2 - t);
}
__device__ __forceinline__ void ct_bfly_lazy(uint32_t& x, uint32_t& y, uint32_t w, uint32_t wp,
                                             const Mod30& m) {
  ct_bfly(x, y, w, wp, m);
}
// GS: u, v in [0, 2q) -> (u + v) in [0, 2q), (u - v) w in [0, 2q).
__device__ __forceinline__ void gs_bfly(uint32_t& x, uint32_t& y, uint32_t w, uint32_t wp,
                                        const Mod30& m) {
  const uint32_t u = x, v = y;
  x = csub<uint32_t>(u + v, m.q2);
  y = shoup_lazy(u - v + m.q2, w, wp, Mod<uint32_t>{m.q, m.nq});
}
// Canonical Shoup product of any x < 2^32 (the inverse's folded last stage).
__device__ __forceinline__ uint32_t shoup_mul(uint32_t x, uint32_t w, uint32_t wp, const Mod30& m) {
  return csub<uint32_t>(shoup_lazy(x, w, wp, Mod<uint32_t>{m.q, m.nq}), m.q);
}
// ---- 62-bit moduli in 64-bit words: the same Harvey-lazy butterflies -------
// With q < 2^62, 4q < 2^64 gives the u64 path the two bits of headroom the
// 30-bit u32 bases have, so the product path runs the same lazy ranges
// (forward CT values in [0, 4q), inverse GS values in [0, 2q)): one 64-bit
// conditional subtraction per CT butterfly instead of three (the Shoup
// product's, add_mod's, sub_mod's), and one per GS butterfly instead of two.
// A 64-bit reduction is a two-word subtract, a 64-bit compare and two
// selects, so each one saved is five VALU ops on the VALU-bound u64 path
// ("The u64 path").  The reference's 40-, 61- and 62-bit
// primes all qualify; a 63-bit prime keeps the canonical kernels.
struct Mod62 {
  uint64_t q;   // modulus, < 2^62
  uint64_t q2;  // 2q
};
__device__ __forceinline__ uint64_t shoup_lazy(uint64_t x, uint64_t w, uint64_t wp, const Mod62& m) {
  return x * w - mulhi(x, wp) * m.q;  // [0, 2q) for any x < 2^64
}
__device__ __forceinline__ void ct_bfly(uint64_t& x, uint64_t& y, uint64_t w, uint64_t wp, const Mod62& m) {
  const uint64_t t = shoup_lazy(y, w, wp, m);                          // [0, 2q)
  const uint64_t u = csub<uint64_t>(x, m.q2);                          // [0, 2q)
  x = u + t;
  y = u + (m.q2 - t);
}
__device__ __forceinline__ void ct_bfly_lazy(uint64_t& x, uint64_t& y, uint64_t w, uint64_t wp,
                                             const Mod62& m) {
  ct_bfly(x, y, w, wp, m);
}
__device__ __forceinline__ void gs_bfly(uint64_t& x, uint64_t& y, uint64_t w, uint64_t wp, const Mod62& m) {
  const uint64_t u = x, v = y;
  x = csub<uint64_t>(u + v, m.q2);
  y = shoup_lazy(u - v + m.q2, w, wp, m);
}
__device__ __forceinline__ uint64_t shoup_mul(uint64_t x, uint64_t w, uint64_t wp, const Mod62& m) {
  return csub<uint64_t>(shoup_lazy(x, w, wp, m), m.q);
}

// What the GS difference u - v is biased by to stay non-negative.
template <class W>
__device__ __forceinline__ W gs_bias(const Mod<W>& m) { return m.q; }   // u, v in [0, q)
__device__ __forceinline__ uint32_t gs_bias(const Mod30& m) { return m.q2; }  // u, v in [0, 2q)
__device__ __forceinline__ uint64_t gs_bias(const Mod62& m) { return m.q2; }  // u, v in [0, 2q)

// m mod q for a 64-bit magnitude m, canonical.  The 32-bit path splits m
// into halves, hi * (2^32 mod q) + lo, each reduced by a Shoup product, so
// there is no 64-bit division (a long software sequence on the device); the
// 64-bit path uses %.
template <class W>
__device__ __forceinline__ W mag_mod(uint64_t m, const LimbConst<W>& lc) {
  if constexpr (sizeof(W) == 4) {
    const uint32_t a = shoup_mul<uint32_t>((uint32_t)(m >> 32), lc.rmod, lc.rmod_p, lc.q);
    const uint32_t b = shoup_mul<uint32_t>((uint32_t)m, 1u, lc.one_p, lc.q);
    return add_mod<uint32_t>(a, b, lc.q);
  } else {
    return (W)(m % (uint64_t)lc.q);
  }
}

// c.rem_euclid(q) (from_coeffs, poly.rs:55-61), |c| <= 2^63.
template <class W>
__device__ __forceinline__ W rem_euclid(int64_t c, const LimbConst<W>& lc) {
  if (c >= 0) return mag_mod<W>((uint64_t)c, lc);
  const W r = mag_mod<W>((uint64_t)(-(c + 1)) + 1u, lc);  // |c| without overflow
  return r == 0 ? (W)0 : (W)(lc.q - r);
}

}  // namespace rnt
