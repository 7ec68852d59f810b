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
template <class W>
__host__ __device__ __forceinline__ W csub(W x, W q) {
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

// Montgomery product a*b*2^-w mod q (a, b in [0, q)); qinv = q^-1 mod 2^w.
template <class W>
__host__ __device__ __forceinline__ W mont_mul(W a, W b, W q, W qinv);

template <>
__host__ __device__ __forceinline__ uint32_t mont_mul<uint32_t>(uint32_t a, uint32_t b, uint32_t q,
                                                                 uint32_t qinv) {
  uint64_t t = (uint64_t)a * b;
  uint32_t m = (uint32_t)t * qinv;
  uint32_t hi = (uint32_t)(t >> 32);
  uint32_t mh = mulhi(m, q);
  return sub_mod<uint32_t>(hi, mh, q);  // (t - m q) / 2^32, exact; hi, mh < q
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

// CT butterfly (forward, merged twist): (x, y) -> (x + w y, x - w y)
template <class W>
__device__ __forceinline__ void ct_bfly(W& x, W& y, W w, W wp, W q) {
  W t = shoup_mul<W>(y, w, wp, q);
  W u = x;
  x = add_mod<W>(u, t, q);
  y = sub_mod<W>(u, t, q);
}

// GS butterfly (inverse): (x, y) -> (x + y, (x - y) w)
template <class W>
__device__ __forceinline__ void gs_bfly(W& x, W& y, W w, W wp, W q) {
  W u = x, v = y;
  x = add_mod<W>(u, v, q);
  y = shoup_mul<W>(u - v + q, w, wp, q);  // u - v + q in (0, 2q): any x < 2^w is fine
}

}  // namespace rnt
