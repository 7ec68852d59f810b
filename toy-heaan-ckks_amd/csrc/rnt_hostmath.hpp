// rnt_hostmath.hpp -- host-side number theory for basis setup (one-time).
//
// Restates the reference's setup rules so the device tables hold exactly
// the residues the reference's NttTable would:
//   is_prime (deterministic Miller-Rabin)   src/math/primes.rs:67-93
//   is_ntt_friendly_prime                   src/math/primes.rs:125-131
//   get_first_prime_down                    src/math/primes.rs:199-219
//   generate_primes                         src/math/utils.rs:47-80
//   find_primitive_root (psi rule)          src/rings/backends/rns_ntt/basis.rs:217-237
//   mod_inverse                             basis.rs:198-210
#pragma once
#include <stdint.h>

namespace rnt {
namespace host {

typedef unsigned __int128 u128;

inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) { return (uint64_t)((u128)a * b % q); }

inline uint64_t powmod(uint64_t b, uint64_t e, uint64_t q) {
  uint64_t r = 1 % q;
  b %= q;
  while (e) {
    if (e & 1) r = mulmod(r, b, q);
    b = mulmod(b, b, q);
    e >>= 1;
  }
  return r;
}

// inverse of v mod m (gcd must be 1); returns 0 when not invertible.
inline uint64_t invmod(uint64_t v, uint64_t m) {
  __int128 r0 = m, r1 = v % m, s0 = 0, s1 = 1;
  while (r1 != 0) {
    __int128 qt = r0 / r1, t = r0 - qt * r1;
    r0 = r1;
    r1 = t;
    t = s0 - qt * s1;
    s0 = s1;
    s1 = t;
  }
  if (r0 != 1) return 0;
  __int128 x = s0 % (__int128)m;
  if (x < 0) x += m;
  return (uint64_t)x;
}

inline bool is_prime(uint64_t n) {
  static const uint64_t bases[12] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
  if (n < 2) return false;
  if (n < 4) return true;
  if ((n & 1) == 0) return false;
  uint64_t d = n - 1;
  unsigned r = 0;
  while ((d & 1) == 0) {
    d >>= 1;
    ++r;
  }
  for (uint64_t a : bases) {
    if (a >= n) continue;
    uint64_t x = powmod(a, d, n);
    if (x == 1 || x == n - 1) continue;
    bool composite = true;
    for (unsigned i = 1; i < r; ++i) {
      x = mulmod(x, x, n);
      if (x == n - 1) {
        composite = false;
        break;
      }
    }
    if (composite) return false;
  }
  return true;
}

inline bool is_ntt_friendly(uint64_t p, uint64_t n) {
  if (n == 0 || n > UINT64_MAX / 2) return false;
  return is_prime(p) && p % (2 * n) == 1;
}

// largest prime p < bound with p = 1 mod 2n, or 0
inline uint64_t prime_down(uint64_t bound, uint64_t n) {
  if (n == 0 || bound <= 2) return 0;
  const uint64_t step = 2 * n;
  uint64_t c = bound - 1;
  c -= (c % step + step - 1) % step;  // largest value <= bound-1 that is 1 mod step
  for (;;) {
    if (c <= 2) return 0;
    if (is_prime(c)) return c;
    if (c < step) return 0;
    c -= step;
  }
}

// generate_primes: 0 on success, -1 when the reference would panic.
inline int generate_primes(uint32_t bits, uint64_t count, uint64_t degree, uint64_t* out) {
  if (bits < 4 || bits > 63 || count == 0 || degree == 0) return -1;
  const uint64_t upper = (1ull << bits) - 1, lower = 1ull << (bits - 1);
  uint64_t cur = prime_down(upper + 1, degree);
  if (cur == 0) return -1;
  uint64_t k = 0;
  while (k < count) {
    if (cur < lower) break;
    out[k++] = cur;
    const uint64_t nx = prime_down(cur, degree);
    if (nx == 0) break;
    cur = nx;
  }
  return k == count ? 0 : -1;
}

// psi = c^((q-1)/2n) for the smallest c >= 2 whose power has order exactly
// 2n (2n is a power of two, so "order exactly 2n" == "psi^n != 1").
inline uint64_t find_psi(uint64_t q, uint64_t n) {
  const uint64_t order = 2 * n;
  const uint64_t e = (q - 1) / order;
  for (uint64_t c = 2; c < q; ++c) {
    const uint64_t r = powmod(c, e, q);
    if (r == 1) continue;
    if (powmod(r, order / 2, q) == 1) continue;
    return r;
  }
  return 0;
}

inline uint64_t brv(uint64_t v, unsigned bits) {
  uint64_t r = 0;
  for (unsigned i = 0; i < bits; ++i) {
    r = (r << 1) | (v & 1);
    v >>= 1;
  }
  return r;
}

// Shoup companion floor(w * 2^wbits / q), wbits in {32, 64}
inline uint64_t shoup_companion(uint64_t w, uint64_t q, unsigned wbits) {
  if (wbits == 32) return (uint64_t)((((u128)w) << 32) / q);
  return (uint64_t)((((u128)w) << 64) / q);
}

// q^-1 mod 2^wbits (q odd)
inline uint64_t neg_free_qinv(uint64_t q, unsigned wbits) {
  uint64_t x = q;
  for (int i = 0; i < 6; ++i) x *= 2 - q * x;
  return wbits == 32 ? (x & 0xffffffffull) : x;
}

}  // namespace host
}  // namespace rnt
