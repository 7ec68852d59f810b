/*
 * oracle.c -- CPU restatement of the reference RNS-NTT path.
 * TEST INFRASTRUCTURE ONLY (see oracle.h header).  Citations are
 * path:line in the reference repository (oiwn/toy-heaan-ckks).
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef unsigned __int128 u128;
typedef __int128 i128;

/* ------------------------------------------------------------------ */
/* scalar helpers                                                      */
/* ------------------------------------------------------------------ */

/* poly.rs:651-653 */
uint64_t or_mul_mod(uint64_t a, uint64_t b, uint64_t q) {
  return (uint64_t)(((u128)a * (u128)b) % (u128)q);
}
/* poly.rs:642-645 (a+b computed in u64: safe because q < 2^63) */
uint64_t or_add_mod(uint64_t a, uint64_t b, uint64_t q) {
  uint64_t s = a + b;
  return s >= q ? s - q : s;
}
/* poly.rs:647-649 */
uint64_t or_sub_mod(uint64_t a, uint64_t b, uint64_t q) {
  return a >= b ? a - b : a + q - b;
}
/* poly.rs:629-640 / basis.rs:185-196 */
uint64_t or_mod_pow(uint64_t base, uint64_t e, uint64_t q) {
  uint64_t r = 1;
  base %= q;
  while (e > 0) {
    if (e & 1) r = (uint64_t)(((u128)r * base) % q);
    base = (uint64_t)(((u128)base * base) % q);
    e >>= 1;
  }
  return r;
}
/* basis.rs:198-210: i128 extended GCD (recursive in the reference; the
 * iterative form computes the same Bezout coefficient). */
uint64_t or_mod_inverse(uint64_t v, uint64_t m) {
  i128 a = (i128)v, b = (i128)m;
  /* extended_gcd(a, b) returning x with a*x + b*y = gcd */
  i128 old_r = a, r = b, old_s = 1, s = 0;
  while (r != 0) {
    i128 qt = old_r / r;
    i128 t = old_r - qt * r; old_r = r; r = t;
    t = old_s - qt * s; old_s = s; s = t;
  }
  if (old_r != 1 && old_r != -1) return 0; /* reference: assert gcd == 1 */
  if (old_r == -1) old_s = -old_s;
  i128 mm = (i128)m;
  return (uint64_t)(((old_s % mm) + mm) % mm);
}

/* ------------------------------------------------------------------ */
/* primes: src/math/primes.rs                                           */
/* ------------------------------------------------------------------ */

static const uint64_t MR_BASES[12] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};

/* primes.rs:67-93 (deterministic Miller-Rabin) */
int or_is_prime(uint64_t n) {
  if (n == 0 || n == 1) return 0;
  if (n == 2 || n == 3) return 1;
  if ((n & 1) == 0) return 0;
  uint64_t d = n - 1;
  uint32_t r = 0;
  while ((d & 1) == 0) { d >>= 1; r++; } /* decompose, primes.rs:48-57 */
  for (int bi = 0; bi < 12; bi++) {
    uint64_t a = MR_BASES[bi];
    if (a >= n) continue;
    uint64_t x = or_mod_pow(a, d, n);
    if (x == 1 || x == n - 1) continue;
    int witness = 1;
    for (uint32_t i = 1; i < r; i++) {
      x = or_mul_mod(x, x, n);
      if (x == n - 1) { witness = 0; break; }
    }
    if (witness) return 0;
  }
  return 1;
}

/* primes.rs:96-114 */
int or_is_prime_reference(uint64_t n) {
  if (n < 2) return 0;
  if (n == 2 || n == 3) return 1;
  if (n % 2 == 0 || n % 3 == 0) return 0;
  for (uint64_t i = 5;; i += 6) {
    u128 sq = (u128)i * i;
    if (sq > n) break;
    if (n % i == 0 || n % (i + 2) == 0) return 0;
  }
  return 1;
}

/* primes.rs:125-131 */
int or_is_ntt_friendly_prime(uint64_t p, uint64_t n) {
  if (n == 0 || n > UINT64_MAX / 2) return 0; /* reference panics */
  uint64_t m = n * 2;
  return or_is_prime(p) && p % m == 1;
}

/* primes.rs:134-148 */
static uint64_t snap_up(uint64_t value, uint64_t modulus) {
  uint64_t rem = value % modulus;
  if (rem == 1) return value;
  uint64_t delta = (modulus + 1 - rem) % modulus;
  return value + delta;
}
/* primes.rs:151-161 */
static uint64_t snap_down(uint64_t value, uint64_t modulus) {
  uint64_t rem = value % modulus;
  uint64_t delta = (rem + modulus - 1) % modulus;
  return value - delta;
}

/* primes.rs:171-188 */
uint64_t or_get_first_prime_up(uint32_t logq, uint64_t n) {
  if (logq >= 64 || n == 0) return 0;
  uint64_t step = n * 2;
  uint64_t c = snap_up((1ULL << logq) + 1, step);
  for (;;) {
    if (or_is_prime(c)) return c;
    c += step;
  }
}

/* primes.rs:199-219 */
uint64_t or_get_first_prime_down(uint64_t bound, uint64_t n) {
  if (n == 0) return 0;
  if (bound <= 2) return 0;
  uint64_t step = n * 2;
  uint64_t c = snap_down(bound - 1, step); /* saturating_sub(1) */
  for (;;) {
    if (c <= 2) return 0;
    if (or_is_prime(c)) return c;
    if (c < step) return 0; /* checked_sub -> None */
    c -= step;
  }
}

/* utils.rs:47-80 */
size_t or_generate_primes(uint32_t bit_size, size_t count, uint64_t degree,
                          uint64_t* out) {
  if (bit_size < 4 || bit_size > 63 || count == 0 || degree == 0) return 0;
  uint64_t upper = (1ULL << bit_size) - 1;
  uint64_t lower = 1ULL << (bit_size - 1);
  uint64_t cursor = or_get_first_prime_down(upper + 1, degree);
  if (cursor == 0) return 0;
  size_t k = 0;
  while (k < count) {
    if (cursor < lower) break;
    out[k++] = cursor;
    uint64_t next = or_get_first_prime_down(cursor, degree);
    if (next == 0) break;
    cursor = next;
  }
  return k == count ? k : 0;
}

/* ------------------------------------------------------------------ */
/* tables: basis.rs                                                    */
/* ------------------------------------------------------------------ */

/* basis.rs:217-237 with distinct_prime_factors (basis.rs:239-255) */
uint64_t or_find_primitive_root(uint64_t modulus, uint64_t order) {
  uint64_t exponent = (modulus - 1) / order;
  uint64_t factors[64];
  int nf = 0;
  uint64_t v = order;
  for (uint64_t d = 2; d * d <= v; d++) {
    if (v % d == 0) {
      factors[nf++] = d;
      while (v % d == 0) v /= d;
    }
  }
  if (v > 1) factors[nf++] = v;
  for (uint64_t cand = 2; cand < modulus; cand++) {
    uint64_t root = or_mod_pow(cand, exponent, modulus);
    if (root == 1) continue;
    int ok = 1;
    for (int f = 0; f < nf; f++)
      if (or_mod_pow(root, order / factors[f], modulus) == 1) { ok = 0; break; }
    if (ok) return root;
  }
  return 0;
}

static int is_pow2(size_t n) { return n != 0 && (n & (n - 1)) == 0; }

/* basis.rs:20-84 */
int or_table_new(or_table* t, size_t n, uint64_t modulus) {
  memset(t, 0, sizeof(*t));
  if (!is_pow2(n)) return OR_INVALID_DEGREE;
  if (!or_is_ntt_friendly_prime(modulus, n)) return OR_NON_NTT_FRIENDLY;
  uint64_t psi = or_find_primitive_root(modulus, 2 * n);
  uint64_t omega = or_mod_pow(psi, 2, modulus);
  uint64_t omega_inv = or_mod_inverse(omega, modulus);
  uint64_t psi_inv = or_mod_inverse(psi, modulus);
  t->modulus = modulus;
  t->psi = psi;
  t->forward_roots = (uint64_t*)malloc(n * sizeof(uint64_t));
  t->inverse_roots = (uint64_t*)malloc(n * sizeof(uint64_t));
  t->twist_factors = (uint64_t*)malloc(n * sizeof(uint64_t));
  t->untwist_factors = (uint64_t*)malloc(n * sizeof(uint64_t));
  /* The reference calls mod_pow per index (basis.rs:50-73); a running
   * product yields the identical residues. */
  uint64_t f = 1, iv = 1, tw = 1, ut = 1;
  for (size_t i = 0; i < n; i++) {
    t->forward_roots[i] = f;
    t->inverse_roots[i] = iv;
    t->twist_factors[i] = tw;
    t->untwist_factors[i] = ut;
    f = or_mul_mod(f, omega, modulus);
    iv = or_mul_mod(iv, omega_inv, modulus);
    tw = or_mul_mod(tw, psi, modulus);
    ut = or_mul_mod(ut, psi_inv, modulus);
  }
  t->n_inv = or_mod_inverse((uint64_t)n % modulus, modulus);
  return OR_OK;
}

void or_table_free(or_table* t) {
  free(t->forward_roots);
  free(t->inverse_roots);
  free(t->twist_factors);
  free(t->untwist_factors);
  memset(t, 0, sizeof(*t));
}

/* basis.rs:97-106 */
int or_basis_new(or_basis* b, size_t n, const uint64_t* moduli, size_t count) {
  memset(b, 0, sizeof(*b));
  if (count == 0) return OR_EMPTY_BASIS;
  b->n = n;
  b->channels = count;
  b->moduli = (uint64_t*)malloc(count * sizeof(uint64_t));
  b->tables = (or_table*)calloc(count, sizeof(or_table));
  b->owns_tables = 1;
  memcpy(b->moduli, moduli, count * sizeof(uint64_t));
  for (size_t i = 0; i < count; i++) {
    int rc = or_table_new(&b->tables[i], n, moduli[i]);
    if (rc != OR_OK) {
      b->channels = i; /* free the ones built so far */
      or_basis_free(b);
      return rc;
    }
  }
  return OR_OK;
}

void or_basis_free(or_basis* b) {
  if (b->owns_tables && b->tables)
    for (size_t i = 0; i < b->channels; i++) or_table_free(&b->tables[i]);
  if (b->owns_tables) free(b->tables);
  free(b->moduli);
  memset(b, 0, sizeof(*b));
}

/* basis.rs:121-134 */
int or_basis_drop_last(const or_basis* b, size_t drop_count, or_basis* out) {
  memset(out, 0, sizeof(*out));
  if (drop_count >= b->channels) return OR_INVALID_MOD_DROP;
  size_t keep = b->channels - drop_count;
  out->n = b->n;
  out->channels = keep;
  out->moduli = (uint64_t*)malloc(keep * sizeof(uint64_t));
  memcpy(out->moduli, b->moduli, keep * sizeof(uint64_t));
  out->tables = b->tables;
  out->owns_tables = 0;
  return OR_OK;
}

/* basis.rs:140-145 */
uint32_t or_basis_total_bits(const or_basis* b) {
  uint32_t s = 0;
  for (size_t i = 0; i < b->channels; i++) s += 63 - (uint32_t)__builtin_clzll(b->moduli[i]);
  return s;
}

/* basis.rs:158-180 */
int64_t or_reconstruct_centered(const or_basis* b, const uint64_t* r) {
  u128 q = 1;
  for (size_t i = 0; i < b->channels; i++) q *= (u128)b->moduli[i];
  u128 acc = 0;
  for (size_t i = 0; i < b->channels; i++) {
    uint64_t m = b->moduli[i];
    u128 qi = q / m;
    uint64_t qi_inv = or_mod_inverse((uint64_t)(qi % m), m);
    u128 s = ((u128)r[i] * qi_inv) % m;
    u128 term = s * qi % q;
    acc = (acc + term) % q;
  }
  if (acc > q / 2) return (int64_t)((i128)acc - (i128)q);
  return (int64_t)acc;
}

/* ------------------------------------------------------------------ */
/* polynomial ops: poly.rs                                             */
/* ------------------------------------------------------------------ */

/* poly.rs:49-67 */
void or_from_coeffs(const or_basis* b, const int64_t* coeffs, uint64_t* out) {
  for (size_t ch = 0; ch < b->channels; ch++) {
    i128 q = (i128)b->moduli[ch];
    for (size_t i = 0; i < b->n; i++) {
      i128 v = (i128)coeffs[i] % q;
      if (v < 0) v += q;
      out[ch * b->n + i] = (uint64_t)v;
    }
  }
}

/* poly.rs:73-99: count check then reducedness scan */
int or_from_channels_check(const or_basis* b, const uint64_t* ch, size_t count) {
  if (count != b->channels) return OR_CHANNEL_COUNT_MISMATCH;
  for (size_t c = 0; c < count; c++)
    for (size_t i = 0; i < b->n; i++)
      if (ch[c * b->n + i] >= b->moduli[c]) return OR_NON_REDUCED;
  return OR_OK;
}

static size_t reverse_bits(size_t v, unsigned bits) {
  size_t r = 0;
  for (unsigned i = 0; i < bits; i++) { r = (r << 1) | (v & 1); v >>= 1; }
  return r;
}

/* poly.rs:617-625 */
static void bit_reverse_permute(uint64_t* v, size_t n) {
  unsigned bits = (unsigned)__builtin_ctzll(n);
  for (size_t i = 0; i < n; i++) {
    size_t j = reverse_bits(i, bits);
    if (i < j) { uint64_t t = v[i]; v[i] = v[j]; v[j] = t; }
  }
}

/* poly.rs:593-615 */
static void cooley_tukey_ntt(uint64_t* values, const uint64_t* roots, size_t n,
                             uint64_t q) {
  for (size_t len = 2; len <= n; len *= 2) {
    size_t half = len / 2, step = n / len;
    for (size_t start = 0; start < n; start += len)
      for (size_t off = 0; off < half; off++) {
        size_t l = start + off, r = l + half;
        uint64_t tw = roots[off * step];
        uint64_t t = or_mul_mod(values[r], tw, q);
        uint64_t u = values[l];
        values[l] = or_add_mod(u, t, q);
        values[r] = or_sub_mod(u, t, q);
      }
  }
}

/* poly.rs:574-580 */
void or_forward_ntt(const or_table* t, size_t n, uint64_t* v) {
  bit_reverse_permute(v, n);
  cooley_tukey_ntt(v, t->forward_roots, n, t->modulus);
}
/* poly.rs:582-591 */
void or_inverse_ntt(const or_table* t, size_t n, uint64_t* v) {
  bit_reverse_permute(v, n);
  cooley_tukey_ntt(v, t->inverse_roots, n, t->modulus);
  for (size_t i = 0; i < n; i++) v[i] = or_mul_mod(v[i], t->n_inv, t->modulus);
}

/* one channel of to_ntt_domain (poly.rs:140-146) */
static void channel_to_ntt(const or_table* t, size_t n, uint64_t* v) {
  for (size_t j = 0; j < n; j++) v[j] = or_mul_mod(v[j], t->twist_factors[j], t->modulus);
  or_forward_ntt(t, n, v);
}
/* one channel of to_coeff_domain (poly.rs:158-164) */
static void channel_to_coeff(const or_table* t, size_t n, uint64_t* v) {
  or_inverse_ntt(t, n, v);
  for (size_t j = 0; j < n; j++) v[j] = or_mul_mod(v[j], t->untwist_factors[j], t->modulus);
}

/* poly.rs:136-148 */
void or_to_ntt_domain(const or_basis* b, uint64_t* poly) {
  for (size_t ch = 0; ch < b->channels; ch++) channel_to_ntt(&b->tables[ch], b->n, poly + ch * b->n);
}
/* poly.rs:154-166 */
void or_to_coeff_domain(const or_basis* b, uint64_t* poly) {
  for (size_t ch = 0; ch < b->channels; ch++) channel_to_coeff(&b->tables[ch], b->n, poly + ch * b->n);
}

/* poly.rs:404-427 */
void or_to_coeffs(const or_basis* b, const uint64_t* poly, int in_ntt, int64_t* out) {
  size_t n = b->n, L = b->channels;
  uint64_t* tmp = (uint64_t*)malloc(L * n * sizeof(uint64_t));
  memcpy(tmp, poly, L * n * sizeof(uint64_t));
  if (in_ntt) or_to_coeff_domain(b, tmp);
  uint64_t* res = (uint64_t*)malloc(L * sizeof(uint64_t));
  for (size_t i = 0; i < n; i++) {
    for (size_t ch = 0; ch < L; ch++) res[ch] = tmp[ch * n + i];
    out[i] = or_reconstruct_centered(b, res);
  }
  free(res);
  free(tmp);
}

/* The per-channel body of the coefficient-domain MulAssign branch
 * (poly.rs:310-328): twist+fwd(self), twist+fwd(clone of rhs), pointwise,
 * inv+untwist(self). */
static void channel_mul_coeff(const or_table* t, size_t n, uint64_t* a,
                              const uint64_t* rhs, uint64_t* scratch) {
  uint64_t q = t->modulus;
  channel_to_ntt(t, n, a);
  memcpy(scratch, rhs, n * sizeof(uint64_t)); /* rhs.channels.clone() :312 */
  channel_to_ntt(t, n, scratch);
  for (size_t j = 0; j < n; j++) a[j] = or_mul_mod(a[j], scratch[j], q);
  channel_to_coeff(t, n, a);
}

/* poly.rs:277-331 */
int or_mul_assign(const or_basis* b, uint64_t* a, int a_ntt, const uint64_t* rhs, int rhs_ntt) {
  if (a_ntt != rhs_ntt) return OR_DOMAIN_MISMATCH;
  size_t n = b->n;
  if (a_ntt) {
    for (size_t ch = 0; ch < b->channels; ch++) {
      uint64_t q = b->moduli[ch];
      for (size_t j = 0; j < n; j++) a[ch * n + j] = or_mul_mod(a[ch * n + j], rhs[ch * n + j], q);
    }
    return OR_OK;
  }
  uint64_t* scratch = (uint64_t*)malloc(n * sizeof(uint64_t));
  for (size_t ch = 0; ch < b->channels; ch++)
    channel_mul_coeff(&b->tables[ch], n, a + ch * n, rhs + ch * n, scratch);
  free(scratch);
  return OR_OK;
}

/* poly.rs:339-367 */
void or_mul_assign_naive(const or_basis* b, uint64_t* a, const uint64_t* rhs) {
  size_t n = b->n;
  uint64_t* result = (uint64_t*)malloc(n * sizeof(uint64_t));
  for (size_t ch = 0; ch < b->channels; ch++) {
    uint64_t q = b->moduli[ch];
    const uint64_t* l = a + ch * n;
    const uint64_t* r = rhs + ch * n;
    memset(result, 0, n * sizeof(uint64_t));
    for (size_t i = 0; i < n; i++)
      for (size_t j = 0; j < n; j++) {
        uint64_t prod = or_mul_mod(l[i], r[j], q);
        if (i + j < n) result[i + j] = or_add_mod(result[i + j], prod, q);
        else result[i + j - n] = or_sub_mod(result[i + j - n], prod, q);
      }
    memcpy(a + ch * n, result, n * sizeof(uint64_t));
  }
  free(result);
}

/* poly.rs:254-275 */
int or_add_assign(const or_basis* b, uint64_t* a, int a_ntt, const uint64_t* rhs, int rhs_ntt) {
  if (a_ntt != rhs_ntt) return OR_DOMAIN_MISMATCH;
  size_t n = b->n;
  for (size_t ch = 0; ch < b->channels; ch++) {
    uint64_t q = b->moduli[ch];
    for (size_t j = 0; j < n; j++) a[ch * n + j] = or_add_mod(a[ch * n + j], rhs[ch * n + j], q);
  }
  return OR_OK;
}

/* poly.rs:370-385 */
void or_neg(const or_basis* b, uint64_t* a) {
  size_t n = b->n;
  for (size_t ch = 0; ch < b->channels; ch++) {
    uint64_t q = b->moduli[ch];
    for (size_t j = 0; j < n; j++) {
      uint64_t c = a[ch * n + j];
      if (c != 0) a[ch * n + j] = q - c;
    }
  }
}

/* poly.rs:187-228 */
int or_rescale(const or_basis* b, const uint64_t* in, int in_ntt, uint64_t* out) {
  size_t L = b->channels, n = b->n;
  if (L < 2) return OR_INVALID_MOD_DROP;
  const uint64_t* ch = in;
  uint64_t* tmp = NULL;
  if (in_ntt) {
    tmp = (uint64_t*)malloc(L * n * sizeof(uint64_t));
    memcpy(tmp, in, L * n * sizeof(uint64_t));
    or_to_coeff_domain(b, tmp);
    ch = tmp;
  }
  size_t last = L - 1;
  uint64_t q_last = b->moduli[last];
  for (size_t i = 0; i < last; i++) {
    uint64_t qi = b->moduli[i];
    uint64_t inv = or_mod_inverse(q_last % qi, qi);
    for (size_t j = 0; j < n; j++) {
      uint64_t ci = ch[i * n + j];
      uint64_t cl = ch[last * n + j] % qi;
      uint64_t diff = or_sub_mod(ci, cl, qi);
      out[i * n + j] = or_mul_mod(diff, inv, qi);
    }
  }
  free(tmp);
  return OR_OK;
}

/* poly.rs:492-541 */
void or_automorphism(const or_basis* b, const uint64_t* in, int in_ntt, uint64_t g,
                     uint64_t* out, int* out_ntt) {
  size_t L = b->channels, n = b->n;
  uint64_t two_n = 2 * (uint64_t)n;
  uint64_t e = g % two_n;
  if (e == 0) { /* :508-511 returns self.clone() (domain preserved) */
    memcpy(out, in, L * n * sizeof(uint64_t));
    *out_ntt = in_ntt;
    return;
  }
  const uint64_t* ch = in;
  uint64_t* tmp = NULL;
  if (in_ntt) {
    tmp = (uint64_t*)malloc(L * n * sizeof(uint64_t));
    memcpy(tmp, in, L * n * sizeof(uint64_t));
    or_to_coeff_domain(b, tmp);
    ch = tmp;
  }
  memset(out, 0, L * n * sizeof(uint64_t));
  for (size_t c = 0; c < L; c++) {
    uint64_t q = b->moduli[c];
    for (size_t i = 0; i < n; i++) {
      uint64_t coeff = ch[c * n + i];
      uint64_t jf = ((uint64_t)i * e) % two_n; /* i*e < 2N*2N fits u64 for N<=2^31 */
      size_t j = (size_t)(jf % n);
      int sign = jf >= n;
      if (coeff == 0) continue;
      out[c * n + j] = sign ? q - coeff : coeff;
    }
  }
  *out_ntt = 0;
  free(tmp);
}

/* poly.rs:546-569 */
void or_rotate_slots(const or_basis* b, const uint64_t* in, int in_ntt, int32_t k,
                     uint64_t* out, int* out_ntt) {
  uint64_t two_n = 2 * (uint64_t)b->n;
  uint64_t rot = k >= 0 ? (uint64_t)k : (uint64_t)(-(int64_t)k);
  uint64_t e = or_mod_pow(5, rot, two_n);
  if (k >= 0) {
    or_automorphism(b, in, in_ntt, e, out, out_ntt);
  } else {
    size_t sz = b->channels * b->n;
    uint64_t* tmp = (uint64_t*)malloc(sz * sizeof(uint64_t));
    int tmp_ntt;
    or_automorphism(b, in, in_ntt, e, tmp, &tmp_ntt);
    or_automorphism(b, tmp, tmp_ntt, two_n - 1, out, out_ntt);
    free(tmp);
  }
}

/* ------------------------------------------------------------------ */
/* engine.rs key-switching                                              */
/* ------------------------------------------------------------------ */

/* engine.rs:505-528 (relin) == engine.rs:429-452 (rotation) */
void or_gadget_keyswitch(const or_basis* b, const uint64_t* d, const uint64_t* key_a,
                         const uint64_t* key_b, uint64_t* acc0, uint64_t* acc1) {
  size_t L = b->channels, n = b->n, sz = L * n;
  uint64_t* alpha = (uint64_t*)malloc(sz * sizeof(uint64_t));
  uint64_t* tb = (uint64_t*)malloc(sz * sizeof(uint64_t));
  memset(acc0, 0, sz * sizeof(uint64_t));
  memset(acc1, 0, sz * sizeof(uint64_t));
  for (size_t i = 0; i < L; i++) {
    for (size_t j = 0; j < L; j++) {
      uint64_t qj = b->moduli[j];
      for (size_t k = 0; k < n; k++) alpha[j * n + k] = d[i * n + k] % qj; /* :507-516 */
    }
    memcpy(tb, alpha, sz * sizeof(uint64_t));
    or_mul_assign(b, tb, 0, key_b + i * sz, 0); /* :521-523 */
    or_add_assign(b, acc0, 0, tb, 0);
    or_mul_assign(b, alpha, 0, key_a + i * sz, 0); /* :525-527 */
    or_add_assign(b, acc1, 0, alpha, 0);
  }
  free(alpha);
  free(tb);
}

/* engine.rs:473-539 */
void or_mul_ciphertexts_gadget(const or_basis* b, const uint64_t* c0, const uint64_t* c1,
                               const uint64_t* c0p, const uint64_t* c1p,
                               const uint64_t* key_a, const uint64_t* key_b,
                               uint64_t* out0, uint64_t* out1) {
  size_t sz = b->channels * b->n;
  uint64_t* d1b = (uint64_t*)malloc(sz * sizeof(uint64_t));
  uint64_t* d2 = (uint64_t*)malloc(sz * sizeof(uint64_t));
  uint64_t* r0 = (uint64_t*)malloc(sz * sizeof(uint64_t));
  uint64_t* r1 = (uint64_t*)malloc(sz * sizeof(uint64_t));
  memcpy(out0, c0, sz * 8); or_mul_assign(b, out0, 0, c0p, 0);       /* d0 :481-482 */
  memcpy(out1, c0, sz * 8); or_mul_assign(b, out1, 0, c1p, 0);       /* d1a :484-485 */
  memcpy(d1b, c1, sz * 8); or_mul_assign(b, d1b, 0, c0p, 0);         /* d1b :486-487 */
  or_add_assign(b, out1, 0, d1b, 0);                                 /* :488-489 */
  memcpy(d2, c1, sz * 8); or_mul_assign(b, d2, 0, c1p, 0);           /* d2 :491-493 */
  or_gadget_keyswitch(b, d2, key_a, key_b, r0, r1);                  /* :498-528 */
  or_add_assign(b, out0, 0, r0, 0);                                  /* :530 */
  or_add_assign(b, out1, 0, r1, 0);                                  /* :531 */
  free(d1b); free(d2); free(r0); free(r1);
}

/* engine.rs:412-463 */
void or_rotate_ciphertext(const or_basis* b, const uint64_t* c0, const uint64_t* c1, int32_t k,
                          const uint64_t* key_a, const uint64_t* key_b,
                          uint64_t* out0, uint64_t* out1) {
  size_t sz = b->channels * b->n;
  uint64_t* c1r = (uint64_t*)malloc(sz * sizeof(uint64_t));
  uint64_t* ks0 = (uint64_t*)malloc(sz * sizeof(uint64_t));
  int f0, f1;
  or_rotate_slots(b, c0, 0, k, out0, &f0);  /* :417 */
  or_rotate_slots(b, c1, 0, k, c1r, &f1);   /* :418 */
  or_gadget_keyswitch(b, c1r, key_a, key_b, ks0, out1); /* :426-452 */
  or_add_assign(b, out0, 0, ks0, 0);        /* :454-455 */
  free(c1r); free(ks0);
}

/* ------------------------------------------------------------------ */
/* CPU baseline driver                                                  */
/* ------------------------------------------------------------------ */

typedef struct {
  const or_basis* b;
  uint64_t* a;
  const uint64_t* rhs;
  size_t items;
  size_t next;
  pthread_mutex_t mu;
} mt_job;

static void* mt_worker(void* arg) {
  mt_job* job = (mt_job*)arg;
  size_t n = job->b->n, L = job->b->channels;
  uint64_t* scratch = (uint64_t*)malloc(n * sizeof(uint64_t));
  for (;;) {
    pthread_mutex_lock(&job->mu);
    size_t it = job->next++;
    pthread_mutex_unlock(&job->mu);
    if (it >= job->items) break;
    size_t poly = it / L, ch = it % L;
    size_t off = (poly * L + ch) * n;
    channel_mul_coeff(&job->b->tables[ch], n, job->a + off, job->rhs + off, scratch);
  }
  free(scratch);
  return NULL;
}

double or_polymul_batch_mt(const or_basis* b, uint64_t* a, const uint64_t* rhs,
                           size_t count, int threads) {
  if (threads < 1) threads = 1;
  mt_job job;
  job.b = b; job.a = a; job.rhs = rhs;
  job.items = count * b->channels;
  job.next = 0;
  pthread_mutex_init(&job.mu, NULL);
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  pthread_t* th = (pthread_t*)malloc((size_t)threads * sizeof(pthread_t));
  for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, mt_worker, &job);
  for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  free(th);
  pthread_mutex_destroy(&job.mu);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ------------------------------------------------------------------ */
/* Channel-parallel key-switch (test infrastructure: the same per-channel  */
/* arithmetic as or_gadget_keyswitch / or_mul_ciphertexts_gadget /          */
/* or_rotate_ciphertext, spread over threads so the oracle can check the    */
/* BASELINE config-4/5 rings in seconds).  Every target channel j of the   */
/* gadget sum depends only on d[*] and channel j of the keys               */
/* (engine.rs:505-528: alpha_i[j] = d[i] mod q_j, then channel-wise ring   */
/* products), so channels are independent work items.                      */
/* ------------------------------------------------------------------ */

typedef void (*chan_fn)(void* ctx, size_t ch, uint64_t* scratch);
typedef struct {
  chan_fn fn;
  void* ctx;
  size_t items, next, scratch_words;
  pthread_mutex_t mu;
} par_job;

static void* par_worker(void* arg) {
  par_job* job = (par_job*)arg;
  uint64_t* scratch = (uint64_t*)malloc(job->scratch_words * sizeof(uint64_t));
  for (;;) {
    pthread_mutex_lock(&job->mu);
    size_t it = job->next++;
    pthread_mutex_unlock(&job->mu);
    if (it >= job->items) break;
    job->fn(job->ctx, it, scratch);
  }
  free(scratch);
  return NULL;
}

static void par_for(size_t items, int threads, size_t scratch_words, chan_fn fn, void* ctx) {
  if (threads < 1) threads = 1;
  if ((size_t)threads > items) threads = (int)(items ? items : 1);
  par_job job;
  job.fn = fn; job.ctx = ctx; job.items = items; job.next = 0; job.scratch_words = scratch_words;
  pthread_mutex_init(&job.mu, NULL);
  pthread_t* th = (pthread_t*)malloc((size_t)threads * sizeof(pthread_t));
  for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, par_worker, &job);
  for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
  free(th);
  pthread_mutex_destroy(&job.mu);
}

typedef struct {
  const or_basis* b;
  const uint64_t *d, *key_a, *key_b;
  uint64_t *acc0, *acc1;
} ks_ctx;

/* target channel j of engine.rs:505-528 */
static void ks_channel(void* vc, size_t j, uint64_t* scratch) {
  ks_ctx* c = (ks_ctx*)vc;
  const or_basis* b = c->b;
  size_t L = b->channels, n = b->n, sz = L * n;
  uint64_t qj = b->moduli[j];
  uint64_t* alpha = scratch;
  uint64_t* tb = scratch + n;
  uint64_t* mul_scratch = scratch + 2 * n;
  uint64_t* a0 = c->acc0 + j * n;
  uint64_t* a1 = c->acc1 + j * n;
  memset(a0, 0, n * sizeof(uint64_t));
  memset(a1, 0, n * sizeof(uint64_t));
  for (size_t i = 0; i < L; i++) {
    for (size_t k = 0; k < n; k++) alpha[k] = c->d[i * n + k] % qj; /* :507-516 */
    memcpy(tb, alpha, n * sizeof(uint64_t));
    channel_mul_coeff(&b->tables[j], n, tb, c->key_b + i * sz + j * n, mul_scratch); /* :521-523 */
    for (size_t k = 0; k < n; k++) a0[k] = or_add_mod(a0[k], tb[k], qj);
    channel_mul_coeff(&b->tables[j], n, alpha, c->key_a + i * sz + j * n, mul_scratch); /* :525-527 */
    for (size_t k = 0; k < n; k++) a1[k] = or_add_mod(a1[k], alpha[k], qj);
  }
}

void or_gadget_keyswitch_mt(const or_basis* b, const uint64_t* d, const uint64_t* key_a,
                            const uint64_t* key_b, uint64_t* acc0, uint64_t* acc1, int threads) {
  ks_ctx c = {b, d, key_a, key_b, acc0, acc1};
  par_for(b->channels, threads, 3 * b->n, ks_channel, &c);
}

typedef struct {
  const or_basis* b;
  const uint64_t *c0, *c1, *c0p, *c1p;
  uint64_t *out0, *out1, *d2;
} tensor_ctx;

/* channel ch of the tensor product engine.rs:480-493 */
static void tensor_channel(void* vc, size_t ch, uint64_t* scratch) {
  tensor_ctx* c = (tensor_ctx*)vc;
  const or_basis* b = c->b;
  size_t n = b->n, o = ch * n;
  uint64_t q = b->moduli[ch];
  const or_table* t = &b->tables[ch];
  uint64_t* d1b = scratch;
  uint64_t* ms = scratch + n;
  memcpy(c->out0 + o, c->c0 + o, n * 8); channel_mul_coeff(t, n, c->out0 + o, c->c0p + o, ms);
  memcpy(c->out1 + o, c->c0 + o, n * 8); channel_mul_coeff(t, n, c->out1 + o, c->c1p + o, ms);
  memcpy(d1b, c->c1 + o, n * 8); channel_mul_coeff(t, n, d1b, c->c0p + o, ms);
  for (size_t k = 0; k < n; k++) c->out1[o + k] = or_add_mod(c->out1[o + k], d1b[k], q);
  memcpy(c->d2 + o, c->c1 + o, n * 8); channel_mul_coeff(t, n, c->d2 + o, c->c1p + o, ms);
}

void or_mul_ciphertexts_gadget_mt(const or_basis* b, const uint64_t* c0, const uint64_t* c1,
                                  const uint64_t* c0p, const uint64_t* c1p,
                                  const uint64_t* key_a, const uint64_t* key_b,
                                  uint64_t* out0, uint64_t* out1, int threads) {
  size_t sz = b->channels * b->n;
  uint64_t* d2 = (uint64_t*)malloc(sz * sizeof(uint64_t));
  uint64_t* r0 = (uint64_t*)malloc(sz * sizeof(uint64_t));
  uint64_t* r1 = (uint64_t*)malloc(sz * sizeof(uint64_t));
  tensor_ctx tc = {b, c0, c1, c0p, c1p, out0, out1, d2};
  par_for(b->channels, threads, 2 * b->n, tensor_channel, &tc);
  or_gadget_keyswitch_mt(b, d2, key_a, key_b, r0, r1, threads);
  or_add_assign(b, out0, 0, r0, 0); /* :530 */
  or_add_assign(b, out1, 0, r1, 0); /* :531 */
  free(d2); free(r0); free(r1);
}

void or_rotate_ciphertext_mt(const or_basis* b, const uint64_t* c0, const uint64_t* c1, int32_t k,
                             const uint64_t* key_a, const uint64_t* key_b,
                             uint64_t* out0, uint64_t* out1, int threads) {
  size_t sz = b->channels * b->n;
  uint64_t* c1r = (uint64_t*)malloc(sz * sizeof(uint64_t));
  uint64_t* ks0 = (uint64_t*)malloc(sz * sizeof(uint64_t));
  int f0, f1;
  or_rotate_slots(b, c0, 0, k, out0, &f0); /* :417 */
  or_rotate_slots(b, c1, 0, k, c1r, &f1);  /* :418 */
  or_gadget_keyswitch_mt(b, c1r, key_a, key_b, ks0, out1, threads); /* :426-452 */
  or_add_assign(b, out0, 0, ks0, 0);       /* :454-455 */
  free(c1r); free(ks0);
}
