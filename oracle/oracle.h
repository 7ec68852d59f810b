/*
 * oracle.h -- CPU restatement of oiwn/toy-heaan-ckks's RNS-NTT path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (include/, the
 * toy-heaan-ckks_amd/ package) may link, load or call this code.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it,
 * and only as the checker / the timed CPU baseline.
 *
 * Every function restates one reference function, with the same loop
 * structure and the same u128 `%` arithmetic, and cites its source
 * (paths relative to the reference repository root).  Storage is the
 * reference's `Vec<[u64; N]>`, i.e. a contiguous [L][N] uint64_t array per
 * polynomial, heap-allocated (the reference uses stack arrays, which
 * overflow at N = 2^16).
 *
 * Parity pinning: the reference is Rust and no Rust toolchain exists here,
 * so the reference itself cannot be built (oracle/_ref stays empty).  This
 * restatement is pinned by the reference's own known-answer tests
 * (tests/golden/reference_kats.json, transcribed from poly.rs / basis.rs /
 * primes.rs / utils.rs #[test] blocks) and by an independent pure-Python
 * big-integer restatement (tests/golden/make_golden.py).
 */
#ifndef TOY_HEAAN_ORACLE_H
#define TOY_HEAAN_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes mirror RnsNttError (src/rings/backends/rns_ntt/errors.rs:4-20). */
enum {
  OR_OK = 0,
  OR_INVALID_DEGREE = 1,
  OR_EMPTY_BASIS = 2,
  OR_NON_NTT_FRIENDLY = 3,
  OR_INVALID_MOD_DROP = 4,
  OR_CHANNEL_COUNT_MISMATCH = 5,
  OR_NON_REDUCED = 6,
  OR_DOMAIN_MISMATCH = 7,
  OR_BAD_ARGUMENT = 11,
};

/* ---- scalar modular helpers: poly.rs:629-653, basis.rs:185-210 ---------- */
uint64_t or_mul_mod(uint64_t a, uint64_t b, uint64_t q);
uint64_t or_add_mod(uint64_t a, uint64_t b, uint64_t q);
uint64_t or_sub_mod(uint64_t a, uint64_t b, uint64_t q);
uint64_t or_mod_pow(uint64_t base, uint64_t e, uint64_t q);
uint64_t or_mod_inverse(uint64_t v, uint64_t q); /* returns 0 if not coprime */

/* ---- primes: src/math/primes.rs:21-219, src/math/utils.rs:47-80 -------- */
int or_is_prime(uint64_t n);
int or_is_prime_reference(uint64_t n);
int or_is_ntt_friendly_prime(uint64_t p, uint64_t n);
uint64_t or_get_first_prime_up(uint32_t logq, uint64_t n);
/* returns 0 for None */
uint64_t or_get_first_prime_down(uint64_t bound, uint64_t n);
/* returns number of primes written (== count on success, 0 on the panic paths) */
size_t or_generate_primes(uint32_t bit_size, size_t count, uint64_t degree,
                          uint64_t* out);

/* ---- NTT tables / basis: basis.rs:5-180 ---------------------------------- */
typedef struct {
  uint64_t modulus;
  uint64_t n_inv;
  uint64_t psi;
  uint64_t* forward_roots;   /* [N] omega^i         */
  uint64_t* inverse_roots;   /* [N] omega^{-i}      */
  uint64_t* twist_factors;   /* [N] psi^j           */
  uint64_t* untwist_factors; /* [N] psi^{-j}        */
} or_table;

typedef struct {
  size_t n;
  size_t channels;
  uint64_t* moduli;
  or_table* tables;
  int owns_tables; /* 0 for drop_last views */
} or_basis;

uint64_t or_find_primitive_root(uint64_t modulus, uint64_t order);
int or_table_new(or_table* t, size_t n, uint64_t modulus);
void or_table_free(or_table* t);
int or_basis_new(or_basis* b, size_t n, const uint64_t* moduli, size_t count);
void or_basis_free(or_basis* b);
/* basis.rs:121-134: keeps a prefix; the view shares the parent's tables. */
int or_basis_drop_last(const or_basis* b, size_t drop_count, or_basis* out);
uint32_t or_basis_total_bits(const or_basis* b);
/* basis.rs:158-180 (requires Q < 2^128) */
int64_t or_reconstruct_centered(const or_basis* b, const uint64_t* residues);

/* ---- polynomial ops on one [L][N] poly: poly.rs ------------------------- */
void or_from_coeffs(const or_basis* b, const int64_t* coeffs, uint64_t* out);
int or_from_channels_check(const or_basis* b, const uint64_t* ch, size_t count);
void or_to_coeffs(const or_basis* b, const uint64_t* poly, int in_ntt,
                  int64_t* out);
void or_forward_ntt(const or_table* t, size_t n, uint64_t* v);
void or_inverse_ntt(const or_table* t, size_t n, uint64_t* v);
void or_to_ntt_domain(const or_basis* b, uint64_t* poly);
void or_to_coeff_domain(const or_basis* b, uint64_t* poly);
/* MulAssign (poly.rs:277-331); a and b must be in the same domain
 * (the reference debug_asserts this; we return OR_DOMAIN_MISMATCH). */
int or_mul_assign(const or_basis* b, uint64_t* a, int a_ntt,
                  const uint64_t* rhs, int rhs_ntt);
void or_mul_assign_naive(const or_basis* b, uint64_t* a, const uint64_t* rhs);
int or_add_assign(const or_basis* b, uint64_t* a, int a_ntt,
                  const uint64_t* rhs, int rhs_ntt);
void or_neg(const or_basis* b, uint64_t* a);
/* rescale_into (poly.rs:187-228): out has L-1 channels, coefficient domain */
int or_rescale(const or_basis* b, const uint64_t* in, int in_ntt,
               uint64_t* out);
/* automorphism (poly.rs:492-541).  *out_ntt receives the output domain
 * flag (the g mod 2N == 0 early return clones self, domain included). */
void or_automorphism(const or_basis* b, const uint64_t* in, int in_ntt,
                     uint64_t g, uint64_t* out, int* out_ntt);
/* rotate_slots (poly.rs:546-569) */
void or_rotate_slots(const or_basis* b, const uint64_t* in, int in_ntt,
                     int32_t k, uint64_t* out, int* out_ntt);

/* ---- engine-level key-switch: src/crypto/engine.rs ---------------------- */
/* Gadget sum (engine.rs:505-528 / 429-452): d (coefficient domain) ->
 * acc0 = sum_i alpha_i(d) * key_b[i], acc1 = sum_i alpha_i(d) * key_a[i].
 * key_a/key_b: L polys each, [L][L][N], coefficient domain. */
void or_gadget_keyswitch(const or_basis* b, const uint64_t* d,
                         const uint64_t* key_a, const uint64_t* key_b,
                         uint64_t* acc0, uint64_t* acc1);
/* mul_ciphertexts_gadget (engine.rs:473-539), coefficient-domain inputs. */
void or_mul_ciphertexts_gadget(const or_basis* b, const uint64_t* c0,
                               const uint64_t* c1, const uint64_t* c0p,
                               const uint64_t* c1p, const uint64_t* key_a,
                               const uint64_t* key_b, uint64_t* out0,
                               uint64_t* out1);
/* rotate_ciphertext (engine.rs:412-463) */
void or_rotate_ciphertext(const or_basis* b, const uint64_t* c0,
                          const uint64_t* c1, int32_t k,
                          const uint64_t* key_a, const uint64_t* key_b,
                          uint64_t* out0, uint64_t* out1);

/* Channel-parallel forms of the three above (identical results; `threads`
 * workers over target channels).  Test infrastructure for the config-4/5
 * rings only. */
void or_gadget_keyswitch_mt(const or_basis* b, const uint64_t* d,
                            const uint64_t* key_a, const uint64_t* key_b,
                            uint64_t* acc0, uint64_t* acc1, int threads);
void or_mul_ciphertexts_gadget_mt(const or_basis* b, const uint64_t* c0,
                                  const uint64_t* c1, const uint64_t* c0p,
                                  const uint64_t* c1p, const uint64_t* key_a,
                                  const uint64_t* key_b, uint64_t* out0,
                                  uint64_t* out1, int threads);
void or_rotate_ciphertext_mt(const or_basis* b, const uint64_t* c0,
                             const uint64_t* c1, int32_t k,
                             const uint64_t* key_a, const uint64_t* key_b,
                             uint64_t* out0, uint64_t* out1, int threads);

/* ---- CPU baseline driver (bench.py cpu_baseline leg) ---------------------- */
/* Runs `count` coefficient-domain poly-muls a[i] *= b[i] ([count][L][N] each)
 * with `threads` std::thread-style workers over (poly, limb) work items.
 * Each work item is the reference's per-channel MulAssign body
 * (poly.rs:310-328).  Returns wall seconds. */
double or_polymul_batch_mt(const or_basis* b, uint64_t* a, const uint64_t* rhs,
                           size_t count, int threads);

#ifdef __cplusplus
}
#endif
#endif
