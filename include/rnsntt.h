/*
 * rnsntt.h -- C-ABI of the MI355X-native RNS-NTT backend (librnsntt.so).
 *
 * Drop-in boundary for oiwn/toy-heaan-ckks's `RnsPoly<N>` / `RnsBasis<N>`
 * (src/rings/backends/rns_ntt/) and the key-switch / rescale loops of
 * `CkksEngine` (src/crypto/engine.rs).  Each entry point names the reference
 * interface it replaces (paths relative to the reference repository root).
 *
 * Conventions
 *  - Every function returns an `int` status: 0 = OK, otherwise one of
 *    RNT_ERR_*.  No exception, abort or panic crosses this boundary.
 *    `rnt_last_error()` returns a thread-local human-readable message for the
 *    last failing call on the calling thread.
 *  - Host polynomial data is exactly the reference's memory: a polynomial is
 *    `Vec<[u64; N]>`, i.e. `uint64_t[L][N]` (limb-major, "channels"); a batch
 *    of B polynomials is `uint64_t[B][L][N]`.  Rust passes
 *    `channels.as_ptr() as *const u64`.
 *  - NTT-domain data crossing the boundary is in the reference's natural
 *    order: index k holds a(psi^(2k+1)) mod q_i (poly.rs:136-148).  The
 *    device-internal order is private.
 *  - Ops are asynchronous on the context's stream; `rnt_sync` waits.
 *    Uploads and downloads are synchronous (they validate / return host
 *    data).
 *  - Threading: a context is immutable after creation and may be shared by
 *    any number of host threads (it is the reference's `Arc<RnsBasis>`).  A
 *    buffer must not be used by two threads at once (the reference's `&mut`).
 */
#ifndef RNSNTT_H
#define RNSNTT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RNT_ABI_VERSION 4

/* Status codes.  1..6 mirror RnsNttError in order
 * (src/rings/backends/rns_ntt/errors.rs:4-20). */
enum {
  RNT_OK = 0,
  RNT_ERR_INVALID_DEGREE = 1,      /* RnsNttError::InvalidDegree          */
  RNT_ERR_EMPTY_BASIS = 2,         /* RnsNttError::EmptyBasis             */
  RNT_ERR_NON_NTT_FRIENDLY = 3,    /* RnsNttError::NonNttFriendlyModulus  */
  RNT_ERR_INVALID_MOD_DROP = 4,    /* RnsNttError::InvalidModDrop         */
  RNT_ERR_CHANNEL_COUNT = 5,       /* RnsNttError::ChannelCountMismatch   */
  RNT_ERR_NON_REDUCED = 6,         /* RnsNttError::NonReducedCoefficient  */
  RNT_ERR_DOMAIN_MISMATCH = 7,     /* reference: debug_assert only (poly.rs:264-267, 292-295) */
  RNT_ERR_BASIS_MISMATCH = 8,      /* reference: debug_assert Arc::ptr_eq (poly.rs:260-263, 288-291) */
  RNT_ERR_DEVICE = 9,              /* HIP runtime error                   */
  RNT_ERR_OUT_OF_MEMORY = 10,
  RNT_ERR_BAD_ARGUMENT = 11,
  /* A valid reference input beyond this backend's capacity (no reference
   * variant: the reference accepts it).  Today only ring degrees above
   * 2^17 (rnt_ctx_create); fields = {degree, max_degree}. */
  RNT_ERR_UNSUPPORTED = 12
};

typedef struct rnt_ctx rnt_ctx; /* == Arc<RnsBasis<N>> (basis.rs:90-94) */
typedef struct rnt_buf rnt_buf; /* == device storage of B RnsPoly (poly.rs:25-30) */

/* ---- library / diagnostics ------------------------------------------- */
int rnt_abi_version(void);
const char* rnt_last_error(void);
const char* rnt_status_string(int status);
/* The RnsNttError fields (src/rings/backends/rns_ntt/errors.rs:4-20) of the
 * calling thread's last failing call, so a binding can rebuild the
 * reference's variant exactly.  Returns that call's status and writes
 *   1 InvalidDegree          fields = {degree, 0}
 *   2 EmptyBasis             fields = {0, 0}
 *   3 NonNttFriendlyModulus  fields = {modulus, degree}
 *   4 InvalidModDrop         fields = {drop_count, channel_count}
 *   5 ChannelCountMismatch   fields = {expected, actual}
 *   6 NonReducedCoefficient  fields = {coefficient, modulus}
 *  12 Unsupported            fields = {degree, max_degree} (no reference variant)
 * and {0, 0} for the statuses 7..11, which have no reference variant.
 * 0 (and {0, 0}) if no call on this thread has failed. */
int rnt_last_error_detail(uint64_t fields[2]);

/* Number of visible HIP devices (0 without a GPU; never fails on CPU-only
 * hosts). */
int rnt_device_count(int* n);

/* ---- per-kernel timing (diagnostics; not thread-safe) ------------------ */
/* When enabled on a context, every kernel the library launches on that
 * context's stream is bracketed by HIP events; rnt_profile_read syncs and
 * returns, for one kernel name ("col_fwd", "row_fwd", "row_inv",
 * "row_mul", "col_inv", "elementwise", "rescale", "automorphism",
 * "ks_decompose", "ks_rows", "tensor_rows", "import", "export", "crt", "sfft",
 * "sample", "copy", "plane_fused", "mf_ntt_fwd", "mf_ntt_inv", "whole_fwd",
 * "whole_inv", "whole_mul", "ks_whole", "tensor_whole", "mf_tensor", "mf_mul"), the
 * launch count and summed device milliseconds since enabling. */
int rnt_profile_enable(const rnt_ctx* ctx, int enable);
int rnt_profile_read(const rnt_ctx* ctx, const char* kernel, uint64_t* launches,
                     double* total_ms);
/* Test hook for the deferred-error path: records a failed cleanup call
 * (HIP error `hip_error`, named "rnt_debug_defer") on the calling thread,
 * as a block leaving the device cache would.  The next launch on the thread
 * reports it as RNT_ERR_DEVICE; free / destroy / trim entry points report
 * only their own cleanup failures and leave it pending. */
int rnt_debug_defer(int hip_error);

/* ---- host-side number theory (no device needed) ----------------------- */
/* is_ntt_friendly_prime (src/math/primes.rs:125-131); writes 0/1. */
int rnt_is_ntt_friendly_prime(uint64_t p, uint64_t degree, int* out);
/* generate_primes (src/math/utils.rs:47-80): `count` descending NTT-friendly
 * primes of exactly `bit_size` bits for `degree`. */
int rnt_generate_primes(uint32_t bit_size, size_t count, uint64_t degree,
                        uint64_t* out);
/* psi of NttTable::new (basis.rs:39-40, find_primitive_root :217-237). */
int rnt_find_psi(uint64_t modulus, uint64_t degree, uint64_t* psi);

/* ---- context == RnsBasis ---------------------------------------------- */
/* RnsBasis::new (basis.rs:97-106) + NttTable::new per modulus (:20-84):
 * validates like the reference (EmptyBasis, then per modulus InvalidDegree
 * for a degree that is not a power of two and NonNttFriendlyModulus), builds
 * the device tables on `device`.  A power-of-two degree above 2^17, which the
 * reference accepts, is RNT_ERR_UNSUPPORTED (this backend's table and grid
 * limit), never InvalidDegree. */
int rnt_ctx_create(uint32_t log_n, const uint64_t* moduli, size_t count,
                   int device, rnt_ctx** out);
/* Releases the caller's handle; like dropping an Arc, the context (and its
 * device tables) stays alive until every buffer allocated on it is freed. */
int rnt_ctx_destroy(rnt_ctx* ctx);
/* RnsBasis::drop_last (basis.rs:121-134): a prefix view sharing the
 * parent's device tables (no table copy). */
int rnt_ctx_drop_last(const rnt_ctx* ctx, size_t drop_count, rnt_ctx** out);
int rnt_ctx_degree(const rnt_ctx* ctx, size_t* n);
int rnt_ctx_channel_count(const rnt_ctx* ctx, size_t* count); /* basis.rs:116-118 */
int rnt_ctx_moduli(const rnt_ctx* ctx, uint64_t* out);       /* basis.rs:108-110 */
int rnt_ctx_total_bits(const rnt_ctx* ctx, uint32_t* bits);  /* basis.rs:140-145 */
int rnt_ctx_psi(const rnt_ctx* ctx, size_t limb, uint64_t* psi);
/* The HIP stream (hipStream_t) the context's ops are queued on. */
int rnt_ctx_stream(const rnt_ctx* ctx, void** stream);
/* Queue later ops on the caller's `stream` (a hipStream_t of the context's
 * device; NULL restores the context's own stream), ordered after everything
 * already queued.  Applies to every context sharing the tables (drop_last
 * views).  Call it while no other thread issues ops on those contexts; a
 * caller's stream must outlive the context or be replaced first.  This is
 * SURVEY §8b's per-op stream: set it around the ops that belong on it. */
int rnt_ctx_set_stream(const rnt_ctx* ctx, void* stream);
int rnt_sync(const rnt_ctx* ctx);

/* ---- captured op sequences (hipGraph) --------------------------------- */
/* The reference engine calls one ciphertext at a time
 * (mul_ciphertexts_gadget engine.rs:473-539, rotate_ciphertext :412-463), so
 * a fixed per-ciphertext op sequence is launch-bound.  rnt_capture_begin
 * starts recording every op the calling thread then queues on ctx's stream
 * (any context sharing its tables) into a graph instead of running it;
 * rnt_capture_end instantiates it; rnt_graph_launch replays it, with the
 * same buffers, on the context's current stream.  Record only device ops
 * (no upload, download, rnt_sync or allocation that misses the block cache)
 * and run the sequence once un-recorded first, so its workspaces are cached;
 * the graph keeps the workspace blocks its ops took until
 * rnt_graph_destroy (recorded ops share one call-scoped workspace, so N
 * recorded key-switches keep one block, not N).  Buffers the graph reads
 * and writes must outlive it, and so must their private scratch: while a
 * graph is alive, do not run an op on a larger batch into one of its output
 * buffers (an op that grows a buffer's scratch releases the old block, which
 * the graph's replays still write).  rnt_graph_workspace reports the blocks
 * and bytes the graph holds. */
typedef struct rnt_graph rnt_graph;
int rnt_capture_begin(const rnt_ctx* ctx);
int rnt_capture_end(const rnt_ctx* ctx, rnt_graph** out);
int rnt_graph_launch(rnt_graph* graph);
int rnt_graph_destroy(rnt_graph* graph);
int rnt_graph_workspace(const rnt_graph* graph, size_t* blocks, size_t* bytes);

/* ---- buffers == batches of RnsPoly ------------------------------------ */
/* Allocates device storage for n_polys polynomials over ctx's basis, all
 * zero, coefficient domain (RnsPoly::zero, poly.rs:36-43).  The zeroing is
 * queued on the context's stream (rnt_ctx_stream) like every op: a reader on
 * another stream (e.g. through rnt_buf_device_ptr) must order itself after
 * that stream or call rnt_sync first. */
int rnt_buf_alloc(const rnt_ctx* ctx, size_t n_polys, rnt_buf** out);
/* The same buffer with unspecified contents: for an op's output, which the
 * op overwrites entirely (no zero fill queued; the reference has no such
 * constructor -- RnsPoly::zero is rnt_buf_alloc). */
int rnt_buf_alloc_uninit(const rnt_ctx* ctx, size_t n_polys, rnt_buf** out);
/* Frees without waiting for the device: the buffer's device blocks go to a
 * per-device cache behind an event on the context stream, and a later
 * allocation's stream waits on that event before reusing them. */
int rnt_buf_free(rnt_buf* buf);
/* Returns every idle cached block of `device` (-1: all devices) to the HIP
 * allocator, e.g. before a caller's own allocation that failed is retried;
 * writes the bytes released when freed_bytes is non-NULL.  The cache holds
 * at most RNT_WS_POOL_MB MiB (default 1/8 of the device's memory) idle. */
int rnt_pool_trim(int device, size_t* freed_bytes);
int rnt_buf_n_polys(const rnt_buf* buf, size_t* n);
int rnt_buf_is_ntt(const rnt_buf* buf, int* in_ntt); /* is_ntt_domain, poly.rs:127-129 */
/* RnsPoly::from_channels (poly.rs:73-99) for a batch: host
 * uint64_t[n_polys][channels][N]; `channels` must equal the basis' channel
 * count (else RNT_ERR_CHANNEL_COUNT); every residue must be < q_i (else
 * RNT_ERR_NON_REDUCED).  `in_ntt` != 0: natural-order NTT-domain data. */
int rnt_upload(rnt_buf* buf, const uint64_t* host, size_t n_polys,
               size_t channels, int in_ntt);
/* RnsPoly::from_coeffs (poly.rs:49-67) for a batch: host int64_t[n_polys][N]
 * reduced by rem_euclid per channel; result in coefficient domain. */
int rnt_upload_coeffs(rnt_buf* buf, const int64_t* coeffs, size_t n_polys);
/* RnsPoly::channels (poly.rs:119-121): copies uint64_t[n_polys][L][N] out,
 * in the buffer's current domain (natural order when NTT). */
int rnt_download(const rnt_buf* buf, uint64_t* host, size_t n_polys);
/* channels() of polys [first, first + count) of a batch: uint64_t[count][L][N],
 * in the buffer's current domain (natural order when NTT).  A range outside
 * the batch -> RNT_ERR_BAD_ARGUMENT. */
int rnt_download_polys(const rnt_buf* buf, uint64_t* host, size_t first, size_t count);
int rnt_copy(rnt_buf* dst, const rnt_buf* src); /* Clone */
/* PolyRing::to_coeffs (poly.rs:404-427) for a batch: per coefficient the CRT
 * value centred in (-Q/2, Q/2] (reconstruct_centered_coeff, basis.rs:158-180)
 * as int64_t[n_polys][N] -- the value's low 64 bits in two's complement,
 * exactly the reference's result wherever it is defined (Q < 2^128).  An
 * NTT-domain buffer is converted on a temporary copy. */
int rnt_to_coeffs(const rnt_buf* buf, int64_t* host, size_t n_polys);
/* The same centred CRT value without truncation: `words` 64-bit
 * little-endian two's-complement words per coefficient,
 * uint64_t[n_polys][N][words] (the reference's u128 path
 * cannot represent Q >= 2^128).  1 <= words <= 64. */
int rnt_crt_centered(const rnt_buf* buf, uint64_t* host, size_t n_polys, size_t words);
/* Device-memory interop for multi-GPU pipelines (collectives run by the
 * caller, e.g. RCCL through torch.distributed):
 * rnt_buf_wrap makes a NON-owning buffer over caller device memory laid out
 * [L][n_polys][N] in the context's word width (device-internal order when
 * in_ntt); rnt_buf_device_ptr exposes a buffer's storage and word width.
 * Library writes to that storage (including rnt_buf_alloc's zeroing) are
 * queued on the context's stream: order external reads after it (or call
 * rnt_sync). */
int rnt_buf_wrap(const rnt_ctx* ctx, void* device_ptr, size_t n_polys, int in_ntt,
                 rnt_buf** out);
int rnt_buf_device_ptr(const rnt_buf* buf, void** device_ptr, size_t* word_bytes);

/* ---- ring ops (batched; every poly of the buffers participates) -------- */
/* to_ntt_domain / to_coeff_domain (poly.rs:136-166); no-ops when already
 * in the target domain. */
int rnt_ntt_fwd(rnt_buf* buf);
int rnt_ntt_inv(rnt_buf* buf);
/* MulAssign (poly.rs:277-331) as out = a * b: both NTT -> pointwise, result
 * NTT; both coefficient -> negacyclic product, result coefficient.  Mixed
 * domains -> RNT_ERR_DOMAIN_MISMATCH.  out may alias a or b. */
int rnt_mul(rnt_buf* out, const rnt_buf* a, const rnt_buf* b);
/* AddAssign (poly.rs:254-275) as out = a + b, either domain (must match). */
int rnt_add(rnt_buf* out, const rnt_buf* a, const rnt_buf* b);
int rnt_sub(rnt_buf* out, const rnt_buf* a, const rnt_buf* b);
/* Neg (poly.rs:370-385), either domain. */
int rnt_neg(rnt_buf* out, const rnt_buf* a);
/* rescale_into (poly.rs:187-228): `out` belongs to a context equal to
 * drop_last(1) of `in`'s; result coefficient domain, floor division by the
 * last prime. */
int rnt_rescale(rnt_buf* out, const rnt_buf* in);
/* mod_drop_last (poly.rs:169-177): out (a context equal to drop_last(k) of
 * in's) receives the first L-k channels; domain preserved. */
int rnt_mod_drop_last(rnt_buf* out, const rnt_buf* in);
/* automorphism X -> X^g (poly.rs:492-541). Output coefficient domain, except
 * g mod 2N == 0 which copies `in` (domain preserved) like the reference. */
int rnt_automorphism(rnt_buf* out, const rnt_buf* in, uint64_t g);
/* rotate_slots (poly.rs:546-569): g = 5^k mod 2N (k >= 0); for k < 0 the
 * reference's automorphism(5^|k|) then automorphism(2N-1). */
int rnt_rotate_slots(rnt_buf* out, const rnt_buf* in, int32_t k);

/* ---- samplers (PolySampler, src/rings/traits.rs:74-127) */
/* Fill every poly of `out` (coefficient domain) from the counter-based
 * Philox4x32-10 stream (seed, stream): a draw depends only on (seed, stream,
 * sampler, poly, limb, index), never on launch geometry or batch split.  The
 * reference's ChaCha20 streams are not reproduced.
 *   uniform  : residues uniform in [0, q_l), independent per limb
 *              (sample_uniform, poly.rs:438-444);
 *   gaussian : round(N(0, std_dev)) per coefficient, reduced into every limb
 *              (sample_gaussian, poly.rs:447-459); std_dev must be finite > 0;
 *   ternary  : exactly hamming_weight coefficients +-1, the rest 0
 *              (sample_tribits, poly.rs:462-469); hamming_weight <= N. */
int rnt_sample_uniform(rnt_buf* out, uint64_t seed, uint64_t stream);
int rnt_sample_gaussian(rnt_buf* out, double std_dev, uint64_t seed, uint64_t stream);
int rnt_sample_ternary(rnt_buf* out, size_t hamming_weight, uint64_t seed, uint64_t stream);

/* ---- CKKS encoder / decoder (src/encoding) ---------- */
/* CkksEncoder::encode_complex (ckks_encoder.rs:85-122) for every poly of
 * `out`: values = [n_polys][n_values] complex slots as interleaved (re, im)
 * doubles, n_values <= N/2 (zero-padded to N/2, build_conjugate_slots,
 * special_fft.rs:158-178); slots times 2^scale_bits -> the inverse canonical
 * embedding (special_idft, special_fft.rs:194-220, as an O(N log N) special
 * FFT) -> coefficients rounded like f64::round -> residues like from_coeffs
 * (poly.rs:49-67).  `out` becomes coefficient domain.  n_values > N/2 or
 * scale_bits == 0 -> RNT_ERR_BAD_ARGUMENT (the reference panics). */
int rnt_encode(rnt_buf* out, const double* values, size_t n_values, uint32_t scale_bits);
/* CkksEncoder::decode_complex (ckks_encoder.rs:134-156): centred CRT
 * coefficients (to_coeffs, poly.rs:404-427, its i64 result) -> the canonical
 * embedding (special_dft, special_fft.rs:224-242) -> the first n_values
 * slots / 2^scale_bits into values ([n_polys][n_values] (re, im) pairs). */
int rnt_decode(const rnt_buf* in, double* values, size_t n_values, uint32_t scale_bits);

/* ---- engine-level fused ops (src/crypto/engine.rs) -------------------- */
/* A gadget key (RnsGadgetRelinKey / RnsGadgetRotationKey, engine.rs:224-253):
 * key_a and key_b are buffers of one poly per gadget (source) limb i
 * (poly i = a_i / b_i): L polys for rnt_keyswitch, the global limb count for
 * a limb shard's rnt_keyswitch_ext (validated by the key-switch calls).  They
 * are kept device-resident in the NTT domain; rnt_key_prepare transforms
 * them once. */
int rnt_key_prepare(rnt_buf* key_a, rnt_buf* key_b);
/* Gadget key-switch sum (engine.rs:505-528 / :429-452): for every poly of d
 * (coefficient domain): acc0 = sum_i alpha_i(d) * key_b[i],
 * acc1 = sum_i alpha_i(d) * key_a[i]; outputs coefficient domain. */
int rnt_keyswitch(rnt_buf* acc0, rnt_buf* acc1, const rnt_buf* d,
                  const rnt_buf* key_a, const rnt_buf* key_b);
/* mul_ciphertexts_gadget (engine.rs:473-539) for a batch of ciphertext
 * pairs: tensor product + gadget relinearization.  Inputs coefficient
 * domain; outputs coefficient domain. */
int rnt_ct_mul_relin(rnt_buf* out0, rnt_buf* out1, const rnt_buf* c0,
                     const rnt_buf* c1, const rnt_buf* c0p, const rnt_buf* c1p,
                     const rnt_buf* key_a, const rnt_buf* key_b);
/* mul_ciphertexts_gadget followed by rescale_ciphertext (engine.rs:473-539,
 * then :263-282), the engine's ct-mul call pair, as one op: out0/out1 are on
 * drop_last(1) of the inputs' basis (one shared context, as rnt_ct_rescale);
 * the result equals rnt_ct_mul_relin + rnt_ct_rescale word for word.  The
 * rescale runs as the key-switch inverse's epilogue, so the un-rescaled
 * product never reaches memory (N >= 2^14 with the four-step key-switch;
 * smaller rings run the two ops). */
int rnt_ct_mul_relin_rescale(rnt_buf* out0, rnt_buf* out1, const rnt_buf* c0,
                             const rnt_buf* c1, const rnt_buf* c0p, const rnt_buf* c1p,
                             const rnt_buf* key_a, const rnt_buf* key_b);
/* rotate_ciphertext (engine.rs:412-463). */
int rnt_ct_rotate(rnt_buf* out0, rnt_buf* out1, const rnt_buf* c0,
                  const rnt_buf* c1, int32_t k, const rnt_buf* key_a,
                  const rnt_buf* key_b);
/* rescale_ciphertext (engine.rs:263-282): both components onto the same
 * dropped basis. */
int rnt_ct_rescale(rnt_buf* out0, rnt_buf* out1, const rnt_buf* c0,
                   const rnt_buf* c1);

/* ---- limb-sharded building blocks ------------------------ */
/* A rank owning a contiguous run of the global basis' limbs holds every
 * ciphertext restricted to them (a context over those moduli).  The join
 * steps take the other ranks' limbs as raw device arrays gathered by the
 * caller. */
/* Tensor product of mul_ciphertexts_gadget (engine.rs:480-493) on the local
 * limbs: d0 = c0 c0', d1 = c0 c1' + c1 c0' (NTT domain, device order: the
 * seeds of rnt_keyswitch_ext), d2 = c1 c1' (coefficient domain). */
int rnt_ct_tensor(rnt_buf* d0, rnt_buf* d1, rnt_buf* d2, const rnt_buf* c0,
                  const rnt_buf* c1, const rnt_buf* c0p, const rnt_buf* c1p);
/* Gadget sum (engine.rs:505-528) for the local (target) limbs of acc0/acc1
 * over `src_limbs` source limbs held at `src` ([src_limbs][B][N] words,
 * coefficient domain, B = acc0's batch): acc = INV(seed + sum_i
 * NTT(src_i mod q_j) key[i]); key_a/key_b hold src_limbs polys over acc's
 * basis (prepared); init0/init1 NTT-domain seeds or NULL. */
int rnt_keyswitch_ext(rnt_buf* acc0, rnt_buf* acc1, const void* src, size_t src_limbs,
                      const rnt_buf* key_a, const rnt_buf* key_b, const rnt_buf* init0,
                      const rnt_buf* init1);
/* rescale_into (poly.rs:187-228) by an external last modulus q_last whose
 * residues (coefficient domain, [B][N] words) are at `last_limb`: every
 * local limb l -> (c_l - (c_last mod q_l)) (q_last mod q_l)^-1.  If q_last is
 * the input's own last modulus (the shard that owns it) that limb is
 * dropped, so `out` must be drop_last(1) of `in`'s context; otherwise `out`
 * shares `in`'s context. */
int rnt_rescale_ext(rnt_buf* out, const rnt_buf* in, const void* last_limb, uint64_t q_last);

#ifdef __cplusplus
}
#endif
#endif /* RNSNTT_H */
