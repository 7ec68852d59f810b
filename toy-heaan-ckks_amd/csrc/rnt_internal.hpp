// rnt_internal.hpp -- private types shared by the C-ABI layer (rnt_api.cpp)
// and the kernels (rnt_kernels.hip).
//
// Device layout (private):
//   A buffer of B polynomials over L limbs is one allocation of W words laid
//   out [L][B][N] (limb-major, so a limb shard is contiguous and one prime's
//   twiddles serve a whole contiguous launch range).  W = uint32_t when every
//   modulus is < 2^31, else uint64_t.
//   NTT-domain data is stored in bit-reversed order of the natural
//   evaluation index (the output order of the merged negacyclic CT
//   transform), i.e. device[brv(k)] = a(psi^(2k+1)).  Upload / download
//   permute to and from the reference's natural order.
//
// Transform decomposition: N = R * C.  The column pass does the top log2(R)
// CT stages (a stride-C radix-R butterfly network per column, in
// registers); the row pass does the remaining log2(C) stages per row of C
// contiguous words through LDS in radix-16 register passes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace rnt {

constexpr int kMaxLogN = 17;
constexpr int kRowElems = 16;  // elements per thread per operand in the row pass
// threads per row-pass workgroup (at least one row's C/16 threads)
constexpr int kRowThreads = 256;

template <class W>
struct LimbConst {
  W q;       // modulus
  W qinv;    // q^-1 mod 2^w (Montgomery)
  W one_p;   // floor(2^w / q): Shoup companion of 1 (canonical reduction of x < 2^w)
  W rmod;    // 2^w mod q
  W rmod_p;
  W c1;      // n^-1                      (last inverse stage, plain)
  W c1_p;
  W c2;      // psi_inv_rev[1] * n^-1
  W c2_p;
  W c1r;     // n^-1 * 2^w                (last inverse stage, Montgomery-folded)
  W c1r_p;
  W c2r;     // psi_inv_rev[1] * n^-1 * 2^w
  W c2r_p;
  W c1t;     // 4 n^-1 * 2^w             (last stage after a product truncated two stages early)
  W c1t_p;
  W c2t;     // psi_inv_rev[1] * 4 n^-1 * 2^w
  W c2t_p;
};

// A twiddle and its Shoup companion, interleaved so one load fetches both.
template <class W>
struct alignas(2 * sizeof(W)) Tw {
  W w;  // psi^{+-brv(g)} mod q
  W p;  // floor(w * 2^w / q)
};

// Shared, immutable device tables of a root basis.  drop_last views hold a
// shared_ptr to the same tables (no copy, unlike basis.rs:130-133).
// Device pointers of the centred-CRT constants (rnt_kernels.hip k_crt).
struct CrtConsts {
  const uint32_t* qi_words;  // [L][MW]  Q / q_l
  const uint32_t* q_words;   // [MW]     Q
  const uint32_t* qh_words;  // [MW]     floor(Q / 2)
  const uint64_t* inv;       // [L]      (Q/q_l)^-1 mod q_l
  const uint64_t* inv_p;     // [L]      its Shoup companion (device word width)
  const double* rq;          // [L]      1 / q_l
};
struct CrtDev {
  void* dev = nullptr;
  uint32_t mw = 0;
  CrtConsts cc{};
};

struct Tables {
  int device = 0;
  int wide = 0;            // 0: W = u32, 1: W = u64
  bool lazy30 = false;     // every modulus < 2^30: Harvey-lazy product path (u32)
  bool lazy62 = false;     // u64 words, every modulus < 2^62: the same for u64
  bool ks_diag = true;     // ct-mul key-switch diagonal from the tensor's d2^ (RNT_KS_DIAG)
  int rot_fuse = 1;        // rotation: sigma(c0) gathered by the key-switch inverse (RNT_ROT_FUSE: 1 one ct, 2 any, 0 off)
  int plane = 0;           // the whole-plane kernels where they apply (plane_ok, mf_ok);
  int mf_mul = 1;          // rnt_mul at N = 2^16 on the matrix-core transforms (RNT_MF_MUL=0: k_plane_fused)
                           // RNT_PLANE=0: the four-step kernels everywhere
  uint32_t dec_jg = 0;     // key-switch decomposition: target limbs per workgroup (0 = auto)
  size_t ks_ws_bytes = (size_t)4096 << 20;  // key-switch scratch cap per chunk (RNT_KS_WS_MB)
  uint32_t log_n = 0;
  size_t n = 0;
  size_t L = 0;            // channel count of the root basis
  std::vector<uint64_t> moduli;
  std::vector<uint64_t> psi;
  void* tw_fwd = nullptr;   // [L][N] Tw<W>{psi^{brv(g)}, companion}, heap order g in [1, N)
  void* tw_inv = nullptr;   // [L][N] Tw<W>{psi^{-brv(g)}, companion}
  void* lconst = nullptr;   // [L] LimbConst<W>
  void* resc = nullptr;     // [L][L]: resc[l][i] = (q_l mod q_i)^-1 mod q_i, i < l
  void* resc_p = nullptr;   // [L][L] Shoup companions
  hipStream_t stream = nullptr;      // where every op is queued (rnt_ctx_set_stream)
  hipStream_t own_stream = nullptr;  // created with the context
  // rnt_rescale_ext constants per external last modulus: device arrays
  // {inv[L], invp[L]} with inv[l] = (q_last mod q_l)^-1 mod q_l.
  std::mutex resc_mu;
  std::vector<std::pair<uint64_t, void*>> resc_ext;
  // centred-CRT constants per limb count (rnt_to_coeffs / rnt_crt_centered)
  std::vector<std::pair<size_t, struct CrtDev>> crt_cache;
  // CKKS special-FFT twiddles (rnt_encode.hip), [N/2] double2, built on
  // first encode/decode
  std::mutex sfft_mu;
  void* sfft_tw = nullptr;
  struct Prof* prof = nullptr;  // per-kernel event timing (rnt_profile_*)
  // MFMA transform tables (rnt_mfma.hip: matrix operands, compensations and
  // twists per limb), built by rnt_ctx_create where mf_supported()
  void* mf = nullptr;
  ~Tables();
};

// Kernel ids for rnt_profile_read.
enum KernelId {
  K_COL_FWD, K_ROW_FWD, K_ROW_INV, K_ROW_MUL, K_COL_INV, K_ELEMENTWISE, K_RESCALE,
  K_AUTOMORPHISM, K_KS_DECOMPOSE, K_KS_ROWS, K_TENSOR_ROWS, K_IMPORT, K_EXPORT, K_CRT,
  K_SFFT, K_SAMPLE, K_COPY, K_PLANE_FUSED, K_MF_NTT_FWD, K_MF_NTT_INV, K_WHOLE_FWD, K_WHOLE_INV, K_WHOLE_MUL,
  K_KS_WHOLE, K_TENSOR_WHOLE, K_MF_TENSOR, K_MF_MUL, K_COUNT
};

struct Prof {
  std::mutex mu;
  bool on = false;
  struct Rec {
    int id;
    hipEvent_t a, b;
  };
  std::vector<Rec> pending;
  std::vector<hipEvent_t> pool;
  uint64_t launches[K_COUNT] = {};
  double ms[K_COUNT] = {};
  // the first failure of a profiling call (event create / record / elapsed
  // time): profiling turns itself off and rnt_profile_read reports it; it
  // never aborts or fails a launch
  hipError_t err = hipSuccess;
  const char* err_where = nullptr;
};

}  // namespace rnt

// Arc<RnsBasis> semantics: a context lives until rnt_ctx_destroy has been
// called AND every buffer allocated on it has been freed, so handles may be
// released in any order (e.g. by a garbage collector).
struct rnt_ctx {
  std::shared_ptr<rnt::Tables> t;
  size_t L = 0;  // channel count of this (possibly dropped) basis
  std::atomic<long> refs{1};  // 1 for the creator + 1 per live buffer
};

struct rnt_buf {
  const rnt_ctx* ctx = nullptr;
  size_t n_polys = 0;
  void* data = nullptr;       // [L][B][N] words
  size_t data_bytes = 0;      // size of the block holding `data` (owned buffers)
  int in_ntt = 0;
  // lazily grown per-buffer workspace (buffers are never used by two
  // threads at once, so this needs no lock)
  void* ws = nullptr;
  size_t ws_bytes = 0;
  void* stage = nullptr;      // u64 host-format staging for upload/download
  size_t stage_bytes = 0;
  bool owns = true;           // false: rnt_buf_wrap view of caller memory
};

namespace rnt {

// Geometry of the N = R * C split.
struct Geom {
  uint32_t log_n, log_r, log_c;
  size_t n, r, c;
};
Geom geom_for(uint32_t log_n);

// Kernel argument bundle common to all launches.
struct Launch {
  const Tables* t;
  size_t L;            // limbs processed (prefix of the root basis)
  size_t B;            // polys per buffer
  hipStream_t s;
  size_t Ls = 0;       // key-switch source limbs (0: same as L)
  // The ct-mul key-switch's diagonal (source limb i == target limb i, the
  // same basis): the tensor launches write the exact d2^ here ([L][B][N],
  // limb stride d2hat_ls), the decomposition skips those planes and the
  // key-switch rows read them instead of transforming S (nullptr: off)
  void* d2hat = nullptr;
  uint64_t d2hat_ls = 0;
  // The rotation's sigma_g(c0) read straight from c0 by the key-switch
  // inverse's addend (g^-1 mod 2N, odd; 0: the addend as it is): no
  // separate automorphism launch for c0 (tiled column grids only)
  uint32_t add_ginv = 0;
  size_t src_limbs() const { return Ls ? Ls : L; }
};

// ---- launchers (rnt_kernels.hip), W-dispatched by t->wide ---------------
// All arrays are [limb][poly][N] with an explicit limb stride `*_ls` (words);
// k.B polys (a batch or a chunk of one) and k.L limbs are processed.
// Forward column pass on up to two operands (in0->out0, in1->out1).
// lazy (all three): the product path's Harvey-lazy 30-bit variant (q < 2^30,
// see rnt_modarith.hpp Mod30) where lazy_ok(); the intermediates between
// the three launches are then unreduced, the product's output canonical.
bool lazy_ok(const Tables* t);
hipError_t launch_col_fwd(const Launch& k, void* out0, const void* in0, void* out1,
                          const void* in1, uint64_t in_ls, uint64_t out_ls, bool lazy = false);
// Row pass.  mode 0: forward rows (in place on x); 1: inverse rows (in place
// on x); 2: poly-mul rows: x <- INVrow(FWDrow(x) (.) FWDrow(y) * 2^-w).
hipError_t launch_row(const Launch& k, int mode, void* x, const void* y, uint64_t ls,
                      bool lazy = false);
// The whole-plane product for u32 canonical bases at N = 2^16 (rnt_plane.hip;
// 5 planes of HBM traffic per (poly, limb) instead of the four-step path's
// 9): out = a * b in the coefficient domain (out may alias a or b; scratch:
// one word per output word, a^ in a private layout).
bool plane_ok(const Tables* t);
hipError_t launch_plane_fused(const Launch& k, void* out, const void* a, const void* b, void* scratch, uint64_t ls);
// Scratch slots indexed by the CU a 160-KiB-LDS workgroup runs on (XCC_ID
// and HW_ID bits 15..8): k_plane_fused_slots, k_mf_tensor from this many
// (poly, limb) pairs on.
constexpr uint32_t kPlaneSlots = 1u << 11;
// scratch planes (of N words) launch_plane_fused needs for B L pairs
uint64_t plane_scratch_planes(uint64_t planes);
// The standalone transforms at the same size (rnt_mfma.hip): radix-16 passes
// as i8 matrix products, in place.  mf_supported: u32 bases at N = 2^16;
// mf_build: the per-limb tables into t->mf (0 ok, else err).
inline bool mf_supported(const Tables* t) { return t->plane != 0 && !t->wide && t->log_n == 16; }
int mf_build(Tables* t, std::string* err);
hipError_t launch_mf_ntt(const Launch& k, int inverse, void* data, uint64_t ls);
// The ciphertext tensor product at N = 2^16 on the matrix-core transforms
// (k_mf_tensor, mf_supported bases): coefficient-domain c0, c1, c0', c1' at
// limb stride ils -> NTT-domain d0^, d1^ (Montgomery-scaled key-switch seeds)
// and coefficient-domain d2 at limb stride ols; scratch: plane_scratch_planes(B L)
// planes of N words.
hipError_t launch_mf_tensor(const Launch& k, void* d0, void* d1, void* d2, uint64_t ols, const void* c0,
                            const void* c1, const void* c0p, const void* c1p, uint64_t ils, void* scratch);
// The coefficient-domain product c = a b at N = 2^16 on the matrix-core
// transforms (k_mf_mul, mf_supported bases; in place allowed); scratch:
// plane_scratch_planes(B L) planes of N words.
hipError_t launch_mf_mul(const Launch& k, void* c, const void* a, const void* b, uint64_t ls, void* scratch);
// Whether rnt_mul's row kernel stops its transforms two stages early and
// multiplies degree-3 residues (u32 canonical bases, row length 2^(4k));
// its inverse column pass then takes rfold = 2.
bool mul_truncated(const Tables* t);
// The whole-plane row path at 2^10 <= N <= 2^14 (u32 and u64; rnt_kernels.hip
// k_row<..., WHOLE>): one launch per transform or product, every plane one
// row.  mode 0: forward in place (x); 1: inverse in place (x); 2: out = x * y
// in the coefficient domain (out may alias x or y).  whole_ok: the path serves
// this mode on this basis.
bool whole_ok(const Tables* t, int mode);
hipError_t launch_whole(const Launch& k, int mode, void* out, void* x, const void* y, uint64_t ls);
// Inverse column pass with n^-1 folded into the last stage; rfold adds the
// Montgomery factor 2^w.  addend (optional, coefficient domain, out layout).
// ColRescArgs (tiled grids, log R >= 5, col_resc_ok): limb0 offsets the
// launch's limbs in the basis' tables (in/out point at the first one); with
// `last` ([B][N], the dropped limb's coefficient plane) the output is
// rescaled: (c_l - (c_last mod q_l)) inv[l], inv/invp the rows
// resc_inv_row(t, last limb, 0 / 1) of the rescale table.
struct ColRescArgs {
  const void* last = nullptr;
  const void* inv = nullptr;
  const void* invp = nullptr;
  uint32_t limb0 = 0;
};
hipError_t launch_col_inv(const Launch& k, void* out, uint64_t out_ls, const void* in,
                          uint64_t in_ls, int rfold, const void* addend, bool lazy = false,
                          const ColRescArgs& ra = ColRescArgs{});
bool col_resc_ok(const Tables* t);
const void* resc_inv_row(const Tables* t, size_t last, int which);
// Elementwise over k.L*k.B*N contiguous words: op 0 add, 1 sub, 2 neg,
// 3 pointwise mul (canonical a*b mod q), 4 Montgomery product (a*b*2^-w).
hipError_t launch_elementwise(const Launch& k, int op, void* out, const void* a,
                              const void* b);
// Plain device copy of `bytes` (16-byte aligned pointers, bytes % 16 == 0):
// every lane moves 4 x 16 B, loads before stores (Clone, rnt_copy).
hipError_t launch_copy(hipStream_t s, void* dst, const void* src, uint64_t bytes);
// k.L = limbs of the input; output has k.L - 1 (same poly count / stride B*N).
hipError_t launch_rescale(const Launch& k, void* out, const void* in);
// Centred CRT of every coefficient (coefficient-domain `in`, k.L limbs) into
// `out_words` 64-bit two's-complement words each ([B][N][out_words]);
// `consts` points to a host CrtConsts of device arrays, mw = 32-bit words of Q.
hipError_t launch_crt(const Launch& k, uint64_t* out, const void* in, const void* consts,
                      uint32_t mw, uint32_t out_words);
// out limb l = (in_l - (last mod q_l)) * inv[l] (Shoup pair inv/invp, device
// arrays of k.L words); `last` is a [B][N] plane of residues mod q_last.
hipError_t launch_rescale_ext(const Launch& k, void* out, const void* in, const void* last,
                              const void* inv, const void* invp);
hipError_t launch_automorphism(const Launch& k, void* out, const void* in, uint64_t g);
// host u64 [B][L][N] staging <-> device; err_index receives the smallest
// offending flat index (UINT64_MAX if none) for non-reduced input.
hipError_t launch_import(const Launch& k, void* dst, const uint64_t* stage, int to_brv,
                         unsigned long long* err_index);
hipError_t launch_import_coeffs(const Launch& k, void* dst, const int64_t* stage);
// k.B polys starting at src; ls = limb stride in words (0: k.B * N)
hipError_t launch_export(const Launch& k, uint64_t* stage, const void* src, int from_brv,
                         uint64_t ls = 0);
// Key-switch pieces.  S: [L_target][L_source][k.B][N] scratch (chunk-local).
hipError_t launch_ks_decompose(const Launch& k, void* S, const void* d, uint64_t d_ls);
// u0 rows <- INVrow(sum_i FWDrow(S[j][i]) (.) key_b[i][j] (+ init0)), u1 with
// key_a.  init0/init1 may be null (NTT-domain rows, Montgomery-scaled).
hipError_t launch_ks_rows(const Launch& k, void* u0, void* u1, uint64_t u_ls, const void* S,
                          const void* key_a, const void* key_b, uint64_t key_ls,
                          const void* init0, const void* init1, uint64_t init_ls);
// The whole-plane key-switch at 2^10 <= N <= 2^13 (k_ks_whole, one launch,
// no S): out0 = INV(sum_i NTT(src_i mod q_j) (.) key_b[i][j] + init0) (+ add0),
// out1 likewise with key_a; src is [k.src_limbs()][k.B][N] coefficient-domain
// at limb stride src_ls, out0/out1/add0 at out_ls, init0/init1 (NTT domain,
// Montgomery-scaled, may be null) at init_ls.  ks_whole_ok: it serves this basis.
bool ks_whole_ok(const Tables* t);
hipError_t launch_ks_whole(const Launch& k, void* out0, void* out1, uint64_t out_ls, const void* src,
                           uint64_t src_ls, const void* key_a, const void* key_b, uint64_t key_ls,
                           const void* init0, const void* init1, uint64_t init_ls, const void* add0);
// Tensor rows for ct x ct: inputs are column-transformed c0,c1,c0p,c1p.
// Writes d0hat, d1hat (NTT rows, Montgomery-scaled) and the inverse-row
// output of d2 into d2row.  All arrays share limb stride ls.
// The whole-plane tensor (k_tensor_rows<..., WHOLE>, 2^10 <= N <= 2^13;
// u64 bases N <= 2^12): coefficient-domain c0, c1, c0', c1' -> NTT-domain
// d0^, d1^ and coefficient-domain d2 in one launch.
bool tensor_whole_ok(const Tables* t);
hipError_t launch_tensor_whole(const Launch& k, void* d0hat, void* d1hat, void* d2, uint64_t ls,
                               const void* c0, const void* c1, const void* c0p, const void* c1p,
                               uint64_t in_ls);
hipError_t launch_tensor_rows(const Launch& k, void* d0hat, void* d1hat, void* d2row,
                              const void* c0, const void* c1, const void* c0p,
                              const void* c1p, uint64_t ls);
// Device samplers (rnt_sample.hip): kind 0 uniform residues, 1 rounded
// Gaussian (sigma), 2 ternary with exactly `hamming_weight` nonzeros; every
// poly of `out` ([k.L][k.B][N], limb stride k.B * N) in the coefficient domain.
struct SampleKey {
  uint32_t k0, k1;  // Philox key: seed low word, seed high word ^ stream high word
  uint32_t stream;  // stream low word (a counter word)
};
hipError_t launch_sample(const Launch& k, int kind, void* out, SampleKey s, double sigma,
                         uint32_t hamming_weight);
// CKKS canonical embedding (rnt_encode.hip).  Twiddle table: N/2 complex
// doubles (interleaved re, im).  encode: values [B][n_values] double2 ->
// coeffs [B][N] i64 (work: [B][N/2] double2); decode: centred i64 coeffs
// [B][N] -> work [B][N/2] double2 slots / 2^scale_bits.
bool sfft_supported(uint32_t log_n);
std::vector<double> sfft_twiddles(uint32_t log_n);
hipError_t launch_sfft_encode(const Launch& k, int64_t* coeffs, void* work, const void* values,
                              uint32_t n_values, uint32_t scale_bits, const void* tw);
hipError_t launch_sfft_decode(const Launch& k, void* work, const int64_t* coeffs,
                              uint32_t scale_bits, const void* tw);

}  // namespace rnt
