// rns_ntt.hpp -- C++ host mirror of the reference's RNS ring backend over
// the C-ABI (include/rnsntt.h).
//
// The reference is Rust (src/rings/backends/rns_ntt/{basis,poly}.rs); with no
// Rust toolchain in this image the host side above the ABI is C++ with the
// reference's names and meanings:
//   Arc<RnsBasis<N>>            -> std::shared_ptr<RnsBasis<N>> (BasisRef<N>)
//   RnsPoly<N> (+=, *=, Neg)    -> RnsPoly<N> (+=, *=, unary -)
//   channels() -> &[[u64; N]]   -> const std::vector<std::array<uint64_t, N>>&
//                                  (a host mirror synced lazily from HBM)
//   RnsNttResult<T> / errors    -> return T, or throw RnsNttError{kind}
//   debug_assert (domain/basis) -> RnsNttError{DomainMismatch/BasisMismatch}
// Every ring operation runs on the GPU through librnsntt; there is no host
// arithmetic path (the schoolbook product the reference keeps for its tests
// lives in the tests).
#pragma once

#include <array>
#include <cmath>
#include <complex>
#include <cstdint>
#include <memory>
#include <optional>
#include <random>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "rnsntt.h"

namespace rns_ntt {

// errors.rs:4-20 (+ the ABI's device / argument failures)
enum class RnsNttErrorKind {
  InvalidDegree = RNT_ERR_INVALID_DEGREE,
  EmptyBasis = RNT_ERR_EMPTY_BASIS,
  NonNttFriendlyModulus = RNT_ERR_NON_NTT_FRIENDLY,
  InvalidModDrop = RNT_ERR_INVALID_MOD_DROP,
  ChannelCountMismatch = RNT_ERR_CHANNEL_COUNT,
  NonReducedCoefficient = RNT_ERR_NON_REDUCED,
  DomainMismatch = RNT_ERR_DOMAIN_MISMATCH,
  BasisMismatch = RNT_ERR_BASIS_MISMATCH,
  Device = RNT_ERR_DEVICE,
  OutOfMemory = RNT_ERR_OUT_OF_MEMORY,
  BadArgument = RNT_ERR_BAD_ARGUMENT,
  Unsupported = RNT_ERR_UNSUPPORTED,  // beyond the backend's capacity (N > 2^17)
};

// The variant and its fields, as the reference's struct variants carry them
// (InvalidDegree{degree}, NonNttFriendlyModulus{modulus, degree},
// InvalidModDrop{drop_count, channel_count}, ChannelCountMismatch{expected,
// actual}, NonReducedCoefficient{coefficient, modulus}); fields a variant
// does not have stay 0.
class RnsNttError : public std::runtime_error {
 public:
  RnsNttError(int status, const char* msg, uint64_t f0 = 0, uint64_t f1 = 0)
      : std::runtime_error(std::string(rnt_status_string(status)) + ": " + (msg ? msg : "")),
        kind((RnsNttErrorKind)status) {
    switch (kind) {
      case RnsNttErrorKind::InvalidDegree: degree = f0; break;
      case RnsNttErrorKind::NonNttFriendlyModulus: modulus = f0; degree = f1; break;
      case RnsNttErrorKind::InvalidModDrop: drop_count = f0; channel_count = f1; break;
      case RnsNttErrorKind::ChannelCountMismatch: expected = f0; actual = f1; break;
      case RnsNttErrorKind::NonReducedCoefficient: coefficient = f0; modulus = f1; break;
      case RnsNttErrorKind::Unsupported: degree = f0; max_degree = f1; break;
      default: break;
    }
  }
  RnsNttErrorKind kind;
  uint64_t degree = 0, modulus = 0, drop_count = 0, channel_count = 0, expected = 0, actual = 0,
           coefficient = 0, max_degree = 0;
};

// Throws the failing call's variant with the fields rnt_last_error_detail
// reports for it.
inline void check(int status) {
  if (status == RNT_OK) return;
  uint64_t f[2] = {0, 0};
  if (rnt_last_error_detail(f) != status) f[0] = f[1] = 0;
  throw RnsNttError(status, rnt_last_error(), f[0], f[1]);
}

template <size_t N>
class RnsBasis;
template <size_t N>
using BasisRef = std::shared_ptr<const RnsBasis<N>>;

inline uint32_t log2_exact(size_t n) {
  uint32_t l = 0;
  while (((size_t)1 << l) < n) ++l;
  return l;
}

// RnsBasis<N> (basis.rs:90-180): the moduli and their device NTT tables.
template <size_t N>
class RnsBasis : public std::enable_shared_from_this<RnsBasis<N>> {
 public:
  // RnsBasis::new (basis.rs:97-106): InvalidDegree / EmptyBasis /
  // NonNttFriendlyModulus like the reference.
  static BasisRef<N> create(const std::vector<uint64_t>& moduli, int device = 0) {
    if (moduli.empty())  // basis.rs:98-100 comes before NttTable::new's degree check
      throw RnsNttError(RNT_ERR_EMPTY_BASIS, "RNS basis must contain at least one modulus");
    if (((size_t)1 << log2_exact(N)) != N)
      throw RnsNttError(RNT_ERR_INVALID_DEGREE, "N is not a power of two", N);
    rnt_ctx* c = nullptr;
    check(rnt_ctx_create(log2_exact(N), moduli.data(), moduli.size(), device, &c));
    return BasisRef<N>(new RnsBasis(c));
  }
  ~RnsBasis() { rnt_ctx_destroy(ctx_); }
  RnsBasis(const RnsBasis&) = delete;
  RnsBasis& operator=(const RnsBasis&) = delete;

  std::vector<uint64_t> moduli() const {
    std::vector<uint64_t> m(channel_count());
    check(rnt_ctx_moduli(ctx_, m.data()));
    return m;
  }
  size_t channel_count() const {
    size_t l = 0;
    check(rnt_ctx_channel_count(ctx_, &l));
    return l;
  }
  uint32_t total_bits() const {
    uint32_t b = 0;
    check(rnt_ctx_total_bits(ctx_, &b));
    return b;
  }
  uint64_t psi(size_t limb) const {
    uint64_t p = 0;
    check(rnt_ctx_psi(ctx_, limb, &p));
    return p;
  }
  // drop_last (basis.rs:121-134): InvalidModDrop if nothing would remain
  BasisRef<N> drop_last(size_t k) const {
    rnt_ctx* c = nullptr;
    check(rnt_ctx_drop_last(ctx_, k, &c));
    return BasisRef<N>(new RnsBasis(c));
  }
  rnt_ctx* ctx() const { return ctx_; }
  void sync() const { check(rnt_sync(ctx_)); }
  // hipStream_t the ops are queued on; set_stream(nullptr) restores the own one
  void* stream() const {
    void* s = nullptr;
    check(rnt_ctx_stream(ctx_, &s));
    return s;
  }
  void set_stream(void* s) const { check(rnt_ctx_set_stream(ctx_, s)); }

 private:
  explicit RnsBasis(rnt_ctx* c) : ctx_(c) {}
  rnt_ctx* ctx_;
};

// RnsPoly<N> (poly.rs:25-570): one polynomial resident in HBM.
template <size_t N>
class RnsPoly {
 public:
  using Channel = std::array<uint64_t, N>;

  // zero (poly.rs:36-43)
  static RnsPoly zero(BasisRef<N> basis) { return RnsPoly(std::move(basis)); }

  // from_coeffs (poly.rs:49-67): rem_euclid per channel
  static RnsPoly from_coeffs(const std::vector<int64_t>& coeffs, BasisRef<N> basis) {
    if (coeffs.size() < N) throw std::invalid_argument("from_coeffs: fewer than N coefficients");
    RnsPoly p(std::move(basis));
    check(rnt_upload_coeffs(p.buf_, coeffs.data(), 1));
    return p;
  }
  static RnsPoly from_coeffs(const std::array<int64_t, N>& coeffs, BasisRef<N> basis) {
    return from_coeffs(std::vector<int64_t>(coeffs.begin(), coeffs.end()), std::move(basis));
  }

  // from_channels (poly.rs:73-99): ChannelCountMismatch / NonReducedCoefficient
  static RnsPoly from_channels(const std::vector<Channel>& channels, BasisRef<N> basis, bool in_ntt) {
    RnsPoly p(std::move(basis));
    check(rnt_upload(p.buf_, channels.empty() ? nullptr : channels[0].data(), 1, channels.size(),
                     in_ntt ? 1 : 0));
    p.host_ = channels;
    return p;
  }

  // Clone (a device copy)
  RnsPoly(const RnsPoly& o) : RnsPoly(o.basis_) {
    check(rnt_copy(buf_, o.buf_));
    host_ = o.host_;
  }
  RnsPoly(RnsPoly&& o) noexcept : basis_(std::move(o.basis_)), buf_(o.buf_), host_(std::move(o.host_)) {
    o.buf_ = nullptr;
  }
  RnsPoly& operator=(RnsPoly&& o) noexcept {
    std::swap(basis_, o.basis_);
    std::swap(buf_, o.buf_);
    std::swap(host_, o.host_);
    return *this;
  }
  RnsPoly& operator=(const RnsPoly&) = delete;
  ~RnsPoly() {
    if (buf_) rnt_buf_free(buf_);
  }

  // channels (poly.rs:119-121): the current domain (natural order if NTT)
  const std::vector<Channel>& channels() const {
    if (!host_) {
      std::vector<Channel> h(basis_->channel_count());
      check(rnt_download(buf_, h.empty() ? nullptr : h[0].data(), 1));
      host_ = std::move(h);
    }
    return *host_;
  }
  bool is_ntt_domain() const {
    int f = 0;
    check(rnt_buf_is_ntt(buf_, &f));
    return f != 0;
  }
  const BasisRef<N>& basis() const { return basis_; }
  rnt_buf* handle() const { return buf_; }

  // to_ntt_domain / to_coeff_domain (poly.rs:136-166), no-ops when there
  void to_ntt_domain() {
    check(rnt_ntt_fwd(buf_));
    host_.reset();
  }
  void to_coeff_domain() {
    check(rnt_ntt_inv(buf_));
    host_.reset();
  }

  // AddAssign / MulAssign (poly.rs:254-331), Neg (:370-385)
  RnsPoly& operator+=(const RnsPoly& rhs) {
    check(rnt_add(buf_, buf_, rhs.buf_));
    host_.reset();
    return *this;
  }
  RnsPoly& operator*=(const RnsPoly& rhs) {
    check(rnt_mul(buf_, buf_, rhs.buf_));
    host_.reset();
    return *this;
  }
  RnsPoly operator-() const {
    RnsPoly out(basis_);
    check(rnt_neg(out.buf_, buf_));
    return out;
  }

  // rescale_into / rescale (poly.rs:187-249): coefficient-domain result
  RnsPoly rescale_into(BasisRef<N> new_basis) const {
    RnsPoly out(std::move(new_basis));
    check(rnt_rescale(out.buf_, buf_));
    return out;
  }
  RnsPoly rescale() const {
    if (basis_->channel_count() < 2)
      throw RnsNttError(RNT_ERR_INVALID_MOD_DROP, "rescale needs at least two channels", 1,
                        basis_->channel_count());
    return rescale_into(basis_->drop_last(1));
  }
  // mod_drop_last (poly.rs:169-177)
  RnsPoly mod_drop_last(size_t k) const {
    RnsPoly out(basis_->drop_last(k));
    check(rnt_mod_drop_last(out.buf_, buf_));
    return out;
  }

  // automorphism / rotate_slots (poly.rs:492-569)
  RnsPoly automorphism(uint64_t g) const {
    RnsPoly out(basis_);
    check(rnt_automorphism(out.buf_, buf_, g));
    return out;
  }
  RnsPoly rotate_slots(int32_t k) const {
    RnsPoly out(basis_);
    check(rnt_rotate_slots(out.buf_, buf_, k));
    return out;
  }

  // PolyRing::to_coeffs (poly.rs:404-427): centred CRT on the device
  std::array<int64_t, N> to_coeffs() const {
    std::array<int64_t, N> out{};
    check(rnt_to_coeffs(buf_, out.data(), 1));
    return out;
  }

  // PolySampler (traits.rs:74-127; poly.rs:438-477), sampled on the
  // device (rnt_sample_*, Philox4x32-10).  The caller's Rng supplies only a
  // 64-bit seed per call, so a seeded Rng fixes every sample, as in the
  // reference; its ChaCha20 sample values are not reproduced.
  template <class Rng>
  static RnsPoly sample_uniform(const BasisRef<N>& basis, Rng& rng) {
    RnsPoly p(basis);
    check(rnt_sample_uniform(p.buf_, draw_seed(rng), 0));
    return p;
  }
  // sample_tribits: exactly hamming_weight coefficients +-1; a weight above
  // N is a panic in the reference (sampling.rs:71-80), BadArgument here
  template <class Rng>
  static RnsPoly sample_tribits(size_t hamming_weight, const BasisRef<N>& basis, Rng& rng) {
    RnsPoly p(basis);
    check(rnt_sample_ternary(p.buf_, hamming_weight, draw_seed(rng), 0));
    return p;
  }
  template <class Rng>
  static RnsPoly sample_gaussian(double std_dev, const BasisRef<N>& basis, Rng& rng) {
    RnsPoly p(basis);
    check(rnt_sample_gaussian(p.buf_, std_dev, draw_seed(rng), 0));
    return p;
  }
  // sample_noise (poly.rs:471-477): Gaussian with std_dev = sqrt(variance)
  template <class Rng>
  static RnsPoly sample_noise(double variance, const BasisRef<N>& basis, Rng& rng) {
    return sample_gaussian(std::sqrt(variance), basis, rng);
  }

 private:
  template <size_t M>
  friend class CkksEncoder;
  explicit RnsPoly(BasisRef<N> basis) : basis_(std::move(basis)) {
    check(rnt_buf_alloc(basis_->ctx(), 1, &buf_));
  }
  template <class Rng>
  static uint64_t draw_seed(Rng& rng) {
    return std::uniform_int_distribution<uint64_t>()(rng);
  }
  void touch() { host_.reset(); }
  BasisRef<N> basis_;
  rnt_buf* buf_ = nullptr;
  mutable std::optional<std::vector<Channel>> host_;
};

// Plaintext (crypto/types.rs): an encoded polynomial, its scale and slot count.
template <size_t N>
struct Plaintext {
  RnsPoly<N> poly;
  uint32_t scale_bits;
  size_t slots;
};

// CkksEncoder<DEGREE> (ckks_encoder.rs:32-157).  The canonical embedding
// runs on the device (rnt_encode / rnt_decode: the O(N log N) special FFT
// in f64) instead of the reference's O(N^2) Vandermonde sums.
template <size_t N>
class CkksEncoder {
 public:
  explicit CkksEncoder(uint32_t scale_bits) : scale_bits_(scale_bits) {
    if (((size_t)1 << log2_exact(N)) != N) throw std::invalid_argument("CkksEncoder: DEGREE must be a power of two");
    if (scale_bits == 0) throw std::invalid_argument("CkksEncoder: scale_bits must be positive");
  }
  double scale_factor() const { return std::ldexp(1.0, (int)scale_bits_); }
  size_t max_slots() const { return N / 2; }

  // encode (ckks_encoder.rs:65-82) / encode_complex (:85-99); more than N/2
  // values is a panic in the reference, std::invalid_argument here
  Plaintext<N> encode(const std::vector<double>& values, BasisRef<N> basis) const {
    std::vector<std::complex<double>> c(values.begin(), values.end());
    return encode_complex(c, std::move(basis), "encode");
  }
  Plaintext<N> encode_complex(const std::vector<std::complex<double>>& values, BasisRef<N> basis,
                              const char* name = "encode_complex") const {
    if (values.size() > N / 2)
      throw std::invalid_argument(std::string(name) + ": " + std::to_string(values.size()) +
                                  " values exceed max slots " + std::to_string(N / 2));
    RnsPoly<N> p(std::move(basis));
    check(rnt_encode(p.buf_, reinterpret_cast<const double*>(values.data()), values.size(), scale_bits_));
    return Plaintext<N>{std::move(p), scale_bits_, values.size()};
  }

  // decode (:129-131) / decode_complex (:134-156)
  std::vector<double> decode(const Plaintext<N>& pt) const {
    std::vector<double> out;
    for (const auto& z : decode_complex(pt)) out.push_back(z.real());
    return out;
  }
  std::vector<std::complex<double>> decode_complex(const Plaintext<N>& pt) const {
    std::vector<std::complex<double>> out(pt.slots);
    check(rnt_decode(pt.poly.handle(), reinterpret_cast<double*>(out.data()), pt.slots, pt.scale_bits));
    return out;
  }

 private:
  uint32_t scale_bits_;
};

}  // namespace rns_ntt
