// test_rns_poly.cpp -- the reference's RnsPoly unit tests
// (src/rings/backends/rns_ntt/poly.rs:658-1060) against the C++ host mirror
// (toy-heaan-ckks_amd/host/rns_ntt.hpp), every op on the GPU.  Names and
// assertions follow the Rust tests one for one; the RNG-driven tests keep
// their distributional checks (the ChaCha20 streams are not reproduced).
//
// Build: __graft_entry__.build() -> tests/cpp/bin/test_rns_poly; run by
// tests/test_cpp_host.py (-m gpu).  Exit status = number of failed tests.
#include <cmath>
#include <complex>
#include <cstdio>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "rns_ntt.hpp"

using namespace rns_ntt;
using Poly = RnsPoly<8>;

static int g_failed = 0, g_run = 0;
#define CHECK(cond)                                                                 \
  do {                                                                              \
    if (!(cond)) throw std::runtime_error(std::string("CHECK failed: ") + #cond);   \
  } while (0)

static void run(const char* name, const std::function<void()>& f) {
  ++g_run;
  try {
    f();
    std::printf("ok   %s\n", name);
  } catch (const std::exception& e) {
    ++g_failed;
    std::printf("FAIL %s: %s\n", name, e.what());
  }
}

static BasisRef<8> basis_17_97() { return RnsBasis<8>::create({17, 97}); }
static BasisRef<8> basis_three() { return RnsBasis<8>::create({17, 97, 113}); }

template <class F>
static bool throws_kind(F&& f, RnsNttErrorKind kind) {
  try {
    f();
  } catch (const RnsNttError& e) {
    return e.kind == kind;
  }
  return false;
}

// the error a call throws (kind None-equivalent: BadArgument if none)
template <class F>
static RnsNttError caught(F&& f) {
  try {
    f();
  } catch (const RnsNttError& e) {
    return e;
  }
  return RnsNttError(RNT_ERR_BAD_ARGUMENT, "no error thrown");
}

// the reference's mul_assign_naive (poly.rs:339-367): schoolbook negacyclic
// product per channel -- a test-side helper, as in the reference
static std::vector<Poly::Channel> mul_naive(const Poly& a, const Poly& b) {
  const auto mods = a.basis()->moduli();
  std::vector<Poly::Channel> out(mods.size());
  for (size_t l = 0; l < mods.size(); ++l) {
    const unsigned __int128 q = mods[l];
    out[l].fill(0);
    for (size_t i = 0; i < 8; ++i)
      for (size_t j = 0; j < 8; ++j) {
        const uint64_t p = (uint64_t)((unsigned __int128)a.channels()[l][i] * b.channels()[l][j] % q);
        const size_t k = (i + j) % 8;
        if (i + j < 8)
          out[l][k] = (uint64_t)((out[l][k] + (unsigned __int128)p) % q);
        else
          out[l][k] = (uint64_t)((out[l][k] + q - p) % q);
      }
  }
  return out;
}

int main() {
  // ── Construction ──────────────────────────────────────────────────────────
  run("zero_poly_is_all_zeros", [] {
    Poly poly = Poly::zero(basis_17_97());
    for (auto& ch : poly.channels())
      for (auto c : ch) CHECK(c == 0);
    CHECK(!poly.is_ntt_domain());
  });
  run("from_coeffs_reduces_correctly", [] {
    Poly poly = Poly::from_coeffs(std::array<int64_t, 8>{-1, 2, -3, 4, 0, 0, 0, 0}, basis_17_97());
    CHECK(poly.channels()[0][0] == 16);
    CHECK(poly.channels()[0][1] == 2);
    CHECK(poly.channels()[0][2] == 14);
    CHECK(poly.channels()[1][0] == 96);
  });
  run("from_channels_rejects_unreduced_coefficient", [] {
    std::vector<Poly::Channel> bad(2);
    bad[0].fill(17);
    bad[1].fill(0);
    CHECK(throws_kind([&] { Poly::from_channels(bad, basis_17_97(), false); },
                      RnsNttErrorKind::NonReducedCoefficient));
  });
  run("from_channels_rejects_wrong_channel_count", [] {
    std::vector<Poly::Channel> too_few(1);
    too_few[0].fill(0);
    CHECK(throws_kind([&] { Poly::from_channels(too_few, basis_17_97(), false); },
                      RnsNttErrorKind::ChannelCountMismatch));
  });
  // ── NTT roundtrip ─────────────────────────────────────────────────────────
  run("ntt_roundtrip_preserves_coefficients", [] {
    Poly poly = Poly::from_coeffs(std::array<int64_t, 8>{1, -2, 3, 4, -5, 6, 7, -8}, basis_17_97());
    const auto original = poly.channels();
    poly.to_ntt_domain();
    CHECK(poly.is_ntt_domain());
    poly.to_coeff_domain();
    CHECK(!poly.is_ntt_domain());
    CHECK(poly.channels() == original);
  });
  run("to_ntt_is_idempotent", [] {
    Poly poly = Poly::from_coeffs(std::array<int64_t, 8>{1, 2, 3, 4, 5, 6, 7, 8}, basis_17_97());
    poly.to_ntt_domain();
    const auto after_first = poly.channels();
    poly.to_ntt_domain();
    CHECK(poly.channels() == after_first);
  });
  // ── Mod-drop ──────────────────────────────────────────────────────────────
  run("mod_drop_removes_last_channels", [] {
    Poly poly = Poly::from_coeffs(std::array<int64_t, 8>{1, 2, 3, 4, 5, 6, 7, 8}, basis_three());
    Poly dropped = poly.mod_drop_last(1);
    CHECK(dropped.basis()->channel_count() == 2);
    CHECK(dropped.channels().size() == 2);
  });
  // ── Arithmetic ────────────────────────────────────────────────────────────
  run("add_assign_computes_correct_sum", [] {
    auto basis = basis_17_97();
    Poly a = Poly::from_coeffs(std::array<int64_t, 8>{1, 2, 3, 4, 5, 6, 7, 8}, basis);
    Poly b = Poly::from_coeffs(std::array<int64_t, 8>{8, 7, 6, 5, 4, 3, 2, 1}, basis);
    a += b;
    for (auto c : a.channels()[0]) CHECK(c == 9);
    for (auto c : a.channels()[1]) CHECK(c == 9);
  });
  run("add_assign_wraps_at_modulus", [] {
    auto basis = basis_17_97();
    Poly a = Poly::from_coeffs(std::array<int64_t, 8>{16, 0, 0, 0, 0, 0, 0, 0}, basis);
    Poly b = Poly::from_coeffs(std::array<int64_t, 8>{2, 0, 0, 0, 0, 0, 0, 0}, basis);
    a += b;
    CHECK(a.channels()[0][0] == 1);
  });
  run("neg_negates_coefficients", [] {
    Poly poly = Poly::from_coeffs(std::array<int64_t, 8>{3, 0, 0, 0, 0, 0, 0, 0}, basis_17_97());
    Poly neg = -poly;
    CHECK(neg.channels()[0][0] == 14);
    CHECK(neg.channels()[0][1] == 0);
  });
  run("mul_assign_schoolbook_small", [] {
    auto basis = basis_17_97();
    Poly a = Poly::from_coeffs(std::array<int64_t, 8>{1, 1, 0, 0, 0, 0, 0, 0}, basis);
    Poly b = Poly::from_coeffs(std::array<int64_t, 8>{1, 1, 0, 0, 0, 0, 0, 0}, basis);
    a *= b;
    const auto coeffs = a.to_coeffs();
    CHECK(coeffs[0] == 1 && coeffs[1] == 2 && coeffs[2] == 1);
    for (size_t i = 3; i < 8; ++i) CHECK(coeffs[i] == 0);
  });
  run("mul_assign_wraps_around_quotient", [] {
    auto basis = basis_17_97();
    Poly a = Poly::from_coeffs(std::array<int64_t, 8>{0, 0, 0, 0, 0, 0, 0, 1}, basis);
    Poly b = Poly::from_coeffs(std::array<int64_t, 8>{0, 1, 0, 0, 0, 0, 0, 0}, basis);
    a *= b;
    const auto coeffs = a.to_coeffs();
    CHECK(coeffs[0] == -1);
    for (size_t i = 1; i < 8; ++i) CHECK(coeffs[i] == 0);
  });
  // ── PolyRing trait ────────────────────────────────────────────────────────
  run("to_coeffs_roundtrips_from_coeffs", [] {
    const std::array<int64_t, 8> input{1, -2, 3, -4, 5, -6, 7, -8};
    CHECK(Poly::from_coeffs(input, basis_17_97()).to_coeffs() == input);
  });
  run("to_coeffs_works_from_ntt_domain", [] {
    const std::array<int64_t, 8> input{1, -2, 3, -4, 5, -6, 7, -8};
    Poly poly = Poly::from_coeffs(input, basis_17_97());
    poly.to_ntt_domain();
    CHECK(poly.to_coeffs() == input);
    CHECK(poly.is_ntt_domain());
  });
  // ── PolySampler trait ─────────────────────────────────────────────────────
  run("sample_uniform_stays_in_range", [] {
    auto basis = basis_17_97();
    std::mt19937_64 rng(42);
    Poly poly = Poly::sample_uniform(basis, rng);
    const auto mods = basis->moduli();
    for (size_t l = 0; l < mods.size(); ++l)
      for (auto c : poly.channels()[l]) CHECK(c < mods[l]);
  });
  run("mul_assign_ntt_domain_matches_coeff_domain", [] {
    auto basis = basis_17_97();
    const std::array<int64_t, 8> ac{1, -2, 3, -4, 5, -6, 7, -8}, bc{2, 1, -1, 3, 0, -2, 4, 1};
    Poly a_coeff = Poly::from_coeffs(ac, basis);
    a_coeff *= Poly::from_coeffs(bc, basis);
    const auto expected = a_coeff.to_coeffs();
    Poly a_ntt = Poly::from_coeffs(ac, basis), b_ntt = Poly::from_coeffs(bc, basis);
    a_ntt.to_ntt_domain();
    b_ntt.to_ntt_domain();
    a_ntt *= b_ntt;
    CHECK(a_ntt.is_ntt_domain());
    CHECK(a_ntt.to_coeffs() == expected);
  });
  run("automorphism_identity_preserves_coefficients", [] {
    const std::array<int64_t, 8> coeffs{1, 2, 3, 4, 5, 6, 7, 8};
    Poly poly = Poly::from_coeffs(coeffs, basis_17_97());
    CHECK(poly.automorphism(1).to_coeffs() == coeffs);
    CHECK(poly.automorphism(16).to_coeffs() == coeffs);
  });
  run("automorphism_applies_sign_change_correctly", [] {
    Poly poly = Poly::from_coeffs(std::array<int64_t, 8>{1, 1, 0, 0, 0, 0, 0, 0}, basis_17_97());
    const auto result = poly.automorphism(9).to_coeffs();
    CHECK(result[0] == 1 && result[1] == -1);
    for (size_t i = 2; i < 8; ++i) CHECK(result[i] == 0);
  });
  run("rotate_slots_works_for_simple_case", [] {
    Poly poly = Poly::from_coeffs(std::array<int64_t, 8>{1, 0, 2, 0, 3, 0, 4, 0}, basis_17_97());
    CHECK(poly.rotate_slots(1).to_coeffs().size() == 8);
  });
  run("rotate_slots_negative_uses_conjugate", [] {
    Poly poly = Poly::from_coeffs(std::array<int64_t, 8>{1, 2, 3, 4, 5, 6, 7, 8}, basis_17_97());
    CHECK(poly.rotate_slots(-1).to_coeffs().size() == 8);
  });
  run("automorphism_preserves_ntt_domain_flag", [] {
    Poly poly = Poly::from_coeffs(std::array<int64_t, 8>{1, 2, 3, 4, 5, 6, 7, 8}, basis_17_97());
    poly.to_ntt_domain();
    CHECK(poly.is_ntt_domain());
    CHECK(!poly.automorphism(3).is_ntt_domain());
  });
  run("mul_assign_matches_naive", [] {
    auto basis = basis_17_97();
    const std::array<int64_t, 8> ac{3, 1, -2, 0, 4, -1, 2, -3}, bc{1, -1, 0, 2, -2, 3, 1, -1};
    Poly a_ntt = Poly::from_coeffs(ac, basis);
    Poly b = Poly::from_coeffs(bc, basis);
    const auto naive = mul_naive(a_ntt, b);
    a_ntt *= b;
    CHECK(a_ntt.channels() == naive);
  });
  run("sample_tribits_has_correct_hamming_weight", [] {
    std::mt19937_64 rng(7);
    Poly poly = Poly::sample_tribits(3, basis_17_97(), rng);
    size_t nz = 0;
    for (auto c : poly.channels()[0]) nz += c != 0;
    CHECK(nz == 3);
  });
  // ── Rescale ───────────────────────────────────────────────────────────────
  run("rescale_drops_channel_count", [] {
    Poly poly = Poly::from_coeffs(std::array<int64_t, 8>{1, 2, 3, 4, 5, 6, 7, 8}, basis_three());
    Poly r = poly.rescale();
    CHECK(r.basis()->channel_count() == 2);
    CHECK(r.channels().size() == 2);
    CHECK(!r.is_ntt_domain());
  });
  run("rescale_on_single_channel_errors", [] {
    Poly poly = Poly::from_coeffs(std::array<int64_t, 8>{1, 2, 3, 4, 5, 6, 7, 8},
                                  RnsBasis<8>::create({17}));
    CHECK(throws_kind([&] { poly.rescale(); }, RnsNttErrorKind::InvalidModDrop));
  });
  run("rescale_is_exact_division_by_last_prime", [] {
    std::vector<int64_t> coeffs(8, 113 * 2);
    const auto out = Poly::from_coeffs(coeffs, basis_three()).rescale().to_coeffs();
    for (auto x : out) CHECK(x == 2);
  });
  run("rescale_from_ntt_domain_matches_coeff_domain", [] {
    auto basis = basis_three();
    const std::array<int64_t, 8> c{3, -1, 2, 0, -4, 5, -2, 1};
    const auto expected = Poly::from_coeffs(c, basis).rescale().to_coeffs();
    Poly p = Poly::from_coeffs(c, basis);
    p.to_ntt_domain();
    CHECK(p.rescale().to_coeffs() == expected);
  });
  // ── boundary checks the reference only debug_asserts ─────────────────────
  run("mixed_domains_are_rejected", [] {
    auto basis = basis_17_97();
    Poly a = Poly::from_coeffs(std::array<int64_t, 8>{1, 2, 3, 4, 5, 6, 7, 8}, basis);
    Poly b = Poly::from_coeffs(std::array<int64_t, 8>{1, 2, 3, 4, 5, 6, 7, 8}, basis);
    b.to_ntt_domain();
    CHECK(throws_kind([&] { a *= b; }, RnsNttErrorKind::DomainMismatch));
  });
  run("different_bases_are_rejected", [] {
    Poly a = Poly::from_coeffs(std::array<int64_t, 8>{1, 0, 0, 0, 0, 0, 0, 0}, basis_17_97());
    Poly b = Poly::from_coeffs(std::array<int64_t, 8>{1, 0, 0, 0, 0, 0, 0, 0}, basis_17_97());
    CHECK(throws_kind([&] { a += b; }, RnsNttErrorKind::BasisMismatch));
  });
  run("basis_validation_matches_reference", [] {
    CHECK(throws_kind([] { RnsBasis<8>::create({}); }, RnsNttErrorKind::EmptyBasis));
    CHECK(throws_kind([] { RnsBasis<8>::create({19}); }, RnsNttErrorKind::NonNttFriendlyModulus));
  });

  run("error_variants_carry_reference_fields", [] {
    // errors.rs:4-20: the struct variants' payloads cross the C-ABI
    // (rnt_last_error_detail) and come back with the reference's meaning
    std::vector<Poly::Channel> bad(2);
    bad[0].fill(3);
    bad[0][5] = 17;
    bad[1].fill(0);
    auto e = caught([&] { Poly::from_channels(bad, basis_17_97(), false); });
    CHECK(e.kind == RnsNttErrorKind::NonReducedCoefficient && e.coefficient == 17 && e.modulus == 17);
    std::vector<Poly::Channel> one(1);
    one[0].fill(0);
    e = caught([&] { Poly::from_channels(one, basis_17_97(), false); });
    CHECK(e.kind == RnsNttErrorKind::ChannelCountMismatch && e.expected == 2 && e.actual == 1);
    e = caught([] { RnsBasis<8>::create({19}); });
    CHECK(e.kind == RnsNttErrorKind::NonNttFriendlyModulus && e.modulus == 19 && e.degree == 8);
    e = caught([] { basis_17_97()->drop_last(2); });
    CHECK(e.kind == RnsNttErrorKind::InvalidModDrop && e.drop_count == 2 && e.channel_count == 2);
    Poly single = Poly::from_coeffs(std::array<int64_t, 8>{1, 2, 3, 4, 5, 6, 7, 8}, RnsBasis<8>::create({17}));
    e = caught([&] { single.rescale(); });
    CHECK(e.kind == RnsNttErrorKind::InvalidModDrop && e.drop_count == 1 && e.channel_count == 1);
  });

  // ---- CkksEncoder (ckks_encoder.rs:161-228 tests), on the device --------
  // basis {97, 113}, scale_bits 5, epsilon 0.1, as in the reference module
  const auto enc_basis = [] { return RnsBasis<8>::create({97, 113}); };
  const auto near = [](double a, double b, double eps) { return std::fabs(a - b) <= eps; };
  run("encoder_roundtrip_real_values", [&] {
    CkksEncoder<8> enc(5);
    const std::vector<double> values{1.0, -1.0, 0.5, -0.5};
    const auto out = enc.decode(enc.encode(values, enc_basis()));
    for (size_t i = 0; i < values.size(); ++i) CHECK(near(values[i], out[i], 0.1));
  });
  run("encoder_roundtrip_complex_values", [&] {
    CkksEncoder<8> enc(5);
    const std::vector<std::complex<double>> values{{1.0, 0.5}, {-0.5, 0.25}};
    const auto out = enc.decode_complex(enc.encode_complex(values, enc_basis()));
    for (size_t i = 0; i < values.size(); ++i) {
      CHECK(near(values[i].real(), out[i].real(), 0.1));
      CHECK(near(values[i].imag(), out[i].imag(), 0.1));
    }
  });
  run("encoder_single_value_roundtrip", [&] {
    CkksEncoder<8> enc(5);
    CHECK(near(enc.decode(enc.encode({3.0}, enc_basis()))[0], 3.0, 0.1));
  });
  run("encoder_slot_count_preserved", [&] {
    CkksEncoder<8> enc(5);
    CHECK(enc.decode(enc.encode({1.0, 2.0, 3.0}, enc_basis())).size() == 3);
  });
  run("encoder_max_slots_is_half_degree", [] { CHECK(CkksEncoder<8>(10).max_slots() == 4); });
  run("encoder_panics_on_too_many_values", [&] {
    CkksEncoder<8> enc(5);
    bool threw = false;
    try {
      enc.encode(std::vector<double>(5, 0.0), enc_basis());
    } catch (const std::invalid_argument& e) {
      threw = std::string(e.what()).find("exceed max slots") != std::string::npos;
    }
    CHECK(threw);
  });

  // ---- samplers (sampling.rs:98-242), on the device ----------------------
  run("sample_gaussian_has_reasonable_mean_and_variance", [] {
    std::mt19937_64 rng(17);
    double sum = 0, sq = 0;
    size_t cnt = 0;
    for (int t = 0; t < 256; ++t) {
      const auto c = Poly::sample_gaussian(3.2, basis_17_97(), rng).to_coeffs();
      for (int64_t v : c) {
        sum += (double)v;
        sq += (double)v * v;
        ++cnt;
      }
    }
    const double mean = sum / cnt, var = sq / cnt - mean * mean;
    CHECK(std::fabs(mean) < 0.5 && std::fabs(var - 3.2 * 3.2) < 2.5);
  });
  run("sample_tribits_handles_weight_extremes", [] {
    std::mt19937_64 rng(5);
    for (size_t hw : {size_t(0), size_t(8)}) {
      const auto c = Poly::sample_tribits(hw, basis_17_97(), rng).to_coeffs();
      size_t nz = 0;
      for (int64_t v : c) {
        CHECK(v >= -1 && v <= 1);
        nz += v != 0;
      }
      CHECK(nz == hw);
    }
    CHECK(throws_kind([&] { Poly::sample_tribits(9, basis_17_97(), rng); }, RnsNttErrorKind::BadArgument));
  });
  run("sample_gaussian_rejects_non_positive_std_dev", [] {
    std::mt19937_64 rng(1);
    CHECK(throws_kind([&] { Poly::sample_gaussian(0.0, basis_17_97(), rng); }, RnsNttErrorKind::BadArgument));
    CHECK(throws_kind([&] { Poly::sample_gaussian(-1.0, basis_17_97(), rng); }, RnsNttErrorKind::BadArgument));
  });
  std::printf("%d/%d passed\n", g_run - g_failed, g_run);
  return g_failed;
}
