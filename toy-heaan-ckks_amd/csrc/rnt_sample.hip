// rnt_sample.hip -- device samplers: PolySampler for RnsPoly
// (traits.rs:74-127; poly.rs:438-477; math/sampling.rs:9-90), SURVEY §8f
// row 2 (key generation on the device).
//
// Randomness is Philox4x32-10 (Salmon et al., SC'11; Random123), counter
// based: every draw is a pure function of (seed, stream, sampler, poly,
// limb, index, attempt), so a sample does not depend on the launch
// geometry, the batch split or the device.  The reference draws from
// ChaCha20 through rand/rand_distr, whose streams cannot be reproduced here
// (SURVEY §8c/§8f), so parity is (a) bit-exact against the CPU restatement
// of THIS construction (oracle/sampler.py) and (b) the reference's own
// statistical sampler tests and key relations.
//
//   uniform   every (limb, poly, index) independently uniform in [0, q_l)
//             (sample_uniform, poly.rs:438-444): 64-bit draws with
//             rejection above the largest multiple of q (no modulo bias)
//   gaussian  one rounded N(0, sigma) integer per (poly, index), reduced
//             into every limb like from_coeffs (sample_gaussian,
//             poly.rs:447-459): Box-Muller on 53-bit uniforms, f64::round
//   ternary   exactly h coefficients +-1, the rest 0 (sample_tribits,
//             poly.rs:462-469; ternary_coefficients, sampling.rs:71-90):
//             position i gets the key (philox << 17) | i (unique), the h
//             smallest keys are selected by an 8-bit radix select in LDS
//             (one workgroup per poly), and each selected coefficient takes
//             a sign from a second draw.  Uniform over h-subsets, like the
//             reference's shuffle.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "rnt_internal.hpp"
#include "rnt_modarith.hpp"

namespace rnt {

namespace {

enum : uint32_t { kDrawUniform = 1, kDrawGauss = 2, kDrawTernKey = 3, kDrawTernSign = 4 };

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = make_uint4((uint32_t)(p1 >> 32) ^ c.y ^ k.x, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k.y,
                   (uint32_t)p0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

// Counter layout: (index | attempt << 20, poly, limb | kind << 16, stream);
// key: (seed_lo, seed_hi ^ stream_hi).
__device__ __forceinline__ uint4 draw(const SampleKey& s, uint32_t index, uint32_t attempt,
                                      uint32_t poly, uint32_t limb, uint32_t kind) {
  return philox4x32_10(make_uint4(index | (attempt << 20), poly, limb | (kind << 16), s.stream),
                       make_uint2(s.k0, s.k1));
}

__device__ __forceinline__ uint64_t lo64(uint4 v) { return (uint64_t)v.x | ((uint64_t)v.y << 32); }
__device__ __forceinline__ uint64_t hi64(uint4 v) { return (uint64_t)v.z | ((uint64_t)v.w << 32); }

template <class W>
__device__ __forceinline__ void sample_uniform_one(W* __restrict__ out, const LimbConst<W>* __restrict__ lc,
                                                   SampleKey s, uint32_t log_n, uint32_t B, uint64_t gid) {
  const uint32_t k = (uint32_t)(gid & ((1ull << log_n) - 1));
  const uint64_t lp = gid >> log_n;
  const uint32_t l = (uint32_t)(lp / B);
  const uint32_t p = (uint32_t)(lp - (uint64_t)l * B);
  const uint64_t q = (uint64_t)lc[l].q;
  const uint64_t rem = (uint64_t)mag_mod<W>(0 - q, lc[l]);  // 2^64 mod q = (2^64 - q) mod q
  const uint64_t lim = 0 - rem;      // accept x < 2^64 - rem (all x when rem == 0)
  uint64_t x = 0;
  for (uint32_t att = 0; att < 16; ++att) {  // a miss has probability < q / 2^64 per draw
    const uint4 v = draw(s, k, att, p, l, kDrawUniform);
    x = lo64(v);
    if (rem == 0 || x < lim) break;
    x = hi64(v);
    if (x < lim) break;  // (rem != 0 here)
  }
  out[gid] = mag_mod<W>(x, lc[l]);
}
template <class W>
__global__ void __launch_bounds__(256)
k_sample_uniform(W* __restrict__ out, const LimbConst<W>* __restrict__ lc, SampleKey s,
                 uint32_t log_n, uint32_t B, uint64_t total) {
  // [L][B][N]; grid-stride (a dispatch holds fewer than 2^32 work-items,
  // and 4096 polys x 16 limbs at 2^16 are 2^32 words)
  for (uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; gid < total;
       gid += (uint64_t)gridDim.x * blockDim.x)
    sample_uniform_one<W>(out, lc, s, log_n, B, gid);
}

// f64::round (ties away from zero), then `as i64` (saturating).
__device__ __forceinline__ int64_t round_away(double z) {
  double r = trunc(z);
  if (fabs(z - r) >= 0.5) r += copysign(1.0, z);
  if (r >= 9223372036854775807.0) return INT64_MAX;
  if (r <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)r;
}

template <class W>
__global__ void __launch_bounds__(256)
k_sample_gaussian(W* __restrict__ out, const LimbConst<W>* __restrict__ lc, SampleKey s,
                  double sigma, uint32_t log_n, uint32_t L, uint32_t B, uint64_t total) {
  // [B][N], grid-stride as k_sample_uniform
  for (uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; gid < total;
       gid += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t k = (uint32_t)(gid & ((1ull << log_n) - 1));
    const uint32_t p = (uint32_t)(gid >> log_n);
    const uint4 v = draw(s, k, 0, p, 0, kDrawGauss);
    const double u1 = (double)((lo64(v) >> 11) + 1) * 0x1.0p-53;  // (0, 1]
    const double u2 = (double)(hi64(v) >> 11) * 0x1.0p-53;        // [0, 1)
    const double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2) * sigma;
    const int64_t e = round_away(z);
    const uint64_t ls = (uint64_t)B << log_n;
    for (uint32_t l = 0; l < L; ++l) out[l * ls + gid] = rem_euclid<W>(e, lc[l]);
  }
}

constexpr uint32_t kTernThreads = 1024;

__device__ __forceinline__ uint64_t tern_key(const SampleKey& s, uint32_t i, uint32_t p) {
  return ((uint64_t)draw(s, i, 0, p, 0, kDrawTernKey).x << 17) | i;
}

template <class W>
__global__ void __launch_bounds__(kTernThreads)
k_sample_ternary(W* __restrict__ out, const LimbConst<W>* __restrict__ lc, SampleKey s,
                 uint32_t h, uint32_t log_n, uint32_t L, uint32_t B) {
  __shared__ uint32_t hist[256];
  __shared__ uint64_t s_prefix;
  __shared__ uint32_t s_rank;
  const uint32_t N = 1u << log_n;
  const uint32_t p = blockIdx.x, t = threadIdx.x;
  // the h-th smallest key (1-based) by radix select over 7 digits of 8 bits
  // (keys are < 2^49); with h == 0 nothing is selected
  uint64_t prefix = 0, mask = 0;
  if (t == 0) s_rank = h;
  for (int shift = 48; shift >= 0 && h > 0; shift -= 8) {
    if (t < 256) hist[t] = 0;
    __syncthreads();
    for (uint32_t i = t; i < N; i += kTernThreads) {
      const uint64_t key = tern_key(s, i, p);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (t == 0) {
      uint32_t r = s_rank, d = 0;
      while (hist[d] < r) r -= hist[d++];  // the rank-th key of this subset lies in digit d
      s_rank = r;
      s_prefix = prefix | ((uint64_t)d << shift);
    }
    __syncthreads();
    prefix = s_prefix;
    mask |= (uint64_t)255 << shift;
    __syncthreads();
  }
  const uint64_t ls = (uint64_t)B << log_n;
  for (uint32_t i = t; i < N; i += kTernThreads) {
    int64_t c = 0;
    if (h > 0 && tern_key(s, i, p) <= prefix)
      c = (draw(s, i, 0, p, 0, kDrawTernSign).x & 1u) ? 1 : -1;
    const uint64_t off = (uint64_t)p * N + i;
    for (uint32_t l = 0; l < L; ++l) out[l * ls + off] = rem_euclid<W>(c, lc[l]);
  }
}

// Blocks of 256 for `total` items, capped so a dispatch stays under 2^32
// work-items (the kernels stride over the rest).
unsigned grid_for_total(uint64_t total) {
  const uint64_t b = (total + 255) / 256;
  return (unsigned)(b < (1ull << 22) ? b : (1ull << 22));
}

template <class W>
hipError_t sample_impl(const Launch& k, int kind, void* out, SampleKey s, double sigma,
                       uint32_t h) {
  const uint32_t log_n = k.t->log_n;
  const auto* lc = (const LimbConst<W>*)k.t->lconst;
  if (k.B == 0 || k.L == 0) return hipSuccess;
  if (kind == 0) {
    const uint64_t total = (uint64_t)k.L * k.B << log_n;
    hipLaunchKernelGGL(k_sample_uniform<W>, dim3(grid_for_total(total)), dim3(256), 0, k.s, (W*)out,
                       lc, s, log_n, (uint32_t)k.B, total);
  } else if (kind == 1) {
    const uint64_t total = (uint64_t)k.B << log_n;
    hipLaunchKernelGGL(k_sample_gaussian<W>, dim3(grid_for_total(total)), dim3(256), 0, k.s,
                       (W*)out, lc, s, sigma, log_n, (uint32_t)k.L, (uint32_t)k.B, total);
  } else {
    hipLaunchKernelGGL(k_sample_ternary<W>, dim3((unsigned)k.B), dim3(kTernThreads), 0, k.s,
                       (W*)out, lc, s, h, log_n, (uint32_t)k.L, (uint32_t)k.B);
  }
  return hipGetLastError();
}

}  // namespace

hipError_t launch_sample(const Launch& k, int kind, void* out, SampleKey s, double sigma,
                         uint32_t hamming_weight) {
  return k.t->wide ? sample_impl<uint64_t>(k, kind, out, s, sigma, hamming_weight)
                   : sample_impl<uint32_t>(k, kind, out, s, sigma, hamming_weight);
}

}  // namespace rnt
