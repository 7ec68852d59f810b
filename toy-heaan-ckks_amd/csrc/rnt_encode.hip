// rnt_encode.hip -- the CKKS canonical embedding on the device (SURVEY §8f
// row 4): CkksEncoder::encode_complex / decode_complex
// (ckks_encoder.rs:85-156) without the reference's O(N^2) Vandermonde
// evaluation (special_fft.rs:194-242).
//
// With M = N/2 slots, zeta = exp(i pi / N) and a the (centred integer)
// plaintext coefficients:
//
//   decode: u_j = a_j + i a_{j+M} (j < M);  z_k = sum_j u_j zeta^{5^k j}.
//     This is a(zeta^{5^k}) because zeta^{M 5^k} = i (5^k = 1 mod 4); the
//     reference's special_dft output index k (after its reversal) evaluates
//     a at conj(slot_roots[N-1-k]) = zeta^{5^k}: the same value.
//   encode: w_j = (1/M) sum_{k<M} v_k zeta^{-5^k j};  coefficient j = Re w_j,
//     coefficient j+M = Im w_j.  The reference's special_idft of the
//     conjugate-symmetric slot vector (special_fft.rs:158-178) reduces to
//     exactly this (its other half adds the complex conjugate).
//
// Both are the "special FFT" of size M over the rotation group 5^k: a
// decimation-in-time network after a bit reversal (decode) and its
// decimation-in-frequency inverse followed by a bit reversal (encode).
// Stage s (len = 2^s) pairs positions p, p + len/2 (p mod len < len/2) with
// the twiddle zeta^{(5^j mod 4 len) * 2N / (4 len)}, j = p mod len; the host
// table holds stage s's 2^(s-1) twiddles at heap offset 2^(s-1).
//
// Arithmetic is f64 complex (double2), so parity with the reference is
// tolerance-based, like the reference's own tests.  Rounding to integer
// coefficients is Rust's f64::round (ties away from zero) then `as i64`.
//
// Kernels (all over [B][M] double2 planes, 16 B per point):
//   k_sfft_low   stages inside 1024-point contiguous blocks, through LDS
//   k_sfft_high  stages across blocks: a workgroup holds 32 adjacent columns
//                of the (M/1024)-row grid (rows at stride 1024) in LDS
//   k_sfft_pack_coeffs / k_sfft_pack_slots / k_sfft_round: format changes
//                fused with the bit reversal and the power-of-two scalings
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <cmath>
#include <vector>

#include "rnt_internal.hpp"

namespace rnt {

namespace {

constexpr uint32_t kLowLog = 10;  // 1024 points (16 KiB) per low-pass block
constexpr uint32_t kHighLog = 6;  // at most 64 rows (32 KiB) per high-pass workgroup
constexpr uint32_t kHighTC = 32;  // columns per high-pass workgroup
constexpr uint32_t kSfThreads = 256;

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}

// DIT butterfly (x, y) -> (x + y w, x - y w); DIF inverse
// (x, y) -> (x + y, (x - y) conj(w)).
template <bool INV>
__device__ __forceinline__ void sbfly(double2* px, double2* py, double2 w) {
  const double2 x = *px, y = *py;
  if (!INV) {
    const double2 t = cmul(y, w);
    *px = make_double2(x.x + t.x, x.y + t.y);
    *py = make_double2(x.x - t.x, x.y - t.y);
  } else {
    *px = make_double2(x.x + y.x, x.y + y.y);
    *py = cmul(make_double2(x.x - y.x, x.y - y.y), make_double2(w.x, -w.y));
  }
}

__device__ __forceinline__ uint32_t brv32(uint32_t p, uint32_t bits) {
  return bits ? __brev(p) >> (32 - bits) : 0u;
}

// Stages 1..log_blk (forward) or log_blk..1 (inverse) of block blockIdx.x
// (2^log_blk contiguous points) of poly blockIdx.y.
template <bool INV>
__global__ void __launch_bounds__(kSfThreads)
k_sfft_low(double2* __restrict__ data, const double2* __restrict__ tw, uint32_t log_m,
           uint32_t log_blk) {
  __shared__ double2 s[1u << kLowLog];
  const uint32_t blk = 1u << log_blk;
  double2* d = data + ((uint64_t)blockIdx.y << log_m) + ((uint64_t)blockIdx.x << log_blk);
  for (uint32_t t = threadIdx.x; t < blk; t += kSfThreads) s[t] = d[t];
  __syncthreads();
  const uint32_t half = blk >> 1;
  for (uint32_t k = 0; k < log_blk; ++k) {
    const uint32_t st = INV ? log_blk - k : k + 1;
    const uint32_t lenh = 1u << (st - 1);
    for (uint32_t b = threadIdx.x; b < half; b += kSfThreads) {
      const uint32_t j = b & (lenh - 1);
      const uint32_t i0 = ((b >> (st - 1)) << st) | j;
      sbfly<INV>(&s[i0], &s[i0 + lenh], tw[lenh + j]);
    }
    __syncthreads();
  }
  for (uint32_t t = threadIdx.x; t < blk; t += kSfThreads) d[t] = s[t];
}

// Stages log_blk+1..log_m (forward) or log_m..log_blk+1 (inverse): the
// points of one column (equal low log_blk bits) are 2^(log_m - log_blk)
// rows at stride 2^log_blk; a workgroup holds kHighTC adjacent columns.
template <bool INV>
__global__ void __launch_bounds__(kSfThreads)
k_sfft_high(double2* __restrict__ data, const double2* __restrict__ tw, uint32_t log_m,
            uint32_t log_blk) {
  extern __shared__ double2 hs[];  // [rows][kHighTC]
  const uint32_t log_rows = log_m - log_blk;
  const uint32_t rows = 1u << log_rows;
  const uint32_t c0 = blockIdx.x * kHighTC;
  double2* d = data + ((uint64_t)blockIdx.y << log_m);
  for (uint32_t e = threadIdx.x; e < rows * kHighTC; e += kSfThreads)
    hs[e] = d[((e / kHighTC) << log_blk) + c0 + (e % kHighTC)];
  __syncthreads();
  const uint32_t nb = rows * kHighTC / 2;
  for (uint32_t k = 0; k < log_rows; ++k) {
    const uint32_t rb = INV ? log_rows - 1 - k : k;  // row bit of this stage
    const uint32_t lenh = 1u << (log_blk + rb);
    for (uint32_t b = threadIdx.x; b < nb; b += kSfThreads) {
      const uint32_t cc = b % kHighTC, rr = b / kHighTC;
      const uint32_t r0 = ((rr >> rb) << (rb + 1)) | (rr & ((1u << rb) - 1u));
      const uint32_t j = ((r0 << log_blk) + c0 + cc) & (2 * lenh - 1);
      sbfly<INV>(&hs[r0 * kHighTC + cc], &hs[(r0 | (1u << rb)) * kHighTC + cc], tw[lenh + j]);
    }
    __syncthreads();
  }
  for (uint32_t e = threadIdx.x; e < rows * kHighTC; e += kSfThreads)
    d[((e / kHighTC) << log_blk) + c0 + (e % kHighTC)] = hs[e];
}

// decode input: centred integer coefficients ([B][N] i64, k_crt's output)
// -> u at bit-reversed positions, scaled by 2^-scale_bits (exact: a power of
// two commutes with every rounding of the network, so this equals the
// reference's division of the slots by Delta).
__global__ void __launch_bounds__(256)
k_sfft_pack_coeffs(double2* __restrict__ out, const int64_t* __restrict__ a, uint32_t log_m,
                   double scale, uint64_t total) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const uint32_t M = 1u << log_m;
  const uint64_t p = gid >> log_m;
  const uint32_t j = brv32((uint32_t)gid & (M - 1), log_m);
  const int64_t* ap = a + (p << (log_m + 1));
  out[gid] = make_double2((double)ap[j] * scale, (double)ap[j + M] * scale);
}

// encode input: nv slot values per poly ([B][nv] double2) -> [B][M] in
// natural order, zero-padded (build_conjugate_slots), times 2^scale_bits.
__global__ void __launch_bounds__(256)
k_sfft_pack_slots(double2* __restrict__ out, const double2* __restrict__ v, uint32_t log_m,
                  uint32_t nv, double scale, uint64_t total) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const uint64_t p = gid >> log_m;
  const uint32_t k = (uint32_t)gid & ((1u << log_m) - 1u);
  double2 x = make_double2(0.0, 0.0);
  if (k < nv) x = v[p * nv + k];
  out[gid] = make_double2(x.x * scale, x.y * scale);
}

// f64::round (ties away from zero) then `as i64` (saturating, NaN -> 0).
__device__ __forceinline__ int64_t round_i64(double x) {
  if (!(x == x)) return 0;
  double r = trunc(x);
  if (fabs(x - r) >= 0.5) r += copysign(1.0, x);
  if (r >= 9223372036854775807.0) return INT64_MAX;
  if (r <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)r;
}

// encode output: after the inverse network position p holds M w_{brv p};
// coefficient brv(p) = round(Re / M), brv(p) + M = round(Im / M)
// (ckks_encoder.rs:112-115).
__global__ void __launch_bounds__(256)
k_sfft_round(int64_t* __restrict__ c, const double2* __restrict__ w, uint32_t log_m,
             double inv_m, uint64_t total) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const uint32_t M = 1u << log_m;
  const uint64_t p = gid >> log_m;
  const uint32_t j = brv32((uint32_t)gid & (M - 1), log_m);
  int64_t* cp = c + (p << (log_m + 1));
  const double2 x = w[gid];
  cp[j] = round_i64(x.x * inv_m);
  cp[j + M] = round_i64(x.y * inv_m);
}

unsigned grid_1d(uint64_t total) { return (unsigned)((total + 255) / 256); }

// Run the stages of the network over `planes` planes of 2^log_m points.
hipError_t sfft_network(hipStream_t s, double2* x, const double2* tw, uint32_t log_m,
                        uint64_t planes, bool inv) {
  const uint32_t log_blk = log_m < kLowLog ? log_m : kLowLog;
  const dim3 lgrid((unsigned)(1u << (log_m - log_blk)), (unsigned)planes);
  const bool high = log_m > log_blk;
  const uint32_t rows = 1u << (log_m - log_blk);
  const dim3 hgrid((unsigned)((1u << log_blk) / kHighTC), (unsigned)planes);
  const size_t hlds = (size_t)rows * kHighTC * sizeof(double2);
  if (!inv) {
    if (log_blk)
      hipLaunchKernelGGL(k_sfft_low<false>, lgrid, dim3(kSfThreads), 0, s, x, tw, log_m, log_blk);
    if (high)
      hipLaunchKernelGGL(k_sfft_high<false>, hgrid, dim3(kSfThreads), hlds, s, x, tw, log_m, log_blk);
  } else {
    if (high)
      hipLaunchKernelGGL(k_sfft_high<true>, hgrid, dim3(kSfThreads), hlds, s, x, tw, log_m, log_blk);
    if (log_blk)
      hipLaunchKernelGGL(k_sfft_low<true>, lgrid, dim3(kSfThreads), 0, s, x, tw, log_m, log_blk);
  }
  return hipGetLastError();
}

}  // namespace

std::vector<double> sfft_twiddles(uint32_t log_n) {
  // stage s (len = 2^s, s = 1..log2 M): tw[2^(s-1) + j] =
  // exp(2 pi i (5^j mod 4 len) / (4 len)), j < len / 2  (entry 0 unused)
  const uint64_t M = log_n ? (1ull << (log_n - 1)) : 0;
  std::vector<double> tab(2 * (M ? M : 1), 0.0);
  for (uint64_t len = 2; len <= M; len <<= 1) {
    const uint64_t lenq = 4 * len, lenh = len / 2;
    uint64_t r = 1;  // 5^j mod 4 len
    for (uint64_t j = 0; j < lenh; ++j) {
      const long double ang = 2.0L * 3.141592653589793238462643383279502884L * (long double)r /
                              (long double)lenq;
      tab[2 * (lenh + j)] = (double)cosl(ang);
      tab[2 * (lenh + j) + 1] = (double)sinl(ang);
      r = r * 5 % lenq;
    }
  }
  return tab;
}

bool sfft_supported(uint32_t log_n) { return log_n >= 1 && log_n - 1 <= kLowLog + kHighLog; }

hipError_t launch_sfft_encode(const Launch& k, int64_t* coeffs, void* work, const void* values,
                              uint32_t n_values, uint32_t scale_bits, const void* tw) {
  const uint32_t log_m = k.t->log_n - 1;
  const uint64_t total = (uint64_t)k.B << log_m;
  if (total == 0) return hipSuccess;
  double2* x = (double2*)work;
  hipLaunchKernelGGL(k_sfft_pack_slots, dim3(grid_1d(total)), dim3(256), 0, k.s, x,
                     (const double2*)values, log_m, n_values, std::ldexp(1.0, (int)scale_bits),
                     total);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = sfft_network(k.s, x, (const double2*)tw, log_m, k.B, true);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_sfft_round, dim3(grid_1d(total)), dim3(256), 0, k.s, coeffs,
                     (const double2*)x, log_m, std::ldexp(1.0, -(int)log_m), total);
  return hipGetLastError();
}

hipError_t launch_sfft_decode(const Launch& k, void* work, const int64_t* coeffs,
                              uint32_t scale_bits, const void* tw) {
  const uint32_t log_m = k.t->log_n - 1;
  const uint64_t total = (uint64_t)k.B << log_m;
  if (total == 0) return hipSuccess;
  double2* x = (double2*)work;
  hipLaunchKernelGGL(k_sfft_pack_coeffs, dim3(grid_1d(total)), dim3(256), 0, k.s, x, coeffs,
                     log_m, std::ldexp(1.0, -(int)scale_bits), total);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return sfft_network(k.s, x, (const double2*)tw, log_m, k.B, false);
}

}  // namespace rnt
