// rnt_kernels.hip -- hand-written gfx950 kernels for the RNS-NTT hot path.
//
// Reference behaviour being replaced (oiwn/toy-heaan-ckks):
//   to_ntt_domain / to_coeff_domain   src/rings/backends/rns_ntt/poly.rs:136-166
//   forward_ntt / inverse_ntt / CT    poly.rs:574-625
//   MulAssign (both domains)          poly.rs:277-331
//   AddAssign / Neg                   poly.rs:254-275, 370-385
//   rescale_into                      poly.rs:187-228
//   automorphism                      poly.rs:492-541
//   gadget key-switch sum             src/crypto/engine.rs:505-528, 429-452
//   tensor product                    engine.rs:480-493
//
// Transform: merged negacyclic Cooley-Tukey (twist folded into the
// twiddles: psi_rev[g] = psi^{brv(g)} over the heap g in [1, N)), output in
// bit-reversed order; inverse is the matching Gentleman-Sande network with
// n^-1 folded into its last stage.  Values equal the reference's
// a(psi^(2k+1)) exactly; only the order is private.
// Twiddles are stored interleaved with their Shoup companions ({w, w'}
// pairs) so one 8-byte load fetches both.
//
// Decomposition N = R * C (see rnt_internal.hpp):
//   column pass: stages with distance >= C, one column (stride C) per
//                thread, R <= 16 registers, coalesced 256 B per wave load;
//   row pass:    stages with distance < C, one row of C contiguous words per
//                C/16 threads, radix-16 register passes, LDS exchanges with a
//                1-in-16 pad (conflict-free for every pass distribution).
//                The row geometry is a template (RowGeo<LOG_C>): pass bit
//                ranges, LDS offsets and twiddle-subtree shapes are all
//                compile-time, so only one base address per thread is live.
#include <hip/hip_runtime.h>

#include <climits>

#include "rnt_internal.hpp"
#include "rnt_modarith.hpp"

namespace rnt {

template <class W>
struct TabPtrs {
  const Tw<W>* tw;   // [L][N] forward {w, w'}
  const Tw<W>* itw;  // [L][N] inverse {w, w'}
  const LimbConst<W>* lc;
  const W* resc;
  const W* rescp;
  uint32_t Lroot;
};

template <class W>
static TabPtrs<W> tab_ptrs(const Tables* t) {
  TabPtrs<W> p;
  p.tw = (const Tw<W>*)t->tw_fwd;
  p.itw = (const Tw<W>*)t->tw_inv;
  p.lc = (const LimbConst<W>*)t->lconst;
  p.resc = (const W*)t->resc;
  p.rescp = (const W*)t->resc_p;
  p.Lroot = (uint32_t)t->L;
  return p;
}

template <class W>
__device__ __forceinline__ Mod<W> mod_of(const LimbConst<W>& lc) {
  return Mod<W>{lc.q, (W)(W(0) - lc.q)};
}

// The product path's modulus bundle: LZ = Harvey-lazy 30-bit arithmetic
// (rnt_modarith.hpp Mod30; u32 words and q < 2^30 only).
template <class W, bool LZ>
__device__ __forceinline__ auto mod_for(const LimbConst<W>& lc) {
  static_assert(!LZ || sizeof(W) == 4, "lazy 30-bit arithmetic needs 32-bit words");
  if constexpr (LZ) {
    const uint32_t q = (uint32_t)lc.q;
    return Mod30{q, 0u - q, 2u * q};
  } else {
    return mod_of(lc);
  }
}

// Buffer-resource view of a wave-uniform base (a (limb, poly) plane or a
// limb's twiddle table): loads/stores take a 32-bit per-lane element offset
// plus a wave-uniform one that lands in the instruction's SGPR soffset, so
// strided column access costs no VALU address arithmetic.
// Cache-policy bits (`aux`) of the plane loads and stores: the default
// policy (non-temporal was within run-to-run spread).
constexpr int kBufAux = 0;
// Measurement builds only (tools/build_variant.sh -DRNT_MEAS=...; never the
// shipped library): 1 = the product kernels (k_colt_fwd, k_row<2>,
// k_colt_inv) move no plane data through memory (synthetic loads, stores
// kept behind a never-true compare), 2 = their butterflies are skipped.
// They time the VALU-only and memory/LDS-only parts of the poly-mul
// ("ceiling").
#ifndef RNT_MEAS
#define RNT_MEAS 0
#endif
constexpr int kMeas = RNT_MEAS;
// 3 and 4 keep every butterfly and move the poly-mul's plane traffic of a
// lower-traffic design: the intermediate planes named below are replaced
// by synthetic values (loads) and never-true stores, so the three kernels
// move 5 planes per (poly, limb) (3: a's column output and the row
// output are not written, a's column output and the column-inverse input
// not read) or 7 (4: only the row -> inverse-column plane is skipped) --
// the energy model's what-ifs measured directly.
// Sites: 0 k_colt_fwd operand-0 store, 1 k_row<2> load of operand 0,
// 2 k_row<2> store, 3 k_colt_inv load.
constexpr bool meas_virtual(int site) {
  return (kMeas == 3 && site <= 3) || (kMeas == 4 && (site == 2 || site == 3));
}
template <class W>
__device__ __forceinline__ W meas_val(uint32_t v, uint32_t s) {
  return (W)((v * 2654435761u + s) & 0x3fffffffu);
}
template <class W>
__device__ __forceinline__ W gload(const W* p, uint64_t i) {
  if constexpr (kMeas == 1) return meas_val<W>((uint32_t)i, 0u);
  return p[i];
}
template <class W>
__device__ __forceinline__ void gstore(W* p, uint64_t i, W x) {
  if constexpr (kMeas == 1) {
    if (x == (W)0xffffffffu) p[i] = x;
    return;
  }
  p[i] = x;
}

template <class W>
struct BufView {
  __amdgpu_buffer_rsrc_t r;
  __device__ BufView(const W* base, uint32_t elems)
      : r(__builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)(elems * sizeof(W)), 0x00020000)) {}
  __device__ __forceinline__ W ld(uint32_t v, uint32_t s) const {
    if constexpr (kMeas == 1) return meas_val<W>(v, s);
    if constexpr (sizeof(W) == 4) {
      return __builtin_amdgcn_raw_buffer_load_b32(r, v * 4u, s * 4u, kBufAux);
    } else {
      return __builtin_bit_cast(W, __builtin_amdgcn_raw_buffer_load_b64(r, v * 8u, s * 8u, kBufAux));
    }
  }
  // four consecutive words (the compiler does not merge the raw buffer
  // builtins into wide loads by itself)
  __device__ __forceinline__ void ld4(W (&o)[4], uint32_t v, uint32_t s) const {
    if constexpr (sizeof(W) == 4) {
      const auto q = __builtin_amdgcn_raw_buffer_load_b128(r, v * 4u, s * 4u, kBufAux);
      o[0] = q[0];
      o[1] = q[1];
      o[2] = q[2];
      o[3] = q[3];
    } else {
      const auto a = __builtin_amdgcn_raw_buffer_load_b128(r, v * 8u, s * 8u, kBufAux);
      const auto b = __builtin_amdgcn_raw_buffer_load_b128(r, v * 8u + 16u, s * 8u, kBufAux);
      o[0] = (uint64_t)a[0] | ((uint64_t)a[1] << 32);
      o[1] = (uint64_t)a[2] | ((uint64_t)a[3] << 32);
      o[2] = (uint64_t)b[0] | ((uint64_t)b[1] << 32);
      o[3] = (uint64_t)b[2] | ((uint64_t)b[3] << 32);
    }
  }
  __device__ __forceinline__ void st(W x, uint32_t v, uint32_t s) const {
    if constexpr (kMeas == 1) {
      if (x != (W)0xffffffffu) return;
    }
    if constexpr (sizeof(W) == 4) {
      __builtin_amdgcn_raw_buffer_store_b32(x, r, v * 4u, s * 4u, kBufAux);
    } else {
      using V2 = decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0));
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(V2, x), r, v * 8u, s * 8u, kBufAux);
    }
  }
};

// Twiddle sources for the pass templates: a plain pointer (row kernels,
// whose limb may vary across a workgroup) or a buffer view of one limb's
// table (column kernels: one limb per workgroup).
// tw_get(src, nb, m): twiddle nb + m where nb is the stage's (per-lane or
// uniform) heap base and m a compile-time index -- kept apart so the buffer
// form puts m into the instruction (inline-constant soffset) and holds ONE
// offset register per stage instead of one per twiddle.
template <class W>
__device__ __forceinline__ Tw<W> tw_get(const Tw<W>* p, uint32_t nb, uint32_t m) {
  return p[nb + m];
}
template <class W>
struct TwBuf {
  __amdgpu_buffer_rsrc_t r;
  __device__ TwBuf(const Tw<W>* base, uint32_t n)
      : r(__builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)(n * sizeof(Tw<W>)), 0x00020000)) {}
};
template <class W>
__device__ __forceinline__ Tw<W> tw_get(const TwBuf<W>& b, uint32_t nb, uint32_t m) {
  Tw<W> t;
  if constexpr (sizeof(W) == 4) {
    const uint64_t v =
        __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(b.r, nb * 8u, m * 8u, 0));
    t.w = (uint32_t)v;
    t.p = (uint32_t)(v >> 32);
  } else {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(b.r, nb * 16u, m * 16u, 0);
    t.w = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
    t.p = (uint64_t)v[2] | ((uint64_t)v[3] << 32);
  }
  return t;
}

Geom geom_for(uint32_t log_n) {
  Geom g;
  g.log_n = log_n;
  if (log_n < 4) {  // tiny rings: one row holds the whole polynomial
    g.log_r = 0;
    g.log_c = log_n;
  } else if (log_n < 8) {
    g.log_r = log_n - 4;
    g.log_c = 4;
  } else {
    // balance the stages between the (memory-bound) column passes and the
    // (ALU-bound) row pass: R = 2^floor(log_n / 2), at least 16
    g.log_r = log_n / 2 > 4 ? log_n / 2 : 4;
    g.log_c = log_n - g.log_r;
  }
  g.n = (size_t)1 << log_n;
  g.r = (size_t)1 << g.log_r;
  g.c = (size_t)1 << g.log_c;
  return g;
}

// ---------------------------------------------------------------------------
// column passes
// ---------------------------------------------------------------------------

template <class W, int LOG_R>
__device__ __forceinline__ void col_ct(W (&x)[1 << LOG_R], const Tw<W>* tw, const Mod<W>& m) {
  constexpr int R = 1 << LOG_R;
#pragma unroll
  for (int k = 0; k < LOG_R; ++k) {
    const int d = R >> (k + 1);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      if (i & d) continue;
      const Tw<W> t = tw[(1 << k) + (i >> (LOG_R - k))];
      // outputs that the next stage only multiplies stay unreduced
      if (k + 1 < LOG_R && (i & (d >> 1)))
        ct_bfly_lazy<W>(x[i], x[i + d], t.w, t.p, m);
      else
        ct_bfly<W>(x[i], x[i + d], t.w, t.p, m);
    }
  }
}

// x <- GS network over the column with the last (distance N/2) stage scaled
// by c1 (upper) and c2 (lower).
template <class W, int LOG_R>
__device__ __forceinline__ void col_gs(W (&x)[1 << LOG_R], const Tw<W>* itw, const Mod<W>& m,
                                       W c1, W c1p, W c2, W c2p) {
  const W q = m.q;
  constexpr int R = 1 << LOG_R;
#pragma unroll
  for (int sl = 0; sl < LOG_R; ++sl) {
    const int d = 1 << sl;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      if (i & d) continue;
      if (sl == LOG_R - 1) {
        W u = x[i], v = x[i + d];
        x[i] = shoup_mul<W>(u + v, c1, c1p, m);
        x[i + d] = shoup_mul<W>(u - v + q, c2, c2p, m);
      } else {
        const Tw<W> t = itw[(1 << (LOG_R - 1 - sl)) + (i >> (sl + 1))];
        gs_bfly<W>(x[i], x[i + d], t.w, t.p, m);
      }
    }
  }
  if (LOG_R == 0) x[0] = shoup_mul<W>(x[0], c1, c1p, m);
}

// Forward column pass.  Thread = (limb l, poly p, column j1); j1 fastest.
// Operand 1 is processed first: out0 may alias in1 (out = a * b, out == b).
template <class W, int LOG_R>
__global__ void __launch_bounds__(256)
k_col_fwd(W* out0, const W* in0, W* out1, const W* in1, TabPtrs<W> tp, uint32_t log_n,
          uint32_t log_c, uint32_t B, uint64_t in_ls, uint64_t out_ls, uint64_t total) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  constexpr int R = 1 << LOG_R;
  const uint32_t C = 1u << log_c;
  const uint64_t N = 1ull << log_n;
  const uint32_t j1 = (uint32_t)(gid & (C - 1));
  const uint64_t lp = gid >> log_c;
  const uint32_t l = (uint32_t)(lp / B);
  const uint32_t p = (uint32_t)(lp - (uint64_t)l * B);
  const uint64_t ib = (uint64_t)l * in_ls + (uint64_t)p * N + j1;
  const uint64_t ob = (uint64_t)l * out_ls + (uint64_t)p * N + j1;
  const Mod<W> m = mod_of(tp.lc[l]);
  const Tw<W>* tw = tp.tw + (uint64_t)l * N;
  W x[R];
  if (in1 != nullptr) {
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = in1[ib + (uint64_t)i * C];
    col_ct<W, LOG_R>(x, tw, m);
#pragma unroll
    for (int i = 0; i < R; ++i) out1[ob + (uint64_t)i * C] = x[i];
  }
#pragma unroll
  for (int i = 0; i < R; ++i) x[i] = in0[ib + (uint64_t)i * C];
  col_ct<W, LOG_R>(x, tw, m);
#pragma unroll
  for (int i = 0; i < R; ++i) out0[ob + (uint64_t)i * C] = x[i];
}

template <class W, int LOG_R>
__global__ void __launch_bounds__(256)
k_col_inv(W* out, const W* in, const W* addend, TabPtrs<W> tp, uint32_t log_n, uint32_t log_c,
          uint32_t B, uint64_t in_ls, uint64_t out_ls, uint64_t total, int rfold) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  constexpr int R = 1 << LOG_R;
  const uint32_t C = 1u << log_c;
  const uint64_t N = 1ull << log_n;
  const uint32_t j1 = (uint32_t)(gid & (C - 1));
  const uint64_t lp = gid >> log_c;
  const uint32_t l = (uint32_t)(lp / B);
  const uint32_t p = (uint32_t)(lp - (uint64_t)l * B);
  const uint64_t ib = (uint64_t)l * in_ls + (uint64_t)p * N + j1;
  const uint64_t base = (uint64_t)l * out_ls + (uint64_t)p * N + j1;
  const LimbConst<W> lc = tp.lc[l];
  const Tw<W>* itw = tp.itw + (uint64_t)l * N;
  W x[R];
#pragma unroll
  for (int i = 0; i < R; ++i) x[i] = in[ib + (uint64_t)i * C];
  if (rfold == 2)
    col_gs<W, LOG_R>(x, itw, mod_of(lc), lc.c1t, lc.c1t_p, lc.c2t, lc.c2t_p);
  else if (rfold)
    col_gs<W, LOG_R>(x, itw, mod_of(lc), lc.c1r, lc.c1r_p, lc.c2r, lc.c2r_p);
  else
    col_gs<W, LOG_R>(x, itw, mod_of(lc), lc.c1, lc.c1_p, lc.c2, lc.c2_p);
  if (addend != nullptr) {
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = add_mod<W>(x[i], addend[base + (uint64_t)i * C], lc.q);
  }
#pragma unroll
  for (int i = 0; i < R; ++i) out[base + (uint64_t)i * C] = x[i];
}

// Key-switch decomposition + forward column pass (engine.rs:507-516 fused
// with the first half of alpha_i's forward NTT): thread = (target limb j,
// source limb i, poly p, column j1); reads limb i of d, reduces mod q_j
// canonically (R5), transforms with q_j's tables, writes S[j][i][p].
template <class W, int LOG_R>
__global__ void __launch_bounds__(256)
k_ks_decompose(W* __restrict__ S, const W* __restrict__ d, TabPtrs<W> tp, uint32_t log_n,
               uint32_t log_c, uint32_t L, uint32_t B, uint64_t d_ls, uint64_t total) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  constexpr int R = 1 << LOG_R;
  const uint32_t C = 1u << log_c;
  const uint64_t N = 1ull << log_n;
  const uint32_t j1 = (uint32_t)(gid & (C - 1));
  uint64_t rest = gid >> log_c;  // ((j*L + i)*B + p), L = source limbs
  const uint32_t p = (uint32_t)(rest % B);
  rest /= B;
  const uint32_t i = (uint32_t)(rest % L);
  const uint32_t j = (uint32_t)(rest / L);
  const LimbConst<W> lc = tp.lc[j];
  const Tw<W>* tw = tp.tw + (uint64_t)j * N;
  const uint64_t src = (uint64_t)i * d_ls + (uint64_t)p * N + j1;
  const uint64_t dst = (((uint64_t)j * L + i) * B + p) * N + j1;
  W x[R];
#pragma unroll
  for (int t = 0; t < R; ++t) x[t] = shoup_mul<W>(d[src + (uint64_t)t * C], (W)1, lc.one_p, lc.q);
  col_ct<W, LOG_R>(x, tw, mod_of(lc));
#pragma unroll
  for (int t = 0; t < R; ++t) S[dst + (uint64_t)t * C] = x[t];
}

// ---------------------------------------------------------------------------
// row passes
// ---------------------------------------------------------------------------

// Radix-16 pass schedule of one transform of length 2^LOGX held by T
// threads x E registers.  Passes run from the top bits down: full radix-16
// passes on bits [bb, bb+4), then (if LOGX % 4) a partial pass on bits
// [0, REM) with register bits [0, 4).  LOGX < 4: one thread holds it all.
template <int LOGX>
struct PassSched {
  static constexpr int LOGX_ = LOGX;
  static constexpr int LOGE = LOGX < 4 ? LOGX : 4;
  static constexpr int E = 1 << LOGE;
  static constexpr int LOG_T = LOGX - LOGE;
  static constexpr int T = 1 << LOG_T;
  static constexpr int X = 1 << LOGX;
  static constexpr int FULL = LOGX >= 4 ? LOGX / LOGE : 0;
  static constexpr int REM = LOGX >= 4 ? LOGX % LOGE : LOGX;
  static constexpr int P = FULL + (REM ? 1 : 0);
  static constexpr int bb(int p) { return (p >= 0 && p < FULL) ? LOGX - LOGE * (p + 1) : 0; }
  static constexpr int k(int p) { return p < FULL ? LOGE : REM; }
  static constexpr int BB0 = bb(0);
  static constexpr int BBL = bb(P - 1);
  // transform-local index of register i in the distribution with register
  // bits [b, b+LOGE): base(tau, b) | (i << b)
  __device__ static __forceinline__ uint32_t base(uint32_t tau, int b) {
    const uint32_t lowmask = (1u << b) - 1u;
    return (tau & lowmask) | ((tau >> b) << (b + LOGE));
  }
};

// Rows: RPW rows of C = 2^LOG_C contiguous words per workgroup; each row has
// its own LDS region with a 1-in-16 pad.  swz(base | (i<<b)) =
// swz(base) + (i<<b) + ((i<<b)>>4) because base has zero bits in [b, b+4).
template <int LOG_C>
struct RowGeo : PassSched<LOG_C> {
  using S = PassSched<LOG_C>;
  static constexpr int LOGC = LOG_C;
  static constexpr int C = 1 << LOG_C;
  // one pad word per 2^PADSH words (16 for the radix-16 passes)
  static constexpr int PADSH = S::LOGE == 3 ? 3 : 4;
  static constexpr int PADC = C + (C >> PADSH);
  static constexpr int THREADS = S::T > kRowThreads ? S::T : kRowThreads;
  static constexpr int RPW = THREADS / S::T;  // rows per workgroup
  static constexpr int REGION = RPW * PADC;   // LDS words per operand
  __device__ static __forceinline__ uint32_t slot_of(uint32_t tid) { return tid >> S::LOG_T; }
  __device__ static __forceinline__ uint32_t tau_of(uint32_t tid) { return tid & (S::T - 1); }
  __device__ static __forceinline__ uint32_t lds_off(uint32_t slot, uint32_t j) {
    return slot * PADC + j + (j >> PADSH);
  }
  static constexpr uint32_t lds_ioff(int i, int b) {
    return ((uint32_t)i << b) + (((uint32_t)i << b) >> PADSH);
  }
};

// Column tiles: TC = 2^LOG_TC adjacent columns of a stride-C, length-R
// column transform per workgroup; LDS is [j][TC] so consecutive lanes hit
// consecutive banks.  TC = 64 (C >= 64) makes a wave's 64 lanes one tau, so
// every twiddle a wave needs is wave-uniform: they come through scalar loads
// into SGPRs (no VGPRs, no vector memory ops); TC = 32 (C = 32) keeps them
// per-lane.
template <int LOG_R, int LOG_TC>
struct ColGeo : PassSched<LOG_R> {
  using S = PassSched<LOG_R>;
  static constexpr int LOGTC = LOG_TC;
  static constexpr int TC = 1 << LOG_TC;
  static constexpr bool UNIFORM = TC == 64;
  static constexpr int THREADS = TC * S::T;
  static constexpr int REGION = S::X * TC;
  __device__ static __forceinline__ uint32_t slot_of(uint32_t tid) { return tid & (TC - 1); }
  __device__ static __forceinline__ uint32_t tau_of(uint32_t tid) {
    if constexpr (UNIFORM) return __builtin_amdgcn_readfirstlane(tid >> LOG_TC);
    else return tid >> LOG_TC;
  }
  __device__ static __forceinline__ uint32_t lds_off(uint32_t slot, uint32_t j) {
    return j * TC + slot;
  }
  static constexpr uint32_t lds_ioff(int i, int b) { return ((uint32_t)i << b) * TC; }
};

// Wave-uniform twiddle source: a constant-address-space view, so uniform
// indices become s_load into SGPRs.  (The host pass of hipcc parses the
// kernels too and has no address space 4.)
#if defined(__HIP_DEVICE_COMPILE__)
#define RNT_CONST_AS __attribute__((address_space(4)))
#else
#define RNT_CONST_AS
#endif
template <class W>
struct TwScalar {
  const RNT_CONST_AS Tw<W>* p;
};
template <class W>
__device__ __forceinline__ Tw<W> tw_get(const TwScalar<W>& t, uint32_t nb, uint32_t m) {
  return t.p[nb + m];
}
template <class W, bool UNIFORM>
__device__ __forceinline__ auto col_twiddles(const Tw<W>* base, uint32_t n) {
  if constexpr (UNIFORM) {
    return TwScalar<W>{(const RNT_CONST_AS Tw<W>*)base};
  } else {
    return TwBuf<W>(base, n);
  }
}

// Last-stage constants of the inverse network (n^-1 folded, optionally with
// the Montgomery factor): x <- (u+v) c1, y <- (u-v) c2.
template <class W>
struct Fold {
  W c1, c1p, c2, c2p;
};

// CT stages on bits [BB, BB+K) for NOPS operands sharing twiddles.  `node0`
// = heap index base of register 0: (heap root of this transform) * 2^LOGX +
// its transform-local index, so stage s's node is node0 >> (s+1) + (i >> ...).
// SLMIN > 0 stops SLMIN stages early (the truncated product transform); the
// last stage run then leaves its outputs canonical.
template <class W, int NOPS, int LOGE, int K, int BB, class TS, class MO, int SLMIN = 0>
__device__ __forceinline__ void pass_ct(W (&x)[NOPS][1 << LOGE], uint32_t node0, const TS& tw,
                                        const MO& mo) {
  if constexpr (kMeas == 2) return;
  constexpr int E = 1 << LOGE;
#pragma unroll
  for (int sl = K - 1; sl >= SLMIN; --sl) {
    constexpr int H = E > 1 ? E / 2 : 1;
    const int cnt = H >> sl;  // distinct twiddles at this stage
    const uint32_t nb = node0 >> (BB + sl + 1);
    Tw<W> t[H];
#pragma unroll
    for (int m = 0; m < H; ++m)
      if (m < cnt) t[m] = tw_get<W>(tw, nb, (uint32_t)m);
    const int d = 1 << sl;
#pragma unroll
    for (int i = 0; i < E; ++i) {
      if (i & d) continue;
      const int m = i >> (sl + 1);
      // inside a pass, outputs the next stage only multiplies stay unreduced
      const bool lazy = sl > SLMIN && (i & (d >> 1));
#pragma unroll
      for (int o = 0; o < NOPS; ++o) {
        if (lazy)
          ct_bfly_lazy(x[o][i], x[o][i | d], t[m].w, t[m].p, mo);
        else
          ct_bfly(x[o][i], x[o][i | d], t[m].w, t[m].p, mo);
      }
    }
  }
}

// GS stages; with FOLD the transform's top stage (bit LOGX-1, distance N/2
// of the whole network) applies the folded n^-1 constants instead.
template <class W, int NOPS, int LOGE, int K, int BB, int LOGX, bool FOLD, class TS, class MO,
          int SLMIN = 0>
__device__ __forceinline__ void pass_gs(W (&x)[NOPS][1 << LOGE], uint32_t node0, const TS& itw,
                                        const MO& mo, const Fold<W>& f) {
  if constexpr (kMeas == 2) return;
  const W bias = gs_bias(mo);
  constexpr int E = 1 << LOGE;
#pragma unroll
  for (int sl = SLMIN; sl < K; ++sl) {
    constexpr int H = E > 1 ? E / 2 : 1;
    const int d = 1 << sl;
    if (FOLD && BB + sl + 1 == LOGX) {
#pragma unroll
      for (int i = 0; i < E; ++i) {
        if (i & d) continue;
#pragma unroll
        for (int o = 0; o < NOPS; ++o) {
          const W u = x[o][i], v = x[o][i | d];
          x[o][i] = shoup_mul(u + v, f.c1, f.c1p, mo);
          x[o][i | d] = shoup_mul(u - v + bias, f.c2, f.c2p, mo);
        }
      }
      continue;
    }
    const int cnt = H >> sl;
    const uint32_t nb = node0 >> (BB + sl + 1);
    Tw<W> t[H];
#pragma unroll
    for (int m = 0; m < H; ++m)
      if (m < cnt) t[m] = tw_get<W>(itw, nb, (uint32_t)m);
#pragma unroll
    for (int i = 0; i < E; ++i) {
      if (i & d) continue;
      const int m = i >> (sl + 1);
#pragma unroll
      for (int o = 0; o < NOPS; ++o) gs_bfly(x[o][i], x[o][i | d], t[m].w, t[m].p, mo);
    }
  }
}

// Minimum resident waves per SIMD requested for the row kernels (caps their
// VGPR budget at 512 / kRowMinWaves) and for the key-switch rows.
constexpr int kRowMinWaves = 6;
constexpr int kKsMinWaves = 4;
// Key rows of the key-switch rows kernel go global -> LDS directly
// (global_load_lds, no registers) for u32 rows of >= 64 words, except in the
// WIDE (small-batch) grid below 2^9-word rows, where staging them through
// registers measured faster (profiles/r02_ab_ks_small_batch.txt).
constexpr int kKsGldsWideMinLogC = 9;

// Move NOPS register sets from distribution BF to BT through LDS.  Several
// operands go one after the other through a single LDS region, so occupancy
// is bounded by VGPRs rather than LDS, at two barriers per operand.
template <class G, class W, int NOPS, int BF, int BT>
__device__ __forceinline__ void xchg(W (&x)[NOPS][G::E], W* lds, uint32_t slot, uint32_t tau) {
  const uint32_t wb = G::lds_off(slot, G::base(tau, BF));
  const uint32_t rb = G::lds_off(slot, G::base(tau, BT));
#pragma unroll
  for (int o = 0; o < NOPS; ++o) {
#pragma unroll
    for (int i = 0; i < G::E; ++i) lds[wb + G::lds_ioff(i, BF)] = x[o][i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < G::E; ++i) x[o][i] = lds[rb + G::lds_ioff(i, BT)];
    __syncthreads();
  }
}

// Per-thread transform coordinates: `slot` (which transform of the
// workgroup), `tau` (thread within it), `heap` (heap index of the
// transform's root times its length: node0 = heap + local index).
struct XPos {
  uint32_t slot, tau;
  uint32_t heap;
};

template <class G, class W, int NOPS, int PP, int SLMIN = 0, class TS, class MO>
__device__ __forceinline__ void fwd_pass(W (&x)[NOPS][G::E], const XPos& xp, W* lds, const TS& tw,
                                         const MO& q) {
  constexpr int BB = G::bb(PP);
  if constexpr (PP > 0) xchg<G, W, NOPS, G::bb(PP - 1), BB>(x, lds, xp.slot, xp.tau);
  pass_ct<W, NOPS, G::LOGE, G::k(PP), BB, TS, MO, SLMIN>(x, xp.heap + G::base(xp.tau, BB), tw, q);
}

template <class G, class W, int NOPS, int PP, bool FOLD, int SLMIN = 0, class TS, class MO>
__device__ __forceinline__ void inv_pass(W (&x)[NOPS][G::E], const XPos& xp, W* lds, const TS& itw,
                                         const MO& q, const Fold<W>& f) {
  constexpr int BB = G::bb(PP);
  if constexpr (PP < G::P - 1) xchg<G, W, NOPS, G::bb(PP + 1), BB>(x, lds, xp.slot, xp.tau);
  pass_gs<W, NOPS, G::LOGE, G::k(PP), BB, G::LOGX_, FOLD, TS, MO, SLMIN>(
      x, xp.heap + G::base(xp.tau, BB), itw, q, f);
}

// All forward passes (first-pass distribution in, last-pass out).
template <class G, class W, int NOPS, class TS, class MO>
__device__ __forceinline__ void xf_fwd(W (&x)[NOPS][G::E], const XPos& xp, W* lds, const TS& tw,
                                       const MO& q) {
  if constexpr (G::P > 0) fwd_pass<G, W, NOPS, 0>(x, xp, lds, tw, q);
  if constexpr (G::P > 1) fwd_pass<G, W, NOPS, 1>(x, xp, lds, tw, q);
  if constexpr (G::P > 2) fwd_pass<G, W, NOPS, 2>(x, xp, lds, tw, q);
  if constexpr (G::P > 3) fwd_pass<G, W, NOPS, 3>(x, xp, lds, tw, q);
}

// All inverse passes (last-pass distribution in, first-pass out).
template <class G, class W, int NOPS, bool FOLD = false, class TS, class MO>
__device__ __forceinline__ void xf_inv(W (&x)[NOPS][G::E], const XPos& xp, W* lds, const TS& itw,
                                       const MO& q, const Fold<W>& f = Fold<W>{}) {
  if constexpr (G::P > 3) inv_pass<G, W, NOPS, 3, FOLD>(x, xp, lds, itw, q, f);
  if constexpr (G::P > 2) inv_pass<G, W, NOPS, 2, FOLD>(x, xp, lds, itw, q, f);
  if constexpr (G::P > 1) inv_pass<G, W, NOPS, 1, FOLD>(x, xp, lds, itw, q, f);
  if constexpr (G::P > 0) inv_pass<G, W, NOPS, 0, FOLD>(x, xp, lds, itw, q, f);
}

// Row coordinates of this thread.
struct RowPos {
  XPos xp;
  uint32_t l, p, r;
  bool active;
};

// Row coordinates with the poly index fastest: row = ((l * R + r) * B + p).
// Consecutive rows of a workgroup then share (limb, row r), so whatever they
// read per (limb, r) -- gadget-key rows, twiddles -- is fetched from HBM once
// and hit in cache by the rest of the batch.
template <class G>
__device__ __forceinline__ RowPos row_pos_pfast(uint32_t log_n, uint32_t B, uint64_t rows_total) {
  RowPos rp;
  rp.xp.slot = G::slot_of(threadIdx.x);
  rp.xp.tau = G::tau_of(threadIdx.x);
  uint64_t row = (uint64_t)blockIdx.x * G::RPW + rp.xp.slot;
  rp.active = row < rows_total;
  if (!rp.active) row = 0;
  const uint32_t log_r = log_n - G::LOGC;
  const uint64_t lr = row / B;
  rp.p = (uint32_t)(row - lr * B);
  rp.r = (uint32_t)(lr & ((1u << log_r) - 1u));
  rp.l = (uint32_t)(lr >> log_r);
  rp.xp.heap = (1u << log_n) + rp.r * (uint32_t)G::C;  // (R + r) * C
  return rp;
}

// ---------------------------------------------------------------------------
// tiled column passes (log2 R >= 5): a workgroup owns TC = 32 adjacent
// columns of one (limb, poly) and runs the R-point network over the row
// index j (stride C) through LDS.  The column transform is the top of the
// heap: node0 = R + j.  Output stays in place (row j, column c).
// ---------------------------------------------------------------------------

struct ColPos {
  XPos xp;
  uint32_t l, p;
  uint32_t col;
};

// Grid: x = poly * (C / TC) + column tile, y = limb (no integer division,
// so limb and poly stay in SGPRs and the buffer descriptors built from them
// are provably wave-uniform).
template <class G>
__device__ __forceinline__ ColPos col_pos(uint32_t log_c) {
  ColPos cp;
  cp.xp.slot = G::slot_of(threadIdx.x);
  cp.xp.tau = G::tau_of(threadIdx.x);
  const uint32_t tpp_log = log_c - G::LOGTC;  // column tiles per (limb, poly)
  cp.l = blockIdx.y;
  cp.p = blockIdx.x >> tpp_log;
  const uint32_t ct = blockIdx.x & ((1u << tpp_log) - 1);
  cp.col = (ct << G::LOGTC) + cp.xp.slot;
  cp.xp.heap = (uint32_t)G::X;
  return cp;
}

// Per-lane element offset of register 0 and the wave-uniform register
// stride of a column tile in distribution bits [BB, BB+LOGE).
template <class G, int BB>
struct ColAddr {
  uint32_t v, s;
  __device__ ColAddr(const ColPos& cp, uint32_t log_c)
      : v(cp.col + (G::base(cp.xp.tau, BB) << log_c)), s(1u << (log_c + BB)) {}
  // Opaque redefinition of the stride: stops the compiler from keeping all
  // E soffsets (i * s) live across a transform, which spills them to VGPRs
  // and turns every buffer op into a waterfall loop.
  __device__ __forceinline__ void refresh() { asm volatile("" : "+s"(s)); }
};

template <class W, int LOG_R, int LOG_TC, bool LZ = false>
__global__ void __launch_bounds__((ColGeo<LOG_R, LOG_TC>::THREADS))
k_colt_fwd(W* out0, const W* in0, W* out1, const W* in1, TabPtrs<W> tp, uint32_t log_n,
           uint32_t log_c, uint32_t B, uint64_t in_ls, uint64_t out_ls) {
  using G = ColGeo<LOG_R, LOG_TC>;
  constexpr int E = G::E;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  W* lds = (W*)smem_raw;
  const ColPos cp = col_pos<G>(log_c);
  const uint32_t N = 1u << log_n;
  const uint64_t ip = (uint64_t)cp.l * in_ls + (uint64_t)cp.p * N;
  const uint64_t op = (uint64_t)cp.l * out_ls + (uint64_t)cp.p * N;
  ColAddr<G, G::BB0> a0(cp, log_c);
  ColAddr<G, G::BBL> al(cp, log_c);
  const auto tw = col_twiddles<W, G::UNIFORM>(tp.tw + (uint64_t)cp.l * N, N);
  const auto m = mod_for<W, LZ>(tp.lc[cp.l]);  // LZ: outputs in [0, 4q)
  W x[1][E];
  const BufView<W> src(in0 + ip, N), dst(out0 + op, N);
  // operand 1 first: out0 may alias in1 (out = a * b with out == b).  With
  // wave-uniform twiddles the registers are cheap, so operand 0's loads are
  // issued up front and land while operand 1 is transformed.
  if (in1 != nullptr) {
    const BufView<W> src1(in1 + ip, N), dst1(out1 + op, N);
    W y[1][E];
#pragma unroll
    for (int i = 0; i < E; ++i) y[0][i] = src1.ld(a0.v, i * a0.s);
    if constexpr (G::UNIFORM) {
#pragma unroll
      for (int i = 0; i < E; ++i) x[0][i] = src.ld(a0.v, i * a0.s);
    }
    xf_fwd<G, W, 1>(y, cp.xp, lds, tw, m);
#pragma unroll
    for (int i = 0; i < E; ++i) dst1.st(y[0][i], al.v, i * al.s);
    a0.refresh();
    al.refresh();
    if constexpr (!G::UNIFORM) {
#pragma unroll
      for (int i = 0; i < E; ++i) x[0][i] = src.ld(a0.v, i * a0.s);
    }
  } else {
#pragma unroll
    for (int i = 0; i < E; ++i) x[0][i] = src.ld(a0.v, i * a0.s);
  }
  xf_fwd<G, W, 1>(x, cp.xp, lds, tw, m);
#pragma unroll
  for (int i = 0; i < E; ++i) {
    if constexpr (meas_virtual(0)) {
      if (x[0][i] != (W)0xffffffffu) continue;
    }
    dst.st(x[0][i], al.v, i * al.s);
  }
}

template <class W, int LOG_R, int LOG_TC, bool LZ = false>
__global__ void __launch_bounds__((ColGeo<LOG_R, LOG_TC>::THREADS))
k_colt_inv(W* out, const W* in, const W* addend, TabPtrs<W> tp, uint32_t log_n, uint32_t log_c,
           uint32_t B, uint64_t in_ls, uint64_t out_ls, int rfold) {
  using G = ColGeo<LOG_R, LOG_TC>;
  constexpr int E = G::E;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  W* lds = (W*)smem_raw;
  const ColPos cp = col_pos<G>(log_c);
  const uint32_t N = 1u << log_n;
  const uint64_t ip = (uint64_t)cp.l * in_ls + (uint64_t)cp.p * N;
  const uint64_t op = (uint64_t)cp.l * out_ls + (uint64_t)cp.p * N;
  ColAddr<G, G::BB0> a0(cp, log_c);
  const ColAddr<G, G::BBL> al(cp, log_c);
  const LimbConst<W> lc = tp.lc[cp.l];
  const auto itw = col_twiddles<W, G::UNIFORM>(tp.itw + (uint64_t)cp.l * N, N);
  const Fold<W> f = rfold == 2 ? Fold<W>{lc.c1t, lc.c1t_p, lc.c2t, lc.c2t_p}
                  : rfold ? Fold<W>{lc.c1r, lc.c1r_p, lc.c2r, lc.c2r_p}
                          : Fold<W>{lc.c1, lc.c1_p, lc.c2, lc.c2_p};
  const BufView<W> src(in + ip, N), dst(out + op, N);
  W x[1][E];
#pragma unroll
  for (int i = 0; i < E; ++i)
    x[0][i] = meas_virtual(3) ? meas_val<W>(al.v, (uint32_t)i * al.s) : src.ld(al.v, i * al.s);
  xf_inv<G, W, 1, true>(x, cp.xp, lds, itw, mod_for<W, LZ>(lc), f);  // canonical out
  a0.refresh();
  if (addend != nullptr) {
    const BufView<W> ad(addend + op, N);
#pragma unroll
    for (int i = 0; i < E; ++i) x[0][i] = add_mod<W>(x[0][i], ad.ld(a0.v, i * a0.s), lc.q);
  }
  a0.refresh();
#pragma unroll
  for (int i = 0; i < E; ++i) dst.st(x[0][i], a0.v, i * a0.s);
}

// Tiled key-switch decomposition: grid x = group of jg target limbs j
// (fastest, so the workgroups that reduce one source tile of d mod every q_j
// run back to back and read it from L2; each loads the tile once and loops
// over its group), y = p * (C / TC) + column tile, z = source limb i.
template <class W, int LOG_R, int LOG_TC>
__global__ void __launch_bounds__((ColGeo<LOG_R, LOG_TC>::THREADS))
k_colt_decompose(W* __restrict__ S, const W* __restrict__ d, TabPtrs<W> tp, uint32_t log_n,
                 uint32_t log_c, uint32_t L, uint32_t B, uint64_t d_ls, uint32_t Lt,
                 uint32_t jg, uint32_t lift_csub) {
  using G = ColGeo<LOG_R, LOG_TC>;
  constexpr int E = G::E;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  W* lds = (W*)smem_raw;
  const uint32_t N = 1u << log_n;
  const uint32_t tpp_log = log_c - G::LOGTC;
  const uint32_t p = blockIdx.y >> tpp_log;
  const uint32_t ct = blockIdx.y & ((1u << tpp_log) - 1);
  const uint32_t i = blockIdx.z;
  // this workgroup's target limbs: [j0, j1), the source tile loaded once
  const uint32_t j0 = blockIdx.x * jg;
  const uint32_t j1 = j0 + jg < Lt ? j0 + jg : Lt;
  ColPos cp;
  cp.xp.slot = G::slot_of(threadIdx.x);
  cp.xp.tau = G::tau_of(threadIdx.x);
  cp.xp.heap = (uint32_t)G::X;
  cp.col = (ct << G::LOGTC) + cp.xp.slot;
  const ColAddr<G, G::BB0> a0(cp, log_c);
  ColAddr<G, G::BBL> al(cp, log_c);
  const BufView<W> src(d + (uint64_t)i * d_ls + (uint64_t)p * N, N);
  W raw[E];
#pragma unroll
  for (int e = 0; e < E; ++e) raw[e] = src.ld(a0.v, e * a0.s);
#pragma unroll 1
  for (uint32_t j = j0; j < j1; ++j) {
    const BufView<W> dst(S + (((uint64_t)j * L + i) * B + p) * N, N);
    const LimbConst<W> lc = tp.lc[j];
    W x[1][E];
    // alpha_i mod q_j: one conditional subtraction when every word is below
    // 2 q_j (u32 words, all target q_j > 2^30), else a Shoup reduction
    if (lift_csub) {
#pragma unroll
      for (int e = 0; e < E; ++e) x[0][e] = csub<W>(raw[e], lc.q);
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) x[0][e] = shoup_mul<W>(raw[e], (W)1, lc.one_p, lc.q);
    }
    // (the transform's LDS exchange ends in a barrier: the next j may reuse it)
    xf_fwd<G, W, 1>(x, cp.xp, lds, col_twiddles<W, G::UNIFORM>(tp.tw + (uint64_t)j * N, N),
                    mod_of(lc));
    al.refresh();
#pragma unroll
    for (int e = 0; e < E; ++e) dst.st(x[0][e], al.v, e * al.s);
  }
}

// ---- the truncated product (rnt_mul's row kernel, u32 canonical bases) ----
// The forward transforms stop two stages early: block b of 4 consecutive
// device-order words then holds the residue of the operand mod X^4 - zeta_b,
// zeta_b = psi_rev[N/4 + b]^2 = (-1)^b psi_rev[N/8 + b/2] (the heap's
// children square to their parent's root, and the odd child carries -1).
// The product of two such residues is a degree-3 negacyclic-style product;
// the inverse transforms skip the same two stages, and the inverse column
// pass folds 4/N instead of 1/N (LimbConst c1t/c2t).  Exact arithmetic, so
// the coefficient-domain result is bit-identical to the full transform's.
template <int LOG_C>
struct Trunc {
  static constexpr bool on = LOG_C >= 4 && LOG_C % 4 == 0;  // last row pass = a whole radix-16 pass
};
template <class W, int LOG_C, bool LZ>
constexpr bool trunc_mul() {
  return sizeof(W) == 4 && !LZ && Trunc<LOG_C>::on;
}

// (T * 2^-32) mod q for T < 4 q^2 (a sum of four products of canonical
// residues, q < 2^31): m = T q^-1 mod 2^32 makes T - m q a multiple of 2^32,
// and hi(T) - hi(m q) lies in (-q, 2q).
__device__ __forceinline__ uint32_t redc_sum4(uint64_t T, uint32_t q, uint32_t qinv) {
  const uint32_t m = (uint32_t)T * qinv;
  uint32_t t;
  const bool neg = __builtin_sub_overflow((uint32_t)(T >> 32), mulhi(m, q), &t);
  return neg ? t + q : csub<uint32_t>(t, q);
}

// c = a b mod (X^4 - zeta) for canonical residues, result * 2^-32 (the
// product path's Montgomery factor, folded out by the inverse column pass).
__device__ __forceinline__ void mul_mod_x4(uint32_t (&c)[4], const uint32_t* a, const uint32_t* b,
                                           uint32_t zeta, uint32_t zeta_p, uint32_t q,
                                           uint32_t qinv) {
  const Mod<uint32_t> m{q, 0u - q};
  const uint32_t b1 = shoup_mul(b[1], zeta, zeta_p, m);
  const uint32_t b2 = shoup_mul(b[2], zeta, zeta_p, m);
  const uint32_t b3 = shoup_mul(b[3], zeta, zeta_p, m);
  const uint64_t t0 = mad64(a[3], b1, mad64(a[2], b2, mad64(a[1], b3, mul64(a[0], b[0]))));
  const uint64_t t1 = mad64(a[3], b2, mad64(a[2], b3, mad64(a[1], b[0], mul64(a[0], b[1]))));
  const uint64_t t2 = mad64(a[3], b3, mad64(a[2], b[0], mad64(a[1], b[1], mul64(a[0], b[2]))));
  const uint64_t t3 = mad64(a[3], b[0], mad64(a[2], b[1], mad64(a[1], b[2], mul64(a[0], b[3]))));
  c[0] = redc_sum4(t0, q, qinv);
  c[1] = redc_sum4(t1, q, qinv);
  c[2] = redc_sum4(t2, q, qinv);
  c[3] = redc_sum4(t3, q, qinv);
}

// rnt_mul runs the Harvey-lazy kernels exactly when lazy30_ok(); otherwise
// its u32 row kernel truncates when the row length allows (Trunc<LOG_C>).
bool lazy30_ok(const Tables* t);
bool mul_truncated(const Tables* t) {
  if (t->wide || lazy30_ok(t)) return false;
  const Geom g = geom_for(t->log_n);
  return g.log_c >= 4 && g.log_c % 4 == 0;
}

// mode 0: forward rows in place; 1: inverse rows in place;
// 2: poly-mul rows: x <- INV(FWD(x) (.) FWD(y)) with Montgomery pointwise.
template <class W, int MODE, int LOG_C, bool LZ = false>
__global__ void __launch_bounds__(RowGeo<LOG_C>::THREADS, sizeof(W) == 4 ? kRowMinWaves : 1)
k_row(W* __restrict__ xg, const W* __restrict__ yg, TabPtrs<W> tp, uint32_t log_n, uint32_t B,
      uint64_t ls, uint64_t rows_total) {
  using G = RowGeo<LOG_C>;
  constexpr int E = G::E;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  W* lds = (W*)smem_raw;
  // poly index fastest: a workgroup's rows share (limb, row r) and with it
  // every twiddle, which then comes from L1 (profiles/r02_ab_row_pfast.txt)
  const RowPos rp = row_pos_pfast<G>(log_n, B, rows_total);
  const uint64_t N = 1ull << log_n;
  const uint64_t base = (uint64_t)rp.l * ls + (uint64_t)rp.p * N + (uint64_t)rp.r * G::C;
  const LimbConst<W> lc = tp.lc[rp.l];
  const Tw<W>* tw = tp.tw + (uint64_t)rp.l * N;
  const Tw<W>* itw = tp.itw + (uint64_t)rp.l * N;
  const uint32_t b0 = G::base(rp.xp.tau, G::BB0);
  const uint32_t bl = G::base(rp.xp.tau, G::BBL);
  if constexpr (MODE == 2) {
    W v[2][E];
#pragma unroll
    for (int i = 0; i < E; ++i) {
      v[0][i] = meas_virtual(1) ? meas_val<W>((uint32_t)(base + b0) + (uint32_t)i, 7u)
                                : gload(xg, base + b0 + ((uint32_t)i << G::BB0));
      v[1][i] = gload(yg, base + b0 + ((uint32_t)i << G::BB0));
    }
    const auto mo = mod_for<W, LZ>(lc);
    W z[1][E];
    if constexpr (trunc_mul<W, LOG_C, LZ>()) {
      // every pass but the last in full, the last without its two stages
      if constexpr (G::P > 1) fwd_pass<G, W, 2, 0>(v, rp.xp, lds, tw, mo);
      if constexpr (G::P > 2) fwd_pass<G, W, 2, 1>(v, rp.xp, lds, tw, mo);
      if constexpr (G::P > 3) fwd_pass<G, W, 2, 2>(v, rp.xp, lds, tw, mo);
      fwd_pass<G, W, 2, G::P - 1, 2>(v, rp.xp, lds, tw, mo);
      // blocks t of 4 registers: device positions r*C + tau*E + 4t (G::BBL == 0)
      static_assert(G::BBL == 0 && E == 16, "truncated product layout");
      const uint32_t zb = (uint32_t)(N >> 3) + ((rp.r * (uint32_t)G::C) >> 3) + (rp.xp.tau << 1);
      const Tw<W> zw[2] = {tw[zb], tw[zb + 1]};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const Tw<W> w = zw[t >> 1];
        const uint32_t zeta = (t & 1) ? (uint32_t)lc.q - w.w : w.w;  // (-1)^b psi_rev[N/8 + b/2]
        const uint32_t zeta_p = (t & 1) ? ~w.p : w.p;                  // Shoup companion of q - w
        uint32_t c[4];
        mul_mod_x4(c, &v[0][4 * t], &v[1][4 * t], zeta, zeta_p, lc.q, lc.qinv);
#pragma unroll
        for (int k = 0; k < 4; ++k) z[0][4 * t + k] = c[k];
      }
      inv_pass<G, W, 1, G::P - 1, false, 2>(z, rp.xp, lds, itw, mo, Fold<W>{});
      if constexpr (G::P > 3) inv_pass<G, W, 1, 2, false>(z, rp.xp, lds, itw, mo, Fold<W>{});
      if constexpr (G::P > 2) inv_pass<G, W, 1, 1, false>(z, rp.xp, lds, itw, mo, Fold<W>{});
      if constexpr (G::P > 1) inv_pass<G, W, 1, 0, false>(z, rp.xp, lds, itw, mo, Fold<W>{});
    } else {
    xf_fwd<G, W, 2>(v, rp.xp, lds, tw, mo);
    if constexpr (LZ) {
      // [0, 4q) inputs -> [0, 2q); a b < 4q^2 < q 2^32, so the Montgomery
      // quotient leaves (ab + mq) / 2^32 < 2q: the GS passes' input range
#pragma unroll
      for (int i = 0; i < E; ++i) {
        const uint32_t a = csub<uint32_t>(v[0][i], mo.q2), b = csub<uint32_t>(v[1][i], mo.q2);
        const uint64_t t = mul64(a, b);
        const uint32_t mm = (uint32_t)t * (0u - (uint32_t)lc.qinv);
        z[0][i] = (uint32_t)(mad64(mm, (uint32_t)lc.q, t) >> 32);
      }
    } else {
#pragma unroll
      for (int i = 0; i < E; ++i) z[0][i] = mont_mul<W>(v[0][i], v[1][i], lc.q, lc.qinv);
    }
    xf_inv<G, W, 1>(z, rp.xp, lds, itw, mo);
    }
    if (rp.active) {
#pragma unroll
      for (int i = 0; i < E; ++i) {
        if constexpr (meas_virtual(2)) {
          if (z[0][i] != (W)0xffffffffu) continue;
        }
        gstore(xg, base + b0 + ((uint32_t)i << G::BB0), z[0][i]);
      }
    }
  } else if constexpr (MODE == 0) {
    W v[1][E];
#pragma unroll
    for (int i = 0; i < E; ++i) v[0][i] = xg[base + b0 + ((uint32_t)i << G::BB0)];
    xf_fwd<G, W, 1>(v, rp.xp, lds, tw, mod_of(lc));
    if (rp.active) {
#pragma unroll
      for (int i = 0; i < E; ++i) xg[base + bl + ((uint32_t)i << G::BBL)] = v[0][i];
    }
  } else {
    W v[1][E];
#pragma unroll
    for (int i = 0; i < E; ++i) v[0][i] = xg[base + bl + ((uint32_t)i << G::BBL)];
    xf_inv<G, W, 1>(v, rp.xp, lds, itw, mod_of(lc));
    if (rp.active) {
#pragma unroll
      for (int i = 0; i < E; ++i) xg[base + b0 + ((uint32_t)i << G::BB0)] = v[0][i];
    }
  }
}

// ---- whole-plane product (rnt_mul at N = 2^16, u32 canonical bases) ------
// Two launches per batch instead of three, 5 planes of HBM traffic per
// (poly, limb) instead of 9 (the 5-plane traffic measured
// 142k poly-muls/s against 122k for the shipped 9):
//   k_plane_fwd: a -> a^ (the whole truncated forward transform of one
//                plane in one workgroup's registers; a^ goes to a private
//                layout), 2 planes;
//   k_plane_mul: b -> b^ the same way, a^ (x) b^ (degree-3 block products),
//                the whole truncated inverse, c, 3 planes.
// A workgroup = 1024 threads holds one 2^16-word plane, 64 words a thread.
// Thread t = (w << 6) | lam (wave w, lane lam); the 16-bit index i is split
// three ways:
//   L0  i = (r << 10) | (w << 6) | lam     registers: bits 15..10, coalesced
//   L1  i = (w << 12) | (r << 6) | lam     registers: bits 11..6
//   L2  i = (w << 12) | (lam << 6) | r     registers: bits 5..0
// and the network is the same merged negacyclic CT / GS heap as the
// four-step kernels (node = (2^16 + i) >> (b + 1) at bit b), so a^ and the
// product equal theirs word for word.  Pass A runs bits 15..10 in L0, pass
// B bits 9..6 in L1 (both with wave-uniform twiddle nodes: scalar loads),
// pass C bits 5..2 in L2 (bits 1..0 are the truncated stages).
//   X1 (L0 <-> L1) keeps the lanes and moves words between waves: 128 KiB
//      of LDS in two rounds, split on index bit 10 (a register bit on both
//      sides, so a round reads back exactly the registers it wrote).
//   X2 (L1 <-> L2) stays inside each wave: lane bits 5, 4 trade places with
//      register bits 5, 4 through v_permlane32_swap / v_permlane16_swap,
//      and the remaining 16 x 16 transposes go through a wave-private LDS
//      buffer in four rounds, with no workgroup barrier.
// The physical register of a logical one is a compile-time permutation
// (slot1, shared by L1 and L2).
#ifndef RNT_PLANE_EXP
#define RNT_PLANE_EXP 0
#endif
namespace plane {
constexpr int T = 1024;
constexpr int XS = 17;                  // X2 buffer row stride (words): conflict-free both ways
constexpr int XW = 64 * XS;             // words of one X2 buffer
constexpr int LDS_WORDS = 16 * 2 * XW;  // two X2 buffers per wave; >= 2^15 (an X1 round)
static_assert(LDS_WORDS >= (1 << 15), "X1 round");
__host__ __device__ constexpr int slot0(int r) { return r; }
__host__ __device__ constexpr int slot1(int r) { return 2 * (((r >> 5) << 4) | (r & 15)) + ((r >> 4) & 1); }
__host__ __device__ constexpr int slot2(int r) { return slot1(r); }
template <int L>
__host__ __device__ constexpr int slot(int r) {
  return L == 0 ? slot0(r) : slot1(r);
}
}  // namespace plane

// CT stages on logical register bits SLHI .. SLLO of layout LY (index bits
// [BB, BB + 6)); node0 = 2^16 + the thread's index with register bits 0.
// Twiddles in chunks of CH per stage (bounded registers beside the plane).
// As in pass_ct, outputs the next stage of the pass only multiplies stay
// in [0, 2q); the last stage leaves everything canonical.  Stages and
// chunks are template recursions, so every register index is a
// compile-time constant (a loop the unroller gave up on would put the
// plane in scratch memory).
template <int LY, int BB, int SL, int SLLO, int M0, int CH, class TS>
__device__ __forceinline__ void plane_ct_chunks(uint32_t (&x)[64], uint32_t nb, const TS& tw,
                                                const Mod<uint32_t>& mo) {
  constexpr int d = 1 << SL, cnt = 32 >> SL, n = (cnt - M0) < CH ? (cnt - M0) : CH;
  Tw<uint32_t> t[n];
#pragma unroll
  for (int j = 0; j < n; ++j)
    t[j] = (RNT_PLANE_EXP & 8) ? Tw<uint32_t>{12345u + (uint32_t)j, 54321u} : tw_get<uint32_t>(tw, nb, (uint32_t)(M0 + j));
#pragma unroll
  for (int j = 0; j < n; ++j) {
#pragma unroll
    for (int e = 0; e < d; ++e) {
      const int i = ((M0 + j) << (SL + 1)) | e;
      if (SL > SLLO && (i & (d >> 1)))
        ct_bfly_lazy(x[plane::slot<LY>(i)], x[plane::slot<LY>(i | d)], t[j].w, t[j].p, mo);
      else
        ct_bfly(x[plane::slot<LY>(i)], x[plane::slot<LY>(i | d)], t[j].w, t[j].p, mo);
    }
  }
  if constexpr (M0 + CH < cnt) plane_ct_chunks<LY, BB, SL, SLLO, M0 + CH, CH>(x, nb, tw, mo);
}
template <int LY, int BB, int SL, int SLLO, int CH, class TS>
__device__ __forceinline__ void plane_ct(uint32_t (&x)[64], uint32_t node0, const TS& tw,
                                         const Mod<uint32_t>& mo) {
  plane_ct_chunks<LY, BB, SL, SLLO, 0, CH>(x, node0 >> (BB + SL + 1), tw, mo);
  if constexpr (SL > SLLO) plane_ct<LY, BB, SL - 1, SLLO, CH>(x, node0, tw, mo);
}

// GS stages on logical register bits SLLO .. SLHI; FOLD: the stage at
// index bit 15 applies the folded constants (4/N with the Montgomery
// factor, LimbConst c1t/c2t) instead of its twiddle.
template <int LY, int BB, int SL, int M0, int CH, class TS>
__device__ __forceinline__ void plane_gs_chunks(uint32_t (&x)[64], uint32_t nb, const TS& itw,
                                                const Mod<uint32_t>& mo) {
  constexpr int d = 1 << SL, cnt = 32 >> SL, n = (cnt - M0) < CH ? (cnt - M0) : CH;
  Tw<uint32_t> t[n];
#pragma unroll
  for (int j = 0; j < n; ++j)
    t[j] = (RNT_PLANE_EXP & 8) ? Tw<uint32_t>{12345u + (uint32_t)j, 54321u} : tw_get<uint32_t>(itw, nb, (uint32_t)(M0 + j));
#pragma unroll
  for (int j = 0; j < n; ++j) {
#pragma unroll
    for (int e = 0; e < d; ++e) {
      const int i = ((M0 + j) << (SL + 1)) | e;
      gs_bfly(x[plane::slot<LY>(i)], x[plane::slot<LY>(i | d)], t[j].w, t[j].p, mo);
    }
  }
  if constexpr (M0 + CH < cnt) plane_gs_chunks<LY, BB, SL, M0 + CH, CH>(x, nb, itw, mo);
}
template <int LY, int BB, int SL, int SLHI, int CH, bool FOLD, class TS>
__device__ __forceinline__ void plane_gs(uint32_t (&x)[64], uint32_t node0, const TS& itw,
                                         const Mod<uint32_t>& mo, const Fold<uint32_t>& f) {
  constexpr int d = 1 << SL;
  if constexpr (FOLD && BB + SL + 1 == 16) {
#pragma unroll
    for (int e = 0; e < d; ++e) {  // the top stage: d = 32, one group
      const uint32_t u = x[plane::slot<LY>(e)], v = x[plane::slot<LY>(e | d)];
      x[plane::slot<LY>(e)] = shoup_mul(u + v, f.c1, f.c1p, mo);
      x[plane::slot<LY>(e | d)] = shoup_mul(u - v + mo.q, f.c2, f.c2p, mo);
    }
  } else {
    plane_gs_chunks<LY, BB, SL, 0, CH>(x, node0 >> (BB + SL + 1), itw, mo);
  }
  if constexpr (SL < SLHI) plane_gs<LY, BB, SL + 1, SLHI, CH, FOLD>(x, node0, itw, mo, f);
}

// X1, L0 <-> L1 through LDS.  Round h carries the words with index bit
// 10 == h: L0 registers 2k + h, L1 logical registers r1 = ((k >> 4) << 5) |
// (h << 4) | (k & 15), both in physical register 2k + h.  LDS word = the 15
// other index bits; every access is 64 consecutive words per wave.
// SYNC_FIRST: other waves may still be reading their X2 buffers.
template <bool TO_L1, bool SYNC_FIRST>
__device__ __forceinline__ void plane_x1(uint32_t (&x)[64], uint32_t* lds, uint32_t t) {
  const uint32_t w = t >> 6, lam = t & 63u;
  if constexpr ((RNT_PLANE_EXP & 16) != 0) return;
  if constexpr (SYNC_FIRST) __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const uint32_t j0 = ((uint32_t)k << 10) | t;
      const uint32_t j1 = ((((w << 1) | ((uint32_t)k >> 4))) << 10) | (((uint32_t)k & 15u) << 6) | lam;
      lds[TO_L1 ? j0 : j1] = x[2 * k + h];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const uint32_t j0 = ((uint32_t)k << 10) | t;
      const uint32_t j1 = ((((w << 1) | ((uint32_t)k >> 4))) << 10) | (((uint32_t)k & 15u) << 6) | lam;
      x[2 * k + h] = lds[TO_L1 ? j1 : j0];
    }
    __syncthreads();
  }
}

// Lane bit 5 <-> L1 register bit 5 and lane bit 4 <-> register bit 4
// (self-inverse; the two commute).
__device__ __forceinline__ void plane_swap54(uint32_t (&x)[64]) {
#pragma unroll
  for (int m = 0; m < 64; ++m) {
    if (m & 32) continue;
    const auto r = __builtin_amdgcn_permlane32_swap(x[plane::slot1(m)], x[plane::slot1(m | 32)], false, false);
    x[plane::slot1(m)] = r[0];
    x[plane::slot1(m | 32)] = r[1];
  }
#pragma unroll
  for (int m = 0; m < 64; ++m) {
    if (m & 16) continue;
    const auto r = __builtin_amdgcn_permlane16_swap(x[plane::slot1(m)], x[plane::slot1(m | 16)], false, false);
    x[plane::slot1(m)] = r[0];
    x[plane::slot1(m | 16)] = r[1];
  }
}

// X2, L1 <-> L2 inside each wave.  After plane_swap54 a lane holds index
// bits 11, 10 (lane bits 5, 4) and 3..0, a register m holds bits 5, 4
// (m >> 4) and 9..6 (m & 15); per group g = m >> 4 the 16 x 16 blocks of
// (m & 15) x (lane & 15) transpose through the wave's LDS buffer: word
// (lane, m & 15) at lane * 17 + (m & 15), read back by lane' as register
// (g << 4) | c from lane (lane' & 48) | c, column lane' & 15 (both
// directions 64 distinct banks).  LDS instructions of one wave execute in
// order, so the reads see the same wave's writes; two buffers alternate.
template <bool TO_L2>
__device__ __forceinline__ void plane_x2(uint32_t (&x)[64], uint32_t* lds, uint32_t t) {
  const uint32_t w = t >> 6, lam = t & 63u;
  if constexpr ((RNT_PLANE_EXP & 16) != 0) return;
  if constexpr (TO_L2) plane_swap54(x);
  const uint32_t a15 = lam * plane::XS;                          // + (m & 15)
  const uint32_t a2 = (lam & 48u) * plane::XS + (lam & 15u);     // + c * XS
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    uint32_t* buf = lds + (w * 2u + (uint32_t)(g & 1)) * plane::XW;
#pragma unroll
    for (int j = 0; j < 16; ++j) buf[TO_L2 ? a15 + j : a2 + j * plane::XS] = x[plane::slot1((g << 4) | j)];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int c = 0; c < 16; ++c) x[plane::slot1((g << 4) | c)] = buf[TO_L2 ? a2 + c * plane::XS : a15 + c];
    __builtin_amdgcn_wave_barrier();
  }
  if constexpr (!TO_L2) plane_swap54(x);
}

// One workgroup per CU and equal work per workgroup keep every CU's load,
// compute and store phases in step across the chip, so the loads of all
// CUs meet at the HBM together while the VALUs idle, and then the other
// way round.  Delaying the first workgroup of every other CU by `ticks`
// of the 100 MHz real-time counter once shifts that CU's phase for the
// rest of the launch (its next workgroups start when the previous one
// ends), so half the CUs load while the other half compute.
__device__ __forceinline__ void plane_stagger(uint32_t ticks) {
  if (ticks == 0) return;
  const uint32_t id = blockIdx.x + blockIdx.y * gridDim.x;
  if (id >= 256u || !((id >> 3) & 1u)) return;  // first wave, every other CU of each XCD
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

// Phase timeline of the plane kernels (measurement build only:
// tools/build_variant.sh trace -DRNT_PLANE_TRACE; tools/plane_trace.py).
// Lane 0 of every wave of the first 4096 workgroups waits for the wave's
// own memory operations and stamps the 100 MHz real-time counter at each
// phase boundary.
#ifdef RNT_PLANE_TRACE
constexpr int kTraceWg = 4096, kTraceStamps = 16;
__device__ uint64_t g_plane_trace[2 * kTraceWg * 16 * kTraceStamps];
#define PLANE_STAMP(K, S)                                                                       \
  do {                                                                                          \
    const uint32_t wg_ = trace_id;                                                              \
    if ((threadIdx.x & 63u) == 0 && wg_ < (uint32_t)kTraceWg) {                                 \
      __builtin_amdgcn_s_waitcnt(0);                                                            \
      g_plane_trace[(((K) * kTraceWg + wg_) * 16 + (threadIdx.x >> 6)) * kTraceStamps + (S)] =  \
          __builtin_amdgcn_s_memrealtime();                                                     \
    }                                                                                           \
  } while (0)
#else
#define PLANE_STAMP(K, S) \
  do {                    \
  } while (0)
#endif

// Measurement builds (tools/build_variant.sh, wrong results by design):
// RNT_PLANE_EXP bit 0: pass C / inverse pass C twiddles wave-uniform;
// bit 1: no plane loads (synthetic words); bit 2: no plane stores;
// bit 3: no twiddle loads in the passes (one constant); bit 4: no X1 / X2.

// Load the L0 plane at src (64 coalesced dword loads a thread).
__device__ __forceinline__ void plane_load(uint32_t (&x)[64], const uint32_t* src, uint32_t t) {
  if constexpr ((RNT_PLANE_EXP & 2) != 0) {
#pragma unroll
    for (int r = 0; r < 64; ++r) x[r] = (t * 2654435761u + (uint32_t)r * 40503u) >> 2;
    return;
  }
  const BufView<uint32_t> g(src, 1u << 16);
#pragma unroll
  for (int r = 0; r < 64; ++r) x[r] = g.ld(t, (uint32_t)r << 10);
}

// The truncated forward transform of the plane in x (L0 in, L2 out).
// SYNC1: other waves may still be using the LDS (their X2 buffers of an
// earlier transform) when X1 starts.
template <int K, bool SYNC1>
__device__ __forceinline__ void plane_fwd(uint32_t (&x)[64], uint32_t* lds, uint32_t t,
                                          const Tw<uint32_t>* tw, const Mod<uint32_t>& mo, uint32_t trace_id) {
  (void)trace_id;
  const uint32_t N = 1u << 16;
  const TwScalar<uint32_t> tws{(const RNT_CONST_AS Tw<uint32_t>*)tw};
  // pass A's twiddle nodes ((2^16 + i) >> (b + 1), b >= 10) depend on
  // register bits only, pass B's (b >= 6) on register and wave bits: both
  // wave-uniform (scalar loads)
  plane_ct<0, 10, 5, 0, 32>(x, N, tws, mo);
  PLANE_STAMP(K, 2);
  plane_x1<true, SYNC1>(x, lds, t);
  PLANE_STAMP(K, 3);
  const uint32_t wu = __builtin_amdgcn_readfirstlane(t >> 6);
  plane_ct<1, 6, 3, 0, 16>(x, N + (wu << 12), tws, mo);
  PLANE_STAMP(K, 4);
  plane_x2<true>(x, lds, t);
  PLANE_STAMP(K, 5);
  if constexpr ((RNT_PLANE_EXP & 1) != 0)
    plane_ct<2, 0, 5, 2, 8>(x, N, tws, mo);
  else
    plane_ct<2, 0, 5, 2, 8>(x, N + (t << 6), tw, mo);
  PLANE_STAMP(K, 6);
}

// The rest of the product once b^ is in x (L2): the degree-3 block
// products with a^ (ah: the private layout, block kk of thread t at
// ah[kk * 1024 + t]), the whole truncated inverse, c stored in L0.
template <int K>
__device__ __forceinline__ void plane_mul_tail(uint32_t (&x)[64], uint32_t* lds, uint32_t t, const uint4* ah,
                                               uint32_t* c, const Tw<uint32_t>* tw, const Tw<uint32_t>* itw,
                                               const LimbConst<uint32_t>& lc, const Mod<uint32_t>& mo,
                                               uint32_t trace_id) {
  (void)trace_id;
  const uint32_t n0 = 1u << 16;
  // degree-3 block products: block (t << 4) | kk, zeta = (-1)^kk psi_rev[N/8 + (t << 3) + kk/2]
  const uint32_t zb = (n0 >> 3) + (t << 3);
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    const uint4 av = (RNT_PLANE_EXP & 2) != 0 ? make_uint4(t * 7u + kk, t * 11u, t + 3u * kk, t ^ 0x55u)
                                              : ah[kk * 1024 + t];
    const uint32_t aa[4] = {av.x, av.y, av.z, av.w};
    const uint32_t bb[4] = {x[plane::slot2(4 * kk)], x[plane::slot2(4 * kk + 1)], x[plane::slot2(4 * kk + 2)],
                            x[plane::slot2(4 * kk + 3)]};
    const Tw<uint32_t> w = tw[zb + (kk >> 1)];
    const uint32_t zeta = (kk & 1) ? lc.q - w.w : w.w;
    const uint32_t zeta_p = (kk & 1) ? ~w.p : w.p;
    uint32_t cc[4];
    mul_mod_x4(cc, aa, bb, zeta, zeta_p, lc.q, lc.qinv);
#pragma unroll
    for (int e = 0; e < 4; ++e) x[plane::slot2(4 * kk + e)] = cc[e];
  }
  PLANE_STAMP(K, 7);
  const TwScalar<uint32_t> itws{(const RNT_CONST_AS Tw<uint32_t>*)itw};
  if constexpr ((RNT_PLANE_EXP & 1) != 0)
    plane_gs<2, 0, 2, 5, 8, false>(x, n0, itws, mo, Fold<uint32_t>{});
  else
    plane_gs<2, 0, 2, 5, 8, false>(x, n0 + (t << 6), itw, mo, Fold<uint32_t>{});
  PLANE_STAMP(K, 8);
  plane_x2<false>(x, lds, t);
  PLANE_STAMP(K, 9);
  const uint32_t wu = __builtin_amdgcn_readfirstlane(t >> 6);
  plane_gs<1, 6, 0, 3, 16, false>(x, n0 + (wu << 12), itws, mo, Fold<uint32_t>{});
  PLANE_STAMP(K, 10);
  plane_x1<false, true>(x, lds, t);  // other waves may still be in their X2
  PLANE_STAMP(K, 11);
  plane_gs<0, 10, 0, 5, 32, true>(x, n0, itws, mo, Fold<uint32_t>{lc.c1t, lc.c1t_p, lc.c2t, lc.c2t_p});
  PLANE_STAMP(K, 12);
  if ((RNT_PLANE_EXP & 4) != 0 && x[0] != 0xffffffffu) return;
  const BufView<uint32_t> dst(c, n0);
#pragma unroll
  for (int r = 0; r < 64; ++r) dst.st(x[r], t, (uint32_t)r << 10);
  PLANE_STAMP(K, 13);
}

// a^ in the private layout: block kk (4 words) of thread t at (kk * 1024 + t) * 4
__device__ __forceinline__ void plane_store_hat(uint4* dst, const uint32_t (&x)[64], uint32_t t) {
  if ((RNT_PLANE_EXP & 4) != 0 && x[0] != 0xffffffffu) return;
#pragma unroll
  for (int kk = 0; kk < 16; ++kk)
    dst[kk * 1024 + t] = make_uint4(x[plane::slot2(4 * kk)], x[plane::slot2(4 * kk + 1)],
                                    x[plane::slot2(4 * kk + 2)], x[plane::slot2(4 * kk + 3)]);
}

// One workgroup per plane, grid (B, L).
__global__ void __launch_bounds__(plane::T, 1)
k_plane_fwd(uint32_t* __restrict__ ahat, const uint32_t* __restrict__ a, TabPtrs<uint32_t> tp, uint64_t ls,
            uint32_t stagger) {
  plane_stagger(stagger);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  uint32_t* lds = (uint32_t*)smem_raw;
  const uint32_t t = threadIdx.x, poly = blockIdx.x, l = blockIdx.y;
  const uint32_t trace_id = poly + l * gridDim.x;
  PLANE_STAMP(0, 0);
  const uint64_t N = 1ull << 16;
  const uint64_t off = (uint64_t)l * ls + (uint64_t)poly * N;
  uint32_t x[64];
  plane_load(x, a + off, t);
  PLANE_STAMP(0, 1);
  plane_fwd<0, false>(x, lds, t, tp.tw + (uint64_t)l * N, mod_of(tp.lc[l]), trace_id);
  plane_store_hat((uint4*)(ahat + off), x, t);
  PLANE_STAMP(0, 7);
}

__global__ void __launch_bounds__(plane::T, 1)
k_plane_mul(uint32_t* __restrict__ c, const uint32_t* __restrict__ b, const uint32_t* __restrict__ ahat,
            TabPtrs<uint32_t> tp, uint64_t ls, uint32_t stagger) {
  plane_stagger(stagger);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  uint32_t* lds = (uint32_t*)smem_raw;
  const uint32_t t = threadIdx.x, poly = blockIdx.x, l = blockIdx.y;
  const uint32_t trace_id = poly + l * gridDim.x;
  PLANE_STAMP(1, 0);
  const uint64_t N = 1ull << 16;
  const uint64_t off = (uint64_t)l * ls + (uint64_t)poly * N;
  const LimbConst<uint32_t> lc = tp.lc[l];
  const Mod<uint32_t> mo = mod_of(lc);
  const Tw<uint32_t>* tw = tp.tw + (uint64_t)l * N;
  uint32_t x[64];
  plane_load(x, b + off, t);
  PLANE_STAMP(1, 1);
  plane_fwd<1, false>(x, lds, t, tw, mo, trace_id);
  plane_mul_tail<1>(x, lds, t, (const uint4*)(ahat + off), c + off, tw, tp.itw + (uint64_t)l * N, lc, mo, trace_id);
}

// Both halves in one workgroup (RNT_PLANE=3): a -> a^ through the scratch
// plane, which the same threads read back ~40 us later (so the read is
// served by the Infinity Cache or L2 rather than HBM), then b -> c as
// k_plane_mul.  One launch per batch; the store of a^ and the load of b
// are back to back and overlap.
__global__ void __launch_bounds__(plane::T, 1)
k_plane_fused(uint32_t* __restrict__ c, const uint32_t* a, const uint32_t* b, uint32_t* __restrict__ scratch,
              TabPtrs<uint32_t> tp, uint64_t ls) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  uint32_t* lds = (uint32_t*)smem_raw;
  const uint32_t t = threadIdx.x, poly = blockIdx.x, l = blockIdx.y;
  const uint32_t trace_id = poly + l * gridDim.x;
  const uint64_t N = 1ull << 16;
  const uint64_t off = (uint64_t)l * ls + (uint64_t)poly * N;
  const LimbConst<uint32_t> lc = tp.lc[l];
  const Mod<uint32_t> mo = mod_of(lc);
  const Tw<uint32_t>* tw = tp.tw + (uint64_t)l * N;
  uint4* ah = (uint4*)(scratch + off);
  uint32_t x[64];
  plane_load(x, a + off, t);
  plane_fwd<0, false>(x, lds, t, tw, mo, trace_id);
  plane_store_hat(ah, x, t);
  plane_load(x, b + off, t);
  plane_fwd<1, true>(x, lds, t, tw, mo, trace_id);
  // a^ comes back from this thread's own stores above; an opaque copy of
  // the base keeps the compiler from holding the 16 store addresses live
  // (in scratch) across b's transform
  const uint4* ah2 = ah;
  asm volatile("" : "+s"(ah2));
  plane_mul_tail<1>(x, lds, t, ah2, c + off, tw, tp.itw + (uint64_t)l * N, lc, mo, trace_id);
}

#ifdef RNT_PLANE_TRACE
extern "C" __attribute__((visibility("default"))) int rnt_debug_plane_trace(uint64_t* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_plane_trace), sizeof(g_plane_trace));
}
#endif

// Words per padded LDS key row: C + C/16 (ks_pad's 4 per 64), rounded up to
// a whole 16-byte unit (the host sizes the LDS with the same formula).
template <class W>
__host__ __device__ constexpr int ks_kpad_words(int c) {
  constexpr int V = 16 / (int)sizeof(W);
  return (c + (c >> 4) + V - 1) / V * V;
}
// Padded LDS position of key word w: 4 pad words per 64, so the 16-byte
// reads of 16 lanes at 64-byte strides (a row's E = 16 consecutive words per
// thread) start on 16 distinct 4-bank groups, and 16-byte alignment holds.
__device__ __forceinline__ uint32_t ks_pad(uint32_t w) { return w + ((w >> 6) << 2); }
// 16 bytes of LDS into registers (p is 16-byte aligned by construction:
// key rows start on ks_kpad_words boundaries, and ks_pad keeps every
// thread's run of E words within a row on a 16-byte boundary).
template <class W>
__device__ __forceinline__ void ks_lds_read16(W (&o)[16 / sizeof(W)], const W* p) {
  const uint4 v = *(const uint4*)p;
  if constexpr (sizeof(W) == 4) {
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  } else {
    o[0] = (uint64_t)v.x | ((uint64_t)v.y << 32);
    o[1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
  }
}

// Lazy multiply-accumulate of the u32 key-switch sum (q < 2^31): the
// accumulator lives in [0, 2q) and a term is the Montgomery product without
// its final subtraction, t = (x k + m q) / 2^32 in [0, 2q).  acc + t < 4q
// needs 33 bits: the add's carry and the borrow of subtracting 2q decide the
// select (acc + t >= 2q iff carry or no borrow), so a term costs the three
// half-rate products plus add, subtract and select, where mont_mul + add_mod
// took two more full-rate ops.  The sum is made canonical once, after the
// source-limb loop.
__device__ __forceinline__ uint32_t mac_lazy(uint32_t acc, uint32_t x, uint32_t k, uint32_t q,
                                             uint32_t q2, uint32_t nqinv) {
  const uint64_t T = mul64(x, k);
  const uint32_t m = (uint32_t)T * nqinv;  // -T q^-1 mod 2^32
  const uint32_t t = (uint32_t)(mad64(m, q, T) >> 32);
  uint32_t s, d;
  const bool carry = __builtin_add_overflow(acc, t, &s);
  const bool borrow = __builtin_sub_overflow(s, q2, &d);
  return (carry || !borrow) ? d : s;
}

// Key-switch rows.  A workgroup owns row r of target limb j for RPW
// consecutive polys p (grid: (j, r) major, poly group minor, dealt so the
// workgroups of one (j, r) share an XCD).  For every source limb i: forward
// rows of S[j][i][p], multiply-accumulate with the NTT-resident keys; then
// the inverse rows of both accumulators.  The key rows of (i, j, r) are the
// same for every poly of the workgroup, so its threads load them once per i,
// cooperatively and together with the S rows, into a double-buffered LDS
// slot, and the accumulate reads them back from LDS: one global round trip
// per source limb instead of three (S, then key_b, then key_a), and 2 key
// words per thread instead of 2E (A/B: profiles/r02_ab_ks_rows.txt).
template <class W, int LOG_C, int NP>
__global__ void __launch_bounds__(RowGeo<LOG_C>::THREADS, sizeof(W) == 4 ? kKsMinWaves : 1)
k_ks_rows(W* __restrict__ u0, W* __restrict__ u1, const W* __restrict__ S,
          const W* __restrict__ key_a, const W* __restrict__ key_b, uint64_t key_ls,
          const W* __restrict__ init0, const W* __restrict__ init1, uint64_t init_ls,
          TabPtrs<W> tp, uint32_t log_n, uint32_t L, uint32_t B, uint64_t ls, uint32_t pgroups,
          uint32_t nblocks) {
  using G = RowGeo<LOG_C>;
  constexpr int E = G::E;
  constexpr int C = G::C;
  // padded key row (ks_pad), rounded up to 16 bytes so every key row --
  // hence every thread's 16-byte LDS read -- starts 16-byte aligned also for
  // short rows (C = 16/32, where C + C/16 alone is 17 or 34 words)
  constexpr int KPAD = ks_kpad_words<W>(C);
  // NP polys x KROWS consecutive rows per workgroup (NP = RPW: one row r
  // for RPW polys; NP = 1: one poly, RPW rows); the key rows of a source
  // limb are staged per workgroup, KROWS of each key
  static_assert(NP >= 1 && G::RPW % NP == 0, "polys per workgroup");
  constexpr int KROWS = G::RPW / NP;
  constexpr bool WIDE = NP < G::RPW;
  constexpr int KPT = (2 * KROWS * C + G::THREADS - 1) / G::THREADS;  // key words per thread per i
  constexpr bool kKeyGlds = sizeof(W) == 4 && C >= 64 && (NP > 1 || LOG_C >= kKsGldsWideMinLogC);
  // two key buffers (the next limb's keys are written while the last ones
  // may still be read) when they fit beside the exchange region in a
  // quarter of the LDS; else one buffer and a barrier per limb
  constexpr bool KDOUBLE =
      (size_t)(G::REGION + 4 * KROWS * KPAD) * sizeof(W) <= 40u * 1024u || KROWS == 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  W* lds = (W*)smem_raw;
  // [buffers][key_b rows | key_a rows]
  W* kbuf = lds + G::REGION;
  // XCD-aware deal: hardware block b runs on XCD b % 8; consecutive logical
  // blocks (one (j, r), successive poly groups) get the same b % 8
  const uint32_t per_xcd = (nblocks + 7) / 8;
  const uint32_t wg = (blockIdx.x & 7u) * per_xcd + (blockIdx.x >> 3);
  if (wg >= nblocks) return;  // the whole workgroup: no barrier is left waiting
  const uint32_t log_r = log_n - G::LOGC;
  const uint32_t pg = wg % pgroups;
  const uint32_t jr = wg / pgroups;
  RowPos rp;
  rp.xp.slot = G::slot_of(threadIdx.x);
  rp.xp.tau = G::tau_of(threadIdx.x);
  uint32_t rbase;  // first row of the workgroup's key rows
  if constexpr (WIDE) {
    // jr = (j, row group of KROWS rows); slot = row-in-group * NP + poly-in-group
    const uint32_t lg = log_r - (uint32_t)__builtin_ctz(KROWS);
    rbase = (jr & ((1u << lg) - 1u)) * KROWS;
    rp.r = rbase + rp.xp.slot / NP;
    rp.l = jr >> lg;
    const uint32_t p = pg * NP + rp.xp.slot % NP;
    rp.active = p < B;
    rp.p = rp.active ? p : B - 1;
  } else {
    rp.r = jr & ((1u << log_r) - 1u);
    rbase = rp.r;
    rp.l = jr >> log_r;
    const uint32_t p = pg * G::RPW + rp.xp.slot;
    rp.active = p < B;
    rp.p = rp.active ? p : B - 1;  // inactive slots read a valid row, store nothing
  }
  rp.xp.heap = (1u << log_n) + rp.r * (uint32_t)G::C;
  const uint64_t N = 1ull << log_n;
  const uint32_t j = rp.l;
  const uint64_t rowoff = (uint64_t)rp.r * G::C;
  const uint64_t ibase = (uint64_t)j * init_ls + (uint64_t)rp.p * N + rowoff;
  const LimbConst<W> lc = tp.lc[j];
  const Tw<W>* tw = tp.tw + (uint64_t)j * N;
  const Tw<W>* itw = tp.itw + (uint64_t)j * N;
  const uint32_t b0 = G::base(rp.xp.tau, G::BB0);
  const uint32_t bl = G::base(rp.xp.tau, G::BBL);
  // u32: the lazy [0, 2q) accumulation (mac_lazy); u64: mont_mul + add_mod
  constexpr bool kLazy = sizeof(W) == 4;
  W nqinv = (W)0 - lc.qinv;
  asm volatile("" : "+s"(nqinv));  // keeps T * (-q^-1) one multiply (not -(T q^-1))
  const W q2 = lc.q + lc.q;
  W acc[2][E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const uint32_t pos = bl + ((uint32_t)e << G::BBL);
    acc[0][e] = init0 ? init0[ibase + pos] : (W)0;
    acc[1][e] = init1 ? init1[ibase + pos] : (W)0;
  }
#pragma unroll 1
  for (uint32_t i = 0; i < L; ++i) {
    // this limb's key rows (key poly i, limb j, rows rbase ..; limb stride
    // key_ls) and S rows: one batch of loads, one wait
    const uint64_t sbase = (((uint64_t)j * L + i) * B + rp.p) * N + rowoff;
    const uint64_t kbase = (uint64_t)j * key_ls + (uint64_t)i * N + (WIDE ? (uint64_t)rbase * G::C : rowoff);
    constexpr uint32_t KW = (uint32_t)(KROWS * C);  // words per key
    W x[1][E];
    // one key buffer: every thread's reads of the previous limb's keys
    // finish before it is rewritten
    if constexpr (!KDOUBLE) __syncthreads();
    W* kb = KDOUBLE ? kbuf + (i & 1u) * 2 * KROWS * KPAD : kbuf;
    if constexpr (kKeyGlds) {
      // u32 rows of >= 64 words: the key rows go global -> LDS directly, one
      // 64-word segment (one ks_pad run) per wave instruction, no registers
      constexpr uint32_t SEG = KW / 64;  // segments per key
      constexpr int WAVES = G::THREADS / 64;
      const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
      const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
      for (int m = 0; m < (int)((2 * SEG + WAVES - 1) / WAVES); ++m) {
        const uint32_t sg = wave + (uint32_t)m * WAVES;
        if (sg < 2 * SEG) {
          const uint32_t kk = sg >= SEG, rs = kk ? sg - SEG : sg;  // key, segment within it
          const W* src = (kk ? key_a : key_b) + kbase + rs * 64u + lane;
          W* dst = kb + kk * (KROWS * KPAD) + (rs / (C / 64)) * KPAD + ks_pad((rs % (C / 64)) * 64u);
          __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                           (__attribute__((address_space(3))) void*)dst, 4, 0, 0);
        }
      }
      // pin the order: the LDS-DMA key loads issue before the S loads, so the
      // (in-order) vmcnt wait for x below also covers them; the exchange
      // barriers after it then publish kb to the other waves
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int e = 0; e < E; ++e) x[0][e] = S[sbase + b0 + ((uint32_t)e << G::BB0)];
      if constexpr (G::P < 2) {
        // no exchange barrier follows: wait for this wave's DMA explicitly
        // before the barrier below publishes kb
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      W kr[KPT];
#pragma unroll
      for (int m = 0; m < KPT; ++m) {
        const uint32_t w = threadIdx.x + (uint32_t)m * G::THREADS;
        if (w < 2u * KW) kr[m] = w < KW ? key_b[kbase + w] : key_a[kbase + w - KW];
      }
#pragma unroll
      for (int e = 0; e < E; ++e) x[0][e] = S[sbase + b0 + ((uint32_t)e << G::BB0)];
#pragma unroll
      for (int m = 0; m < KPT; ++m) {
        const uint32_t w = threadIdx.x + (uint32_t)m * G::THREADS;
        if (w < 2u * KW) {
          const uint32_t wk = w < KW ? w : w - KW;  // word within its key's rows
          kb[(w < KW ? 0u : KROWS * KPAD) + (wk / C) * KPAD + ks_pad(wk & (C - 1))] = kr[m];
        }
      }
    }
    // the transform's LDS exchange ends in barriers that publish kb (and
    // order the reads of this slot two limbs ago before this write); a
    // single-pass row has none, so it gets one here
    if constexpr (G::P < 2) __syncthreads();
    xf_fwd<G, W, 1>(x, rp.xp, lds, tw, mod_of(lc));
    __builtin_amdgcn_sched_barrier(0);
    // the last pass leaves a thread's E values at consecutive positions
    // (G::BBL == 0): the keys come back 16 bytes at a time, one key after
    // the other
    static_assert(G::BBL == 0, "last row pass distribution");
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      const W* kk = kb + o * KROWS * KPAD + (WIDE ? (rp.xp.slot / NP) * KPAD : 0u) + ks_pad(bl);
      constexpr int V = 16 / sizeof(W);
#pragma unroll
      for (int e0 = 0; e0 < E; e0 += V) {
        W kv[V];
        if constexpr (E % V == 0) {
          ks_lds_read16<W>(kv, kk + e0);
        } else {
#pragma unroll
          for (int v = 0; v < V; ++v) kv[v] = e0 + v < E ? kk[e0 + v] : (W)0;
        }
#pragma unroll
        for (int v = 0; v < V; ++v) {
          if (e0 + v >= E) continue;
          if constexpr (kLazy)
            acc[o][e0 + v] = mac_lazy(acc[o][e0 + v], x[0][e0 + v], kv[v], lc.q, q2, nqinv);
          else
            acc[o][e0 + v] = add_mod<W>(acc[o][e0 + v], mont_mul<W>(x[0][e0 + v], kv[v], lc.q, lc.qinv), lc.q);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // the two accumulators' inverse rows one after the other (half the live
  // registers of a two-operand pass).  The thread coordinates pass through
  // an opaque copy, so the inverse passes' twiddle and store addresses are
  // derived here rather than computed before the loop and spilled across it
  XPos xq = rp.xp;
  uint32_t pq = rp.p;
  asm volatile("" : "+v"(xq.tau), "+v"(pq));
  const uint64_t oq = (uint64_t)j * ls + (uint64_t)pq * N + rowoff;
  const uint32_t b0q = G::base(xq.tau, G::BB0);
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    W v[1][E];
#pragma unroll
    for (int e = 0; e < E; ++e) v[0][e] = kLazy ? csub<W>(acc[o][e], lc.q) : acc[o][e];
    xf_inv<G, W, 1>(v, xq, lds, itw, mod_of(lc));
    W* uo = o == 0 ? u0 : u1;
    if (rp.active) {
#pragma unroll
      for (int e = 0; e < E; ++e) uo[oq + b0q + ((uint32_t)e << G::BB0)] = v[0][e];
    }
  }
}

// 4 waves per SIMD (<= 128 VGPRs; unconstrained it takes 134-154 and runs
// at 3): tensor_rows 1.74 -> 1.64 ms per 64 cts (profiles/r02_ab_tensor_waves.txt)
constexpr int kTensorMinWaves = 4;
template <class W, int LOG_C>
__global__ void __launch_bounds__(RowGeo<LOG_C>::THREADS, sizeof(W) == 4 ? kTensorMinWaves : 1)
k_tensor_rows(W* __restrict__ d0hat, W* __restrict__ d1hat, W* __restrict__ d2row,
              const W* __restrict__ c0, const W* __restrict__ c1, const W* __restrict__ c0p,
              const W* __restrict__ c1p, TabPtrs<W> tp, uint32_t log_n, uint32_t B, uint64_t ls,
              uint64_t rows_total) {
  using G = RowGeo<LOG_C>;
  constexpr int E = G::E;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  W* lds = (W*)smem_raw;
  const RowPos rp = row_pos_pfast<G>(log_n, B, rows_total);  // shared twiddles, as in k_row
  const uint64_t N = 1ull << log_n;
  const uint64_t base = (uint64_t)rp.l * ls + (uint64_t)rp.p * N + (uint64_t)rp.r * G::C;
  const LimbConst<W> lc = tp.lc[rp.l];
  const Tw<W>* tw = tp.tw + (uint64_t)rp.l * N;
  const Tw<W>* itw = tp.itw + (uint64_t)rp.l * N;
  const uint32_t b0 = G::base(rp.xp.tau, G::BB0);
  const uint32_t bl = G::base(rp.xp.tau, G::BBL);
  W a[2][E], b[2][E];
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const uint32_t e = b0 + ((uint32_t)i << G::BB0);
    a[0][i] = c0[base + e];
    a[1][i] = c1[base + e];
  }
  xf_fwd<G, W, 2>(a, rp.xp, lds, tw, mod_of(lc));
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const uint32_t e = b0 + ((uint32_t)i << G::BB0);
    b[0][i] = c0p[base + e];
    b[1][i] = c1p[base + e];
  }
  xf_fwd<G, W, 2>(b, rp.xp, lds, tw, mod_of(lc));
  W d2[1][E];
  W nqi = (W)0 - lc.qinv;
  asm volatile("" : "+v"(nqi));  // one multiply per REDC (see mont_mul_nq)
#pragma unroll
  for (int i = 0; i < E; ++i) {
    const W q = lc.q, qi = lc.qinv;
    W d0, d1;
    if constexpr (sizeof(W) == 4) {
      d0 = mont_mul_nq(a[0][i], b[0][i], q, nqi);
      // one REDC of the two-product sum: T < 2q^2 and T + m q < 2^64, the
      // result (T + m q) / 2^32 < 2q (q < 2^31)
      const uint64_t T = mad64(a[1][i], b[0][i], mul64(a[0][i], b[1][i]));
      const uint32_t m = (uint32_t)T * nqi;
      d1 = csub<uint32_t>((uint32_t)(mad64(m, q, T) >> 32), q);
      d2[0][i] = mont_mul_nq(a[1][i], b[1][i], q, nqi);
    } else {
      d0 = mont_mul<W>(a[0][i], b[0][i], q, qi);
      d1 = add_mod<W>(mont_mul<W>(a[0][i], b[1][i], q, qi), mont_mul<W>(a[1][i], b[0][i], q, qi), q);
      d2[0][i] = mont_mul<W>(a[1][i], b[1][i], q, qi);
    }
    if (rp.active) {
      const uint32_t pos = bl + ((uint32_t)i << G::BBL);
      d0hat[base + pos] = d0;
      d1hat[base + pos] = d1;
    }
  }
  xf_inv<G, W, 1>(d2, rp.xp, lds, itw, mod_of(lc));
  if (rp.active) {
#pragma unroll
    for (int i = 0; i < E; ++i) d2row[base + b0 + ((uint32_t)i << G::BB0)] = d2[0][i];
  }
}

// ---------------------------------------------------------------------------
// elementwise / permutation kernels
// ---------------------------------------------------------------------------

template <class W, int OP>
__device__ __forceinline__ W elementwise_op(W x, W y, const LimbConst<W>& lc) {
  if constexpr (OP == 0) return add_mod<W>(x, y, lc.q);
  else if constexpr (OP == 1) return sub_mod<W>(x, y, lc.q);
  else if constexpr (OP == 2) return x == 0 ? (W)0 : (W)(lc.q - x);
  else if constexpr (OP == 3) return shoup_mul<W>(mont_mul<W>(x, y, lc.q, lc.qinv), lc.rmod, lc.rmod_p, lc.q);
  else return mont_mul<W>(x, y, lc.q, lc.qinv);
}

// Coefficient-wise ops (poly.rs:254-306, 370-385).  Grid: x = chunks of one
// limb's B*N words, y = limb, so the limb constants are wave-uniform (no
// per-thread division).  VEC: every thread moves 16 bytes per operand
// (callers check 16-byte alignment and a limb length divisible by it).
template <class W, int OP, bool VEC>
__global__ void __launch_bounds__(256)
k_elementwise(W* __restrict__ out, const W* __restrict__ a, const W* __restrict__ b,
              TabPtrs<W> tp, uint64_t limb_words) {
  constexpr int V = VEC ? 16 / (int)sizeof(W) : 1;
  const uint32_t l = blockIdx.y;
  const uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * V;
  if (i >= limb_words) return;
  const LimbConst<W> lc = tp.lc[l];
  const uint64_t g = (uint64_t)l * limb_words + i;
  if constexpr (VEC) {
    const uint4 xa = *reinterpret_cast<const uint4*>(a + g);
    uint4 xb = xa;
    if constexpr (OP != 2) xb = *reinterpret_cast<const uint4*>(b + g);
    W x[V], y[V], r[V];
    __builtin_memcpy(x, &xa, 16);
    __builtin_memcpy(y, &xb, 16);
#pragma unroll
    for (int v = 0; v < V; ++v) r[v] = elementwise_op<W, OP>(x[v], y[v], lc);
    uint4 o;
    __builtin_memcpy(&o, r, 16);
    *reinterpret_cast<uint4*>(out + g) = o;
  } else {
    out[g] = elementwise_op<W, OP>(a[g], OP == 2 ? (W)0 : b[g], lc);
  }
}

// rescale_into (poly.rs:212-225): out[l] = (c_l - (c_last mod q_l)) * q_last^-1.
template <class W>
__global__ void __launch_bounds__(256)
k_rescale(W* __restrict__ out, const W* __restrict__ in, const W* __restrict__ lastp,
          const W* __restrict__ inv_t, const W* __restrict__ invp_t, TabPtrs<W> tp,
          uint64_t ls_in, uint64_t ls_out, uint64_t poly_words, uint32_t limbs) {
  // one thread per coefficient position over every kept limb: c_last is read
  // once per position, not once per limb (the per-(limb, position) form read
  // the last plane L - 1 times)
  const uint64_t off = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (off >= poly_words) return;
  const W last = lastp[off];
#pragma unroll 4
  for (uint32_t l = 0; l < limbs; ++l) {
    const LimbConst<W> lc = tp.lc[l];
    const W inv = inv_t[l];  // (q_last mod q_l)^-1 mod q_l
    const W invp = invp_t[l];
    const W ci = in[(uint64_t)l * ls_in + off];
    const W cl = shoup_mul<W>(last, (W)1, lc.one_p, lc.q);  // canonical c_last mod q_l (R5)
    out[(uint64_t)l * ls_out + off] = shoup_mul<W>(sub_mod<W>(ci, cl, lc.q), inv, invp, lc.q);
  }
}

// Gather kernels: grid y = limb, x = the limb's B*N words (no per-thread
// division).  XCD-aware deal along x: hardware block b of a row runs on XCD
// b % 8 (gridDim.x is a multiple of 8), so logical block (b % 8) *
// (gridDim.x / 8) + b / 8 gives every XCD a contiguous run of the limb --
// whole polys, whose scattered gathers then stay in that XCD's L2 instead
// of every XCD fetching every poly.
__device__ __forceinline__ uint64_t xcd_gid() {
  const uint32_t per_xcd = gridDim.x >> 3;
  const uint32_t wg = (blockIdx.x & 7u) * per_xcd + (blockIdx.x >> 3);
  return (uint64_t)wg * blockDim.x + threadIdx.x;
}

// automorphism for odd g: out[t] gathers its unique source (poly.rs:520-537).
template <class W>
__global__ void __launch_bounds__(256)
k_automorph_odd(W* __restrict__ out, const W* __restrict__ in, TabPtrs<W> tp, uint32_t log_n,
                uint64_t ginv, uint64_t poly_words, uint64_t total) {
  const uint64_t i = xcd_gid();
  if (i >= poly_words) return;
  const uint64_t N = 1ull << log_n;
  const uint32_t l = blockIdx.y;
  const uint64_t gid = (uint64_t)l * poly_words + i;
  const uint64_t jo = i & (N - 1);
  const uint64_t pbase = gid - jo;
  const uint64_t t = (jo * ginv) & (2 * N - 1);
  const W q = tp.lc[l].q;
  W v;
  if (t < N) {
    v = in[pbase + t];
  } else {
    const W c = in[pbase + t - N];
    v = c == 0 ? (W)0 : (W)(q - c);
  }
  out[gid] = v;
}

// automorphism for even g != 0 mod 2N (not a ring automorphism): the
// reference's scatter loop keeps, per output slot, the LAST (largest i)
// non-zero writer (poly.rs:520-537).  g = 2^e * h, h odd; i*g = r (mod 2N)
// iff 2^e | r and i = (r >> e) * h^-1 (mod M), M = 2N >> e.
template <class W>
__global__ void __launch_bounds__(256)
k_automorph_even(W* __restrict__ out, const W* __restrict__ in, TabPtrs<W> tp, uint32_t log_n,
                 uint32_t e, uint64_t hinv, uint64_t poly_words, uint64_t total) {
  const uint64_t i = xcd_gid();
  if (i >= poly_words) return;
  const uint64_t N = 1ull << log_n;
  const uint32_t l = blockIdx.y;
  const uint64_t gid = (uint64_t)l * poly_words + i;
  const uint64_t jo = i & (N - 1);
  const uint64_t pbase = gid - jo;
  const uint64_t M = (2 * N) >> e;
  const W q = tp.lc[l].q;
  int64_t best = -1;
  int best_neg = 0;
  W best_val = 0;
  for (int h = 0; h < 2; ++h) {
    const uint64_t r = jo + (h ? N : 0);
    if (r & ((1ull << e) - 1)) continue;
    const uint64_t i0 = ((r >> e) * hinv) & (M - 1);
    if (i0 >= N) continue;
    // largest i = i0 + k*M < N with a non-zero coefficient
    uint64_t kmax = (N - 1 - i0) / M;
    for (int64_t k = (int64_t)kmax; k >= 0; --k) {
      const uint64_t i = i0 + (uint64_t)k * M;
      if ((int64_t)i <= best) break;
      const W c = in[pbase + i];
      if (c != 0) {
        best = (int64_t)i;
        best_neg = h;
        best_val = c;
        break;
      }
    }
  }
  W v = 0;
  if (best >= 0) v = best_neg ? (W)(q - best_val) : best_val;
  out[gid] = v;
}

__device__ __forceinline__ uint64_t brv_dev(uint64_t k, uint32_t bits) {
  return bits == 0 ? 0 : (__brevll(k) >> (64 - bits));
}

// host [B][L][N] u64 staging -> device [L][B][N] W (with validation).
template <class W>
__global__ void __launch_bounds__(256)
k_import(W* __restrict__ dst, const uint64_t* __restrict__ stage, TabPtrs<W> tp, uint32_t log_n,
         uint32_t L, uint64_t ls, int to_brv, unsigned long long* err, uint64_t total) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const uint64_t N = 1ull << log_n;
  const uint64_t k = gid & (N - 1);
  const uint64_t pl = gid >> log_n;  // p*L + l
  const uint32_t l = (uint32_t)(pl % L);
  const uint64_t p = pl / L;
  const uint64_t v = stage[gid];
  const uint64_t q = (uint64_t)tp.lc[l].q;
  if (v >= q) atomicMin(err, (unsigned long long)gid);
  const uint64_t pos = to_brv ? brv_dev(k, log_n) : k;
  dst[(uint64_t)l * ls + p * N + pos] = (W)(v >= q ? 0 : v);
}

// from_coeffs (poly.rs:55-61): rem_euclid per channel.
template <class W>
__global__ void __launch_bounds__(256)
k_import_coeffs(W* __restrict__ dst, const int64_t* __restrict__ coeffs, TabPtrs<W> tp,
                uint32_t L, uint64_t ls, uint64_t total) {
  // one thread per coefficient ([B][N] = the [L][B][N] offset within a
  // limb): read it once, write its residue into every limb
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const int64_t c = coeffs[gid];
  for (uint32_t l = 0; l < L; ++l) dst[(uint64_t)l * ls + gid] = rem_euclid<W>(c, tp.lc[l]);
}

template <class W>
__global__ void __launch_bounds__(256)
k_export(uint64_t* __restrict__ stage, const W* __restrict__ src, uint32_t log_n, uint32_t L,
         uint64_t ls, int from_brv, uint64_t total) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const uint64_t N = 1ull << log_n;
  const uint64_t k = gid & (N - 1);
  const uint64_t pl = gid >> log_n;
  const uint32_t l = (uint32_t)(pl % L);
  const uint64_t p = pl / L;
  const uint64_t pos = from_brv ? brv_dev(k, log_n) : k;
  stage[gid] = (uint64_t)src[(uint64_t)l * ls + p * N + pos];
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------

static inline unsigned grid_for(uint64_t total, unsigned block) {
  return (unsigned)((total + block - 1) / block);
}

template <class K>
static hipError_t allow_lds(K kernel, size_t bytes) {
  if (bytes <= 65536) return hipSuccess;
  return hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)bytes);
}

#define RNT_DISPATCH_LOGR(LOGR, MACRO) \
  switch (LOGR) {                      \
    case 0: MACRO(0); break;           \
    case 1: MACRO(1); break;           \
    case 2: MACRO(2); break;           \
    case 3: MACRO(3); break;           \
    case 4: MACRO(4); break;           \
    default: return hipErrorInvalidValue; \
  }

#define RNT_DISPATCH_LOGC(LOGC, MACRO) \
  switch (LOGC) {                      \
    case 0: MACRO(0);                  \
    case 1: MACRO(1);                  \
    case 2: MACRO(2);                  \
    case 3: MACRO(3);                  \
    case 4: MACRO(4);                  \
    case 5: MACRO(5);                  \
    case 6: MACRO(6);                  \
    case 7: MACRO(7);                  \
    case 8: MACRO(8);                  \
    case 9: MACRO(9);                  \
    default: return hipErrorInvalidValue; \
  }

template <class W, int LOG_C>
static size_t row_lds(int nops) {
  using G = RowGeo<LOG_C>;
  (void)nops;  // operands share one region (xchg)
  return (size_t)G::RPW * G::PADC * sizeof(W);
}

#define RNT_DISPATCH_LOGRT(LOGR, MACRO) \
  switch (LOGR) {                       \
    case 5: MACRO(5); break;            \
    case 6: MACRO(6); break;            \
    case 7: MACRO(7); break;            \
    case 8: MACRO(8); break;            \
    default: return hipErrorInvalidValue; \
  }

template <class W, int LOG_R, int LOG_TC>
static size_t col_lds() {
  return (size_t)ColGeo<LOG_R, LOG_TC>::REGION * sizeof(W);
}

// Tiled column grid: x = poly * (C / TC) + column tile, y, z as given
// (limb; source x target limb for the key-switch decomposition).  grid.x = 0
// flags a shape beyond the hardware grid limits.
static int col_log_tc(const Geom& g) { return g.log_c >= 6 ? 6 : 5; }
static dim3 col_grid(const Launch& k, const Geom& g, uint32_t y, uint32_t z) {
  const uint64_t x = (uint64_t)k.B << (g.log_c - col_log_tc(g));
  if (x > 0x7fffffffull || y > 65535u || z > 65535u) return dim3(0, 1, 1);
  return dim3((unsigned)x, y, z);
}

template <class W, bool LZ>
static hipError_t col_fwd_t(const Launch& k, void* out0, const void* in0, void* out1,
                            const void* in1, uint64_t in_ls, uint64_t out_ls) {
  const Geom g = geom_for(k.t->log_n);
  const TabPtrs<W> tp = tab_ptrs<W>(k.t);
  if ((uint64_t)k.L * k.B == 0) return hipSuccess;
  if (g.log_r >= 5) {
    const dim3 grid = col_grid(k, g, (uint32_t)k.L, 1);
    if (grid.x == 0) return hipErrorInvalidConfiguration;
    hipError_t e = hipSuccess;
#define RNT_L2(R, TC)                                                                           \
  e = allow_lds(k_colt_fwd<W, R, TC, LZ>, col_lds<W, R, TC>());                                 \
  if (e != hipSuccess) return e;                                                                \
  hipLaunchKernelGGL((k_colt_fwd<W, R, TC, LZ>), grid, dim3(ColGeo<R, TC>::THREADS),                \
                     (col_lds<W, R, TC>()), k.s, (W*)out0, (const W*)in0, (W*)out1, (const W*)in1, \
                     tp, g.log_n, g.log_c, (uint32_t)k.B, in_ls, out_ls)
#define RNT_L(R)                          \
  if (col_log_tc(g) == 6) {               \
    RNT_L2(R, 6);                         \
  } else {                                \
    RNT_L2(R, 5);                         \
  }
    RNT_DISPATCH_LOGRT(g.log_r, RNT_L)
#undef RNT_L
#undef RNT_L2
    return hipGetLastError();
  }
  const uint64_t total = (uint64_t)k.L * k.B * g.c;
#define RNT_L(R)                                                                              \
  hipLaunchKernelGGL((k_col_fwd<W, R>), dim3(grid_for(total, 256)), dim3(256), 0, k.s,      \
                     (W*)out0, (const W*)in0, (W*)out1, (const W*)in1, tp, g.log_n, g.log_c, \
                     (uint32_t)k.B, in_ls, out_ls, total)
  RNT_DISPATCH_LOGR(g.log_r, RNT_L)
#undef RNT_L
  return hipGetLastError();
}

template <class W, bool LZ>
static hipError_t col_inv_t(const Launch& k, void* out, uint64_t out_ls, const void* in,
                            uint64_t in_ls, int rfold, const void* addend) {
  const Geom g = geom_for(k.t->log_n);
  const TabPtrs<W> tp = tab_ptrs<W>(k.t);
  if ((uint64_t)k.L * k.B == 0) return hipSuccess;
  if (g.log_r >= 5) {
    const dim3 grid = col_grid(k, g, (uint32_t)k.L, 1);
    if (grid.x == 0) return hipErrorInvalidConfiguration;
    hipError_t e = hipSuccess;
#define RNT_L2(R, TC)                                                                        \
  e = allow_lds(k_colt_inv<W, R, TC, LZ>, col_lds<W, R, TC>());                              \
  if (e != hipSuccess) return e;                                                             \
  hipLaunchKernelGGL((k_colt_inv<W, R, TC, LZ>), grid, dim3(ColGeo<R, TC>::THREADS),             \
                     (col_lds<W, R, TC>()), k.s, (W*)out, (const W*)in, (const W*)addend, tp, \
                     g.log_n, g.log_c, (uint32_t)k.B, in_ls, out_ls, rfold)
#define RNT_L(R)                          \
  if (col_log_tc(g) == 6) {               \
    RNT_L2(R, 6);                         \
  } else {                                \
    RNT_L2(R, 5);                         \
  }
    RNT_DISPATCH_LOGRT(g.log_r, RNT_L)
#undef RNT_L
#undef RNT_L2
    return hipGetLastError();
  }
  const uint64_t total = (uint64_t)k.L * k.B * g.c;
#define RNT_L(R)                                                                          \
  hipLaunchKernelGGL((k_col_inv<W, R>), dim3(grid_for(total, 256)), dim3(256), 0, k.s,  \
                     (W*)out, (const W*)in, (const W*)addend, tp, g.log_n, g.log_c,      \
                     (uint32_t)k.B, in_ls, out_ls, total, rfold)
  RNT_DISPATCH_LOGR(g.log_r, RNT_L)
#undef RNT_L
  return hipGetLastError();
}

template <class W, int MODE, int LOG_C, bool LZ = false>
static hipError_t row_launch(const Launch& k, void* x, const void* y, uint64_t ls) {
  using G = RowGeo<LOG_C>;
  const Geom g = geom_for(k.t->log_n);
  const uint64_t rows = (uint64_t)k.L * k.B * g.r;
  if (rows == 0) return hipSuccess;
  const unsigned blocks = (unsigned)((rows + G::RPW - 1) / G::RPW);
  const size_t lds = row_lds<W, LOG_C>(MODE == 2 ? 2 : 1);
  hipError_t e = allow_lds(k_row<W, MODE, LOG_C, LZ>, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_row<W, MODE, LOG_C, LZ>), dim3(blocks), dim3(G::THREADS), lds, k.s, (W*)x,
                     (const W*)y, tab_ptrs<W>(k.t), g.log_n, (uint32_t)k.B, ls, rows);
  return hipGetLastError();
}

template <class W>
static hipError_t row_t(const Launch& k, int mode, void* x, const void* y, uint64_t ls, bool lz) {
  const Geom g = geom_for(k.t->log_n);
#define RNT_L0(C) return row_launch<W, 0, C>(k, x, y, ls)
#define RNT_L1(C) return row_launch<W, 1, C>(k, x, y, ls)
#define RNT_L2(C) return row_launch<W, 2, C>(k, x, y, ls)
#define RNT_L2Z(C) return row_launch<W, 2, C, true>(k, x, y, ls)
  if constexpr (sizeof(W) == 4) {
    if (mode == 2 && lz) {
      RNT_DISPATCH_LOGC(g.log_c, RNT_L2Z)
    }
  }
  if (mode == 0) {
    RNT_DISPATCH_LOGC(g.log_c, RNT_L0)
  } else if (mode == 1) {
    RNT_DISPATCH_LOGC(g.log_c, RNT_L1)
  } else {
    RNT_DISPATCH_LOGC(g.log_c, RNT_L2)
  }
#undef RNT_L0
#undef RNT_L1
#undef RNT_L2
#undef RNT_L2Z
  return hipErrorInvalidValue;
}

template <class W>
static hipError_t elementwise_t(const Launch& k, int op, void* out, const void* a,
                                const void* b) {
  const uint64_t limb_words = (uint64_t)k.B << k.t->log_n;
  if (limb_words == 0 || k.L == 0) return hipSuccess;
  constexpr int V = 16 / (int)sizeof(W);
  const bool vec = limb_words % V == 0 && ((uintptr_t)out | (uintptr_t)a | (uintptr_t)b) % 16 == 0;
  const uint64_t per = vec ? limb_words / V : limb_words;
  const uint64_t bx = (per + 255) / 256;
  if (bx > 0x7fffffffull || k.L > 65535) return hipErrorInvalidConfiguration;
  const dim3 grid((unsigned)bx, (unsigned)k.L);
#define RNT_EW(OP)                                                                              \
  if (vec)                                                                                      \
    hipLaunchKernelGGL((k_elementwise<W, OP, true>), grid, dim3(256), 0, k.s, (W*)out,         \
                       (const W*)a, (const W*)b, tab_ptrs<W>(k.t), limb_words);                \
  else                                                                                          \
    hipLaunchKernelGGL((k_elementwise<W, OP, false>), grid, dim3(256), 0, k.s, (W*)out,        \
                       (const W*)a, (const W*)b, tab_ptrs<W>(k.t), limb_words);
  switch (op) {
    case 0: RNT_EW(0) break;
    case 1: RNT_EW(1) break;
    case 2: RNT_EW(2) break;
    case 3: RNT_EW(3) break;
    default: RNT_EW(4) break;
  }
#undef RNT_EW
  return hipGetLastError();
}

// Clone: 4 x 16 B per lane, all four loads issued before the stores.
__global__ void __launch_bounds__(256)
k_copy16(uint4* __restrict__ dst, const uint4* __restrict__ src, uint64_t n16) {
  const uint64_t base = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
  uint4 v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (base + u * 256 < n16) v[u] = src[base + u * 256];
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (base + u * 256 < n16) dst[base + u * 256] = v[u];
}

hipError_t launch_copy(hipStream_t s, void* dst, const void* src, uint64_t bytes) {
  const uint64_t n16 = bytes / 16;
  if (n16 == 0) return hipSuccess;
  const uint64_t blocks = (n16 + 1023) / 1024;
  if (blocks > 0x7fffffffull) return hipErrorInvalidConfiguration;
  hipLaunchKernelGGL(k_copy16, dim3((unsigned)blocks), dim3(256), 0, s, (uint4*)dst,
                     (const uint4*)src, n16);
  return hipGetLastError();
}

// k.L = limbs of the INPUT; output has k.L - 1.
template <class W>
static hipError_t rescale_t(const Launch& k, void* out, const void* in) {
  const uint64_t pw = (uint64_t)k.B << k.t->log_n;
  const uint64_t total = pw * (k.L - 1);
  if (total == 0) return hipSuccess;
  const TabPtrs<W> tp = tab_ptrs<W>(k.t);
  const uint64_t last = k.L - 1;
  hipLaunchKernelGGL((k_rescale<W>), dim3(grid_for(pw, 256)), dim3(256), 0, k.s, (W*)out,
                     (const W*)in, (const W*)in + last * pw, tp.resc + last * tp.Lroot,
                     tp.rescp + last * tp.Lroot, tp, pw, pw, pw, (uint32_t)last);
  return hipGetLastError();
}

// Rescale by a limb held outside the buffer (limb-sharded pipelines: the
// broadcast last limb of the global basis): out limbs 0..k.L-1 from in's.
template <class W>
static hipError_t rescale_ext_t(const Launch& k, void* out, const void* in, const void* lastp,
                                const void* inv, const void* invp) {
  const uint64_t pw = (uint64_t)k.B << k.t->log_n;
  const uint64_t total = pw * k.L;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL((k_rescale<W>), dim3(grid_for(pw, 256)), dim3(256), 0, k.s, (W*)out,
                     (const W*)in, (const W*)lastp, (const W*)inv, (const W*)invp, tab_ptrs<W>(k.t),
                     pw, pw, pw, (uint32_t)k.L);
  return hipGetLastError();
}

static uint64_t inv_mod_pow2(uint64_t h, uint64_t M) {
  // h odd, M power of two: Newton iteration for h^-1 mod 2^64, then mask.
  uint64_t x = h;  // correct to 3 bits
  for (int i = 0; i < 6; ++i) x *= 2 - h * x;
  return x & (M - 1);
}

template <class W>
static hipError_t automorphism_t(const Launch& k, void* out, const void* in, uint64_t g) {
  const uint64_t N = 1ull << k.t->log_n;
  const uint64_t two_n = 2 * N;
  const uint64_t e = g % two_n;
  const uint64_t pw = (uint64_t)k.B * N;
  const uint64_t total = pw * k.L;
  if (total == 0) return hipSuccess;
  if (k.L > 65535) return hipErrorInvalidConfiguration;
  const dim3 grid8((grid_for(pw, 256) + 7u) & ~7u, (unsigned)k.L);  // xcd_gid(): x a multiple of 8
  if (e & 1) {
    const uint64_t ginv = inv_mod_pow2(e, two_n);
    hipLaunchKernelGGL((k_automorph_odd<W>), grid8, dim3(256), 0, k.s,
                       (W*)out, (const W*)in, tab_ptrs<W>(k.t), k.t->log_n, ginv, pw, total);
  } else {
    uint32_t ex = 0;
    uint64_t h = e;
    while ((h & 1) == 0) {
      h >>= 1;
      ++ex;
    }
    const uint64_t M = two_n >> ex;
    const uint64_t hinv = inv_mod_pow2(h, M);
    hipLaunchKernelGGL((k_automorph_even<W>), grid8, dim3(256), 0, k.s,
                       (W*)out, (const W*)in, tab_ptrs<W>(k.t), k.t->log_n, ex, hinv, pw, total);
  }
  return hipGetLastError();
}

template <class W>
static hipError_t import_t(const Launch& k, void* dst, const uint64_t* stage, int to_brv,
                           unsigned long long* err) {
  const uint64_t total = ((uint64_t)k.B * k.L) << k.t->log_n;
  if (total == 0) return hipSuccess;
  const uint64_t ls = (uint64_t)k.B << k.t->log_n;
  hipLaunchKernelGGL((k_import<W>), dim3(grid_for(total, 256)), dim3(256), 0, k.s, (W*)dst,
                     stage, tab_ptrs<W>(k.t), k.t->log_n, (uint32_t)k.L, ls, to_brv, err, total);
  return hipGetLastError();
}

template <class W>
static hipError_t import_coeffs_t(const Launch& k, void* dst, const int64_t* stage) {
  const uint64_t total = (uint64_t)k.B << k.t->log_n;
  if (total == 0 || k.L == 0) return hipSuccess;
  hipLaunchKernelGGL((k_import_coeffs<W>), dim3(grid_for(total, 256)), dim3(256), 0, k.s,
                     (W*)dst, stage, tab_ptrs<W>(k.t), (uint32_t)k.L, total, total);
  return hipGetLastError();
}

template <class W>
static hipError_t export_t(const Launch& k, uint64_t* stage, const void* src, int from_brv,
                           uint64_t ls) {
  const uint64_t total = ((uint64_t)k.B * k.L) << k.t->log_n;
  if (total == 0) return hipSuccess;
  if (ls == 0) ls = (uint64_t)k.B << k.t->log_n;
  hipLaunchKernelGGL((k_export<W>), dim3(grid_for(total, 256)), dim3(256), 0, k.s, stage,
                     (const W*)src, k.t->log_n, (uint32_t)k.L, ls, from_brv, total);
  return hipGetLastError();
}

template <class W>
static hipError_t ks_decompose_t(const Launch& k, void* S, const void* d, uint64_t d_ls) {
  const Geom g = geom_for(k.t->log_n);
  if ((uint64_t)k.L * k.B == 0) return hipSuccess;
  const TabPtrs<W> tp = tab_ptrs<W>(k.t);
  const uint32_t Ls = (uint32_t)k.src_limbs();  // source limbs i; target limbs j = k.L
  if (g.log_r >= 5) {
    const dim3 g0 = col_grid(k, g, Ls, (uint32_t)k.L);
    if (g0.x == 0 || g0.x > 65535u) return hipErrorInvalidConfiguration;
    // target limbs per workgroup (Tables::dec_jg; 0 = auto): the source tile
    // is read once per group instead of once per target limb.  Auto takes
    // groups of 16 (vs one limb per group: ks_decompose -8%, profiles/r01_ab_dec_jg.txt) and
    // halves them while the grid would fall under 4 workgroups per CU.
    uint32_t jg = k.t->dec_jg;
    if (jg == 0) {
      jg = 16;
      while (jg > 1 && ((uint32_t)k.L + jg - 1) / jg * (uint64_t)g0.x * Ls < 1024u) jg >>= 1;
    }
    const dim3 grid(((uint32_t)k.L + jg - 1) / jg, g0.x, Ls);
    // u32 words hold residues of moduli < 2^31 (wider bases take u64), so
    // alpha_i < 2^31 <= 2 q_j when every target modulus is >= 2^30: one
    // conditional subtraction reduces it (the root basis' smallest modulus
    // bounds every drop_last view's)
    uint64_t qmin = ~0ull;
    for (uint64_t q : k.t->moduli) qmin = q < qmin ? q : qmin;
    const uint32_t lift_csub = sizeof(W) == 4 && qmin >= (1ull << 30) ? 1u : 0u;
    hipError_t e = hipSuccess;
#define RNT_L2(R, TC)                                                                         \
  e = allow_lds(k_colt_decompose<W, R, TC>, col_lds<W, R, TC>());                             \
  if (e != hipSuccess) return e;                                                              \
  hipLaunchKernelGGL((k_colt_decompose<W, R, TC>), grid, dim3(ColGeo<R, TC>::THREADS),        \
                     (col_lds<W, R, TC>()), k.s, (W*)S, (const W*)d, tp, g.log_n, g.log_c,      \
                     Ls, (uint32_t)k.B, d_ls, (uint32_t)k.L, jg, lift_csub)
#define RNT_L(R)                          \
  if (col_log_tc(g) == 6) {               \
    RNT_L2(R, 6);                         \
  } else {                                \
    RNT_L2(R, 5);                         \
  }
    RNT_DISPATCH_LOGRT(g.log_r, RNT_L)
#undef RNT_L
#undef RNT_L2
    return hipGetLastError();
  }
  const uint64_t total = (uint64_t)k.L * Ls * k.B * g.c;
#define RNT_L(R)                                                                               \
  hipLaunchKernelGGL((k_ks_decompose<W, R>), dim3(grid_for(total, 256)), dim3(256), 0, k.s,  \
                     (W*)S, (const W*)d, tp, g.log_n, g.log_c, Ls, (uint32_t)k.B, d_ls, total)
  RNT_DISPATCH_LOGR(g.log_r, RNT_L)
#undef RNT_L
  return hipGetLastError();
}

template <class W, int LOG_C, int NP>
static hipError_t ks_rows_launch(const Launch& k, void* u0, void* u1, uint64_t ls, const void* S,
                                 const void* key_a, const void* key_b, uint64_t key_ls,
                                 const void* init0, const void* init1, uint64_t init_ls) {
  using G = RowGeo<LOG_C>;
  constexpr int KROWS = G::RPW / NP;
  constexpr size_t KPADB = (size_t)ks_kpad_words<W>(G::C) * sizeof(W);
  const Geom g = geom_for(k.t->log_n);
  if (k.L == 0 || k.B == 0) return hipSuccess;
  if (g.r % KROWS) return hipErrorInvalidValue;
  // one workgroup per (target limb, group of KROWS rows, group of NP polys)
  const uint64_t pgroups = (k.B + NP - 1) / NP;
  const uint64_t blocks = (uint64_t)k.L * (g.r / KROWS) * pgroups;
  if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
  const unsigned launched = (unsigned)((blocks + 7) / 8 * 8);  // whole XCD rounds
  // exchange region + one or two buffers of {key_b, key_a} x KROWS rows
  // (the kernel's KDOUBLE rule)
  const size_t region = row_lds<W, LOG_C>(1);
  const bool kdouble = region + 4 * KROWS * KPADB <= 40u * 1024u || KROWS == 1;
  const size_t lds = region + (kdouble ? 4 : 2) * KROWS * KPADB;
  hipError_t e = allow_lds(k_ks_rows<W, LOG_C, NP>, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_ks_rows<W, LOG_C, NP>), dim3(launched), dim3(G::THREADS), lds, k.s,
                     (W*)u0, (W*)u1, (const W*)S, (const W*)key_a, (const W*)key_b, key_ls,
                     (const W*)init0, (const W*)init1, init_ls, tab_ptrs<W>(k.t), g.log_n,
                     (uint32_t)k.src_limbs(), (uint32_t)k.B, ls, (uint32_t)pgroups,
                     (uint32_t)blocks);
  return hipGetLastError();
}

// Polys per workgroup: the poly-per-slot grid (NP = RPW) shares each key
// row among RPW polys but leaves slots idle when RPW does not divide B.
// u32 rows of >= 64 words pick, among NP = RPW and smaller powers of two
// (2..8 for the configs' 2^8- and 2^9-word rows, 1 for every row length),
// the one that fills the most row slots, the larger on a tie (more key
// sharing).  B < RPW/2 used to run at B/RPW of the grid.
template <class W, int LOG_C>
static hipError_t ks_rows_pick(const Launch& k, void* u0, void* u1, uint64_t ls, const void* S,
                               const void* key_a, const void* key_b, uint64_t key_ls,
                               const void* init0, const void* init1, uint64_t init_ls) {
  using G = RowGeo<LOG_C>;
  constexpr int RPW = G::RPW;
  const Geom g = geom_for(k.t->log_n);
  // NP = polys per workgroup (each key row is loaded once for NP polys).
  // Take the largest NP whose grid fills at least 90% of its row slots:
  // slot fill alone would pick NP = 1 (always 100% full, no key sharing,
  // the most expensive grid) for every odd batch, e.g. a 63-poly last chunk
  // of a 1023-ciphertext batch.  Below that fill (small batches, B < RPW
  // mostly) the best-filled grid wins, the larger NP on a tie.
  int np = RPW;
  if (sizeof(W) == 4 && G::C >= 64 && RPW > 1) {
    double best = -1.0;
    int best_np = RPW;
    bool chosen = false;
    for (int c = RPW; c >= 1; c >>= 1) {
      const bool have = c == RPW || c == 1 || ((LOG_C == 8 || LOG_C == 9) && c <= 8);
      if (!have || g.r % (RPW / c)) continue;
      const double fill = (double)k.B / (double)(((k.B + c - 1) / c) * c);
      if (fill >= 0.9) {
        np = c;
        chosen = true;
        break;
      }
      if (fill > best + 1e-9) { best = fill; best_np = c; }
    }
    if (!chosen) np = best_np;
  }
#define RNT_NP(V) \
  if (np == (V) && RPW % (V) == 0) \
    return ks_rows_launch<W, LOG_C, (RPW % (V) == 0 ? (V) : RPW)>(k, u0, u1, ls, S, key_a, key_b, key_ls, init0, init1, init_ls);
  if constexpr (sizeof(W) == 4 && G::C >= 64 && RPW > 1) {
    RNT_NP(1)
    if constexpr (LOG_C == 8 || LOG_C == 9) {
      RNT_NP(2)
      RNT_NP(4)
      RNT_NP(8)
    }
  }
#undef RNT_NP
  return ks_rows_launch<W, LOG_C, RPW>(k, u0, u1, ls, S, key_a, key_b, key_ls, init0, init1, init_ls);
}

template <class W>
static hipError_t ks_rows_t(const Launch& k, void* u0, void* u1, uint64_t ls, const void* S,
                            const void* key_a, const void* key_b, uint64_t key_ls,
                            const void* init0, const void* init1, uint64_t init_ls) {
  const Geom g = geom_for(k.t->log_n);
#define RNT_L(C) \
  return ks_rows_pick<W, C>(k, u0, u1, ls, S, key_a, key_b, key_ls, init0, init1, init_ls)
  RNT_DISPATCH_LOGC(g.log_c, RNT_L)
#undef RNT_L
  return hipErrorInvalidValue;
}

template <class W, int LOG_C>
static hipError_t tensor_rows_launch(const Launch& k, void* d0hat, void* d1hat, void* d2row,
                                     const void* c0, const void* c1, const void* c0p,
                                     const void* c1p, uint64_t ls) {
  using G = RowGeo<LOG_C>;
  const Geom g = geom_for(k.t->log_n);
  const uint64_t rows = (uint64_t)k.L * k.B * g.r;
  if (rows == 0) return hipSuccess;
  const unsigned blocks = (unsigned)((rows + G::RPW - 1) / G::RPW);
  const size_t lds = row_lds<W, LOG_C>(2);
  hipError_t e = allow_lds(k_tensor_rows<W, LOG_C>, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_tensor_rows<W, LOG_C>), dim3(blocks), dim3(G::THREADS), lds, k.s,
                     (W*)d0hat, (W*)d1hat, (W*)d2row, (const W*)c0, (const W*)c1,
                     (const W*)c0p, (const W*)c1p, tab_ptrs<W>(k.t), g.log_n, (uint32_t)k.B, ls,
                     rows);
  return hipGetLastError();
}

template <class W>
static hipError_t tensor_rows_t(const Launch& k, void* d0hat, void* d1hat, void* d2row,
                                const void* c0, const void* c1, const void* c0p,
                                const void* c1p, uint64_t ls) {
  const Geom g = geom_for(k.t->log_n);
#define RNT_L(C) return tensor_rows_launch<W, C>(k, d0hat, d1hat, d2row, c0, c1, c0p, c1p, ls)
  RNT_DISPATCH_LOGC(g.log_c, RNT_L)
#undef RNT_L
  return hipErrorInvalidValue;
}

// W dispatch -----------------------------------------------------------------
#define RNT_WIDE(CALL32, CALL64) return k.t->wide ? (CALL64) : (CALL32)

bool lazy30_ok(const Tables* t) {
  return !t->wide && t->lazy30 && geom_for(t->log_n).log_r >= 5;
}
hipError_t launch_col_fwd(const Launch& k, void* out0, const void* in0, void* out1,
                          const void* in1, uint64_t in_ls, uint64_t out_ls, bool lazy) {
  if (lazy && lazy30_ok(k.t))
    return col_fwd_t<uint32_t, true>(k, out0, in0, out1, in1, in_ls, out_ls);
  RNT_WIDE((col_fwd_t<uint32_t, false>(k, out0, in0, out1, in1, in_ls, out_ls)),
           (col_fwd_t<uint64_t, false>(k, out0, in0, out1, in1, in_ls, out_ls)));
}
// The whole-plane product (k_plane_fwd + k_plane_mul) serves rnt_mul for
// u32 canonical bases at N = 2^16 when Tables::plane is set (RNT_PLANE).
// The whole-plane kernels take every u32 basis at N = 2^16 (their
// canonical arithmetic holds for any q < 2^31, so 30-bit bases too: 131k
// against the lazy four-step kernels' 114k products/s).
bool plane_ok(const Tables* t) {
  return t->plane != 0 && !t->wide && t->log_n == 16;
}

hipError_t launch_plane(const Launch& k, int which, void* out, const void* in, const void* ahat,
                        uint64_t ls) {
  if (k.B == 0 || k.L == 0) return hipSuccess;
  if (k.B > 0x7fffffffull || k.L > 65535) return hipErrorInvalidConfiguration;
  const size_t lds = (size_t)plane::LDS_WORDS * 4;
  const dim3 grid((unsigned)k.B, (unsigned)k.L);
  const uint32_t st = k.t->plane_stagger;
  if (which == 0) {
    hipError_t e = allow_lds(k_plane_fwd, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_plane_fwd, grid, dim3(plane::T), lds, k.s, (uint32_t*)out, (const uint32_t*)in,
                       tab_ptrs<uint32_t>(k.t), ls, st);
  } else {
    hipError_t e = allow_lds(k_plane_mul, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_plane_mul, grid, dim3(plane::T), lds, k.s, (uint32_t*)out, (const uint32_t*)in,
                       (const uint32_t*)ahat, tab_ptrs<uint32_t>(k.t), ls, st);
  }
  return hipGetLastError();
}

hipError_t launch_plane_fused(const Launch& k, void* out, const void* a, const void* b, void* scratch, uint64_t ls) {
  if (k.B == 0 || k.L == 0) return hipSuccess;
  if (k.B > 0x7fffffffull || k.L > 65535) return hipErrorInvalidConfiguration;
  const size_t lds = (size_t)plane::LDS_WORDS * 4;
  hipError_t e = allow_lds(k_plane_fused, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_plane_fused, dim3((unsigned)k.B, (unsigned)k.L), dim3(plane::T), lds, k.s, (uint32_t*)out,
                     (const uint32_t*)a, (const uint32_t*)b, (uint32_t*)scratch, tab_ptrs<uint32_t>(k.t), ls);
  return hipGetLastError();
}

hipError_t launch_row(const Launch& k, int mode, void* x, const void* y, uint64_t ls, bool lazy) {
  const bool lz = lazy && lazy30_ok(k.t);
  RNT_WIDE(row_t<uint32_t>(k, mode, x, y, ls, lz), row_t<uint64_t>(k, mode, x, y, ls, false));
}
hipError_t launch_col_inv(const Launch& k, void* out, uint64_t out_ls, const void* in,
                          uint64_t in_ls, int rfold, const void* addend, bool lazy) {
  if (lazy && lazy30_ok(k.t))
    return col_inv_t<uint32_t, true>(k, out, out_ls, in, in_ls, rfold, addend);
  RNT_WIDE((col_inv_t<uint32_t, false>(k, out, out_ls, in, in_ls, rfold, addend)),
           (col_inv_t<uint64_t, false>(k, out, out_ls, in, in_ls, rfold, addend)));
}
hipError_t launch_elementwise(const Launch& k, int op, void* out, const void* a, const void* b) {
  RNT_WIDE(elementwise_t<uint32_t>(k, op, out, a, b), elementwise_t<uint64_t>(k, op, out, a, b));
}
// ---------------------------------------------------------------------------
// decode-side CRT (basis.rs:158-180, poly.rs:404-427)
// ---------------------------------------------------------------------------

// Per coefficient, with residues r_l (coefficient domain):
//   s_l = r_l * (Q/q_l)^-1 mod q_l,   x = sum_l s_l * (Q/q_l) - k * Q,
//   k = floor(sum_l s_l / q_l)  (double precision, then a +-Q correction),
// centred into (-Q/2, Q/2] and written as `out_words` little-endian 64-bit
// two's-complement words.  Multi-word values are MW 32-bit words; the
// constants (Q/q_l words, Q, floor(Q/2)) are wave-uniform scalar loads.
// (CrtConsts: rnt_internal.hpp)

template <int MW>
__device__ __forceinline__ bool mw_ge(const uint32_t (&a)[MW + 1], const RNT_CONST_AS uint32_t* b) {
  if (a[MW] != 0) return true;
#pragma unroll
  for (int w = MW - 1; w >= 0; --w) {
    if (a[w] != b[w]) return a[w] > b[w];
  }
  return true;
}
template <int MW>
__device__ __forceinline__ void mw_sub(uint32_t (&a)[MW + 1], const RNT_CONST_AS uint32_t* b) {
  uint64_t borrow = 0;
#pragma unroll
  for (int w = 0; w < MW; ++w) {
    const uint64_t d = (uint64_t)a[w] - b[w] - borrow;
    a[w] = (uint32_t)d;
    borrow = (d >> 32) & 1;
  }
  a[MW] -= (uint32_t)borrow;
}
template <int MW>
__device__ __forceinline__ void mw_add(uint32_t (&a)[MW + 1], const RNT_CONST_AS uint32_t* b) {
  uint64_t carry = 0;
#pragma unroll
  for (int w = 0; w < MW; ++w) {
    const uint64_t t = (uint64_t)a[w] + b[w] + carry;
    a[w] = (uint32_t)t;
    carry = t >> 32;
  }
  a[MW] += (uint32_t)carry;
}

template <class W, int MW>
__global__ void __launch_bounds__(256)
k_crt(uint64_t* __restrict__ out, const W* __restrict__ in, CrtConsts cc, TabPtrs<W> tp,
      uint32_t L, uint64_t ls, uint32_t out_words, uint64_t total) {
  const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const RNT_CONST_AS uint32_t* qi = (const RNT_CONST_AS uint32_t*)cc.qi_words;
  const RNT_CONST_AS uint32_t* qw = (const RNT_CONST_AS uint32_t*)cc.q_words;
  const RNT_CONST_AS uint32_t* qh = (const RNT_CONST_AS uint32_t*)cc.qh_words;
  uint32_t acc[MW + 1];
#pragma unroll
  for (int w = 0; w <= MW; ++w) acc[w] = 0;
  double f = 0.0;
  for (uint32_t l = 0; l < L; ++l) {
    const LimbConst<W> lc = tp.lc[l];
    const W s = shoup_mul<W>(in[(uint64_t)l * ls + gid], (W)cc.inv[l], (W)cc.inv_p[l], lc.q);
    f += (double)s * cc.rq[l];
    // acc += s * (Q/q_l), s split into 32-bit halves
    const RNT_CONST_AS uint32_t* row = qi + (uint64_t)l * MW;
#pragma unroll
    for (int half = 0; half < (sizeof(W) == 8 ? 2 : 1); ++half) {
      const uint32_t sh = (uint32_t)((uint64_t)s >> (32 * half));
      uint64_t carry = 0;
#pragma unroll
      for (int w = 0; w + half < MW; ++w) {
        const uint64_t t = (uint64_t)sh * row[w] + acc[w + half] + carry;
        acc[w + half] = (uint32_t)t;
        carry = t >> 32;
      }
#pragma unroll
      for (int w = MW - half; w <= MW; ++w) {  // propagate into the top word(s)
        const uint64_t t = (uint64_t)acc[w] + carry;
        acc[w] = (uint32_t)t;
        carry = t >> 32;
      }
    }
  }
  // subtract k*Q, k = floor(f) < L; then correct by at most one Q either way
  const uint32_t k = (uint32_t)f;
  {
    uint64_t borrow = 0;
    uint64_t carry = 0;
#pragma unroll
    for (int w = 0; w < MW; ++w) {
      const uint64_t kq = (uint64_t)k * qw[w] + carry;
      carry = kq >> 32;
      const uint64_t d = (uint64_t)acc[w] - (uint32_t)kq - borrow;
      acc[w] = (uint32_t)d;
      borrow = (d >> 32) & 1;
    }
    acc[MW] = acc[MW] - (uint32_t)carry - (uint32_t)borrow;
  }
  if ((int32_t)acc[MW] < 0) mw_add<MW>(acc, qw);
  if (mw_ge<MW>(acc, qw)) mw_sub<MW>(acc, qw);
  // centre: x > floor(Q/2)  <=>  x > Q/2 (Q odd)  ->  x - Q
  uint32_t t2[MW + 1];
#pragma unroll
  for (int w = 0; w <= MW; ++w) t2[w] = acc[w];
  bool gt = false;
  {
    bool decided = false;
#pragma unroll
    for (int w = MW - 1; w >= 0; --w) {
      if (!decided && t2[w] != qh[w]) {
        gt = t2[w] > qh[w];
        decided = true;
      }
    }
  }
  if (gt) mw_sub<MW>(acc, qw);  // negative: two's complement with sign in acc[MW]
  const uint32_t sign = (int32_t)acc[MW] < 0 ? 0xffffffffu : 0u;
  uint64_t* o = out + gid * out_words;
  for (uint32_t w = 0; w < out_words; ++w) {
    const uint32_t lo = 2 * w < (uint32_t)MW ? acc[2 * w] : sign;
    const uint32_t hi = 2 * w + 1 < (uint32_t)MW ? acc[2 * w + 1] : sign;
    o[w] = (uint64_t)lo | ((uint64_t)hi << 32);
  }
}

template <class W>
static hipError_t crt_t(const Launch& k, uint64_t* out, const void* in, const CrtConsts& cc,
                        uint32_t mw, uint32_t out_words) {
  const uint64_t total = (uint64_t)k.B << k.t->log_n;
  if (total == 0) return hipSuccess;
  const uint64_t ls = total;
#define RNT_L(MW)                                                                                \
  hipLaunchKernelGGL((k_crt<W, MW>), dim3(grid_for(total, 256)), dim3(256), 0, k.s, out,       \
                     (const W*)in, cc, tab_ptrs<W>(k.t), (uint32_t)k.L, ls, out_words, total); \
  return hipGetLastError()
  if (mw <= 4) { RNT_L(4); }
  if (mw <= 8) { RNT_L(8); }
  if (mw <= 16) { RNT_L(16); }
  if (mw <= 32) { RNT_L(32); }
  if (mw <= 64) { RNT_L(64); }
  if (mw <= 128) { RNT_L(128); }
#undef RNT_L
  return hipErrorInvalidValue;
}

hipError_t launch_rescale(const Launch& k, void* out, const void* in) {
  RNT_WIDE(rescale_t<uint32_t>(k, out, in), rescale_t<uint64_t>(k, out, in));
}
hipError_t launch_crt(const Launch& k, uint64_t* out, const void* in, const void* consts,
                      uint32_t mw, uint32_t out_words) {
  const CrtConsts cc = *(const CrtConsts*)consts;
  RNT_WIDE(crt_t<uint32_t>(k, out, in, cc, mw, out_words),
           crt_t<uint64_t>(k, out, in, cc, mw, out_words));
}
hipError_t launch_rescale_ext(const Launch& k, void* out, const void* in, const void* last,
                              const void* inv, const void* invp) {
  RNT_WIDE(rescale_ext_t<uint32_t>(k, out, in, last, inv, invp),
           rescale_ext_t<uint64_t>(k, out, in, last, inv, invp));
}
hipError_t launch_automorphism(const Launch& k, void* out, const void* in, uint64_t g) {
  RNT_WIDE(automorphism_t<uint32_t>(k, out, in, g), automorphism_t<uint64_t>(k, out, in, g));
}
hipError_t launch_import(const Launch& k, void* dst, const uint64_t* stage, int to_brv,
                         unsigned long long* err) {
  RNT_WIDE(import_t<uint32_t>(k, dst, stage, to_brv, err),
           import_t<uint64_t>(k, dst, stage, to_brv, err));
}
hipError_t launch_import_coeffs(const Launch& k, void* dst, const int64_t* stage) {
  RNT_WIDE(import_coeffs_t<uint32_t>(k, dst, stage), import_coeffs_t<uint64_t>(k, dst, stage));
}
hipError_t launch_export(const Launch& k, uint64_t* stage, const void* src, int from_brv,
                         uint64_t ls) {
  RNT_WIDE(export_t<uint32_t>(k, stage, src, from_brv, ls),
           export_t<uint64_t>(k, stage, src, from_brv, ls));
}
hipError_t launch_ks_decompose(const Launch& k, void* S, const void* d, uint64_t d_ls) {
  RNT_WIDE(ks_decompose_t<uint32_t>(k, S, d, d_ls), ks_decompose_t<uint64_t>(k, S, d, d_ls));
}
hipError_t launch_ks_rows(const Launch& k, void* u0, void* u1, uint64_t u_ls, const void* S,
                          const void* key_a, const void* key_b, uint64_t key_ls,
                          const void* init0, const void* init1, uint64_t init_ls) {
  RNT_WIDE(ks_rows_t<uint32_t>(k, u0, u1, u_ls, S, key_a, key_b, key_ls, init0, init1, init_ls),
           ks_rows_t<uint64_t>(k, u0, u1, u_ls, S, key_a, key_b, key_ls, init0, init1, init_ls));
}
hipError_t launch_tensor_rows(const Launch& k, void* d0hat, void* d1hat, void* d2row,
                              const void* c0, const void* c1, const void* c0p, const void* c1p,
                              uint64_t ls) {
  RNT_WIDE(tensor_rows_t<uint32_t>(k, d0hat, d1hat, d2row, c0, c1, c0p, c1p, ls),
           tensor_rows_t<uint64_t>(k, d0hat, d1hat, d2row, c0, c1, c0p, c1p, ls));
}

}  // namespace rnt
