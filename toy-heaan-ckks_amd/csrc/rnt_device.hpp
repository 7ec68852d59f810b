// rnt_device.hpp -- device helpers shared by the kernel translation units
// (rnt_kernels.hip: four-step transforms, key-switch, elementwise; rnt_plane.hip:
// the whole-plane poly-mul): table pointers, buffer-resource views, twiddle
// sources, the truncated product's degree-3 block product, LDS opt-in.
#pragma once
#include <hip/hip_runtime.h>

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

// The product path's modulus bundle: LZ = Harvey-lazy arithmetic
// (rnt_modarith.hpp Mod30: u32 words, q < 2^30; Mod62: u64 words, q < 2^62).
template <class W, bool LZ>
__device__ __forceinline__ auto mod_for(const LimbConst<W>& lc) {
  if constexpr (LZ && sizeof(W) == 4) {
    const uint32_t q = (uint32_t)lc.q;
    return Mod30{q, 0u - q, 2u * q};
  } else if constexpr (LZ) {
    const uint64_t q = (uint64_t)lc.q;
    return Mod62{q, 2ull * q};
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
template <class W>
__device__ __forceinline__ W gload(const W* p, uint64_t i) {
  return p[i];
}
template <class W>
__device__ __forceinline__ void gstore(W* p, uint64_t i, W x) {
  p[i] = x;
}

template <class W>
struct BufView {
  __amdgpu_buffer_rsrc_t r;
  __device__ BufView(const W* base, uint32_t elems)
      : r(__builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)(elems * sizeof(W)), 0x00020000)) {}
  __device__ __forceinline__ W ld(uint32_t v, uint32_t s) const {
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

// k_colt_inv's optional limb offset and fused rescale (ColRescArgs).
template <class W>
struct ColResc {
  const W* last = nullptr;
  const W* inv = nullptr;
  const W* invp = nullptr;
  uint32_t limb0 = 0;
};

// Last-stage constants of the inverse network (n^-1 folded, optionally with
// the Montgomery factor): x <- (u+v) c1, y <- (u-v) c2.
template <class W>
struct Fold {
  W c1, c1p, c2, c2p;
};

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

template <class K>
static hipError_t allow_lds(K kernel, size_t bytes) {
  if (bytes <= 65536) return hipSuccess;
  return hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)bytes);
}
}  // namespace rnt
