// rnt_mfma.hip -- the whole-plane poly-mul and transforms at N = 2^16 (u32
// bases) on the matrix cores: radix-16 passes as i8 MFMA products.
//
// Reference unit: one coefficient-domain `a *= &b` (poly.rs:307-329:
// to_ntt_domain of both operands, the pointwise mul_mod, to_coeff_domain)
// and the standalone to_ntt_domain / to_coeff_domain (poly.rs:136-166).
// The network is the four-step kernels' merged negacyclic CT / GS heap, so
// the NTT-domain words are the same (device order = the in-place CT order)
// and the product is the reference's word for word (R1: exact arithmetic).
//
// ---- the transform as four 16 x 16 matrix passes ----------
// Pass p (p = 0..3) runs the four CT stages at index bits 15-4p .. 12-4p.
// On each group of 16 words that differ only in those bits (k = the 4-bit
// group index) it is one 16 x 16 matrix M_U, U = the index bits above the
// pass: M_U[j][k] = z_{U,j}^k (a Vandermonde matrix on the 16 roots of the
// group's modulus), and M_U = F . diag(beta_U^k) with ONE matrix F for every
// pass and U (beta_U = psi_rev[(N >> (b_lo + 1)) + 8U], the heap node of the
// pass's last stage at the group's first word; tools/mfma_model.py checks
// both facts and the four passes against the oracle).  So:
//   pass 0: M_0 itself (one matrix);
//   pass 1: M_U with U = the wave's 4 bits (one matrix per wave);
//   passes 2, 3: F, with the twist beta_U^k applied to the data first (one
//            signed Montgomery product per word, twiddles from a table).
// The inverse runs the inverse matrices in the mirror order (the twist
// after F^-1); n^-1 and, after a product, the Montgomery factor 2^32 of the
// pointwise product are folded into its last matrix.
//
// ---- exact integer matrix products on the i8 matrix cores -----------------
// Words travel between passes as signed representatives r, |r| < q/2 + 2^14,
// packed as four balanced byte digits: (r + 0x80808080) ^ 0x80808080 (byte b
// of that is digit b, in [-128, 128)).  A pass computes, for each output j,
//   T_j = sum_{k,b} E[j][k][b] * x_k^(b),   E[j][k][b] = centred(W[j][k] 2^(8b) 2^32 mod q)
// with E split into four digit planes too: v_mfma_i32_16x16x64_i8 forms the
// digit sums C_a (K = 64 = 16 words x 4 data digits, |C_a| <= 2^20), and
//   T = (C_0 + 2^8 C_1) + 2^16 (C_2 + 2^8 C_3),  |T| < 2^46,
//   r' = (T + m q) / 2^32,  m = T (-q^-1) mod 2^32  (signed Montgomery),
// gives r' = sum_k W[j][k] x_k mod q in (-q/2 - 2^14, q/2 + 2^14), which packs
// again (the +0x80808080 rides in the reduction's 64-bit addend).  About 7
// VALU instructions per word per pass (10 with a twist) instead of 22 for
// four radix-2 CT stages; the MFMAs (4 per 256 words) run beside them.
//
// ---- layouts -----------------------------------------------------------------
// One 1024-thread workgroup per (poly, limb) plane, 64 words a thread as 16
// chunks c of 4 registers i.  Thread t = (wave w, lane lam = 16 g + n).  An
// MFMA tile is one chunk of one wave: K is split over the lane group g and
// the chunk's 4 registers, the 16 columns (or rows) are n.  The index bits
// of each layout (g = lane bits 5,4; n = lane bits 3..0):
//   P1: i=(15,14) g=(13,12) n=(5,4,3,2) w=(11,9,8,6) c=(7,10,1,0)  [loads: 16 B/lane]
//   P2: i=(11,10) g=(9,8)   n=(3..0)    w=(15..12)   c=(7,6,5,4)
//   P3: i=(7,6)   g=(5,4)   n=(3..0)    w=(15..12)   c=(11..8)
//   P4: i=(1,0)   g=(3,2)   n=(7..4)    w=(15..12)   c=(11..8)   [NTT-domain stores: 16 B/lane]
//   Q3: i=(5,4)   g=(7,6)   n=(3..0)    w=(15..12)   c=(11..8)   (inverse)
// P1 -> P2 goes through LDS (two rounds of 128 KiB split on bit 7, the pass
// of one round's chunks running while the other round's words move); P2 ->
// P3 and Q3 -> P2 trade lane bits 5,4 with two register bits
// (v_permlane32_swap / v_permlane16_swap); P3 -> P4 and P4 -> Q3 are free:
// the pass takes the data as the MFMA's A operand, whose result puts the
// output index on the lanes and the data rows on lane group and register
// (D[row][col] at lane 16 (row >> 2) + col, register row & 3).
#include <hip/hip_runtime.h>

#include <vector>

#include "rnt_internal.hpp"
#include "rnt_hostmath.hpp"
#include "rnt_modarith.hpp"
#include "rnt_device.hpp"

namespace rnt {

// Phase timeline of k_mf_ntt (measurement build only: MF_ONLY=1
// tools/build_variant.sh mftrace -DRNT_MF_TRACE; tools/mf_trace.py): lane 0
// of every wave of the first kMfTraceWg workgroups stamps the 100 MHz
// real-time counter at each phase boundary (waiting only for the stamp's own
// scalar read, so the plane's loads and stores stay asynchronous).
#ifdef RNT_MF_TRACE
constexpr int kMfTraceWg = 4096, kMfTraceSt = 16;
__device__ uint64_t g_mf_trace[kMfTraceWg * 16 * kMfTraceSt];
#define MF_STAMP(S)                                                                                  \
  do {                                                                                               \
    const uint32_t wg_ = blockIdx.x + blockIdx.y * gridDim.x;                                        \
    if ((threadIdx.x & 63u) == 0 && wg_ < (uint32_t)kMfTraceWg)                                      \
      g_mf_trace[(wg_ * 16 + (threadIdx.x >> 6)) * kMfTraceSt + (S)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define MF_STAMP(S) \
  do {              \
  } while (0)
#endif

namespace mf {

typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int kT = 1024;
constexpr uint32_t kN = 1u << 16;
constexpr uint32_t K32 = 0x80808080u;

// ---- per-limb table (v4i units): MFMA operands, compensations, twists ----
// Matrix slot s, digit plane a, lane lam: operand bytes of that lane.
// F1..F4: the forward passes (F2: one per U), I4..I1: the inverse's.
constexpr int S_F1 = 0, S_F2 = 1, S_F3 = 17, S_F4 = 18, S_I4 = 19, S_I3 = 20, S_I2 = 21, S_I1 = 37;
constexpr int kSlots = 38;
constexpr int kMat = 0;
constexpr int kCompF1 = kSlots * 4 * 64;  // [lam]: digit-0 accumulator start of pass 0 (input bias)
constexpr int kCompI4 = kCompF1 + 64;     // [lam]: the same for the standalone inverse's first pass
constexpr int kTw3f = kCompI4 + 64;       // [w][g][c], element i: pass 2 twist, P2 positions
constexpr int kTw4f = kTw3f + 1024;       // [w][c][lam]: pass 3 twist, P4 positions
constexpr int kTw4i = kTw4f + 16384;      // [w][c][lam]: inverse pass 3 twist, Q3 positions
constexpr int kTw3i = kTw4i + 16384;      // [w][c][g]: inverse pass 2 twist, Q3 positions
// F4S: F4 times 2^32 (k_mf_mul's fwd(a), so a Montgomery product of its
// output with b^ is the exact product), a matrix slot past the twists (the
// offsets before it stay as they were: moving them cost hipcc SGPRs and
// 170 bytes a lane of spills in k_mf_mul)
constexpr int S_F4S = (kTw3i + 1024 + 255) / 256;
constexpr int kLimb = (S_F4S + 1) * 256;
// LDS: the P1 <-> P2 exchange (128 KiB: half a plane per round) and the
// inverse's stash (10 KiB a wave); one workgroup per CU either way
constexpr size_t kLdsBytes = (size_t)160 * 1024;
// k_mf_tensor indexes its scratch slot by the CU it runs on: that needs one
// resident workgroup per CU, which more than half the CU's 160 KiB of LDS
// guarantees (as k_plane_fused_slots asserts for its own slots)
static_assert(kLdsBytes > 80 * 1024, "one workgroup per CU");

// Registers of a P3 / P4 / Q3 chunk (c, i) after the P2 -> P3 swap, as
// physical slots of the P2 numbering 4c + i (see the header).
__host__ __device__ constexpr int p3(int c, int i) {
  return 4 * (8 * (i >> 1) + 4 * (i & 1) + 2 * ((c >> 1) & 1) + (c & 1)) + 2 * (c >> 3) + ((c >> 2) & 1);
}
// P2 chunk (c, i) after the inverse's Q3 -> P2 swap.
__host__ __device__ constexpr int q2(int c, int i) {
  return p3(8 * (i >> 1) + 4 * (i & 1) + 2 * (c >> 3) + ((c >> 2) & 1), 2 * ((c >> 1) & 1) + (c & 1));
}

struct Mc {
  int32_t q;       // modulus < 2^31
  uint32_t nqinv;  // -q^-1 mod 2^32
  int64_t K;       // 0x80808080 << 32: the digit bias, added in a reduction's addend
  int64_t K0;      // 0 (opaque)
  int32_t one;     // opaque 1 and 2^16 (SGPR operands of v_mad_i64_i32)
  int32_t s16;
};

// Every global access goes through a buffer descriptor (base and range in
// SGPRs): a lane offset in a VGPR, the rest as the SGPR offset, so no 64-bit
// addresses live in VGPRs.
typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)bytes, 0x00020000);
}
// RNT_MF_NT: the cache-policy bits of the plane loads and stores that
// stream (the operand planes in, the result out): 2 = nt, so they do not
// push the re-read lines (the tables, the a^ slot) out of the L2.
#ifndef RNT_MF_NT
#define RNT_MF_NT 2
#endif
constexpr int kStreamAux = RNT_MF_NT;
// RNT_MF_LAST_NT: the same hint on k_mf_tensor's last reads of its
// temporaries (c0^, c1^, t in the last epilogue) and its final d0, d1
// stores (-2.8% tensor time; on k_mf_mul's a^ reads it measured -0.3%, so
// those keep the default, profiles/r05/ab_mf_nt.txt)
#ifndef RNT_MF_LAST_NT
#define RNT_MF_LAST_NT 2
#endif
constexpr int kLastAux = RNT_MF_LAST_NT;
template <int AUX = 0>
__device__ __forceinline__ v4i bld(Rsrc r, uint32_t voff, uint32_t soff) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, AUX);
  return v4i{(int)v[0], (int)v[1], (int)v[2], (int)v[3]};
}
template <int AUX = 0>
__device__ __forceinline__ void bst(v4i x, Rsrc r, uint32_t voff, uint32_t soff) {
  using V4 = decltype(__builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, 0));
  V4 v;
  v[0] = (uint32_t)x[0];
  v[1] = (uint32_t)x[1];
  v[2] = (uint32_t)x[2];
  v[3] = (uint32_t)x[3];
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, soff, AUX);
  // The store reads its 128-bit data after issue, and hipcc pads nothing
  // for a buffer store with an SGPR soffset: a VALU write of the data
  // registers 0-1 wait states later lost single lanes of stored words (r05,
  // profiles/r05/ab_mf_ntt_split_load.txt).  The empty statement keeps v
  // live, 2 wait states on, so nothing overwrites it sooner
  // (tools/isa_check.py rule S1 checks every kernel).
  asm volatile("s_nop 1" ::"v"(v));
}

// Output word from its four digit sums: r = T 2^-32 mod q (signed
// representative), + 0x80808080 when WK (then ^ K32 packs it).
template <bool WK>
__device__ __forceinline__ int32_t recomb(int32_t c0, int32_t c1, int32_t c2, int32_t c3, const Mc& m) {
  const int32_t lo = c0 + (int32_t)((uint32_t)c1 << 8);
  const int32_t hi = c2 + (int32_t)((uint32_t)c3 << 8);
  int64_t t;
  if constexpr (WK) {
    // the digit bias rides in the addend's high word; the multiplier is the
    // inline constant 1 (as lo * m.one + m.K, two SGPR operands exceed the
    // one-scalar operand limit and hipcc kept K in a VGPR pair all kernel)
    uint64_t cc;
    asm("v_mad_i64_i32 %0, %1, %2, 1, %3" : "=v"(t), "=s"(cc) : "v"(lo), "s"(m.K));
  } else {
    t = (int64_t)lo;  // sign extension: one shift instead of a 64-bit multiply-add
  }
  t = (int64_t)hi * m.s16 + t;
  const uint32_t mm = (uint32_t)t * m.nqinv;
  const int64_t v = (int64_t)(int32_t)mm * m.q + t;
  return (int32_t)(v >> 32);
}
// Signed Montgomery product a b 2^-32 mod q, + 0x80808080 when WK.  Any
// |a|, |b| < q < 2^31: |a b + m q| < q^2 + 2^31 q < 2^63 and the result lies
// in (-q, q); the bias K only adds to the high word (its low word is 0), so
// a wrap of the 64-bit sum does not change the returned word mod 2^32.
// Where the result is handed on in the packed byte form (k_mf_mul's
// product), the operands are pass outputs, |a|, |b| < q/2 + 2^14, so
// |v| < (q/2 + 2^14)^2 / 2^32 + q/2 + 1 < 5q/8 + 1 < 0x7F7F7F7F, inside the
// packed range [-0x80808080, 0x7F7F7F7F] (mf_build checks it per prime).
template <bool WK>
__device__ __forceinline__ int32_t mont(int32_t a, int32_t b, const Mc& m) {
  // one v_mad_i64_i32 (left to itself hipcc widens a -- the high word of
  // the previous reduction -- to a 64-bit multiply of six instructions)
  int64_t p;
  uint64_t cc;
  asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=v"(p), "=s"(cc) : "v"(a), "v"(b), "s"(WK ? m.K : m.K0));
  const uint32_t mm = (uint32_t)p * m.nqinv;
  const int64_t v = (int64_t)(int32_t)mm * m.q + p;
  return (int32_t)(v >> 32);
}
// The end of one tile's work: hipcc would otherwise hoist later tiles'
// MFMAs and loads above it and keep their digit sums live (spills).
__device__ __forceinline__ void tile_fence() { __builtin_amdgcn_sched_barrier(0); }
// Pins a tile's four outputs as computed at this point: IR-level code motion
// (sched_barrier orders only the machine scheduler) would otherwise sink the
// reductions to the words' next use and keep their partial sums live.
__device__ __forceinline__ void pin4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  asm volatile("" ::"v"(a), "v"(b), "v"(c), "v"(d));
}
__device__ __forceinline__ uint32_t pk_canon(uint32_t x) { return (x + 0x40808080u) ^ K32; }  // x - 2^30, packed
__device__ __forceinline__ uint32_t canon(int32_t r, int32_t q) { return (uint32_t)(r + ((r >> 31) & q)); }

// One MFMA tile: the four digit planes of a 16 x 16 x 64 product, hazard-safe
// by construction ("MFMA hazards"; tools/isa_check.py checks
// the built code).  The four MFMAs are one asm statement:
//  - the results are early-clobber outputs, so no MFMA's D overlaps any
//    operand of the tile (hipcc's own allocation let the last MFMA's D take
//    the data operand's registers, wholly or in part: the case that gave
//    k_mf_tensor its wrong words, r04);
//  - `s_nop 1` first: the operands hipcc's VALU just wrote are 2 wait
//    states old when the first MFMA reads them (hipcc pads nothing it cannot
//    see, and an asm MFMA is invisible to it);
//  - `s_nop 7` last: nothing after the statement -- hipcc's code or an asm
//    writer such as mont()'s v_mad_i64_i32, which its hazard recognizer does
//    not check against MFMAs -- reads or writes a register any of the four
//    MFMAs reads or writes until 8 wait states after the last one issued,
//    the XDL write -> VALU access window of a 4-pass MFMA on gfx950 (the
//    window hipcc itself pads for its own reads of a builtin MFMA's D).
// DA: the data is the A operand (the matrix the B operand).  HC: the first
// digit plane accumulates onto c0 (otherwise the inline constant 0).
template <bool DA, bool HC>
__device__ __forceinline__ void tile(v4i (&D)[4], const v4i (&M)[4], v4i dat, v4i c0) {
#define RNT_MF4(A0, B0, A1, B1, A2, B2, A3, B3, C0)                                  \
  "s_nop 1\n\t"                                                                      \
  "v_mfma_i32_16x16x64_i8 %0, " A0 ", " B0 ", " C0 "\n\t"                            \
  "v_mfma_i32_16x16x64_i8 %1, " A1 ", " B1 ", 0\n\t"                                 \
  "v_mfma_i32_16x16x64_i8 %2, " A2 ", " B2 ", 0\n\t"                                 \
  "v_mfma_i32_16x16x64_i8 %3, " A3 ", " B3 ", 0\n\t"                                 \
  "s_nop 7"
  if constexpr (DA && HC)
    asm volatile(RNT_MF4("%4", "%5", "%4", "%6", "%4", "%7", "%4", "%8", "%9")
                 : "=&v"(D[0]), "=&v"(D[1]), "=&v"(D[2]), "=&v"(D[3])
                 : "v"(dat), "v"(M[0]), "v"(M[1]), "v"(M[2]), "v"(M[3]), "v"(c0));
  else if constexpr (DA)
    asm volatile(RNT_MF4("%4", "%5", "%4", "%6", "%4", "%7", "%4", "%8", "0")
                 : "=&v"(D[0]), "=&v"(D[1]), "=&v"(D[2]), "=&v"(D[3])
                 : "v"(dat), "v"(M[0]), "v"(M[1]), "v"(M[2]), "v"(M[3]));
  else if constexpr (HC)
    asm volatile(RNT_MF4("%5", "%4", "%6", "%4", "%7", "%4", "%8", "%4", "%9")
                 : "=&v"(D[0]), "=&v"(D[1]), "=&v"(D[2]), "=&v"(D[3])
                 : "v"(dat), "v"(M[0]), "v"(M[1]), "v"(M[2]), "v"(M[3]), "v"(c0));
  else
    asm volatile(RNT_MF4("%5", "%4", "%6", "%4", "%7", "%4", "%8", "%4", "0")
                 : "=&v"(D[0]), "=&v"(D[1]), "=&v"(D[2]), "=&v"(D[3])
                 : "v"(dat), "v"(M[0]), "v"(M[1]), "v"(M[2]), "v"(M[3]));
#undef RNT_MF4
}
// the table of one limb; lo = lam * 16 (the lane's 16 bytes of an operand row)
__device__ __forceinline__ void load_mat(v4i (&M)[4], Rsrc tab, uint32_t slot, uint32_t lo) {
#pragma unroll
  for (int a = 0; a < 4; ++a) M[a] = bld(tab, lo, (uint32_t)(kMat + (slot * 4 + a) * 64) * 16u);
}

// The thread's coordinates.  Lane-derived values are recomputed at each use
// from an opaque copy of the thread id: hipcc would otherwise keep every
// offset derived from them live across the whole kernel (and spill them).
struct Th {
  uint32_t tid0, w;
  __device__ explicit Th(uint32_t tt) : tid0(tt), w(__builtin_amdgcn_readfirstlane(tt >> 6)) {}
  __device__ __forceinline__ uint32_t t() const {
    uint32_t v = tid0;
    asm volatile("" : "+v"(v));
    return v;
  }
  __device__ __forceinline__ uint32_t lam() const { return t() & 63u; }
  __device__ __forceinline__ uint32_t g() const { return (t() >> 4) & 3u; }
  __device__ __forceinline__ uint32_t n() const { return t() & 15u; }
};

// ---- P1 <-> P2 through LDS ----------------------------------------------------
// LDS word of index bits (bit 7 = the round) -- conflict-free for 4-byte
// accesses from both layouts (32-lane halves vary bits 12,5..2 in P1 and
// 8,3..0 in P2):
//   (b0^b4) + 2(b1^b5) + 4b2 + 8b3 + 16(b8^b12) + 32b10 + 64b14 + 128b15
//   + 256b6 + 512b11 + 1024b4 + 2048b5 + 4096b12 + 8192b13 + 16384b9
// Per thread: a base per value of the two register bits inside an XOR term,
// the other register bits as instruction offsets.
__device__ __forceinline__ void p1_bases(uint32_t (&wb)[4], const Th& h) {
  const uint32_t n0 = h.n() & 1, n1 = (h.n() >> 1) & 1, n2 = (h.n() >> 2) & 1, n3 = h.n() >> 3;
  const uint32_t g0 = h.g() & 1, g1 = h.g() >> 1;
  const uint32_t w0 = h.w & 1, w1 = (h.w >> 1) & 1, w2 = (h.w >> 2) & 1, w3 = h.w >> 3;
  const uint32_t rest = 4 * n0 + 8 * n1 + 16 * (w1 ^ g0) + 256 * w0 + 512 * w3 + 1024 * n2 + 2048 * n3 +
                        4096 * g0 + 8192 * g1 + 16384 * w2;
#pragma unroll
  for (uint32_t e = 0; e < 4; ++e) wb[e] = rest + ((e & 1) ^ n2) + 2 * ((e >> 1) ^ n3);
}
__device__ __forceinline__ void p2_bases(uint32_t (&rb)[4], const Th& h) {
  const uint32_t n0 = h.n() & 1, n1 = (h.n() >> 1) & 1, n2 = (h.n() >> 2) & 1, n3 = h.n() >> 3;
  const uint32_t g0 = h.g() & 1, g1 = h.g() >> 1;
  const uint32_t w0 = h.w & 1, w1 = (h.w >> 1) & 1, w2 = (h.w >> 2) & 1, w3 = h.w >> 3;
  const uint32_t rest = 4 * n2 + 8 * n3 + 16 * (g0 ^ w0) + 64 * w2 + 128 * w3 + 4096 * w0 + 8192 * w1 + 16384 * g1;
#pragma unroll
  for (uint32_t e = 0; e < 4; ++e) rb[e] = rest + (n0 ^ (e & 1)) + 2 * (n1 ^ (e >> 1)) + 1024 * (e & 1) + 2048 * (e >> 1);
}
// P1 register (c, i) / P2 register (c, i): word offset beside the base.
__host__ __device__ constexpr uint32_t p1_off(int c, int i) { return 32u * ((c >> 2) & 1) + 64u * (i & 1) + 128u * (i >> 1); }
__host__ __device__ constexpr uint32_t p2_off(int c, int i) { return 32u * (i & 1) + 512u * (i >> 1) + 256u * ((c >> 2) & 1); }

// LDS reads with the register part of the address as the instruction
// offset: left to itself hipcc pairs them into ds_read2_b32, whose 8-bit
// offsets cannot hold it, and keeps one address VGPR per pair (spilled).
// The reads are asm, so hipcc does not count them: lds_wait() (every
// destination named as read-write) ends each group before its first use.
template <uint32_t OFF>
__device__ __forceinline__ uint32_t lds_rd(uint32_t addr) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
template <int B0>
__device__ __forceinline__ void lds_wait8(uint32_t (&x)[64]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(x[B0 + 0]), "+v"(x[B0 + 1]), "+v"(x[B0 + 2]), "+v"(x[B0 + 3]), "+v"(x[B0 + 4]),
                 "+v"(x[B0 + 5]), "+v"(x[B0 + 6]), "+v"(x[B0 + 7]));
}

// Round H of P1 -> P2: P1 chunks 8H .. 8H+7 out, P2 chunks 8H .. 8H+7 in.
template <int H>
__device__ __forceinline__ void x_write_p1(const uint32_t (&x1)[64], uint32_t* lds, const uint32_t (&wb)[4]) {
#pragma unroll
  for (int c = 8 * H; c < 8 * H + 8; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) lds[wb[c & 3] + p1_off(c, i)] = x1[4 * c + i];
}
template <int H, int C, int I>
__device__ __forceinline__ void x_read_p2_one(uint32_t (&x2)[64], uint32_t lds0, const uint32_t (&rb)[4]) {
  x2[4 * C + I] = lds_rd<p2_off(C, I) * 4u>(lds0 + rb[C & 3] * 4u);
}
template <int H>
__device__ __forceinline__ void x_read_p2(uint32_t (&x2)[64], const uint32_t* lds, const uint32_t (&rb)[4]) {
  const uint32_t l0 = (uint32_t)(uintptr_t)lds;
#define RNT_MF_RD(C)                      \
  x_read_p2_one<H, C, 0>(x2, l0, rb);     \
  x_read_p2_one<H, C, 1>(x2, l0, rb);     \
  x_read_p2_one<H, C, 2>(x2, l0, rb);     \
  x_read_p2_one<H, C, 3>(x2, l0, rb);
  RNT_MF_RD(8 * H + 0) RNT_MF_RD(8 * H + 1) RNT_MF_RD(8 * H + 2) RNT_MF_RD(8 * H + 3)
  RNT_MF_RD(8 * H + 4) RNT_MF_RD(8 * H + 5) RNT_MF_RD(8 * H + 6) RNT_MF_RD(8 * H + 7)
#undef RNT_MF_RD
  lds_wait8<32 * H + 0>(x2);
  lds_wait8<32 * H + 8>(x2);
  lds_wait8<32 * H + 16>(x2);
  lds_wait8<32 * H + 24>(x2);
}
// ---- the quarter-plane (64 KiB) P1 -> P2 exchange ---------------------------
// k_mf_mul's fwd(b) exchanges in four rounds so the LDS above 64 KiB can hold
// six of a^'s sixteen tiles a wave.  The LDS word function above without
// index bit 10 (weight 32): bits (7, 10) pick the round -- P1 chunk bits 3
// and 2, P2 chunk bit 3 and register bit i0 -- and the weights above 32
// halve.  The low five address bits are unchanged, so both layouts stay
// conflict-free.
__device__ __forceinline__ void p1_bases4(uint32_t (&wb)[4], const Th& h) {
  const uint32_t n0 = h.n() & 1, n1 = (h.n() >> 1) & 1, n2 = (h.n() >> 2) & 1, n3 = h.n() >> 3;
  const uint32_t g0 = h.g() & 1, g1 = h.g() >> 1;
  const uint32_t w0 = h.w & 1, w1 = (h.w >> 1) & 1, w2 = (h.w >> 2) & 1, w3 = h.w >> 3;
  const uint32_t rest = 4 * n0 + 8 * n1 + 16 * (w1 ^ g0) + 128 * w0 + 256 * w3 + 512 * n2 + 1024 * n3 +
                        2048 * g0 + 4096 * g1 + 8192 * w2;
#pragma unroll
  for (uint32_t e = 0; e < 4; ++e) wb[e] = rest + ((e & 1) ^ n2) + 2 * ((e >> 1) ^ n3);
}
__device__ __forceinline__ void p2_bases4(uint32_t (&rb)[4], const Th& h) {
  const uint32_t n0 = h.n() & 1, n1 = (h.n() >> 1) & 1, n2 = (h.n() >> 2) & 1, n3 = h.n() >> 3;
  const uint32_t g0 = h.g() & 1, g1 = h.g() >> 1;
  const uint32_t w0 = h.w & 1, w1 = (h.w >> 1) & 1, w2 = (h.w >> 2) & 1, w3 = h.w >> 3;
  const uint32_t rest = 4 * n2 + 8 * n3 + 16 * (g0 ^ w0) + 32 * w2 + 64 * w3 + 2048 * w0 + 4096 * w1 + 8192 * g1;
#pragma unroll
  for (uint32_t e = 0; e < 4; ++e) rb[e] = rest + (n0 ^ (e & 1)) + 2 * (n1 ^ (e >> 1)) + 512 * (e & 1) + 1024 * (e >> 1);
}
__host__ __device__ constexpr uint32_t p1_off4(int, int i) { return 32u * (i & 1) + 64u * (i >> 1); }
__host__ __device__ constexpr uint32_t p2_off4(int c, int i) { return 256u * (i >> 1) + 128u * ((c >> 2) & 1); }
// Round Q: P1 chunks 4Q .. 4Q+3 out; P2 chunks 8(Q >> 1) .. +7, registers
// i = Q & 1 and (Q & 1) + 2, in.
template <int Q>
__device__ __forceinline__ void x_write_p1q(const uint32_t (&x1)[64], uint32_t* lds, const uint32_t (&wb)[4]) {
#pragma unroll
  for (int c = 4 * Q; c < 4 * Q + 4; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) lds[wb[c & 3] + p1_off4(c, i)] = x1[4 * c + i];
}
template <int C, int I>
__device__ __forceinline__ void x_read_p2q_one(uint32_t (&x2)[64], uint32_t lds0, const uint32_t (&rb)[4]) {
  x2[4 * C + I] = lds_rd<p2_off4(C, I) * 4u>(lds0 + rb[C & 3] * 4u);
}
template <int Q>
__device__ __forceinline__ void x_read_p2q(uint32_t (&x2)[64], const uint32_t* lds, const uint32_t (&rb)[4]) {
  constexpr int H = Q >> 1, X = Q & 1;
  const uint32_t l0 = (uint32_t)(uintptr_t)lds;
#define RNT_MF_RDQ(C)                    \
  x_read_p2q_one<C, X>(x2, l0, rb);      \
  x_read_p2q_one<C, X + 2>(x2, l0, rb);
  RNT_MF_RDQ(8 * H + 0) RNT_MF_RDQ(8 * H + 1) RNT_MF_RDQ(8 * H + 2) RNT_MF_RDQ(8 * H + 3)
  RNT_MF_RDQ(8 * H + 4) RNT_MF_RDQ(8 * H + 5) RNT_MF_RDQ(8 * H + 6) RNT_MF_RDQ(8 * H + 7)
#undef RNT_MF_RDQ
  constexpr int B = 32 * H + X;
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(x2[B + 0]), "+v"(x2[B + 2]), "+v"(x2[B + 4]), "+v"(x2[B + 6]), "+v"(x2[B + 8]),
                 "+v"(x2[B + 10]), "+v"(x2[B + 12]), "+v"(x2[B + 14]), "+v"(x2[B + 16]), "+v"(x2[B + 18]),
                 "+v"(x2[B + 20]), "+v"(x2[B + 22]), "+v"(x2[B + 24]), "+v"(x2[B + 26]), "+v"(x2[B + 28]),
                 "+v"(x2[B + 30]));
}
// the inverse direction: P2 words at q2(c, i) out, P1 words in
template <int H>
__device__ __forceinline__ void x_write_p2(const uint32_t (&x2)[64], uint32_t* lds, const uint32_t (&rb)[4]) {
#pragma unroll
  for (int c = 8 * H; c < 8 * H + 8; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) lds[rb[c & 3] + p2_off(c, i)] = x2[q2(c, i)];
}
template <int H, int C, int I>
__device__ __forceinline__ void x_read_p1_one(uint32_t (&x1)[64], uint32_t lds0, const uint32_t (&wb)[4]) {
  x1[4 * C + I] = lds_rd<p1_off(C, I) * 4u>(lds0 + wb[C & 3] * 4u);
}
template <int H>
__device__ __forceinline__ void x_read_p1(uint32_t (&x1)[64], const uint32_t* lds, const uint32_t (&wb)[4]) {
  const uint32_t l0 = (uint32_t)(uintptr_t)lds;
#define RNT_MF_RD(C)                      \
  x_read_p1_one<H, C, 0>(x1, l0, wb);     \
  x_read_p1_one<H, C, 1>(x1, l0, wb);     \
  x_read_p1_one<H, C, 2>(x1, l0, wb);     \
  x_read_p1_one<H, C, 3>(x1, l0, wb);
  RNT_MF_RD(8 * H + 0) RNT_MF_RD(8 * H + 1) RNT_MF_RD(8 * H + 2) RNT_MF_RD(8 * H + 3)
  RNT_MF_RD(8 * H + 4) RNT_MF_RD(8 * H + 5) RNT_MF_RD(8 * H + 6) RNT_MF_RD(8 * H + 7)
#undef RNT_MF_RD
  lds_wait8<32 * H + 0>(x1);
  lds_wait8<32 * H + 8>(x1);
  lds_wait8<32 * H + 16>(x1);
  lds_wait8<32 * H + 24>(x1);
}

// Lane bits 5, 4 <-> the register bits of chunk bits 1, 0: P2 -> P3.
__device__ __forceinline__ void swap_p2p3(uint32_t (&x)[64]) {
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    if (c & 2) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const auto r = __builtin_amdgcn_permlane32_swap(x[4 * c + i], x[4 * (c | 2) + i], false, false);
      x[4 * c + i] = r[0];
      x[4 * (c | 2) + i] = r[1];
    }
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    if (c & 1) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const auto r = __builtin_amdgcn_permlane16_swap(x[4 * c + i], x[4 * (c | 1) + i], false, false);
      x[4 * c + i] = r[0];
      x[4 * (c | 1) + i] = r[1];
    }
  }
}
// Q3 -> P2 (the inverse): Q3 chunk bits 1, 0 (index bits 9, 8) <-> lane bits 5, 4.
__device__ __forceinline__ void swap_q3p2(uint32_t (&x)[64]) {
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    if (c & 2) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const auto r = __builtin_amdgcn_permlane32_swap(x[p3(c, i)], x[p3(c | 2, i)], false, false);
      x[p3(c, i)] = r[0];
      x[p3(c | 2, i)] = r[1];
    }
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    if (c & 1) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const auto r = __builtin_amdgcn_permlane16_swap(x[p3(c, i)], x[p3(c | 1, i)], false, false);
      x[p3(c, i)] = r[0];
      x[p3(c | 1, i)] = r[1];
    }
  }
}

// ---- the passes -------------------------------------------------------------
// Progress priority (RNT_MF_PRIO) over the forward's barrier-free stretch
// (pass 1's second half, pass 2, pass 3: tiles p = 0..39): a wave lowers its
// priority 3 -> 0 as it advances, so a wave that fell behind outranks the
// ones ahead of it and the sixteen finish together instead of in age order
// (r05 trace: the last wave of a CU ended 11 us after the first).
#ifndef RNT_MF_PRIO
#define RNT_MF_PRIO 1
#endif
// k_mf_tensor: each forward's exchange fenced after its own last read
#ifndef RNT_MF_TENSOR_SYNCX
#define RNT_MF_TENSOR_SYNCX 1
#endif
#ifndef RNT_MF_TENSOR_PARK
#define RNT_MF_TENSOR_PARK 0
#endif
#ifndef RNT_MF_TENSOR_MEAS
#define RNT_MF_TENSOR_MEAS 0
#endif
#ifndef RNT_MF_TENSOR_PARK4
#define RNT_MF_TENSOR_PARK4 0
#endif
// the same over the inverse's first stretch (its passes 3, 2 and the first
// half of 1: 40 tiles between the plane load and the first exchange)
#ifndef RNT_MF_IPRIO
#define RNT_MF_IPRIO 1
#endif
// RNT_MF_PRIO_VAR: where the steps fall (0: tiles 0, 10, 20, 30; 1: 0, 20,
// 28, 34); p is a constant after unrolling
#ifndef RNT_MF_PRIO_VAR
#define RNT_MF_PRIO_VAR 0
#endif
template <bool ON>
__device__ __forceinline__ void mf_prio(int p) {
  if constexpr (ON) {
    constexpr int s1 = RNT_MF_PRIO_VAR ? 20 : 10, s2 = RNT_MF_PRIO_VAR ? 28 : 20, s3 = RNT_MF_PRIO_VAR ? 34 : 30;
    if (p == 0) __builtin_amdgcn_s_setprio(3);
    if (p == s1) __builtin_amdgcn_s_setprio(2);
    if (p == s2) __builtin_amdgcn_s_setprio(1);
    if (p == s3) __builtin_amdgcn_s_setprio(0);
  }
}
// pass 0 on P1 chunks [C0, C0 + 8): input canonical (BIAS: packed with the
// -2^30 shift its compensation undoes) or packed; output packed.
template <int C0, bool BIAS>
__device__ __forceinline__ void pass_p1(uint32_t (&x1)[64], const v4i (&M)[4], v4i comp, const Mc& m) {
#pragma unroll
  for (int c = C0; c < C0 + 8; ++c) {
    v4i b;
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = (int)(BIAS ? pk_canon(x1[4 * c + i]) : x1[4 * c + i]);
    v4i D[4];
    tile<false, BIAS>(D, M, b, comp);
#pragma unroll
    for (int i = 0; i < 4; ++i) x1[4 * c + i] = (uint32_t)recomb<true>(D[0][i], D[1][i], D[2][i], D[3][i], m) ^ K32;
    pin4(x1[4 * c + 0], x1[4 * c + 1], x1[4 * c + 2], x1[4 * c + 3]);
    tile_fence();
  }
}
// pass 1 (per-wave matrix) on P2 chunks [C0, C0 + 8), then the pass-2 twist
// (TW: the table in P2 positions).
template <int C0>
__device__ __forceinline__ void pass_p2(uint32_t (&x2)[64], const v4i (&M)[4], Rsrc tab, uint32_t tvo, uint32_t tso,
                                        const Mc& m) {
  const v4i z = {0, 0, 0, 0};
#pragma unroll
  for (int c = C0; c < C0 + 8; ++c) {
    if constexpr (C0 == 8) mf_prio<RNT_MF_PRIO != 0>(c - 8);
    v4i b;
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = (int)x2[4 * c + i];
    // (the twists of a 16 KiB table: cache hits, loaded at the tile -- a
    // tile-ahead prefetch measured 4 more spilled registers)
    const v4i tv = bld(tab, tvo, tso + (uint32_t)c * 16u);
    v4i D[4];
    tile<false, false>(D, M, b, z);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int32_t r = recomb<false>(D[0][i], D[1][i], D[2][i], D[3][i], m);
      x2[4 * c + i] = (uint32_t)mont<true>(r, tv[i], m) ^ K32;
    }
    pin4(x2[4 * c + 0], x2[4 * c + 1], x2[4 * c + 2], x2[4 * c + 3]);
    tile_fence();
  }
}
// pass 2 (F, data as A: P3 -> P4 positions), then the pass-3 twist.
__device__ __forceinline__ void pass_p3(uint32_t (&x)[64], const v4i (&M)[4], Rsrc tab, uint32_t tvo, uint32_t tso,
                                        const Mc& m) {
  const v4i z = {0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    mf_prio<RNT_MF_PRIO != 0>(8 + c);
    v4i a;
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = (int)x[p3(c, i)];
    const v4i tv = bld(tab, tvo, tso + (uint32_t)c * 1024u);
    v4i D[4];
    tile<true, false>(D, M, a, z);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int32_t r = recomb<false>(D[0][i], D[1][i], D[2][i], D[3][i], m);
      x[p3(c, i)] = (uint32_t)mont<true>(r, tv[i], m) ^ K32;
    }
    pin4(x[p3(c, 0)], x[p3(c, 1)], x[p3(c, 2)], x[p3(c, 3)]);
    tile_fence();
  }
}
// pass 3 (F, P4 in place): each tile's centred outputs go to EPI(c, r, x)
// at once (stored, or multiplied into the product), so no 64-bit reduction
// result stays live beyond its tile.
template <class EPI>
__device__ __forceinline__ void pass_p4(uint32_t (&x)[64], const v4i (&M)[4], const Mc& m, const EPI& epi) {
  const v4i z = {0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    mf_prio<RNT_MF_PRIO != 0>(24 + c);
    v4i b;
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = (int)x[p3(c, i)];
    v4i D[4];
    tile<false, false>(D, M, b, z);
    int32_t r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = recomb<false>(D[0][i], D[1][i], D[2][i], D[3][i], m);
    epi(c, r, x);
    tile_fence();
  }
}
// The inverse's first two passes hold the whole plane and two matrices'
// worth of operands in registers: the outputs of ipass_p4's first kStash
// tiles wait in a per-wave LDS stash (the LDS is idle until the exchanges)
// until ipass_p3 takes them, instead of being spilled to scratch memory.
constexpr int kStash = 10;  // the most that fits: fewer measured more spills (8: 52 B a lane in the inverse)
static_assert((size_t)kStash * 16 * 1024 <= kLdsBytes, "sixteen waves' stashes in the LDS");
__device__ __forceinline__ uint32_t stash_addr(const uint32_t* lds, const Th& h) {
  return (uint32_t)(uintptr_t)lds + (h.w * (kStash * 64u) + h.lam()) * 16u;
}
__device__ __forceinline__ void stash_put(uint32_t addr, int c, uint32_t a, uint32_t b, uint32_t d, uint32_t e) {
  asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(addr), "v"(v4i{(int)a, (int)b, (int)d, (int)e}), "i"(c * 1024)
               : "memory");
}
__device__ __forceinline__ v4i stash_get(uint32_t addr, int c) {
  v4i v;
  asm volatile("ds_read_b128 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr), "i"(c * 1024) : "memory");
  return v;
}
// inverse pass 3 (F^-1, data as A: P4 -> Q3) on the canonical words as
// loaded (biased here, comp undoes it), then its twist; packed output.
// tv: tile 0's twists (each tile loads the next one's).
// PK: the words are already in the passes' packed signed form (a product
// epilogue's Montgomery output), so no bias and no compensation.
template <bool PK = false>
__device__ __forceinline__ void ipass_p4(uint32_t (&x)[64], const v4i (&M)[4], v4i comp, v4i tv, Rsrc tab,
                                         uint32_t tvo, uint32_t tso, const Mc& m, uint32_t* lds, const Th& h) {
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    mf_prio<RNT_MF_IPRIO != 0>(c);
    v4i a;
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = (int)(PK ? x[p3(c, i)] : pk_canon(x[p3(c, i)]));
    const v4i tn = c + 1 < 16 ? bld(tab, tvo, tso + (uint32_t)(c + 1) * 1024u) : tv;
    v4i D[4];
    if constexpr (PK)
      tile<true, false>(D, M, a, v4i{0, 0, 0, 0});
    else
      tile<true, true>(D, M, a, comp);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int32_t r = recomb<false>(D[0][i], D[1][i], D[2][i], D[3][i], m);
      x[p3(c, i)] = (uint32_t)mont<true>(r, tv[i], m) ^ K32;
    }
    if (c < kStash)
      stash_put(stash_addr(lds, h), c, x[p3(c, 0)], x[p3(c, 1)], x[p3(c, 2)], x[p3(c, 3)]);
    else
      pin4(x[p3(c, 0)], x[p3(c, 1)], x[p3(c, 2)], x[p3(c, 3)]);
    tv = tn;
    tile_fence();
  }
}
// inverse pass 2 (F^-1 in Q3), then its twist; packed output.
__device__ __forceinline__ void ipass_p3(uint32_t (&x)[64], const v4i (&M)[4], Rsrc tab, uint32_t tvo, uint32_t tso,
                                         const Mc& m, uint32_t* lds, const Th& h) {
  const v4i z = {0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    mf_prio<RNT_MF_IPRIO != 0>(16 + c);
    v4i b;
    if (c < kStash) {
      b = stash_get(stash_addr(lds, h), c);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) b[i] = (int)x[p3(c, i)];
    }
    const v4i tv = bld(tab, tvo, tso + (uint32_t)c * 64u);
    v4i D[4];
    tile<false, false>(D, M, b, z);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int32_t r = recomb<false>(D[0][i], D[1][i], D[2][i], D[3][i], m);
      x[p3(c, i)] = (uint32_t)mont<true>(r, tv[i], m) ^ K32;
    }
    pin4(x[p3(c, 0)], x[p3(c, 1)], x[p3(c, 2)], x[p3(c, 3)]);
    tile_fence();
  }
}
// inverse pass 1 (per-wave matrix) on P2 chunks [C0, C0 + 8) at q2 slots
// (the registers after the Q3 -> P2 swap); packed output.
template <int C0>
__device__ __forceinline__ void ipass_p2(uint32_t (&x)[64], const v4i (&M)[4], const Mc& m) {
  const v4i z = {0, 0, 0, 0};
#pragma unroll
  for (int c = C0; c < C0 + 8; ++c) {
    if constexpr (C0 == 0) mf_prio<RNT_MF_IPRIO != 0>(32 + c);
    v4i b;
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = (int)x[q2(c, i)];
    v4i D[4];
    tile<false, false>(D, M, b, z);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      x[q2(c, i)] = (uint32_t)recomb<true>(D[0][i], D[1][i], D[2][i], D[3][i], m) ^ K32;
    pin4(x[q2(c, 0)], x[q2(c, 1)], x[q2(c, 2)], x[q2(c, 3)]);
    tile_fence();
  }
}
// inverse pass 0 on P1 chunks [C0, C0 + 8): canonical output; every four
// chunks (the words of one 16-byte store per register) go to memory at once.
template <int C0>
__device__ __forceinline__ void ipass_p1(uint32_t (&x1)[64], const v4i (&M)[4], const Mc& m, Rsrc dst,
                                         const Th& h);

// P1 plane byte offsets of load / store (i, hc): 4 consecutive words,
// chunks c = 4 hc + e, e = 0..3.  Lane part (VGPR), wave part and the
// register part (SGPR).
__device__ __forceinline__ uint32_t p1_lane(const Th& h) { return ((h.g() << 12) | (h.n() << 2)) * 4u; }
__device__ __forceinline__ uint32_t p1_wave(const Th& h) {
  const uint32_t w = h.w;
  return (((w >> 3) << 11) | (((w >> 2) & 1) << 9) | (((w >> 1) & 1) << 8) | ((w & 1) << 6)) * 4u;
}
__host__ __device__ constexpr uint32_t p1_reg(int i, int hc) {
  return (((uint32_t)i << 14) | ((uint32_t)(hc & 1) << 10) | ((uint32_t)(hc >> 1) << 7)) * 4u;
}
__device__ __forceinline__ void load_p1(uint32_t (&x1)[64], Rsrc src, const Th& h) {
  const uint32_t lo = p1_lane(h), wo = p1_wave(h);
#pragma unroll
  for (int hc = 0; hc < 4; ++hc)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const v4i v = bld<kStreamAux>(src, lo, wo + p1_reg(i, hc));
#pragma unroll
      for (int e = 0; e < 4; ++e) x1[4 * (4 * hc + e) + i] = (uint32_t)v[e];
    }
}
template <int C0>
__device__ __forceinline__ void ipass_p1(uint32_t (&x1)[64], const v4i (&M)[4], const Mc& m, Rsrc dst,
                                         const Th& h) {
  const v4i z = {0, 0, 0, 0};
#pragma unroll
  for (int c = C0; c < C0 + 8; ++c) {
    v4i b;
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = (int)x1[4 * c + i];
    v4i D[4];
    tile<false, false>(D, M, b, z);
#pragma unroll
    for (int i = 0; i < 4; ++i) x1[4 * c + i] = canon(recomb<false>(D[0][i], D[1][i], D[2][i], D[3][i], m), m.q);
    if ((c & 3) == 3) {
      const int hc = c >> 2;
      const uint32_t lo = p1_lane(h), wo = p1_wave(h);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v4i v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (int)x1[4 * (4 * hc + e) + i];
        bst<kStreamAux>(v, dst, lo, wo + p1_reg(i, hc));
      }
    } else {
      pin4(x1[4 * c + 0], x1[4 * c + 1], x1[4 * c + 2], x1[4 * c + 3]);
    }
    tile_fence();
  }
}

// P4 (NTT-domain device order): chunk c's 4 words are consecutive.
__device__ __forceinline__ uint32_t p4_lane(const Th& h) { return ((h.n() << 4) | (h.g() << 2)) * 4u; }
__device__ __forceinline__ uint32_t p4_soff(const Th& h, int c) { return ((h.w << 12) | ((uint32_t)c << 8)) * 4u; }

struct Tabs {
  Rsrc tab;  // this limb's table
  Mc m;
};
__device__ __forceinline__ Tabs tabs_of(const void* mf, const LimbConst<uint32_t>& lc, uint32_t l) {
  Tabs r;
  r.tab = rsrc((const v4i*)mf + (size_t)l * kLimb, (uint32_t)kLimb * 16u);
  r.m.q = (int32_t)lc.q;
  r.m.nqinv = 0u - lc.qinv;
  int64_t K = (int64_t)((uint64_t)K32 << 32), K0 = 0;
  int32_t one = 1, s16 = 65536;
  asm volatile("" : "+s"(one), "+s"(s16), "+s"(K), "+s"(K0));
  r.m.K = K;
  r.m.K0 = K0;
  r.m.one = one;
  r.m.s16 = s16;
  return r;
}

// The forward transform: canonical plane at src (P1) -> x2 in P4 positions,
// centred representatives.  SYNC1: the LDS may still be in use by other waves.
// EPI(c, r, x2): the last pass's per-tile epilogue (the standalone forward
// stores each tile from it).
struct NoEpi {
  __device__ void operator()(int, const int32_t (&)[4], uint32_t (&)[64]) const {}
};
// Q4: the exchange in four quarter-plane rounds (the LDS above 64 KiB stays
// free); SYNCX: a barrier after the last exchange read (the caller writes
// the exchange region's upper half from the last pass on).
// NPARK: P2 chunks 0..NPARK-1 (idle through pass 1's second half) wait in
// the LDS at byte PBASE + wave * PSTRIDE from SYNCX to the P2 -> P3 swap,
// instead of being spilled to scratch memory (whose write-back is HBM
// traffic); the caller guarantees no other wave touches that LDS then.
template <int NPARK, uint32_t PBASE, uint32_t PSTRIDE>
__device__ __forceinline__ uint32_t park_addr(const uint32_t* lds, const Th& h) {
  static_assert(NPARK * 1024 <= (int)PSTRIDE && PBASE + 16 * PSTRIDE <= kLdsBytes, "park area");
  return (uint32_t)(uintptr_t)lds + PBASE + h.w * PSTRIDE + h.lam() * 16u;
}
template <bool SYNC1, int F4 = S_F4, bool Q4 = false, bool SYNCX = false, int NPARK = 0, uint32_t PBASE = 0,
          uint32_t PSTRIDE = 0, class EPI = NoEpi>
__device__ __forceinline__ void fwd(uint32_t (&x2)[64], Rsrc src, uint32_t* lds, const Th& h, const Tabs& T,
                                    const EPI& epi = EPI{}) {
  // the first pass's operands load ahead of the plane (cache hits, needed
  // first): its first tile then waits only for its own words
  const Mc& m = T.m;
  const uint32_t lo = h.lam() * 16u;
  v4i M[4];
  load_mat(M, T.tab, S_F1, lo);
  const v4i comp = bld(T.tab, lo, (uint32_t)kCompF1 * 16u);
  uint32_t x1[64];
  load_p1(x1, src, h);
  MF_STAMP(1);
  pass_p1<0, true>(x1, M, comp, m);
  MF_STAMP(2);
  if constexpr (SYNC1) __syncthreads();
  uint32_t wb[4], rb[4];
  const uint32_t t3v = h.g() * 256u, t3s = (uint32_t)(kTw3f + h.w * 64) * 16u;
  if constexpr (Q4) {
    p1_bases4(wb, h);
    x_write_p1q<0>(x1, lds, wb);
    pass_p1<8, true>(x1, M, comp, m);
    __syncthreads();
    p2_bases4(rb, h);
    x_read_p2q<0>(x2, lds, rb);
    __syncthreads();
    p1_bases4(wb, h);
    x_write_p1q<1>(x1, lds, wb);
    __syncthreads();
    p2_bases4(rb, h);
    x_read_p2q<1>(x2, lds, rb);
    __syncthreads();
    p1_bases4(wb, h);
    x_write_p1q<2>(x1, lds, wb);
    load_mat(M, T.tab, S_F2 + h.w, lo);
    pass_p2<0>(x2, M, T.tab, t3v, t3s, m);
    __syncthreads();
    p2_bases4(rb, h);
    x_read_p2q<2>(x2, lds, rb);
    __syncthreads();
    p1_bases4(wb, h);
    x_write_p1q<3>(x1, lds, wb);
    __syncthreads();
    p2_bases4(rb, h);
    x_read_p2q<3>(x2, lds, rb);
  } else {
  p1_bases(wb, h);
  x_write_p1<0>(x1, lds, wb);
  pass_p1<8, true>(x1, M, comp, m);
  MF_STAMP(3);
  __syncthreads();
  MF_STAMP(4);
  p2_bases(rb, h);
  x_read_p2<0>(x2, lds, rb);
  __syncthreads();
  MF_STAMP(5);
  p1_bases(wb, h);
  x_write_p1<1>(x1, lds, wb);
  load_mat(M, T.tab, S_F2 + h.w, lo);
  pass_p2<0>(x2, M, T.tab, t3v, t3s, m);
  MF_STAMP(6);
  __syncthreads();
  MF_STAMP(7);
  p2_bases(rb, h);
  x_read_p2<1>(x2, lds, rb);
  }
  if constexpr (SYNCX) __syncthreads();
  static_assert(NPARK == 0 || SYNCX, "the park area is free only past SYNCX");
#pragma unroll
  for (int c = 0; c < NPARK; ++c)
    stash_put(park_addr<NPARK, PBASE, PSTRIDE>(lds, h), c, x2[4 * c], x2[4 * c + 1], x2[4 * c + 2], x2[4 * c + 3]);
  pass_p2<8>(x2, M, T.tab, t3v, t3s, m);
  MF_STAMP(8);
#pragma unroll
  for (int c = 0; c < NPARK; ++c) {
    const v4i v = stash_get(park_addr<NPARK, PBASE, PSTRIDE>(lds, h), c);
#pragma unroll
    for (int i = 0; i < 4; ++i) x2[4 * c + i] = (uint32_t)v[i];
  }
  swap_p2p3(x2);
  load_mat(M, T.tab, S_F3, lo);
  pass_p3(x2, M, T.tab, lo, (uint32_t)(kTw4f + h.w * 1024) * 16u, m);
  MF_STAMP(9);
  load_mat(M, T.tab, F4, lo);
  pass_p4(x2, M, m, epi);
  MF_STAMP(10);
}

// The inverse in place: the NTT-domain plane (device order, P4 positions)
// to the canonical coefficients (P1).  The first pass's digit-0
// accumulators start at the input bias's compensation (canonical input
// words travel as x - 2^30).  The first pass's operands load ahead of the
// plane (cache hits, needed first); its first tile then waits only for
// its own words.  In place: a wave stores only after the exchanges'
// barriers, which it passes once it has used (so read) every word it loaded.
// LOAD = false: the plane is already in x2 (P4 positions, canonical), as a
// forward pass's epilogue left it; the LDS may still be read by other waves.
template <bool LOAD, bool PK = false>
__device__ __forceinline__ void inv_x(uint32_t (&x2)[64], Rsrc pr, uint32_t* lds, const Th& h, const Tabs& T) {
  const Mc& m = T.m;
  const uint32_t lo = h.lam() * 16u;
  v4i M[4];
  load_mat(M, T.tab, S_I4, lo);
  const v4i comp = bld(T.tab, lo, (uint32_t)kCompI4 * 16u);
  const uint32_t t4s = (uint32_t)(kTw4i + h.w * 1024) * 16u;
  const v4i tv0 = bld(T.tab, lo, t4s);
  if constexpr (LOAD) {
#pragma unroll
    for (int cc = 0; cc < 16; ++cc) {
      const v4i v = bld<kStreamAux>(pr, p4_lane(h), p4_soff(h, cc));
#pragma unroll
      for (int i = 0; i < 4; ++i) x2[p3(cc, i)] = (uint32_t)v[i];
    }
  } else {
    __syncthreads();  // ipass_p4's stash reuses the LDS of the last exchange
  }
  ipass_p4<PK>(x2, M, comp, tv0, T.tab, lo, t4s, m, lds, h);
  load_mat(M, T.tab, S_I3, lo);
  ipass_p3(x2, M, T.tab, h.g() * 16u, (uint32_t)(kTw3i + h.w * 64) * 16u, m, lds, h);
  swap_q3p2(x2);
  load_mat(M, T.tab, S_I2 + h.w, lo);
  uint32_t wb[4], rb[4];
  uint32_t x1[64];
  ipass_p2<0>(x2, M, m);
  __syncthreads();  // other waves may still read the LDS (the last forward exchange)
  p2_bases(rb, h);
  x_write_p2<0>(x2, lds, rb);
  ipass_p2<8>(x2, M, m);
  __syncthreads();
  p1_bases(wb, h);
  x_read_p1<0>(x1, lds, wb);
  __syncthreads();
  p2_bases(rb, h);
  x_write_p2<1>(x2, lds, rb);
  load_mat(M, T.tab, S_I1, lo);
  ipass_p1<0>(x1, M, m, pr, h);
  __syncthreads();
  p1_bases(wb, h);
  x_read_p1<1>(x1, lds, wb);
  ipass_p1<8>(x1, M, m, pr, h);
}
__device__ __forceinline__ void inv(Rsrc pr, uint32_t* lds, const Th& h, const Tabs& T) {
  uint32_t x2[64];
  inv_x<true>(x2, pr, lds, h, T);
}

// ---- two virtual waves a wave (k_mf_mul2) -----------------------------------
// fwd and inv_x for a 512-thread workgroup whose wave p carries the sixteen-
// wave layout's waves 2p (ha, xa) and 2p + 1 (hb, xb): every pass runs once
// for each, the barriers once for both.  The per-wave state of the 1024-thread
// layout (x, a^, the VGPRs of the working set) is then held by half as many
// threads, and the register file left over keeps a^ tiles on the CU.
template <bool SYNC1, int F4, bool Q4, bool SYNCX, int NPARK, uint32_t PBASE, uint32_t PSTRIDE, class EA, class EB>
__device__ __forceinline__ void fwd2(uint32_t (&xa)[64], uint32_t (&xb)[64], Rsrc src, uint32_t* lds, const Th& ha,
                                     const Th& hb, const Tabs& T, const EA& epa, const EB& epb) {
  const Mc& m = T.m;
  const uint32_t lo = ha.lam() * 16u;
  v4i M[4];
  load_mat(M, T.tab, S_F1, lo);
  const v4i comp = bld(T.tab, lo, (uint32_t)kCompF1 * 16u);
  uint32_t x1a[64], x1b[64];
  load_p1(x1a, src, ha);
  load_p1(x1b, src, hb);
  pass_p1<0, true>(x1a, M, comp, m);
  pass_p1<0, true>(x1b, M, comp, m);
  if constexpr (SYNC1) __syncthreads();
  uint32_t wb[4], rb[4];
  const uint32_t t3v = ha.g() * 256u;
  auto t3s = [](const Th& h) { return (uint32_t)(kTw3f + h.w * 64) * 16u; };
  if constexpr (Q4) {
    p1_bases4(wb, ha); x_write_p1q<0>(x1a, lds, wb);
    p1_bases4(wb, hb); x_write_p1q<0>(x1b, lds, wb);
    pass_p1<8, true>(x1a, M, comp, m);
    pass_p1<8, true>(x1b, M, comp, m);
    __syncthreads();
    p2_bases4(rb, ha); x_read_p2q<0>(xa, lds, rb);
    p2_bases4(rb, hb); x_read_p2q<0>(xb, lds, rb);
    __syncthreads();
    p1_bases4(wb, ha); x_write_p1q<1>(x1a, lds, wb);
    p1_bases4(wb, hb); x_write_p1q<1>(x1b, lds, wb);
    __syncthreads();
    p2_bases4(rb, ha); x_read_p2q<1>(xa, lds, rb);
    p2_bases4(rb, hb); x_read_p2q<1>(xb, lds, rb);
    __syncthreads();
    p1_bases4(wb, ha); x_write_p1q<2>(x1a, lds, wb);
    p1_bases4(wb, hb); x_write_p1q<2>(x1b, lds, wb);
    load_mat(M, T.tab, S_F2 + ha.w, lo);
    pass_p2<0>(xa, M, T.tab, t3v, t3s(ha), m);
    load_mat(M, T.tab, S_F2 + hb.w, lo);
    pass_p2<0>(xb, M, T.tab, t3v, t3s(hb), m);
    __syncthreads();
    p2_bases4(rb, ha); x_read_p2q<2>(xa, lds, rb);
    p2_bases4(rb, hb); x_read_p2q<2>(xb, lds, rb);
    __syncthreads();
    p1_bases4(wb, ha); x_write_p1q<3>(x1a, lds, wb);
    p1_bases4(wb, hb); x_write_p1q<3>(x1b, lds, wb);
    __syncthreads();
    p2_bases4(rb, ha); x_read_p2q<3>(xa, lds, rb);
    p2_bases4(rb, hb); x_read_p2q<3>(xb, lds, rb);
  } else {
    p1_bases(wb, ha); x_write_p1<0>(x1a, lds, wb);
    p1_bases(wb, hb); x_write_p1<0>(x1b, lds, wb);
    pass_p1<8, true>(x1a, M, comp, m);
    pass_p1<8, true>(x1b, M, comp, m);
    __syncthreads();
    p2_bases(rb, ha); x_read_p2<0>(xa, lds, rb);
    p2_bases(rb, hb); x_read_p2<0>(xb, lds, rb);
    __syncthreads();
    p1_bases(wb, ha); x_write_p1<1>(x1a, lds, wb);
    p1_bases(wb, hb); x_write_p1<1>(x1b, lds, wb);
    load_mat(M, T.tab, S_F2 + ha.w, lo);
    pass_p2<0>(xa, M, T.tab, t3v, t3s(ha), m);
    load_mat(M, T.tab, S_F2 + hb.w, lo);
    pass_p2<0>(xb, M, T.tab, t3v, t3s(hb), m);
    __syncthreads();
    p2_bases(rb, ha); x_read_p2<1>(xa, lds, rb);
    p2_bases(rb, hb); x_read_p2<1>(xb, lds, rb);
  }
  if constexpr (SYNCX) __syncthreads();
  static_assert(NPARK == 0 || SYNCX, "the park area is free only past SYNCX");
#pragma unroll
  for (int c = 0; c < NPARK; ++c) {
    stash_put(park_addr<NPARK, PBASE, PSTRIDE>(lds, ha), c, xa[4 * c], xa[4 * c + 1], xa[4 * c + 2], xa[4 * c + 3]);
    stash_put(park_addr<NPARK, PBASE, PSTRIDE>(lds, hb), c, xb[4 * c], xb[4 * c + 1], xb[4 * c + 2], xb[4 * c + 3]);
  }
  load_mat(M, T.tab, S_F2 + ha.w, lo);
  pass_p2<8>(xa, M, T.tab, t3v, t3s(ha), m);
  load_mat(M, T.tab, S_F2 + hb.w, lo);
  pass_p2<8>(xb, M, T.tab, t3v, t3s(hb), m);
#pragma unroll
  for (int c = 0; c < NPARK; ++c) {
    const v4i va = stash_get(park_addr<NPARK, PBASE, PSTRIDE>(lds, ha), c);
    const v4i vb = stash_get(park_addr<NPARK, PBASE, PSTRIDE>(lds, hb), c);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      xa[4 * c + i] = (uint32_t)va[i];
      xb[4 * c + i] = (uint32_t)vb[i];
    }
  }
  swap_p2p3(xa);
  swap_p2p3(xb);
  load_mat(M, T.tab, S_F3, lo);
  pass_p3(xa, M, T.tab, lo, (uint32_t)(kTw4f + ha.w * 1024) * 16u, m);
  pass_p3(xb, M, T.tab, lo, (uint32_t)(kTw4f + hb.w * 1024) * 16u, m);
  load_mat(M, T.tab, F4, lo);
  pass_p4(xa, M, m, epa);
  pass_p4(xb, M, m, epb);
}

// inv_x<false, true> for two virtual waves: the product (packed signed form,
// P4 positions) in xa / xb to the canonical coefficients stored at pr.
__device__ __forceinline__ void inv2(uint32_t (&xa)[64], uint32_t (&xb)[64], Rsrc pr, uint32_t* lds, const Th& ha,
                                     const Th& hb, const Tabs& T) {
  const Mc& m = T.m;
  const uint32_t lo = ha.lam() * 16u;
  v4i M[4];
  load_mat(M, T.tab, S_I4, lo);
  const v4i comp = {0, 0, 0, 0};  // (PK: no input bias)
  auto t4s = [](const Th& h) { return (uint32_t)(kTw4i + h.w * 1024) * 16u; };
  __syncthreads();  // ipass_p4's stash reuses the LDS of the last exchange and the a^ tiles
  ipass_p4<true>(xa, M, comp, bld(T.tab, lo, t4s(ha)), T.tab, lo, t4s(ha), m, lds, ha);
  ipass_p4<true>(xb, M, comp, bld(T.tab, lo, t4s(hb)), T.tab, lo, t4s(hb), m, lds, hb);
  load_mat(M, T.tab, S_I3, lo);
  ipass_p3(xa, M, T.tab, ha.g() * 16u, (uint32_t)(kTw3i + ha.w * 64) * 16u, m, lds, ha);
  ipass_p3(xb, M, T.tab, hb.g() * 16u, (uint32_t)(kTw3i + hb.w * 64) * 16u, m, lds, hb);
  swap_q3p2(xa);
  swap_q3p2(xb);
  uint32_t wb[4], rb[4];
  uint32_t x1a[64], x1b[64];
  load_mat(M, T.tab, S_I2 + ha.w, lo);
  ipass_p2<0>(xa, M, m);
  load_mat(M, T.tab, S_I2 + hb.w, lo);
  ipass_p2<0>(xb, M, m);
  __syncthreads();  // every wave's stash reads are done
  p2_bases(rb, ha); x_write_p2<0>(xa, lds, rb);
  p2_bases(rb, hb); x_write_p2<0>(xb, lds, rb);
  load_mat(M, T.tab, S_I2 + ha.w, lo);
  ipass_p2<8>(xa, M, m);
  load_mat(M, T.tab, S_I2 + hb.w, lo);
  ipass_p2<8>(xb, M, m);
  __syncthreads();
  p1_bases(wb, ha); x_read_p1<0>(x1a, lds, wb);
  p1_bases(wb, hb); x_read_p1<0>(x1b, lds, wb);
  __syncthreads();
  p2_bases(rb, ha); x_write_p2<1>(xa, lds, rb);
  p2_bases(rb, hb); x_write_p2<1>(xb, lds, rb);
  load_mat(M, T.tab, S_I1, lo);
  ipass_p1<0>(x1a, M, m, pr, ha);
  ipass_p1<0>(x1b, M, m, pr, hb);
  __syncthreads();
  p1_bases(wb, ha); x_read_p1<1>(x1a, lds, wb);
  p1_bases(wb, hb); x_read_p1<1>(x1b, lds, wb);
  ipass_p1<8>(x1a, M, m, pr, ha);
  ipass_p1<8>(x1b, M, m, pr, hb);
}

}  // namespace mf

// Standalone transforms in place (rnt_ntt_fwd / rnt_ntt_inv at N = 2^16),
// grid (B, L): one workgroup per (poly, limb) plane.
template <bool INV>
__global__ void __launch_bounds__(mf::kT, 1)
k_mf_ntt(uint32_t* __restrict__ data, const void* __restrict__ mft, const LimbConst<uint32_t>* __restrict__ lcs,
         uint64_t ls) {
  using namespace mf;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  uint32_t* lds = (uint32_t*)smem_raw;
  const Th h(threadIdx.x);
  const uint32_t poly = blockIdx.x, l = blockIdx.y;
  MF_STAMP(0);
  uint32_t* p = data + (uint64_t)l * ls + (uint64_t)poly * kN;
  const Tabs T = tabs_of(mft, lcs[l], l);
  const Rsrc pr = rsrc(p, kN * 4u);
  if constexpr (!INV) {
    uint32_t x[64];
    // the last pass stores each tile, canonical, in the device order (in
    // place: every wave read its words of the plane before the first
    // exchange's barrier)
    fwd<false>(x, pr, lds, h, T, [&](int cc, const int32_t (&r)[4], uint32_t (&)[64]) {
      bst<kStreamAux>(v4i{(int)canon(r[0], T.m.q), (int)canon(r[1], T.m.q), (int)canon(r[2], T.m.q), (int)canon(r[3], T.m.q)}, pr,
          p4_lane(h), p4_soff(h, cc));
    });
  } else {
    inv(pr, lds, h, T);
  }
#ifdef RNT_MF_TRACE
  __builtin_amdgcn_s_waitcnt(0);  // the plane's stores have left the CU
  MF_STAMP(11);
#endif
}

// The ciphertext tensor product at N = 2^16 (rnt_ct_tensor and the
// relinearised ct-mul, engine.rs:480-493) on the matrix-core transforms, one
// workgroup per (poly, limb): the four forward transforms run one after the
// other, each last pass's epilogue combining tile by tile with what the
// earlier ones left in memory at the same device-order positions (written
// and read back by the same thread):
//   fwd c0  -> c0^ into d1's plane (a temporary);  fwd c1 -> c1^ into the
//   CU's scratch slot (k_plane_fused_slots' indexing, or the pair's own
//   plane below kPlaneSlots pairs);  fwd c0' -> d0 = c0^ c0'^ (final) and
//   t = c1^ c0'^ into d2's plane;  fwd c1' -> d1 = t + c0^ c1'^ (final) and
//   d2 = c1^ c1'^ 2^32 in registers, inverse-transformed from there into
//   d2's plane (coefficient domain).
// d0, d1 carry the Montgomery factor 2^-32 as k_tensor_rows' do (key-switch
// seeds); the same words.  HBM: the 4 operand planes in, 3 planes out (the
// temporaries are rewritten within the workgroup's life and the slot is
// the CU's), against 17 planes through the column and row kernels.
__global__ void __launch_bounds__(mf::kT, 1)
k_mf_tensor(uint32_t* __restrict__ d0, uint32_t* __restrict__ d1, uint32_t* __restrict__ d2, uint64_t ols,
            const uint32_t* __restrict__ c0, const uint32_t* __restrict__ c1, const uint32_t* __restrict__ c0p,
            const uint32_t* __restrict__ c1p, uint64_t ils, uint32_t* __restrict__ scratch, uint32_t slots,
            const void* __restrict__ mft, const LimbConst<uint32_t>* __restrict__ lcs,
            uint32_t* __restrict__ d2hat) {
  using namespace mf;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  uint32_t* lds = (uint32_t*)smem_raw;
  const Th h(threadIdx.x);
  const uint32_t poly = blockIdx.x, l = blockIdx.y;
  const uint64_t oo = (uint64_t)l * ols + (uint64_t)poly * kN, io = (uint64_t)l * ils + (uint64_t)poly * kN;
  const LimbConst<uint32_t> lc = lcs[l];
  const Tabs T = tabs_of(mft, lc, l);
  const uint32_t q = lc.q, nqi = T.m.nqinv;
  uint64_t so;
  if (slots) {
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u;          // hwreg(HW_REG_XCC_ID)
    const uint32_t cu = (__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 8) & 0xffu;  // hwreg(HW_REG_HW_ID)[15:8]
    so = (uint64_t)((xcc << 8) | cu) << 16;
  } else {
    so = (uint64_t)(poly + l * gridDim.x) << 16;
  }
  const Rsrc R0 = rsrc(d0 + oo, kN * 4u), R1 = rsrc(d1 + oo, kN * 4u), R2 = rsrc(d2 + oo, kN * 4u);
  const Rsrc RS = rsrc(scratch + so, kN * 4u);
  // the exact d2^ (c1^ c1'^, canonical, device order): the key-switch's
  // diagonal source row (k_ks_rows), when asked for
  const bool want_hat = d2hat != nullptr;
  const Rsrc RH = rsrc(want_hat ? d2hat + oo : d2 + oo, kN * 4u);
  // The lane offset is computed once per kernel, and the epilogues'
  // products are plain C++.
  const uint32_t pl = p4_lane(h);
  auto canon4 = [q](const int32_t (&r)[4]) {
    return v4i{(int)canon(r[0], (int32_t)q), (int)canon(r[1], (int32_t)q), (int)canon(r[2], (int32_t)q),
               (int)canon(r[3], (int32_t)q)};
  };
  auto mmul = [q, nqi](uint32_t a, uint32_t b) {  // a b 2^-32 mod q, canonical
    const uint64_t t = (uint64_t)a * b;
    const uint32_t mm = (uint32_t)t * nqi;
    const uint32_t r = (uint32_t)((t + (uint64_t)mm * q) >> 32);
    return r >= q ? r - q : r;
  };
  const uint32_t rm = lc.rmod, rmp = lc.rmod_p;
  uint32_t x[64];
  // each forward's LDS exchange is fenced by a barrier right after its own
  // last exchange read (SYNCX: the waves are together there) rather than
  // before the next forward's first write (SYNC1, after a drift of three
  // passes); RNT_MF_TENSOR_SYNCX=0 keeps the latter
  constexpr bool SX = RNT_MF_TENSOR_SYNCX != 0;
  // RNT_MF_TENSOR_PARK: P2 chunks parked past SYNCX in [128 KiB, 160 KiB),
  // which the exchanges (the lower 128 KiB) leave free: spills 128 -> 88
  // bytes a lane, the kernel flat to -0.6% (profiles/r05/ab_mf_tensor_syncx.txt),
  // off by default
  constexpr int NP = SX ? RNT_MF_TENSOR_PARK : 0;
  constexpr uint32_t PB = 128u * 1024u, PS = 2048u;
  // RNT_MF_TENSOR_MEAS (measurement builds only, wrong results by design;
  // profiles/r06/tensor_traffic.json): 1 drops c1^'s round trip through the
  // scratch slot (its store and both reads), 2 drops t's (its store into
  // d2's plane and its read), 3 drops c0^'s (its store into d1's plane and
  // both reads); the PMC bytes each build saves say whether that temporary
  // leaves the L2
  constexpr int MEAS = RNT_MF_TENSOR_MEAS;
  fwd<false, S_F4, false, SX, NP, PB, PS>(x, rsrc(c0 + io, kN * 4u), lds, h, T, [&](int cc, const int32_t (&r)[4], uint32_t (&)[64]) {
    if constexpr (MEAS != 3) bst(canon4(r), R1, pl, p4_soff(h, cc));
  });
  fwd<!SX, S_F4, false, SX, NP, PB, PS>(x, rsrc(c1 + io, kN * 4u), lds, h, T, [&](int cc, const int32_t (&r)[4], uint32_t (&)[64]) {
    if constexpr (MEAS != 1) bst(canon4(r), RS, pl, p4_soff(h, cc));
  });
  fwd<!SX, S_F4, false, SX, NP, PB, PS>(x, rsrc(c0p + io, kN * 4u), lds, h, T, [&](int cc, const int32_t (&r)[4], uint32_t (&)[64]) {
    const v4i a0 = MEAS == 3 ? canon4(r) : bld(R1, pl, p4_soff(h, cc));
    const v4i a1 = MEAS == 1 ? canon4(r) : bld(RS, pl, p4_soff(h, cc));
    const v4i b = canon4(r);
    v4i o0, t;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o0[i] = (int)mmul((uint32_t)a0[i], (uint32_t)b[i]);
      t[i] = (int)mmul((uint32_t)a1[i], (uint32_t)b[i]);
    }
    bst<kLastAux>(o0, R0, pl, p4_soff(h, cc));
    if constexpr (MEAS != 2) bst(t, R2, pl, p4_soff(h, cc));
  });
  fwd<!SX, S_F4, false, RNT_MF_TENSOR_PARK4 && SX, RNT_MF_TENSOR_PARK4 ? NP : 0, PB, PS>(x, rsrc(c1p + io, kN * 4u), lds, h, T, [&](int cc, const int32_t (&r)[4], uint32_t (&xx)[64]) {
    const v4i b = canon4(r);
    const v4i a0 = MEAS == 3 ? b : bld<kLastAux>(R1, pl, p4_soff(h, cc));
    const v4i a1 = MEAS == 1 ? b : bld<kLastAux>(RS, pl, p4_soff(h, cc));
    const v4i t = MEAS == 2 ? b : bld<kLastAux>(R2, pl, p4_soff(h, cc));
    v4i o1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t s = (uint32_t)t[i] + mmul((uint32_t)a0[i], (uint32_t)b[i]);
      o1[i] = (int)(s >= q ? s - q : s);
      // c1^ c1'^ 2^-32, times 2^32 (Shoup by 2^32 mod q): the exact product
      const uint32_t m = mmul((uint32_t)a1[i], (uint32_t)b[i]);
      const uint32_t qh = (uint32_t)(((uint64_t)m * rmp) >> 32);
      const uint32_t v = m * rm - qh * q;
      xx[p3(cc, i)] = v >= q ? v - q : v;
    }
    pin4(xx[p3(cc, 0)], xx[p3(cc, 1)], xx[p3(cc, 2)], xx[p3(cc, 3)]);  // (as in k_mf_mul)
    bst<kLastAux>(o1, R1, pl, p4_soff(h, cc));
    if (want_hat)
      bst<kLastAux>(v4i{(int)xx[p3(cc, 0)], (int)xx[p3(cc, 1)], (int)xx[p3(cc, 2)], (int)xx[p3(cc, 3)]}, RH, pl,
                    p4_soff(h, cc));
  });
  inv_x<false>(x, R2, lds, h, T);
}

// RNT_MF_MUL_Q4: fwd(b) exchanges in quarter-plane rounds, and six a^
// tiles a wave stay in the LDS above 64 KiB (else two above 128 KiB)
#ifndef RNT_MF_MUL_Q4
#define RNT_MF_MUL_Q4 1
#endif
#ifndef RNT_MF_MUL_NOSYNC1
#define RNT_MF_MUL_NOSYNC1 1
#endif
// RNT_MF_MUL_PARK: P2 chunks parked in the LDS over pass 1's second half
// (fwd(a): in the wave's own a^ tile area, not yet written; fwd(b): in its
// 4 KiB of the quarter-round region, behind a SYNCX barrier)
#ifndef RNT_MF_MUL_PARK
#define RNT_MF_MUL_PARK 4
#endif
// RNT_MF_MUL_MEAS (measurement build only, wrong results by design): the
// a^ tiles that go through memory are neither stored nor read back -- the
// rate a design keeping all of a^ on the CU could reach at best
#ifndef RNT_MF_MUL_MEAS
#define RNT_MF_MUL_MEAS 0
#endif
// RNT_MF_SLOT_ST_AUX: cache-policy bits of k_mf_mul's a^ slot stores (0:
// default; 2: nt; 16: sc1, which drops the line from the L2 -- the slot is
// read back from HBM in any case, profiles/r06/ab_mf_mul_slot_skip.txt)
#ifndef RNT_MF_SLOT_ST_AUX
#define RNT_MF_SLOT_ST_AUX 0
#endif
// RNT_MF_MUL_MEAS_SKIP: the same for the first SKIP slot tiles only (the
// slot's footprint per XCD shrinks from 32 x 160 KiB: does the rest then stay
// in the L2?)
#ifndef RNT_MF_MUL_MEAS_SKIP
#define RNT_MF_MUL_MEAS_SKIP (RNT_MF_MUL_MEAS ? 16 - kMulLdsTiles : 0)
#endif
// RNT_MF_MUL_V2: rnt_mul at 2^16 runs k_mf_mul2 (512 threads, two virtual
// waves a wave) instead of k_mf_mul.  Off: bit-identical, but two waves a
// SIMD measured 11% slower at the same power (7.08 against 6.27 ms, the clock
// 17% higher: issue-bound, not power-bound), and the registers it frees hold
// about one a^ tile a virtual wave (+1.5%), not the ten that cost k_mf_mul
// 7.8% (profiles/r06/ab_mf_mul2.txt, ab_mf_mul_ahat_ceiling.txt)
#ifndef RNT_MF_MUL_V2
#define RNT_MF_MUL_V2 0
#endif
constexpr int kMulLdsTiles = RNT_MF_MUL_Q4 ? 6 : 2;  // a^ tiles per wave kept in the LDS (k_mf_mul)
constexpr uint32_t kMulLdsBase = RNT_MF_MUL_Q4 ? (1u << 14) : (1u << 15);  // words
static_assert(kMulLdsBase * 4 + (size_t)kMulLdsTiles * 16 * 1024 <= mf::kLdsBytes, "in the LDS");
// The coefficient-domain product c = a b at N = 2^16 (rnt_mul, poly.rs:307-329)
// on the matrix-core transforms, one workgroup per (poly, limb): fwd a -> a^
// into the CU's scratch slot (k_mf_tensor's indexing); fwd b, whose last
// pass multiplies each tile by a^ (read back by the same thread) and keeps
// the exact product in registers; the inverse from there stores c.  c may
// be a or b: every wave has read its words of both before the exchange
// barriers that precede the inverse's stores.
__global__ void __launch_bounds__(mf::kT, 1)
k_mf_mul(uint32_t* c, const uint32_t* a, const uint32_t* b, uint64_t ls, uint32_t* __restrict__ scratch,
         uint32_t slots, const void* __restrict__ mft, const LimbConst<uint32_t>* __restrict__ lcs) {
  using namespace mf;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  uint32_t* lds = (uint32_t*)smem_raw;
  const Th h(threadIdx.x);
  const uint32_t poly = blockIdx.x, l = blockIdx.y;
  const uint64_t o = (uint64_t)l * ls + (uint64_t)poly * kN;
  const LimbConst<uint32_t> lc = lcs[l];
  const Tabs T = tabs_of(mft, lc, l);
  uint64_t so;
  if (slots) {
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u;          // hwreg(HW_REG_XCC_ID)
    const uint32_t cu = (__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 8) & 0xffu;  // hwreg(HW_REG_HW_ID)[15:8]
    so = (uint64_t)((xcc << 8) | cu) << 16;
  } else {
    so = (uint64_t)(poly + l * gridDim.x) << 16;
  }
  const Rsrc RS = rsrc(scratch + so, kN * 4u);
  uint32_t x[64];
  // a^ 2^32: fwd(a)'s last pass runs on F4 2^32 (slot S_F4S)
  // the signed representatives (|r| < q) go to the slot as they are; the
  // last kMulLdsTiles tiles of each wave stay in the LDS past the exchange
  // region (free until the inverse's stash), 1 KiB a tile per wave
  // (recomputed where used from the opaque thread index, as is the lane
  // offset p4_lane: kept live across the passes they cost 16-byte spills)
  auto hat = [&](int t) -> v4i& { return ((v4i*)(lds + kMulLdsBase) + h.w * (kMulLdsTiles * 64) + h.lam())[t * 64]; };
  // (with Q4 the tiles overlap fwd(a)'s exchange region: SYNCX holds every
  // wave's last pass until all have read their last exchange words)
  constexpr int NP = RNT_MF_MUL_Q4 ? RNT_MF_MUL_PARK : 0;
  fwd<false, S_F4S, false, RNT_MF_MUL_Q4 != 0, NP, kMulLdsBase * 4, kMulLdsTiles * 1024>(x, rsrc(a + o, kN * 4u), lds, h, T, [&](int cc, const int32_t (&r)[4], uint32_t (&)[64]) {
    if (cc >= 16 - kMulLdsTiles)
      hat(cc - (16 - kMulLdsTiles)) = v4i{r[0], r[1], r[2], r[3]};
    else if (cc >= RNT_MF_MUL_MEAS_SKIP)
      bst<RNT_MF_SLOT_ST_AUX>(v4i{r[0], r[1], r[2], r[3]}, RS, p4_lane(h), p4_soff(h, cc));
  });
  // fwd(b) needs no barrier before its first exchange write with Q4: every
  // wave passed fwd(a)'s SYNCX after its last read of fwd(a)'s exchange,
  // and fwd(b)'s quarter rounds stay below the a^ tiles
  fwd<!(RNT_MF_MUL_Q4 && RNT_MF_MUL_NOSYNC1), S_F4, RNT_MF_MUL_Q4 != 0, (NP > 0), NP, 0, 4096>(x, rsrc(b + o, kN * 4u), lds, h, T, [&](int cc, const int32_t (&r)[4], uint32_t (&xx)[64]) {
    const v4i ah = cc >= 16 - kMulLdsTiles ? hat(cc - (16 - kMulLdsTiles))
                   : cc < RNT_MF_MUL_MEAS_SKIP ? v4i{r[0], r[1], r[2], r[3]} : bld(RS, p4_lane(h), p4_soff(h, cc));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // (a^ 2^32) b^ 2^-32, a signed Montgomery product of two pass
      // outputs (|a^|, |b^| < q/2 + 2^14, so |v| < 5q/8 + 1, inside the
      // packed range; mont() and mf_build): the exact product, in the
      // packed signed form the inverse's first pass takes as it is
      // (inv_x<false, true>)
      xx[p3(cc, i)] = (uint32_t)mont<true>(ah[i], r[i], T.m) ^ K32;
    }
    // computed here: left free, hipcc sinks each reduction to the inverse's
    // first use of the word and keeps its 64-bit partial live (232 bytes a
    // lane of spills)
    pin4(xx[p3(cc, 0)], xx[p3(cc, 1)], xx[p3(cc, 2)], xx[p3(cc, 3)]);
  });
  inv_x<false, true>(x, rsrc(c + o, kN * 4u), lds, h, T);
}

// RNT_MF_MUL2_REG: a^ tiles a virtual wave keeps in registers (k_mf_mul2):
// tiles 10 - REG .. 9 (10 .. 15 stay in the LDS as in k_mf_mul; the first
// 10 - REG go through the scratch slot)
#ifndef RNT_MF_MUL2_REG
#define RNT_MF_MUL2_REG 6
#endif
#ifndef RNT_MF_MUL2_PARK
#define RNT_MF_MUL2_PARK 0
#endif
// k_mf_mul with 512 threads, each wave the two virtual waves 2p, 2p + 1 of
// k_mf_mul's sixteen-wave layout (mf::fwd2 / inv2): the same plane
// positions, LDS layout, tables and scratch slot indexing, so the same words
// out; RNT_MF_MUL2_REG of the ten a^ tiles a virtual wave sent through the
// scratch slot stay in registers instead.
__global__ void __launch_bounds__(mf::kT / 2, 1)
k_mf_mul2(uint32_t* c, const uint32_t* a, const uint32_t* b, uint64_t ls, uint32_t* __restrict__ scratch,
          uint32_t slots, const void* __restrict__ mft, const LimbConst<uint32_t>* __restrict__ lcs) {
  using namespace mf;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  uint32_t* lds = (uint32_t*)smem_raw;
  // virtual thread ids: wave p's lane l is thread 128p + l of wave 2p and
  // 128p + 64 + l of wave 2p + 1
  const uint32_t tv = 2u * threadIdx.x - (threadIdx.x & 63u);
  const Th ha(tv), hb(tv + 64u);
  const uint32_t poly = blockIdx.x, l = blockIdx.y;
  const uint64_t o = (uint64_t)l * ls + (uint64_t)poly * kN;
  const LimbConst<uint32_t> lc = lcs[l];
  const Tabs T = tabs_of(mft, lc, l);
  uint64_t so;
  if (slots) {
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u;          // hwreg(HW_REG_XCC_ID)
    const uint32_t cu = (__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 8) & 0xffu;  // hwreg(HW_REG_HW_ID)[15:8]
    so = (uint64_t)((xcc << 8) | cu) << 16;
  } else {
    so = (uint64_t)(poly + l * gridDim.x) << 16;
  }
  const Rsrc RS = rsrc(scratch + so, kN * 4u);
  constexpr int R = RNT_MF_MUL2_REG;
  static_assert(R >= 0 && R <= 16 - kMulLdsTiles, "a^ register tiles");
  constexpr int MEM = 16 - kMulLdsTiles - R;  // tiles 0 .. MEM-1 through the slot
  v4i ra[R > 0 ? R : 1], rbv[R > 0 ? R : 1];
  auto hat = [&](const Th& h, int t) -> v4i& {
    return ((v4i*)(lds + kMulLdsBase) + h.w * (kMulLdsTiles * 64) + h.lam())[t * 64];
  };
  uint32_t xa[64], xb[64];
  auto put = [&](const Th& h, v4i (&reg)[R > 0 ? R : 1], int cc, const int32_t (&r)[4]) {
    const v4i v = {r[0], r[1], r[2], r[3]};
    if (cc >= 16 - kMulLdsTiles)
      hat(h, cc - (16 - kMulLdsTiles)) = v;
    else if (cc >= MEM)
      reg[cc - MEM] = v;
    else
      bst(v, RS, p4_lane(h), p4_soff(h, cc));
  };
  constexpr int NP = RNT_MF_MUL2_PARK;
  fwd2<false, S_F4S, false, true, NP, kMulLdsBase * 4, kMulLdsTiles * 1024>(
      xa, xb, rsrc(a + o, kN * 4u), lds, ha, hb, T,
      [&](int cc, const int32_t (&r)[4], uint32_t (&)[64]) { put(ha, ra, cc, r); },
      [&](int cc, const int32_t (&r)[4], uint32_t (&)[64]) { put(hb, rbv, cc, r); });
  auto mul = [&](const Th& h, v4i (&reg)[R > 0 ? R : 1], int cc, const int32_t (&r)[4], uint32_t (&xx)[64]) {
    const v4i ah = cc >= 16 - kMulLdsTiles ? hat(h, cc - (16 - kMulLdsTiles))
                   : cc >= MEM             ? reg[cc - MEM]
                                           : bld(RS, p4_lane(h), p4_soff(h, cc));
#pragma unroll
    for (int i = 0; i < 4; ++i) xx[p3(cc, i)] = (uint32_t)mont<true>(ah[i], r[i], T.m) ^ K32;  // (as k_mf_mul)
    pin4(xx[p3(cc, 0)], xx[p3(cc, 1)], xx[p3(cc, 2)], xx[p3(cc, 3)]);
  };
  fwd2<false, S_F4, true, (NP > 0), NP, 0, 4096>(
      xa, xb, rsrc(b + o, kN * 4u), lds, ha, hb, T,
      [&](int cc, const int32_t (&r)[4], uint32_t (&xx)[64]) { mul(ha, ra, cc, r, xx); },
      [&](int cc, const int32_t (&r)[4], uint32_t (&xx)[64]) { mul(hb, rbv, cc, r, xx); });
  inv2(xa, xb, rsrc(c + o, kN * 4u), lds, ha, hb, T);
}

// ---------------------------------------------------------------------------
// host: the per-limb table
// ---------------------------------------------------------------------------
namespace {
using host::brv;
using host::invmod;
using host::mulmod;
using host::powmod;

int32_t centred(uint64_t v, uint64_t q) {
  v %= q;
  return v > q / 2 ? (int32_t)((int64_t)v - (int64_t)q) : (int32_t)v;
}

// W[out][in] (mod q) as MFMA operand bytes of digit planes a = 0..3 for the
// 64 lanes (4 words each): E[o][k][b] = centred(W[o][k] 2^(8b) 2^32), its
// balanced byte digits.  DA: the matrix is the B operand (lane 16 g + col,
// output col); else the A operand (lane 16 g + row, output kappa(row >> 2,
// row & 3)).  kappa(g, i) = 4i + g (KAP 0) or 4g + i (KAP 1): the group
// index of the data in lane group g, register i.
void expand(const uint64_t (&W)[16][16], uint64_t q, uint64_t R, bool DA, int KAP, int32_t* out) {
  int32_t E[16][16][4];
  for (int o = 0; o < 16; ++o)
    for (int k = 0; k < 16; ++k)
      for (int b = 0; b < 4; ++b) E[o][k][b] = centred(mulmod(mulmod(W[o][k], (1ull << (8 * b)) % q, q), R, q), q);
  for (int a = 0; a < 4; ++a)
    for (int lam = 0; lam < 64; ++lam)
      for (int i = 0; i < 4; ++i) {
        const int g = lam >> 4, r = lam & 15;
        const int kin = KAP ? 4 * g + i : 4 * i + g;
        const int jout = DA ? r : (KAP ? r : 4 * (r & 3) + (r >> 2));
        uint32_t wd = 0;
        for (int b = 0; b < 4; ++b) {
          const uint32_t u = (uint32_t)E[jout][kin][b] + 0x80808080u;
          wd |= ((((u >> (8 * a)) & 0xFFu) ^ 0x80u) & 0xFFu) << (8 * b);
        }
        out[(a * 64 + lam) * 4 + i] = (int32_t)wd;
      }
}

}  // namespace

// Builds the MFMA tables of every limb (u32 bases at N = 2^16) into t->mf.
int mf_build(Tables* t, std::string* err) {
  using namespace mf;
  const size_t L = t->L;
  const uint64_t n = kN;
  std::vector<int32_t> all((size_t)L * kLimb * 4);
  std::vector<uint64_t> tw(n), itw(n), pw(n), ipw(n);
  for (size_t l = 0; l < L; ++l) {
    const uint64_t q = t->moduli[l], psi = t->psi[l], psinv = invmod(psi, q);
    uint64_t x = 1, y = 1;
    for (uint64_t j = 0; j < n; ++j) {
      pw[j] = x;
      ipw[j] = y;
      x = mulmod(x, psi, q);
      y = mulmod(y, psinv, q);
    }
    for (uint64_t g = 0; g < n; ++g) {
      tw[g] = pw[brv(g, 16)];
      itw[g] = ipw[brv(g, 16)];
    }
    const uint64_t R = (uint64_t)(((host::u128)1 << 32) % q);
    // k_mf_mul hands its product to the inverse in the packed byte form:
    // with pass outputs |r| < q/2 + 2^14 the Montgomery product's bound
    // (q/2 + 2^14)^2 / 2^32 + q/2 + 1 must stay inside [-0x80808080,
    // 0x7F7F7F7F] (mont(); holds for every q < 2^31)
    {
      const double rb = (double)q / 2 + 16384.0;
      if (rb * rb / 4294967296.0 + (double)q / 2 + 1 >= (double)0x7F7F7F7Fu) {
        *err = "MFMA tables: the product bound exceeds the packed digit range for this prime";
        return -1;
      }
    }
    // pass 0's matrix by running its four CT stages on unit vectors
    uint64_t M0[16][16];
    for (int k = 0; k < 16; ++k) {
      uint64_t v[16] = {};
      v[k] = 1;
      for (int sb = 3; sb >= 0; --sb) {
        const int b = 12 + sb;
        for (int kk = 0; kk < 16; ++kk) {
          if (kk & (1 << sb)) continue;
          const uint64_t i = (uint64_t)kk << 12;
          const uint64_t w = tw[(n + i) >> (b + 1)];
          const uint64_t x = v[kk], y = v[kk | (1 << sb)];
          const uint64_t tt = mulmod(w, y, q);
          v[kk] = (x + tt) % q;
          v[kk | (1 << sb)] = (x + q - tt) % q;
        }
      }
      for (int j = 0; j < 16; ++j) M0[j][k] = v[j];
    }
    const uint64_t beta1i = itw[8];
    uint64_t F[16][16], Fi[16][16];
    const uint64_t inv16 = invmod(16 % q, q);
    for (int j = 0; j < 16; ++j)
      for (int k = 0; k < 16; ++k) F[j][k] = mulmod(M0[j][k], powmod(beta1i, (uint64_t)k, q), q);
    for (int j = 0; j < 16; ++j)
      for (int k = 0; k < 16; ++k) Fi[k][j] = mulmod(inv16, invmod(F[j][k], q), q);
    // F Fi == I (F is a DFT on the 16 roots of unity; checked, not assumed)
    for (int j = 0; j < 16; ++j)
      for (int k = 0; k < 16; ++k) {
        uint64_t s = 0;
        for (int x = 0; x < 16; ++x) s = (s + mulmod(F[j][x], Fi[x][k], q)) % q;
        if (s != (j == k ? 1u : 0u)) {
          *err = "MFMA tables: F is not invertible as a DFT";
          return -1;
        }
      }
    int32_t* lt = all.data() + l * (size_t)kLimb * 4;
    auto slot = [&](int s) { return lt + (size_t)(kMat + s * 4 * 64) * 4; };
    uint64_t W[16][16];
    expand(M0, q, R, false, 0, slot(S_F1));
    for (int U = 0; U < 16; ++U) {
      const uint64_t be = tw[128 + 8 * U], bei = itw[128 + 8 * U];
      for (int j = 0; j < 16; ++j)
        for (int k = 0; k < 16; ++k) W[j][k] = mulmod(F[j][k], powmod(be, (uint64_t)k, q), q);
      expand(W, q, R, false, 0, slot(S_F2 + U));
      for (int k = 0; k < 16; ++k)
        for (int j = 0; j < 16; ++j) W[k][j] = mulmod(powmod(bei, (uint64_t)k, q), Fi[k][j], q);
      expand(W, q, R, false, 0, slot(S_I2 + U));
    }
    expand(F, q, R, true, 0, slot(S_F3));
    expand(F, q, R, false, 1, slot(S_F4));
    for (int j = 0; j < 16; ++j)
      for (int k = 0; k < 16; ++k) W[j][k] = mulmod(F[j][k], R, q);
    expand(W, q, R, false, 1, slot(S_F4S));
    expand(Fi, q, R, true, 1, slot(S_I4));
    expand(Fi, q, R, false, 1, slot(S_I3));
    for (int k = 0; k < 16; ++k)
      for (int j = 0; j < 16; ++j) W[k][j] = mulmod(powmod(beta1i, (uint64_t)k, q), Fi[k][j], q);
    expand(W, q, R, false, 0, slot(S_I1));
    // input-bias compensations: the data digits carry x - 2^30
    const uint64_t bias = mulmod(R, (1ull << 30) % q, q);
    {
      int32_t cf[16], ci[16];
      for (int j = 0; j < 16; ++j) {
        uint64_t s0 = 0, s1 = 0;
        for (int k = 0; k < 16; ++k) {
          s0 = (s0 + M0[j][k]) % q;
          s1 = (s1 + Fi[j][k]) % q;
        }
        cf[j] = centred(mulmod(bias, s0, q), q);
        ci[j] = centred(mulmod(bias, s1, q), q);
      }
      int32_t* c1 = lt + (size_t)kCompF1 * 4;
      int32_t* c4 = lt + (size_t)kCompI4 * 4;
      for (int lam = 0; lam < 64; ++lam)
        for (int i = 0; i < 4; ++i) {
          c1[lam * 4 + i] = cf[4 * i + (lam >> 4)];
          c4[lam * 4 + i] = ci[lam & 15];
        }
    }
    // twists (Montgomery form, centred)
    auto mr = [&](uint64_t v) { return centred(mulmod(v, R, q), q); };
    int32_t* t3f = lt + (size_t)kTw3f * 4;
    int32_t* t3i = lt + (size_t)kTw3i * 4;
    for (int w = 0; w < 16; ++w)
      for (int g = 0; g < 4; ++g)
        for (int c = 0; c < 16; ++c)
          for (int i = 0; i < 4; ++i) {
            const int U3 = (w << 4) | (i << 2) | g;
            t3f[((w * 4 + g) * 16 + c) * 4 + i] = mr(powmod(tw[2048 + 8 * U3], (uint64_t)c, q));
          }
    for (int w = 0; w < 16; ++w)
      for (int c = 0; c < 16; ++c)
        for (int g = 0; g < 4; ++g)
          for (int i = 0; i < 4; ++i) {
            const int U3 = (w << 4) | c;
            t3i[((w * 16 + c) * 4 + g) * 4 + i] = mr(powmod(itw[2048 + 8 * U3], (uint64_t)(4 * g + i), q));
          }
    int32_t* t4f = lt + (size_t)kTw4f * 4;
    int32_t* t4i = lt + (size_t)kTw4i * 4;
    for (int w = 0; w < 16; ++w)
      for (int c = 0; c < 16; ++c)
        for (int lam = 0; lam < 64; ++lam)
          for (int i = 0; i < 4; ++i) {
            const int g = lam >> 4, nn = lam & 15;
            const int Uf = (w << 8) | (c << 4) | nn;
            t4f[((w * 16 + c) * 64 + lam) * 4 + i] = mr(powmod(tw[32768 + 8 * Uf], (uint64_t)(4 * g + i), q));
            const int Ui = (w << 8) | (c << 4) | (4 * g + i);
            t4i[((w * 16 + c) * 64 + lam) * 4 + i] = mr(powmod(itw[32768 + 8 * Ui], (uint64_t)nn, q));
          }
  }
  // t->mf is set only once the tables are on the device: a failed build
  // leaves no half-built table behind
  const size_t bytes = all.size() * sizeof(int32_t);
  void* dev = nullptr;
  if (hipError_t e = hipMalloc(&dev, bytes); e != hipSuccess) {
    *err = std::string("hipMalloc(MFMA tables): ") + hipGetErrorString(e);
    return -3;
  }
  if (hipError_t e = hipMemcpy(dev, all.data(), bytes, hipMemcpyHostToDevice); e != hipSuccess) {
    (void)hipFree(dev);
    *err = std::string("hipMemcpy(MFMA tables): ") + hipGetErrorString(e);
    return -2;
  }
  t->mf = dev;
  return 0;
}

static hipError_t launch_ntt_t(const Launch& k, const void* fn, void* data, uint64_t ls) {
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mf::kLdsBytes);
  if (e != hipSuccess) return e;
  uint32_t* d = (uint32_t*)data;
  const void* mft = k.t->mf;
  const LimbConst<uint32_t>* lcs = (const LimbConst<uint32_t>*)k.t->lconst;
  void* args[] = {&d, &mft, &lcs, &ls};
  return hipLaunchKernel(fn, dim3((unsigned)k.B, (unsigned)k.L), dim3(mf::kT), args, mf::kLdsBytes, k.s);
}

hipError_t launch_mf_tensor(const Launch& k, void* d0, void* d1, void* d2, uint64_t ols, const void* c0,
                            const void* c1, const void* c0p, const void* c1p, uint64_t ils, void* scratch) {
  if (k.B == 0 || k.L == 0) return hipSuccess;
  if (k.B > 0x7fffffffull || k.L > 65535) return hipErrorInvalidConfiguration;
  const void* fn = (const void*)k_mf_tensor;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mf::kLdsBytes);
  if (e != hipSuccess) return e;
  uint32_t slots = (uint64_t)k.B * k.L >= kPlaneSlots ? 1u : 0u;  // plane_scratch_planes
  const void* mft = k.t->mf;
  const LimbConst<uint32_t>* lcs = (const LimbConst<uint32_t>*)k.t->lconst;
  void* d2hat = k.d2hat;  // the exact d2^ for the key-switch's diagonal (its stride is ols)
  void* args[] = {&d0, &d1, &d2, &ols, &c0, &c1, &c0p, &c1p, &ils, &scratch, &slots, &mft, &lcs, &d2hat};
  return hipLaunchKernel(fn, dim3((unsigned)k.B, (unsigned)k.L), dim3(mf::kT), args, mf::kLdsBytes, k.s);
}

hipError_t launch_mf_mul(const Launch& k, void* c, const void* a, const void* b, uint64_t ls, void* scratch) {
  if (k.B == 0 || k.L == 0) return hipSuccess;
  if (k.B > 0x7fffffffull || k.L > 65535) return hipErrorInvalidConfiguration;
  const void* fn = RNT_MF_MUL_V2 ? (const void*)k_mf_mul2 : (const void*)k_mf_mul;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mf::kLdsBytes);
  if (e != hipSuccess) return e;
  uint32_t slots = (uint64_t)k.B * k.L >= kPlaneSlots ? 1u : 0u;  // plane_scratch_planes
  const void* mft = k.t->mf;
  const LimbConst<uint32_t>* lcs = (const LimbConst<uint32_t>*)k.t->lconst;
  void* args[] = {&c, &a, &b, &ls, &scratch, &slots, &mft, &lcs};
  return hipLaunchKernel(fn, dim3((unsigned)k.B, (unsigned)k.L), dim3(RNT_MF_MUL_V2 ? mf::kT / 2 : mf::kT), args,
                         mf::kLdsBytes, k.s);
}

#ifdef RNT_MF_TRACE
extern "C" __attribute__((visibility("default"))) int rnt_debug_mf_trace(uint64_t* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mf_trace), sizeof(g_mf_trace));
}
#endif

hipError_t launch_mf_ntt(const Launch& k, int inverse, void* data, uint64_t ls) {
  if (k.B == 0 || k.L == 0) return hipSuccess;
  if (k.B > 0x7fffffffull || k.L > 65535) return hipErrorInvalidConfiguration;
  return inverse ? launch_ntt_t(k, (const void*)k_mf_ntt<true>, data, ls)
                 : launch_ntt_t(k, (const void*)k_mf_ntt<false>, data, ls);
}

}  // namespace rnt
