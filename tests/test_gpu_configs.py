"""BASELINE configs 4 and 5 at their real ring sizes, bit-exact against the
oracle (VERDICT r01 "what's weak" #1).

* Config 4 (N=2^16, 16 x 31-bit primes): mul_ciphertexts_gadget
  (engine.rs:473-539) + rescale_ciphertext (engine.rs:263-282) on a batch of
  66 ciphertext pairs.  With the key-switch workspace cap set to 4 GiB of S
  (RNT_KS_WS_MB=4096; S = [L][L][Bc][N] words, rnt_api.cpp ks_chunk; the
  default 16 GiB gives 256) the chunks are 64, so the
  batch runs as two chunks, [0, 64) and [64, 66); the checked pairs sit on
  both sides of the boundary and at the end.  The decomposition's target
  limb groups (auto: 16 for the first chunk, 2 for the 8-tile second) are
  both exercised.
* Config 5 (N=2^17, 32 x 31-bit primes): rotate_ciphertext (engine.rs:412-463)
  of one ciphertext for k = 1, -3, 2^15 over all 32 limbs.
* Edge operands on the metric's 31-bit path at N=2^16: all-(q-1), zero and
  monomial operands (one bit of headroom: 2q < 2^32 < 3q).
* Explicit decomposition groups (RNT_DEC_JG, read at rnt_ctx_create): 3 (a
  partial last group) and 16, for mul_ciphertexts_gadget and for
  rnt_keyswitch_ext with 5 target limbs over 8 source limbs.

The oracle runs channel-parallel (oracle.c or_*_mt: the reference's
per-channel arithmetic on host threads) so a full-size check takes seconds.
"""
from __future__ import annotations

import numpy as np
import pytest

import pyoracle as orc

pytestmark = pytest.mark.gpu

T = orc.host_threads()


def _rand(rng, mod, n, batch):
    return orc.uniform_poly(mod, n, rng, batch=batch)


def _ct_batch(rng, mod, n, B, distinct_at):
    """[B][L][N] batch: a few distinct polys placed at `distinct_at`, the rest
    tiled (a chunk-placement bug cannot hide behind equal values at the
    checked positions)."""
    uniq = _rand(rng, mod, n, len(distinct_at) + 1)
    out = np.empty((B, len(mod), n), dtype=np.uint64)
    out[:] = uniq[-1]
    for j, p in enumerate(distinct_at):
        out[p] = uniq[j]
    return out


def test_config4_ct_mul_relin_rescale_two_chunks(gpu, monkeypatch):
    monkeypatch.setenv("RNT_KS_WS_MB", "4096")  # chunks of 64 (read at rnt_ctx_create)
    rn = gpu
    n, L, B = 1 << 16, 16, 66
    mod = rn.generate_primes(31, L, n)
    Bd, Bo = rn.RnsBasis(mod, n), orc.Basis(mod, n)
    rng = np.random.default_rng(404)
    checked = (0, 63, 64, 65)  # first, last of chunk 0; first, last of chunk 1
    c0, c1, c0p, c1p = (_ct_batch(rng, mod, n, B, checked) for _ in range(4))
    ka, kb = _rand(rng, mod, n, L), _rand(rng, mod, n, L)
    rlk = rn.RnsGadgetKey.from_channels(ka, kb, Bd)
    up = lambda x: rn.RnsPoly.from_channels(x, Bd)  # noqa: E731
    ct1 = rn.Ciphertext(up(c0), up(c1), 31, Bd.total_bits())
    ct2 = rn.Ciphertext(up(c0p), up(c1p), 31, Bd.total_bits())
    out = rn.mul_ciphertexts_gadget(ct1, ct2, rlk)
    res = rn.rescale_ciphertext(out)
    o0, o1 = out.c0.channels(), out.c1.channels()
    r0, r1 = res.c0.channels(), res.c1.channels()
    assert res.c0.basis.channel_count() == L - 1 and res.logp == 62 - mod[-1].bit_length()
    for p in checked:
        w0, w1 = orc.mul_ciphertexts_gadget(Bo, c0[p], c1[p], c0p[p], c1p[p], ka, kb, threads=T)
        assert np.array_equal(o0[p], w0) and np.array_equal(o1[p], w1), p
        assert np.array_equal(r0[p], orc.rescale(Bo, w0)), p
        assert np.array_equal(r1[p], orc.rescale(Bo, w1)), p
    # the tiled positions agree with each other (one value per chunk)
    tile = [p for p in range(B) if p not in checked]
    assert np.array_equal(o0[tile[0]], o0[tile[-1]]) and np.array_equal(o1[tile[0]], o1[tile[-1]])


def test_config4_full_1024_ct_batch(gpu):
    """BASELINE config 4 at its stated batch: 1024 ciphertext pairs through
    mul_ciphertexts_gadget (engine.rs:473-539) + rescale_ciphertext
    (engine.rs:263-282) in one call, i.e. 4 key-switch chunks of 256 (the
    default 16 GiB S cap).  The
    operands are drawn on the device (Philox, rnt_sample_uniform: 32 GiB of
    host data otherwise); the chunk-boundary ciphertexts 0, 255, 256 and the
    last, 1023, are read back with their inputs and checked against the
    oracle."""
    rn = gpu
    n, L, B = 1 << 16, 16, 1024
    mod = rn.generate_primes(31, L, n)
    Bd, Bo = rn.RnsBasis(mod, n), orc.Basis(mod, n)
    drng = rn.DeviceRng(1024)
    c0, c1, c0p, c1p = (rn.RnsPoly.sample_uniform(Bd, drng, B) for _ in range(4))
    rng = np.random.default_rng(1025)
    ka, kb = _rand(rng, mod, n, L), _rand(rng, mod, n, L)
    rlk = rn.RnsGadgetKey.from_channels(ka, kb, Bd)
    ct1 = rn.Ciphertext(c0, c1, 31, Bd.total_bits())
    ct2 = rn.Ciphertext(c0p, c1p, 31, Bd.total_bits())
    out = rn.mul_ciphertexts_gadget(ct1, ct2, rlk)
    res = rn.rescale_ciphertext(out)
    assert res.c0.basis.channel_count() == L - 1
    for p in (0, 255, 256, B - 1):
        x0, x1, y0, y1 = (t.channels_of(p)[0] for t in (c0, c1, c0p, c1p))
        w0, w1 = orc.mul_ciphertexts_gadget(Bo, x0, x1, y0, y1, ka, kb, threads=T)
        assert np.array_equal(out.c0.channels_of(p)[0], w0), p
        assert np.array_equal(out.c1.channels_of(p)[0], w1), p
        assert np.array_equal(res.c0.channels_of(p)[0], orc.rescale(Bo, w0)), p
        assert np.array_equal(res.c1.channels_of(p)[0], orc.rescale(Bo, w1)), p


@pytest.mark.parametrize("k", [1, -3, 1 << 15])
def test_config5_rotation_full_32_limbs(gpu, k):
    rn = gpu
    n, L = 1 << 17, 32
    mod = rn.generate_primes(31, L, n)
    Bd, Bo = rn.RnsBasis(mod, n), orc.Basis(mod, n)
    rng = np.random.default_rng(500 + (k & 0xffff))
    c0, c1 = _rand(rng, mod, n, 1)[0], _rand(rng, mod, n, 1)[0]
    ka, kb = _rand(rng, mod, n, L), _rand(rng, mod, n, L)
    rotk = rn.RnsGadgetKey.from_channels(ka, kb, Bd, rotation=k)
    r = rn.rotate_ciphertext(rn.Ciphertext(rn.RnsPoly.from_channels(c0, Bd), rn.RnsPoly.from_channels(c1, Bd)),
                             rotk)
    w0, w1 = orc.rotate_ciphertext(Bo, c0, c1, k, ka, kb, threads=T)
    assert np.array_equal(r.c0.channels(), w0)
    assert np.array_equal(r.c1.channels(), w1)


@pytest.mark.parametrize("plane", [None, "0"])
def test_metric_path_edge_operands(gpu, monkeypatch, plane):
    """All-(q-1), zero and monomial operands through the default 31-bit
    poly-mul (the metric's path: the fused whole-plane kernel), and through
    the four-step kernels (RNT_PLANE=0), against the oracle."""
    if plane is not None:
        monkeypatch.setenv("RNT_PLANE", plane)
    rn = gpu
    n, L = 1 << 16, 16
    mod = rn.generate_primes(31, L, n)
    Bd, Bo = rn.RnsBasis(mod, n), orc.Basis(mod, n)
    q = np.array(mod, dtype=np.uint64)[:, None]
    rng = np.random.default_rng(16)
    full = np.broadcast_to(q - 1, (L, n)).copy()
    zero = np.zeros((L, n), dtype=np.uint64)
    mono = np.zeros((L, n), dtype=np.uint64)
    mono[:, n - 1] = (q - 1)[:, 0]  # -(x^(N-1)): wraps negacyclically
    mono1 = np.zeros((L, n), dtype=np.uint64)
    mono1[:, 1] = 1
    rnd = _rand(rng, mod, n, 1)[0]
    pairs = [(full, full), (full, rnd), (zero, rnd), (mono, full), (mono, mono), (mono1, rnd), (rnd, full)]
    a = rn.RnsPoly.from_channels(np.stack([p[0] for p in pairs]), Bd)
    b = rn.RnsPoly.from_channels(np.stack([p[1] for p in pairs]), Bd)
    got = (a * b).channels()
    for i, (x, y) in enumerate(pairs):
        assert np.array_equal(got[i], orc.mul(Bo, x, y)), i
    # NTT round trip of the extreme operands
    t = a.clone()
    t.to_ntt_domain()
    assert np.array_equal(t.channels()[0], orc.to_ntt(Bo, full))
    t.to_coeff_domain()
    assert np.array_equal(t.channels(), a.channels())


@pytest.mark.parametrize("mf_mul", [None, "0"])
def test_plane_product_matches_oracle(gpu, monkeypatch, mf_mul):
    """rnt_mul through the whole-plane products at N = 2^16 on u32 bases --
    the default matrix-core one (k_mf_mul) and, with RNT_MF_MUL=0, the VALU
    one (k_plane_fused) -- bit-exact against the oracle's poly.rs:307-329
    product on random, all-(q-1), zero and negacyclic-monomial operands, and
    in both in-place forms (out aliasing a, out aliasing b)."""
    monkeypatch.delenv("RNT_PLANE", raising=False)
    if mf_mul is None:
        monkeypatch.delenv("RNT_MF_MUL", raising=False)
    else:
        monkeypatch.setenv("RNT_MF_MUL", mf_mul)
    rn = gpu
    n, L = 1 << 16, 3
    mod = rn.generate_primes(31, L, n)
    Bd, Bo = rn.RnsBasis(mod, n), orc.Basis(mod, n)
    q = np.array(mod, dtype=np.uint64)[:, None]
    rng = np.random.default_rng(65536)
    full = np.broadcast_to(q - 1, (L, n)).copy()
    mono = np.zeros((L, n), dtype=np.uint64)
    mono[:, n - 1] = 1
    r1, r2 = _rand(rng, mod, n, 1)[0], _rand(rng, mod, n, 1)[0]
    pairs = [(r1, r2), (full, full), (full, r1), (np.zeros_like(r1), r2), (mono, mono), (mono, r2)]
    a_h = np.stack([p[0] for p in pairs])
    b_h = np.stack([p[1] for p in pairs])
    a = rn.RnsPoly.from_channels(a_h, Bd)
    b = rn.RnsPoly.from_channels(b_h, Bd)
    got = (a * b).channels()
    for i, (x, y) in enumerate(pairs):
        assert np.array_equal(got[i], orc.mul(Bo, x, y)), i
    a *= b  # out aliases a
    assert np.array_equal(a.channels(), got)
    b2 = rn.RnsPoly.from_channels(b_h, Bd)
    a2 = rn.RnsPoly.from_channels(a_h, Bd)
    from rns_ntt import _lib
    rn.check(rn.load().rnt_mul(b2.handle, a2.handle, b2.handle))  # out aliases b
    assert np.array_equal(b2.channels(), got)


@pytest.mark.parametrize("env", [{}, {"RNT_MF_MUL": "0"}, {"RNT_PLANE": "0"}], ids=["mf_mul", "plane_fused", "four_step"])
def test_metric_batch_1024_sampled_pairs(gpu, monkeypatch, env):
    """The metric's own shape and batch (N = 2^16, L = 16 x 31-bit, 1024
    pairs, operands drawn on the device as in bench.py): eight pairs --
    the first, the last, both sides of the 512 midpoint and four random
    ones -- bit-exact against the oracle's poly.rs:307-329 product, and the
    same batch through the in-place form (a *= b, out aliasing a); the
    default path (k_mf_mul), the VALU whole-plane product (RNT_MF_MUL=0) and
    the four-step kernels (RNT_PLANE=0)."""
    monkeypatch.delenv("RNT_MF_MUL", raising=False)
    monkeypatch.delenv("RNT_PLANE", raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rn = gpu
    n, L, B = 1 << 16, 16, 1024
    mod = rn.generate_primes(31, L, n)
    Bd, Bo = rn.RnsBasis(mod, n), orc.Basis(mod, n)
    drng = rn.DeviceRng(2024)
    a = rn.RnsPoly.sample_uniform(Bd, drng, B)
    b = rn.RnsPoly.sample_uniform(Bd, drng, B)
    c = a * b
    rng = np.random.default_rng(1024)
    picks = sorted({0, B - 1, 511, 512, *rng.integers(1, B - 1, size=4).tolist()})
    a_h = {p: a.channels_of(p)[0] for p in picks}
    b_h = {p: b.channels_of(p)[0] for p in picks}
    for p in picks:
        assert np.array_equal(c.channels_of(p)[0], orc.mul(Bo, a_h[p], b_h[p])), p
    a *= b
    for p in picks[:3]:
        assert np.array_equal(a.channels_of(p)[0], c.channels_of(p)[0]), p


@pytest.mark.parametrize("mf_mul", [None, "0"])
def test_metric_product_full_output_vs_four_step(gpu, monkeypatch, mf_mul):
    """Every word of 128 pairs x 16 limbs (2048 planes: the CU-indexed
    scratch slots) of the whole-plane product -- the default matrix-core one
    (k_mf_mul) and, with RNT_MF_MUL=0, the VALU one (k_plane_fused_slots) --
    against the four-step kernels' (RNT_PLANE=0), on the same device-drawn
    operands and on all-(q-1) operands (the largest sums)."""
    rn = gpu
    n, L, B = 1 << 16, 16, 128
    mod = rn.generate_primes(31, L, n)
    q = np.array(mod, dtype=np.uint64)[:, None]
    if mf_mul is None:
        monkeypatch.delenv("RNT_MF_MUL", raising=False)
    else:
        monkeypatch.setenv("RNT_MF_MUL", mf_mul)
    out = {}
    for plane in (None, "0"):
        if plane is None:
            monkeypatch.delenv("RNT_PLANE", raising=False)
        else:
            monkeypatch.setenv("RNT_PLANE", plane)
        Bd = rn.RnsBasis(mod, n)
        drng = rn.DeviceRng(77)
        a = rn.RnsPoly.sample_uniform(Bd, drng, B)
        b = rn.RnsPoly.sample_uniform(Bd, drng, B)
        out[plane] = (a * b).channels_batch()
        full = rn.RnsPoly.from_channels(np.broadcast_to(q - 1, (2, L, n)), Bd)
        out[(plane, "full")] = (full * full).channels_batch()
        del a, b, full, Bd
    assert int((out[None] != out["0"]).sum()) == 0
    assert np.array_equal(out[(None, "full")], out[("0", "full")])


@pytest.mark.parametrize("jg", [3, 16])
def test_decomposition_groups(gpu, monkeypatch, jg):
    """RNT_DEC_JG fixes the key-switch decomposition's target limbs per
    workgroup; 3 leaves a partial last group at L = 8 and at 5 targets."""
    rn = gpu
    monkeypatch.setenv("RNT_DEC_JG", str(jg))
    n, L, B = 1 << 14, 8, 3
    mod = rn.generate_primes(31, L, n)
    Bd, Bo = rn.RnsBasis(mod, n), orc.Basis(mod, n)
    rng = np.random.default_rng(30 + jg)
    c0, c1, c0p, c1p = (_rand(rng, mod, n, B) for _ in range(4))
    ka, kb = _rand(rng, mod, n, L), _rand(rng, mod, n, L)
    rlk = rn.RnsGadgetKey.from_channels(ka, kb, Bd)
    up = lambda x: rn.RnsPoly.from_channels(x, Bd)  # noqa: E731
    out = rn.mul_ciphertexts_gadget(rn.Ciphertext(up(c0), up(c1)), rn.Ciphertext(up(c0p), up(c1p)), rlk)
    o0, o1 = out.c0.channels(), out.c1.channels()
    for p in (0, B - 1):
        w0, w1 = orc.mul_ciphertexts_gadget(Bo, c0[p], c1[p], c0p[p], c1p[p], ka, kb, threads=T)
        assert np.array_equal(o0[p], w0) and np.array_equal(o1[p], w1), p
    # keyswitch_ext: 5 target limbs (a limb shard) over the 8 source limbs
    Lt = 5
    Bt = rn.RnsBasis(mod[:Lt], n)
    d = up(c1)
    key_t = rn.RnsGadgetKey.from_channels(np.ascontiguousarray(ka[:, :Lt]), np.ascontiguousarray(kb[:, :Lt]), Bt)
    ptr, _ = d.device_ptr()
    a0, a1 = rn.keyswitch_ext(ptr, L, key_t, Bt, B)
    g0, g1 = a0.channels(), a1.channels()
    for p in (0, B - 1):
        w0, w1 = orc.keyswitch(Bo, c1[p], ka, kb, threads=T)
        assert np.array_equal(g0[p], w0[:Lt]) and np.array_equal(g1[p], w1[:Lt]), p


# (log_n, B) -> the grid ks_rows_pick chooses (NP polys x RPW/NP rows per
# workgroup; RPW = 64, 32, 16, 8 rows at N = 2^12, 2^14, 2^16, 2^17): the
# largest NP whose grid fills >= 90% of its row slots, else the best fill.
# NP = 2/4/8 exist for 2^8- and 2^9-word rows (N = 2^16, 2^17) only.
_KS_GRIDS = [(12, 1, 1), (12, 3, 1), (12, 40, 1), (12, 127, 64), (14, 2, 1), (14, 9, 1), (14, 33, 1),
             (14, 63, 32), (16, 1, 1), (16, 2, 2), (16, 5, 1), (16, 8, 8), (16, 12, 4), (16, 16, 16),
             (16, 17, 2), (16, 63, 16), (17, 1, 1), (17, 2, 2), (17, 3, 1), (17, 4, 4), (17, 6, 2),
             (17, 8, 8)]


def _ks_np(log_n, B):
    """Python restatement of ks_rows_pick (rnt_kernels.hip) for the table."""
    rpw = {12: 64, 14: 32, 16: 16, 17: 8}[log_n]
    have = [c for c in (64, 32, 16, 8, 4, 2, 1) if c <= rpw and (c in (rpw, 1) or (log_n in (16, 17) and c <= 8))]
    best, best_c = -1.0, rpw
    for c in have:
        fill = B / (-(-B // c) * c)
        if fill >= 0.9:
            return c
        if fill > best + 1e-9:
            best, best_c = fill, c
    return best_c


def test_keyswitch_grid_table_matches_picker():
    assert [(ln, B, _ks_np(ln, B)) for ln, B, _ in _KS_GRIDS] == _KS_GRIDS


@pytest.mark.parametrize("log_n,B,np_", _KS_GRIDS)
def test_keyswitch_row_grids(gpu, log_n, B, np_):
    """rnt_keyswitch's rows kernel picks its grid by batch (ks_rows_pick):
    NP polys x RPW/NP consecutive rows per workgroup, the largest NP whose
    grid fills at least 90% of its row slots (key rows shared by NP polys),
    else the best-filled grid; key rows are staged through registers or by
    direct global->LDS loads by row length and grid (kKeyGlds).  The table
    runs every NP the picker can choose at each ring (NP = 1, 2, 4, 8 and
    RPW), including odd large batches (63, 127) that keep the shared-key
    grid, first and last poly of the batch, against the oracle's gadget sum
    (engine.rs:505-528)."""
    rn = gpu
    n, L = 1 << log_n, 4
    mod = rn.generate_primes(31, L, n)
    Bd, Bo = rn.RnsBasis(mod, n), orc.Basis(mod, n)
    rng = np.random.default_rng(900 + 31 * log_n + B)
    d = _rand(rng, mod, n, B)  # [B][L][N]
    ka, kb = _rand(rng, mod, n, L), _rand(rng, mod, n, L)
    key = rn.RnsGadgetKey.from_channels(ka, kb, Bd)
    a0, a1 = rn.keyswitch(rn.RnsPoly.from_channels(d, Bd), key)
    for p in sorted({0, B - 1}):
        w0, w1 = orc.keyswitch(Bo, d[p], ka, kb, threads=T)
        assert np.array_equal(a0.channels_of(p)[0], w0), (log_n, B, p)
        assert np.array_equal(a1.channels_of(p)[0], w1), (log_n, B, p)


@pytest.mark.parametrize("log_n,L,B,bits", [(16, 16, 66, 31), (14, 8, 5, 31), (12, 4, 3, 31), (14, 3, 3, 61)])
def test_fused_mul_relin_rescale_equals_two_calls(gpu, monkeypatch, log_n, L, B, bits):
    """rnt_ct_mul_relin_rescale (the rescale fused into the key-switch
    inverse) equals mul_ciphertexts_gadget + rescale_ciphertext word for word
    -- at config 4's ring over two key-switch chunks (66 pairs), config 3's,
    a whole-plane ring (2^12, the two-op fallback) and a 61-bit u64 basis --
    and the oracle on the first and last pair."""
    monkeypatch.setenv("RNT_KS_WS_MB", "4096")  # config 4: chunks of 64, so 66 pairs are two
    rn = gpu
    n = 1 << log_n
    mod = rn.generate_primes(bits, L, n)
    Bd, Bo = rn.RnsBasis(mod, n), orc.Basis(mod, n)
    rng = np.random.default_rng(700 + log_n)
    c0, c1, c0p, c1p = (_ct_batch(rng, mod, n, B, (0, B - 1)) for _ in range(4))
    ka, kb = _rand(rng, mod, n, L), _rand(rng, mod, n, L)
    rlk = rn.RnsGadgetKey.from_channels(ka, kb, Bd)
    up = lambda x: rn.RnsPoly.from_channels(x, Bd)  # noqa: E731
    ct1 = rn.Ciphertext(up(c0), up(c1), 31, Bd.total_bits())
    ct2 = rn.Ciphertext(up(c0p), up(c1p), 31, Bd.total_bits())
    fused = rn.mul_ciphertexts_gadget_rescale(ct1, ct2, rlk)
    two = rn.rescale_ciphertext(rn.mul_ciphertexts_gadget(ct1, ct2, rlk))
    assert fused.c0.basis.channel_count() == L - 1 and (fused.logp, fused.logq) == (two.logp, two.logq)
    f0, f1 = fused.c0.channels(), fused.c1.channels()
    assert np.array_equal(f0, two.c0.channels()) and np.array_equal(f1, two.c1.channels())
    for p in (0, B - 1):
        w0, w1 = orc.mul_ciphertexts_gadget(Bo, c0[p], c1[p], c0p[p], c1p[p], ka, kb, threads=T)
        assert np.array_equal(f0[p], orc.rescale(Bo, w0)), p
        assert np.array_equal(f1[p], orc.rescale(Bo, w1)), p


def test_fused_mul_relin_rescale_errors(gpu):
    """The fused op checks the output basis as rnt_ct_rescale does."""
    rn = gpu
    n = 1 << 14
    mod = rn.generate_primes(31, 4, n)
    Bd = rn.RnsBasis(mod, n)
    rng = np.random.default_rng(9)
    x = rn.RnsPoly.from_channels(_rand(rng, mod, n, 2), Bd)
    ka, kb = _rand(rng, mod, n, 4), _rand(rng, mod, n, 4)
    rlk = rn.RnsGadgetKey.from_channels(ka, kb, Bd)
    lib = rn.load()
    same = rn.RnsPoly(Bd, 2)  # full basis: not drop_last(1)
    with pytest.raises(rn.RnsNttError) as e:
        rn.check(lib.rnt_ct_mul_relin_rescale(same.handle, rn.RnsPoly(Bd, 2).handle, x.handle, x.handle,
                                              x.handle, x.handle, rlk.a.handle, rlk.b.handle))
    assert e.value.kind == "BasisMismatch"


@pytest.mark.parametrize("log_n,L,B,bits", [(16, 16, 3, 31), (14, 8, 5, 31), (14, 3, 3, 61), (15, 4, 3, 31)])
def test_keyswitch_diagonal_from_tensor(gpu, monkeypatch, log_n, L, B, bits):
    """The ct-mul key-switch takes its diagonal (source limb i of target limb
    i) from the tensor's exact d2^ instead of transforming S (the matrix-core
    tensor at 2^16, the four-step tensor rows elsewhere, u32 and u64): the
    relinearised product equals the RNT_KS_DIAG=0 path, which transforms
    every (i, j), word for word, and the oracle on the first pair."""
    rn = gpu
    n = 1 << log_n
    mod = rn.generate_primes(bits, L, n)
    Bo = orc.Basis(mod, n)
    rng = np.random.default_rng(900 + log_n)
    c0, c1, c0p, c1p = (_rand(rng, mod, n, B) for _ in range(4))
    ka, kb = _rand(rng, mod, n, L), _rand(rng, mod, n, L)
    outs = []
    for diag in ("1", "0"):
        monkeypatch.setenv("RNT_KS_DIAG", diag)  # read at rnt_ctx_create
        Bd = rn.RnsBasis(mod, n)
        rlk = rn.RnsGadgetKey.from_channels(ka, kb, Bd)
        up = lambda x: rn.RnsPoly.from_channels(x, Bd)  # noqa: E731
        r = rn.mul_ciphertexts_gadget(rn.Ciphertext(up(c0), up(c1)), rn.Ciphertext(up(c0p), up(c1p)), rlk)
        outs.append((r.c0.channels(), r.c1.channels()))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    w0, w1 = orc.mul_ciphertexts_gadget(Bo, c0[0], c1[0], c0p[0], c1p[0], ka, kb, threads=T)
    assert np.array_equal(outs[0][0][0], w0) and np.array_equal(outs[0][1][0], w1)


@pytest.mark.parametrize("log_n,L,B,k", [(14, 8, 5, 3), (16, 6, 3, -7), (17, 4, 2, 1 << 12)])
def test_rotation_fused_sigma_c0(gpu, monkeypatch, log_n, L, B, k):
    """rnt_ct_rotate gathers sigma(c0) inside the key-switch's inverse column
    pass (k_colt_inv's addend with g^-1 mod 2N) instead of a launch of its
    own: word for word the RNT_ROT_FUSE=0 path (k_automorph_odd into a
    scratch plane), over several key-switch chunks (RNT_KS_WS_MB=1 at 2^14),
    and the in-place call (out0 = c0, which keeps the separate launch), and
    the oracle on the first and last ciphertext (engine.rs:412-463)."""
    rn = gpu
    n = 1 << log_n
    mod = rn.generate_primes(31, L, n)
    Bo = orc.Basis(mod, n)
    rng = np.random.default_rng(1300 + log_n)
    c0, c1 = _rand(rng, mod, n, B), _rand(rng, mod, n, B)
    ka, kb = _rand(rng, mod, n, L), _rand(rng, mod, n, L)
    if log_n == 14:
        monkeypatch.setenv("RNT_KS_WS_MB", "1")  # one ciphertext a chunk: five chunks
    outs = []
    for fuse in ("2", "0"):
        monkeypatch.setenv("RNT_ROT_FUSE", fuse)  # read at rnt_ctx_create (2: fused at any batch)
        Bd = rn.RnsBasis(mod, n)
        rotk = rn.RnsGadgetKey.from_channels(ka, kb, Bd, rotation=k)
        x0, x1 = rn.RnsPoly.from_channels(c0, Bd), rn.RnsPoly.from_channels(c1, Bd)
        r = rn.rotate_ciphertext(rn.Ciphertext(x0, x1), rotk)
        outs.append((r.c0.channels(), r.c1.channels()))
        if fuse == "2":
            o1 = rn.RnsPoly(Bd, B)
            rn.check(rn.load().rnt_ct_rotate(x0.handle, o1.handle, x0.handle, x1.handle, int(k),
                                              rotk.a.handle, rotk.b.handle))
            outs.append((x0.channels(), o1.channels()))
    for o in outs[1:]:
        assert np.array_equal(outs[0][0], o[0]) and np.array_equal(outs[0][1], o[1])
    for p in (0, B - 1):
        w0, w1 = orc.rotate_ciphertext(Bo, c0[p], c1[p], k, ka, kb, threads=T)
        assert np.array_equal(outs[0][0][p], w0) and np.array_equal(outs[0][1][p], w1), p
