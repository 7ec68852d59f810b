"""The C-ABI boundary on the device: the reference's error payloads, the
device block cache (buffers freed without a host wait, their blocks reused
by later allocations on the same or another stream), and every runtime knob
the library still reads, each on its non-default setting, bit-exact against
the oracle.

Knobs (read when a context is created, or per call for the cache cap):
* RNT_LAZY30=0   -- 30-bit bases take the canonical product path instead of
                    the Harvey-lazy one;
* RNT_KS_WS_MB   -- key-switch scratch cap: 1 MiB cuts a config-3-shaped
                    batch into one ciphertext per chunk;
* RNT_WS_POOL_MB -- idle bytes the device cache keeps: 0 releases every
                    freed block at once;
* RNT_DEC_JG     -- covered by test_gpu_configs.py::test_decomposition_groups.
"""
from __future__ import annotations

import numpy as np
import pytest

import pyoracle as orc

pytestmark = pytest.mark.gpu

T = orc.host_threads()


def _rand(rng, mod, n, batch=None):
    return orc.uniform_poly(mod, n, rng, batch=batch)


def test_error_payloads_match_reference_variants(gpu):
    """errors.rs:4-20 struct variants, rebuilt from rnt_last_error_detail."""
    rn = gpu
    Bd = rn.RnsBasis([17, 97], 8)
    bad = np.zeros((2, 8), dtype=np.uint64)
    bad[1, 3] = 100  # not reduced modulo 97 (poly.rs:83-93)
    with pytest.raises(rn.RnsNttError) as e:
        rn.RnsPoly.from_channels(bad, Bd)
    assert e.value.kind == "NonReducedCoefficient"
    assert e.value.fields == {"coefficient": 100, "modulus": 97}
    with pytest.raises(rn.RnsNttError) as e:
        rn.RnsPoly.from_channels(np.zeros((1, 8), dtype=np.uint64), Bd)
    assert e.value.fields == {"expected": 2, "actual": 1} and e.value.kind == "ChannelCountMismatch"
    with pytest.raises(rn.RnsNttError) as e:
        Bd.drop_last(2)  # basis.rs:121-134
    assert e.value.kind == "InvalidModDrop" and e.value.fields == {"drop_count": 2, "channel_count": 2}
    one = rn.RnsPoly.from_channels(np.ones((1, 8), dtype=np.uint64), rn.RnsBasis([17], 8))
    with pytest.raises(rn.RnsNttError) as e:
        one.rescale()  # poly.rs:191-197
    assert e.value.kind == "InvalidModDrop" and e.value.fields == {"drop_count": 1, "channel_count": 1}
    # the gadget key must hold one poly per channel
    d = rn.RnsPoly.from_channels(_rand(np.random.default_rng(1), [17, 97], 8, 1), Bd)
    key = rn.RnsGadgetKey.from_channels(np.zeros((1, 2, 8), np.uint64), np.zeros((1, 2, 8), np.uint64), Bd)
    with pytest.raises(rn.RnsNttError) as e:
        rn.keyswitch(d, key)
    assert e.value.kind == "ChannelCountMismatch" and e.value.fields == {"expected": 2, "actual": 1}


def _hip_runtime():
    """The process's one HIP runtime (the copy torch loaded, which the
    library binds too), by its mapped path: loading another copy by name
    would start a second runtime."""
    import ctypes

    with open("/proc/self/maps") as f:
        paths = {ln.split()[-1] for ln in f if "libamdhip64" in ln and "/" in ln}
    assert len(paths) == 1, paths
    rt = ctypes.CDLL(paths.pop())
    rt.hipSetDevice.argtypes = [ctypes.c_int]
    rt.hipSetDevice.restype = ctypes.c_int
    rt.hipGetLastError.restype = ctypes.c_int
    return rt


def test_pending_hip_error_is_reported_not_dropped(gpu):
    """A HIP error some other code left in the runtime's last-error slot is
    reported by the next launch as DeviceError, pending from an earlier
    call (r04's clear_stale_error dropped it), and the launch after that
    runs normally."""
    rn = gpu
    n, L = 1 << 12, 2
    mod = rn.generate_primes(31, L, n)
    Bd = rn.RnsBasis(mod, n)
    x = rn.RnsPoly.from_channels(_rand(np.random.default_rng(9), mod, n, 2), Bd)
    x.to_ntt_domain()
    Bd.sync()
    rt = _hip_runtime()
    assert rt.hipSetDevice(4096) != 0  # invalid device: the slot now holds the error
    with pytest.raises(rn.RnsNttError) as e:
        x.to_coeff_domain()
    assert e.value.kind == "DeviceError" and "pending" in str(e.value), str(e.value)
    assert rt.hipGetLastError() == 0  # reported, so no longer pending
    x.to_coeff_domain()  # the op itself was never launched: x is still NTT-domain
    assert not x.is_ntt_domain()


def test_freed_blocks_are_reused_without_host_wait(gpu):
    """Buffers freed while their kernels may still be queued hand their
    blocks to later allocations; results and zero-initialisation stay exact.
    A second context (its own stream) takes blocks freed on the first."""
    rn = gpu
    lib = rn.load()
    n, L = 1 << 12, 4
    mod = rn.generate_primes(31, L, n)
    Bd, Bo = rn.RnsBasis(mod, n), orc.Basis(mod, n)
    other = rn.RnsBasis(mod, n)  # same moduli, another stream
    rng = np.random.default_rng(7)
    a_h, b_h = _rand(rng, mod, n, 8), _rand(rng, mod, n, 8)
    want = np.stack([orc.mul(Bo, a_h[i], b_h[i]) for i in range(8)])
    a, b = rn.RnsPoly.from_channels(a_h, Bd), rn.RnsPoly.from_channels(b_h, Bd)
    for it in range(6):
        out = rn.RnsPoly(Bd, 8)  # fresh output (and workspace) each time
        rn.check(lib.rnt_mul(out.handle, a.handle, b.handle))
        if it % 2:
            got = out.channels()
            assert np.array_equal(got, want), it
        del out  # freed right after queueing its product: no host wait
        z = rn.RnsPoly(other if it % 3 == 0 else Bd, 8)  # takes the freed block
        assert not z.channels().any(), it  # RnsPoly::zero
        del z
    freed = rn.pool_trim()
    assert freed > 0
    assert rn.pool_trim() == 0


def test_pool_cap_zero_releases_every_block(gpu, monkeypatch):
    """RNT_WS_POOL_MB=0: no idle block is kept; a ct-mul loop that makes
    fresh outputs every step stays exact."""
    rn = gpu
    monkeypatch.setenv("RNT_WS_POOL_MB", "0")
    n, L, B = 1 << 12, 4, 2
    mod = rn.generate_primes(31, L, n)
    Bd, Bo = rn.RnsBasis(mod, n), orc.Basis(mod, n)
    rng = np.random.default_rng(8)
    c = [_rand(rng, mod, n, B) for _ in range(4)]
    ka, kb = _rand(rng, mod, n, L), _rand(rng, mod, n, L)
    rlk = rn.RnsGadgetKey.from_channels(ka, kb, Bd)
    up = lambda x: rn.RnsPoly.from_channels(x, Bd)  # noqa: E731
    w0, w1 = orc.mul_ciphertexts_gadget(Bo, c[0][1], c[1][1], c[2][1], c[3][1], ka, kb)
    for _ in range(3):
        out = rn.mul_ciphertexts_gadget(rn.Ciphertext(up(c[0]), up(c[1])), rn.Ciphertext(up(c[2]), up(c[3])), rlk)
        assert np.array_equal(out.c0.channels()[1], w0) and np.array_equal(out.c1.channels()[1], w1)
        del out
    assert rn.pool_trim() == 0  # nothing was kept


def test_lazy30_off_takes_canonical_path(gpu, monkeypatch):
    """RNT_LAZY30=0 on a 30-bit basis: the canonical 31-bit product kernels
    run instead of the Harvey-lazy ones; products stay bit-exact."""
    rn = gpu
    monkeypatch.setenv("RNT_LAZY30", "0")
    n, L = 1 << 14, 6
    mod = rn.generate_primes(30, L, n)
    Bd, Bo = rn.RnsBasis(mod, n), orc.Basis(mod, n)
    q = np.array(mod, dtype=np.uint64)[:, None]
    rng = np.random.default_rng(30)
    full = np.broadcast_to(q - 1, (L, n)).copy()
    x = np.stack([_rand(rng, mod, n), full, _rand(rng, mod, n)])
    y = np.stack([_rand(rng, mod, n), full, full])
    got = (rn.RnsPoly.from_channels(x, Bd) * rn.RnsPoly.from_channels(y, Bd)).channels()
    for i in range(3):
        assert np.array_equal(got[i], orc.mul(Bo, x[i], y[i])), i


def test_small_keyswitch_scratch_chunks_every_ciphertext(gpu, monkeypatch):
    """RNT_KS_WS_MB=1 at N=2^12, L=8 (S per ciphertext = 1 MiB): each
    ciphertext is its own key-switch chunk, for the relinearisation and for
    a limb shard's keyswitch_ext."""
    rn = gpu
    monkeypatch.setenv("RNT_KS_WS_MB", "1")
    n, L, B = 1 << 12, 8, 3
    mod = rn.generate_primes(31, L, n)
    Bd, Bo = rn.RnsBasis(mod, n), orc.Basis(mod, n)
    rng = np.random.default_rng(12)
    c = [_rand(rng, mod, n, B) for _ in range(4)]
    ka, kb = _rand(rng, mod, n, L), _rand(rng, mod, n, L)
    rlk = rn.RnsGadgetKey.from_channels(ka, kb, Bd)
    up = lambda x: rn.RnsPoly.from_channels(x, Bd)  # noqa: E731
    out = rn.mul_ciphertexts_gadget(rn.Ciphertext(up(c[0]), up(c[1])), rn.Ciphertext(up(c[2]), up(c[3])), rlk)
    o0, o1 = out.c0.channels(), out.c1.channels()
    for p in range(B):
        w0, w1 = orc.mul_ciphertexts_gadget(Bo, c[0][p], c[1][p], c[2][p], c[3][p], ka, kb)
        assert np.array_equal(o0[p], w0) and np.array_equal(o1[p], w1), p
    Lt = 3
    Bt = rn.RnsBasis(mod[:Lt], n)
    key_t = rn.RnsGadgetKey.from_channels(np.ascontiguousarray(ka[:, :Lt]), np.ascontiguousarray(kb[:, :Lt]), Bt)
    d = up(c[1])
    ptr, _ = d.device_ptr()
    a0, a1 = rn.keyswitch_ext(ptr, L, key_t, Bt, B)
    g0, g1 = a0.channels(), a1.channels()
    for p in range(B):
        w0, w1 = orc.keyswitch(Bo, c[1][p], ka, kb)
        assert np.array_equal(g0[p], w0[:Lt]) and np.array_equal(g1[p], w1[:Lt]), p



def test_download_polys_reads_a_sub_batch(gpu):
    """rnt_download_polys: channels() of a range of a batch, in either
    domain; ranges outside the batch are BadArgument."""
    rn = gpu
    n, L, B = 1 << 12, 3, 5
    mod = rn.generate_primes(31, L, n)
    Bd = rn.RnsBasis(mod, n)
    x = _rand(np.random.default_rng(3), mod, n, B)
    p = rn.RnsPoly.from_channels(x, Bd)
    assert np.array_equal(p.channels_of(1, 3), x[1:4])
    assert np.array_equal(p.channels_of(4), x[4:5])
    p.to_ntt_domain()
    full = p.channels()
    assert np.array_equal(p.channels_of(2, 2), full[2:4])
    assert p.channels_of(5, 0).shape == (0, L, n)
    with pytest.raises(rn.RnsNttError) as e:
        p.channels_of(4, 2)
    assert e.value.kind == "BadArgument"


def test_ops_follow_a_caller_stream(gpu):
    """rnt_ctx_set_stream: with torch's stream bound, a product over wrapped
    torch tensors waits for the torch work queued before it (a device sleep,
    then the operand copies) and torch reads the result on the same stream,
    with no host wait in between.  NULL restores the basis' own stream."""
    import torch

    rn = gpu
    lib = rn.load()
    n, L, B = 1 << 12, 4, 4
    mod = rn.generate_primes(31, L, n)
    Bd, Bo = rn.RnsBasis(mod, n), orc.Basis(mod, n)
    own = Bd.stream()
    rng = np.random.default_rng(21)
    a_h, b_h = _rand(rng, mod, n, B), _rand(rng, mod, n, B)
    want = np.stack([orc.mul(Bo, a_h[i], b_h[i]) for i in range(B)])
    dev = torch.device("cuda", Bd.device)
    # device layout [L][B][N] of 32-bit words (residues < 2^31 fit int32)
    lay = lambda x: torch.from_numpy(np.ascontiguousarray(x.transpose(1, 0, 2)).astype(np.int32))  # noqa: E731
    a_src, b_src = lay(a_h).to(dev), lay(b_h).to(dev)
    torch.cuda.synchronize(dev)
    a_t, b_t = torch.zeros_like(a_src), torch.zeros_like(b_src)
    out_t = torch.zeros_like(a_src)
    a = rn.RnsPoly.wrap(Bd, a_t.data_ptr(), B, owner=a_t)
    b = rn.RnsPoly.wrap(Bd, b_t.data_ptr(), B, owner=b_t)
    out = rn.RnsPoly.wrap(Bd, out_t.data_ptr(), B, owner=out_t)
    s = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(s):
        torch.cuda._sleep(20_000_000)  # the operands land well after the launch
        a_t.copy_(a_src)
        b_t.copy_(b_src)
    Bd.set_stream(s)
    assert Bd.stream() == s.cuda_stream
    rn.check(lib.rnt_mul(out.handle, a.handle, b.handle))
    with torch.cuda.stream(s):
        res = out_t.clone()
    s.synchronize()
    got = res.cpu().numpy().astype(np.uint64).transpose(1, 0, 2)
    assert np.array_equal(got, want)
    Bd.set_stream(None)
    assert Bd.stream() == own
    # the own stream is ordered after the caller's: a download sees the product
    assert np.array_equal(out.channels(), want)


def _reupload(rn, buf, channels):
    """from_channels into an existing buffer (same device memory)."""
    import ctypes

    ch = np.ascontiguousarray(channels, dtype=np.uint64)
    if ch.ndim == 2:
        ch = ch[None]
    rn.check(rn.load().rnt_upload(buf.handle, ch.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                  ch.shape[0], ch.shape[1], 0))


def test_graph_capture_replays_the_engine_call_shape(gpu):
    """rnt_capture_begin/end + rnt_graph_launch: one ciphertext's
    mul_ciphertexts_gadget + rescale_ciphertext (engine.rs:473-539,
    263-282) and a rotate_ciphertext (:412-463), recorded once and replayed
    after the input buffers were overwritten in place: every replay
    recomputes from the buffers' current contents, bit-exact against the
    oracle; recording does not run the ops."""
    rn = gpu
    n, L = 1 << 12, 4
    mods = rn.generate_primes(31, L, n)
    Bd, Bo = rn.RnsBasis(mods, n), orc.Basis(mods, n)
    rng = np.random.default_rng(77)
    x = [_rand(rng, mods, n) for _ in range(4)]
    ka, kb = _rand(rng, mods, n, L), _rand(rng, mods, n, L)
    ra, rb = _rand(rng, mods, n, L), _rand(rng, mods, n, L)
    key = rn.RnsGadgetKey.from_channels(ka, kb, Bd)
    rkey = rn.RnsGadgetKey.from_channels(ra, rb, Bd)
    c = [rn.RnsPoly.from_channels(v, Bd) for v in x]
    lib = rn.load()
    Bd1 = Bd.drop_last(1)
    o0, o1, r0, r1 = rn.RnsPoly(Bd), rn.RnsPoly(Bd), rn.RnsPoly(Bd1), rn.RnsPoly(Bd1)
    t0, t1 = rn.RnsPoly(Bd), rn.RnsPoly(Bd)
    k = -3

    def seq():
        rn.check(lib.rnt_ct_mul_relin(o0.handle, o1.handle, c[0].handle, c[1].handle, c[2].handle,
                                      c[3].handle, key.a.handle, key.b.handle))
        rn.check(lib.rnt_ct_rescale(r0.handle, r1.handle, o0.handle, o1.handle))
        rn.check(lib.rnt_ct_rotate(t0.handle, t1.handle, c[0].handle, c[1].handle, k, rkey.a.handle,
                                   rkey.b.handle))

    seq()  # warm: the workspaces are cached before recording
    Bd.sync()
    for p in (r0, r1, t0, t1):
        _reupload(rn, p, np.zeros((p.basis.channel_count(), n), np.uint64))
    with Bd.capture() as g:
        seq()
    Bd.sync()
    assert not r0.channels().any() and not t1.channels().any()  # recorded, not run
    for it in range(2):
        x = [_rand(rng, mods, n) for _ in range(4)]
        for buf, v in zip(c, x):
            _reupload(rn, buf, v)
        g.replay()
        g.replay()
        Bd.sync()
        w0, w1 = orc.mul_ciphertexts_gadget(Bo, x[0], x[1], x[2], x[3], ka, kb)
        assert np.array_equal(r0.channels(), orc.rescale(Bo, w0)), it
        assert np.array_equal(r1.channels(), orc.rescale(Bo, w1)), it
        v0, v1 = orc.rotate_ciphertext(Bo, x[0], x[1], k, ra, rb)
        assert np.array_equal(t0.channels(), v0) and np.array_equal(t1.channels(), v1), it
    del g  # returns the graph's workspace blocks to the cache
    seq()
    Bd.sync()
    assert np.array_equal(t0.channels(), v0)


def test_graph_records_share_one_keyswitch_workspace(gpu):
    """N recorded key-switch ops keep one call-scoped workspace block (the
    recorded ops are ordered on the one captured stream, so the second op
    reuses the block the first handed back while recording), and the
    replays of the 4-rotation graph are bit-exact against the oracle.  A
    capture whose body raises destroys its graph (no leaked workspace)."""
    rn = gpu
    n, L = 1 << 12, 4
    mods = rn.generate_primes(31, L, n)
    Bd, Bo = rn.RnsBasis(mods, n), orc.Basis(mods, n)
    rng = np.random.default_rng(78)
    x0, x1 = _rand(rng, mods, n), _rand(rng, mods, n)
    ra, rb = _rand(rng, mods, n, L), _rand(rng, mods, n, L)
    rkey = rn.RnsGadgetKey.from_channels(ra, rb, Bd)
    c0, c1 = rn.RnsPoly.from_channels(x0, Bd), rn.RnsPoly.from_channels(x1, Bd)
    lib = rn.load()
    outs = [(rn.RnsPoly(Bd), rn.RnsPoly(Bd)) for _ in range(4)]

    def rec(m):
        for t0, t1 in outs[:m]:
            rn.check(lib.rnt_ct_rotate(t0.handle, t1.handle, c0.handle, c1.handle, 1, rkey.a.handle,
                                       rkey.b.handle))

    rec(4)  # warm
    Bd.sync()
    with Bd.capture() as g1:
        rec(1)
    with Bd.capture() as g4:
        rec(4)
    b1, by1 = g1.workspace()
    b4, by4 = g4.workspace()
    # one block either way (g4's may be another cached block of a different
    # size: g1 holds the first); four ops do not keep four
    assert b1 >= 1 and b4 == b1 and by4 < 2 * by1, ((b1, by1), (b4, by4))
    g4.replay()
    Bd.sync()
    v0, v1 = orc.rotate_ciphertext(Bo, x0, x1, 1, ra, rb)
    for t0, t1 in outs:
        assert np.array_equal(t0.channels(), v0) and np.array_equal(t1.channels(), v1)
    del g1, g4
    with pytest.raises(ZeroDivisionError):
        with Bd.capture():
            rec(1)
            1 / 0
    # the context records again after the failed capture
    with Bd.capture() as g:
        rec(2)
    g.replay()
    Bd.sync()
    assert np.array_equal(outs[1][0].channels(), v0)


def test_deferred_failure_survives_an_intervening_free(gpu):
    """a free / destroy reports only its own cleanup failures.  A
    failure deferred earlier on the thread (rnt_debug_defer stands in for a
    block that failed to leave the cache) is neither consumed nor blamed by
    an intervening rnt_buf_free -- whose status the bindings' __del__ drops
    -- and reaches the next launch, which reports it and does not run."""
    rn = gpu
    lib = rn.load()
    n, L = 1 << 12, 2
    mod = rn.generate_primes(31, L, n)
    Bd = rn.RnsBasis(mod, n)
    x = rn.RnsPoly.from_channels(_rand(np.random.default_rng(3), mod, n, 2), Bd)
    tmp = rn.RnsPoly(Bd, 4)
    Bd.sync()
    assert lib.rnt_debug_defer(1) == 0  # hipErrorInvalidValue, deferred
    assert lib.rnt_buf_free(tmp.handle) == 0  # its own cleanup succeeded: OK, not the earlier failure
    tmp._h = None
    with pytest.raises(rn.RnsNttError) as e:
        x.to_ntt_domain()
    assert e.value.kind == "DeviceError" and "rnt_debug_defer" in str(e.value), str(e.value)
    assert not x.is_ntt_domain()  # reported before any launch
    x.to_ntt_domain()  # reported once: the next launch runs
    assert x.is_ntt_domain()
