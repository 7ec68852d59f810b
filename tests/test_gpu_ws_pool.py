"""Key-switch workspace reuse (rnt_api.cpp ensure_ws / rnt_buf_free pool).

Every gadget multiply below gets fresh output buffers, so from the second
call on its workspace comes from blocks earlier, freed buffers left behind
(dirty).  The results must not depend on that: all calls agree with each
other and with the oracle's mul_ciphertexts_gadget (pyoracle, via the
sharded tests' helper)."""
import numpy as np
import pytest

from test_sharded import _inputs, _oracle_reference


@pytest.mark.gpu
def test_gadget_mul_with_reused_workspace_matches_oracle(gpu):
    rn = gpu
    n, L, B = 4096, 8, 3
    mods = rn.generate_primes(31, L, n)
    cts, key_a, key_b = _inputs(mods, n, B, 21)
    basis = rn.RnsBasis(mods, n)
    c = [rn.RnsPoly.from_channels(x, basis) for x in cts]
    key = rn.RnsGadgetKey.from_channels(key_a, key_b, basis)
    first = None
    for it in range(6):
        m = rn.mul_ciphertexts_gadget(rn.Ciphertext(c[0], c[1]), rn.Ciphertext(c[2], c[3]), key)
        got = (m.c0.channels(), m.c1.channels())
        del m  # frees the buffers: their workspace goes back to the pool
        if first is None:
            first = got
        else:
            assert all(np.array_equal(g, f) for g, f in zip(got, first)), f"call {it} differs"
    want = _oracle_reference(mods, n, [x[:1] for x in cts], key_a, key_b)
    assert np.array_equal(first[0][:1], want[0]) and np.array_equal(first[1][:1], want[1])
