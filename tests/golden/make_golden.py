#!/usr/bin/env python3
"""Generate tests/golden/vectors.npz with an independent pure-Python
big-integer restatement of the reference's RNS-NTT path.

Nothing here shares code with oracle/oracle.c or with the HIP backend:
NTT-domain values come from direct evaluation a(psi^(2k+1)) (the value the
reference's to_ntt_domain computes at index k), products
from the schoolbook negacyclic convolution (the reference's own oracle,
poly.rs:339-367), and psi from the reference's root-selection rule
(basis.rs:217-237).  After generation every vector is cross-checked against
the C oracle so the two restatements pin each other.

Usage:  python tests/golden/make_golden.py      (writes vectors.npz)
"""
from __future__ import annotations

import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

# --- number theory (primes.rs:67-219, utils.rs:47-80, basis.rs:217-237) ---
MR_BASES = [2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37]


def is_prime(n: int) -> bool:
    if n < 2:
        return False
    if n < 4:
        return True
    if n % 2 == 0:
        return False
    d, r = n - 1, 0
    while d % 2 == 0:
        d //= 2
        r += 1
    for a in MR_BASES:
        if a >= n:
            continue
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(r - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def prime_down(bound: int, n: int):
    if bound <= 2:
        return None
    step = 2 * n
    c = bound - 1
    c -= (c % step + step - 1) % step
    while True:
        if c <= 2:
            return None
        if is_prime(c):
            return c
        if c < step:
            return None
        c -= step


def generate_primes(bits: int, count: int, degree: int) -> list[int]:
    upper, lower = (1 << bits) - 1, 1 << (bits - 1)
    cur = prime_down(upper + 1, degree)
    out = []
    while len(out) < count and cur is not None and cur >= lower:
        out.append(cur)
        cur = prime_down(cur, degree)
    assert len(out) == count
    return out


def find_psi(q: int, n: int) -> int:
    e = (q - 1) // (2 * n)
    for c in range(2, q):
        r = pow(c, e, q)
        if r != 1 and pow(r, n, q) != 1:
            return r
    raise ValueError


# --- ring ops on lists of ints ------------------------------------------------


def negacyclic(a, b, q):
    n = len(a)
    out = [0] * n
    for i, ai in enumerate(a):
        if ai == 0:
            continue
        for j, bj in enumerate(b):
            k = i + j
            if k < n:
                out[k] += ai * bj
            else:
                out[k - n] -= ai * bj
    return [x % q for x in out]


def ntt_natural(a, q, psi):
    """index k -> a(psi^(2k+1)) mod q."""
    n = len(a)
    res = []
    for k in range(n):
        x = pow(psi, 2 * k + 1, q)
        acc = 0
        for c in reversed(a):  # Horner
            acc = (acc * x + c) % q
        res.append(acc)
    return res


def rescale(ch, moduli):
    L = len(moduli)
    ql = moduli[-1]
    out = []
    for i in range(L - 1):
        qi = moduli[i]
        inv = pow(ql % qi, -1, qi)
        out.append([((c - cl % qi) * inv) % qi for c, cl in zip(ch[i], ch[L - 1])])
    return out


def automorphism(ch, moduli, g):
    """poly.rs:506-540 (last non-zero writer wins for non-odd g)."""
    n = len(ch[0])
    e = g % (2 * n)
    if e == 0:
        return [list(c) for c in ch]
    out = []
    for c, q in zip(ch, moduli):
        o = [0] * n
        for i, v in enumerate(c):
            jf = i * e % (2 * n)
            if v == 0:
                continue
            o[jf % n] = (q - v) if jf >= n else v
        out.append(o)
    return out


def rotation_exponent(k, n):
    e = pow(5, abs(k), 2 * n)
    return e if k >= 0 else (e * (2 * n - 1)) % (2 * n)


def poly_mul(x, y, moduli):
    return [negacyclic(a, b, q) for a, b, q in zip(x, y, moduli)]


def poly_add(x, y, moduli):
    return [[(u + v) % q for u, v in zip(a, b)] for a, b, q in zip(x, y, moduli)]


def keyswitch(d, key_a, key_b, moduli):
    L = len(moduli)
    n = len(d[0])
    acc0 = [[0] * n for _ in range(L)]
    acc1 = [[0] * n for _ in range(L)]
    for i in range(L):
        alpha = [[v % qj for v in d[i]] for qj in moduli]
        acc0 = poly_add(acc0, poly_mul(alpha, key_b[i], moduli), moduli)
        acc1 = poly_add(acc1, poly_mul(alpha, key_a[i], moduli), moduli)
    return acc0, acc1


def rand_poly(rng, moduli, n):
    return [[rng.randrange(q) for _ in range(n)] for q in moduli]


def arr(x):
    return np.array(x, dtype=np.uint64)


def main():
    rng = random.Random(20261015)
    vec = {}
    manifest = {}

    def ring_case(name, bits, L, n, extras=True):
        moduli = generate_primes(bits, L, n)
        psis = [find_psi(q, n) for q in moduli]
        a, b = rand_poly(rng, moduli, n), rand_poly(rng, moduli, n)
        vec[f"{name}/moduli"] = arr(moduli)
        vec[f"{name}/psi"] = arr(psis)
        vec[f"{name}/a"] = arr(a)
        vec[f"{name}/b"] = arr(b)
        vec[f"{name}/mul"] = arr(poly_mul(a, b, moduli))
        vec[f"{name}/ntt_a"] = arr([ntt_natural(c, q, p) for c, q, p in zip(a, moduli, psis)])
        vec[f"{name}/add"] = arr(poly_add(a, b, moduli))
        if L >= 2:
            vec[f"{name}/rescale_a"] = arr(rescale(a, moduli))
        if extras:
            for g in (3, 2 * n - 1, rotation_exponent(3, n), 2, n):
                vec[f"{name}/auto_{g}"] = arr(automorphism(a, moduli, g))
        manifest[name] = {"bits": bits, "L": L, "n": n}
        print(name, "done", flush=True)

    ring_case("n8_q20x2", 20, 2, 8)
    ring_case("n16_q31x3", 31, 3, 16)  # config 1 primes (examples/encrypt_add.rs:41)
    ring_case("n64_q40x3", 40, 3, 64)
    ring_case("n256_q61x2", 61, 2, 256)
    ring_case("n1024_q31x3", 31, 3, 1024, extras=True)
    ring_case("n1024_q62x2", 62, 2, 1024, extras=False)

    # key-switch / ciphertext pipeline (engine.rs:412-539) at N=64, L=3
    for name, bits in (("ks_n64_q31x3", 31), ("ks_n32_q62x2", 62)):
        L = 3 if bits == 31 else 2
        n = 64 if bits == 31 else 32
        moduli = generate_primes(bits, L, n)
        c0, c1, c0p, c1p = (rand_poly(rng, moduli, n) for _ in range(4))
        key_a = [rand_poly(rng, moduli, n) for _ in range(L)]
        key_b = [rand_poly(rng, moduli, n) for _ in range(L)]
        d2 = poly_mul(c1, c1p, moduli)
        acc0, acc1 = keyswitch(d2, key_a, key_b, moduli)
        d0 = poly_mul(c0, c0p, moduli)
        d1 = poly_add(poly_mul(c0, c1p, moduli), poly_mul(c1, c0p, moduli), moduli)
        out0, out1 = poly_add(d0, acc0, moduli), poly_add(d1, acc1, moduli)
        vec.update({f"{name}/moduli": arr(moduli), f"{name}/c0": arr(c0), f"{name}/c1": arr(c1),
                    f"{name}/c0p": arr(c0p), f"{name}/c1p": arr(c1p), f"{name}/key_a": arr(key_a),
                    f"{name}/key_b": arr(key_b), f"{name}/relin_out0": arr(out0),
                    f"{name}/relin_out1": arr(out1)})
        for k in (1, -1, 3):
            g = rotation_exponent(k, n)
            s0, s1 = automorphism(c0, moduli, g), automorphism(c1, moduli, g)
            r0, r1 = keyswitch(s1, key_a, key_b, moduli)
            vec[f"{name}/rot{k}_out0"] = arr(poly_add(s0, r0, moduli))
            vec[f"{name}/rot{k}_out1"] = arr(r1)
        manifest[name] = {"bits": bits, "L": L, "n": n}
        print(name, "done", flush=True)

    # BASELINE config prime chains (SURVEY §8a a14 restated) and psi
    configs = {"cfg1_n16": (31, 3, 16), "cfg2_n4096": (31, 4, 4096), "cfg3_n16384": (31, 8, 16384),
               "cfg4_n65536": (31, 16, 65536), "cfg5_n131072": (31, 32, 131072)}
    for name, (bits, L, n) in configs.items():
        moduli = generate_primes(bits, L, n)
        vec[f"{name}/moduli"] = arr(moduli)
        vec[f"{name}/psi"] = arr([find_psi(q, n) for q in moduli])
        manifest[name] = {"bits": bits, "L": L, "n": n}

    out = os.path.join(HERE, "vectors.npz")
    np.savez_compressed(out, **vec)
    with open(os.path.join(HERE, "vectors_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote", out, len(vec), "arrays")

    # cross-check with the C oracle (the two restatements pin each other)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pyoracle as orc  # noqa: E402

    for name, m in manifest.items():
        moduli = [int(x) for x in vec[f"{name}/moduli"]]
        assert orc.generate_primes(m["bits"], m["L"], m["n"]) == moduli, name
        if f"{name}/a" in vec:
            B = orc.Basis(moduli, m["n"])
            a, b = vec[f"{name}/a"], vec[f"{name}/b"]
            assert [B.psi(i) for i in range(B.L)] == [int(x) for x in vec[f"{name}/psi"]]
            assert np.array_equal(orc.mul(B, a, b), vec[f"{name}/mul"]), name
            assert np.array_equal(orc.to_ntt(B, a), vec[f"{name}/ntt_a"]), name
    print("oracle cross-check OK")


if __name__ == "__main__":
    main()
