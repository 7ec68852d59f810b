"""C-ABI checks that need no GPU: the library loads, exports exactly what
include/rnsntt.h declares, its host-side setup math matches the oracle and
the reference KATs, and validation errors come back as the reference's
RnsNttError variants."""
from __future__ import annotations

import ctypes
import os
import re
import sys

import numpy as np
import pytest

import pyoracle as orc
import rns_ntt
from rns_ntt import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    text = open(os.path.join(REPO, "include", "rnsntt.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rnt_[a-z0-9_]+)\s*\(", text)))


def test_library_loads_and_exports_every_declared_symbol():
    lib = rns_ntt.load()
    assert lib.rnt_abi_version() == 4
    names = declared_functions()
    assert len(names) >= 35
    for n in names:
        assert hasattr(lib, n), n
    # the Python binding types every declared function
    assert sorted(_lib.SIGNATURES) == names


def test_status_strings_mirror_rnsntt_error():
    lib = rns_ntt.load()
    want = ["ok", "InvalidDegree", "EmptyBasis", "NonNttFriendlyModulus", "InvalidModDrop",
            "ChannelCountMismatch", "NonReducedCoefficient", "DomainMismatch", "BasisMismatch",
            "DeviceError", "OutOfMemory", "BadArgument", "Unsupported"]
    for code, name in enumerate(want):
        assert lib.rnt_status_string(code).decode() == name
        if code:
            assert _lib.STATUS_NAMES[code] == name


def test_generate_primes_matches_oracle_and_configs(vectors, manifest):
    for name, m in manifest.items():
        mods = rns_ntt.generate_primes(m["bits"], m["L"], m["n"])
        assert mods == [int(x) for x in vectors[f"{name}/moduli"]], name
        assert mods == orc.generate_primes(m["bits"], m["L"], m["n"])
        if f"{name}/psi" in vectors:
            for q, psi in zip(mods, vectors[f"{name}/psi"]):
                assert rns_ntt.find_psi(q, m["n"]) == int(psi)


def test_prime_kats(kats):
    k = kats["primes"]
    f = k["ntt_friendly_condition"]
    assert all(rns_ntt.is_ntt_friendly_prime(p, f["n"]) for p in f["friendly"])
    assert not any(rns_ntt.is_ntt_friendly_prime(p, f["n"]) for p in f["not_friendly"])
    g = k["generates_ntt_primes_in_range"]
    ps = rns_ntt.generate_primes(g["bits"], g["count"], g["degree"])
    assert all((1 << 19) <= q < (1 << 20) and rns_ntt.is_ntt_friendly_prime(q, 1024) for q in ps)
    g = k["panics_when_not_enough_primes"]
    with pytest.raises(rns_ntt.RnsNttError):
        rns_ntt.generate_primes(g["bits"], g["count"], g["degree"])
    # primality through the friendly test at degree 1 (p = 1 mod 2 <=> odd prime)
    for p in k["is_prime_large"]["prime"] + k["near_u64_limit"]["prime"]:
        assert rns_ntt.is_ntt_friendly_prime(p, 1)
    for c in k["is_prime_large"]["composite"] + k["tricky_composites"]["composite"]:
        assert not rns_ntt.is_ntt_friendly_prime(c, 1)
    for lo, hi in k["miller_rabin_matches_reference_ranges"]["ranges"]:
        for n in range(lo, hi + 1):
            want = orc.lib().or_is_prime(n) and n % 2 == 1
            assert rns_ntt.is_ntt_friendly_prime(n, 1) == bool(want), n


def test_psi_matches_oracle_random_primes():
    rng = np.random.default_rng(5)
    for logn in (1, 3, 8, 12, 16, 17):
        n = 1 << logn
        for bits in (20, 31, 40, 62):
            if bits <= logn + 8:
                continue
            for q in rns_ntt.generate_primes(bits, 2, n):
                assert rns_ntt.find_psi(q, n) == orc.lib().or_find_primitive_root(q, 2 * n)


def test_ctx_validation_errors_without_gpu(kats):
    """RnsBasis::new error order (basis.rs:97-106) -- checked before any HIP call."""
    lib = rns_ntt.load()
    h = ctypes.c_void_p()
    arr = np.zeros(1, dtype=np.uint64)
    assert lib.rnt_ctx_create(3, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 0, 0, ctypes.byref(h)) == 2
    with pytest.raises(rns_ntt.RnsNttError) as e:
        rns_ntt.RnsBasis([], 8)
    assert e.value.kind == "EmptyBasis" and e.value.fields == {}
    bad = kats["basis_n8"]["rejects_non_friendly_modulus"]["modulus"]
    with pytest.raises(rns_ntt.RnsNttError) as e:
        rns_ntt.RnsBasis([bad], 8)
    # NonNttFriendlyModulus { modulus, degree } (errors.rs:9-10, basis.rs:26-29)
    assert e.value.kind == "NonNttFriendlyModulus"
    assert e.value.fields == {"modulus": bad, "degree": 8} and e.value.modulus == bad
    with pytest.raises(rns_ntt.RnsNttError) as e:
        rns_ntt.RnsBasis([17], 12)
    assert e.value.kind == "InvalidDegree" and e.value.fields == {"degree": 12}
    q18 = rns_ntt.generate_primes(31, 1, 1 << 18)[0]
    with pytest.raises(rns_ntt.RnsNttError) as e:
        rns_ntt.RnsBasis([q18], 1 << 18)
    # a valid degree the reference accepts, beyond this backend's 2^17 limit:
    # the capacity status, not the reference's InvalidDegree (basis.rs:22-24)
    assert e.value.kind == "Unsupported" and e.value.code == 12
    assert e.value.fields == {"degree": 1 << 18, "max_degree": 1 << 17}
    # EmptyBasis comes before the degree check (basis.rs:97-100)
    with pytest.raises(rns_ntt.RnsNttError) as e:
        rns_ntt.RnsBasis([], 12)
    assert e.value.kind == "EmptyBasis"


def test_error_detail_through_the_abi():
    """rnt_last_error_detail returns the failing call's status and the
    reference variant's fields (errors.rs:4-20), per thread."""
    lib = rns_ntt.load()
    f = (ctypes.c_uint64 * 2)()
    psi = ctypes.c_uint64()
    assert lib.rnt_find_psi(19, 8, ctypes.byref(psi)) == 3
    assert lib.rnt_last_error_detail(f) == 3 and (f[0], f[1]) == (19, 8)
    assert lib.rnt_find_psi(17, 12, ctypes.byref(psi)) == 1
    assert lib.rnt_last_error_detail(f) == 1 and (f[0], f[1]) == (12, 0)
    assert lib.rnt_last_error_detail(None) == 1
    # a failure without a reference variant clears the fields
    assert lib.rnt_find_psi(17, 8, None) == 11
    assert lib.rnt_last_error_detail(f) == 11 and (f[0], f[1]) == (0, 0)
    # equality compares variant and payload, like the reference's PartialEq
    a = rns_ntt.RnsNttError(6, "x", {"coefficient": 17, "modulus": 17})
    assert a == rns_ntt.RnsNttError(6, "y", {"coefficient": 17, "modulus": 17})
    assert a != rns_ntt.RnsNttError(6, "x", {"coefficient": 18, "modulus": 17})


# ---- INTEGRATION.md's Rust extern block against include/rnsntt.h ----------

_C_SCALARS = {"int": "c_int", "uint64_t": "u64", "int64_t": "i64", "uint32_t": "u32",
              "int32_t": "i32", "size_t": "usize", "double": "f64", "char": "c_char",
              "void": "c_void", "rnt_ctx": "rnt_ctx", "rnt_buf": "rnt_buf", "rnt_graph": "rnt_graph"}


def _c_type_to_rust(ctype: str) -> str:
    """`const uint64_t*` -> `*const u64`, `rnt_ctx**` -> `*mut *mut rnt_ctx`,
    `uint64_t fields[2]` (array parameter) -> `*mut u64`."""
    t = ctype.strip()
    const = t.startswith("const ")
    base = t[6:] if const else t
    stars = base.count("*")
    base = base.replace("*", "").strip()
    rust = _C_SCALARS[base]
    if stars == 0:
        return rust
    out = ("*const " if const else "*mut ") + rust
    for _ in range(stars - 1):
        out = "*mut " + out
    return out


def _header_prototypes():
    text = open(os.path.join(REPO, "include", "rnsntt.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(rnt_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", text):
        ret, name, params = m.group(1).strip(), m.group(2), " ".join(m.group(3).split())
        args = []
        if params != "void":
            for p in params.split(","):
                p = p.strip()
                arr = re.match(r"(.*?)\s*(\w+)\s*\[\d*\]$", p)
                if arr:  # T name[k] decays to T*
                    args.append(_c_type_to_rust(arr.group(1) + "*"))
                else:
                    pm = re.match(r"(.*?[\s\*])(\w+)$", p)
                    args.append(_c_type_to_rust(pm.group(1)))
        protos[name] = (_c_type_to_rust(ret), args)
    return protos


def _rust_block_prototypes():
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    block = re.search(r'extern "C" \{(.*?)\n\}', text, flags=re.S).group(1)
    block = re.sub(r"//[^\n]*", "", block)
    protos = {}
    for m in re.finditer(r"pub fn (rnt_\w+)\((.*?)\)\s*(?:->\s*([^;]+))?;", block, flags=re.S):
        name, params, ret = m.group(1), " ".join(m.group(2).split()), (m.group(3) or "()").strip()
        args = [p.split(":", 1)[1].strip() for p in params.split(",") if p.strip()]
        assert name not in protos, f"{name} declared twice in INTEGRATION.md"
        protos[name] = (" ".join(ret.split()), [" ".join(a.split()) for a in args])
    return protos


def test_integration_rust_block_matches_header():
    """Every function of include/rnsntt.h has exactly one line in
    INTEGRATION.md's Rust extern block, with the same arity and the
    corresponding argument and return types (the block must
    carry rnt_to_coeffs, rnt_mod_drop_last, rnt_sub and the basis getters
    the shim needs for traits.rs:28-64 and basis.rs:108-145)."""
    c = _header_prototypes()
    r = _rust_block_prototypes()
    assert sorted(c) == declared_functions()
    assert sorted(r) == sorted(c), (sorted(set(c) - set(r)), sorted(set(r) - set(c)))
    for name, (ret, args) in c.items():
        rret, rargs = r[name]
        assert rret == ret, (name, rret, ret)
        assert len(rargs) == len(args), (name, rargs, args)
        assert rargs == args, (name, rargs, args)
    for needed in ("rnt_to_coeffs", "rnt_mod_drop_last", "rnt_sub", "rnt_ctx_moduli",
                   "rnt_ctx_total_bits", "rnt_ctx_channel_count"):
        assert needed in r


# ---- the Makefile's dependency lists against the sources' #include lines ---

def _local_includes(path, seen=None):
    """Every header `path` includes with #include "...", transitively, as
    repo-relative paths."""
    import re

    seen = set() if seen is None else seen
    base = os.path.dirname(path)
    for line in open(path):
        m = re.match(r'\s*#\s*include\s+"([^"]+)"', line)
        if not m:
            continue
        h = os.path.normpath(os.path.join(base, m.group(1)))
        rel = os.path.relpath(h, REPO)
        if rel not in seen:
            seen.add(rel)
            _local_includes(h, seen)
    return seen


def test_makefile_dependencies_match_includes():
    """a `make` build must rebuild an object when any
    header it includes changes, so each DEP_<tu> list in the Makefile equals
    the transitive closure of that translation unit's #include lines, every
    TU build() compiles has one, and `all` runs the ISA hazard check."""
    import re

    sys.path.insert(0, REPO)
    import __graft_entry__ as ge

    mk = open(os.path.join(REPO, "Makefile")).read().replace("\\\n", " ")
    deps = {m.group(1): set(m.group(2).split()) for m in re.finditer(r"^DEP_(\w+)\s*:=\s*(.*)$", mk, re.M)}
    for src in ge.SOURCES:
        tu = os.path.splitext(src)[0]
        assert tu in deps, f"Makefile has no DEP_{tu}"
        want = _local_includes(os.path.join(ge.CSRC, src))
        got = {d.replace("$(CSRC)", "toy-heaan-ckks_amd/csrc") for d in deps[tu]}
        assert got == want, f"DEP_{tu}: Makefile {sorted(got)} vs #include closure {sorted(want)}"
        assert re.search(rf"^\$\(LIBDIR\)/{tu}\.o:\s*\$\(CSRC\)/{re.escape(src)}\s+\$\(DEP_{tu}\)\s*$", mk, re.M), tu
    all_line = re.search(r"^all:(.*)$", mk, re.M).group(1)
    assert "isa_check.ok" in all_line
    assert re.search(r"^\t.*tools/isa_check\.py \$\(OBJS\)", mk, re.M)
