"""The C++ host mirror (toy-heaan-ckks_amd/host/rns_ntt.hpp) and its port of
the reference's RnsPoly unit tests (src/rings/backends/rns_ntt/poly.rs:658-1060,
tests/cpp/test_rns_poly.cpp)."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "cpp", "test_rns_poly.cpp")
LIB = os.path.join(REPO, "toy-heaan-ckks_amd", "lib")
BIN = os.path.join(REPO, "tests", "cpp", "bin", "test_rns_poly")


def _compile(out):
    subprocess.run(
        ["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(REPO, "include"),
         "-I", os.path.join(REPO, "toy-heaan-ckks_amd", "host"), SRC, "-L", LIB, "-lrnsntt",
         f"-Wl,-rpath,{LIB}", "-o", out],
        check=True, capture_output=True, text=True)


def test_host_mirror_compiles_and_links(tmp_path):
    """The header and the test build warning-free against the C-ABI library."""
    if not os.path.exists(os.path.join(LIB, "librnsntt.so")):
        pytest.skip("librnsntt.so not built (run __graft_entry__.build())")
    _compile(str(tmp_path / "t"))


@pytest.mark.gpu
def test_reference_poly_tests_pass_through_cpp_mirror(tmp_path):
    exe = BIN
    if not os.path.exists(exe):
        exe = str(tmp_path / "t")
        _compile(exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "FAIL" not in r.stdout
    last = r.stdout.strip().splitlines()[-1]
    done, total = last.split()[0].split("/")
    assert done == total and int(total) >= 28
