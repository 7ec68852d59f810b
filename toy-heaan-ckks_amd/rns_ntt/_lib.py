"""ctypes binding of librnsntt.so (include/rnsntt.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make``) into ``toy-heaan-ckks_amd/lib/librnsntt.so``.  There is no CPU
fallback: if the library is missing, importing the compute API raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_int, c_int32, c_int64, c_size_t, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "librnsntt.so")

# status codes (include/rnsntt.h); 1..6 mirror RnsNttError
# (src/rings/backends/rns_ntt/errors.rs:4-20)
OK = 0
INVALID_DEGREE = 1
EMPTY_BASIS = 2
NON_NTT_FRIENDLY = 3
INVALID_MOD_DROP = 4
CHANNEL_COUNT = 5
NON_REDUCED = 6
DOMAIN_MISMATCH = 7
BASIS_MISMATCH = 8
DEVICE = 9
OUT_OF_MEMORY = 10
BAD_ARGUMENT = 11
UNSUPPORTED = 12  # beyond this backend's capacity (degree > 2^17); no reference variant

STATUS_NAMES = {
    1: "InvalidDegree",
    2: "EmptyBasis",
    3: "NonNttFriendlyModulus",
    4: "InvalidModDrop",
    5: "ChannelCountMismatch",
    6: "NonReducedCoefficient",
    7: "DomainMismatch",
    8: "BasisMismatch",
    9: "DeviceError",
    10: "OutOfMemory",
    11: "BadArgument",
    12: "Unsupported",
}


# the fields of each reference variant, in rnt_last_error_detail's order
FIELD_NAMES = {
    1: ("degree",),
    2: (),
    3: ("modulus", "degree"),
    4: ("drop_count", "channel_count"),
    5: ("expected", "actual"),
    6: ("coefficient", "modulus"),
    12: ("degree", "max_degree"),
}


class RnsNttError(Exception):
    """Mirror of RnsNttError (errors.rs:4-20) plus the C-ABI's extra codes.

    ``kind`` is the variant name and ``fields`` its payload, e.g.
    ``NonReducedCoefficient`` carries ``{"coefficient": c, "modulus": q}``;
    each field is also an attribute (``err.coefficient``)."""

    def __init__(self, code: int, message: str, fields: dict | None = None):
        self.code = code
        self.kind = STATUS_NAMES.get(code, "Unknown")
        self.fields = dict(fields or {})
        for k, v in self.fields.items():
            setattr(self, k, v)
        super().__init__(f"{self.kind}: {message}")

    def __eq__(self, other):  # variant equality, like the reference's PartialEq
        return isinstance(other, RnsNttError) and (self.code, self.fields) == (other.code, other.fields)

    __hash__ = Exception.__hash__


_P = c_void_p
_U64P = POINTER(c_uint64)
_I64P = POINTER(c_int64)

# name -> (restype, argtypes); every declaration of include/rnsntt.h
SIGNATURES = {
    "rnt_abi_version": (c_int, []),
    "rnt_last_error": (c_char_p, []),
    "rnt_last_error_detail": (c_int, [_U64P]),
    "rnt_pool_trim": (c_int, [c_int, POINTER(c_size_t)]),
    "rnt_status_string": (c_char_p, [c_int]),
    "rnt_device_count": (c_int, [POINTER(c_int)]),
    "rnt_profile_enable": (c_int, [_P, c_int]),
    "rnt_profile_read": (c_int, [_P, c_char_p, POINTER(c_uint64), POINTER(ctypes.c_double)]),
    "rnt_debug_defer": (c_int, [c_int]),
    "rnt_is_ntt_friendly_prime": (c_int, [c_uint64, c_uint64, POINTER(c_int)]),
    "rnt_generate_primes": (c_int, [c_uint32, c_size_t, c_uint64, _U64P]),
    "rnt_find_psi": (c_int, [c_uint64, c_uint64, _U64P]),
    "rnt_ctx_create": (c_int, [c_uint32, _U64P, c_size_t, c_int, POINTER(_P)]),
    "rnt_ctx_destroy": (c_int, [_P]),
    "rnt_ctx_drop_last": (c_int, [_P, c_size_t, POINTER(_P)]),
    "rnt_ctx_degree": (c_int, [_P, POINTER(c_size_t)]),
    "rnt_ctx_channel_count": (c_int, [_P, POINTER(c_size_t)]),
    "rnt_ctx_moduli": (c_int, [_P, _U64P]),
    "rnt_ctx_total_bits": (c_int, [_P, POINTER(c_uint32)]),
    "rnt_ctx_psi": (c_int, [_P, c_size_t, _U64P]),
    "rnt_ctx_stream": (c_int, [_P, POINTER(_P)]),
    "rnt_ctx_set_stream": (c_int, [_P, c_void_p]),
    "rnt_sync": (c_int, [_P]),
    "rnt_capture_begin": (c_int, [_P]),
    "rnt_capture_end": (c_int, [_P, POINTER(_P)]),
    "rnt_graph_launch": (c_int, [_P]),
    "rnt_graph_destroy": (c_int, [_P]),
    "rnt_graph_workspace": (c_int, [_P, POINTER(c_size_t), POINTER(c_size_t)]),
    "rnt_buf_alloc": (c_int, [_P, c_size_t, POINTER(_P)]),
    "rnt_buf_alloc_uninit": (c_int, [_P, c_size_t, POINTER(_P)]),
    "rnt_buf_free": (c_int, [_P]),
    "rnt_buf_n_polys": (c_int, [_P, POINTER(c_size_t)]),
    "rnt_buf_is_ntt": (c_int, [_P, POINTER(c_int)]),
    "rnt_upload": (c_int, [_P, _U64P, c_size_t, c_size_t, c_int]),
    "rnt_upload_coeffs": (c_int, [_P, _I64P, c_size_t]),
    "rnt_download": (c_int, [_P, _U64P, c_size_t]),
    "rnt_download_polys": (c_int, [_P, _U64P, c_size_t, c_size_t]),
    "rnt_copy": (c_int, [_P, _P]),
    "rnt_to_coeffs": (c_int, [_P, c_void_p, c_size_t]),
    "rnt_crt_centered": (c_int, [_P, c_void_p, c_size_t, c_size_t]),
    "rnt_buf_wrap": (c_int, [_P, c_void_p, c_size_t, c_int, POINTER(c_void_p)]),
    "rnt_buf_device_ptr": (c_int, [_P, POINTER(c_void_p), POINTER(c_size_t)]),
    "rnt_ct_tensor": (c_int, [_P, _P, _P, _P, _P, _P, _P]),
    "rnt_keyswitch_ext": (c_int, [_P, _P, c_void_p, c_size_t, _P, _P, _P, _P]),
    "rnt_rescale_ext": (c_int, [_P, _P, c_void_p, c_uint64]),
    "rnt_ntt_fwd": (c_int, [_P]),
    "rnt_ntt_inv": (c_int, [_P]),
    "rnt_mul": (c_int, [_P, _P, _P]),
    "rnt_add": (c_int, [_P, _P, _P]),
    "rnt_sub": (c_int, [_P, _P, _P]),
    "rnt_neg": (c_int, [_P, _P]),
    "rnt_rescale": (c_int, [_P, _P]),
    "rnt_mod_drop_last": (c_int, [_P, _P]),
    "rnt_automorphism": (c_int, [_P, _P, c_uint64]),
    "rnt_rotate_slots": (c_int, [_P, _P, c_int32]),
    "rnt_key_prepare": (c_int, [_P, _P]),
    "rnt_keyswitch": (c_int, [_P, _P, _P, _P, _P]),
    "rnt_ct_mul_relin": (c_int, [_P, _P, _P, _P, _P, _P, _P, _P]),
    "rnt_ct_mul_relin_rescale": (c_int, [_P, _P, _P, _P, _P, _P, _P, _P]),
    "rnt_ct_rotate": (c_int, [_P, _P, _P, _P, c_int32, _P, _P]),
    "rnt_ct_rescale": (c_int, [_P, _P, _P, _P]),
    "rnt_encode": (c_int, [_P, c_void_p, c_size_t, c_uint32]),
    "rnt_decode": (c_int, [_P, c_void_p, c_size_t, c_uint32]),
    "rnt_sample_uniform": (c_int, [_P, c_uint64, c_uint64]),
    "rnt_sample_gaussian": (c_int, [_P, ctypes.c_double, c_uint64, c_uint64]),
    "rnt_sample_ternary": (c_int, [_P, c_size_t, c_uint64, c_uint64]),
}

_lib = None


def load(path: str | None = None) -> ctypes.CDLL:
    """Load librnsntt.so once; raise loudly if it was not built.  RNSNTT_LIB
    overrides the path (tools/ab.sh compares build variants of the same
    library on one box)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("RNSNTT_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError(
            f"librnsntt.so not found at {path}: build it with `make` or "
            "`python -c 'import __graft_entry__ as g; g.build()'` (there is no CPU fallback)"
        )
    # One HIP runtime per process: the torch wheel bundles its own
    # libamdhip64.so.7, and whichever copy loads first serves both.  Loading
    # /opt/rocm's first leaves torch without a GPU ("No HIP GPUs are
    # available"), so when torch is installed it is imported before the
    # library binds its runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error_fields(status: int) -> dict:
    """The reference variant's fields of the last failing call on this
    thread (rnt_last_error_detail), named as in errors.rs:4-20."""
    raw = (c_uint64 * 2)()
    if load().rnt_last_error_detail(raw) != status:
        return {}
    return {name: int(raw[i]) for i, name in enumerate(FIELD_NAMES.get(status, ()))}


def check(status: int) -> None:
    if status != OK:
        msg = load().rnt_last_error()
        raise RnsNttError(status, msg.decode() if msg else "", last_error_fields(status))
