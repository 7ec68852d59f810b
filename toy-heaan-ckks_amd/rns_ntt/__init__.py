"""Host-side mirror of oiwn/toy-heaan-ckks's RNS-NTT ring interface over the
MI355X C-ABI (include/rnsntt.h).

Names, argument meaning and error behaviour follow the reference:

* :class:`RnsBasis`  -- ``RnsBasis<N>`` (src/rings/backends/rns_ntt/basis.rs:90-180)
* :class:`RnsPoly`   -- ``RnsPoly<N>`` (src/rings/backends/rns_ntt/poly.rs:25-570);
  one object holds a *batch* of ``n_polys`` polynomials that every op
  processes together (``n_polys=1`` is the reference's single polynomial).
* :func:`mul_ciphertexts_gadget`, :func:`rotate_ciphertext`,
  :func:`rescale_ciphertext` -- ``CkksEngine`` (src/crypto/engine.rs:263-539).
* :class:`RnsNttError` -- ``RnsNttError`` (errors.rs:4-20), raised with the
  same variant name.

All arithmetic runs in librnsntt.so on the GPU.  Host code here only moves
data across the boundary (``from_channels`` / ``channels``) and does the
reference's decode-side u128 CRT in :meth:`RnsPoly.to_coeffs`.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import RnsNttError, check, load

__all__ = [
    "device_count",
    "RnsNttError",
    "RnsBasis",
    "RnsPoly",
    "RnsGadgetKey",
    "Ciphertext",
    "generate_primes",
    "is_ntt_friendly_prime",
    "find_psi",
    "keyswitch",
    "mul_ciphertexts_gadget",
    "mul_ciphertexts_gadget_rescale",
    "rotate_ciphertext",
    "rescale_ciphertext",
    "Plaintext",
    "CkksEncoder",
    "DeviceRng",
    "pool_trim",
    "Graph",
]


def _u64p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def _i64p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))


# ---------------------------------------------------------------------------
# host-side number theory (setup)
# ---------------------------------------------------------------------------


def device_count() -> int:
    """Visible HIP devices (0 on a CPU-only host)."""
    r = ctypes.c_int(0)
    check(load().rnt_device_count(ctypes.byref(r)))
    return int(r.value)


def pool_trim(device: int = -1) -> int:
    """Release the device block cache's idle blocks (of one device, or all
    with -1) back to HIP; returns the bytes released.  Call it when another
    allocator (torch's) runs out of memory before retrying."""
    freed = ctypes.c_size_t(0)
    check(load().rnt_pool_trim(int(device), ctypes.byref(freed)))
    return int(freed.value)


def generate_primes(bit_size: int, count: int, degree: int) -> list[int]:
    """src/math/utils.rs:47-80."""
    out = np.zeros(max(count, 1), dtype=np.uint64)
    check(load().rnt_generate_primes(bit_size, count, degree, _u64p(out)))
    return [int(x) for x in out[:count]]


def is_ntt_friendly_prime(p: int, n: int) -> bool:
    """src/math/primes.rs:125-131."""
    r = ctypes.c_int(0)
    check(load().rnt_is_ntt_friendly_prime(p, n, ctypes.byref(r)))
    return bool(r.value)


def find_psi(modulus: int, degree: int) -> int:
    """psi of NttTable::new (basis.rs:39-40, 217-237)."""
    r = ctypes.c_uint64(0)
    check(load().rnt_find_psi(modulus, degree, ctypes.byref(r)))
    return int(r.value)


class DeviceRng:
    """The seeded generator passed where the reference passes ``&mut rng``
    to a PolySampler (traits.rs:74-127).  Every sampler call takes the next
    stream of the device's counter-based Philox4x32-10 generator
    (rnt_sample_*), so a seed fixes every later sample, as a seeded
    ChaCha20Rng does in the reference (whose streams are not reproduced)."""

    def __init__(self, seed: int):
        self.seed = int(seed) & ((1 << 64) - 1)
        self.stream = 0

    def next_stream(self) -> int:
        s = self.stream
        self.stream += 1
        return s


# ---------------------------------------------------------------------------
# RnsBasis
# ---------------------------------------------------------------------------


class RnsBasis:
    """``Arc<RnsBasis<N>>``: an immutable RNS basis with device NTT tables.

    ``RnsBasis(moduli, degree)`` validates like ``RnsBasis::new``
    (basis.rs:97-106): ``EmptyBasis`` for no moduli, ``InvalidDegree`` for a
    non power-of-two degree, ``NonNttFriendlyModulus`` otherwise; a valid
    degree above 2^17 raises ``Unsupported`` (this backend's capacity).
    """

    def __init__(self, moduli: Sequence[int], degree: int, device: int = 0):
        lib = load()
        # basis.rs:97-106 order: EmptyBasis first (rnt_ctx_create checks it),
        # then per modulus NttTable::new's InvalidDegree (basis.rs:22-24: not a
        # power of two) and NonNttFriendlyModulus.  A power-of-two degree
        # above this backend's 2^17 is Unsupported (status 12), never
        # InvalidDegree.
        if len(moduli) and (degree <= 0 or degree & (degree - 1)):
            raise RnsNttError(_lib.INVALID_DEGREE, f"ring degree must be a power of two, got {degree}",
                              {"degree": degree})
        log_n = degree.bit_length() - 1 if degree > 0 and not degree & (degree - 1) else 0
        arr = np.ascontiguousarray(np.array(list(moduli), dtype=np.uint64)) if len(moduli) else np.zeros(1, np.uint64)
        h = ctypes.c_void_p()
        check(lib.rnt_ctx_create(log_n, _u64p(arr), len(moduli), device, ctypes.byref(h)))
        self._h = h
        self._parent = None
        self.degree = degree
        self.device = device

    @classmethod
    def _from_handle(cls, h, parent: "RnsBasis") -> "RnsBasis":
        self = cls.__new__(cls)
        self._h = h
        self._parent = parent  # keeps the shared tables' owner reachable
        self.degree = parent.degree
        self.device = parent.device
        return self

    @property
    def handle(self):
        return self._h

    def moduli(self) -> list[int]:
        out = np.zeros(self.channel_count(), dtype=np.uint64)
        check(load().rnt_ctx_moduli(self._h, _u64p(out)))
        return [int(x) for x in out]

    def channel_count(self) -> int:
        r = ctypes.c_size_t(0)
        check(load().rnt_ctx_channel_count(self._h, ctypes.byref(r)))
        return int(r.value)

    def drop_last(self, drop_count: int) -> "RnsBasis":
        """basis.rs:121-134 (a view sharing the device tables)."""
        h = ctypes.c_void_p()
        check(load().rnt_ctx_drop_last(self._h, drop_count, ctypes.byref(h)))
        return RnsBasis._from_handle(h, self)

    def total_bits(self) -> int:
        r = ctypes.c_uint32(0)
        check(load().rnt_ctx_total_bits(self._h, ctypes.byref(r)))
        return int(r.value)

    def psi(self, limb: int) -> int:
        r = ctypes.c_uint64(0)
        check(load().rnt_ctx_psi(self._h, limb, ctypes.byref(r)))
        return int(r.value)

    def stream(self) -> int:
        r = ctypes.c_void_p()
        check(load().rnt_ctx_stream(self._h, ctypes.byref(r)))
        return int(r.value or 0)

    def set_stream(self, stream=None) -> None:
        """Queue later ops on ``stream`` (a raw hipStream_t address or a
        ``torch.cuda.Stream``; None: the basis' own stream), after everything
        queued so far.  Shared with every drop_last view of this basis."""
        if stream is not None and not isinstance(stream, int):
            stream = int(stream.cuda_stream)
        check(load().rnt_ctx_set_stream(self._h, ctypes.c_void_p(stream or None)))

    def sync(self) -> None:
        check(load().rnt_sync(self._h))

    def capture(self) -> "Graph":
        """Record the device ops this thread queues on the basis' stream
        inside ``with basis.capture() as g:`` into a HIP graph instead of
        running them; ``g.replay()`` then re-runs the whole sequence (same
        buffers) as one launch (rnt_capture_begin / rnt_graph_launch).  Run
        the sequence once before recording it, so its workspaces are cached;
        only device ops may be recorded (no from_channels / channels / sync)."""
        return Graph(self)

    def profile_enable(self, enable: bool = True) -> None:
        """Bracket every kernel launched on this basis' stream with HIP events."""
        check(load().rnt_profile_enable(self._h, 1 if enable else 0))

    def profile_read(self, kernel: str) -> tuple[int, float]:
        """(launches, summed device ms) for one kernel since profile_enable."""
        n = ctypes.c_uint64(0)
        ms = ctypes.c_double(0)
        check(load().rnt_profile_read(self._h, kernel.encode(), ctypes.byref(n), ctypes.byref(ms)))
        return int(n.value), float(ms.value)

    def reconstruct_centered_coeff(self, residues: Sequence[int]) -> int:
        """basis.rs:158-180 (host-side decode; the reference needs Q < 2^128)."""
        mods = self.moduli()
        Q = 1
        for m in mods:
            Q *= m
        if Q >= 1 << 128:
            raise OverflowError("reconstruct_centered_coeff requires Q < 2^128 (basis.rs:152-157)")
        acc = 0
        for r, m in zip(residues, mods):
            qi = Q // m
            acc = (acc + (int(r) * pow(qi % m, -1, m) % m) * qi) % Q
        return acc - Q if acc > Q // 2 else acc

    def __del__(self, _lib=_lib):  # module globals may be gone at interpreter exit
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib is not None and _lib._lib is not None:
            _lib._lib.rnt_ctx_destroy(h)
            self._h = None


class Graph:
    """A recorded op sequence (see RnsBasis.capture)."""

    def __init__(self, basis: "RnsBasis"):
        self.basis = basis
        self._h = None

    def __enter__(self) -> "Graph":
        check(load().rnt_capture_begin(self.basis.handle))
        return self

    def __exit__(self, exc_type, exc, tb) -> None:
        h = ctypes.c_void_p()
        rc = load().rnt_capture_end(self.basis.handle, ctypes.byref(h))
        if exc_type is None:
            check(rc)
            self._h = h
        elif rc == 0 and h.value:
            # the body raised: the graph (and the workspace it holds) is never replayed
            load().rnt_graph_destroy(h)

    def workspace(self) -> tuple[int, int]:
        """(blocks, bytes) of device workspace the recorded graph holds."""
        if self._h is None:
            raise RuntimeError("graph was not recorded")
        blocks, nbytes = ctypes.c_size_t(), ctypes.c_size_t()
        check(load().rnt_graph_workspace(self._h, ctypes.byref(blocks), ctypes.byref(nbytes)))
        return int(blocks.value), int(nbytes.value)

    def replay(self) -> None:
        if self._h is None:
            raise RuntimeError("graph was not recorded")
        check(load().rnt_graph_launch(self._h))

    def __del__(self, _lib=_lib):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib is not None and _lib._lib is not None:
            _lib._lib.rnt_graph_destroy(h)
            self._h = None


# ---------------------------------------------------------------------------
# RnsPoly
# ---------------------------------------------------------------------------


class RnsPoly:
    """A batch of ``n_polys`` polynomials in Z_{q_0} x ... x Z_{q_{L-1}}[X]/(X^N+1).

    Mirrors ``RnsPoly<N>`` (poly.rs:25-570).  Operators follow the Rust ones:
    ``a *= b`` (MulAssign), ``a += b`` (AddAssign), ``-a`` (Neg).

    An object is either the reference's single polynomial (built without a
    batch count: ``RnsPoly(basis)``, ``from_channels([L][N])``,
    ``from_coeffs([N])``, ``sample_*(...)`` without ``n_polys``) or a batch
    (``RnsPoly(basis, B)``, ``from_channels([B][L][N])`` ...), and every
    result of an op is of the same kind as its input.  Host views follow the
    kind, never the batch size: ``channels()`` is [L][N] for a single
    polynomial and [B][L][N] for a batch (also when B == 1);
    ``channels_batch()`` is always [B][L][N].
    """

    def __init__(self, basis: RnsBasis, n_polys: Optional[int] = None, _uninit: bool = False):
        lib = load()
        h = ctypes.c_void_p()
        count = 1 if n_polys is None else int(n_polys)
        alloc = lib.rnt_buf_alloc_uninit if _uninit else lib.rnt_buf_alloc
        check(alloc(basis.handle, count, ctypes.byref(h)))
        self._h = h
        self.basis = basis
        self.n_polys = count
        self.batched = n_polys is not None

    def _like(self, basis: Optional[RnsBasis] = None) -> "RnsPoly":
        """An op output of this object's kind and batch on ``basis``: its
        contents are unspecified until the op (which writes every word)
        fills it, so no zero fill is queued (rnt_buf_alloc_uninit)."""
        return RnsPoly(basis or self.basis, self.n_polys if self.batched else None, _uninit=True)

    # -- constructors (poly.rs:34-114) --------------------------------------
    @classmethod
    def zero(cls, basis: RnsBasis, n_polys: Optional[int] = None) -> "RnsPoly":
        return cls(basis, n_polys)

    @classmethod
    def from_coeffs(cls, coeffs, basis: RnsBasis) -> "RnsPoly":
        """poly.rs:49-67; ``coeffs`` is [N] or [B][N] signed integers."""
        c = np.asarray(coeffs, dtype=np.int64)
        single = c.ndim == 1
        if single:
            c = c[None, :]
        if c.shape[1] < basis.degree:
            raise ValueError(f"from_coeffs: need at least {basis.degree} coefficients, got {c.shape[1]}")
        c = np.ascontiguousarray(c[:, : basis.degree])
        p = cls(basis, None if single else c.shape[0])
        check(load().rnt_upload_coeffs(p._h, _i64p(c), c.shape[0]))
        return p

    @classmethod
    def from_channels(cls, channels, basis: RnsBasis, in_ntt_domain: bool = False) -> "RnsPoly":
        """poly.rs:73-99; ``channels`` is [L][N] or [B][L][N] residues.

        Raises ChannelCountMismatch / NonReducedCoefficient like the reference.
        """
        ch = np.asarray(channels, dtype=np.uint64)
        single = ch.ndim == 2
        if single:
            ch = ch[None, :, :]
        if ch.ndim != 3 or ch.shape[2] != basis.degree:
            raise ValueError("from_channels: expected [L][N] or [B][L][N] with N == degree")
        ch = np.ascontiguousarray(ch)
        p = cls(basis, None if single else ch.shape[0])
        check(load().rnt_upload(p._h, _u64p(ch), ch.shape[0], ch.shape[1], 1 if in_ntt_domain else 0))
        return p

    @classmethod
    def wrap(cls, basis: RnsBasis, device_ptr: int, n_polys: int, in_ntt_domain: bool = False,
             owner=None) -> "RnsPoly":
        """A non-owning view of caller device memory laid out [L][n_polys][N]
        in the basis' device word width (``word_bytes``); ``owner`` (e.g. the
        torch tensor holding the memory) is kept alive with the view.  Used
        by the limb-sharded pipeline to hand buffers to RCCL collectives."""
        p = cls.__new__(cls)
        h = ctypes.c_void_p()
        check(load().rnt_buf_wrap(basis.handle, ctypes.c_void_p(device_ptr), n_polys,
                                  1 if in_ntt_domain else 0, ctypes.byref(h)))
        p._h = h
        p.basis = basis
        p.n_polys = n_polys
        p.batched = True
        p._owner = owner
        return p

    # -- PolySampler (traits.rs:74-127; poly.rs:438-477), on the device -----
    @classmethod
    def sample_uniform(cls, basis: RnsBasis, rng: DeviceRng, n_polys: Optional[int] = None) -> "RnsPoly":
        p = cls(basis, n_polys)
        check(load().rnt_sample_uniform(p._h, rng.seed, rng.next_stream()))
        return p

    @classmethod
    def sample_gaussian(cls, std_dev: float, basis: RnsBasis, rng: DeviceRng, n_polys: Optional[int] = None) -> "RnsPoly":
        p = cls(basis, n_polys)
        check(load().rnt_sample_gaussian(p._h, float(std_dev), rng.seed, rng.next_stream()))
        return p

    @classmethod
    def sample_tribits(cls, hamming_weight: int, basis: RnsBasis, rng: DeviceRng, n_polys: Optional[int] = None) -> "RnsPoly":
        p = cls(basis, n_polys)
        check(load().rnt_sample_ternary(p._h, int(hamming_weight), rng.seed, rng.next_stream()))
        return p

    @classmethod
    def sample_noise(cls, variance: float, basis: RnsBasis, rng: DeviceRng, n_polys: Optional[int] = None) -> "RnsPoly":
        """poly.rs:471-477: Gaussian with std_dev = sqrt(variance)."""
        return cls.sample_gaussian(float(np.sqrt(variance)), basis, rng, n_polys)

    def device_ptr(self) -> tuple[int, int]:
        """(device address of the [L][B][N] storage, word bytes)."""
        ptr = ctypes.c_void_p()
        wb = ctypes.c_size_t()
        check(load().rnt_buf_device_ptr(self._h, ctypes.byref(ptr), ctypes.byref(wb)))
        return int(ptr.value or 0), int(wb.value)

    # -- accessors (poly.rs:118-129) ----------------------------------------
    @property
    def handle(self):
        return self._h

    def channels(self) -> np.ndarray:
        """poly.rs:119-121: [L][N] for a single polynomial, [B][L][N] for a
        batch object (whatever its size; see the class docstring)."""
        out = self.channels_batch()
        return out if self.batched else out[0]

    def channels_batch(self) -> np.ndarray:
        """[B][L][N] always (B = 1 for a single polynomial)."""
        out = np.zeros((self.n_polys, self.basis.channel_count(), self.basis.degree), dtype=np.uint64)
        check(load().rnt_download(self._h, _u64p(out), self.n_polys))
        return out

    def channels_of(self, first: int, count: int = 1) -> np.ndarray:
        """[count][L][N]: channels of polys first .. first+count-1 of the batch."""
        out = np.zeros((count, self.basis.channel_count(), self.basis.degree), dtype=np.uint64)
        check(load().rnt_download_polys(self._h, _u64p(out), int(first), int(count)))
        return out

    def is_ntt_domain(self) -> bool:
        r = ctypes.c_int(0)
        check(load().rnt_buf_is_ntt(self._h, ctypes.byref(r)))
        return bool(r.value)

    def clone(self) -> "RnsPoly":
        p = self._like()
        check(load().rnt_copy(p._h, self._h))
        return p

    # -- domain conversion (poly.rs:136-166) --------------------------------
    def to_ntt_domain(self) -> None:
        check(load().rnt_ntt_fwd(self._h))

    def to_coeff_domain(self) -> None:
        check(load().rnt_ntt_inv(self._h))

    # -- arithmetic (poly.rs:254-385) ---------------------------------------
    def __imul__(self, rhs: "RnsPoly") -> "RnsPoly":
        check(load().rnt_mul(self._h, self._h, rhs._h))
        return self

    def __iadd__(self, rhs: "RnsPoly") -> "RnsPoly":
        check(load().rnt_add(self._h, self._h, rhs._h))
        return self

    def __isub__(self, rhs: "RnsPoly") -> "RnsPoly":
        check(load().rnt_sub(self._h, self._h, rhs._h))
        return self

    def __mul__(self, rhs: "RnsPoly") -> "RnsPoly":
        out = self._like()
        check(load().rnt_mul(out._h, self._h, rhs._h))
        return out

    def __add__(self, rhs: "RnsPoly") -> "RnsPoly":
        out = self._like()
        check(load().rnt_add(out._h, self._h, rhs._h))
        return out

    def __sub__(self, rhs: "RnsPoly") -> "RnsPoly":
        out = self._like()
        check(load().rnt_sub(out._h, self._h, rhs._h))
        return out

    def __neg__(self) -> "RnsPoly":
        out = self._like()
        check(load().rnt_neg(out._h, self._h))
        return out

    # -- rescale / mod-drop (poly.rs:168-249) -------------------------------
    def rescale_into(self, new_basis: RnsBasis) -> "RnsPoly":
        out = self._like(new_basis)
        check(load().rnt_rescale(out._h, self._h))
        return out

    def rescale(self) -> "RnsPoly":
        if self.basis.channel_count() < 2:
            raise RnsNttError(_lib.INVALID_MOD_DROP,
                              f"invalid mod-drop count 1 for {self.basis.channel_count()} channels",
                              {"drop_count": 1, "channel_count": self.basis.channel_count()})
        return self.rescale_into(self.basis.drop_last(1))

    def mod_drop_last(self, drop_count: int) -> "RnsPoly":
        nb = self.basis.drop_last(drop_count)
        out = self._like(nb)
        check(load().rnt_mod_drop_last(out._h, self._h))
        return out

    # -- automorphisms (poly.rs:482-570) ------------------------------------
    def automorphism(self, exponent: int) -> "RnsPoly":
        out = self._like()
        check(load().rnt_automorphism(out._h, self._h, exponent))
        return out

    def rotate_slots(self, k: int) -> "RnsPoly":
        out = self._like()
        check(load().rnt_rotate_slots(out._h, self._h, k))
        return out

    # -- PolyRing::to_coeffs (poly.rs:404-427) ------------------------------
    def to_coeffs(self) -> np.ndarray:
        """PolyRing::to_coeffs (poly.rs:404-427): the centred CRT value of each
        coefficient as i64 (its low 64 bits, like the reference), computed on
        the device (rnt_to_coeffs)."""
        out = np.zeros((self.n_polys, self.basis.degree), dtype=np.int64)
        check(load().rnt_to_coeffs(self._h, out.ctypes.data_as(ctypes.c_void_p), self.n_polys))
        return out if self.batched else out[0]

    def to_coeffs_exact(self) -> list:
        """The centred CRT values as Python ints for any Q (rnt_crt_centered):
        [N] for a single polynomial, [B][N] nested lists for a batch object."""
        bits = sum(int(q).bit_length() for q in self.basis.moduli())
        words = max(1, (bits + 1 + 63) // 64)
        raw = np.zeros((self.n_polys, self.basis.degree, words), dtype=np.uint64)
        check(load().rnt_crt_centered(self._h, raw.ctypes.data_as(ctypes.c_void_p), self.n_polys, words))
        out = []
        for b in range(self.n_polys):
            row = []
            for i in range(self.basis.degree):
                v = 0
                for w in range(words - 1, -1, -1):
                    v = (v << 64) | int(raw[b, i, w])
                if v >> (64 * words - 1):  # two's complement sign
                    v -= 1 << (64 * words)
                row.append(v)
            out.append(row)
        return out if self.batched else out[0]

    def __del__(self, _lib=_lib):  # module globals may be gone at interpreter exit
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib is not None and _lib._lib is not None:
            _lib._lib.rnt_buf_free(h)
            self._h = None


# ---------------------------------------------------------------------------
# engine-level ops (src/crypto/engine.rs)
# ---------------------------------------------------------------------------


class RnsGadgetKey:
    """RnsGadgetRelinKey / RnsGadgetRotationKey (engine.rs:224-253).

    ``a`` and ``b`` are RnsPoly batches holding the L key polynomials; they
    are made NTT-resident once by :meth:`prepare`.
    """

    def __init__(self, a: RnsPoly, b: RnsPoly, rotation: Optional[int] = None):
        self.a = a
        self.b = b
        self.rotation = rotation
        check(load().rnt_key_prepare(a.handle, b.handle))

    @classmethod
    def from_channels(cls, a_channels, b_channels, basis: RnsBasis, rotation: Optional[int] = None):
        """a_channels / b_channels: [L][L][N] coefficient-domain residues."""
        return cls(RnsPoly.from_channels(a_channels, basis), RnsPoly.from_channels(b_channels, basis), rotation)


@dataclass
class Ciphertext:
    """types.rs:27-35."""

    c0: RnsPoly
    c1: RnsPoly
    logp: int = 0
    logq: int = 0


def keyswitch(d: RnsPoly, key: RnsGadgetKey) -> tuple[RnsPoly, RnsPoly]:
    """Gadget sum (engine.rs:505-528 / 429-452) on a coefficient-domain batch."""
    acc0, acc1 = d._like(), d._like()
    check(load().rnt_keyswitch(acc0.handle, acc1.handle, d.handle, key.a.handle, key.b.handle))
    return acc0, acc1


def mul_ciphertexts_gadget(ct1: Ciphertext, ct2: Ciphertext, rlk: RnsGadgetKey) -> Ciphertext:
    """engine.rs:473-539."""
    assert ct1.logq == ct2.logq, "logq mismatch in gadget multiplication"
    basis = ct1.c0.basis
    out0, out1 = ct1.c0._like(basis), ct1.c0._like(basis)
    check(load().rnt_ct_mul_relin(out0.handle, out1.handle, ct1.c0.handle, ct1.c1.handle,
                                  ct2.c0.handle, ct2.c1.handle, rlk.a.handle, rlk.b.handle))
    return Ciphertext(out0, out1, ct1.logp + ct2.logp, ct1.logq)


def rotate_ciphertext(ct: Ciphertext, rotk: RnsGadgetKey) -> Ciphertext:
    """engine.rs:412-463."""
    basis = ct.c0.basis
    out0, out1 = ct.c0._like(basis), ct.c0._like(basis)
    check(load().rnt_ct_rotate(out0.handle, out1.handle, ct.c0.handle, ct.c1.handle,
                               int(rotk.rotation or 0), rotk.a.handle, rotk.b.handle))
    return Ciphertext(out0, out1, ct.logp, ct.logq)


def mul_ciphertexts_gadget_rescale(ct1: Ciphertext, ct2: Ciphertext, rlk: RnsGadgetKey) -> Ciphertext:
    """mul_ciphertexts_gadget then rescale_ciphertext (engine.rs:473-539,
    :263-282) as one op (rnt_ct_mul_relin_rescale): equal word for word to
    the two calls, with the rescale fused into the key-switch inverse."""
    assert ct1.logq == ct2.logq, "logq mismatch in gadget multiplication"
    q_last = ct1.c0.basis.moduli()[-1]
    bits_dropped = q_last.bit_length()
    new_basis = ct1.c0.basis.drop_last(1)
    out0, out1 = ct1.c0._like(new_basis), ct1.c0._like(new_basis)
    check(load().rnt_ct_mul_relin_rescale(out0.handle, out1.handle, ct1.c0.handle, ct1.c1.handle,
                                          ct2.c0.handle, ct2.c1.handle, rlk.a.handle, rlk.b.handle))
    return Ciphertext(out0, out1, ct1.logp + ct2.logp - bits_dropped, ct1.logq - bits_dropped)


def rescale_ciphertext(ct: Ciphertext) -> Ciphertext:
    """engine.rs:263-282: both components onto one shared dropped basis."""
    q_last = ct.c0.basis.moduli()[-1]
    bits_dropped = q_last.bit_length()
    new_basis = ct.c0.basis.drop_last(1)
    out0, out1 = ct.c0._like(new_basis), ct.c0._like(new_basis)
    check(load().rnt_ct_rescale(out0.handle, out1.handle, ct.c0.handle, ct.c1.handle))
    return Ciphertext(out0, out1, ct.logp - bits_dropped, ct.logq - bits_dropped)


# ---------------------------------------------------------------------------
# CKKS encoder (src/encoding/ckks_encoder.rs)
# ---------------------------------------------------------------------------


@dataclass
class Plaintext:
    """types.rs Plaintext: an encoded RnsPoly batch (one row of slots per
    poly), its scale and slot count."""

    poly: RnsPoly
    scale_bits: int
    slots: int


class CkksEncoder:
    """``CkksEncoder<DEGREE>`` (ckks_encoder.rs:32-157).  The canonical
    embedding runs on the device as an O(N log N) special FFT
    (rnt_encode / rnt_decode) instead of the reference's O(N^2) Vandermonde
    evaluation; a 2-D ``values`` encodes one poly per row."""

    def __init__(self, degree: int, scale_bits: int):
        if degree <= 0 or degree & (degree - 1):
            raise ValueError("CkksEncoder: DEGREE must be a power of two")
        if scale_bits <= 0:
            raise ValueError("CkksEncoder: scale_bits must be positive")
        self.degree = degree
        self.scale_bits = scale_bits

    def scale_factor(self) -> float:
        return 2.0 ** self.scale_bits

    def max_slots(self) -> int:
        return self.degree // 2

    def encode(self, values, basis: RnsBasis) -> Plaintext:
        """ckks_encoder.rs:65-82: real values, imaginary parts zero."""
        return self.encode_complex(np.asarray(values, dtype=np.float64), basis, _name="encode")

    def encode_complex(self, values, basis: RnsBasis, _name: str = "encode_complex") -> Plaintext:
        """ckks_encoder.rs:85-99."""
        if basis.degree != self.degree:
            raise ValueError(f"{_name}: basis degree {basis.degree} != encoder degree {self.degree}")
        v = np.asarray(values, dtype=np.complex128)
        rows = v.reshape(1, -1) if v.ndim <= 1 else v
        if rows.ndim != 2:
            raise ValueError(f"{_name}: values must be 1-D (one poly) or 2-D (one row per poly)")
        n_values = rows.shape[1]
        if n_values > self.degree // 2:
            raise ValueError(f"{_name}: {n_values} values exceed max slots {self.degree // 2}")
        buf = np.ascontiguousarray(rows)
        poly = RnsPoly(basis, None if v.ndim <= 1 else rows.shape[0])
        check(load().rnt_encode(poly.handle, buf.ctypes.data_as(ctypes.c_void_p), n_values, self.scale_bits))
        return Plaintext(poly, self.scale_bits, n_values)

    def decode(self, pt: Plaintext) -> np.ndarray:
        """ckks_encoder.rs:129-131."""
        return self.decode_complex(pt).real

    def decode_complex(self, pt: Plaintext) -> np.ndarray:
        """ckks_encoder.rs:134-156 (one row per poly of a batch object)."""
        B = pt.poly.n_polys
        out = np.zeros((B, pt.slots), dtype=np.complex128)
        check(load().rnt_decode(pt.poly.handle, out.ctypes.data_as(ctypes.c_void_p), pt.slots, pt.scale_bits))
        return out if pt.poly.batched else out[0]


# ---------------------------------------------------------------------------
# limb-sharded building blocks (include/rnsntt.h)
# ---------------------------------------------------------------------------


def ct_tensor(c0: RnsPoly, c1: RnsPoly, c0p: RnsPoly, c1p: RnsPoly,
              d2_out: Optional[RnsPoly] = None) -> tuple[RnsPoly, RnsPoly, RnsPoly]:
    """Tensor product (engine.rs:480-493) on this basis' limbs: d0, d1 in the
    NTT domain (key-switch seeds), d2 in the coefficient domain (written into
    ``d2_out`` when given, e.g. a wrapped collective buffer)."""
    d0, d1 = c0._like(), c0._like()
    d2 = d2_out if d2_out is not None else c0._like()
    check(load().rnt_ct_tensor(d0.handle, d1.handle, d2.handle, c0.handle, c1.handle,
                               c0p.handle, c1p.handle))
    return d0, d1, d2


def keyswitch_ext(src_ptr: int, src_limbs: int, key: RnsGadgetKey, basis: RnsBasis, n_polys: int,
                  init0: Optional[RnsPoly] = None, init1: Optional[RnsPoly] = None,
                  out0: Optional[RnsPoly] = None, out1: Optional[RnsPoly] = None
                  ) -> tuple[RnsPoly, RnsPoly]:
    """Gadget sum (engine.rs:505-528) for this basis' (target) limbs over
    ``src_limbs`` coefficient-domain source limbs at device address
    ``src_ptr`` ([src_limbs][n_polys][N] words); seeds in the NTT domain."""
    acc0 = out0 if out0 is not None else RnsPoly(basis, n_polys)
    acc1 = out1 if out1 is not None else RnsPoly(basis, n_polys)
    check(load().rnt_keyswitch_ext(acc0.handle, acc1.handle, ctypes.c_void_p(src_ptr), src_limbs,
                                   key.a.handle, key.b.handle,
                                   init0.handle if init0 is not None else None,
                                   init1.handle if init1 is not None else None))
    return acc0, acc1


def rescale_ext(x: RnsPoly, last_ptr: int, q_last: int, out_basis: RnsBasis,
                out: Optional[RnsPoly] = None) -> RnsPoly:
    """rescale_into (poly.rs:187-228) by an external last limb: residues mod
    ``q_last`` ([n_polys][N] words, coefficient domain) at ``last_ptr``."""
    o = out if out is not None else x._like(out_basis)
    check(load().rnt_rescale_ext(o.handle, x.handle, ctypes.c_void_p(last_ptr), int(q_last)))
    return o
