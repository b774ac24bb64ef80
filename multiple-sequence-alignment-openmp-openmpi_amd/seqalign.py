"""Host-side mirror of the reference's hot-path interface over the C-ABI.

The reference (yangxvlin/multiple-sequence-alignment-openMP-openMPI) exposes
the path as three C++ functions; this module keeps their names, argument
meaning and results, and runs every DP cell on the MI355X through
``lib/libnwk.so`` (include/nwk.h).  There is no CPU fallback: without the
built library or a HIP device the calls raise ``NwkError``.

    getMinimumPenalties(genes, k, pxy, pgap, penalties) -> hash
        seqalign-mpi-skeleton.cpp:117-175, submit/xuliny-seqalkway.cpp:232-364
    getMinimumPenalty(x, y, pxy, pgap) -> (penalty, align1, align2)
        seqalign-mpi-skeleton.cpp:186-280 + trim 135-154
    do_MPI_task(...)  ->  Engine.align_pairs(pair_ids, ...)
        submit/xuliny-seqalkway.cpp:369-417 (one rank's share of the pairs)
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# NWK_LIB: an A/B build variant of the library (profiles/r04/scripts/col_variant.sh); default the in-tree build
LIB_PATH = os.environ.get("NWK_LIB") or os.path.join(HERE, "lib", "libnwk.so")

NWK_OK = 0
ERRORS = {-1: "EINVAL", -2: "ENOMEM", -3: "EDEVICE", -4: "EKERNEL", -5: "ECOMM"}
MODES = {0: "profile", 1: "compare", 2: "literal", 3: "affine", 4: "packed-profile", 5: "packed-band-pairs",
         7: "packed-affine-band-pairs", 8: "bit-sliced-planes", 9: "bit-sliced-strips", 10: "bit-parallel-columns",
         11: "bit-sliced-affine"}
# fill kernel of each mode (csrc/nwk_kernels.hip), as rocprofv3 names it
KERNELS = {0: "nw_align", 1: "nw_align", 2: "nw_align", 3: "nw_align_affine", 4: "nw_align_pk", 5: "nw_align_pk2",
           7: "nw_align_pka", 8: "nw_align_bits", 9: "nw_align_strip", 10: "nw_align_col", 11: "nw_align_gotoh"}


class NwkError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("nwk error %d (%s): %s" % (code, ERRORS.get(code, "?"), msg))
        self.code = code


class Opts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("ngpus", ctypes.c_int32), ("bits", ctypes.c_int32),
                ("host_threads", ctypes.c_int32), ("workspace_bytes", ctypes.c_int64),
                ("verbose", ctypes.c_int32), ("finalize", ctypes.c_int32),
                ("linear_space", ctypes.c_int32), ("kernel", ctypes.c_int32), ("collective", ctypes.c_int32),
                ("task_order", ctypes.c_int32)]


class Stats(ctypes.Structure):
    _fields_ = [("fill_ms", ctypes.c_double), ("traceback_ms", ctypes.c_double),
                ("total_ms", ctypes.c_double), ("cells", ctypes.c_double),
                ("matrix_bytes", ctypes.c_int64), ("batches", ctypes.c_int32),
                ("bits", ctypes.c_int32), ("mode", ctypes.c_int32),
                ("fill_launches", ctypes.c_int32), ("device_finalized", ctypes.c_int32),
                ("linear_space_pairs", ctypes.c_int32), ("window_retries", ctypes.c_int32),
                ("window", ctypes.c_int32), ("guard_checked", ctypes.c_int32),
                ("guard_reruns", ctypes.c_int32)]


# Every exported symbol of include/nwk.h with its ctypes signature.
_P = ctypes.c_void_p
_I32, _I64 = ctypes.c_int32, ctypes.c_int64
SIGNATURES = {
    "nwk_opts_default": (None, [_P]),
    "nwk_last_error": (ctypes.c_char_p, []),
    "nwk_device_count": (ctypes.c_int, []),
    "nwk_ctx_create": (ctypes.c_int, [_P, _P]),
    "nwk_ctx_destroy": (None, [_P]),
    "nwk_set_sequences": (ctypes.c_int, [_P, _P, _P, _I32]),
    "nwk_align_pairs": (ctypes.c_int, [_P, _P, _I64, _I32, _I32, _P, _P]),
    "nwk_last_stats": (ctypes.c_int, [_P, _P]),
    "nwk_get_minimum_penalties": (ctypes.c_int, [_P, _P, _I32, _I32, _I32, _P, _P, _P]),
    "nwk_get_minimum_penalty": (ctypes.c_int, [_P, _P, _I32, _P, _I32, _I32, _I32, _P, _P, _P, _P]),
    "nwk_align_pairs_affine": (ctypes.c_int, [_P, _P, _I64, _I32, _I32, _I32, _P, _P]),
    "nwk_align_all": (ctypes.c_int, [_P, _I32, _I32, _P, _P, _P]),
    "nwk_align_all_affine": (ctypes.c_int, [_P, _I32, _I32, _I32, _P, _P, _P]),
    "nwk_get_minimum_penalty_affine": (ctypes.c_int, [_P, _P, _I32, _P, _I32, _I32, _I32, _I32, _P, _P, _P, _P]),
    "nwk_get_minimum_penalties_affine": (ctypes.c_int, [_P, _P, _I32, _I32, _I32, _I32, _P, _P, _P]),
    "nwk_msa": (ctypes.c_int, [_P, _I32, _I32, _P, _P, _I64, _P, _P]),
    "nwk_shard_pairs": (ctypes.c_int, [_P, _I32, _I32, _I32, _P, _P]),
    "nwk_chain_hash": (ctypes.c_int, [_P, _I64, _P]),
    "nwk_finalize_moves": (ctypes.c_int, [_P, _I32, _P, _I32, _I32, _I32, _P, _I64, _P, _P, _P, _P, _P]),
    "nwk_sha512_hex": (None, [_P, _I64, _P]),
    "nwk_align_pairs_begin": (ctypes.c_int, [_P, _P, _I64, _I32, _I32]),
    "nwk_align_pairs_end": (ctypes.c_int, [_P, _P, _P]),
    "nwk_align_pairs_poll": (ctypes.c_int, [_P, _I64, _P, _P, _P]),
    "nwk_chain_create": (ctypes.c_int, [_I64, _P]),
    "nwk_chain_feed": (ctypes.c_int, [_P, _P, _P, _P, _I64]),
    "nwk_chain_finish": (ctypes.c_int, [_P, _P, _P, _P]),
    "nwk_chain_destroy": (None, [_P]),
    "nwk_comm_unique_id": (ctypes.c_int, [_P]),
    "nwk_comm_create": (ctypes.c_int, [_I32, _P, _I32, _I32, _P]),
    "nwk_comm_all_gather": (ctypes.c_int, [_P, _P, _I64, _P]),
    "nwk_comm_all_reduce_max_f64": (ctypes.c_int, [_P, _P, _I64]),
    "nwk_comm_destroy": (None, [_P]),
    "nwk_device_synchronize": (ctypes.c_int, [_I32]),
}
COMM_ID_BYTES = 128

_lib = None

# Source files that determine each fill kernel's code object (plus the build
# flags in the Makefile): kernel_source_id() hashes them, so a roofline's
# per-launch counters (profiles/<round>/pmc_<workload>.json) can be tied to the
# kernel build that produced them.
KERNEL_SOURCES = {
    "nw_align_bits": ("csrc/nwk_bits.hip", "csrc/nwk_bits_dev.h", "csrc/nwk_sha_dev.h", "csrc/nwk_internal.h",
                      "Makefile"),
    "nw_align_strip": ("csrc/nwk_bits.hip", "csrc/nwk_bits_dev.h", "csrc/nwk_sha_dev.h", "csrc/nwk_internal.h",
                       "Makefile"),
    "nw_align_col": ("csrc/nwk_col.hip", "csrc/nwk_bits_dev.h", "csrc/nwk_sha_dev.h", "csrc/nwk_internal.h",
                     "Makefile"),
    "nw_align_gotoh": ("csrc/nwk_gotoh.hip", "csrc/nwk_gotoh_planes.h", "csrc/nwk_bits_dev.h", "csrc/nwk_sha_dev.h",
                       "csrc/nwk_internal.h", "Makefile"),
    "nw_align_pka": ("csrc/nwk_kernels.hip", "csrc/nwk_internal.h", "Makefile"),
    "nw_align_pk2": ("csrc/nwk_kernels.hip", "csrc/nwk_internal.h", "Makefile"),
    "nw_align_pk": ("csrc/nwk_kernels.hip", "csrc/nwk_internal.h", "Makefile"),
    "nw_align_affine": ("csrc/nwk_kernels.hip", "csrc/nwk_internal.h", "Makefile"),
    "nw_align": ("csrc/nwk_kernels.hip", "csrc/nwk_internal.h", "Makefile"),
    "nw_profile": ("csrc/nwk_kernels.hip", "csrc/nwk_prof.h", "csrc/nwk_internal.h", "Makefile"),
}


def kernel_source_id(kernel):
    """sha256 (16 hex digits) of the sources a fill kernel is compiled from."""
    import hashlib

    h = hashlib.sha256()
    for rel in KERNEL_SOURCES.get(kernel, ()):
        with open(os.path.join(HERE, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read())
    return h.hexdigest()[:16] if kernel in KERNEL_SOURCES else None


def load_library(path=LIB_PATH):
    """Loads lib/libnwk.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise NwkError(-3, "HIP extension not built: %s (run __graft_entry__.build())" % path)
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _check(rc):
    if rc != NWK_OK:
        raise NwkError(rc, _lib.nwk_last_error().decode("utf-8", "replace"))


def _as_bytes(s):
    if isinstance(s, bytes):
        return s
    if isinstance(s, str):
        return s.encode("latin-1")
    return bytes(s)


def pack_genes(genes):
    """Concatenated bytes + int64 offsets[k+1] (the C-ABI's sequence set)."""
    bs = [_as_bytes(g) for g in genes]
    offs = np.zeros(len(bs) + 1, dtype=np.int64)
    if bs:
        offs[1:] = np.cumsum([len(b) for b in bs])
    data = np.frombuffer(b"".join(bs) or b"\0", dtype=np.uint8).copy()
    return data, offs


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def device_count():
    return load_library().nwk_device_count()


def pair_index(i, j):
    """Canonical pair id of (i, j), i > j (skel:122-123)."""
    return i * (i - 1) // 2 + j


def pair_ij(p):
    i = int((1 + (1 + 8 * p) ** 0.5) // 2)
    while i * (i - 1) // 2 > p:
        i -= 1
    while (i + 1) * i // 2 <= p:
        i += 1
    return i, p - i * (i - 1) // 2


class Engine:
    """One device context: pooled HBM workspace + streams (nwk_ctx)."""

    FINALIZE = {"auto": 0, "host": 1, "device": 2, "fused": 3}

    KERNEL = {"auto": 0, "nw_align": 1, "nw_align_pk": 2, "nw_align_pk2": 3, "nw_align_bits": 4, "nw_align_strip": 5,
              "nw_align_col": 6, "nw_align_gotoh": 7}

    def __init__(self, device=0, bits=0, workspace_bytes=0, host_threads=0, verbose=False, finalize="auto",
                 linear_space=0, kernel="auto", task_order=0):
        """finalize: where rows, penalty and SHA-512 of each pair are computed --
        "auto" (per batch, by estimated cost), "host" threads, "device" (nw_rows +
        nw_hash after each fill launch) or "fused" (inside the bits kernels' fill
        launch, records streaming to the host as pairs finish: align_pairs_poll)."""
        self.lib = load_library()
        o = Opts()
        self.lib.nwk_opts_default(ctypes.byref(o))
        o.device, o.bits, o.workspace_bytes = device, bits, workspace_bytes
        o.host_threads, o.verbose = host_threads, int(verbose)
        o.finalize = self.FINALIZE[finalize]
        # linear-space traceback: 0 only where the matrix does not fit,
        # -1 never, G > 0 every pair with G bands per recompute group
        o.linear_space = linear_space
        # linear fill kernel (tests / A/B): "auto", "nw_align", "nw_align_pk", "nw_align_pk2", "nw_align_bits"
        o.kernel = self.KERNEL[kernel]
        o.task_order = int(task_order)
        self._ctx = ctypes.c_void_p()
        _check(self.lib.nwk_ctx_create(ctypes.byref(o), ctypes.byref(self._ctx)))
        self.k = 0
        self._offs = None
        self._pending = 0

    def close(self):
        if self._ctx:
            self.lib.nwk_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_sequences(self, genes):
        data, offs = pack_genes(genes)
        _check(self.lib.nwk_set_sequences(self._ctx, _ptr(data), _ptr(offs), len(genes)))
        self.k = len(genes)
        self._offs = offs

    def align_pairs(self, pair_ids, pxy, pgap):
        """The worker loop of one rank: returns (penalties int32[n], raw hashes uint8[n,64])."""
        ids = np.ascontiguousarray(pair_ids, dtype=np.int64)
        n = ids.size
        pen = np.zeros(max(n, 1), dtype=np.int32)
        hs = np.zeros((max(n, 1), 64), dtype=np.uint8)
        _check(self.lib.nwk_align_pairs(self._ctx, _ptr(ids), n, pxy, pgap, _ptr(pen), _ptr(hs)))
        return pen[:n], hs[:n]

    def align_pairs_begin(self, pair_ids, pxy, pgap):
        """Starts align_pairs on the context's host thread and returns at once
        (nwk_align_pairs_begin); align_pairs_end() collects the result."""
        ids = np.ascontiguousarray(pair_ids, dtype=np.int64)
        _check(self.lib.nwk_align_pairs_begin(self._ctx, _ptr(ids), ids.size, pxy, pgap))
        self._pending = ids.size
        self._poll_pen = np.zeros(max(ids.size, 1), dtype=np.int32)
        self._poll_hs = np.zeros((max(ids.size, 1), 64), dtype=np.uint8)

    def align_pairs_poll(self, start=0):
        """While align_pairs_begin's call runs: (upto, penalties, hashes) of the
        pairs pair_ids[start:upto] whose results are final (nwk_align_pairs_poll).
        With the bits kernels' fused device finalize they stream in as each
        pair's traceback ends; otherwise a batch's pairs arrive together."""
        upto = ctypes.c_int64(0)
        _check(self.lib.nwk_align_pairs_poll(self._ctx, int(start), _ptr(self._poll_pen), _ptr(self._poll_hs),
                                             ctypes.addressof(upto)))
        u = upto.value
        return u, self._poll_pen[start:u].copy(), self._poll_hs[start:u].copy()

    def align_pairs_end(self):
        n = self._pending
        pen = np.zeros(max(n, 1), dtype=np.int32)
        hs = np.zeros((max(n, 1), 64), dtype=np.uint8)
        _check(self.lib.nwk_align_pairs_end(self._ctx, _ptr(pen), _ptr(hs)))
        return pen[:n], hs[:n]

    def align_all(self, pxy, pgap, affine=None):
        """All pairs of the current set + the chained answer hash (getMinimumPenalties
        on this context): returns (hash, penalties int32[P], raw hashes uint8[P,64]).
        affine=(go, ge) selects the affine-gap variant."""
        P = self.k * (self.k - 1) // 2
        pen = np.zeros(max(P, 1), dtype=np.int32)
        hs = np.zeros((max(P, 1), 64), dtype=np.uint8)
        out = ctypes.create_string_buffer(129)
        if affine:
            _check(self.lib.nwk_align_all_affine(self._ctx, pxy, affine[0], affine[1], _ptr(pen), _ptr(hs), out))
        else:
            _check(self.lib.nwk_align_all(self._ctx, pxy, pgap, _ptr(pen), _ptr(hs), out))
        return out.value.decode(), pen[:P], hs[:P]

    def align_pairs_affine(self, pair_ids, pxy, go, ge):
        """Affine-gap variant of align_pairs."""
        ids = np.ascontiguousarray(pair_ids, dtype=np.int64)
        n = ids.size
        pen = np.zeros(max(n, 1), dtype=np.int32)
        hs = np.zeros((max(n, 1), 64), dtype=np.uint8)
        _check(self.lib.nwk_align_pairs_affine(self._ctx, _ptr(ids), n, pxy, go, ge, _ptr(pen), _ptr(hs)))
        return pen[:n], hs[:n]

    def get_minimum_penalty_affine(self, x, y, pxy, go, ge):
        xb, yb = _as_bytes(x), _as_bytes(y)
        m, n = len(xb), len(yb)
        a1 = ctypes.create_string_buffer(max(m + n, 1))
        a2 = ctypes.create_string_buffer(max(m + n, 1))
        alen, pen = ctypes.c_int32(), ctypes.c_int32()
        _check(self.lib.nwk_get_minimum_penalty_affine(self._ctx, xb, m, yb, n, pxy, go, ge, a1, a2,
                                                       ctypes.byref(alen), ctypes.byref(pen)))
        self.k = 2
        return pen.value, a1.raw[:alen.value], a2.raw[:alen.value]

    def stats(self):
        s = Stats()
        _check(self.lib.nwk_last_stats(self._ctx, ctypes.byref(s)))
        return {f: getattr(s, f) for f, _ in Stats._fields_ if f != "reserved"}

    def get_minimum_penalty(self, x, y, pxy, pgap):
        xb, yb = _as_bytes(x), _as_bytes(y)
        m, n = len(xb), len(yb)
        a1 = ctypes.create_string_buffer(max(m + n, 1))
        a2 = ctypes.create_string_buffer(max(m + n, 1))
        alen, pen = ctypes.c_int32(), ctypes.c_int32()
        _check(self.lib.nwk_get_minimum_penalty(self._ctx, xb, m, yb, n, pxy, pgap, a1, a2,
                                                ctypes.byref(alen), ctypes.byref(pen)))
        self.k = 2
        return pen.value, a1.raw[:alen.value], a2.raw[:alen.value]

    def msa(self, pxy, pgap, penalties=None):
        """Progressive sum-of-pairs MSA of the current set (nwk_msa):
        returns (rows: list of k bytes, '_' = gap, SoP score).  penalties: the
        pairwise penalties in canonical order (computed with align_all when None)."""
        if penalties is None:
            penalties = self.align_all(pxy, pgap)[1] if self.k > 1 else np.zeros(0, np.int32)
        pen = np.ascontiguousarray(penalties, dtype=np.int32)
        cap = max(int(self._offs[-1]) if self._offs is not None else 0, 1)
        rows = np.zeros((max(self.k, 1), cap), dtype=np.uint8)
        ln, sop = ctypes.c_int64(), ctypes.c_int64()
        _check(self.lib.nwk_msa(self._ctx, pxy, pgap, _ptr(pen) if pen.size else None, _ptr(rows), cap,
                                ctypes.byref(ln), ctypes.byref(sop)))
        return [bytes(rows[r, :ln.value]) for r in range(self.k)], sop.value


class ChainStream:
    """nwk_chain_*: the skel:159 chain over P pairs, advanced by a C++ worker
    thread as records are fed in any order; finish() -> (hash, penalties[P],
    hashes[P, 64]) in canonical order."""

    def __init__(self, P):
        self.lib = load_library()
        self.P = P
        self._ch = ctypes.c_void_p()
        _check(self.lib.nwk_chain_create(P, ctypes.byref(self._ch)))

    def feed(self, ids, penalties, hashes):
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        pen = np.ascontiguousarray(penalties, dtype=np.int32)
        hs = np.ascontiguousarray(hashes, dtype=np.uint8).reshape(-1, 64)
        if ids.size:
            _check(self.lib.nwk_chain_feed(self._ch, _ptr(ids), _ptr(pen), _ptr(hs), ids.size))

    def finish(self):
        out = ctypes.create_string_buffer(129)
        pen = np.zeros(max(self.P, 1), dtype=np.int32)
        hs = np.zeros((max(self.P, 1), 64), dtype=np.uint8)
        _check(self.lib.nwk_chain_finish(self._ch, out, _ptr(pen), _ptr(hs)))
        return out.value.decode(), pen[:self.P], hs[:self.P]

    def close(self):
        if self._ch:
            self.lib.nwk_chain_destroy(self._ch)
            self._ch = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Comm:
    """nwk_comm_*: one RCCL rank of a multi-process job, held by the library
    (the rank process binds only the library's HIP runtime and RCCL).  The
    rendezvous -- rank 0's id handed to the others -- is the caller's
    (dist.rccl_comm does it through a file on the node)."""

    def __init__(self, device, uid, world, rank):
        self.lib = load_library()
        self.device, self.world, self.rank = device, world, rank
        self._c = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * COMM_ID_BYTES).from_buffer_copy(bytes(uid).ljust(COMM_ID_BYTES, b"\0"))
        _check(self.lib.nwk_comm_create(device, buf, world, rank, ctypes.byref(self._c)))

    @staticmethod
    def unique_id():
        lib = load_library()
        buf = (ctypes.c_uint8 * COMM_ID_BYTES)()
        _check(lib.nwk_comm_unique_id(buf))
        return bytes(buf)

    def all_gather(self, block):
        """block: a C-contiguous numpy array (the same shape on every rank) ->
        (world,) + block.shape, every rank's block in rank order."""
        b = np.ascontiguousarray(block)
        out = np.empty((self.world,) + b.shape, dtype=b.dtype)
        _check(self.lib.nwk_comm_all_gather(self._c, _ptr(b), b.nbytes, _ptr(out)))
        return out

    def all_reduce_max(self, values):
        v = np.ascontiguousarray(values, dtype=np.float64).copy()
        _check(self.lib.nwk_comm_all_reduce_max_f64(self._c, _ptr(v), v.size))
        return v

    def barrier(self):
        self.all_reduce_max(np.zeros(1))

    def close(self):
        if self._c:
            self.lib.nwk_comm_destroy(self._c)
            self._c = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def device_synchronize(device):
    _check(load_library().nwk_device_synchronize(int(device)))


def chain_hash(problem_hashes):
    """skel:159 chain over raw 64-byte problem hashes in canonical order."""
    lib = load_library()
    h = np.ascontiguousarray(problem_hashes, dtype=np.uint8).reshape(-1, 64)
    out = ctypes.create_string_buffer(129)
    _check(lib.nwk_chain_hash(_ptr(h), h.shape[0], out))
    return out.value.decode()


def finalize_moves(x, y, pxy, pgap, moves):
    """Host finalize (skel:263-272 prefix, 135-157 trim/rows/hash) of a traceback
    given as moves in walk order from (m, n): (penalty, align1, align2, raw problemhash)."""
    lib = load_library()
    xb, yb, mv = _as_bytes(x), _as_bytes(y), _as_bytes(moves)
    cap = max(len(xb) + len(yb), 1)
    a1 = ctypes.create_string_buffer(cap)
    a2 = ctypes.create_string_buffer(cap)
    alen, pen = ctypes.c_int32(), ctypes.c_int32()
    ph = ctypes.create_string_buffer(64)
    _check(lib.nwk_finalize_moves(xb, len(xb), yb, len(yb), pxy, pgap, mv, len(mv), a1, a2, ctypes.byref(alen),
                                  ctypes.byref(pen), ph))
    return pen.value, a1.raw[:alen.value], a2.raw[:alen.value], ph.raw


def moves_of(a1, a2, m, n):
    """Walk-order moves (from (m, n)) of an alignment's rows: the inverse of the
    finalize, for tests.  Columns are read back to front; the prefix run (one
    row exhausted) is not part of the walk."""
    out = bytearray()
    i, j = m, n
    for c1, c2 in zip(reversed(a1), reversed(a2)):
        if i == 0 or j == 0:
            break
        if c1 != ord("_") and c2 != ord("_"):
            out.append(ord("D")); i -= 1; j -= 1
        elif c2 == ord("_"):
            out.append(ord("U")); i -= 1
        else:
            out.append(ord("L")); j -= 1
    return bytes(out)


def sha512_hex(data):
    lib = load_library()
    b = _as_bytes(data)
    out = ctypes.create_string_buffer(129)
    lib.nwk_sha512_hex(b, len(b), out)
    return out.value.decode()


def shard_pairs(lengths, rank, world):
    """This rank's canonical pair ids under the engine's LPT cell-cost shard."""
    lib = load_library()
    offs = np.zeros(len(lengths) + 1, dtype=np.int64)
    if len(lengths):
        offs[1:] = np.cumsum(lengths)
    k = len(lengths)
    P = k * (k - 1) // 2
    out = np.zeros(max(P, 1), dtype=np.int64)
    n = ctypes.c_int64()
    _check(lib.nwk_shard_pairs(_ptr(offs), k, rank, world, _ptr(out), ctypes.byref(n)))
    return out[:n.value].copy()


def getMinimumPenalties(genes, k, pxy, pgap, penalties, ngpus=1, bits=0, verbose=False, collective=False):
    """skel:117-175: fills penalties[0..P) in canonical order, returns the hash.
    ngpus > 1 (or collective=True) shards the pairs over devices 0..ngpus-1 and
    collects the result records with one in-process ncclAllGather."""
    lib = load_library()
    genes = list(genes)[:k]
    data, offs = pack_genes(genes)
    P = k * (k - 1) // 2
    pen = np.zeros(max(P, 1), dtype=np.int32)
    out = ctypes.create_string_buffer(129)
    o = Opts()
    lib.nwk_opts_default(ctypes.byref(o))
    o.ngpus, o.bits, o.verbose, o.collective = ngpus, bits, int(verbose), int(collective)
    _check(lib.nwk_get_minimum_penalties(_ptr(data), _ptr(offs), k, pxy, pgap, _ptr(pen), out,
                                         ctypes.byref(o)))
    for p in range(P):
        penalties[p] = int(pen[p])
    return out.value.decode()


def getMinimumPenaltiesAffine(genes, k, pxy, go, ge, penalties, ngpus=1, verbose=False):
    """Affine-gap variant of getMinimumPenalties (go=0, ge=pgap == linear)."""
    lib = load_library()
    genes = list(genes)[:k]
    data, offs = pack_genes(genes)
    P = k * (k - 1) // 2
    pen = np.zeros(max(P, 1), dtype=np.int32)
    out = ctypes.create_string_buffer(129)
    o = Opts()
    lib.nwk_opts_default(ctypes.byref(o))
    o.ngpus, o.verbose = ngpus, int(verbose)
    _check(lib.nwk_get_minimum_penalties_affine(_ptr(data), _ptr(offs), k, pxy, go, ge, _ptr(pen), out,
                                                ctypes.byref(o)))
    for p in range(P):
        penalties[p] = int(pen[p])
    return out.value.decode()


def getMinimumPenalty(x, y, pxy, pgap, device=0):
    """skel:186-280 + trim: (penalty, align1, align2) for one pair."""
    with Engine(device=device) as e:
        return e.get_minimum_penalty(x, y, pxy, pgap)


def parse_fasta(text):
    """FASTA records in file order: header lines start with '>',
    sequence lines are concatenated with whitespace removed, ';' lines are
    comments; sequence text before the first header is an unnamed record.
    Same rules as the driver's --fasta (csrc/seqalkway_main.cpp read_fasta)."""
    if isinstance(text, str):
        text = text.encode("latin-1")
    genes, cur = [], None
    for line in text.split(b"\n"):
        if line.startswith(b">"):
            cur = bytearray()
            genes.append(cur)
            continue
        if not line.strip() or line.startswith(b";"):
            continue
        if cur is None:
            cur = bytearray()
            genes.append(cur)
        cur += b"".join(line.split())
    return [bytes(g) for g in genes]


def read_input(path, pxy=3, pgap=2):
    """(pxy, pgap, genes) from the reference's token format, or from FASTA
    (first non-blank character '>') with the given penalties."""
    data = open(path, "rb").read()
    if data.lstrip().startswith(b">"):
        return pxy, pgap, parse_fasta(data)
    return parse_input(data)


def parse_input(text):
    """Rank-0 stdin parse of skel:40-47 (cin >> tokens): (pxy, pgap, genes)."""
    if isinstance(text, str):
        text = text.encode("latin-1")
    tok = text.split()
    pxy, pgap, k = int(tok[0]), int(tok[1]), int(tok[2])
    genes = [tok[3 + i] if 3 + i < len(tok) else b"" for i in range(max(k, 0))]
    return pxy, pgap, genes
