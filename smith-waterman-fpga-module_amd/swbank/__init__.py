"""swbank — Python host over libswbank.so (ctypes), mirroring the reference ScoreBank surface.

The reference's "host" for this path is the ScoreBank testbench (ScoreBank/ScoreBank_v1_tb.sv)
and the CAPI C host (capi_sample_aligner/software-C,C++/src/main_test.c).  This module keeps
their order of operations:

    bank = ScoreBank()                                  # ScoreBank_v2 instance + reset
    bank.set_penalties(5, -4, -12, -4)                  # ld_penalties   (ScoreBank_v2.v:161)
    bank.load_query(encode("AGGGCG..."))                # ld_sequence q  (ScoreBank_v2.v:162)
    scores = bank.score_batch(targets)                  # target records -> results/IDs/vld

Everything goes through the C ABI declared in include/swbank.h; there is no Python compute
path and no CPU fallback: if libswbank.so is missing, or no gfx950 device is present,
construction raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Iterable, Optional, Sequence, Tuple

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("SWBANK_LIB", os.path.join(_PKG, "lib", "libswbank.so"))
CLI_PATH = os.path.join(_PKG, "bin", "swbank")

OK = 0
ERR_ARG, ERR_NO_DEVICE, ERR_HIP, ERR_RANGE, ERR_STATE, ERR_NOMEM, ERR_IO, ERR_UNSUPPORTED = \
    -1, -2, -3, -4, -5, -6, -7, -8
ERR_TIMEOUT = -9  # a device-side hand-off wait ran out (ABI 5): the call's scores are invalid
ALPHABET_DNA, ALPHABET_PROTEIN = 0, 1
GAP_MERGED, GAP_GOTOH = 0, 1
DNA_ALPHA, PROTEIN_ALPHA = 5, 24

# Every symbol include/swbank.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "sw_abi_version", "sw_status_string", "sw_device_count", "sw_max_query_len",
    "sw_config_default", "sw_bank_create", "sw_bank_destroy", "sw_last_error",
    "sw_set_penalties", "sw_set_matrix", "sw_load_query", "sw_score_batch",
    "sw_score_batch_device", "sw_best_hit", "sw_encode_ascii", "sw_pack_2bit",
    "sw_unpack_2bit", "sw_fill_matrix", "sw_bank_set_timing", "sw_bank_timing",
    "sw_last_kernel", "sw_load_query_record", "sw_score_records", "sw_score_records_device",
    "sw_best_hit_device", "sw_batch_best", "sw_bank_devices", "sw_load_queries",
    "sw_query_count", "sw_score_batch_device_range", "sw_bank_counters",
    "sw_bank_counters_ex", "sw_bank_sync", "sw_score_batch_device_multi",
)
ABI_VERSION = 6
COUNTERS = ("stream_calls", "stream_reruns", "stream_declined", "chunked_calls", "device_sorts",
            "gather_timeouts", "mixed_chunks", "mixed_runs", "balanced_calls",
            "balanced_timeouts", "tail_timeouts", "handoff_reruns", "wave_balanced_timeouts",
            "h2d_bytes")
MAX_DEVICES = 16
RECORD_BYTES, RECORD_MAX_BASES = 64, 232


class SwbankError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"swbank status {status}: {msg}")
        self.status = status


class DeviceBatch(ctypes.Structure):
    """sw_device_batch (ABI 6): one device's resident batch for sw_score_batch_device_multi."""
    _fields_ = [("d_residues", ctypes.c_void_p), ("d_offsets", ctypes.c_void_p),
                ("d_lens", ctypes.c_void_p), ("n", ctypes.c_size_t),
                ("min_len", ctypes.c_uint32), ("max_len", ctypes.c_uint32),
                ("d_scores", ctypes.c_void_p), ("stream", ctypes.c_void_p)]


class _Config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("alphabet", ctypes.c_int32),
                ("gap_model", ctypes.c_int32), ("max_query_len", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("n_devices", ctypes.c_int32),
                ("devices", ctypes.c_int32 * 16)]


_LIB: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    """Load libswbank.so (raises if it has not been built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise SwbankError(ERR_UNSUPPORTED, f"{LIB_PATH} not built (run make in {_PKG})")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 (same SONAME). If
    # torch is imported first, libswbank binds to that copy, so torch tensors and streams can
    # be handed across the ABI; loading /opt/rocm's copy first would leave torch unable to
    # initialise its own.  So import torch (when present) before dlopen-ing the library.
    if os.environ.get("SWBANK_STANDALONE_HIP") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = ctypes.CDLL(LIB_PATH)
    if L.sw_abi_version() != ABI_VERSION:
        raise SwbankError(ERR_UNSUPPORTED, f"{LIB_PATH}: ABI {L.sw_abi_version()}, want {ABI_VERSION}")
    P, i32, u32, u64, sz = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64,
                            ctypes.c_size_t)
    sig = {
        "sw_abi_version": (i32, []),
        "sw_status_string": (ctypes.c_char_p, [i32]),
        "sw_device_count": (i32, []),
        "sw_max_query_len": (u32, []),
        "sw_config_default": (i32, [P]),
        "sw_bank_create": (i32, [ctypes.POINTER(P), P]),
        "sw_bank_destroy": (None, [P]),
        "sw_last_error": (ctypes.c_char_p, [P]),
        "sw_set_penalties": (i32, [P, i32, i32, i32, i32]),
        "sw_set_matrix": (i32, [P, P, i32, i32, i32]),
        "sw_load_query": (i32, [P, u64, P, u32]),
        "sw_score_batch": (i32, [P, P, sz, P, P, P, sz, P]),
        "sw_score_batch_device": (i32, [P, P, P, P, P, sz, u32, P, P]),
        "sw_score_batch_device_range": (i32, [P, P, P, P, P, sz, u32, u32, P, P]),
        "sw_bank_counters": (i32, [P, P]),
        "sw_bank_counters_ex": (i32, [P, P, sz]),
        "sw_bank_sync": (i32, [P]),
        "sw_batch_best": (i32, [P, P, P, P]),
        "sw_bank_devices": (i32, [P, P, i32]),
        "sw_best_hit": (i32, [P, P, P, sz, P, P]),
        "sw_encode_ascii": (sz, [i32, ctypes.c_char_p, sz, P]),
        "sw_pack_2bit": (sz, [ctypes.c_char_p, sz, P]),
        "sw_unpack_2bit": (sz, [P, sz, P]),
        "sw_fill_matrix": (i32, [i32, i32, i32, P]),
        "sw_bank_set_timing": (i32, [P, i32]),
        "sw_bank_timing": (i32, [P, P, P, P]),
        "sw_last_kernel": (ctypes.c_char_p, [P]),
        "sw_load_query_record": (i32, [P, P]),
        "sw_score_records": (i32, [P, P, sz, P]),
        "sw_score_records_device": (i32, [P, P, sz, P, P]),
        "sw_best_hit_device": (i32, [P, P, P, sz, P, P]),
        "sw_load_queries": (i32, [P, sz, P, P, P, P]),
        "sw_query_count": (sz, [P]),
        "sw_score_batch_device_multi": (i32, [P, P, sz, P, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = L
    return L


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def status_string(st: int) -> str:
    return lib().sw_status_string(st).decode()


def device_count() -> int:
    return int(lib().sw_device_count())


# ---- host helpers (no device) --------------------------------------------------------------
def encode(seq: str | bytes, alphabet: int = ALPHABET_DNA) -> np.ndarray:
    """ASCII -> codes (sw_encode_ascii; ConvertToBase for DNA)."""
    b = seq.encode() if isinstance(seq, str) else bytes(seq)
    out = np.zeros(max(len(b), 1), dtype=np.uint8)
    lib().sw_encode_ascii(alphabet, b, len(b), _p(out))
    return out[:len(b)]


def pack_2bit(seq: str | bytes) -> np.ndarray:
    """charTo2bit packing (sw_pack_2bit)."""
    b = seq.encode() if isinstance(seq, str) else bytes(seq)
    out = np.zeros(max((len(b) + 3) // 4, 1), dtype=np.uint8)
    lib().sw_pack_2bit(b, len(b), _p(out))
    return out[:(len(b) + 3) // 4]


def unpack_2bit(packed: np.ndarray, n: int) -> np.ndarray:
    packed = np.ascontiguousarray(packed, dtype=np.uint8)
    out = np.zeros(max(n, 1), dtype=np.uint8)
    lib().sw_unpack_2bit(_p(packed), n, _p(out))
    return out[:n]


def make_records(seqs: Sequence[np.ndarray], ids: Optional[Sequence[int]] = None) -> np.ndarray:
    """DNA code arrays (0..3) -> CAPI `sequence_t` records, one 64-byte row each
    (aligner_Header.h:19-24: u32 ID, u16 length, 58 bytes of 2-bit codes LSB-first)."""
    out = np.zeros((len(seqs), RECORD_BYTES), dtype=np.uint8)
    if isinstance(seqs, np.ndarray) and seqs.ndim == 2:  # equal lengths: vectorised
        n, L = seqs.shape
        if L > RECORD_MAX_BASES or (seqs.size and seqs.max() > 3):
            raise ValueError(f"records need <= {RECORD_MAX_BASES} ACGT codes")
        idv = np.arange(n, dtype=np.uint32) if ids is None else np.asarray(ids, np.uint32)
        out[:, 0:4] = idv.view(np.uint8).reshape(n, 4)
        out[:, 4:6] = np.full(n, L, np.uint16).view(np.uint8).reshape(n, 2)
        q = np.zeros((n, (L + 3) // 4 * 4), dtype=np.uint8)
        q[:, :L] = seqs
        q = q.reshape(n, -1, 4)
        out[:, 6:6 + q.shape[1]] = q[..., 0] | q[..., 1] << 2 | q[..., 2] << 4 | q[..., 3] << 6
        return out
    for k, sq in enumerate(seqs):
        c = np.asarray(sq, dtype=np.uint8)
        if len(c) > RECORD_MAX_BASES or (len(c) and c.max() > 3):
            raise ValueError(f"record {k}: needs <= {RECORD_MAX_BASES} ACGT codes")
        out[k, 0:4] = np.frombuffer(np.uint32(k if ids is None else ids[k]).tobytes(), np.uint8)
        out[k, 4:6] = np.frombuffer(np.uint16(len(c)).tobytes(), np.uint8)
        q = np.zeros((len(c) + 3) // 4 * 4, dtype=np.uint8)
        q[:len(c)] = c
        q = q.reshape(-1, 4)
        out[k, 6:6 + len(q)] = q[:, 0] | q[:, 1] << 2 | q[:, 2] << 4 | q[:, 3] << 6
    return out


def fill_matrix(alphabet: int, match: int = 5, mismatch: int = -4) -> np.ndarray:
    a = DNA_ALPHA if alphabet == ALPHABET_DNA else PROTEIN_ALPHA
    m = np.zeros((a, a), dtype=np.int8)
    st = lib().sw_fill_matrix(alphabet, match, mismatch, _p(m))
    if st != OK:
        raise SwbankError(st, status_string(st))
    return m


def pack_targets(seqs: Sequence[np.ndarray]) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Concatenate code arrays -> (residues, offsets u64, lens u32)."""
    lens = np.array([len(s) for s in seqs], dtype=np.uint32)
    offs = np.zeros(len(seqs), dtype=np.uint64)
    if len(seqs) > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    res = np.concatenate([np.asarray(s, dtype=np.uint8) for s in seqs]) if len(seqs) else None
    if res is None or res.size == 0:
        res = np.zeros(1, dtype=np.uint8)
    return res, offs, lens


def validate_batch(residues, offsets, lens, ids=None):
    """Host batch -> contiguous (residues u8, offsets u64, lens u32, ids u64 | None), or
    ValueError when the arrays disagree: the C feeder reads offsets[k], lens[k] (and ids[k])
    for every k < len(lens), so a short array would be a host over-read inside the library
    rather than a Python error.  Each target's range against the residues is checked by the
    library itself (sw_score_batch takes the residue count; SW_ERR_ARG, nothing read past it),
    inside the feeder pass that reads the offsets anyway."""
    res = np.ascontiguousarray(residues, dtype=np.uint8).reshape(-1)
    ln = np.ascontiguousarray(lens, dtype=np.uint32).reshape(-1)
    off_in = np.asarray(offsets).reshape(-1)
    if off_in.size != ln.size:
        raise ValueError(f"{off_in.size} offsets for {ln.size} lengths")
    if off_in.size and np.issubdtype(off_in.dtype, np.signedinteger) and off_in.min() < 0:
        raise ValueError("negative offset")
    offs = np.ascontiguousarray(off_in, dtype=np.uint64)
    idv = None
    if ids is not None:
        idv = np.ascontiguousarray(ids, dtype=np.uint64).reshape(-1)
        if idv.size != ln.size:
            raise ValueError(f"{idv.size} ids for {ln.size} targets")
    return res, offs, ln, idv


# ---- the bank ----------------------------------------------------------------------------
class ScoreBank:
    """One ScoreBank_v2 instance (sw_bank_create): on one GPU, or with ``devices=[...]`` a
    multi-device bank that deals every host batch over those GPUs (the RTL's MODULES,
    ScoreBank_v2.v:76-148) and gathers the scores back with RCCL."""

    def __init__(self, device: int = -1, alphabet: int = ALPHABET_DNA,
                 gap_model: int = GAP_MERGED, max_query_len: int = 0,
                 devices: Optional[Sequence[int]] = None):
        L = lib()
        cfg = _Config()
        L.sw_config_default(ctypes.byref(cfg))
        cfg.device, cfg.alphabet, cfg.gap_model, cfg.max_query_len = (
            device, alphabet, gap_model, max_query_len)
        if devices is not None:
            devices = list(devices)
            if not 1 <= len(devices) <= MAX_DEVICES:
                raise ValueError(f"devices: 1..{MAX_DEVICES} ordinals")
            cfg.n_devices = len(devices)
            for i, d in enumerate(devices):
                cfg.devices[i] = d
        h = ctypes.c_void_p()
        st = L.sw_bank_create(ctypes.byref(h), ctypes.byref(cfg))
        if st != OK:
            raise SwbankError(st, status_string(st))
        self._h = h
        self.alphabet = alphabet
        self.gap_model = gap_model

    # errors
    def _check(self, st: int):
        if st != OK:
            raise SwbankError(st, f"{status_string(st)}: {lib().sw_last_error(self._h).decode()}")

    def close(self):
        if getattr(self, "_h", None):
            lib().sw_bank_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ld_penalties
    def set_penalties(self, match: int, mismatch: int, gap_open: int, gap_extend: int):
        self._check(lib().sw_set_penalties(self._h, match, mismatch, gap_open, gap_extend))

    def set_matrix(self, matrix: np.ndarray, gap_open: int, gap_extend: int):
        m = np.ascontiguousarray(matrix, dtype=np.int8)
        self._check(lib().sw_set_matrix(self._h, _p(m), m.shape[0], gap_open, gap_extend))

    # ld_sequence (query)
    def load_query(self, codes: np.ndarray, qid: int = 0):
        c = np.ascontiguousarray(codes, dtype=np.uint8)
        buf = c if c.size else np.zeros(1, np.uint8)
        self._check(lib().sw_load_query(self._h, qid, _p(buf), len(c)))

    def load_queries(self, queries, ids=None):
        """A query set (sw_load_queries): every following score_batch_device call scores the
        batch against each query, scores query-major (len(queries) x n)."""
        qs = [np.ascontiguousarray(q, dtype=np.uint8) for q in queries]
        if not qs:
            raise ValueError("an empty query set")
        codes, offs, lens = pack_targets(qs)
        idv = None
        if ids is not None:
            idv = np.ascontiguousarray(ids, dtype=np.uint64)
            if idv.size != len(qs):
                raise ValueError(f"{idv.size} ids for {len(qs)} queries")
        buf = codes if codes.size else np.zeros(1, np.uint8)
        self._check(lib().sw_load_queries(self._h, len(qs), None if idv is None else _p(idv),
                                          _p(buf), _p(offs), _p(lens)))

    def query_count(self) -> int:
        return int(lib().sw_query_count(self._h))

    # target stream
    def score_batch(self, residues: np.ndarray, offsets: np.ndarray, lens: np.ndarray,
                    ids: Optional[np.ndarray] = None,
                    out: Optional[np.ndarray] = None) -> np.ndarray:
        """Scores of targets residues[offsets[k] : offsets[k] + lens[k]] in input order; ids
        (optional, one per target) tag the batch best hit (best()); out (optional, int32,
        contiguous, one per target) is filled and returned instead of a new array."""
        res, offs, ln, idv = validate_batch(residues, offsets, lens, ids)
        if out is None:
            out = np.empty(len(ln), dtype=np.int32)  # every entry written by the library
        elif (out.dtype != np.int32 or out.shape != (len(ln),)
              or not out.flags["C_CONTIGUOUS"] or not out.flags["WRITEABLE"]):
            raise ValueError("out: a writable contiguous int32 array with one entry per target")
        if len(ln) == 0:
            return out
        self._check(lib().sw_score_batch(self._h, _p(res), res.size, _p(offs), _p(ln),
                                         _p(idv) if idv is not None else None, len(ln), _p(out)))
        return out

    def best(self) -> Tuple[int, int, int]:
        """Best hit of the last batch call (sw_batch_best, ≙ max / vld_max):
        (id, score, index) — lowest index among equal maxima."""
        bid, bsc, bix = ctypes.c_uint64(), ctypes.c_int32(), ctypes.c_uint64()
        self._check(lib().sw_batch_best(self._h, ctypes.byref(bid), ctypes.byref(bsc),
                                        ctypes.byref(bix)))
        return int(bid.value), int(bsc.value), int(bix.value)

    def devices(self) -> list:
        arr = (ctypes.c_int32 * MAX_DEVICES)()
        n = lib().sw_bank_devices(self._h, arr, MAX_DEVICES)
        return [int(arr[i]) for i in range(n)]

    def score_targets(self, seqs: Iterable[np.ndarray]) -> np.ndarray:
        return self.score_batch(*pack_targets(list(seqs)))

    def score_batch_device(self, d_res: int, d_offs: int, d_lens: int, n: int, max_len: int,
                           d_scores: int, stream: int = 0, d_ids: int = 0,
                           min_len: Optional[int] = None):
        """Device pointers (ints, e.g. torch.Tensor.data_ptr()); async on `stream`.  With d_ids
        the call also records the batch best hit on the device (best()).  With min_len (every
        length in [min_len, max_len]) the call is sw_score_batch_device_range: a range of one
        length skips the on-device length sort.  stream 0 is the BANK's own non-blocking stream
        (the C ABI's NULL), not HIP's default stream; torch's default current stream has handle
        0 on ROCm, so pass a torch.cuda.Stream's cuda_stream (or sync()) before torch reads the
        scores."""
        if min_len is None:
            self._check(lib().sw_score_batch_device(self._h, d_res, d_offs, d_lens,
                                                    d_ids or None, n, max_len, d_scores,
                                                    stream or None))
        else:
            self._check(lib().sw_score_batch_device_range(self._h, d_res, d_offs, d_lens,
                                                          d_ids or None, n, min_len, max_len,
                                                          d_scores, stream or None))

    def score_batch_device_multi(self, batches, d_gathered: int = 0, stream: int = 0):
        """sw_score_batch_device_multi (ABI 6): batches[d] = dict(d_res, d_offs, d_lens, n,
        max_len, min_len=0, d_scores=0, stream=0) resident on the bank's d-th device; each device
        scores its own batch in place, the int32 scores are gathered to the root into d_gathered
        (query-major over the concatenated batch) and/or left in each d_scores.  Async."""
        arr = (DeviceBatch * len(batches))()
        for i, bt in enumerate(batches):
            arr[i] = DeviceBatch(bt["d_res"] or None, bt["d_offs"] or None, bt["d_lens"] or None,
                                 bt["n"], bt.get("min_len", 0), bt["max_len"],
                                 bt.get("d_scores", 0) or None, bt.get("stream", 0) or None)
        self._check(lib().sw_score_batch_device_multi(self._h, arr, len(batches),
                                                      d_gathered or None, stream or None))

    def counters(self) -> dict:
        """sw_bank_counters: feeder / fallback counts since the bank was created."""
        c = (ctypes.c_uint64 * len(COUNTERS))()
        self._check(lib().sw_bank_counters_ex(self._h, ctypes.byref(c), ctypes.sizeof(c)))
        return dict(zip(COUNTERS, (int(x) for x in c)))

    def sync(self):
        """sw_bank_sync: wait for the bank's last scoring call; raises SwbankError(ERR_TIMEOUT)
        when a device call since the last synchronising call had a hand-off wait run out."""
        self._check(lib().sw_bank_sync(self._h))

    # CAPI record path (sequence_t arrays, 2-bit codes)
    def load_query_record(self, record: np.ndarray):
        r = np.ascontiguousarray(record, dtype=np.uint8).reshape(-1)
        if r.size != RECORD_BYTES:
            raise ValueError("a record is 64 bytes")
        self._check(lib().sw_load_query_record(self._h, _p(r)))

    def score_records(self, records: np.ndarray) -> np.ndarray:
        r = np.ascontiguousarray(records, dtype=np.uint8).reshape(-1, RECORD_BYTES)
        out = np.zeros(len(r), dtype=np.int32)
        if len(r):
            self._check(lib().sw_score_records(self._h, _p(r), len(r), _p(out)))
        return out

    def score_records_device(self, d_records: int, n: int, d_scores: int, stream: int = 0):
        self._check(lib().sw_score_records_device(self._h, d_records, n, d_scores,
                                                  stream or None))

    def best_hit(self, scores: np.ndarray, ids: Optional[np.ndarray] = None) -> Tuple[int, int]:
        """ScoreBank max / vld_max: (id of the best target, its score)."""
        s = np.ascontiguousarray(scores, dtype=np.int32)
        bid, bsc = ctypes.c_uint64(), ctypes.c_int32()
        ida = np.ascontiguousarray(ids, dtype=np.uint64) if ids is not None else None
        self._check(lib().sw_best_hit(self._h, _p(s), _p(ida) if ida is not None else None,
                                      len(s), ctypes.byref(bid), ctypes.byref(bsc)))
        return int(bid.value), int(bsc.value)

    def best_hit_device(self, d_scores: int, n: int, d_out: int, d_ids: int = 0,
                        stream: int = 0):
        """Device best hit: d_out (2 x uint64) <- (best id, best score); async on `stream`."""
        self._check(lib().sw_best_hit_device(self._h, d_scores, d_ids or None, n, d_out,
                                             stream or None))

    # profiling
    def set_timing(self, enable: bool = True):
        self._check(lib().sw_bank_set_timing(self._h, 1 if enable else 0))

    def last_kernel(self) -> str:
        """The kernel the last score call ran (e.g. "tile f16 R=32 W=4 segs=1 grid=998")."""
        return lib().sw_last_kernel(self._h).decode()

    def timing(self) -> Tuple[int, float, float]:
        """(launches, pack_ms, score_ms) accumulated since the previous call."""
        n, pm, sm = ctypes.c_uint64(), ctypes.c_double(), ctypes.c_double()
        self._check(lib().sw_bank_timing(self._h, ctypes.byref(n), ctypes.byref(pm),
                                         ctypes.byref(sm)))
        return int(n.value), float(pm.value), float(sm.value)
