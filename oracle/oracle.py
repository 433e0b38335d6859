"""Oracle for the Smith-Waterman scoring path — TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg may import this
module.  It is the checker: the product library (libswbank.so) never calls into it.

Contents
* ``liboracle_sw.so`` loader (C restatement in ``sw_oracle.c``; file:line citations there).
* An independent pure-Python restatement (``py_score_merged`` / ``py_score_gotoh``) for small
  cases, used to cross-check the C code.
* Alphabets and matrices the reference uses: DNA codes of ``ConvertToBase``
  (ScoreBank/ScoreBank_v1_tb.sv:44-52: A=10b, G=11b, T=00b, C=01b; anything else -> code 4,
  which mismatches everything, since the testbench's ``2'bZZ`` is undefined), the constants of
  ``data/smith-waterman.py:6-10``; BLOSUM62 for protein mode (build-supplied, not in the
  reference: protein parity is unpinned by the reference).
* FASTA reader matching the testbench's tokeniser (``ScoreBank_v1_tb.sv:185-212``: '>' name
  token, then one sequence token) and tolerant of multi-line records.
* Golden-fixture loaders (tests/golden/*.tsv written by tests/golden/make_golden.py).
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, List, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLDEN = os.path.join(REPO, "tests", "golden")

GAP_MERGED = 0
GAP_GOTOH = 1

# Reference penalties: data/smith-waterman.py:6-10
REF_MATCH, REF_MISMATCH, REF_GAP_OPEN, REF_GAP_EXTEND = 5, -4, -12, -4

# ---------------------------------------------------------------------------------------
# alphabets
DNA_ALPHA = 5  # T C A G N
_DNA_CODE = np.full(256, 4, dtype=np.uint8)
for _ch, _c in (("T", 0), ("C", 1), ("A", 2), ("G", 3)):
    _DNA_CODE[ord(_ch)] = _c
    _DNA_CODE[ord(_ch.lower())] = _c

PROT_LETTERS = "ARNDCQEGHILKMFPSTWYVBZX*"
PROT_ALPHA = 24
_PROT_CODE = np.full(256, PROT_LETTERS.index("X"), dtype=np.uint8)
for _i, _ch in enumerate(PROT_LETTERS):
    _PROT_CODE[ord(_ch)] = _i
    _PROT_CODE[ord(_ch.lower())] = _i

_BLOSUM62_ROWS = """
 4 -1 -2 -2  0 -1 -1  0 -2 -1 -1 -1 -1 -2 -1  1  0 -3 -2  0 -2 -1  0 -4
-1  5  0 -2 -3  1  0 -2  0 -3 -2  2 -1 -3 -2 -1 -1 -3 -2 -3 -1  0 -1 -4
-2  0  6  1 -3  0  0  0  1 -3 -3  0 -2 -3 -2  1  0 -4 -2 -3  3  0 -1 -4
-2 -2  1  6 -3  0  2 -1 -1 -3 -4 -1 -3 -3 -1  0 -1 -4 -3 -3  4  1 -1 -4
 0 -3 -3 -3  9 -3 -4 -3 -3 -1 -1 -3 -1 -2 -3 -1 -1 -2 -2 -1 -3 -3 -2 -4
-1  1  0  0 -3  5  2 -2  0 -3 -2  1  0 -3 -1  0 -1 -2 -1 -2  0  3 -1 -4
-1  0  0  2 -4  2  5 -2  0 -3 -3  1 -2 -3 -1  0 -1 -3 -2 -2  1  4 -1 -4
 0 -2  0 -1 -3 -2 -2  6 -2 -4 -4 -2 -3 -3 -2  0 -2 -2 -3 -3 -1 -2 -1 -4
-2  0  1 -1 -3  0  0 -2  8 -3 -3 -1 -2 -1 -2 -1 -2 -2  2 -3  0  0 -1 -4
-1 -3 -3 -3 -1 -3 -3 -4 -3  4  2 -3  1  0 -3 -2 -1 -3 -1  3 -3 -3 -1 -4
-1 -2 -3 -4 -1 -2 -3 -4 -3  2  4 -2  2  0 -3 -2 -1 -2 -1  1 -4 -3 -1 -4
-1  2  0 -1 -3  1  1 -2 -1 -3 -2  5 -1 -3 -1  0 -1 -3 -2 -2  0  1 -1 -4
-1 -1 -2 -3 -1  0 -2 -3 -2  1  2 -1  5  0 -2 -1 -1 -1 -1  1 -3 -1 -1 -4
-2 -3 -3 -3 -2 -3 -3 -3 -1  0  0 -3  0  6 -4 -2 -2  1  3 -1 -3 -3 -1 -4
-1 -2 -2 -1 -3 -1 -1 -2 -2 -3 -3 -1 -2 -4  7 -1 -1 -4 -3 -2 -2 -1 -2 -4
 1 -1  1  0 -1  0  0  0 -1 -2 -2  0 -1 -2 -1  4  1 -3 -2 -2  0  0  0 -4
 0 -1  0 -1 -1 -1 -1 -2 -2 -1 -1 -1 -1 -2 -1  1  5 -2 -2  0 -1 -1  0 -4
-3 -3 -4 -4 -2 -2 -3 -2 -2 -3 -2 -3 -1  1 -4 -3 -2 11  2 -3 -4 -3 -2 -4
-2 -2 -2 -3 -2 -1 -2 -3  2 -1 -1 -2 -1  3 -3 -2 -2  2  7 -1 -3 -2 -1 -4
 0 -3 -3 -3 -1 -2 -2 -3 -3  3  1 -2  1 -1 -2 -2  0 -3 -1  4 -3 -2 -1 -4
-2 -1  3  4 -3  0  1 -1  0 -3 -4  0 -3 -3 -2  0 -1 -4 -3 -3  4  1 -1 -4
-1  0  0  1 -3  3  4 -2  0 -3 -3  1 -1 -3 -1  0 -1 -3 -2 -2  1  4 -1 -4
 0 -1 -1 -1 -2 -1 -1 -1 -1 -1 -1 -1 -1 -1 -2  0  0 -2 -1 -1 -1 -1 -1 -4
-4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4 -4  1
"""
BLOSUM62 = np.array([[int(x) for x in r.split()] for r in _BLOSUM62_ROWS.strip().splitlines()],
                    dtype=np.int8)


def encode_dna(seq: str | bytes) -> np.ndarray:
    b = seq.encode() if isinstance(seq, str) else bytes(seq)
    return _DNA_CODE[np.frombuffer(b, dtype=np.uint8)]


def encode_protein(seq: str | bytes) -> np.ndarray:
    b = seq.encode() if isinstance(seq, str) else bytes(seq)
    return _PROT_CODE[np.frombuffer(b, dtype=np.uint8)]


def dna_matrix(match: int = REF_MATCH, mismatch: int = REF_MISMATCH) -> np.ndarray:
    """5x5: equal A/C/G/T codes score ``match`` (PE LUT, SW_ProcessingElement_v1.0.v:119),
    everything else — including N vs N — ``mismatch``."""
    m = np.full((DNA_ALPHA, DNA_ALPHA), mismatch, dtype=np.int8)
    for c in range(4):
        m[c, c] = match
    return m


# ---------------------------------------------------------------------------------------
# FASTA + fixtures
def read_fasta(path: str) -> List[Tuple[str, str]]:
    """[(name, sequence)] — '>' starts a record; sequence lines are concatenated."""
    recs: List[Tuple[str, str]] = []
    name, chunks = None, []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            if line.startswith(">"):
                if name is not None:
                    recs.append((name, "".join(chunks)))
                name, chunks = line[1:].split()[0] if len(line) > 1 else "", []
            else:
                chunks.append(line)
    if name is not None:
        recs.append((name, "".join(chunks)))
    return recs


def golden_fasta(name: str) -> str:
    return os.path.join(GOLDEN, "fasta", name)


def load_ref_scores() -> List[Tuple[str, str, str, str, int]]:
    rows = []
    with open(os.path.join(GOLDEN, "ref_scores.tsv")) as f:
        next(f)
        for line in f:
            src, lib, q, t, s = line.rstrip("\n").split("\t")
            rows.append((src, lib, q, t, int(s)))
    return rows


def load_swalign_control() -> Dict[str, int]:
    out = {}
    with open(os.path.join(GOLDEN, "swalign_control.tsv")) as f:
        next(f)
        for line in f:
            _, _, t, s = line.rstrip("\n").split("\t")
            out[t] = int(s)
    return out


# ---------------------------------------------------------------------------------------
# pure-Python restatements (small cases only; independent of the C file)
def py_score_merged(q: Sequence[int], t: Sequence[int], sub: np.ndarray, go: int, ge: int,
                    col0_rule: bool = True) -> int:
    """§8.0 merged-I recurrence (SW_ProcessingElement_v1.0.v:119-141,287-291,411-420).
    col0_rule=False gives the textbook form (neighbours also used in the first column)."""
    n = len(t)
    Mp, Ip = [0] * n, [0] * n
    best = 0
    for qi in q:
        srow = sub[qi]
        dM = dI = lM = lI = 0
        for j in range(n):
            uM, uI = Mp[j], Ip[j]
            m = max(0, max(dM, dI) + int(srow[t[j]]))
            if j == 0 and col0_rule:
                i_ = max(go + ge, ge)
            else:
                i_ = max(max(uM, lM) + go + ge, max(uI, lI) + ge)
            best = max(best, m, i_)
            dM, dI, lM, lI = uM, uI, m, i_
            Mp[j], Ip[j] = m, i_
    return best


def py_score_gotoh(q: Sequence[int], t: Sequence[int], sub: np.ndarray, go: int, ge: int) -> int:
    NEG = -(1 << 30)
    n = len(t)
    Hp, Fp = [0] * n, [NEG] * n
    best = 0
    for qi in q:
        srow = sub[qi]
        dH = lH = 0
        E = NEG
        for j in range(n):
            uH = Hp[j]
            E = max(lH + go + ge, E + ge)
            F = max(uH + go + ge, Fp[j] + ge)
            h = max(0, dH + int(srow[t[j]]), E, F)
            best = max(best, h)
            dH, lH, Hp[j], Fp[j] = uH, h, h, F
    return best


# ---------------------------------------------------------------------------------------
# C oracle
_LIB = None


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle_sw.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "liboracle_sw.so"], cwd=HERE)
        L = ctypes.CDLL(path)
        P = ctypes.c_void_p
        i32 = ctypes.c_int32
        L.swo_score_pair.restype = i32
        L.swo_score_pair.argtypes = [P, i32, P, i32, P, i32, i32, i32, i32]
        L.swo_score_pair_rtl.restype = i32
        L.swo_score_pair_rtl.argtypes = [P, i32, P, i32, P, i32, i32, i32, i32]
        L.swo_score_batch.restype = None
        L.swo_score_batch.argtypes = [P, i32, P, P, P, ctypes.c_size_t, P, i32, i32, i32, i32, P, i32]
        L.swo_score_pairs.restype = None
        L.swo_score_pairs.argtypes = [P, P, P, P, P, P, P, P, ctypes.c_size_t, P, i32, i32, i32, i32,
                                      P, i32]
        _LIB = L
    return _LIB


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def score_pair(q: np.ndarray, t: np.ndarray, sub: np.ndarray, go: int, ge: int,
               model: int = GAP_MERGED) -> int:
    q = np.ascontiguousarray(q, dtype=np.uint8)
    t = np.ascontiguousarray(t, dtype=np.uint8)
    sub = np.ascontiguousarray(sub, dtype=np.int8)
    return lib().swo_score_pair(_ptr(q), len(q), _ptr(t), len(t), _ptr(sub), sub.shape[0], go, ge,
                                model)


def score_pair_rtl(q: np.ndarray, t: np.ndarray, sub: np.ndarray, go: int, ge: int,
                   width: int = 12) -> int:
    q = np.ascontiguousarray(q, dtype=np.uint8)
    t = np.ascontiguousarray(t, dtype=np.uint8)
    sub = np.ascontiguousarray(sub, dtype=np.int8)
    return lib().swo_score_pair_rtl(_ptr(q), len(q), _ptr(t), len(t), _ptr(sub), sub.shape[0], go,
                                    ge, width)


def pack_residues(seqs: Sequence[np.ndarray]) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    lens = np.array([len(s) for s in seqs], dtype=np.uint32)
    offs = np.zeros(len(seqs), dtype=np.uint64)
    if len(seqs):
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    res = np.concatenate([np.asarray(s, dtype=np.uint8) for s in seqs]) if len(seqs) else \
        np.zeros(0, np.uint8)
    if res.size == 0:
        res = np.zeros(1, np.uint8)
    return res, offs, lens


def score_batch(q: np.ndarray, res: np.ndarray, offs: np.ndarray, lens: np.ndarray,
                sub: np.ndarray, go: int, ge: int, model: int = GAP_MERGED,
                nthreads: int = 0) -> np.ndarray:
    q = np.ascontiguousarray(q, dtype=np.uint8)
    res = np.ascontiguousarray(res, dtype=np.uint8)
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    sub = np.ascontiguousarray(sub, dtype=np.int8)
    out = np.zeros(len(lens), dtype=np.int32)
    lib().swo_score_batch(_ptr(q), len(q), _ptr(res), _ptr(offs), _ptr(lens), len(lens), _ptr(sub),
                          sub.shape[0], go, ge, model, _ptr(out), nthreads)
    return out


def score_pairs(qres, qoffs, qlens, tres, toffs, tlens, qidx, tidx, sub, go, ge,
                model: int = GAP_MERGED, nthreads: int = 0) -> np.ndarray:
    arrs = [np.ascontiguousarray(a, dtype=d) for a, d in (
        (qres, np.uint8), (qoffs, np.uint64), (qlens, np.uint32), (tres, np.uint8),
        (toffs, np.uint64), (tlens, np.uint32), (qidx, np.uint32), (tidx, np.uint32))]
    sub = np.ascontiguousarray(sub, dtype=np.int8)
    out = np.zeros(len(arrs[6]), dtype=np.int32)
    lib().swo_score_pairs(*[_ptr(a) for a in arrs], len(arrs[6]), _ptr(sub), sub.shape[0], go, ge,
                          model, _ptr(out), nthreads)
    return out


# ---------------------------------------------------------------------------------------
# seeded synthetic workloads (splitmix64, shared with bench.py so both draw the same data)
def splitmix64_bytes(seed: int, n: int, start: int = 0) -> np.ndarray:
    """Bytes [start, start + n) of a splitmix64 stream (vectorised, deterministic; word i of the
    stream depends on i alone, so any window is generated without its prefix)."""
    w0 = start // 8
    words = (start + n + 7) // 8 - w0
    idx = np.arange(w0 + 1, w0 + words + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    o = start - 8 * w0
    return z.view(np.uint8)[o:o + n].copy()


def random_codes(seed: int, n: int, alpha: int, start: int = 0) -> np.ndarray:
    """Uniform i.i.d. codes in [0, alpha) (like data/generate.py:7,13, but seeded): codes
    [start, start + n) of the seed's stream."""
    b = splitmix64_bytes(seed, n, start).astype(np.uint32)
    return (b * alpha >> 8).astype(np.uint8)
