"""GPU: streamed host batches (sw_score_batch on equal-length DNA targets): one kernel launch
for the whole call, chunks of whole tiles published to the running kernel as their copies land
(swbank_stream.hip stream_feed, swbank_ktile.hip STREAM variants).  Scores must equal the
chunked feeder's (SWBANK_STREAM=0, itself checked against the oracle in test_gpu_feeder.py) and
the oracle's on a sample; the best hit the lowest index of the maximum; a bad code or a target
outside the residues fails the call and leaves the bank usable."""
import numpy as np
import pytest

import swbank as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu

REF = (5, -4, -12, -4)


def _uniform(rng, n, L, p_n=0.0):
    res = rng.integers(0, 4, n * L, dtype=np.uint8)
    if p_n:
        res[rng.random(res.size) < p_n] = 4
    return res, np.arange(n, dtype=np.uint64) * L, np.full(n, L, np.uint32)


def _check(monkeypatch, bank, q, res, offs, lens, params, gotoh, rng, extra=()):
    got = bank.score_batch(res, offs, lens)
    kern = bank.last_kernel()
    best = bank.best()
    assert "streamed=" in kern, kern
    monkeypatch.setenv("SWBANK_STREAM", "0")
    ref = bank.score_batch(res, offs, lens)
    assert "streamed=" not in bank.last_kernel()
    monkeypatch.delenv("SWBANK_STREAM")
    assert np.array_equal(got, ref), kern
    top = int(np.argmax(got))
    assert best[1] == int(got[top]) and best[2] == top, (best, top)
    n = len(lens)
    sel = np.unique(np.concatenate([rng.choice(n, min(n, 600), replace=False),
                                    np.arange(min(n, 130)), np.arange(max(0, n - 130), n),
                                    np.asarray(extra, dtype=np.int64)]))
    L = int(lens[0])
    sub = [res[int(offs[k]):int(offs[k]) + L] for k in sel]
    want = O.score_batch(q, *S.pack_targets(sub), O.dna_matrix(*params[:2]), *params[2:],
                         O.GAP_GOTOH if gotoh else O.GAP_MERGED)
    assert np.array_equal(got[sel], want), kern
    return kern


@pytest.mark.parametrize("L", [150, 33, 1])
def test_stream_pair_f16(monkeypatch, L):
    """The headline form: f16 letter-pair tables, 2-bit chunks, a full-size batch (>= two
    rounds of resident workgroups) and a forced small one (fewer tiles than chunks' minimum)."""
    rng = np.random.default_rng(L)
    n = 300_000 if L == 150 else 5_000
    if L != 150:
        monkeypatch.setenv("SWBANK_STREAM", "2")
    res, offs, lens = _uniform(rng, n, L)
    q = rng.integers(0, 4, 100, dtype=np.uint8)
    for k in range(0, n, 4001):  # local homologs: high scores, a best hit that is not 0
        a = int(rng.integers(0, 50))
        m = min(L, 100 - a)
        res[k * L:k * L + m] = q[a:a + m]
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        if L != 150:
            monkeypatch.setenv("SWBANK_STREAM", "2")
        kern = _check(monkeypatch, bank, q, res, offs, lens, REF, False, rng)
        if L != 150:
            monkeypatch.delenv("SWBANK_STREAM", raising=False)
    assert " pair " in kern or L == 1, kern


@pytest.mark.parametrize("case", ["nibble-mid", "nibble-all", "u16", "gotoh-f16", "gotoh-u16",
                                  "lut-f16", "gotoh-lut", "gotoh-f16-256"])
def test_stream_variants(monkeypatch, case):
    """4-bit chunks from the first chunk holding an N on; the row-LUT variants (u16, Gotoh
    R = 16, f16 without pair tables)."""
    monkeypatch.setenv("SWBANK_STREAM", "2")
    rng = np.random.default_rng(len(case) * 7)
    n, L = 40_000, 120
    res, offs, lens = _uniform(rng, n, L)
    extra = []
    if case == "nibble-mid":  # N codes only from target 25000 on: 2-bit chunks, then 4-bit
        tail = res[25000 * L:]
        tail[rng.random(tail.size) < 0.01] = 4
        extra = list(range(24900, 25100))
    if case == "nibble-all":
        res[rng.random(res.size) < 0.02] = 4
    if case in ("lut-f16", "gotoh-lut"):
        monkeypatch.setenv("SWBANK_PAIR", "0")
    if case in ("u16", "gotoh-u16"):
        monkeypatch.setenv("SWBANK_F16", "0")
    gotoh = case.startswith("gotoh")
    params = (5, -4, -10, -1) if gotoh else REF
    # (256 rows: a 16-wave Gotoh workgroup, the largest pair table beside the ring)
    q = rng.integers(0, 4, 256 if case.endswith("256") else 140, dtype=np.uint8)
    with S.ScoreBank(gap_model=S.GAP_GOTOH if gotoh else S.GAP_MERGED) as bank:
        bank.set_penalties(*params)
        bank.load_query(q)
        got = bank.score_batch(res, offs, lens)
        kern = bank.last_kernel()
        monkeypatch.setenv("SWBANK_STREAM", "0")
        ref = bank.score_batch(res, offs, lens)
        monkeypatch.setenv("SWBANK_STREAM", "2")
    assert "streamed=" in kern, kern
    if case in ("u16", "gotoh-u16"):
        assert kern.startswith("tile u16"), kern
    if case in ("lut-f16", "gotoh-lut"):
        assert kern.startswith("tile f16 R=") and " pair " not in kern, kern
    if case.startswith("gotoh-f16"):
        assert kern.startswith("tile f16 pair R=32"), kern
    assert np.array_equal(got, ref), kern
    sel = np.unique(np.concatenate([rng.choice(n, 500, replace=False), np.asarray(extra, int),
                                    np.arange(n - 128, n)]))
    sub = [res[int(offs[k]):int(offs[k]) + L] for k in sel]
    want = O.score_batch(q, *S.pack_targets(sub), O.dna_matrix(*params[:2]), *params[2:],
                         O.GAP_GOTOH if gotoh else O.GAP_MERGED)
    assert np.array_equal(got[sel], want), kern


@pytest.mark.parametrize("where", ["first", "middle", "last"])
@pytest.mark.parametrize("kind", ["code", "range"])
def test_stream_errors(monkeypatch, where, kind, poisoned_buffers):
    """A code outside the alphabet or a target past the residues, in the first, a middle or the
    last chunk: SW_ERR_ARG naming the target; the kernel drains (the chunks never sent are
    released as aborted) and the next call on the bank scores correctly."""
    monkeypatch.setenv("SWBANK_STREAM", "2")
    rng = np.random.default_rng(5)
    n, L = 30_000, 64
    res, offs, lens = _uniform(rng, n, L)
    k = {"first": 3, "middle": 17_000, "last": n - 2}[where]
    bad_res, bad_offs = res.copy(), offs.copy()
    if kind == "code":
        bad_res[k * L + 5] = 9
    else:
        bad_offs[k] = res.size - L + 1
    q = rng.integers(0, 4, 80, dtype=np.uint8)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        with pytest.raises(S.SwbankError) as ei:
            bank.score_batch(bad_res, bad_offs, lens)
        assert ei.value.status == S.ERR_ARG
        assert f"target {k}" in str(ei.value), str(ei.value)
        got = bank.score_batch(res, offs, lens)
        assert "streamed=" in bank.last_kernel()
    sel = rng.choice(n, 300, replace=False)
    sub = [res[int(offs[j]):int(offs[j]) + L] for j in sel]
    assert np.array_equal(got[sel], O.score_batch(q, *S.pack_targets(sub), O.dna_matrix(), -12, -4))


def test_stream_repeat_calls(monkeypatch):
    """Back-to-back calls reuse the codes buffer, the layout words and the records (no stale
    chunk from the previous call is read): different batches, different lengths."""
    monkeypatch.setenv("SWBANK_STREAM", "2")
    rng = np.random.default_rng(9)
    q = rng.integers(0, 4, 90, dtype=np.uint8)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        for n, L in [(20_000, 100), (9_000, 40), (20_000, 100), (50_000, 7)]:
            res, offs, lens = _uniform(rng, n, L, p_n=0.005 if L == 40 else 0.0)
            got = bank.score_batch(res, offs, lens)
            assert "streamed=" in bank.last_kernel()
            sel = rng.choice(n, 300, replace=False)
            sub = [res[int(offs[j]):int(offs[j]) + L] for j in sel]
            assert np.array_equal(got[sel], O.score_batch(q, *S.pack_targets(sub),
                                                          O.dna_matrix(), -12, -4))


def test_stream_same_shape_new_data(monkeypatch):
    """Two streamed calls of the same shape (the same chunk ranges of the reused device buffer)
    with different codes: the second call's scores are all exact (no line of the first call's
    codes is read stale), against the chunked feeder on every target."""
    rng = np.random.default_rng(5)
    q = rng.integers(0, 4, 128, dtype=np.uint8)
    n, L = 300_000, 128
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        first = _uniform(rng, n, L)
        bank.score_batch(*first)
        res, offs, lens = _uniform(rng, n, L)
        res[: 100 * L] = np.tile(q[:L], 100)[: 100 * L]  # a different best hit
        got = bank.score_batch(res, offs, lens)
        assert "streamed=" in bank.last_kernel(), bank.last_kernel()
        monkeypatch.setenv("SWBANK_STREAM", "0")
        ref = bank.score_batch(res, offs, lens)
    assert np.array_equal(got, ref)


def test_stream_memory_cap_falls_back(monkeypatch):
    """A batch past the streamed path's memory cap (SWBANK_STREAM_MB) runs through the bounded
    chunked feeder with the same scores; the decline is counted (sw_bank_counters)."""
    rng = np.random.default_rng(6)
    q = rng.integers(0, 4, 100, dtype=np.uint8)
    res, offs, lens = _uniform(rng, 300_000, 150)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        ref = bank.score_batch(res, offs, lens)
        assert "streamed=" in bank.last_kernel()
        monkeypatch.setenv("SWBANK_STREAM_MB", "1")
        got = bank.score_batch(res, offs, lens)
        assert "streamed=" not in bank.last_kernel(), bank.last_kernel()
        c = bank.counters()
    assert c["stream_declined"] == 1 and c["stream_calls"] == 1 and c["chunked_calls"] == 1, c
    assert np.array_equal(got, ref)


def test_stream_with_other_banks(monkeypatch):
    """With several other banks (and their streams) open in the process, so streams share the
    process's hardware queues, the streamed call still runs streamed (its kernel on a queue of
    its own: no copy marker stuck behind it) and matches the chunked feeder."""
    rng = np.random.default_rng(21)
    q = rng.integers(0, 4, 100, dtype=np.uint8)
    others = [S.ScoreBank() for _ in range(4)]
    try:
        small = _uniform(rng, 3000, 90)
        for o in others:
            o.set_penalties(*REF)
            o.load_query(q)
            o.score_batch(*small)
        res, offs, lens = _uniform(rng, 300_000, 150)
        with S.ScoreBank() as bank:
            bank.set_penalties(*REF)
            bank.load_query(q)
            for _ in range(3):
                got = bank.score_batch(res, offs, lens)
                assert "streamed=" in bank.last_kernel(), bank.last_kernel()
            monkeypatch.setenv("SWBANK_STREAM", "0")
            ref = bank.score_batch(res, offs, lens)
        assert np.array_equal(got, ref)
    finally:
        for o in others:
            o.close()


def test_stream_stalled_chunk_reruns(monkeypatch, poisoned_buffers):
    """A chunk published past the kernel's wait bound (SWBANK_STREAM_HOLD_MS): the waiting waves
    mark it aborted, the kernel drains, and the call re-runs through the chunked feeder with
    exact scores; the bank stays usable for a streamed call afterwards."""
    import time
    monkeypatch.setenv("SWBANK_STREAM", "2")
    rng = np.random.default_rng(33)
    n, L = 40_000, 100
    res, offs, lens = _uniform(rng, n, L)
    q = rng.integers(0, 4, 90, dtype=np.uint8)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        monkeypatch.setenv("SWBANK_STREAM_HOLD_MS", "8000")
        t0 = time.perf_counter()
        got = bank.score_batch(res, offs, lens)
        dt = time.perf_counter() - t0
        kern = bank.last_kernel()
        monkeypatch.delenv("SWBANK_STREAM_HOLD_MS")
        print(f"stalled call {dt:.2f} s, {kern}")
        assert "streamed=" not in kern, kern  # the chunked re-run
        c = bank.counters()
        assert c["stream_reruns"] == 1 and c["chunked_calls"] == 1 and c["stream_calls"] == 0, c
        again = bank.score_batch(res, offs, lens)
        assert "streamed=" in bank.last_kernel()
        assert bank.counters()["stream_calls"] == 1
    assert np.array_equal(got, again)
    sel = rng.choice(n, 300, replace=False)
    sub = [res[int(offs[j]):int(offs[j]) + L] for j in sel]
    assert np.array_equal(got[sel], O.score_batch(q, *S.pack_targets(sub), O.dna_matrix(), -12, -4))


@pytest.mark.parametrize("layout", ["back-to-back", "reversed", "gaps", "partly"])
def test_stream_runs(monkeypatch, layout):
    """Parts whose targets lie back to back pack as one run; reversed order, gaps between
    targets, or a batch only partly back to back go target by target: the same scores either
    way (SWBANK_STREAM_RUNS=0 packs every target on its own), and the oracle's on a sample."""
    monkeypatch.setenv("SWBANK_STREAM", "2")
    rng = np.random.default_rng(len(layout))
    n, L = 30_000, 128
    seqs = rng.integers(0, 4, (n, L), dtype=np.uint8)
    if layout == "back-to-back":
        res, offs = seqs.reshape(-1), np.arange(n, dtype=np.uint64) * L
    elif layout == "reversed":
        res, offs = seqs[::-1].reshape(-1).copy(), (n - 1 - np.arange(n, dtype=np.uint64)) * L
    else:
        gap = 5 if layout == "gaps" else 0
        res = np.full(n * (L + gap) + L + 64, 3, np.uint8)
        offs = np.arange(n, dtype=np.uint64) * (L + gap)
        if layout == "partly":  # back to back, except one target every 7000 moved to the end
            for k in range(0, n, 7000):
                offs[k] = n * L  # all share one copy at the end
            res[n * L:n * L + L] = seqs[0]
            for k in range(0, n, 7000):
                seqs[k] = seqs[0]
        for k in range(n):
            if layout == "gaps" or offs[k] < n * L:
                res[int(offs[k]):int(offs[k]) + L] = seqs[k]
    lens = np.full(n, L, np.uint32)
    q = rng.integers(0, 4, 100, dtype=np.uint8)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        got = bank.score_batch(res, offs, lens)
        assert "streamed=" in bank.last_kernel()
        monkeypatch.setenv("SWBANK_STREAM_RUNS", "0")
        per = bank.score_batch(res, offs, lens)
    assert np.array_equal(got, per)
    sel = np.unique(np.concatenate([rng.choice(n, 300, replace=False), np.arange(0, n, 7000)]))
    want = O.score_batch(q, *S.pack_targets([seqs[k] for k in sel]), O.dna_matrix(), -12, -4)
    assert np.array_equal(got[sel], want)


def test_stream_concurrent_banks():
    """Two banks streaming on the same device from two host threads at once (ctypes releases
    the GIL): both kernels wait only on their own call's copies, so both finish, streamed or
    through the chunked re-run, with exact scores."""
    import threading
    rng = np.random.default_rng(44)
    qs = [rng.integers(0, 4, 100, dtype=np.uint8) for _ in range(2)]
    batches = [_uniform(rng, 300_000, 128) for _ in range(2)]
    out, kern, errs = [None, None], [None, None], []

    def work(i):
        try:
            with S.ScoreBank() as bank:
                bank.set_penalties(*REF)
                bank.load_query(qs[i])
                for _ in range(3):
                    out[i] = bank.score_batch(*batches[i])
                kern[i] = bank.last_kernel()
        except Exception as e:  # reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in th), "a streamed call did not return"
    assert not errs, errs
    print("kernels:", kern)
    for i in range(2):
        res, offs, lens = batches[i]
        sel = rng.choice(len(lens), 300, replace=False)
        sub = [res[int(offs[j]):int(offs[j]) + 128] for j in sel]
        want = O.score_batch(qs[i], *S.pack_targets(sub), O.dna_matrix(), -12, -4)
        assert np.array_equal(out[i][sel], want)


@pytest.mark.parametrize("L", [100, 232, 37, 1])
def test_stream_records(monkeypatch, L):
    """Equal-length CAPI records (sw_score_records) stream their 2-bit data bytes: the same
    scores as the byte path and the oracle, and the batch best hit carries the record's ID."""
    monkeypatch.setenv("SWBANK_STREAM", "2")
    rng = np.random.default_rng(L)
    n = 40_000
    seqs = [rng.integers(0, 4, L, dtype=np.uint8) for _ in range(n)]
    ids = rng.integers(0, 2**31, n)
    recs = S.make_records(seqs, ids)
    q = rng.integers(0, 4, 120, dtype=np.uint8)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        got = bank.score_records(recs)
        assert "streamed=" in bank.last_kernel(), bank.last_kernel()
        bid, bsc, bix = bank.best()
        ref = bank.score_targets(seqs)
    assert np.array_equal(got, ref)
    top = int(np.argmax(got))
    assert (bid, bsc, bix) == (int(ids[top]), int(got[top]), top)
    sel = rng.choice(n, 300, replace=False)
    want = O.score_batch(q, *S.pack_targets([seqs[k] for k in sel]), O.dna_matrix(), -12, -4)
    assert np.array_equal(got[sel], want)


@pytest.mark.parametrize("where", ["chunk0", "later", "too-long"])
def test_stream_records_other_lengths(monkeypatch, where, poisoned_buffers):
    """A record of another length ends streaming: in chunk 0 before the launch, later after
    the kernel drains; the chunked feeder then scores the call (exact), or reports a length
    past 232 (SW_ERR_ARG)."""
    monkeypatch.setenv("SWBANK_STREAM", "2")
    rng = np.random.default_rng(len(where))
    n, L = 40_000, 90
    seqs = [rng.integers(0, 4, L, dtype=np.uint8) for _ in range(n)]
    k = {"chunk0": 5, "later": 35_000, "too-long": 30_000}[where]
    seqs[k] = rng.integers(0, 4, 50, dtype=np.uint8)
    recs = S.make_records(seqs)
    if where == "too-long":
        recs[k, 4:6] = np.frombuffer(np.uint16(300).tobytes(), np.uint8)
    q = rng.integers(0, 4, 80, dtype=np.uint8)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        if where == "too-long":
            with pytest.raises(S.SwbankError) as ei:
                bank.score_records(recs)
            assert ei.value.status == S.ERR_ARG
            return
        got = bank.score_records(recs)
        assert "streamed=" not in bank.last_kernel(), bank.last_kernel()
    sel = np.unique(np.concatenate([rng.choice(n, 300, replace=False), [k]]))
    want = O.score_batch(q, *S.pack_targets([seqs[j] for j in sel]), O.dna_matrix(), -12, -4)
    assert np.array_equal(got[sel], want)


def _ragged(rng, n, lo, hi, p_n=0.0, gap=0):
    lens = rng.integers(lo, hi + 1, n).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gap)
    res = rng.integers(0, 4, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    if p_n:
        res[rng.random(res.size) < p_n] = 4
    return res, offs, lens


@pytest.mark.parametrize("case", ["2bit", "nibble", "empty", "gaps", "big", "u16", "gotoh",
                                  "shuffled", "noruns", "long"])
def test_stream_ragged(monkeypatch, poisoned_buffers, case):
    """Ragged batches stream (SWBANK_STREAM_RAGGED): each chunk carries its mixed offset words,
    lengths and longest-first order (placed while packing) ahead of its codes, the targets in
    2-bit codes or, when they hold an N, 4-bit codes; parts whose targets lie back to back pack
    as runs.  Scores equal the chunked feeder's (SWBANK_STREAM_RAGGED=0) and the oracle's on a
    sample."""
    if case != "big":
        monkeypatch.setenv("SWBANK_STREAM", "2")
    monkeypatch.setenv("SWBANK_STREAM_RAGGED", "1")
    if case == "noruns":
        monkeypatch.setenv("SWBANK_MIXED_RUNS", "0")
    rng = np.random.default_rng(len(case) * 13)
    n = 300_000 if case == "big" else 6_000 if case == "long" else 30_000
    lo, hi = {"empty": (0, 40), "big": (64, 150), "long": (300, 1500)}.get(case, (20, 200))
    p_n = 0.002 if case in ("nibble", "big", "shuffled", "noruns", "long") else 0.0
    res, offs, lens = _ragged(rng, n, lo, hi, p_n=p_n, gap=3 if case == "gaps" else 0)
    if case == "shuffled":  # offsets out of order: no part is a run
        perm = rng.permutation(n)
        offs, lens = offs[perm].copy(), lens[perm].copy()
    gotoh = case == "gotoh"
    params = (5, -4, -10, -1) if gotoh else REF
    if case == "u16":
        monkeypatch.setenv("SWBANK_F16", "0")
    q = rng.integers(0, 4, 110, dtype=np.uint8)
    with S.ScoreBank(gap_model=S.GAP_GOTOH if gotoh else S.GAP_MERGED) as bank:
        bank.set_penalties(*params)
        bank.load_query(q)
        got = bank.score_batch(res, offs, lens)
        kern = bank.last_kernel()
        best = bank.best()
        c = bank.counters()
        monkeypatch.setenv("SWBANK_STREAM_RAGGED", "0")
        ref = bank.score_batch(res, offs, lens)
    assert "streamed=" in kern, kern
    assert c["stream_calls"] == 1 and c["mixed_chunks"] >= 1, c
    if case in ("shuffled", "noruns"):
        assert c["mixed_runs"] == 0, c
    elif case != "empty":
        assert c["mixed_runs"] >= 1, c
    assert np.array_equal(got, ref), kern
    top = int(np.argmax(got))
    assert best[1:] == (int(got[top]), top)
    sel = np.unique(np.concatenate([rng.choice(n, 400, replace=False), np.arange(n - 130, n)]))
    sub = [res[int(offs[k]):int(offs[k]) + int(lens[k])] for k in sel]
    want = O.score_batch(q, *S.pack_targets(sub), O.dna_matrix(*params[:2]), *params[2:],
                         O.GAP_GOTOH if gotoh else O.GAP_MERGED)
    assert np.array_equal(got[sel], want), kern


def test_stream_ragged_back_to_back(monkeypatch, poisoned_buffers):
    """Three ragged streamed calls on one bank with other data and lengths each time: every
    call's scores are exact (no stale chunk codes, orders or offset words)."""
    monkeypatch.setenv("SWBANK_STREAM", "2")
    monkeypatch.setenv("SWBANK_STREAM_RAGGED", "1")
    rng = np.random.default_rng(5)
    q = rng.integers(0, 4, 96, dtype=np.uint8)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        for seed in range(3):
            res, offs, lens = _ragged(np.random.default_rng(100 + seed), 20_000, 30, 160,
                                      p_n=0.003)
            got = bank.score_batch(res, offs, lens)
            assert "streamed=" in bank.last_kernel()
            sel = rng.choice(len(lens), 300, replace=False)
            sub = [res[int(offs[j]):int(offs[j]) + int(lens[j])] for j in sel]
            want = O.score_batch(q, *S.pack_targets(sub), O.dna_matrix(), -12, -4)
            assert np.array_equal(got[sel], want), seed


@pytest.mark.parametrize("kind", ["code", "range"])
def test_stream_ragged_errors(monkeypatch, kind, poisoned_buffers):
    """A bad code or a target past the residues in a ragged streamed batch: SW_ERR_ARG naming
    the target, and the bank scores the next call.  The chunks never sent are released to the
    running kernel as aborted; with poisoned buffers their regions hold 0x3C bytes, which the
    kernel once read as offsets and visiting order (an illegal address): aborted targets now
    read as empty."""
    monkeypatch.setenv("SWBANK_STREAM", "2")
    monkeypatch.setenv("SWBANK_STREAM_RAGGED", "1")  # opt-in
    rng = np.random.default_rng(71)
    res, offs, lens = _ragged(rng, 30_000, 10, 120)
    k = 21_000
    bad_res, bad_offs = res.copy(), offs.copy()
    if kind == "code":
        bad_res[int(offs[k]) + 2] = 7
        lens[k] = max(lens[k], 5)
    else:
        bad_offs[k] = res.size - 1
        lens[k] = max(lens[k], 5)
    q = rng.integers(0, 4, 70, dtype=np.uint8)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        with pytest.raises(S.SwbankError) as ei:
            bank.score_batch(bad_res, bad_offs, lens)
        assert ei.value.status == S.ERR_ARG and f"target {k}" in str(ei.value), str(ei.value)
        got = bank.score_batch(res, offs, lens)
        assert "streamed=" in bank.last_kernel()
    sel = rng.choice(len(lens), 300, replace=False)
    sub = [res[int(offs[j]):int(offs[j]) + int(lens[j])] for j in sel]
    assert np.array_equal(got[sel], O.score_batch(q, *S.pack_targets(sub), O.dna_matrix(), -12, -4))


@pytest.mark.parametrize("seed", range(24))
def test_stream_ragged_fuzz(monkeypatch, seed):
    """Seeded ragged streamed batches: random lengths (incl. empty), N rates, gaps between and
    shuffles of the targets in the residues, match/mismatch/gap penalties, both gap models and
    f16/u16 -- every call equal to the chunked feeder's scores and to the oracle on a sample."""
    rng = np.random.default_rng(9000 + seed)
    monkeypatch.setenv("SWBANK_STREAM", "2")
    monkeypatch.setenv("SWBANK_STREAM_RAGGED", "1")
    if rng.random() < 0.3:
        monkeypatch.setenv("SWBANK_F16", "0")
    if rng.random() < 0.2:
        monkeypatch.setenv("SWBANK_MIXED_RUNS", "0")
    n = int(rng.integers(300, 20_000))
    lo = int(rng.integers(0, 60))
    hi = lo + int(rng.integers(1, 400))
    res, offs, lens = _ragged(rng, n, lo, hi, p_n=float(rng.choice([0.0, 0.0005, 0.01, 0.2])),
                              gap=int(rng.choice([0, 0, 1, 5])))
    if rng.random() < 0.25:
        perm = rng.permutation(n)
        offs, lens = offs[perm].copy(), lens[perm].copy()
    ma, mm = int(rng.integers(1, 8)), -int(rng.integers(1, 8))
    go, ge = -int(rng.integers(1, 16)), -int(rng.integers(1, 5))
    gotoh = rng.random() < 0.4
    q = rng.integers(0, 4, int(rng.integers(1, 200)), dtype=np.uint8)
    with S.ScoreBank(gap_model=S.GAP_GOTOH if gotoh else S.GAP_MERGED) as bank:
        bank.set_penalties(ma, mm, go, ge)
        bank.load_query(q)
        got = bank.score_batch(res, offs, lens)
        kern = bank.last_kernel()
        monkeypatch.setenv("SWBANK_STREAM_RAGGED", "0")
        ref = bank.score_batch(res, offs, lens)
    assert np.array_equal(got, ref), kern
    sel = np.unique(np.concatenate([rng.choice(n, min(n, 200), replace=False), [n - 1]]))
    sub = [res[int(offs[k]):int(offs[k]) + int(lens[k])] for k in sel]
    want = O.score_batch(q, *S.pack_targets(sub), O.dna_matrix(ma, mm), go, ge,
                         O.GAP_GOTOH if gotoh else O.GAP_MERGED)
    assert np.array_equal(got[sel], want), kern
