"""GPU: the host-buffer feeder of sw_score_batch / sw_score_records (chunks in input order,
pinned staging slots, copy stream, a longest-first permutation per chunk).

Forced to many small chunks (SWBANK_CHUNK_MB=1) with ragged lengths, so several chunks are in
flight at once and each carries its own permutation; the scores must equal the device-API
path's (one launch over the whole batch, caller's order) and the oracle's."""
import numpy as np
import pytest

import swbank as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu

REF = (5, -4, -12, -4)


def _ragged(rng, n, lo, hi, A=4):
    lens = rng.integers(lo, hi + 1, n).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    res = rng.integers(0, A, int(lens.sum()), dtype=np.uint8)
    return res, offs, lens


def _device_scores(bank, res, offs, lens):
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.astype(np.int32)).to(dev)
    d_sc = torch.zeros(len(lens), dtype=torch.int32, device=dev)
    s = torch.cuda.Stream()
    bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), len(lens),
                            int(lens.max()), d_sc.data_ptr(), s.cuda_stream)
    s.synchronize()
    return d_sc.cpu().numpy()


@pytest.mark.parametrize("host_dsort", ["1", "0"])
@pytest.mark.parametrize("chunk_mb", ["1", "3"])
def test_feeder_many_chunks_ragged(monkeypatch, chunk_mb, host_dsort):
    """ragged chunks visited longest first, the order sorted on the device into each chunk's
    slot (SWBANK_HOST_DSORT=1, default) or on the host (0)"""
    monkeypatch.setenv("SWBANK_CHUNK_MB", chunk_mb)
    monkeypatch.setenv("SWBANK_HOST_DSORT", host_dsort)
    rng = np.random.default_rng(11)
    res, offs, lens = _ragged(rng, 60000, 0, 220)  # ~6.6 MB of codes: 2-7 chunks
    q = rng.integers(0, 4, 100, dtype=np.uint8)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        got = bank.score_batch(res, offs, lens)
        dev = _device_scores(bank, res, offs, lens)
    assert np.array_equal(got, dev)
    sel = rng.choice(len(lens), 3000, replace=False)
    sub = [res[int(offs[k]):int(offs[k]) + int(lens[k])] for k in sel]
    want = O.score_batch(q, *S.pack_targets(sub), O.dna_matrix(*REF[:2]), *REF[2:])
    assert np.array_equal(got[sel], want)


def test_feeder_scattered_offsets(monkeypatch):
    """offsets in any order and with gaps (the caller's layout, not the feeder's)"""
    monkeypatch.setenv("SWBANK_CHUNK_MB", "1")
    rng = np.random.default_rng(12)
    res, offs, lens = _ragged(rng, 30000, 1, 150)
    n = len(lens)
    perm = rng.permutation(n)                 # target j of the new batch = old target perm[j]
    lens2 = lens[perm]
    gap = np.full(int(lens.sum()) + 7 * n, 3, np.uint8)
    offs2 = np.zeros(n, np.uint64)
    cursor = 0
    for j in rng.permutation(n):              # laid out in memory in yet another order
        offs2[j] = cursor
        k = int(perm[j])
        gap[cursor:cursor + int(lens2[j])] = res[int(offs[k]):int(offs[k]) + int(lens[k])]
        cursor += int(lens2[j]) + 7
    q = rng.integers(0, 4, 64, dtype=np.uint8)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        base = bank.score_batch(res, offs, lens)
        got = bank.score_batch(gap, offs2, lens2)
    assert np.array_equal(got, base[perm])


def test_feeder_bad_code_in_late_chunk(monkeypatch):
    monkeypatch.setenv("SWBANK_CHUNK_MB", "1")
    rng = np.random.default_rng(13)
    res, offs, lens = _ragged(rng, 30000, 50, 150)
    bad = 27000
    res[int(offs[bad]) + 3] = 9
    q = rng.integers(0, 4, 64, dtype=np.uint8)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        with pytest.raises(S.SwbankError) as ei:
            bank.score_batch(res, offs, lens)
        assert ei.value.status == S.ERR_ARG and f"target {bad} code 9" in str(ei.value)
        res[int(offs[bad]) + 3] = 1  # the bank stays usable after the error
        got = bank.score_batch(res, offs, lens)
        assert np.array_equal(got, _device_scores(bank, res, offs, lens))


@pytest.mark.parametrize("point", [3, 5])
def test_feeder_hip_failure_mid_call(monkeypatch, point):
    """a HIP failure reported while chunk jobs are still queued on the launch thread
    (SWBANK_FEED_FAULT=k, a test hook: sync point k fails) returns SW_ERR_HIP after draining
    the launch thread and the streams, and the bank scores the next batch exactly"""
    monkeypatch.setenv("SWBANK_CHUNK_MB", "1")
    rng = np.random.default_rng(14)
    res, offs, lens = _ragged(rng, 60000, 40, 180)  # ~6.6 MB of codes: 7 chunks
    q = rng.integers(0, 4, 64, dtype=np.uint8)
    k = point
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        want = _device_scores(bank, res, offs, lens)
        monkeypatch.setenv("SWBANK_FEED_FAULT", str(k))
        with pytest.raises(S.SwbankError) as ei:
            bank.score_batch(res, offs, lens)
        assert ei.value.status == S.ERR_HIP, str(ei.value)
        monkeypatch.delenv("SWBANK_FEED_FAULT")
        for _ in range(2):
            assert np.array_equal(bank.score_batch(res, offs, lens), want)


def test_feeder_records_many_chunks(monkeypatch):
    monkeypatch.setenv("SWBANK_CHUNK_MB", "1")
    rng = np.random.default_rng(14)
    n = 50000  # 3.2 MB of records: 4 chunks
    L = rng.integers(1, S.RECORD_MAX_BASES + 1, n)
    seqs = [rng.integers(0, 4, int(l), dtype=np.uint8) for l in L]
    recs = S.make_records(seqs)
    q = rng.integers(0, 4, 120, dtype=np.uint8)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        got = bank.score_records(recs)
        want = bank.score_targets(seqs)
        assert np.array_equal(got, want)
        recs[40000, 4:6] = np.frombuffer(np.uint16(S.RECORD_MAX_BASES + 1).tobytes(), np.uint8)
        with pytest.raises(S.SwbankError) as ei:
            bank.score_records(recs)
        assert ei.value.status == S.ERR_ARG and "record 40000" in str(ei.value)


@pytest.mark.parametrize("avx2", ["1", "0"])
@pytest.mark.parametrize("case", ["merged", "gotoh", "profile", "long-query", "wave"])
def test_feeder_two_bit_chunks(monkeypatch, case, avx2):
    """DNA chunks without N cross PCIe as the 2-bit stream (SWK_PACK_STREAM, each target from
    a byte boundary); the chunk holding an N and those after it cross as 4-bit codes
    (SWK_PACK_NIBBLE).  Ragged lengths 0-300
    (every residue count mod 4/8/16, empty targets), N only in the middle of the batch, several
    chunks in flight: the scores equal the byte path's (SWBANK_PACK2=0) and the oracle's."""
    monkeypatch.setenv("SWBANK_CHUNK_MB", "1")
    monkeypatch.setenv("SWBANK_AVX2", avx2)
    if case == "profile":
        monkeypatch.setenv("SWBANK_PROFILE", "1")
    if case == "wave":
        monkeypatch.setenv("SWBANK_KERNEL", "wave")
    rng = np.random.default_rng(len(case) * 7919)
    res, offs, lens = _ragged(rng, 24000, 0, 300)  # ~3.6 MB of codes: 3-4 chunks
    mid = slice(int(offs[10000]), int(offs[10400]))
    res[mid][rng.random(mid.stop - mid.start) < 0.05] = 4  # N in one chunk only
    qlen = 700 if case == "long-query" else 120
    q = rng.integers(0, 4, qlen, dtype=np.uint8)
    gotoh = case == "gotoh"
    params = (5, -4, -10, -1) if gotoh else REF
    with S.ScoreBank(gap_model=S.GAP_GOTOH if gotoh else S.GAP_MERGED) as bank:
        bank.set_penalties(*params)
        bank.load_query(q)
        got = bank.score_batch(res, offs, lens)
        kern = bank.last_kernel()
        monkeypatch.setenv("SWBANK_PACK2", "0")
        ref = bank.score_batch(res, offs, lens)
    assert np.array_equal(got, ref), kern
    if case == "wave":
        assert kern.startswith("wave"), kern
    sel = np.concatenate([np.arange(10000, 10400), rng.choice(len(lens), 1500, replace=False)])
    sub = [res[int(offs[k]):int(offs[k]) + int(lens[k])] for k in sel]
    want = O.score_batch(q, *S.pack_targets(sub), O.dna_matrix(*params[:2]), *params[2:],
                         O.GAP_GOTOH if gotoh else O.GAP_MERGED)
    assert np.array_equal(got[sel], want), kern


@pytest.mark.parametrize("case", ["2bit", "nibble", "protein", "wave", "long-query", "opt16"])
def test_feeder_uniform_chunks(monkeypatch, case):
    """Equal-length chunks cross PCIe as codes only (no per-target offsets / lengths: the
    kernels compute them from the chunk's length and stride); the scores equal the headers path
    (SWBANK_UNIFORM=0) and the oracle's, for 2-bit, 4-bit and byte chunks, both kernels, a
    segmented query and an optimistic f16 pass with its u16 re-score."""
    monkeypatch.setenv("SWBANK_CHUNK_MB", "1")
    rng = np.random.default_rng(len(case) * 31)
    prot = case == "protein"
    A = 20 if prot else 4
    L = {"long-query": 90, "opt16": 300}.get(case, 133)
    n = 20000
    lens = np.full(n, L, np.uint32)
    offs = np.arange(n, dtype=np.uint64) * L
    res = rng.integers(0, A, n * L, dtype=np.uint8)
    if case == "nibble":
        res[rng.random(res.size) < 0.01] = 4
    if case == "wave":
        monkeypatch.setenv("SWBANK_KERNEL", "wave")
    qlen = {"long-query": 1100, "opt16": 600}.get(case, 100)
    q = rng.integers(0, A, qlen, dtype=np.uint8)
    if case == "opt16":  # near-copies of the query: scores far past 2048 (u16 re-score)
        for k in range(0, n, 97):
            res[k * L:(k + 1) * L] = q[:L]
    kw = dict(alphabet=S.ALPHABET_PROTEIN, gap_model=S.GAP_GOTOH) if prot else {}
    with S.ScoreBank(**kw) as bank:
        if prot:
            bank.set_matrix(O.BLOSUM62, -11, -1)
        else:
            bank.set_penalties(*REF)
        bank.load_query(q)
        got = bank.score_batch(res, offs, lens)
        kern = bank.last_kernel()
        monkeypatch.setenv("SWBANK_UNIFORM", "0")
        ref = bank.score_batch(res, offs, lens)
    assert np.array_equal(got, ref), kern
    sel = rng.choice(n, 400, replace=False)
    if case == "opt16":
        sel = np.concatenate([sel, np.arange(0, n, 97)[:60]])
    sub = [res[int(offs[k]):int(offs[k]) + L] for k in sel]
    if prot:
        want = O.score_batch(q, *S.pack_targets(sub), O.BLOSUM62, -11, -1, O.GAP_GOTOH)
    else:
        want = O.score_batch(q, *S.pack_targets(sub), O.dna_matrix(*REF[:2]), *REF[2:])
    assert np.array_equal(got[sel], want), kern


@pytest.mark.parametrize("case", ["sparse-n", "dense-n", "no-n", "tiny", "one-tile", "gotoh",
                                  "long-query"])
def test_feeder_mixed_chunks(monkeypatch, poisoned_buffers, case):
    """Ragged DNA chunks as SWK_PACK_MIXED: each target in 2-bit codes from an even byte, or in
    4-bit codes from an odd byte when it holds an N, u32 offsets, the longest-first order
    sorted on the device after the codes.  Equal to the whole-chunk layouts (SWBANK_MIXED=0)
    and to the oracle; the counter shows the chunks took the mixed layout."""
    monkeypatch.setenv("SWBANK_CHUNK_MB", "1")
    monkeypatch.setenv("SWBANK_KERNEL", "tile")
    rng = np.random.default_rng(len(case) * 13)
    n, lo, hi = {"tiny": (20_000, 0, 9), "one-tile": (100, 0, 300)}.get(case, (30_000, 1, 250))
    res, offs, lens = _ragged(rng, n, lo, hi)
    p_n = {"sparse-n": 0.001, "dense-n": 0.05, "no-n": 0.0, "tiny": 0.02}.get(case, 0.003)
    res[rng.random(res.size) < p_n] = 4
    qlen = 700 if case == "long-query" else 100
    q = rng.integers(0, 4, qlen, dtype=np.uint8)
    for k in range(0, n, 97):  # homologs (high scores, long gapped alignments)
        m = min(int(lens[k]), qlen)
        res[int(offs[k]):int(offs[k]) + m] = q[:m]
    gotoh = case == "gotoh"
    params = (5, -4, -10, -1) if gotoh else REF
    with S.ScoreBank(gap_model=S.GAP_GOTOH if gotoh else S.GAP_MERGED) as bank:
        bank.set_penalties(*params)
        bank.load_query(q)
        got = bank.score_batch(res, offs, lens)
        mixed = bank.counters()["mixed_chunks"]
        monkeypatch.setenv("SWBANK_MIXED", "0")
        ref = bank.score_batch(res, offs, lens)
        assert bank.counters()["mixed_chunks"] == mixed
    assert mixed >= 1, case
    assert np.array_equal(got, ref), np.nonzero(got != ref)[0][:8]
    sel = np.unique(np.concatenate([rng.choice(n, min(n, 700), replace=False),
                                    np.arange(0, n, 97), np.arange(max(0, n - 130), n)]))
    sub = [res[int(offs[k]):int(offs[k]) + int(lens[k])] for k in sel]
    want = O.score_batch(q, *S.pack_targets(sub), O.dna_matrix(*params[:2]), *params[2:],
                         O.GAP_GOTOH if gotoh else O.GAP_MERGED)
    assert np.array_equal(got[sel], want)


@pytest.mark.parametrize("layout", ["runs", "gaps", "empties", "shuffled", "runs-off"])
def test_feeder_mixed_runs(monkeypatch, poisoned_buffers, layout):
    """Mixed chunks whose pool parts hold targets back to back in the residues pack each part
    as ONE run (targets start inside a byte, offset word = 2-bit position << 1; the N targets
    found from the run packer's positions and re-packed in 4-bit codes): "runs" back to back,
    "gaps" small gaps between targets (packed with the run), "empties" zero-length targets at
    offset 0 in between, "shuffled" offsets out of order (one packer call per target), and
    "runs-off" (SWBANK_MIXED_RUNS=0).  Scores equal the whole-chunk layouts and the oracle; the
    counter shows which form ran."""
    monkeypatch.setenv("SWBANK_CHUNK_MB", "1")
    monkeypatch.setenv("SWBANK_KERNEL", "tile")
    if layout == "runs-off":
        monkeypatch.setenv("SWBANK_MIXED_RUNS", "0")
    rng = np.random.default_rng(17 + len(layout))
    n = 40_000
    lens = rng.integers(1, 180, n).astype(np.uint32)
    gap = rng.integers(0, 4, n) if layout == "gaps" else np.zeros(n, np.int64)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gap[:-1].astype(np.uint64))
    total = int(offs[-1] + lens[-1])
    res = rng.integers(0, 4, total + 8, dtype=np.uint8)
    res[rng.random(res.size) < 0.002] = 4  # N, also in the gaps (must not mark a neighbour)
    if layout == "empties":
        e = rng.random(n) < 0.05
        lens[e] = 0
        offs[e] = 0
    if layout == "shuffled":
        p = rng.permutation(n)
        offs, lens = offs[p].copy(), lens[p].copy()
    q = rng.integers(0, 4, 120, dtype=np.uint8)
    for k in range(0, n, 89):  # homologs: high scores that a wrong code would change
        m = min(int(lens[k]), 120)
        res[int(offs[k]):int(offs[k]) + m] = q[:m]
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        got = bank.score_batch(res, offs, lens)
        c = bank.counters()
        monkeypatch.setenv("SWBANK_MIXED", "0")
        ref = bank.score_batch(res, offs, lens)
    assert c["mixed_chunks"] >= 1
    if layout in ("runs", "gaps", "empties"):
        assert c["mixed_runs"] >= c["mixed_chunks"], c
    else:
        assert c["mixed_runs"] == 0, c
    assert np.array_equal(got, ref), np.nonzero(got != ref)[0][:8]
    sel = np.unique(np.concatenate([rng.choice(n, 800, replace=False), np.arange(0, n, 89),
                                    np.arange(n - 130, n)]))
    sub = [res[int(offs[k]):int(offs[k]) + int(lens[k])] for k in sel]
    want = O.score_batch(q, *S.pack_targets(sub), O.dna_matrix(*REF[:2]), *REF[2:])
    assert np.array_equal(got[sel], want)


def test_feeder_mixed_bad_code(monkeypatch):
    """A code outside the alphabet in a mixed chunk: the byte path reports the target."""
    monkeypatch.setenv("SWBANK_CHUNK_MB", "1")
    rng = np.random.default_rng(5)
    res, offs, lens = _ragged(rng, 30_000, 5, 200)
    res[rng.random(res.size) < 0.002] = 4
    k = 20_000
    bad = res.copy()
    bad[int(offs[k]) + 1] = 9
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(rng.integers(0, 4, 100, dtype=np.uint8))
        with pytest.raises(S.SwbankError) as ei:
            bank.score_batch(bad, offs, lens)
        assert ei.value.status == S.ERR_ARG and f"target {k}" in str(ei.value)
        assert (bank.score_batch(res, offs, lens) >= 0).all()


@pytest.mark.parametrize("n,want_chunks", [(12_500, 1), (60_000, None)])
def test_feeder_wave_batch_chunk_floor(monkeypatch, n, want_chunks):
    """A host batch the wave kernel takes (configs[4]'s protein shape) is cut in chunks of at
    least one unit per resident wave slot: 12,500 x 1,000 aa go as ONE launch (they went as
    three, each leaving SIMDs idle for a unit's time), a larger batch as several whose every
    launch still fills the slots; scores equal the device API's and the oracle's."""
    torch = pytest.importorskip("torch")
    monkeypatch.delenv("SWBANK_CHUNK_MB", raising=False)
    rng = np.random.default_rng(n)
    L = 1000
    res = rng.integers(0, 20, n * L, dtype=np.uint8)
    offs = np.arange(n, dtype=np.uint64) * L
    lens = np.full(n, L, np.uint32)
    q = rng.integers(0, 20, 512, dtype=np.uint8)
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN, gap_model=S.GAP_GOTOH) as bank:
        bank.set_matrix(O.BLOSUM62, -11, -1)
        bank.load_query(q)
        bank.timing()
        bank.set_timing(True)
        got = bank.score_batch(res, offs, lens)
        launches, _, _ = bank.timing()
        bank.set_timing(False)
        kern = bank.last_kernel()
        dev = torch.device("cuda", 0)
        d_sc = torch.full((n,), -1, dtype=torch.int32, device=dev)
        d_res = torch.from_numpy(res).to(dev)
        d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
        d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, L,
                                d_sc.data_ptr(), min_len=L)
        torch.cuda.synchronize()
    assert kern.startswith("wave"), kern
    if want_chunks is not None:
        assert launches == want_chunks, (launches, kern)
    else:
        assert 1 < launches <= n // 12_000, (launches, kern)  # each >= 16 x 768 targets
    assert np.array_equal(got, d_sc.cpu().numpy())
    sel = rng.choice(n, 120, replace=False)
    sub = [res[int(offs[k]):int(offs[k]) + L] for k in sel]
    want = O.score_batch(q, *S.pack_targets(sub), O.BLOSUM62, -11, -1, O.GAP_GOTOH)
    assert np.array_equal(got[sel], want), kern
