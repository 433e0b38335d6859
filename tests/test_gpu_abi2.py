"""GPU: the ABI-2 surface — scores past the 16-bit lanes (int32 re-score), the batch best hit
with caller ids (≙ ScoreBank_v2.v:39-43 results/IDs/max), the on-device length sort of ragged
device batches, device records with corrupt lengths, and multi-device banks (the RTL's
MODULES, ScoreBank_v2.v:76-148) with their RCCL / copy score gather.

Every score is checked bit-exact against the oracle (test infrastructure only)."""
import os

import numpy as np
import pytest

import swbank as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu

REF = (5, -4, -12, -4)


def _codes(rng, n, alpha=4):
    return rng.integers(0, alpha, n, dtype=np.uint8)


def _mutate(rng, s, p, alpha=4):
    t = s.copy()
    m = rng.random(len(t)) < p
    t[m] = rng.integers(0, alpha, int(m.sum()), dtype=np.uint8)
    return t


# ---- int32: scores past 65535 -------------------------------------------------------------
@pytest.mark.parametrize("kernel", ["tile", "wave"])
def test_scores_past_16_bits_dna(kernel, monkeypatch):
    """A 14,000-bp query against near-copies of itself: self score 70,000 > 65,535.  The
    16-bit pass flags those pairs and the int32 kernel re-scores them exactly."""
    monkeypatch.setenv("SWBANK_KERNEL", kernel)
    rng = np.random.default_rng(11)
    q = _codes(rng, 14000)
    seqs = [q.copy(), _mutate(rng, q, 0.01), _mutate(rng, q, 0.2), q[:9000].copy(),
            _codes(rng, 300), np.zeros(0, np.uint8), q[5000:].copy()]
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        got = bank.score_targets(seqs)
        kern = bank.last_kernel()
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)
    assert want[0] == 70000 and want.max() > 65535
    assert (got == want).all(), (kern, got.tolist(), want.tolist())
    assert "+i32-rescore" in kern


def test_scores_past_16_bits_protein_gotoh():
    """BLOSUM62 / Gotoh: a 13,000-aa query (SWB_MAX_QUERY is 65,536 now) against itself and
    mutants; the self score is above the 16-bit bound."""
    rng = np.random.default_rng(12)
    q = rng.integers(0, 20, 13000, dtype=np.uint8)
    seqs = [q.copy(), _mutate(rng, q, 0.05, 20), rng.integers(0, 20, 700, dtype=np.uint8)]
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN, gap_model=S.GAP_GOTOH) as bank:
        bank.set_matrix(O.BLOSUM62, -11, -1)
        bank.load_query(q)
        got = bank.score_targets(seqs)
        kern = bank.last_kernel()
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.BLOSUM62, -11, -1, O.GAP_GOTOH)
    assert want[0] > 65535
    assert (got == want).all(), (kern, got.tolist(), want.tolist())


@pytest.mark.parametrize("case", ["dna-ref", "dna-col0", "dna-gotoh", "prot-merged",
                                  "prot-gotoh", "dna-N"])
@pytest.mark.parametrize("qlen", [1, 5, 63, 64, 255, 256, 257, 700])
def test_int32_kernel_everywhere(case, qlen, monkeypatch):
    """SWBANK_I32=1 routes every pair through the int32 kernel (after the 16-bit pass), so the
    kernel itself is checked on random shapes, both gap models, the HDL column-0 rule, protein
    and N codes, across strip boundaries (256 rows)."""
    monkeypatch.setenv("SWBANK_I32", "1")
    rng = np.random.default_rng(hash((case, qlen)) % 2**32)
    prot = case.startswith("prot")
    alpha = 20 if prot else 4
    model = S.GAP_GOTOH if case.endswith("gotoh") else S.GAP_MERGED
    q = rng.integers(0, alpha, qlen, dtype=np.uint8)
    seqs = [rng.integers(0, alpha, int(rng.integers(0, 400)), dtype=np.uint8) for _ in range(150)]
    seqs += [_mutate(rng, q, 0.1, alpha), q[: qlen // 2].copy()]
    if case == "dna-N":
        for t in seqs[:40]:
            t[rng.random(len(t)) < 0.1] = 4
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN if prot else S.ALPHABET_DNA,
                     gap_model=model) as bank:
        if prot:
            sub, go, ge = O.BLOSUM62, -11, -1
            bank.set_matrix(sub, go, ge)
        else:
            pen = {"dna-col0": (9, -3, -2, -1)}.get(case, REF)
            sub, go, ge = O.dna_matrix(pen[0], pen[1]), pen[2], pen[3]
            bank.set_penalties(*pen)
        bank.load_query(q)
        got = bank.score_targets(seqs)
        assert "+i32-rescore" in bank.last_kernel()
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, sub.astype(np.int8), go, ge, model)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), int(lens[i]), int(got[i]), int(want[i])) for i in bad[:6]]


def test_int32_kernel_on_records(monkeypatch):
    monkeypatch.setenv("SWBANK_I32", "1")
    rng = np.random.default_rng(5)
    q = _codes(rng, 300)
    seqs = [_codes(rng, int(rng.integers(0, 233))) for _ in range(300)]
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        got = bank.score_records(S.make_records(seqs))
    res, offs, lens = O.pack_residues(seqs)
    assert (got == O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)).all()


# ---- batch best hit with ids ---------------------------------------------------------------
def test_batch_best_host_device_and_records():
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(21)
    q = _codes(rng, 128)
    seqs = [_codes(rng, int(rng.integers(1, 200))) for _ in range(3000)]
    seqs[1234] = q.copy()                      # the unique best
    seqs[2345] = q.copy()                      # a tie: the lower index wins
    ids = (np.arange(len(seqs), dtype=np.uint64) * 7919 + (1 << 40))
    res, offs, lens = O.pack_residues(seqs)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        sc = bank.score_batch(res, offs, lens, ids=ids)
        assert bank.best() == (int(ids[1234]), 640, 1234)
        bank.score_batch(res, offs, lens)      # no ids: the id is the index
        assert bank.best() == (1234, 640, 1234)
        dev = torch.device("cuda", torch.cuda.current_device())
        d_res = torch.from_numpy(res).to(dev)
        d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
        d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
        d_ids = torch.from_numpy(ids.view(np.int64)).to(dev)
        d_sc = torch.zeros(len(seqs), dtype=torch.int32, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(),
                                len(seqs), int(lens.max()), d_sc.data_ptr(), st,
                                d_ids=d_ids.data_ptr())
        assert bank.best() == (int(ids[1234]), 640, 1234)
        assert (d_sc.cpu().numpy() == sc).all()
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(),
                                len(seqs), int(lens.max()), d_sc.data_ptr(), st)
        with pytest.raises(S.SwbankError) as e:  # a device call without ids records nothing
            bank.best()
        assert e.value.status == S.ERR_STATE
        short = [s[:232] for s in seqs]
        rec = S.make_records(short, ids=[int(i) & 0xFFFFFFFF for i in ids])
        rs = bank.score_records(rec)
        b = int(np.argmax(rs))
        assert bank.best() == (int(ids[b]) & 0xFFFFFFFF, int(rs[b]), b)


# ---- ragged device batches: on-device length sort -------------------------------------------
@pytest.mark.parametrize("lo,hi", [(64, 128), (1, 150), (0, 1000), (100, 101), (128, 128)])
def test_device_sort_ragged(lo, hi, monkeypatch):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(lo * 1000 + hi)
    q = _codes(rng, 150)
    n = 20000
    lens0 = rng.integers(lo, hi + 1, n)
    seqs = [_codes(rng, int(l)) for l in lens0]
    for t in seqs[::97]:
        t[rng.random(len(t)) < 0.05] = 4
    res, offs, lens = O.pack_residues(seqs)
    dev = torch.device("cuda", torch.cuda.current_device())
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    out = {}
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        for dsort in ("1", "0"):
            monkeypatch.setenv("SWBANK_DSORT", dsort)
            d_sc = torch.full((n,), -1, dtype=torch.int32, device=dev)
            bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n,
                                    max(int(lens.max()), 1), d_sc.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            out[dsort] = d_sc.cpu().numpy()
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)
    assert (out["1"] == want).all() and (out["0"] == want).all()


@pytest.mark.parametrize("lo,hi", [(128, 128), (100, 101), (64, 150), (0, 3000)])
def test_device_range_skips_sort_on_one_length(lo, hi):
    """sw_score_batch_device_range: with the caller's length range the sort kernels run only
    when the lengths span more than one sort bin (last_kernel names " dsort", the bank counts
    it); a fixed-length batch keeps the caller's order with no sort launch at all.  Scores equal
    the oracle's either way."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(lo + 7 * hi)
    q = _codes(rng, 128)
    n = 40000
    lens0 = rng.integers(lo, hi + 1, n)
    seqs = [_codes(rng, int(l)) for l in lens0]
    res, offs, lens = O.pack_residues(seqs)
    dev = torch.device("cuda", torch.cuda.current_device())
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    d_sc = torch.full((n,), -1, dtype=torch.int32, device=dev)
    mn, mx = int(lens.min()), max(int(lens.max()), 1)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, mx,
                                d_sc.data_ptr(), torch.cuda.current_stream().cuda_stream,
                                min_len=mn)
        torch.cuda.synchronize()
        kern, c = bank.last_kernel(), bank.counters()
        with pytest.raises(S.SwbankError) as e:  # an empty range
            bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n,
                                    mx, d_sc.data_ptr(), 0, min_len=mx + 1)
        assert e.value.status == S.ERR_ARG
    sorted_ = mx - mn >= 1  # max_len < 2048: one length per bin
    assert (" dsort" in kern) == sorted_ and c["device_sorts"] == int(sorted_), (kern, c)
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)
    assert (d_sc.cpu().numpy() == want).all()


# ---- device records with a corrupt length field --------------------------------------------
def test_device_records_clamp_corrupt_lengths():
    """A device record whose length field exceeds 232 is read as 232 bases (the kernels clamp
    it): no read past the data field or the buffer, same score as the 232-base
    record, with a query of several segments too (edge rows sized for 232 columns)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(3)
    seqs = [_codes(rng, 232) for _ in range(300)]
    rec = S.make_records(seqs)
    bad = rec.copy()
    bad[::3, 4:6] = np.frombuffer(np.uint16(60000).tobytes(), np.uint8)
    bad[1::3, 4:6] = np.frombuffer(np.uint16(233).tobytes(), np.uint8)
    dev = torch.device("cuda", torch.cuda.current_device())
    for qlen in (100, 1500):
        q = _codes(rng, qlen)
        with S.ScoreBank() as bank:
            bank.set_penalties(*REF)
            bank.load_query(q)
            good = bank.score_records(rec)
            d_rec = torch.from_numpy(bad.reshape(-1)).to(dev)
            d_sc = torch.full((len(seqs),), -1, dtype=torch.int32, device=dev)
            bank.score_records_device(d_rec.data_ptr(), len(seqs), d_sc.data_ptr(),
                                      torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            assert (d_sc.cpu().numpy() == good).all()


# ---- multi-device banks ---------------------------------------------------------------------
def _ragged_batch(seed, n=5000):
    rng = np.random.default_rng(seed)
    q = _codes(rng, 150)
    seqs = [_codes(rng, int(l)) for l in rng.integers(0, 1200, n)]
    seqs[n // 2] = q.copy()
    return q, seqs


@pytest.mark.parametrize("devices,gather", [([0, 0], "copy"), ([0, 0, 0], "copy"),
                                            ([0], "rccl"), ([0], "copy")])
def test_multi_device_bank_equals_single(devices, gather, monkeypatch):
    """A multi-device bank on the one GPU of the box: [0, 0] deals the batch over two child
    banks and gathers with device copies (RCCL refuses two ranks on one device); [0] with
    SWBANK_GATHER=rccl runs the real ncclCommInitAll + ncclGather path on a 1-rank comm.
    Scores must equal the single bank's bit for bit, in input order, with the best hit."""
    monkeypatch.setenv("SWBANK_GATHER", gather)
    q, seqs = _ragged_batch(len(devices) * 10 + len(gather))
    res, offs, lens = O.pack_residues(seqs)
    ids = np.arange(len(seqs), dtype=np.uint64) + 500
    with S.ScoreBank() as one:
        one.set_penalties(*REF)
        one.load_query(q)
        want = one.score_batch(res, offs, lens)
    with S.ScoreBank(devices=devices) as multi:
        assert multi.devices() == devices
        multi.set_penalties(*REF)
        multi.load_query(q)
        got = multi.score_batch(res, offs, lens, ids=ids)
        kern = multi.last_kernel()
        assert kern.startswith(f"multi[{len(devices)}] gather={gather}"), kern
        assert (got == want).all()
        b = int(np.argmax(want))
        assert multi.best() == (int(ids[b]), int(want[b]), b)
        # records through the same bank
        short = [s[:232] for s in seqs]
        r_multi = multi.score_records(S.make_records(short))
    res2, offs2, lens2 = O.pack_residues(short)
    assert (r_multi == O.score_batch(q, res2, offs2, lens2, O.dna_matrix(), -12, -4)).all()
    assert (want == O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)).all()


@pytest.mark.parametrize("nib", ["1", "0", "pipe"])
@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0], [0]])
def test_multi_device_bank_device_api(devices, nib, poisoned_buffers, monkeypatch):
    """ABI 4/5: a multi-device bank takes device buffers (on the root device): the batch is
    sorted longest first on the root and dealt round robin (length-balanced, as the host path),
    each device copies its share into its own HBM, scores it there and copies its scores back,
    asynchronous on the caller's stream (ScoreBank_v2.v:117-137: each module latches its own
    target copy).  Bit-exact against a single bank for a ragged batch with the best hit, a
    uniform batch on another stream right after (the staging reuse is ordered), a query set
    (every query broadcast to every device, ScoreBank_v2.v:101-102), and device records.
    nib="pipe": 4-bit shares cut into chunks of 700 targets, each scored while the next copies
    (the pipelined deal; without the knob only a share of more than one round of the tile
    kernel's slots on another device is cut)."""
    torch = pytest.importorskip("torch")
    # (round 6: DNA shares cross as 4-bit codes)
    monkeypatch.setenv("SWBANK_DEAL_NIB", "0" if nib == "0" else "1")
    if nib == "pipe":
        monkeypatch.setenv("SWBANK_DEAL_CHUNK", "700")
    dev = torch.device("cuda", 0)
    q, seqs = _ragged_batch(40 + len(devices), 6000)
    res, offs, lens = O.pack_residues(seqs)
    n = len(seqs)
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    d_ids = torch.from_numpy((np.arange(n, dtype=np.uint64) + 7).view(np.int64)).to(dev)
    qs = [q, q[:90].copy(), _codes(np.random.default_rng(9), 300)]
    short = [t[:232] for t in seqs]
    d_rec = torch.from_numpy(S.make_records(short).reshape(-1)).to(dev)
    L = int(lens.max())

    def run(bank):
        st = torch.cuda.Stream()
        one = torch.full((n,), -1, dtype=torch.int32, device=dev)
        bank.set_penalties(*REF)
        bank.load_query(q)
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, L,
                                one.data_ptr(), st.cuda_stream, d_ids=d_ids.data_ptr())
        best = bank.best()
        kern = bank.last_kernel()
        st2 = torch.cuda.Stream()  # a uniform batch (4000 targets cut to 60) right after
        uni = torch.full((4000,), -1, dtype=torch.int32, device=dev)
        bank.score_batch_device(d_res.data_ptr(), d_o60.data_ptr(), d_u60.data_ptr(), 4000, 60,
                                uni.data_ptr(), st2.cuda_stream, min_len=60)
        st2.synchronize()
        rec = torch.full((n,), -1, dtype=torch.int32, device=dev)
        bank.score_records_device(d_rec.data_ptr(), n, rec.data_ptr(), st.cuda_stream)
        bank.load_queries(qs)
        assert bank.query_count() == len(qs)
        sets = torch.full((len(qs), n), -1, dtype=torch.int32, device=dev)
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, L,
                                sets.data_ptr(), st.cuda_stream, min_len=int(lens.min()))
        st.synchronize()
        bank.sync()
        return (one.cpu().numpy(), best, rec.cpu().numpy(), sets.cpu().numpy(),
                uni.cpu().numpy(), kern)

    offs60 = np.ascontiguousarray(offs[np.nonzero(lens >= 60)[0][:4000]])
    lens60 = np.full(4000, 60, np.uint32)
    d_o60 = torch.from_numpy(offs60.view(np.int64)).to(dev)
    d_u60 = torch.from_numpy(lens60.view(np.int32)).to(dev)
    with S.ScoreBank() as single:
        want = run(single)
    with S.ScoreBank(devices=devices) as multi:
        got = run(multi)
        if len(devices) > 1:
            assert got[5].startswith(f"multi[{len(devices)}] device deal longest-first"), got[5]
            assert (" 4-bit" in got[5]) == (nib != "0"), got[5]
            assert (" pipelined x" in got[5]) == (nib == "pipe"), got[5]
    assert (got[0] == want[0]).all() and got[1] == want[1]
    assert (got[2] == want[2]).all() and (got[3] == want[3]).all()
    assert (got[4] == want[4]).all()
    assert (want[4] == O.score_batch(q, res, offs60, lens60, O.dna_matrix(), -12, -4)).all()
    assert (want[0] == O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)).all()
    res2, offs2, lens2 = O.pack_residues(short)
    assert (want[2] == O.score_batch(q, res2, offs2, lens2, O.dna_matrix(), -12, -4)).all()
    for i, qq in enumerate(qs):
        assert (want[3][i] == O.score_batch(qq, res, offs, lens, O.dna_matrix(), -12, -4)).all()


def test_multi_device_bank_bad_input_leaves_bank_usable(monkeypatch):
    """A code outside the alphabet on one device's share fails the call before any gather is
    issued (no rank is left waiting in the collective) and the bank stays usable."""
    monkeypatch.setenv("SWBANK_GATHER", "copy")
    q, seqs = _ragged_batch(3, 2000)
    bad = [s.copy() for s in seqs]
    bad[1500] = np.array([9, 9, 9], np.uint8)
    with S.ScoreBank(devices=[0, 0]) as multi:
        multi.set_penalties(*REF)
        multi.load_query(q)
        with pytest.raises(S.SwbankError) as e:
            multi.score_targets(bad)
        assert e.value.status == S.ERR_ARG
        got = multi.score_targets(seqs)
    res, offs, lens = O.pack_residues(seqs)
    assert (got == O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)).all()


def test_multi_device_rccl_gather_failure_leaves_bank_usable(monkeypatch):
    """A device that fails inside the RCCL gather phase (SWBANK_GATHER_FAULT=d: it reports a
    failure instead of joining ncclGather): the call returns SW_ERR_HIP, every communicator is
    aborted (ncclCommAbort) rather than left waiting for the missing rank, and the next call
    creates them again and returns exact scores.  (The box has one GPU, so this is the real
    ncclCommInitAll / ncclGather / ncclCommAbort on a 1-rank communicator; the timeout path for a
    peer that never arrives needs two devices.)"""
    monkeypatch.setenv("SWBANK_GATHER", "rccl")
    q, seqs = _ragged_batch(4, 3000)
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)
    with S.ScoreBank(devices=[0]) as multi:
        multi.set_penalties(*REF)
        multi.load_query(q)
        assert (multi.score_batch(res, offs, lens) == want).all()
        monkeypatch.setenv("SWBANK_GATHER_FAULT", "0")
        with pytest.raises(S.SwbankError) as e:
            multi.score_batch(res, offs, lens)
        assert e.value.status == S.ERR_HIP and "aborted" in str(e.value), str(e.value)
        monkeypatch.delenv("SWBANK_GATHER_FAULT")
        got = multi.score_batch(res, offs, lens)
        assert multi.last_kernel().startswith("multi[1] gather=rccl"), multi.last_kernel()
        assert multi.counters()["gather_timeouts"] == 0
    assert (got == want).all()


def test_cli_device_list(tmp_path, monkeypatch):
    """swbank -d 0,0: the CLI's multi-device bank reproduces the single-device transcript."""
    import subprocess
    monkeypatch.setenv("SWBANK_GATHER", "copy")
    q, lib = O.golden_fasta("query100.fa"), O.golden_fasta("data500.fa")
    one = subprocess.run([S.CLI_PATH, "-q", q, "-l", lib], capture_output=True, text=True)
    two = subprocess.run([S.CLI_PATH, "-q", q, "-l", lib, "-d", "0,0", "-b"], capture_output=True,
                         text=True)
    assert one.returncode == 0 and two.returncode == 0, two.stderr
    assert one.stdout == two.stdout and one.stdout.count("score:") == 499
    assert two.stderr.startswith("best: >")


def test_host_batch_target_outside_residues():
    """sw_score_batch checks every target against the residue count before reading it."""
    rng = np.random.default_rng(8)
    q = _codes(rng, 64)
    seqs = [_codes(rng, 100) for _ in range(5000)]
    res, offs, lens = O.pack_residues(seqs)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        with pytest.raises(S.SwbankError) as e:
            bank.score_batch(res[:-1], offs, lens)
        assert e.value.status == S.ERR_ARG and "outside" in str(e.value)
        bad = offs.copy()
        bad[4000] = np.uint64(2**63)  # huge offset: no overflow into a small address
        with pytest.raises(S.SwbankError):
            bank.score_batch(res, bad, lens)
        got = bank.score_batch(res, offs, lens)  # still usable
    assert (got == O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)).all()


@pytest.mark.parametrize("n", [1, 2, 5, 129])
def test_multi_device_deal_small_batches(n, poisoned_buffers):
    """The device-call deal with fewer targets than devices (some devices get none), a single
    target, empty targets, a batch of one length and a ragged one: exact against the oracle,
    the best hit with ids, device records dealt as contiguous ranges."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(n)
    q = _codes(rng, 60)
    seqs = [_codes(rng, int(rng.integers(0, 90))) for _ in range(n)]
    seqs[0] = q[:40].copy()
    if n > 2:
        seqs[1] = np.zeros(0, np.uint8)
    res, offs, lens = O.pack_residues(seqs)
    res = np.concatenate([res, np.zeros(16, np.uint8)])
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    d_ids = torch.from_numpy((np.arange(n, dtype=np.uint64) * 3 + 1).view(np.int64)).to(dev)
    d_rec = torch.from_numpy(S.make_records(seqs).reshape(-1)).to(dev)
    with S.ScoreBank(devices=[0, 0, 0]) as multi:
        multi.set_penalties(*REF)
        multi.load_query(q)
        sc = torch.full((n,), -5, dtype=torch.int32, device=dev)
        multi.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n,
                                 max(1, int(lens.max())), sc.data_ptr(), d_ids=d_ids.data_ptr())
        best = multi.best()
        rec = torch.full((n,), -5, dtype=torch.int32, device=dev)
        multi.score_records_device(d_rec.data_ptr(), n, rec.data_ptr())
        multi.sync()
        got, got_rec = sc.cpu().numpy(), rec.cpu().numpy()
    assert np.array_equal(got, want), (got.tolist(), want.tolist())
    assert np.array_equal(got_rec, want)
    k = int(np.argmax(want))
    assert best == (k * 3 + 1, int(want[k]), k)


#  SWBANK_DEAL_SOAK_SEEDS=n (default 3) / SWBANK_DEAL_SOAK_BASE=b: seeds b .. b+n-1
_DS_BASE = int(os.environ.get("SWBANK_DEAL_SOAK_BASE", "0"))
_DS_SEEDS = int(os.environ.get("SWBANK_DEAL_SOAK_SEEDS", "3"))


@pytest.mark.parametrize("seed", range(_DS_BASE, _DS_BASE + _DS_SEEDS))
def test_multi_device_deal_soak(seed, monkeypatch):
    """Seeded device calls on multi-device banks (2-4 devices, every one the box's GPU): random
    batch sizes, ragged lengths with empties, N codes, scattered offsets, half of them with the
    shares cut into random chunks (the pipelined deal); the deal (sort, gather to each device's
    staging, copies, scatter back) equals a one-device bank on every target."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(90_000 + seed)
    D = int(rng.integers(2, 5))
    n = int(rng.choice([int(rng.integers(1, 64)), int(rng.integers(64, 5000)),
                        int(rng.integers(5000, 60000))]))
    maxl = int(rng.choice([8, 31, 150, 600]))
    q = _codes(rng, int(rng.integers(20, 300)))
    lens = rng.integers(0, maxl + 1, n).astype(np.uint32)
    gap = rng.integers(0, 9, n).astype(np.uint64) if rng.random() < 0.5 else np.zeros(n, np.uint64)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.uint64) + gap[:-1])
    total = int(offs[-1] + lens[-1]) + 16
    res = rng.integers(0, 4, total, dtype=np.uint8)
    res[rng.random(total) < 0.005] = 4
    perm = rng.permutation(n) if rng.random() < 0.5 else np.arange(n)
    offs, lens = np.ascontiguousarray(offs[perm]), np.ascontiguousarray(lens[perm])
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    L = max(1, int(lens.max()))
    chunk = int(rng.integers(1, 3000)) if rng.random() < 0.5 else 0

    def run(devices):
        monkeypatch.setenv("SWBANK_DEAL_CHUNK", str(chunk if len(devices) > 1 else 0))
        with S.ScoreBank(devices=devices) as bank:
            bank.set_penalties(*REF)
            bank.load_query(q)
            sc = torch.full((n,), -5, dtype=torch.int32, device=dev)
            bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, L,
                                    sc.data_ptr())
            bank.sync()
            return sc.cpu().numpy()

    got = run([0] * D)
    want = run([0])
    assert np.array_equal(got, want), (D, n, maxl, chunk, int((got != want).sum()))


@pytest.mark.parametrize("devices,gather", [([0, 0], "copy"), ([0, 0, 0], "copy"),
                                            ([0], "rccl"), (None, None)])
def test_multi_device_resident_batches(devices, gather, monkeypatch, poisoned_buffers):
    """ABI 6, sw_score_batch_device_multi: each device's batch already sits in its own HBM (the
    RTL's modules each latch their own targets, ScoreBank_v2.v:117-137) and is scored in place;
    only the int32 scores are gathered to the root -- by ncclGather on a real 1-rank
    communicator for [0] with SWBANK_GATHER=rccl, by peer copies for a device listed twice.
    Ragged, uniform and empty per-device batches, a query set, the per-device score buffers and
    the gathered vector: bit-exact against the oracle on every target, twice in a row on
    different streams (the shared gather buffer's reuse is ordered)."""
    torch = pytest.importorskip("torch")
    if gather:
        monkeypatch.setenv("SWBANK_GATHER", gather)
    dev = torch.device("cuda", 0)
    D = len(devices) if devices else 1
    rng = np.random.default_rng(500 + D)
    q = _codes(rng, 130)
    shapes = [(3000, 0, 180), (2049, 90, 90), (0, 0, 1), (777, 1, 300)][:D]
    if D == 1:
        shapes = [(4500, 0, 200)]
    per, want, dev_bufs = [], [], []
    for n, lo, hi in shapes:
        seqs = [_codes(rng, int(l)) for l in rng.integers(lo, hi + 1, n)]
        if n > 10:  # a homolog, within the batch's length range (d_lens <= max_len)
            seqs[n // 3] = q[:len(seqs[n // 3])].copy()
        res, offs, lens = O.pack_residues(seqs) if n else (np.zeros(16, np.uint8),
                                                           np.zeros(0, np.uint64),
                                                           np.zeros(0, np.uint32))
        res = np.concatenate([res, np.zeros(16, np.uint8)])
        want.append((res, offs, lens))
        t = [torch.from_numpy(res).to(dev), torch.from_numpy(offs.view(np.int64)).to(dev),
             torch.from_numpy(lens.view(np.int32)).to(dev)]
        dev_bufs.append(t)
        per.append((n, lo, max(hi, 1)))
    qs = [q, q[:70].copy(), _codes(rng, 260)]
    N = sum(n for n, _, _ in per)

    def oracle_rows(qq):
        return np.concatenate([O.score_batch(qq, r, o, l, O.dna_matrix(), -12, -4) if len(l) else
                               np.zeros(0, np.int32) for r, o, l in want])

    kw = dict(devices=devices) if devices else {}
    with S.ScoreBank(**kw) as bank:
        bank.set_penalties(*REF)
        for rnd, queries in enumerate([[q], qs]):
            if len(queries) == 1:
                bank.load_query(queries[0])
            else:
                bank.load_queries(queries)
            nq = len(queries)
            own = [torch.full((nq, max(n, 1)), -3, dtype=torch.int32, device=dev) for n, _, _ in per]
            gathered = torch.full((nq, N), -3, dtype=torch.int32, device=dev)
            st = torch.cuda.Stream()
            batches = [dict(d_res=b[0].data_ptr(), d_offs=b[1].data_ptr(), d_lens=b[2].data_ptr(),
                            n=n, min_len=lo, max_len=hi, d_scores=o.data_ptr())
                       for b, (n, lo, hi), o in zip(dev_bufs, per, own)]
            bank.score_batch_device_multi(batches, gathered.data_ptr(), st.cuda_stream)
            st.synchronize()
            bank.sync()
            if devices:
                assert bank.last_kernel().startswith(f"multi[{D}] resident gather={gather}"), \
                    bank.last_kernel()
            g = gathered.cpu().numpy()
            for i, qq in enumerate(queries):
                ref = oracle_rows(qq)
                bad = np.nonzero(g[i] != ref)[0]
                assert len(bad) == 0, (rnd, i, len(bad), bad[:8].tolist(), g[i][bad[:8]].tolist(),
                                       ref[bad[:8]].tolist(), per)
                at = 0
                for (n, _, _), o in zip(per, own):
                    assert np.array_equal(o.cpu().numpy()[i][:n], ref[at:at + n])
                    at += n
        # gathered only (no per-device buffers), the bank's own streams
        bank.load_query(q)
        only = torch.full((N,), -3, dtype=torch.int32, device=dev)
        bank.score_batch_device_multi([dict(d_res=b[0].data_ptr(), d_offs=b[1].data_ptr(),
                                            d_lens=b[2].data_ptr(), n=n, min_len=lo, max_len=hi)
                                       for b, (n, lo, hi) in zip(dev_bufs, per)], only.data_ptr())
        bank.sync()
        torch.cuda.synchronize()
        assert np.array_equal(only.cpu().numpy(), oracle_rows(q))
        with pytest.raises(S.SwbankError) as e:  # one batch per device, exactly
            bank.score_batch_device_multi([], only.data_ptr())
        assert e.value.status == S.ERR_ARG


def test_multi_device_ragged_gather_knob(monkeypatch):
    """with SWBANK_RAGGED_GATHER=1/2 a child's launch copied the batch in its sorted
    order into the same buffers the multi-device deal had handed it as input (in place, so lanes
    overwrote targets others had not read).  The sorted copy now has its own buffers: a [0, 0]
    deal large enough for the children's ragged balanced ranges, bit-exact with the knob."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(77)
    q = _codes(rng, 128)
    n = 1_300_000  # each child's share must allow ragged balanced ranges (>= 4,864 tiles)
    lens = rng.integers(64, 151, n).astype(np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    res = rng.integers(0, 4, int(lens.sum()) + 16, dtype=np.uint8)
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)
    d = [torch.from_numpy(x).to(dev) for x in (res, offs.view(np.int64), lens.view(np.int32))]
    for mode in ("1", "2", "nib"):
        # "nib": the default deal (4-bit shares, round 6) -- the children's ragged balanced
        # ranges read 4-bit codes; the gather knob applies to byte shares only
        monkeypatch.setenv("SWBANK_DEAL_NIB", "1" if mode == "nib" else "0")
        monkeypatch.setenv("SWBANK_RAGGED_GATHER", "0" if mode == "nib" else mode)
        with S.ScoreBank(devices=[0, 0]) as bank:
            bank.set_penalties(*REF)
            bank.load_query(q)
            sc = torch.full((n,), -3, dtype=torch.int32, device=dev)
            bank.score_batch_device(d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(), n, 150,
                                    sc.data_ptr(), min_len=64)
            bank.sync()
            kern = bank.last_kernel()
            got = sc.cpu().numpy()
        assert "balanced" in kern and ("gather" in kern) == (mode != "nib"), kern
        assert ("4-bit" in kern) == (mode == "nib"), kern
        assert np.array_equal(got, want), (mode, int((got != want).sum()))
