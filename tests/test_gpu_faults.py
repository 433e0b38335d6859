"""GPU: device-side hand-off waits that run out fail loudly (ABI 5, include/swbank.h).

Two launch shapes hand work between workgroups of one launch: balanced chunk ranges (a tile's
column state from workgroup g - 1 to g) and the segmented protein tail (a pair's
bottom rows from segment s to s + 1).  Each wait is bounded; one that runs out marks
the launch's fault word instead of hanging, and the host turns the mark into an error -- the
reference host's convention of failing a call on the AFU's error bits
(capi_sample_aligner/software-C,C++/src/main_test.c:64-100):
  * a device call (asynchronous) latches SW_ERR_TIMEOUT until the next synchronising call
    (sw_bank_sync, sw_batch_best, sw_bank_timing) or the next device scoring call returns it;
  * a host-buffer call re-runs itself without hand-offs and returns exact scores.
The test hooks: SWBANK_STALL=g makes the producer the g-th waiter depends on skip its hand-off,
SWBANK_POLL_LIMIT bounds the waits to a few hundred microseconds."""
import numpy as np
import pytest

import swbank as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu

REF = (5, -4, -12, -4)


def _uniform_batch(torch, n=340_000, L=128, qlen=128):
    dev = torch.device("cuda", 0)
    q = O.random_codes(11, qlen, 4)
    res = O.random_codes(12, n * L, 4)
    for k in range(0, n, 97):  # homologous targets: a lost column state shows
        res[k * L:k * L + min(L, qlen)] = q[:min(L, qlen)]
    offs = np.arange(n, dtype=np.uint64) * L
    lens = np.full(n, L, np.uint32)
    d = (torch.from_numpy(res).to(dev), torch.from_numpy(offs.view(np.int64)).to(dev),
         torch.from_numpy(lens.view(np.int32)).to(dev))
    return q, res, offs, lens, d


def test_balanced_stall_device_call(monkeypatch):
    """A balanced-range tail visit whose predecessor never publishes: the call itself returns
    (asynchronous), sw_bank_sync returns SW_ERR_TIMEOUT once, the counter shows it, and the next
    call on the same bank is exact again."""
    torch = pytest.importorskip("torch")
    q, res, offs, lens, (d_res, d_offs, d_lens) = _uniform_batch(torch)
    n, L = len(lens), int(lens[0])
    sc = torch.full((n,), -7, dtype=torch.int32, device=d_res.device)
    with S.ScoreBank() as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        monkeypatch.setenv("SWBANK_STALL", "5")
        monkeypatch.setenv("SWBANK_POLL_LIMIT", "2000")
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, L,
                                sc.data_ptr(), min_len=L)
        assert "balanced" in bank.last_kernel()
        with pytest.raises(S.SwbankError) as ei:
            bank.sync()
        assert ei.value.status == S.ERR_TIMEOUT
        bank.sync()  # reported once
        assert bank.counters()["balanced_timeouts"] == 1

        # the next device scoring call returns a fault latched before it (no sync in between)
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, L,
                                sc.data_ptr(), min_len=L)
        torch.cuda.synchronize()
        with pytest.raises(S.SwbankError) as ei:
            bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, L,
                                    sc.data_ptr(), min_len=L)
        assert ei.value.status == S.ERR_TIMEOUT

        # the batch best hit: sw_batch_best reports the fault instead of a best of wrong scores
        ids = torch.arange(n, dtype=torch.int64, device=d_res.device)
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, L,
                                sc.data_ptr(), d_ids=ids.data_ptr(), min_len=L)
        with pytest.raises(S.SwbankError) as ei:
            bank.best()
        assert ei.value.status == S.ERR_TIMEOUT
        assert bank.counters()["balanced_timeouts"] == 3

        monkeypatch.delenv("SWBANK_STALL")
        monkeypatch.delenv("SWBANK_POLL_LIMIT")
        sc.fill_(-7)
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, L,
                                sc.data_ptr(), d_ids=ids.data_ptr(), min_len=L)
        bank.sync()
        got = sc.cpu().numpy()
        best = bank.best()
        assert bank.counters()["balanced_timeouts"] == 3
    rows = np.unique(np.concatenate([np.arange(0, n, 97), np.arange(1000)]))
    want = O.score_batch(q, res, np.ascontiguousarray(offs[rows]),
                         np.ascontiguousarray(lens[rows]), O.dna_matrix(*REF[:2]), *REF[2:])
    assert np.array_equal(got[rows], want)
    assert best[1] == int(got.max()) and best[2] == int(np.argmax(got))


def _protein_batch(rng, n, qlen):
    q = rng.integers(0, 20, qlen, dtype=np.uint8)
    seqs = [rng.integers(0, 20, int(rng.integers(200, 400)), dtype=np.uint8) for _ in range(n)]
    for k in range(n - 30, n, 3):  # homologous tail targets
        t = np.resize(q, 380).copy()
        t[::11] = rng.integers(0, 20, len(t[::11]))
        seqs[k] = t
    return q, seqs


@pytest.mark.parametrize("model", [S.GAP_MERGED, S.GAP_GOTOH])
def test_tail_stall_host_call_reruns(monkeypatch, model):
    """A segmented protein tail whose first segment never publishes, in a host-buffer call: the
    call re-runs without hand-offs (counted) and returns exact scores."""
    rng = np.random.default_rng(model + 3)
    n, qlen = 600, 400
    q, seqs = _protein_batch(rng, n, qlen)
    monkeypatch.setenv("SWBANK_KERNEL", "wave")
    monkeypatch.setenv("SWBANK_WAVE_SPLIT", "20")
    monkeypatch.setenv("SWBANK_WAVE_SPLIT_P", "8")
    want = O.score_batch(q, *O.pack_residues(seqs), O.BLOSUM62, -11, -1,
                         O.GAP_GOTOH if model == S.GAP_GOTOH else O.GAP_MERGED)
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN, gap_model=model) as bank:
        bank.set_matrix(O.BLOSUM62, -11, -1)
        bank.load_query(q)
        got0 = bank.score_targets(seqs)
        assert "tail=20/8" in bank.last_kernel(), bank.last_kernel()
        assert bank.counters()["handoff_reruns"] == 0
        monkeypatch.setenv("SWBANK_STALL", "3")
        monkeypatch.setenv("SWBANK_POLL_LIMIT", "500")
        got = bank.score_targets(seqs)
        ctr = bank.counters()
        kern = bank.last_kernel()
    assert np.array_equal(got0, want)
    assert ctr["handoff_reruns"] == 1 and ctr["tail_timeouts"] == 1, ctr
    assert "tail=" not in kern, kern  # the re-run ran without the segmented tail
    assert np.array_equal(got, want)


def test_tail_stall_device_call(monkeypatch):
    """The same stall in a device call: SW_ERR_TIMEOUT at sw_bank_sync; the next call is exact."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(9)
    n, qlen = 600, 512
    q, seqs = _protein_batch(rng, n, qlen)
    res, offs, lens = O.pack_residues(seqs)
    dev = torch.device("cuda", 0)
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    d_sc = torch.full((n,), -9, dtype=torch.int32, device=dev)
    monkeypatch.setenv("SWBANK_KERNEL", "wave")
    monkeypatch.setenv("SWBANK_WAVE_SPLIT", "20")
    monkeypatch.setenv("SWBANK_WAVE_SPLIT_P", "8")
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN) as bank:
        bank.set_matrix(O.BLOSUM62, -11, -1)
        bank.load_query(q)
        monkeypatch.setenv("SWBANK_STALL", "20")
        monkeypatch.setenv("SWBANK_POLL_LIMIT", "500")
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n,
                                int(lens.max()), d_sc.data_ptr())
        assert "tail=20/8" in bank.last_kernel()
        with pytest.raises(S.SwbankError) as ei:
            bank.sync()
        assert ei.value.status == S.ERR_TIMEOUT
        assert bank.counters()["tail_timeouts"] == 1
        monkeypatch.delenv("SWBANK_STALL")
        monkeypatch.delenv("SWBANK_POLL_LIMIT")
        d_sc.fill_(-9)
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n,
                                int(lens.max()), d_sc.data_ptr())
        bank.sync()
    want = O.score_batch(q, res, offs, lens, O.BLOSUM62, -11, -1)
    assert np.array_equal(d_sc.cpu().numpy(), want)


def test_multi_device_bank_sync_reports_child_fault(monkeypatch):
    """A multi-device bank (both children on device 0) reports a child's fault at sw_bank_sync."""
    torch = pytest.importorskip("torch")
    q, res, offs, lens, (d_res, d_offs, d_lens) = _uniform_batch(torch, n=700_000)
    n, L = len(lens), int(lens[0])
    sc = torch.full((n,), -7, dtype=torch.int32, device=d_res.device)
    with S.ScoreBank(devices=[0, 0]) as bank:
        bank.set_penalties(*REF)
        bank.load_query(q)
        monkeypatch.setenv("SWBANK_STALL", "5")
        monkeypatch.setenv("SWBANK_POLL_LIMIT", "2000")
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), n, L,
                                sc.data_ptr(), min_len=L)
        with pytest.raises(S.SwbankError) as ei:
            bank.sync()
        assert ei.value.status == S.ERR_TIMEOUT
        assert bank.counters()["balanced_timeouts"] >= 1
        bank.sync()
