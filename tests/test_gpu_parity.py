"""GPU parity: the HIP path (through the C ABI) against the golden vectors and the oracle.

Bar: bit-exact int32 scores.  Every test here runs the product path (libswbank.so on a
gfx950 device); the oracle is only the checker.
"""
import os
import subprocess

import numpy as np
import pytest

import swbank as S
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["tile", "tile-lut", "tile-u16", "wave", "wave-u16"])
def kernel_choice(request, monkeypatch):
    """Run every parity test through each score kernel: the tile kernel (waves = row blocks,
    lanes = targets) and the wave kernel (lanes = rows, DPP hand-off), each with its f16
    arithmetic where eligible ("tile", "wave": exact below the f16 bound, optimistic with a
    u16 re-score above it) and forced to u16 ("-u16").  "tile" takes the letter-pair table
    for DNA queries of <= 128 rows; "tile-lut" forces the per-row LUT lookup instead.  Past
    1024 rows the wave kernel runs the query as 1024-row segments."""
    kern = request.param.split("-")[0]
    monkeypatch.setenv("SWBANK_KERNEL", kern)
    monkeypatch.setenv("SWBANK_F16", "0" if request.param.endswith("-u16") else "1")
    monkeypatch.setenv("SWBANK_PAIR", "0" if request.param.endswith("-lut") else "1")
    return request.param


REF = (5, -4, -12, -4)


@pytest.fixture(scope="module")
def bank():
    b = S.ScoreBank()
    yield b
    b.close()


def _lib_records(name):
    return O.read_fasta(O.golden_fasta(name))


def test_every_golden_score(bank):
    """730 HDL transcript + 598 ssearch36 + 1 CAPI scores, keyed by target name."""
    rows = O.load_ref_scores()
    bank.set_penalties(*REF)
    checked = 0
    for q in sorted({r[2] for r in rows}):
        bank.load_query(O.encode_dna(_lib_records(q)[0][1]))
        for lib in sorted({r[1] for r in rows if r[2] == q}):
            recs = _lib_records(lib)
            got = dict(zip([n for n, _ in recs],
                           bank.score_targets([O.encode_dna(s) for _, s in recs])))
            for src, l, qq, t, s in rows:
                if l == lib and qq == q:
                    assert got[t] == s, (src, lib, q, t, s, got[t])
                    checked += 1
    assert checked == len(rows) == 1329


def test_swalign_control_differs(bank):
    bank.set_penalties(*REF)
    bank.load_query(O.encode_dna(_lib_records("query1.fa")[0][1]))
    recs = dict(_lib_records("data1.fa"))
    ctrl = O.load_swalign_control()
    names = sorted(ctrl)
    got = bank.score_targets([O.encode_dna(recs[n]) for n in names])
    diff = sorted(n for n, g in zip(names, got) if g != ctrl[n])
    assert diff == ["db10", "db12", "db13", "db8"]


def _random_case(rng, qlen, ntargets, maxlen, alpha=5, p_n=0.02):
    q = rng.integers(0, 4, qlen, dtype=np.uint8)
    q[rng.random(qlen) < p_n] = 4
    seqs = []
    for _ in range(ntargets):
        t = rng.integers(0, 4, int(rng.integers(0, maxlen + 1)), dtype=np.uint8)
        t[rng.random(len(t)) < p_n] = 4
        seqs.append(t)
    return q, seqs


@pytest.mark.parametrize("params", [REF, (5, -4, -10, -1), (2, -3, -5, -2), (1, -1, -1, -1),
                                    (20, -4, -2, -1), (3, 0, -6, -1)])
@pytest.mark.parametrize("qlen", [1, 7, 16, 17, 31, 32, 33, 63, 64, 65, 100, 128, 150, 255, 256,
                                  300, 512])
def test_random_vs_oracle(bank, params, qlen):
    rng = np.random.default_rng(qlen * 1009 + params[0] * 31 + params[3])
    q, seqs = _random_case(rng, qlen, 300, 260)
    # homologous targets exercise long gapped alignments
    for k in range(0, 300, 10):
        m = q.copy()
        if len(m):
            cut = rng.integers(0, len(m) + 1)
            m = np.concatenate([m[:cut], rng.integers(0, 4, rng.integers(0, 8), dtype=np.uint8),
                                m[cut + rng.integers(0, 4):]])
        seqs[k] = m[:300]
    bank.set_penalties(*params)
    bank.load_query(q)
    got = bank.score_targets(seqs)
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(params[0], params[1]), params[2],
                         params[3])
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), int(lens[i]), int(got[i]), int(want[i])) for i in bad[:8]]


def test_edge_shapes(bank):
    bank.set_penalties(*REF)
    bank.load_query(O.encode_dna("ACGT"))
    # empty batch, empty targets, single-base targets, all-N target
    assert bank.score_targets([]).size == 0
    got = bank.score_targets([np.zeros(0, np.uint8), O.encode_dna("A"), O.encode_dna("NNNN"),
                              O.encode_dna("ACGT")])
    assert got.tolist() == [0, 5, 0, 20]
    # empty query scores 0 everywhere
    bank.load_query(np.zeros(0, np.uint8))
    assert bank.score_targets([O.encode_dna("ACGT")]).tolist() == [0]
    # ragged tile tails: n not a multiple of the 128-target tile
    rng = np.random.default_rng(2)
    q, seqs = _random_case(rng, 128, 129, 140)
    bank.load_query(q)
    got = bank.score_targets(seqs)
    res, offs, lens = O.pack_residues(seqs)
    assert (got == O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)).all()


@pytest.mark.parametrize("qlen", [200, 407, 408, 409, 410, 512])
@pytest.mark.parametrize("match", [5, 8, 9, 16])
def test_f16_bound_edges(bank, qlen, match, kernel_choice):
    """Scores at and past the f16 kernel's exact range (exact f16 while min(|q|, max|t|) *
    max(s) + max(s) <= 2048, optimistic f16 + u16 re-score past it); match 9 has a non-zero
    f16 low byte, so it runs on the 2-byte profile; perfect and near-perfect matches put the
    optimum right at the bound."""
    rng = np.random.default_rng(qlen * 7 + match)
    q = rng.integers(0, 4, qlen, dtype=np.uint8)
    near = q.copy()
    near[qlen // 2] = (near[qlen // 2] + 1) % 4
    gapped = np.concatenate([q[:qlen // 3], q[qlen // 3 + 2:]])
    seqs = [q, near, gapped, q[: qlen // 2], rng.integers(0, 4, qlen, dtype=np.uint8)]
    seqs += [q] * 130  # a second tile
    params = (match, -4, -12, -4)
    bank.set_penalties(*params)
    bank.load_query(q)
    got = bank.score_targets(seqs)
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(match, -4), -12, -4)
    assert got[0] == match * qlen
    if kernel_choice in ("tile", "tile-lut"):
        # exact f16 within the bound; past it optimistic f16 with a u16 re-score of the pairs
        # above 2048 - max(s); a score with a non-zero f16 low byte (9) cannot use the
        # one-byte LUT and runs on the 2-byte f16 profile instead
        want_k = ("tile f16" + ("" if qlen * match + match <= 2048 else "+u16-rescore") +
                  ("-profile " if match == 9 else " "))
        assert bank.last_kernel().startswith(want_k), bank.last_kernel()
    elif kernel_choice == "tile-u16":
        assert bank.last_kernel().startswith("tile u16")
    assert (got == want).all(), [(i, int(got[i]), int(want[i])) for i in np.nonzero(got != want)[0][:8]]


def test_errors(bank):
    bank.set_penalties(*REF)
    with pytest.raises(S.SwbankError) as e:
        bank.load_query(np.zeros(S.lib().sw_max_query_len() + 1, np.uint8))
    assert e.value.status == S.ERR_UNSUPPORTED
    with pytest.raises(S.SwbankError) as e:
        bank.load_query(np.array([0, 1, 9], np.uint8))
    assert e.value.status == S.ERR_ARG
    with pytest.raises(S.SwbankError) as e:
        bank.set_penalties(5, -4, 3, -1)
    assert e.value.status == S.ERR_ARG
    fresh = S.ScoreBank()
    with pytest.raises(S.SwbankError) as e:
        fresh.score_targets([O.encode_dna("ACGT")])
    assert e.value.status == S.ERR_STATE
    # a substitution range past the 8-bit LUT is refused, not wrapped
    fresh.set_penalties(127, -128, -12, -4)
    fresh.load_query(np.zeros(16, np.uint8))
    with pytest.raises(S.SwbankError) as e:
        fresh.score_targets([np.zeros(20, np.uint8)])
    assert e.value.status == S.ERR_RANGE
    # the largest DNA scores fit the u16 lanes: 127 * 512 + S
    fresh.set_penalties(127, -4, -12, -4)
    fresh.load_query(np.zeros(512, np.uint8))
    assert fresh.score_targets([np.zeros(600, np.uint8)]).tolist() == [127 * 512]
    fresh.close()


def test_device_api_with_torch_buffers(bank):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(9)
    q, seqs = _random_case(rng, 128, 1000, 128, p_n=0.0)
    res, offs, lens = O.pack_residues(seqs)
    dev = torch.device("cuda", torch.cuda.current_device())
    d_res = torch.from_numpy(res).to(dev)
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    d_sc = torch.full((len(seqs),), -1, dtype=torch.int32, device=dev)
    bank.set_penalties(*REF)
    bank.load_query(q)
    stream = torch.cuda.current_stream()
    bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), len(seqs),
                            int(lens.max()), d_sc.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)
    assert (d_sc.cpu().numpy() == want).all()


def test_bench_scale_properties(bank):
    """query100 x 499*64 synthetic 128-bp targets (the bench's shape at reduced replication):
    a seeded subset is checked against the oracle, and size-independent properties hold for
    the whole batch: duplicated targets score identically, scores are permutation-equivariant,
    and every score is bounded by 5 * min(|q|, |t|)."""
    q = O.encode_dna(_lib_records("query100.fa")[0][1])
    n, L = 499 * 64, 128
    codes = O.random_codes(2024, n * L, 4).reshape(n, L)
    codes[1::7] = codes[0::7][: len(codes[1::7])]
    seqs = list(codes)
    bank.set_penalties(*REF)
    bank.load_query(q)
    got = bank.score_targets(seqs)
    assert (got[1::7] == got[0::7][: len(got[1::7])]).all()
    perm = np.random.default_rng(4).permutation(n)
    got_p = bank.score_targets([seqs[i] for i in perm])
    assert (got_p == got[perm]).all()
    assert got.min() >= 0 and got.max() <= 5 * L
    idx = np.random.default_rng(5).choice(n, 2000, replace=False)
    res, offs, lens = O.pack_residues([seqs[i] for i in idx])
    assert (got[idx] == O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)).all()


def test_cli_reproduces_transcript():
    out = subprocess.run([S.CLI_PATH, "-q", O.golden_fasta("query100.fa"), "-l",
                          O.golden_fasta("data100.fa")], capture_output=True, text=True,
                         check=True).stdout
    got = {}
    for line in out.splitlines():
        name, _, score = line.partition(" score: ")
        got[name.lstrip(">")] = int(score)
    want = {t: s for src, lib, q, t, s in O.load_ref_scores() if lib == "data100.fa"}
    assert all(got[t] == s for t, s in want.items()) and len(want) == 99


def test_cli_ssearch_R_writer_matches_score500(tmp_path):
    """Row f3: `swbank -R` writes data/score500.txt's per-target lines byte for byte (name,
    length, score, record index, byte offset in the library file)."""
    rfile = tmp_path / "score500.txt"
    subprocess.run([S.CLI_PATH, "-q", O.golden_fasta("query100.fa"), "-l",
                    O.golden_fasta("data500.fa"), "-R", str(rfile), "-o", os.devnull], check=True)
    got = [ln for ln in rfile.read_text().splitlines() if ln.startswith("db")]
    want = open(os.path.join(O.GOLDEN, "score500_R_lines.txt")).read().splitlines()
    assert len(got) == len(want) == 499
    bad = [(g, w) for g, w in zip(got, want) if g != w]
    assert not bad, bad[:3]


def test_cli_fasta_robustness(tmp_path):
    """Row f4: CRLF line ends, wrapped sequence lines, lower case, blank lines and header
    descriptions parse to the same records as the reference's one-line FASTA."""
    recs = _lib_records("data10.fa")
    messy = tmp_path / "data10_messy.fa"
    with open(messy, "w", newline="") as f:
        for k, (name, seq) in enumerate(recs):
            f.write(f">{name} some description\r\n\r\n")
            body = seq.lower() if k % 2 else seq
            for i in range(0, len(body), 60):
                f.write(body[i:i + 60] + "\r\n")
    def run(lib):
        out = subprocess.run([S.CLI_PATH, "-q", O.golden_fasta("query100.fa"), "-l", str(lib)],
                             capture_output=True, text=True, check=True).stdout
        return out.splitlines()
    assert run(messy) == run(O.golden_fasta("data10.fa"))
    assert len(run(messy)) == len(recs)


# ---- Gotoh / protein / profile-mode kernels ---------------------------------------------
def _load_generated():
    import json
    return json.load(open(os.path.join(O.GOLDEN, "generated.json")))["cases"]


@pytest.mark.parametrize("case", _load_generated(), ids=lambda c: c["name"])
def test_generated_golden(case):
    """configs[3]/[4] shapes and merged!=Gotoh parameters (fixtures from the pinned oracle)."""
    prot = case["alphabet"] == "protein"
    alphabet = S.ALPHABET_PROTEIN if prot else S.ALPHABET_DNA
    model = S.GAP_GOTOH if case["gap_model"] == "gotoh" else S.GAP_MERGED
    with S.ScoreBank(alphabet=alphabet, gap_model=model) as bank:
        if prot:
            bank.set_matrix(O.BLOSUM62, case["gap_open"], case["gap_extend"])
        else:
            bank.set_penalties(*case["match_mismatch"], case["gap_open"], case["gap_extend"])
        bank.load_query(S.encode(case["query"], alphabet))
        got = bank.score_targets([S.encode(t, alphabet) for t in case["targets"]])
    assert got.tolist() == case["scores"]


@pytest.mark.parametrize("params", [(5, -4, -12, -4), (5, -4, -10, -1), (2, -3, -5, -2),
                                    (1, -1, -1, -1)])
@pytest.mark.parametrize("qlen", [1, 17, 32, 64, 100, 150, 256, 512])
def test_gotoh_dna_random_vs_oracle(params, qlen):
    rng = np.random.default_rng(qlen * 7 + params[3])
    q, seqs = _random_case(rng, qlen, 260, 300)
    with S.ScoreBank(gap_model=S.GAP_GOTOH) as bank:
        bank.set_penalties(*params)
        bank.load_query(q)
        got = bank.score_targets(seqs)
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(params[0], params[1]), params[2],
                         params[3], O.GAP_GOTOH)
    assert (got == want).all()


@pytest.mark.parametrize("case", ["dna-gotoh", "prot-merged", "prot-gotoh"])
def test_f16_gotoh_and_profile_paths(case, kernel_choice):
    """The f16 Gotoh column and the 2-byte f16 query profile are taken when the score bound
    allows (and not under SWBANK_F16=0), and agree with the oracle around the bound."""
    rng = np.random.default_rng(len(case))
    dna = case.startswith("dna")
    model = S.GAP_GOTOH if case.endswith("gotoh") else S.GAP_MERGED
    A = 4 if dna else 20
    for qlen in (40, 150):
        q = rng.integers(0, A, qlen, dtype=np.uint8)
        seqs = [rng.integers(0, A, int(rng.integers(0, 220)), dtype=np.uint8) for _ in range(300)]
        for k in range(0, 300, 5):
            seqs[k] = q.copy()
            seqs[k][::9] = rng.integers(0, A, len(seqs[k][::9]))
        seqs[1] = q.copy()  # the bound itself: a perfect match
        with S.ScoreBank(alphabet=S.ALPHABET_DNA if dna else S.ALPHABET_PROTEIN,
                         gap_model=model) as bank:
            if dna:
                bank.set_penalties(5, -4, -10, -1)
                sub, go, ge = O.dna_matrix(5, -4), -10, -1
            else:
                bank.set_matrix(O.BLOSUM62, -11, -1)
                sub, go, ge = O.BLOSUM62, -11, -1
            bank.load_query(q)
            got = bank.score_targets(seqs)
            kern = bank.last_kernel()
        res, offs, lens = O.pack_residues(seqs)
        want = O.score_batch(q, res, offs, lens, sub, go, ge, model)
        assert (got == want).all(), (kern, np.nonzero(got != want)[0][:5])
        smax = 5 if dna else 11
        if kernel_choice in ("tile", "tile-lut"):
            f16 = min(qlen, max(lens)) * smax + smax <= 2048
            assert kern.startswith("tile f16" + ("" if f16 else "+u16-rescore")), kern
        elif kernel_choice == "tile-u16":
            assert kern.startswith("tile u16"), kern


@pytest.mark.parametrize("model", [S.GAP_MERGED, S.GAP_GOTOH])
@pytest.mark.parametrize("gaps", [(-11, -1), (-10, -2), (-2, -1)])
@pytest.mark.parametrize("qlen", [5, 33, 200, 512])
def test_protein_random_vs_oracle(model, gaps, qlen):
    rng = np.random.default_rng(qlen + 100 * model - gaps[0])
    q = rng.integers(0, 24, qlen, dtype=np.uint8)
    seqs = [rng.integers(0, 24, int(rng.integers(0, 400)), dtype=np.uint8) for _ in range(200)]
    for k in range(0, 200, 8):  # homologous targets
        seqs[k] = q[rng.integers(0, max(1, qlen // 2)):][:300].copy()
        seqs[k][::7] = rng.integers(0, 20, len(seqs[k][::7]))
    with S.ScoreBank(alphabet=S.ALPHABET_PROTEIN, gap_model=model) as bank:
        bank.set_matrix(O.BLOSUM62, *gaps)
        bank.load_query(q)
        got = bank.score_targets(seqs)
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.BLOSUM62, gaps[0], gaps[1], model)
    assert (got == want).all()


@pytest.mark.parametrize("model", [S.GAP_MERGED, S.GAP_GOTOH])
def test_dna_profile_mode_equals_lut_mode(model, monkeypatch):
    """The query-profile (LDS) lookup and the SGPR-LUT lookup are interchangeable."""
    rng = np.random.default_rng(31)
    q, seqs = _random_case(rng, 128, 300, 200)
    outs = []
    for prof in ("0", "1"):
        monkeypatch.setenv("SWBANK_PROFILE", prof)
        with S.ScoreBank(gap_model=model) as bank:
            bank.set_penalties(5, -4, -10, -1)
            bank.load_query(q)
            outs.append(bank.score_targets(seqs))
    assert (outs[0] == outs[1]).all()
    res, offs, lens = O.pack_residues(seqs)
    assert (outs[0] == O.score_batch(q, res, offs, lens, O.dna_matrix(), -10, -1, model)).all()


def test_custom_dna_matrix_routes_to_profile_kernel():
    """A DNA matrix with a non-uniform N column cannot use the 4-entry LUT; it must still be
    exact (profile kernel)."""
    m = O.dna_matrix(5, -4).copy()
    m[4, :] = -1
    m[:, 4] = -1
    m[4, 4] = 2
    m[0, 1] = m[1, 0] = -2  # transition/transversion-like asymmetry in the 4x4 block
    rng = np.random.default_rng(8)
    q, seqs = _random_case(rng, 77, 200, 150, p_n=0.1)
    with S.ScoreBank() as bank:
        bank.set_matrix(m, -12, -4)
        bank.load_query(q)
        got = bank.score_targets(seqs)
    res, offs, lens = O.pack_residues(seqs)
    assert (got == O.score_batch(q, res, offs, lens, m, -12, -4)).all()


def test_capi_records_path(bank, kernel_choice):
    """Row f2: CAPI sequence_t records (2-bit codes read by the kernel) score exactly like the
    byte path and the oracle; query from a record; lengths 0..232; device API."""
    import torch

    rng = np.random.default_rng(17)
    bank.set_penalties(*REF)
    q = rng.integers(0, 4, 100, dtype=np.uint8)
    lens = [0, 1, 7, 8, 9, 100, 231, 232] + list(rng.integers(0, 233, 300))
    seqs = [rng.integers(0, 4, int(n), dtype=np.uint8) for n in lens]
    for k in range(10, 300, 9):  # homologous targets
        seqs[k] = q[: min(len(q), 232)].copy()
    recs = S.make_records(seqs)
    bank.load_query_record(S.make_records([q])[0])
    got = bank.score_records(recs)
    res, offs, ln = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, ln, O.dna_matrix(5, -4), -12, -4)
    assert (got == want).all(), np.nonzero(got != want)[0][:8]
    assert (bank.score_targets(seqs) == want).all()
    # device-resident records, unsorted
    dev = torch.device("cuda", 0)
    d_rec = torch.from_numpy(recs.reshape(-1)).to(dev)
    d_sc = torch.zeros(len(seqs), dtype=torch.int32, device=dev)
    bank.score_records_device(d_rec.data_ptr(), len(seqs), d_sc.data_ptr(),
                              torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert (d_sc.cpu().numpy() == want).all()
    # main_test_output.txt: query1 vs db18 -> result 102 (CAPI host fixture)
    q1 = O.encode_dna(_lib_records("query1.fa")[0][1])
    db = dict(_lib_records("data1.fa"))
    bank.load_query_record(S.make_records([q1])[0])
    assert bank.score_records(S.make_records([O.encode_dna(db["db18"])])).tolist() == [102]
    # too long a record is refused
    bad = S.make_records([np.zeros(10, np.uint8)])
    bad[0, 4:6] = np.frombuffer(np.uint16(233).tobytes(), np.uint8)
    with pytest.raises(S.SwbankError):
        bank.score_records(bad)


def test_best_hit_device(bank):
    """Row f1 on the device: highest score, lowest index among ties, optional 64-bit IDs."""
    import torch

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    for n in (1, 7, 256, 1000, 300001):
        sc = rng.integers(-5, 2000, n).astype(np.int32)
        if n > 10:
            sc[n // 3] = sc[2 * n // 3] = sc.max() + 1  # a tie: the lower index wins
        ids = rng.integers(0, 2**63, n, dtype=np.uint64)
        d_sc = torch.from_numpy(sc).to(dev)
        d_ids = torch.from_numpy(ids.view(np.int64)).to(dev)
        d_out = torch.zeros(2, dtype=torch.int64, device=dev)
        stream = torch.cuda.current_stream().cuda_stream
        bank.best_hit_device(d_sc.data_ptr(), n, d_out.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        bi = int(np.argmax(sc))
        assert d_out.cpu().numpy().tolist() == [bi, int(sc[bi])]
        assert bank.best_hit(sc) == (bi, int(sc[bi]))
        bank.best_hit_device(d_sc.data_ptr(), n, d_out.data_ptr(), d_ids=d_ids.data_ptr(),
                             stream=stream)
        torch.cuda.synchronize()
        out = d_out.cpu().numpy().view(np.uint64)
        assert int(out[0]) == int(ids[bi]) and int(out[1]) == int(sc[bi])


def test_back_to_back_queries_on_a_user_stream():
    """ld_sequence between asynchronous device batches on the caller's own stream: the new
    query's tables are uploaded only after the previous launch has read the old ones, and the
    next launch waits for the upload (no host synchronisation in between)."""
    import torch

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(21)
    n, L = 20000, 200
    tg = rng.integers(0, 4, (n, L), dtype=np.uint8)
    queries = [rng.integers(0, 4, int(rng.integers(100, 700)), dtype=np.uint8) for _ in range(6)]
    for k in range(0, n, 97):  # homologs of the queries
        qq = queries[k % 6]
        a = int(rng.integers(0, max(1, len(qq) - L)))
        tg[k, :len(qq[a:a + L])] = qq[a:a + L]
    d_res = torch.from_numpy(tg.reshape(-1)).to(dev)
    d_offs = torch.arange(n, dtype=torch.int64, device=dev) * L
    d_lens = torch.full((n,), L, dtype=torch.int32, device=dev)
    d_sc = torch.zeros((len(queries), n), dtype=torch.int32, device=dev)
    user = torch.cuda.Stream()
    with S.ScoreBank() as bank:
        bank.set_penalties(5, -4, -12, -4)
        for rep in range(2):
            for k, qq in enumerate(queries):
                bank.load_query(qq)
                bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(),
                                        n, L, d_sc[k].data_ptr(), user.cuda_stream)
        user.synchronize()
    got = d_sc.cpu().numpy()
    idx = np.arange(0, n, 7)
    offs = (idx * L).astype(np.uint64)
    for k, qq in enumerate(queries):
        want = O.score_batch(qq, tg.reshape(-1), offs, np.full(len(idx), L, np.uint32),
                             O.dna_matrix(), -12, -4)
        assert (got[k][idx] == want).all(), k


@pytest.mark.parametrize("qlen", [1, 8, 31, 32, 33, 64, 97, 127, 128])
@pytest.mark.parametrize("params", [REF, (2, -3, -5, -2), (4, 0, -8, -2)])
def test_pair_table_path(bank, qlen, params, kernel_choice):
    """The letter-pair table (tile f16, DNA merged gaps, queries of 17-128 rows): all 25 letter
    pairs incl. N on both sides (dense N), ragged lengths, several workgroup heights, and the
    path assertion: "tile" takes the pair table, "tile-lut" the per-row LUT."""
    rng = np.random.default_rng(qlen * 31 + params[0])
    q, seqs = _random_case(rng, qlen, 300, 180, p_n=0.25)
    seqs += [q.copy() for _ in range(3)]
    bank.set_penalties(*params)
    bank.load_query(q)
    got = bank.score_targets(seqs)
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(params[0], params[1]), params[2],
                         params[3])
    kern = bank.last_kernel()
    assert (got == want).all(), (kern, [(i, int(got[i]), int(want[i]))
                                        for i in np.nonzero(got != want)[0][:8]])
    if kernel_choice == "tile" and qlen > 16:  # <= 16 rows: the R = 16 LUT kernel
        assert kern.startswith("tile f16 pair R=32"), kern
    elif kernel_choice == "tile-lut":
        assert kern.startswith("tile f16 R=") and "pair" not in kern, kern


@pytest.mark.parametrize("qlen", [5, 17, 100, 128, 129, 255, 256, 257, 400, 512, 513, 1000])
@pytest.mark.parametrize("params", [(5, -4, -10, -1), (2, -3, -5, -2), (4, 0, -8, -2)])
def test_gotoh_pair_table_path(qlen, params, kernel_choice, poisoned_buffers):
    """The letter-pair table in the Gotoh f16 tile column (R = 32; R = 16 for <= 16 rows):
    one table per query segment (512 rows; 4-column chunks when the table and the segment
    edges leave no room for 8), all 25 letter pairs incl. dense N, ragged lengths with empty
    targets, homologs near the f16 bound; "tile" takes the pair table, "tile-lut" the
    per-row LUT, "tile-u16" the u16 column (R = 16 up to 256 rows), all equal to the oracle."""
    rng = np.random.default_rng(qlen * 13 + params[0])
    q, seqs = _random_case(rng, qlen, 400, 300, p_n=0.25)
    seqs += [rng.integers(0, 4, int(n), dtype=np.uint8) for n in rng.integers(0, 7, 200)]
    for k in range(0, 400, 37):  # homologs: long gapped local alignments
        m = q[rng.integers(0, max(1, qlen // 3)):][:300].copy()
        m[::11] = rng.integers(0, 4, len(m[::11]))
        seqs[k] = m
    with S.ScoreBank(gap_model=S.GAP_GOTOH) as bank:
        bank.set_penalties(*params)
        bank.load_query(q)
        got = bank.score_targets(seqs)
        kern = bank.last_kernel()
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(params[0], params[1]), params[2],
                         params[3], O.GAP_GOTOH)
    assert (got == want).all(), (kern, [(i, int(lens[i]), int(got[i]), int(want[i]))
                                        for i in np.nonzero(got != want)[0][:8]])
    if kernel_choice == "tile":
        assert kern.startswith("tile f16") and " pair R=" in kern, kern
    elif kernel_choice == "tile-lut":
        assert " pair" not in kern, kern


@pytest.mark.parametrize("qlen", [32, 64, 128])
@pytest.mark.parametrize("tail", [1, 10, 63, 64, 65, 121, 127])
def test_partial_last_tile_full_chunks(bank, qlen, tail):
    """A last tile whose high-half lanes lie past the batch end while every valid target is
    long (whole 8-code chunks for all valid lanes): the lanes past the end must not disturb
    their low-half partners (the pair table feeds both halves from one slot)."""
    rng = np.random.default_rng(qlen + 1000 * tail)
    q = rng.integers(0, 4, qlen, dtype=np.uint8)
    seqs = [rng.integers(0, 4, int(rng.integers(96, 120)), dtype=np.uint8)
            for _ in range(3 * 128 + tail)]
    bank.set_penalties(*REF)
    bank.load_query(q)
    got = bank.score_targets(seqs)
    res, offs, lens = O.pack_residues(seqs)
    want = O.score_batch(q, res, offs, lens, O.dna_matrix(), -12, -4)
    assert (got == want).all(), [(i, int(got[i]), int(want[i]))
                                 for i in np.nonzero(got != want)[0][:8]]


def test_device_codes_past_n_read_as_n(bank):
    """Device API: codes 5..7 (not validated there) score like N (code 4) in every kernel."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(5)
    q, seqs = _random_case(rng, 100, 300, 150, p_n=0.0)
    res, offs, lens = O.pack_residues(seqs)
    hit = rng.random(len(res)) < 0.1
    res_hi = res.copy()
    res_hi[hit] = rng.integers(5, 8, int(hit.sum()))
    res_n = res.copy()
    res_n[hit] = 4
    bank.set_penalties(*REF)
    bank.load_query(q)
    out = []
    for r in (res_hi, res_n):
        dev = torch.device("cuda", 0)
        d_res = torch.from_numpy(r).to(dev)
        d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
        d_lens = torch.from_numpy(lens.astype(np.int32)).to(dev)
        d_sc = torch.zeros(len(lens), dtype=torch.int32, device=dev)
        bank.score_batch_device(d_res.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), len(lens),
                                int(lens.max()), d_sc.data_ptr(), 0)
        torch.cuda.synchronize()
        out.append(d_sc.cpu().numpy())
    assert (out[0] == out[1]).all()
    assert (out[1] == O.score_batch(q, res_n, offs, lens, O.dna_matrix(), -12, -4)).all()
