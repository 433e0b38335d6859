"""C-ABI checks that need no GPU: the library loads, exports every symbol include/swbank.h
declares, its host helpers agree with the oracle/reference encoders, and the bank refuses to
run without a gfx950 device (no CPU fallback)."""
import os
import re
import subprocess

import numpy as np
import pytest

import swbank as S
from oracle import oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "swbank.h")


def _declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sw_[a-z0-9_]+)\s*\(", txt)))


def test_header_declarations_match_python_exports():
    assert _declared() == sorted(S.EXPORTS)


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", S.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if l.strip()}
    missing = [s for s in _declared() if s not in syms]
    assert not missing, missing
    L = S.lib()
    for s in _declared():
        assert hasattr(L, s)


def test_abi_version_and_status_strings():
    assert S.lib().sw_abi_version() == S.ABI_VERSION == 6
    assert "timed out" in S.status_string(S.ERR_TIMEOUT)
    assert S.status_string(0) == "ok"
    assert "gfx950" in S.status_string(S.ERR_NO_DEVICE)
    assert S.lib().sw_max_query_len() >= 128


def test_encode_matches_convert_to_base():
    seq = "ACGTacgtNnRX-"
    got = S.encode(seq)
    assert got.tolist() == [2, 1, 3, 0, 2, 1, 3, 0, 4, 4, 4, 4, 4]
    assert (got == O.encode_dna(seq)).all()
    prot = "ARNDCQEGHILKMFPSTWYVBZX*arnduoj"
    assert (S.encode(prot, S.ALPHABET_PROTEIN) == O.encode_protein(prot)).all()


def test_pack_2bit_matches_capi_fixture():
    want = open(os.path.join(O.GOLDEN, "charto2bit_query1.hex")).read().split()
    q = O.read_fasta(O.golden_fasta("query1.fa"))[0][1]
    assert [f"{b:02x}" for b in S.pack_2bit(q)] == want
    assert (S.unpack_2bit(S.pack_2bit(q), len(q)) == S.encode(q)).all()


def test_records_match_capi_sequence_t():
    """make_records builds main_test.c's sequence_t (aligner_Header.h:19-24): ID, length and
    the charTo2bit bytes the reference host printed for query1."""
    want = open(os.path.join(O.GOLDEN, "charto2bit_query1.hex")).read().split()
    q = O.read_fasta(O.golden_fasta("query1.fa"))[0][1]
    rec = S.make_records([S.encode(q)], ids=[7])
    assert rec.shape == (1, S.RECORD_BYTES)
    assert int.from_bytes(rec[0, 0:4].tobytes(), "little") == 7
    assert int.from_bytes(rec[0, 4:6].tobytes(), "little") == len(q)
    assert [f"{b:02x}" for b in rec[0, 6:6 + len(want)]] == want
    assert not rec[0, 6 + len(want):].any()
    with pytest.raises(ValueError):
        S.make_records([np.zeros(233, np.uint8)])
    with pytest.raises(ValueError):
        S.make_records([np.array([4], np.uint8)])  # N has no 2-bit code


REF_LIB = os.path.join(REPO, "oracle", "_ref", "libaligner_ref.so")


@pytest.mark.skipif(not os.path.exists(REF_LIB), reason="oracle/_ref not built")
def test_pack_2bit_matches_reference_charto2bit():
    """The reference's own charTo2bit (aligner_Header.c:14-47), compiled into oracle/_ref/."""
    import ctypes
    ref = ctypes.CDLL(REF_LIB)
    ref.charTo2bit.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    libc = ctypes.CDLL(None)
    libc.fflush.argtypes = [ctypes.c_void_p]
    rng = np.random.default_rng(1)
    for n in (1, 3, 4, 31, 32, 128, 232):
        seq = "".join(rng.choice(list("ACGTacgtN"), n))
        buf = np.zeros(64, np.uint8)
        # the reference prints a debug trace per base (_DEBUGGING_); run it in a child
        # process-free way by muting stdout at the fd level
        fd = os.dup(1)
        with open(os.devnull, "w") as dn:
            os.dup2(dn.fileno(), 1)
            try:
                ref.charTo2bit(seq.encode(), buf.ctypes.data)
                libc.fflush(None)
            finally:
                os.dup2(fd, 1)
                os.close(fd)
        ours = S.pack_2bit(seq)
        assert (buf[:len(ours)] == ours).all(), seq


def test_fill_matrix_matches_oracle():
    assert (S.fill_matrix(S.ALPHABET_DNA, 5, -4) == O.dna_matrix(5, -4)).all()
    assert (S.fill_matrix(S.ALPHABET_PROTEIN) == O.BLOSUM62).all()


def test_no_cpu_fallback_without_gpu():
    if S.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(S.SwbankError) as ei:
        S.ScoreBank()
    assert ei.value.status == S.ERR_NO_DEVICE


def test_cli_usage_and_missing_inputs():
    r = subprocess.run([S.CLI_PATH], capture_output=True, text=True)
    assert r.returncode == 1 and "Input files missing" in r.stderr


def test_batch_validation_rejects_mismatched_arrays():
    """ScoreBank.score_batch validates on the host before the C feeder reads anything
    (a short offsets array or an out-of-range target would otherwise be a host over-read)."""
    res = np.zeros(10, np.uint8)
    r, o, l, i = S.validate_batch(res, [0, 4], [4, 6], ids=[7, 8])
    assert o.dtype == np.uint64 and l.dtype == np.uint32 and i.tolist() == [7, 8]
    with pytest.raises(ValueError):
        S.validate_batch(res, [0], [4, 6])            # fewer offsets than lengths
    with pytest.raises(ValueError):
        S.validate_batch(res, [0, -1], [4, 6])        # negative offset
    with pytest.raises(ValueError):
        S.validate_batch(res, [0, 4], [4, 6], ids=[1])  # ids count
    assert S.validate_batch(np.zeros(0, np.uint8), [], [])[2].size == 0


def test_multi_device_config_without_gpu():
    """A multi-device bank needs every listed device: none here, so it fails like a single
    bank (no CPU fallback), and more than SW_MAX_DEVICES ordinals is an argument error."""
    with pytest.raises(ValueError):
        S.ScoreBank(devices=[0] * (S.MAX_DEVICES + 1))
    if S.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(S.SwbankError) as ei:
        S.ScoreBank(devices=[0, 0])
    assert ei.value.status == S.ERR_NO_DEVICE


def test_cli_rejects_bad_device_list():
    r = subprocess.run([S.CLI_PATH, "-q", "x", "-l", "y", "-d", "0,a"], capture_output=True,
                       text=True)
    assert r.returncode == 1
