"""The C ABI from a plain C99 client (tests/c/abi_client.c), compiled with gcc against
include/swbank.h and linked to libswbank.so — the way the reference's C host would bind it.
Host-only checks run on CPU; scoring runs on the GPU and must reproduce the golden scores."""
import os
import subprocess

import pytest

import swbank as S
from oracle import oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tests", "c", "abi_client.c")


@pytest.fixture(scope="module")
def client(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("abi") / "abi_client")
    libdir = os.path.dirname(S.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror",
                    "-I", os.path.join(REPO, "include"), SRC, "-o", exe, "-L", libdir,
                    "-lswbank", f"-Wl,-rpath,{libdir}"], check=True)
    return exe


def test_c_client_host_checks(client):
    r = subprocess.run([client, "host"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "host ok"


@pytest.mark.parametrize("arg", ["", ",", "0,x", ",".join(["0"] * 17)])
def test_cli_bad_device_list(arg):
    """-d with an empty list, a bad entry, or more devices than a bank holds is a usage error
    (exit 1), never a read of an unset device ordinal."""
    q, lib = O.golden_fasta("query1.fa"), O.golden_fasta("data1.fa")
    r = subprocess.run([S.CLI_PATH, "-q", q, "-l", lib, "-d", arg], capture_output=True, text=True)
    assert r.returncode == 1 and "usage" in r.stderr, (r.returncode, r.stderr)


@pytest.mark.gpu
@pytest.mark.parametrize("lib", ["data500.fa", "data100.fa", "data10.fa"])
def test_c_client_scores_golden(client, lib):
    r = subprocess.run([client, "score", O.golden_fasta("query100.fa"), O.golden_fasta(lib)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[0].startswith("kernel ") and lines[-1] == "score ok"
    assert lines[-3].startswith("best ") and lines[-2].startswith("counters host_calls=")
    got = dict(ln.split() for ln in lines[1:-3])
    want = {t: s for src, lb, q, t, s in O.load_ref_scores()
            if lb == lib and q == "query100.fa" and src == "hdl"}
    assert want and all(int(got[t]) == s for t, s in want.items())
    best = max(want.values())
    assert int(lines[-3].split()[2]) == best


@pytest.fixture(scope="module")
def cli_asan(tmp_path_factory):
    """The CLI host built with AddressSanitizer + UBSan (host code only; the library and the
    GPU kernels are not instrumented)."""
    exe = str(tmp_path_factory.mktemp("asan") / "swbank_asan")
    libdir = os.path.dirname(S.LIB_PATH)
    pkg = os.path.dirname(libdir)
    subprocess.run(["gcc", "-std=c11", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
                    "-I", os.path.join(REPO, "include"), "-I", os.path.join(pkg, "csrc"),
                    os.path.join(pkg, "csrc", "swbank_cli.c"), "-o", exe, "-L", libdir,
                    "-lswbank", f"-Wl,-rpath,{libdir}"], check=True)
    return exe


ASAN_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0")


def _messy_fasta(path):
    with open(path, "w", newline="") as f:
        f.write(">a some description\r\nACGTNN\r\nacgt\r\n\r\n>b\r\n>c x\nGGGTTTAACC")
        f.write("\n>" + "n" * 300 + "\n" + "ACGT" * 200)  # long name, long record, no EOL


def test_cli_parsing_under_asan(cli_asan, tmp_path):
    fa = tmp_path / "messy.fa"
    _messy_fasta(fa)
    r = subprocess.run([cli_asan, "-q", str(fa), "-l", str(fa), "-R", str(tmp_path / "r.txt")],
                       capture_output=True, text=True, env=ASAN_ENV)
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
    assert r.returncode in (0, 3), r.stderr  # 3: no GPU here (no CPU fallback)
    for args in (["-q", "/nonexistent.fa", "-l", str(fa)], ["-p", "1,2", "-q", str(fa)], []):
        r = subprocess.run([cli_asan] + args, capture_output=True, text=True, env=ASAN_ENV)
        assert "AddressSanitizer" not in r.stderr and r.returncode in (1, 2)


@pytest.mark.gpu
def test_cli_scores_under_asan(cli_asan, tmp_path):
    fa = tmp_path / "messy.fa"
    _messy_fasta(fa)
    out = subprocess.run([cli_asan, "-q", O.golden_fasta("query100.fa"), "-l", str(fa), "-R",
                          str(tmp_path / "r.txt")], capture_output=True, text=True, env=ASAN_ENV)
    assert out.returncode == 0, out.stderr
    assert "AddressSanitizer" not in out.stderr and "runtime error" not in out.stderr
    ref = subprocess.run([S.CLI_PATH, "-q", O.golden_fasta("query100.fa"), "-l", str(fa)],
                         capture_output=True, text=True, check=True)
    assert out.stdout == ref.stdout and len(out.stdout.splitlines()) == 4
