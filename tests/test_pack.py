"""The host feeder's 2-bit / 4-bit packers (csrc/swbank_pack.h, header-inline, the code
libswbank.so runs) compiled into a CPU harness (tests/c/pack_check.cc) and checked against a
byte-at-a-time restatement: SSE2 forms, and the AVX2 forms with vector tails when the CPU has
AVX2."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "smith-waterman-fpga-module_amd", "csrc")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("pack") / "pack_check")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-Werror", "-I", CSRC,
                    os.path.join(REPO, "tests", "c", "pack_check.cc"), "-o", exe], check=True)
    return exe


def _has_avx2():
    try:
        return " avx2" in open("/proc/cpuinfo").read()
    except OSError:
        return False


@pytest.mark.parametrize("isa", ["sse2", "avx2"])
def test_packers_vs_bytewise(harness, isa):
    if isa == "avx2" and not _has_avx2():
        pytest.skip("no AVX2 on this host")
    r = subprocess.run([harness, isa], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == f"pack ok ({isa})"
