"""The per-lane decode code of the GPU kernels, run on the CPU (no GPU needed).

tests/emu/extract.py lifts the REAL lane-walk functions out of loona_amd/csrc (lit12_body,
lit12_step with its end detection, lit12_load/status, lo_decode, and the huge-literal phase's
per-piece functions) into a host header; tests/emu/shim.h stands in for the handful of HIP builtins
they use (alignbit, ubfe, perm, clz). tests/emu/emu.cpp replays the kernels' per-lane protocols — the
wave kernel's body steps then both tails (LUT3 and LUT2), the fill kernel's (LUT2), the huge-literal
phase's passes and fix rounds — on random literals (text, 5-bit-only text that reaches the decoded
bound, random bytes, EOS runs, bad and too-long padding) in exact-bound regions back to back, against
the oracle (oracle/hpk_oracle.c, the checker). What it cannot cover — LDS, waves, the fills' staging —
is the GPU suite's job (tests/test_gpu.py)."""

import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def emu(tmp_path_factory):
    if not shutil.which("g++") or not shutil.which("gcc"):
        pytest.skip("no host C/C++ compiler")
    d = tmp_path_factory.mktemp("emu")
    subprocess.check_call(["python3", os.path.join(HERE, "emu", "extract.py"), os.path.join(REPO, "loona_amd", "csrc"),
                           str(d / "walk.h")])
    shutil.copy(os.path.join(HERE, "emu", "shim.h"), d / "shim.h")
    subprocess.check_call(["gcc", "-O2", "-std=c11", "-D_GNU_SOURCE", "-c", os.path.join(REPO, "oracle", "hpk_oracle.c"),
                           "-o", str(d / "oracle.o")])
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I", str(d), "-c", os.path.join(HERE, "emu", "emu.cpp"), "-o",
                           str(d / "emu.o")])
    subprocess.check_call(["g++", "-o", str(d / "emu"), str(d / "emu.o"), str(d / "oracle.o"), "-lpthread"])
    return str(d / "emu")


@pytest.mark.parametrize("seed", [1, 2])
def test_lane_walk_emulation_matches_oracle(emu, seed):
    p = subprocess.run([emu, str(seed), "6"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "ok: 0 mismatches" in p.stdout
