"""The decode kernel's two-symbol table (hpk_code.h, LUT2 layout) checked entry by entry on the host:
tests/lut2_check.cpp re-decodes every 12-bit prefix from the canonical code and compares each field
(symbols, first-code length, both codes' length, bits held, code count, the two range flags) with
what the lane step reads. CPU only (g++)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "loona_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_lut2_fields_match_a_code_by_code_decode(tmp_path):
    exe = tmp_path / "lut2_check"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-I", CSRC, "-o", str(exe), os.path.join(HERE, "lut2_check.cpp")])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout + out.stderr
