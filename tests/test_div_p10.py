"""div_p10 (csrc/rl_tb_chain.h): the decimal step's strtod division x / 10^k as
five fma-based operations with RN(10^-k), checked against IEEE division on
the host (scripts/div_p10_check.c restates the device function in C; gfx950's
v_fma_f64 is the IEEE fused multiply-add, as the host's fma())."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "..", "scripts", "div_p10_check.c")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_div_p10_matches_ieee_division(tmp_path):
    exe = str(tmp_path / "div_p10_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, SRC, "-lm"], check=True)
    out = subprocess.run([exe, "2000000"], check=False, capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "0 mismatches" in out.stdout
