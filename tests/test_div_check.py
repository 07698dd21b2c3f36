"""The exact constant-divisor division of the combine_ICP pass's tap computation
(csrc/dpft_ic.hip div_const, used by make_taps_xy) equals the IEEE division on the inputs
that can move a tap: a quick stride of tools/div_check.c (host C, the same IEEE binary32
arithmetic as the GPU: round to nearest, fused multiply-add, denormals kept)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no host C compiler")
def test_constant_divisor_division_is_exact(tmp_path):
    exe = tmp_path / "div_check"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), os.path.join(ROOT, "tools", "div_check.c"),
                    "-lm"], check=True)
    r = subprocess.run([str(exe), "2"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "total bad 0" in r.stdout, r.stdout[-2000:]
