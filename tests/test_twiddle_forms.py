"""The planner's Arith32P twiddle tables, checked on the host (tests/host/twiddle_forms.cpp): every
forward / inverse entry is the Plantard pair of the reference table value (nttmul_table's
mixed_powers_rev / inv_mixed_powers_rev), in the unsigned or signed-input form the kernels use it
in (arith_select.hpp p_signed_fw_entry), exact for every multiplicand of its class."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ntt-based-polynomial-multiplier-fpga_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_planner_twiddle_forms(tmp_path):
    exe = tmp_path / "twiddle_forms"
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"), "-I", CSRC,
                    "-o", str(exe), os.path.join(ROOT, "tests", "host", "twiddle_forms.cpp"),
                    os.path.join(CSRC, "planner.cpp"), os.path.join(CSRC, "hostapi.cpp")],
                   check=True)
    env = dict(os.environ)
    env.pop("LD_PRELOAD", None)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert "twiddle forms ok" in out.stdout
