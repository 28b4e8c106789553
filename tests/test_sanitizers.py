"""an ASan/UBSan CPU build of the host-only code — the planner and host API of
libnttmul (csrc/planner.cpp, csrc/hostapi.cpp) and the CPU oracle (oracle/nttmul_oracle.c) —
driven by tests/sanitize/san_driver.cpp, which also checks the results (planner tables == oracle
tables, restated products == schoolbook).  Any sanitizer report fails the run
(-fno-sanitize-recover=all)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ntt-based-polynomial-multiplier-fpga_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="no gcc")
def test_asan_ubsan_host_code(tmp_path):
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
           "-g", "-O1"]
    oracle_o = tmp_path / "oracle.o"
    subprocess.run(["gcc", "-std=gnu11", "-c", *san, "-o", str(oracle_o),
                    os.path.join(ROOT, "oracle", "nttmul_oracle.c")], check=True)
    exe = tmp_path / "san_driver"
    subprocess.run(["g++", "-std=c++17", *san, "-I", os.path.join(ROOT, "include"), "-I", CSRC,
                    "-o", str(exe), os.path.join(ROOT, "tests", "sanitize", "san_driver.cpp"),
                    os.path.join(CSRC, "planner.cpp"), os.path.join(CSRC, "hostapi.cpp"),
                    str(oracle_o)], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    out = subprocess.run([str(exe), os.path.join(ROOT, "tests", "golden"), str(tmp_path)],
                         capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-4000:]
    assert "sanitizer run ok" in out.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_tsan_copy_pool(tmp_path):
    """csrc/copy_pool.hpp (the host-buffer path's split staging copies; round 6: concurrent calls
    share the workers through a job queue instead of queueing on one call lock) under
    ThreadSanitizer: four caller threads start together and share the process-wide pool with
    varied sizes (3 MiB + 2 among them: the ceiling split) and split counts; every copy is
    compared byte for byte, and the run fails unless at least two split copies were in flight at
    once (tests/sanitize/tsan_copy_pool.cpp)."""
    exe = tmp_path / "tsan_copy_pool"
    subprocess.run(["g++", "-std=c++17", "-fsanitize=thread", "-g", "-O1", "-I", CSRC, "-o",
                    str(exe), os.path.join(ROOT, "tests", "sanitize", "tsan_copy_pool.cpp"),
                    "-pthread"], check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    out = subprocess.run([str(exe), "4", "40", "2"], capture_output=True, text=True, timeout=300,
                         env=env)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "copy pool tsan run ok" in out.stdout
