"""One bench.py line run against another build of libnttmul.so, for a same-box A/B of bench lines
(e.g. this round's library against the previous round's, interleaved in one GPU session):

    python tools/bench_ab.py <path/to/libnttmul.so> [bench.py args...]

The binding loads the given library instead of lib/libnttmul.so; the line's `build` and
profile-derived fields (traffic, valu_roofline) describe the in-tree build and are dropped, so
only the measured fields (value, kernel_ms, power, ...) are reported, with the library's path and
code object id under `ab_library`.  Run each side in its own process."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ntt-based-polynomial-multiplier-fpga_amd"))
sys.path.insert(0, ROOT)


def main():
    if len(sys.argv) < 2 or sys.argv[1] in ("-h", "--help"):
        print(__doc__.strip().splitlines()[0])
        print("usage: python tools/bench_ab.py <libnttmul.so> [bench.py args...]")
        return 0
    lib = os.path.abspath(sys.argv[1])
    import nttmul
    nttmul.LIB_PATH = lib
    import bench
    import contextlib
    import io
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main(sys.argv[2:] + ["--clock-seconds", "0", "--no-cpu-baseline"])
    line = json.loads([ln for ln in buf.getvalue().splitlines() if ln.startswith("{")][-1])
    for k in ("build", "valu_roofline", "in_kernel_clock"):
        line.pop(k, None)
    for k in ("traffic", "traffic_source"):
        line["roofline"].pop(k, None)
    line["ab_library"] = {"path": os.path.relpath(lib, ROOT), "code_object": nttmul.code_object_id(lib)}
    print(json.dumps(line))
    return 0


if __name__ == "__main__":
    sys.exit(main())
