"""Emit tools/kbench/bin/kb_rows_pl.inc (or <argv[1]>/kb_rows_pl.inc): csrc/kernels_dev.hpp's k_rows with its arguments reordered
(a, b, c, units, P) as k_rows_pl, for the kernel-argument preload A/B (KB_PL=1 builds with
-mllvm -amdgpu-kernarg-preload-count=N: LLVM preloads only leading non-aggregate arguments, and
k_rows takes its KParams aggregate first).  Generated, not committed, so the product kernel has
one source."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
s = open(os.path.join(R, "ntt-based-polynomial-multiplier-fpga_amd", "csrc", "kernels_dev.hpp")).read()
head = ("template <class A, class TIn, class TOut, int LOGS, int L1, bool PRIO = false>\n"
        "__global__ __launch_bounds__(rows_threads(LOGS), rows_min_waves(LOGS)) void k_rows(\n"
        "    KParams<A> P, const TIn *__restrict__ a, const TIn *__restrict__ b, TOut *__restrict__ c,\n"
        "    size_t units) {")
a = s.index(head)
b = s.index("  CLK_STAMP(1);\n}\n", a) + len("  CLK_STAMP(1);\n}\n")
body = s[a + len(head):b]
out = ("template <class A, class TIn, class TOut, int LOGS, int L1, bool PRIO = false>\n"
       "__global__ __launch_bounds__(rows_threads(LOGS), rows_min_waves(LOGS)) void k_rows_pl(\n"
       "    const TIn *__restrict__ a, const TIn *__restrict__ b, TOut *__restrict__ c,\n"
       "    size_t units, KParams<A> P) {" + body)
dst = sys.argv[1] if len(sys.argv) > 1 else os.path.join(R, "tools", "kbench", "bin")
os.makedirs(dst, exist_ok=True)
open(os.path.join(dst, "kb_rows_pl.inc"), "w").write(out)
