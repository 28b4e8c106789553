"""tools/ holds only what runs against HEAD (verdict r5 item 6): every script passes a syntax check
(bash -n, py_compile, hipcc -fsyntax-only for the microbenchmarks), the ones with a usage line
print it, every tools/ path a kept script names exists, and every tools/ path the documents cite
either exists or is listed in tools/archive/MANIFEST.md with the commit that holds it."""
import os
import py_compile
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, "tools")
HIPCC = "/opt/rocm/bin/hipcc"


def _tracked(suffixes):
    out = subprocess.run(["git", "ls-files", "tools"], capture_output=True, text=True, cwd=ROOT)
    if out.returncode != 0:  # not a git checkout (the GPU box's snapshot): walk the tree
        files = [os.path.relpath(os.path.join(d, f), ROOT) for d, _, fs in os.walk(TOOLS)
                 for f in fs]
    else:
        files = out.stdout.split()
    return sorted(f for f in files if f.endswith(suffixes) and "/bin/" not in f)


@pytest.mark.parametrize("path", _tracked((".sh",)))
def test_shell_scripts_parse(path):
    r = subprocess.run(["bash", "-n", os.path.join(ROOT, path)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.parametrize("path", _tracked((".py",)))
def test_python_tools_compile(path, tmp_path):
    py_compile.compile(os.path.join(ROOT, path), cfile=str(tmp_path / "x.pyc"), doraise=True)


@pytest.mark.parametrize("cmd", [
    ["bash", "tools/kbench/ab_power.sh", "--help"],
    ["bash", "tools/gpu_check.sh", "--help"],
    [sys.executable, "tools/energy_budget.py", "--help"],
    [sys.executable, "tools/server_latency.py", "--help"],
])
def test_usage_lines(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert r.returncode == 0 and r.stdout.strip(), r.stderr[-2000:]


@pytest.mark.parametrize("path", _tracked((".hip", ".cpp")))
def test_device_tools_compile(path):
    """The microbenchmarks and kbench sources are valid translation units (kb_kernels.hip's
    variant builds are checked flag by flag in tests/test_abi.py)."""
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not present")
    if path.endswith("kb_kernels.hip"):
        pytest.skip("covered by tests/test_abi.py::test_kbench_sources_compile")
    inc = ["-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "ntt-based-polynomial-multiplier-fpga_amd", "csrc"),
           "-I" + os.path.join(TOOLS, "kbench")]
    lang = ["-x", "hip"] if path.endswith(".hip") or "kbench" in path else []
    if path.endswith("kbench.cpp"):  # built with the variant's name (tools/kbench/build.sh)
        lang += ["-DVARIANT=\"syntax\""]
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-std=c++17", "-fsyntax-only", *inc, *lang,
                        os.path.join(ROOT, path)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]


def _named_tools_paths(text):
    return {m.rstrip(".,;:)`'\"") for m in re.findall(r"tools/[\w./-]+", text)}


def test_kept_scripts_name_existing_tools():
    for path in _tracked((".sh", ".py")):
        text = open(os.path.join(ROOT, path), encoding="utf-8").read()
        for p in _named_tools_paths(text):
            if "/bin/" in p or p.endswith(("/bin", "libenergy.so")) or "archive" in p:
                continue
            if "MANIFEST" in text and p.startswith("tools/r"):
                continue
            # a named path exists, or it is a historical reference the manifest lists
            assert os.path.exists(os.path.join(ROOT, p)) or p in _manifest(), (path, p)


def _manifest():
    text = open(os.path.join(TOOLS, "archive", "MANIFEST.md"), encoding="utf-8").read()
    return {m for m in re.findall(r"`(tools/[^`]+)`", text)}


def test_cited_tools_exist_or_are_archived():
    """DESIGN.md / README.md / INTEGRATION.md cite scripts by path: each cited file exists, or is
    archived (tools/archive/MANIFEST.md), or is a directory of either."""
    listed = _manifest()
    dirs = {os.path.dirname(p) for p in listed}
    for doc in ("DESIGN.md", "README.md", "INTEGRATION.md"):
        text = open(os.path.join(ROOT, doc), encoding="utf-8").read()
        for p in _named_tools_paths(text):
            p = p.rstrip("/")
            if "/bin" in p or "*" in p or p.endswith("libenergy.so"):
                continue
            ok = (os.path.exists(os.path.join(ROOT, p)) or p in listed or p in dirs
                  or any(x.startswith(p + "/") for x in listed))
            assert ok, (doc, p)
