"""Host-side logic of bench.py that the driver's numbers depend on (CPU only): Infinity-Cache
rotation, the fail-closed profile lookups keyed by code object, the code-object id of the built
library, and the workload labels."""
import json
import os
import struct

import pytest

import bench
import nttmul


def test_buffer_sets():
    assert bench.buffer_sets(3 * 4096 * 4 * 65536) == 1            # C3: 3 GiB, HBM anyway
    c2 = 3 * 1024 * 4 * 4096                                        # C2: 48 MiB
    assert bench.buffer_sets(c2) == 16 and 16 * c2 >= 3 * bench.IC_BYTES
    assert bench.buffer_sets(c2, 1) == 1                            # explicit --rotate 1
    assert bench.buffer_sets(bench.IC_BYTES) == 3


def test_workload_names():
    assert bench.workload_name(4096, 2013265921, 65536, 1) == "C3"
    assert bench.workload_name(4096, 2013265921, 1 << 20, 8) == "C4"
    assert bench.workload_name(1024, 2013265921, 4096, 1) == "C2"
    assert bench.workload_name(65536, 0x3FFFFFFFFFE80001, 1024, 1) == "C5"
    assert bench.workload_name(2048, 2013265921, 10, 1) == "custom"


def _elf(sections: dict) -> bytes:
    """A minimal ELF64 image holding a .shstrtab and the given {name: bytes} sections."""
    names = b"\0.shstrtab\0" + b"".join(k.encode() + b"\0" for k in sections)
    blobs, off = [], 64 + len(names)
    for data in sections.values():
        blobs.append((off, data))
        off += len(data)
    sh_off = off + (-off) % 8
    nsec = 2 + len(sections)
    hdr = bytearray(64)
    hdr[:4] = b"\x7fELF"
    hdr[4] = 2                                   # ELFCLASS64
    hdr[5] = 1
    struct.pack_into("<Q", hdr, 0x28, sh_off)    # e_shoff
    struct.pack_into("<HHH", hdr, 0x3A, 64, nsec, 1)  # e_shentsize, e_shnum, e_shstrndx
    secs = bytearray(64 * nsec)
    struct.pack_into("<IIQQQQ", secs, 64, 1, 3, 0, 0, 64, len(names))         # .shstrtab
    name_off = 11
    for i, (k, (o, data)) in enumerate(zip(sections, blobs)):
        struct.pack_into("<IIQQQQ", secs, 64 * (2 + i), name_off, 1, 0, 0, o, len(data))
        name_off += len(k) + 1
    body = bytes(hdr) + names + b"".join(d for _, d in blobs)
    return body + b"\0" * (sh_off - len(body)) + bytes(secs)


def _elf_with_fatbin(path, payload: bytes):
    """A minimal ELF64 with a .hip_fatbin section."""
    with open(path, "wb") as f:
        f.write(_elf({".hip_fatbin": payload}))


def _bundle(entries) -> bytes:
    """A clang offload bundle of (triple, image) entries."""
    head = len(b"__CLANG_OFFLOAD_BUNDLE__") + 8 + sum(24 + len(t) for t, _ in entries)
    out, table, off = b"", b"", head
    for triple, image in entries:
        table += struct.pack("<QQQ", off, len(image), len(triple)) + triple
        off += len(image)
    out = b"__CLANG_OFFLOAD_BUNDLE__" + struct.pack("<Q", len(entries)) + table
    return out + b"".join(image for _, image in entries)


def test_code_object_id_reads_machine_code(tmp_path):
    """The id follows each amdgcn code object's .text / .rodata / .note and ignores its symbol
    tables (the compiler's __hip_cuid_* marker changes with any source edit) and host entries."""
    def lib(path, text, dynsym, host=b"host"):
        co = _elf({".note": b"meta", ".dynsym": dynsym, ".rodata": b"kd", ".text": text})
        _elf_with_fatbin(path, _bundle([(b"host-x86_64-unknown-linux-gnu-", host),
                                        (b"hipv4-amdgcn-amd-amdhsa--gfx950", co)]))
        return nttmul.code_object_id(str(path))
    base = lib(tmp_path / "a.so", b"\x01\x02", b"__hip_cuid_1111")
    assert lib(tmp_path / "b.so", b"\x01\x02", b"__hip_cuid_2222") == base   # cuid only
    assert lib(tmp_path / "c.so", b"\x01\x02", b"__hip_cuid_1111", b"h2") == base
    assert lib(tmp_path / "d.so", b"\x01\x03", b"__hip_cuid_1111") != base   # a kernel changed


def test_code_object_id(tmp_path):
    a, b = tmp_path / "a.so", tmp_path / "b.so"
    _elf_with_fatbin(a, b"kernels v1")
    _elf_with_fatbin(b, b"kernels v2")
    ia, ib = nttmul.code_object_id(str(a)), nttmul.code_object_id(str(b))
    assert len(ia) == 16 and ia != ib
    assert nttmul.code_object_id(str(a)) == ia                      # deterministic
    (tmp_path / "x.txt").write_bytes(b"not an elf")
    with pytest.raises(ValueError):
        nttmul.code_object_id(str(tmp_path / "x.txt"))
    if os.path.exists(nttmul.LIB_PATH):                              # the built library has one
        assert len(nttmul.code_object_id()) == 16


def test_profile_lookup_fails_closed(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    entry = {"n": 4096, "q": 2013265921, "batch": 65536, "code_object": "aaaa",
             "hbm_bytes_per_launch": 2.0e9, "source": "x_pmc.json", "method": "m"}
    (prof / "pmc_traffic.json").write_text(json.dumps({"entries": [entry]}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    t, src = bench.load_traffic(4096, 2013265921, 32768, "aaaa")
    assert t == 1.0e9 and "aaaa" in src                            # scaled to the batch
    t, src = bench.load_traffic(4096, 2013265921, 65536, "bbbb")   # another build
    assert t is None and "bbbb" in src
    assert bench.load_valu_bound(4096, 2013265921, "aaaa") is None  # no file: None


def test_power_probe_summary():
    """bench.power_probe: medians over the gfx-busy samples, the cap, the PPT-limiter count, and
    None without a reader (amdsmi replaced by a canned sampler)."""
    it = iter(range(10 ** 6))

    def read():
        i = next(it)
        return {"w": 1399 if i % 2 else 1397, "mhz": 1900 + (i % 3) * 50, "busy": 100 if i else 0,
                "ppt": True, "ppt_pct": 100}

    steps = []
    out = bench.power_probe(lambda: steps.append(1), lambda: None, 0.7, (read, 1400.0, 3),
                            units_per_step=1000)
    assert out["board_uj_per_unit"] == pytest.approx(
        out["socket_power_w_median"] / out["rate_during_probe"] * 1e6)
    assert steps and out["amd_smi_gpu"] == 3 and out["socket_power_cap_w"] == 1400.0
    assert out["busy_samples"] == out["samples"] - 1 >= 1
    assert out["socket_power_w_median"] in (1397, 1398, 1399)
    assert out["ppt_limiter_active"] == f"{out['busy_samples']}/{out['busy_samples']}"
    assert bench.power_probe(lambda: None, lambda: None, 0.01, None) is None
    assert bench.power_reader("", 0) is None or callable(bench.power_reader("", 0)[0])


def test_host_cores_rule(monkeypatch):
    """cpu_baseline's thread count: every core of the affinity mask, capped by the cgroup quota
    and OMP_NUM_THREADS (each reported beside the choice)."""
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    c = bench.host_cores()
    assert c["threads"] == min(x for x in (c["sched_getaffinity"], c["cgroup_cpu_quota"], 3) if x)
    assert c["OMP_NUM_THREADS"] == 3 and c["os_cpu_count"] >= c["sched_getaffinity"] >= 1
    monkeypatch.delenv("OMP_NUM_THREADS")
    c = bench.host_cores()
    assert c["OMP_NUM_THREADS"] is None and c["threads"] <= c["sched_getaffinity"]


def test_c1_single_product_line():
    """BASELINE configs[0] (C1): one unoptimized-CT product on one core, checked vs the oracle."""
    c1 = bench.c1_single(target_s=0.05)
    assert c1["matches_oracle"] and c1["cores"] == 1 and c1["n"] == 1024
    assert c1["q"] == 2013265921 and c1["value"] > 0
    assert c1["us_per_polymult"] == pytest.approx(1e6 / c1["value"])


def test_weak_scaling_batch_is_constant():
    """--batch-per-gpu is the same at every N (no switch to C4's slice at 8 ranks)."""
    assert bench.parse([]).batch_per_gpu == 65536
    assert bench.parse(["--gpus", "8"]).batch_per_gpu == 65536


def test_settle_runs_untimed_chunks_until_the_wall_time():
    """bench.settle: synchronised chunks doubling while under 10 ms, stopping once `ms` passed."""
    t = {"now": 0.0, "steps": 0, "syncs": 0}

    def step():
        t["steps"] += 1
        t["now"] += 1e-3          # each step costs 1 ms of (fake) wall time

    def sync():
        t["syncs"] += 1

    n, ms = bench.settle(step, 100.0, sync, clock=lambda: t["now"])
    assert n == t["steps"] and ms >= 100.0
    assert n < 200                # chunks stop doubling at 10 ms, so little overshoot
    assert t["syncs"] >= 5        # paced: never one unsynchronised burst
    assert bench.settle(step, 0, sync) == (0, 0.0)


def test_op_defaults_to_the_product():
    """The default step is the product (the BASELINE metric); --op forward / inverse / pointwise
    time the standalone entry points with their own unit and bytes moved."""
    assert bench.parse([]).op == "multiply"
    assert bench.OPS["multiply"] == ("polymults/s", 3)
    assert bench.OPS["forward"][1] == bench.OPS["inverse"][1] == 2   # read x, write its transform
    assert bench.OPS["pointwise"][1] == 3
    assert bench.parse(["--op", "inverse"]).op == "inverse"
    with pytest.raises(SystemExit):
        bench.parse(["--op", "square"])


def test_committed_profiles_describe_the_shipped_library():
    """The driver's bench line reads traffic and valu_roofline from the committed profiles only
    when they were measured on this build's code object (bench.py fails closed otherwise): the
    in-tree libnttmul.so must have a PMC entry for C3, C2 and C5 and a VALU bound for C3 / C2."""
    if not os.path.exists(nttmul.LIB_PATH):
        pytest.skip("libnttmul.so not built")
    co = nttmul.code_object_id()
    for n, q, batch in ((4096, 2013265921, 65536), (1024, 2013265921, 4096),
                        (65536, 0x3FFFFFFFFFE80001, 1024)):
        traffic, why = bench.load_traffic(n, q, batch, co)
        assert traffic is not None, why
    for n in (4096, 1024):
        assert bench.load_valu_bound(n, 2013265921, co) is not None, f"no VALU bound of {co} at n={n}"
