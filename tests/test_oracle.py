"""CPU tests of the oracle (oracle/nttmul_oracle.c): pinned against the reference compiled from its
own sources (oracle/_ref, when /root/reference is present) and against tests/golden/ fixtures
(always).  No GPU needed."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

Q0 = 12289
needs_ref = pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built (no reference tree)")


def _kat_arrays(kat, n):
    out = []
    for key in ("a", "b", "c"):
        v = np.zeros(n, dtype=np.uint64)
        for i, x in kat[key].items():
            v[int(i)] = x
        out.append(v)
    return out


def test_kats_golden(golden_dir):
    """test_prod_ntt256.c:47-56 and friends: (1+2x)*3 = 3+6x etc., at (256, 12289), psi = 1002."""
    data = json.load(open(os.path.join(golden_dir, "kat256.json")))
    P = O.Plan(256, Q0, 1002)
    assert len(data["kats"]) >= 5
    for kat in data["kats"]:
        a, b, c = _kat_arrays(kat, 256)
        for f in (P.product1, P.product4, P.product_merged):
            assert np.array_equal(f(a, b), c), kat["name"]
        for gs in (False, True):
            assert np.array_equal(P.red_product(a, b, gs), c.astype(np.int32)), kat["name"]
        assert np.array_equal(O.schoolbook(a, b, 256, Q0), c)


def test_ref256_golden(golden_dir):
    """All four reference products on the reference's own coefficient files + 63 more inputs."""
    g = np.load(os.path.join(golden_dir, "ref256.npz"))
    P = O.Plan(256, Q0, 1002)
    for i in range(g["a"].shape[0]):
        a, b = g["a"][i], g["b"][i]
        assert np.array_equal(P.product1(a, b), g["ntt256_product1"][i])
        assert np.array_equal(P.product4(a, b), g["ntt256_product4"][i])
        assert np.array_equal(P.red_product(a, b, False), g["ntt_red256_product1"][i].astype(np.int32))
        assert np.array_equal(P.red_product(a, b, True), g["ntt_red256_product4"][i].astype(np.int32))


def test_ref_generic_golden(golden_dir):
    """ntt.C generic-n loops at n = 512..2048, q = 12289, planner-generated tables."""
    g = np.load(os.path.join(golden_dir, "ref_generic_12289.npz"))
    for n in (512, 1024, 2048):
        P = O.Plan(n, Q0)
        assert P.psi == int(g[f"n{n}_psi"][0])
        for a, b, c in zip(g[f"n{n}_a"], g[f"n{n}_b"], g[f"n{n}_c"]):
            assert np.array_equal(P.product1(a, b), c)
            assert np.array_equal(P.product4(a, b), c)
            assert np.array_equal(P.product_merged(a, b), c)


def test_schoolbook_bigint_golden(golden_dir):
    """BASELINE moduli (31-bit, full 32-bit, 62-bit): pinned to the big-int restatement of
    schoolbook.py:23-46 (the reference cannot run these q)."""
    g = np.load(os.path.join(golden_dir, "schoolbook_bigint.npz"))
    keys = sorted({k.rsplit("_", 1)[0] for k in g.files})
    assert len(keys) == 6
    for key in keys:
        n = int(key.split("_")[0][1:])
        q = int(key.split("_")[1][1:])
        P = O.Plan(n, q)
        for a, b, c in zip(g[key + "_a"], g[key + "_b"], g[key + "_c"]):
            assert np.array_equal(P.product4(a, b), c), key
            assert np.array_equal(P.product_merged(a, b), c), key
            if n <= 1024:
                assert np.array_equal(O.schoolbook(a, b, n, q), c), key


@needs_ref
def test_tables_match_reference():
    """The 12 tables of ntt256_tables.C equal the planner's formulas (ntt.h:63-183)."""
    R = O.Ref()
    P = O.Plan(256, Q0, 1002)
    for name in O.TABLES:
        assert np.array_equal(R.table("ntt256_" + name), P.table(name).astype(np.int64)), name
    red = ["psi_powers", "omega_powers", "omega_powers_rev", "inv_omega_powers",
           "inv_omega_powers_rev", "scaled_inv_psi_powers"]
    for k, name in enumerate(red):
        assert np.array_equal(R.table("ntt_red256_" + name, signed=True), P.kred_table(k)), name


@needs_ref
def test_transforms_match_reference():
    """Every restated ntt.C loop is bit-exact with the compiled reference loop."""
    R = O.Ref()
    rng = np.random.default_rng(7)
    cases = [("ntt_ct_rev2std", "omega_powers"), ("ntt_ct_std2rev", "omega_powers_rev"),
             ("ntt_gs_rev2std", "omega_powers_rev"), ("ntt_gs_std2rev", "omega_powers"),
             ("mulntt_ct_rev2std", "mixed_powers"), ("mulntt_ct_std2rev", "mixed_powers_rev"),
             ("nttmul_gs_rev2std", "inv_mixed_powers_rev"), ("nttmul_gs_std2rev", "inv_mixed_powers"),
             ("ntt_ct_rev2std_v1", "psi_powers"), ("mul_table", "psi_powers")]
    for n in (256, 1024, 2048):
        P = O.Plan(n, Q0, 1002 if n == 256 else 0)
        for _ in range(5):
            a = rng.integers(0, Q0, n)
            for name, tab in cases:
                t = P.table(tab)
                ref_name = "mul_array16" if name == "mul_table" else name
                assert np.array_equal(R.transform(ref_name, a, t.astype(np.uint16)),
                                      P.transform(name, a, tab).astype(np.int32)), (n, name)


WRAPPERS = {  # NTT/ntt256.h:20-69: wrapper -> (ntt.C loop, ntt256 table)
    "ntt256_ct_rev2std": ("ntt_ct_rev2std", "omega_powers"),
    "ntt256_gs_rev2std": ("ntt_gs_rev2std", "omega_powers_rev"),
    "ntt256_ct_std2rev": ("ntt_ct_std2rev", "omega_powers_rev"),
    "ntt256_gs_std2rev": ("ntt_gs_std2rev", "omega_powers"),
    "intt256_ct_rev2std": ("ntt_ct_rev2std", "inv_omega_powers"),
    "intt256_gs_rev2std": ("ntt_gs_rev2std", "inv_omega_powers_rev"),
    "intt256_ct_std2rev": ("ntt_ct_std2rev", "inv_omega_powers_rev"),
    "intt256_gs_std2rev": ("ntt_gs_std2rev", "inv_omega_powers"),
    "mulntt256_ct_rev2std": ("mulntt_ct_rev2std", "mixed_powers"),
    "mulntt256_ct_std2rev": ("mulntt_ct_std2rev", "mixed_powers_rev"),
    "inttmul256_gs_rev2std": ("nttmul_gs_rev2std", "inv_mixed_powers_rev"),
    "inttmul256_gs_std2rev": ("nttmul_gs_std2rev", "inv_mixed_powers"),
}


def test_wrappers_golden(golden_dir):
    """The oracle's loops reproduce the compiled reference's twelve ntt256 wrappers
    (tests/golden/ref256_wrappers.npz) on all 32 fixture inputs."""
    g = np.load(os.path.join(golden_dir, "ref256_wrappers.npz"))
    P = O.Plan(256, Q0, 1002)
    for name, (fn, tab) in WRAPPERS.items():
        for x, exp in zip(g["x"], g[name]):
            got = P.transform(fn, x.astype(np.uint64), tab)
            assert np.array_equal(got, exp.astype(np.uint64)), name


def _bitrev_perm(v):
    b = int(np.log2(len(v)))
    return v[[int(format(i, f"0{b}b")[::-1], 2) for i in range(len(v))]]


def test_order_identities():
    """rev2std = P o std2rev o P (P = bit reversal) for every loop pair, and CT == GS per order:
    what lets the library run every wrapper with its two transform kernels."""
    rng = np.random.default_rng(3)
    for n, q in ((256, Q0), (1024, 2013265921), (4096, 2013265921)):
        P = O.Plan(n, q)
        x = rng.integers(0, q, n).astype(np.uint64)
        T = P.transform
        for fwd, rev in ((("mulntt_ct_std2rev", "mixed_powers_rev"), ("mulntt_ct_rev2std", "mixed_powers")),
                         (("ntt_ct_std2rev", "omega_powers_rev"), ("ntt_ct_rev2std", "omega_powers")),
                         (("nttmul_gs_rev2std", "inv_mixed_powers_rev"), ("nttmul_gs_std2rev", "inv_mixed_powers")),
                         (("ntt_gs_rev2std", "inv_omega_powers_rev"), ("ntt_gs_std2rev", "inv_omega_powers"))):
            assert np.array_equal(T(rev[0], x, rev[1]), _bitrev_perm(T(fwd[0], _bitrev_perm(x), fwd[1])))
        assert np.array_equal(T("ntt_gs_std2rev", x, "omega_powers"), T("ntt_ct_std2rev", x, "omega_powers_rev"))
        assert np.array_equal(T("ntt_gs_rev2std", x, "omega_powers_rev"), T("ntt_ct_rev2std", x, "omega_powers"))


@needs_ref
def test_random_products_match_reference():
    R = O.Ref()
    P = O.Plan(256, Q0, 1002)
    rng = np.random.default_rng(11)
    for _ in range(300):
        a = rng.integers(0, Q0, 256)
        b = rng.integers(0, Q0, 256)
        exp = R.product("ntt256_product4", a, b)
        assert np.array_equal(P.product4(a, b), exp)
        assert np.array_equal(P.product1(a, b), exp)
        assert np.array_equal(R.product("ntt_red256_product1", a, b), exp)


def test_planner_params():
    assert O.is_prime(2013265921) and O.is_prime(4293918721) and O.is_prime(0x3FFFFFFFFFE80001)
    assert not O.is_prime(2013265923)
    assert O.smallest_psi(256, Q0) == 3           # generate_params.C:25-44 rule
    for n, q in ((1024, 2013265921), (4096, 2013265921), (4096, 4293918721),
                 (65536, 0x3FFFFFFFFFE80001)):
        P = O.Plan(n, q)
        assert pow(P.psi, n, q) == q - 1
        assert P.psi == O.smallest_psi(n, q)
    with pytest.raises(ValueError):
        O.Plan(4096, Q0)                          # 12289 has no 8192-th root of unity
    with pytest.raises(ValueError):
        O.Plan(1000, 2013265921)                  # n not a power of two


def test_fast_cpu_baseline_matches():
    """The CPU baseline (lazy Shoup, psi-merged) equals the restated P4 sequence."""
    for n, q in ((1024, 2013265921), (4096, 2013265921), (256, Q0), (2048, 1073479681)):
        P = O.Plan(n, q)
        a, b = O.fill_inputs(n, q, 5, 6)
        a[0] = q - 1
        b[0] = q - 1
        c, sec = P.fast_batch_u32(a.astype(np.uint32), b.astype(np.uint32), threads=2)
        assert sec >= 0
        for i in range(6):
            assert np.array_equal(c[i].astype(np.uint64), P.product4(a[i], b[i])), (n, q, i)
        c4, _ = P.product_batch(a, b, gs=True, threads=2)
        assert np.array_equal(c4, c.astype(np.uint64))


def test_eval_check_62bit_65536():
    """C5 size: 62-bit q, n = 65536 — the O(n) evaluation property c(r) = a(r) b(r) at roots of
    x^n + 1, and linearity."""
    n, q = 65536, 0x3FFFFFFFFFE80001
    P = O.Plan(n, q)
    a, b = O.fill_inputs(n, q, 0, 1)
    c = P.product_merged(a[0], b[0])
    assert P.eval_check(c, a[0], b[0], points=4) == 0
    bad = c.copy()
    bad[123] = (int(bad[123]) + 1) % q
    assert P.eval_check(bad, a[0], b[0], points=1) == 1


def test_inputs_counter_based():
    a, b = O.fill_inputs(64, 2013265921, 10, 3)
    a2, b2 = O.fill_inputs(64, 2013265921, 11, 1)
    assert np.array_equal(a[1], a2[0]) and np.array_equal(b[1], b2[0])
    assert int(a.max()) < 2013265921


@needs_ref
def test_reference_anchors_run_and_agree():
    """bench.py's single-core anchors on the reference's own objects: every anchor is reported
    only when its product equals the oracle's, so all six keys present = all six agree."""
    r = O.ref_anchors(reps256=50, reps1024=10)
    assert len(r) == 6, r
    assert all(0 < v < 1e-2 for v in r.values())


def test_c5_oracle_vs_bigint_golden(golden_dir):
    """C5 size (n = 65536, 62-bit q): the oracle's restated P4 product equals the golden digests
    of tests/golden/c5_bigint.json, which were computed by Kronecker substitution with Python big
    integers (no NTT anywhere; tests/golden/make_c5_bigint.py) -- an independent pin of the
    restatement at the size the reference cannot run."""
    import hashlib
    import json
    g = json.load(open(os.path.join(golden_dir, "c5_bigint.json")))
    n, q = g["n"], g["q"]
    P = O.Plan(n, q)
    for case in g["cases"]:
        a, b = O.fill_inputs(n, q, case["p0"], 1, g["seed"])
        if case["a"] == "all_q_minus_1":
            a[0][:] = q - 1
        c = P.product_batch(a, b)[0].reshape(n)
        assert hashlib.sha256(c.astype("<u8").tobytes()).hexdigest() == case["sha256"], case["p0"]
        assert [int(x) for x in c[:8]] == case["head"] and int(c[-1]) == case["last"]
