"""Generate the golden fixtures under tests/golden/ (run in the build container only).

The expected outputs come from the reference ITSELF, compiled from its own sources under
/root/reference by oracle/Makefile into oracle/_ref/libntt_ref.so, or — where the reference cannot
run (32-bit / 62-bit q, n > 2048) — from a pure-Python big-int restatement of the reference's own
definition of a correct product, colab_programs/schoolbook.py:23-46 (oracle.schoolbook_py).
Fixtures are data only (inputs and expected outputs); no reference source text is stored.

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

REF_DIR = "/root/reference/Multiplier_NTT_Based/NTT_Software/NTT_Software_Evaluations/NTT-256"
Q0 = 12289


def read_coeffs(path):
    # time_testing256.c:17-44 ler_coeficientes: whitespace-separated decimal int32
    with open(path) as f:
        vals = [int(x) for x in f.read().split()]
    return np.array((vals + [0] * 256)[:256], dtype=np.int64)


# NTT/ntt256.h:20-69: wrapper -> (ntt.C loop, ntt256 table it passes)
WRAPPERS = {
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


def wrappers(R):
    """The twelve n = 256 transform wrappers through the compiled reference's own loops, on 32
    inputs (one all-(q-1), one all-zero, one unit impulse, the rest random)."""
    rng = np.random.default_rng(0x57A9)
    X = rng.integers(0, Q0, (32, 256))
    X[0] = Q0 - 1; X[1] = 0; X[2] = 0; X[2, 1] = 1
    P256 = O.Plan(256, Q0, 1002)
    t = {k: P256.table(k).astype(np.uint16) for k in O.TABLES}
    out = {"x": X.astype(np.int32)}
    for name, (fn, tab) in WRAPPERS.items():
        out[name] = np.array([R.transform(fn, x, t[tab]) for x in X], dtype=np.int32)
        # the oracle's restatement of the same loop must agree (pins oracle/nttmul_oracle.c)
        ora = np.array([P256.transform(fn, x.astype(np.uint64), tab) for x in X])
        assert np.array_equal(ora.astype(np.int64), out[name].astype(np.int64)), name
    np.savez_compressed(os.path.join(HERE, "ref256_wrappers.npz"), **out)
    print("ref256_wrappers.npz written")


def main():
    if not O.ref_available():
        sys.exit("oracle/_ref/libntt_ref.so missing: run `make -C oracle` with /root/reference present")
    R = O.Ref()

    # 1. KATs at (256, 12289): test_prod_ntt256.c:47-56, NTT_PCIECommunicationv2.c:157-158,
    #    NTT_PolyMul_test.v:110-195.  Expected = the compiled reference's product.
    kats = []
    for name, a_c, b_c in [("test_prod_(1+2x)*3", [1, 2], [3]),
                           ("pcie_v2_(1+2x+3x^2)*2", [1, 2, 3], [2]),
                           ("polymul_tb_(1+2x+3x^2)(2+2x)", [1, 2, 3], [2, 2]),
                           ("time_testing_init_polyABC", {0: 1, 1: 2, 4: 2}, {0: 3, 1: 3, 3: 1}),
                           ("wrap_x^255*x^255", {255: 1}, {255: 1})]:
        a = np.zeros(256, dtype=np.int64)
        b = np.zeros(256, dtype=np.int64)
        for arr, spec in ((a, a_c), (b, b_c)):
            items = spec.items() if isinstance(spec, dict) else enumerate(spec)
            for i, v in items:
                arr[i] = v
        outs = {nm: R.product(nm, a, b).tolist() for nm in
                ("ntt256_product1", "ntt256_product4", "ntt_red256_product1", "ntt_red256_product4")}
        first = outs["ntt256_product1"]
        assert all(v == first for v in outs.values()), name
        nz = {i: v for i, v in enumerate(first) if v}
        kats.append({"name": name, "a": {str(i): int(v) for i, v in enumerate(a) if v},
                     "b": {str(i): int(v) for i, v in enumerate(b) if v},
                     "c": {str(i): int(v) for i, v in nz.items()}})
    with open(os.path.join(HERE, "kat256.json"), "w") as f:
        json.dump({"n": 256, "q": Q0, "source": "oracle/_ref (reference compiled from source)",
                   "kats": kats}, f, indent=1)

    # 2. n=256, q=12289: the reference's own input files + seeded random + edge cases,
    #    outputs of all four reference products.
    rng = np.random.default_rng(20251212)
    A = [read_coeffs(os.path.join(REF_DIR, "coeficientes_a.txt"))]
    B = [read_coeffs(os.path.join(REF_DIR, "coeficientes_b.txt"))]
    A.append(np.full(256, Q0 - 1)); B.append(np.full(256, Q0 - 1))
    A.append(np.zeros(256, dtype=np.int64)); B.append(rng.integers(0, Q0, 256))
    for _ in range(61):
        A.append(rng.integers(0, Q0, 256)); B.append(rng.integers(0, Q0, 256))
    A = np.array(A); B = np.array(B)
    outs = {nm: np.array([R.product(nm, a, b) for a, b in zip(A, B)]) for nm in
            ("ntt256_product1", "ntt256_product4", "ntt_red256_product1", "ntt_red256_product4")}
    np.savez_compressed(os.path.join(HERE, "ref256.npz"), a=A.astype(np.uint32),
                        b=B.astype(np.uint32),
                        **{k: v.astype(np.uint32) for k, v in outs.items()})

    # 2b. standalone transforms at (256, 12289, psi = 1002) through the reference's own loops:
    #     forward = mul_array16(psi_powers) + ntt_ct_std2rev(omega_powers_rev)  (ntt256.C:6-7)
    #     inverse = ntt_gs_rev2std(inv_omega_powers_rev) + mul_array16(scaled_inv_psi) (:22-23)
    P256 = O.Plan(256, Q0, 1002)
    t = {k: P256.table(k).astype(np.uint16) for k in O.TABLES}
    fwd = np.array([R.transform("ntt_ct_std2rev", R.transform("mul_array16", x, t["psi_powers"]),
                                t["omega_powers_rev"]) for x in A])
    fwd_gs = np.array([R.transform("ntt_gs_std2rev", R.transform("mul_array16", x, t["psi_powers"]),
                                   t["omega_powers"]) for x in A])
    assert np.array_equal(fwd, fwd_gs)
    inv = np.array([R.transform("mul_array16", R.transform("ntt_gs_rev2std", x,
                                                           t["inv_omega_powers_rev"]),
                                t["scaled_inv_psi_powers"]) for x in A])
    np.savez_compressed(os.path.join(HERE, "ref256_transforms.npz"), x=A.astype(np.uint32),
                        forward=fwd.astype(np.uint32), inverse=inv.astype(np.uint32))

    # 3. n = 512, 1024, 2048 at q = 12289 through the reference's generic-n loops (ntt.C) fed with
    #    tables from the oracle planner (psi = smallest order-2n element, generate_params.C:25-44).
    gen = {}
    for n in (512, 1024, 2048):
        P = O.Plan(n, Q0)
        a = rng.integers(0, Q0, (8, n)); b = rng.integers(0, Q0, (8, n))
        a[0] = Q0 - 1; b[0] = Q0 - 1
        c1 = np.array([R.generic_product(False, x, y, P) for x, y in zip(a, b)])
        c4 = np.array([R.generic_product(True, x, y, P) for x, y in zip(a, b)])
        assert np.array_equal(c1, c4)
        gen[f"n{n}_a"] = a.astype(np.uint32); gen[f"n{n}_b"] = b.astype(np.uint32)
        gen[f"n{n}_c"] = c1.astype(np.uint32); gen[f"n{n}_psi"] = np.array([P.psi])
    np.savez_compressed(os.path.join(HERE, "ref_generic_12289.npz"), **gen)

    # 2c. cyclic transforms through the reference's plain (non-psi) loops, ntt256.h:37,49:
    #     ntt_ct_std2rev(omega_powers_rev) and ntt_gs_rev2std(inv_omega_powers_rev) + n^-1
    cfw = np.array([R.transform("ntt_ct_std2rev", x, t["omega_powers_rev"]) for x in A])
    cinv = np.array([R.scalar_mul_array(R.transform("ntt_gs_rev2std", x, t["inv_omega_powers_rev"]),
                                        P256.inv_n) for x in A])
    np.savez_compressed(os.path.join(HERE, "ref256_cyclic.npz"), x=A.astype(np.uint32),
                        omega=np.array([P256.omega]), forward=cfw.astype(np.uint32),
                        inverse=cinv.astype(np.uint32))

    # 2d. the FPGA's own committed simulation vectors (Hardware_Multiplier/simulation/modelsim/
    #     test/*.txt, data files of the reference) + the cyclic product of its POLY_A x POLY_B
    hm = "/root/reference/Multiplier_NTT_Based/Hardware_Multiplier/simulation/modelsim/test"
    def rd(name):
        vals = []
        for line in open(os.path.join(hm, name)):
            line = line.strip()
            if line and not line.startswith("//"):
                vals.append(int(line.split()[0], 16))
        return np.array(vals, dtype=np.uint64)
    prm = rd("PARAM.txt")  # N, q, w, w_inv, psi, psi_inv, n_inv*R, R
    fv = {k: rd(k.upper() + ".txt") for k in ("ntt_din", "ntt_dout", "intt_din", "intt_dout",
                                                  "w", "winv", "poly_a_hex", "poly_b_hex")}
    n_f, q_f = int(prm[0]), int(prm[1])
    fv["poly_c_cyclic"] = O.cyclic_schoolbook(fv["poly_a_hex"], fv["poly_b_hex"], n_f, q_f)
    np.savez_compressed(os.path.join(HERE, "fpga_vectors.npz"), param=prm, **fv)
    # text fixtures for the reference's file formats (copies of its data files)
    import shutil
    for name in ("coeficientes_a.txt", "coeficientes_b.txt"):
        shutil.copy(os.path.join(REF_DIR, name), os.path.join(HERE, name))
    shutil.copy(os.path.join(hm, "POLY_A_HEX.txt"), os.path.join(HERE, "POLY_A_HEX.txt"))

    # 4. BASELINE moduli the reference cannot run: big-int schoolbook (schoolbook.py:23-46).
    sb = {}
    cases = [(1024, 2013265921, 3), (4096, 2013265921, 2), (1024, 4293918721, 2),
             (4096, 4293918721, 1), (1024, 0x3FFFFFFFFFE80001, 2), (256, 0x3FFFFFFFFFE80001, 2)]
    for n, q, cnt in cases:
        a, b = O.fill_inputs(n, q, 0, cnt)
        a = a.copy(); b = b.copy()
        a[0, :] = q - 1                      # all (q-1) edge case
        if cnt > 1:
            b[1, :] = 0; b[1, n - 1] = 1     # x^(n-1) * a : wrap-around sign
        c = np.array([O.schoolbook_py(x.tolist(), y.tolist(), n, q) for x, y in zip(a, b)],
                     dtype=np.uint64)
        key = f"n{n}_q{q}"
        sb[key + "_a"] = a; sb[key + "_b"] = b; sb[key + "_c"] = c
        print("schoolbook", key, "done", flush=True)
    np.savez_compressed(os.path.join(HERE, "schoolbook_bigint.npz"), **sb)
    wrappers(R)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    if sys.argv[1:] == ["wrappers"]:
        if not O.ref_available():
            sys.exit("oracle/_ref/libntt_ref.so missing")
        wrappers(O.Ref())
    else:
        main()
