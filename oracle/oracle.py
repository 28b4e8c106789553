"""ctypes front-end to the CPU oracle (oracle/liboracle.so) and to the reference build (oracle/_ref).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, never by the product (the nttmul package fails loudly instead of falling back here).

Every function here forwards to nttmul_oracle.c, which restates the reference's
NTT_Software/NTT_Software_Evaluations/NTT-256 code; see that file's header for file:line anchors.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_LIB_PATH = os.path.join(HERE, "_ref", "libntt_ref.so")

# table ids, in the order of the enum in nttmul_oracle.c
TABLES = [
    "psi_powers", "inv_psi_powers", "inv_psi_powers_rev", "scaled_inv_psi_powers",
    "omega_powers", "omega_powers_rev", "inv_omega_powers", "inv_omega_powers_rev",
    "mixed_powers", "mixed_powers_rev", "inv_mixed_powers", "inv_mixed_powers_rev",
]

_u64p = ctypes.POINTER(ctypes.c_uint64)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_i32p = ctypes.POINTER(ctypes.c_int32)


def build() -> None:
    """Compile liboracle.so (and oracle/_ref when /root/reference is present)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        build()
    lib = ctypes.CDLL(LIB_PATH)
    lib.orc_plan_create.restype = ctypes.c_void_p
    lib.orc_plan_create.argtypes = [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64]
    lib.orc_plan_destroy.argtypes = [ctypes.c_void_p]
    lib.orc_plan_table.restype = _u64p
    lib.orc_plan_table.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.orc_plan_params.argtypes = [ctypes.c_void_p, _u64p]
    lib.orc_smallest_psi.restype = ctypes.c_uint64
    lib.orc_smallest_psi.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
    lib.orc_is_prime.restype = ctypes.c_int
    lib.orc_is_prime.argtypes = [ctypes.c_uint64]
    lib.orc_powmod.restype = ctypes.c_uint64
    lib.orc_powmod.argtypes = [ctypes.c_uint64] * 3
    for name in ("orc_product1", "orc_product4", "orc_product_merged"):
        f = getattr(lib, name)
        f.argtypes = [ctypes.c_void_p, _u64p, _u64p, _u64p]
    for name in ("orc_ntt_ct_rev2std_v1", "orc_ntt_ct_rev2std", "orc_mulntt_ct_rev2std",
                 "orc_ntt_ct_std2rev", "orc_mulntt_ct_std2rev", "orc_ntt_gs_rev2std",
                 "orc_nttmul_gs_rev2std", "orc_ntt_gs_std2rev", "orc_nttmul_gs_std2rev",
                 "orc_mul_table"):
        getattr(lib, name).argtypes = [_u64p, ctypes.c_uint32, _u64p, ctypes.c_uint64]
    lib.orc_mul_array.argtypes = [_u64p, ctypes.c_uint32, _u64p, _u64p, ctypes.c_uint64]
    lib.orc_scalar_mul_array.argtypes = [_u64p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64]
    lib.orc_bitrev_shuffle.argtypes = [_u64p, ctypes.c_uint32]
    lib.orc_schoolbook.argtypes = [_u64p, _u64p, _u64p, ctypes.c_uint32, ctypes.c_uint64]
    lib.orc_cyclic_schoolbook.argtypes = [_u64p, _u64p, _u64p, ctypes.c_uint32, ctypes.c_uint64]
    lib.orc_eval_check.restype = ctypes.c_int
    lib.orc_eval_check.argtypes = [ctypes.c_void_p, _u64p, _u64p, _u64p, ctypes.c_uint32]
    lib.orc_red_product.restype = ctypes.c_int
    lib.orc_red_product.argtypes = [ctypes.c_void_p, ctypes.c_int, _i32p, _i32p, _i32p]
    lib.orc_kred_table.restype = ctypes.c_int
    lib.orc_kred_table.argtypes = [ctypes.c_void_p, ctypes.c_int, _i32p]
    lib.orc_fill_inputs.argtypes = [_u64p, _u64p, ctypes.c_uint32, ctypes.c_uint64,
                                    ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
    lib.orc_fast_batch_u32.restype = ctypes.c_double
    lib.orc_fast_batch_u32.argtypes = [ctypes.c_void_p, _u32p, _u32p, _u32p, ctypes.c_uint64,
                                       ctypes.c_int]
    lib.orc_product_batch.restype = ctypes.c_double
    lib.orc_product_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, _u64p, _u64p, _u64p,
                                      ctypes.c_uint64, ctypes.c_int]
    lib.orc_num_threads.restype = ctypes.c_int
    lib.orc_time_single.restype = ctypes.c_double
    lib.orc_time_single.argtypes = [ctypes.c_void_p, ctypes.c_int, _u64p, _u64p, _u64p,
                                    ctypes.c_int]
    return lib


_LIB: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        _LIB = _load()
    return _LIB


def _p64(x: np.ndarray):
    assert x.dtype == np.uint64 and x.flags.c_contiguous
    return x.ctypes.data_as(_u64p)


def _p32(x: np.ndarray):
    assert x.dtype == np.uint32 and x.flags.c_contiguous
    return x.ctypes.data_as(_u32p)


def _pi32(x: np.ndarray):
    assert x.dtype == np.int32 and x.flags.c_contiguous
    return x.ctypes.data_as(_i32p)


SEED = 0x4E54544D554C  # "NTTMUL" 


class Plan:
    """(n, q, psi) plan with the 12 tables of NTT/ntt.h:63-183."""

    def __init__(self, n: int, q: int, psi: int = 0):
        self._lib = lib()
        self._p = self._lib.orc_plan_create(n, q, psi)
        if not self._p:
            raise ValueError(f"oracle: invalid parameters n={n} q={q} psi={psi}")
        self.n, self.q = n, q
        prm = np.zeros(6, dtype=np.uint64)
        self._lib.orc_plan_params(self._p, _p64(prm))
        self.psi, self.omega, self.inv_psi, self.inv_omega, self.inv_n = (int(v) for v in prm[:5])
        self.logn = int(prm[5])

    def __del__(self):
        if getattr(self, "_p", None):
            self._lib.orc_plan_destroy(self._p)
            self._p = None

    def table(self, name: str) -> np.ndarray:
        ptr = self._lib.orc_plan_table(self._p, TABLES.index(name))
        return np.ctypeslib.as_array(ptr, shape=(self.n,)).copy()

    def _prod(self, fn, a, b) -> np.ndarray:
        a = np.array(a, dtype=np.uint64, copy=True)
        b = np.array(b, dtype=np.uint64, copy=True)
        c = np.zeros(self.n, dtype=np.uint64)
        fn(self._p, _p64(c), _p64(a), _p64(b))
        return c

    def product1(self, a, b) -> np.ndarray:
        """ntt256.C:5-13 sequence (CT) at this plan's (n, q)."""
        return self._prod(self._lib.orc_product1, a, b)

    def product4(self, a, b) -> np.ndarray:
        """ntt256.C:16-24 sequence (GS) at this plan's (n, q)."""
        return self._prod(self._lib.orc_product4, a, b)

    def product_merged(self, a, b) -> np.ndarray:
        """psi-merged product."""
        return self._prod(self._lib.orc_product_merged, a, b)

    def red_product(self, a, b, gs: bool) -> np.ndarray:
        """ntt_red256.C:5-27 / :30-51 (K-RED, q = 12289 only)."""
        a = np.array(a, dtype=np.int32, copy=True)
        b = np.array(b, dtype=np.int32, copy=True)
        c = np.zeros(self.n, dtype=np.int32)
        if self._lib.orc_red_product(self._p, int(gs), _pi32(c), _pi32(a), _pi32(b)) != 0:
            raise ValueError("K-RED product needs q = 12289")
        return c

    def kred_table(self, which: int) -> np.ndarray:
        out = np.zeros(self.n, dtype=np.int32)
        if self._lib.orc_kred_table(self._p, which, _pi32(out)) != 0:
            raise ValueError("K-RED tables need q = 12289")
        return out

    def transform(self, name: str, a, table: str) -> np.ndarray:
        """Run one of the restated ntt.C loops (orc_<name>) on a copy of a."""
        a = np.array(a, dtype=np.uint64, copy=True)
        t = self.table(table)
        getattr(self._lib, "orc_" + name)(_p64(a), self.n, _p64(t), self.q)
        return a

    def eval_check(self, c, a, b, points: int = 8) -> int:
        c = np.ascontiguousarray(c, dtype=np.uint64)
        a = np.ascontiguousarray(a, dtype=np.uint64)
        b = np.ascontiguousarray(b, dtype=np.uint64)
        return self._lib.orc_eval_check(self._p, _p64(c), _p64(a), _p64(b), points)

    def fast_batch_u32(self, a: np.ndarray, b: np.ndarray, threads: int = 0):
        """CPU baseline: psi-merged lazy-Shoup product over a batch; returns (c, seconds)."""
        a = np.ascontiguousarray(a, dtype=np.uint32)
        b = np.ascontiguousarray(b, dtype=np.uint32)
        c = np.zeros_like(a)
        cnt = a.size // self.n
        sec = self._lib.orc_fast_batch_u32(self._p, _p32(c), _p32(a), _p32(b), cnt, threads)
        if sec < 0:
            raise ValueError("fast_batch_u32 needs q < 2^31")
        return c, sec

    def time_single(self, a, b, gs: bool = False, reps: int = 30):
        """One product on one core, timed as time_testing256.c:147-187 (inputs restored untimed
        before each of `reps` calls, CLOCK_MONOTONIC around the call); returns (c, seconds per
        product).  gs=False: the unoptimized CT sequence ntt256.C:5-13."""
        a = np.ascontiguousarray(a, dtype=np.uint64)
        b = np.ascontiguousarray(b, dtype=np.uint64)
        c = np.zeros(self.n, dtype=np.uint64)
        sec = self._lib.orc_time_single(self._p, int(gs), _p64(c), _p64(a), _p64(b), reps)
        return c, sec

    def product_batch(self, a: np.ndarray, b: np.ndarray, gs: bool = True, threads: int = 0):
        a = np.ascontiguousarray(a, dtype=np.uint64)
        b = np.ascontiguousarray(b, dtype=np.uint64)
        c = np.zeros_like(a)
        cnt = a.size // self.n
        sec = self._lib.orc_product_batch(self._p, int(gs), _p64(c), _p64(a), _p64(b), cnt,
                                          threads)
        return c, sec


def schoolbook(a, b, n: int, q: int) -> np.ndarray:
    """colab_programs/schoolbook.py:23-46, in C."""
    a = np.array(a, dtype=np.uint64, copy=True)
    b = np.array(b, dtype=np.uint64, copy=True)
    c = np.zeros(n, dtype=np.uint64)
    lib().orc_schoolbook(_p64(c), _p64(a), _p64(b), n, q)
    return c


def cyclic_schoolbook(a, b, n: int, q: int) -> np.ndarray:
    """c = a*b mod (x^n - 1, q): the FPGA's cyclic product (Hardware_Multiplier/PolyMult.v)."""
    a = np.array(a, dtype=np.uint64, copy=True)
    b = np.array(b, dtype=np.uint64, copy=True)
    c = np.zeros(n, dtype=np.uint64)
    lib().orc_cyclic_schoolbook(_p64(c), _p64(a), _p64(b), n, q)
    return c


def schoolbook_py(a, b, n: int, q: int) -> list:
    """Pure-Python big-int restatement of schoolbook.py:23-46 (small cases only)."""
    conv = [0] * (2 * n - 1)
    for i in range(n):
        ai = int(a[i]) % q
        if ai == 0:
            continue
        for j in range(n):
            conv[i + j] += ai * (int(b[j]) % q)
    for k in range(len(conv)):
        conv[k] %= q
    return [(conv[k] - (conv[k + n] if k + n < len(conv) else 0)) % q for k in range(n)]


def fill_inputs(n: int, q: int, p0: int, count: int, seed: int = SEED):
    """SURVEY §8d counter-based inputs: returns (a, b) uint64 [count, n]."""
    a = np.zeros((count, n), dtype=np.uint64)
    b = np.zeros((count, n), dtype=np.uint64)
    lib().orc_fill_inputs(_p64(a), _p64(b), n, q, seed, p0, count)
    return a, b


def smallest_psi(n: int, q: int) -> int:
    return int(lib().orc_smallest_psi(n, q))


def is_prime(q: int) -> bool:
    return bool(lib().orc_is_prime(q))


def num_threads() -> int:
    return int(lib().orc_num_threads())


# ---------------------------------------------------------------------------------------------
# The reference itself, compiled from /root/reference by oracle/Makefile (present only in the
# build container and in snapshots taken from it).
# ---------------------------------------------------------------------------------------------

def ref_available() -> bool:
    return os.path.exists(REF_LIB_PATH)


ANCHOR_LIB_PATH = os.path.join(HERE, "_ref", "libref_anchor.so")


def ref_anchors(reps256: int = 20000, reps1024: int = 4000, seed: int = SEED) -> dict:
    """Seconds per product of the reference's own compiled objects (oracle/ref_anchor.c), single
    thread: the four n = 256 products and the ntt.C generic loops at n = 1024 with planner tables
    (q = 12289).  Each result is checked against the oracle before its time is reported."""
    if not os.path.exists(ANCHOR_LIB_PATH):
        return {}
    L = ctypes.CDLL(ANCHOR_LIB_PATH)
    L.anchor_product256.restype = ctypes.c_double
    L.anchor_product256.argtypes = [ctypes.c_int, _i32p, _i32p, _i32p, ctypes.c_int]
    L.anchor_product_generic.restype = ctypes.c_double
    u16p = ctypes.POINTER(ctypes.c_uint16)
    L.anchor_product_generic.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(u16p),
                                         _i32p, _i32p, _i32p, ctypes.c_int]
    out = {}
    q = 12289
    P = Plan(256, q, 1002)                     # the reference tables' psi (ntt256_tables.h:20)
    a, b = fill_inputs(256, q, 0, 1, seed)
    a32, b32 = a[0].astype(np.int32), b[0].astype(np.int32)
    want = P.product_merged(a[0], b[0])
    for i, name in enumerate(("ntt256_product1", "ntt256_product4", "ntt_red256_product1",
                              "ntt_red256_product4")):
        c = np.zeros(256, dtype=np.int32)
        s = L.anchor_product256(i, _pi32(a32), _pi32(b32), _pi32(c), reps256)
        if np.array_equal(c.astype(np.uint64), want):
            out[f"{name} n=256 q=12289"] = s
    n = 1024
    P = Plan(n, q)
    names = ("psi_powers", "omega_powers", "omega_powers_rev", "inv_omega_powers",
             "inv_omega_powers_rev", "scaled_inv_psi_powers")
    tabs = [np.ascontiguousarray(P.table(k).astype(np.uint16)) for k in names]
    tp = (u16p * 6)(*[t.ctypes.data_as(u16p) for t in tabs])
    a, b = fill_inputs(n, q, 0, 1, seed)
    a32, b32 = a[0].astype(np.int32), b[0].astype(np.int32)
    want = P.product_merged(a[0], b[0])
    for gs, name in ((0, "ntt.C CT loops (product1 shape)"), (1, "ntt.C GS loops (product4 shape)")):
        c = np.zeros(n, dtype=np.int32)
        s = L.anchor_product_generic(gs, n, tp, _pi32(a32), _pi32(b32), _pi32(c), reps1024)
        if np.array_equal(c.astype(np.uint64), want):
            out[f"{name} n=1024 q=12289"] = s
    return out


class Ref:
    """Direct bindings to the reference's own objects (n = 256, q = 12289 products; generic-n
    loops of ntt.C with caller-supplied uint16 tables)."""

    def __init__(self):
        self.lib = ctypes.CDLL(REF_LIB_PATH)
        for name in ("ntt256_product1", "ntt256_product4", "ntt_red256_product1",
                     "ntt_red256_product4"):
            getattr(self.lib, name).argtypes = [_i32p, _i32p, _i32p]
        _u16p = ctypes.POINTER(ctypes.c_uint16)
        for name in ("ntt_ct_rev2std_v1", "ntt_ct_rev2std", "mulntt_ct_rev2std", "ntt_ct_std2rev",
                     "mulntt_ct_std2rev", "ntt_gs_rev2std", "nttmul_gs_rev2std", "ntt_gs_std2rev",
                     "nttmul_gs_std2rev", "mul_array16"):
            getattr(self.lib, name).argtypes = [_i32p, ctypes.c_uint32, _u16p]
        self.lib.mul_array.argtypes = [_i32p, ctypes.c_uint32, _i32p, _i32p]
        self.lib.scalar_mul_array.argtypes = [_i32p, ctypes.c_uint32, ctypes.c_int32]
        self.lib.bitrev_shuffle.argtypes = [_i32p, ctypes.c_uint32]
        self._u16p = _u16p

    def product(self, name: str, a, b) -> np.ndarray:
        a = np.array(a, dtype=np.int32, copy=True)
        b = np.array(b, dtype=np.int32, copy=True)
        c = np.zeros(256, dtype=np.int32)
        getattr(self.lib, name)(_pi32(c), _pi32(a), _pi32(b))
        return c

    def table(self, name: str, signed: bool = False) -> np.ndarray:
        ct = ctypes.c_int16 if signed else ctypes.c_uint16
        arr = (ct * 256).in_dll(self.lib, name)
        return np.array(arr[:], dtype=np.int64)

    def transform(self, name: str, a, table) -> np.ndarray:
        a = np.array(a, dtype=np.int32, copy=True)
        t = np.ascontiguousarray(np.asarray(table, dtype=np.uint16))
        getattr(self.lib, name)(_pi32(a), len(a), t.ctypes.data_as(self._u16p))
        return a

    def mul_array(self, a, b) -> np.ndarray:
        a = np.ascontiguousarray(a, dtype=np.int32)
        b = np.ascontiguousarray(b, dtype=np.int32)
        c = np.zeros_like(a)
        self.lib.mul_array(_pi32(c), len(a), _pi32(a), _pi32(b))
        return c

    def scalar_mul_array(self, a, s: int) -> np.ndarray:
        a = np.array(a, dtype=np.int32, copy=True)
        self.lib.scalar_mul_array(_pi32(a), len(a), s)
        return a

    def bitrev_shuffle(self, a) -> np.ndarray:
        a = np.array(a, dtype=np.int32, copy=True)
        self.lib.bitrev_shuffle(_pi32(a), len(a))
        return a

    def generic_product(self, gs: bool, a, b, plan: Plan) -> np.ndarray:
        """ntt256.C:5-24 sequence driven through the reference's generic-n loops with tables
        generated by the oracle planner (valid for q = 12289, n <= 2048: uint16 tables)."""
        n = plan.n
        t = {k: plan.table(k).astype(np.uint16) for k in TABLES}
        a = self.transform("mul_array16", a, t["psi_powers"])
        b = self.transform("mul_array16", b, t["psi_powers"])
        if gs:
            a = self.transform("ntt_gs_std2rev", a, t["omega_powers"])
            b = self.transform("ntt_gs_std2rev", b, t["omega_powers"])
        else:
            a = self.transform("ntt_ct_std2rev", a, t["omega_powers_rev"])
            b = self.transform("ntt_ct_std2rev", b, t["omega_powers_rev"])
        c = self.mul_array(a, b)
        if gs:
            c = self.transform("ntt_gs_rev2std", c, t["inv_omega_powers_rev"])
        else:
            c = self.transform("ntt_ct_rev2std", c, t["inv_omega_powers"])
        c = self.transform("mul_array16", c, t["scaled_inv_psi_powers"])
        assert len(c) == n
        return c
