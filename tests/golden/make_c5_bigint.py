"""Golden digests of C5 products (n = 65536, q = 0x3FFFFFFFFFE80001) computed WITHOUT any NTT:
Kronecker substitution with Python's built-in big-integer multiplication, then the negacyclic
fold c_k = p_k - p_(k+n) (mod q) -- the definition of colab_programs/schoolbook.py:23-46
(negacyclic_multiply) evaluated by an independent algorithm.  Inputs are the counter-based
synthetic polynomials of SURVEY §8d (oracle.fill_inputs, also k_fill on the device), so a fixture
is only (seed, index) plus the SHA-256 of the expected 64-bit words and a few coefficients.

    python tests/golden/make_c5_bigint.py        (build container; ~1 min)
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402

N, Q = 65536, 0x3FFFFFFFFFE80001
SLOT = 18  # bytes per Kronecker slot: n q^2 < 2^140 < 2^144


def kron_product(a, b, n=N, q=Q):
    """c = a * b mod (x^n + 1, q) by one big-integer multiplication."""
    def pack(v):
        buf = bytearray(SLOT * n)
        for i, x in enumerate(v):
            buf[SLOT * i:SLOT * i + 8] = int(x).to_bytes(8, "little")
        return int.from_bytes(bytes(buf), "little")
    p = (pack(a) * pack(b)).to_bytes(SLOT * 2 * n, "little")
    coef = [int.from_bytes(p[SLOT * k:SLOT * (k + 1)], "little") for k in range(2 * n)]
    return np.array([(coef[k] - coef[k + n]) % q for k in range(n)], dtype=np.uint64)


def digest(c):
    return hashlib.sha256(np.ascontiguousarray(c, dtype="<u8").tobytes()).hexdigest()


def main():
    cases = []
    for p0 in (0, 1, 1023):                       # C5 batch positions (global counter index)
        a, b = O.fill_inputs(N, Q, p0, 1)
        c = kron_product(a[0], b[0])
        cases.append({"p0": p0, "a": "counter", "sha256": digest(c),
                      "head": [int(x) for x in c[:8]], "mid": int(c[N // 2]), "last": int(c[-1])})
    a, b = O.fill_inputs(N, Q, 7, 1)              # edge: a = all (q - 1), b counter-based
    a_edge = np.full(N, Q - 1, dtype=np.uint64)
    c = kron_product(a_edge, b[0])
    cases.append({"p0": 7, "a": "all_q_minus_1", "sha256": digest(c),
                  "head": [int(x) for x in c[:8]], "mid": int(c[N // 2]), "last": int(c[-1])})
    out = {"n": N, "q": Q, "seed": O.SEED, "method": "Kronecker substitution (Python big int), "
           "negacyclic fold; independent of every NTT in this repository", "cases": cases}
    with open(os.path.join(HERE, "c5_bigint.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
