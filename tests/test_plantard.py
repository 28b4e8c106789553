"""CPU checks of the arithmetic identities the Arith32P kernels rest on (csrc/modarith.hpp).

The GPU parity tests prove the products bit-exact end to end; these pin the number theory of
each step on its worst cases, in Python integers, so a change of modulus range or constant is
caught without a GPU:
  - Plantard's product (T. Plantard, IEEE TETC 2021): t = floor((hi32(x BR mod 2^64) + 1) q / 2^32)
    with BR = (-w 2^64 mod q) q^-1 mod 2^64 is the canonical residue of x w for EVERY 32-bit x
    when q < 2^31 (this is what lets a butterfly correct one operand instead of two);
  - the signed-input form (v_mul_hi_i32 and the high word c + (b0 >> 31), addend ceil(1.5 q)) is
    canonical for every int32 x in (-q, q);
  - the base multiplication's fold of a 4-term sum by 2^32 mod q keeps the Montgomery sum below
    2^64 and the quotient below 2q.
"""
import random

import pytest

M64 = 1 << 64
# the benchmark modulus, both ends of the 2^30..2^31 range, a mid-range NTT prime, and the small
# moduli the dispatcher also sends to Arith32P (the reference's 12289, the FPGA's 7681, ~2^20, ~2^29)
QS = [2013265921, 2147352577, 1073872897, 1811939329,
      12289, 7681, 1032193, 536813569]   # small and mid-size q: Arith32P serves every q < 2^31


def pair(w, q, signed=False):
    """planner.cpp tw_pair for Arith32P: (b0, b1), b1 adjusted for the signed-input form."""
    qinv = pow(q, -1, M64)
    b = (-w * pow(2, 64, q)) % q
    br = (b * qinv) % M64
    b0, b1 = br & 0xFFFFFFFF, br >> 32
    if signed:
        b1 = (b1 + (b0 >> 31)) & 0xFFFFFFFF
    return b0, b1


def pmul(x, b0, b1, q):
    th = (((x * b0) >> 32) + x * b1) & 0xFFFFFFFF
    return (th * q + q) >> 32


def pmul_s(x, b0, b1, q):
    b0s = b0 - (1 << 32) if b0 >= 1 << 31 else b0        # v_mul_hi_i32 reads b0 as int32
    th = (((x * b0s) >> 32) + x * b1) & 0xFFFFFFFF        # x is an int32 value here
    return (th * q + (3 * q + 1) // 2) >> 32


def edge_words(q):
    return [0, 1, q - 1, q, q + 1, 2 * q - 1, 2 * q, (1 << 31) - 1, 1 << 31, (1 << 32) - 1]


@pytest.mark.parametrize("q", QS)
def test_plantard_canonical_for_any_word(q):
    rng = random.Random(q)
    ws = [1, 2, q - 1, q - 2] + [rng.randrange(1, q) for _ in range(60)]
    xs = edge_words(q) + [rng.getrandbits(32) for _ in range(300)]
    for w in ws:
        b0, b1 = pair(w, q)
        for x in xs:
            t = pmul(x, b0, b1, q)
            assert t == (x * w) % q, (q, w, x)
    # the one inequality the proof needs: x B < 2^32 (2^32 - q) for all x < 2^32, B < q
    assert (1 << 32) * (q - 1) < (1 << 32) * ((1 << 32) - q)


@pytest.mark.parametrize("q", QS)
def test_plantard_signed_input(q):
    rng = random.Random(q + 1)
    ws = [1, q - 1] + [rng.randrange(1, q) for _ in range(60)]
    xs = [0, 1, -1, q - 1, -(q - 1), q // 2, -(q // 2)] + [rng.randrange(-q + 1, q) for _ in range(300)]
    a = (3 * q + 1) // 2
    lo, hi = q + ((1 << 31) * q + (1 << 32) - 1) // (1 << 32), (1 << 32) - ((1 << 31) * q) // (1 << 32)
    assert lo <= a < hi, "the addend window of the signed form must be non-empty"
    for w in ws:
        b0, b1 = pair(w, q, signed=True)
        for x in xs:
            assert pmul_s(x, b0, b1, q) == (x * w) % q, (q, w, x)


@pytest.mark.parametrize("q", QS)
def test_basemul_fold_bounds(q):
    """Arith32P::basemul: s < 4 (q-1)^2; s2 = hi(s) c32 + lo(s); (s2 + m q) / 2^32 < 2q."""
    c32 = (1 << 32) % q
    qneg = (-pow(q, -1, 1 << 32)) % (1 << 32)
    rng = random.Random(q + 2)
    worst = 4 * (q - 1) ** 2
    for s in [worst, worst - 1, 0, (1 << 32) - 1] + [rng.randrange(worst) for _ in range(2000)]:
        s2 = (s >> 32) * c32 + (s & 0xFFFFFFFF)
        m = ((s2 & 0xFFFFFFFF) * qneg) & 0xFFFFFFFF
        assert s2 + m * q < M64
        r = (s2 + m * q) >> 32
        assert r < 2 * q
        assert r % q == (s * pow(2, -32, q)) % q


@pytest.mark.parametrize("q", QS)
def test_p3_halfway_fold_bounds(q):
    """Arith32P3::basemul (8-coefficient blocks): four products, fold, four more products, fold,
    Montgomery; arith_select.hpp p3_fold_ok admits q only when the halfway sum fits 64 bits."""
    c32 = (1 << 32) % q
    qneg = (-pow(q, -1, 1 << 32)) % (1 << 32)
    half = 4 * (q - 1) ** 2
    ok = ((half >> 32) * c32 + 0xFFFFFFFF + half) < M64
    if not ok:
        pytest.skip("q not eligible for D = 3 (the launcher keeps D = 2)")
    rng = random.Random(q + 3)
    for s1, s2 in [(half, half), (0, 0), (half, 0), (0, half)] + \
            [(rng.randrange(half), rng.randrange(half)) for _ in range(2000)]:
        s = (s1 >> 32) * c32 + (s1 & 0xFFFFFFFF) + s2
        assert s < M64
        f = (s >> 32) * c32 + (s & 0xFFFFFFFF)
        m = ((f & 0xFFFFFFFF) * qneg) & 0xFFFFFFFF
        r = (f + m * q) >> 32
        assert r < 2 * q and r % q == ((s1 + s2) * pow(2, -32, q)) % q
