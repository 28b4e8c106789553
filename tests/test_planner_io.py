"""CPU tests of the host-only C-ABI functions: planner API, FPGA-compat twiddle
stream (row 3) and the reference's text formats (row 4).  No GPU needed."""
import ctypes
import os

import numpy as np
import pytest

import nttmul
from oracle import oracle as O

Q0 = 12289


def test_tables_match_oracle_and_reference():
    for n, q, psi in ((256, Q0, 1002), (1024, Q0, 0), (4096, 2013265921, 0), (2048, 4293918721, 0)):
        P = O.Plan(n, q, psi)
        for name in nttmul.TABLES:
            assert np.array_equal(nttmul.table(n, q, name, psi), P.table(name)), (n, q, name)
    if O.ref_available():
        R = O.Ref()
        for name in nttmul.TABLES:
            assert np.array_equal(nttmul.table(256, Q0, name, 1002).astype(np.int64),
                                  R.table("ntt256_" + name)), name


def test_prime_and_roots():
    assert nttmul.is_prime(2013265921) and not nttmul.is_prime(2013265923)
    assert nttmul.smallest_psi(256, Q0) == O.smallest_psi(256, Q0) == 3
    for n, bits in ((256, 14), (4096, 31), (4096, 32), (65536, 62), (1024, 30)):
        q = nttmul.find_prime(n, bits)
        assert nttmul.is_prime(q) and O.is_prime(q) and (q - 1) % (2 * n) == 0
        assert q.bit_length() == bits
        # it is the largest such prime below 2^bits
        assert all(not O.is_prime(c) for c in range(q + 2 * n, 1 << bits, 2 * n))
    assert nttmul.find_prime(256, 14) == 15361 and (Q0 - 1) % 512 == 0  # 12289 is a smaller one
    w = nttmul.smallest_omega(256, 7681)
    assert pow(w, 128, 7681) == 7680
    with pytest.raises(nttmul.NttmulError):
        nttmul.table(4096, Q0, "psi_powers")                       # no 8192-th root mod 12289


def test_fpga_twiddle_stream_matches_reference_vectors(golden_dir):
    """generate_twiddles (generate_params.C:54-73) == the reference's committed W.txt / WINV.txt
    (PolyMult.v stream for N = 256, q = 7681, PE_NUMBER = 8, R = 2^18)."""
    g = np.load(os.path.join(golden_dir, "fpga_vectors.npz"))
    n, q, w, w_inv, psi, psi_inv, ninvR, R = (int(v) for v in g["param"][:8])
    assert nttmul.fpga_R(n, 13) == R == 1 << 18                    # K = 13 (test_generator.py)
    W = nttmul.fpga_twiddles(n, q, w, R)
    WI = nttmul.fpga_twiddles(n, q, w_inv, R)
    assert len(W) == 272                                           # W_COUNT, v2 communicator :33
    assert np.array_equal(W, g["w"]) and np.array_equal(WI, g["winv"])


def test_read_coefficients(golden_dir, tmp_path):
    a = nttmul.read_coefficients(os.path.join(golden_dir, "coeficientes_a.txt"), 256)
    g = np.load(os.path.join(golden_dir, "ref256.npz"))
    assert len(a) == 256 and np.array_equal(a.astype(np.uint32), g["a"][0])
    p = tmp_path / "short.txt"
    p.write_text("1 2\n3 x 4\n")                                   # stops at the invalid token
    assert list(nttmul.read_coefficients(str(p), 256)) == [1, 2, 3]
    with pytest.raises(OSError):
        nttmul.read_coefficients(str(tmp_path / "missing.txt"), 4)


def test_hex_round_trip(golden_dir, tmp_path):
    h = nttmul.read_hex(os.path.join(golden_dir, "POLY_A_HEX.txt"), 1024)
    g = np.load(os.path.join(golden_dir, "fpga_vectors.npz"))
    assert np.array_equal(h, g["poly_a_hex"])
    out = tmp_path / "x.txt"
    nttmul.write_hex(str(out), h)
    assert out.read_text() == open(os.path.join(golden_dir, "POLY_A_HEX.txt")).read()


def test_print_array_format(tmp_path):
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    path = tmp_path / "p.txt"
    f = libc.fopen(str(path).encode(), b"w")
    a = np.arange(20, dtype=np.int32) * 613
    nttmul.load_library().nttmul_print_array(f, a.ctypes.data, 20)
    libc.fclose(f)
    # time_testing256.c:46-64: "  " + 16 x "%5d" separated by " ", newline; remainder row
    exp = "  " + " ".join("%5d" % v for v in a[:16]) + "\n" + "  " + " ".join("%5d" % v for v in a[16:]) + " \n"
    assert path.read_text() == exp
