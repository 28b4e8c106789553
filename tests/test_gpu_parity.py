"""GPU parity tests: the HIP path (through the C ABI) against the oracle and the golden fixtures.

Bit-exact integer results are required everywhere.  At BASELINE.json's full sizes (C2, C3, the C4
rank-7 slice, C5) every product of the batch is compared with the oracle's OpenMP batch product on
the host cores (inputs are counter-based, so the oracle regenerates the whole batch); smaller cases
use the restated reference loops directly.
"""
import json
import os

import numpy as np
import pytest

import nttmul
from oracle import oracle as O

pytestmark = pytest.mark.gpu

Q0 = 12289
Q31 = 2013265921            # 15 * 2^27 + 1, the benchmark modulus
Q30 = 1073479681            # < 2^30
Q32 = 4293918721            # 0xFFF00001, full 32-bit word
Q62 = 0x3FFFFFFFFFE80001    # 62-bit, 2^17 | q - 1
# the ends of the Arith32 range (2^30 < q < 2^31), where the typed butterflies' bounds are
# tightest (signed Montgomery in (-0.75 q, 0.75 q), unsigned in [0, 2q)); 2^17 | q - 1
Q31HI = 2147352577
Q31LO = 1073872897


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _ctx(n, q, psi=0, **kw):
    return nttmul.Context(n, q, psi=psi, **kw)


def test_native_library_is_loaded_and_on_gpu(torch_cuda):
    ctx = _ctx(4096, Q31)
    assert ctx.info.ndev >= 1 and ctx.word_bits == 32 and ctx.info.kernel == 1
    # the kernel the bench line names is the dispatched one (D = 3 blocks at n = 4096)
    assert ctx.kernel_name(32) == "k_rows<Arith32P3,u32,u32,12,0>"
    assert ctx.kernel_name(64) == "k_rows<Arith32P3,u64,u64,12,0>"
    assert _ctx(1024, Q31).kernel_name() == "k_rows<Arith32P,u32,u32,10,0>"
    assert os.path.samefile(nttmul.LIB_PATH, nttmul.load_library()._name)


def test_dispatch_names_of_the_bench_configs(torch_cuda):
    """The kernels the library dispatches for the bench's C3, C2 and C5 batches are the ones the
    CPU suite's BENCH_DISPATCH table names (tests/test_bench_host.py), whose per-kernel hashes key
    the committed profiles; each is a kernel of the loaded library."""
    from test_bench_host import BENCH_DISPATCH
    for (n, q, batch), names in BENCH_DISPATCH.items():
        ctx = _ctx(n, q)
        assert ctx.kernel_name(batch=batch) == names, (n, q, batch)
        assert len(nttmul.dispatched_kernel_hashes(names)) == len(names.split("+"))


def _kats(golden_dir):
    data = json.load(open(os.path.join(golden_dir, "kat256.json")))
    for kat in data["kats"]:
        vecs = []
        for key in ("a", "b", "c"):
            v = np.zeros(256, dtype=np.int32)
            for i, x in kat[key].items():
                v[int(i)] = x
            vecs.append(v)
        yield kat["name"], vecs


def test_compat_shims_kats(golden_dir, torch_cuda):
    """ntt256_product1/4 and ntt_red256_product1/4 with the reference's signatures."""
    for name, (a, b, c) in _kats(golden_dir):
        for fn in (nttmul.ntt256_product1, nttmul.ntt256_product4, nttmul.ntt_red256_product1,
                   nttmul.ntt_red256_product4):
            out = np.zeros(256, dtype=np.int32)
            fn(out, a.copy(), b.copy())
            assert np.array_equal(out, c), (name, fn.__name__)


def test_ref256_golden(golden_dir, torch_cuda):
    """The reference's own coefficient files + 63 vectors: all four reference products agree with
    the GPU (batched, psi = 1002 as ntt256_tables.h:20)."""
    g = np.load(os.path.join(golden_dir, "ref256.npz"))
    ctx = _ctx(256, Q0, psi=1002)
    c = ctx.multiply(g["a"], g["b"])
    for name in ("ntt256_product1", "ntt256_product4", "ntt_red256_product1", "ntt_red256_product4"):
        assert np.array_equal(c, g[name]), name
    out = np.zeros(256, dtype=np.int32)
    nttmul.ntt256_product4(out, g["a"][0].astype(np.int32), g["b"][0].astype(np.int32))
    assert np.array_equal(out, g["ntt256_product4"][0].astype(np.int32))


def test_ref_generic_golden(golden_dir, torch_cuda):
    g = np.load(os.path.join(golden_dir, "ref_generic_12289.npz"))
    for n in (512, 1024, 2048):
        ctx = _ctx(n, Q0)
        assert ctx.psi == int(g[f"n{n}_psi"][0])
        assert np.array_equal(ctx.multiply(g[f"n{n}_a"], g[f"n{n}_b"]), g[f"n{n}_c"]), n


def test_schoolbook_bigint_golden(golden_dir, torch_cuda):
    g = np.load(os.path.join(golden_dir, "schoolbook_bigint.npz"))
    keys = sorted({k.rsplit("_", 1)[0] for k in g.files})
    for key in keys:
        n = int(key.split("_")[0][1:])
        q = int(key.split("_")[1][1:])
        ctx = _ctx(n, q)
        dt = np.uint32 if q < (1 << 32) else np.uint64
        c = ctx.multiply(g[key + "_a"].astype(dt), g[key + "_b"].astype(dt))
        assert np.array_equal(c.astype(np.uint64), g[key + "_c"]), key
        if q < (1 << 32):  # u32 words through the 64-bit kernels as well
            c64 = ctx.multiply(g[key + "_a"], g[key + "_b"], dtype=np.uint64)
            assert np.array_equal(c64, g[key + "_c"]), key


@pytest.mark.parametrize("n", [256, 512, 1024, 2048, 4096])
@pytest.mark.parametrize("q", [Q31, Q30, Q32, Q62, Q31HI, Q31LO])
def test_random_vs_oracle(n, q, torch_cuda):
    """Ragged batch sizes (partial blocks) against the restated psi-merged product."""
    P = O.Plan(n, q)
    ctx = _ctx(n, q)
    for batch in (1, 3, 17):
        a, b = O.fill_inputs(n, q, 1000 + batch, batch)
        if batch == 17:
            a[0] = q - 1; b[0] = q - 1          # all (q-1)
            a[1] = 0                            # zero polynomial
            a[2] = 0; a[2, n - 1] = 1           # x^(n-1) * x^(n-1) = -x^(n-2)
            b[2] = 0; b[2, n - 1] = 1
        dt = np.uint32 if q < (1 << 32) else np.uint64
        c = ctx.multiply(a.astype(dt), b.astype(dt)).astype(np.uint64)
        for i in range(batch):
            assert np.array_equal(c[i], P.product_merged(a[i], b[i])), (n, q, batch, i)
        if batch == 17:
            assert not c[1].any()
            exp = np.zeros(n, dtype=np.uint64); exp[n - 2] = q - 1
            assert np.array_equal(c[2], exp)


def _random_primes(bits_list, step_log, seed):
    """One random prime q = k 2^step_log + 1 of each bit length (oracle's Miller-Rabin)."""
    rng = np.random.default_rng(seed)
    out = []
    for bits in bits_list:
        bits = max(bits, step_log + 4)  # enough candidates k of that length
        while True:
            k = int(rng.integers(1 << (bits - step_log - 1), 1 << (bits - step_log)))
            q = (k << step_log) + 1
            if q.bit_length() == bits and O.is_prime(q):
                out.append(q)
                break
    return out


# every word/arithmetic class: Arith32P (incl. the D = 3 fold at n = 4096) below 2^31, Arith32W
# in [2^31, 2^32), Arith64 above; the bit lengths straddle each class boundary
_SWEEP_BITS = [14, 16, 20, 24, 28, 29, 30, 31, 31, 32, 32, 33, 36, 44, 52, 60, 61, 62, 62]


@pytest.mark.parametrize("n", [256, 1024, 4096])
def test_random_prime_sweep(n, torch_cuda):
    """Random NTT-friendly primes of every bit length 14..62 (seeded, 2n | q - 1): a ragged
    batch of random and extreme (all q - 1) operands, every product against the restated
    reference product (NTT/ntt.C:342-371 / :428-451), in the native word and in 64-bit words."""
    step = n.bit_length()  # 2n | q - 1
    for q in _random_primes(_SWEEP_BITS, step, seed=n):
        P = O.Plan(n, q)
        ctx = _ctx(n, q)
        a, b = O.fill_inputs(n, q, q & 0xFFFF, 5)
        a[4] = q - 1
        b[4] = q - 1
        exp = np.stack([P.product_merged(a[i], b[i]) for i in range(5)])
        dt = np.uint32 if q < (1 << 32) else np.uint64
        c = ctx.multiply(a.astype(dt), b.astype(dt)).astype(np.uint64)
        assert np.array_equal(c, exp), (n, q)
        if dt == np.uint32:
            assert np.array_equal(ctx.multiply(a, b, dtype=np.uint64), exp), (n, q, "u64 io")


@pytest.mark.parametrize("n", [8192, 65536])
def test_random_prime_sweep_multipass(n, torch_cuda):
    """The multi-pass product over random primes of each word class (2^17 | q - 1)."""
    for q in _random_primes([20, 30, 31, 32, 40, 62], 17, seed=n):
        P = O.Plan(n, q)
        ctx = _ctx(n, q)
        a, b = O.fill_inputs(n, q, q & 0xFFFF, 2)
        b[1] = q - 1
        dt = np.uint32 if q < (1 << 32) else np.uint64
        c = ctx.multiply(a.astype(dt), b.astype(dt)).astype(np.uint64)
        for i in range(2):
            assert np.array_equal(c[i], P.product_merged(a[i], b[i])), (n, q, i)


@pytest.mark.parametrize("n", [8192, 16384, 32768, 65536])
@pytest.mark.parametrize("q", [Q31, Q30, Q32, Q62, Q31HI, Q31LO])
def test_multipass_vs_oracle(n, q, torch_cuda):
    """n > 4096: column pass + fused rows + inverse column pass, ragged batch of 3 (and 17 at
    n = 8192) against the restated reference product (OpenMP batch) and evaluation at roots."""
    P = O.Plan(n, q)
    ctx = _ctx(n, q, validate=True)
    assert ctx.info.kernel == 2
    # 64-bit words at n = 65536 take the square 256 x 256 split (k_cols8, tiled intermediates),
    # every other multi-pass product the 2^L1 x 4096 split
    wb = 32 if q < (1 << 32) else 64
    if n == 65536 and wb == 64:
        assert ctx.kernel_name(64) == ("k_cols8<Arith64,u64,fwd> + k_rows<Arith64,u64,u64,8,8>"
                                       " + k_cols8<Arith64,u64,inv>")
    else:
        assert ctx.kernel_name(wb).startswith("k_cols_fwd<")
    for batch in ((3, 17) if n == 8192 else (3,)):
        a, b = O.fill_inputs(n, q, 7 + batch, batch)
        a[1] = q - 1
        b[2] = 0; b[2, n - 1] = 1                    # multiply by x^(n-1): a negacyclic rotation
        dt = np.uint32 if q < (1 << 32) else np.uint64
        c = ctx.multiply(a.astype(dt), b.astype(dt)).astype(np.uint64)
        ref = P.product_batch(a, b)[0].reshape(batch, n)
        bad = np.flatnonzero((c != ref).any(axis=1))
        assert bad.size == 0, (n, q, batch, bad[:8])
        rot = np.concatenate([(q - a[2, 1:]) % q, a[2, :1]]).astype(np.uint64)  # a x^(n-1)
        assert np.array_equal(c[2], rot)
    assert P.eval_check(c[0], a[0], b[0], points=2) == 0


def _torch_dtype(torch, word_bits):
    return torch.int32 if word_bits == 32 else torch.int64


def _as_np(t, word_bits):
    arr = t.cpu().numpy()
    return arr.view(np.uint32 if word_bits == 32 else np.uint64)


def _oracle_batch(P, q, a, b):
    """The oracle's whole-batch product (OpenMP over the host cores): the lazy-Shoup port for
    q < 2^31 (checked against the restated reference in test_oracle.py), else the restated
    P4 sequence (ntt256.C:16-24 on the generic ntt.C loops) in 128-bit arithmetic."""
    if q < (1 << 31):
        return P.fast_batch_u32(a.astype(np.uint32), b.astype(np.uint32))[0].astype(np.uint64)
    return P.product_batch(a, b)[0]


def _check_whole_batch(n, q, word_bits, p0, count, a, b, c, chunk=8192):
    """Every product of a device batch (global counter positions p0 .. p0 + count) against the
    oracle, in host chunks: inputs regenerated and compared, products recomputed and compared.
    Returns the number of products checked."""
    P = O.Plan(n, q)
    checked = 0
    for s0 in range(0, count, chunk):
        cnt = min(chunk, count - s0)
        ea, eb = O.fill_inputs(n, q, p0 + s0, cnt)
        sl = slice(s0 * n, (s0 + cnt) * n)
        assert np.array_equal(_as_np(a[sl], word_bits).reshape(cnt, n).astype(np.uint64), ea)
        assert np.array_equal(_as_np(b[sl], word_bits).reshape(cnt, n).astype(np.uint64), eb)
        got = _as_np(c[sl], word_bits).reshape(cnt, n).astype(np.uint64)
        bad = np.flatnonzero((got != _oracle_batch(P, q, ea, eb)).any(axis=1))
        assert bad.size == 0, f"{bad.size} mismatching products, first at {p0 + s0 + bad[0]}"
        checked += cnt
    return checked


@pytest.mark.parametrize("n,q,word_bits,batch,scratch_mb", [
    (4096, Q31, 32, 65536, 0), (1024, Q31, 32, 4096, 0), (65536, Q62, 64, 1024, 0),
    (65536, Q62, 64, 1024, 64), (65536, Q62, 64, 1000, 96), (8192, Q31, 32, 2500, 32),
    (16384, Q31, 32, 3000, 0)])
def test_full_size_device_path(n, q, word_bits, batch, scratch_mb, torch_cuda):
    """BASELINE configs C3, C2 and C5 at full size on device-resident data; C5 also in 8 and in
    6 ragged multi-pass sub-batches and n = 8192 in three (nttmul_params.scratch_mb bounds each
    scratch buffer): every product against the oracle, bit-exact."""
    torch = torch_cuda
    ctx = _ctx(n, q, scratch_mb=scratch_mb)
    dt = _torch_dtype(torch, word_bits)
    a = torch.empty(batch * n, dtype=dt, device="cuda")
    b = torch.empty_like(a)
    c = torch.empty_like(a)
    stream = torch.cuda.current_stream().cuda_stream
    ctx.fill_random_device(a, b, 0, batch, word_bits, stream=stream)
    ctx.multiply_device(c, a, b, batch, word_bits, stream=stream)
    # what ran is what the dry-run dispatch names for this batch (one stream: no overlap rule)
    assert ctx.last_kernel_name() == ctx.kernel_name(word_bits, batch) != ""
    torch.cuda.synchronize()
    assert _check_whole_batch(n, q, word_bits, 0, batch, a, b, c) == batch


@pytest.mark.parametrize("n,q", [(256, Q31), (512, Q31), (1024, Q31), (1024, Q30), (2048, Q31),
                                 (4096, Q31), (4096, Q31HI)])
def test_issue_priority_variants(n, q, torch_cuda):
    """The fused product has two launch forms (kernels.hip rows_prio): batches of at most 4 waves
    per SIMD run k_rows<..., PRIO = true> (issue priority lowered as each wave completes its
    transforms), larger ones the oldest-first kernel.  On both sides of the threshold the library
    names the kernel it launches and every product equals the oracle's."""
    torch = torch_cuda
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    waves_per_product = max(1, n // 16 // 64)           # n / 16 threads per product
    products_per_wave = max(1, 64 // (n // 16))
    limit = 16 * cus * products_per_wave // waves_per_product  # 4 waves x 4 SIMDs per CU
    ctx = _ctx(n, q)
    stream = torch.cuda.current_stream().cuda_stream
    for batch, prio in ((limit, True), (limit + 1 + 16, False), (7, True)):
        name = ctx.kernel_name(32, batch)
        assert name.endswith(",prio>") == prio, (batch, name)
        a = torch.empty(batch * n, dtype=torch.int32, device="cuda")
        b = torch.empty_like(a)
        c = torch.empty_like(a)
        ctx.fill_random_device(a, b, 0, batch, 32, stream=stream)
        ctx.multiply_device(c, a, b, batch, 32, stream=stream)
        torch.cuda.synchronize()
        assert _check_whole_batch(n, q, 32, 0, batch, a, b, c) == batch
    assert not ctx.kernel_name(32).endswith(",prio>")   # batch 0: a large batch


@pytest.mark.parametrize("mode", [1, -1])
def test_issue_priority_forced_by_params(mode, torch_cuda):
    """nttmul_params.issue_prio = 1 / -1 forces the issue-prioritised / oldest-first fused kernel
    for every batch size and stream pattern; products stay exact."""
    torch = torch_cuda
    n, q, batch = 1024, Q31, 300
    ctx = _ctx(n, q, issue_prio=mode)
    want = mode > 0
    for b in (7, 1 << 20):
        assert ctx.kernel_name(32, b).endswith(",prio>") == want, (mode, b)
    a = torch.empty(batch * n, dtype=torch.int32, device="cuda")
    b_, c = torch.empty_like(a), torch.empty_like(a)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    ctx.fill_random_device(a, b_, 0, batch, 32, stream=s1.cuda_stream)
    torch.cuda.synchronize()
    for st in (s1, s2, s1):
        ctx.multiply_device(c, a, b_, batch, 32, stream=st.cuda_stream)
        assert ctx.last_kernel_name().endswith(",prio>") == want
    torch.cuda.synchronize()
    assert _check_whole_batch(n, q, 32, 0, batch, a, b_, c) == batch


@pytest.mark.parametrize("zc,path", [(0, 2), (-1, 0)])
def test_zero_copy_knob(zc, path, torch_cuda):
    """nttmul_params.zero_copy_kb: a one-product n = 256 host call runs zero-copy on the pinned
    staging buffers by default (path 2) and staged through device buffers with -1 (path 0);
    both give the oracle's product.  (small_server = -1: such a call otherwise goes to the
    resident device server, path 3.)"""
    n, q = 256, Q31
    ctx = _ctx(n, q, zero_copy_kb=zc, small_server=-1)
    a, b = O.fill_inputs(n, q, 3, 1)
    got = ctx.multiply(a.astype(np.uint32), b.astype(np.uint32)).astype(np.uint64)
    assert ctx.last_host_path() == path
    assert np.array_equal(got[0], O.Plan(n, q).product_merged(a[0], b[0]))


def test_issue_priority_follows_streams(torch_cuda):
    """Calls alternating over two streams overlap, so the library leaves the issue priority off
    for them (nttmul.cpp run_device); consecutive calls on one stream get it.  The last launch is
    named by nttmul_last_kernel_name, and the products stay exact either way."""
    torch = torch_cuda
    n, q, batch = 1024, Q31, 256
    ctx = _ctx(n, q)
    assert ctx.last_kernel_name() == ""
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    a = torch.empty(batch * n, dtype=torch.int32, device="cuda")
    b = torch.empty_like(a)
    c1, c2 = torch.empty_like(a), torch.empty_like(a)
    ctx.fill_random_device(a, b, 0, batch, 32, stream=s1.cuda_stream)
    torch.cuda.synchronize()
    ctx.multiply_device(c1, a, b, batch, 32, stream=s1.cuda_stream)
    assert ctx.last_kernel_name() == "k_rows<Arith32P,u32,u32,10,0,prio>"   # first call
    ctx.multiply_device(c2, a, b, batch, 32, stream=s2.cuda_stream)
    assert ctx.last_kernel_name() == "k_rows<Arith32P,u32,u32,10,0>"        # stream changed
    ctx.multiply_device(c2, a, b, batch, 32, stream=s2.cuda_stream)
    assert ctx.last_kernel_name() == "k_rows<Arith32P,u32,u32,10,0,prio>"   # same stream again
    ctx.multiply_device(c1, a, b, batch, 32)                                 # null stream
    assert ctx.last_kernel_name() == "k_rows<Arith32P,u32,u32,10,0>"
    torch.cuda.synchronize()
    assert _check_whole_batch(n, q, 32, 0, batch, a, b, c1) == batch
    assert _check_whole_batch(n, q, 32, 0, batch, a, b, c2) == batch


def test_c5_bigint_golden(golden_dir, torch_cuda):
    """C5 products (n = 65536, q = 0x3FFFFFFFFFE80001) on the device, through the product path the
    bench runs (device-resident, counter-based inputs at their C5 batch positions): every output
    word's SHA-256 equals tests/golden/c5_bigint.json, computed by Kronecker substitution with
    Python big integers -- no NTT, independent of the oracle."""
    import hashlib
    torch = torch_cuda
    g = json.load(open(os.path.join(golden_dir, "c5_bigint.json")))
    n, q = g["n"], g["q"]
    ctx = _ctx(n, q)
    s = torch.cuda.current_stream().cuda_stream
    for case in g["cases"]:
        a = torch.empty(n, dtype=torch.int64, device="cuda")
        b = torch.empty_like(a)
        c = torch.empty_like(a)
        ctx.fill_random_device(a, b, case["p0"], 1, 64, seed=g["seed"], stream=s)
        if case["a"] == "all_q_minus_1":
            a.fill_(q - 1)
        ctx.multiply_device(c, a, b, 1, 64, stream=s)
        torch.cuda.synchronize()
        got = _as_np(c, 64)
        assert hashlib.sha256(got.astype("<u8").tobytes()).hexdigest() == case["sha256"], case
        assert [int(x) for x in got[:8]] == case["head"] and int(got[-1]) == case["last"]


def test_c4_last_rank_slice(torch_cuda):
    """C4 (n = 4096, 2^20 products over 8 GPUs): the slice rank 7 owns, at its full size
    (131,072 products from global index 7 * 131,072), generated and multiplied on this device as
    bench.py does; every product against the oracle at its global counter position."""
    import bench
    torch = torch_cuda
    n, q, world, rank = 4096, Q31, 8, 7
    p0, p1 = bench.shard(1 << 20, rank, world)
    count = p1 - p0
    assert count == 131072
    ctx = _ctx(n, q)
    a = torch.empty(count * n, dtype=torch.int32, device="cuda")
    b = torch.empty_like(a)
    c = torch.empty_like(a)
    stream = torch.cuda.current_stream().cuda_stream
    ctx.fill_random_device(a, b, p0, count, 32, stream=stream)
    ctx.multiply_device(c, a, b, count, 32, stream=stream)
    torch.cuda.synchronize()
    assert _check_whole_batch(n, q, 32, p0, count, a, b, c) == count


@pytest.mark.parametrize("scratch_mb", [0, 32])
def test_device_calls_on_two_streams(scratch_mb, torch_cuda):
    """Two multi-pass products enqueued back to back on two different streams share the
    context's scratch (nttmul.cpp Scratch, event-ordered), also when each call runs in
    sub-batches through it (scratch_mb 32: three per call)."""
    torch = torch_cuda
    n, q, batch = 16384, Q31, 1200
    ctx = _ctx(n, q, scratch_mb=scratch_mb)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    a = torch.empty(batch * n, dtype=torch.int32, device="cuda")
    b = torch.empty_like(a)
    a2, b2 = torch.empty_like(a), torch.empty_like(a)
    c, c2 = torch.empty_like(a), torch.empty_like(a)
    ctx.fill_random_device(a, b, 0, batch, 32, stream=s1.cuda_stream)
    ctx.fill_random_device(a2, b2, batch, batch, 32, stream=s2.cuda_stream)
    torch.cuda.synchronize()
    for _ in range(3):
        ctx.multiply_device(c, a, b, batch, 32, stream=s1.cuda_stream)
        ctx.multiply_device(c2, a2, b2, batch, 32, stream=s2.cuda_stream)
    torch.cuda.synchronize()
    assert _check_whole_batch(n, q, 32, 0, batch, a, b, c) == batch
    assert _check_whole_batch(n, q, 32, batch, batch, a2, b2, c2) == batch


def test_validate_flag(torch_cuda):
    ctx = _ctx(1024, Q31, validate=True)
    a, b = O.fill_inputs(1024, Q31, 0, 2)
    a = a.astype(np.uint32); b = b.astype(np.uint32)
    ctx.multiply(a, b)
    a[1, 5] = Q31
    with pytest.raises(nttmul.NttmulError) as ei:
        ctx.multiply(a, b)
    assert ei.value.status == nttmul.NTTMUL_ERANGE


def test_empty_and_invalid_calls(torch_cuda):
    """Edge cases of the product entry points: an empty batch is a successful no-op on both paths
    (null pointers allowed, nothing written), a non-empty batch with a null operand, a word size
    other than 32/64 or 32-bit words for a 62-bit q are NTTMUL_EINVAL, on the host path as on the
    device path."""
    import ctypes
    lib = nttmul.load_library()
    ctx = _ctx(1024, Q31)
    h = ctx._h
    md = lib.nttmul_multiply_batch_device
    s = torch_cuda.cuda.current_stream().cuda_stream
    c = torch_cuda.full((1024,), 7, dtype=torch_cuda.int32, device="cuda")
    assert md(h, None, None, None, 0, 32, 0, ctypes.c_void_p(s)) == nttmul.NTTMUL_OK
    assert md(h, c.data_ptr(), c.data_ptr(), c.data_ptr(), 0, 32, 0, ctypes.c_void_p(s)) == 0
    torch_cuda.cuda.synchronize()
    assert bool((c == 7).all())                                   # nothing written
    assert md(h, None, c.data_ptr(), c.data_ptr(), 1, 32, 0, None) == nttmul.NTTMUL_EINVAL
    assert md(h, c.data_ptr(), c.data_ptr(), c.data_ptr(), 0, 7, 0, None) == nttmul.NTTMUL_EINVAL
    mh = lib.nttmul_multiply_batch_u32
    assert mh(h, None, None, None, 0) == nttmul.NTTMUL_OK
    buf = np.zeros(1024, dtype=np.uint32)
    assert mh(h, buf.ctypes.data, None, buf.ctypes.data, 1) == nttmul.NTTMUL_EINVAL
    out = ctx.multiply(np.zeros((0, 1024), np.uint32), np.zeros((0, 1024), np.uint32))
    assert out.shape == (0, 1024)
    c62 = _ctx(1024, Q62)
    for bt in (0, 1):    # 32-bit words cannot hold a 62-bit q's residues, empty batch or not
        assert lib.nttmul_multiply_batch_u32(c62._h, buf.ctypes.data, buf.ctypes.data,
                                             buf.ctypes.data, bt) == nttmul.NTTMUL_EINVAL
        assert md(c62._h, c.data_ptr(), c.data_ptr(), c.data_ptr(), bt, 32, 0,
                  None) == nttmul.NTTMUL_EINVAL


def test_single_multiply_entry(torch_cuda):
    a, b = O.fill_inputs(4096, Q31, 3, 1)
    c = nttmul.multiply(a[0], b[0], 4096, Q31)
    assert np.array_equal(c.astype(np.uint64), O.Plan(4096, Q31).product_merged(a[0], b[0]))


@pytest.mark.parametrize("n,q,ndev,batch", [(2048, Q31, 2, 9), (4096, Q31, 2, 1537),
                                             (4096, Q31, 3, 3001), (65536, Q62, 2, 9),
                                             (1024, Q62, 4, 2049)])
def test_multi_device_context_split(n, q, ndev, batch, torch_cuda):
    """The host-buffer call split over `ndev` context devices, each slice driven by its own host
    thread (nttmul.cpp run_host).  NTTMUL_FLAG_SHARE_DEVICES maps the slices round-robin over the
    visible devices, so on a one-GPU box every slice shares it (own streams, slots and scratch);
    with ndev real GPUs each slice gets its own.  Every product is checked, staged and direct."""
    ctx = _ctx(n, q, ndev=ndev, share_devices=True)
    assert ctx.info.ndev == ndev
    a, b = O.fill_inputs(n, q, 5, batch)
    dt = np.uint32 if q < (1 << 32) else np.uint64
    ref = O.Plan(n, q).product_batch(a, b)[0].reshape(batch, n)
    c = ctx.multiply(a.astype(dt), b.astype(dt)).astype(np.uint64)
    assert np.array_equal(c, ref)
    assert ctx.last_host_path() in (0, 2)
    ap, bp, cp = (nttmul.host_empty((batch, n), dt) for _ in range(3))
    ap[...] = a
    bp[...] = b
    cp[...] = 0
    ctx.multiply(ap, bp, out=cp)
    assert ctx.last_host_path() == 1
    assert np.array_equal(cp.astype(np.uint64), ref)


# ---------------------------------------------------------------------------------------------
# Standalone transforms
# ---------------------------------------------------------------------------------------------

def test_transforms_ref256_golden(golden_dir, torch_cuda):
    """forward == the reference's mul_array16(psi) + ntt_ct_std2rev (and the GS variant);
    inverse == ntt_gs_rev2std + mul_array16(scaled_inv_psi), on the reference's own inputs."""
    g = np.load(os.path.join(golden_dir, "ref256_transforms.npz"))
    ctx = _ctx(256, Q0, psi=1002)
    assert np.array_equal(ctx.forward(g["x"]), g["forward"])
    assert np.array_equal(ctx.inverse(g["x"]), g["inverse"])


@pytest.mark.parametrize("n", [256, 1024, 4096, 8192, 65536])
@pytest.mark.parametrize("q", [Q31, Q30, Q32, Q62, Q31HI])
def test_transforms_vs_oracle(n, q, torch_cuda):
    P = O.Plan(n, q)
    ctx = _ctx(n, q)
    a, b = O.fill_inputs(n, q, 11, 3)
    a[0] = q - 1
    dt = np.uint32 if q < (1 << 32) else np.uint64
    fa = ctx.forward(a.astype(dt)).astype(np.uint64)
    fb = ctx.forward(b.astype(dt)).astype(np.uint64)
    for i in range(3):
        assert np.array_equal(fa[i], P.transform("mulntt_ct_std2rev", a[i], "mixed_powers_rev"))
    assert np.array_equal(ctx.inverse(fa.astype(dt)).astype(np.uint64), a)      # round trip
    pw = ctx.pointwise(fa.astype(dt), fb.astype(dt)).astype(np.uint64)
    exp = np.array([[int(x) * int(y) % q for x, y in zip(r, s)] for r, s in zip(fa, fb)],
                   dtype=np.uint64)
    assert np.array_equal(pw, exp)
    c = ctx.inverse(pw.astype(dt)).astype(np.uint64)                           # = a * b
    assert np.array_equal(c, ctx.multiply(a.astype(dt), b.astype(dt)).astype(np.uint64))


def test_transforms_device_path(torch_cuda):
    torch = torch_cuda
    n, q, batch = 4096, Q31, 4096
    ctx = _ctx(n, q)
    a = torch.empty(batch * n, dtype=torch.int32, device="cuda")
    b = torch.empty_like(a)
    s = torch.cuda.current_stream().cuda_stream
    ctx.fill_random_device(a, b, 0, batch, 32, stream=s)
    fa, fb, pw, c, c2 = (torch.empty_like(a) for _ in range(5))
    ctx.forward_device(fa, a, batch, 32, stream=s)
    ctx.forward_device(fb, b, batch, 32, stream=s)
    ctx.pointwise_device(pw, fa, fb, batch, 32, stream=s)
    ctx.inverse_device(c, pw, batch, 32, stream=s)
    ctx.multiply_device(c2, a, b, batch, 32, stream=s)
    torch.cuda.synchronize()
    assert torch.equal(c, c2)


# ---------------------------------------------------------------------------------------------
# FPGA-compat cyclic mode and the reference's timing harness (row 4)
# ---------------------------------------------------------------------------------------------

def test_cyclic_reference_loops(golden_dir, torch_cuda):
    """Cyclic mode's transforms are the reference's plain ntt256_ct_std2rev / gs_rev2std (+ n^-1)."""
    g = np.load(os.path.join(golden_dir, "ref256_cyclic.npz"))
    ctx = _ctx(256, Q0, psi=int(g["omega"][0]), cyclic=True)
    assert ctx.info.cyclic == 1
    assert np.array_equal(ctx.forward(g["x"]), g["forward"])
    assert np.array_equal(ctx.inverse(g["x"]), g["inverse"])


def test_cyclic_fpga_vectors(golden_dir, torch_cuda):
    """The FPGA's committed ModelSim vectors (q = 7681, w = 3844): NTT_DIN -> NTT_DOUT, the
    inverse back, and the cyclic product of POLY_A x POLY_B (Hardware_Multiplier/PolyMult.v)."""
    g = np.load(os.path.join(golden_dir, "fpga_vectors.npz"))
    n, q, w = (int(v) for v in g["param"][:3])
    ctx = _ctx(n, q, psi=w, cyclic=True)
    assert np.array_equal(ctx.forward(g["ntt_din"]).astype(np.uint64), g["ntt_dout"])
    assert np.array_equal(ctx.inverse(g["ntt_dout"]).astype(np.uint64), g["ntt_din"])
    c = ctx.multiply(g["poly_a_hex"], g["poly_b_hex"]).astype(np.uint64)
    assert np.array_equal(c, g["poly_c_cyclic"])
    a = np.zeros(n, np.uint32); a[:3] = [1, 2, 3]                # NTT_PolyMul_test.v:110-195 KAT
    b = np.zeros(n, np.uint32); b[:2] = [2, 2]
    assert list(ctx.multiply(a, b)[:5]) == [2, 6, 10, 6, 0]


@pytest.mark.parametrize("n,q", [(1024, Q31), (4096, Q31), (8192, Q31), (4096, Q30), (8192, Q30),
                                 (2048, Q62)])
def test_cyclic_vs_schoolbook(n, q, torch_cuda):
    ctx = _ctx(n, q, cyclic=True)
    a, b = O.fill_inputs(n, q, 3, 2)
    a[1] = q - 1
    dt = np.uint32 if q < (1 << 32) else np.uint64
    c = ctx.multiply(a.astype(dt), b.astype(dt)).astype(np.uint64)
    for i in range(2):
        assert np.array_equal(c[i], O.cyclic_schoolbook(a[i], b[i], n, q)), (n, q, i)


def _horner(coeffs, y, q):
    acc = 0
    for v in reversed([int(x) for x in coeffs]):
        acc = (acc * y + v) % q
    return acc


@pytest.mark.parametrize("n,q", [(65536, Q62), (65536, Q32), (32768, Q31), (16384, Q62)])
def test_cyclic_multipass(n, q, torch_cuda):
    """Cyclic products (NTTMUL_FLAG_CYCLIC, the FPGA flow's x^n - 1) on the multi-pass kernels,
    including the square split at n = 65536 with 64-bit words, where a schoolbook check is out of
    reach: a monomial product is an exact rotation, and a random product agrees with
    a(w^r) b(w^r) at random n-th roots of unity (c = a b mod x^n - 1 evaluates multiplicatively
    there)."""
    ctx = _ctx(n, q, cyclic=True)
    assert ctx.info.cyclic == 1 and ctx.info.kernel == 2
    omega = int(ctx.info.omega)
    assert pow(omega, n, q) == 1 and pow(omega, n // 2, q) == q - 1
    a, b = O.fill_inputs(n, q, 91, 3)
    rng = np.random.default_rng(n ^ (q & 0xFFFF))
    k = int(rng.integers(1, n - 1))
    b[1] = 0; b[1, n - 1] = 1                       # a x^(n-1): c[j] = a[(j + 1) mod n]
    b[2] = 0; b[2, k] = 1                           # a x^k:     c[j] = a[(j - k) mod n]
    dt = np.uint32 if q < (1 << 32) else np.uint64
    c = ctx.multiply(a.astype(dt), b.astype(dt)).astype(np.uint64)
    assert np.array_equal(c[1], np.roll(a[1], -1)), (n, q)
    assert np.array_equal(c[2], np.roll(a[2], k)), (n, q, k)
    for r in (int(x) for x in rng.integers(1, n, 3)):
        y = pow(omega, r, q)
        assert _horner(c[0], y, q) == _horner(a[0], y, q) * _horner(b[0], y, q) % q, (n, q, r)


def test_time_testing_gpu_app(golden_dir, torch_cuda):
    """apps/time_testing_gpu (time_testing256.c on the C ABI) prints the reference's product of
    the reference's own coefficient files."""
    import subprocess
    exe = os.path.join(os.path.dirname(nttmul.LIB_PATH), "..", "apps", "time_testing_gpu")
    out = subprocess.run([exe, os.path.join(golden_dir, "coeficientes_a.txt"),
                          os.path.join(golden_dir, "coeficientes_b.txt"), "5", "1024"],
                         capture_output=True, text=True, timeout=120, check=True).stdout
    g = np.load(os.path.join(golden_dir, "ref256.npz"))
    vals = [int(x) for line in out.split("Resultado C = A * B):")[1].split("\n") for x in line.split()]
    assert vals == [int(v) for v in g["ntt256_product4"][0]]
    assert "Batch 1024" in out


@pytest.mark.parametrize("n,batch", [(256, 1), (256, 4), (256, 3), (512, 2), (1024, 1)])
def test_small_server_products(n, batch, torch_cuda):
    """Host calls of at most 1024 words per operand run on the resident device server
    (nttmul.cpp run_server, kernels.hip k_server: the mailbox in page-locked memory, GO / done
    sequence words): last_host_path 3, products equal the oracle's, over many back-to-back
    calls with changing inputs (every request a new sequence number); small_server = -1 takes
    the launch-per-call path (2) with the same results."""
    q = Q31
    P = O.Plan(n, q)
    srv, launch = _ctx(n, q), _ctx(n, q, small_server=-1)
    for it in range(40):
        a, b = O.fill_inputs(n, q, 100 * it, batch)
        a, b = a.astype(np.uint32), b.astype(np.uint32)
        if it == 7:
            a[0] = q - 1
        got = srv.multiply(a, b).astype(np.uint64)
        assert srv.last_host_path() == 3
        for i in range(batch):
            assert np.array_equal(got[i], P.product_merged(a[i], b[i])), (it, i)
        if it % 10 == 0:
            assert np.array_equal(launch.multiply(a, b).astype(np.uint64), got)
            assert launch.last_host_path() == 2


@pytest.mark.parametrize("cyclic", [False, True])
def test_small_server_two_wave_path(cyclic, torch_cuda):
    """Single n = 256 products take the server's two-wave path (kernels.hip server wide path:
    4 coefficients per lane, the planner's twiddles re-typed in LDS, the base multiplication's
    sign chosen per lane): random primes of every Plantard width (2n | q - 1, 14..31 bits),
    random and all-(q - 1) operands, negacyclic against the restated reference product and
    cyclic (FPGA-compat) against the schoolbook product."""
    n = 256
    for q in _random_primes([14, 17, 20, 24, 28, 30, 31], 9, seed=11 + cyclic) + [Q0, Q31, Q31HI]:
        P = O.Plan(n, q)
        ctx = _ctx(n, q, cyclic=cyclic)
        for it in range(4):
            a, b = O.fill_inputs(n, q, 7 * it + (q & 0xFF), 1)
            if it == 1:
                a[0] = q - 1
            if it == 2:
                a[0] = b[0] = q - 1
            got = ctx.multiply(a.astype(np.uint32), b.astype(np.uint32)).astype(np.uint64)
            assert ctx.last_host_path() == 3
            exp = O.cyclic_schoolbook(a[0], b[0], n, q) if cyclic else P.product_merged(a[0], b[0])
            assert np.array_equal(got[0], exp), (q, cyclic, it)


def test_small_server_two_contexts(torch_cuda):
    """Two contexts in one process each run their own resident server (two kernels polling two
    mailboxes at once): interleaved calls with different n and q stay exact, and destroying one
    context (its server stopped) leaves the other serving."""
    P1, P2 = O.Plan(256, Q0, 1002), O.Plan(512, Q31)
    c1 = _ctx(256, Q0, psi=1002)
    c2 = _ctx(512, Q31)
    for it in range(30):
        a1, b1 = O.fill_inputs(256, Q0, it, 1)
        a2, b2 = O.fill_inputs(512, Q31, 1000 + it, 2)
        g1 = c1.multiply(a1.astype(np.uint32), b1.astype(np.uint32)).astype(np.uint64)
        g2 = c2.multiply(a2.astype(np.uint32), b2.astype(np.uint32)).astype(np.uint64)
        assert c1.last_host_path() == 3 and c2.last_host_path() == 3
        assert np.array_equal(g1[0], P1.product_merged(a1[0], b1[0])), it
        for i in range(2):
            assert np.array_equal(g2[i], P2.product_merged(a2[i], b2[i])), (it, i)
    c1.close()
    for it in range(5):
        a2, b2 = O.fill_inputs(512, Q31, 2000 + it, 1)
        g2 = c2.multiply(a2.astype(np.uint32), b2.astype(np.uint32)).astype(np.uint64)
        assert c2.last_host_path() == 3
        assert np.array_equal(g2[0], P2.product_merged(a2[0], b2[0])), it


def test_small_server_answers_promptly(torch_cuda):
    """A request is answered while the server kernel keeps running, not when it leaves: 200
    back-to-back n = 256 products through the server take well under the 20 ms idle exit each
    (round 4: with plain stores to the host-coherent mailbox c stayed in the GPU's L2 until the
    kernel ended, and every call took 20 ms while staying bit-exact)."""
    import time
    n, q = 256, 12289
    ctx = _ctx(n, q, psi=1002)
    a, b = O.fill_inputs(n, q, 5, 1)
    a, b = a.astype(np.uint32), b.astype(np.uint32)
    ctx.multiply(a, b)
    ts = []
    for _ in range(200):
        t0 = time.perf_counter()
        ctx.multiply(a, b)
        ts.append(time.perf_counter() - t0)
        assert ctx.last_host_path() == 3
    ts.sort()
    assert ts[100] < 1e-3, f"median {ts[100] * 1e6:.1f} us per server call"


def test_small_server_restarts(torch_cuda):
    """The server kernel leaves after 1 ms without a request and at most 50 ms after its launch;
    the host stops and relaunches it past its own 0.5 ms / 25 ms margins.  Calls across idle gaps
    and past the lifetime stay exact; a context destroyed while its server runs stops it; the
    reference-width validation (NTTMUL_FLAG_VALIDATE) is done on the host for this path."""
    import time
    n, q = 256, 12289
    P = O.Plan(n, q, 1002)
    ctx = _ctx(n, q, psi=1002, validate=True)
    t0 = time.time()
    k = 0
    for gap in (0, 0.0003, 0.0007, 0.002, 0.0, 0.005, 0.03):
        time.sleep(gap)
        a, b = O.fill_inputs(n, q, k, 1)
        k += 1
        got = ctx.multiply(a.astype(np.uint32), b.astype(np.uint32)).astype(np.uint64)
        assert ctx.last_host_path() == 3
        assert np.array_equal(got[0], P.product_merged(a[0], b[0]))
    while time.time() - t0 < 0.2:     # past the host's 25 ms and the kernel's 50 ms lifetime
        a, b = O.fill_inputs(n, q, k, 1)
        k += 1
        got = ctx.multiply(a.astype(np.uint32), b.astype(np.uint32)).astype(np.uint64)
        assert np.array_equal(got[0], P.product_merged(a[0], b[0])), k
    bad = a.astype(np.uint32)
    bad[0, 5] = q
    with pytest.raises(nttmul.NttmulError) as ei:
        ctx.multiply(bad, b.astype(np.uint32))
    assert ei.value.status == nttmul.NTTMUL_ERANGE
    ctx.close()                       # stops the running server kernel
    ctx2 = _ctx(n, q, psi=1002)
    got = ctx2.multiply(a.astype(np.uint32), b.astype(np.uint32)).astype(np.uint64)
    assert np.array_equal(got[0], P.product_merged(a[0], b[0]))


def test_small_server_yields_to_other_work(torch_cuda):
    """Advisor r4: a resident server kernel holds its hardware queue, so work that lands in that
    queue waits until the kernel leaves.  The context stops its own server before it enqueues
    anything else, and the kernel leaves 1 ms after its last request, so (1) a device-API product
    of the same context, (2) a torch kernel and synchronize on the default stream and (3) another
    context's server call from another thread, each issued right after a server call, finish far
    below the old 20 ms idle window -- and every result stays exact.
    (2) has a control (verdict r5 item 5): the same torch kernel and synchronize with no server
    resident (the context's device-API call stops it first), interleaved with the timed ones; the
    after-server median may exceed the control median by less than 2 ms.  Round 5's one failure
    here (93.10 ms for (2), the device-API call of the same run 0.10 ms) was torch's first launch
    of its own add / sum kernels in the process -- code-object load and allocator warm-up, a
    one-time cost that the timed loop met in its first iteration -- which is why torch's kernels
    run once before anything is timed."""
    import statistics
    import threading
    import time
    torch = torch_cuda
    n, q = 256, Q31
    P = O.Plan(n, q)
    ctx = _ctx(n, q)
    a, b = O.fill_inputs(n, q, 31, 1)
    a, b = a.astype(np.uint32), b.astype(np.uint32)
    exp = P.product_merged(a[0].astype(np.uint64), b[0].astype(np.uint64))
    da = torch.from_numpy(a.view(np.int32).ravel()).cuda()
    db = torch.from_numpy(b.view(np.int32).ravel()).cuda()
    dc = torch.empty_like(da)
    s = torch.cuda.current_stream().cuda_stream
    (da + 1).sum()                      # torch's own kernels loaded before anything is timed
    ctx.multiply_device(dc, da, db, 1, 32, stream=s)
    torch.cuda.synchronize()
    worst, after, control = {}, [], []

    def torch_op():
        t0 = time.perf_counter()
        x = (da + 1).sum()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        assert int(x) == int(da.sum()) + n
        return dt
    for it in range(10):
        ctx.multiply(a, b)
        assert ctx.last_host_path() == 3
        t0 = time.perf_counter()
        ctx.multiply_device(dc, da, db, 1, 32, stream=s)   # (1) stops the server first
        torch.cuda.synchronize()
        worst["device_api"] = max(worst.get("device_api", 0), time.perf_counter() - t0)
        assert np.array_equal(dc.cpu().numpy().view(np.uint32).astype(np.uint64), exp)
        control.append(torch_op())                          # control: no server resident
        ctx.multiply(a, b)
        assert ctx.last_host_path() == 3
        after.append(torch_op())                            # (2) right after a server call
    worst["torch_sync"] = max(after)
    other = _ctx(512, q)
    a2, b2 = O.fill_inputs(512, q, 7, 1)
    P2 = O.Plan(512, q)
    res = {}

    def call():
        t0 = time.perf_counter()
        res["c"] = other.multiply(a2.astype(np.uint32), b2.astype(np.uint32))
        res["t"] = time.perf_counter() - t0
    other.multiply(a2.astype(np.uint32), b2.astype(np.uint32))   # its server launched once
    for it in range(10):
        ctx.multiply(a, b)
        th = threading.Thread(target=call)                   # (3) another context, another thread
        th.start()
        th.join()
        worst["other_context"] = max(worst.get("other_context", 0), res["t"])
        assert np.array_equal(res["c"][0].astype(np.uint64), P2.product_merged(a2[0], b2[0]))
        assert other.last_host_path() == 3
    assert ctx.server_status() == (0, "") and other.server_status() == (0, "")   # no fallback
    report = {k: f"{v * 1e3:.2f} ms" for k, v in worst.items()}
    report["torch after server / control, medians"] = (
        f"{statistics.median(after) * 1e3:.3f} / {statistics.median(control) * 1e3:.3f} ms")
    assert statistics.median(after) - statistics.median(control) < 2e-3, report
    # worst cases: below the old 20 ms idle window with room for host scheduling jitter (advisor r5)
    assert all(t < 15e-3 for t in worst.values()), report


@pytest.mark.parametrize("n,q,batch", [(4096, Q31, 1537), (256, Q30, 20000), (1024, Q62, 1100),
                                       (8192, Q31, 600), (65536, Q31, 70), (65536, Q62, 40)])
def test_host_path_pipeline(n, q, batch, torch_cuda):
    """The host-buffer ABI path streams 8 MiB chunks through 3 pipeline slots (nttmul.cpp
    run_host): several chunks, a partial last chunk and slot reuse, every product checked.  At
    n > 4096 the slots' multi-pass products run concurrently, each on its own scratch."""
    ctx = _ctx(n, q)
    a, b = O.fill_inputs(n, q, 11, batch)
    dt = np.uint32 if q < (1 << 32) else np.uint64
    c = ctx.multiply(a.astype(dt), b.astype(dt)).astype(np.uint64)
    ref = O.Plan(n, q).product_batch(a, b)[0]
    assert np.array_equal(c, ref.reshape(batch, n))
    # the standalone transforms take the same path
    fa = ctx.forward(a.astype(dt))
    assert np.array_equal(ctx.inverse(fa).astype(np.uint64), a)


@pytest.mark.parametrize("n,q,batch", [(4096, Q31, 1537), (1024, Q62, 1100), (65536, Q62, 20)])
def test_host_path_pinned_direct(n, q, batch, torch_cuda):
    """Page-locked operands (nttmul.host_empty = nttmul_host_alloc) take the direct-DMA branch of
    run_host (no staging copies; several chunks over the slots): every product equals the
    oracle's and the pageable path's; mixing pinned and pageable buffers takes the staged path."""
    ctx = _ctx(n, q)
    a, b = O.fill_inputs(n, q, 23, batch)
    dt = np.uint32 if q < (1 << 32) else np.uint64
    ap, bp, cp = (nttmul.host_empty((batch, n), dt) for _ in range(3))
    ap[...] = a
    bp[...] = b
    cp[...] = 0
    assert ctx.multiply(ap, bp, out=cp) is cp
    assert ctx.last_host_path() == 1                  # the direct-DMA branch really ran
    ref = O.Plan(n, q).product_batch(a, b)[0].reshape(batch, n)
    assert np.array_equal(cp.astype(np.uint64), ref)
    mixed = ctx.multiply(ap, b.astype(dt))            # c pageable: staged
    assert ctx.last_host_path() == 0
    assert np.array_equal(mixed.astype(np.uint64), ref)
    # operands that are views into one larger pinned block (each range inside that allocation)
    big = nttmul.host_empty((2 * batch, n), dt)
    big[:batch] = a
    big[batch:] = b
    c2 = nttmul.host_empty((batch, n), dt)
    ctx.multiply(big[:batch], big[batch:], out=c2)
    assert np.array_equal(c2.astype(np.uint64), ref) and ctx.last_host_path() == 1


def test_bench_host_io_leg(torch_cuda):
    """bench.py --host-io's leg (the PCIe-inclusive rate, never the bench value): the pageable
    call writes into the caller's reused output array, the page-locked call runs the direct-DMA
    branch, and both give the device path's products."""
    import bench
    torch = torch_cuda
    n, q, batch = 4096, Q31, 1000                       # 15.6 MiB per operand: two chunks
    ctx = _ctx(n, q)
    a = torch.empty(batch * n, dtype=torch.int32, device="cuda")
    b, c = torch.empty_like(a), torch.empty_like(a)
    s = torch.cuda.current_stream().cuda_stream
    ctx.fill_random_device(a, b, 5, batch, 32, stream=s)
    ctx.multiply_device(c, a, b, batch, 32, stream=s)
    torch.cuda.synchronize()
    line = bench.host_io(ctx, a, b, batch, n, 32, reps=2)
    assert line["value"] > 0 and line["pinned"].get("matches_pageable") is True, line
    got = ctx.multiply(a.cpu().numpy().view(np.uint32).reshape(batch, n),
                       b.cpu().numpy().view(np.uint32).reshape(batch, n))
    assert np.array_equal(got, c.cpu().numpy().view(np.uint32).reshape(batch, n))


# ---------------------------------------------------------------------------------------------
# The reference's whole transform wrapper set (NTT/ntt256.h:20-69) and its general form
# ---------------------------------------------------------------------------------------------

def test_ntt256_wrappers_golden(golden_dir, torch_cuda):
    """The twelve exported ntt256 wrappers equal the compiled reference's, in place, on the
    fixture's 32 inputs (edge rows: all q-1, all 0, unit impulse)."""
    g = np.load(os.path.join(golden_dir, "ref256_wrappers.npz"))
    for name in nttmul.NTT256_WRAPPERS:
        for x, exp in zip(g["x"], g[name]):
            a = np.ascontiguousarray(x, dtype=np.int32)
            nttmul.ntt256_transform(name, a)
            assert np.array_equal(a, exp), name


def _xf_expected(P, x, mode, cyclic, n, q):
    inv, rev = mode & nttmul.XF_INVERSE, mode & nttmul.XF_REV2STD
    if not inv:
        fn, tab = ((("ntt_ct_rev2std", "omega_powers") if rev else ("ntt_ct_std2rev", "omega_powers_rev"))
                   if cyclic else
                   (("mulntt_ct_rev2std", "mixed_powers") if rev else ("mulntt_ct_std2rev", "mixed_powers_rev")))
    else:
        fn, tab = ((("ntt_gs_rev2std", "inv_omega_powers_rev") if rev else ("ntt_gs_std2rev", "inv_omega_powers"))
                   if cyclic else
                   (("nttmul_gs_rev2std", "inv_mixed_powers_rev") if rev else ("nttmul_gs_std2rev", "inv_mixed_powers")))
    y = P.transform(fn, x, tab)
    if inv and not (mode & nttmul.XF_UNSCALED):
        inv_n = pow(n, q - 2, q)
        y = np.array([int(v) * inv_n % q for v in y], dtype=np.uint64)
    return y


@pytest.mark.parametrize("cyclic", [False, True])
@pytest.mark.parametrize("n,q", [(256, Q30), (1024, Q31), (4096, Q31), (4096, Q32), (4096, Q62),
                                 (8192, Q30), (16384, Q32), (65536, Q62)])
def test_transform_modes_vs_oracle(n, q, cyclic, torch_cuda):
    """nttmul_transform_*: every (direction, order, scaling) equals the reference's loop of the
    same name (restated in the oracle; pinned by test_oracle.py::test_wrappers_golden)."""
    P = O.Plan(n, q)
    ctx = _ctx(n, q, psi=P.omega if cyclic else 0, cyclic=cyclic)  # same omega = psi^2
    x, _ = O.fill_inputs(n, q, 21, 2)
    x[1, :] = q - 1
    dt = np.uint32 if q < (1 << 32) else np.uint64
    for mode in (0, 2, 1, 3, 1 | 4, 3 | 4):
        got = ctx.transform(x.astype(dt), mode).astype(np.uint64)
        for i in range(2):
            assert np.array_equal(got[i], _xf_expected(P, x[i], mode, cyclic, n, q)), (mode, i)


def test_transform_modes_device(torch_cuda):
    torch = torch_cuda
    n, q, batch = 4096, Q31, 1024
    ctx = _ctx(n, q)
    a = torch.empty(batch * n, dtype=torch.int32, device="cuda")
    b = torch.empty_like(a)
    s = torch.cuda.current_stream().cuda_stream
    ctx.fill_random_device(a, b, 0, batch, 32, stream=s)
    f, back = torch.empty_like(a), torch.empty_like(a)
    for fwd, inv in ((nttmul.XF_REV2STD, nttmul.XF_INVERSE | nttmul.XF_STD2REV),
                     (nttmul.XF_STD2REV, nttmul.XF_INVERSE | nttmul.XF_REV2STD)):
        ctx.transform_device(f, a, fwd, batch, 32, stream=s)
        ctx.transform_device(back, f, inv, batch, 32, stream=s)
        torch.cuda.synchronize()
        assert torch.equal(back, a)


@pytest.mark.parametrize("world,batch", [(2, 4096), (8, 1024), (8, None)])
def test_bench_ranks_on_one_gpu(world, batch, tmp_path, torch_cuda):
    """bench.py's N > 1 path as the driver launches it (torch.distributed.run, one process per
    rank, gloo control plane: barrier + all_reduce(MAX) + all_gather), with every rank on this
    box's GPU(s): 2 ranks, and the 8-rank SCALE run's control plane (--gpus 8, 1024 products per
    rank).  The JSON line reports n_gpus and the global batch, one rate per rank, the aggregate
    roofline (all ranks' bytes over the max-over-ranks wall time against N x 8 TB/s) and rank 0's
    CPU baseline with its cores (run after the final barrier at every N, verdict r4 item 2); the
    products each rank dumps from its own contiguous slice [k batch, (k + 1) batch)
    equal the oracle's at their global counter positions.  batch None: the driver's default
    arguments at 8 ranks, which run C4 (2^20 across 8, 131,072 per rank; verdict r5 item 4)."""
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    prefix = str(tmp_path / "samples")
    out = subprocess.run(
        [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
         str(world), "--master-addr", "127.0.0.1", "--master-port", str(port),
         os.path.join(root, "bench.py"), "--gpus", str(world), "--steps", "3", "--warmup", "1",
         "--settle-ms", "20", "--cpu-seconds", "0.5", "--dump-samples", prefix]
        + (["--batch-per-gpu", str(batch)] if batch else []),
        capture_output=True, text=True, timeout=300, cwd=root)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    if batch is None:  # default arguments: C4 at 8 ranks
        batch = 131072
        assert line["config"]["workload"].startswith("C4: ")
        assert line["config"]["global_batch"] == 1 << 20
        assert line["config"]["batch_rule"].startswith("default")
    else:
        assert line["config"]["batch_rule"] == "--batch-per-gpu"
    assert line["n_gpus"] == world and line["config"]["global_batch"] == world * batch
    assert line["config"]["batch_per_gpu"] == batch and line["value"] > 0
    assert line["scaling"] == "weak"
    ranks = line["ranks"]
    assert len(ranks["rates"]) == world and all(r > 0 for r in ranks["rates"])
    assert ranks["min"] == min(ranks["rates"]) and ranks["max"] == max(ranks["rates"])
    assert len(ranks["kernel_ms"]) == world
    agg = line["roofline"]["aggregate"]
    assert agg["peak"] == 8000.0 * world
    # value = global batch per max-over-ranks wall time, so the aggregate is the same quantity
    assert agg["achieved"] == pytest.approx(line["value"] * 3 * 4096 * 4 / 1e9, rel=1e-9)
    assert 0 < agg["frac"] < 1
    cpu = line["cpu_baseline"]
    assert cpu and cpu["value"] > 0 and cpu["cores"] >= 1 and cpu["kind"] == "port"
    assert cpu["host_cores"]["threads"] == cpu["cores"] and f"of {world}" in cpu["note"]
    P = O.Plan(4096, Q31)
    for r in range(world):
        d = np.load(f"{prefix}.rank{r}.npz")
        assert int(d["p0"]) == r * batch and int(d["p1"]) == (r + 1) * batch
        assert int(d["world"]) == world and int(d["global_batch"]) == world * batch
        for i, row in zip(d["idx"], d["c"]):
            ea, eb = O.fill_inputs(4096, Q31, int(d["p0"]) + int(i), 1)
            assert np.array_equal(row, P.product_merged(ea[0], eb[0])), (r, int(i))
