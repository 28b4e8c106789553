"""Multi-process (gloo, world size 2) coverage of the N>1 bench path on CPU: contiguous batch
shards that cover the global batch exactly once, the contract's barrier/sync timing harness and the
max-over-ranks reduction.  The per-rank work is the oracle's CPU product on that rank's slice (the
GPU kernel is covered by tests/test_gpu_parity.py); results are checked against a one-process run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from oracle import oracle as O

N, Q, GLOBAL = 256, 2013265921, 12


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p0, p1 = bench.shard(GLOBAL, rank, world)
    a, b = O.fill_inputs(N, Q, p0, p1 - p0)          # counter-based: any rank regenerates any slice
    plan = O.Plan(N, Q)
    out = {}

    def step():
        out["c"], _ = plan.fast_batch_u32(a.astype(np.uint32), b.astype(np.uint32), threads=1)

    wall = bench.timed_steps(step, steps=3, warmup=1, sync=lambda: None, barrier=dist.barrier)
    wmax = bench.max_over_ranks(wall + rank, dist, torch.device("cpu"))   # rank 1 is "slowest"
    # per-rank rows for the bench line's per-rank rates and aggregate roofline
    rows = bench.gather_ranks([wall + rank, 0.5 + rank, float(p1 - p0)], dist)
    np.save(os.path.join(outdir, f"c{rank}.npy"), out["c"])
    np.save(os.path.join(outdir, f"t{rank}.npy"), np.array([p0, p1, wall, wmax]))
    np.save(os.path.join(outdir, f"r{rank}.npy"), np.array(rows))
    dist.destroy_process_group()


def test_shards_cover_batch():
    for g, w in ((12, 2), (65536, 8), (7, 3), (1 << 20, 8)):
        edges = [bench.shard(g, r, w) for r in range(w)]
        assert edges[0][0] == 0 and edges[-1][1] == g
        assert all(edges[r][1] == edges[r + 1][0] for r in range(w - 1))


def test_two_rank_gloo(tmp_path):
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, str(tmp_path)), nprocs=2, start_method="spawn")
    c = np.concatenate([np.load(tmp_path / f"c{r}.npy") for r in range(2)])
    a, b = O.fill_inputs(N, Q, 0, GLOBAL)
    plan = O.Plan(N, Q)
    ref, _ = plan.fast_batch_u32(a.astype(np.uint32), b.astype(np.uint32), threads=1)
    assert np.array_equal(c, ref)
    t = [np.load(tmp_path / f"t{r}.npy") for r in range(2)]
    assert t[0][1] == t[1][0] == GLOBAL // 2
    # both ranks see the same max, and it is at least rank 1's own (wall + 1)
    assert t[0][3] == t[1][3] >= t[1][2] + 1
    # every rank gathered every rank's row, in rank order
    rows = [np.load(tmp_path / f"r{r}.npy") for r in range(2)]
    assert np.array_equal(rows[0], rows[1]) and rows[0].shape == (2, 3)
    assert rows[0][1][0] == t[1][2] + 1 and rows[0][1][1] == 1.5
    agg, per = bench.rank_summary(rows[0].tolist(), 3, 3 * N * 4, 2, float(t[0][3]))
    assert per["rates"][1] == pytest.approx(GLOBAL // 2 * 3 / (t[1][2] + 1))
    assert per["min"] == min(per["rates"]) and per["max"] == max(per["rates"])
    assert per["kernel_ms"] == [0.5, 1.5]
    # the aggregate: all ranks' bytes over the slowest rank's wall time, against 2 x 8 TB/s
    assert agg["peak"] == 16000.0
    assert agg["achieved"] == pytest.approx(GLOBAL * 3 * N * 4 * 3 / t[0][3] / 1e9)
    assert agg["frac"] == pytest.approx(agg["achieved"] / 16000.0)
