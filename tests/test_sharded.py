"""Multi-rank (corpus-row-sharded) path on CPU with the gloo backend,
world_size 2 and 3: partitioning, global index bases, the gather layout and
the k-way merge order.  The per-shard top-k is the CPU oracle here (test
infrastructure); on MI355X the same orchestration calls libpmm (the GPU merge
kernel is covered by tests/test_gpu_parity.py::test_device_api_sharded_merge_equals_full)."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from polars_matmul.sharded import ShardedTopK, shard_bounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _okey(v: np.ndarray) -> np.ndarray:
    """Monotone unsigned key of f32 ranking values (NaN lowest, -0 == +0)."""
    v = np.where(v == 0, np.float32(0), v).astype(np.float32)
    u = v.view(np.uint32).astype(np.uint64)
    k = np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)
    return np.where(np.isnan(v), 0, k)


def cpu_merge(gathered, k, metric, out_i, out_s):
    """Restatement of the merge kernel's semantics (best-first, ties -> lower
    index, empty slots skipped) over the gathered [world][2][M][k] layout
    (per rank an index plane and a score plane), used as the CPU stand-in."""
    g = gathered.numpy()
    li = g[:, 0].view(np.uint32)  # [world][M][k]
    ls = g[:, 1].view(np.float32)
    m = li.shape[1]
    for r in range(m):
        idx = li[:, r].reshape(-1)
        sc = ls[:, r].reshape(-1)
        keep = idx != 0xFFFFFFFF
        idx, sc = idx[keep], sc[keep]
        rank_v = -sc if metric == oracle.EUCLIDEAN else sc
        order = np.lexsort((idx, -_okey(rank_v).astype(np.float64)))[:k]
        out_i[r, : len(order)] = torch.from_numpy(idx[order].view(np.int32))
        out_s[r, : len(order)] = torch.from_numpy(sc[order])


def cpu_local_topk(q, c, k, metric, base, out_i, out_s, ws):
    idx, sc = oracle.topk(q.numpy(), c.numpy(), k, metric)
    kk = idx.shape[1]
    out_i.fill_(-1)
    out_s.fill_(float("nan"))
    out_i[:, :kk] = torch.from_numpy((idx.astype(np.int64) + base).astype(np.uint32).view(np.int32))
    out_s[:, :kk] = torch.from_numpy(sc.astype(np.float32))


def _worker(rank, world, port, q, c, k, metric, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard_bounds(c.shape[0], world, rank)
        st = ShardedTopK(torch.from_numpy(q), torch.from_numpy(c[lo:hi].copy()), lo, k, metric,
                         local_topk=cpu_local_topk, merge=cpu_merge)
        i, s = st.run()
        st.run()  # state is reusable across passes
        if rank == 0:
            np.save(os.path.join(outdir, "idx.npy"), i.numpy())
            np.save(os.path.join(outdir, "score.npy"), s.numpy())
    finally:
        dist.destroy_process_group()


def test_shard_bounds_partition():
    for n in (1, 7, 1000, 1_000_003):
        for world in (1, 2, 3, 8):
            b = [shard_bounds(n, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[r][1] == b[r + 1][0] for r in range(world - 1))
            sizes = [hi - lo for lo, hi in b]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("metric", [oracle.COSINE, oracle.EUCLIDEAN])
def test_sharded_equals_unsharded_gloo(tmp_path, world, metric):
    rs = np.random.RandomState(world * 10 + metric)
    q = rs.randn(40, 32).astype(np.float32)
    c = rs.randn(500, 32).astype(np.float32)
    c[100] = c[400]  # an exact tie across shards: lower global index must win
    k = 25
    mp.spawn(_worker, args=(world, _free_port(), q, c, k, metric, str(tmp_path)), nprocs=world, join=True)
    got_i = np.load(tmp_path / "idx.npy").view(np.uint32)
    got_s = np.load(tmp_path / "score.npy")
    want_i, want_s = oracle.topk(q, c, k, metric)
    assert np.array_equal(got_i, want_i)
    np.testing.assert_array_equal(got_s, want_s.astype(np.float32))


def test_small_shards_pad_with_empty_slots(tmp_path):
    # 3 ranks over 10 corpus rows with k = 8 > rows per shard
    rs = np.random.RandomState(1)
    q = rs.randn(5, 16).astype(np.float32)
    c = rs.randn(10, 16).astype(np.float32)
    mp.spawn(_worker, args=(3, _free_port(), q, c, 8, oracle.DOT, str(tmp_path)), nprocs=3, join=True)
    want_i, _ = oracle.topk(q, c, 8, oracle.DOT)
    assert np.array_equal(np.load(tmp_path / "idx.npy").view(np.uint32), want_i)
