"""GPU parity at the BASELINE workloads' own sizes.

configs[2] c3: 100,000 x 1,000,000 x 768 f32 cosine k=100
configs[3] c4: the same embeddings rounded to bf16 (RNE), f32 accumulation
configs[4] c5 shape: D = 1024, k = 100, the corpus row-sharded 8 ways
          (sharded.shard_bounds), per-shard top-k with index_base + the k-way
          merge, on one GPU at N = 1,048,576 corpus rows

Inputs are generated on the device exactly as bench.py does (torch.randn,
seed 42 for the queries, 1_000_003 for the corpus), so these tests check the
bench's own numbers.  Every run goes through the C ABI (pmm_topk_f32_device /
pmm_topk_bf16_device / pmm_merge_topk_device).

What is checked (the oracle is the CPU restatement, oracle/pmm_oracle.c):
  * a row sample (whole-query-block rows and split-unit rows) against
    oracle.topk over the FULL corpus: f32 bit-exact (indices identical, f32
    scores equal bit for bit); bf16 tie-aware against the float64 truth of
    the rounded rows, strict exact-match rate vs the oracle printed;
  * every row (all 100k): indices unique and in range, the list best-first
    under the documented total order (score, then lower index), each score
    equal to the oracle's exact re-score of its (row, index) pair (f32 bit for
    bit; bf16 within 1e-5, accumulation order), and nothing outside the list
    scoring better than its k-th entry by more than 1e-5 (a torch f32 GEMM of
    the whole score matrix in row chunks on the device).
"""
from __future__ import annotations

import os

import numpy as np
import pytest

import oracle
from parity import check_topk

pytestmark = pytest.mark.gpu

M, N, D, K = 100_000, 1_000_000, 768, 100
QSEED, CSEED = 42, 1_000_003
COS = 0
THREADS = min(16, os.cpu_count() or 1)


def _torch():
    import torch
    torch.backends.cuda.matmul.allow_tf32 = False
    return torch


def _gen(rows, d, seed, dev):
    from bench import synth_rows  # the bench's own generator (one seeded generator per block)

    return synth_rows(0, rows, d, seed, dev)


def _sample_rows(m, qb_rows):
    # spread over the whole range, plus both sides of the boundary between
    # whole-query-block units (rows < qb_rows) and split units
    rows = set(np.linspace(0, m - 1, 56).astype(int).tolist())
    for r in (0, 1, 255, 256, qb_rows - 1, qb_rows, qb_rows + 1, m - 1):
        if 0 <= r < m:
            rows.add(r)
    return np.array(sorted(rows), dtype=np.int64)


def _run_topk(q, c, k, metric=COS, index_base=0):
    from polars_matmul import _native
    from polars_matmul.sharded import ShardedTopK

    torch = _torch()
    compute = _native.COMPUTE_BF16 if q.dtype == torch.bfloat16 else _native.COMPUTE_F32
    ws = torch.empty(_native.workspace_bytes(q.shape[0], c.shape[0], q.shape[1], k, metric, compute),
                     dtype=torch.uint8, device=q.device)
    oi, osc = ShardedTopK(q, c, index_base, k, metric, workspace=ws).run()
    torch.cuda.synchronize()
    return oi.cpu().numpy().view(np.uint32).copy(), osc.cpu().numpy().copy()


def _check_lists(idx, sc, n, label):
    """Unique in-range indices, best-first under (score desc, index asc)."""
    assert idx.max() < n, f"{label}: index out of range"
    srt = np.sort(idx, axis=1)
    assert np.all(srt[:, 1:] != srt[:, :-1]), f"{label}: duplicate index in a row"
    assert not np.isnan(sc).any(), f"{label}: NaN score"
    a, b = sc[:, :-1], sc[:, 1:]
    ok = (a > b) | ((a == b) & (idx[:, :-1] < idx[:, 1:]))
    assert ok.all(), f"{label}: {int((~ok).sum())} adjacent pairs out of order"


def _check_nothing_better_outside(q, c, idx, sc, tol, label, chunk=2048):
    """For every row: max over corpus rows NOT returned of a torch f32 cosine
    score <= the row's k-th returned score + tol (no better row was missed)."""
    torch = _torch()
    qf, cf = q.float(), c.float()
    cinv = 1.0 / cf.norm(dim=1)
    ti = torch.from_numpy(idx.astype(np.int64)).to(q.device)
    kth = torch.from_numpy(sc[:, -1].astype(np.float32)).to(q.device)
    worst = -1.0
    for r0 in range(0, q.shape[0], chunk):
        r1 = min(r0 + chunk, q.shape[0])
        s = qf[r0:r1] @ cf.T
        s *= cinv[None, :]
        s *= (1.0 / qf[r0:r1].norm(dim=1))[:, None]
        s.scatter_(1, ti[r0:r1], float("-inf"))
        excess = (s.max(dim=1).values - kth[r0:r1]).max().item()
        worst = max(worst, excess)
        del s
    assert worst <= tol, f"{label}: a non-returned row beats the k-th by {worst:.3g}"
    return worst


@pytest.fixture(scope="module")
def c3_data():
    torch = _torch()
    dev = torch.device("cuda:0")
    q = _gen(M, D, QSEED, dev)
    c = _gen(N, D, CSEED, dev)
    yield q, c
    del q, c
    torch.cuda.empty_cache()


def test_c3_fullsize_f32_bitexact(c3_data):
    q, c = c3_data
    idx, sc = _run_topk(q, c, K)
    qh, ch = q.cpu().numpy(), c.cpu().numpy()
    # rows < 65536 run as whole query blocks (256 rows x 256 workgroups), the
    # rest as (split, block) units
    rows = _sample_rows(M, 65536)
    oi, osc = oracle.topk(qh[rows], ch, K, oracle.COSINE, nthreads=THREADS)
    rate = float(np.mean(np.all(idx[rows] == oi, axis=1)))
    print(f"c3 f32 sample of {len(rows)} rows vs oracle: strict exact-match rate {rate:.4f}")
    assert rate == 1.0
    assert np.array_equal(sc[rows], osc.astype(np.float32))
    _check_lists(idx, sc, N, "c3 f32")
    resc = oracle.pair_scores(qh, ch, idx, oracle.COSINE, nthreads=THREADS)
    assert np.array_equal(resc.view(np.uint32), sc.view(np.uint32)), \
        f"c3 f32: {int((resc != sc).sum())} of {sc.size} scores differ from the oracle re-score"
    worst = _check_nothing_better_outside(q, c, idx, sc, 1e-5, "c3 f32")
    print(f"c3 f32 all {M} rows: indices/order/scores bit-exact; best non-returned - kth <= {worst:.3g}")


def test_c4_fullsize_bf16(c3_data):
    torch = _torch()
    q32, c32 = c3_data
    qb, cb = q32.to(torch.bfloat16), c32.to(torch.bfloat16)
    idx, sc = _run_topk(qb, cb, K)
    qr, cr = qb.float(), cb.float()  # bf16 -> f32 is exact
    qh, ch = qr.cpu().numpy(), cr.cpu().numpy()
    rows = _sample_rows(M, 98304)  # 128-row blocks: 768 = 3 x 256 workgroups run whole
    # float64 truth of the sampled rows against the whole rounded corpus
    qd, cd = qr[torch.from_numpy(rows).to(qr.device)].double(), cr.double()
    truth = ((qd @ cd.T) / (qd.norm(dim=1, keepdim=True) * cd.norm(dim=1)[None, :])).cpu().numpy()
    del qd, cd
    check_topk(idx[rows], sc[rows], truth, True, rtol=1e-5, atol=1e-5, label="c4 bf16 sample")
    oi, _ = oracle.topk(qh[rows], ch, K, oracle.COSINE, nthreads=THREADS)
    rate = float(np.mean(np.all(idx[rows] == oi, axis=1)))
    elem = float(np.mean(idx[rows] == oi))
    print(f"c4 bf16 sample of {len(rows)} rows vs oracle on the rounded rows: strict row exact-match "
          f"{rate:.4f}, element match {elem:.4f}")
    # the bf16 MFMA sums in its own order: only near-ties (f32 accumulation
    # order) may swap against the oracle's chain on the rounded rows
    assert elem >= 0.995, f"c4 bf16: element match {elem:.4f} vs the oracle on the rounded rows"
    _check_lists(idx, sc, N, "c4 bf16")
    # SURVEY 8c's bf16 bar on every row: recall@100 against the f32 lists of
    # the same (unrounded) rows
    fi, _ = _run_topk(q32, c32, K)
    from bench import recall_at_k

    rec = recall_at_k(idx, fi)
    print(f"c4 bf16 recall@{K} vs the c3 f32 lists, all {M} rows: {rec:.4f}")
    assert rec >= 0.95, rec
    resc = oracle.pair_scores(qh, ch, idx, oracle.COSINE, nthreads=THREADS)
    err = float(np.max(np.abs(resc.astype(np.float64) - sc)))
    assert err <= 1e-5, f"c4 bf16: max |score - oracle re-score| {err:.3g}"
    worst = _check_nothing_better_outside(qb, cb, idx, sc, 1e-5, "c4 bf16")
    print(f"c4 bf16 all {M} rows: max |score - re-score| {err:.3g}; best non-returned - kth <= {worst:.3g}")


def test_c5_shape_sharded_1m_bitexact():
    # BASELINE configs[4] shape on one GPU: D = 1024, k = 100, 8 corpus shards
    torch = _torch()
    from polars_matmul import _native
    from polars_matmul.sharded import shard_bounds

    dev = torch.device("cuda:0")
    m, n, d, k, world = 2048, 1 << 20, 1024, 100, 8
    q = _gen(m, d, QSEED, dev)
    c = _gen(n, d, CSEED, dev)
    full_i, full_s = _run_topk(q, c, k)
    from polars_matmul.sharded import _device_merge

    # the per-rank lists as the RCCL gather lands them on rank 0 (sharded.py):
    # [world][2][m][k] = per rank an index plane and a score plane
    gathered = torch.empty((world, 2, m, k), dtype=torch.int32, device=dev)
    lists_i = torch.empty((m, world, k), dtype=torch.int32, device=dev)
    lists_s = torch.empty((m, world, k), dtype=torch.float32, device=dev)
    for r in range(world):
        a, b = shard_bounds(n, world, r)
        li, ls = _run_topk(q, c[a:b], k, index_base=a)
        gathered[r, 0] = torch.from_numpy(li.view(np.int32)).to(dev)
        gathered[r, 1] = torch.from_numpy(ls.view(np.int32)).to(dev)
        lists_i[:, r] = torch.from_numpy(li.view(np.int32)).to(dev)
        lists_s[:, r] = torch.from_numpy(ls).to(dev)
    mi = torch.empty((m, k), dtype=torch.int32, device=dev)
    ms = torch.empty((m, k), dtype=torch.float32, device=dev)
    _device_merge(gathered, k, COS, mi, ms)  # the N > 1 rank-0 merge, in place
    torch.cuda.synchronize()
    got_i, got_s = mi.cpu().numpy().view(np.uint32), ms.cpu().numpy()
    assert np.array_equal(got_i, full_i) and np.array_equal(got_s, full_s)
    # the [m][lists][k] entry point gives the same
    mi.zero_()
    _native.merge_device(lists_i.data_ptr(), lists_s.data_ptr(), m, world, k, k, COS, mi.data_ptr(),
                         ms.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(mi.cpu().numpy().view(np.uint32), full_i)
    qh, ch = q.cpu().numpy(), c.cpu().numpy()
    rows = np.linspace(0, m - 1, 24).astype(np.int64)
    oi, osc = oracle.topk(qh[rows], ch, k, oracle.COSINE, nthreads=THREADS)
    assert np.array_equal(got_i[rows], oi) and np.array_equal(got_s[rows], osc.astype(np.float32))
    _check_lists(got_i, got_s, n, "c5-shape")
    resc = oracle.pair_scores(qh, ch, got_i, oracle.COSINE, nthreads=THREADS)
    assert np.array_equal(resc.view(np.uint32), got_s.view(np.uint32))
    _check_nothing_better_outside(q, c, got_i, got_s, 1e-5, "c5-shape")


def _oracle_topk_chunked(qh, c_dev, k, chunk=1 << 21):
    """oracle.topk of a few query rows against a corpus too large to copy to
    the host at once: the oracle over each corpus chunk (global indices), then
    the best k of the chunk lists under the same total order (score desc, then
    lower index) -- the oracle's result over the whole corpus, since each
    chunk's list holds that chunk's top k."""
    n = c_dev.shape[0]
    idx, sc = [], []
    for lo in range(0, n, chunk):
        ch = c_dev[lo:lo + chunk].cpu().numpy()
        oi, osc = oracle.topk(qh, ch, k, oracle.COSINE, nthreads=THREADS)
        idx.append(oi.astype(np.int64) + lo)
        sc.append(osc)
        del ch
    idx, sc = np.concatenate(idx, axis=1), np.concatenate(sc, axis=1)
    order = np.lexsort((idx, -sc), axis=1)[:, :k]  # score desc, then index asc
    return (np.take_along_axis(idx, order, axis=1).astype(np.uint32),
            np.take_along_axis(sc, order, axis=1))


def _pair_scores_chunked(qh, c_dev, idx):
    """oracle.pair_scores over a device corpus, gathering only the corpus rows
    the lists name (the full corpus need not cross to the host)."""
    torch = _torch()
    uniq, inv = np.unique(idx, return_inverse=True)
    rows = c_dev[torch.from_numpy(uniq.astype(np.int64)).to(c_dev.device)].cpu().numpy()
    return oracle.pair_scores(qh, rows, inv.reshape(idx.shape).astype(np.uint32), oracle.COSINE,
                              nthreads=THREADS)


def test_c5_full_corpus_10m_sharded_8way_bitexact():
    # BASELINE configs[4] at its corpus size on one GPU: the full 10,000,000 x
    # 1024 f32 corpus (41 GB, bench.synth_rows: the bench's own rows), 4096
    # queries.  The 8 shard_bounds shards run through the per-rank path
    # (fused top-k with index_base) and the rank-0 merge (_device_merge on the
    # [world][2][m][k] gather layout); that equals the unsharded run bit for
    # bit, a 24-row sample equals oracle.topk over the whole 10M corpus, and
    # every returned pair equals its oracle re-score.
    torch = _torch()
    from polars_matmul.sharded import _device_merge, shard_bounds

    dev = torch.device("cuda:0")
    m, n, d, k, world = 4096, 10_000_000, 1024, 100, 8
    q = _gen(m, d, QSEED, dev)
    c = _gen(n, d, CSEED, dev)
    full_i, full_s = _run_topk(q, c, k)
    gathered = torch.empty((world, 2, m, k), dtype=torch.int32, device=dev)
    for r in range(world):
        a, b = shard_bounds(n, world, r)
        li, ls = _run_topk(q, c[a:b], k, index_base=a)
        gathered[r, 0] = torch.from_numpy(li.view(np.int32)).to(dev)
        gathered[r, 1] = torch.from_numpy(ls.view(np.int32)).to(dev)
    mi = torch.empty((m, k), dtype=torch.int32, device=dev)
    ms = torch.empty((m, k), dtype=torch.float32, device=dev)
    _device_merge(gathered, k, COS, mi, ms)
    torch.cuda.synchronize()
    got_i, got_s = mi.cpu().numpy().view(np.uint32), ms.cpu().numpy()
    assert np.array_equal(got_i, full_i) and np.array_equal(got_s.view(np.uint32), full_s.view(np.uint32))
    _check_lists(got_i, got_s, n, "c5 10M")
    qh = q.cpu().numpy()
    rows = np.linspace(0, m - 1, 24).astype(np.int64)
    oi, osc = _oracle_topk_chunked(qh[rows], c, k)
    assert np.array_equal(got_i[rows], oi)
    assert np.array_equal(got_s[rows], osc.astype(np.float32))
    resc = _pair_scores_chunked(qh, c, got_i)
    assert np.array_equal(resc.view(np.uint32), got_s.view(np.uint32)), \
        f"c5 10M: {int((resc != got_s).sum())} scores differ from the oracle re-score"
    worst = _check_nothing_better_outside(q, c, got_i, got_s, 1e-5, "c5 10M", chunk=256)
    print(f"c5 {m}x{n}x{d}: 8 shards + merge == unsharded; 24 rows == oracle over 10M; "
          f"all {m * k} pairs == oracle re-score; best non-returned - kth <= {worst:.3g}")
    del q, c, gathered
    torch.cuda.empty_cache()


def test_c5_per_rank_shape_one_launch():
    # One launch of the per-GPU share of BASELINE configs[4] on 8 GPUs: all
    # 1,000,000 queries against one 1,250,000-row shard (rows [0, 1.25M) of
    # the bench corpus), D = 1024, k = 100 -- 2.56 PFLOP, ~18 s.  Every row:
    # list properties and every returned pair equal to its oracle re-score; a
    # 32-row sample equal to oracle.topk; no better row missed on a 65,536-row
    # sample (torch f32 GEMM).  Prints the kernel time and MFMA fraction.
    torch = _torch()
    from polars_matmul import _native

    dev = torch.device("cuda:0")
    m, n, d, k = 1_000_000, 1_250_000, 1024, 100
    q = _gen(m, d, QSEED, dev)
    c = _gen(n, d, CSEED, dev)
    _native.timing_reset()
    _native.timing_enable(True)
    idx, sc = _run_topk(q, c, k)
    _native.timing_enable(False)
    ms, launches = _native.timing_read("gemm_f32_topk")
    tflops = 2.0 * m * n * d / (ms / 1000.0) / 1e12
    print(f"c5 per-rank shape {m}x{n}x{d}: fused kernel {ms:.1f} ms ({launches} launch), "
          f"{tflops:.1f} TFLOP/s = {tflops / 157.3:.3f} of the f32 MFMA peak")
    _check_lists(idx, sc, n, "c5 per-rank")
    qh, ch = q.cpu().numpy(), c.cpu().numpy()
    resc = oracle.pair_scores(qh, ch, idx, oracle.COSINE, nthreads=THREADS)
    assert np.array_equal(resc.view(np.uint32), sc.view(np.uint32)), \
        f"c5 per-rank: {int((resc != sc).sum())} of {sc.size} scores differ from the oracle re-score"
    rows = np.linspace(0, m - 1, 32).astype(np.int64)
    oi, osc = oracle.topk(qh[rows], ch, k, oracle.COSINE, nthreads=THREADS)
    assert np.array_equal(idx[rows], oi) and np.array_equal(sc[rows], osc.astype(np.float32))
    del qh, ch
    sub = torch.arange(0, m, m // 65536, device=dev)[:65536]
    worst = _check_nothing_better_outside(q[sub], c, idx[sub.cpu().numpy()], sc[sub.cpu().numpy()], 1e-5,
                                          "c5 per-rank")
    print(f"c5 per-rank: all {m} rows re-scored bit-exact; best non-returned - kth <= {worst:.3g}")
    del q, c
    torch.cuda.empty_cache()
