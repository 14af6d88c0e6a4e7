"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
NumPy float64 truth, on the reference's KATs, seeded fixtures and edge cases.

Parity bar:
  f32 path vs the oracle: BIT-EXACT.  The f32 MFMA kernel feeds K in natural
          order (each output is the oracle's k-ordered fmaf chain), the norms
          follow the same ndarray order and the epilogue the same operation
          order, so indices are identical (exact-match rate == 1.0) and scores
          equal bit for bit, on every fixture and at BASELINE configs[0/1].
  vs the float64 truth (and for bf16 / the f64 path): |s - truth| <=
          1e-5*|truth| + 1e-5 (+ 2e-6*|q||c| for raw f32 dot products, whose
          absolute error scales with the operand norms); indices tie-aware
          (tests/parity.py).
"""
from __future__ import annotations

import json
import os
import threading

import numpy as np
import pyarrow as pa
import pytest

import oracle
from parity import check_matrix, check_topk, dot_scale, exact_match_rate

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
METRICS = {"cosine": 0, "dot": 1, "euclidean": 2}


@pytest.fixture(scope="module")
def pmm():
    import polars_matmul
    from polars_matmul import _native

    assert _native.device_count() > 0, "no HIP device visible"
    return polars_matmul


def _native():
    from polars_matmul import _native as n
    return n


def gpu_topk(q, c, k, metric):
    n = _native()
    kk = min(k, c.shape[0])
    return n.topk_host(np.ascontiguousarray(q), np.ascontiguousarray(c), kk, METRICS[metric])


def assert_bitexact(idx, sc, oi, osc, label=""):
    """Device f32 top-k == oracle top-k: same indices, same f32 scores bit for
    bit (the oracle widens its f32 scores to f64 exactly, matmul.rs:447)."""
    assert idx.shape == oi.shape, (label, idx.shape, oi.shape)
    rate = exact_match_rate(idx, oi)
    assert rate == 1.0, f"{label}: exact index match {rate:.4f}"
    got = np.asarray(sc, dtype=np.float32)
    want = np.asarray(osc).astype(np.float32)
    assert np.array_equal(np.asarray(osc, np.float64), want.astype(np.float64), equal_nan=True), label
    same = (got.view(np.uint32) == want.view(np.uint32)) | (np.isnan(got) & np.isnan(want))
    assert same.all(), f"{label}: {int((~same).sum())} scores differ, e.g. {got[~same][:3]} vs {want[~same][:3]}"


def kats(op):
    with open(os.path.join(GOLD, "kat.json")) as f:
        return [c for c in json.load(f)["cases"] if c["op"] == op]


def _arrow(rows, dtype):
    t = pa.float32() if dtype == "f32" else pa.float64()
    return pa.array(rows, type=pa.list_(t))


@pytest.mark.parametrize("case", kats("topk"), ids=lambda c: c["name"])
def test_kat_topk_through_extension(pmm, case):
    from polars_matmul._polars_matmul import _topk

    out = _topk(_arrow(case["q"], case["dtype"]), _arrow(case["c"], case["dtype"]), case["k"], case["metric"])
    assert out.type == pa.large_list(pa.struct([("index", pa.uint32()), ("score", pa.float64())]))
    rows = out.to_pylist()
    if "expect_len" in case:
        assert [len(r) for r in rows] == case["expect_len"]
    tol = case.get("tol", 1e-6)
    for i, (ei, es) in enumerate(case.get("expect_top", [])):
        assert rows[i][0]["index"] == ei
        assert abs(rows[i][0]["score"] - es) < tol
    for i, exp in enumerate(case.get("expect_rows", [])):
        for j, (ei, es) in enumerate(exp):
            assert rows[i][j]["index"] == ei, (case["name"], rows[i])
            assert abs(rows[i][j]["score"] - es) < tol


@pytest.mark.parametrize("case", kats("topk"), ids=lambda c: c["name"])
def test_kat_topk_f32_path(pmm, case):
    # the same KATs on the fused f32 kernel (the reference's f32 branch)
    q = np.array(case["q"], dtype=np.float32)
    c = np.array(case["c"], dtype=np.float32)
    idx, sc = gpu_topk(q, c, case["k"], case["metric"])
    oi, os_ = oracle.topk(q, c, case["k"], oracle.metric_from_str(case["metric"]))
    assert_bitexact(idx, sc, oi, os_, case["name"])


@pytest.mark.parametrize("case", kats("matmul"), ids=lambda c: c["name"])
def test_kat_matmul_through_extension(pmm, case):
    from polars_matmul._polars_matmul import _matmul

    out = _matmul(_arrow(case["q"], case["dtype"]), _arrow(case["c"], case["dtype"]))
    inner = pa.float32() if case["dtype"] == "f32" else pa.float64()
    assert out.type == pa.list_(inner, len(case["c"]))
    got = np.array(out.to_pylist())
    check_matrix(got, case["expect"], rtol=case["rtol"], atol=0)
    if "expect_flat" in case:
        np.testing.assert_allclose(got.reshape(-1), case["expect_flat"], rtol=case["rtol"])


def test_mixed_f32_f64_uses_f64(pmm):
    # tests/test_polars_matmul.py:434-447
    from polars_matmul._polars_matmul import _matmul

    out = _matmul(_arrow([[1.0, 2.0]], "f32"), _arrow([[1.0, 0.0]], "f64"))
    assert out.type == pa.list_(pa.float64(), 1)


def test_ref_cosine_all_k_f64(pmm):
    # tests/test_polars_matmul.py:264-296 (f64 inputs -> f64 GPU path)
    z = np.load(os.path.join(GOLD, "rand_ref_cosine_5x20x16.npz"))
    idx, sc = gpu_topk(z["q"], z["c"], 20, "cosine")
    for i in range(5):
        np.testing.assert_allclose(sc[i], np.sort(z["cosine"][i])[::-1], rtol=1e-5)
    check_topk(idx, sc, z["cosine"], True, label="ref cosine f64")
    oi, _ = oracle.topk(z["q"], z["c"], 20, oracle.COSINE)
    assert exact_match_rate(idx, oi) == 1.0


def test_ref_matmul_f64_and_f32(pmm):
    z = np.load(os.path.join(GOLD, "rand_ref_matmul_10x20x32.npz"))
    check_matrix(pmm.matmul(z["q"], z["c"]), z["dot"], rtol=1e-5, atol=1e-12)
    got32 = pmm.matmul(z["q"].astype(np.float32), z["c"].astype(np.float32))
    assert got32.dtype == np.float32
    check_matrix(got32, oracle.matmul(z["q"].astype(np.float32), z["c"].astype(np.float32)), rtol=1e-5, atol=1e-5)


def test_bench_verify_f64(pmm):
    # examples/benchmark_topk.py:191-203
    z = np.load(os.path.join(GOLD, "rand_bench_verify_100x500x64.npz"))
    idx, sc = gpu_topk(z["q"], z["c"], 10, "cosine")
    np.testing.assert_allclose(sc, -np.sort(-z["cosine"], axis=1)[:, :10], rtol=1e-4)
    check_topk(idx, sc, z["cosine"], True, label="bench verify")


@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
@pytest.mark.parametrize("k", [1, 10, 100, 1000])
def test_f32_fixture_vs_oracle(pmm, metric, k):
    z = np.load(os.path.join(GOLD, "rand_f32_48x1000x256.npz"))
    idx, sc = gpu_topk(z["q"], z["c"], k, metric)
    scale = dot_scale(z["q"], z["c"]) if metric == "dot" else None
    check_topk(idx, sc, z[metric], metric != "euclidean", rtol=1e-5, atol=1e-5, scale=scale,
               label=f"gpu f32 {metric} k={k}")
    oi, osc = oracle.topk(z["q"], z["c"], k, METRICS[metric])
    assert_bitexact(idx, sc, oi, osc, f"f32 fixture {metric} k={k}")


@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
def test_f64_fixture_vs_oracle(pmm, metric):
    z = np.load(os.path.join(GOLD, "rand_f32_48x1000x256.npz"))
    q, c = z["q"].astype(np.float64), z["c"].astype(np.float64)
    idx, sc = gpu_topk(q, c, 50, metric)
    assert sc.dtype == np.float64
    check_topk(idx, sc, z[metric], metric != "euclidean", rtol=1e-9, atol=1e-9, label=f"gpu f64 {metric}")
    oi, _ = oracle.topk(q, c, 50, METRICS[metric])
    assert exact_match_rate(idx, oi) == 1.0


# ---- the fused f64 path (pmm_f64.hip): chunked scan
# with a running per-row k-th, against the oracle (src/metrics.rs:258-311 +
# src/topk.rs:6-39 restated) and the materialised path (PMM_F64_FUSED=0) ----
@pytest.mark.parametrize("m,n,d,k", [(48, 1000, 256, 50), (33, 30011, 37, 10), (7, 9000, 100, 1),
                                     (64, 20000, 64, 100), (5, 3000, 16, 1000), (130, 700, 200, 700)])
@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
@pytest.mark.parametrize("tile", ["64", "128"])
def test_f64_fused_vs_oracle_and_materialised(pmm, m, n, d, k, metric, tile, monkeypatch):
    # tile: the fused kernel's workgroup tile (PMM_F64_TILE: 64 x 64 by
    # default, 128 x 128 forced) -- K order is the same, so the same bits
    monkeypatch.setenv("PMM_F64_TILE", tile)
    rs = np.random.RandomState(m * 7 + n + d + k)
    q = rs.randn(m, d)
    c = rs.randn(n, d)
    c[n - 30:] = c[:30]  # exact ties across chunk boundaries
    c[n // 2] = 0.0      # a zero-norm corpus row
    q[0] = c[5]          # a query equal to a corpus row
    q[-1] = 0.0 if m > 1 else q[-1]  # a zero-norm query row (every cosine score 0)
    monkeypatch.setenv("PMM_F64_FUSED", "1")  # (by size these shapes take the materialised path)
    idx, sc = gpu_topk(q, c, k, metric)
    assert sc.dtype == np.float64 and idx.shape == (m, min(k, n))
    oi, osc = oracle.topk(q, c, k, METRICS[metric])
    assert exact_match_rate(idx, oi) == 1.0, f"f64 fused vs oracle {metric}"
    np.testing.assert_allclose(sc, osc, rtol=1e-12, atol=1e-12)
    # the materialised path scores with the same GEMM tile (pmm_f64.hip
    # f64_tile) and the same epilogue: the same lists bit for bit
    monkeypatch.setenv("PMM_F64_FUSED", "0")
    mi, ms = gpu_topk(q, c, k, metric)
    assert np.array_equal(mi, idx)
    assert np.array_equal(ms.view(np.uint64), sc.view(np.uint64))


@pytest.mark.parametrize("fused", ["1", "0"])
def test_f64_fused_scores_bitwise_vs_oracle(pmm, fused, monkeypatch):
    # v_mfma_f64_16x16x4_f64 fed K in natural order (lane kq holds k0 + 4s + kq
    # at step s): if the instruction accumulates its four products as a
    # k-ordered fma chain, every score equals the oracle's bit for bit (fused
    # scan and materialised scores alike)
    monkeypatch.setenv("PMM_F64_FUSED", fused)
    rs = np.random.RandomState(77)
    q, c = rs.randn(40, 256), rs.randn(5000, 256)
    for metric in ("dot", "cosine", "euclidean"):
        idx, sc = gpu_topk(q, c, 20, metric)
        oi, osc = oracle.topk(q, c, 20, METRICS[metric])
        assert np.array_equal(idx, oi)
        assert np.array_equal(sc.view(np.uint64), osc.view(np.uint64)), metric


@pytest.mark.parametrize("k", [5, 40, 120, 700, 1500])
def test_f64_cosine_division_skip_at_threshold_edges(pmm, k, monkeypatch):
    # the fused f64 kernel drops cosine elements whose dot is below the row's
    # threshold bound without dividing (pmm_f64.hip): thresholds here land on
    # positive scores, on exact zeros (orthogonal rows, zero-norm rows: no
    # bound), on negative scores, and on runs of exact ties -- the lists must
    # equal the oracle's and the materialised path's bit for bit
    monkeypatch.setenv("PMM_F64_FUSED", "1")
    rs = np.random.RandomState(k)
    n, d = 3000, 8
    q = np.zeros((6, d))
    q[:, 0] = 1.0
    q[3] = rs.randn(d)
    q[5] = 0.0                                  # a zero-norm query row
    c = rs.randn(n, d)
    c[:100, 0] = np.abs(c[:100, 0]) + 0.5       # 100 positive scores for the e1 queries
    c[100:1100, 0] = 0.0                        # 1000 exact zeros (orthogonal)
    c[1100:1600] = c[1100]                      # 500 exact ties
    c[1600:1700] = 0.0                          # zero-norm corpus rows (score 0 by rule)
    c[1700:, 0] = -np.abs(c[1700:, 0]) - 0.1    # negative scores
    idx, sc = gpu_topk(q, c, k, "cosine")
    oi, osc = oracle.topk(q, c, k, METRICS["cosine"])
    assert np.array_equal(idx, oi), f"k={k}"
    assert np.array_equal(sc.view(np.uint64), osc.view(np.uint64)), f"k={k}"
    monkeypatch.setenv("PMM_F64_FUSED", "0")
    mi, ms = gpu_topk(q, c, k, "cosine")
    assert np.array_equal(mi, idx) and np.array_equal(ms.view(np.uint64), sc.view(np.uint64))


def test_f64_cosine_division_skip_tiny_scores(pmm, monkeypatch):
    # cosine scores around 1e-300 (products near the subnormal
    # range, where the skip's rounding margin would not hold) and thresholds
    # on exact ties among them: the skip must stand aside there -- fused ==
    # oracle == materialised, bit for bit
    monkeypatch.setenv("PMM_F64_FUSED", "1")
    rs = np.random.RandomState(3)
    n, d, k = 4000, 4, 50
    q = np.zeros((4, d))
    q[:, 0] = 1.0
    q[:, 1] = [1e-300, 3e-301, 1e-305, 2.5e-290]
    c = np.zeros((n, d))
    c[:, 1] = rs.randint(-40, 41, size=n) * 1.0   # many exact ties
    c[:, 2] = 1.0                                  # corpus norms ~ |c[:, 1]|
    c[::7, 1] = rs.randn(len(c[::7])) * 1e-3
    idx, sc = gpu_topk(q, c, k, "cosine")
    oi, osc = oracle.topk(q, c, k, METRICS["cosine"])
    assert np.array_equal(idx, oi)
    assert np.array_equal(sc.view(np.uint64), osc.view(np.uint64))
    assert np.all(np.abs(sc[np.isfinite(sc)]) < 1e-280)
    monkeypatch.setenv("PMM_F64_FUSED", "0")
    mi, ms = gpu_topk(q, c, k, "cosine")
    assert np.array_equal(mi, idx) and np.array_equal(ms.view(np.uint64), sc.view(np.uint64))


def test_f64_fused_overflow_falls_back(pmm, monkeypatch):
    # adversarial order: every corpus row beats every earlier one, so each
    # chunk's survivors overflow the buffers; the call must still be exact
    # (materialised fallback)
    monkeypatch.setenv("PMM_F64_FUSED", "1")
    n, d = 20000, 16
    q = np.ones((4, d))
    c = np.repeat(np.arange(n, dtype=np.float64)[:, None], d, axis=1) / n
    idx, sc = gpu_topk(q, c, 10, "dot")
    assert idx.tolist() == [list(range(n - 1, n - 11, -1))] * 4
    oi, osc = oracle.topk(q, c, 10, METRICS["dot"])
    assert np.array_equal(idx, oi) and np.array_equal(sc, osc)


@pytest.mark.parametrize("fused", ["1", "1-128", "0"])
def test_f64_nan_rows_and_k_equals_n(pmm, fused, monkeypatch):
    if fused == "1-128":
        fused = "1"
        monkeypatch.setenv("PMM_F64_TILE", "128")
    monkeypatch.setenv("PMM_F64_FUSED", fused)
    rs = np.random.RandomState(5)
    q, c = rs.randn(9, 24), rs.randn(1500, 24)
    c[[3, 700, 1499]] = np.nan
    for metric in ("cosine", "dot", "euclidean"):
        for k in (10, 1500):
            idx, sc = gpu_topk(q, c, k, metric)
            oi, osc = oracle.topk(q, c, k, METRICS[metric])
            assert exact_match_rate(idx, oi) == 1.0, (metric, k)
            np.testing.assert_allclose(sc, osc, rtol=1e-12, atol=1e-12, equal_nan=True)


@pytest.mark.parametrize("k", [1, 10, 100])
def test_f64_fused_long_corpus_stays_fused(pmm, k, monkeypatch):
    # Random rows over a long corpus: the chunk schedule is sized for the
    # tail of the per-row survivor count (pmm_capi.hip, topk_f64_device_impl),
    # so no row's buffer overflows and the call never falls back to the
    # materialised path (whose score launches would show in the timers).
    # With the growth sized for the mean, k = 1 overflowed ~13% of the rows.
    n = _native()
    rs = np.random.RandomState(900 + k)
    q, c = rs.randn(256, 32), rs.randn(300_000, 32)
    monkeypatch.setenv("PMM_F64_FUSED", "1")
    n.timing_reset()
    n.timing_enable(True)
    try:
        idx, sc = gpu_topk(q, c, k, "cosine")
    finally:
        n.timing_enable(False)
    assert n.timing_read("gemm_f64_topk")[1] >= 2
    assert n.timing_read("gemm_f64_scores")[1] == 0, "the fused scan overflowed and fell back"
    oi, osc = oracle.topk(q[:16], c, k, METRICS["cosine"])
    assert np.array_equal(idx[:16], oi)
    assert np.array_equal(sc[:16].view(np.uint64), osc.view(np.uint64))


def test_f64_device_api_equals_host(pmm):
    import torch

    n = _native()
    rs = np.random.RandomState(8)
    q, c = rs.randn(100, 70), rs.randn(8000, 70)
    want = n.topk_host(q, c, 25, METRICS["cosine"])
    dev = torch.device("cuda", 0)
    ld = 80  # >= roundup(70, 16), zero-padded
    qd = torch.zeros((100, ld), dtype=torch.float64, device=dev)
    cd = torch.zeros((8000, ld), dtype=torch.float64, device=dev)
    qd[:, :70] = torch.from_numpy(q).to(dev)
    cd[:, :70] = torch.from_numpy(c).to(dev)
    oi = torch.empty((100, 25), dtype=torch.int32, device=dev)
    os_ = torch.empty((100, 25), dtype=torch.float64, device=dev)
    n.topk_f64_device(qd.data_ptr(), ld, 100, cd.data_ptr(), ld, 8000, 70, 25, METRICS["cosine"], oi.data_ptr(),
                      os_.data_ptr(), index_base=1000, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(oi.cpu().numpy().view(np.uint32) - 1000, want[0])
    assert np.array_equal(os_.cpu().numpy(), want[1])


@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
def test_edge_fixture_exact(pmm, metric):
    # zero-norm rows, exact duplicate corpus rows (ties), d=37 (padded to 64)
    z = np.load(os.path.join(GOLD, "edge_f32_6x70x37.npz"))
    idx, sc = gpu_topk(z["q"], z["c"], 70, metric)
    oi, osc = oracle.topk(z["q"], z["c"], 70, METRICS[metric])
    scale = dot_scale(z["q"], z["c"]) if metric == "dot" else None
    check_topk(idx, sc, z[metric], metric != "euclidean", rtol=1e-5, atol=1e-5, scale=scale, label=f"edge {metric}")
    assert_bitexact(idx, sc, oi, osc, f"edge {metric}")
    for i in range(6):
        row = idx[i].tolist()
        assert row.index(3) < row.index(11) < row.index(40)  # equal scores -> lower index first
    if metric == "cosine":
        assert np.all(sc[2] == 0.0) and idx[2].tolist() == list(range(70))
        for i in range(6):
            assert sc[i, idx[i].tolist().index(5)] == 0.0


@pytest.mark.parametrize("m,n,d,k", [
    (1, 1, 1, 1), (3, 5, 2, 5), (130, 257, 33, 7), (129, 1000, 64, 100), (7, 300, 1024, 16),
    (257, 4099, 96, 64), (64, 2000, 32, 1024),
])
@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
def test_ragged_shapes(pmm, m, n, d, k, metric):
    rs = np.random.RandomState(m * 7 + n + d)
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(n, d).astype(np.float32)
    idx, sc = gpu_topk(q, c, k, metric)
    from golden.make_golden import truth_scores
    truth = truth_scores(q, c, metric)
    scale = dot_scale(q, c) if metric == "dot" else None
    check_topk(idx, sc, truth, metric != "euclidean", rtol=1e-5, atol=1e-5, scale=scale,
               label=f"{m}x{n}x{d} k={k} {metric}")
    oi, osc = oracle.topk(q, c, k, METRICS[metric])
    assert_bitexact(idx, sc, oi, osc, f"{m}x{n}x{d} k={k} {metric}")


def test_large_k_materialised_path(pmm):
    # k > 1024 goes through the materialise + row-select kernels
    rs = np.random.RandomState(11)
    q = rs.randn(20, 48).astype(np.float32)
    c = rs.randn(3000, 48).astype(np.float32)
    for k in (1500, 3000):
        idx, sc = gpu_topk(q, c, k, "cosine")
        oi, osc = oracle.topk(q, c, k, oracle.COSINE)
        from golden.make_golden import truth_scores
        check_topk(idx, sc, truth_scores(q, c, "cosine"), True, rtol=1e-5, atol=1e-5, label=f"k={k}")
        assert_bitexact(idx, sc, oi, osc, f"materialised k={k}")


def test_k_zero_returns_empty_lists(pmm):
    from polars_matmul._polars_matmul import _topk
    out = _topk(_arrow([[1.0, 0.0], [0.0, 1.0]], "f32"), _arrow([[1.0, 0.0]], "f32"), 0, "cosine")
    assert [len(r) for r in out.to_pylist()] == [0, 0]


def test_nan_query_row_ranks_by_index(pmm):
    q = np.array([[np.nan, 1.0], [1.0, 0.0]], dtype=np.float32)
    c = np.array([[1.0, 0.0], [0.0, 1.0], [2.0, 0.0]], dtype=np.float32)
    idx, sc = gpu_topk(q, c, 3, "dot")
    assert idx[0].tolist() == [0, 1, 2] and np.all(np.isnan(sc[0]))
    assert idx[1].tolist() == [2, 0, 1]


def test_config2_dot_k10_vs_oracle(pmm):
    # BASELINE configs[1]: 1000 x 10000 x 256 f32 dot k=10, inputs as
    # examples/benchmark_topk.py:69-71 (seed 42, randn -> f32)
    np.random.seed(42)
    q = np.random.randn(1000, 256).astype(np.float32)
    c = np.random.randn(10000, 256).astype(np.float32)
    idx, sc = gpu_topk(q, c, 10, "dot")
    oi, osc = oracle.topk(q, c, 10, oracle.DOT)
    truth = q.astype(np.float64) @ c.astype(np.float64).T
    check_topk(idx, sc, truth, True, rtol=1e-5, atol=1e-5, scale=dot_scale(q, c), label="config2")
    assert_bitexact(idx, sc, oi, osc, "config2")


def test_config1_cosine_k10_vs_oracle(pmm):
    # BASELINE configs[0] workload (the reference's benchmark), on the GPU
    np.random.seed(42)
    q = np.random.randn(1000, 256).astype(np.float32)
    c = np.random.randn(10000, 256).astype(np.float32)
    idx, sc = gpu_topk(q, c, 10, "cosine")
    oi, osc = oracle.topk(q, c, 10, oracle.COSINE)
    assert_bitexact(idx, sc, oi, osc, "config1")


@pytest.mark.parametrize("m,n,d", [(1, 1, 1), (67, 301, 37), (256, 512, 256), (130, 700, 768), (40, 333, 1024)])
def test_matmul_f32_bitwise_vs_oracle(pmm, m, n, d):
    # the GEMM alone (.pmm.matmul, store mode of the same MFMA main loop):
    # natural K order -> every element is the oracle's fmaf chain bit for bit
    rs = np.random.RandomState(m + n + d)
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(n, d).astype(np.float32)
    got = _native().matmul_host(q, c)
    want = oracle.matmul(q, c)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), \
        f"{int((got != want).sum())} of {got.size} elements differ"


@pytest.mark.parametrize("d", [1, 37, 256, 768, 1024])
@pytest.mark.parametrize("squared", [False, True])
def test_norms_bitwise_vs_oracle(pmm, d, squared):
    # compute_norms_f32 / compute_squared_norms_f32 (src/metrics.rs:368-393):
    # the device norms (ndarray unrolled_dot order, no contraction) equal the
    # oracle's bit for bit, f32 and f64, with a padded row stride
    import torch

    n = _native()
    rs = np.random.RandomState(d)
    rows = 1000
    dev = torch.device("cuda:0")
    for dt, tdt in ((np.float32, torch.float32), (np.float64, torch.float64)):
        a = (rs.randn(rows, d) * rs.uniform(0.1, 10.0, (rows, 1))).astype(dt)
        ld = d + 5
        buf = torch.zeros((rows, ld), dtype=tdt, device=dev)
        buf[:, :d] = torch.from_numpy(a).to(dev)
        out = torch.empty(rows, dtype=tdt, device=dev)
        n.norms_device(buf.data_ptr(), ld, rows, d, squared, out.data_ptr(), f64=dt == np.float64,
                       stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        want = oracle.norms(a, squared=squared)
        ui = np.uint32 if dt == np.float32 else np.uint64
        assert np.array_equal(got.view(ui), want.view(ui)), (dt, int((got != want).sum()))


def test_concurrent_calls_are_reentrant(pmm):
    # two .pmm expressions evaluated concurrently (tests/test_polars_matmul.py:551-572)
    rs = np.random.RandomState(5)
    q = rs.randn(200, 64).astype(np.float32)
    c1 = rs.randn(3000, 64).astype(np.float32)
    c2 = rs.randn(2000, 64).astype(np.float32)
    want1 = gpu_topk(q, c1, 20, "cosine")
    want2 = gpu_topk(q, c2, 20, "euclidean")
    res = {}

    def run(name, c, metric):
        for _ in range(5):
            res[name] = gpu_topk(q, c, 20, metric)

    ts = [threading.Thread(target=run, args=("a", c1, "cosine")),
          threading.Thread(target=run, args=("b", c2, "euclidean"))]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert np.array_equal(res["a"][0], want1[0]) and np.array_equal(res["a"][1], want1[1])
    assert np.array_equal(res["b"][0], want2[0]) and np.array_equal(res["b"][1], want2[1])


def test_device_api_sharded_merge_equals_full(pmm):
    # corpus row-sharding: per-shard top-k with index_base, then
    # the k-way merge, equals the unsharded result
    import torch

    n = _native()
    rs = np.random.RandomState(9)
    m, N, d, k = 300, 5000, 128, 50
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(N, d).astype(np.float32)
    full_i, full_s = gpu_topk(q, c, k, "cosine")
    dev = torch.device("cuda:0")
    tq = torch.from_numpy(q).to(dev)
    shards = [(0, 1700), (1700, 3400), (3400, 5000)]
    gi = torch.empty((m, len(shards), k), dtype=torch.int32, device=dev)
    gs = torch.empty((m, len(shards), k), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    for si, (a, b) in enumerate(shards):
        tc = torch.from_numpy(c[a:b]).to(dev)
        oi = torch.empty((m, k), dtype=torch.int32, device=dev)
        osc = torch.empty((m, k), dtype=torch.float32, device=dev)
        n.topk_device(tq.data_ptr(), d, m, tc.data_ptr(), d, b - a, d, k, 0, oi.data_ptr(), osc.data_ptr(),
                      index_base=a, stream=stream)
        gi[:, si] = oi
        gs[:, si] = osc
    mi = torch.empty((m, k), dtype=torch.int32, device=dev)
    ms = torch.empty((m, k), dtype=torch.float32, device=dev)
    n.merge_device(gi.data_ptr(), gs.data_ptr(), m, len(shards), k, k, 0, mi.data_ptr(), ms.data_ptr(), stream=stream)
    torch.cuda.synchronize()
    got_i = mi.cpu().numpy().view(np.uint32)
    got_s = ms.cpu().numpy()
    assert np.array_equal(got_i, full_i)
    assert np.array_equal(got_s, full_s)


# ---- the list merge on random inputs against a NumPy merge: final order by
# rank counting (k_out <= 128, up to 16384 rows) and by the bitonic sort
# (k_out > 128, or more rows); ties in score, empty slots, fewer valid entries
# than k_out, compactions during the load ----
@pytest.mark.parametrize("m,lists,k_in,k_out,metric,empty,tied", [
    (37, 3, 50, 20, 0, 0.0, False), (20, 1, 30, 20, 1, 0.0, False), (64, 8, 100, 100, 0, 0.0, True),
    (16, 64, 16, 128, 1, 0.0, False), (16, 2, 700, 100, 2, 0.0, False), (16, 5, 400, 128, 0, 0.3, True),
    (16, 4, 40, 100, 2, 0.5, False), (16, 9, 300, 1, 0, 0.0, True), (16, 64, 40, 64, 1, 0.2, True),
    (8, 3, 300, 129, 0, 0.1, False), (8, 70, 10, 100, 0, 0.0, False), (300, 8, 128, 128, 2, 0.05, True),
    (20000, 4, 64, 100, 0, 0.1, True)])
def test_merge_random_lists(m, lists, k_in, k_out, metric, empty, tied):
    import torch
    n = _native()
    rs = np.random.RandomState(m * 1000 + lists * 10 + k_out)
    L = lists * k_in
    idx = np.stack([rs.permutation(8 * L)[:L] * 512 + rs.randint(512) for _ in range(m)]).astype(np.uint32)
    sc = (rs.randint(0, 40, size=idx.shape) / 40.0 if tied else rs.randn(*idx.shape)).astype(np.float32)
    if metric == 2:
        sc = np.abs(sc)
    drop = rs.rand(*idx.shape) < empty
    idx[drop] = 0xFFFFFFFF
    sc[drop] = np.nan
    dev = torch.device("cuda:0")
    ti = torch.from_numpy(idx.reshape(m, lists, k_in).view(np.int32)).to(dev)
    ts = torch.from_numpy(sc.reshape(m, lists, k_in)).to(dev)
    oi = torch.full((m, k_out), 7, dtype=torch.int32, device=dev)
    os_ = torch.full((m, k_out), 7.0, dtype=torch.float32, device=dev)
    n.merge_device(ti.data_ptr(), ts.data_ptr(), m, lists, k_in, k_out, metric, oi.data_ptr(), os_.data_ptr())
    torch.cuda.synchronize()
    gi, gsc = oi.cpu().numpy().view(np.uint32), os_.cpu().numpy()
    for r in range(m):
        ok = idx[r] != 0xFFFFFFFF
        fi, fs = idx[r][ok], sc[r][ok]
        order = np.lexsort((fi, fs if metric == 2 else -fs))[:k_out]
        nv = len(order)
        assert np.array_equal(gi[r, :nv], fi[order]), f"row {r}"
        assert np.array_equal(gsc[r, :nv], fs[order]), f"row {r}"
        assert np.all(gi[r, nv:] == 0xFFFFFFFF) and np.all(np.isnan(gsc[r, nv:])), f"row {r}"


# ---- the sorted-list merge (pmm_merge_sorted_topk_strided_device: each
# list best-first, as every top-k output is; the prefix fast path, with the
# general path for rows whose prefixes cannot hold the answer) against the
# general merge and NumPy, in the [lists][2][m][k_in] layout of the gather ----
@pytest.mark.parametrize("m,lists,k_in,k_out,metric,empty,tied,skew", [
    (3000, 8, 100, 100, 0, 0.0, False, "none"), (3000, 8, 100, 100, 2, 0.0, True, "none"),
    (500, 8, 100, 100, 1, 0.0, False, "one"), (500, 8, 100, 100, 0, 0.0, False, "two"),
    (400, 2, 300, 256, 0, 0.1, False, "none"), (400, 3, 40, 100, 1, 0.5, False, "none"),
    (400, 16, 64, 100, 0, 0.05, True, "none"), (200, 64, 10, 64, 2, 0.0, False, "none"),
    (200, 70, 8, 100, 0, 0.0, False, "none"), (200, 8, 50, 300, 1, 0.0, False, "none"),
    (300, 1, 120, 100, 0, 0.2, True, "none"), (300, 5, 7, 30, 0, 0.0, False, "none"),
    (300, 6, 40, 200, 2, 0.1, False, "none"), (300, 7, 20, 100, 0, 0.0, True, "none"),
    (70000, 8, 100, 100, 0, 0.0, False, "none")])
def test_merge_sorted_lists(m, lists, k_in, k_out, metric, empty, tied, skew):
    import torch
    n = _native()
    rs = np.random.RandomState(m + lists * 7 + k_in * 3 + k_out)
    # distinct global indices per row (shard g's rows are [g * 2^20, (g + 1) * 2^20))
    idx = np.stack([np.concatenate([g * (1 << 20) + rs.permutation(1 << 12)[:k_in] for g in range(lists)])
                    for _ in range(m)]).reshape(m, lists, k_in).astype(np.uint32)
    sc = (rs.randint(0, 40, size=idx.shape) / 40.0 if tied else rs.randn(*idx.shape)).astype(np.float32)
    if skew == "one":    # every row's answer from list 0 (the prefixes cannot hold it)
        sc[:, 0] += 10.0
    elif skew == "two":  # lists 0 and 1 dominate
        sc[:, :2] += 10.0
    if metric == 2:
        sc = np.abs(sc) if skew == "none" else np.abs(sc - 20.0)
    drop = rs.rand(*idx.shape) < empty
    idx[drop] = 0xFFFFFFFF
    sc[drop] = np.nan
    # best first under the total order: score (desc; euclidean asc), then lower index; empty slots last
    for r in range(m):
        for g in range(lists):
            ii, ss = idx[r, g], sc[r, g]
            key = np.where(ii == 0xFFFFFFFF, np.inf, -ss if metric != 2 else ss)
            o = np.lexsort((ii, key))
            idx[r, g], sc[r, g] = ii[o], ss[o]
    dev = torch.device("cuda:0")
    buf = torch.empty((lists, 2, m, k_in), dtype=torch.int32, device=dev)
    buf[:, 0] = torch.from_numpy(np.ascontiguousarray(idx.transpose(1, 0, 2)).view(np.int32)).to(dev)
    buf[:, 1] = torch.from_numpy(np.ascontiguousarray(sc.transpose(1, 0, 2)).view(np.int32)).to(dev)
    outs = {}
    for srt in (False, True):
        oi = torch.full((m, k_out), 7, dtype=torch.int32, device=dev)
        os_ = torch.full((m, k_out), 7.0, dtype=torch.float32, device=dev)
        n.merge_strided_device(buf.data_ptr(), buf[0, 1].data_ptr(), m, lists, k_in, k_in, 2 * m * k_in, k_out,
                               metric, oi.data_ptr(), os_.data_ptr(), sorted_lists=srt)
        torch.cuda.synchronize()
        outs[srt] = (oi.cpu().numpy().view(np.uint32), os_.cpu().numpy())
    assert np.array_equal(outs[True][0], outs[False][0])
    assert np.array_equal(outs[True][1].view(np.uint32), outs[False][1].view(np.uint32))
    gi, gsc = outs[True]
    fi_all, fs_all = idx.reshape(m, -1), sc.reshape(m, -1)
    for r in range(0, m, max(1, m // 50)):
        ok = fi_all[r] != 0xFFFFFFFF
        fi, fs = fi_all[r][ok], fs_all[r][ok]
        order = np.lexsort((fi, fs if metric == 2 else -fs))[:k_out]
        nv = len(order)
        assert np.array_equal(gi[r, :nv], fi[order]), f"row {r}"
        assert np.array_equal(gsc[r, :nv], fs[order]), f"row {r}"
        assert np.all(gi[r, nv:] == 0xFFFFFFFF) and np.all(np.isnan(gsc[r, nv:])), f"row {r}"


def test_c5_shape_corpus_sharded_8way(pmm):
    # BASELINE configs[4] (1M x 10M x 1024 cosine k=100 on 8 GPUs, corpus
    # row-sharded) at a size one GPU checks in seconds: D = 1024, k = 100,
    # 8 contiguous corpus shards (sharded.shard_bounds), per-shard fused top-k
    # with index_base + the k-way merge == the unsharded fused top-k, and
    # both == float64 truth
    import torch

    from golden.make_golden import truth_scores
    from polars_matmul.sharded import shard_bounds

    n = _native()
    rs = np.random.RandomState(1024)
    m, N, d, k, world = 96, 24_000, 1024, 100, 8
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(N, d).astype(np.float32)
    full_i, full_s = gpu_topk(q, c, k, "cosine")
    dev = torch.device("cuda:0")
    tq = torch.from_numpy(q).to(dev)
    gi = torch.empty((m, world, k), dtype=torch.int32, device=dev)
    gs = torch.empty((m, world, k), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    for r in range(world):
        a, b = shard_bounds(N, world, r)
        tc = torch.from_numpy(c[a:b]).to(dev)
        oi = torch.empty((m, k), dtype=torch.int32, device=dev)
        osc = torch.empty((m, k), dtype=torch.float32, device=dev)
        n.topk_device(tq.data_ptr(), d, m, tc.data_ptr(), d, b - a, d, k, 0, oi.data_ptr(), osc.data_ptr(),
                      index_base=a, stream=stream)
        gi[:, r] = oi
        gs[:, r] = osc
    mi = torch.empty((m, k), dtype=torch.int32, device=dev)
    ms = torch.empty((m, k), dtype=torch.float32, device=dev)
    n.merge_device(gi.data_ptr(), gs.data_ptr(), m, world, k, k, 0, mi.data_ptr(), ms.data_ptr(), stream=stream)
    torch.cuda.synchronize()
    got_i = mi.cpu().numpy().view(np.uint32)
    got_s = ms.cpu().numpy()
    # the same f32 arithmetic per (query, corpus row) whatever the shard
    assert np.array_equal(got_i, full_i)
    assert np.array_equal(got_s, full_s)
    check_topk(got_i, got_s, truth_scores(q, c, "cosine"), True, label="c5-shape 8-way sharded")


@pytest.mark.parametrize("compute", ["f32", "bf16"])
def test_whole_query_block_schedule(pmm, compute, monkeypatch):
    # the schedule full-size runs take (query blocks >= grid: whole blocks
    # carry their rows' state over every corpus tile, then split units),
    # forced at a checkable size by planning for 8 workgroups
    from golden.make_golden import truth_scores
    from parity import round_bf16

    n = _native()
    rs = np.random.RandomState(77)
    m, N, d, k = 2500, 9000, 768, 50
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(N, d).astype(np.float32)
    monkeypatch.setenv("PMM_CUS", "8")
    for metric in ("cosine", "euclidean"):
        if compute == "f32":
            idx, sc = gpu_topk(q, c, k, metric)
            truth = truth_scores(q, c, metric)
        else:
            idx, sc = gpu_topk_bf16(q, c, k, metric)
            truth = truth_scores(round_bf16(q), round_bf16(c), metric)
        check_topk(idx, sc, truth, metric != "euclidean", label=f"whole-block {compute} {metric}")
    monkeypatch.delenv("PMM_CUS")
    want = gpu_topk(q, c, k, "cosine") if compute == "f32" else gpu_topk_bf16(q, c, k, "cosine")
    monkeypatch.setenv("PMM_CUS", "8")
    got = gpu_topk(q, c, k, "cosine") if compute == "f32" else gpu_topk_bf16(q, c, k, "cosine")
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])


@pytest.mark.parametrize("flags", ["0", "1", "2", "3", "4", "7"])
@pytest.mark.parametrize("shape", ["whole+split", "many-lists"])
def test_merge_schedules_same_lists(pmm, flags, shape, monkeypatch):
    # merge_kernel's row order (kMergeReverse), pipelined candidate loads
    # (kMergePipelined) and four waves per row (kMergeSplitRow, few rows with
    # many lists and k <= 64) change when and where work happens, never the
    # result: every combination equals the default, which equals the oracle.
    # "whole+split": whole-block rows (one segment) and split rows (many
    # segments, several batches each); "many-lists": the c1 shape's schedule
    # (every row split over dozens of corpus ranges, k = 10)
    import oracle

    rs = np.random.RandomState(31)
    if shape == "whole+split":
        m, N, d, k = 1200, 20000, 64, 100
        monkeypatch.setenv("PMM_CUS", "4")  # 10 query blocks: 8 whole, 2 as split units
    else:
        m, N, d, k = 700, 30011, 96, 10
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(N, d).astype(np.float32)
    want = gpu_topk(q, c, k, "cosine")
    monkeypatch.setenv("PMM_MERGE_FLAGS", flags)
    got = gpu_topk(q, c, k, "cosine")
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    rows = np.arange(0, m, 97)
    oi, osc = oracle.topk(q[rows], c, k, oracle.COSINE)
    assert_bitexact(got[0][rows], got[1][rows], oi, osc, label=f"merge flags {flags}")


@pytest.mark.parametrize("variant", ["0", "1", "2", "3", "4", "5", "5:whole"])
def test_every_tile_variant_same_lists(pmm, variant, monkeypatch):
    # each f32 tile variant forced in turn (PMM_GEMM_VARIANT, per call): the
    # 128-wide ones with the per-lane flag pre-filter, the 256-wide ones with
    # the two-pass one (flags, wave OR, appends at flagged positions); every
    # variant returns the default's lists bit for bit, and the oracle's.  A
    # variant whose LDS carve does not hold the candidate buffers of a k
    # falls back to the chosen one (k = 300 on 256 x 256).
    # ("5": the column split, two waves per SIMD splitting each tile's
    # columns, two candidate segments per row and split; "5:whole" plans for 4
    # workgroups so most query blocks run whole)
    if variant.endswith(":whole"):
        variant = variant.split(":")[0]
        monkeypatch.setenv("PMM_CUS", "4")
    rs = np.random.RandomState(41)
    m, N, d = 700, 9001, 80
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(N, d).astype(np.float32)
    c[17] = 0.0  # a zero-norm corpus row (cosine 0.0, src/metrics.rs:334-337)
    q[5] = 0.0
    rows = np.arange(0, m, 53)
    for metric, mid in (("cosine", oracle.COSINE), ("dot", oracle.DOT), ("euclidean", oracle.EUCLIDEAN)):
        for k in (1, 37, 100, 300):
            monkeypatch.delenv("PMM_GEMM_VARIANT", raising=False)
            want = gpu_topk(q, c, k, metric)
            monkeypatch.setenv("PMM_GEMM_VARIANT", variant)
            got = gpu_topk(q, c, k, metric)
            assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]), (variant, metric, k)
            oi, osc = oracle.topk(q[rows], c, k, mid)
            assert_bitexact(got[0][rows], got[1][rows], oi, osc, label=f"variant {variant} {metric} k={k}")


def test_merge_bytes_counts_the_candidates_left(pmm):
    # the reduction's algorithmic bytes (bench.py "reduction_roofline"):
    # counts + thresholds + output, plus 8 B per candidate the GEMM left --
    # at least k per row, at most S * capg per row
    import torch

    n = _native()
    rs = np.random.RandomState(5)
    m, N, d, k = 200, 6000, 64, 20
    dev = torch.device("cuda:0")
    tq = torch.from_numpy(rs.randn(m, d).astype(np.float32)).to(dev)
    tc = torch.from_numpy(rs.randn(N, d).astype(np.float32)).to(dev)
    wb = n.workspace_bytes(m, N, d, k, 0)
    ws = torch.zeros(wb, dtype=torch.uint8, device=dev)
    oi = torch.empty((m, k), dtype=torch.int32, device=dev)
    osc = torch.empty((m, k), dtype=torch.float32, device=dev)
    n.topk_device(tq.data_ptr(), d, m, tc.data_ptr(), d, N, d, k, 0, oi.data_ptr(), osc.data_ptr(),
                  workspace=ws.data_ptr(), workspace_bytes=wb,
                  stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    b = n.merge_bytes(ws.data_ptr(), m, N, d, k, 0)
    fixed = m * 8 + m * k * 8
    assert b >= fixed + m * k * 8 + m * 4
    assert b <= fixed + m * 4 * N + m * N * 8
    assert n.merge_bytes(ws.data_ptr(), 0, N, d, k, 0) == 0


def test_device_corpus_handle_matches_host_api(pmm):
    # corpus uploaded once, many calls
    n = _native()
    rs = np.random.RandomState(21)
    q = rs.randn(150, 70).astype(np.float32)
    c = rs.randn(4000, 70).astype(np.float32)
    dc = n.DeviceCorpus(c)
    for metric in ("cosine", "dot", "euclidean"):
        want = gpu_topk(q, c, 33, metric)
        got = dc.topk(q, 33, METRICS[metric])
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    dc.close()


def test_device_api_logical_d_matches_host_api(pmm):
    # device API with d = 70 (not a multiple of 32 or 8): rows zero-padded to
    # a stride of 96, norms over exactly 70 elements -> bit-identical to the
    # host API, which pads internally
    import torch
    from polars_matmul.sharded import ShardedTopK

    rs = np.random.RandomState(23)
    q = rs.randn(90, 70).astype(np.float32)
    c = rs.randn(3000, 70).astype(np.float32)
    dev = torch.device("cuda:0")
    for metric in ("cosine", "dot", "euclidean"):
        st = ShardedTopK(torch.from_numpy(q).to(dev), torch.from_numpy(c).to(dev), 0, 17,
                         METRICS[metric])
        assert st.q.stride(0) == 96 and st.q.shape[1] == 70
        oi, osc = st.run()
        torch.cuda.synchronize()
        want = gpu_topk(q, c, 17, metric)
        assert np.array_equal(oi.cpu().numpy().view(np.uint32), want[0])
        assert np.array_equal(osc.cpu().numpy(), want[1])


def test_arrow_corpus_cache_through_extension(pmm):
    from polars_matmul import _polars_matmul as ext

    ext.clear_corpus_cache()
    rs = np.random.RandomState(22)
    c = rs.randn(6000, 64).astype(np.float32)  # 1.5 MB: cached
    carr = pa.FixedSizeListArray.from_arrays(pa.array(c.reshape(-1)), 64)
    q1 = pa.FixedSizeListArray.from_arrays(pa.array(rs.randn(40 * 64).astype(np.float32)), 64)
    q2 = pa.FixedSizeListArray.from_arrays(pa.array(rs.randn(30 * 64).astype(np.float32)), 64)
    r1 = ext._topk(q1, carr, 12, "cosine")
    assert len(ext._cache) == 1
    r2 = ext._topk(q2, carr, 12, "cosine")
    assert len(ext._cache) == 1  # second batch hits the device-resident corpus
    for qa, r in ((q1, r1), (q2, r2)):
        qn = np.asarray(qa.values).reshape(-1, 64)
        want_i, want_s = gpu_topk(qn, c, 12, "cosine")
        got = r.to_pylist()
        assert [[x["index"] for x in row] for row in got] == want_i.tolist()
    ext.clear_corpus_cache()
    assert len(ext._cache) == 0


# ---- Float64 corpus handles (SURVEY 8f rank 4 for the
# reference's f64 branch, src/matmul.rs:449-468): the rows and their f64 norms
# stay in HBM; each call uploads only the queries ----
@pytest.mark.parametrize("fused", ["1", "0"])
def test_f64_device_corpus_handle_matches_host_api(pmm, fused, monkeypatch):
    n = _native()
    monkeypatch.setenv("PMM_F64_FUSED", fused)
    rs = np.random.RandomState(31)
    q = rs.randn(120, 70)
    c = rs.randn(5000, 70)
    c[4000:4030] = c[:30]  # exact ties
    c[77] = 0.0            # a zero-norm row (cosine score 0, src/metrics.rs:277-288)
    dc = n.DeviceCorpus(c)
    assert dc.dtype == np.float64 and dc.device_dtype == n.DTYPE_F64
    for metric in ("cosine", "dot", "euclidean"):
        for k in (1, 25, 1100):  # 1100 > 1024: the materialised path either way
            want_i, want_s = n.topk_host(q, c, k, METRICS[metric])
            got_i, got_s = dc.topk(q, k, METRICS[metric])
            assert got_s.dtype == np.float64
            assert np.array_equal(got_i, want_i), (metric, k)
            assert np.array_equal(got_s.view(np.uint64), want_s.view(np.uint64)), (metric, k)
        oi, osc = oracle.topk(q[:24], c, 25, METRICS[metric])
        gi, gs = dc.topk(q[:24], 25, METRICS[metric])
        assert np.array_equal(gi, oi), metric
        np.testing.assert_allclose(gs, osc, rtol=1e-12, atol=1e-12)
    dc.close()


def test_f64_corpus_handle_fused_scan_uses_cached_norms(pmm, monkeypatch):
    # a shape the library scans fused by size (m x n x 8 B > 256 MB): no corpus
    # norm launch per call -- only the queries' -- and the same lists as the
    # host API, which computes both
    n = _native()
    rs = np.random.RandomState(32)
    q, c = rs.randn(300, 48), rs.randn(120_000, 48)
    dc = n.DeviceCorpus(c)
    want = n.topk_host(q, c, 10, METRICS["cosine"])
    n.timing_reset()
    n.timing_enable(True)
    try:
        got = dc.topk(q, 10, METRICS["cosine"])
    finally:
        n.timing_enable(False)
    assert n.timing_read("gemm_f64_topk")[1] >= 1 and n.timing_read("gemm_f64_scores")[1] == 0
    h2d_ms, h2d_n = n.timing_read("h2d")
    assert h2d_n == 1  # the queries only
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1].view(np.uint64), want[1].view(np.uint64))
    dc.close()


def test_corpus_handle_dtype_mismatch_raises(pmm):
    n = _native()
    rs = np.random.RandomState(33)
    c32 = rs.randn(300, 16).astype(np.float32)
    c64 = c32.astype(np.float64)
    h32, h64 = n.DeviceCorpus(c32), n.DeviceCorpus(c64)
    assert h32.device_dtype == n.DTYPE_F32 and h64.device_dtype == n.DTYPE_F64
    q64 = np.ascontiguousarray(rs.randn(4, 16))
    q32 = q64.astype(np.float32)
    idx = np.empty((4, 5), np.uint32)
    for fn, h, q, sc in ((n.lib().pmm_topk_f64_corpus, h32, q64, np.empty((4, 5))),
                         (n.lib().pmm_topk_f32_corpus, h64, q32, np.empty((4, 5), np.float32))):
        rc = fn(h._h, n.ptr(q), 4, 5, 0, n.ptr(idx), n.ptr(sc))
        assert rc == n.PMM_ERR_ARG and "corpus handle holds" in n.last_error()
    h32.close()
    h64.close()


def test_arrow_f64_corpus_cache_through_extension(pmm):
    # Polars' default Float64 column as the corpus: cached on the device like
    # an f32 one (one entry, hit on the second batch), the results the host
    # API's; the same buffers searched by f32 queries (-> the f64 branch,
    # src/matmul.rs:427) and by f64 ones share the f64 entry, while an f32
    # column searched by f32 queries is its own (f32) entry
    from polars_matmul import _polars_matmul as ext

    ext.clear_corpus_cache()
    rs = np.random.RandomState(34)
    c = rs.randn(5000, 64)  # 2.6 MB of f64 (1.3 MB as f32): cached either way
    carr = pa.FixedSizeListArray.from_arrays(pa.array(c.reshape(-1)), 64)
    q1 = pa.FixedSizeListArray.from_arrays(pa.array(rs.randn(40 * 64)), 64)
    q2 = pa.FixedSizeListArray.from_arrays(pa.array(rs.randn(30 * 64).astype(np.float32)), 64)
    r1 = ext._topk(q1, carr, 12, "cosine")
    assert len(ext._cache) == 1
    r2 = ext._topk(q2, carr, 12, "euclidean")
    assert len(ext._cache) == 1  # same corpus, same compute dtype: a hit
    (key, (_, dc)), = ext._cache.items()
    assert dc.dtype == np.float64
    for qa, r, metric in ((q1, r1, "cosine"), (q2, r2, "euclidean")):
        qn = np.asarray(qa.values).reshape(-1, 64).astype(np.float64)
        want_i, want_s = gpu_topk(qn, c, 12, metric)
        got = r.to_pylist()
        assert [[x["index"] for x in row] for row in got] == want_i.tolist()
        assert [[x["score"] for x in row] for row in got] == want_s.tolist()
    c32 = pa.FixedSizeListArray.from_arrays(pa.array(c.reshape(-1).astype(np.float32)), 64)
    ext._topk(q2, c32, 12, "cosine")
    assert len(ext._cache) == 2 and sorted(v[1].dtype.str for v in ext._cache.values()) == ["<f4", "<f8"]
    ext.clear_corpus_cache()
    assert len(ext._cache) == 0


# ---------------------------------------------------------------------------
# bf16 compute path (PMM_COMPUTE_BF16, BASELINE configs[3]).  Truth = the
# metric of the bf16-rounded rows in float64; the device accumulates the
# bf16 products in f32, so the f32 tolerance applies (rtol 1e-5 + the
# |q||c|-scaled dot term).  SURVEY 8c's own bar for bf16 (recall@k >= 0.95
# vs the f32 result) is checked separately.
# ---------------------------------------------------------------------------
def gpu_topk_bf16(q, c, k, metric, n=None):
    n = n or _native()
    kk = min(k, c.shape[0])
    return n.topk_host(np.ascontiguousarray(q, dtype=np.float32),
                       np.ascontiguousarray(c, dtype=np.float32), kk, METRICS[metric],
                       compute=n.COMPUTE_BF16)


def _bf16_truth_check(q, c, k, metric, idx, sc, label):
    from golden.make_golden import truth_scores
    from parity import round_bf16

    qb, cb = round_bf16(q), round_bf16(c)
    truth = truth_scores(qb, cb, metric)
    scale = dot_scale(qb, cb) if metric == "dot" else None
    check_topk(idx, sc, truth, metric != "euclidean", rtol=1e-5, atol=1e-5, scale=scale, label=label)


@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
@pytest.mark.parametrize("k", [1, 10, 100, 900])
def test_bf16_fixture_vs_bf16_truth(pmm, metric, k):
    z = np.load(os.path.join(GOLD, "rand_f32_48x1000x256.npz"))
    idx, sc = gpu_topk_bf16(z["q"], z["c"], k, metric)
    _bf16_truth_check(z["q"], z["c"], k, metric, idx, sc, f"bf16 {metric} k={k}")


@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
def test_bf16_edge_fixture(pmm, metric):
    # zero-norm rows, exact duplicates (ties -> lower index first), d=37 -> 128
    z = np.load(os.path.join(GOLD, "edge_f32_6x70x37.npz"))
    idx, sc = gpu_topk_bf16(z["q"], z["c"], 70, metric)
    _bf16_truth_check(z["q"], z["c"], 70, metric, idx, sc, f"bf16 edge {metric}")
    for i in range(6):
        row = idx[i].tolist()
        assert row.index(3) < row.index(11) < row.index(40)
    if metric == "cosine":
        assert np.all(sc[2] == 0.0) and idx[2].tolist() == list(range(70))


@pytest.mark.parametrize("m,n,d,k", [
    (1, 1, 1, 1), (3, 5, 2, 5), (130, 257, 33, 7), (129, 1000, 128, 100), (7, 300, 768, 16),
    (257, 4099, 200, 64), (300, 2000, 768, 448),
])
@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
def test_bf16_ragged_shapes(pmm, m, n, d, k, metric):
    rs = np.random.RandomState(m * 5 + n + d)
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(n, d).astype(np.float32)
    idx, sc = gpu_topk_bf16(q, c, k, metric)
    _bf16_truth_check(q, c, k, metric, idx, sc, f"bf16 {m}x{n}x{d} k={k} {metric}")


@pytest.mark.parametrize("m,n,d,k", [(130, 257, 33, 7), (257, 4099, 200, 64), (300, 2000, 768, 100)])
@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
def test_bf16_one_wave_per_simd_kernel(pmm, m, n, d, k, metric, monkeypatch):
    # PMM_BF16_WS=0: the 4-wave kernel (pmm_bf16_kernel.h) on shapes the
    # wave-specialised kernel serves by default (it still serves k > 448)
    monkeypatch.setenv("PMM_BF16_WS", "0")
    rs = np.random.RandomState(m + n + d + k)
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(n, d).astype(np.float32)
    idx, sc = gpu_topk_bf16(q, c, k, metric)
    _bf16_truth_check(q, c, k, metric, idx, sc, f"bf16 classic {m}x{n}x{d} k={k} {metric}")


@pytest.mark.parametrize("m,n,d", [(300, 20000, 768), (140, 9000, 200), (70, 8200, 128), (64, 8500, 384),
                                   (100, 9100, 512), (129, 8300, 640), (200, 40000, 256)])
@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
def test_bf16_seeded_threshold_is_exact(pmm, m, n, d, metric, monkeypatch):
    # the wave-specialised kernel starts each row from the k-th best of the
    # first ns columns (seed_bf16_ws_kernel + seed_select_kernel): those
    # scores are bit-identical to the main pass's, so the seed is an exact
    # lower bound and the lists equal the unseeded run's bit for bit --
    # including exact ties inside and across the sample
    rs = np.random.RandomState(m + n + d)
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(n, d).astype(np.float32)
    c[5000:5040] = c[:40]        # sample columns duplicated past the sample
    c[300:310] = c[700:710]      # duplicates inside the sample
    q[7] = c[3]                  # a query equal to a sample column
    c[100, 5] = np.nan           # NaN scores inside the sample ...
    c[n - 3, 0] = np.nan         # ... and past it
    q[11, 2] = np.nan            # a query row whose every score is NaN
    for k, ns in ((1, None), (10, None), (100, None), (256, None), (10, "64"), (50, "512"), (100, "2048"),
                  (100, "4096")):  # (2048 / 4096: a seed only where n >= 8 ns)
        monkeypatch.setenv("PMM_BF16_SEED", "0")
        want = gpu_topk_bf16(q, c, k, metric)
        monkeypatch.setenv("PMM_BF16_SEED", "1")
        if ns:
            monkeypatch.setenv("PMM_SEED_NS", ns)
        got = gpu_topk_bf16(q, c, k, metric)
        monkeypatch.delenv("PMM_SEED_NS", raising=False)
        assert np.array_equal(got[0], want[0]), (metric, k, ns, float(np.mean(got[0] == want[0])))
        assert np.array_equal(got[1].view(np.uint32), want[1].view(np.uint32)), (metric, k, ns)


def test_bf16_recall_vs_f32(pmm):
    # SURVEY 8c bf16 criterion: recall@k >= 0.95 against the f32 result
    rs = np.random.RandomState(31)
    q = rs.randn(200, 768).astype(np.float32)
    c = rs.randn(20000, 768).astype(np.float32)
    bi, bs = gpu_topk_bf16(q, c, 100, "cosine")
    fi, fs = gpu_topk(q, c, 100, "cosine")
    recall = np.mean([len(set(bi[i]) & set(fi[i])) / 100.0 for i in range(len(q))])
    assert recall >= 0.95, recall
    assert np.max(np.abs(bs - fs)) < 1e-2


def test_bf16_device_api_many_splits(pmm):
    # device bf16 rows (torch.bfloat16), a corpus long enough for several
    # splits and many tiles per unit; truth from float64 on device
    import torch

    n = _native()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    m, N, d, k = 700, 60000, 768, 100
    q = torch.randn((m, d), generator=g, device=dev).to(torch.bfloat16)
    c = torch.randn((N, d), generator=g, device=dev).to(torch.bfloat16)
    oi = torch.empty((m, k), dtype=torch.int32, device=dev)
    osc = torch.empty((m, k), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    n.topk_bf16_device(q.data_ptr(), d, m, c.data_ptr(), d, N, d, k, METRICS["cosine"],
                       oi.data_ptr(), osc.data_ptr(), index_base=7, stream=stream)
    torch.cuda.synchronize()
    qd, cd = q.double(), c.double()
    s = (qd @ cd.T) / (qd.norm(dim=1, keepdim=True) * cd.norm(dim=1)[None, :])
    ref_s, ref_i = torch.topk(s, k, dim=1)
    got_i = oi.long() - 7
    assert int(got_i.min()) >= 0 and int(got_i.max()) < N
    got_true = torch.gather(s, 1, got_i)
    kth = ref_s[:, -1:]
    assert bool((got_true >= kth - 2e-5).all())
    assert float((osc.double() - got_true).abs().max()) < 1e-5
    assert float((got_i == ref_i).float().mean()) > 0.97


@pytest.mark.parametrize("whole", ["0", "1"])
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_bf16_whole_block_runs(pmm, metric, whole, monkeypatch):
    # M >= BM x grid query rows (BM = 128 for the wave-specialised kernel).
    # PMM_BF16_WHOLE=1 (default): the first 256 query
    # blocks run whole (split by split, row state carried across splits), the
    # remaining 2-3 blocks as split units; 0: every unit a split unit.  Every
    # row vs float64 truth.
    import torch

    monkeypatch.setenv("PMM_BF16_WHOLE", whole)

    n = _native()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    m, N, d, k = 33000, 30000, 256, 50
    q = torch.randn((m, d), generator=g, device=dev).to(torch.bfloat16)
    c = torch.randn((N, d), generator=g, device=dev).to(torch.bfloat16)
    oi = torch.empty((m, k), dtype=torch.int32, device=dev)
    osc = torch.empty((m, k), dtype=torch.float32, device=dev)
    n.topk_bf16_device(q.data_ptr(), d, m, c.data_ptr(), d, N, d, k, METRICS[metric],
                       oi.data_ptr(), osc.data_ptr(),
                       stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    cd = c.double()
    got_i = oi.long()
    assert int(got_i.min()) >= 0 and int(got_i.max()) < N
    match = 0.0
    for r0 in range(0, m, 8192):
        qd = q[r0:r0 + 8192].double()
        if metric == "cosine":
            s = (qd @ cd.T) / (qd.norm(dim=1, keepdim=True) * cd.norm(dim=1)[None, :])
            ref_s, ref_i = torch.topk(s, k, dim=1)
        else:
            s = torch.cdist(qd, cd)
            ref_s, ref_i = torch.topk(s, k, dim=1, largest=False)
        gi = got_i[r0:r0 + 8192]
        got_true = torch.gather(s, 1, gi)
        kth = ref_s[:, -1:]
        if metric == "cosine":
            assert bool((got_true >= kth - 2e-5).all())
        else:
            assert bool((got_true <= kth + 2e-4).all())
        tol = 1e-5 if metric == "cosine" else 2e-4
        assert float((osc[r0:r0 + 8192].double() - got_true).abs().max()) < tol
        match += float((gi == ref_i).float().sum())
    assert match / (m * k) > 0.97


@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
def test_compaction_trigger_leaves_lists_unchanged(pmm, metric, monkeypatch):
    # PMM_CTRIG (the count above which a row's candidate buffer is compacted
    # and its threshold raised) changes how many survivors are queued, never
    # the result: bf16 (whole blocks + split units, the split units re-reading
    # the shared thresholds at every drain) and f32, bit for bit against the
    # default trigger.
    import torch

    n = _native()
    monkeypatch.setenv("PMM_CUS", "16")
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    m, N, d, k = 4480, 60000, 256, 100
    q = torch.randn((m, d), generator=g, device=dev).to(torch.bfloat16)
    c = torch.randn((N, d), generator=g, device=dev).to(torch.bfloat16)

    def run_bf16():
        oi = torch.empty((m, k), dtype=torch.int32, device=dev)
        osc = torch.empty((m, k), dtype=torch.float32, device=dev)
        n.topk_bf16_device(q.data_ptr(), d, m, c.data_ptr(), d, N, d, k, METRICS[metric],
                           oi.data_ptr(), osc.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        return oi.cpu().numpy(), osc.cpu().numpy()

    qf = q[:512].float().cpu().numpy()
    cf = c[:20000].float().cpu().numpy()
    monkeypatch.delenv("PMM_CTRIG", raising=False)
    ref_b = run_bf16()
    ref_f = gpu_topk(qf, cf, k, metric)
    for t in ("108", "160", "300"):
        monkeypatch.setenv("PMM_CTRIG", t)
        got_b = run_bf16()
        assert np.array_equal(got_b[0], ref_b[0]), (metric, t)
        assert np.array_equal(got_b[1].view(np.uint32), ref_b[1].view(np.uint32)), (metric, t)
        got_f = gpu_topk(qf, cf, k, metric)
        assert np.array_equal(got_f[0], ref_f[0]), (metric, t)
        assert np.array_equal(np.asarray(got_f[1], np.float64), np.asarray(ref_f[1], np.float64)), (metric, t)


@pytest.mark.parametrize("d,k", [(800, 50), (1024, 100), (300, 1000), (1024, 1500)])
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_bf16_beyond_kernel_limits_widened(pmm, d, k, metric):
    # bf16 compute past the bf16 kernels' limits (d > 768:
    # configs[4]'s 1024; k > 960) runs on the rounded rows widened to f32, so
    # it equals the f32 path on the bf16-rounded inputs bit for bit -- and
    # through the device API with a caller's workspace of the size
    # pmm_topk_workspace_bytes names
    import torch

    n = _native()
    rs = np.random.RandomState(d + k)
    q = rs.randn(70, d).astype(np.float32)
    c = rs.randn(3000, d).astype(np.float32)
    got = n.topk_host(q, c, k, METRICS[metric], compute=n.COMPUTE_BF16)
    qr = torch.from_numpy(q).to(torch.bfloat16).float().numpy()
    cr = torch.from_numpy(c).to(torch.bfloat16).float().numpy()
    want = n.topk_host(qr, cr, k, METRICS[metric])
    assert np.array_equal(got[0], want[0])
    assert np.array_equal(got[1].view(np.uint32), want[1].view(np.uint32))
    dev = torch.device("cuda:0")
    db = (d + 127) // 128 * 128
    tq = torch.zeros((70, db), dtype=torch.bfloat16, device=dev)
    tc = torch.zeros((3000, db), dtype=torch.bfloat16, device=dev)
    tq[:, :d] = torch.from_numpy(q).to(dev).to(torch.bfloat16)
    tc[:, :d] = torch.from_numpy(c).to(dev).to(torch.bfloat16)
    wb = n.workspace_bytes(70, 3000, db, k, METRICS[metric], n.COMPUTE_BF16)
    ws = torch.empty(wb, dtype=torch.uint8, device=dev)
    oi = torch.empty((70, k), dtype=torch.int32, device=dev)
    osc = torch.empty((70, k), dtype=torch.float32, device=dev)
    n.topk_bf16_device(tq.data_ptr(), db, 70, tc.data_ptr(), db, 3000, d, k, METRICS[metric], oi.data_ptr(),
                       osc.data_ptr(), workspace=ws.data_ptr(), workspace_bytes=wb,
                       stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(oi.cpu().numpy().view(np.uint32), want[0])
    assert np.array_equal(osc.cpu().numpy().view(np.uint32), want[1].view(np.uint32))


def test_bf16_numpy_api_and_sharded_runner(pmm):
    # polars_matmul.topk(compute="bf16") and ShardedTopK over bf16 tensors
    # (d = 200 -> zero-padded to a 256 stride) agree with each other
    import torch
    from polars_matmul.sharded import ShardedTopK

    rs = np.random.RandomState(41)
    q = rs.randn(77, 200).astype(np.float32)
    c = rs.randn(2500, 200).astype(np.float32)
    i1, s1 = pmm.topk(q, c, 25, "euclidean", compute="bf16")
    _bf16_truth_check(q, c, 25, "euclidean", i1, s1, "bf16 numpy api")
    dev = torch.device("cuda:0")
    st = ShardedTopK(torch.from_numpy(q).to(dev).to(torch.bfloat16),
                     torch.from_numpy(c).to(dev).to(torch.bfloat16), 0, 25, METRICS["euclidean"])
    assert st.q.stride(0) == 256
    oi, osc = st.run()
    torch.cuda.synchronize()
    assert np.array_equal(oi.cpu().numpy().view(np.uint32), i1)
    assert np.array_equal(osc.cpu().numpy().astype(np.float64), s1)


@pytest.mark.parametrize("k,d", [(1, 256), (10, 256), (100, 256), (10, 72), (10, 768)])
def test_threshold_seeding_changes_nothing(pmm, k, d, monkeypatch):
    # small problems seed each row's threshold from the corpus's first rows
    # (seed_dots_kernel: the sample's scores as fmaf chains, bit-identical to
    # the fused kernel's MFMA chain; PMM_SEED_GEMM=1: the store-mode GEMM +
    # seed_select_kernel) and start the main pass from (the sample's k-th
    # composite key - 1); the result must equal the unseeded run bit for bit,
    # ties (duplicated corpus rows) included
    from golden.make_golden import truth_scores

    rs = np.random.RandomState(31 + k + d)
    m, N = 700, 9000
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(N, d).astype(np.float32)
    c[4000:4600] = c[:600]  # duplicates of sampled rows, later in the corpus
    for metric in ("cosine", "dot", "euclidean"):
        monkeypatch.setenv("PMM_SEED", "0")
        want = gpu_topk(q, c, k, metric)
        monkeypatch.setenv("PMM_SEED", "1")
        got = gpu_topk(q, c, k, metric)
        monkeypatch.setenv("PMM_SEED_GEMM", "1")
        got_g = gpu_topk(q, c, k, metric)
        monkeypatch.delenv("PMM_SEED_GEMM")
        monkeypatch.setenv("PMM_SEED_LDS", "1")  # the LDS-staged seed blocks (opt-in)
        got_f = gpu_topk(q, c, k, metric)
        monkeypatch.delenv("PMM_SEED_LDS")
        outs = [got, got_g, got_f]
        for mf in ("0", "1"):  # fmaf-chain seed blocks / MFMA seed blocks (ns = 256 only)
            monkeypatch.setenv("PMM_SEED_MFMA", mf)
            outs.append(gpu_topk(q, c, k, metric))
        monkeypatch.delenv("PMM_SEED_MFMA")
        monkeypatch.delenv("PMM_SEED")
        for g in outs:
            assert np.array_equal(g[0], want[0]), metric
            assert np.array_equal(g[1], want[1]), metric
        check_topk(got[0], got[1], truth_scores(q, c, metric), metric != "euclidean",
                   label=f"seeded k={k} {metric}")


@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
@pytest.mark.parametrize("seed_mode", ["lds", "rows", "mfma"])
@pytest.mark.parametrize("d", [256, 96, 37, 1000])
def test_seed_scores_equal_main_pass_when_topk_is_in_the_sample(pmm, metric, seed_mode, d, monkeypatch):
    # Every row's true top-k lies inside the seed sample (the corpus's first
    # ns = 256 rows hold 16 near-copies of each query).  The seed's threshold
    # is (the sample's k-th composite) - 1, so if the seed scored the k-th
    # element even one ulp above the main pass, the main pass would reject
    # that element and the list would lose it: bit-exactness against the
    # oracle here checks that the seed (LDS-staged or row-streaming blocks) computes
    # the main pass's scores bit for bit
    rs = np.random.RandomState(17 + METRICS[metric] + d)
    m, N, k = 16, 4096, 10
    q = rs.randn(m, d).astype(np.float32)
    c = (rs.randn(N, d) * 0.3).astype(np.float32)
    c[:256] = q[np.arange(256) % m] + 0.05 * rs.randn(256, d).astype(np.float32)
    # (the seed blocks: LDS-staged fmaf chains, row-streaming fmaf chains, or
    # v_mfma_f32_16x16x4_f32 chains)
    monkeypatch.setenv("PMM_SEED", "1")
    monkeypatch.setenv("PMM_SEED_LDS", "1" if seed_mode == "lds" else "0")
    monkeypatch.setenv("PMM_SEED_MFMA", "1" if seed_mode == "mfma" else "0")
    idx, sc = gpu_topk(q, c, k, metric)
    assert int(idx.max()) < 256  # the top-k really is inside the sample
    oi, osc = oracle.topk(q, c, k, METRICS[metric])
    assert_bitexact(idx, sc, oi, osc, f"seed-sample top-k {metric} {seed_mode}")


@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
def test_host_chunked_upload_equals_one_launch(pmm, metric, monkeypatch):
    # pmm_topk_f32 over a corpus >= 256 MB uploads it in chunks overlapped with
    # compute (per-chunk top-k with carried thresholds + in-place chunk merge);
    # the result must equal the one-upload, one-launch result bit for bit,
    # exact cross-chunk ties included (lower global index first)
    rs = np.random.RandomState(3 + METRICS[metric])
    m, n, d = 300, 90_000, 768
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(n, d).astype(np.float32)
    c[80_000:80_050] = c[10:60]      # chunk 3 duplicates rows of chunk 0
    c[40_000:40_020] = c[30_000:30_020]  # chunk 2 duplicates rows of chunk 1
    for k in (1, 100, 1000):
        monkeypatch.setenv("PMM_CHUNKED_UPLOAD", "0")
        want = gpu_topk(q, c, k, metric)
        monkeypatch.delenv("PMM_CHUNKED_UPLOAD")
        got = gpu_topk(q, c, k, metric)
        assert np.array_equal(got[0], want[0]), (metric, k)
        assert np.array_equal(got[1].view(np.uint32), want[1].view(np.uint32)), (metric, k)
    oi, osc = oracle.topk(q[:40], c, 100, METRICS[metric])
    got = gpu_topk(q[:40], c, 100, metric)
    assert_bitexact(got[0], got[1], oi, osc, f"chunked {metric}")


# ---- multi-GPU through the drop-in boundary (pmm_set_devices) ----
# The box has one GPU: listing device 0 several times runs every shard on it
# through the same code path as distinct GPUs (per-shard top-k with global
# indices, peer copy of each [2][m][k] list into the root's gather buffer,
# k-way merge there).  The result must equal the one-device result bit for bit.

@pytest.fixture
def device_list():
    n = _native()
    yield n
    n.set_devices([])


@pytest.mark.parametrize("shards", [2, 3, 8])
@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
def test_set_devices_sharded_host_topk_bitexact(pmm, device_list, shards, metric):
    n = device_list
    rs = np.random.RandomState(shards * 7 + len(metric))
    m, N, d, k = 300, 20011, 200, 100
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(N, d).astype(np.float32)
    c[N - 40:] = c[:40]  # exact ties across shard boundaries
    want = n.topk_host(q, c, k, METRICS[metric])
    n.set_devices([0] * shards)
    assert n.get_devices() == [0] * shards
    got = n.topk_host(q, c, k, METRICS[metric])
    assert np.array_equal(got[0], want[0]), float(np.mean(got[0] == want[0]))
    assert np.array_equal(got[1].view(np.uint32), want[1].view(np.uint32))
    oi, osc = oracle.topk(q, c, k, METRICS[metric])
    assert_bitexact(got[0], got[1], oi, osc, f"set_devices x{shards} {metric}")


def test_set_devices_shards_smaller_than_k(pmm, device_list):
    # 8 shards of 12-13 rows with k = 64: every shard's list is padded with
    # empty slots, which the merge skips
    n = device_list
    rs = np.random.RandomState(3)
    q = rs.randn(40, 48).astype(np.float32)
    c = rs.randn(100, 48).astype(np.float32)
    want = n.topk_host(q, c, 64, METRICS["cosine"])
    n.set_devices([0] * 8)
    got = n.topk_host(q, c, 64, METRICS["cosine"])
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    n.set_devices([0] * 5)
    got = n.topk_host(q, c[:3], 3, METRICS["cosine"])  # fewer rows than devices: 3 shards of one row
    assert np.array_equal(got[0], n.topk_host(q, c[:3], 3, METRICS["cosine"])[0])


def test_set_devices_bf16_compute(pmm, device_list):
    n = device_list
    rs = np.random.RandomState(9)
    q = rs.randn(257, 384).astype(np.float32)
    c = rs.randn(30000, 384).astype(np.float32)
    want = n.topk_host(q, c, 50, METRICS["cosine"], compute=n.COMPUTE_BF16)
    n.set_devices([0, 0, 0])
    got = n.topk_host(q, c, 50, METRICS["cosine"], compute=n.COMPUTE_BF16)
    # each shard is the exact top-k of the bf16 rows up to f32 accumulation
    # order, checked against the truth of the rounded rows
    _bf16_truth_check(q, c, 50, "cosine", got[0], got[1], "bf16 x3 devices")
    assert float(np.mean(got[0] == want[0])) > 0.99


def test_set_devices_sharded_corpus_handle(pmm, device_list):
    # a corpus handle created under a device list is row-sharded at creation
    # (per-device corpus cache); its searches equal the one-device handle's
    n = device_list
    rs = np.random.RandomState(21)
    q = rs.randn(500, 256).astype(np.float32)
    c = rs.randn(50000, 256).astype(np.float32)
    one = n.DeviceCorpus(c)
    assert one.shards == 1
    n.set_devices([0, 0, 0, 0])
    four = n.DeviceCorpus(c)
    assert four.shards == 4
    for metric in ("cosine", "euclidean", "dot"):
        a = one.topk(q, 100, METRICS[metric])
        b = four.topk(q, 100, METRICS[metric])
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), metric
    one.close()
    four.close()


def test_set_devices_through_extension_and_cache(pmm, device_list):
    from polars_matmul import _polars_matmul as pm

    rs = np.random.RandomState(5)
    q = rs.randn(64, 128).astype(np.float32)
    c = rs.randn(9000, 128).astype(np.float32)
    carr = pa.FixedSizeListArray.from_arrays(pa.array(c.reshape(-1)), 128)
    qarr = pa.FixedSizeListArray.from_arrays(pa.array(q.reshape(-1)), 128)
    want = pm._topk(qarr, carr, 10, "cosine").to_pylist()
    pm.set_devices([0, 0])
    try:
        for _ in range(2):  # second call: the (sharded) cached handle
            assert pm._topk(qarr, carr, 10, "cosine").to_pylist() == want
    finally:
        pm.clear_corpus_cache()


def test_set_devices_one_entry_runs_there(pmm, device_list):
    # a one-entry list is not ignored -- host calls run on that
    # device (device 0 is the only one on the one-GPU box; the plan is the
    # one-device plan) and corpus handles are created there, unsharded
    n = device_list
    rs = np.random.RandomState(13)
    q = rs.randn(50, 96).astype(np.float32)
    c = rs.randn(3000, 96).astype(np.float32)
    want = n.topk_host(q, c, 20, METRICS["cosine"])
    n.set_devices([0])
    assert n.get_devices() == [0]
    got = n.topk_host(q, c, 20, METRICS["cosine"])
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1].view(np.uint32), want[1].view(np.uint32))
    oi, osc = oracle.topk(q, c, 20, METRICS["cosine"])
    assert_bitexact(got[0], got[1], oi, osc, "one-entry device list")
    dc = n.DeviceCorpus(c)
    assert dc.shards == 1
    assert np.array_equal(dc.topk(q, 1500, METRICS["dot"])[0], n.topk_host(q, c, 1500, METRICS["dot"])[0])
    dc.close()


@pytest.mark.parametrize("shards", [2, 3, 8])
@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
def test_set_devices_sharded_f64_bitexact(pmm, device_list, shards, metric, monkeypatch):
    # the f64 branch (Polars' default Float64 columns,
    # src/matmul.rs:449-468) sharded under a device list: every shard's f64
    # top-k with global indices, merged on the root -- bit-equal to one
    # device (indices and f64 scores), on both f64 paths, with ties across
    # shard boundaries, through the host API and a sharded f64 corpus handle
    n = device_list
    rs = np.random.RandomState(shards * 11 + len(metric))
    m, N, d, k = 120, 9001, 64, 100
    q = rs.randn(m, d)
    c = rs.randn(N, d)
    c[N - 30:] = c[:30]  # exact ties across shard boundaries
    for fused in ("1", "0"):
        monkeypatch.setenv("PMM_F64_FUSED", fused)
        n.set_devices([])
        want = n.topk_host(q, c, k, METRICS[metric])
        one = n.DeviceCorpus(c)
        n.set_devices([0] * shards)
        got = n.topk_host(q, c, k, METRICS[metric])
        assert np.array_equal(got[0], want[0]), (fused, float(np.mean(got[0] == want[0])))
        assert np.array_equal(got[1].view(np.uint64), want[1].view(np.uint64)), fused
        dc = n.DeviceCorpus(c)
        assert dc.shards == shards and one.shards == 1
        gc = dc.topk(q, k, METRICS[metric])
        assert np.array_equal(gc[0], want[0]) and np.array_equal(gc[1].view(np.uint64), want[1].view(np.uint64))
        oc = one.topk(q, k, METRICS[metric])
        assert np.array_equal(oc[0], want[0])
        dc.close()
        one.close()
    oi, osc = oracle.topk(q, c, k, METRICS[metric])
    assert np.array_equal(got[0], oi) and np.array_equal(got[1].view(np.uint64), osc.view(np.uint64))


def test_set_devices_f64_shards_smaller_than_k_and_large_k(pmm, device_list):
    # shards shorter than k (their lists padded with empty slots) and k above
    # the fused limit (every shard materialised): still the one-device lists
    n = device_list
    rs = np.random.RandomState(17)
    q = rs.randn(30, 40)
    c = rs.randn(101, 40)
    want = n.topk_host(q, c, 64, METRICS["cosine"])
    n.set_devices([0] * 8)  # 8 shards of 12-13 rows, k = 64
    got = n.topk_host(q, c, 64, METRICS["cosine"])
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1].view(np.uint64), want[1].view(np.uint64))
    n.set_devices([])
    c2 = rs.randn(6000, 40)
    want = n.topk_host(q, c2, 1500, METRICS["dot"])
    n.set_devices([0, 0, 0])
    got = n.topk_host(q, c2, 1500, METRICS["dot"])
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1].view(np.uint64), want[1].view(np.uint64))


def test_set_devices_f64_through_extension_and_cache(pmm, device_list):
    from polars_matmul import _polars_matmul as pm

    rs = np.random.RandomState(8)
    q = rs.randn(40, 96)
    c = rs.randn(7000, 96)
    carr = pa.FixedSizeListArray.from_arrays(pa.array(c.reshape(-1)), 96)
    qarr = pa.FixedSizeListArray.from_arrays(pa.array(q.reshape(-1)), 96)
    want = pm._topk(qarr, carr, 25, "euclidean").to_pylist()
    pm.set_devices([0, 0, 0])
    try:
        for _ in range(2):  # second call: the sharded cached f64 handle
            assert pm._topk(qarr, carr, 25, "euclidean").to_pylist() == want
    finally:
        pm.clear_corpus_cache()


def _visible_gpus():
    try:
        return _native().device_count()
    except Exception:
        return 0


needs_2gpu = pytest.mark.skipif(_visible_gpus() < 2, reason="needs >= 2 visible GPUs (distinct-device branch)")


@needs_2gpu
@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
def test_set_devices_distinct_gpus(pmm, device_list, metric):
    # the distinct-device branch of topk_sharded -- one DevPlan per
    # device, concurrent launches, cross-device event waits, peer copies into
    # the root -- bit-equal to one GPU, through host top-k and a sharded
    # corpus handle, and with the root on another device than the first
    n = device_list
    G = min(4, n.device_count())
    rs = np.random.RandomState(31)
    q = rs.randn(400, 256).astype(np.float32)
    c = rs.randn(60011, 256).astype(np.float32)
    c[-50:] = c[:50]  # ties across shard boundaries
    want = n.topk_host(q, c, 100, METRICS[metric])
    n.set_devices(list(range(G)))
    got = n.topk_host(q, c, 100, METRICS[metric])
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1].view(np.uint32), want[1].view(np.uint32))
    dc = n.DeviceCorpus(c)
    assert dc.shards == G
    got = dc.topk(q, 100, METRICS[metric])
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1].view(np.uint32), want[1].view(np.uint32))
    dc.close()
    n.set_devices(list(reversed(range(G))))  # root on the last device
    got = n.topk_host(q, c, 100, METRICS[metric])
    assert np.array_equal(got[0], want[0])
    # the f64 branch over the same distinct devices
    q64, c64 = q[:100].astype(np.float64), c[:20000].astype(np.float64)
    n.set_devices([])
    want64 = n.topk_host(q64, c64, 100, METRICS[metric])
    n.set_devices(list(range(G)))
    got64 = n.topk_host(q64, c64, 100, METRICS[metric])
    assert np.array_equal(got64[0], want64[0]) and np.array_equal(got64[1].view(np.uint64), want64[1].view(np.uint64))


# ---- the fire-and-forget 256-row bf16 kernel (pmm_bf16_ff_kernel.h,
# PMM_BF16_FF=1): a different kernel structure (256 query rows on one wave per
# SIMD, a guessed static threshold, survivors stored fire-and-forget, re-scored
# and bucketed afterwards, unprovable rows re-run on the shipped kernel) over
# the SAME MFMA chain as the shipped wave-specialised kernel
# (v_mfma_f32_16x16x32_bf16 per 16 x 16 block, K in natural order), so the two
# return the same lists bit for bit: the shipped kernel's cross-check (it
# replaced the lab-only r64 kernel's, which ran the 32x32x16 chain).  Every
# list also passes the bf16 truth check (the exact top-k of the rounded rows
# up to f32 summation order). ----
# The ff kernel is not in the product library: it lives in the test library
# libpmm_ff.so (`make ff`; the product's sources plus the ff kernel), bound
# here as a second ctypes module beside libpmm.so.  The shipped results come
# from libpmm.so, the cross-check's from libpmm_ff.so with PMM_BF16_FF set.
@pytest.fixture(scope="module")
def ffn(pmm):
    import importlib.util

    from polars_matmul import _native as base

    path = os.path.join(os.path.dirname(base.__file__), "libpmm_ff.so")
    assert os.path.exists(path), "libpmm_ff.so not built (make -C polars-matmul_amd ff)"
    spec = importlib.util.spec_from_file_location("polars_matmul._native_ff", base.__file__)
    mod = importlib.util.module_from_spec(spec)
    old = os.environ.get("PMM_LIB")
    os.environ["PMM_LIB"] = "libpmm_ff.so"
    try:
        spec.loader.exec_module(mod)
    finally:
        if old is None:
            os.environ.pop("PMM_LIB", None)
        else:
            os.environ["PMM_LIB"] = old
    assert mod.LIB_PATH.endswith("libpmm_ff.so") and mod.lib() is not base.lib()
    return mod


def _ws_and_ff(q, c, k, metric, monkeypatch, ffn, ff="1"):
    monkeypatch.setenv("PMM_BF16_FF", ff)
    fi, fsc = gpu_topk_bf16(q, c, k, metric, n=ffn)
    monkeypatch.setenv("PMM_BF16_FF", "0")
    wi, wsc = gpu_topk_bf16(q, c, k, metric)
    return (fi, fsc), (wi, wsc)


def test_product_library_has_no_ff_kernel(pmm, ffn, monkeypatch):
    # PMM_BF16_FF has no effect on libpmm.so (the kernel is not compiled in):
    # no "gemm_bf16_topk/ff" launch there, one in the test library
    rs = np.random.RandomState(3)
    q = rs.randn(300, 256).astype(np.float32)
    c = rs.randn(70000, 256).astype(np.float32)
    monkeypatch.setenv("PMM_BF16_FF", "1")
    for lib, want in ((_native(), 0), (ffn, 1)):
        lib.timing_reset()
        lib.timing_enable(True)
        try:
            gpu_topk_bf16(q, c, 10, "cosine", n=lib)
        finally:
            lib.timing_enable(False)
        assert lib.timing_read("gemm_bf16_topk/ff")[1] == want


@pytest.mark.parametrize("m,n,d,k", [(300, 70000, 256, 10), (520, 200000, 768, 100), (257, 131072, 384, 32),
                                     (1000, 100003, 128, 20), (70, 90000, 640, 8), (33, 66000, 500, 16)])
@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
def test_bf16_ff_equals_ws(pmm, ffn, m, n, d, k, metric, monkeypatch):
    rs = np.random.RandomState(m + n + d + k + 13)
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(n, d).astype(np.float32)
    c[n // 2:n // 2 + 20] = c[:20]  # exact ties across the corpus
    q[m // 2] = 0.0                  # a zero-norm query row
    (fi, fsc), (wi, wsc) = _ws_and_ff(q, c, k, metric, monkeypatch, ffn)
    _bf16_truth_check(q, c, k, metric, fi, fsc, f"bf16 ff {m}x{n}x{d} k={k} {metric}")
    assert np.array_equal(fi, wi)
    assert np.array_equal(fsc.view(np.uint32), wsc.view(np.uint32))


@pytest.mark.parametrize("m,n,d,k", [(300, 5000, 256, 10), (70, 3000, 500, 192), (257, 20011, 768, 100),
                                     (1, 1000, 256, 1), (600, 999, 700, 64), (130, 9000, 384, 120)])
@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
def test_bf16_ff_forced_equals_ws_small(pmm, ffn, m, n, d, k, metric, monkeypatch):
    # corpora too short for the ff kernel's guess (PMM_BF16_FF=2 runs it
    # anyway): most rows are re-run on the shipped kernel, the rest must
    # match it bit for bit; odd D (zero-padded to 128), k up to 192, one row
    rs = np.random.RandomState(m + n + d + k + 11)
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(n, d).astype(np.float32)
    c[n // 2:n // 2 + 20] = c[:20]
    q[m // 2] = 0.0
    (fi, fsc), (wi, wsc) = _ws_and_ff(q, c, min(k, n), metric, monkeypatch, ffn, ff="2")
    assert np.array_equal(fi, wi)
    assert np.array_equal(fsc.view(np.uint32), wsc.view(np.uint32))


@pytest.mark.parametrize("metric", ["cosine", "euclidean", "dot"])
def test_bf16_ws_whole_blocks_equal_ff(pmm, ffn, metric, monkeypatch):
    # PMM_CUS=16: 258 query blocks of 128 rows on 16 workgroups, so 256 run
    # whole on the shipped kernel (row state carried across splits) and two
    # as split units; the ff kernel runs split units only: bit-equal
    import torch

    monkeypatch.setenv("PMM_CUS", "16")
    n = _native()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(29)
    m, N, d, k = 33000, 40000, 512, 40
    q = torch.randn((m, d), generator=g, device=dev).to(torch.bfloat16)
    c = torch.randn((N, d), generator=g, device=dev).to(torch.bfloat16)
    outs = []
    for ff in ("2", "0"):
        monkeypatch.setenv("PMM_BF16_FF", ff)
        lib = ffn if ff != "0" else n
        oi = torch.empty((m, k), dtype=torch.int32, device=dev)
        osc = torch.empty((m, k), dtype=torch.float32, device=dev)
        lib.topk_bf16_device(q.data_ptr(), d, m, c.data_ptr(), d, N, d, k, METRICS[metric],
                           oi.data_ptr(), osc.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        outs.append((oi.cpu().numpy(), osc.cpu().numpy()))
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1].view(np.uint32), outs[1][1].view(np.uint32))


def test_bf16_ws_seeded_300k_rows_equal_ff(pmm, ffn, monkeypatch):
    # a corpus long enough for the threshold seed (n >= 8 ns) and for
    # compactions, queue overflows and catch-ups in early tiles: bit-equal
    import torch

    n = _native()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(31)
    m, N, d, k = 2048, 300000, 768, 100
    q = torch.randn((m, d), generator=g, device=dev).to(torch.bfloat16)
    c = torch.randn((N, d), generator=g, device=dev).to(torch.bfloat16)
    outs = []
    for ff in ("1", "0"):
        monkeypatch.setenv("PMM_BF16_FF", ff)
        lib = ffn if ff != "0" else n
        oi = torch.empty((m, k), dtype=torch.int32, device=dev)
        osc = torch.empty((m, k), dtype=torch.float32, device=dev)
        lib.topk_bf16_device(q.data_ptr(), d, m, c.data_ptr(), d, N, d, k, METRICS["cosine"],
                           oi.data_ptr(), osc.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        outs.append((oi.cpu().numpy(), osc.cpu().numpy()))
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1].view(np.uint32), outs[1][1].view(np.uint32))


@pytest.mark.parametrize("knobs", [{"PMM_FF_J": "1"}, {"PMM_FF_CAP": "256"}, {"PMM_FF_J": "1", "PMM_FF_CAP": "64"}])
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_bf16_ff_reruns_rows_it_cannot_prove(pmm, ffn, knobs, metric, monkeypatch):
    # a guess at the sample's best (j = 1: about n / ns scores per row pass,
    # fewer than k for many rows) and/or survivor regions far too small
    # (dropped items): the affected rows must be re-run, and every list must
    # still be the exact top-k of the rounded rows
    rs = np.random.RandomState(71 + len(knobs) + METRICS[metric])
    m, n, d, k = 400, 70000, 256, 60
    q = rs.randn(m, d).astype(np.float32)
    c = rs.randn(n, d).astype(np.float32)
    monkeypatch.setenv("PMM_BF16_FF", "2")  # forced, whatever the guess leaves
    for kk, v in knobs.items():
        monkeypatch.setenv(kk, v)
    fi, fsc = gpu_topk_bf16(q, c, k, metric, n=ffn)
    _bf16_truth_check(q, c, k, metric, fi, fsc, f"bf16 ff rerun {knobs} {metric}")
    for kk in knobs:
        monkeypatch.delenv(kk)
    monkeypatch.setenv("PMM_BF16_FF", "0")
    wi, wsc = gpu_topk_bf16(q, c, k, metric)
    assert np.array_equal(fi, wi)
    assert np.array_equal(fsc.view(np.uint32), wsc.view(np.uint32))


def test_bf16_ff_device_api_whole_problem(pmm, ffn, monkeypatch):
    # the device entry point at a size with several splits per query block:
    # every row vs float64 truth on device, indices distinct
    import torch

    monkeypatch.setenv("PMM_BF16_FF", "1")
    n = ffn
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(37)
    m, N, d, k = 3000, 400000, 768, 100
    q = torch.randn((m, d), generator=g, device=dev).to(torch.bfloat16)
    c = torch.randn((N, d), generator=g, device=dev).to(torch.bfloat16)
    oi = torch.empty((m, k), dtype=torch.int32, device=dev)
    osc = torch.empty((m, k), dtype=torch.float32, device=dev)
    n.topk_bf16_device(q.data_ptr(), d, m, c.data_ptr(), d, N, d, k, METRICS["cosine"],
                       oi.data_ptr(), osc.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    qd, cd = q.double(), c.double()
    s = (qd @ cd.T) / (qd.norm(dim=1, keepdim=True) * cd.norm(dim=1)[None, :])
    ref_s, _ = torch.topk(s, k, dim=1)
    got_true = torch.gather(s, 1, oi.long())
    kth = ref_s[:, -1:]
    ok = got_true >= kth - (1e-5 * kth.abs() + 1e-5)
    assert bool(ok.all()), float(ok.float().mean())
    assert float((osc.double() - got_true).abs().max()) < 1e-4
    srt = torch.sort(oi, dim=1).values
    assert bool((srt[:, 1:] != srt[:, :-1]).all())


@pytest.mark.parametrize("m", [33, 300])
@pytest.mark.parametrize("metric", ["cosine", "euclidean"])
def test_bf16_ws_d128_long_corpus_truth(pmm, m, metric, monkeypatch):
    # padded D = 128 (one K-step per tile) over 2188 tiles: the wave-specialised
    # kernel's survivor drain must run before the column-norm ring overwrites
    # the queued survivors' norms (a 4-tile drain period did not: wrong cosine
    # and euclidean scores in sparsely surviving row groups)
    rs = np.random.RandomState(m + 5)
    q = rs.randn(m, 128).astype(np.float32)
    c = rs.randn(70000, 128).astype(np.float32)
    idx, sc = gpu_topk_bf16(q, c, 50, metric)
    _bf16_truth_check(q, c, 50, metric, idx, sc, f"bf16 ws d128 m={m} {metric}")
