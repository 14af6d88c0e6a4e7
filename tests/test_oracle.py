"""Pin the CPU oracle (oracle/pmm_oracle.c) against the reference's known
answers and the NumPy fixtures (tests/golden/).  CPU only."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

import oracle
from parity import check_matrix, check_topk, dot_scale

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
METRICS = {"cosine": oracle.COSINE, "dot": oracle.DOT, "euclidean": oracle.EUCLIDEAN}


def load_kats():
    with open(os.path.join(GOLD, "kat.json")) as f:
        return json.load(f)["cases"]


def _dt(case):
    return np.float32 if case.get("dtype") == "f32" else np.float64


@pytest.mark.parametrize("case", [c for c in load_kats() if c["op"] == "topk"], ids=lambda c: c["name"])
def test_oracle_topk_kat(case):
    dt = _dt(case)
    q = np.array(case["q"], dtype=dt)
    c = np.array(case["c"], dtype=dt)
    idx, sc = oracle.topk(q, c, case["k"], METRICS[case["metric"]])
    if "expect_len" in case:
        assert [idx.shape[1]] * idx.shape[0] == case["expect_len"]
    tol = case.get("tol", 1e-6)
    for i, (ei, es) in enumerate(case.get("expect_top", [])):
        assert idx[i, 0] == ei
        assert abs(sc[i, 0] - es) < tol
    for i, row in enumerate(case.get("expect_rows", [])):
        for j, (ei, es) in enumerate(row):
            assert idx[i, j] == ei, (case["name"], i, j, idx[i])
            assert abs(sc[i, j] - es) < tol


@pytest.mark.parametrize("case", [c for c in load_kats() if c["op"] == "matmul"], ids=lambda c: c["name"])
def test_oracle_matmul_kat(case):
    dt = _dt(case)
    out = oracle.matmul(np.array(case["q"], dtype=dt), np.array(case["c"], dtype=dt))
    assert out.dtype == dt
    check_matrix(out, case["expect"], rtol=case["rtol"], atol=0)
    if "expect_flat" in case:
        np.testing.assert_allclose(out.reshape(-1), case["expect_flat"], rtol=case["rtol"])


@pytest.mark.parametrize("case", [c for c in load_kats() if c["op"] == "similarity"], ids=lambda c: c["name"])
def test_oracle_similarity_kat(case):
    dt = _dt(case)
    s = oracle.similarity(np.array(case["q"], dtype=dt), np.array(case["c"], dtype=dt), METRICS[case["metric"]])
    for i, j, v in case["expect_cells"]:
        assert abs(s[i, j] - v) < case["tol"]


@pytest.mark.parametrize("case", [c for c in load_kats() if c["op"] == "select"], ids=lambda c: c["name"])
@pytest.mark.parametrize("algo", ["total", "rust"])
def test_oracle_select_kat(case, algo):
    # the Rust-select restatement (the CPU baseline's select) must pass the
    # reference's own select KATs too (src/topk.rs:83-125: no ties there)
    for dt in (np.float32, np.float64):
        idx, _ = oracle.select_topk(np.array(case["s"], dtype=dt), case["k"], case["higher_is_better"], algo=algo)
        assert idx.tolist() == case["expect_idx"]


@pytest.mark.parametrize("m,n,k", [(40, 10000, 10), (20, 1000, 1), (20, 1000, 1000), (30, 5000, 100),
                                   (5, 17, 16), (5, 17, 17), (7, 3, 2), (3, 100000, 100)])
def test_rust_select_equals_checker_select(m, n, k):
    # the baseline's select (Rust's select_nth_unstable_by
    # + stable sort_by, restated in pmm_oracle.c) keeps the same k best scores
    # in the same order as the checker's total-order select; only the order of
    # equal scores may differ (unspecified in the reference, src/topk.rs:55-59)
    rs = np.random.RandomState(m + n + k)
    for dt in (np.float32, np.float64):
        s = rs.randn(m, n).astype(dt)
        s[:, ::7] = s[:, :1]  # runs of equal scores (the equal-pivot path)
        for hib in (True, False):
            i1, s1 = oracle.select_topk(s, k, hib)
            i2, s2 = oracle.select_topk(s, k, hib, algo="rust")
            assert np.array_equal(s1, s2), (dt, hib)
            assert np.array_equal(np.take_along_axis(s, i2.astype(np.int64), 1), s2)
            assert all(len(set(r)) == k for r in i2.tolist())


def test_oracle_metric_parse():
    # src/metrics.rs:20-27
    assert oracle.metric_from_str("cosine") == oracle.COSINE
    assert oracle.metric_from_str("COSINE") == oracle.COSINE
    assert oracle.metric_from_str("Dot") == oracle.DOT
    assert oracle.metric_from_str("euclidean") == oracle.EUCLIDEAN
    assert oracle.metric_from_str("l2") == oracle.EUCLIDEAN
    assert oracle.metric_from_str("L2") == oracle.EUCLIDEAN
    assert oracle.metric_from_str("invalid_metric") == -1
    assert oracle.metric_from_str("") == -1


def test_oracle_ref_cosine_all_k():
    # tests/test_polars_matmul.py:264-296: sorted scores match NumPy at rtol=1e-5
    z = np.load(os.path.join(GOLD, "rand_ref_cosine_5x20x16.npz"))
    idx, sc = oracle.topk(z["q"], z["c"], 20, oracle.COSINE)
    for i in range(5):
        np.testing.assert_allclose(sc[i], np.sort(z["cosine"][i])[::-1], rtol=1e-5)
    check_topk(idx, sc, z["cosine"], True, label="ref_cosine")


def test_oracle_ref_matmul():
    # tests/test_polars_matmul.py:186-202
    z = np.load(os.path.join(GOLD, "rand_ref_matmul_10x20x32.npz"))
    check_matrix(oracle.matmul(z["q"], z["c"]), z["dot"], rtol=1e-5, atol=0)
    check_matrix(oracle.matmul(z["q"].astype(np.float32), z["c"].astype(np.float32)), z["dot"], rtol=1e-4, atol=1e-5)


def test_oracle_bench_verify():
    # examples/benchmark_topk.py:122-138 + :191-203 (rtol 1e-4 on sorted scores)
    z = np.load(os.path.join(GOLD, "rand_bench_verify_100x500x64.npz"))
    idx, sc = oracle.topk(z["q"], z["c"], 10, oracle.COSINE)
    want = -np.sort(-z["cosine"], axis=1)[:, :10]
    np.testing.assert_allclose(sc, want, rtol=1e-4)
    check_topk(idx, sc, z["cosine"], True, label="bench_verify")


@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
@pytest.mark.parametrize("k", [1, 10, 100, 1000])
def test_oracle_f32_fixture(metric, k):
    z = np.load(os.path.join(GOLD, "rand_f32_48x1000x256.npz"))
    idx, sc = oracle.topk(z["q"], z["c"], k, METRICS[metric])
    assert idx.shape == (48, min(k, 1000))
    scale = dot_scale(z["q"], z["c"]) if metric == "dot" else None
    check_topk(idx, sc, z[metric], metric != "euclidean", rtol=1e-5, atol=1e-5, label=f"f32 {metric}",
               scale=scale)


@pytest.mark.parametrize("metric", ["cosine", "dot", "euclidean"])
def test_oracle_edge_fixture(metric):
    z = np.load(os.path.join(GOLD, "edge_f32_6x70x37.npz"))
    idx, sc = oracle.topk(z["q"], z["c"], 70, METRICS[metric])
    scale = dot_scale(z["q"], z["c"]) if metric == "dot" else None
    check_topk(idx, sc, z[metric], metric != "euclidean", rtol=1e-5, atol=1e-5, label=f"edge {metric}",
               scale=scale)
    if metric == "cosine":
        # zero-norm query row -> all scores 0.0, ties broken by lower index
        assert np.all(sc[2] == 0.0)
        assert idx[2].tolist() == list(range(70))
        # zero-norm corpus row scores exactly 0
        for i in range(6):
            pos = int(np.nonzero(idx[i] == 5)[0][0])
            assert sc[i, pos] == 0.0
    # exact duplicates c[3] == c[11] == c[40]: equal scores, lower index first
    for i in range(6):
        row = idx[i].tolist()
        assert row.index(3) < row.index(11) < row.index(40)


def _unrolled_dot_py(x):
    """Pure-Python restatement of ndarray 0.16 unrolled_dot on f32 (small sizes)."""
    f = np.float32
    p = [f(0)] * 8
    n = len(x)
    i = 0
    while i + 8 <= n:
        for j in range(8):
            p[j] = f(p[j] + f(x[i + j] * x[i + j]))
        i += 8
    s = f(0)
    s = f(s + f(p[0] + p[4]))
    s = f(s + f(p[1] + p[5]))
    s = f(s + f(p[2] + p[6]))
    s = f(s + f(p[3] + p[7]))
    while i < n:
        s = f(s + f(x[i] * x[i]))
        i += 1
    return s


def test_oracle_norms_ndarray_order():
    rs = np.random.RandomState(3)
    a = rs.randn(9, 45).astype(np.float32) * 3
    sq = oracle.norms(a, squared=True)
    nr = oracle.norms(a, squared=False)
    for r in range(a.shape[0]):
        want = _unrolled_dot_py(a[r].tolist() and a[r])
        assert sq[r] == want
        assert nr[r] == np.sqrt(want, dtype=np.float32)


def test_oracle_k_zero_and_nan_order():
    q = np.array([[1.0, 0.0]], dtype=np.float32)
    c = np.array([[np.nan, 0.0], [1.0, 0.0], [0.5, 0.0]], dtype=np.float32)
    idx, sc = oracle.topk(q, c, 0, oracle.DOT)
    assert idx.shape == (1, 0)
    idx, sc = oracle.topk(q, c, 3, oracle.DOT)
    # NaN ranks last (the reference leaves its placement unspecified)
    assert idx[0].tolist() == [1, 2, 0]
    assert np.isnan(sc[0, 2])
