"""Generate the golden fixtures under tests/golden/ (committed with this script).

Two kinds of fixtures, both data only:

1. ``kat.json`` -- the known-answer cases the reference's own tests assert,
   restated as literal inputs and expected outputs (reference file:line in
   each case's "source").  The reference cannot be built or imported here
   (no Rust toolchain, no polars), so its KATs are the
   anchor that pins the CPU oracle.

2. ``rand_*.npz`` -- seeded NumPy inputs generated exactly as the reference's
   tests / benchmark do (legacy ``np.random.seed(42)`` + ``randn``), with the
   expected scores computed independently in float64 NumPy (the reference's
   own tests compare against NumPy at rtol=1e-5:
   tests/test_polars_matmul.py:186-202, :264-296; tests/test_performance.py:78-97;
   examples/benchmark_topk.py:122-138).

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def truth_scores(q: np.ndarray, c: np.ndarray, metric: str) -> np.ndarray:
    """float64 NumPy restatement of the metric (src/metrics.rs:258-311)."""
    q = q.astype(np.float64)
    c = c.astype(np.float64)
    dot = q @ c.T
    if metric == "dot":
        return dot
    if metric == "cosine":
        qn = np.sqrt((q * q).sum(1))
        cn = np.sqrt((c * c).sum(1))
        den = np.outer(qn, cn)
        out = np.where(den > 0, dot / np.where(den > 0, den, 1.0), 0.0)
        out[qn <= 1e-10, :] = 0.0
        out[:, cn <= 1e-10] = 0.0
        return out
    if metric == "euclidean":
        qs = (q * q).sum(1)
        cs = (c * c).sum(1)
        sq = qs[:, None] + cs[None, :] - 2.0 * dot
        return np.sqrt(np.maximum(sq, 0.0))
    raise ValueError(metric)


def kat_cases():
    cases = []
    # tests/test_polars_matmul.py:13-53 -- cosine, q = e0,e1 vs c = I3, k=2
    cases.append(dict(
        name="cosine_basic", source="tests/test_polars_matmul.py:13-53", op="topk",
        q=[[1.0, 0.0, 0.0], [0.0, 1.0, 0.0]], c=[[1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]],
        k=2, metric="cosine", dtype="f64",
        expect_top=[[0, 1.0], [1, 1.0]], expect_len=[2, 2], tol=1e-6))
    # :55-75 explode/unnest -> 4 rows
    cases.append(dict(
        name="explode_unnest", source="tests/test_polars_matmul.py:55-75", op="topk",
        q=[[1.0, 0.0], [0.0, 1.0]], c=[[1.0, 0.0], [0.0, 1.0], [0.5, 0.5]],
        k=2, metric="cosine", dtype="f64", expect_len=[2, 2]))
    # :77-95 dot: q=[2,0], c=[[1,0],[3,0]] -> top (1, 6.0)
    cases.append(dict(
        name="dot_basic", source="tests/test_polars_matmul.py:77-95", op="topk",
        q=[[2.0, 0.0]], c=[[1.0, 0.0], [3.0, 0.0]], k=2, metric="dot", dtype="f64",
        expect_top=[[1, 6.0]], expect_rows=[[[1, 6.0], [0, 2.0]]], tol=1e-6))
    # :97-115 euclidean: q=[0,0], c=[[3,4],[1,0]] -> ascending (1,1.0) then (0,5.0)
    cases.append(dict(
        name="euclidean_basic", source="tests/test_polars_matmul.py:97-115", op="topk",
        q=[[0.0, 0.0]], c=[[3.0, 4.0], [1.0, 0.0]], k=2, metric="euclidean", dtype="f64",
        expect_top=[[1, 1.0]], expect_rows=[[[1, 1.0], [0, 5.0]]], tol=1e-6))
    # :117-133 k > N -> N results
    cases.append(dict(
        name="k_gt_n", source="tests/test_polars_matmul.py:117-133", op="topk",
        q=[[1.0, 0.0]], c=[[1.0, 0.0], [0.0, 1.0]], k=10, metric="cosine", dtype="f64",
        expect_len=[2], expect_rows=[[[0, 1.0], [1, 0.0]]], tol=1e-6))
    # :135-163 join: top-2 of e0 against I3 -> index 0 first
    cases.append(dict(
        name="join_metadata", source="tests/test_polars_matmul.py:135-163", op="topk",
        q=[[1.0, 0.0, 0.0]], c=[[1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]],
        k=2, metric="cosine", dtype="f64", expect_top=[[0, 1.0]], expect_len=[2], tol=1e-6))
    # :169-184 matmul identity
    cases.append(dict(
        name="matmul_basic", source="tests/test_polars_matmul.py:169-184", op="matmul",
        q=[[1.0, 2.0], [3.0, 4.0]], c=[[1.0, 0.0], [0.0, 1.0]], dtype="f64",
        expect=[[1.0, 2.0], [3.0, 4.0]], rtol=1e-5))
    # :204-222 flatten -> [1,0,0,1,1,1]
    cases.append(dict(
        name="matmul_flatten", source="tests/test_polars_matmul.py:204-222", op="matmul",
        q=[[1.0, 0.0], [0.0, 1.0], [1.0, 1.0]], c=[[1.0, 0.0], [0.0, 1.0]], dtype="f64",
        expect=[[1.0, 0.0], [0.0, 1.0], [1.0, 1.0]], expect_flat=[1.0, 0.0, 0.0, 1.0, 1.0, 1.0],
        rtol=1e-5))
    # :241-258 Array input d=4
    cases.append(dict(
        name="matmul_array", source="tests/test_polars_matmul.py:241-258", op="matmul",
        q=[[1.0, 2.0, 3.0, 4.0], [5.0, 6.0, 7.0, 8.0]],
        c=[[1.0, 0.0, 0.0, 0.0], [0.0, 1.0, 0.0, 0.0]], dtype="f64",
        expect=[[1.0, 2.0], [5.0, 6.0]], rtol=1e-5))
    # :369-387 f32 matmul
    cases.append(dict(
        name="matmul_f32", source="tests/test_polars_matmul.py:369-387", op="matmul",
        q=[[1.0, 2.0], [3.0, 4.0]], c=[[1.0, 0.0], [0.0, 1.0]], dtype="f32",
        expect=[[1.0, 2.0], [3.0, 4.0]], rtol=1e-5))
    # :449-464 f32 Array d=8
    cases.append(dict(
        name="matmul_f32_array", source="tests/test_polars_matmul.py:449-464", op="matmul",
        q=[[1.0] * 8, [2.0] * 8], c=[[1.0] * 8, [0.5] * 8], dtype="f32",
        expect=[[8.0, 4.0], [16.0, 8.0]], rtol=1e-5))
    # :753-768 f32 Array topk d=8 (k=1): rows [1]*8,[2]*8,[0.5]*8 vs [1]*8,[0]*8
    cases.append(dict(
        name="topk_f32_array_zero_corpus_row", source="tests/test_polars_matmul.py:753-768",
        op="topk", q=[[1.0] * 8, [2.0] * 8, [0.5] * 8], c=[[1.0] * 8, [0.0] * 8], k=1,
        metric="cosine", dtype="f32", expect_rows=[[[0, 1.0]], [[0, 1.0]], [[0, 1.0]]], tol=1e-6))
    # src/metrics.rs:401-411 dot f64 2x3
    cases.append(dict(
        name="rust_dot_f64", source="src/metrics.rs:401-411", op="similarity",
        q=[[1.0, 0.0], [0.0, 1.0]], c=[[1.0, 0.0], [0.0, 1.0], [1.0, 1.0]], metric="dot",
        dtype="f64", expect_cells=[[0, 0, 1.0], [0, 1, 0.0], [1, 1, 1.0]], tol=1e-10))
    # src/metrics.rs:413-423 dot f32
    cases.append(dict(
        name="rust_dot_f32", source="src/metrics.rs:413-423", op="similarity",
        q=[[1.0, 0.0], [0.0, 1.0]], c=[[1.0, 0.0], [0.0, 1.0], [1.0, 1.0]], metric="dot",
        dtype="f32", expect_cells=[[0, 0, 1.0], [0, 1, 0.0], [1, 1, 1.0]], tol=1e-5))
    # src/metrics.rs:425-434 cosine f64 2x2
    cases.append(dict(
        name="rust_cosine_f64", source="src/metrics.rs:425-434", op="similarity",
        q=[[1.0, 0.0], [0.0, 1.0]], c=[[2.0, 0.0], [0.0, 3.0]], metric="cosine", dtype="f64",
        expect_cells=[[0, 0, 1.0], [1, 1, 1.0], [1, 0, 0.0]], tol=1e-10))
    # src/topk.rs:83-125 select on a fixed matrix
    cases.append(dict(
        name="rust_select_higher", source="src/topk.rs:83-97,99-111", op="select",
        s=[[0.1, 0.9, 0.5], [0.8, 0.2, 0.6]], k=2, higher_is_better=True,
        expect_idx=[[1, 2], [0, 2]]))
    cases.append(dict(
        name="rust_select_lower", source="src/topk.rs:113-125", op="select",
        s=[[0.1, 0.9, 0.5], [0.8, 0.2, 0.6]], k=2, higher_is_better=False,
        expect_idx=[[0, 2], [1, 2]]))
    return cases


def main():
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump({"cases": kat_cases()}, f, indent=1)

    # tests/test_polars_matmul.py:264-296: seed 42, randn(5,16) vs randn(20,16), cosine, k=20
    np.random.seed(42)
    q = np.random.randn(5, 16)
    c = np.random.randn(20, 16)
    np.savez(os.path.join(HERE, "rand_ref_cosine_5x20x16.npz"), q=q, c=c,
             cosine=truth_scores(q, c, "cosine"))

    # tests/test_polars_matmul.py:186-202 and tests/test_performance.py:78-97:
    # seed 42, randn(10,32) vs randn(20,32), matmul f64
    np.random.seed(42)
    q = np.random.randn(10, 32)
    c = np.random.randn(20, 32)
    np.savez(os.path.join(HERE, "rand_ref_matmul_10x20x32.npz"), q=q, c=c, dot=q @ c.T)

    # examples/benchmark_topk.py:193-203 correctness verification: seed 42,
    # randn(100,64) vs randn(500,64) f64, cosine k=10
    np.random.seed(42)
    q = np.random.randn(100, 64)
    c = np.random.randn(500, 64)
    np.savez(os.path.join(HERE, "rand_bench_verify_100x500x64.npz"), q=q, c=c,
             cosine=truth_scores(q, c, "cosine"))

    # examples/benchmark_topk.py:69-71 generation (seed 42, randn -> f32) at a
    # reduced size, all three metrics, with f64 truth on the f32 inputs
    np.random.seed(42)
    q = np.random.randn(48, 256).astype(np.float32)
    c = np.random.randn(1000, 256).astype(np.float32)
    np.savez(os.path.join(HERE, "rand_f32_48x1000x256.npz"), q=q, c=c,
             cosine=truth_scores(q, c, "cosine"), dot=truth_scores(q, c, "dot"),
             euclidean=truth_scores(q, c, "euclidean"))

    # edge fixture: zero-norm query and corpus rows, exact duplicates (ties),
    # ragged d (not a multiple of 32)
    rs = np.random.RandomState(7)
    q = rs.randn(6, 37).astype(np.float32)
    c = rs.randn(70, 37).astype(np.float32)
    q[2] = 0.0
    c[5] = 0.0
    c[11] = c[3]
    c[40] = c[3]
    c[12] = 2.0 * c[4]
    np.savez(os.path.join(HERE, "edge_f32_6x70x37.npz"), q=q, c=c,
             cosine=truth_scores(q, c, "cosine"), dot=truth_scores(q, c, "dot"),
             euclidean=truth_scores(q, c, "euclidean"))


if __name__ == "__main__":
    main()
