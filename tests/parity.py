"""Parity checks shared by the CPU and GPU tests.

Score parity: |score - truth[row, idx]| <= atol + rtol * |truth| with the
reference's own tolerance (rtol = 1e-5: tests/test_polars_matmul.py:202,
:295; tests/test_performance.py:95).

Index parity is tie-aware: the f32 GEMM of the
reference (faer) and of this build accumulate in different orders, so two
corpus rows whose scores differ by less than the score tolerance may swap.
A returned list passes iff (a) indices are in range and unique per row,
(b) every returned index scores at least the k-th best truth minus the
tolerance, (c) every non-returned index scores at most the k-th best truth
plus the tolerance, and (d) the list is ordered best-first up to the
tolerance.  The strict exact-match rate against the oracle is reported too.
"""
from __future__ import annotations

import numpy as np


def check_topk(idx, score, truth, higher_is_better=True, rtol=1e-5, atol=1e-6, label="",
               scale=None, ulp=2e-6):
    """scale (M x N, optional): per-element magnitude of the f32 dot product
    (|q|*|c|); adds ulp*scale to the tolerance, since an f32 dot of D terms
    carries an absolute error proportional to |q||c|, not to its value."""
    idx = np.asarray(idx).astype(np.int64)
    score = np.asarray(score, dtype=np.float64)
    truth = np.asarray(truth, dtype=np.float64)
    m, k = idx.shape
    n = truth.shape[1]
    assert truth.shape[0] == m, (label, truth.shape, idx.shape)
    if k == 0:
        return
    assert idx.min() >= 0 and idx.max() < n, f"{label}: index out of range"
    r = truth if higher_is_better else -truth
    for i in range(m):
        row = idx[i]
        assert len(set(row.tolist())) == k, f"{label}: duplicate index in row {i}: {row}"
        t = truth[i, row]
        extra = 0.0 if scale is None else ulp * np.asarray(scale)[i]
        tol = atol + rtol * np.abs(t) + (0.0 if scale is None else extra[row])
        bad = np.abs(score[i] - t) > tol
        assert not bad.any(), (
            f"{label}: row {i} score mismatch at {np.nonzero(bad)[0][:5]}: "
            f"got {score[i][bad][:5]} want {t[bad][:5]}"
        )
        rr = r[i]
        kth = np.sort(rr)[::-1][k - 1]
        band = 2 * (atol + rtol * abs(kth) + (0.0 if scale is None else float(np.max(extra))))
        got = rr[row]
        assert got.min() >= kth - band, f"{label}: row {i} returned a non-top-k index"
        mask = np.ones(n, dtype=bool)
        mask[row] = False
        if mask.any():
            assert rr[mask].max() <= kth + band, f"{label}: row {i} missed a top-k index"
        d = np.diff(got)
        order_tol = 2 * (atol + rtol * np.abs(got[1:])) + (0.0 if scale is None else 2 * float(np.max(extra)))
        assert np.all(d <= order_tol), f"{label}: row {i} not ordered best-first"


def exact_match_rate(idx_a, idx_b) -> float:
    a = np.asarray(idx_a)
    b = np.asarray(idx_b)
    if a.size == 0:
        return 1.0
    return float(np.mean(np.all(a == b, axis=1)))


def check_matrix(got, want, rtol=1e-5, atol=1e-6, label=""):
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    assert got.shape == want.shape, (label, got.shape, want.shape)
    np.testing.assert_allclose(got, want, rtol=rtol, atol=atol, err_msg=label)


def dot_scale(q, c):
    """|q_i| * |c_j| in float64 (tolerance scale for f32 dot products)."""
    q = np.asarray(q, dtype=np.float64)
    c = np.asarray(c, dtype=np.float64)
    return np.outer(np.sqrt((q * q).sum(1)), np.sqrt((c * c).sum(1)))


def round_bf16(x: np.ndarray) -> np.ndarray:
    """f32 -> nearest-even bf16, returned as f32 (the device's v_cvt_pk_bf16_f32
    for finite inputs; NaN stays NaN)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    u = x.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    out = r.view(np.float32).copy()
    nan = np.isnan(x)
    out[nan] = np.nan
    return out
