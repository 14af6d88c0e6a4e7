"""
polars-matmul (MI355X-native): similarity search for Polars embedding columns.

Drop-in for the reference package ``polars_matmul`` (NivekNey/polars-matmul
v0.1.4): importing it registers the ``pmm`` expression namespace on Polars
(python/polars_matmul/__init__.py:39 in the reference) with the same
``topk(corpus, k, metric)`` and ``matmul(corpus, flatten)`` methods, result
dtypes and errors.  The numerics run on MI355X through hand-written HIP
kernels (``libpmm.so``, C ABI in ``include/pmm.h``); there is no CPU path.

Usage:
    >>> import polars as pl
    >>> import polars_matmul  # registers the .pmm namespace
    >>> queries.with_columns(pl.col("embedding").pmm.topk(corpus["embedding"], k=2))

Without Polars, the same extension functions accept pyarrow arrays or numpy
matrices (``polars_matmul._polars_matmul._topk``), and ``topk`` / ``matmul``
below are numpy-level conveniences.

Multi-GPU (an extension; the reference is single-process): ``set_devices([0,
1, ..., 7])`` -- or ``PMM_DEVICES=all`` / ``PMM_DEVICES=0,1,2,3`` in the
environment -- row-shards the corpus of every later ``.pmm.topk`` over those
GPUs inside the one Polars process and merges the per-GPU lists on the first
(include/pmm.h ``pmm_set_devices``); results are identical to one GPU's.
"""
from __future__ import annotations

from typing import Literal

import numpy as np

from polars_matmul._polars_matmul import (  # noqa: F401
    PanicException,
    _matmul,
    _topk,
    get_devices,
    set_devices,
)
from polars_matmul import _native

__version__ = "0.1.4"
__all__ = ["PmmNamespace", "topk", "matmul", "set_devices", "get_devices"]

Metric = Literal["cosine", "dot", "euclidean"]
Compute = Literal["f32", "bf16"]

try:
    import polars as pl  # type: ignore
except Exception:  # polars is optional (not installable in this image)
    pl = None


def topk(queries: np.ndarray, corpus: np.ndarray, k: int, metric: Metric = "cosine",
         compute: Compute = "f32"):
    """numpy-level top-k: returns (indices uint32 [m, k'], scores float64 [m, k'])
    with k' = min(k, len(corpus)); f32 compute iff both inputs are float32
    (src/matmul.rs:427), scores widened to f64 (src/matmul.rs:447).
    compute="bf16" (an extension, not in the reference): f32 inputs rounded to
    bf16 on the device, bf16 MFMA with f32 accumulation (include/pmm.h
    PMM_COMPUTE_BF16: the bf16 kernels up to d = 768 and k = 960, the rounded
    rows widened to f32 beyond)."""
    q = np.asarray(queries)
    c = np.asarray(corpus)
    if compute not in ("f32", "bf16"):
        raise ValueError(f"compute must be 'f32' or 'bf16', not {compute!r}")
    dt = np.float32 if (q.dtype == np.float32 and c.dtype == np.float32) else np.float64
    if compute == "bf16":
        dt = np.float32
    q = np.ascontiguousarray(q, dtype=dt)
    c = np.ascontiguousarray(c, dtype=dt)
    if q.shape[1] != c.shape[1]:
        raise RuntimeError(
            f"Dimension mismatch: left has {q.shape[1]} dimensional vectors, "
            f"right has {c.shape[1]} dimensional vectors"
        )
    kk = min(int(k), c.shape[0])
    mode = _native.COMPUTE_BF16 if compute == "bf16" else _native.COMPUTE_F32
    idx, sc = _native.topk_host(q, c, kk, _native.metric_from_str(metric), compute=mode)
    return idx, sc.astype(np.float64, copy=False)


def matmul(queries: np.ndarray, corpus: np.ndarray) -> np.ndarray:
    """numpy-level Q @ C^T on the GPU (f32 iff both inputs are float32)."""
    q = np.asarray(queries)
    c = np.asarray(corpus)
    dt = np.float32 if (q.dtype == np.float32 and c.dtype == np.float32) else np.float64
    return _native.matmul_host(np.ascontiguousarray(q, dtype=dt), np.ascontiguousarray(c, dtype=dt))


if pl is not None:

    @pl.api.register_expr_namespace("pmm")
    class PmmNamespace:
        """Polars Expression API for similarity search (reference
        python/polars_matmul/__init__.py:39-196)."""

        def __init__(self, expr: "pl.Expr"):
            self._expr = expr

        def topk(self, corpus: "pl.Series", k: int, metric: Metric = "cosine") -> "pl.Expr":
            """Top-k matches per embedding: List[Struct{index: u32, score: f64}]."""
            if isinstance(corpus, pl.Expr):
                raise TypeError(
                    "corpus must be a Polars Series, not an Expression. "
                    "Use corpus['column_name'] or corpus.get_column('column_name')."
                )
            return self._expr.map_batches(
                lambda s: _topk(s, corpus, k, metric),
                is_elementwise=True,
                return_dtype=pl.List(pl.Struct({"index": pl.UInt32, "score": pl.Float64})),
            )

        def matmul(self, corpus: "pl.Series", flatten: bool = False) -> "pl.Expr":
            """All pairwise dot products: Array[f32|f64, N] per row, or one flat
            column (row-major) with flatten=True."""
            if isinstance(corpus, pl.Expr):
                raise TypeError(
                    "corpus must be a Polars Series, not an Expression. "
                    "Use corpus['column_name'] or corpus.get_column('column_name')."
                )
            n_corpus = len(corpus)
            try:
                is_f32 = corpus.dtype.inner == pl.Float32
            except Exception:
                is_f32 = False
            if flatten:
                inner_dtype = pl.Float32 if is_f32 else pl.Float64

                def _matmul_flatten(s: "pl.Series") -> "pl.Series":
                    return _matmul(s, corpus).explode()

                return self._expr.map_batches(
                    _matmul_flatten, is_elementwise=False, return_dtype=inner_dtype
                )
            dtype = pl.Array(pl.Float32 if is_f32 else pl.Float64, n_corpus)
            return self._expr.map_batches(
                lambda s: _matmul(s, corpus), is_elementwise=True, return_dtype=dtype
            )

else:

    class PmmNamespace:  # type: ignore[no-redef]
        """Placeholder: Polars is not importable, so no namespace is registered."""

        def __init__(self, *_a, **_k):
            raise ImportError("polars is not installed; use polars_matmul._topk / topk instead")
