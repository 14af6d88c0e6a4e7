"""``polars_matmul._polars_matmul`` -- the extension-module surface of the reference
(src/lib.rs:15-62, module path pyproject.toml:114), re-implemented over the HIP
C ABI.  Exports ``_topk(left, right, k, metric)`` and ``_matmul(left, right)``
with the reference's argument meaning, result dtypes, error texts and edge
rules:

* input extraction / marshalling ..... src/matmul.rs:12-286
* ``_matmul`` -> ``matmul_impl`` ...... src/matmul.rs:295-417
* ``_topk``   -> ``topk_impl`` ........ src/matmul.rs:420-519

Inputs may be a Polars ``Series`` (``List``/``Array`` of floats; converted with
``rechunk().to_arrow()``, zero-copy for ``Array[f32|f64]``), a pyarrow
``(Large)List`` / ``FixedSizeList`` array or chunked array, or a 2-D numpy
array.  The result is a Polars ``Series`` when Polars is importable and the
query input was a Polars ``Series``, otherwise a pyarrow array of the same
logical type:

* ``_topk``   -> ``List[Struct{index: UInt32, score: Float64}]`` named "topk"
* ``_matmul`` -> ``Array[Float32|Float64, N]`` named "matmul"

Errors: the reference maps ``PolarsError`` to ``RuntimeError`` (src/lib.rs:28,
53); the same message texts are raised here.  A negative ``k`` raises
``OverflowError`` (pyo3's usize conversion); a List row longer than the first
row raises ``PanicException`` (the reference panics on the ndarray index,
src/matmul.rs:276-283).
"""
from __future__ import annotations

import collections
import os
import threading
import time

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc

from . import _native

try:  # Polars is optional: the HIP path does not need it.
    import polars as _pl  # type: ignore
except Exception:  # pragma: no cover - polars is not installed in this image
    _pl = None


# Host-side phase timer for bench.py's end-to-end breakdown: when set to a
# dict, _topk / _matmul add the seconds of each phase (extract: Arrow/numpy ->
# contiguous matrices; device: the C-ABI call -- upload, kernels, download;
# assemble: result dtype widening and Arrow assembly).  None (default): off.
PHASES = None


def _lap(name: str, t0: float) -> float:
    t = time.perf_counter()
    ph = PHASES
    if ph is not None:
        ph[name] = ph.get(name, 0.0) + (t - t0)
    return t


class PanicException(BaseException):
    """Mirror of pyo3's PanicException (a BaseException subclass)."""


def _compute_error(msg: str) -> RuntimeError:
    return RuntimeError(msg)


# ---------------------------------------------------------------------------
# Input normalisation
# ---------------------------------------------------------------------------
def _is_polars_series(obj) -> bool:
    return _pl is not None and isinstance(obj, _pl.Series)


def _to_arrow(obj):
    """Return a single-chunk pyarrow Array (List / LargeList / FixedSizeList) or a
    2-D numpy array."""
    if _is_polars_series(obj):
        obj = obj.rechunk().to_arrow()
    if isinstance(obj, np.ndarray):
        if obj.ndim != 2:
            raise TypeError(f"expected a 2-D array of embeddings, got shape {obj.shape}")
        return obj
    if isinstance(obj, pa.ChunkedArray):
        obj = obj.combine_chunks() if obj.num_chunks != 1 else obj.chunk(0)
    if isinstance(obj, pa.Array):
        return obj
    if isinstance(obj, (list, tuple)):
        return pa.array(obj)
    raise TypeError(f"unsupported embedding container: {type(obj).__name__}")


def _is_f32(arr) -> bool:
    """src/matmul.rs:13-19: List[f32] or Array[f32, d]."""
    if isinstance(arr, np.ndarray):
        return arr.dtype == np.float32
    t = arr.type
    if pa.types.is_list(t) or pa.types.is_large_list(t) or pa.types.is_fixed_size_list(t):
        return t.value_type == pa.float32()
    return False


def _nrows(arr) -> int:
    return arr.shape[0] if isinstance(arr, np.ndarray) else len(arr)


def _values_numpy(values: pa.Array, np_dtype) -> np.ndarray:
    """Child values cast to the compute dtype, nulls -> 0.0 (src/matmul.rs:192, 224)."""
    target = pa.float32() if np_dtype == np.float32 else pa.float64()
    if values.type != target:
        values = pc.cast(values, target)
    if values.null_count:
        values = values.fill_null(0.0)
    return values.to_numpy(zero_copy_only=False)


def _series_to_matrix(arr, np_dtype) -> np.ndarray:
    """series_to_matrix{,_f32} (src/matmul.rs:131-286): a C-contiguous (rows, d)
    matrix of the compute dtype.  Zero-copy when the input is already a
    contiguous Array of that dtype (src/matmul.rs:22-95)."""
    n = _nrows(arr)
    if n == 0:
        raise _compute_error("Empty series")
    if isinstance(arr, np.ndarray):
        if arr.shape[1] == 0:
            raise _compute_error("Zero-dimensional vectors")
        return np.ascontiguousarray(arr, dtype=np_dtype)
    t = arr.type
    if pa.types.is_fixed_size_list(t):
        d = t.list_size
        if d == 0:
            raise _compute_error("Zero-dimensional vectors")
        child = arr.values.slice(arr.offset * d, n * d)
        if arr.null_count == 0:
            vals = _values_numpy(child, np_dtype)
            return np.ascontiguousarray(vals.reshape(n, d))
        # null outer rows carry null children in Polars: they read as zeros
        vals = _values_numpy(child, np_dtype).reshape(n, d).copy()
        valid = np.asarray(arr.is_valid().to_numpy(zero_copy_only=False), dtype=bool)
        vals[~valid] = 0
        return vals
    if pa.types.is_list(t) or pa.types.is_large_list(t):
        if not arr[0].is_valid:
            raise _compute_error("First element is null")
        offsets = np.asarray(arr.offsets.to_numpy(zero_copy_only=False), dtype=np.int64)
        lens = np.diff(offsets)
        d = int(lens[0])
        if d == 0:
            raise _compute_error("Zero-dimensional vectors")
        valid = (
            np.asarray(arr.is_valid().to_numpy(zero_copy_only=False), dtype=bool)
            if arr.null_count
            else np.ones(n, dtype=bool)
        )
        lens = np.where(valid, lens, 0)
        if np.any(lens > d):
            bad = int(np.argmax(lens > d))
            raise PanicException(
                f"ndarray: index out of bounds: row {bad} has {int(lens[bad])} elements, "
                f"the first row has {d}"
            )
        lo, hi = int(offsets[0]), int(offsets[-1])
        vals = _values_numpy(arr.values.slice(lo, hi - lo), np_dtype)
        if valid.all() and np.all(lens == d):
            return np.ascontiguousarray(vals.reshape(n, d))
        out = np.zeros((n, d), dtype=np_dtype)
        rows = np.repeat(np.arange(n), lens)
        starts = offsets[:-1] - lo
        cols = np.arange(rows.size) - np.repeat(np.cumsum(lens) - lens, lens)
        src = np.repeat(starts, lens) + cols
        out[rows, cols] = vals[src]
        return out
    raise _compute_error(f"expected List or Array of numbers, got {t}")


def _dim_mismatch(dl: int, dr: int) -> RuntimeError:
    return _compute_error(
        f"Dimension mismatch: left has {dl} dimensional vectors, "
        f"right has {dr} dimensional vectors"
    )


def _as_usize(k) -> int:
    if isinstance(k, bool) or not isinstance(k, (int, np.integer)):
        raise TypeError(f"'{type(k).__name__}' object cannot be interpreted as an integer")
    k = int(k)
    if k < 0:
        raise OverflowError("can't convert negative int to unsigned")
    return k


# ---------------------------------------------------------------------------
# Device-resident corpus cache, for both branches of the
# reference (f32 and f64 rows; src/matmul.rs:427-468).  Polars' map_batches may
# call _topk repeatedly with the same corpus Series.  Only corpora that came
# in as Polars Series or Arrow arrays are cached (their buffers persist across
# calls; a Python list or numpy matrix is rebuilt or mutable, so it would only
# fill the cache), identified by the buffers' addresses and sizes while the
# cache holds a reference to the Arrow array (the addresses cannot be reused
# meanwhile).  Arrow data is immutable by contract: a Series that shares
# memory with a numpy array the caller then writes to in place gives stale
# cached results -- clear_corpus_cache() or PMM_CORPUS_CACHE=0 in that case.
# PMM_CORPUS_CACHE_BYTES bounds the HBM the cache holds (default 8 GiB), and
# a corpus is cached only while it takes at most half of the device's free HBM
# (pmm_device_memory), so the cache never crowds out the searches themselves.
# Handles are reference-counted (DeviceCorpus.acquire/release), so evicting
# or clearing never frees a corpus another thread is searching.
# ---------------------------------------------------------------------------

_cache_lock = threading.Lock()
_cache: "collections.OrderedDict" = collections.OrderedDict()
_CACHE_ON = os.environ.get("PMM_CORPUS_CACHE", "1") != "0"
_CACHE_BYTES = int(os.environ.get("PMM_CORPUS_CACHE_BYTES", str(8 << 30)))
_CACHE_MIN_BYTES = 1 << 20  # small corpora are cheaper to upload than to cache


def _fits_device(nbytes: int) -> bool:
    try:
        free, _ = _native.device_memory()
    except _native.PmmError:
        return False
    return nbytes <= free // 2


def _arrow_key(arr):
    if not isinstance(arr, pa.Array):
        return None
    bufs = tuple((b.address, b.size) if b is not None else None for b in arr.buffers())
    return (str(arr.type), arr.offset, len(arr), bufs)


def _cached_corpus(original, rv, c: np.ndarray):
    """An ACQUIRED DeviceCorpus for this corpus (the caller releases it), or
    None when the corpus is not cacheable."""
    # Only inputs whose Arrow buffers persist across calls: a single-chunk
    # Polars Series (rechunk() then returns the same buffers; a multi-chunk
    # one is concatenated into a fresh buffer on every call, whose address
    # key would never hit while each miss pinned host and device memory), an
    # Arrow array, or a single-chunk ChunkedArray.
    if _is_polars_series(original):
        if original.n_chunks() != 1:
            return None
    elif not (isinstance(original, pa.Array)
              or (isinstance(original, pa.ChunkedArray) and original.num_chunks == 1)):
        return None
    key = _arrow_key(rv)
    if key is not None:
        # the compute dtype: an f32 column searched by f64 queries runs the
        # f64 branch (src/matmul.rs:427) on an f64 copy of the same buffers;
        # a handle is sharded over the device list of its creation
        key = key + (c.dtype.str, tuple(_native.get_devices()))
    dev_bytes = _native.corpus_device_bytes(c.shape[0], c.shape[1], c.dtype)
    if not _CACHE_ON or key is None or c.nbytes < _CACHE_MIN_BYTES or dev_bytes > _CACHE_BYTES:
        return None
    with _cache_lock:
        hit = _cache.get(key)
        if hit is not None:
            _cache.move_to_end(key)
            return hit[1].acquire()
        if not _fits_device(dev_bytes):
            return None
        dc = _native.DeviceCorpus(c)
        _cache[key] = (rv, dc)
        total = sum(v[1].nbytes for v in _cache.values())
        while total > _CACHE_BYTES and len(_cache) > 1:
            _, (_, old) = _cache.popitem(last=False)
            total -= old.nbytes
            old.close()  # freed now, or by its last in-flight user
        return dc.acquire()


def clear_corpus_cache() -> None:
    with _cache_lock:
        while _cache:
            _, (_, dc) = _cache.popitem()
            dc.close()


# ---------------------------------------------------------------------------
# Device list (multi-GPU through the drop-in: include/pmm.h pmm_set_devices).
# PMM_DEVICES = "all" or a comma list is applied on the first top-k call (not
# at import: counting devices initialises the HIP runtime).
# ---------------------------------------------------------------------------
_devices_env_done = False


def _parse_devices(spec: str, count: int):
    spec = spec.strip().lower()
    if spec in ("", "0-0"):
        return []
    if spec == "all":
        return list(range(count))
    return [int(x) for x in spec.split(",") if x.strip()]


def _apply_devices_env() -> None:
    global _devices_env_done
    if _devices_env_done:
        return
    _devices_env_done = True
    spec = os.environ.get("PMM_DEVICES")
    if spec:
        set_devices(_parse_devices(spec, _native.device_count()))


def set_devices(ids) -> None:
    """Row-shard the corpus of later top-k calls over these GPUs (results
    merged on the first, identical to one GPU's); [] = one GPU."""
    global _devices_env_done
    _devices_env_done = True  # an explicit choice overrides PMM_DEVICES
    _native.set_devices(list(ids))


def get_devices():
    return _native.get_devices()


# ---------------------------------------------------------------------------
# Output builders
# ---------------------------------------------------------------------------
_TOPK_STRUCT = pa.struct([("index", pa.uint32()), ("score", pa.float64())])


def _topk_arrow(idx: np.ndarray, scores: np.ndarray, m: int, k: int) -> pa.Array:
    struct = pa.StructArray.from_arrays(
        [pa.array(idx.reshape(-1), type=pa.uint32()), pa.array(scores.reshape(-1), type=pa.float64())],
        fields=list(_TOPK_STRUCT),
    )
    offsets = np.arange(m + 1, dtype=np.int64) * k
    return pa.LargeListArray.from_arrays(pa.array(offsets, type=pa.int64()), struct)


def _wrap(arrow_arr: pa.Array, name: str, polars_out: bool):
    if polars_out:
        return _pl.Series(name, arrow_arr)
    return arrow_arr


# ---------------------------------------------------------------------------
# Public extension functions
# ---------------------------------------------------------------------------
def _topk(left, right, k, metric):
    """src/lib.rs:33-55 -> src/matmul.rs:473-519 topk_impl."""
    k = _as_usize(k)
    if not isinstance(metric, str):
        raise TypeError(f"argument 'metric': '{type(metric).__name__}' object cannot be converted to 'PyString'")
    polars_out = _is_polars_series(left)
    t = time.perf_counter()
    lv = _to_arrow(left)
    rv = _to_arrow(right)
    if _nrows(lv) == 0:  # src/matmul.rs:480-487
        empty = pa.array([], type=pa.large_list(_TOPK_STRUCT))
        return _wrap(empty, "topk", polars_out)
    try:
        metric_id = _native.metric_from_str(metric)
    except _native.PmmError as e:  # src/metrics.rs:25 text
        raise _compute_error(str(e)) from None
    use_f32 = _is_f32(lv) and _is_f32(rv)  # src/matmul.rs:427
    dt = np.float32 if use_f32 else np.float64
    q = _series_to_matrix(lv, dt)
    c = _series_to_matrix(rv, dt)
    t = _lap("extract", t)
    if q.shape[1] != c.shape[1]:  # src/matmul.rs:433-441
        raise _dim_mismatch(q.shape[1], c.shape[1])
    kk = min(k, c.shape[0])  # src/matmul.rs:443
    m = q.shape[0]
    if kk == 0:
        idx = np.zeros((m, 0), dtype=np.uint32)
        sc = np.zeros((m, 0), dtype=np.float64)
    else:
        _apply_devices_env()
        # (an f32 handle sharded over several GPUs serves k <= 1024; larger k
        # runs on one GPU, the device list's first.  An f64 handle is sharded
        # the same way and serves any k.)
        dc = (_cached_corpus(right, rv, c)
              if (not use_f32 or kk <= 1024 or len(_native.get_devices()) <= 1) else None)
        if dc is not None:
            try:
                idx, sc = dc.topk(q, kk, metric_id)
            finally:
                dc.release()
        else:
            idx, sc = _native.topk_host(q, c, kk, metric_id)
        t = _lap("device", t)
        sc = sc.astype(np.float64, copy=False)  # src/matmul.rs:447 (f32 -> f64)
    out = _wrap(_topk_arrow(idx, sc, m, kk), "topk", polars_out)
    _lap("assemble", t)
    return out


def _matmul(left, right):
    """src/lib.rs:15-30 -> src/matmul.rs:295-417 matmul_impl."""
    polars_out = _is_polars_series(left)
    t = time.perf_counter()
    lv = _to_arrow(left)
    rv = _to_arrow(right)
    use_f32 = _is_f32(lv) and _is_f32(rv)  # src/matmul.rs:298, :308
    dt = np.float32 if use_f32 else np.float64
    pa_t = pa.float32() if use_f32 else pa.float64()
    if _nrows(lv) == 0:  # src/matmul.rs:297-305: empty List (not Array)
        return _wrap(pa.array([], type=pa.large_list(pa_t)), "matmul", polars_out)
    q = _series_to_matrix(lv, dt)
    c = _series_to_matrix(rv, dt)
    t = _lap("extract", t)
    if q.shape[1] != c.shape[1]:
        raise _dim_mismatch(q.shape[1], c.shape[1])
    out = _native.matmul_host(q, c)
    t = _lap("device", t)
    n = c.shape[0]
    arr = pa.FixedSizeListArray.from_arrays(pa.array(out.reshape(-1), type=pa_t), n)
    res = _wrap(arr, "matmul", polars_out)
    _lap("assemble", t)
    return res


__all__ = ["_matmul", "_topk", "PanicException", "clear_corpus_cache", "set_devices", "get_devices"]
