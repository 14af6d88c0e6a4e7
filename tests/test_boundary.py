"""CPU tests of the drop-in boundary: libpmm.so loads and exports every symbol
include/pmm.h declares; the host-side mirror of the reference's extension
functions (input extraction, dtype dispatch, error texts and edge rules of
src/matmul.rs / src/lib.rs) behaves as the reference does before any device
work is issued.  No compute calls without a GPU."""
from __future__ import annotations

import collections
import ctypes
import os
import re
import subprocess

import numpy as np
import pyarrow as pa
import pytest

import polars_matmul
from polars_matmul import _native
from polars_matmul._polars_matmul import PanicException, _matmul, _series_to_matrix, _topk

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pmm.h")


def header_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pmm_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_match_binding_list():
    assert header_symbols() == sorted(_native.EXPORTED_SYMBOLS)


def test_library_exports_every_header_symbol():
    lib = ctypes.CDLL(_native.LIB_PATH)
    for name in header_symbols():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True).stdout
    for name in header_symbols():
        assert re.search(rf"\bT {name}\b", out), f"{name} not exported"


def test_library_targets_gfx950_only():
    # the code objects embedded in libpmm.so are gfx950 only (no dual paths)
    blob = open(_native.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_version_and_metric_parse_via_c_abi():
    assert _native.version().startswith("0.1.4")
    assert _native.metric_from_str("cosine") == _native.METRIC_COSINE
    assert _native.metric_from_str("COSINE") == _native.METRIC_COSINE
    assert _native.metric_from_str("dot") == _native.METRIC_DOT
    assert _native.metric_from_str("euclidean") == _native.METRIC_EUCLIDEAN
    assert _native.metric_from_str("l2") == _native.METRIC_EUCLIDEAN
    with pytest.raises(_native.PmmError) as ei:
        _native.metric_from_str("invalid_metric")
    # src/metrics.rs:25
    assert str(ei.value) == "Unknown metric: 'invalid_metric'. Supported: cosine, dot, euclidean"
    assert _native.lib().pmm_metric_higher_is_better(_native.METRIC_EUCLIDEAN) == 0
    assert _native.lib().pmm_metric_higher_is_better(_native.METRIC_COSINE) == 1


def L(rows, t=pa.float64()):
    return pa.array(rows, type=pa.list_(t))


# ---- error texts / edge rules checked before any device call ----

def test_topk_empty_query_returns_empty_typed():
    # src/matmul.rs:480-487 (checked before the metric, so even a bad metric passes)
    out = _topk(L([]), L([[1.0, 0.0]]), 1, "not_a_metric")
    assert len(out) == 0
    assert out.type == pa.large_list(pa.struct([("index", pa.uint32()), ("score", pa.float64())]))


def test_topk_unknown_metric():
    with pytest.raises(RuntimeError, match="Unknown metric"):
        _topk(L([[1.0, 0.0]]), L([[1.0, 0.0]]), 1, "invalid_metric")


def test_topk_empty_corpus():
    # tests/test_polars_matmul.py:335-343
    with pytest.raises(RuntimeError, match="Empty"):
        _topk(L([[1.0, 0.0]]), L([]), 1, "cosine")


def test_topk_dimension_mismatch():
    # tests/test_polars_matmul.py:355-363
    with pytest.raises(RuntimeError, match="Dimension mismatch: left has 2 dimensional vectors, right has 3"):
        _topk(L([[1.0, 2.0]]), L([[1.0, 2.0, 3.0]]), 1, "cosine")


def test_matmul_dimension_mismatch():
    # tests/test_polars_matmul.py:345-353
    with pytest.raises(RuntimeError, match="Dimension mismatch"):
        _matmul(L([[1.0, 2.0]]), L([[1.0, 2.0, 3.0]]))


def test_matmul_empty_left_is_empty_list():
    # src/matmul.rs:297-305: empty List (not Array), f32 iff both f32
    out = _matmul(L([], pa.float32()), L([[1.0]], pa.float32()))
    assert len(out) == 0 and out.type == pa.large_list(pa.float32())
    out = _matmul(L([], pa.float32()), L([[1.0]]))
    assert out.type == pa.large_list(pa.float64())


def test_negative_k_overflow_and_type_errors():
    with pytest.raises(OverflowError):
        _topk(L([[1.0]]), L([[1.0]]), -1, "cosine")
    with pytest.raises(TypeError):
        _topk(L([[1.0]]), L([[1.0]]), 1.5, "cosine")
    with pytest.raises(TypeError):
        _topk(L([[1.0]]), L([[1.0]]), 1, 3)


def test_first_element_null_and_zero_dim():
    with pytest.raises(RuntimeError, match="First element is null"):
        _topk(L([None, [1.0]]), L([[1.0]]), 1, "dot")
    with pytest.raises(RuntimeError, match="Zero-dimensional vectors"):
        _topk(L([[]]), L([[1.0]]), 1, "dot")
    with pytest.raises(RuntimeError, match="Zero-dimensional vectors"):
        _topk(pa.array([[]], type=pa.list_(pa.float32(), 0)), L([[1.0]]), 1, "dot")


def test_longer_row_panics():
    # src/matmul.rs:276-283: d from row 0, a longer row indexes out of bounds
    with pytest.raises(PanicException):
        _topk(L([[1.0, 2.0], [1.0, 2.0, 3.0]]), L([[1.0, 2.0]]), 1, "dot")


# ---- extraction (src/matmul.rs:131-286) ----

def test_extract_list_with_nulls_and_short_rows():
    arr = pa.array([[1.0, 2.0, 3.0], None, [4.0, None], [5.0, 6.0, 7.0]], type=pa.list_(pa.float64()))
    m = _series_to_matrix(arr, np.float64)
    assert m.tolist() == [[1.0, 2.0, 3.0], [0.0, 0.0, 0.0], [4.0, 0.0, 0.0], [5.0, 6.0, 7.0]]


def test_extract_sliced_large_list_and_chunked():
    arr = pa.array([[9.0, 9.0], [1.0, 2.0], [3.0, 4.0]], type=pa.large_list(pa.float32())).slice(1)
    assert _series_to_matrix(arr, np.float32).tolist() == [[1.0, 2.0], [3.0, 4.0]]
    ch = pa.chunked_array([pa.array([[1.0, 2.0]], type=pa.list_(pa.float32())),
                           pa.array([[3.0, 4.0]], type=pa.list_(pa.float32()))])
    from polars_matmul._polars_matmul import _to_arrow
    assert _series_to_matrix(_to_arrow(ch), np.float32).tolist() == [[1.0, 2.0], [3.0, 4.0]]


def test_extract_fixed_size_list_zero_copy_and_slice():
    base = np.arange(24, dtype=np.float32)
    arr = pa.FixedSizeListArray.from_arrays(pa.array(base), 4)
    m = _series_to_matrix(arr, np.float32)
    assert m.shape == (6, 4) and m.dtype == np.float32
    # src/matmul.rs:22-95: an Array[f32] of one chunk with no nulls is borrowed,
    # not copied -- the matrix IS the Arrow child buffer
    child = np.frombuffer(arr.values.buffers()[1], dtype=np.float32)
    assert np.shares_memory(m, child)
    assert m.ctypes.data == child.ctypes.data
    s = arr.slice(2, 3)
    assert _series_to_matrix(s, np.float32).tolist() == base.reshape(6, 4)[2:5].tolist()
    # f32 Array into the f64 path is cast
    assert _series_to_matrix(s, np.float64).dtype == np.float64


def test_extract_fixed_size_list_null_rows_are_zero():
    arr = pa.array([[1.0, 2.0], None, [3.0, 4.0]], type=pa.list_(pa.float64(), 2))
    assert _series_to_matrix(arr, np.float64).tolist() == [[1.0, 2.0], [0.0, 0.0], [3.0, 4.0]]


def test_dtype_dispatch_rules():
    from polars_matmul._polars_matmul import _is_f32
    assert _is_f32(pa.array([[1.0]], type=pa.list_(pa.float32())))
    assert _is_f32(pa.array([[1.0]], type=pa.list_(pa.float32(), 1)))
    assert not _is_f32(pa.array([[1.0]], type=pa.list_(pa.float64())))
    assert not _is_f32(pa.array([[1]], type=pa.list_(pa.int64())))
    # ints go through the f64 path with a cast (src/matmul.rs:143)
    m = _series_to_matrix(pa.array([[1, 2]], type=pa.list_(pa.int64())), np.float64)
    assert m.dtype == np.float64 and m.tolist() == [[1.0, 2.0]]


def test_compute_fails_loudly_without_device():
    if _native.device_count() > 0:
        pytest.skip("a GPU is visible: covered by the gpu tests")
    with pytest.raises(RuntimeError):
        _topk(L([[1.0, 0.0]]), L([[1.0, 0.0]]), 1, "cosine")
    with pytest.raises(RuntimeError):
        polars_matmul.matmul(np.ones((2, 2)), np.ones((2, 2)))


def test_null_buffers_are_refused_before_any_device_call():
    # a non-empty call with a null buffer is an argument error, not a fault;
    # checked before the device is touched, so it runs here without a GPU
    lib = _native.lib()
    a = np.ones((4, 8), dtype=np.float32)
    a64 = a.astype(np.float64)
    oi = np.zeros(4, dtype=np.uint32)
    os_ = np.zeros(4, dtype=np.float32)
    os64 = np.zeros(4, dtype=np.float64)
    P = lambda x: x.ctypes.data  # noqa: E731
    calls = [
        lambda: lib.pmm_topk_f32(None, 4, P(a), 4, 8, 1, 0, P(oi), P(os_)),
        lambda: lib.pmm_topk_f32(P(a), 4, None, 4, 8, 1, 0, P(oi), P(os_)),
        lambda: lib.pmm_topk_f32(P(a), 4, P(a), 4, 8, 1, 0, None, P(os_)),
        lambda: lib.pmm_topk_f32(P(a), 4, P(a), 4, 8, 1, 0, P(oi), None),
        lambda: lib.pmm_topk_f64(P(a64), 4, None, 4, 8, 1, 0, P(oi), P(os64)),
        lambda: lib.pmm_topk_f64(P(a64), 4, P(a64), 4, 8, 1, 0, P(oi), None),
        lambda: lib.pmm_matmul_f32(P(a), 4, P(a), 4, 8, None),
        lambda: lib.pmm_matmul_f64(None, 4, P(a64), 4, 8, P(os64)),
    ]
    for call in calls:
        assert call() == _native.PMM_ERR_ARG
        assert _native.last_error() == "null argument"
    h = ctypes.c_void_p()
    assert lib.pmm_corpus_create_f32(None, 4, 8, ctypes.byref(h)) == _native.PMM_ERR_ARG
    assert not h.value
    # empty calls need no buffers (src/matmul.rs:480-487 returns before any work)
    assert lib.pmm_topk_f32(None, 0, None, 4, 8, 1, 0, None, None) == 0
    assert lib.pmm_matmul_f32(None, 0, None, 4, 8, None) == 0


def test_pmm_namespace_placeholder_without_polars():
    try:
        import polars  # noqa: F401
    except Exception:
        with pytest.raises(ImportError):
            polars_matmul.PmmNamespace(None)


def test_import_does_not_import_torch():
    # the product package needs no torch: only the HIP runtime library torch
    # ships is preloaded by path (so torch, if imported later, shares it)
    code = ("import sys; sys.path.insert(0, %r); import polars_matmul; "
            "print('torch' in sys.modules)") % os.path.join(ROOT, "polars-matmul_amd")
    out = subprocess.run([os.sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "False"


def test_device_corpus_refcount_defers_destroy(monkeypatch):
    # a cache eviction must not free a corpus another thread is
    # searching -- close() with a use in flight defers the destroy to release()
    destroyed = []

    class StubLib:
        def pmm_corpus_destroy(self, h):
            destroyed.append(h.value)
            return 0

    monkeypatch.setattr(_native, "_lib", StubLib())
    dc = object.__new__(_native.DeviceCorpus)
    import threading
    dc._h = ctypes.c_void_p(1234)
    dc._lock = threading.Lock()
    dc._refs = 0
    dc._closing = False
    dc.acquire()
    dc.close()
    assert destroyed == [] and not dc.closed
    with pytest.raises(RuntimeError):
        dc.acquire()  # closing: no new users
    dc.release()
    assert destroyed == [1234] and dc.closed
    dc.close()
    assert destroyed == [1234]


def test_corpus_cache_respects_free_device_memory(monkeypatch):
    # the cache takes at most half of the free HBM -- a
    # corpus larger than that is searched uncached, one that fits is cached
    from polars_matmul import _polars_matmul as pm

    created = []

    class StubCorpus:
        def __init__(self, c):
            self.nbytes = c.nbytes
            created.append(self)

        def acquire(self):
            return self

        def close(self):
            pass

    free = {"bytes": 0}
    monkeypatch.setattr(_native, "DeviceCorpus", StubCorpus)
    monkeypatch.setattr(_native, "device_memory", lambda: (free["bytes"], 1 << 40))
    monkeypatch.setattr(pm, "_CACHE_ON", True)
    monkeypatch.setattr(pm, "_cache", collections.OrderedDict())
    c = np.zeros((4096, 128), dtype=np.float32)  # 2 MiB: above the caching floor
    arr = pa.FixedSizeListArray.from_arrays(pa.array(c.reshape(-1)), 128)
    free["bytes"] = 3 << 20  # half of it (1.5 MiB) is below the corpus
    assert pm._cached_corpus(arr, arr, c) is None and created == []
    free["bytes"] = 8 << 20
    dc = pm._cached_corpus(arr, arr, c)
    assert dc is created[0] and len(pm._cache) == 1
    assert pm._cached_corpus(arr, arr, c) is dc and len(created) == 1  # hit


def test_corpus_cache_skips_multi_chunk_polars_series(monkeypatch):
    # a multi-chunk Polars Series is concatenated into a
    # fresh buffer by every rechunk(), so its address key never hits -- it
    # must not be cached at all (no entry, no device upload per call)
    from polars_matmul import _polars_matmul as pm

    created = []

    class StubCorpus:
        def __init__(self, c):
            self.nbytes = c.nbytes
            created.append(self)

        def acquire(self):
            return self

        def close(self):
            pass

    c = np.zeros((4096, 128), dtype=np.float32)
    arr = pa.FixedSizeListArray.from_arrays(pa.array(c.reshape(-1)), 128)

    class FakeSeries:
        def __init__(self, chunks):
            self.chunks = chunks

        def n_chunks(self):
            return self.chunks

        def rechunk(self):
            return self

        def to_arrow(self):
            return arr

    monkeypatch.setattr(pm, "_is_polars_series", lambda o: isinstance(o, FakeSeries))
    monkeypatch.setattr(_native, "DeviceCorpus", StubCorpus)
    monkeypatch.setattr(_native, "device_memory", lambda: (1 << 40, 1 << 40))
    monkeypatch.setattr(pm, "_CACHE_ON", True)
    monkeypatch.setattr(pm, "_cache", collections.OrderedDict())
    multi = FakeSeries(2)
    for _ in range(2):
        assert pm._cached_corpus(multi, arr, c) is None
    assert created == [] and len(pm._cache) == 0
    single = FakeSeries(1)
    dc = pm._cached_corpus(single, arr, c)
    assert dc is created[0] and len(pm._cache) == 1


def test_corpus_cache_sizes_entries_by_device_footprint():
    # the device holds rows padded to 32 floats plus four
    # norm arrays, so d = 72 takes 96 floats per row on the device
    assert _native.corpus_device_bytes(1000, 72) == 1000 * 96 * 4 + 1000 * 16
    assert _native.corpus_device_bytes(10, 32) == 10 * 32 * 4 + 10 * 16
    # an f64 corpus (pmm_corpus_create_f64): rows padded to 16 doubles, two
    # f64 norm arrays
    assert _native.corpus_device_bytes(1000, 70, np.float64) == 1000 * 80 * 8 + 1000 * 16
    assert _native.corpus_device_bytes(10, 16, np.float64) == 10 * 16 * 8 + 10 * 16


def test_device_list_parse_and_validation():
    # multi-GPU through the drop-in (include/pmm.h pmm_set_devices): the
    # PMM_DEVICES spec, an empty list, and an invalid device id
    from polars_matmul import _polars_matmul as pm

    assert pm._parse_devices("all", 8) == list(range(8))
    assert pm._parse_devices("0,1, 3", 8) == [0, 1, 3]
    assert pm._parse_devices("", 8) == []
    _native.set_devices([])
    assert _native.get_devices() == []
    with pytest.raises(_native.PmmError) as ei:
        _native.set_devices([_native.device_count() + 5])
    assert ei.value.code == _native.PMM_ERR_NODEVICE
    assert _native.get_devices() == []


def test_pinned_pool_recycles_blocks_and_falls_back(monkeypatch):
    # .pmm.matmul results land in recycled page-locked
    # blocks (no page faults, D2H at link rate); a block returns to the pool
    # when its array (or the Arrow buffer viewing it) is freed.  The
    # allocator is stubbed here (no HIP runtime work on CPU).
    import gc

    store = {}
    frees = []

    class StubLib:
        def pmm_host_alloc(self, nbytes, out):
            b = ctypes.create_string_buffer(nbytes)
            store[ctypes.addressof(b)] = b
            out._obj.value = ctypes.addressof(b)
            return 0

        def pmm_host_free(self, p):
            frees.append(p)
            return 0

    monkeypatch.setattr(_native, "_lib", StubLib())
    pool = _native.PinnedPool(64 << 20)
    monkeypatch.setattr(_native, "pinned_pool", pool)
    a = _native.pinned_empty((1024, 1024), np.float32)  # 4 MiB: pooled
    assert a.flags.writeable and a.shape == (1024, 1024)
    a[:] = 3.0
    arr = pa.array(a.reshape(-1))  # Arrow view keeps the block alive
    p = a.ctypes.data
    del a
    gc.collect()
    assert pool.idle_bytes() == 0 and float(arr[5].as_py()) == 3.0
    del arr
    gc.collect()
    assert pool.idle_bytes() == 4 << 20  # back in the pool
    b = _native.pinned_empty((1024, 1024), np.float32)
    assert b.ctypes.data == p and pool.idle_bytes() == 0  # recycled, not reallocated
    small = _native.pinned_empty((4, 4), np.float32)  # below MIN_BYTES: plain numpy
    assert small.base is None or not hasattr(small.base, "_pmm_block")
    del b
    gc.collect()
    pool.clear()
    assert frees == [p]


def test_pinned_pool_finaliser_inside_take_does_not_deadlock(monkeypatch):
    # a block finalised by a GC pass that starts inside `take`
    # (on the same thread, while the pool works) must not wait on the pool's
    # lock.  Simulate it: the stub allocator drops the last reference to a
    # live block while `take` runs; with a lock taken in the finaliser this
    # would hang.
    store = {}
    pending = []

    class StubLib:
        def pmm_host_alloc(self, nbytes, out):
            pending.clear()  # finalises the held block right here
            b = ctypes.create_string_buffer(nbytes)
            store[ctypes.addressof(b)] = b
            out._obj.value = ctypes.addressof(b)
            return 0

        def pmm_host_free(self, p):
            return 0

    monkeypatch.setattr(_native, "_lib", StubLib())
    pool = _native.PinnedPool(64 << 20)
    got = pool.take(2 << 20)
    pending.append(got[1])
    del got
    with pool.lock:  # finaliser runs while the lock is held: must not block
        pending.clear()
    pending.append(pool.take(2 << 20)[1])  # reuses the returned block, no alloc
    t = pool.take(3 << 20)  # allocates; the stub finalises the 2 MiB block inside
    assert t is not None
    assert pool.idle_bytes() == 2 << 20


def test_pinned_pool_frees_over_cap_blocks_without_a_later_take(monkeypatch):
    # blocks returned past the pool's cap are freed when they
    # come back (an opportunistic, non-blocking drain in the finaliser path),
    # not only on the next take(): a burst of large results freed at the end of
    # a workload does not stay page-locked
    import gc

    store = {}
    frees = []

    class StubLib:
        def pmm_host_alloc(self, nbytes, out):
            b = ctypes.create_string_buffer(nbytes)
            store[ctypes.addressof(b)] = b
            out._obj.value = ctypes.addressof(b)
            return 0

        def pmm_host_free(self, p):
            frees.append(p)
            return 0

    monkeypatch.setattr(_native, "_lib", StubLib())
    pool = _native.PinnedPool(3 << 20)  # holds at most one 2 MiB block idle
    monkeypatch.setattr(_native, "pinned_pool", pool)
    arrs = [_native.pinned_empty((512, 1024), np.float32) for _ in range(4)]  # 2 MiB each
    ptrs = [a.ctypes.data for a in arrs]
    del arrs
    gc.collect()
    # no take() since: one block kept idle, the other three already freed
    assert len(frees) == 3 and set(frees) < set(ptrs)
    assert pool.pending_bytes() == 0 and pool.idle == 2 << 20
    # a block returned while the pool's lock is held (a finaliser inside
    # take) waits in the deque, counted, and is handled by the next drain
    with pool.lock:
        pool._give_back(999, 2 << 20)
        assert pool.pending_bytes() == 2 << 20
    pool.drain()
    assert 999 in frees and pool.pending_bytes() == 0
    pool.clear()
    assert len(frees) == 4 + 1
