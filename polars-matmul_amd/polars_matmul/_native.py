"""ctypes binding of ``libpmm.so`` (the C ABI declared in ``include/pmm.h``).

The reference binds its numerics through pyo3 (src/lib.rs:15-62); this module
is the equivalent binding for the HIP library.  ctypes releases the GIL for
the duration of every foreign call, as ``py.detach`` does in src/lib.rs:25/45.

There is no CPU fallback: if ``libpmm.so`` is missing, importing this module
raises ImportError; if no gfx950 device is visible, every compute call raises
RuntimeError with the library's message.
"""
from __future__ import annotations

import atexit
import collections
import ctypes
import importlib.util
import os
import sys
import threading

import numpy as np

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        # diagnostics only: PMM_LIB=libpmm_stats.so (make stats) adds the
                        # bf16 kernels' per-phase cycle counters (PMM_STATS=1)
                        os.environ.get("PMM_LIB", "libpmm.so"))

PMM_OK = 0
PMM_ERR_ARG = 1
PMM_ERR_HIP = 2
PMM_ERR_UNSUPPORTED = 3
PMM_ERR_NODEVICE = 4

METRIC_COSINE = 0
METRIC_DOT = 1
METRIC_EUCLIDEAN = 2

COMPUTE_F32 = 0
COMPUTE_BF16 = 1

# Every symbol include/pmm.h declares (checked by tests/test_boundary.py).
EXPORTED_SYMBOLS = (
    "pmm_version",
    "pmm_last_error",
    "pmm_metric_from_str",
    "pmm_metric_higher_is_better",
    "pmm_device_count",
    "pmm_device_memory",
    "pmm_set_device",
    "pmm_set_devices",
    "pmm_get_devices",
    "pmm_shard_plan",
    "pmm_topk_f32",
    "pmm_topk_f32_ex",
    "pmm_topk_f64",
    "pmm_topk_f64_device",
    "pmm_matmul_f32",
    "pmm_matmul_f64",
    "pmm_host_alloc",
    "pmm_host_free",
    "pmm_topk_workspace_bytes",
    "pmm_topk_merge_bytes",
    "pmm_topk_f32_device",
    "pmm_topk_bf16_device",
    "pmm_merge_topk_device",
    "pmm_merge_topk_strided_device",
    "pmm_merge_sorted_topk_strided_device",
    "pmm_norms_f32_device",
    "pmm_norms_f64_device",
    "pmm_corpus_create_f32",
    "pmm_corpus_create_f64",
    "pmm_corpus_dtype",
    "pmm_corpus_destroy",
    "pmm_corpus_info",
    "pmm_corpus_shards",
    "pmm_topk_f32_corpus",
    "pmm_topk_f64_corpus",
    "pmm_timing_enable",
    "pmm_timing_reset",
    "pmm_timing_read",
)

def _preload_hip_runtime() -> None:
    """PyTorch-ROCm ships its own libamdhip64.so (SONAME libamdhip64.so.7, as
    /opt/rocm's).  Whichever is loaded first serves the whole process; if
    libpmm.so pulled in /opt/rocm's runtime first, a later `import torch`
    would run on a runtime it was not built against.  When torch is installed
    (and not yet imported), its runtime library is loaded here by path --
    without importing torch -- so libpmm.so and any later torch share it and
    torch device pointers / streams can be passed to the C ABI."""
    if os.environ.get("PMM_NO_TORCH_PRELOAD") == "1" or "torch" in sys.modules:
        return
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is None or not spec.origin:
        return
    hip = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(hip):
        try:
            ctypes.CDLL(hip, mode=ctypes.RTLD_GLOBAL)
        except OSError:
            pass


_preload_hip_runtime()

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"polars_matmul: HIP library not built ({LIB_PATH} missing). "
        "Run `make -C polars-matmul_amd` or `python -c 'import __graft_entry__ as g; g.build()'`."
    )

_lib = ctypes.CDLL(LIB_PATH)

_vp, _i64, _i32, _sz = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_size_t
_u32 = ctypes.c_uint32

_SIGS = {
    "pmm_version": ([], ctypes.c_char_p),
    "pmm_last_error": ([], ctypes.c_char_p),
    "pmm_metric_from_str": ([ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)], _i32),
    "pmm_metric_higher_is_better": ([_i32], _i32),
    "pmm_device_count": ([ctypes.POINTER(ctypes.c_int)], _i32),
    "pmm_device_memory": ([ctypes.POINTER(_sz), ctypes.POINTER(_sz)], _i32),
    "pmm_set_device": ([_i32], _i32),
    "pmm_set_devices": ([ctypes.POINTER(ctypes.c_int), _i32], _i32),
    "pmm_get_devices": ([ctypes.POINTER(ctypes.c_int), _i32, ctypes.POINTER(ctypes.c_int)], _i32),
    "pmm_shard_plan": ([ctypes.POINTER(ctypes.c_int), _i32, _i64, _i64, _i64, _i64, _i32, _i32, _i32,
                        ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                        ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                        ctypes.POINTER(ctypes.c_int)], _i32),
    "pmm_topk_f32": ([_vp, _i64, _vp, _i64, _i64, _i64, _i32, _vp, _vp], _i32),
    "pmm_topk_f32_ex": ([_vp, _i64, _vp, _i64, _i64, _i64, _i32, _i32, _vp, _vp], _i32),
    "pmm_topk_f64": ([_vp, _i64, _vp, _i64, _i64, _i64, _i32, _vp, _vp], _i32),
    "pmm_topk_f64_device": ([_vp, _i64, _i64, _vp, _i64, _i64, _i64, _i64, _i32, _u32, _vp, _vp, _vp], _i32),
    "pmm_matmul_f32": ([_vp, _i64, _vp, _i64, _i64, _vp], _i32),
    "pmm_matmul_f64": ([_vp, _i64, _vp, _i64, _i64, _vp], _i32),
    "pmm_host_alloc": ([_sz, ctypes.POINTER(ctypes.c_void_p)], _i32),
    "pmm_host_free": ([_vp], _i32),
    "pmm_topk_workspace_bytes": ([_i64, _i64, _i64, _i64, _i32, _i32], _sz),
    "pmm_topk_merge_bytes": ([_vp, _i64, _i64, _i64, _i64, _i32, _i32, ctypes.POINTER(ctypes.c_uint64)], _i32),
    "pmm_topk_f32_device": (
        [_vp, _i64, _i64, _vp, _i64, _i64, _i64, _i64, _i32, _i32, _u32, _vp, _vp, _vp, _sz, _vp],
        _i32,
    ),
    "pmm_topk_bf16_device": (
        [_vp, _i64, _i64, _vp, _i64, _i64, _i64, _i64, _i32, _u32, _vp, _vp, _vp, _sz, _vp], _i32
    ),
    "pmm_merge_topk_device": ([_vp, _vp, _i64, _i64, _i64, _i64, _i32, _vp, _vp, _vp], _i32),
    "pmm_merge_topk_strided_device": (
        [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _vp, _vp, _vp], _i32),
    "pmm_merge_sorted_topk_strided_device": (
        [_vp, _vp, _i64, _i64, _i64, _i64, _i64, _i64, _i32, _vp, _vp, _vp], _i32),
    "pmm_norms_f32_device": ([_vp, _i64, _i64, _i64, _i32, _vp, _vp], _i32),
    "pmm_norms_f64_device": ([_vp, _i64, _i64, _i64, _i32, _vp, _vp], _i32),
    "pmm_corpus_create_f32": ([_vp, _i64, _i64, ctypes.POINTER(ctypes.c_void_p)], _i32),
    "pmm_corpus_create_f64": ([_vp, _i64, _i64, ctypes.POINTER(ctypes.c_void_p)], _i32),
    "pmm_corpus_dtype": ([_vp, ctypes.POINTER(ctypes.c_int)], _i32),
    "pmm_corpus_destroy": ([_vp], _i32),
    "pmm_corpus_info": (
        [_vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int)],
        _i32,
    ),
    "pmm_corpus_shards": ([_vp, ctypes.POINTER(ctypes.c_int)], _i32),
    "pmm_topk_f32_corpus": ([_vp, _vp, _i64, _i64, _i32, _vp, _vp], _i32),
    "pmm_topk_f64_corpus": ([_vp, _vp, _i64, _i64, _i32, _vp, _vp], _i32),
    "pmm_timing_enable": ([_i32], _i32),
    "pmm_timing_reset": ([], _i32),
    "pmm_timing_read": (
        [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)],
        _i32,
    ),
}
for _name, (_args, _res) in _SIGS.items():
    _fn = getattr(_lib, _name)
    _fn.argtypes = _args
    _fn.restype = _res


def lib() -> ctypes.CDLL:
    return _lib


class PmmError(RuntimeError):
    """A failing libpmm call; ``code`` is the PMM_ERR_* value."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


def last_error() -> str:
    return (_lib.pmm_last_error() or b"").decode(errors="replace")


def check(rc: int) -> None:
    if rc != PMM_OK:
        raise PmmError(rc, last_error())


def ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def version() -> str:
    return _lib.pmm_version().decode()


def device_count() -> int:
    n = ctypes.c_int(0)
    check(_lib.pmm_device_count(ctypes.byref(n)))
    return n.value


def device_memory():
    """(free, total) bytes of HBM on the device host calls run on."""
    f, t = _sz(0), _sz(0)
    check(_lib.pmm_device_memory(ctypes.byref(f), ctypes.byref(t)))
    return f.value, t.value


def set_devices(ids) -> None:
    """Row-shard the corpus of later host top-k calls (and corpus handles
    created afterwards) over these HIP devices, results merged on ids[0]
    (pmm_set_devices).  An empty list returns to one device."""
    ids = [int(i) for i in ids]
    arr = (ctypes.c_int * max(1, len(ids)))(*ids)
    check(_lib.pmm_set_devices(arr, len(ids)))


def get_devices():
    """The current device list (pmm_get_devices); [] = one device."""
    n = ctypes.c_int(0)
    check(_lib.pmm_get_devices(None, 0, ctypes.byref(n)))
    arr = (ctypes.c_int * max(1, n.value))()
    check(_lib.pmm_get_devices(arr, n.value, ctypes.byref(n)))
    return list(arr[:n.value])


def shard_plan(devs, m: int, n: int, d: int, k: int, metric: int, compute: int = COMPUTE_F32,
               host_rows: bool = True):
    """The sharded search's memory plan (pmm_shard_plan; pure, no GPU):
    (plan_of[g], [(device, bytes) per distinct-device plan], list_offsets[g])."""
    G = len(devs)
    arr = (ctypes.c_int * G)(*[int(x) for x in devs])
    plan_of = (ctypes.c_int * G)()
    plan_dev = (ctypes.c_int * G)()
    plan_bytes = (ctypes.c_uint64 * G)()
    offs = (ctypes.c_uint64 * G)()
    npl = ctypes.c_int(0)
    check(_lib.pmm_shard_plan(arr, G, m, n, d, k, metric, compute, 1 if host_rows else 0, plan_of, plan_dev,
                              plan_bytes, offs, ctypes.byref(npl)))
    return (list(plan_of), [(plan_dev[j], int(plan_bytes[j])) for j in range(npl.value)], [int(x) for x in offs])


def metric_from_str(s: str) -> int:
    out = ctypes.c_int(-1)
    check(_lib.pmm_metric_from_str(s.encode(), ctypes.byref(out)))
    return out.value


def topk_host(q: np.ndarray, c: np.ndarray, k: int, metric: int, compute: int = COMPUTE_F32):
    """Host-buffer top-k.  q: (m, d), c: (n, d) C-contiguous, both f32 or both f64;
    0 <= k <= n.  Returns (idx uint32 (m, k), scores (m, k) in the input dtype)."""
    m, d = q.shape
    n = c.shape[0]
    idx = np.empty((m, k), dtype=np.uint32)
    sc = np.empty((m, k), dtype=q.dtype)
    if q.dtype == np.float32:
        rc = _lib.pmm_topk_f32_ex(ptr(q), m, ptr(c), n, d, k, metric, compute, ptr(idx), ptr(sc))
    else:
        rc = _lib.pmm_topk_f64(ptr(q), m, ptr(c), n, d, k, metric, ptr(idx), ptr(sc))
    check(rc)
    return idx, sc


class _PinnedBlock:
    """One page-locked host block of the result pool; returns itself to the
    pool when the last array / Arrow buffer viewing it is released."""

    __slots__ = ("ptr", "nbytes", "pool", "__weakref__")

    def __init__(self, ptr_value: int, nbytes: int, pool: "PinnedPool"):
        self.ptr, self.nbytes, self.pool = ptr_value, nbytes, pool

    def __del__(self):  # pragma: no cover - exercised through the GC
        try:
            self.pool._give_back(self.ptr, self.nbytes)
        except Exception:
            pass


class PinnedPool:
    """Recycled page-locked result buffers (pmm_host_alloc).  A `.pmm.matmul`
    result (m x n values) lands in one of these: no page faults, D2H at link
    rate, and the buffer becomes the Arrow child buffer of the result Series
    without a copy.  Blocks come back when their arrays are freed; at most
    `cap_bytes` of idle blocks are kept (PMM_PINNED_POOL_BYTES, default 1 GiB;
    0 disables the pool).

    Re-entrancy: a block's finaliser can run inside any allocation (a cyclic
    GC pass), including one made by `take` on the same thread.  So returning a
    block takes no lock and allocates nothing: `_give_back` appends
    (ptr, nbytes) to a deque (append is atomic), and `take` moves returned
    blocks into the free lists under the lock, where nothing is allocated
    either (the lists are preallocated per size; Python objects for the result
    are built after the lock is released)."""

    MIN_BYTES = 1 << 20  # smaller results: a plain numpy array

    def __init__(self, cap_bytes: int):
        self.cap = cap_bytes
        self.free = {}  # nbytes -> [ptr, ...]
        self.idle = 0
        self.lock = threading.Lock()
        self.returned = collections.deque()  # (ptr, nbytes) from finalisers, lock-free

    def _absorb(self):
        """Move finalised blocks into the free lists (lock held by caller).
        Returns the pointers that exceed the cap, to be freed after the lock
        is released."""
        over = []
        while True:
            try:
                p, nbytes = self.returned.popleft()
            except IndexError:
                return over
            if self.idle + nbytes <= self.cap:
                self.free.setdefault(nbytes, []).append(p)
                self.idle += nbytes
            else:
                over.append(p)

    def take(self, nbytes: int):
        """A (pointer, owner) for nbytes, or None (pool off, too small, or the
        allocation failed)."""
        if self.cap <= 0 or nbytes < self.MIN_BYTES:
            return None
        p = None
        with self.lock:
            over = self._absorb()
            lst = self.free.get(nbytes)
            if lst:
                self.idle -= nbytes
                p = lst.pop()
        for q in over:
            _lib.pmm_host_free(q)
        if p is None:
            out = ctypes.c_void_p()
            if _lib.pmm_host_alloc(nbytes, ctypes.byref(out)) != PMM_OK or not out.value:
                return None
            p = out.value
        return p, _PinnedBlock(p, nbytes, self)

    def _give_back(self, p: int, nbytes: int) -> None:
        # runs from finalisers: never waits on the lock (the finaliser may run
        # inside `take` on the thread that holds it), allocates nothing beyond
        # the deque node before it tries the lock
        self.returned.append((p, nbytes))
        # opportunistic drain: blocks past the cap are freed as they come back,
        # not left page-locked until a later take(); when the lock
        # is busy, its holder or the next call drains them.  Not at interpreter
        # shutdown (module globals may be gone; the process exit frees them)
        if sys.is_finalizing() or _lib is None:
            return
        self.drain(blocking=False)

    def drain(self, blocking: bool = True) -> None:
        """Move returned blocks into the free lists and free those past the cap."""
        if not self.lock.acquire(blocking=blocking):
            return
        try:
            over = self._absorb()
        finally:
            self.lock.release()
        for q in over:
            _lib.pmm_host_free(q)

    def pending_bytes(self) -> int:
        """Bytes returned by finalisers and not yet absorbed (from the deque
        itself, so no unlocked counter can drift)."""
        return sum(n for _, n in list(self.returned))

    def idle_bytes(self) -> int:
        with self.lock:
            over = self._absorb()
            n = self.idle
        for q in over:
            _lib.pmm_host_free(q)
        return n

    def clear(self) -> None:
        with self.lock:
            over = self._absorb()
            ptrs = [p for lst in self.free.values() for p in lst] + over
            self.free.clear()
            self.idle = 0
        for p in ptrs:
            _lib.pmm_host_free(p)


pinned_pool = PinnedPool(int(os.environ.get("PMM_PINNED_POOL_BYTES", str(1 << 30))))
atexit.register(pinned_pool.clear)  # idle page-locked blocks go back to the OS at exit


def pinned_empty(shape, dtype) -> np.ndarray:
    """np.empty in a pooled page-locked block when one is available (the block
    is owned by the returned array's buffer chain), else np.empty."""
    dtype = np.dtype(dtype)
    nbytes = int(np.prod(shape)) * dtype.itemsize
    got = pinned_pool.take(nbytes)
    if got is None:
        return np.empty(shape, dtype=dtype)
    p, owner = got
    raw = (ctypes.c_char * nbytes).from_address(p)
    raw._pmm_block = owner  # the array's base holds the block until released
    return np.frombuffer(raw, dtype=dtype).reshape(shape)


def matmul_host(q: np.ndarray, c: np.ndarray) -> np.ndarray:
    m, d = q.shape
    n = c.shape[0]
    out = pinned_empty((m, n), q.dtype)
    fn = _lib.pmm_matmul_f32 if q.dtype == np.float32 else _lib.pmm_matmul_f64
    check(fn(ptr(q), m, ptr(c), n, d, ptr(out)))
    return out


def topk_device(q_ptr: int, ldq: int, m: int, c_ptr: int, ldc: int, n: int, d: int, k: int,
                metric: int, out_idx_ptr: int, out_score_ptr: int, *, index_base: int = 0,
                compute: int = COMPUTE_F32, workspace: int = 0, workspace_bytes: int = 0,
                stream: int = 0) -> None:
    """Device-resident fused top-k (pointers are HBM addresses, e.g. torch data_ptr())."""
    check(_lib.pmm_topk_f32_device(q_ptr, ldq, m, c_ptr, ldc, n, d, k, metric, compute,
                                   index_base, out_idx_ptr, out_score_ptr, workspace or None,
                                   workspace_bytes, stream or None))


def topk_f64_device(q_ptr: int, ldq: int, m: int, c_ptr: int, ldc: int, n: int, d: int, k: int,
                    metric: int, out_idx_ptr: int, out_score_ptr: int, *, index_base: int = 0,
                    stream: int = 0) -> None:
    """Device-resident f64 top-k (pmm_topk_f64_device; row strides >= roundup(d, 16))."""
    check(_lib.pmm_topk_f64_device(q_ptr, ldq, m, c_ptr, ldc, n, d, k, metric, index_base, out_idx_ptr,
                                   out_score_ptr, stream or None))


def topk_bf16_device(q_ptr: int, ldq: int, m: int, c_ptr: int, ldc: int, n: int, d: int, k: int,
                     metric: int, out_idx_ptr: int, out_score_ptr: int, *, index_base: int = 0,
                     workspace: int = 0, workspace_bytes: int = 0, stream: int = 0) -> None:
    """Device-resident bf16 top-k (bf16 row bit patterns in HBM, e.g. a
    torch.bfloat16 tensor's data_ptr()); row strides >= roundup(d, 128)."""
    check(_lib.pmm_topk_bf16_device(q_ptr, ldq, m, c_ptr, ldc, n, d, k, metric, index_base,
                                    out_idx_ptr, out_score_ptr, workspace or None, workspace_bytes,
                                    stream or None))


def merge_device(idx_ptr: int, score_ptr: int, m: int, lists: int, k_in: int, k_out: int,
                 metric: int, out_idx_ptr: int, out_score_ptr: int, stream: int = 0) -> None:
    check(_lib.pmm_merge_topk_device(idx_ptr, score_ptr, m, lists, k_in, k_out, metric,
                                     out_idx_ptr, out_score_ptr, stream or None))


def merge_strided_device(idx_ptr: int, score_ptr: int, m: int, lists: int, k_in: int,
                         row_stride: int, list_stride: int, k_out: int, metric: int,
                         out_idx_ptr: int, out_score_ptr: int, stream: int = 0, *,
                         sorted_lists: bool = False) -> None:
    """k-way merge of strided lists; sorted_lists=True: every list is
    best-first (a top-k or merge output), so the prefix fast path applies
    (pmm_merge_sorted_topk_strided_device)."""
    fn = _lib.pmm_merge_sorted_topk_strided_device if sorted_lists else _lib.pmm_merge_topk_strided_device
    check(fn(idx_ptr, score_ptr, m, lists, k_in, row_stride, list_stride, k_out, metric, out_idx_ptr,
             out_score_ptr, stream or None))


def norms_device(a_ptr: int, ld: int, rows: int, d: int, squared: bool, out_ptr: int, *,
                 f64: bool = False, stream: int = 0) -> None:
    """Row norms (or squared norms) of device rows in the reference's order
    (pmm_norms_f32_device / pmm_norms_f64_device)."""
    fn = _lib.pmm_norms_f64_device if f64 else _lib.pmm_norms_f32_device
    check(fn(a_ptr, ld, rows, d, 1 if squared else 0, out_ptr, stream or None))


def workspace_bytes(m: int, n: int, d: int, k: int, metric: int, compute: int = COMPUTE_F32) -> int:
    return int(_lib.pmm_topk_workspace_bytes(m, n, d, k, metric, compute))


def merge_bytes(workspace_ptr: int, m: int, n: int, d: int, k: int, metric: int,
                compute: int = COMPUTE_F32) -> int:
    """Algorithmic bytes of the last fused top-k's merge pass (measurement only)."""
    out = ctypes.c_uint64(0)
    check(_lib.pmm_topk_merge_bytes(workspace_ptr, m, n, d, k, metric, compute, ctypes.byref(out)))
    return int(out.value)


def timing_enable(on: bool = True) -> None:
    check(_lib.pmm_timing_enable(1 if on else 0))


def timing_reset() -> None:
    check(_lib.pmm_timing_reset())


def timing_read(kernel: str):
    ms = ctypes.c_double(0.0)
    n = ctypes.c_int64(0)
    check(_lib.pmm_timing_read(kernel.encode(), ctypes.byref(ms), ctypes.byref(n)))
    return ms.value, n.value


DTYPE_F32 = 0
DTYPE_F64 = 1


def corpus_device_bytes(n: int, d: int, dtype=np.float32) -> int:
    """HBM a DeviceCorpus of n x d rows holds.  f32 (pmm_corpus_create_f32):
    the rows padded to a multiple of 32 floats plus four norm arrays (cosine
    norms and pre-filter factors, euclidean squared norms and factors).  f64
    (pmm_corpus_create_f64): the rows padded to a multiple of 16 doubles plus
    two norm arrays (cosine norms, euclidean squared norms)."""
    if np.dtype(dtype) == np.float64:
        dp = -(-d // 16) * 16
        return n * dp * 8 + n * 2 * 8
    dp = -(-d // 32) * 32
    return n * dp * 4 + n * 4 * 4


class DeviceCorpus:
    """A corpus uploaded once to HBM with its norms (pmm_corpus_*), f32 or f64
    rows by the dtype of ``c`` (the reference's two branches,
    src/matmul.rs:427-468).

    Reference-counted: ``acquire()`` / ``release()`` bracket a use (``topk``
    does so itself); ``close()`` frees the device memory at once if no use is
    in flight, else when the last one releases it -- a cache may evict a
    handle while another thread is still searching it."""

    def __init__(self, c: np.ndarray):
        self.dtype = np.dtype(np.float64 if np.asarray(c).dtype == np.float64 else np.float32)
        c = np.ascontiguousarray(c, dtype=self.dtype)
        h = ctypes.c_void_p()
        create = _lib.pmm_corpus_create_f64 if self.dtype == np.float64 else _lib.pmm_corpus_create_f32
        check(create(ptr(c), c.shape[0], c.shape[1], ctypes.byref(h)))
        self._h = h
        self._lock = threading.Lock()
        self._refs = 0
        self._closing = False
        self.n, self.d = c.shape
        self.nbytes = corpus_device_bytes(self.n, self.d, self.dtype)  # device footprint, not host bytes

    def acquire(self) -> "DeviceCorpus":
        with self._lock:
            if self._closing or not self._h:
                raise RuntimeError("DeviceCorpus is closed")
            self._refs += 1
        return self

    def release(self) -> None:
        with self._lock:
            self._refs -= 1
            if self._refs == 0 and self._closing:
                self._destroy()

    def topk(self, q: np.ndarray, k: int, metric: int):
        """(idx uint32 (m, k), scores (m, k) in the corpus dtype); q is
        converted to the corpus dtype."""
        q = np.ascontiguousarray(q, dtype=self.dtype)
        if q.shape[1] != self.d:
            raise ValueError("dimension mismatch")
        m = q.shape[0]
        idx = np.empty((m, k), dtype=np.uint32)
        sc = np.empty((m, k), dtype=self.dtype)
        fn = _lib.pmm_topk_f64_corpus if self.dtype == np.float64 else _lib.pmm_topk_f32_corpus
        self.acquire()
        try:
            check(fn(self._h, ptr(q), m, k, metric, ptr(idx), ptr(sc)))
        finally:
            self.release()
        return idx, sc

    def _destroy(self) -> None:  # with self._lock held
        if self._h:
            _lib.pmm_corpus_destroy(self._h)
            self._h = ctypes.c_void_p()

    @property
    def shards(self) -> int:
        """Device shards of this corpus (pmm_corpus_shards)."""
        n = ctypes.c_int(0)
        check(_lib.pmm_corpus_shards(self._h, ctypes.byref(n)))
        return n.value

    @property
    def device_dtype(self) -> int:
        """DTYPE_F32 / DTYPE_F64 as the library reports it (pmm_corpus_dtype)."""
        v = ctypes.c_int(-1)
        check(_lib.pmm_corpus_dtype(self._h, ctypes.byref(v)))
        return v.value

    @property
    def closed(self) -> bool:
        return not self._h

    def close(self) -> None:
        with self._lock:
            self._closing = True
            if self._refs == 0:
                self._destroy()

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass
