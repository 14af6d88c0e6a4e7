#!/usr/bin/env python3
"""Headline benchmark: cosine top-k queries/sec on MI355X.

Workload (BASELINE.json configs[2], the config its metric is quoted on; it fits
one GPU): 100,000 queries x 1,000,000 corpus rows x 768 dims, f32, cosine,
k = 100.  Synthetic N(0,1) f32 embeddings generated on device in blocks of
65,536 rows, each block from its own seeded torch generator (so every rank can
generate any corpus row range, and the corpus is the same whatever the number
of GPUs); inputs are resident in HBM before the timed region.

One step = one full top-k pass of all M queries against the corpus:
  N = 1: fused GEMM + top-k (libpmm.so, pmm_topk_f32_device) over the corpus.
  N > 1: the corpus is row-sharded over the ranks (one process per GPU);
         each rank runs the fused top-k on its shard (global indices via
         index_base), rank 0 gathers the per-shard M x k lists over RCCL
         (torch.distributed "nccl" = RCCL; one gather of a [2][M][k] block per
         rank) and k-way merges them in place (pmm_merge_topk_strided_device).
         Total work is fixed: "scaling": "strong".

Run: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c4|c5|c1|c2]
  --gpus N > 1 without a torch.distributed launcher: this process starts N rank
  processes itself (before touching the GPU) and exits with their status;
  under torch.distributed.run, WORLD_SIZE must equal N.

Prints ONE JSON line on rank 0 with the metric, the dominant kernel's roofline
(achieved TFLOP/s from HIP events on its launch stream vs the 157.3 TFLOP/s
f32 MFMA peak) and CPU baselines (the oracle -- a port of the reference's
algorithm -- on a bounded query sample on this host's cores; the reference's
own benchmark size configs[0] in full under extra.c1).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "polars-matmul_amd"), os.path.join(ROOT, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

CONFIGS = {
    # name: (M, N, D, k, metric, compute dtype)
    "c3": (100_000, 1_000_000, 768, 100, "cosine", "f32"),
    "c4": (100_000, 1_000_000, 768, 100, "cosine", "bf16"),
    "c5": (1_000_000, 10_000_000, 1024, 100, "cosine", "f32"),
    # configs[4]'s per-GPU work on one GPU: all 1M queries against rank 0's
    # shard of the 8-way row split (corpus rows [0, 1.25M) of c5's corpus)
    "c5_rank": (1_000_000, 1_250_000, 1024, 100, "cosine", "f32"),
    "c2": (1_000, 10_000, 256, 10, "dot", "f32"),
    "c1": (1_000, 10_000, 256, 10, "cosine", "f32"),
}
# the reference's own benchmark (examples/benchmark_topk.py:69-71): seed-42
# NumPy randn inputs, generated on the host
REF_INPUT_CONFIGS = ("c1", "c2")
MFMA_PEAK_TFLOPS = {"f32": 157.3, "bf16": 2516.6}  # MI355X dense matrix peaks (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
QSEED, CSEED = 42, 1_000_003
GEN_BLOCK = 65536


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def available_parallelism() -> int:
    """The thread count faer's Parallelism::Rayon(0) gets (metrics.rs:244-251):
    rayon's default pool is std::thread::available_parallelism(), i.e. the
    CPUs this process may run on (sched_getaffinity), capped by a cgroup v2
    CPU quota (cpu.max) when one is set."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def recall_at_k(a: np.ndarray, b: np.ndarray) -> float:
    """Mean over rows of |a_row & b_row| / k for index lists without
    duplicates inside a row (SURVEY 8c's bf16 criterion)."""
    both = np.concatenate([a, b], axis=1)
    both.sort(axis=1)
    return float(np.mean((both[:, 1:] == both[:, :-1]).sum(axis=1) / a.shape[1]))


# ---------------------------------------------------------------------------
# N-rank launcher (no GPU work in this process)
# ---------------------------------------------------------------------------
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int, argv, extra_env=None) -> int:
    """Start n rank processes running this script with argv (one per GPU,
    torchrun-style env: RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT) and
    return the first non-zero exit status (0 if all succeed).  Children are
    started fresh; this process never touches the GPU."""
    env = dict(os.environ)
    env.update({"WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(_free_port())})
    env.update(extra_env or {})
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=e))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            r = p.poll()
            if r is None:
                continue
            pending.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for o in pending:  # a failed rank would leave the others waiting in a collective
                    o.terminate()
        time.sleep(0.05)
    return rc


# ---------------------------------------------------------------------------
# synthetic inputs
# ---------------------------------------------------------------------------
def synth_rows(lo: int, hi: int, d: int, seed: int, dev):
    """Rows [lo, hi) of an (unbounded) N(0,1) f32 matrix: block b of GEN_BLOCK
    rows comes from torch.randn on a generator seeded with seed * 2^20 + b."""
    import torch

    out = torch.empty((hi - lo, d), dtype=torch.float32, device=dev)
    if hi <= lo:
        return out
    g = torch.Generator(device=dev)
    for b in range(lo // GEN_BLOCK, (hi - 1) // GEN_BLOCK + 1):
        g.manual_seed(seed * (1 << 20) + b)
        blk = torch.randn((GEN_BLOCK, d), generator=g, device=dev, dtype=torch.float32)
        a0, a1 = max(lo, b * GEN_BLOCK), min(hi, (b + 1) * GEN_BLOCK)
        out[a0 - lo:a1 - lo] = blk[a0 - b * GEN_BLOCK:a1 - b * GEN_BLOCK]
        del blk
    return out


def ref_inputs(M, N, D):
    """examples/benchmark_topk.py:69-71: np.random.seed(42); randn(M, D),
    randn(N, D) in float64, cast to float32."""
    np.random.seed(42)
    q = np.random.randn(M, D).astype(np.float32)
    c = np.random.randn(N, D).astype(np.float32)
    return q, c


METRIC_OVERRIDE = None  # --metric: the main config's metric replaced (no traffic record applies)


def load_traffic(config: str):
    """(HBM bytes per launch of the dominant kernel, its source record) from
    the committed rocprofv3 --pmc summary of this build (profiles/
    pmc_traffic_<config>.json, written by tools/traffic_json.py), corrected as
    MI355X_MICROARCH.md prescribes."""
    path = os.path.join(ROOT, "profiles", f"pmc_traffic_{config}.json")
    if METRIC_OVERRIDE or not os.path.exists(path):  # the records are of the configs' own metric
        return None, None
    try:
        with open(path) as f:
            rec = json.load(f)
        return rec.get("hbm_bytes_per_launch"), {
            "source": rec.get("source"), "traffic_over_algorithmic": rec.get("traffic_over_algorithmic"),
            "algorithmic_bytes_per_launch": rec.get("algorithmic_bytes_per_launch"),
            "l2_hit_rate": rec.get("l2_hit_rate")}
    except Exception:
        return None, None


# ---------------------------------------------------------------------------
# CPU baselines (rank 0, N = 1 only)
# ---------------------------------------------------------------------------
def cpu_oracle_qps(q, c, k, metric, threads, reps=1, warm=0):
    """The oracle (the reference's structure: threaded GEMM, single-threaded
    epilogue + per-row select); median seconds of `reps` timed calls."""
    import oracle

    mid = oracle.metric_from_str(metric)
    for _ in range(warm):
        oracle.topk(q, c, k, mid, nthreads=threads)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        oracle.topk(q, c, k, mid, nthreads=threads)
        ts.append(time.perf_counter() - t0)
    dt = float(np.median(ts))
    return q.shape[0] / dt, dt


def cpu_blas_qps(q, c, k, metric, threads, reps=1, warm=0):
    """the reference's structure with a BLAS-class GEMM
    (oracle.topk_blas: ndarray-order norms, OpenBLAS sgemm through NumPy on
    `threads` threads in the role of faer's Parallelism::Rayon(0)
    (src/metrics.rs:244-251) into the M x N matrix, then the oracle's
    single-threaded epilogue and per-row select).  Median seconds of `reps`
    calls and the phase split of the median call."""
    import oracle

    mid = oracle.metric_from_str(metric)
    for _ in range(warm):
        oracle.topk_blas(q, c, k, mid, nthreads=threads)
    runs = []
    for _ in range(reps):
        ph = {}
        t0 = time.perf_counter()
        oracle.topk_blas(q, c, k, mid, nthreads=threads, timings=ph)
        runs.append((time.perf_counter() - t0, ph))
    runs.sort(key=lambda r: r[0])
    dt, ph = runs[len(runs) // 2]
    return q.shape[0] / dt, dt, {kk: round(v * 1000.0, 2) for kk, v in ph.items()}


def blas_name() -> str:
    try:
        cfg = np.show_config(mode="dicts")
        b = cfg["Build Dependencies"]["blas"]
        return f"{b.get('name', 'blas')} {b.get('version', '')}".strip()
    except Exception:
        return "NumPy BLAS"


def numpy_comparator(q, c, k, reps=1, warm=0):
    """SURVEY 8d CPU baseline (2): the README's NumPy comparator
    (examples/benchmark_topk.py:14-33 in the reference) restated -- L2-normalise
    both sides, one BLAS GEMM, a per-row partial selection of k, then a sort
    of those k.  Cosine only; BLAS threads as the environment sets them."""
    def once():
        qn = q / np.sqrt((q * q).sum(axis=1, keepdims=True))
        cn = c / np.sqrt((c * c).sum(axis=1, keepdims=True))
        sim = qn @ cn.T
        cut = sim.shape[1] - k
        part = np.argpartition(sim, cut, axis=1)[:, cut:]
        vals = np.take_along_axis(sim, part, axis=1)
        order = np.argsort(-vals, axis=1)
        return np.take_along_axis(part, order, axis=1)

    for _ in range(warm):
        once()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        once()
        ts.append(time.perf_counter() - t0)
    dt = float(np.median(ts))
    return q.shape[0] / dt, dt


def link_ceilings(out_bytes, in_bytes, reps=5):
    """The box's host <-> device copy rates: one
    hipMemcpyAsync (torch copy_) of out_bytes device -> page-locked host, and
    of in_bytes host -> device from page-locked and from pageable memory,
    median of `reps` after one warm-up each."""
    import torch

    dev = torch.device("cuda", torch.cuda.current_device())
    d_out = torch.empty(out_bytes // 4, dtype=torch.float32, device=dev)
    h_out = torch.empty(out_bytes // 4, dtype=torch.float32, pin_memory=True)
    d_in = torch.empty(in_bytes // 4, dtype=torch.float32, device=dev)
    h_in_pinned = torch.ones(in_bytes // 4, dtype=torch.float32, pin_memory=True)
    h_in_pageable = torch.ones(in_bytes // 4, dtype=torch.float32)

    def rate(dst, src, nbytes):
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            dst.copy_(src, non_blocking=True)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return round(nbytes / float(np.median(ts)) / 1e9, 2)

    out = {"d2h_pinned_gbs": rate(h_out, d_out, out_bytes), "h2d_pinned_gbs": rate(d_in, h_in_pinned, in_bytes),
           "h2d_pageable_gbs": rate(d_in, h_in_pageable, in_bytes), "out_bytes": out_bytes, "in_bytes": in_bytes}
    del d_out, h_out, d_in, h_in_pinned, h_in_pageable
    return out


def matmul_line(args, reps=20, warm=3):
    """SURVEY 8f row 1, `.pmm.matmul` (matmul.rs:295-417): the f32 GEMM in store
    mode through the host C ABI (pmm_matmul_f32: host Q, C in; the M x N f32
    result in a host buffer), at the reference benchmark's size (configs[0]
    inputs, seed 42).  Per call: median wall time of `reps` calls, the device
    GEMM's average (HIP events) and the result's relative error against a
    float64 product; CPU baseline: NumPy's f32 BLAS product (the role of the
    reference's faer GEMM, matmul.rs:244-251)."""
    from polars_matmul import _native

    M, N, D = CONFIGS["c1"][:3]
    qh, ch = ref_inputs(M, N, D)
    out = _native.matmul_host(qh, ch)
    ref = qh.astype(np.float64) @ ch.astype(np.float64).T
    err = float(np.max(np.abs(out.astype(np.float64) - ref) / np.maximum(1.0, np.abs(ref))))
    del ref, out
    for _ in range(warm):
        _native.matmul_host(qh, ch)
    _native.timing_reset()
    _native.timing_enable(True)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        _native.matmul_host(qh, ch)
        ts.append(time.perf_counter() - t0)
    # the same call into a caller's reused (faulted-in, pageable) output
    # buffer; matmul_host's results come from the page-locked result pool
    # (a dropped result's block serves the next call)
    import ctypes

    reuse = np.zeros((M, N), np.float32)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        _native.check(_native._lib.pmm_matmul_f32(vp(qh), M, vp(ch), N, D, vp(reuse)))
        rts.append(time.perf_counter() - t0)
    _native.timing_enable(False)
    kms, kn = _native.timing_read("gemm_f32_matmul")
    dt = float(np.median(ts))
    rdt = float(np.median(rts))
    flops = 2.0 * M * N * D
    link = link_ceilings(out_bytes=M * N * 4, in_bytes=(M + N) * D * 4)
    link_floor_ms = (M + N) * D * 4 / (link["h2d_pageable_gbs"] * 1e9) * 1000.0 + \
        M * N * 4 / (link["d2h_pinned_gbs"] * 1e9) * 1000.0
    line = {
        "metric": f"matmul calls/s ({M}x{N}x{D} f32, host buffers in and out)", "value": round(1.0 / dt, 2),
        "unit": "calls/s", "ms_per_call": round(dt * 1000.0, 3),
        "kernel_ms_avg": round(kms / kn, 4) if kn else None,
        "kernel_tflops": round(flops / (kms / kn / 1000.0) / 1e12, 2) if kn else None,
        "ms_per_call_reused_out": round(rdt * 1000.0, 3),
        "out_gbs": round(M * N * 4 / dt / 1e9, 2), "max_rel_err_vs_f64": err,
        "d2h_ceiling_gbs": link["d2h_pinned_gbs"], "out_frac_of_d2h": round(M * N * 4 / dt / 1e9 / link["d2h_pinned_gbs"], 3),
        "link": link,
        # the call's bytes over the link at the measured rates (inputs from
        # pageable NumPy memory, the result into page-locked blocks), serialised
        "link_floor_ms": round(link_floor_ms, 3), "link_frac": round(link_floor_ms / (dt * 1000.0), 3),
        "note": "result bytes M*N*4 = 40 MB per call, copied into a pooled page-locked block: the "
                "PCIe copy, not the GEMM, bounds the call",
    }
    line["sweep"] = matmul_sweep(cpu=bool(args.cpu_sample))
    if args.cpu_sample:
        for _ in range(2):
            qh @ ch.T
        cts = []
        for _ in range(5):
            t0 = time.perf_counter()
            qh @ ch.T
            cts.append(time.perf_counter() - t0)
        cdt = float(np.median(cts))
        line["cpu_baseline"] = {
            "value": round(1.0 / cdt, 2), "unit": "calls/s",
            "cores": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)),
            "host_nproc": os.cpu_count(), "available_parallelism": available_parallelism(), "kind": "port",
            "sample": f"the full product, NumPy f32 BLAS q @ c.T, median of 5 after 2 warm-ups: {cdt * 1000:.2f} ms",
        }
    return line


def root_merge_line(reps=10, warm=2, shards=8):
    """configs[4]'s root merge at full size: rank 0's k-way
    merge of the 8 gathered per-shard top-100 lists of 1M query rows, the one
    piece of the 8-GPU step besides the RCCL gather that one GPU can time.
    Input: the gather buffer [8][2][1M][100] (per shard an index plane and a
    score plane) generated on device, each shard's list of a row sorted best
    first (i.i.d. N(0,1) scores: the lists interleave as equal shards' top-k
    do).  Timed with HIP events on the launch stream: the sorted-list merge the
    sharded paths use (pmm_merge_sorted_topk_strided_device: prefixes first)
    and the general merge (any list order) on the same buffer.  Algorithmic
    bytes per launch (G + 1) M k 8: every list entry read once, the output
    written once."""
    import torch
    from polars_matmul import _native

    M, k, G = 1_000_000, 100, shards
    dev = torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    buf = torch.empty((G, 2, M, k), dtype=torch.int32, device=dev)
    step = 1 << 17
    for r0 in range(0, M, step):
        r1 = min(M, r0 + step)
        vals = torch.randn((G, r1 - r0, k), generator=g, device=dev)
        vals, _ = torch.sort(vals, dim=2, descending=True)
        buf[:, 1, r0:r1] = vals.view(torch.int32)
        base = (torch.arange(G, device=dev, dtype=torch.int64) * 1_250_000).view(G, 1, 1)
        ids = torch.randint(0, 1_250_000, (G, r1 - r0, k), generator=g, device=dev) + base
        buf[:, 0, r0:r1] = ids.to(torch.int32)
        del vals, ids
    oi = torch.empty((M, k), dtype=torch.int32, device=dev)
    osc = torch.empty((M, k), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream()
    out = {}
    for name, srt in (("sorted", True), ("general", False)):
        def run():
            _native.merge_strided_device(buf.data_ptr(), buf[0, 1].data_ptr(), M, G, k, k, 2 * M * k, k,
                                         _native.metric_from_str("cosine"), oi.data_ptr(), osc.data_ptr(),
                                         stream=stream.cuda_stream, sorted_lists=srt)
        for _ in range(warm):
            run()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
        for i in range(reps):
            ev[2 * i].record(stream)
            run()
            ev[2 * i + 1].record(stream)
        torch.cuda.synchronize()
        ms = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(reps))
        avg = sum(ms) / reps
        # spot check 4096 rows against torch over the concatenated lists
        rows = torch.arange(0, M, M // 4096, device=dev)[:4096]
        sc_all = buf[:, 1, rows].view(torch.float32).permute(1, 0, 2).reshape(len(rows), G * k)
        id_all = buf[:, 0, rows].permute(1, 0, 2).reshape(len(rows), G * k)
        ts, ti = torch.topk(sc_all, k, dim=1)
        ok = bool(torch.equal(torch.gather(id_all, 1, ti), oi[rows])) and bool(torch.equal(ts, osc[rows]))
        alg = (G + 1) * M * k * 8
        out[name] = {"kernel_ms_avg": round(avg, 4), "kernel_ms_median": round(ms[reps // 2], 4),
                     "achieved": round(alg / (avg / 1000.0) / 1e9, 1), "frac": round(alg / (avg / 1000.0) / 1e9 / HBM_PEAK_GBS, 4),
                     "spot_check_4096_rows_exact": ok}
    c = min(k, 256 // G)
    line = {
        "metric": f"root k-way merge of {G} x {M} x {k} sorted (index, score) lists", "unit": "GB/s",
        "bound": "hbm", "peak": HBM_PEAK_GBS, "bytes_per_launch": (G + 1) * M * k * 8,
        "kernel": "merge_kernel<1> (sorted: prefix fast path; general: every entry)",
        "value": out["sorted"]["achieved"], "frac": out["sorted"]["frac"],
        "kernel_ms_avg": out["sorted"]["kernel_ms_avg"],
        "sorted_prefix_bytes_min": M * G * c * 8 + M * k * 8,
        "sorted": out["sorted"], "general": out["general"],
        "data": "device-generated: per shard and row 100 i.i.d. N(0,1) scores sorted best first, indices in the "
                "shard's row range",
    }
    del buf, oi, osc
    torch.cuda.empty_cache()
    return line


def _median_time(fn, reps, warm):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), ts


def boundary_rates(q_dev, c_dev, k, metric_id, compute=0, reps=5, warm=1):
    """Host-boundary rates: host f32 buffers in, host idx/score
    out, through the C ABI, median of `reps` calls after `warm` full-size
    warm-ups (untimed by the contract's clock):
      host_api: pmm_topk_f32 -- uploads Q and C (pageable host memory; the
        corpus in chunks overlapped with compute), computes, downloads;
      cached_corpus: pmm_topk_f32_corpus -- corpus resident (uploaded once,
        as the Arrow-keyed cache does across map_batches calls), Q uploaded
        and results downloaded per call."""
    from polars_matmul import _native

    qh = q_dev.cpu().numpy()
    ch = c_dev.cpu().numpy()
    M = qh.shape[0]
    out = {"reps": reps, "warmup": warm}
    _native.topk_host(qh[:1024], ch[:4096], k, metric_id, compute=compute)  # first-call setup
    dt, ts = _median_time(lambda: _native.topk_host(qh, ch, k, metric_id, compute=compute), reps, warm)
    out["host_api_qps"] = round(M / dt, 2)
    out["host_api_s"] = [round(t, 4) for t in ts]
    if compute != _native.COMPUTE_F32:
        return out  # the corpus handle is f32-only
    t0 = time.perf_counter()
    dc = _native.DeviceCorpus(ch)
    out["corpus_upload_s"] = round(time.perf_counter() - t0, 3)
    dc.topk(qh[:1024], k, metric_id)  # first-call allocations
    dt, ts = _median_time(lambda: dc.topk(qh, k, metric_id), reps, warm)
    out["cached_corpus_qps"] = round(M / dt, 2)
    out["cached_corpus_s"] = [round(t, 4) for t in ts]
    dc.close()
    return out


# ---------------------------------------------------------------------------
# The reference's own benchmarks, end to end through the extension surface
# 
# ---------------------------------------------------------------------------
def _arrow_rows(a, fixed):
    """a's rows as a Polars List[f] column's Arrow form (LargeList) or as an
    Array[f, d] (FixedSizeList) -- what `.cast(pl.List(..))` / `pl.Array`
    hand the plugin (benchmark_topk.py:76-82, benchmark_matmul.py:54-60)."""
    import pyarrow as pa

    m, d = a.shape
    vals = pa.array(a.reshape(-1))
    if fixed:
        return pa.FixedSizeListArray.from_arrays(vals, d)
    return pa.LargeListArray.from_arrays(pa.array(np.arange(m + 1, dtype=np.int64) * d), vals)


def _explode_unnest(res, qid):
    """`.explode("m").unnest("m")` of benchmark_topk.py:56-60 on Arrow: the
    query id repeated per hit, the index and score columns."""
    import pyarrow.compute as pc

    parents = pc.list_parent_indices(res)
    flat = res.flatten()
    return qid.take(parents), flat.field("index"), flat.field("score")


def _native_split():
    """(h2d, kernels, d2h) ms of the library's event records since the last reset."""
    from polars_matmul import _native

    tot, _ = _native.timing_read("")
    h2d, _ = _native.timing_read("h2d")
    d2h, _ = _native.timing_read("d2h")
    return h2d, tot - h2d - d2h, d2h


def e2e_topk_line(reps=5, warm=2):
    """benchmark_topk.py:48-64 / :79-91 at its base size (BASELINE configs[0]/
    [1] shape: 1000 x 10000 x 256, k = 10, cosine, seed-42 inputs): the whole
    `.pmm.topk` call (`_topk` on the Arrow form of a Polars List[f32] column,
    then explode + unnest), median of `reps` after `warm` warm-ups, as the
    reference times it.  Legs: List and Array (FixedSizeList) inputs, f32 and
    f64 (the reference's "Varying Dtype"); `cached` = repeated calls with the
    same corpus column (the device corpus cache -- f32 or f64 rows -- hits
    after the first call: only the queries are uploaded), `first_call` = the
    cache cleared before each call (corpus uploaded and its norms computed
    every time).  Per leg the median call's split: extract
    (Arrow -> contiguous matrices), h2d / kernels / d2h (HIP events of the
    library), device_other (host time in the C-ABI call outside the events'
    span: staging, launch, sync), assemble (f64 widening + Arrow List[Struct])
    and explode_unnest."""
    import pyarrow as pa

    from polars_matmul import _native
    from polars_matmul import _polars_matmul as pm

    M, N, D, k, metric = CONFIGS["c1"][:5]
    qid = pa.array(np.arange(M, dtype=np.int64))
    out = {"workload": f"{M}x{N}x{D} {metric} k={k}, seed-42 inputs (benchmark_topk.py:69-71)",
           "reps": reps, "warmup": warm}
    for dt_name, dtype in (("f32", np.float32), ("f64", np.float64)):
        np.random.seed(42)
        qh = np.random.randn(M, D).astype(dtype)
        ch = np.random.randn(N, D).astype(dtype)
        for fixed in (False, True):
            qa, ca = _arrow_rows(qh, fixed), _arrow_rows(ch, fixed)
            legs = ("cached", "first_call")  # f32 and f64 corpora are both cached on the device
            for leg in legs:
                def call():
                    if leg == "first_call":
                        pm.clear_corpus_cache()
                    res = pm._topk(qa, ca, k, metric)
                    _explode_unnest(res, qid)

                for _ in range(warm):
                    call()
                runs = []
                for _ in range(reps):
                    ph = {}
                    pm.PHASES = ph
                    _native.timing_reset()
                    _native.timing_enable(True)
                    t0 = time.perf_counter()
                    res = None
                    if leg == "first_call":
                        pm.clear_corpus_cache()
                    t1 = time.perf_counter()
                    res = pm._topk(qa, ca, k, metric)
                    t2 = time.perf_counter()
                    _explode_unnest(res, qid)
                    t3 = time.perf_counter()
                    _native.timing_enable(False)
                    pm.PHASES = None
                    h2d, kern, d2h = _native_split()
                    ph["explode_unnest"] = t3 - t2
                    runs.append((t3 - t1, t0, ph, h2d, kern, d2h))
                runs.sort(key=lambda r: r[0])
                tot, _, ph, h2d, kern, d2h = runs[len(runs) // 2]
                name = f"{dt_name}_{'array' if fixed else 'list'}_{leg}"
                dev_ms = ph.get("device", 0.0) * 1000.0
                out[name] = {
                    "ms_per_call": round(tot * 1000.0, 3), "queries_per_s": round(M / tot, 1),
                    "all_ms": sorted(round(r[0] * 1000.0, 3) for r in runs),
                    "split_ms": {"extract": round(ph.get("extract", 0.0) * 1000.0, 3),
                                 "h2d": round(h2d, 3), "kernels": round(kern, 3), "d2h": round(d2h, 3),
                                 "device_other": round(max(0.0, dev_ms - h2d - kern - d2h), 3),
                                 "assemble": round(ph.get("assemble", 0.0) * 1000.0, 3),
                                 "explode_unnest": round(ph.get("explode_unnest", 0.0) * 1000.0, 3)},
                }
                log(f"e2e {name}: {out[name]}")
        pm.clear_corpus_cache()
    # the README's figure for the reference on its (unstated) hardware
    out["reference_readme_ms"] = 45.0
    return out


def matmul_sweep(reps=10, warm=3, cpu=True):
    """benchmark_matmul.py:110-143: `.pmm.matmul` (`_matmul` on the Arrow form
    of the columns) over its points -- queries 500/1000/2000, corpus
    5000/10000/20000, dim 128/256/512 around 1000 x 10000 x 256, f32 and f64,
    Array and List inputs -- median of `reps` calls after `warm` warm-ups, as
    the reference times it (:33-41), with NumPy's BLAS product (np.dot, :23-30)
    on this host beside it."""
    from polars_matmul import _polars_matmul as pm

    base = (1000, 10000, 256)
    pts = []
    for qq in (500, 1000, 2000):
        pts.append((qq, base[1], base[2], "f32", "array"))
    for cc in (5000, 20000):
        pts.append((base[0], cc, base[2], "f32", "array"))
    for dd in (128, 512):
        pts.append((base[0], base[1], dd, "f32", "array"))
    pts.append((*base, "f64", "array"))
    pts.append((*base, "f32", "list"))
    pts.append((*base, "f64", "list"))
    rows = []
    for (m, n, d, dt_name, kind) in pts:
        dtype = np.float32 if dt_name == "f32" else np.float64
        np.random.seed(42)
        qh = np.random.randn(m, d).astype(dtype)
        ch = np.random.randn(n, d).astype(dtype)
        qa, ca = _arrow_rows(qh, kind == "array"), _arrow_rows(ch, kind == "array")
        t, _ = _median_time(lambda: pm._matmul(qa, ca), reps, warm)
        row = {"queries": m, "corpus": n, "dim": d, "dtype": dt_name, "input": kind,
               "pmm_ms": round(t * 1000.0, 3)}
        if cpu:
            tn, _ = _median_time(lambda: np.dot(qh, ch.T), reps, warm)
            row["numpy_ms"] = round(tn * 1000.0, 3)
            row["ratio"] = round(t / tn, 3)
        rows.append(row)
        log(f"matmul sweep {row}")
    return rows


# ---------------------------------------------------------------------------
# GPU measurement
# ---------------------------------------------------------------------------
def make_inputs(name, rank, world, dev):
    """(q, corpus shard, shard row offset, shard rows) on this rank's device."""
    import torch

    M, N, D, k, metric, cdt = CONFIGS[name]
    lo, hi = N * rank // world, N * (rank + 1) // world
    if name in REF_INPUT_CONFIGS:
        qh, ch = ref_inputs(M, N, D)
        q = torch.from_numpy(qh).to(dev)
        c = torch.from_numpy(ch[lo:hi].copy()).to(dev)
    else:
        q = synth_rows(0, M, D, QSEED, dev)
        c = synth_rows(lo, hi, D, CSEED, dev)
    if cdt == "bf16":
        # BASELINE configs[3]: the same f32 embeddings rounded to bf16 (RNE) on
        # device, resident before the timed region
        q, c = q.to(torch.bfloat16), c.to(torch.bfloat16)
    return q, c, lo, hi - lo


def timed_steps(runner, steps, warmup, dist, stride=1):
    """K timed steps; the library's per-kernel HIP events are recorded on
    every `stride`-th step of the timed region (1 = every step)."""
    import torch
    from polars_matmul import _native

    for _ in range(warmup):
        runner.run()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    _native.timing_reset()
    t0 = time.perf_counter()
    out = None
    if stride <= 0:
        # a sub-millisecond step: the events themselves (8 records per step)
        # add ~20 us to it (c1 0.142 ms with them on every step, 0.119 on
        # every 64th; profiles/r3_c1/timing_stride.txt), so they sample it
        stride = 1 if steps <= 20 else 50
    for i in range(steps):
        if stride > 1:
            _native.timing_enable(i % stride == 0)
        elif i == 0:
            _native.timing_enable(True)
        out = runner.run()
        if steps <= 50:
            log(f"step {i + 1}/{steps} issued")
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    _native.timing_enable(False)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=torch.device("cuda", torch.cuda.current_device()))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, out


def kernel_stats(bf16):
    from polars_matmul import _native

    names = {"gemm": "gemm_bf16_topk" if bf16 else "gemm_f32_topk",
             "seed": "seed_bf16" if bf16 else "gemm_f32_seed",
             "merge": "merge_topk", "shard_merge": "merge_shards", "norms": "norms_",
             "ff_bucket": "ff_bucket"}
    out = {}
    for key, nm in names.items():
        ms, n = _native.timing_read(nm)
        out[key] = (ms / n if n else None, n)
    if bf16:
        # which bf16 kernel ran (the library's timer names carry it); the
        # fire-and-forget kernel's re-run rows go through the ws kernel, timed
        # apart from it (per step, not per launch)
        out["bf16_kernel"] = next((v for v in ("ff", "ws", "one-wave")
                                   if _native.timing_read("gemm_bf16_topk/" + v)[1]), "ws")
        ms, n = _native.timing_read("gemm_bf16_topk/" + out["bf16_kernel"])
        out["gemm"] = (ms / n if n else None, n)
        if out["bf16_kernel"] == "ff":
            rms, rn = _native.timing_read("gemm_bf16_topk/ws")
            out["ff_rerun"] = (rms, rn)
    return out


BF16_KERNEL_NAMES = {
    "ff": "gemm_bf16_ff_kernel (256 query rows per CU on 16x16x32 MFMAs, pre-filter against a guessed "
          "static threshold, survivors stored fire-and-forget; + seed_bf16_ws_kernel in achieved)",
    "ws": "gemm_bf16_ws_kernel (wave-specialised fused GEMM + metric + top-k on 16x16x32 MFMAs; "
          "+ seed_bf16_ws_kernel in achieved)",
    "one-wave": "gemm_bf16_kernel (one-wave fused GEMM + metric + top-k)",
}


def spot_check(q, c, lo, k, metric, out_i, out_s, rows, dist, world, rank):
    """Correctness spot check on a few query rows (untimed): the f64 top-k of
    every shard on its own rank (torch on device), gathered to rank 0 and
    merged there, vs the returned global lists."""
    import torch

    dev = q.device
    qd = q[rows].double()
    cd = c.double()
    s = qd @ cd.T
    if metric == "cosine":
        s = s / (qd.norm(dim=1, keepdim=True) * cd.norm(dim=1)[None, :])
    largest = metric != "euclidean"
    if metric == "euclidean":
        s = torch.cdist(qd, cd)
    kk = min(k, s.shape[1])
    v, i = torch.topk(s, kk, dim=1, largest=largest)
    loc = torch.full((len(rows), k), float("nan"), dtype=torch.float64, device=dev)
    loc_i = torch.full((len(rows), k), -1, dtype=torch.int64, device=dev)
    loc[:, :kk] = v
    loc_i[:, :kk] = i + lo
    if world > 1:
        gv = [torch.empty_like(loc) for _ in range(world)] if rank == 0 else None
        gi = [torch.empty_like(loc_i) for _ in range(world)] if rank == 0 else None
        dist.gather(loc, gv, dst=0)
        dist.gather(loc_i, gi, dst=0)
        if rank != 0:
            return None
        allv, alli = torch.cat(gv, dim=1), torch.cat(gi, dim=1)
        fill = float("-inf") if largest else float("inf")
        allv = torch.where(torch.isnan(allv), torch.full_like(allv, fill), allv)
        ref_v, pos = torch.topk(allv, k, dim=1, largest=largest)
        ref_i = torch.gather(alli, 1, pos)
    else:
        ref_v, ref_i = loc, loc_i
    got_i = out_i[rows].long()
    got_s = out_s[rows].double()
    kth = ref_v[:, -1:]
    band = 1e-5 * kth.abs() + 1e-5
    ok = (got_s >= kth - band) if largest else (got_s <= kth + band)
    return {
        "rows": int(len(rows)),
        "valid_topk_frac": float(ok.float().mean().item()),
        "exact_index_match_frac": float((got_i == ref_i).float().mean().item()),
        "max_abs_score_err_vs_f64_topk": float((got_s - ref_v).abs().max().item()),
    }


def measure(name, steps, warmup, rank, world, dist, dev, check_rows=8, stride=1):
    """One config's timed line (inputs resident, K steps bracketed by barrier
    + synchronize, max over ranks).  Returns (fields, q, corpus shard)."""
    import torch
    from polars_matmul import _native
    from polars_matmul.sharded import ShardedTopK

    M, N, D, k, metric, cdt = CONFIGS[name]
    bf16 = cdt == "bf16"
    compute = _native.COMPUTE_BF16 if bf16 else _native.COMPUTE_F32
    mid = _native.metric_from_str(metric)
    q, c, lo, n_loc = make_inputs(name, rank, world, dev)
    ws = torch.empty(_native.workspace_bytes(M, n_loc, D, k, mid, compute), dtype=torch.uint8, device=dev)
    runner = ShardedTopK(q, c, lo, k, mid, workspace=ws)
    torch.cuda.synchronize()
    elapsed, (out_i, out_s) = timed_steps(runner, steps, warmup, dist, stride)
    ks = kernel_stats(bf16)
    merge_bytes = _native.merge_bytes(ws.data_ptr(), M, n_loc, D, k, mid, compute) if ks["merge"][1] else None
    check = None
    if check_rows:
        rows = torch.arange(0, M, max(1, M // check_rows), device=dev)[:check_rows]
        check = spot_check(q, c, lo, k, metric, out_i, out_s, rows, dist, world, rank)
    flops = 2.0 * M * n_loc * D
    peak = MFMA_PEAK_TFLOPS[cdt]
    traffic, traffic_rec = load_traffic(name) if world == 1 else (None, None)
    gemm_ms, _ = ks["gemm"]
    seed_ms, _ = ks["seed"]
    all_gemm_ms = (gemm_ms or 0.0) + (seed_ms or 0.0)
    ms_step = elapsed / steps * 1000.0
    # the dominant (fused) kernel alone: its algorithmic flops over its own
    # average launch time (HIP events on its stream); the seed / prologue
    # launch and the whole step are reported beside it, labelled
    ach = flops / (gemm_ms / 1000.0) / 1e12 if gemm_ms else None
    ach_seed = flops / (all_gemm_ms / 1000.0) / 1e12 if gemm_ms and seed_ms else None
    roof = {
        "bound": "mfma",
        "kernel": (BF16_KERNEL_NAMES[ks["bf16_kernel"]] if bf16 else
                   "gemm_f32_kernel (fused GEMM + metric + top-k)"),
        "achieved": round(ach, 2) if ach else None,
        "peak": peak, "unit": "TFLOP/s",
        "frac": round(ach / peak, 4) if ach else None,
        "fused_frac": round(ach / peak, 4) if ach else None,
        "with_seed_frac": round(ach_seed / peak, 4) if ach_seed else None,
        "traffic": traffic,
        "traffic_record": traffic_rec,
        # per launch of the dominant kernel; the threshold seed (small
        # problems and bf16) is a launch of its own, counted
        # only in "with_seed_frac" and "step_frac"
        "kernel_ms_avg": round(gemm_ms, 3) if gemm_ms else None,
        "kernel_launches_timed": ks["gemm"][1],
        "seed_ms_avg": round(seed_ms, 3) if seed_ms else None,
        "seed_us": round(seed_ms * 1000.0, 2) if seed_ms else None,
        "flops_per_launch": flops,
        # the whole step (norms, fills, seed, GEMM, merge, gather) against the peak
        "step_frac": round(flops / (ms_step / 1000.0) / 1e12 / peak, 4),
        "merge_ms_avg": round(ks["merge"][0], 3) if ks["merge"][0] else None,
        "shard_merge_ms_avg": round(ks["shard_merge"][0], 3) if ks["shard_merge"][0] else None,
        "norms_ms_avg": round(ks["norms"][0], 3) if ks["norms"][0] else None,
    }
    if ks["ff_bucket"][1]:
        roof["ff_bucket_ms_avg"] = round(ks["ff_bucket"][0], 3)
    if "ff_rerun" in ks:
        # total re-run kernel time over the timed launches' steps, and its launches
        roof["ff_rerun_ms_total"] = round(ks["ff_rerun"][0], 3)
        roof["ff_rerun_launches"] = ks["ff_rerun"][1]
    reduction = None
    if ks["merge"][1] and merge_bytes:
        mavg = ks["merge"][0] / 1000.0
        gbs = merge_bytes / mavg / 1e9
        reduction = {
            "kernel": "merge_kernel (per-row merge of the split candidate buffers)",
            "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_launch": merge_bytes,
            "kernel_ms_avg": round(mavg * 1000.0, 3),
        }
        if ks["shard_merge"][1]:
            # rank 0's k-way merge of the world x M x k (index, score) lists
            sbytes = (world + 1) * M * k * 8
            savg = ks["shard_merge"][0] / 1000.0
            reduction["shard_merge"] = {"bytes_per_launch": sbytes, "kernel_ms_avg": round(savg * 1000.0, 3),
                                        "achieved": round(sbytes / savg / 1e9, 1), "unit": "GB/s"}
    small = None
    if not bf16 and seed_ms and M * n_loc * D < 10**11:
        # each small launch of a reference-size step against
        # its own floor.  The prologue (seed + norms + fills, one launch):
        # reads Q and C once, writes the norms / pre-filter factors and the
        # seeded thresholds, and runs the sample's dot products (2 M ns D
        # flops) and the norms (2 (M + N) D) on the vector ALUs.  The merge:
        # merge_bytes (the split counts, surviving candidates, thresholds,
        # the M x k output).  floor = max(bytes / HBM peak, flops / f32 peak).
        ns = min(n_loc, 1 << max(8, (8 * k - 1).bit_length()))
        pbytes = (M + n_loc) * D * 4 + (M + 2 * n_loc) * 4 + M * 8
        pflops = 2.0 * M * ns * D + 2.0 * (M + n_loc) * D
        small = {"prologue": {"kernel": "prologue_kernel (seed dots + norms + fills)", "us_avg": round(seed_ms * 1000.0, 2),
                              "bytes": pbytes, "flops": pflops, "seed_rows": ns}}
        if ks["merge"][0] and merge_bytes:
            small["merge"] = {"kernel": "merge_kernel", "us_avg": round(ks["merge"][0] * 1000.0, 2), "bytes": merge_bytes,
                              "flops": 0.0}
        for v in small.values():
            floor_s = max(v["bytes"] / (HBM_PEAK_GBS * 1e9), v["flops"] / (MFMA_PEAK_TFLOPS["f32"] * 1e12))
            v["floor_us"] = round(floor_s * 1e6, 2)
            v["gbs"] = round(v["bytes"] / (v["us_avg"] * 1e-6) / 1e9, 1)
            v["frac_of_floor"] = round(floor_s * 1e6 / v["us_avg"], 3)
        small["fused_us_avg"] = round(gemm_ms * 1000.0, 2) if gemm_ms else None
    lists = out_i.cpu().numpy() if (world == 1 or rank == 0) else None
    fields = {
        "config": {"workload": f"{M}x{N}x{D} {cdt} {metric} k={k} ({name})", "queries": M, "corpus": N,
                   "dim": D, "k": k, "metric": metric,
                   "parallelism": f"corpus-row-shard x{world}" if world > 1 else "single GPU"},
        "dtype": cdt, "value": round(M * steps / elapsed, 2), "unit": "queries/s",
        "ms_per_step": round(ms_step, 3), "steps": steps, "warmup": warmup,
        "roofline": roof, "reduction_roofline": reduction, "check": check,
    }
    if small:
        fields["small_kernels"] = small
    del runner, ws
    return fields, q, c, lists


def cpu_selftest(args, rank, world):
    """Launcher / gather / merge plumbing on CPU (gloo): a small synthetic
    problem whose per-shard top-k and merge are plain torch on the host.  Used
    by tests/test_bench_launcher.py; measures nothing."""
    import torch
    import torch.distributed as dist

    from polars_matmul.sharded import ShardedTopK, shard_bounds

    if world > 1:
        dist.init_process_group("gloo")
    g = torch.Generator()
    g.manual_seed(7)
    M, N, D, k = 24, 300, 16, 10
    q = torch.randn((M, D), generator=g)
    c = torch.randn((N, D), generator=g)
    lo, hi = shard_bounds(N, world, rank)

    def local(qq, cc, kk, metric, base, oi, os_, ws):
        v, i = torch.topk(qq @ cc.T, kk, dim=1)
        oi.copy_(i.to(torch.int32) + base)
        os_.copy_(v)

    def merge(gathered, kk, metric, oi, os_):
        ii = gathered[:, 0].permute(1, 0, 2).reshape(M, -1)
        ss = gathered[:, 1].view(torch.float32).permute(1, 0, 2).reshape(M, -1)
        v, pos = torch.topk(ss, kk, dim=1)
        oi.copy_(torch.gather(ii, 1, pos))
        os_.copy_(v)

    st = ShardedTopK(q, c[lo:hi].contiguous(), lo, k, 1, local_topk=local, merge=merge)
    oi, osc = st.run()
    if rank == 0:
        v, i = torch.topk(q @ c.T, k, dim=1)
        ok = bool(torch.equal(oi.long(), i)) and bool(torch.allclose(osc, v))
        print(json.dumps({"metric": "cpu selftest", "n_gpus": world, "ranks_ok": ok}), flush=True)
    if world > 1:
        dist.destroy_process_group()


F64_MFMA_PEAK_TFLOPS = 78.6  # MI355X FP64 matrix, AMD spec (MI355X_MICROARCH.md lists no f64 row)


F64_LARGE = (4096, 1_000_000, 256, 10, "cosine")  # the f64 path where the M x N matrix (32 GB) must not exist


def f64_line(steps=200, warmup=10, large=False):
    """the f64 top-k (what Polars' default Float64 columns
    take; src/matmul.rs:449-468) resident in HBM: pmm_topk_f64_device per
    step, fused (PMM_F64_FUSED=1) and materialised (PMM_F64_FUSED=0) timed one
    after the other, plus the library's default choice; the GEMM launches'
    roofline against the f64 MFMA peak.  large=False: the reference
    benchmark's size, c1 inputs as f64 (seed 42, cosine, k = 10);
    large=True: F64_LARGE, device-generated N(0,1) rows (seed 7)."""
    import torch
    from polars_matmul import _native

    dev = torch.device("cuda", torch.cuda.current_device())
    if large:
        M, N, D, k, metric = F64_LARGE
        g = torch.Generator(device=dev)
        g.manual_seed(7)
        q = torch.randn((M, D), dtype=torch.float64, device=dev, generator=g)
        c = torch.randn((N, D), dtype=torch.float64, device=dev, generator=g)
        qh, ch = None, None
    else:
        M, N, D, k, metric = CONFIGS["c1"][:5]
        qh, ch = ref_inputs(M, N, D)
        q = torch.from_numpy(qh.astype(np.float64)).to(dev)
        c = torch.from_numpy(ch.astype(np.float64)).to(dev)
    mid = _native.metric_from_str(metric)
    oi = torch.empty((M, k), dtype=torch.int32, device=dev)
    os_ = torch.empty((M, k), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def run():
        _native.topk_f64_device(q.data_ptr(), D, M, c.data_ptr(), D, N, D, k, mid, oi.data_ptr(), os_.data_ptr(),
                                stream=stream)

    out = {"workload": f"{M}x{N}x{D} f64 {metric} k={k} " +
           ("(device N(0,1) rows)" if large else "(c1 inputs as f64)"), "dtype": "f64"}
    for mode in ("fused", "materialised", "default"):
        if mode != "default":
            os.environ["PMM_F64_FUSED"] = "1" if mode == "fused" else "0"
        try:
            for _ in range(warmup):
                run()
            torch.cuda.synchronize()
            _native.timing_reset()
            _native.timing_enable(True)
            t0 = time.perf_counter()
            for _ in range(steps):
                run()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            _native.timing_enable(False)
        finally:
            os.environ.pop("PMM_F64_FUSED", None)
        gms, gn = _native.timing_read("gemm_f64_topk")
        if not gn:
            gms, gn = _native.timing_read("gemm_f64_scores")
        tot, tn = _native.timing_read("")
        ach = 2.0 * M * N * D / (gms / steps / 1000.0) / 1e12 if gn else None
        rec = {"value": round(M * steps / el, 2), "unit": "queries/s", "ms_per_step": round(el / steps * 1000.0, 4),
               "steps": steps, "warmup": warmup, "gemm_ms_per_step": round(gms / steps, 4) if gn else None,
               "gemm_launches_per_step": gn // steps if gn else None,
               "kernels_ms_per_step": round(tot / steps, 4) if tn else None}
        if ach:
            rec["roofline"] = {"bound": "mfma", "achieved": round(ach, 2), "peak": F64_MFMA_PEAK_TFLOPS,
                               "unit": "TFLOP/s", "frac": round(ach / F64_MFMA_PEAK_TFLOPS, 4),
                               "peak_source": "AMD spec (FP64 matrix); not in MI355X_MICROARCH.md"}
        out[mode] = rec
        log(f"f64 {mode}: {rec}")
    # exactness of this run's lists against the oracle (first rows)
    import oracle

    nr = 4 if large else 64
    got = oi.cpu().numpy().view(np.uint32)
    if large:
        qh, ch = q[:nr].cpu().numpy(), c.cpu().numpy()
    oi_, _ = oracle.topk(qh[:nr].astype(np.float64), ch.astype(np.float64), k, oracle.metric_from_str(metric))
    out["check"] = {"rows": nr, "exact_index_match_frac": float(np.mean(got[:nr] == oi_))}
    del q, c
    torch.cuda.empty_cache()
    return out


def inproc_child(args) -> None:
    """the drop-in boundary's own multi-GPU transport, in ONE
    fresh process (started by rank 0 after the RCCL ranks are done, before
    anything here touches the GPU): pmm_set_devices(0..N-1), a corpus handle
    row-sharded over the N devices at creation (pmm_corpus_create_f32), then
    pmm_topk_f32_corpus per step -- host queries uploaded to every device,
    every device's fused top-k concurrently, the [2][M][k] lists copied peer
    to peer into device 0 and merged there, results downloaded.  Prints one
    JSON line."""
    import torch
    from polars_matmul import _native

    n = args.inproc_child
    M, N, D, k, metric, cdt = CONFIGS[args.config]
    if cdt != "f32":
        print(json.dumps({"error": "in-process transport measured for f32 configs only"}), flush=True)
        return
    mid = _native.metric_from_str(metric)
    dev0 = torch.device("cuda", 0)
    # the same rows bench.py's ranks generate, brought to the host
    qh = synth_rows(0, M, D, QSEED, dev0).cpu().numpy()
    ch = synth_rows(0, N, D, CSEED, dev0).cpu().numpy()
    torch.cuda.empty_cache()
    # (rehearsal on a one-GPU box: PMM_BENCH_INPROC_DEVICES=0,0 lists device 0 twice)
    devs = os.environ.get("PMM_BENCH_INPROC_DEVICES")
    _native.set_devices([int(x) for x in devs.split(",")] if devs else list(range(n)))
    t0 = time.perf_counter()
    dc = _native.DeviceCorpus(ch)
    up = time.perf_counter() - t0
    del ch
    steps, warm = max(1, min(args.steps, 5)), max(1, min(args.warmup, 1))
    for _ in range(warm):
        dc.topk(qh, k, mid)
    _native.timing_reset()
    _native.timing_enable(True)
    ts = []
    for _ in range(steps):
        t1 = time.perf_counter()
        out_i, _ = dc.topk(qh, k, mid)
        ts.append(time.perf_counter() - t1)
    _native.timing_enable(False)
    gms, gn = _native.timing_read("gemm_f32_topk")
    mms, mn = _native.timing_read("merge_devices")
    h2d, hn = _native.timing_read("h2d")
    dt = float(np.median(ts))
    print(json.dumps({
        "transport": "in-process (pmm_set_devices + sharded corpus handle; peer copies into device 0)",
        "n_gpus": n, "devices": _native.get_devices(), "shards": dc.shards, "workload": f"{M}x{N}x{D} {cdt} {metric} k={k} ({args.config})",
        "value": round(M / dt, 2), "unit": "queries/s", "ms_per_call": round(dt * 1000.0, 3),
        "steps": steps, "warmup": warm, "all_ms": [round(t * 1000.0, 3) for t in ts],
        "shard_kernel_ms_avg": round(gms / gn, 3) if gn else None, "shard_kernel_launches": gn,
        "root_merge_ms_avg": round(mms / mn, 3) if mn else None,
        "h2d_ms_per_call": round(h2d / steps, 3) if hn else None,
        "corpus_upload_s": round(up, 3),
        "note": "host queries in, host lists out (the .pmm.topk boundary): the H2D of the queries to every "
                "device and the D2H of the merged lists are inside the call",
    }), flush=True)
    dc.close()


class EarlySpawner:
    """A helper process forked BEFORE this process touches the GPU, which later
    starts one program on request and returns its exit status and output.  A
    process that has initialised the GPU must not exec another program; the
    helper never initialises it, so the program it starts is clean."""

    def __init__(self):
        r1, w1 = os.pipe()
        r2, w2 = os.pipe()
        pid = os.fork()
        if pid == 0:  # the helper: no GPU, no torch
            os.close(w1)
            os.close(r2)
            code = 0
            try:
                with os.fdopen(r1, "rb") as f:
                    req = f.read()
                if req:
                    job = json.loads(req)
                    try:
                        r = subprocess.run(job["cmd"], env=job["env"], capture_output=True, text=True,
                                           timeout=job["timeout"])
                        res = {"rc": r.returncode, "stdout": r.stdout, "stderr": r.stderr}
                    except subprocess.TimeoutExpired:
                        res = {"rc": None, "stdout": "", "stderr": f"timed out after {job['timeout']} s"}
                    with os.fdopen(w2, "wb") as f:
                        f.write(json.dumps(res).encode())
            except Exception:
                code = 1
            os._exit(code)
        os.close(r1)
        os.close(w2)
        self.pid, self.w, self.r = pid, w1, r2

    def run(self, cmd, env, timeout):
        with os.fdopen(self.w, "wb") as f:
            f.write(json.dumps({"cmd": cmd, "env": env, "timeout": timeout}).encode())
        self.w = None
        with os.fdopen(self.r, "rb") as f:
            out = f.read()
        self.r = None
        os.waitpid(self.pid, 0)
        return json.loads(out) if out else {"rc": None, "stdout": "", "stderr": "helper failed"}

    def close(self):
        if self.w is not None:  # never used: let the helper exit
            os.close(self.w)
            os.close(self.r)
            os.waitpid(self.pid, 0)
            self.w = self.r = None


def run_inproc_child(args, world, spawner):
    """Start the in-process transport measurement as a fresh child process
    (through the early helper; no torch.distributed env) and return its JSON
    record."""
    env = {kk: v for kk, v in os.environ.items()
           if kk not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                         "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE", "TORCHELASTIC_RUN_ID")}
    cmd = [sys.executable, os.path.abspath(__file__), "--inproc-child", str(world), "--config", args.config,
           "--steps", str(args.steps), "--warmup", str(args.warmup)] + (["--metric", args.metric] if args.metric else [])
    # (c5's child synthesises a 40 GB host corpus, uploads it sharded and runs
    # ~18 s steps: a longer limit for problems of that size)
    M, N, D = CONFIGS[args.config][:3]
    timeout = args.inproc_timeout if args.inproc_timeout > 0 else (900 if M * N * D > 1e15 else 300)
    r = spawner.run(cmd, env, timeout)
    lines = [x for x in r["stdout"].splitlines() if x.startswith("{")]
    if r["rc"] != 0 or not lines:
        return {"error": f"in-process child rc={r['rc']}", "stderr_tail": r["stderr"][-800:]}
    return json.loads(lines[-1])


def extra_line(name, steps, warmup, dev, args):
    """Secondary workload on this GPU (N = 1 runs only), reported under
    "extra"; the reference-size configs also carry their CPU baselines timed
    in full (configs[0] = c1: examples/benchmark_topk.py)."""
    import torch

    M, N, D = CONFIGS[name][:3]
    small = M * N * D < 10**11  # sub-millisecond steps: time more of them
    st, wu = (max(steps, 200), max(warmup, 10)) if small else (steps, warmup)
    if name == "c5_rank":
        st, wu = 2, 1  # ~18 s per step: 1 warm-up + 2 timed steps keep the default run within minutes
    fields, q, c, lists = measure(name, st, wu, 0, 1, None, dev, check_rows=8, stride=args.timing_stride)
    ref = args.ref_lists.get(CONFIGS[name][:5])
    if CONFIGS[name][5] == "bf16" and ref is not None and fields["check"] is not None:
        # SURVEY 8c's bf16 bar: recall@k of the bf16 lists against the f32
        # lists of the same rows (the main line's c3 output, same inputs)
        fields["check"]["recall_at_k_vs_f32_all_rows"] = round(recall_at_k(lists, ref), 6)
    del lists
    if name == "c1":
        # the reference's own benchmark, end to end through `_topk` on Arrow
        # List / Array columns (host buffers in, Arrow List[Struct] out)
        fields["boundary"] = e2e_topk_line()
    if name in REF_INPUT_CONFIGS and args.cpu_sample:
        k, metric = CONFIGS[name][3], CONFIGS[name][4]
        qh, ch = ref_inputs(M, N, D)
        qps, dt, ph = cpu_blas_qps(qh, ch, k, metric, args.cpu_threads, reps=5, warm=2)
        fields["cpu_baseline"] = {
            "value": round(qps, 2), "unit": "queries/s", "cores": args.cpu_threads,
            "host_nproc": os.cpu_count(), "available_parallelism": available_parallelism(), "kind": "port",
            "gemm": f"{blas_name()} sgemm via NumPy, {args.cpu_threads} threads (faer Rayon(0)'s role)",
            "sample": f"the full {M}x{N}x{D} {metric} k={k} workload (seed-42 inputs, "
                      f"benchmark_topk.py:69-71), median of 5 after 2 warm-ups: {dt * 1000:.1f} ms; the "
                      "reference's structure (norms, threaded BLAS GEMM, 1-thread epilogue + per-row select; "
                      "oracle.topk_blas)",
            "phases_ms": ph,
        }
        oqps, odt = cpu_oracle_qps(qh, ch, k, metric, args.cpu_threads, reps=5, warm=2)
        fields["cpu_baseline_oracle_loop"] = {
            "value": round(oqps, 2), "unit": "queries/s", "cores": args.cpu_threads, "kind": "port",
            "sample": f"full workload, median of 5 after 2 warm-ups: {odt * 1000:.1f} ms; oracle/pmm_oracle.c "
                      "with its own scalar-blocked GEMM (the checker)",
        }
        if metric == "cosine":
            nq, ndt = numpy_comparator(qh, ch, k, reps=5, warm=2)
            fields["cpu_baseline_numpy"] = {
                "value": round(nq, 2), "unit": "queries/s",
                "cores": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)),
                "host_nproc": os.cpu_count(), "available_parallelism": available_parallelism(), "kind": "port",
                "sample": f"full workload, median of 5 after 2 warm-ups: {ndt * 1000:.1f} ms; the reference "
                          "README's NumPy comparator (benchmark_topk.py:14-33)",
            }
    del q, c
    torch.cuda.empty_cache()
    return fields


def _brief(rec):
    """value / ms per step / roofline fraction of one line (None-free)."""
    out = {}
    for key in ("value", "ms_per_step", "ms_per_call"):
        if rec.get(key) is not None:
            out[key] = rec[key]
    roof = rec.get("roofline") or {}
    if roof.get("frac") is not None:
        out["frac"] = roof["frac"]
    if roof.get("kernel_ms_avg") is not None:
        out["kernel_ms"] = roof["kernel_ms_avg"]
    return out


def summary_of(line):
    """A compact digest of the whole line (the headline and every extra's
    value, ms per step and roofline fraction), printed as the line's LAST key
    so that a reader of only the tail of stdout (the driver keeps the last
    16 kB) sees every config's numbers."""
    out = {"headline": dict(_brief(line), config=line["config"]["workload"])}
    for name, rec in (line.get("extra") or {}).items():
        if not isinstance(rec, dict):
            continue
        if name in ("c1_f64", "f64_large"):
            b = _brief(rec.get("default") or {})
            b["fused_ms"] = (rec.get("fused") or {}).get("ms_per_step")
            b["materialised_ms"] = (rec.get("materialised") or {}).get("ms_per_step")
            out[name] = b
            continue
        if name == "c5_root_merge":
            out[name] = {"gbs": rec.get("value"), "frac": rec.get("frac"), "kernel_ms": rec.get("kernel_ms_avg"),
                         "general_frac": (rec.get("general") or {}).get("frac")}
            continue
        b = _brief(rec)
        if rec.get("roofline", {}).get("step_frac") is not None and name in ("c1", "c2"):
            b["step_frac"] = rec["roofline"]["step_frac"]
            b["seed_us"] = rec["roofline"].get("seed_us")
        if name == "matmul":
            b["link_frac"] = rec.get("link_frac")
        if name == "c1" and isinstance(rec.get("boundary"), dict):
            b["e2e_ms"] = {leg: v["ms_per_call"] for leg, v in rec["boundary"].items()
                           if isinstance(v, dict) and "ms_per_call" in v}
            b["e2e_h2d_ms"] = {leg: v["split_ms"]["h2d"] for leg, v in rec["boundary"].items()
                               if isinstance(v, dict) and "split_ms" in v}
        if rec.get("reduction_roofline"):
            b["merge_frac_hbm"] = rec["reduction_roofline"].get("frac")
        if rec.get("small_kernels"):
            b["small_kernels_us"] = {kk: (v.get("us_avg") if isinstance(v, dict) else v)
                                     for kk, v in rec["small_kernels"].items()}
        if rec.get("cpu_baseline"):
            b["cpu_baseline"] = rec["cpu_baseline"].get("value")
        out[name] = b
    cpu = line.get("cpu_baseline")
    if cpu:
        out["cpu_baseline"] = {"value": cpu.get("value"), "unit": cpu.get("unit"), "cores": cpu.get("cores")}
    return out


def descendants(pid: int):
    """Live descendant processes of pid (via /proc/<pid>/task/*/children)."""
    out, todo = [], [pid]
    while todo:
        p = todo.pop()
        try:
            tasks = os.listdir(f"/proc/{p}/task")
        except OSError:
            continue
        for t in tasks:
            try:
                with open(f"/proc/{p}/task/{t}/children") as f:
                    kids = [int(x) for x in f.read().split()]
            except (OSError, ValueError):
                continue
            for kid in kids:
                try:
                    with open(f"/proc/{kid}/cmdline", "rb") as f:
                        cmd = f.read().replace(b"\0", b" ").decode(errors="replace").strip()
                except OSError:
                    cmd = "?"
                out.append((kid, p, cmd))
                todo.append(kid)
    return out


def report_descendants(tag: str) -> None:
    """the driver saw one process alive at the end of the
    bench (procs_at_end: 1) while an N = 1 run starts none on purpose; name
    every descendant still alive (and this process's threads) on stderr."""
    kids = descendants(os.getpid())
    try:
        nthreads = len(os.listdir(f"/proc/{os.getpid()}/task"))
    except OSError:
        nthreads = -1
    log(f"[bench] {tag}: pid {os.getpid()}, {nthreads} threads, {len(kids)} live descendant process(es)"
        + "".join(f"\n[bench]   pid {k} (parent {p}): {c[:200]}" for k, p, c in kids))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-sample", type=int, default=512,
                    help="queries timed on the CPU baseline vs the full corpus (0 = skip CPU baselines)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="oracle baseline threads (0 = available_parallelism(), as faer's Rayon(0))")
    ap.add_argument("--boundary", type=int, default=1, help="also time the host-buffer C ABI (N=1)")
    ap.add_argument("--extra", default="c4,c1,c2,c1_f64,f64_large,matmul,c5_rank,c5_root_merge",
                    help="comma-separated secondary configs measured after the main line (N=1; 'none' = none; "
                         "'matmul' = .pmm.matmul at the c1 size; 'c1_f64' = the f64 top-k at the c1 size; "
                         "'f64_large' = the f64 top-k at 4096 x 1M x 256; 'c5_rank' = configs[4]'s per-GPU "
                         "share, 1M x 1.25M x 1024, 1 warm-up + 2 timed steps; 'c5_root_merge' = configs[4]'s root "
                         "merge of 8 x 1M x 100 gathered lists)")
    ap.add_argument("--metric", choices=("cosine", "dot", "euclidean"), default=None,
                    help="replace the main config's metric (the extras keep theirs)")
    ap.add_argument("--check", type=int, default=8, help="query rows spot-checked against an f64 top-k")
    ap.add_argument("--timing-stride", type=int, default=0,
                    help="record the per-kernel HIP events on every n-th timed step (0: every step of "
                         "a run of at most 20 steps, every 50th of a longer one)")
    ap.add_argument("--cpu-selftest", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--inproc", type=int, default=1,
                    help="N > 1: after the RCCL ranks, also measure the in-process transport (one child "
                         "process driving all N GPUs through pmm_set_devices) under extra.inproc")
    ap.add_argument("--inproc-timeout", type=int, default=0, help=argparse.SUPPRESS)  # 0: by problem size
    ap.add_argument("--inproc-child", type=int, default=0, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.metric and args.metric != CONFIGS[args.config][4]:
        global METRIC_OVERRIDE
        METRIC_OVERRIDE = args.metric
        CONFIGS[args.config] = CONFIGS[args.config][:4] + (args.metric,) + CONFIGS[args.config][5:]
    if args.inproc_child:
        inproc_child(args)
        return

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # this process only launches: no torch.cuda / HIP call happens here
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
        sys.exit(2)
    if args.cpu_selftest:
        cpu_selftest(args, rank, world)
        return
    if args.cpu_threads <= 0:
        args.cpu_threads = available_parallelism()
    # rank 0 of an N > 1 run starts the in-process transport's measurement
    # after the RCCL one: fork its helper now, before anything touches the GPU
    spawner = EarlySpawner() if (world > 1 and rank == 0 and args.inproc) else None

    import torch

    dist = None
    # rehearsal of the N > 1 path on a one-GPU box: every rank on device 0 and
    # the gloo backend (RCCL refuses two ranks on one GPU); the numbers of such
    # a run measure nothing, the line says so
    share = world > 1 and os.environ.get("PMM_BENCH_SHARE_GPU") == "1"
    if share:
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
        os.environ.setdefault("PMM_BENCH_INPROC_DEVICES", ",".join("0" * world))
    elif world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from polars_matmul import _native

    _native.check(_native.lib().pmm_set_device(torch.cuda.current_device()))

    M, N, D, k, metric, cdt = CONFIGS[args.config]
    fields, q, c, lists = measure(args.config, args.steps, args.warmup, rank, world, dist, dev, args.check,
                                  args.timing_stride)
    if fields["check"]:
        log(f"spot check: {fields['check']}")
    # f32 lists of this workload's (M, N, D, k, metric) for the bf16 recall check of an extra line
    args.ref_lists = {CONFIGS[args.config][:5]: lists} if cdt == "f32" and lists is not None else {}
    del lists

    boundary = None
    if args.boundary and world == 1 and args.config not in ("c5",):
        boundary = boundary_rates(q.float(), c.float(), k, _native.metric_from_str(metric),
                                  _native.COMPUTE_BF16 if cdt == "bf16" else _native.COMPUTE_F32)
        log(f"boundary: {boundary}")

    cpu = cpu_np = cpu_oracle = None
    if args.cpu_sample and world == 1 and rank == 0:
        n_s = min(args.cpu_sample, M)
        qh = q[:n_s].float().cpu().numpy()
        ch = c.float().cpu().numpy()
        # bf16: the baselines on the bf16-rounded rows (widened to f32, exact)
        cpu_qps, cpu_dt, cpu_ph = cpu_blas_qps(qh, ch, k, metric, args.cpu_threads)
        cpu = {
            "value": round(cpu_qps, 2), "unit": "queries/s", "cores": args.cpu_threads,
            "host_nproc": os.cpu_count(), "available_parallelism": available_parallelism(), "kind": "port",
            "gemm": f"{blas_name()} sgemm via NumPy, {args.cpu_threads} threads (faer Rayon(0)'s role)",
            "sample": f"first {n_s} queries x full {N}-row corpus, {D}d {cdt} {metric} k={k}; the reference's "
                      f"structure (matmul.rs:420-469): norms, threaded BLAS GEMM into the M x N matrix, "
                      f"1-thread epilogue + per-row select (oracle.topk_blas), {cpu_dt:.1f}s",
            "phases_ms": cpu_ph,
        }
        o_qps, o_dt = cpu_oracle_qps(qh[:min(n_s, 128)], ch, k, metric, args.cpu_threads)
        cpu_oracle = {
            "value": round(o_qps, 2), "unit": "queries/s", "cores": args.cpu_threads, "kind": "port",
            "sample": f"first {min(n_s, 128)} queries x full corpus; oracle/pmm_oracle.c's own scalar-blocked "
                      f"GEMM (the checker's k-ordered chain), {o_dt:.1f}s",
        }
        if metric == "cosine":
            np_qps, np_dt = numpy_comparator(qh, ch, k)
            cpu_np = {
                "value": round(np_qps, 2), "unit": "queries/s",
                "cores": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)),
                "host_nproc": os.cpu_count(), "available_parallelism": available_parallelism(), "kind": "port",
                "sample": f"first {n_s} queries x full {N}-row corpus; the reference README's NumPy "
                          f"comparator (normalise, BLAS GEMM, argpartition, argsort), {np_dt:.1f}s",
            }
        del ch

    extra = None
    if args.extra and world == 1:
        del q, c
        torch.cuda.empty_cache()
        extra = {}
        for name in [x for x in args.extra.split(",") if x and x not in (args.config, "none")]:
            extra[name] = (matmul_line(args) if name == "matmul" else f64_line() if name == "c1_f64"
                           else f64_line(steps=3, warmup=1, large=True) if name == "f64_large"
                           else root_merge_line() if name == "c5_root_merge"
                           else extra_line(name, args.steps, args.warmup, dev, args))
            log(f"extra {name}: {json.dumps(extra[name])}")

    if rank != 0:
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return
    inproc = None
    if world > 1:
        dist.barrier()  # the other ranks leave after this barrier
    if world > 1 and args.inproc:
        # the RCCL measurement is complete on every rank; free this rank's
        # device memory and let the other ranks exit, then one fresh process
        # drives all N GPUs through the drop-in boundary
        del q, c
        torch.cuda.empty_cache()
        inproc = run_inproc_child(args, world, spawner)
        log(f"inproc: {inproc}")

    line = {
        "metric": f"{metric} top-k queries/sec",
        "value": fields["value"],
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": fields["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": cdt,
        "data": ("synthetic N(0,1) f32 embeddings generated on device (torch.randn, one seeded generator "
                 "per 65,536-row block)" if args.config not in REF_INPUT_CONFIGS else
                 "seed-42 NumPy randn inputs (examples/benchmark_topk.py:69-71)")
                + (", rounded to bf16 on device" if cdt == "bf16" else ""),
        "config": fields["config"],
        "roofline": fields["roofline"],
        "reduction_roofline": fields["reduction_roofline"],
        "cpu_baseline": cpu,
        "cpu_baseline_numpy": cpu_np,
        "cpu_baseline_oracle_loop": cpu_oracle,
        "boundary": boundary,
        "extra": extra if inproc is None else dict(extra or {}, inproc=inproc),
        "check": fields["check"],
    }
    if share:
        line["rehearsal"] = "PMM_BENCH_SHARE_GPU=1: every rank on device 0, gloo; not a measurement"
    line["summary"] = summary_of(line)  # (last key: see summary_of)
    if spawner:
        spawner.close()
    if dist:
        dist.destroy_process_group()
    report_descendants("before the result line")
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
