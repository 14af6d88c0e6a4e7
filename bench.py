#!/usr/bin/env python3
"""Headline benchmark: cosine top-k queries/sec on MI355X.

Workload (BASELINE.json configs[2], the config its metric is quoted on; it fits
one GPU): 100,000 queries x 1,000,000 corpus rows x 768 dims, f32, cosine,
k = 100.  Synthetic N(0,1) f32 embeddings generated on device (torch.randn,
seeded); inputs are resident in HBM before the timed region.

One step = one full top-k pass of all M queries against the corpus:
  N = 1: fused GEMM + top-k (libpmm.so, pmm_topk_f32_device) over the corpus.
  N > 1: the corpus is row-sharded over the ranks (one process per GPU);
         each rank runs the fused top-k on its shard (global indices via
         index_base), rank 0 gathers the per-shard M x k lists over RCCL
         (torch.distributed "nccl" = RCCL) and k-way merges them
         (pmm_merge_topk_device).  Total work is fixed: "scaling": "strong".

Run: python bench.py [--gpus N] [--steps K] [--warmup W]
     (N > 1 under torch.distributed.run, one rank per GPU)

Prints ONE JSON line on rank 0 with the metric, the dominant kernel's roofline
(achieved TFLOP/s from HIP events on its launch stream vs the 157.3 TFLOP/s
f32 MFMA peak) and a CPU baseline (the oracle, a port of the reference's
algorithm, on a bounded query sample on this host's cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "polars-matmul_amd"), os.path.join(ROOT, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

CONFIGS = {
    # name: (M, N, D, k, metric, compute dtype)
    "c3": (100_000, 1_000_000, 768, 100, "cosine", "f32"),
    "c4": (100_000, 1_000_000, 768, 100, "cosine", "bf16"),
    "c2": (1_000, 10_000, 256, 10, "dot", "f32"),
    "c1": (1_000, 10_000, 256, 10, "cosine", "f32"),
}
MFMA_PEAK_TFLOPS = {"f32": 157.3, "bf16": 2516.6}  # MI355X dense matrix peaks (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_traffic(config: str):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3
    --pmc summary (profiles/), corrected as MI355X_MICROARCH.md prescribes."""
    path = os.path.join(ROOT, "profiles", f"pmc_traffic_{config}.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except Exception:
        return None


def cpu_baseline(q_dev, c_dev, k, metric, n_sample, threads):
    """Time the oracle (reference structure: threaded GEMM, single-threaded
    epilogue + per-row select) on the first n_sample queries vs the full
    corpus; returns queries/sec."""
    import oracle

    q = q_dev[:n_sample].float().cpu().numpy()
    c = c_dev.float().cpu().numpy()
    mid = oracle.metric_from_str(metric)
    t0 = time.perf_counter()
    oracle.topk(q, c, k, mid, nthreads=threads)
    dt = time.perf_counter() - t0
    return n_sample / dt, dt


def numpy_comparator_qps(q_dev, c_dev, k, n_sample):
    """SURVEY 8d CPU baseline (2): the README's NumPy comparator
    (examples/benchmark_topk.py:14-33 in the reference) restated -- L2-normalise
    both sides, one BLAS GEMM, a per-row partial selection of k, then a sort
    of those k -- on the first n_sample queries against the full corpus.
    Cosine only; BLAS threads as the environment sets them."""
    q = q_dev[:n_sample].float().cpu().numpy()
    c = c_dev.float().cpu().numpy()
    t0 = time.perf_counter()
    qn = q / np.sqrt((q * q).sum(axis=1, keepdims=True))
    cn = c / np.sqrt((c * c).sum(axis=1, keepdims=True))
    sim = qn @ cn.T
    cut = sim.shape[1] - k
    part = np.argpartition(sim, cut, axis=1)[:, cut:]
    vals = np.take_along_axis(sim, part, axis=1)
    order = np.argsort(-vals, axis=1)
    np.take_along_axis(part, order, axis=1)
    dt = time.perf_counter() - t0
    return n_sample / dt, dt


def boundary_rates(q_dev, c_dev, k, metric_id, compute=0):
    """Host-boundary rates: host f32 buffers in, host idx/score
    out, through the C ABI, one call each (untimed by the contract's clock):
      host_api: pmm_topk_f32 -- pads+uploads Q and C, computes, downloads;
      cached_corpus: pmm_topk_f32_corpus -- corpus resident (uploaded once,
        as the Arrow-keyed cache does across map_batches calls), Q uploaded
        and results downloaded per call."""
    from polars_matmul import _native

    qh = q_dev.cpu().numpy()
    ch = c_dev.cpu().numpy()
    M = qh.shape[0]
    out = {}
    t0 = time.perf_counter()
    _native.topk_host(qh, ch, k, metric_id, compute=compute)
    out["host_api_qps"] = round(M / (time.perf_counter() - t0), 2)
    if compute != _native.COMPUTE_F32:
        return out  # the corpus handle is f32-only
    t0 = time.perf_counter()
    dc = _native.DeviceCorpus(ch)
    out["corpus_upload_s"] = round(time.perf_counter() - t0, 3)
    dc.topk(qh[:1024], k, metric_id)  # first-call allocations
    t0 = time.perf_counter()
    dc.topk(qh, k, metric_id)
    out["cached_corpus_qps"] = round(M / (time.perf_counter() - t0), 2)
    dc.close()
    return out


def measure_extra(name, steps, warmup, dev):
    """Secondary workload on this GPU (N = 1 runs only): the same timing as the
    main line (inputs resident, K steps bracketed by synchronize), reported
    under "extra" -- e.g. c4, BASELINE configs[3] (bf16 compute)."""
    from polars_matmul import _native
    from polars_matmul.sharded import ShardedTopK

    M, N, D, k, metric, cdt = CONFIGS[name]
    mid = _native.metric_from_str(metric)
    bf16 = cdt == "bf16"
    g = torch.Generator(device=dev)
    g.manual_seed(42)
    q = torch.randn((M, D), generator=g, device=dev, dtype=torch.float32)
    g.manual_seed(1_000_003)
    c = torch.randn((N, D), generator=g, device=dev, dtype=torch.float32)
    if bf16:
        q, c = q.to(torch.bfloat16), c.to(torch.bfloat16)
    compute = _native.COMPUTE_BF16 if bf16 else _native.COMPUTE_F32
    ws = torch.empty(_native.workspace_bytes(M, N, D, k, mid, compute), dtype=torch.uint8, device=dev)
    runner = ShardedTopK(q, c, 0, k, mid, workspace=ws)
    for _ in range(warmup):
        runner.run()
    torch.cuda.synchronize()
    _native.timing_reset()
    _native.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        runner.run()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    _native.timing_enable(False)
    kms, kn = _native.timing_read("gemm_bf16_topk" if bf16 else "gemm_f32_topk")
    sms, sn = _native.timing_read("gemm_f32_seed")
    ach =2.0 * M * N * D / (kms / kn / 1000.0) / 1e12 if kn else None
    out = {
        "config": {"workload": f"{M}x{N}x{D} {cdt} {metric} k={k} ({name})"},
        "dtype": cdt, "value": round(M * steps / el, 2), "unit": "queries/s",
        "ms_per_step": round(el / steps * 1000.0, 3), "steps": steps, "warmup": warmup,
        "roofline": {"bound": "mfma", "achieved": round(ach, 2) if ach else None,
                     "peak": MFMA_PEAK_TFLOPS[cdt], "unit": "TFLOP/s",
                     "frac": round(ach / MFMA_PEAK_TFLOPS[cdt], 4) if ach else None,
                     "kernel_ms_avg": round(kms / kn, 3) if kn else None,
                     "seed_ms_avg": round(sms / sn, 3) if sn else None},
    }
    del runner, ws, q, c
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-sample", type=int, default=512,
                    help="queries timed on the CPU baseline vs the full corpus (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--boundary", type=int, default=1, help="also time the host-buffer C ABI (N=1)")
    ap.add_argument("--extra", default="c4,c1,c2",
                    help="comma-separated secondary configs measured after the main line (N=1; 'none' = none)")
    ap.add_argument("--check", type=int, default=8, help="query rows spot-checked against an f64 torch top-k")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from polars_matmul import _native

    _native.check(_native.lib().pmm_set_device(torch.cuda.current_device()))

    M, N, D, k, metric, cdt = CONFIGS[args.config]
    bf16 = cdt == "bf16"
    compute = _native.COMPUTE_BF16 if bf16 else _native.COMPUTE_F32
    mid = _native.metric_from_str(metric)
    lo = N * rank // world
    hi = N * (rank + 1) // world
    n_loc = hi - lo

    g = torch.Generator(device=dev)
    g.manual_seed(42)
    q = torch.randn((M, D), generator=g, device=dev, dtype=torch.float32)
    g.manual_seed(1_000_003 + rank)
    c = torch.randn((n_loc, D), generator=g, device=dev, dtype=torch.float32)
    if bf16:
        # BASELINE configs[3]: the same f32 embeddings rounded to bf16 (RNE) on
        # device, resident before the timed region
        q, c = q.to(torch.bfloat16), c.to(torch.bfloat16)
    ws_bytes = _native.workspace_bytes(M, n_loc, D, k, mid, compute)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    from polars_matmul.sharded import ShardedTopK

    runner = ShardedTopK(q, c, lo, k, mid, workspace=ws)
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        runner.run()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    _native.timing_reset()
    _native.timing_enable(True)
    t0 = time.perf_counter()
    for i in range(args.steps):
        out_i, out_s = runner.run()
        log(f"[rank {rank}] step {i + 1}/{args.steps} issued")
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    _native.timing_enable(False)
    kern_ms, kern_n = _native.timing_read("gemm_bf16_topk" if bf16 else "gemm_f32_topk")
    merge_ms, merge_n = _native.timing_read("merge_topk")
    seed_ms, seed_n = _native.timing_read("gemm_f32_seed")
    shard_ms, shard_n = _native.timing_read("merge_shards")
    # algorithmic bytes of this rank's last merge pass (the reduction's HBM
    # roofline), read from the workspace after the timed region
    merge_bytes = _native.merge_bytes(ws.data_ptr(), M, n_loc, D, k, mid, compute) if merge_n else None
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # correctness spot check on a few rows (f64 torch on device; untimed)
    check = None
    if args.check and world == 1:
        rows = torch.arange(0, M, max(1, M // args.check), device=dev)[: args.check]
        qd = q[rows].double()
        cd = c.double()
        s = qd @ cd.T
        if metric == "cosine":
            s = s / (qd.norm(dim=1, keepdim=True) * cd.norm(dim=1)[None, :])
        ref_s, ref_i = torch.topk(s, k, dim=1)
        got_i = out_i[rows].long()
        got_s = out_s[rows].double()
        kth = ref_s[:, -1:]
        band = 1e-5 * kth.abs() + 1e-5
        in_set = torch.gather(s, 1, got_i) >= (kth - band)
        check = {
            "rows": int(rows.numel()),
            "valid_topk_frac": float(in_set.float().mean().item()),
            "exact_index_match_frac": float((got_i == ref_i).float().mean().item()),
            "max_abs_score_err": float((got_s - torch.gather(s, 1, got_i)).abs().max().item()),
        }
        log(f"spot check: {check}")

    boundary = None
    if args.boundary and world == 1:
        boundary = boundary_rates(q.float(), c.float(), k, mid, compute)
        log(f"boundary: {boundary}")

    extra = None
    if args.extra and world == 1:
        del runner, ws
        torch.cuda.empty_cache()
        extra = {}
        for name in [x for x in args.extra.split(",") if x and x not in (args.config, "none")]:
            M_, N_, D_ = CONFIGS[name][:3]
            small = M_ * N_ * D_ < 10**11  # sub-millisecond steps: time more of them
            extra[name] = measure_extra(name, max(args.steps, 50) if small else args.steps,
                                        max(args.warmup, 3) if small else args.warmup, dev)
            log(f"extra {name}: {extra[name]}")

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    ms_per_step = elapsed / args.steps * 1000.0
    qps = M * args.steps / elapsed
    flops_launch = 2.0 * M * n_loc * D
    avg_kern_s = (kern_ms / kern_n / 1000.0) if kern_n else None
    achieved = flops_launch / avg_kern_s / 1e12 if avg_kern_s else None
    peak = MFMA_PEAK_TFLOPS[cdt]
    roofline = {
        "bound": "mfma",
        "kernel": f"gemm_{cdt}_kernel (fused GEMM + metric + top-k)",
        "achieved": round(achieved, 2) if achieved else None,
        "peak": peak,
        "unit": "TFLOP/s",
        "frac": round(achieved / peak, 4) if achieved else None,
        "traffic": load_traffic(args.config),
        "kernel_ms_avg": round(kern_ms / kern_n, 3) if kern_n else None,
        "flops_per_launch": flops_launch,
        "merge_ms_avg": round(merge_ms / merge_n, 3) if merge_n else None,
        "shard_merge_ms_avg": round(shard_ms / shard_n, 3) if shard_n else None,
        # threshold-seeding pass (small problems only): its own
        # gemm_f32_kernel launch, not in kernel_ms_avg, counted in ms_per_step
        "seed_ms_avg": round(seed_ms / seed_n, 3) if seed_n else None,
    }
    reduction = None
    if merge_n and merge_bytes:
        mavg = merge_ms / merge_n / 1000.0
        gbs = merge_bytes / mavg / 1e9
        reduction = {
            "kernel": "merge_kernel (per-row merge of the split candidate buffers)",
            "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_launch": merge_bytes,
            "kernel_ms_avg": round(mavg * 1000.0, 3),
        }
        if shard_n:
            # rank 0's k-way merge of the world x M x k (index, score) lists
            sbytes = (world + 1) * M * k * 8
            savg = shard_ms / shard_n / 1000.0
            reduction["shard_merge"] = {"bytes_per_launch": sbytes, "kernel_ms_avg": round(savg * 1000.0, 3),
                                        "achieved": round(sbytes / savg / 1e9, 1), "unit": "GB/s"}
    cpu = None
    if args.cpu_sample and world == 1:
        n_s = min(args.cpu_sample, M)
        # bf16: the oracle on the bf16-rounded rows (widened to f32, exact)
        cpu_qps, cpu_dt = cpu_baseline(q, c, k, metric, n_s, args.cpu_threads)
        cpu = {
            "value": round(cpu_qps, 2),
            "unit": "queries/s",
            "cores": args.cpu_threads,
            "kind": "port",
            "sample": f"first {n_s} queries x full {N}-row corpus, {D}d {cdt} {metric} k={k}; "
                      f"oracle/pmm_oracle.c (threaded GEMM, 1-thread epilogue+select), {cpu_dt:.1f}s",
        }
    cpu_np = None
    if args.cpu_sample and world == 1 and metric == "cosine":
        n_s = min(args.cpu_sample, M)
        np_qps, np_dt = numpy_comparator_qps(q, c, k, n_s)
        cpu_np = {
            "value": round(np_qps, 2), "unit": "queries/s",
            "cores": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)),
            "kind": "port",
            "sample": f"first {n_s} queries x full {N}-row corpus; the reference README's NumPy "
                      f"comparator (normalise, BLAS GEMM, argpartition, argsort), {np_dt:.1f}s",
        }
    line = {
        "metric": "cosine top-k queries/sec",
        "value": round(qps, 2),
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": cdt,
        "data": "synthetic N(0,1) f32 embeddings generated on device (torch.randn, seeded)"
                + (", rounded to bf16 on device" if bf16 else ""),
        "config": {"workload": f"{M}x{N}x{D} {cdt} {metric} k={k} ({args.config})", "queries": M,
                   "corpus": N, "dim": D, "k": k, "metric": metric,
                   "parallelism": f"corpus-row-shard x{world}" if world > 1 else "single GPU"},
        "roofline": roofline,
        "reduction_roofline": reduction,
        "cpu_baseline": cpu,
        "cpu_baseline_numpy": cpu_np,
        "boundary": boundary,
        "extra": extra,
        "check": check,
    }
    print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
