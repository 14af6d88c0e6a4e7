"""bench.py's N-rank launcher on CPU (gloo): `python bench.py --gpus 2`
without a torch.distributed launcher starts 2 rank processes itself, they
rendezvous on 127.0.0.1, run the sharded orchestration (one packed gather of
the per-rank [2][M][k] lists, merge of the [world][2][M][k] buffer) and rank 0
prints one JSON line with n_gpus = 2.  The per-shard top-k and merge are plain
torch on the host here (--cpu-selftest); on MI355X they are libpmm's kernels."""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=300)


def test_launcher_spawns_two_ranks():
    r = _run(["--gpus", "2", "--cpu-selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["ranks_ok"] is True


def test_launcher_three_ranks():
    r = _run(["--gpus", "3", "--cpu-selftest"])
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["n_gpus"] == 3 and out["ranks_ok"] is True


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--cpu-selftest"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE" in r.stderr


def test_early_spawner_runs_a_program_and_returns_its_output():
    # bench.py forks this helper before the GPU is touched; later the helper
    # starts the in-process transport's child (a clean process) and hands back
    # its status and output
    import bench

    sp = bench.EarlySpawner()
    r = sp.run([sys.executable, "-c", "import sys; print('{\"ok\": 1}'); sys.exit(3)"], dict(os.environ), 60)
    assert r["rc"] == 3 and r["stdout"].strip() == '{"ok": 1}'
    sp.close()  # already used: no-op
    unused = bench.EarlySpawner()
    unused.close()  # the helper exits without running anything


def _bench_module():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_summary_is_the_last_key_and_carries_every_extra():
    # the driver keeps only the tail of stdout; the line's
    # last key digests the headline and every extra
    b = _bench_module()
    line = {
        "value": 93000.0, "ms_per_step": 1070.0, "config": {"workload": "c3"},
        "roofline": {"frac": 0.91, "kernel_ms_avg": 1068.0},
        "cpu_baseline": {"value": 176.0, "unit": "queries/s", "cores": 16},
        "extra": {
            "c4": {"value": 700000.0, "ms_per_step": 140.0, "roofline": {"frac": 0.45, "kernel_ms_avg": 134.0}},
            "c1": {"value": 1e7, "ms_per_step": 0.1, "roofline": {"frac": 0.31},
                   "boundary": {"f32_list_cached": {"ms_per_call": 0.5, "split_ms": {"h2d": 0.04}},
                                "reps": 5},
                   "small_kernels": {"prologue": {"us_avg": 17.0}, "fused_us_avg": 72.0}},
            "c1_f64": {"default": {"value": 3e6, "ms_per_step": 0.3, "roofline": {"frac": 0.1}},
                       "fused": {"ms_per_step": 0.35}, "materialised": {"ms_per_step": 0.3}},
            "matmul": {"value": 900.0, "ms_per_call": 1.1},
            "c5_rank": {"value": 55000.0, "ms_per_step": 18000.0, "roofline": {"frac": 0.9}},
        },
    }
    line["summary"] = b.summary_of(line)
    text = json.dumps(line)
    assert list(json.loads(text))[-1] == "summary"
    sm = line["summary"]
    assert set(sm) >= {"headline", "c4", "c1", "c1_f64", "matmul", "c5_rank", "cpu_baseline"}
    assert sm["c4"]["frac"] == 0.45 and sm["c5_rank"]["ms_per_step"] == 18000.0
    assert sm["c1"]["e2e_ms"] == {"f32_list_cached": 0.5} and sm["c1"]["small_kernels_us"]["prologue"] == 17.0
    assert sm["c1_f64"]["fused_ms"] == 0.35 and sm["matmul"]["ms_per_call"] == 1.1
    assert len(json.dumps(sm)) < 4000


def test_descendants_names_a_live_child():
    b = _bench_module()
    p = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(30)"])
    try:
        kids = b.descendants(os.getpid())
        assert any(k == p.pid and "sleep" in c for k, _, c in kids), kids
    finally:
        p.kill()
        p.wait()
