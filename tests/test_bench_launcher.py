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
