#!/usr/bin/env python3
"""Regenerate profiles/pmc_traffic_<config>.json (the bench line's
roofline.traffic) from a tools/profile.sh output directory of the CURRENT
build.

    python tools/traffic_json.py <prof_dir> <config> <kernel_substring> <summary_out>

Runs tools/pmc_summary.py on the directory, writes its JSON to <summary_out>
(a committed copy under profiles/), and writes profiles/pmc_traffic_<config>.json
with the HBM bytes per launch (FETCH_SIZE x1024 x2 + WRITE_SIZE x1024, the
gfx950 corrections of MI355X_MICROARCH.md "HBM") next to the ALGORITHMIC bytes
of one launch (Q and C read once: (M + N) * D * elem, plus the M x k lists)
and their ratio -- the re-read factor the tiling costs."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = {  # M, N, D, k, element bytes
    "c3": (100_000, 1_000_000, 768, 100, 4),
    "c4": (100_000, 1_000_000, 768, 100, 2),
    "c1": (1_000, 10_000, 256, 10, 4),
    "c2": (1_000, 10_000, 256, 10, 4),
}

prof, cfg, kern, summary_out = sys.argv[1:5]
res = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), prof, kern],
                     check=True, capture_output=True, text=True)
summ = json.loads(res.stdout)
os.makedirs(os.path.dirname(os.path.abspath(summary_out)), exist_ok=True)
with open(summary_out, "w") as f:
    json.dump(summ, f, indent=1)
M, N, D, k, eb = CONFIGS[cfg]
alg = (M + N) * D * eb + M * k * 8
hbm = summ.get("hbm_bytes_per_launch")
out = {
    "config": cfg,
    "kernel": kern,
    "hbm_bytes_per_launch": hbm,
    "hbm_read_bytes_per_launch": summ.get("hbm_read_bytes_per_launch"),
    "hbm_write_bytes_per_launch": summ.get("hbm_write_bytes_per_launch"),
    "algorithmic_bytes_per_launch": alg,
    "traffic_over_algorithmic": round(hbm / alg, 1) if hbm else None,
    "source": f"{os.path.relpath(summary_out, ROOT)} (tools/profile.sh passes of this build: rocprofv3 "
              "--pmc FETCH_SIZE / WRITE_SIZE in separate passes; FETCH_SIZE x1024 x2, WRITE_SIZE x1024 per "
              "MI355X_MICROARCH.md)",
    "l2_hit_rate": summ.get("l2_hit_rate"),
    "trace_avg_ms": summ.get("avg_ms"),
    "effective_clock_ghz": summ.get("effective_clock_ghz"),
    "mfma_busy_frac": summ.get("mfma_busy_frac"),
}
with open(os.path.join(ROOT, "profiles", f"pmc_traffic_{cfg}.json"), "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out, indent=1))
