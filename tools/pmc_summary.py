#!/usr/bin/env python3
"""Summarise a tools/profile.sh output directory for one kernel.

    python tools/pmc_summary.py gpurun_out/prof_<tag> [kernel_substring]

Prints per-launch kernel time (trace pass), PMC counters per launch, and the
derived quantities the bench reports: effective clock (GRBM_GUI_ACTIVE / 8 /
wall), MFMA busy fraction, HBM bytes per launch with the gfx950 correction
(FETCH_SIZE is in KiB and reads 1/2 of a wide coalesced stream's bytes:
MI355X_MICROARCH.md "HBM"), and the L2 hit rate.
"""
import collections
import csv
import json
import os
import sys

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "gemm_f32_kernel"


def launches(path):
    rows = list(csv.DictReader(open(path)))
    return [r for r in rows if kern in r["Kernel_Name"]]


out = {"kernel": kern}
tr = os.path.join(d, "trace", "run_kernel_trace.csv")
if os.path.exists(tr):
    ls = launches(tr)
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in ls]
    out["launches"] = len(durs)
    out["avg_ms"] = sum(durs) / max(1, len(durs))
    out["vgpr"] = ls[0].get("VGPR_Count") if ls else None
    out["agpr"] = ls[0].get("Accum_VGPR_Count") if ls else None
    out["lds"] = ls[0].get("LDS_Block_Size") if ls else None
agg = collections.defaultdict(float)
n_dispatch = collections.defaultdict(set)
dur = {}
for p in ("fetch", "write", "sq", "cache"):
    f = os.path.join(d, p, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in launches(f):
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        n_dispatch[r["Counter_Name"]].add(r["Dispatch_Id"])
        dur[(p, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9
per = {k: v / max(1, len(n_dispatch[k])) for k, v in agg.items()}
out["counters_per_launch"] = per
sq_durs = [v for (p, _), v in dur.items() if p == "sq"]
if "GRBM_GUI_ACTIVE" in per and sq_durs:
    wall = sum(sq_durs) / len(sq_durs)
    clk = per["GRBM_GUI_ACTIVE"] / 8 / wall
    out["effective_clock_ghz"] = clk / 1e9
    if "SQ_VALU_MFMA_BUSY_CYCLES" in per:
        out["mfma_busy_frac"] = per["SQ_VALU_MFMA_BUSY_CYCLES"] / (wall * clk * 1024)
if "FETCH_SIZE" in per:
    out["hbm_read_bytes_per_launch"] = per["FETCH_SIZE"] * 1024 * 2
if "WRITE_SIZE" in per:
    out["hbm_write_bytes_per_launch"] = per["WRITE_SIZE"] * 1024
if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
    out["hbm_bytes_per_launch"] = out["hbm_read_bytes_per_launch"] + out["hbm_write_bytes_per_launch"]
if "TCC_HIT_sum" in per:
    out["l2_hit_rate"] = per["TCC_HIT_sum"] / (per["TCC_HIT_sum"] + per["TCC_MISS_sum"])
if "SQ_INSTS_VALU" in per and per.get("SQ_INSTS_MFMA"):
    out["valu_per_mfma"] = (per["SQ_INSTS_VALU"] - per["SQ_INSTS_MFMA"]) / per["SQ_INSTS_MFMA"]
if "hbm_bytes_per_launch" in out and out.get("avg_ms"):
    out["hbm_gbs"] = out["hbm_bytes_per_launch"] / (out["avg_ms"] / 1000.0) / 1e9
print(json.dumps(out, indent=1))
