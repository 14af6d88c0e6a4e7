"""Summarise tools/experiments/ws_clock.sh: per run, the ws kernel's duration,
GRBM_GUI_ACTIVE cycles per XCD and the effective clock."""
import collections
import csv
import glob
import os

for d in sorted(glob.glob("gpurun_out/clk/*/")):
    kt = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    cc = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    ws = [r for r in kt if "ws_kernel" in r["Kernel_Name"]]
    dur = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ws) / 1e9
    agg = collections.defaultdict(float)
    for r in cc:
        if "ws_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    gui = agg["GRBM_GUI_ACTIVE"] / 8
    print(f"{os.path.basename(d.rstrip('/')):24s} {dur * 1e3:8.2f} ms  {gui / 1e6:8.1f} Mcyc/XCD  "
          f"{gui / dur / 1e9:5.3f} GHz  LDS insts {agg['SQ_INSTS_LDS'] / 1e6:8.1f} M")
