#!/bin/bash
# A/B of two builds of the library on one box (PMM_LIB), alternated twice:
# the c3 merge, c1 and c4 lines.  Usage: tools/gpu_lib_ab.sh libA.so libB.so
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/lib_ab.txt
: > $out
for rep in 1 2; do
  for lib in "$@"; do
    for cfg in ${CFGS:-c3 c1 c4}; do
      if [ $cfg = c1 ] || [ $cfg = c2 ]; then st="--steps 400 --warmup 20"; else st="--steps 3 --warmup 1"; fi
      PMM_LIB=$lib timeout -k 10 180 python -u bench.py --config $cfg $st --extra none --cpu-sample 0 \
        --boundary 0 --check 8 > gpurun_out/libab.json 2> gpurun_out/libab_err.log || exit 1
      python - $lib $cfg gpurun_out/libab.json >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
r, red = d["roofline"], d.get("reduction_roofline") or {}
print(sys.argv[1], sys.argv[2], "step", d["ms_per_step"], "kernel", r["kernel_ms_avg"], "merge", r.get("merge_ms_avg"),
      "red_frac", red.get("frac"), "exact", d["check"]["exact_index_match_frac"])
PY
    done
  done
done
cat $out
