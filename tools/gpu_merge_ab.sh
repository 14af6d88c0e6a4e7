#!/bin/bash
# c3 merge A/B (PMM_MERGE_FLAGS: 1 reverse row order, 2 pipelined candidate
# loads), alternated twice; records merge_ms_avg and reduction frac.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/merge_ab.txt
: > $out
for rep in 1 2; do
  for f in 0 1 2 3; do
    PMM_MERGE_FLAGS=$f timeout -k 10 180 python -u bench.py --config c3 --steps 3 --warmup 1 --extra none \
      --cpu-sample 0 --boundary 0 --check 8 > gpurun_out/mab_$f.json 2> gpurun_out/mab_err.log || exit 1
    python - $f gpurun_out/mab_$f.json >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["reduction_roofline"]
print("flags", sys.argv[1], "merge_ms", r["kernel_ms_avg"], "frac", r["frac"], "step_ms", d["ms_per_step"],
      "exact", d["check"]["exact_index_match_frac"])
PY
  done
done
cat $out
