#!/bin/bash
# c1 GEMM time composition (lab build: PMM_ABLATE 1 = no epilogue, 2 =
# pre-filter only; results wrong, timing only), with and without the seed.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/c1_ablate.txt
: > $out
for rep in 1 2; do
  for v in "0 1" "1 1" "2 1" "0 0" "1 0"; do
    set -- $v
    PMM_LIB=libpmm_lab.so PMM_ABLATE=$1 PMM_SEED=$2 timeout -k 10 120 python -u bench.py --config c1 --steps 400 \
      --warmup 20 --extra none --cpu-sample 0 --boundary 0 --check 0 > gpurun_out/c1abl.json 2> gpurun_out/c1abl_err.log || exit 1
    python - "$1" "$2" gpurun_out/c1abl.json >> $out <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
r = d["roofline"]
print("ablate", sys.argv[1], "seed", sys.argv[2], "step", d["ms_per_step"], "gemm", r["kernel_ms_avg"],
      "seed_ms", r.get("seed_ms_avg"), "merge", r.get("merge_ms_avg"))
PY
  done
done
cat $out
