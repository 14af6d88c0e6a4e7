#!/bin/bash
# c1/c2 small-problem A/B: the bench's c1 line under several planner/tile
# settings, alternated twice (wall time of one GEMM launch varies box to box).
# (Round 3 also ran PMM_F32_WPC=2, a since-removed planner knob: two 128 x 128
# workgroups per CU, slower; profiles/r3_c1/wpc_variant_ab.txt.)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/c1_ab.txt
: > $out
run() {
  local tag=$1; shift
  for cfg in c1 c2; do
    env "$@" timeout -k 10 120 python -u bench.py --config $cfg --steps 400 --warmup 20 --extra none \
      --cpu-sample 0 --boundary 0 --check 8 > gpurun_out/c1ab_${tag}_${cfg}.json 2> gpurun_out/c1ab_err.log || return 1
    python - "$tag" "$cfg" gpurun_out/c1ab_${tag}_${cfg}.json >> $out <<'EOF'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1], sys.argv[2], d["ms_per_step"], r["kernel_ms_avg"], r.get("seed_ms_avg"), r.get("merge_ms_avg"),
      d["check"]["exact_index_match_frac"])
EOF
  done
}
for rep in 1 2; do
  run base PMM_NONE=1 || exit 1
  run v2 PMM_GEMM_VARIANT=2 || exit 3
done
cat $out
