#!/bin/bash
# A/B of library builds or runtime knobs on one GPU box, alternated.
#   tools/gpu_ab.sh <tag> <reps> "<bench.py args>" <variant>...
# A variant is <lib>[:VAR=val[,VAR=val...]] -- a library under
# polars-matmul_amd/polars_matmul/ (PMM_LIB) plus environment settings, e.g.
#   libpmm.so  libpmm_ab_old.so  libpmm_lab.so:PMM_ABLATE=8
# Each run is its own time-limited step; the script stops at the first failure.
# Output: gpurun_out/ab_<tag>/<i>_<variant>.{json,log}; one summary line per
# run on stdout (ms per step, dominant kernel ms, roofline fraction).
set -u
tag=$1; reps=$2; args=$3; shift 3
out=gpurun_out/ab_$tag
mkdir -p "$out"
for i in $(seq 1 "$reps"); do
  for v in "$@"; do
    lib=${v%%:*}
    envs=""
    [ "$lib" != "$v" ] && envs=${v#*:}
    name=$(echo "$v" | tr ':,=/' '____')
    ( export PMM_LIB=$lib
      IFS=',' read -ra kv <<< "$envs"
      for x in "${kv[@]}"; do [ -n "$x" ] && export "$x"; done
      timeout -k 10 ${AB_TIMEOUT:-300} python3 -u bench.py $args ) \
        > "$out/${i}_$name.json" 2> "$out/${i}_$name.log" || { echo "$v run $i failed"; tail -5 "$out/${i}_$name.log"; exit 5; }
    python3 - "$out/${i}_$name.json" "$v" "$i" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[2]:40s} run {sys.argv[3]}: step {d['ms_per_step']} ms, kernel {r['kernel_ms_avg']} ms, "
      f"frac {r['frac']}, seed/prologue {r.get('seed_ms_avg')} ms, merge {r.get('merge_ms_avg')} ms")
EOF
  done
done
echo done
