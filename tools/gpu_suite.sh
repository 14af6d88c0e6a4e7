#!/bin/bash
# One GPU session on the box, steps chosen by name (run in this order):
#   tools/gpu_suite.sh <tag> [tests] [smoke] [bench] [prof:<cfg>[:<pmc 0|1>]]...
#   tests        the whole GPU suite (pytest -m gpu), as the driver runs it
#   smoke        __graft_entry__.smoke()
#   bench        the default bench line (python bench.py)
#   prof:c3:1    tools/profile.sh on one config (kernel trace + stats; with
#                :1 the PMC passes too) and the PMC digest of its kernels
# Output under gpurun_out/<tag>/ (and gpurun_out/prof_<tag>_<cfg>/).  Each
# step runs under its own time limit; the first failing step ends the session.
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
          > "$out/gpu.log" 2>&1
      rc=$?; echo "gpu tests rc=$rc: $(tail -1 "$out/gpu.log")"; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit 4
      tail -1 "$out/smoke.log" ;;
    bench)
      timeout -k 10 900 python -u bench.py > "$out/bench.json" 2> "$out/bench.log" || { tail -20 "$out/bench.log"; exit 5; }
      python3 -c "import json,sys; d=json.load(open('$out/bench.json')); print(json.dumps(d['summary']))" ;;
    prof:*)
      IFS=: read -r _ cfg pmc <<< "$step"
      case $cfg in
        c1|c2) args="--steps 200 --warmup 10" ;;
        c5_rank) args="--steps 1 --warmup 1" ;;
        *) args="--steps 2 --warmup 1" ;;
      esac
      PMC=${pmc:-0} bash tools/profile.sh "${tag}_$cfg" --config "$cfg" $args --extra none --cpu-sample 0 \
          --boundary 0 --check 0 || exit 6
      if [ "${pmc:-0}" = "1" ]; then
        for k in gemm_ prologue_kernel merge_kernel; do
          python3 tools/pmc_summary.py "gpurun_out/prof_${tag}_$cfg" "$k" \
              > "gpurun_out/prof_${tag}_$cfg/summary_$k.json" 2>/dev/null || true
        done
      fi ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
