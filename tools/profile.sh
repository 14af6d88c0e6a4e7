#!/bin/bash
# Collect rocprofv3 summaries for one bench configuration on the GPU box.
#   tools/profile.sh <tag> [bench.py args...]
# Pass 1: kernel trace + stats (per-kernel durations).
# Passes 2..: PMC counters, one group per run (FETCH_SIZE and WRITE_SIZE cannot
# share a pass on gfx950; MI355X_MICROARCH.md "rocprofv3 PMC slots").
# Every pass is its own time-limited step; the script stops at the first failure.
set -u
root=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
out=$root/gpurun_out/prof_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
run() {  # run <name> <rocprofv3 options...>
  local name=$1; shift
  echo "[profile] pass $name" >&2
  timeout -k 10 900 rocprofv3 "$@" --output-format csv -d "$out/$name" -o run -- \
      python3 "$root/bench.py" ${BENCH_ARGS} > "$out/$name.log" 2>&1
  local rc=$?
  echo "[profile] pass $name rc=$rc" >&2
  return $rc
}
BENCH_ARGS="$*"
run trace --kernel-trace --stats || exit 1
[ "${PMC:-1}" = "1" ] || exit 0
run fetch --kernel-trace --pmc FETCH_SIZE || exit 1
run write --kernel-trace --pmc WRITE_SIZE || exit 1
run sq --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
run cache --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY || exit 1
exit 0
