#!/bin/bash
# FETCH_SIZE calibration for the corpus DMA patterns (dma_fetch_calib.hip).
# Two passes: kernel trace (durations) and FETCH_SIZE; each time-limited.
set -u
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/calib
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
bin=$root/tools/calib/dma_fetch_calib
timeout -k 10 120 "$bin" > "$out/plain.log" 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- "$bin" > "$out/trace.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- "$bin" > "$out/fetch.log" 2>&1 || exit 1
cat "$out/plain.log"
exit 0
