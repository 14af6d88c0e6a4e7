#!/bin/bash
# rocprofv3 summaries of the reference-benchmark-size configs (c1 cosine, c2
# dot): kernel trace + PMC passes (tools/profile.sh), then per-kernel summaries.
set -o pipefail
P="--steps 100 --warmup 10 --boundary 0 --extra none --cpu-sample 0 --check 0"
for cfg in c1 c2; do
  bash tools/profile.sh r3b$cfg --config $cfg $P || exit 11
  for k in gemm_f32_kernel merge_kernel prologue_kernel; do
    python tools/pmc_summary.py gpurun_out/prof_r3b$cfg $k > gpurun_out/prof_r3b$cfg/summary_$k.json || exit 12
  done
done
echo profiles ok
