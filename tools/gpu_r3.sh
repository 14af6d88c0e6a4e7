#!/bin/bash
# Round-3 GPU check: the -m gpu suite (verbose, per-test timeout), smoke(),
# then the default bench line.  Each GPU step has its own time limit; the
# first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 780 python -u -m pytest tests -m gpu -x -v --durations=15 --timeout 600 --timeout-method thread \
  > gpurun_out/r3_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r3_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r3_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r3_bench.json

[ $rc -eq 0 ] || exit $rc
# rocprofv3 summaries of the shipped kernels at c3 and c4 (tools/profile.sh:
# a kernel-trace pass, then one PMC group per pass)
P="--steps 2 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0"
bash tools/profile.sh r3c3 --config c3 $P || exit 11
python tools/pmc_summary.py gpurun_out/prof_r3c3 gemm_f32_kernel > gpurun_out/prof_r3c3/summary.json || exit 12
python tools/pmc_summary.py gpurun_out/prof_r3c3 merge_kernel > gpurun_out/prof_r3c3/summary_merge.json || exit 12
bash tools/profile.sh r3c4 --config c4 $P || exit 13
python tools/pmc_summary.py gpurun_out/prof_r3c4 gemm_bf16_ws > gpurun_out/prof_r3c4/summary.json || exit 14
echo profiles ok
