#!/bin/bash
# bf16 seed kernel change: every bf16 GPU test (incl. seeded == unseeded bit
# for bit), then c4 with the previous and the new library alternated.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -k "bf16 or c4" -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/bf16_seed_tests.log 2>&1
rc=$?; echo "bf16 tests rc=$rc"; tail -2 gpurun_out/bf16_seed_tests.log
[ $rc -eq 0 ] || exit $rc
CFGS="c4" bash tools/gpu_lib_ab.sh "$@"
