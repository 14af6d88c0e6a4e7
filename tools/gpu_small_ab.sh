#!/bin/bash
# Small-problem A/Bs in one call: parity of the candidate library first
# (PMM_LIB=$1), then c1/c2 across the libraries given, then the seed sample
# size (shipped library).
set -o pipefail
mkdir -p gpurun_out
cand=$1
PMM_LIB=$cand timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/parity_cand.log 2>&1
rc=$?; echo "parity ($cand) rc=$rc"; tail -2 gpurun_out/parity_cand.log
[ $rc -eq 0 ] || exit $rc
shift
CFGS="c1 c2" bash tools/gpu_lib_ab.sh "$@" || exit 1
cp gpurun_out/lib_ab.txt gpurun_out/lib_ab_small.txt
bash tools/gpu_seedns_ab.sh
