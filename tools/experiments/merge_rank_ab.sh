#!/bin/bash
# merge_kernel final order by rank counting (default) vs bitonic sort (PMM_MERGE_RANK=0):
# the GPU suite, then c3 and c1 alternated.
set -o pipefail
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/mrank_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/mrank_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
for cfg in c3 c1; do
  if [ $cfg = c3 ]; then B="--config c3 --steps 2 --warmup 1"; else B="--config c1 --steps 200 --warmup 10"; fi
  B="$B --extra none --cpu-sample 0 --boundary 0"
  for i in 1 2; do
    for v in 1 0; do
      PMM_MERGE_RANK=$v timeout -k 10 200 python -u bench.py $B > gpurun_out/mrank_${cfg}_${v}_$i.json 2> gpurun_out/mrank_${cfg}_${v}_$i.err || exit 7
      python3 -c "import json;d=json.load(open('gpurun_out/mrank_${cfg}_${v}_$i.json'));r=d['roofline'];m=d['reduction_roofline'];print('$cfg RANK=$v', d['ms_per_step'], r['merge_ms_avg'], m['frac'], d['check'])"
    done
  done
done
