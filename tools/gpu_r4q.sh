#!/bin/bash
# round 4: fire-and-forget mode of the ws kernel with per-register ballots
# (no LDS re-read of survivor values): bit-equality tests, c4 A/B
mkdir -p gpurun_out/r4q
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "wsff" --timeout 300 --timeout-method thread > gpurun_out/r4q/gpu_wsff.log 2>&1
rc=$?; echo "wsff tests rc=$rc"; tail -3 gpurun_out/r4q/gpu_wsff.log; [ $rc -eq 0 ] || exit $rc
B="--config c4 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 8"
run() {  # run <name> <env...>
  local name=$1; shift
  env "$@" PMM_FF_DEBUG=1 timeout -k 10 300 python -u bench.py $B > gpurun_out/r4q/$name.json 2> gpurun_out/r4q/$name.log || { echo "$name failed"; exit 5; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4q/$name.json'));r=d['roofline'];print('$name', d['ms_per_step'], r['kernel_ms_avg'], r['seed_ms_avg'], r['merge_ms_avg'], r.get('ff_bucket_ms_avg'), r.get('ff_rerun_ms_total'), r['frac'], d['check']['exact_index_match_frac'])"
  grep "re-run rows" gpurun_out/r4q/$name.log | tail -1
}
for i in 1 2; do
  run def_$i PMM_BF16_WSFF=0
  run wsff3_$i PMM_BF16_WSFF=1
  run wsff2_$i PMM_BF16_WSFF=1 PMM_WSFF_J=2
done
echo done
