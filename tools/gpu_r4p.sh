#!/bin/bash
# round 4: the wave-specialised kernel's fire-and-forget mode (PMM_BF16_WSFF):
# its bit-equality tests, then c4 alternated with the default mode
mkdir -p gpurun_out/r4p
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "wsff" --timeout 300 --timeout-method thread > gpurun_out/r4p/gpu_wsff.log 2>&1
rc=$?; echo "wsff tests rc=$rc"; tail -3 gpurun_out/r4p/gpu_wsff.log; [ $rc -eq 0 ] || exit $rc
B="--config c4 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 8"
for i in 1 2; do
  for v in 0 1; do
    PMM_BF16_WSFF=$v PMM_FF_DEBUG=1 timeout -k 10 300 python -u bench.py $B > gpurun_out/r4p/wsff${v}_$i.json 2> gpurun_out/r4p/wsff${v}_$i.log || { echo "$v failed"; exit 5; }
    python3 -c "import json;d=json.load(open('gpurun_out/r4p/wsff${v}_$i.json'));r=d['roofline'];print('wsff $v $i', d['ms_per_step'], r['kernel_ms_avg'], r['seed_ms_avg'], r['merge_ms_avg'], r.get('ff_bucket_ms_avg'), r.get('ff_rerun_ms_total'), r['frac'], d['check']['exact_index_match_frac'])"
    grep "re-run rows" gpurun_out/r4p/wsff${v}_$i.log | tail -1
  done
done
for j in 2 5; do
  PMM_BF16_WSFF=1 PMM_WSFF_J=$j PMM_FF_DEBUG=1 timeout -k 10 300 python -u bench.py $B > gpurun_out/r4p/wsff_j$j.json 2> gpurun_out/r4p/wsff_j$j.log || { echo "j$j failed"; exit 6; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4p/wsff_j$j.json'));r=d['roofline'];print('wsff j=$j', d['ms_per_step'], r['kernel_ms_avg'], r['seed_ms_avg'], r.get('ff_bucket_ms_avg'), r.get('ff_rerun_ms_total'), r['frac'])"
  grep "re-run rows" gpurun_out/r4p/wsff_j$j.log | tail -1
done
echo done
