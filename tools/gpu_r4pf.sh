#!/bin/bash
# round 4: per-lane survivor flags + one prefix sum in the small f32
# variants' pre-filter: GPU suite, then c1 / c2 vs the previous build (the lab
# library, built before the change), alternated twice
mkdir -p gpurun_out/r4pf
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4pf/gpu.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r4pf/gpu.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, lib
PMM_LIB=$2 timeout -k 10 300 python -u bench.py --config c1 --steps 1000 --warmup 50 --extra c2 --cpu-sample 0 --boundary 0 --check 8 > gpurun_out/r4pf/c1_$1.json 2> gpurun_out/r4pf/c1_$1.log || exit 5
python3 -c "import json;d=json.load(open('gpurun_out/r4pf/c1_$1.json'));r=d['roofline'];c=d['extra']['c2'];print('$1 c1 step', d['ms_per_step'], 'fused', r.get('kernel_ms_avg'), '| c2 step', c['ms_per_step'], 'fused', c['roofline'].get('kernel_ms_avg'), '| exact', d['check']['exact_index_match_frac'])"
}
for rep in 1 2; do run new libpmm.so; run old libpmm_lab.so; done
echo done
