#!/bin/bash
# round 4: the f32 kernel's small variants at c1 / c2: resident query rows
# (AK), the deep LDS-DMA ring, and the query-row re-stream ablation: f32 parity subset on the product
# build, then c1 / c2 per stage count (lab builds libpmm_s{2,3,4}.so,
# alternated twice), then the 2-stage lab build with PMM_ABLATE 1 / 3 / 4
mkdir -p gpurun_out/r4x
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "f32 or fixture or kat or ref_ or small or matmul or seed" --timeout 300 --timeout-method thread > gpurun_out/r4x/gpu.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4x/gpu.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, lib, ablate, resident query rows
PMM_LIB=$2 PMM_ABLATE=$3 PMM_F32_AK=$4 timeout -k 10 300 python -u bench.py --config c1 --steps 1000 --warmup 50 --extra c2 --cpu-sample 0 --boundary 0 --check 0 > gpurun_out/r4x/c1_$1.json 2> gpurun_out/r4x/c1_$1.log || exit 5
python3 -c "import json;d=json.load(open('gpurun_out/r4x/c1_$1.json'));r=d['roofline'];print('$1 c1', d['ms_per_step'], r.get('kernel_ms_avg'), 'c2', d['extra']['c2']['ms_per_step'], d['extra']['c2']['roofline'].get('kernel_ms_avg'))"
}
for rep in 1 2; do
run s2 libpmm_s2.so 0 0; run s2ak libpmm_s2.so 0 1; run s4 libpmm_s4.so 0 0
done
for ab in 1 3 4; do run ab$ab libpmm_s2.so $ab 0; done
run ab1ak libpmm_s2.so 1 1
echo done
