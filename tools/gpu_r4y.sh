#!/bin/bash
# round 4: f32 small variants with the LDS survivor queue + staged column
# norms, resident query rows (AK) on / off: f32 parity subset both ways, then
# c1 / c2 alternated twice
mkdir -p gpurun_out/r4y
for ak in 1 0; do
PMM_F32_AK=$ak timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "f32 or fixture or kat or ref_ or small or matmul or seed" --timeout 300 --timeout-method thread > gpurun_out/r4y/gpu_ak$ak.log 2>&1
rc=$?; echo "tests ak=$ak rc=$rc"; tail -1 gpurun_out/r4y/gpu_ak$ak.log; [ $rc -eq 0 ] || exit $rc
done
run() {  # tag, AK
PMM_F32_AK=$2 timeout -k 10 300 python -u bench.py --config c1 --steps 1000 --warmup 50 --extra c2 --cpu-sample 0 --boundary 0 --check 8 > gpurun_out/r4y/c1_$1.json 2> gpurun_out/r4y/c1_$1.log || exit 5
python3 -c "import json;d=json.load(open('gpurun_out/r4y/c1_$1.json'));r=d['roofline'];print('$1 c1', d['ms_per_step'], r.get('kernel_ms_avg'), 'c2', d['extra']['c2']['ms_per_step'], d['extra']['c2']['roofline'].get('kernel_ms_avg'), 'check', d.get('check'))"
}
for rep in 1 2; do run ak1 1; run ak0 0; done
echo done
