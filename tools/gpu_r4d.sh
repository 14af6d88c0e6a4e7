#!/bin/bash
# round 4: LDS-staged f32 seed (parity + c1/c2 A/B against the row-streaming
# seed), then the fire-and-forget bf16 kernel's c4 step split (re-run rows,
# rocprofv3 kernel trace)
mkdir -p gpurun_out/r4d
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "seed or kat or fixture or ref_ or norms or small or edge" --timeout 300 --timeout-method thread > gpurun_out/r4d/gpu.log 2>&1
rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/r4d/gpu.log
[ $rc -eq 0 ] || exit $rc
A="--config c1 --steps 2000 --warmup 50 --extra c2 --cpu-sample 0 --boundary 0 --check 8"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $A > gpurun_out/r4d/c1_lds_$i.json 2> gpurun_out/r4d/c1_lds_$i.log || exit 5
  PMM_SEED_LDS=0 timeout -k 10 300 python -u bench.py $A > gpurun_out/r4d/c1_ring_$i.json 2> gpurun_out/r4d/c1_ring_$i.log || exit 6
done
PMM_BF16_FF=1 PMM_FF_DEBUG=1 timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --extra none --cpu-sample 0 --boundary 0 > gpurun_out/r4d/c4_ff.json 2> gpurun_out/r4d/c4_ff.log || exit 7
PMM_BF16_FF=1 PMC=0 bash tools/profile.sh r4ff --config c4 --steps 2 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0 || exit 8
echo done
