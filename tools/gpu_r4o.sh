#!/bin/bash
# round 4: bf16 seed sample size at c4 (PMM_SEED_NS 1024 = default, 2048,
# 4096), alternated twice; bf16 seeded-exactness tests at 4096 first
mkdir -p gpurun_out/r4o
PMM_SEED_NS=4096 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "bf16 and seed" --timeout 300 --timeout-method thread > gpurun_out/r4o/gpu_seed.log 2>&1
rc=$?; echo "seed tests rc=$rc"; tail -2 gpurun_out/r4o/gpu_seed.log; [ $rc -eq 0 ] || exit $rc
B="--config c4 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 8"
for i in 1 2; do
  for ns in 1024 2048 4096; do
    PMM_SEED_NS=$ns timeout -k 10 300 python -u bench.py $B > gpurun_out/r4o/ns${ns}_$i.json 2> gpurun_out/r4o/ns${ns}_$i.log || { echo "$ns failed"; exit 5; }
    python3 -c "import json;d=json.load(open('gpurun_out/r4o/ns${ns}_$i.json'));r=d['roofline'];print('ns $ns $i', d['ms_per_step'], r['kernel_ms_avg'], r['seed_ms_avg'], r['merge_ms_avg'], r['frac'], d['check']['exact_index_match_frac'])"
  done
done
echo done
