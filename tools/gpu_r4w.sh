#!/bin/bash
# round 4: the f32 seed rule (split-unit majority) -- seeding tests, c1/c2
# (still seeded), the per-rank shapes again
mkdir -p gpurun_out/r4w
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "seed or kat or fixture or ref_ or small or bench_verify" --timeout 300 --timeout-method thread > gpurun_out/r4w/gpu.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r4w/gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c1 --steps 1000 --warmup 50 --extra c2 --cpu-sample 0 --boundary 0 --check 8 > gpurun_out/r4w/c1.json 2> gpurun_out/r4w/c1.log || exit 5
python3 -c "import json;d=json.load(open('gpurun_out/r4w/c1.json'));r=d['roofline'];print('c1', d['ms_per_step'], r['seed_ms_avg'], 'c2', d['extra']['c2']['ms_per_step'])"
export SHAPE_VARIANTS='[["f32", 8, {}], ["f32", 2, {}], ["f32", 1, {}]]'
timeout -k 10 600 python -u tools/experiments/shard_shapes.py > gpurun_out/r4w/shapes.jsonl 2> gpurun_out/r4w/shapes.log || exit 6
cat gpurun_out/r4w/shapes.jsonl
echo done
