#!/bin/bash
# round 4: c4 re-check on the final tree (the final bench line read 140.8 ms)
mkdir -p gpurun_out/r4c4
for i in 1 2; do
timeout -k 10 400 python -u bench.py --config c4 --steps 10 --warmup 3 --extra none --cpu-sample 0 --boundary 0 --check 0 > gpurun_out/r4c4/c4_$i.json 2> gpurun_out/r4c4/c4_$i.log || exit 5
python3 -c "import json;d=json.load(open('gpurun_out/r4c4/c4_$i.json'));r=d['roofline'];print('c4', d['ms_per_step'], r['frac'], r.get('kernel_ms_avg'), r.get('seed_ms_avg'))"
done
timeout -k 10 300 python -u bench.py --config c3 --steps 5 --warmup 2 --extra none --cpu-sample 0 --boundary 0 --check 0 > gpurun_out/r4c4/c3.json 2> gpurun_out/r4c4/c3.log || exit 6
python3 -c "import json;d=json.load(open('gpurun_out/r4c4/c3.json'));r=d['roofline'];print('c3', d['ms_per_step'], r['frac'])"
