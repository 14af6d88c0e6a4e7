#!/bin/bash
# round 4: c1 / c2 seed sample size on the final tree (PMM_SEED_NS), alternated twice
mkdir -p gpurun_out/r4ns
for rep in 1 2; do for ns in 256 384 512; do
PMM_SEED_NS=$ns timeout -k 10 300 python -u bench.py --config c1 --steps 1000 --warmup 50 --extra c2 --cpu-sample 0 --boundary 0 --check 8 > gpurun_out/r4ns/c1_$ns.json 2> gpurun_out/r4ns/c1_$ns.log || exit 5
python3 -c "import json;d=json.load(open('gpurun_out/r4ns/c1_$ns.json'));r=d['roofline'];c=d['extra']['c2'];print('ns $ns c1', d['ms_per_step'], r.get('kernel_ms_avg'), r.get('seed_ms_avg'), 'c2', c['ms_per_step'], c['roofline'].get('kernel_ms_avg'), 'exact', d['check']['exact_index_match_frac'])"
done; done
echo done
