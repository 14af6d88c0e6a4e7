#!/bin/bash
# c1/c2 threshold-seed sample size A/B (PMM_SEED_NS), alternated twice.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/seedns_ab.txt
: > $out
for rep in 1 2; do
  for ns in 256 128 192 512; do
    for cfg in c1 c2; do
      PMM_SEED_NS=$ns timeout -k 10 120 python -u bench.py --config $cfg --steps 400 --warmup 20 --extra none \
        --cpu-sample 0 --boundary 0 --check 8 > gpurun_out/seedns.json 2> /dev/null || exit 1
      python -c "import json; d=json.loads(open('gpurun_out/seedns.json').read().strip().splitlines()[-1]); r=d['roofline']; print('ns', $ns, '$cfg', 'step', d['ms_per_step'], 'gemm', r['kernel_ms_avg'], 'seed', r['seed_ms_avg'], 'merge', r['merge_ms_avg'], 'exact', d['check']['exact_index_match_frac'])" >> $out
    done
  done
done
cat $out
