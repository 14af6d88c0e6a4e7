# candidate-buffer capacity (PMM_CAPG) at c1 / c2 with threshold seeding
set -o pipefail
mkdir -p gpurun_out
for cfg in c1 c2; do
for rep in 1 2; do
for v in 0 96 128 256 384 512; do
  PMM_CAPG=$v timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 5 --boundary 0 --extra none --cpu-sample 0 --check 64 > gpurun_out/cab.json 2> gpurun_out/cab.err || exit 1
  echo "[$cfg CAPG=$v] $(python -c "import json;d=json.load(open('gpurun_out/cab.json'));c=d['check'];r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms_avg'],r['seed_ms_avg'],r['merge_ms_avg'],c['exact_index_match_frac'])")"
done; done; done
