# A/B of the seed sample size (PMM_SEED_NS) at c1 / c2
set -o pipefail
mkdir -p gpurun_out
for cfg in c1 c2; do
for rep in 1 2; do
for v in ${NS_LIST:-256 512 1024}; do
  PMM_SEED=1 PMM_SEED_NS=$v timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 5 --boundary 0 --extra none --cpu-sample 0 --check 64 > gpurun_out/sab.json 2> gpurun_out/sab.err || exit 1
  echo "[$cfg NS=$v] $(python -c "import json;d=json.load(open('gpurun_out/sab.json'));c=d['check'];print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms_avg'],c['exact_index_match_frac'],c['max_abs_score_err'])")"
done; done; done
