# Threshold seeding at c3 (f32 100k x 1M x 768 cosine k=100): off vs sample sizes
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for v in 0 1024 4096 16384; do
  if [ $v = 0 ]; then E="PMM_SEED=0"; else E="PMM_SEED=1 PMM_SEED_NS=$v"; fi
  env $E timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 8 > gpurun_out/s3.json 2> gpurun_out/s3.err || exit 1
  echo "[c3 $E] $(python -c "import json;d=json.load(open('gpurun_out/s3.json'));c=d['check'];print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms_avg'],d['roofline']['merge_ms_avg'],c['exact_index_match_frac'])")"
done; done
