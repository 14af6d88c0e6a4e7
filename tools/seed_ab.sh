# GPU tests, then A/B of the threshold seeding (PMM_SEED) at c1 / c2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for cfg in c1 c2; do
for rep in 1 2; do
for v in 0 1; do
  PMM_SEED=$v timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 5 --boundary 0 --extra none --cpu-sample 0 --check 64 > gpurun_out/sab.json 2> gpurun_out/sab.err || exit 1
  echo "[$cfg SEED=$v] $(python -c "import json;d=json.load(open('gpurun_out/sab.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms_avg'],d['roofline']['merge_ms_avg'],d['check'])")"
done; done; done
