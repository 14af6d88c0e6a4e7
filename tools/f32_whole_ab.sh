# f32 whole-block schedule: GPU tests with it on, then c3 A/B (bench only)
mkdir -p gpurun_out
timeout -k 10 300 env PMM_F32_WHOLE=1 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fw_pytest.log 2>&1; rc=$?
echo "pytest (whole) rc=$rc $(tail -1 gpurun_out/fw_pytest.log)"; [ $rc -eq 0 ] || exit $rc
for e in PMM_F32_WHOLE=0 PMM_F32_WHOLE=1 PMM_F32_WHOLE=0 PMM_F32_WHOLE=1; do
  timeout -k 10 300 env $e python bench.py --config c3 --steps 2 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 8 > gpurun_out/fw.json 2> gpurun_out/fw.err || exit 1
  echo "[$e] $(python -c "import json;d=json.load(open('gpurun_out/fw.json'));print(d['value'],d['roofline']['achieved'],d['roofline']['kernel_ms_avg'],d['check']['valid_topk_frac'],d['reduction_roofline']['kernel_ms_avg'],d['reduction_roofline']['bytes_per_launch'])")"
done
