#!/bin/bash
# round 4: the 16x16x32 wave-specialised bf16 kernel (libpmm_ws16.so, lab
# build with -DPMM_WS_MFMA16=1) -- bf16 parity tests on it, its lists against
# the fire-and-forget kernel's (the same MFMA chain), then c4 alternated with
# the 32x32x16 lab build (libpmm_lab.so)
mkdir -p gpurun_out/r4i
PMM_LIB=libpmm_ws16.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "bf16 and not r64 and not ff" --timeout 300 --timeout-method thread > gpurun_out/r4i/gpu_bf16.log 2>&1
rc=$?
echo "bf16 tests (ws16) rc=$rc"; tail -3 gpurun_out/r4i/gpu_bf16.log
[ $rc -eq 0 ] || exit $rc
PMM_LIB=libpmm_ws16.so timeout -k 10 600 python -u tools/experiments/ws16_vs_ff.py > gpurun_out/r4i/ws16_vs_ff.log 2>&1
echo "ws16 vs ff rc=$?"; tail -2 gpurun_out/r4i/ws16_vs_ff.log
B="--config c4 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 8"
for i in 1 2; do
  for L in libpmm_lab.so libpmm_ws16.so; do
    PMM_LIB=$L timeout -k 10 300 python -u bench.py $B > gpurun_out/r4i/c4_${L%.so}_$i.json 2> gpurun_out/r4i/c4_${L%.so}_$i.log || exit 5
    python3 -c "import json;d=json.load(open('gpurun_out/r4i/c4_${L%.so}_$i.json'));r=d['roofline'];print('$L $i', d['ms_per_step'], r['kernel_ms_avg'], r['seed_ms_avg'], r['frac'], d['check'])"
  done
done
echo done
