#!/bin/bash
# round 4: c4 with the 16x16x32 ws kernel -- PMC passes of the default build
# (MFMA busy, clock, traffic), then candidate-capacity / seed settings
# alternated (the epilogue waves' share may have moved with the faster MFMA waves)
mkdir -p gpurun_out/r4k
bash tools/profile.sh r4_c4_ws16 --config c4 --steps 2 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0 || exit 6
B="--config c4 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0"
run() {  # run <name> <env...>
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py $B > gpurun_out/r4k/$name.json 2> gpurun_out/r4k/$name.log || { echo "$name failed"; exit 5; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4k/$name.json'));r=d['roofline'];print('$name', d['ms_per_step'], r['kernel_ms_avg'], r.get('seed_ms_avg'), r.get('merge_ms_avg'), r['frac'])"
}
for i in 1 2; do
  run def_$i PMM_NONE=1
  run capg256_$i PMM_CAPG=256
  run capg512_$i PMM_CAPG=512
  run noseed_$i PMM_BF16_SEED=0
done
echo done
