# A/B of an environment knob on one box (boxes differ by up to ~12% in clock):
#   tools/ab_env.sh VAR "v1 v2" [bench args]   -- alternates v1 v2 v1 v2
set -e
mkdir -p gpurun_out
VAR=$1; VALS=$2; shift 2
B="python bench.py --steps 3 --warmup 1 --boundary 0 --extra none --cpu-sample 0 --check 0 $*"
for rep in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 $B > gpurun_out/ab_$v.json 2>/dev/null
    echo "$VAR=$v $(python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print(d['value'],d['roofline']['achieved'])")"
  done
done
