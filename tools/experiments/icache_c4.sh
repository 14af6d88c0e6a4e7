#!/bin/bash
# instruction-cache counters of the wave-specialised bf16 kernel at c4: list
# the SQC instruction-cache counters the box offers, then one PMC pass with them
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/icache${ICACHE_TAG:-}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$O/counters.txt" 2>&1 || exit 1
grep -oE "SQC?_[A-Z_]*(ICACHE|IFETCH|INST_LEVEL|WAIT_INST)[A-Z_]*" "$O/counters.txt" | sort -u > "$O/names.txt" || true
C=$(grep -E "^(SQC_ICACHE_HITS|SQC_ICACHE_MISSES|SQC_ICACHE_MISSES_DUPLICATE|SQ_IFETCH)$" "$O/names.txt" | tr '\n' ' ')
echo "counters: $C"
[ -n "$C" ] || exit 0
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$O/pmc" -o run -- \
  python3 "$R/bench.py" --config c4 --steps 1 --warmup 0 --boundary 0 --extra none --cpu-sample 0 --check 0 \
  > "$O/pmc.log" 2>&1
