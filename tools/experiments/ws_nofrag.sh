#!/bin/bash
# wave-specialised bf16 kernel at c4 without the epilogue (PMM_ABLATE=1) and
# without epilogue or corpus traffic (3): default build vs a diagnostic build
# whose MFMA waves skip their LDS fragment reads (build it first with
# `make -C polars-matmul_amd wsx WSX=-DPMM_WS_NOFRAG`, loaded as libpmm_wsx.so):
# what do the fragment reads cost?
set -o pipefail
mkdir -p gpurun_out
for lib in libpmm.so libpmm_wsx.so; do
  for ab in 1 3; do
    PMM_LIB=$lib PMM_ABLATE=$ab timeout -k 10 300 python3 -u bench.py --config c4 --steps 3 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0 > gpurun_out/nf_${lib}_$ab.log 2>&1 || exit 2
  done
done
