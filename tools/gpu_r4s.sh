#!/bin/bash
# round 4: PMC of the ws16 kernel's phase-removed lab variants at c4 (clock and
# MFMA busy of the bare MFMA loop, PMM_ABLATE=3, and without the epilogue, =1)
mkdir -p gpurun_out/r4s
for v in 3 1; do
  PMM_LIB=libpmm_lab.so PMM_ABLATE=$v PMC=1 bash tools/profile.sh r4s_abl$v --config c4 --steps 2 --warmup 1 --extra none --cpu-sample 0 --boundary 0 --check 0 || exit 6
done
echo done
