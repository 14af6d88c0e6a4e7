#!/bin/bash
# rows64 probe (256 query rows per CU, bare loop) on its round-3 synthetic
# data (mode 0) and on N(0,1) bf16 data (mode 1, the c4 bench's data)
mkdir -p gpurun_out/probe
cd tools/experiments
for a in 0 1 2; do
  for m in 0 1 0 1; do
    timeout -k 10 120 ./bf16_rows64_probe_a$a 3 $m >> ../../gpurun_out/probe/probe.txt 2>&1 || exit 1
  done
done
