#!/bin/bash
# round 4: the per-rank shapes of the multi-GPU runs (c3 / c4 with 1/2, 1/4,
# 1/8 of the corpus) on one GPU
mkdir -p gpurun_out/r4u
timeout -k 10 600 python -u tools/experiments/shard_shapes.py > gpurun_out/r4u/shapes.jsonl 2> gpurun_out/r4u/shapes.log || exit 5
cat gpurun_out/r4u/shapes.jsonl
echo done
