#!/bin/bash
# round 4: per-rank shapes at 1/4 and 1/8 of the corpus with the seed and the
# whole-block schedule toggled (where the non-GEMM time of a shard goes)
mkdir -p gpurun_out/r4v
export SHAPE_VARIANTS='[["f32", 8, {}], ["f32", 8, {"PMM_SEED": "0"}], ["f32", 4, {}], ["f32", 4, {"PMM_SEED": "0"}], ["bf16", 8, {}], ["bf16", 8, {"PMM_BF16_WHOLE": "0"}], ["bf16", 8, {"PMM_BF16_SEED": "0"}], ["bf16", 4, {}], ["bf16", 4, {"PMM_BF16_WHOLE": "0"}]]'
timeout -k 10 600 python -u tools/experiments/shard_shapes.py > gpurun_out/r4v/shapes.jsonl 2> gpurun_out/r4v/shapes.log || exit 5
cat gpurun_out/r4v/shapes.jsonl
echo done
