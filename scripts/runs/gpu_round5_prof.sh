#!/bin/bash
# round-5 step breakdown at bs1024 and bs256, plus a bs256 bench
set -o pipefail
mkdir -p gpurun_out/r5prof
bash scripts/gpu_prof_step.sh gpurun_out/r5prof/b1024 && \
bash scripts/gpu_prof_step.sh gpurun_out/r5prof/b256 --batch-per-gpu 256 && \
timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 10 > gpurun_out/r5prof/bench256.json 2> gpurun_out/r5prof/bench256.err
