#!/bin/bash
# round 6 tree: step breakdown at bs1024 and bs256 + bench runs
set -o pipefail
mkdir -p gpurun_out/r6z
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
bash scripts/gpu_prof_step.sh gpurun_out/r6z/b1024 > /dev/null && \
bash scripts/gpu_prof_step.sh gpurun_out/r6z/b256 --batch-per-gpu 256 > /dev/null && \
head -3 gpurun_out/r6z/b1024/breakdown.txt && tail -5 gpurun_out/r6z/b1024/breakdown.txt && \
head -3 gpurun_out/r6z/b256/breakdown.txt && tail -5 gpurun_out/r6z/b256/breakdown.txt && \
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/r6z/bench_bs1024.json 2> gpurun_out/r6z/bench_bs1024.err && tail -1 gpurun_out/r6z/bench_bs1024.json | cut -c1-180 && \
timeout -k 10 300 python bench.py --steps 60 --warmup 15 --batch-per-gpu 256 > gpurun_out/r6z/bench_bs256.json 2> gpurun_out/r6z/bench_bs256.err && tail -1 gpurun_out/r6z/bench_bs256.json | cut -c1-180
