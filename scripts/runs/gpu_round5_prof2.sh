#!/bin/bash
# round-5 step breakdown (after ds / stem / big-tile changes) at bs1024 and bs256 + conv probe table
set -o pipefail
mkdir -p gpurun_out/r5prof2
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
bash scripts/gpu_prof_step.sh gpurun_out/r5prof2/b1024 && \
bash scripts/gpu_prof_step.sh gpurun_out/r5prof2/b256 --batch-per-gpu 256 && \
timeout -k 10 400 python scripts/probe_resnet_convs.py > gpurun_out/r5prof2/conv_tflops.txt 2> gpurun_out/r5prof2/conv_tflops.err
