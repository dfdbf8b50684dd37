#!/bin/bash
# final-tree step breakdown at bs1024 and bs256
set -o pipefail
mkdir -p gpurun_out/r5proffinal
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
bash scripts/gpu_prof_step.sh gpurun_out/r5proffinal/b1024 && \
bash scripts/gpu_prof_step.sh gpurun_out/r5proffinal/b256 --batch-per-gpu 256
