#!/bin/bash
# round 6: kernel-trace-only profile at bs256 (current tree): step breakdown + per-queue tail
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
bash scripts/gpu_prof_step.sh gpurun_out/r6b256 --batch-per-gpu 256 > /dev/null && tail -5 gpurun_out/r6b256/breakdown.txt
