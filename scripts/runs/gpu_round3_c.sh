#!/bin/bash
mkdir -p gpurun_out/r3c
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python scripts/probe_wgrad_blas.py > gpurun_out/r3c/wgrad_blas.jsonl 2> gpurun_out/r3c/wgrad_blas.err
rc=$?; cat gpurun_out/r3c/wgrad_blas.jsonl; exit $rc
