#!/bin/bash
mkdir -p gpurun_out/s25
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --timing 10 > gpurun_out/s25/bench_resnet.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --config bert-ssp --steps 20 --warmup 5 --timing 10 > gpurun_out/s25/bench_bert.log 2>&1 || exit $?
exit 0
