#!/bin/bash
# round 6: after the variant prune -- full GPU suite, then the ResNet-50 bench at bs1024 and bs256
O=gpurun_out/r6p
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_full.log 2>&1 || { tail -40 $O/pytest_gpu_full.log; exit 1; }
tail -2 $O/pytest_gpu_full.log
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/bench_bs1024.json 2> $O/bench_bs1024.err || { tail -5 $O/bench_bs1024.err; exit 1; }
tail -1 $O/bench_bs1024.json
timeout -k 10 300 python bench.py --steps 60 --warmup 15 --batch-per-gpu 256 > $O/bench_bs256.json 2> $O/bench_bs256.err || { tail -5 $O/bench_bs256.err; exit 1; }
tail -1 $O/bench_bs256.json
