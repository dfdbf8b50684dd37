#!/bin/bash
mkdir -p gpurun_out/bs
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
for b in 256 768 1024; do
  timeout -k 10 300 python bench.py --steps 15 --warmup 5 --batch-per-gpu $b --json-out gpurun_out/bs/b$b.json > gpurun_out/bs/b$b.log 2>&1 || exit $?
  cat gpurun_out/bs/b$b.json
done
