#!/bin/bash
mkdir -p gpurun_out/s23
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -m pytest tests/test_zoo_gpu.py -q > gpurun_out/s23/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/s23/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --config bert-ssp --steps 20 --warmup 5 > gpurun_out/s23/bench_bert.log 2>&1 || exit $?
exit 0
