#!/bin/bash
# full GPU suite + smoke + default bench + a roctx marker trace of a short ResNet run
mkdir -p gpurun_out/full gpurun_out/marker
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/full/pytest.log; tail -3 gpurun_out/full/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/full/bench.log 2>&1 || exit $?
tail -1 gpurun_out/full/bench.log | cut -c1-200
cd /tmp && timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace -d $R/gpurun_out/marker -o run --output-format csv -- python $R/bench.py --steps 3 --warmup 2 --batch-per-gpu 128 > $R/gpurun_out/marker/run.log 2>&1 || exit $?
ls $R/gpurun_out/marker
