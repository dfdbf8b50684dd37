#!/bin/bash
# full GPU suite + smoke + default bench (after the wgrad LIN path, fused xent, XCD flash, fc v3)
mkdir -p gpurun_out/r3x
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
bash scripts/gpu_tests.sh || exit $?
cp gpurun_out/tests/pytest.log gpurun_out/r3x/pytest_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3x/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r3x/bench.json 2>gpurun_out/r3x/bench.err || exit $?
tail -2 gpurun_out/r3x/smoke.log; cut -c1-250 gpurun_out/r3x/bench.json
