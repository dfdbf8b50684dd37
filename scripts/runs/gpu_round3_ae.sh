#!/bin/bash
# full GPU suite + smoke + default bench of the tree with the patch weight gradient and the bn3 prologue
mkdir -p gpurun_out/r3ae
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
bash scripts/gpu_tests.sh || exit $?
cp gpurun_out/tests/pytest.log gpurun_out/r3ae/pytest_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3ae/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r3ae/bench.json 2>gpurun_out/r3ae/bench.err || exit $?
tail -2 gpurun_out/r3ae/smoke.log; cut -c1-250 gpurun_out/r3ae/bench.json
