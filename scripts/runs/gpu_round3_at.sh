#!/bin/bash
# Final-tree validation after the epilogue spill fix: full GPU suite, smoke, default bench
O=gpurun_out/r3at
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
bash scripts/gpu_tests.sh || exit $?
cp gpurun_out/tests/pytest.log $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
tail -1 $O/bench.json
