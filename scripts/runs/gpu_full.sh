#!/bin/bash
# Round-end style validation: full GPU test suite, smoke(), default bench
mkdir -p gpurun_out/full
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/full/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/full/bench.log 2>&1 || exit $?
exit 0
