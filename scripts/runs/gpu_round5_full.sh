#!/bin/bash
# full GPU suite + smoke on the current tree
set -o pipefail
mkdir -p gpurun_out/r5full
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5full/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r5full/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5full/smoke.log 2>&1
