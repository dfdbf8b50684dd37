#!/bin/bash
# Round-end style validation: full GPU suite, smoke(), default bench, kernel-trace step breakdown
O=gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-200
bash scripts/gpu_prof_step.sh $O/pstep > /dev/null || exit $?
head -8 $O/pstep/breakdown.txt
