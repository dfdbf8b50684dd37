#!/bin/bash
# round 6: remote-write probe tests (AsyncPS / row plane, W=2 processes on cuda:0) + async/plane regressions
O=gpurun_out/r6f
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_remote_probe_gpu.py tests/test_async_ps_gpu.py tests/test_row_plane_gpu.py tests/test_runahead_gpu.py > $O/pytest.log 2>&1; rc=$?
tail -25 $O/pytest.log
exit $rc
