#!/bin/bash
# round 6: async-rows remote-write probe on the GPU + the remaining GPU probe tests
O=gpurun_out/r6ac
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_remote_probe_gpu.py tests/test_async_ps_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
