#!/bin/bash
# round 6: (1) GPU probe tests incl. async rows; (2) host-launch vs GPU-start of the ResNet-50 step (kernel + HIP API trace)
O=gpurun_out/r6ad
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_remote_probe_gpu.py tests/test_async_ps_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --hip-runtime-trace -d $R/$O/prof -o run --output-format csv -- python $R/bench.py --steps 6 --warmup 3 > $R/$O/prof.log 2>&1 || { tail -20 $R/$O/prof.log; exit 1; }
cd $R && ls $O/prof/*/ | head; python scripts/launch_lag.py $(ls $O/prof/*/*kernel_trace.csv | head -1) $(ls $O/prof/*/*hip_api_trace.csv | head -1) 40 > $O/launch_lag.txt && cat $O/launch_lag.txt
