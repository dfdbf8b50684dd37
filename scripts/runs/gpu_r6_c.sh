#!/bin/bash
# round 6: run-ahead allocator test, HIP API trace of the unbounded run-ahead stall, bench with the allocator fields
O=gpurun_out/r6c
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_runahead_gpu.py > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && PS_AMD_MAX_INFLIGHT=0 timeout -k 10 300 rocprofv3 --hip-runtime-trace -d $R/$O/api -o run --output-format csv -- python $R/scripts/probe_stall_alloc.py --steps 12 > $R/$O/api.log 2>&1 || exit $?
cd $R && grep -h '"step"' $O/api.log | cut -c1-100; python scripts/api_trace_top.py $(ls $O/api/*hip_api_trace.csv | head -1) 30 > $O/api_top.txt 2>&1; cat $O/api_top.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
tail -1 $O/bench.json
