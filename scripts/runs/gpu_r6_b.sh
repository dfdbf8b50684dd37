#!/bin/bash
# round 6: GELU epilogue FFN tests + BERT after, run-ahead allocator test, HIP API trace of the stall
O=gpurun_out/r6b
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gelu_ffn_gpu.py tests/test_runahead_gpu.py > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 > $O/bert_after.json 2> $O/bert_after.err || exit $?
tail -1 $O/bert_after.json
PS_AMD_LT_GELU=0 timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 > $O/bert_nolt.json 2> $O/bert_nolt.err || exit $?
tail -1 $O/bert_nolt.json
cd /tmp && PS_AMD_MAX_INFLIGHT=0 timeout -k 10 300 rocprofv3 --hip-runtime-trace -d $R/$O/api -o run --output-format csv -- python $R/scripts/probe_stall_alloc.py --steps 12 > $R/$O/api.log 2>&1 || exit $?
cd $R && grep -h step $O/api.log | cut -c1-120 | head -14; python scripts/api_trace_top.py $(ls $O/api/*hip_api_trace.csv | head -1) 25 > $O/api_top.txt 2>&1; cat $O/api_top.txt
