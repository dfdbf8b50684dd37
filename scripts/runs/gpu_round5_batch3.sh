#!/bin/bash
# Batch 3: layer-2 fused conv3 backward with 8 waves (tests, probe, bench); the 1-bit push at
# Llama-3-8B width (2 ranks on cuda:0, xGMI plane, 60 steps, onebit vs none); the Llama-3-8B serve
# on a CU-masked stream (A/B at 32 / 64 CUs vs the default).
O=gpurun_out/r5b3
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_conv_bwd_fused_gpu.py \
  "tests/test_convgemm_gpu.py::test_fused_bottleneck_matches_module_path" -m gpu > $O/pytest_conv.log 2>&1; rc=$?
tail -3 $O/pytest_conv.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/probe_conv3_bwd.py > $O/probe.jsonl 2> $O/probe.err || exit $?
cat $O/probe.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > $O/bench.json 2> $O/bench.err || exit $?
grep -o '"value": [0-9.]*' $O/bench.json
for c in onebit none; do
  PS_AMD_BENCH_ONE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 scripts/llama_width_onebit.py --compress $c --steps 60 \
    > $O/llama_width_$c.jsonl 2> $O/llama_width_$c.err || exit $?
  tail -c 1500 $O/llama_width_$c.jsonl
done
for cus in 0 64 32; do
  PS_AMD_SERVE_CUS=$cus timeout -k 10 400 python bench.py --config llama-onebit --steps 6 --warmup 3 --timing 3 \
    > $O/llama_w1_cus$cus.json 2> $O/llama_w1_cus$cus.err || exit $?
  python3 -c "import json;d=json.loads(open('$O/llama_w1_cus$cus.json').read().strip().splitlines()[-1]);print('cus $cus', d['value'], d['ms_per_step'], json.dumps(d['config'].get('ps_phase_ms_per_step')))"
done
