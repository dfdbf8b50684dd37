#!/bin/bash
# full GPU suite + smoke + default bench after the flash default / sparse / Philox changes;
# row-kernel roofline again (Philox on 64-bit products)
mkdir -p gpurun_out/r3l
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
bash scripts/gpu_tests.sh || exit $?
cp gpurun_out/tests/pytest.log gpurun_out/r3l/pytest_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3l/smoke.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_server_kernels.py --big 0 --json gpurun_out/r3l/server_kernels.json > gpurun_out/r3l/server_kernels.log 2>&1 || exit $?
timeout -k 10 300 python scripts/probe_fc.py > gpurun_out/r3l/fc_probe.jsonl 2>gpurun_out/r3l/fc_probe.err || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r3l/bench.json 2>gpurun_out/r3l/bench.err || exit $?
grep -E "lazy_init|sorted_runs" gpurun_out/r3l/server_kernels.log | cut -c1-200; cat gpurun_out/r3l/smoke.log | tail -2; cut -c1-300 gpurun_out/r3l/bench.json
cut -c1-250 gpurun_out/r3l/fc_probe.jsonl
