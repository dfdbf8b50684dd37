#!/bin/bash
# final-tree validation: full GPU suite, smoke, default bench, bs256 line, multi-rank plane rehearsal, step trace
mkdir -p gpurun_out/r3al
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
bash scripts/gpu_tests.sh || exit $?
cp gpurun_out/tests/pytest.log gpurun_out/r3al/pytest_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3al/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r3al/bench.json 2>gpurun_out/r3al/bench.err || exit $?
timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 20 --warmup 5 > gpurun_out/r3al/bench_bs256.json 2>>gpurun_out/r3al/bench.err || exit $?
PS_AMD_BENCH_ONE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 --comm-probe 0 \
  --batch-per-gpu 256 --timing 3 > gpurun_out/r3al/n2_rehearsal.json 2> gpurun_out/r3al/n2_rehearsal.err || exit $?
PS_AMD_BENCH_ONE_GPU=1 timeout -k 10 400 python bench.py --gpus 4 --steps 10 --warmup 3 --comm-probe 0 \
  --batch-per-gpu 128 --timing 3 > gpurun_out/r3al/n4_rehearsal.json 2> gpurun_out/r3al/n4_rehearsal.err || exit $?
R=$PWD; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r3al/prof -o run -- \
  python3 $R/bench.py --steps 3 --warmup 5 > $R/gpurun_out/r3al/prof.log 2>&1 || exit $?
cd $R && f=$(find gpurun_out/r3al/prof -name '*kernel_trace.csv' | head -1) && python3 scripts/step_breakdown.py $f > gpurun_out/r3al/step_breakdown.txt
tail -2 gpurun_out/r3al/smoke.log; cut -c1-200 gpurun_out/r3al/bench.json gpurun_out/r3al/bench_bs256.json gpurun_out/r3al/n2_rehearsal.json gpurun_out/r3al/n4_rehearsal.json
head -3 gpurun_out/r3al/step_breakdown.txt
