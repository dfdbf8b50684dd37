#!/bin/bash
# round 6 final-tree checks: full GPU suite, smoke(), bench default (bs1024), bs256, other configs
O=gpurun_out/${OUT:-r6final}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_full.log 2>&1 || { tail -40 $O/pytest_gpu_full.log; exit 1; }
tail -1 $O/pytest_gpu_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-220
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/bench_bs1024.json 2> $O/bench_bs1024.err || { tail -5 $O/bench_bs1024.err; exit 1; }
tail -1 $O/bench_bs1024.json | cut -c1-220
timeout -k 10 300 python bench.py --steps 60 --warmup 15 --batch-per-gpu 256 > $O/bench_bs256.json 2> $O/bench_bs256.err || { tail -5 $O/bench_bs256.err; exit 1; }
tail -1 $O/bench_bs256.json | cut -c1-220
