#!/bin/bash
# round 6, final tree after the stem / epilogue trims: full GPU suite + smoke + bench at both batches
O=gpurun_out/${OUT:-r6aj2}
mkdir -p $O
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log
for b in 1024 256; do
timeout -k 10 300 python bench.py --batch-per-gpu $b > $O/bench_$b.json 2> $O/bench_$b.err && tail -1 $O/bench_$b.json
done
