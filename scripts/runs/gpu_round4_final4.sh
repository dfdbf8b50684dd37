#!/bin/bash
# Round-4 final tree (+ stem max-pool k=3 path): full GPU
# suite, smoke, default bench twice, batch 256 twice, step breakdowns at 1024 and 256.
O=gpurun_out/r4final4
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
step() {  # name seconds command...  (any failure ends the call)
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  tail -2 $O/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step full 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_a 200 python bench.py --steps 20 --warmup 8
step bench256_a 200 python bench.py --batch-per-gpu 256 --steps 20 --warmup 8
step bench_b 200 python bench.py --steps 20 --warmup 8
step bench256_b 200 python bench.py --batch-per-gpu 256 --steps 20 --warmup 8
step prof 400 bash scripts/gpu_prof_step.sh $O/p1024
step prof256 400 bash scripts/gpu_prof_step.sh $O/p256 --batch-per-gpu 256
