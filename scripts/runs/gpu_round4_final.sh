#!/bin/bash
# Round-4 final-tree validation + the last A/Bs: full GPU suite, smoke, default bench (twice),
# batch 256, deep LDS-DMA ring and HIP-graph A/Bs, plain-GEMM probe, step breakdown.
O=gpurun_out/r4final
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
step() {  # name seconds command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  tail -2 $O/$name.log | cut -c1-300
  if [ $rc -ge 124 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step full 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_a 200 python bench.py --steps 20 --warmup 8
step bench_b 200 python bench.py --steps 20 --warmup 8
step bench256 200 python bench.py --batch-per-gpu 256 --steps 20 --warmup 8
step bench_deep 200 env PS_AMD_GLDS_STAGES=3 python bench.py --steps 20 --warmup 8
step bench_graph 300 python bench.py --steps 20 --warmup 8 --graph 1
step bench256_graph 300 python bench.py --batch-per-gpu 256 --steps 20 --warmup 8 --graph 1
step probe2 200 env PROBE_ONLY=plain_gemm python scripts/probe_twosrc.py
step probe3 200 env PS_AMD_GLDS_STAGES=3 PS_AMD_GLDS_DEEP_MIN_NK=4 PROBE_ONLY=plain_gemm python scripts/probe_twosrc.py
step prof 400 bash scripts/gpu_prof_step.sh $O/p1024
