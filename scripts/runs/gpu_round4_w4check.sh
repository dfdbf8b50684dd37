#!/bin/bash
# W = 4 ranks at bs1024 sharing ONE GPU: side stream on vs off (is the slow shared-GPU step the
# side stream or the four-process time slicing?)
O=gpurun_out/r4w4b  # (first run: r4w4 at the default bs1024)
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH PS_AMD_BENCH_ONE_GPU=1
for m in 0 1; do for bpg in 512; do
  timeout -k 10 600 env PS_AMD_WGRAD_STREAM=$m python bench.py --gpus 4 --steps 4 --warmup 2 --comm-probe 0 --timing 2 --batch-per-gpu $bpg > $O/w4_side$m.log 2>&1 || exit $?
  python3 -c "
import json
for l in open('$O/w4_side$m.log'):
    l=l.strip()
    if l.startswith('{') and '\"metric\"' in l:
        d=json.loads(l); p=d['config'].get('ps_phase_ms_per_step',{})
        print('side=$m', d['value'], d['ms_per_step'], 'exposed', p.get('exposed_comm_ms'), 'fwd_bwd', p.get('fwd_bwd_ms'))
"
done; done
