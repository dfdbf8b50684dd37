#!/bin/bash
# round 6: BN-backward apply bandwidth standalone; allocator growth inside the timed region (warmup
# length, expandable segments)
O=gpurun_out/r6q
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 200 python scripts/probe_bn_bwd_apply.py > $O/bn_bwd_apply.jsonl 2> $O/bn_bwd_apply.err || { tail -5 $O/bn_bwd_apply.err; exit 1; }
cat $O/bn_bwd_apply.jsonl
run() {  # name, env..., -- bench args
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py $BARGS > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  python -c "import json;r=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);c=r['config'];print('$n', r['value'], r['ms_per_step'], c['device_allocs_timed'], c['reserved_growth_timed_gb'], c['reserved_gb'])"
}
BARGS="--steps 30 --warmup 10" run base_w10 A=1
BARGS="--steps 30 --warmup 40" run base_w40 A=1
BARGS="--steps 30 --warmup 10" run exp_w10 PYTORCH_HIP_ALLOC_CONF=expandable_segments:True
BARGS="--steps 30 --warmup 40" run exp_w40 PYTORCH_HIP_ALLOC_CONF=expandable_segments:True
