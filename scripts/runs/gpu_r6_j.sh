#!/bin/bash
# round 6: weight-gradient fork order vs the BN backward apply passes (ResNet-50, 1 GPU), interleaved
O=gpurun_out/r6j
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
for rep in 1 2; do
  for o in 0 1 2 3; do
    PS_AMD_FORK_ORDER=$o timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b_o${o}_$rep.json 2> $O/b_o${o}_$rep.err || exit $?
    echo "order $o rep $rep: $(python -c "import json;r=json.load(open('$O/b_o${o}_$rep.json'));print(r['value'], r['ms_per_step'])")"
  done
done
