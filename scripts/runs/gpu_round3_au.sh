#!/bin/bash
# Re-check of the register-staged tuning knobs after the epilogue spill fix (ResNet-50 bs1024)
O=gpurun_out/r3au
mkdir -p $O
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/$tag.json 2> $O/$tag.err || exit 1
  echo "$tag $(python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
}
run default A=1
run nkpro8 PS_AMD_PERSIST_NK_PRO=8
run nkpro2 PS_AMD_PERSIST_NK_PRO=2
run patch64 PS_AMD_CONV_PATCH64=1
run default2 A=1
run nkpro8b PS_AMD_PERSIST_NK_PRO=8
