#!/bin/bash
# stride-2 patch weight gradient: tests, probe of the three 64/128-channel 3x3 shapes vs MIOpen, bench A/B
mkdir -p gpurun_out/r3ac
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_convgemm_gpu.py \
  > gpurun_out/r3ac/pytest.log 2>&1 || { tail -40 gpurun_out/r3ac/pytest.log; exit 1; }
tail -2 gpurun_out/r3ac/pytest.log
timeout -k 10 400 python scripts/probe_wgrad.py --it 10 --only "3x3 56x56 64->64,3x3 56x56 128->128,3x3 28x28 128->128" \
  > gpurun_out/r3ac/wgrad_probe.jsonl 2>gpurun_out/r3ac/probe.err || exit $?
cut -c1-200 gpurun_out/r3ac/wgrad_probe.jsonl
run() { env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 8 >> gpurun_out/r3ac/bench_ab.jsonl 2>>gpurun_out/r3ac/bench.err || exit $?;
        echo "$*: $(tail -1 gpurun_out/r3ac/bench_ab.jsonl | cut -c100-190)"; }
run PS_AMD_WGRAD_PATCH_MAX_C=128
run PS_AMD_WGRAD_PATCH_MAX_C=0
run PS_AMD_WGRAD_PATCH_MAX_C=128 PS_AMD_BN_BWD_PROLOGUE_MAX_C=0
run PS_AMD_WGRAD_PATCH_MAX_C=128
run PS_AMD_WGRAD_PATCH_MAX_C=0
run PS_AMD_WGRAD_PATCH_MAX_C=128 PS_AMD_BN_BWD_PROLOGUE_MAX_C=0
# 1x1 forward GEMMs: timing vs hipBLASLt + one PMC pass (why the bn2-prologue conv3 forward of layers 2-4 runs at 1-3 TB/s)
timeout -k 10 200 python scripts/probe_conv_fwd.py > gpurun_out/r3ac/conv_fwd_probe.jsonl 2>>gpurun_out/r3ac/probe.err || exit $?
R=$PWD; cd /tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA \
  -d $R/gpurun_out/r3ac/pmc1 -o run --output-format csv -- python3 $R/scripts/probe_conv_fwd.py > $R/gpurun_out/r3ac/pmc1.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INST_LEVEL_VMEM TCC_HIT_sum TCC_MISS_sum \
  -d $R/gpurun_out/r3ac/pmc2 -o run --output-format csv -- python3 $R/scripts/probe_conv_fwd.py > $R/gpurun_out/r3ac/pmc2.log 2>&1 || exit $?
cd $R && python3 scripts/pmc_summary.py gpurun_out/r3ac/pmc1 gpurun_out/r3ac/pmc2 --match conv_fwd > gpurun_out/r3ac/pmc_summary.txt
find gpurun_out/r3ac -name '*kernel_trace.csv' -delete
echo done
