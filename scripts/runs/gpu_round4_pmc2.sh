#!/bin/bash
# PMC passes over the final ResNet-50 step (bs1024): per-kernel MFMA busy, waits, VALU/MFMA, LDS conflicts, L2 hit
mkdir -p gpurun_out/r4pmc2
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
cd /tmp
pass() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" -d $R/gpurun_out/r4pmc2/$name -o run --output-format csv \
    -- python3 $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/r4pmc2/$name.log 2>&1
}
pass p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA || exit $?
pass p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU SQ_INST_LEVEL_VMEM TCC_HIT_sum TCC_MISS_sum || exit $?
cd $R && python3 scripts/pmc_summary.py gpurun_out/r4pmc2/p1 gpurun_out/r4pmc2/p2 --match conv_ bn_ stem weight_prep pool > gpurun_out/r4pmc2/summary.txt
find gpurun_out/r4pmc2 -name '*kernel_trace.csv' -delete
find gpurun_out/r4pmc2 -name '*counter_collection.csv' -delete
wc -l gpurun_out/r4pmc2/summary.txt
