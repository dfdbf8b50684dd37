#!/bin/bash
# round 5: HBM bytes per kernel over the ResNet-50 step (FETCH / WRITE passes + a clean trace), and
# SQ / LDS / cache counters of the layer-1 3x3 kernels (planar c64 kernel vs the tall tile)
set -o pipefail
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
mkdir -p gpurun_out/r5pmc
cd /tmp
cpass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $R/gpurun_out/r5pmc/$name -o run --output-format csv \
    -- python3 $R/scripts/probe_conv3x3_c64.py > $R/gpurun_out/r5pmc/$name.log 2>&1
}
for m in 2 0; do
  export PS_AMD_CONV_C64=$m
  cpass c64m${m}_p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA || exit $?
  cpass c64m${m}_p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU SQ_INST_LEVEL_VMEM TCC_HIT_sum TCC_MISS_sum || exit $?
  cpass c64m${m}_p3 FETCH_SIZE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum || exit $?
  cpass c64m${m}_p4 WRITE_SIZE TA_BUSY_avr TA_TA_BUSY_sum || exit $?
done
unset PS_AMD_CONV_C64
cd $R && python3 scripts/pmc_summary.py gpurun_out/r5pmc/c64m2_p1 gpurun_out/r5pmc/c64m2_p2 gpurun_out/r5pmc/c64m2_p3 gpurun_out/r5pmc/c64m2_p4 --match c64s > gpurun_out/r5pmc/c64m2.txt 2>&1
python3 scripts/pmc_summary.py gpurun_out/r5pmc/c64m0_p1 gpurun_out/r5pmc/c64m0_p2 gpurun_out/r5pmc/c64m0_p3 gpurun_out/r5pmc/c64m0_p4 --match "conv_fwd" > gpurun_out/r5pmc/c64m0.txt 2>&1
cd /tmp
spass() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" -d $R/gpurun_out/r5pmc/$name -o run --output-format csv \
    -- python3 $R/bench.py --steps 2 --warmup 2 > $R/gpurun_out/r5pmc/$name.log 2>&1
}
spass fetch FETCH_SIZE || exit $?
spass write WRITE_SIZE || exit $?
mkdir -p $R/gpurun_out/r5pmc/clean
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r5pmc/clean -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 > $R/gpurun_out/r5pmc/clean.log 2>&1 || exit $?
cd $R && python3 scripts/pmc_step_summary.py gpurun_out/r5pmc/fetch gpurun_out/r5pmc/write $(ls gpurun_out/r5pmc/clean/*kernel_trace.csv | head -1) --top 60 > gpurun_out/r5pmc/summary.txt 2>&1
head -5 gpurun_out/r5pmc/summary.txt
