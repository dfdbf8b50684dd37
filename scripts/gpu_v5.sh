#!/bin/bash
# PMC counters of the conv GEMM kernels (quick probe: 2 shapes), one pass
R=$PWD
mkdir -p gpurun_out/v5
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $R/gpurun_out/v5/pmc -o run -- python3 $R/scripts/probe_convgemm.py --quick > $R/gpurun_out/v5/pmc.log 2>&1 || exit $?
exit 0
