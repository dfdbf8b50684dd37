#!/bin/bash
set -o pipefail
O=gpurun_out/r5dbg
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 120 python scripts/debug_big_chain.py $O/big.pt > $O/log2.txt 2>&1 && \
PS_AMD_CONV_BIG=0 timeout -k 10 120 python scripts/debug_big_chain.py $O/nobig.pt >> $O/log2.txt 2>&1 && \
UNFUSED=1 timeout -k 10 120 python scripts/debug_big_chain.py $O/unfused.pt >> $O/log2.txt 2>&1 && \
FP32=1 timeout -k 10 120 python scripts/debug_big_chain.py $O/fp32.pt >> $O/log2.txt 2>&1 && \
DEFER=0 timeout -k 10 120 python scripts/debug_big_chain.py $O/nodefer.pt >> $O/log2.txt 2>&1 && \
echo "== big vs fp32" >> $O/log2.txt && python scripts/debug_big_chain.py --cmp $O/big.pt $O/fp32.pt >> $O/log2.txt && \
echo "== nobig vs fp32" >> $O/log2.txt && python scripts/debug_big_chain.py --cmp $O/nobig.pt $O/fp32.pt >> $O/log2.txt && \
echo "== unfused vs fp32" >> $O/log2.txt && python scripts/debug_big_chain.py --cmp $O/unfused.pt $O/fp32.pt >> $O/log2.txt && \
echo "== nodefer(big) vs fp32" >> $O/log2.txt && python scripts/debug_big_chain.py --cmp $O/nodefer.pt $O/fp32.pt >> $O/log2.txt && \
rm -f $O/*.pt
