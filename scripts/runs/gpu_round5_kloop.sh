#!/bin/bash
# what bounds the 256 x 256 K loop: phase stamps with the MFMAs (9) or MFMAs + fragment reads (8) skipped
set -o pipefail
O=gpurun_out/r5kloop
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 200 python scripts/probe_big_phases.py > $O/phases_full.txt 2>&1 && \
PS_AMD_CONV_BIG_L2PF=9 timeout -k 10 200 python scripts/probe_big_phases.py > $O/phases_nomfma.txt 2>&1 && \
PS_AMD_CONV_BIG_L2PF=8 timeout -k 10 200 python scripts/probe_big_phases.py > $O/phases_dmaonly.txt 2>&1
