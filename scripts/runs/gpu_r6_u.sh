#!/bin/bash
# round 6: host slack of the ResNet-50 step at bs256 / bs1024
O=gpurun_out/r6u
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
timeout -k 10 300 python scripts/probe_host_slack.py 256 60 > $O/slack256.log 2>&1 || { tail -20 $O/slack256.log; exit 1; }
tail -1 $O/slack256.log
timeout -k 10 300 python scripts/probe_host_slack.py 1024 30 > $O/slack1024.log 2>&1 || { tail -20 $O/slack1024.log; exit 1; }
tail -1 $O/slack1024.log
