#!/bin/bash
mkdir -p gpurun_out/stream
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python scripts/probe_stream.py > gpurun_out/stream/probe.jsonl 2>&1 || exit $?
