#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r5host
timeout -k 10 400 python scripts/probe_host_overhead.py --batches 8,256,1024 > gpurun_out/r5host/host.jsonl 2> gpurun_out/r5host/host.err
