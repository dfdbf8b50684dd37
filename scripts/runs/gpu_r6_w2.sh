#!/bin/bash
# round 6: the multi-rank ResNet-50 bench path rehearsed with W=2 and W=4 processes on one GPU (xGMI plane over IPC,
# side stream, step-boundary changes), bs256 per rank
O=gpurun_out/r6w2
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH PS_AMD_BENCH_ONE_GPU=1
for W in 2 4; do
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port 2952$W bench.py --gpus $W --steps 10 --warmup 5 --batch-per-gpu 256 > $O/w$W.json 2> $O/w$W.err || { tail -20 $O/w$W.err; exit 1; }
tail -1 $O/w$W.json | cut -c1-400
done
