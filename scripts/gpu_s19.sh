#!/bin/bash
# Full GPU suite + smoke + all BASELINE configs (1 GPU) + torchrun 1-rank path.
mkdir -p gpurun_out/s19
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/s19/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/s19/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s19/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/s19/bench_torchrun1.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --config bert-ssp --steps 20 --warmup 5 > gpurun_out/s19/bench_bert.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --config dlrm --steps 20 --warmup 5 > gpurun_out/s19/bench_dlrm.log 2>&1 || exit $?
timeout -k 10 900 python bench.py --config llama-onebit --steps 5 --warmup 2 > gpurun_out/s19/bench_llama.log 2>&1 || exit $?
exit 0
