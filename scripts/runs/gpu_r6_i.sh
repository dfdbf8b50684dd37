#!/bin/bash
# round 6: 1-bit pack on its own stream + bf16 error feedback; full-depth Llama-3-8B, W=2 on one GPU
# env: SKIP_TESTS=1 skips the pytest part; LLAMA_MODES="onebit:bf16 none:fp32" (compress:ef)
O=gpurun_out/r6i
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH PS_AMD_BENCH_ONE_GPU=1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k onebit tests/test_plane_gpu.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
for mode in ${LLAMA_MODES:-onebit:bf16:0 none:fp32:0}; do
  IFS=: read c e w <<< "$mode"; w=${w:-0}; tag=${c}_${e}_w${w}
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    scripts/llama_width_onebit.py --layers 32 --ckpt 1 --batch 1 --seq 4096 --steps ${LLAMA_STEPS:-14} --timed 6 --compress $c --ef $e --warmup $w \
    > $O/llama8b_full_$tag.jsonl 2> $O/llama8b_full_$tag.err || { tail -20 $O/llama8b_full_$tag.err; exit 1; }
  tail -2 $O/llama8b_full_$tag.jsonl | cut -c1-1500
done
