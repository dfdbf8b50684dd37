#!/bin/bash
# round 6: 1-bit Adam (momentum compression, frozen owner variance) -- kernel + plane tests, then the
# full-depth Llama-3-8B W=2 quality probe: uncompressed vs 1-bit Adam (10 warm-up rounds)
O=gpurun_out/${OUT:-r6aa}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH PS_AMD_BENCH_ONE_GPU=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_plane_gpu.py -k onebit > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for mode in ${LLAMA_MODES:-onebit:bf16:10:1}; do
  IFS=: read c e w adam r <<< "$mode"; w=${w:-0}; adam=${adam:-0}; r=${r:-0}; tag=${c}_${e}_w${w}_a${adam}_r${r}
  timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    scripts/llama_width_onebit.py --layers 32 --ckpt 1 --batch 1 --seq 4096 --steps ${LLAMA_STEPS:-40} --timed 6 --compress $c --ef $e --warmup $w --adam1bit $adam --refresh $r \
    > $O/llama8b_full_$tag.jsonl 2> $O/llama8b_full_$tag.err || { tail -20 $O/llama8b_full_$tag.err; exit 1; }
  tail -1 $O/llama8b_full_$tag.jsonl | cut -c1-600
done
