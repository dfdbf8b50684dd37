#!/bin/bash
# round 3 batch J: ResNet-50 step profile (bs1024) + bs256 number; Llama rocprof (flash default)
# + exposed_comm_ms at world 1; BERT async vs pipelined re-measure.
mkdir -p gpurun_out/r3j
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
R=$PWD
bash scripts/gpu_prof_step.sh gpurun_out/r3j/rn || exit $?
find gpurun_out/r3j/rn/prof -name '*kernel_trace.csv' -delete
timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 20 --warmup 5 > gpurun_out/r3j/rn_b256.json 2>/dev/null || exit $?
PS_AMD_TIMING=1 timeout -k 10 400 python bench.py --config llama-onebit --steps 6 --warmup 3 > gpurun_out/r3j/llama_timing.json 2>gpurun_out/r3j/llama_timing.err || exit $?
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3j/lprof -o run --output-format csv -- python $R/bench.py --config llama-onebit --steps 3 --warmup 2 > $R/gpurun_out/r3j/lprof.log 2>&1 || exit $?
cd $R && python scripts/kernel_stats_top.py $(ls gpurun_out/r3j/lprof/*kernel_stats.csv | head -1) 30 > gpurun_out/r3j/llama_top.txt || exit $?
find gpurun_out/r3j/lprof -name '*kernel_trace.csv' -delete
for B in 256 1024; do
  for A in 1 0; do
    PS_AMD_BERT_ASYNC=$A timeout -k 10 300 python bench.py --config bert-ssp --batch-per-gpu $B --steps 20 --warmup 5 \
      > gpurun_out/r3j/bert_b${B}_async${A}.json 2> gpurun_out/r3j/bert_b${B}_async${A}.err || exit $?
  done
done
cut -c1-200 gpurun_out/r3j/*.json; head -20 gpurun_out/r3j/llama_top.txt
