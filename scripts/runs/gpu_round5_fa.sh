#!/bin/bash
# round-5: flash-attention kernel changes (stage ring depth; bare v_exp_f32, packed bf16 converts, diag-only mask) -- numerics tests, standalone kernel times, Llama bench
set -o pipefail
O=${O:-gpurun_out/r5fa}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_flash_gpu.py tests/test_transformer_gpu.py tests/test_attention_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/probe_flash.py 4 > $O/probe.json 2> $O/probe.err && cat $O/probe.json && \
R=$PWD && cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python $R/scripts/probe_flash.py 4 > $R/$O/prof.log 2>&1 && cd $R && \
python scripts/kernel_stats_top.py $O/prof/run_kernel_stats.csv | head -8 && \
timeout -k 10 200 python scripts/probe_bert_attn.py > $O/bert_attn.json 2> $O/bert_attn.err && cat $O/bert_attn.json && \
timeout -k 10 500 python bench.py --config llama-onebit --steps 6 --warmup 3 > $O/llama.json 2> $O/llama.err && tail -1 $O/llama.json && \
timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 > $O/bert.json 2> $O/bert.err && tail -1 $O/bert.json
