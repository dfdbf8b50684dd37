#!/bin/bash
# round-5: PyTorch TunableOp over hipBLASLt solutions for the Llama-3-8B GEMMs.  Tuning resumes from
# the table so far (ps_amd/tuning/llama-onebit_partial.csv: the forward shapes), writes the full table,
# then the bench runs with it (lookups only, ps_amd/utils/gemm_tuning.py) vs without.
set -o pipefail
O=${O:-gpurun_out/r5tunable2}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
( while true; do date >> $O/heartbeat.txt; sleep 45; done ) &
HB=$!
[ -f ps_amd/tuning/llama-onebit_partial.csv ] && cp ps_amd/tuning/llama-onebit_partial.csv $O/llama_tuned0.csv  # first run's forward shapes (not kept in the tree)
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_ROCBLAS_ENABLED=0 \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=10 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=3 \
PYTORCH_TUNABLEOP_FILENAME=$O/llama_tuned.csv timeout -k 10 900 python bench.py --config llama-onebit --steps 1 --warmup 1 > $O/llama_tune.json 2> $O/llama_tune.err
rc=$?
kill $HB
[ $rc -ne 0 ] && exit $rc
cat $O/llama_tuned0.csv
PS_AMD_GEMM_TUNING=$O/llama_tuned0.csv timeout -k 10 500 python bench.py --config llama-onebit --steps 6 --warmup 3 > $O/llama_tuned.json 2> $O/llama_tuned.err && tail -1 $O/llama_tuned.json && \
PS_AMD_GEMM_TUNING=off timeout -k 10 500 python bench.py --config llama-onebit --steps 6 --warmup 3 > $O/llama_default.json 2> $O/llama_default.err && tail -1 $O/llama_default.json
