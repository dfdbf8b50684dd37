#!/bin/bash
# round-5 final: full GPU suite + smoke + every BASELINE config (driver flags: --warmup 5) on the final tree
set -o pipefail
O=${O:-gpurun_out/r5final3}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/resnet_default.json 2> $O/resnet_default.err && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/resnet.json 2> $O/resnet.err && \
timeout -k 10 300 python bench.py --batch-per-gpu 256 --steps 30 --warmup 5 > $O/resnet256.json 2> $O/resnet256.err && \
timeout -k 10 300 python bench.py --config bert-ssp --steps 20 --warmup 5 > $O/bert.json 2> $O/bert.err && \
timeout -k 10 300 python bench.py --config dlrm --steps 20 --warmup 5 > $O/dlrm.json 2> $O/dlrm.err && \
timeout -k 10 300 python bench.py --config ctr-async --steps 20 --warmup 5 > $O/ctr.json 2> $O/ctr.err && \
timeout -k 10 500 python bench.py --config llama-onebit --steps 6 --warmup 3 > $O/llama.json 2> $O/llama.err
