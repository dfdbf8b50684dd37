#!/bin/bash
# round 6: world-1 serve inline on the landing stream vs on the comm stream (A/B interleaved on one box)
O=gpurun_out/${OUT:-r6ae}
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_resnet_routes_gpu.py tests/test_ps_gpu.py tests/test_side_stream_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
for v in 0 1; do
PS_AMD_LASTJOIN=$v timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/b1024_i${v}_$i.json 2> $O/b1024_i${v}_$i.err || { tail -5 $O/b1024_i${v}_$i.err; exit 1; }
python -c "import json;r=json.loads(open('$O/b1024_i${v}_$i.json').read().strip().splitlines()[-1]);print('bs1024 lastjoin=$v', r['value'], r['ms_per_step'])"
PS_AMD_LASTJOIN=$v timeout -k 10 300 python bench.py --steps 60 --warmup 15 --batch-per-gpu 256 > $O/b256_i${v}_$i.json 2> $O/b256_i${v}_$i.err || { tail -5 $O/b256_i${v}_$i.err; exit 1; }
python -c "import json;r=json.loads(open('$O/b256_i${v}_$i.json').read().strip().splitlines()[-1]);print('bs256 lastjoin=$v', r['value'], r['ms_per_step'])"
done
done
