#!/bin/bash
# round 6: A/B of the wide weight-gradient LDS ring depth (kWS 4 -> 3: 128 -> 96 KiB, so a compute-stream
# GEMM block may share a CU with a weight-gradient block), interleaved on one box
O=gpurun_out/r6y
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
SO=ps_amd/_C.cpython-310-x86_64-linux-gnu.so
timeout -k 10 200 python -u -m pytest tests/test_convgemm_gpu.py -x -q -k "wgrad or patch" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_p2.log 2>&1 || { tail -30 $O/pytest_p2.log; exit 1; }
tail -1 $O/pytest_p2.log
for i in 1 2; do
for v in ws3 p2; do
cp alt/_C_$v.so $SO
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/b1024_${v}_$i.json 2> $O/b1024_${v}_$i.err || { tail -5 $O/b1024_${v}_$i.err; exit 1; }
python -c "import json;r=json.loads(open('$O/b1024_${v}_$i.json').read().strip().splitlines()[-1]);print('bs1024 $v', r['value'], r['ms_per_step'])"
timeout -k 10 300 python bench.py --steps 60 --warmup 15 --batch-per-gpu 256 > $O/b256_${v}_$i.json 2> $O/b256_${v}_$i.err || { tail -5 $O/b256_${v}_$i.err; exit 1; }
python -c "import json;r=json.loads(open('$O/b256_${v}_$i.json').read().strip().splitlines()[-1]);print('bs256 $v', r['value'], r['ms_per_step'])"
done
done
