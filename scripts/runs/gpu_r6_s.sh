#!/bin/bash
# round 6: one-launch BN finalize (fin3): numerics, finalize-chain probe, ResNet-50 routes test, bench bs1024 / bs256
O=gpurun_out/r6s
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u -m pytest tests/test_bn_finalize_gpu.py tests/test_bn_gpu.py tests/test_resnet_routes_gpu.py tests/test_convgemm_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python scripts/probe_bn_finalize.py > $O/fin_events.jsonl 2> $O/fin_events.err || { tail -5 $O/fin_events.err; exit 1; }
cat $O/fin_events.jsonl
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/bench_bs1024_$i.json 2> $O/bench_bs1024_$i.err || { tail -5 $O/bench_bs1024_$i.err; exit 1; }
tail -1 $O/bench_bs1024_$i.json | cut -c1-200
timeout -k 10 300 python bench.py --steps 60 --warmup 15 --batch-per-gpu 256 > $O/bench_bs256_$i.json 2> $O/bench_bs256_$i.err || { tail -5 $O/bench_bs256_$i.err; exit 1; }
tail -1 $O/bench_bs256_$i.json | cut -c1-200
done
