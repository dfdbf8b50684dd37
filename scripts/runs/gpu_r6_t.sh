#!/bin/bash
# round 6: A/B of the one-launch BN finalize on one box (interleaved), bs1024 and bs256
O=gpurun_out/r6t
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
for i in 1 2; do
for f in 0 1; do
PS_AMD_FIN3=$f timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/b1024_f${f}_$i.json 2> $O/b1024_f${f}_$i.err || { tail -5 $O/b1024_f${f}_$i.err; exit 1; }
python -c "import json;r=json.loads(open('$O/b1024_f${f}_$i.json').read().strip().splitlines()[-1]);print('bs1024 fin3=$f', r['value'], r['ms_per_step'])"
PS_AMD_FIN3=$f timeout -k 10 300 python bench.py --steps 60 --warmup 15 --batch-per-gpu 256 > $O/b256_f${f}_$i.json 2> $O/b256_f${f}_$i.err || { tail -5 $O/b256_f${f}_$i.err; exit 1; }
python -c "import json;r=json.loads(open('$O/b256_f${f}_$i.json').read().strip().splitlines()[-1]);print('bs256 fin3=$f', r['value'], r['ms_per_step'])"
done
done
