export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out/pe
for v in 0; do timeout -k 10 120 python scripts/probe_dgrad_epi.py >> gpurun_out/pe/probe.jsonl 2>gpurun_out/pe/err_$v.log || exit $?; done
cat gpurun_out/pe/probe.jsonl
