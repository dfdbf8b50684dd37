#!/bin/bash
# round 6: VMM-chunked IPC arenas (hipIpcOpenMemHandle hangs above 2 GiB), plane regressions, then full-depth Llama 1-bit
O=gpurun_out/r6l
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ipc_arena_gpu.py > $O/pytest_arena.log 2>&1 || { tail -30 $O/pytest_arena.log; exit 1; }
tail -4 $O/pytest_arena.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_plane_gpu.py tests/test_row_plane_gpu.py tests/test_remote_probe_gpu.py > $O/pytest_plane.log 2>&1 || { tail -30 $O/pytest_plane.log; exit 1; }
tail -2 $O/pytest_plane.log
SKIP_TESTS=1 LLAMA_MODES="onebit:bf16 none:fp32" LLAMA_STEPS=12 bash scripts/runs/gpu_r6_i.sh
