#!/bin/bash
# Final tree: full GPU suite + smoke (the driver's round-end tiers).
O=gpurun_out/r4final7
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/full.log 2>&1 || { tail -30 $O/full.log; exit 1; }
tail -2 $O/full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
