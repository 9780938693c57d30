#!/bin/bash
# round 6 batch A: new robustness / split hand-off tests, the full GPU suite, the bench line with C1 / C3 legs
set -o pipefail
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "stale_outlier or handoff_split" > $O/t_new.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
