#!/bin/bash
# round 6 batch Z: short-K / odd chunk-count cases of the fragment-double-buffered GEMMs
set -o pipefail
O=gpurun_out/r06z
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "w4z or swiglu_dual or gemm_glds_tiles" > $O/tests.log 2>&1 || exit $?
