#!/bin/bash
# round 6 batch L: convert-once int4 GEMM with the conversion on waves 0-3 (before / after their MFMAs)
set -o pipefail
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "w4z or gemm_glds_qkv" > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/prefill_bench.py --T 2048 --iters 3 --ab-w4z 5 > $O/ab_w4z.jsonl 2> $O/ab_w4z.err || exit $?
LLJ_LIB=scratch/w4zafter.so timeout -k 10 300 python -u tools/prefill_bench.py --T 2048 --iters 3 --ab-w4z 5 > $O/ab_w4z_after.jsonl 2> $O/ab_w4z_after.err || exit $?
