#!/bin/bash
# round 6 batch Q: flash prefill with 8 waves (128 queries) per workgroup vs 4, conversion interleave at
# 2 VALU per MFMA as the product default; flash / prefill parity, then the windows
set -o pipefail
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "flash or prefill or w4z" > $O/tests.log 2>&1 || exit $?
LLJ_LIB=scratch/flash_nwq8.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "flash or prefill" > $O/tests_nwq8.log 2>&1 || exit $?
for v in product nwq8 product2 nwq8b; do
  case $v in product*) unset LLJ_LIB;; *) export LLJ_LIB=scratch/flash_nwq8.so;; esac
  timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 4 > $O/prefill_$v.jsonl 2> $O/prefill_$v.err || exit $?
done
