#!/bin/bash
# round 6 batch S: c_fc1 + c_fc2 in one dual pass (llj_gemm_swiglu) and the flash kernel with two K / V
# tiles in flight -- parity, model prefill tests, A/Bs
set -o pipefail
O=gpurun_out/r06s
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "swiglu or w4z or flash or prefill" > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_model_7b_gpu.py tests/test_model_gpu.py -k "prefill or gemm" > $O/tests_model.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --iters 3 --ab-flag GEMM_SWIGLU:4 > $O/ab_swiglu.jsonl 2> $O/ab_swiglu.err || exit $?
for v in product pf1 product2 pf1b; do
  case $v in product*) unset LLJ_LIB;; *) export LLJ_LIB=scratch/flash_pf1.so;; esac
  timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 4 > $O/prefill_$v.jsonl 2> $O/prefill_$v.err || exit $?
done
