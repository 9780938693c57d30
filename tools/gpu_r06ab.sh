#!/bin/bash
# round 6 batch AB: split-K residual GEMMs for few row tiles -- parity, prefill model tests, windows at
# T = 512 / 1024 / 2048 against the unsplit build (LLJ_GEMM_SPLITK=0 variant, alternating processes)
set -o pipefail
O=gpurun_out/r06ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "split_k or w4z or gemm_glds" > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_model_7b_gpu.py tests/test_model_gpu.py -k "prefill or gemm" > $O/tests_model.log 2>&1 || exit $?
for v in product nosplit product2 nosplit2; do
  case $v in product*) unset LLJ_LIB;; *) export LLJ_LIB=scratch/nosplit.so;; esac
  timeout -k 10 200 python -u tools/prefill_bench.py --T 512 1024 2048 --modes gptq.int4 none --iters 4 > $O/prefill_$v.jsonl 2> $O/prefill_$v.err || exit $?
done
