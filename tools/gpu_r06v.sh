#!/bin/bash
# round 6 batch V: fragment double buffering in the LDS-DMA GEMM (chunk t + 1's fragments read during chunk
# t's MFMAs) -- GEMM parity, prefill model tests, windows against the FDB=0 build (alternating processes)
set -o pipefail
O=gpurun_out/r06v
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "gemm or w4z or swiglu" > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_model_7b_gpu.py tests/test_model_gpu.py -k "prefill or gemm" > $O/tests_model.log 2>&1 || exit $?
for v in product fdb0 product2 fdb0b; do
  case $v in product*) unset LLJ_LIB;; *) export LLJ_LIB=scratch/fdb0.so;; esac
  timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 4 > $O/prefill_$v.jsonl 2> $O/prefill_$v.err || exit $?
done
