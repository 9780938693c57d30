#!/bin/bash
# round 6 batch W: schedule knobs of the fragment-double-buffered GEMM (VALU per MFMA 1 / 2 / 3, the
# interleave off, one fragment read per MFMA) -- 7B windows, product run twice
set -o pipefail
O=gpurun_out/r06w
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "w4z or swiglu_dual" > $O/tests.log 2>&1 || exit $?
for v in product vpm3 vpm1 ds1 noiglp product2; do
  case $v in product*) unset LLJ_LIB;; *) export LLJ_LIB=scratch/f_$v.so;; esac
  timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 4 > $O/prefill_$v.jsonl 2> $O/prefill_$v.err || exit $?
done
