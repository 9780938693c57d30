#!/bin/bash
# round 6 batch AG: tile order of the LDS-DMA GEMMs -- n-fastest for the convert-once int4 (product) vs
# m-fastest (mfast), and n-fastest for bf16 too (nfastbf); parity of the int4 GEMMs, then the windows
set -o pipefail
O=gpurun_out/r06ag
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "w4z or swiglu_dual or split_k" > $O/tests.log 2>&1 || exit $?
for v in product mfast nfastbf product2 mfast2 nfastbf2; do
  case $v in product*) unset LLJ_LIB;; mfast*) export LLJ_LIB=scratch/mfast.so;; *) export LLJ_LIB=scratch/nfastbf.so;; esac
  timeout -k 10 200 python -u tools/prefill_bench.py --T 512 2048 --modes gptq.int4 none --iters 4 > $O/prefill_$v.jsonl 2> $O/prefill_$v.err || exit $?
done
