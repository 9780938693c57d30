#!/bin/bash
# round 6 batch AI: grouped tile order (2 / 4 row tiles per group) of the LDS-DMA GEMMs vs the product
# (int4 n-fastest, bf16 m-fastest), 7B windows
set -o pipefail
O=gpurun_out/r06ai
mkdir -p $O
for v in product g2 g4 product2 g2b g4b; do
  case $v in product*) unset LLJ_LIB;; g2*) export LLJ_LIB=scratch/g2.so;; *) export LLJ_LIB=scratch/g4.so;; esac
  timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 4 > $O/prefill_$v.jsonl 2> $O/prefill_$v.err || exit $?
done
