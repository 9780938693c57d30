#!/bin/bash
# round 6 batch AJ: the convert-once interleave knobs re-checked under the n-fastest tile order
set -o pipefail
O=gpurun_out/r06aj
mkdir -p $O
for v in product vpm2 ds1 vpm0 product2 vpm2b ds1b vpm0b; do
  case $v in product*) unset LLJ_LIB;; vpm2*) export LLJ_LIB=scratch/k_vpm2.so;; ds1*) export LLJ_LIB=scratch/k_ds1.so;; *) export LLJ_LIB=scratch/k_vpm0.so;; esac
  timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 --iters 4 > $O/prefill_$v.jsonl 2> $O/prefill_$v.err || exit $?
done
