#!/bin/bash
# round 6 batch AA: flash prefill with two 16-query blocks per wave (LLJ_FLASH_QB=2) on the final build
set -o pipefail
O=gpurun_out/r06aa
mkdir -p $O
for v in qb1 qb2 qb1b qb2b; do
  case $v in qb1*) unset LLJ_FLASH_QB;; *) export LLJ_FLASH_QB=2;; esac
  timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 --iters 4 > $O/prefill_$v.jsonl 2> $O/prefill_$v.err || exit $?
done
