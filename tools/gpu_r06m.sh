#!/bin/bash
# round 6 batch M: convert-once int4 GEMM, conversion interleaved with the MFMAs (8 waves, codes read
# before the fragments, sched_group_barrier 1 MFMA : 3 VALU) and variants, each in an interleaved
# A/B against the default int4 kernel (LLJ_OPT_GEMM_W4Z 1 / 0) in one process
set -o pipefail
O=gpurun_out/r06m
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "w4z or gemm_glds_qkv" > $O/tests.log 2>&1 || exit $?
for v in product noiglp w4after prio; do
  if [ $v = product ]; then unset LLJ_LIB; else export LLJ_LIB=scratch/w4z_$v.so; fi
  timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --iters 3 --ab-w4z 4 > $O/ab_$v.jsonl 2> $O/ab_$v.err || exit $?
done
