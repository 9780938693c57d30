#!/bin/bash
# round 6 batch P: cheaper exact conversion (packed fp32 subtract + v_cvt_pk_bf16_f32) in the
# convert-once int4 GEMM -- its parity tests, then interleaved A/Bs (product, 2 VALU per MFMA)
set -o pipefail
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "w4z or gemm_glds_qkv" > $O/tests.log 2>&1 || exit $?
for v in product vpm2; do
  if [ $v = product ]; then unset LLJ_LIB; else export LLJ_LIB=scratch/w4z_$v.so; fi
  timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --iters 3 --ab-w4z 4 > $O/ab_$v.jsonl 2> $O/ab_$v.err || exit $?
done
