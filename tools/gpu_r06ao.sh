#!/bin/bash
# round 6 batch AO: the dual SwiGLU pass's partial last wave as split-K halves (llj_gemm_swiglu_ws) -- tests,
# the probe (swiglu vs swiglu_ws) and the prefill window against scratch/tail0.so (LLJ_GEMM_SWIGLU_TAIL=0)
set -o pipefail
O=gpurun_out/r06ao
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py -k "swiglu or w4z or split_k or prefill" > $O/tests.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 100 python -u tools/gemm_epi_probe.py > $O/probe_$r.json || exit $?
done
for r in 1 2; do
  timeout -k 10 150 python -u tools/prefill_bench.py --T 512 1024 2048 --modes gptq.int4 --iters 4 > $O/prefill_tail_$r.jsonl 2>> $O/prefill.err || exit $?
  LLJ_LIB=scratch/tail0.so timeout -k 10 150 python -u tools/prefill_bench.py --T 512 1024 2048 --modes gptq.int4 --iters 4 > $O/prefill_old_$r.jsonl 2>> $O/prefill.err || exit $?
done
