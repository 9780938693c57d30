#!/bin/bash
# round 6 batch AM: store / residual / SwiGLU epilogues through LDS -- GEMM and prefill tests, the epilogue
# probe and the prefill window against the previous epilogues (scratch/epi0.so, LLJ_GLDS_LDS_EPI=0), interleaved
set -o pipefail
O=gpurun_out/r06am
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_model_gpu.py -k "gemm or prefill" > $O/tests.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 100 python -u tools/gemm_epi_probe.py > $O/probe_lds_$r.json || exit $?
  LLJ_LIB=scratch/epi0.so timeout -k 10 100 python -u tools/gemm_epi_probe.py > $O/probe_old_$r.json || exit $?
done
for r in 1 2; do
  timeout -k 10 150 python -u tools/prefill_bench.py --T 512 2048 --modes gptq.int4 none --iters 4 > $O/prefill_lds_$r.jsonl 2>> $O/prefill.err || exit $?
  LLJ_LIB=scratch/epi0.so timeout -k 10 150 python -u tools/prefill_bench.py --T 512 2048 --modes gptq.int4 none --iters 4 > $O/prefill_old_$r.jsonl 2>> $O/prefill.err || exit $?
done
