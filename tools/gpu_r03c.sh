#!/bin/bash
# Round-3 GPU batch 3: parity of the 256-row GEMM tiles (bf16 / int8 default, int4 variant) and the
# generalized int8 side-product fast path, then the prefill windows and the int8 GEMV regimes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm or i8 or int8" > gpurun_out/t_c_kern.log 2>&1 &&
LLJ_LIB=scratch/w4bm.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_kernels_gpu.py -k "gemm and not i8" > gpurun_out/t_c_w4bm.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_model_7b_gpu.py \
  -k "prefill or int8" > gpurun_out/t_c_7b.log 2>&1 &&
timeout -k 10 200 python -u tools/i8_bench.py > gpurun_out/i8_bench_c.jsonl 2>&1 &&
timeout -k 10 250 python -u tools/prefill_bench.py --T 512 2048 --modes gptq.int4 none llm.int8 > gpurun_out/pf_c_base.jsonl 2>&1 &&
LLJ_LIB=scratch/w4bm.so timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 > gpurun_out/pf_c_w4bm.jsonl 2>&1 &&
LLJ_LIB=scratch/i8off.so timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes llm.int8 > gpurun_out/pf_c_i8off.jsonl 2>&1
