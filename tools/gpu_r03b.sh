#!/bin/bash
# Round-3 (second session) GPU batch: new kernels' parity, the int8 side-product regimes, the
# decode-attention A/B and the prefill GEMM prefetch-depth A/B. Each step under its own limit;
# the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "i8 or int8 or attention_decode" > gpurun_out/t_i8.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_model_7b_gpu.py \
  -k "prefill or int8" > gpurun_out/t_7bp.log 2>&1 &&
timeout -k 10 200 python -u tools/i8_bench.py > gpurun_out/i8_bench.jsonl 2>&1 &&
timeout -k 10 300 python -u tools/ab_decode.py --variants old:ATTN_DEC=0 dec8:ATTN_DEC=1 dec4:ATTN_DEC=1,ATTN_DEC_SPLIT=4 \
  dec2:ATTN_DEC=1,ATTN_DEC_SPLIT=2 --batch 1 \
  > gpurun_out/ab_att2.jsonl 2> gpurun_out/ab_att2.log &&
timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 none llm.int8 > gpurun_out/pf_base.jsonl 2>&1 &&
LLJ_LIB=scratch/gd2.so timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes none llm.int8 > gpurun_out/pf_gd2.jsonl 2>&1 &&
LLJ_LIB=scratch/gd2w3.so timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 > gpurun_out/pf_gd2w3.jsonl 2>&1 &&
LLJ_LIB=scratch/bm256d2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "gemm and not i8" > gpurun_out/t_bm256.log 2>&1 &&
LLJ_LIB=scratch/bm256.so timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes none > gpurun_out/pf_bm256.jsonl 2>&1 &&
LLJ_LIB=scratch/bm256d2.so timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes none > gpurun_out/pf_bm256d2.jsonl 2>&1
