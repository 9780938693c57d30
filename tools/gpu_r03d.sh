#!/bin/bash
# Round-3 GPU batch 4: LLM.int8 GEMM with pre-gathered outlier matrices (parity), int8 side-product
# speculative-entry A/B (GEMV regimes + C3 model step, one box), LLM.int8 decode counters, prefill
# windows and MFMA busy with the 256-row tiles and the int8 GEMM.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm_i8 or i8_stats" > gpurun_out/t_d_kern.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_model_7b_gpu.py \
  -k "prefill" > gpurun_out/t_d_7b.log 2>&1 &&
timeout -k 10 200 python -u tools/prefill_bench.py --T 512 2048 --modes llm.int8 none gptq.int4 > gpurun_out/pf_d_base.jsonl 2>&1 &&
LLJ_LIB=scratch/d3.so timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes none llm.int8 > gpurun_out/pf_d3.jsonl 2>&1 &&
timeout -k 10 150 python -u tools/i8_bench.py > gpurun_out/i8_d_main.jsonl 2>&1 &&
LLJ_LIB=scratch/spe1.so timeout -k 10 150 python -u tools/i8_bench.py > gpurun_out/i8_d_spe1.jsonl 2>&1 &&
timeout -k 10 200 python -u tools/config_suite.py --only C3 --out gpurun_out/c3_main.json > gpurun_out/c3_main.log 2>&1 &&
LLJ_LIB=scratch/spe1.so timeout -k 10 200 python -u tools/config_suite.py --only C3 --out gpurun_out/c3_spe1.json > gpurun_out/c3_spe1.log 2>&1 &&
timeout -k 10 300 bash tools/profile_c3.sh r03_c3_pmc > gpurun_out/c3_pmc.log 2>&1 &&
timeout -k 10 200 bash tools/profile_prefill_mfma.sh r03_prefill_mfma "gptq.int4 none llm.int8" > gpurun_out/pf_mfma.log 2>&1
