#!/bin/bash
# Round-3 closing GPU batch: int4 GEMM variant A/B (prefill window), the whole GPU suite and smoke().
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 > gpurun_out/pf_f_base.jsonl 2>&1 &&
LLJ_LIB=scratch/w4d1.so timeout -k 10 150 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 > gpurun_out/pf_f_w4d1.jsonl 2>&1 &&
LLJ_LIB=scratch/w4mf.so timeout -k 10 150 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 > gpurun_out/pf_f_w4mf.jsonl 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/t_f_all.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_f.log 2>&1
