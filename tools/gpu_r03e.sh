#!/bin/bash
# Round-3 final GPU batch: int8 parity after the speculative-entry choice, all BASELINE configs,
# the bench line, prefill MFMA busy, and the kernel trace of the bench.
set -o pipefail
mkdir -p gpurun_out/r03e
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "int8 or i8" > gpurun_out/t_e_kern.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_model_7b_gpu.py \
  -k "int8" > gpurun_out/t_e_7b.log 2>&1 &&
timeout -k 10 400 python -u tools/config_suite.py --out gpurun_out/r03e/configs.json > gpurun_out/r03e/configs.log 2>&1 &&
timeout -k 10 240 python -u bench.py > gpurun_out/r03e/bench.json 2> gpurun_out/r03e/bench.err &&
timeout -k 10 200 bash tools/profile_prefill_mfma.sh r03_prefill_mfma "gptq.int4 none llm.int8" > gpurun_out/pf_mfma.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03e -o trace \
  -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r03e/bench_trace.log 2>&1
