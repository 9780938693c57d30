#!/bin/bash
# round 6 batch K: the convert-once int4 prefill GEMM (LLJ_WF_ZINT) -- its parity tests, the GEMM /
# prefill model tests, then an interleaved A/B of the 7B 2048-token window and a kernel trace
set -o pipefail
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "w4z or gemm_glds or gemm_linear_and_resid or gemm_swiglu or gemm_qkv" > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_model_7b_gpu.py tests/test_model_gpu.py -k "prefill or gemm" > $O/tests_model.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/prefill_bench.py --T 2048 --iters 3 --ab-w4z 5 > $O/ab_w4z.jsonl 2> $O/ab_w4z.err || exit $?
timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 3 > $O/prefill.jsonl 2> $O/prefill.err || exit $?
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/r06k_prof -o w4z -- python3 $GRAFT_REPO_ROOT/tools/prefill_bench.py --T 2048 --modes gptq.int4 --iters 2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/kstats_db.py /tmp/r06k_prof > $O/w4z_kernel_stats.csv 2> $O/kstats.log
