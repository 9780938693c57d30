#!/bin/bash
# round 6 batch O: the QKV GEMM epilogue with the row / column index math hoisted (no divisions per
# element) -- GEMM parity tests incl. every QKV epilogue, prefill model tests, then the windows
set -o pipefail
O=gpurun_out/r06o
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "gemm or flash or prefill" > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_model_7b_gpu.py tests/test_model_gpu.py -k "prefill or gemm" > $O/tests_model.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --iters 3 --ab-w4z 4 > $O/ab_w4z.jsonl 2> $O/ab_w4z.err || exit $?
timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 3 > $O/prefill.jsonl 2> $O/prefill.err || exit $?
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/r06o_prof -o w4z -- python3 $GRAFT_REPO_ROOT/tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/kstats_db.py /tmp/r06o_prof > $O/prefill_kernel_stats.csv 2> $O/kstats.log
LLJ_LIB=scratch/flash_slow.so timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 3 > $O/prefill_flash_slow.jsonl 2> $O/prefill_flash_slow.err || exit $?
timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 3 > $O/prefill2.jsonl 2> $O/prefill2.err || exit $?
