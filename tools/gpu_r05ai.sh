#!/bin/bash
# Round-5 batch AI: 7B gptq.int4 2048-token prefill window on the final build: default kernels, the
# LDS-DMA GEMM for every format, and a kernel trace of the default.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ai
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 --iters 3 > $O/default.jsonl 2> $O/default.err
rc=$?; echo "default rc=$rc" >> $O/status.log; [ $rc -eq 0 ] || exit $rc
LLJ_GEMM_GLDS=1 timeout -k 10 300 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 --iters 3 > $O/glds.jsonl 2> $O/glds.err
rc=$?; echo "glds rc=$rc" >> $O/status.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 --iters 2 > $O/prof.log 2>&1
echo "trace rc=$?" >> $O/status.log
exit 0
