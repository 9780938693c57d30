#!/bin/bash
# round 6 batch X: VALU-per-MFMA 1 vs 2 (product) repeated, then a kernel trace of the product's windows
set -o pipefail
O=gpurun_out/r06x
mkdir -p $O
for v in product vpm1 product2 vpm1b product3 vpm1c; do
  case $v in product*) unset LLJ_LIB;; *) export LLJ_LIB=scratch/f_vpm1.so;; esac
  timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes gptq.int4 --iters 4 > $O/prefill_$v.jsonl 2> $O/prefill_$v.err || exit $?
done
unset LLJ_LIB
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/r06x_prof -o pf -- python3 $GRAFT_REPO_ROOT/tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/kstats_db.py /tmp/r06x_prof > $O/prefill_kernel_stats.csv 2> $O/kstats.log
