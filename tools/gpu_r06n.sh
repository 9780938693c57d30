#!/bin/bash
# round 6 batch N: the convert-once int4 GEMM's interleave ratio (VALU per MFMA 2 / 3 / 4 / 6), each an
# interleaved A/B against the default int4 kernel in one process, then a kernel trace of the product
set -o pipefail
O=gpurun_out/r06n
mkdir -p $O
for v in product vpm2 vpm4 vpm6; do
  if [ $v = product ]; then unset LLJ_LIB; else export LLJ_LIB=scratch/w4z_$v.so; fi
  timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --iters 3 --ab-w4z 4 > $O/ab_$v.jsonl 2> $O/ab_$v.err || exit $?
done
unset LLJ_LIB
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/r06n_prof -o w4z -- python3 $GRAFT_REPO_ROOT/tools/prefill_bench.py --T 2048 --modes gptq.int4 none --iters 2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
python3 tools/kstats_db.py /tmp/r06n_prof > $O/prefill_kernel_stats.csv 2> $O/kstats.log
