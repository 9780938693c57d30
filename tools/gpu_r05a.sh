#!/bin/bash
# Round-5 batch A: baseline phase stamps (old-tree trace build), streamed-A GEMV tests, 7B-width
# model tests, decode-only bs=8 / bs=1 and a kernel trace of the bs=8 decode graph.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05a
mkdir -p $O
cd $R
export TMPDIR=/tmp
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 0) ;; *) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "streamed or handoff or multi_tile or fused or generic_int8" > $O/t_kern.log 2>&1
chk "kernel tests" $?
timeout -k 10 300 python -u -m pytest tests/test_fp32_gpu.py tests/test_generic_gpu.py -x -v --timeout 200 --timeout-method thread > $O/t_fp32.log 2>&1
chk "fp32 + generic tests" $?
timeout -k 10 400 python -u -m pytest tests/test_model_7b_gpu.py -x -v --timeout 200 --timeout-method thread > $O/t_7b.log 2>&1
chk "7b tests" $?
timeout -k 10 200 python -u bench.py --decode-only --batch 8 --steps 50 > $O/bs8.log 2>&1
chk "bs8 decode-only" $?
timeout -k 10 200 python -u bench.py --decode-only --batch 1 --steps 50 > $O/bs1.log 2>&1
chk "bs1 decode-only" $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8 -o run -- python -u bench.py --decode-only --batch 8 --steps 50 > $O/prof8.log 2>&1
chk "bs8 kernel trace" $?
find $O/prof8 -name "*kernel_stats.csv" -exec cp {} $O/bs8_kernel_stats.csv \;
rm -rf $O/prof8
exit 0
