#!/bin/bash
# Round-4 batch H: the whole GPU test suite, then the 7B prefill windows under a kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04h
mkdir -p $O
cd $R
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 840 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider > $O/t_all.log 2>&1
chk "gpu tests" $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pf -o prefill -- python3 $R/tools/prefill_bench.py --T 2048 --modes none gptq.int4 --iters 3 > $O/prefill_trace.log 2>&1
chk "prefill trace" $?
find /tmp/pf -name "*kernel_stats.csv" -exec cp {} $O/prefill_kernel_stats.csv \;
exit 0
