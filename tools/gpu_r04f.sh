#!/bin/bash
# Round-4 batch F: every BASELINE config (C3 in its three outlier regimes) and the bs=8 / C3 decode
# graphs under --kernel-trace --stats (in-graph kernel times; --pmc passes over the multi-row GEMVs
# end in a host SIGSEGV inside hipLaunchKernel).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04f
mkdir -p $O
cd $R
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 600 python -u tools/config_suite.py --out $O/configs.json > $O/configs.log 2>&1
chk "config suite" $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/t8 -o bs8 -- python3 $R/bench.py --decode-only --batch 8 --steps 100 --warmup 10 > $O/bs8_trace.log 2>&1
chk "bs8 trace" $?
find /tmp/t8 -name "*kernel_stats.csv" -exec cp {} $O/bs8_kernel_stats.csv \;
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/tc3 -o c3 -- python3 $R/bench.py --decode-only --quantize llm.int8 --batch 8 --steps 50 --warmup 5 > $O/c3_trace.log 2>&1
chk "c3 trace" $?
find /tmp/tc3 -name "*kernel_stats.csv" -exec cp {} $O/c3_kernel_stats.csv \;
exit 0
