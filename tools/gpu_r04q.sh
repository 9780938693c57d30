#!/bin/bash
# Round-4 batch Q (final tree, decode attention 512 x 4): whole GPU suite, smoke(), the default bench
# line, the config suite, and kernel traces of the default bench and of the bs=1 decode graph alone.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04q
mkdir -p $O
cd $R
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 840 python -u -m pytest tests -m gpu -q --timeout 280 --timeout-method thread -p no:cacheprovider > $O/t_all.log 2>&1
chk "gpu tests" $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
chk smoke $?
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
chk bench $?
timeout -k 10 600 python -u tools/config_suite.py --out $O/configs.json > $O/configs.log 2>&1
chk configs $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/gt -o graph -- python3 $R/bench.py --decode-only --steps 100 --warmup 10 > $O/graph_prof.log 2>&1
chk "graph trace" $?
find /tmp/gt -name "*kernel_stats.csv" -exec cp {} $O/graph_kernel_stats.csv \;
timeout -s KILL 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/bt -o bench -- python3 $R/bench.py > $O/bench_prof.log 2>&1
chk "bench trace" $?
find /tmp/bt -name "*kernel_stats.csv" -exec cp {} $O/bench_kernel_stats.csv \;
exit 0
