#!/bin/bash
# Round-4 batch Y (final tree, one-row SwiGLU with 2 chunks in flight): whole GPU suite, smoke(),
# the default bench line, the config suite, kernel traces of the bs=1 decode graph and the default
# bench, and bs=1 FETCH / WRITE passes (-> gpurun_out/r04y_pmc.json).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04y
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
D=/tmp/r04y
mkdir -p $D
SHORT="--steps 4 --warmup 1 --no-bs8 --no-c4 --no-cpu-baseline --eager --prompt-len 80"
for pass in FETCH_SIZE WRITE_SIZE; do
  tag=bs1_$(echo $pass | tr 'A-Z' 'a-z' | cut -d_ -f1)
  timeout -s KILL 150 rocprofv3 --pmc $pass --output-format csv -d $D -o $tag -- python3 $R/bench.py $SHORT > $D/$tag.log 2>&1
  chk "pmc $pass" $?
done
find $D -mindepth 2 -name "*counter_collection.csv" -exec mv {} $D/ \;
python3 $R/tools/profile_summary.py $D $R/gpurun_out/r04y_pmc.json >> $O/status.log 2>&1
exit 0
