#!/bin/bash
# Round-4 batch O: A/B of the QKV epilogue ring-wrap change (scratch/old.so = before) at bs=8 and bs=1,
# interleaved, plus an in-graph kernel trace of the new build at bs=8.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04o
mkdir -p $O
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
cd $R
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = new ]; then unset LLJ_LIB; else export LLJ_LIB=$R/scratch/old.so; fi
    timeout -k 10 150 python3 bench.py --decode-only --batch 8 --steps 300 --warmup 20 > $O/bs8_${v}_$rep.log 2>&1
    chk "bs8 $v $rep" $?
    timeout -k 10 150 python3 bench.py --decode-only --steps 300 --warmup 20 > $O/bs1_${v}_$rep.log 2>&1
    chk "bs1 $v $rep" $?
  done
done
unset LLJ_LIB
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/o_new -o new -- python3 $R/bench.py --decode-only --batch 8 --steps 100 --warmup 10 > $O/trace.log 2>&1
chk trace $?
find /tmp/o_new -name "*kernel_stats.csv" -exec cp {} $O/new_kernel_stats.csv \;
exit 0
