#!/bin/bash
# Round-4 batch M: where the bs=8 multi-row GEMVs spend the time they take beyond their bs=1 form
# (rocprofv3 --pmc crashes on them): in-graph kernel traces of bs=8 decode-only runs with the
# GEMV ablation builds (LLJ_ABL 1: no A prologue, 4: minimal epilogue, 7: neither and no compute;
# outputs invalid, timing only) beside the product build.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04m
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
for v in prod abl1 abl4 abl7; do
  if [ $v = prod ]; then unset LLJ_LIB; else export LLJ_LIB=$R/scratch/$v.so; fi
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/m_$v -o $v -- python3 $R/bench.py --decode-only --batch 8 --steps 100 --warmup 10 > $O/$v.log 2>&1
  chk "trace $v" $?
  find /tmp/m_$v -name "*kernel_stats.csv" -exec cp {} $O/${v}_kernel_stats.csv \;
done
exit 0
