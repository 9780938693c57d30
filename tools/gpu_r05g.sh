#!/bin/bash
# Round-5 batch G: counters (bs=8 int4, C3 GEMVs only: the full C3 pass crashes rocprofv3, bs=1),
# kernel traces of the bs=8 and bs=1 decode graphs.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05g
mkdir -p $O
cd $R
export TMPDIR=/tmp
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 0) ;; *) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
for b in 8 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$b -o run -- python -u bench.py --decode-only --batch $b --steps 50 > $O/prof$b.log 2>&1
  chk "bs$b kernel trace" $?
  find $O/prof$b -name "*kernel_stats.csv" -exec cp {} $O/bs${b}_graph_kernel_stats.csv \;
  rm -rf $O/prof$b
done
PMC_PASSES="bs8 bs1" bash tools/profile_r05.sh r05g_pmc > $O/pmc.log 2>&1
chk "pmc bs8 bs1" $?
PMC_PASSES="c3" PMC_REGEX="gemv_kernel" bash tools/profile_r05.sh r05g_pmc_c3 > $O/pmc_c3.log 2>&1
chk "pmc c3 gemv" $?
exit 0
