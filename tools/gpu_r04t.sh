#!/bin/bash
# Round-4 batch T: the default bench line three times on the final tree (run-to-run spread).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04t
mkdir -p $O
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
cd $R
for rep in 1 2 3; do
  timeout -k 10 400 python -u bench.py > $O/bench_$rep.log 2>&1
  chk "bench $rep" $?
done
exit 0
