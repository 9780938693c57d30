#!/bin/bash
# Round-5 batch H: the whole GPU test suite, smoke, the default bench line, then the PMC repro on the
# remaining C3 kernel families (stops at the first crash).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05h
mkdir -p $O
cd $R
export TMPDIR=/tmp
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 0) ;; *) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_all.log 2>&1
chk "gpu tests" $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
chk "smoke" $?
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
chk "bench" $?
PMC_CASES="prep:8:4096:4096 qw:4096:4096:4096 gemm_i8:128:4096:4096" bash tools/pmc_repro.sh r05h_pmc_repro
echo "pmc repro rc=$?" >> $O/status.log
exit 0
