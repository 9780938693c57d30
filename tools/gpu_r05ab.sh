#!/bin/bash
# Round-5 batch AB (final): full GPU suite, smoke, default bench line, C3 regimes and kernel traces
# (bs=8 int4, C3) of the round-5 end state.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ab
mkdir -p $O
cd $R
export TMPDIR=/tmp
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 0) ;; *) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t_all.log 2>&1
chk "gpu tests" $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
chk "smoke" $?
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
chk "bench" $?
timeout -k 10 300 python -u tools/config_suite.py --only C3,C3-o0,C3-o6x20 --steps 50 > $O/configs.log 2>&1
chk "configs" $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profc3 -o run -- \
  python -u bench.py --decode-only --batch 8 --steps 20 --quantize llm.int8 > $O/profc3.log 2>&1
chk "trace c3" $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof8 -o run -- \
  python -u bench.py --decode-only --batch 8 --steps 20 > $O/prof8.log 2>&1
chk "trace bs8" $?
exit 0
