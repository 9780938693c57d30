#!/bin/bash
# Round-4 batch AD (batched SwiGLU with 2 chunks in flight): whole GPU suite, smoke(), the default
# bench line and the config suite (C3's int8 SwiGLU shares the setting).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04ad
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
exit 0
