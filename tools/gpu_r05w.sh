#!/bin/bash
# Round-5 batch W: streamed int8 workspace rows (AM_I8S) for the norm-fed int8 GEMVs: int8 tests,
# C3 A/B against the LDS image (scratch/noi8s.so), C3 regimes, C3 trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05w
mkdir -p $O
cd $R
export TMPDIR=/tmp
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 0) ;; *) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "int8 or i8 or stat" > $O/t_kern.log 2>&1
chk "kernel tests" $?
timeout -k 10 400 python -u -m pytest tests/test_model_7b_gpu.py tests/test_model_gpu.py tests/test_fulldepth_gpu.py -x -q --timeout 250 --timeout-method thread -k "int8" > $O/t_model.log 2>&1
chk "model tests" $?
timeout -k 10 300 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --quantize llm.int8 --variants \
  i8s noi8s:LIB=scratch/noi8s.so > $O/ab_c3.jsonl 2> $O/ab_c3.err
chk "ab c3" $?
timeout -k 10 300 python -u tools/config_suite.py --only C3,C3-o0,C3-o6x20 --steps 50 > $O/configs.log 2>&1
chk "configs" $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profc3 -o run -- \
  python -u bench.py --decode-only --batch 8 --steps 20 --quantize llm.int8 > $O/profc3.log 2>&1
chk "trace c3" $?
exit 0
