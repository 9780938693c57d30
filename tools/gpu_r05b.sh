#!/bin/bash
# Round-5 batch B: int8 hand-off + full-depth + batch-12 tests, C3 / bs8 decode-only, kernel traces,
# then the PMC counter passes (tools/profile_r05.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05b
mkdir -p $O
cd $R
export TMPDIR=/tmp
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 0) ;; *) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 400 python -u -m pytest tests/test_fulldepth_gpu.py tests/test_model_gpu.py -x -v -s --timeout 300 --timeout-method thread -k "full_depth or batch or int8" > $O/t_model.log 2>&1
chk "model tests" $?
timeout -k 10 300 python -u tools/config_suite.py --only C2-bs8,C3,C3-o0,C3-o6x20 --steps 50 > $O/configs.log 2>&1
chk "configs" $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof8 -o run -- python -u bench.py --decode-only --batch 8 --steps 50 > $O/prof8.log 2>&1
chk "bs8 kernel trace" $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profc3 -o run -- python -u bench.py --decode-only --batch 8 --steps 50 --quantize llm.int8 > $O/profc3.log 2>&1
chk "c3 kernel trace" $?
find $O/prof8 -name "*kernel_stats.csv" -exec cp {} $O/bs8_kernel_stats.csv \;
find $O/profc3 -name "*kernel_stats.csv" -exec cp {} $O/c3_kernel_stats.csv \;
rm -rf $O/prof8 $O/profc3
bash tools/profile_r05.sh r05b_pmc > $O/pmc.log 2>&1
echo "pmc rc=$?" >> $O/status.log
exit 0
