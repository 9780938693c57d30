#!/bin/bash
# Round-5 batch C: interleaved A/B of the batched-decode knobs (tools/ab_decode.py), bs=1 streamed
# single rows, C3 hand-off vs statistics launches.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05c
mkdir -p $O
cd $R
export TMPDIR=/tmp
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 0) ;; *) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "int8_statistics or attention" > $O/t_kern.log 2>&1
chk "kernel tests" $?
timeout -k 10 400 python -u -m pytest tests/test_model_7b_gpu.py -x -v --timeout 200 --timeout-method thread -k "decode" > $O/t_7b.log 2>&1
chk "7b-width tests" $?
timeout -k 10 400 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --variants base tpw1:TPW=1 tpw2:TPW=2 \
  specb:SPECB=1 dm2:LIB=scratch/dm2.so dm6:LIB=scratch/dm6.so drm4:LIB=scratch/drm4.so dms3:LIB=scratch/dms3.so \
  nwm8:LIB=scratch/nwm8.so > $O/ab_bs8.jsonl 2> $O/ab_bs8.err
chk "ab bs8" $?
timeout -k 10 300 python -u tools/ab_decode.py --batch 1 --rounds 4 --steps 60 --variants base s1:STREAM=2,HAND_NORM_MIN_M=1 \
  > $O/ab_bs1.jsonl 2> $O/ab_bs1.err
chk "ab bs1" $?
timeout -k 10 300 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --quantize llm.int8 --variants base \
  stats_launches:I8_HANDOFF=False > $O/ab_c3.jsonl 2> $O/ab_c3.err
chk "ab c3" $?
timeout -k 10 300 python -u tools/config_suite.py --only C3,C3-o0,C3-o6x20 --steps 50 > $O/configs.log 2>&1
chk "configs" $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profc3 -o run -- python -u bench.py --decode-only --batch 8 --steps 50 --quantize llm.int8 > $O/profc3.log 2>&1
chk "c3 kernel trace" $?
find $O/profc3 -name "*kernel_stats.csv" -exec cp {} $O/c3_kernel_stats.csv \;
rm -rf $O/profc3
exit 0
