#!/bin/bash
# Round-5 batch E: LLM.int8 decode fully streamed (norm rows' hand-off blocks): kernel + 7B-width +
# full-depth tests, C3 in three regimes, C3 kernel trace; bs=8 phase stamps (trace build); then batch
# D's A/B (depths, 256-thread attention, batch speculative pass, int8 depth) and the PMC repro bisect.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05e
mkdir -p $O
cd $R
export TMPDIR=/tmp
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 0) ;; *) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "int8" > $O/t_kern.log 2>&1
chk "kernel tests" $?
timeout -k 10 400 python -u -m pytest tests/test_model_7b_gpu.py tests/test_model_gpu.py -x -v --timeout 200 --timeout-method thread -k "int8" > $O/t_model.log 2>&1
chk "model tests" $?
timeout -k 10 300 python -u -m pytest tests/test_fulldepth_gpu.py -x -v -s --timeout 250 --timeout-method thread -k "int8" > $O/t_full.log 2>&1
chk "full depth" $?
timeout -k 10 300 python -u tools/config_suite.py --only C3,C3-o0,C3-o6x20 --steps 50 > $O/configs.log 2>&1
chk "configs" $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profc3 -o run -- python -u bench.py --decode-only --batch 8 --steps 50 --quantize llm.int8 > $O/profc3.log 2>&1
chk "c3 kernel trace" $?
find $O/profc3 -name "*kernel_stats.csv" -exec cp {} $O/c3_kernel_stats.csv \;
rm -rf $O/profc3
timeout -k 10 240 python -u tools/phase_trace.py --batch 8 > $O/trace_bs8.log 2>&1
chk "trace bs8" $?
cp gpurun_out/phase_trace_bs8.json $O/
timeout -k 10 400 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --variants base drm3:LIB=scratch/drm3.so \
  drm2:LIB=scratch/drm2.so dm3:LIB=scratch/dm3.so att256:LIB=scratch/att256.so specb:SPECB=1 \
  att256specb:LIB=scratch/att256.so,SPECB=1 > $O/ab_bs8.jsonl 2> $O/ab_bs8.err
chk "ab bs8" $?
timeout -k 10 300 python -u tools/ab_decode.py --batch 1 --rounds 3 --steps 60 --variants base att256:LIB=scratch/att256.so \
  > $O/ab_bs1.jsonl 2> $O/ab_bs1.err
chk "ab bs1" $?
timeout -k 10 300 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --quantize llm.int8 --variants base \
  di8q3:LIB=scratch/di8q3.so > $O/ab_c3.jsonl 2> $O/ab_c3.err
chk "ab c3" $?
PMC_CASES="w4:8:4096:4096 i8q:8:4096:4096 i8q:8:4096:11008 i8swiglu:8:11008:4096 i8:8:4096:4096" bash tools/pmc_repro.sh r05d_pmc_repro
echo "pmc repro rc=$?" >> $O/status.log
exit 0
