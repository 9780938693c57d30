#!/bin/bash
# Round-5 batch O: row-sum branch restored; SIS with 2 entries; A/B of the load fence (bs=8 int4,
# bs=1, C3); per-workgroup phase traces of the llm.int8 bs=8 GEMVs with and without the in-stream
# side loop (trace builds, scratch/trace*.so); tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05o
mkdir -p $O
cd $R
export TMPDIR=/tmp
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 0) ;; *) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t_kern.log 2>&1
chk "kernel tests" $?
timeout -k 10 400 python -u -m pytest tests/test_model_7b_gpu.py tests/test_model_gpu.py tests/test_fulldepth_gpu.py -x -q --timeout 250 --timeout-method thread > $O/t_model.log 2>&1
chk "model tests" $?
timeout -k 10 300 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --variants new fence:LIB=scratch/fence.so \
  > $O/ab_bs8.jsonl 2> $O/ab_bs8.err
chk "ab bs8" $?
timeout -k 10 300 python -u tools/ab_decode.py --batch 8 --rounds 3 --steps 50 --quantize llm.int8 --variants \
  new fence:LIB=scratch/fence.so > $O/ab_c3.jsonl 2> $O/ab_c3.err
chk "ab c3" $?
timeout -k 10 300 python -u tools/ab_decode.py --batch 1 --rounds 3 --steps 60 --variants new fence:LIB=scratch/fence.so \
  > $O/ab_bs1.jsonl 2> $O/ab_bs1.err
chk "ab bs1" $?
cd lit-llama-ja_amd
timeout -k 10 200 python -u ../tools/phase_trace.py --quantize llm.int8 --batch 8 --lib scratch/trace.so > $O/phase_c3.log 2>&1
chk "phase c3" $?
timeout -k 10 200 python -u ../tools/phase_trace.py --quantize llm.int8 --batch 8 --lib scratch/trace_sidel.so > $O/phase_c3_sidel.log 2>&1
chk "phase c3 sidel" $?
exit 0
