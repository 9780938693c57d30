#!/bin/bash
# Counters for the llm.int8 bs=8 decode kernels (C3) through the C++ harness (tools/micro/pmc_repro),
# one kernel shape per rocprofv3 --pmc run -- the full C3 decode under --pmc crashes rocprofv3 (DESIGN.md
# section 8), each entry point alone does not. Tags c3h_<op>_<pass> -> tools/profile_summary.py ->
# gpurun_out/$1.json. A failing pass ends the script (summarized first).
OUT=$1
R=$GRAFT_REPO_ROOT
D=/tmp/$OUT
mkdir -p $D $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B=$R/tools/micro/pmc_repro
SQ="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_ANY,SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,GRBM_GUI_ACTIVE"
summarize() {
  find $D -mindepth 2 -name "*.csv" -exec mv {} $D/ \;
  python3 $R/tools/profile_summary.py $D $R/gpurun_out/$OUT.json
}
# op tag -> harness args (M N K): QKV / lm_head shapes on the workspace GEMV (AM_I8S, store epilogue),
# SwiGLU, attn.c_proj / mlp.c_proj on the hand-off GEMV (AM_I8Q), the norm + statistics launch
CASES=${C3H_CASES:-"qkv:i8:8:12288:4096 head:i8:8:32000:4096 swiglu:i8swiglu:8:11008:4096 cproj:i8q:8:4096:4096 down:i8q:8:4096:11008 prep:prep:8:4096:4096 attn:atti8:8:4096:144"}
for cc in $CASES; do
  IFS=: read tag op m n k <<< "$cc"
  for pass in fetch write sq; do
    case $pass in fetch) c=FETCH_SIZE;; write) c=WRITE_SIZE;; sq) c=$SQ;; esac
    timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $D -o c3h_${tag}_$pass -- $B $op $m $n $k 5 > $D/c3h_${tag}_$pass.log 2>&1
    rc=$?
    echo "c3h_${tag}_$pass rc=$rc" >> $R/gpurun_out/${OUT}_status.log
    case $rc in 0) ;; *) summarize; exit $rc;; esac
  done
done
summarize
exit 0
