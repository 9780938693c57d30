#!/bin/bash
# Round-4 batch S: RMSNorm row launch with 512-thread blocks (LLJ_NORM_NT=512) vs 256: parity (norm
# kernels + batched decode models), bs=8 decode-only tok/s interleaved, in-graph trace of the 512 form.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04s
mkdir -p $O
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
cd $R
LLJ_NORM_NT=512 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_7b_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "norm or batch or decode or prefill" > $O/t_512.log 2>&1
chk "tests 512" $?
for rep in 1 2 3; do
  for nt in 256 512; do
    LLJ_NORM_NT=$nt timeout -k 10 150 python3 bench.py --decode-only --batch 8 --steps 300 --warmup 20 > $O/bs8_${nt}_$rep.log 2>&1
    chk "bs8 $nt $rep" $?
  done
done
cd /tmp && export TMPDIR=/tmp
LLJ_NORM_NT=512 timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/s512 -o s512 -- python3 $R/bench.py --decode-only --batch 8 --steps 100 --warmup 10 > $O/trace.log 2>&1
chk trace $?
find /tmp/s512 -name "*kernel_stats.csv" -exec cp {} $O/s512_kernel_stats.csv \;
exit 0
