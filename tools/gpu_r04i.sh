#!/bin/bash
# Round-4 batch I: LDS-DMA tile-shape cost A/B on the 7B bf16 window, smoke(), the default bench
# line, and the rocprofv3 kernel-trace summary of that same bench command (profiles/).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04i
mkdir -p $O
cd $R
chk() {
  echo "$1 rc=$2" >> $O/status.log
  case $2 in 124|134|137|139|-6|-11) echo "stopping after $1" >> $O/status.log; exit $2;; esac
}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_7b_gpu.py -k "gemm or prefill" -q --timeout 150 --timeout-method thread > $O/t_gemm.log 2>&1
chk "gemm+prefill tests" $?
for cfg in "LLJ_GLDS_COST128=55" "LLJ_GLDS_COST128=70" "LLJ_GLDS_COST128=85" "LLJ_GLDS_COST128=55"; do
  echo "== $cfg" >> $O/prefill_bench.log
  env $cfg timeout -k 10 200 python -u tools/prefill_bench.py --T 2048 --modes none gptq.int4 --iters 5 >> $O/prefill_bench.log 2>&1
  chk "prefill bench $cfg" $?
done
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
chk smoke $?
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
chk bench $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/bt -o bench -- python3 $R/bench.py > $O/bench_prof.log 2>&1
chk "bench trace" $?
find /tmp/bt -name "*kernel_stats.csv" -exec cp {} $O/bench_kernel_stats.csv \;
exit 0
