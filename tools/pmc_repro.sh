#!/bin/bash
# Bisect the rocprofv3 --pmc crash with tools/micro/pmc_repro (one GEMV entry point per run, no
# Python): each case first without the profiler, then under --pmc FETCH_SIZE. Results appended to
# gpurun_out/$1.log. The first case that crashes ends the script (nothing more runs on the GPU after
# a segfault); order the cases (PMC_CASES="op:M:N:K ...") so the suspects come last.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$1.log
cd /tmp && export TMPDIR=/tmp
B=$R/tools/micro/pmc_repro
CASES=${PMC_CASES:-"w4:8:4096:4096 i8q:8:4096:4096 i8q:8:4096:11008 i8swiglu:8:11008:4096 i8:8:4096:4096"}
for cc in $CASES; do
  c=${cc//:/ }
  timeout -k 5 60 $B $c > /tmp/plain.log 2>&1
  p=$?
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pmcr -o r -- $B $c > /tmp/pmc.log 2>&1
  q=$?
  echo "case [$c] plain rc=$p pmc rc=$q" >> $OUT
  if [ $q -ne 0 ]; then grep -E "pmc_repro|Segmentation|signal|@" /tmp/pmc.log | head -12 >> $OUT; exit $q; fi
  case $p in 0) ;; *) echo "plain run failed: stop" >> $OUT; exit $p;; esac
done
exit 0
