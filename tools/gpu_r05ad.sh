#!/bin/bash
# Round-5 batch AD: counters of the llm.int8 bs=8 decode kernels via the C++ harness.
R=$GRAFT_REPO_ROOT
cd $R
bash tools/pmc_c3_harness.sh r05_pmc_c3_harness
exit 0
