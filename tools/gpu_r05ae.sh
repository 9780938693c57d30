#!/bin/bash
# Round-5 batch AE: counters of the LLM.int8 decode attention (llj_attention_i8) via the C++ harness.
R=$GRAFT_REPO_ROOT
cd $R
C3H_CASES="attn:atti8:8:4096:144" bash tools/pmc_c3_harness.sh r05_pmc_c3_harness_attn
exit 0
