#!/bin/bash
# Round-5 batch AA: one more attempt at the llm.int8 bs=8 counter passes with the final build (the
# round-4/5 builds crashed rocprofv3 here); a crash ends the call.
R=$GRAFT_REPO_ROOT
cd $R
PMC_PASSES="c3" bash tools/profile_r05.sh r05aa_pmc
exit 0
