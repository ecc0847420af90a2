# round-3 evidence: PMC passes (reducer, convs, tgemm), then link curves at the shipped defaults
cd $GRAFT_REPO_ROOT
bash tools/gpu_r3_pmc.sh && bash tools/gpu_r3_links.sh
