# AMDGPU machine-scheduler strategy (max-ilp / max-memory-clause vs default) A/B
cd $GRAFT_REPO_ROOT && bash tools/ab_quick.sh room2m 64 3 base ilp memc
