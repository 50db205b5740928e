# bary stage with record loads issued before the exact division (WF_BARY_EARLY) A/B
cd $GRAFT_REPO_ROOT && bash tools/ab_quick.sh room2m 64 4 base early
