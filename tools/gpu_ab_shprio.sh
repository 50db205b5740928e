# s_setprio for wf_shade waves (finish sooner beside the other pipelines' trace launches) A/B
cd $GRAFT_REPO_ROOT && bash tools/ab_quick.sh room2m 64 3 base sp2 sp3
