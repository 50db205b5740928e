# s_setprio of the latency-bound kernels (wf_long, wf_finish_coop) A/B
cd $GRAFT_REPO_ROOT && bash tools/ab_quick.sh room2m 64 3 base lp2 lfp2 lp3
