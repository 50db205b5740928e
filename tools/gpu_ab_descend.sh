# descent step with selects + unconditional LDS stack write (default) vs the branchy step (RT_DESCEND_BRANCHY) A/B
cd $GRAFT_REPO_ROOT && bash tools/ab_quick.sh room2m 64 4 base sel
