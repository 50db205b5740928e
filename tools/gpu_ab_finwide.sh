# finisher: live-ray count at or below which a wave traces its rays one by one with all lanes (WF_FIN_WIDE) A/B
cd $GRAFT_REPO_ROOT && bash tools/ab_quick.sh room2m 64 3 ${@:-fw1 fw4 fw8 fw16}
