# round 4, first GPU session: the new tests on the default build, the state-machine finisher's
# parity tests, its A/B against the default on the bulk, the phase profile
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh r04c tests:"test_gpu_chain or test_gpu_traversal or configs4" && \
ISAKLM_RT_LIB_OVERRIDE=$PWD/ab_libs/sm.so bash tools/gpu_run.sh r04c_sm tests:"test_gpu_chain or test_gpu_traversal or smoke or configs0 or configs1" && \
MAXD=64 timeout -k 10 900 bash tools/gpu_ab_libs.sh 2 3 128 room2m ab_libs/base.so ab_libs/sm.so ab_libs/sm_s8.so ab_libs/sm_s40.so ab_libs/sm_c8.so ab_libs/sm_w5.so ab_libs/base_w5.so && \
ISAKLM_RT_LIB_OVERRIDE=$PWD/ab_libs/phase.so timeout -k 10 300 python -u tools/phase_profile.py room2m 128
