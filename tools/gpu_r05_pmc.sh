# counter passes over one 16-pass room2m call, per library variant: SQ issue / wait, I-cache
cd "$GRAFT_REPO_ROOT" && O=$GRAFT_REPO_ROOT/gpurun_out/${R05_TAG:-r05s} && mkdir -p $O && export PYTHONUNBUFFERED=1 TMPDIR=/tmp &&
PY=$(python -c "import os, sys; print(os.path.realpath(sys.executable))") && echo "python: $PY" &&
timeout -k 10 200 $PY tools/prof_call.py 2 > $O/warm.log 2>&1 &&
for v in ${R05_VARIANTS:-default noenter}; do
  if [ $v = default ]; then unset ISAKLM_RT_LIB_OVERRIDE; else export ISAKLM_RT_LIB_OVERRIDE=$GRAFT_REPO_ROOT/ab_libs/$v.so; fi
  timeout -s KILL 420 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU --kernel-trace -d $O/${v}_sq -o run --output-format csv -- $PY $GRAFT_REPO_ROOT/tools/prof_call.py 16 > $O/${v}_sq.log 2>&1 || exit 1
  timeout -s KILL 420 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_LDS SQ_INSTS_VMEM_RD --kernel-trace -d $O/${v}_ic -o run --output-format csv -- $PY $GRAFT_REPO_ROOT/tools/prof_call.py 16 > $O/${v}_ic.log 2>&1 || exit 1
  echo $v; $PY tools/pmc_finisher.py $O/${v}_sq; $PY tools/pmc_finisher.py $O/${v}_ic
done
