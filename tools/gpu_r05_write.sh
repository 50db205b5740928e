# WRITE_SIZE / FETCH_SIZE of wf_finish_bvh over one 16-pass room2m call, per library variant
cd "$GRAFT_REPO_ROOT" && O=$GRAFT_REPO_ROOT/gpurun_out/${R05_TAG:-r05ak} && mkdir -p $O && export PYTHONUNBUFFERED=1 TMPDIR=/tmp &&
PY=$(python -c "import os, sys; print(os.path.realpath(sys.executable))") &&
timeout -k 10 200 $PY tools/prof_call.py 2 > $O/warm.log 2>&1 &&
for v in ${R05_VARIANTS:-default park0}; do
  if [ $v = default ]; then unset ISAKLM_RT_LIB_OVERRIDE; else export ISAKLM_RT_LIB_OVERRIDE=$GRAFT_REPO_ROOT/ab_libs/$v.so; fi
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/${v}_w -o run --output-format csv -- $PY $GRAFT_REPO_ROOT/tools/prof_call.py 16 > $O/${v}_w.log 2>&1 || exit 1
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES --kernel-trace -d $O/${v}_i -o run --output-format csv -- $PY $GRAFT_REPO_ROOT/tools/prof_call.py 16 > $O/${v}_i.log 2>&1 || exit 1
  echo $v; $PY tools/pmc_finisher.py $O/${v}_w; $PY tools/pmc_finisher.py $O/${v}_i
done
