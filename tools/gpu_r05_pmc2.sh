# counter passes over one 16-pass room2m call: SQ issue by type, TA / TCP busy and stalls (wf_finish_bvh)
cd "$GRAFT_REPO_ROOT" && O=$GRAFT_REPO_ROOT/gpurun_out/${R05_TAG:-r05ae} && mkdir -p $O && export PYTHONUNBUFFERED=1 TMPDIR=/tmp &&
PY=$(python -c "import os, sys; print(os.path.realpath(sys.executable))") &&
timeout -k 10 200 $PY tools/prof_call.py 2 > $O/warm.log 2>&1 &&
for pass in "sq:SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" "ta:TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "tcp:TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE" "wait:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU"; do
  n=${pass%%:*}; c=${pass#*:}
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace -d $O/$n -o run --output-format csv -- $PY $GRAFT_REPO_ROOT/tools/prof_call.py 16 > $O/$n.log 2>&1 || exit 1
  echo $n; $PY tools/pmc_finisher.py $O/$n
done
