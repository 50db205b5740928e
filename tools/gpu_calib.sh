# FETCH_SIZE calibration on known line counts + the counter list (GPU box)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/calib
cd /tmp && export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 $R/tools/fetch_calibrate.hip -o /tmp/fetch_calibrate || exit 1
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/calib/counters_list.txt 2>&1 || echo "list rc=$?"
grep -E "TCC_EA0_RD|TCC_BUBBLE|TCC_EA0_WR|FETCH_SIZE|WRITE_SIZE|TCC_REQ|TCC_READ" $R/gpurun_out/calib/counters_list.txt | head -40 > $R/gpurun_out/calib/counters_tcc.txt || true
for set in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_BUBBLE_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $set | tr ' ' '_')
  timeout -s KILL 60 rocprofv3 --pmc $set --kernel-trace -d /tmp/cal_$tag -o run --output-format csv -- /tmp/fetch_calibrate > $R/gpurun_out/calib/run_$tag.log 2>&1
  rc=$?
  echo "pass $tag rc=$rc"
  f=$(find /tmp/cal_$tag -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && cp $f $R/gpurun_out/calib/cc_$tag.csv
  if [ $rc -ge 124 ]; then echo "pass $tag killed"; exit 1; fi
done
exit 0
