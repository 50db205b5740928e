set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
P=/tmp/prof; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/wf_kt -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --passes 4 --no-cpu-baseline --kernel wavefront > $R/gpurun_out/prof_wf.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --kernel-trace -d $P/wf_sq -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --passes 4 --no-cpu-baseline --kernel wavefront > $R/gpurun_out/prof_wf_sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --kernel-trace -d $P/mega_sq -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --passes 4 --no-cpu-baseline > $R/gpurun_out/prof_mega_sq.log 2>&1
python3 $R/tools/prof_summary.py $R/gpurun_out/prof_wf_summary.json $P/wf_kt $P/wf_sq $P/mega_sq > /dev/null
