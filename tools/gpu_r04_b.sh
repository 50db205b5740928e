# round 4: the headline bench with chained calls (overlap) vs unchained, calls of 256 / 64 passes,
# the 5-waves/SIMD finisher build, and Msamples/s by passes per call
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04b; mkdir -p $O
export PYTHONUNBUFFERED=1
B="--no-pmc --no-cpu-baseline --steps 20 --warmup 5"
timeout -k 10 300 python bench.py $B > $O/chain_spc4.json 2> $O/chain_spc4.err && tail -c 300 $O/chain_spc4.json | head -c 300; echo && \
timeout -k 10 300 python bench.py $B --steps-per-call 1 > $O/chain_spc1.json 2> $O/chain_spc1.err && tail -c 300 $O/chain_spc1.json | head -c 300; echo && \
timeout -k 10 300 python bench.py $B --overlap 0 > $O/nochain_spc4.json 2> $O/nochain_spc4.err && tail -c 300 $O/nochain_spc4.json | head -c 300; echo && \
ISAKLM_RT_LIB_OVERRIDE=$PWD/ab_libs/base_w5.so timeout -k 10 300 python bench.py $B > $O/w5_chain_spc4.json 2> $O/w5_chain_spc4.err && tail -c 300 $O/w5_chain_spc4.json | head -c 300; echo && \
timeout -k 10 400 python tools/call_granularity.py 256 1,16,64,256 > $O/granularity.jsonl 2> $O/granularity.err; cat $O/granularity.jsonl
