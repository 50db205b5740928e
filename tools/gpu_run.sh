#!/bin/bash
# One parametrised GPU-box run (replaces the per-experiment gpu_r0x_*.sh scripts).
# usage: bash tools/gpu_run.sh OUT STEP [STEP ...]   (run from the repo root on the GPU box)
#   tests            every GPU test          tests:EXPR   pytest -k EXPR
#   smoke            __graft_entry__.smoke()
#   bench:ARGS       python bench.py ARGS   (ARGS with ',' for ' ', e.g. bench:--steps,20,--warmup,5)
#   rocprof:ARGS     rocprofv3 --kernel-trace --stats of bench.py --no-pmc --no-cpu-baseline ARGS
#   py:FILE:ARGS     python FILE ARGS (a tools/ script)
# Every step runs under its own time limit; the first failure ends the run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/$1
shift
mkdir -p "$O"
export PYTHONUNBUFFERED=1
n=0
for step in "$@"; do
    n=$((n + 1))
    kind=${step%%:*}
    arg=""
    [[ "$step" == *:* ]] && arg=${step#*:}
    args=${arg//,/ }
    log="$O/$n.$kind"
    echo "[gpu_run] step $n: $step" >&2
    case "$kind" in
    tests)
        if [ -n "$arg" ]; then
            timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "$arg" > "$log.log" 2>&1
        else
            timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > "$log.log" 2>&1
        fi
        rc=$?; tail -3 "$log.log" ;;
    smoke)
        timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log.log" 2>&1
        rc=$?; tail -2 "$log.log" ;;
    bench)
        timeout -k 10 900 python -u bench.py $args > "$log.json" 2> "$log.err"
        rc=$?; tail -c 400 "$log.json"; echo ;;
    rocprof)
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$log.d" -o run \
            --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-pmc --no-cpu-baseline $args \
            > "$GRAFT_REPO_ROOT/$log.json" 2> "$GRAFT_REPO_ROOT/$log.err")
        rc=$?; tail -c 300 "$log.json"; echo ;;
    py)
        f=${arg%%:*}; a=""; [[ "$arg" == *:* ]] && a=${arg#*:}; a=${a//,/ }
        timeout -k 10 900 python -u "$f" $a > "$log.out" 2> "$log.err"
        rc=$?; tail -5 "$log.out" ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
    if [ $rc -ne 0 ]; then
        echo "[gpu_run] step $n ($step) failed rc=$rc"; tail -20 "$log".* 2>/dev/null | tail -40; exit $rc
    fi
done
