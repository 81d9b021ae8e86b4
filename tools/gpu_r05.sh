#!/bin/bash
# One GPU call of round 5: the GPU test suite, the default bench line and optional extras, each step under its
# own time limit, stopping at the first failure.  Usage: tools/gpu_r05.sh TAG [steps...]
#   steps: tests | tests:<pytest -k expr> | bench | bench:<args> | probe:<dtype> | smoke | prof | pmc:<counters>
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for step in "$@"; do
  name=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  case $name in
    tests)
      if [ -n "$arg" ]; then k=(-k "$arg"); else k=(); fi
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
        > "$out/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/tests.log"; exit 1; } ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 \
        || { echo "smoke failed"; tail -20 "$out/smoke.log"; exit 1; } ;;
    bench)
      timeout -k 10 600 python -u bench.py $arg > "$out/bench_${arg// /_}.json" 2> "$out/bench_${arg// /_}.err" \
        || { echo "bench failed"; tail -20 "$out/bench_${arg// /_}.err"; exit 1; } ;;
    probe)
      timeout -k 10 600 python -u tools/order_probe.py $arg > "$out/probe_$arg.log" 2>&1 \
        || { echo "probe failed"; tail -20 "$out/probe_$arg.log"; exit 1; } ;;
    prof)
      (cd "$out" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d prof -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --variants 0 --cpu-seconds 0 $arg \
        > prof.log 2>&1) || { echo "prof failed"; tail -20 "$out/prof.log"; exit 1; } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $step ok"
done
