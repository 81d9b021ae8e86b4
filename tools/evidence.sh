#!/bin/bash
# HEAD evidence of one round (GPU box): the GPU suite, smoke, every workload's bench line (with its CPU baseline
# and parity blocks) and a rocprofv3 kernel trace + stats of each bench command.  usage: tools/evidence.sh TAG
# -> gpurun_out/TAG/{tests.log, smoke.log, bench_<wl>.json, prof_<wl>/}.  Stops at the first failure.
set -o pipefail
tag=${1:-evidence}; out=gpurun_out/$tag; mkdir -p "$out"
export TMPDIR=/tmp
root=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 \
  || { echo "tests failed"; tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { echo "smoke failed"; exit 1; }
for wl in cfg2 perplant quadrotor stream; do
  timeout -k 10 600 python -u bench.py --workload $wl > "$out/bench_$wl.json" 2> "$out/bench_$wl.err" \
    || { echo "bench $wl failed"; tail -20 "$out/bench_$wl.err"; exit 1; }
  echo "bench $wl ok"
done
for wl in cfg2 perplant quadrotor stream; do
  steps=20; [ $wl = quadrotor ] && steps=3; [ $wl = stream ] && steps=3
  (cd "$out" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d prof_$wl -o run -- python3 "$root/bench.py" \
      --workload $wl --steps $steps --warmup 1 --variants 0 --cpu-seconds 0 --cfg3-strong 0 > prof_$wl.log 2>&1) \
    || { echo "prof $wl failed"; tail -20 "$out/prof_$wl.log"; exit 1; }
  python3 tools/rocpd_export.py "$out/prof_$wl/run_results.db" "$out/${tag}_$wl" > /dev/null || exit 1
  echo "prof $wl ok"
done
exit 0
