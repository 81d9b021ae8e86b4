#!/bin/bash
# Round check on the GPU box: gpu tests, smoke, the benches of every config (with cpu_baseline) and
# rocprofv3 kernel stats for configs 2 and 4.  usage: bash tools/gpu_round.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
o=gpurun_out/${1:-round}; mkdir -p "$o"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || exit $?
timeout -k 10 200 python bench.py > $o/bench_cfg2_f32.json 2> $o/bench_cfg2_f32.err || exit $?
timeout -k 10 200 python bench.py --dtype f64 > $o/bench_cfg2_f64.json 2> $o/bench_cfg2_f64.err || exit $?
timeout -k 10 300 python bench.py --workload perplant --steps 3 --warmup 1 --cpu-seconds 5 > $o/bench_cfg3_f32.json 2> $o/bench_cfg3.err || exit $?
timeout -k 10 300 python bench.py --workload quadrotor --steps 3 --warmup 1 --cpu-seconds 5 > $o/bench_cfg4.json 2> $o/bench_cfg4.err || exit $?
timeout -k 10 300 python bench.py --workload stream --steps 3 --warmup 1 > $o/bench_cfg5_f32.json 2> $o/bench_cfg5.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_cfg2 -o run -- python bench.py --steps 5 --warmup 1 --cpu-seconds 0 > $o/prof_cfg2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_cfg4 -o run -- python bench.py --workload quadrotor --steps 3 --warmup 1 --cpu-seconds 0 > $o/prof_cfg4.log 2>&1
