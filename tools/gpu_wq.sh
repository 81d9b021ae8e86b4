#!/bin/bash
# Dev loop for the tile kernel: tile-path parity tests, then the cfg2 bench f32 / f64 and a kernel
# trace.  usage: bash tools/gpu_wq.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
o=gpurun_out/${1:-wq}; mkdir -p "$o"
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit $?
for dt in f32 f64; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --dtype $dt --cpu-seconds 0 > $o/bench_$dt.json 2> $o/bench_$dt.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o run -- python bench.py --steps 5 --warmup 1 --cpu-seconds 0 > $o/prof.log 2>&1
