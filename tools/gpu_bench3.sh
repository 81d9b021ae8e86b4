#!/bin/bash
# cfg2 bench in the three precisions (dev tool): gpurun_out/b_<dtype>.json
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for dt in ${DTYPES:-mixed f32 f64}; do
  timeout -k 10 200 python bench.py --dtype $dt --steps ${BENCH_STEPS:-10} --warmup 2 --cpu-seconds ${CPU_SECONDS:-2} > gpurun_out/b_$dt.json 2> gpurun_out/b_$dt.err || exit $?
done
exit 0
