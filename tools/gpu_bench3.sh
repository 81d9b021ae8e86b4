#!/bin/bash
# cfg2 bench in the three precisions plus A/B variants (dev tool): gpurun_out/b_<name>.json
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for dt in ${DTYPES:-mixed f32 f64}; do
  timeout -k 10 200 python bench.py --dtype $dt --steps ${BENCH_STEPS:-10} --warmup 2 --cpu-seconds ${CPU_SECONDS:-2} > gpurun_out/b_$dt.json 2> gpurun_out/b_$dt.err || exit $?
done
# A/B lines: "NAME DTYPE ENV..."
while read -r name dt envs; do
  [ -z "$name" ] && continue
  env $envs timeout -k 10 200 python bench.py --dtype $dt --steps ${BENCH_STEPS:-10} --warmup 2 --cpu-seconds 0 > gpurun_out/b_$name.json 2> gpurun_out/b_$name.err || exit $?
done <<< "${AB:-f32_occ2 f32 MPCQ_TILE_OCC=2
f32_tiletail f32 MPCQ_TAIL=tile
mixed_r6 mixed MPCQ_MIX_R=6}"
exit 0
