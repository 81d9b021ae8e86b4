#!/bin/bash
# Round-4 pass o (dev tool): phase-stop A/B of the mixed and f64 tile chains (MPCQ_PHASES, MPCQ_TAIL),
# config 3 as BASELINE writes it (1,048,576 plants on one GPU, f64) and config 5 in f32 and f64.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2 3; do
  while read -r name dt envs; do
    [ -z "$name" ] && continue
    env $envs timeout -k 10 120 python bench.py --dtype $dt --steps 20 --warmup 3 --cpu-seconds 0 --variants 0 > gpurun_out/ph_${name}_$rep.json 2>> gpurun_out/ph.err || exit $?
  done <<AB
mx_def mixed
mx_34 mixed MPCQ_PHASES=3,4
mx_45 mixed MPCQ_PHASES=4,5
mx_5 mixed MPCQ_PHASES=5
mx_3 mixed MPCQ_PHASES=3
mx_24 mixed MPCQ_PHASES=2,4
mx_wt mixed MPCQ_TAIL=wave
f64_def f64
f64_34 f64 MPCQ_PHASES=3,4
f64_45 f64 MPCQ_PHASES=4,5
AB
done
timeout -k 10 300 python bench.py --workload perplant --scaling strong --steps 3 --warmup 1 > gpurun_out/bench_cfg3_strong.json 2> gpurun_out/bench_cfg3_strong.err || exit $?
timeout -k 10 300 python bench.py --workload stream --steps 3 --warmup 1 > gpurun_out/bench_stream_f32.json 2> gpurun_out/bench_stream_f32.err || exit $?
timeout -k 10 300 python bench.py --workload stream --dtype f64 --steps 3 --warmup 1 > gpurun_out/bench_stream_f64.json 2> gpurun_out/bench_stream_f64.err || exit $?
exit 0
