#!/bin/bash
# Round-4 pass p (dev tool): the GPU suite with phase 0 as a work queue (MPCQ_QUEUE=1), then A/B lines:
# queue off / on, with the default stops and (mixed) [75, max].
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
MPCQ_QUEUE=1 timeout -k 10 500 python -u -m pytest tests/ -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_q1.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests_q1.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  while read -r name dt envs; do
    [ -z "$name" ] && continue
    env $envs timeout -k 10 120 python bench.py --dtype $dt --steps 20 --warmup 3 --cpu-seconds 0 --variants 0 > gpurun_out/q_${name}_$rep.json 2>> gpurun_out/q.err || exit $?
  done <<AB
mx_def mixed
mx_q mixed MPCQ_QUEUE=1
mx_3 mixed MPCQ_PHASES=3
mx_3q mixed MPCQ_PHASES=3 MPCQ_QUEUE=1
f64_def f64
f64_q f64 MPCQ_QUEUE=1
f32_def f32
f32_q f32 MPCQ_QUEUE=1
AB
done
exit 0
