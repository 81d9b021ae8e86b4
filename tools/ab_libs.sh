#!/bin/bash
# Library A/B (dev tool): "NAME LIB DTYPE" lines in $AB, each run $REPS times interleaved; gpurun_out/ablib_NAME_i.json
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-3}); do
  while read -r name lib dt; do
    [ -z "$name" ] && continue
    MPCQ_LIBRARY=$lib timeout -k 10 120 python bench.py --dtype $dt --steps 20 --warmup 3 --cpu-seconds 0 --variants 0 > gpurun_out/ablib_${name}_$rep.json 2>> gpurun_out/ablib.err || exit $?
  done <<< "$AB"
done
exit 0
