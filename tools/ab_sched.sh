#!/bin/bash
# Schedule / variant A/B of the cfg2 bench (dev tool): each line "NAME ENV..." runs bench.py once with
# that environment (MPCQ_LIBRARY selects an alternative build; BENCH_ARGS: e.g. --workload perplant);
# results in gpurun_out/ab_NAME.json.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
while read -r name envs; do
  [ -z "$name" ] && continue
  env $envs timeout -k 10 120 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 ${BENCH_ARGS} > gpurun_out/ab_$name.json 2>> gpurun_out/ab.err || exit 1
done <<< "${AB_CASES}"
exit 0
