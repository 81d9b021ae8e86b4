#!/bin/bash
# A/B of env-selected variants of the default bench (dev tool, GPU box).  One line per variant in
# $VARIANTS ("name ENV=.. ENV=.."); each gets a bench JSON and a kernel trace (per-phase durations).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
out=gpurun_out/ab; mkdir -p $out
ARGS=${BENCH_ARGS:---steps 10 --warmup 2 --cpu-seconds 0}
while read -r name envs; do
  [ -z "$name" ] && continue
  env $envs timeout -k 10 200 python bench.py $ARGS > $out/$name.json 2> $out/$name.err || { echo "bench $name rc=$?" >> $out/$name.err; exit 1; }
  if [ -n "$TRACE" ]; then
    env $envs timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $out/tr_$name -o run -- python bench.py --steps 3 --warmup 1 --cpu-seconds 0 $EXTRA > $out/tr_$name.log 2>&1 || { echo "trace $name rc=$?" >> $out/$name.err; exit 1; }
  fi
done <<< "$VARIANTS"
exit 0
