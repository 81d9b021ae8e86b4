#!/bin/bash
# Library / setting A/B (dev tool): lines "NAME LIB [VAR=val ...] -- bench args" in $AB (LIB "-" = the in-tree
# library), each run $REPS times interleaved -> gpurun_out/$TAG/ab_NAME_i.json.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
out=gpurun_out/${TAG:-ab}; mkdir -p "$out"
for rep in $(seq 1 ${REPS:-3}); do
  while read -r name lib rest; do
    [ -z "$name" ] && continue
    envs=${rest%%--*}; args=${rest#*--}
    if [ "$lib" = "-" ]; then lv=(); else lv=(MPCQ_LIBRARY=$lib); fi
    env "${lv[@]}" $envs timeout -k 10 300 python bench.py $args --cpu-seconds 0 --variants 0 --cfg3-strong 0 \
      > "$out/ab_${name}_$rep.json" 2>> "$out/ab.err" || { echo "ab $name failed"; tail -5 "$out/ab.err"; exit 1; }
  done <<< "$AB"
done
python - "$out" <<'PY'
import glob, json, sys, collections
r = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/ab_*.json")):
    name = f.rsplit("/", 1)[1][3:].rsplit("_", 1)[0]
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r[name].append((d["value"] / 1e6, d["roofline"]["frac"], d["roofline"]["kernel_ms"]))
for k, v in r.items():
    print(f"{k:20s} " + "  ".join(f"{a:7.2f}M {b:.4f} {c:.3f}ms" for a, b, c in v))
PY
