# Dev tool: order_key_kernel workgroup-size A/B (MPCQ_ORDER_WG), kernel stats per size, then bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
out=gpurun_out/r05ak; mkdir -p $out
for wg in 1024 512 256; do
  (cd $out && MPCQ_ORDER_WG=$wg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d prof_$wg -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --variants 0 --cpu-seconds 0 > prof_$wg.log 2>&1) || exit 1
done
for rep in 1 2 3; do
  for wg in 1024 512 256; do
    MPCQ_ORDER_WG=$wg timeout -k 10 200 python bench.py --steps 20 --warmup 3 --variants 0 --cpu-seconds 0 > $out/b_${wg}_$rep.json 2>> $out/ab.err || exit 1
  done
done
