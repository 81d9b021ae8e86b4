# f32/f64 bench + kernel trace of the f32 bench (dev loop on the GPU box)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/bench_*.json
for dt in f32 f64; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --dtype $dt --cpu-seconds 0 > gpurun_out/bench_$dt.json 2>gpurun_out/bench_$dt.err || exit $?
done
for v in ${AB_VARIANTS:-}; do
  env $v timeout -k 10 200 python bench.py --steps 5 --warmup 1 --dtype f32 --cpu-seconds 0 > gpurun_out/bench_${v//=/_}.json 2>>gpurun_out/bench_f32.err || exit $?
done
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 3 --warmup 1 --dtype f32 --cpu-seconds 0 > gpurun_out/prof.log 2>&1
