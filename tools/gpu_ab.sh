cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -q -x -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
for occ in 3 4; do
  MPCQ_TILE_OCC=$occ timeout -k 10 200 python bench.py --steps 5 --warmup 1 --dtype f32 --cpu-seconds 0 > gpurun_out/bench_occ$occ.json 2>gpurun_out/bench_occ$occ.err || exit $?
done
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --dtype f64 --cpu-seconds 0 > gpurun_out/bench_f64.json 2>gpurun_out/bench_f64.err || exit $?
MPCQ_TILE_OCC=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3 -o run -- python bench.py --steps 3 --warmup 1 --dtype f32 --cpu-seconds 0 > gpurun_out/prof3.log 2>&1
