# tests + probe + f32/f64 bench (dev loop on the GPU box)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -q -x -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
MPCQ_PHASES=0 timeout -k 10 300 python tools/tile_probe.py f32 > gpurun_out/probe.log 2>&1 || exit $?
for dt in f32 f64; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --dtype $dt --cpu-seconds 0 > gpurun_out/bench_$dt.json 2>gpurun_out/bench_$dt.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 3 --warmup 1 --dtype f32 --cpu-seconds 0 > gpurun_out/prof.log 2>&1
