# Round-end check on the GPU box: gpu tests, smoke, default bench (with cpu_baseline), kernel stats.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/final && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || exit $?
timeout -k 10 200 python bench.py > gpurun_out/final/bench_default.json 2>gpurun_out/final/bench_default.err || exit $?
timeout -k 10 200 python bench.py --dtype f64 > gpurun_out/final/bench_default_f64.json 2>gpurun_out/final/bench_default_f64.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof -o run -- python bench.py --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/final/prof.log 2>&1
