#!/bin/bash
# All GPU tests + smoke, then cfg2 (trace) and cfg3 benches (dev tool).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/c2
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/c2/gpu_tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/c2/smoke.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/c2/cfg2.json 2> gpurun_out/c2/cfg2.err || exit $?
timeout -k 10 300 python bench.py --workload perplant --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/c2/cfg3.json 2> gpurun_out/c2/cfg3.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c2/tr -o run -- python bench.py --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/c2/tr.log 2>&1
