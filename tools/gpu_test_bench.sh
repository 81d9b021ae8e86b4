#!/bin/bash
# All GPU tests, smoke, then the default-bench A/B with kernel traces (dev tool).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/tb
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tb/gpu_tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/tb/smoke.log 2>&1 || exit $?
bash tools/gpu_ab_run.sh
