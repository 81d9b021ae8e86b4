#!/bin/bash
# GPU tests (tile/wave paths) + default-bench A/B variants with kernel traces (dev tool).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/qa
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/qa/gpu_tests.log 2>&1 || exit $?
bash tools/gpu_ab_run.sh
