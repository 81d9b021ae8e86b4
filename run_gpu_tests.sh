#!/bin/bash
# GPU test driver: each GPU step under its own limit; stop at the first abnormal exit.
cd "$GRAFT_REPO_ROOT" || exit 2
timeout -k 10 400 python -m pytest tests/test_gpu.py -q -m gpu -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke.log
exit $rc
