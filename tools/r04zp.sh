#!/bin/bash
# Round-4 pass zp (dev tool): final validation of HEAD: the GPU suite, smoke(), the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/zp_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/zp_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/zp_smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/zp_bench.json 2> gpurun_out/zp_bench.err || exit $?
exit 0
