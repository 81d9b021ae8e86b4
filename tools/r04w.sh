#!/bin/bash
# Round-4 pass w (dev tool): per-plant fp64 kernel at 3 vs 4 waves/SIMD (MPCQ_PLANT_WPE), then the config-3
# evidence of the default kernel (kernel trace + stats, stage isolation, PMC) via tools/prof_cfg3.sh.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
MPCQ_PLANT_WPE=4 timeout -k 10 300 python -u -m pytest tests/test_plants_step.py -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/plant_wpe4.log 2>&1
echo "rc=$?" >> gpurun_out/plant_wpe4.log
for rep in 1 2 3; do
  for w in 3 4; do
    MPCQ_PLANT_WPE=$w timeout -k 10 200 python bench.py --workload perplant --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/w_wpe${w}_$rep.json 2>> gpurun_out/w.err || exit $?
  done
done
for rep in 1 2; do
  for cpw in 6 8 12 16; do
    MPCQ_STREAM_CPW=$cpw timeout -k 10 200 python bench.py --workload stream --dtype f64 --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/w_st_cpw${cpw}_$rep.json 2>> gpurun_out/w.err || exit $?
  done
done
DT=f64 bash tools/prof_cfg3.sh || exit $?
exit 0
