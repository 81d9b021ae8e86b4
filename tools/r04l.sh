#!/bin/bash
# Round-4 pass l (dev tool): GPU suite on the stacked-f64 library, the mixed parity tests at other fp64
# shares (MPCQ_MIX_R), then interleaved A/B lines: base library (HEAD before the change) vs new, and the
# new one at MIX_R 6 / 5 / 4.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
for r in 6 5 4; do
  MPCQ_MIX_R=$r timeout -k 10 300 python -u -m pytest tests/test_gpu.py -s -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -k "mixed_full_batch or mixed_tile_parity" > gpurun_out/mixr_$r.log 2>&1
  echo "rc=$?" >> gpurun_out/mixr_$r.log
done
MPCQ_PLANT_WPE=3 timeout -k 10 300 python -u -m pytest tests/ -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -k "plant or config3" > gpurun_out/plant_wpe3.log 2>&1
echo "rc=$?" >> gpurun_out/plant_wpe3.log
for rep in 1 2 3; do
  while read -r name lib dt envs; do
    [ -z "$name" ] && continue
    wl=cfg2; st=20
    case $name in pp_*) wl=perplant; st=5;; esac
    env MPCQ_LIBRARY=$lib $envs timeout -k 10 120 python bench.py --workload $wl --dtype $dt --steps $st --warmup 2 --cpu-seconds 0 --variants 0 > gpurun_out/ab_${name}_$rep.json 2>> gpurun_out/ab.err || exit $?
  done <<EOF
base_mixed solvempc_amd/libmpcq_base.so mixed
new_mixed solvempc_amd/libmpcq.so mixed
base_f64 solvempc_amd/libmpcq_base.so f64
new_f64 solvempc_amd/libmpcq.so f64
new_mixed_r6 solvempc_amd/libmpcq.so mixed MPCQ_MIX_R=6
new_mixed_r5 solvempc_amd/libmpcq.so mixed MPCQ_MIX_R=5
new_mixed_r4 solvempc_amd/libmpcq.so mixed MPCQ_MIX_R=4
pp_base_f64 solvempc_amd/libmpcq_base.so f64
pp_new_f64 solvempc_amd/libmpcq.so f64
pp_new_f64_w3 solvempc_amd/libmpcq.so f64 MPCQ_PLANT_WPE=3
pp_base_f32 solvempc_amd/libmpcq_base.so f32
pp_new_f32_w3 solvempc_amd/libmpcq.so f32 MPCQ_PLANT_WPE=3
EOF
done
exit 0
