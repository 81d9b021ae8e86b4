#!/bin/bash
# Round-4 evidence pass (dev tool): PMC of the headline (mixed) cfg2 bench, then tail A/B repeats.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
CMD="python bench.py --dtype mixed --steps 3 --warmup 1 --cpu-seconds 0 --variants 0" \
PMC_SETS="FETCH_SIZE
WRITE_SIZE
SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_COUNT" bash tools/pmc.sh mixed gpurun_out/pmc_mixed || exit $?
for rep in 1 2 3; do
  for v in "wave:" "tile:MPCQ_TAIL=tile"; do
    name=${v%%:*}; envs=${v#*:}
    for dt in mixed f32; do
      env $envs timeout -k 10 120 python bench.py --dtype $dt --steps 20 --warmup 3 --cpu-seconds 0 --variants 0 > gpurun_out/ab_${dt}_${name}_$rep.json 2>> gpurun_out/ab.err || exit $?
    done
  done
done
exit 0
