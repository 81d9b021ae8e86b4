#!/bin/bash
# Config-3 evidence (dev tool, on the GPU box): rocprofv3 kernel trace + stats of the perplant bench, the
# stage-isolation timings of tools/plant_profile.py, then PMC passes over the same bench (tools/pmc.sh).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cfg3 -o run -- \
  python bench.py --workload perplant --dtype ${DT:-f32} --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/prof_cfg3.log 2>&1 || exit $?
timeout -k 10 300 python tools/plant_profile.py > gpurun_out/plant_profile.txt 2>&1 || exit $?
CMD="python bench.py --workload perplant --dtype ${DT:-f32} --steps 2 --warmup 1 --cpu-seconds 0" \
PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY
SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
  bash tools/pmc.sh ${DT:-f32} gpurun_out/pmc_cfg3 || exit $?
exit 0
