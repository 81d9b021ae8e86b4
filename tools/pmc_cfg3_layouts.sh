#!/bin/bash
# PMC of the config-3 one-pass kernel, two plants per wave (MPCQ_PLANT_LAYOUT=2) against three (default):
# VALU / LDS / SALU instructions and wave cycles per dispatch.  Usage (GPU box): bash tools/pmc_cfg3_layouts.sh OUTDIR
out=${1:-gpurun_out/pmc_cfg3}
cd "$GRAFT_REPO_ROOT" || exit 2
for lay in 2 3; do
  MPCQ_PLANT_LAYOUT=$lay CMD="python bench.py --workload perplant --steps 2 --warmup 1 --cpu-seconds 0 --variants 0" \
    PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
    timeout -k 10 300 bash tools/pmc.sh f64 "$out/lay$lay" > "$out.lay$lay.log" 2>&1 || exit 1
done
