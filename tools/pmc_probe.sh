#!/bin/bash
# PMC passes over a fixed-iteration probe launch (tools/tile_probe.py), one rocprofv3 run per counter
# set (dev tool, GPU box).  usage: PROBE_ARGS="f32 65536 125" bash tools/pmc_probe.sh <outdir>
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
out=${1:-gpurun_out/pmcp}; mkdir -p "$out"
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d "$out/p$i" -o run -- python tools/tile_probe.py ${PROBE_ARGS:-f32 65536 125} > "$out/p$i.log" 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc" >> "$out/passes.txt"
  if [ $rc -ne 0 ]; then exit $rc; fi
done <<SETS
${PMC_SETS:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE
SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_LDS GRBM_COUNT}
SETS
exit 0
