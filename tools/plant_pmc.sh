#!/bin/bash
# PMC of the config-3 kernel's stages (dev tool, GPU): tools/plant_profile.py (fp64: default, max_iter = 1, 24,
# 25, ...) under one rocprofv3 --pmc pass per counter set -> $1/p<i>/ ; summarise with tools/plant_pmc.py.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
out=${1:-gpurun_out/plant_pmc}; mkdir -p "$out"
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  DTYPES=f64 timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d "$out/p$i" -o run -- python3 tools/plant_profile.py > "$out/p$i.log" 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc" >> "$out/passes.txt"
  [ $rc -eq 0 ] || exit $rc
done <<SETS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE
SETS
exit 0
