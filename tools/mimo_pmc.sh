#!/bin/bash
# PMC passes over tools/mimo_pmc.py (dev tool, GPU box).  usage: bash tools/mimo_pmc.sh <outdir> <mode> [batch]
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
out=${1:-gpurun_out/mpmc}; mode=${2:-gj}; batch=${3:-16384}; mkdir -p "$out"
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d "$out/p$i" -o run -- python tools/mimo_pmc.py $mode $batch > "$out/p$i.log" 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc" >> "$out/passes.txt"
  if [ $rc -ne 0 ]; then exit $rc; fi
done <<SETS
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS
SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE
SETS
exit 0
