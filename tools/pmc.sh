#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 run per counter set; never combined with tracing).
#   usage (on the GPU box): bash tools/pmc.sh <dtype> <outdir>   (CMD=... overrides the profiled program,
#   PMC_SETS=... the counter passes, one line each)
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
dt=${1:-f32}; out=${2:-gpurun_out/pmc_$dt}
mkdir -p "$out"
CMD=${CMD:-"python bench.py --steps 3 --warmup 1 --dtype $dt --cpu-seconds 0 --cfg3-strong 0"}
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$out/p$i" -o run -- $CMD > "$out/p$i.log" 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc" >> "$out/passes.txt"
  if [ $rc -ne 0 ]; then exit $rc; fi
done <<SETS
${PMC_SETS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT
FETCH_SIZE
WRITE_SIZE}
SETS
exit 0
