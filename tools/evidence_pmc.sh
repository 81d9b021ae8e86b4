#!/bin/bash
# HEAD PMC evidence (GPU box): FETCH_SIZE / WRITE_SIZE and the SQ / MFMA set over each workload's bench command
# (tools/gpu.sh pmc steps), the config-3 stage PMC and per-wave stage stamps.  usage: tools/evidence_pmc.sh TAG
set -o pipefail
tag=${1:-evidence}
bash tools/gpu.sh $tag pmc:cfg2,mixed pmc:perplant,f64 pmc:quadrotor,f64 pmc:stream,f64 || exit 1
timeout -k 10 600 bash tools/plant_pmc.sh gpurun_out/$tag/plant_pmc && python3 tools/plant_pmc.py gpurun_out/$tag/plant_pmc \
  > gpurun_out/$tag/plant_pmc/summary.txt || exit 1
if [ -f tools/dbg_r06q/libmpcq.so ]; then
  MPCQ_LIBRARY=tools/dbg_r06q/libmpcq.so timeout -k 10 300 python3 tools/plant_stamps.py > gpurun_out/$tag/plant_stamps.txt 2>&1 || exit 1
fi
exit 0
