#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of the cfg2 bench per dtype (summarise with tools/pmc_traffic.py).
cd "$GRAFT_REPO_ROOT" || exit 2
for dt in f32 f64; do
  PMC_SETS="FETCH_SIZE
WRITE_SIZE" bash tools/pmc.sh $dt gpurun_out/pmct_$dt || exit $?
done
