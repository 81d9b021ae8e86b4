#!/bin/bash
# Round-4 pass s (dev tool): the round's evidence on HEAD: the driver's default bench line, every
# workload's line, a rocprofv3 kernel trace + stats of the default bench, and PMC passes of the mixed
# config-2 kernel (HBM traffic, MFMA busy, MFMA MOPS) for profiles/pmc_*_mixed.json.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/s_default.json 2> gpurun_out/s_default.err || exit $?
timeout -k 10 300 python bench.py --workload perplant > gpurun_out/s_perplant.json 2> gpurun_out/s_perplant.err || exit $?
timeout -k 10 300 python bench.py --workload perplant --scaling strong --steps 3 --warmup 1 > gpurun_out/s_perplant_strong.json 2> gpurun_out/s_perplant_strong.err || exit $?
timeout -k 10 300 python bench.py --workload stream --steps 3 --warmup 1 > gpurun_out/s_stream.json 2> gpurun_out/s_stream.err || exit $?
timeout -k 10 300 python bench.py --workload quadrotor --steps 3 --warmup 1 > gpurun_out/s_quadrotor.json 2> gpurun_out/s_quadrotor.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_s -o run -- python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --variants 0 > gpurun_out/prof_s.log 2>&1 || exit $?
CMD="python bench.py --dtype mixed --steps 3 --warmup 1 --cpu-seconds 0 --variants 0" \
PMC_SETS="FETCH_SIZE
WRITE_SIZE
SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_COUNT" bash tools/pmc.sh mixed gpurun_out/pmc_s_mixed || exit $?
exit 0
