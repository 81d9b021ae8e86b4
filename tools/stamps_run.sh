#!/bin/bash
# Per-wave stage stamps of the tile kernel (dev tool): needs tools/dbglib/libmpcq.so from
# `SRC=mpcq_tile_f64.hip bash tools/build_dbg.sh MPCQ_INFO_STAMPS` (or the f32 source); writes
# gpurun_out/stamps_<dtype>.bin and the tools/stamps.py summary.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for dt in ${DTYPES:-mixed f64}; do
  MPCQ_LIBRARY=${LIB:-tools/dbglib/libmpcq.so} MPCQ_TILE_STAMPS=gpurun_out/stamps_$dt$TAG.bin timeout -k 10 200 \
    python bench.py --dtype $dt --steps 1 --warmup 1 --cpu-seconds 0 --variants 0 > gpurun_out/stamps_bench_$dt$TAG.json 2>&1 || exit $?
  python tools/stamps.py gpurun_out/stamps_$dt$TAG.bin > gpurun_out/stamps_$dt$TAG.txt 2>&1 || exit $?
done
exit 0
