#!/bin/bash
# One GPU call: the GPU test suite, the default bench line and optional extras, each step under its
# own time limit, stopping at the first failure.  Usage: tools/gpu.sh TAG [steps...]
#   steps: tests | tests:<pytest -k expr> | bench | bench:<args> | probe:<dtype> | smoke | prof | pmc:<counters>
#          | envbench:VAR=val,<args> | pmcw:VAR=val,<dtype> | stamps:mimo_setup | tstamps:<dtype> | calib
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for step in "$@"; do
  name=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  case $name in
    tests)
      if [ -n "$arg" ]; then k=(-k "$arg"); else k=(); fi
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
        > "$out/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$out/tests.log"; exit 1; } ;;
    testsk)  # as tests, but failed assertions (pytest exit 1) do not end the call; any other failure does
      if [ -n "$arg" ]; then k=(-k "$arg"); else k=(); fi
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "${k[@]}" \
        > "$out/tests.log" 2>&1; rc=$?
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "tests crashed rc=$rc"; tail -30 "$out/tests.log"; exit 1; }
      grep -E "^(FAILED|ERROR)|passed|failed" "$out/tests.log" | tail -12 ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 \
        || { echo "smoke failed"; tail -20 "$out/smoke.log"; exit 1; } ;;
    bench)  # bench:<args with _ for spaces>, e.g. bench:--workload_quadrotor
      timeout -k 10 600 python -u bench.py ${arg//_/ } > "$out/bench_$arg.json" 2> "$out/bench_$arg.err" \
        || { echo "bench failed"; tail -20 "$out/bench_$arg.err"; exit 1; } ;;
    probe)
      timeout -k 10 600 python -u tools/order_probe.py $arg > "$out/probe_$arg.log" 2>&1 \
        || { echo "probe failed"; tail -20 "$out/probe_$arg.log"; exit 1; } ;;
    prof)
      (cd "$out" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d prof -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --variants 0 --cpu-seconds 0 --cfg3-strong 0 $arg \
        > prof.log 2>&1) || { echo "prof failed"; tail -20 "$out/prof.log"; exit 1; } ;;
    pmc)  # pmc:<workload>,<dtype>[,<extra PMC set>] -> $out/pmc_<workload>_<dtype>/ (FETCH, WRITE, MFMA/VALU passes)
      IFS=, read -r wl dt extra <<< "$arg"
      sets=$'FETCH_SIZE\nWRITE_SIZE\nSQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE'
      [ -n "$extra" ] && sets="$sets"$'\n'"${extra//+/ }"
      CMD="python bench.py --workload $wl --dtype $dt --steps 3 --warmup 1 --cpu-seconds 0 --variants 0 --cfg3-strong 0" \
        PMC_SETS="$sets" timeout -k 10 600 bash tools/pmc.sh "$dt" "$out/pmc_${wl}_$dt" > "$out/pmc_${wl}_$dt.log" 2>&1 \
        || { echo "pmc failed"; cat "$out/pmc_${wl}_$dt/passes.txt"; exit 1; } ;;
    stamps)  # stamps:mimo_setup -> per-stage cycles of mimo_setup_kernel on the debug library built here
             # beforehand (SRC=mpcq_mimo.hip DBGDIR=tools/dbg_r05 bash tools/build_dbg.sh)
      MPCQ_LIBRARY=tools/dbg_r05/libmpcq.so timeout -k 10 300 python -u tools/mimo_setup_stamps.py > "$out/stamps_$arg.log" 2>&1 \
        || { echo "stamps failed"; tail "$out/stamps_$arg.log"; exit 1; } ;;
    tstamps)  # tstamps:<dtype> -> per-wave stage stamps of the tile kernel (debug library tools/dbg_r05t, built
              # here: SRC=mpcq_tile_f64.hip DBGDIR=tools/dbg_r05t bash tools/build_dbg.sh MPCQ_INFO_STAMPS)
      MPCQ_LIBRARY=tools/dbg_r05t/libmpcq.so MPCQ_TILE_STAMPS="$out/tstamps_$arg.bin" timeout -k 10 300 \
        python bench.py --dtype $arg --steps 1 --warmup 1 --cpu-seconds 0 --variants 0 > "$out/tstamps_bench_$arg.json" 2>&1 \
        && python tools/stamps.py "$out/tstamps_$arg.bin" > "$out/tstamps_$arg.txt" 2>&1 \
        || { echo "tstamps failed"; tail "$out/tstamps_bench_$arg.json"; exit 1; } ;;
    sstamps)  # sstamps:<dtype> -> per-wave stamps of the one-launch stream (config 5; debug library tools/dbg_r06s,
              # built here: SRC=mpcq_tile_f64.hip DBGDIR=tools/dbg_r06s bash tools/build_dbg.sh MPCQ_INFO_STAMPS)
      MPCQ_LIBRARY=tools/dbg_r06s/libmpcq.so MPCQ_TILE_STAMPS="$out/sstamps_$arg.bin" timeout -k 10 300 \
        python bench.py --workload stream --dtype $arg --steps 1 --warmup 1 --cpu-seconds 0 --variants 0 > "$out/sstamps_bench_$arg.json" 2>&1 \
        && python tools/stamps.py "$out/sstamps_$arg.bin" > "$out/sstamps_$arg.txt" 2>&1 \
        || { echo "sstamps failed"; tail "$out/sstamps_bench_$arg.json"; exit 1; } ;;
    calib)  # WRITE_SIZE calibration of the finalize's store patterns (tools/calib/write_calib.hip, built here)
      (cd "$out" && timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d calib -o run -- "$GRAFT_REPO_ROOT/tools/calib/write_calib" \
        > calib.log 2>&1) || { echo "calib failed"; tail "$out/calib.log"; exit 1; } ;;
    envbench)  # envbench:VAR=val,<bench args with _ for spaces> -> 3 bench lines with the test hook set
      IFS=, read -r ev rest <<< "$arg"
      for r in 1 2 3; do
        env "$ev" timeout -k 10 300 python -u bench.py ${rest//_/ } --cpu-seconds 0 --variants 0 > "$out/eb_${ev}_$r.json" 2> "$out/eb.err" \
          || { echo "envbench failed"; tail -20 "$out/eb.err"; exit 1; }
      done ;;
    pmcw)  # pmcw:VAR=val,<dtype> -> one WRITE_SIZE pass of the cfg2 bench with the test hook set
      IFS=, read -r ev dt <<< "$arg"
      env "$ev" CMD="python bench.py --dtype $dt --steps 3 --warmup 1 --cpu-seconds 0 --variants 0 --cfg3-strong 0" PMC_SETS=WRITE_SIZE \
        timeout -k 10 300 bash tools/pmc.sh "$dt" "$out/pmcw_${ev}_$dt" > "$out/pmcw_${ev}_$dt.log" 2>&1 \
        || { echo "pmcw failed"; cat "$out/pmcw_${ev}_$dt/passes.txt"; exit 1; } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $step ok"
done
