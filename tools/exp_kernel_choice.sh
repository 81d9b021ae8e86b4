cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/exp && rm -f gpurun_out/exp/*
for k in tile wave; do
  MPCQ_KERNEL=$k timeout -k 10 120 python bench.py --workload stream --steps 2 --warmup 1 --cpu-seconds 0 --ctrl-steps 300 > gpurun_out/exp/stream_$k.json 2>>gpurun_out/exp/err || exit $?
  for b in 4096 16384 32768; do
    MPCQ_KERNEL=$k timeout -k 10 120 python bench.py --batch $b --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/exp/cfg2_${b}_$k.json 2>>gpurun_out/exp/err || exit $?
  done
done
