cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/st1
bash tools/gpu_stamps.sh st1 || exit $?
MPCQ_LIBRARY=$PWD/tools/dbg/libmpcq.so bash tools/gpu_stamps.sh st1w || exit $?
python tools/wave_stamps.py gpurun_out/st1w/stamps.bin > gpurun_out/st1w/wave.txt
