# Kernel + memory-copy trace of one bench step: bash tools/run_trace_copies.sh <outdir> <bench args...>
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace -o b -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-alt-rng --no-extra-lines --no-segmented-line "$@" > $O/trace.log 2>&1 || exit 1
echo ALLDONE
