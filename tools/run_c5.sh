# C5 bench (loader + fused collate/masking + training step) and its kernel trace.
# usage: bash tools/run_c5.sh <tag> [extra bench args]
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 400 python -u bench.py --workload c5 --steps 200 --warmup 20 "$@" > $O/bench_c5.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o c5 -- python3 bench.py --workload c5 --steps 100 --warmup 10 "$@" > $O/trace.log 2>&1 || exit 2
echo ALLDONE
