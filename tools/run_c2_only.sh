# default C2 bench (the driver's command) + kernel trace; usage: bash tools/run_c2_only.sh <tag>
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench_c2.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/trace.log 2>&1 || exit 2
echo ALLDONE
