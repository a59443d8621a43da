set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r04c3f
timeout -k 10 900 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-segmented-line --no-alt-rng > gpurun_out/r04c3f/bench_c3.log 2>&1 || exit 1
echo ALLDONE
