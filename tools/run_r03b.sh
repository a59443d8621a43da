# round-3 checkpoint: full GPU tests, then C2 (short) and C3 (10 GB, streamed balance) bench lines
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra-lines --no-segmented-line > $O/bench_c2.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline --no-segmented-line --no-alt-rng > $O/bench_c3.log 2>&1 || exit 3
echo ALLDONE
