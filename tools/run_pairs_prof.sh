# pair parity tests + a short C2 bench + a kernel trace of it; usage: bash tools/run_pairs_prof.sh <tag>
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py tests/test_native_gpu.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/trace.log 2>&1 || exit 3
echo ALLDONE
