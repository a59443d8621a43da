# pair parity tests + a short C2 bench; usage: bash tools/run_pairs_check.sh <tag>
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py tests/test_native_gpu.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench.log 2>&1 || exit 2
echo ALLDONE
