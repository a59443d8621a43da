set -o pipefail
mkdir -p gpurun_out/r04w
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py > gpurun_out/r04w/tests.log 2>&1 || exit 1
echo tests ok
bash tools/run_trace_copies.sh r04w/trace || exit 1
B="python3 bench.py --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines --steps 1 --warmup 0"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r04w/fetch -o p -- $B > gpurun_out/r04w/fetch.log 2>&1 || exit 4
python3 tools/pmc_summary.py $(find gpurun_out/r04w/fetch -name "*.db" | head -1) > gpurun_out/r04w/fetch.txt || exit 7
echo ALLDONE
