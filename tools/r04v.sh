set -o pipefail
mkdir -p gpurun_out/r04v
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_native_gpu.py -k "wide or bit_exact" > gpurun_out/r04v/tests.log 2>&1 || exit 1
echo tests ok
B="python3 bench.py --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines --steps 1 --warmup 0"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r04v/fetch -o p -- $B > gpurun_out/r04v/fetch.log 2>&1 || exit 4
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r04v/write -o p -- $B > gpurun_out/r04v/write.log 2>&1 || exit 5
for k in fetch write; do python3 tools/pmc_summary.py $(find gpurun_out/r04v/$k -name "*.db" | head -1) > gpurun_out/r04v/$k.txt || exit 7; done
echo ALLDONE
