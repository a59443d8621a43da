set -o pipefail
mkdir -p gpurun_out/r04a
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_loader.py tests/test_collate_gpu.py tests/test_balance.py tests/test_output_gpu.py > gpurun_out/r04a/tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 240 python -u bench.py --workload c5 > gpurun_out/r04a/c5_fork.log 2>&1 || exit 1
echo c5 fork done
timeout -k 10 240 python -u bench.py --workload c5 --c5-mp forkserver > gpurun_out/r04a/c5_forkserver.log 2>&1 || exit 1
echo c5 forkserver done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04a/prof_native -o native -- python3 bench.py --rng native --steps 2 --warmup 1 --no-alt-rng --no-extra-lines --no-segmented-line --no-cpu-baseline > gpurun_out/r04a/native.log 2>&1 || exit 1
echo native done
