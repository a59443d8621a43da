cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t12.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/time_balance.py > gpurun_out/tb12.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b12_c2.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline > gpurun_out/b12_c4.log 2>&1 || exit 4
