cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/trc2 -o b -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/trc2.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/trc4 -o b -- python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/trc4.log 2>&1 || exit 2
