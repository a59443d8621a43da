# pair tests (incl. the large-partition planner path) + trim-parity A/B + C5 with cgroup counters
cd /root/repo
export TMPDIR=/tmp
AB_TESTS="tests/test_pairs_gpu.py tests/test_output_gpu.py" bash tools/ab.sh r03p9 t6 base || exit 1
cat /sys/fs/cgroup/cpu.max > gpurun_out/r03p9/cg.txt 2>&1
timeout -k 10 300 python -u bench.py --workload c5 --steps 100 --warmup 10 > gpurun_out/r03p9/c5cg.out 2>&1 || exit 2
echo ALLDONE
