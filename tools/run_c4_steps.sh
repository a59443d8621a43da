cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/n4
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --steps 4 --rng native > gpurun_out/n4/c4n.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu-baseline --steps 4 > gpurun_out/n4/c4r.log 2>&1 || exit 2
echo ALLDONE
