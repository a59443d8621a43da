# Default bench (C2 + alt RNG + CPU baseline) and C4 (4 steps), JSON lines to gpurun_out/<dir>.
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-bp}
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/c2.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --workload c4 --no-cpu-baseline --steps 4 > $O/c4.log 2>&1 || exit 2
echo ALLDONE
