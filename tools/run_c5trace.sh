cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o c5 -- python3 bench.py --workload c5 --steps 60 --warmup 10 > $O/trace.log 2>&1 || exit 2
echo ALLDONE
