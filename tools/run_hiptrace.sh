# HIP API + kernel trace of a short bench run (finds host-side stalls: allocations, syncs); the
# database is summarised on the box and removed (it exceeds the 64 MiB pull limit).
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d /tmp/ht_trace -o b -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt-rng "$@" > $O/trace.log 2>&1 || exit 1
python3 tools/hip_api_summary.py /tmp/ht_trace > $O/summary.txt 2>&1 || exit 2
echo ALLDONE
