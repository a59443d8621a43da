# HIP API + kernel trace of a short C5 run (which API calls block the training step's host);
# usage: bash tools/run_c5_hiptrace.sh <tag>
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace -d $O/trace -o c5 -- python3 bench.py --workload c5 --steps 30 --warmup 5 > $O/trace.out 2>&1 || exit 1
python3 tools/hip_api_summary.py $O/trace > $O/hip_api.txt || exit 2
rm -rf $O/trace
echo ALLDONE
