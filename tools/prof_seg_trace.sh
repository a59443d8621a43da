cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o b -- python3 tools/seg_bench.py 2 > $O/trace.log 2>&1 && echo ALLDONE
