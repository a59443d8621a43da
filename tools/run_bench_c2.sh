cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-b}
mkdir -p $O
timeout -k 10 500 python -u bench.py > $O/bench_c2.log 2>&1 || exit 1
echo ALLDONE
