# rehearsal of bench.py's N > 1 path on a one-GPU box: `bench.py --gpus 2` launches 2 ranks itself
# (launch_command), sharing cuda:0 over gloo (LDDL_BENCH_SHARE_DEVICE); usage: bash tools/run_bench_n2.sh <tag>
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
LDDL_BENCH_SHARE_DEVICE=1 timeout -k 10 600 python3 bench.py --gpus 2 --steps 2 --warmup 1 > $O/bench_n2.log 2>&1 || exit 1
echo ALLDONE
