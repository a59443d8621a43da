# C5 training step with the loader in the main process (one DataLoader worker per bin), and the --gpus 2
# launcher rehearsal on one GPU; usage: bash tools/run_r03p8.sh <tag>
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u bench.py --workload c5 --steps 100 --warmup 10 --c5-workers 1 > $O/bench_c5_w1.log 2>&1 || exit 1
LDDL_BENCH_SHARE_DEVICE=1 timeout -k 10 600 python -u bench.py --gpus 2 --steps 2 --warmup 1 > $O/bench_n2.log 2>&1 || exit 2

bash tools/prof_counters.sh $1_pmc || exit 3
echo ALLDONE
