# round-3 first check: N=2 rehearsal through bench's own launcher, C5 with the sync-free harness
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
LDDL_BENCH_SHARE_DEVICE=1 timeout -k 10 600 python3 bench.py --gpus 2 --steps 2 --warmup 1 --no-alt-rng > $O/bench_n2.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --workload c5 --steps 200 --warmup 20 > $O/bench_c5.log 2>&1 || exit 2
echo ALLDONE
