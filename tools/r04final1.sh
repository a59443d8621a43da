set -o pipefail
cd /root/repo
export TMPDIR=/tmp
bash tools/run_full.sh r04f1 || exit 1
echo full ok
LDDL_BENCH_SHARE_DEVICE=1 timeout -k 10 600 python -u bench.py --workload c4 --gpus 2 --batch-bytes 2000000000 --steps 3 > gpurun_out/r04f1/bench_c4_n2_share.log 2>&1 || exit 2
echo c4 n2 ok
bash tools/run_trace_copies.sh r04f1/trace_native --rng native || exit 3
echo ALLDONE
