set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r04c4n2
LDDL_BENCH_SHARE_DEVICE=1 timeout -k 10 600 python -u bench.py --workload c4 --gpus 2 --batch-bytes 2000000000 --steps 3 > gpurun_out/r04c4n2/bench_c4_n2_share.log 2>&1 || exit 1
echo ALLDONE
