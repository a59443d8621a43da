# The other configs' bench lines of the current build: C3 (10 GB, seq 512, 64 bins, balance into
# 8 shards), C4 at 25 GB of text per GPU (5 GB sub-batches), C5 (loader + training step), and the
# end-to-end CLI at 1 GB seq 128; usage: bash tools/run_lines.sh <tag>
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u bench.py --workload c3 --no-cpu-baseline --no-segmented-line --no-alt-rng > $O/bench_c3.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --workload c4 --sub-batch-bytes 5000000000 --steps 2 --warmup 1 --no-cpu-baseline --no-segmented-line --no-alt-rng > $O/bench_c4_25GB.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py --workload c5 --steps 200 --warmup 20 > $O/bench_c5.log 2>&1 || exit 3
timeout -k 10 600 python -u tools/cli_e2e.py --bytes 1e9 --num-blocks 1024 > $O/cli_1GB.log 2>&1 || exit 4
echo ALLDONE
