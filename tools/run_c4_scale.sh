# C4-scale runs on one GPU: bench --workload c4 (25 GB of text per GPU, streamed through 5 GB
# sub-batches, peak HBM), then the CLI with --num-shards over the largest corpus the box's disk
# holds with its output (~5 GB in, ~55 GB out); usage: bash tools/run_c4_scale.sh <tag>
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python -u bench.py --workload c4 --sub-batch-bytes 5000000000 --steps 2 --warmup 1 --no-cpu-baseline --no-segmented-line --no-alt-rng > $O/bench_c4_25GB.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/cli_e2e.py --bytes 5e9 --num-blocks 5120 --seq 512 --bin-size 8 --num-shards 8 --files 64 > $O/cli_c4_5GB.log 2>&1 || exit 2
echo ALLDONE
