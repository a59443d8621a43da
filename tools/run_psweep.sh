# C2 bench over partition sizes (replay planner occupancy); usage: bash tools/run_psweep.sh <tag> sizes...
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
for p in "$@"; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines --partition-bytes $p > $O/bench_p$p.log 2>&1 || exit 1
done
echo ALLDONE
