# C2 bench with 1 / 2 / 4 pipelined chunks; usage: bash tools/run_chunks.sh <tag>
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for c in 1 2 4; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines --chunks $c > $O/bench_chunks$c.log 2>&1 || exit 1
done
echo ALLDONE
