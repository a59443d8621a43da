# C2 bench at larger batches per step (more partitions in flight for the replay planner)
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-bsweep}
mkdir -p $O
for gb in 6 8; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-alt-rng --no-segmented-line --steps 3 --batch-bytes $((gb << 30)) > $O/c2_${gb}g.log 2>&1 || exit 1
done
echo ALLDONE
