# C2 bench with arena allocation tracing (which steps allocate); usage: bash tools/run_arena_dbg.sh <tag>
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
LDDL_ARENA_DEBUG=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench.log 2>&1 || exit 1
echo ALLDONE
