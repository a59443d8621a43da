# A/B of a runtime environment variable on the C2 bench stages (2 rounds, same box).
# usage: bash tools/run_env_ab.sh <tag> <VAR> <value>...   (value "-" = unset)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
VAR=$2
shift 2
mkdir -p $O
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = - ]; then unset $VAR; else export $VAR=$v; fi
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_${v}_$r.log 2>&1 || exit 2
    echo "$VAR=$v r$r $(grep -o '"stages_ms": {[^}]*}' $O/bench_${v}_$r.log)" >> $O/summary.txt
  done
done
unset $VAR
echo ALLDONE
