# quick A/B of library variants: C2 bench stages per variant, 2 rounds (no tests; parity-neutral
# changes only). usage: bash tools/run_ab_quick.sh <tag> <variant>...
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
    LDDL_AMD_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_${v}_$r.log 2>&1 || exit 2
    echo "$v r$r $(grep -o '"stages_ms": {[^}]*}' $O/bench_${v}_$r.log)" >> $O/summary.txt
  done
done
echo ALLDONE
