# A/B of library variants on one box: pair parity tests on each variant, then a short C2 bench
# per variant (stages_ms summary). usage: bash tools/run_ab.sh <tag> <variant>... (base = lddl_amd/_lib)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
for v in "$@"; do
  if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
  if [ "$v" != base ]; then
    LDDL_AMD_LIB=$L timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu ${AB_TESTS:-tests/test_pairs_gpu.py tests/test_output_gpu.py} > $O/tests_$v.log 2>&1 || exit 1
  fi
done
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
    LDDL_AMD_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_${v}_$r.log 2>&1 || exit 2
    echo "$v r$r $(grep -o '"stages_ms": {[^}]*}' $O/bench_${v}_$r.log)" >> $O/summary.txt
  done
done
echo ALLDONE
