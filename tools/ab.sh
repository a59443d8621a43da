# Parity tests on the default library, then a quick C2 bench A/B of library variants (2 rounds).
# usage: bash tools/ab.sh <tag> <variant>...   (base = lddl_amd/_lib, else lddl_amd/_lib_<v>)
# AB_TESTS overrides the test files (default: pair + output tests); AB_TESTS=none skips them;
# AB_TEST_VARIANTS lists variant libraries to test as well.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
T=${AB_TESTS:-tests/test_pairs_gpu.py tests/test_output_gpu.py}
if [ "$T" != none ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu $T > $O/tests.log 2>&1 || exit 1
  for v in $AB_TEST_VARIANTS; do  # also test these variant libraries
    LDDL_AMD_LIB=lddl_amd/_lib_$v/liblddl_amd.so timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu $T > $O/tests_$v.log 2>&1 || exit 1
  done
fi
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
    LDDL_AMD_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_${v}_$r.log 2>&1 || exit 2
    echo "$v r$r $(grep -o '"stages_ms": {[^}]*}' $O/bench_${v}_$r.log)" >> $O/summary.txt
  done
done
echo ALLDONE
