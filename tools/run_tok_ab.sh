# tokenizer A/B: parity tests against a variant library, then 2-GiB timing of base and variants
# usage: bash tools/run_tok_ab.sh <tag> <variant> [more variants]
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
for v in "$@"; do
  LDDL_AMD_LIB=lddl_amd/_lib_$v/liblddl_amd.so timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_tokenize_gpu.py > $O/tests_$v.log 2>&1 || exit 1
done
for v in base "$@"; do
  if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
  LDDL_AMD_LIB=$L timeout -k 10 200 python -u tools/tok_bench.py 2147483648 > $O/tok_$v.log 2>&1 || exit 2
done
echo ALLDONE
