# tokenizer A/B: GPU tokenizer tests on each variant, then tok_bench (2 GiB) per variant, 2 rounds
# usage: bash tools/run_tok_ab.sh <tag> <variant>...   (base = lddl_amd/_lib)
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
for v in "$@"; do
  if [ "$v" = base ]; then continue; fi
  LDDL_AMD_LIB=lddl_amd/_lib_$v/liblddl_amd.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_tokenize_gpu.py > $O/tests_$v.log 2>&1 || exit 1
done
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
    echo "== $v r$r" >> $O/tok.log
    LDDL_AMD_LIB=$L timeout -k 10 300 python -u tools/tok_bench.py 2147483648 >> $O/tok.log 2>&1 || exit 2
  done
done
echo ALLDONE
