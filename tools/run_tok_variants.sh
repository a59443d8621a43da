# Tokenizer throughput of library variants: bash tools/run_tok_variants.sh <out> <bytes> <variant>...
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
B=$2
shift 2
mkdir -p $O
for v in "$@"; do
  if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
  echo "== $v" >> $O/tok.log
  LDDL_AMD_LIB=$L timeout -k 10 300 python -u tools/tok_bench.py $B >> $O/tok.log 2>&1 || exit 1
done
echo ALLDONE
