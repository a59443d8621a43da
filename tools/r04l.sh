# tokenizer cost breakdown: tok_bench over 2 GiB on the product library and phase-skipping variants
set -o pipefail
mkdir -p gpurun_out/r04l
export TMPDIR=/tmp
for v in base tnob tnoab tnop tcls; do
  if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
  LDDL_AMD_LIB=$L timeout -k 10 300 python -u tools/tok_bench.py 2147483648 > gpurun_out/r04l/tok_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r04l/tok_$v.log)"
done
