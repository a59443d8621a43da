set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r04tk
for v in base sf128 sf256 ch64 ch256; do
  if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
  LDDL_AMD_LIB=$L timeout -k 10 300 python -u tools/tok_bench.py 2147483648 > gpurun_out/r04tk/tok_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r04tk/tok_$v.log)"
done
