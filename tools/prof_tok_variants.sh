# SQ counters of the tokenizer under library variants (tok_bench, 1 GiB): mix per variant.
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
for v in "$@"; do
  if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
  LDDL_AMD_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD -d $O/p_$v -o p -- python3 tools/tok_bench.py 1073741824 > $O/p_$v.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $(find $O/p_$v -name "*.db" | head -1) tokenize_batch > $O/mix_$v.txt || exit 2
done
echo ALLDONE
