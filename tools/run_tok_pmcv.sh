# tokenizer PMC pass (instruction mix) per library variant; usage: bash tools/run_tok_pmcv.sh <tag> v1 v2 ...
cd /root/repo
T=$1; shift
for v in "$@"; do
  bash tools/pmc_pass.sh $T $v tokenize_batch SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM || exit 1
done
echo ALLDONE
