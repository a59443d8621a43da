# C2 bench (stages) + one PMC pass on the tokenizer; usage: bash tools/run_tok_pmc.sh <tag>
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines --steps 3 --warmup 1 > $O/bench.log 2>&1 || exit 1
bash tools/pmc_pass.sh $1 base tokenize_batch SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM || exit 2
echo ALLDONE
