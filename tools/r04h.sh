set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04h
bash tools/pmc_pass.sh r04h/tlb base gather_kernel TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum || exit 1
bash tools/pmc_pass.sh r04h/sq base gather_kernel SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_INSTS_SALU || exit 1
