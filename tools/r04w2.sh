set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r04w2
B="python3 bench.py --workload c3 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines --steps 1 --warmup 0"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/r04w2/c1 -o p -- $B > gpurun_out/r04w2/c1.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r04w2/fetch -o p -- $B > gpurun_out/r04w2/fetch.log 2>&1 || exit 2
for k in c1 fetch; do python3 tools/pmc_summary.py $(find gpurun_out/r04w2/$k -name "*.db" | head -1) > gpurun_out/r04w2/$k.txt || exit 3; done
echo ALLDONE
