# round 6 final build, part 1: PMC passes + kernel trace of the C2 step, then the GPU test suite
cd /root/repo
bash tools/prof_counters.sh ${1:-r06z} || { echo PMC_FAILED; exit 1; }
bash tools/r06_gpu_all.sh ${1:-r06z} || exit 2
echo ALLDONE_FINAL1
