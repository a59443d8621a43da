# round 6 final build: PMC passes + kernel trace, the PMC JSON written into profiles/ here too (so this
# call's bench lines read the passes of their own build), GPU tests, smoke, C2 / C3 / C4 bench lines
# usage: bash tools/r06_final_all2.sh <tag1> <tag2> <pmc json name> <git head>
cd /root/repo
bash tools/prof_counters.sh $1 || { echo PMC_FAILED; exit 1; }
python3 tools/make_pmc_json.py gpurun_out/$1/pmc 10000000000 "$1: C2 10 GB step, round-6 final build" $4 > profiles/$3 || exit 2
cp profiles/$3 gpurun_out/$1/$3
bash tools/r06_gpu_all.sh $1 || exit 3
WITH_C4=1 bash tools/r06_final2.sh $2 || exit 4
echo ALLDONE_FINAL
