# checkpoint (GPU tests, smoke, default bench) + PMC passes of the same build; usage: bash tools/run_ckpt_pmc.sh
cd /root/repo
export TMPDIR=/tmp
bash tools/run_ckpt.sh r03c7 || exit 1
bash tools/prof_counters.sh r03t || exit 2
echo ALLDONE
