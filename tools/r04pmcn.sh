set -o pipefail
cd /root/repo
export TMPDIR=/tmp
bash tools/prof_counters.sh r04pmcn --rng native || exit 1
echo ALLDONE
