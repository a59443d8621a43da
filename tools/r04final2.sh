set -o pipefail
cd /root/repo
export TMPDIR=/tmp
bash tools/prof_counters.sh r04pmc2 || exit 1
echo pmc ok
bash tools/run_full.sh r04f2 || exit 2
echo full ok
bash tools/run_trace_copies.sh r04f2/trace_native --rng native || exit 3
echo ALLDONE
