# one rocprofv3 --pmc pass of one C2 bench step on a library variant, summarised for one kernel
# usage: bash tools/pmc_pass.sh <tag> <lib variant|base> <kernel-substring> <counters...>
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1; V=$2; K=$3; shift 3
mkdir -p $O
if [ "$V" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$V/liblddl_amd.so; fi
export LDDL_AMD_LIB=$L
timeout -s KILL 300 rocprofv3 --pmc "$@" -d $O/pmc_$V -o p -- python3 bench.py --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines --steps 1 --warmup 0 > $O/pmc_$V.log 2>&1 || exit 1
python3 tools/pmc_summary.py $(find $O/pmc_$V -name "*.db" | head -1) $K > $O/pmc_$V.txt || exit 2
echo ALLDONE
