# planner region stamps (diagnostic library, s_memtime sums per region); usage: bash tools/run_stamps.sh <tag>
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
LDDL_AMD_LIB=lddl_amd/_lib_diag/liblddl_amd.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 1 --warmup 0 --no-alt-rng --no-segmented-line --no-extra-lines > $O/stamps.log 2>&1 || exit 1
echo ALLDONE
