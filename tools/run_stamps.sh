cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/st
LDDL_AMD_LIB=lddl_amd/_lib_diag/liblddl_amd.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 1 --warmup 0 --no-alt-rng --no-segmented-line > gpurun_out/st/s.log 2>&1 || exit 1
echo ALLDONE
