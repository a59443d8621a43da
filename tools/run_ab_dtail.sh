set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r02_dt1
mkdir -p $O
L=lddl_amd/_lib_dtail/liblddl_amd.so
LDDL_AMD_LIB=$L timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py > $O/tests_dtail.log 2>&1 || exit 1
for r in 1 2; do
  for v in base d1024 d2048 d4096; do
    if [ $v = base ]; then L=lddl_amd/_lib/liblddl_amd.so; W=2048; else L=lddl_amd/_lib_dtail/liblddl_amd.so; W=${v#d}; fi
    LDDL_DENSE_WG=$W LDDL_AMD_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines > $O/bench_${v}_$r.log 2>&1 || exit 2
    echo "$v r$r $(grep -o '"stages_ms": {[^}]*}' $O/bench_${v}_$r.log)" >> $O/summary.txt
  done
done
echo ALLDONE
