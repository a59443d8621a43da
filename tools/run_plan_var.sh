# pair parity tests (default library) + C2 bench per (library variant, partition size)
# usage: bash tools/run_plan_var.sh <tag> "<variants>" "<partition sizes>"
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_pairs_gpu.py tests/test_output_gpu.py tests/test_native_gpu.py > $O/tests.log 2>&1 || exit 1
for v in $2; do
  if [ "$v" = base ]; then L=lddl_amd/_lib/liblddl_amd.so; else L=lddl_amd/_lib_$v/liblddl_amd.so; fi
  for p in $3; do
    LDDL_AMD_LIB=$L timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-alt-rng --no-segmented-line --no-extra-lines --partition-bytes $p > $O/bench_${v}_$p.log 2>&1 || exit 2
    echo "$v $p $(grep -o '"stages_ms": {[^}]*}' $O/bench_${v}_$p.log)" >> $O/summary.txt
  done
done
echo ALLDONE
