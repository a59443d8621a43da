set -o pipefail
mkdir -p gpurun_out/r04s
export TMPDIR=/tmp
for c in 1 2 4; do
  timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-alt-rng --no-extra-lines --no-segmented-line --chunks $c > gpurun_out/r04s/chunks$c.log 2>&1 || exit 1
  echo "chunks $c: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r04s/chunks$c.log)"
done
bash tools/run_trace_copies.sh r04s/trace4 --chunks 4 || exit 1
