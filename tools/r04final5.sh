set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r04f5
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04f5/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f5/smoke.log 2>&1 || exit 2
echo ALLDONE
