cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-t}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || exit 1
echo ALLDONE
