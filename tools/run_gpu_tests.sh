# GPU test suite in one process (+ device facts); usage: bash tools/run_gpu_tests.sh <tag> [pytest -k expr]
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/${1:-t}
mkdir -p $O
timeout -k 10 120 python -c "import torch; p=torch.cuda.get_device_properties(0); print(p); print('shared_memory_per_block', getattr(p, 'shared_memory_per_block', None), getattr(p, 'shared_memory_per_block_optin', None))" > $O/device.txt 2>&1 || exit 1
K=${2:+-k "$2"}
timeout -k 10 900 python -u -m pytest --maxfail=10 -v --timeout 300 --timeout-method thread -m gpu tests $K > $O/gpu_tests.log 2>&1 || exit 2
echo ALLDONE
