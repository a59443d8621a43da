# last A/B of the round + checkpoint (full GPU tests, smoke, default bench) of the default build
cd /root/repo
export TMPDIR=/tmp
bash tools/ab.sh r03p11 t8 base || exit 1
bash tools/run_ckpt.sh r03c6 || exit 2
echo ALLDONE
