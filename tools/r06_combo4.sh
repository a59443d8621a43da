cd /root/repo
bash tools/r06_ppw.sh r06u || exit $?
bash tools/r06_gd.sh r06v || exit $?
