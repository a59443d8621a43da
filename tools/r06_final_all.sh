cd /root/repo
bash tools/r06_final1.sh ${1:-r06f1} || exit $?
WITH_C4=1 bash tools/r06_final2.sh ${2:-r06f2} || exit $?
