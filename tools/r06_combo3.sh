# round 6: planner stamps + timeline (diagnostic library), then C4, C5 and the CLI end to end
cd /root/repo
bash tools/run_stamps.sh ${1:-r06t} || exit $?
SKIP_C3=1 bash tools/r06_configs.sh ${2:-r06s} || exit $?
