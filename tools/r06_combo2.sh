cd /root/repo
bash tools/r06_memovar.sh r06r prod mg2 mg4 mg8 || exit $?
bash tools/r06_configs.sh r06q || exit $?
