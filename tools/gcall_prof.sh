mkdir -p gpurun_out
bash tools/profile.sh r03s6c4 --no-extra || exit 6
