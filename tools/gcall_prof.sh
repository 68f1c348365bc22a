mkdir -p gpurun_out
bash tools/profile.sh r03s5c4 --no-extra || exit 6
