# usage: bash tools/gcall_ab.sh TAG CFG NAME1 NAME2 ...   (A/B builds from build/ab, interleaved in one process)
mkdir -p gpurun_out
TAG=$1; CFG=$2; shift 2
for cfg in ${CFG//,/ }; do
  timeout -k 10 400 python3 -u tools/ab.py run cfg=$cfg "$@" > gpurun_out/ab_${TAG}_${cfg}.log 2>&1 || exit 3
done
