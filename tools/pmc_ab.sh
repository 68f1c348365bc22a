# usage: bash tools/pmc_ab.sh TAG "COUNTERS" build1 build2 ... ; writes gpurun_out/pmc_TAG_<build>/
set -e
tag=$1; ctrs=$2; shift 2
export TMPDIR=/tmp
for b in "$@"; do
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc_${tag}_$b -o pmc -- python3 tools/prof_one.py $b enc c4 3 > gpurun_out/pmc_${tag}_$b.log 2>&1
done
