# usage: T=tag CFG=c3 bash tools/pmc_dec_ab.sh build1 build2 ... : WRITE_SIZE / FETCH_SIZE of one config's decode per
# A/B build (tools/prof_one.py), one rocprofv3 pass per counter; writes gpurun_out/pmc_${T}_<build>_<ctr>/
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in "$@"; do
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${T}_${b}_$c -o pmc -- \
      python3 tools/prof_one.py $b dec ${CFG:-c3} 3 > gpurun_out/pmc_${T}_${b}_$c.log 2>&1 || exit 9
  done
done
