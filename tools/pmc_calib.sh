# FETCH_SIZE / WRITE_SIZE calibration: build/membench_calib
# runs known-byte streams at 8 and 16 B per lane, then the shipped RS(10,4)
# encode and 4-erasure decode, in one process; one rocprofv3 pass per counter.
# Summarise with tools/pmc_summary.py <bench prof dir> <out.json> gpurun_out/$TAG.
set -e
TAG=${1:-calib}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 120 ./build/membench_calib calib > $OUT/plain.jsonl 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  d=pmc_fetch; [ $c = WRITE_SIZE ] && d=pmc_write
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --kernel-include-regex "k_cal|rs104" --output-format csv \
      -d $OUT/$d -o run -- ./build/membench_calib calib > $OUT/$d.jsonl 2>&1
done
