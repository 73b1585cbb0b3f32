# Does the slow-allocation mode (decode ~0.744 of peak instead of ~0.78) go
# with address-translation misses? K bench processes (fresh allocations),
# each under one rocprofv3 PMC pass of the TCP UTCL1 counters, restricted to
# the RS kernels; each process prints its own bench line (HIP events).
# Summarise with tools/tlb_summary.py.
set -e
TAG=${1:-tlb}
K=${2:-6}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
for i in $(seq 1 $K); do
  timeout -s KILL 200 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
      TCP_UTCL1_REQUEST_sum TCP_UTCL1_THRASHING_STALL_sum --kernel-trace --kernel-include-regex "rs104" \
      --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-packed > $OUT/bench_$i.log 2>&1
done
find $OUT -name "*counter_collection.csv" | sort
