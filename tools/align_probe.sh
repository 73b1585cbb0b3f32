# VERDICT r04 item 1(c), run once per fresh lease: does a 1 GiB-aligned batch
# base remove the first process's extra UTCL1 translation misses? Processes in
# the order given (e.g. "a1g torch a1g torch"), each a bench.py run under one
# rocprofv3 pass of the TCP UTCL1 counters (RS kernels only); arm a1g =
# --base-align 1073741824, torch = the allocator's own base. Summarise with
# tools/tlb_summary.py gpurun_out/$TAG.
set -e
TAG=${1:-align}
ARMS=${2:-"a1g torch a1g torch"}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for arm in $ARMS; do
  i=$((i+1))
  flag=""; [ "$arm" = a1g ] && flag="--base-align 1073741824"
  echo "$arm" > $OUT/arm_$i.txt
  timeout -s KILL 200 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
      TCP_UTCL1_REQUEST_sum TCP_UTCL1_THRASHING_STALL_sum --kernel-trace --kernel-include-regex "rs104" \
      --output-format csv -d $OUT/p$i -o run -- \
      python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-packed $flag > $OUT/bench_$i.log 2>&1
done
