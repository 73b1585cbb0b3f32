# The first GPU process after a box is acquired: does one allocate/touch/free
# cycle of the batch's size before the real allocation change its speed and
# its translation misses? FIRST = the first process's arm (pre / plain), then
# three more processes alternating plain / pre. UTCL1 PMC pass per process.
set -e
TAG=${1:-first}
FIRST=${2:-pre}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for arm in $FIRST plain pre plain; do
  i=$((i+1))
  flag=""; [ "$arm" = pre ] && flag="--precycle"
  timeout -s KILL 150 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
      TCP_UTCL1_REQUEST_sum TCP_UTCL1_THRASHING_STALL_sum --kernel-trace --kernel-include-regex "rs104" \
      --output-format csv -d $OUT/p$i -o run -- \
      python3 tools/alloc_tlb_probe.py --kind torch $flag > $OUT/p$i.log 2>&1
done
