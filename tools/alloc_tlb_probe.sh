# Alternating processes: the bench batch from torch's allocator vs one
# physically contiguous allocation, each under one rocprofv3 pass of the TCP
# UTCL1 translation counters (RS kernels only). Summarise with
# tools/alloc_tlb_summary.py.
set -e
TAG=${1:-alloc_tlb}
R=${2:-4}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
for r in $(seq 1 $R); do
  for kind in torch contiguous; do
    timeout -s KILL 150 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum \
        TCP_UTCL1_REQUEST_sum TCP_UTCL1_THRASHING_STALL_sum --kernel-trace --kernel-include-regex "rs104" \
        --output-format csv -d $OUT/${kind}_$r -o run -- \
        python3 tools/alloc_tlb_probe.py --kind $kind > $OUT/${kind}_$r.log 2>&1
  done
done
