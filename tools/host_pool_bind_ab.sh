#!/bin/bash
# Same-box A/B: the host worker pools bound to the GPU's NUMA node (default)
# vs unbound (HEC_HOST_POOL_BIND=0), alternating processes: the batched
# degraded read (tools/bench_intervals.py --c-abi-only, median of 7 calls) and
# pageable host batches (tools/pageable_multi_probe.py --single).
# usage: tools/host_pool_bind_ab.sh OUT_JSONL [PAIRS]
set -o pipefail
out=${1:?out.jsonl}
pairs=${2:-3}
: > "$out"
for i in $(seq 1 "$pairs"); do
    for b in 1 0; do
        HEC_HOST_POOL_BIND=$b timeout -k 10 150 python tools/bench_intervals.py --c-abi-only --reps 7 >> "$out" || exit $?
        HEC_HOST_POOL_BIND=$b timeout -k 10 150 python tools/pageable_multi_probe.py --single --rounds 1 \
            | sed "s/^{/{\"host_pool_bind\": \"$b\", /" >> "$out" || exit $?
    done
done
