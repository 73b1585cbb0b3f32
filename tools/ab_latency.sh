# Per-call latency of the drop-in host API (tools/bench_latency.py): pinned
# staging with the kernel's completion flag vs hipStreamSynchronize vs direct
# copies, beside the C oracle, three passes in one call.
TAG=${1:-latab}
mkdir -p gpurun_out/$TAG
for r in 1 2 3; do
  timeout -k 10 200 python tools/bench_latency.py --reps 400 --sizes 1024,4096,16384,65536,262144,1048576 \
    2>/dev/null >> gpurun_out/$TAG/lat.jsonl || exit 1
done
