# Default bench at shard pad 64 KiB vs packed shards, alternating (each run a
# fresh process and allocation, so placement spread is in both arms).
TAG=${1:-abpad}
mkdir -p gpurun_out/$TAG; : > gpurun_out/$TAG/runs.jsonl
for p in ${ORDER:-65536 0 65536 0 0 65536}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --shard-pad $p >> gpurun_out/$TAG/runs.jsonl 2>/dev/null || exit 1
done
