# Run-to-run spread of the default bench on one box: N runs back to back (default 3).
TAG=${1:-rep}
mkdir -p gpurun_out/$TAG; : > gpurun_out/$TAG/bench_runs.jsonl
for i in $(seq 1 ${N:-3}); do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras >> gpurun_out/$TAG/bench_runs.jsonl 2>/dev/null || exit 1
done
