# Run-to-run spread of the default bench on one box: 3 runs back to back.
TAG=${1:-rep}
mkdir -p gpurun_out/$TAG; : > gpurun_out/$TAG/bench_runs.jsonl
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras >> gpurun_out/$TAG/bench_runs.jsonl 2>/dev/null || exit 1
done
