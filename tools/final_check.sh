# The driver's round-end order on one fresh lease: the bench FIRST (the
# driver's BENCH line is the first GPU process on its box), then the GPU
# tests and smoke(). Each step under its own time limit, chained with set -e.
# The bench runs under rocprofv3 --kernel-trace --stats (the program directly
# after --, no wrapper), so the committed trace and kernel stats are of the
# SAME process as the committed bench line: tools/trace_summary.py sets the
# timed dispatches' mean duration beside that process's HIP-event times
# (VERDICT r05 "next" 1).
set -e
TAG=${1:-final}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
python3 tools/trace_summary.py $O/trace/run_kernel_trace.csv $O/bench.json $O/trace_summary.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
