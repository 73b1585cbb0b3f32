# The driver's round-end order on one fresh lease: the bench FIRST (the
# driver's BENCH line is the first GPU process on its box), then the GPU
# tests and smoke(). Each step under its own time limit, chained with set -e.
set -e
TAG=${1:-final}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
