# One GPU call: -m gpu tests, default bench, rocprofv3 kernel trace + PMC
# passes (tools/profile.sh), under per-step time limits. Outputs in gpurun_out/$TAG.
set -e
TAG=${1:-ev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 120 ./build/cabi_bench > $OUT/cabi_bench.json 2>&1
bash tools/profile.sh $TAG
python tools/pmc_summary.py $OUT $OUT/pmc_traffic.json > /dev/null
python tools/sq_summary.py $OUT/pmc_sq/run_counter_collection.csv $OUT/pmc_sq_wave_states.json > /dev/null
