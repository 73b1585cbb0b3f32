# One GPU call of round evidence, in the driver's order: the bench FIRST (the
# driver's BENCH line is the first GPU process on its box), directly under
# rocprofv3 --kernel-trace --stats so its trace and its line are one process
# (tools/trace_summary.py -> trace_summary.json), then the -m gpu
# tests, smoke(), the C-ABI bench, rocprofv3 kernel trace + PMC passes of the
# bench (tools/profile.sh) and of the mixed workload (tools/profile_mixed.sh),
# and the counter calibration on known bytes (tools/pmc_calib.sh). Each step
# under its own time limit, steps chained so the first failure ends the call.
# Outputs in gpurun_out/$TAG; summaries: pmc_traffic.json (calibrated),
# pmc_sq_wave_states.json, pmc_mixed_workload.json.
set -e
TAG=${1:-ev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
python3 tools/trace_summary.py $OUT/trace/run_kernel_trace.csv $OUT/bench.json $OUT/trace_summary.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 120 ./build/cabi_bench > $OUT/cabi_bench.json 2>&1
bash tools/profile.sh $TAG/prof
bash tools/profile_mixed.sh $TAG/profmix
bash tools/pmc_calib.sh $TAG/calib
python tools/pmc_summary.py $OUT/prof $OUT/pmc_traffic.json $OUT/calib > /dev/null
python tools/sq_summary.py $OUT/prof/pmc_sq/run_counter_collection.csv $OUT/pmc_sq_wave_states.json > /dev/null
python tools/pmc_mixed_summary.py $OUT/profmix $OUT/pmc_mixed_workload.json > /dev/null
