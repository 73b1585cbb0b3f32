# rocprofv3 evidence for the bench command (run on the GPU box from the repo root):
#   1) kernel trace + stats of the default bench (kernel durations); the
#      timed dispatches are summarised beside the same process's HIP-event
#      times by tools/trace_summary.py ($OUT/trace_summary.json)
#   2) FETCH_SIZE pass, 3) WRITE_SIZE pass -- separate PMC passes (gfx950 TCC slots),
#      restricted to the RS kernels, 4) SQ wave-state + GRBM pass (tools/sq_summary.py).
#   Outputs under gpurun_out/$TAG/.
set -e
TAG=${1:-prof}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $OUT/bench_trace.log 2>&1
python3 tools/trace_summary.py $OUT/trace/run_kernel_trace.csv $OUT/bench_trace.log $OUT/trace_summary.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex "rs104|rs_apply" --output-format csv \
    -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $OUT/bench_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --kernel-include-regex "rs104|rs_apply" --output-format csv \
    -d $OUT/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $OUT/bench_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --kernel-include-regex "rs104" --output-format csv \
    -d $OUT/pmc_sq -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $OUT/bench_sq.log 2>&1
find $OUT -name "*.csv" | sort
