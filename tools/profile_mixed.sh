# rocprofv3 evidence for the mixed workload (BASELINE config 5, device-resident;
# tools/mixed_probe.py: 512 stripes, 64 KiB..4 MiB, 0..4 erasures): kernel trace
# + stats, then separate FETCH_SIZE and WRITE_SIZE passes restricted to the
# ragged kernels. Summarise with tools/pmc_mixed_summary.py. Outputs under
# gpurun_out/$TAG/.
set -e
TAG=${1:-profmix}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 tools/mixed_probe.py --rounds 2 --reps 5 > $OUT/mixed_trace.jsonl 2> $OUT/mixed_trace.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex "ragged" --output-format csv \
    -d $OUT/pmc_fetch -o run -- python3 tools/mixed_probe.py --rounds 1 --reps 2 > $OUT/mixed_fetch.jsonl 2> $OUT/mixed_fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --kernel-include-regex "ragged" --output-format csv \
    -d $OUT/pmc_write -o run -- python3 tools/mixed_probe.py --rounds 1 --reps 2 > $OUT/mixed_write.jsonl 2> $OUT/mixed_write.err
find $OUT -name "*.csv" | sort
