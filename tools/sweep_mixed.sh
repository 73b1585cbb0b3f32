# Config-5 (mixed workload) sweep under rocprofv3 kernel traces (VERDICT r02
# "next" item 1): is the ragged kernels' gap to the strided ones per byte or
# launch-fixed? Separate processes, one per case:
#   mixed lengths + mixed erasures at 512 / 2048 / 4096 stripes;
#   4096 stripes with only the length mixed (e = 4) and only e mixed (1 MiB);
#   4096 x 1 MiB, e = 4 through the ragged and the strided kernels (same bytes).
# Summarise with tools/sweep_mixed_summary.py gpurun_out/$TAG.
set -e
TAG=${1:-sweep}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
run() {  # name, probe args...
    local name=$1; shift
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- \
        python3 tools/mixed_probe.py --rounds 2 --reps 3 "$@" > $OUT/$name.jsonl 2> $OUT/$name.err
    echo "$name done"
}
run mixed512 --stripes 512
run mixed2048 --stripes 2048
run mixed4096 --stripes 4096
run lenmix4096_e4 --stripes 4096 --fixed-e 4
run emix4096_1m --stripes 4096 --fixed-len 1048576 --strided
run uniform4096 --stripes 4096 --uniform 4 --strided
