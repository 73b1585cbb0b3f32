# Fourth config-5 sweep: the erasure mix against every fixed erasure count on
# the SAME stripes (lengths, layout, bytes) in one process, for the mixed
# lengths and for 1 MiB stripes, plus the XCD-balanced ("dealt") order.
# Summarise with tools/sweep_mixed_summary.py.
set -e
TAG=${1:-sweep4}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
run() {  # name, probe args...
    local name=$1; shift
    timeout -k 10 300 python3 tools/mixed_probe.py --reps 3 --rounds 3 --orders given,dealt,e1,e2,e3,e4 "$@" \
        > $OUT/$name.jsonl 2> $OUT/$name.err
    echo "$name done"
}
run mixed4096 --stripes 4096
run emix4096_1m --stripes 4096 --fixed-len 1048576
