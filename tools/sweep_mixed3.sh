# Third config-5 sweep: does balancing the decode work over the 8 XCDs (the
# descriptor order "dealt": each erasure count split evenly over the map's
# eighths) recover the 3-4% a mixed erasure count costs? Given vs dealt order
# alternate per round in one process. Summarise with tools/sweep_mixed_summary.py.
set -e
TAG=${1:-sweep3}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
run() {  # name, probe args...
    local name=$1; shift
    timeout -k 10 300 python3 tools/mixed_probe.py --reps 3 --rounds 4 --orders given,dealt "$@" \
        > $OUT/$name.jsonl 2> $OUT/$name.err
    echo "$name done"
}
run emix4096_1m --stripes 4096 --fixed-len 1048576 --strided
run mixed4096 --stripes 4096
run mixed2048 --stripes 2048
run mixed512 --stripes 512
