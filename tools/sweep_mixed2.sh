# Second config-5 sweep: the length mix through the strided kernels (one
# launch per length, --grouped) beside the ragged launches, ragged encode
# XCD remap off/on, uniform 4 MiB and 64 KiB stripes ragged vs strided, and
# the 64 KiB shard gap on the mix. Summarise with tools/sweep_mixed_summary.py.
set -e
TAG=${1:-sweep2}
OUT=gpurun_out/$TAG
export TMPDIR=/tmp
mkdir -p $OUT
run() {  # name, probe args...
    local name=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- \
        python3 tools/mixed_probe.py --reps 3 "$@" > $OUT/$name.jsonl 2> $OUT/$name.err
    echo "$name done"
}
run m4096_grouped --stripes 4096 --rounds 3 --grouped --enc-remaps 0,1
run m512_grouped --stripes 512 --rounds 3 --grouped --enc-remaps 0,1
run len4m_e4 --stripes 1024 --fixed-len 4194304 --fixed-e 4 --rounds 3 --strided --enc-remaps 0,1
run len64k_e4 --stripes 16384 --fixed-len 65536 --fixed-e 4 --rounds 3 --strided --enc-remaps 0,1
run m4096_pad --stripes 4096 --rounds 3 --pads 0,65536
