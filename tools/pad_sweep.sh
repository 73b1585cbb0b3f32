# Layout sweep on the BASELINE batch: extra bytes between shards (--pad: the
# shard AND stripe strides grow) and between stripes only (--stripe-pad),
# encode (bit-sliced) and decode, GF and XOR-only twin. Output: gpurun_out/$TAG.
TAG=${1:-pads}
OUT=gpurun_out/$TAG
mkdir -p $OUT; : > $OUT/pads.jsonl
for p in ${PADS:-0 256 1024 2048 8192 65536 0}; do
  timeout -k 10 120 python tools/tune.py --modes 0,1 --vecs 1 --blocks 0 --remaps 1 --encs 1 --rounds 3 --pad $p \
    2>/dev/null >> $OUT/pads.jsonl || exit 1
done
for p in ${SPADS:-4096 65536 1048576}; do
  timeout -k 10 120 python tools/tune.py --modes 0,1 --vecs 1 --blocks 0 --remaps 1 --encs 1 --rounds 3 --stripe-pad $p \
    2>/dev/null >> $OUT/pads.jsonl || exit 1
done
