# Decode with 8 bytes per lane (variant dec8) vs the shipped 16-byte decode
# and a null build, interleaved on one box (tools/tune.py; decode column).
TAG=${1:-dec8}
OUT=gpurun_out/$TAG
mkdir -p $OUT; : > $OUT/ab.log
for v in ${VARS:-ship dec8 null dec8 ship null dec8 ship}; do
  if [ $v = ship ]; then L=""; else L=build/variants/libhec_$v.so; fi
  echo "== $v" >> $OUT/ab.log
  HEC_LIB_PATH=$L timeout -k 10 120 python tools/tune.py --modes 0 --vecs 1 --blocks 0 --remaps 1 --bpcs 0 \
      --encs 1 --rounds 4 2>/dev/null >> $OUT/ab.log || exit 1
done
