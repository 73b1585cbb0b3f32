# Decode A/B of a measurement build (Makefile VARIANTS) against the shipped
# library and a null build, alternating on one box (tools/tune.py).
TAG=${1:-abv}; V=${2:-lf0}
OUT=gpurun_out/$TAG
mkdir -p $OUT; : > $OUT/ab.log
for v in ${ORDER:-ship $V null $V ship null $V ship}; do
  if [ $v = ship ]; then L=""; else L=build/variants/libhec_$v.so; fi
  echo "== $v" >> $OUT/ab.log
  HEC_LIB_PATH=$L timeout -k 10 120 python tools/tune.py --modes 0 --vecs 1 --blocks 0 --remaps 1 --bpcs 0 \
      --encs 1 --rounds 4 2>/dev/null >> $OUT/ab.log || exit 1
done
