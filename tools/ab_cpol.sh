# Cache policy of the shard streams through raw buffer instructions vs the
# shipped global nt accesses, interleaved on one box (Makefile VARIANTS
# s_* / l_*; null = byte-identical kernel file, the method's own spread).
TAG=${1:-cpol}
OUT=gpurun_out/$TAG
mkdir -p $OUT; : > $OUT/ab.log
for r in 1 2; do
 for v in ${VARS:-ship null s_sc1 s_sc0sc1 s_sc0sc1nt s_bufnt l_bufnt}; do
  if [ $v = ship ]; then L=""; else L=build/variants/libhec_$v.so; fi
  echo "== $v" >> $OUT/ab.log
  HEC_LIB_PATH=$L timeout -k 10 120 python tools/tune.py --modes 0 --vecs 1 --blocks 0 --remaps 1 --bpcs 0 \
      --encs 1 --rounds 4 2>/dev/null >> $OUT/ab.log || exit 1
 done
done
