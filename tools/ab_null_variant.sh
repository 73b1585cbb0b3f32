# The A/B method itself: the shipped library against a byte-identical kernel
# build linked as a variant (null), in interleaved order. Spread = method noise.
TAG=${1:-abn}
mkdir -p gpurun_out/$TAG; : > gpurun_out/$TAG/ab.log
for v in ${VARS:-ship null null ship ship null}; do
  if [ $v = ship ]; then L=""; else L=build/variants/libhec_$v.so; fi
  echo "== $v" >> gpurun_out/$TAG/ab.log
  HEC_LIB_PATH=$L timeout -k 10 200 python tools/tune.py --modes 0 --vecs 1 --blocks 0 --remaps 1 --bpcs 0 \
      --encs 0,1 --rounds 5 >> gpurun_out/$TAG/ab.log 2>&1 || exit 1
done
