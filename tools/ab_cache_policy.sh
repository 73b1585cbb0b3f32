# A/B of the shard-stream cache policies (Makefile `variants`: nt loads/stores
# on or off) against the shipped build, alternating on one box.
# Usage: make variants && bash tools/ab_cache_policy.sh TAG
TAG=${1:-abc}
mkdir -p gpurun_out/$TAG; : > gpurun_out/$TAG/ab.log
for r in 1 2; do
  for v in ${VARS:-ship ntl0_nts0 ntl0_nts1 ntl1_nts0}; do
    if [ $v = ship ]; then L=""; else L=build/variants/libhec_$v.so; fi
    echo "== $v" >> gpurun_out/$TAG/ab.log
    HEC_LIB_PATH=$L timeout -k 10 200 python tools/tune.py --modes 0 --vecs 1 --blocks 0 --remaps 1 --bpcs 0 \
      --encs 0,1 --rounds 5 >> gpurun_out/$TAG/ab.log 2>&1 || exit 1
  done
done
