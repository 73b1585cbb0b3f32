# Same-box A/B of the working tree's build against the HEAD build
# (build/variants/libhec_old.so, built from `git archive HEAD`), interleaved:
# GPU suite on the new build first, then tools/tune.py rounds alternating
# builds. Usage: bash tools/ab_old_new.sh TAG [ORDER]
TAG=${1:-abon}
OUT=gpurun_out/$TAG
mkdir -p $OUT; : > $OUT/ab.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for v in ${2:-old new new old old new}; do
  if [ $v = old ]; then L=build/variants/libhec_old.so; else L=""; fi
  echo "== $v" >> $OUT/ab.log
  HEC_LIB_PATH=$L timeout -k 10 200 python tools/tune.py --modes 0,1 --vecs 1 --blocks 0 --remaps 1 --bpcs 0 \
      --encs 1 --rounds 5 >> $OUT/ab.log 2>&1 || exit 1
done
