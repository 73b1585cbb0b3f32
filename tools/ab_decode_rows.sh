# Decode rate by erasure count, working tree vs HEAD build (libhec_old.so),
# alternating on one box, after the GPU suite on the new build.
TAG=${1:-abrows}
OUT=gpurun_out/$TAG
mkdir -p $OUT; : > $OUT/probe.jsonl
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for v in ${ORDER:-old new new old}; do
  if [ $v = old ]; then L=build/variants/libhec_old.so; else L=""; fi
  HEC_LIB_PATH=$L timeout -k 10 200 python tools/decode_pattern_probe.py --rounds 5 2>/dev/null >> $OUT/probe.jsonl || exit 1
done
