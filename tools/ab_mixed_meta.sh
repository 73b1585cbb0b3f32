mkdir -p gpurun_out/mixed_ab
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mixed_ab/gpu_tests.log 2>&1 || exit 1
: > gpurun_out/mixed_ab/mixed.jsonl
for v in old new new old; do
  if [ $v = old ]; then L=build/variants/libhec_old.so; else L=""; fi
  HEC_LIB_PATH=$L timeout -k 10 120 python tools/mixed_probe.py --rounds 3 2>/dev/null >> gpurun_out/mixed_ab/mixed.jsonl || exit 1
done
