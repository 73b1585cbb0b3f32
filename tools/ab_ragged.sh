# Ragged kernels, working tree vs HEAD build (libhec_old.so), alternating on
# one box: the mixed workload (bench config 5) and the bench batch through the
# ragged path (4 and 1 erasures), after the GPU suite on the new build.
TAG=${1:-abrag}
OUT=gpurun_out/$TAG
mkdir -p $OUT; : > $OUT/m.jsonl
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
for v in ${ORDER:-old new new old}; do
  if [ $v = old ]; then L=build/variants/libhec_old.so; else L=""; fi
  HEC_LIB_PATH=$L timeout -k 10 120 python tools/mixed_probe.py --rounds 3 2>/dev/null >> $OUT/m.jsonl || exit 1
  HEC_LIB_PATH=$L timeout -k 10 120 python tools/mixed_probe.py --rounds 2 --uniform 4 --stripes 4096 2>/dev/null >> $OUT/m.jsonl || exit 1
done
