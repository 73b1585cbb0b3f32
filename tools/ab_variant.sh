mkdir -p gpurun_out/s3
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3/gpu_tests.log 2>&1 || exit 1
: > gpurun_out/s3/ab.log
for r in 1 2; do
 for v in old new; do
  if [ $v = old ]; then L=build/variants/libhec_old.so; else L=""; fi
  echo "== $v" >> gpurun_out/s3/ab.log
  HEC_LIB_PATH=$L timeout -k 10 200 python tools/tune.py --modes 0,1 --vecs 1 --blocks 0 --remaps 1 --bpcs 0 --encs 0,1 --rounds 5 >> gpurun_out/s3/ab.log 2>&1 || exit 1
 done
done
