mkdir -p gpurun_out; : > gpurun_out/tune2.log
for v in default ntl0_nts0 ntl0_nts1 ntl1_nts0; do
  if [ $v = default ]; then L=""; else L="build/variants/libhec_$v.so"; fi
  HEC_LIB_PATH=$L timeout -k 10 200 python tools/tune.py --modes 0,1 --vecs 1,2 --blocks 0 --rounds 5 >> gpurun_out/tune2.log 2>&1 || exit 1
done
for pad in 4096 8256 65536; do
  timeout -k 10 200 python tools/tune.py --modes 0,1 --vecs 1,2 --blocks 0 --rounds 5 --pad $pad >> gpurun_out/tune2.log 2>&1 || exit 1
done
grep '^{' gpurun_out/tune2.log
