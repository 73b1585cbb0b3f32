mkdir -p gpurun_out; : > gpurun_out/tune8.log
for tile in 0 16384 32768 65536 131072; do
  timeout -k 10 200 python tools/tune.py --modes 0,1 --vecs 1 --blocks 0 --remaps 0,1 --bpcs 0 --rounds 5 --tile $tile >> gpurun_out/tune8.log 2>&1 || exit 1
done
grep '^{' gpurun_out/tune8.log
