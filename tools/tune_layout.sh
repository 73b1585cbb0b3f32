# Layout sweep: contiguous [S][14][1 MiB] vs tile-interleaved [S*L/T][14][T].
mkdir -p gpurun_out; : > gpurun_out/tune3.log
for tile in 0 1024 2048 4096 8192 16384 65536; do
  timeout -k 10 200 python tools/tune.py --modes 0,1 --vecs 1,2,4 --blocks 0 --rounds 5 --tile $tile >> gpurun_out/tune3.log 2>&1 || exit 1
done
grep '^{' gpurun_out/tune3.log
