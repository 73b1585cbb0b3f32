# Shard-file preallocation (fallocate KEEP_SIZE) on vs off (HEC_NO_PREALLOC=1),
# alternating on one box, fresh files and over existing files.
TAG=${1:-abp}
mkdir -p gpurun_out/$TAG; : > gpurun_out/$TAG/ab.log
for r in 1 2 3; do
  for v in prealloc noprealloc; do
    if [ $v = noprealloc ]; then export HEC_NO_PREALLOC=1; else unset HEC_NO_PREALLOC; fi
    echo "== $v" >> gpurun_out/$TAG/ab.log
    timeout -k 10 250 python tools/file_stages.py --reps 2 --fresh >> gpurun_out/$TAG/ab.log 2>/dev/null || exit 1
    timeout -k 10 250 python tools/file_stages.py --reps 2 >> gpurun_out/$TAG/ab.log 2>/dev/null || exit 1
  done
done
