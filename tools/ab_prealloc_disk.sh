# Preallocation on vs off on a disk filesystem (the box's scratch dir), 4 GiB volume.
TAG=${1:-abpd}; DIR=${2:-$GRAFT_REPO_ROOT/gpurun_scratch}
mkdir -p gpurun_out/$TAG $DIR; : > gpurun_out/$TAG/ab.log
df -T $DIR >> gpurun_out/$TAG/ab.log
for r in 1 2; do
  for v in prealloc noprealloc; do
    if [ $v = noprealloc ]; then export HEC_NO_PREALLOC=1; else unset HEC_NO_PREALLOC; fi
    echo "== $v" >> gpurun_out/$TAG/ab.log
    timeout -k 10 250 python tools/file_stages.py --dir $DIR --gib 4 --reps 2 --fresh >> gpurun_out/$TAG/ab.log 2>/dev/null || exit 1
    timeout -k 10 250 python tools/file_stages.py --dir $DIR --gib 4 --reps 2 >> gpurun_out/$TAG/ab.log 2>/dev/null || exit 1
  done
done
rm -rf $DIR
