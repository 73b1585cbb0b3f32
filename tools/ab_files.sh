# File-layer pipeline variants (slots / job size builds) vs the default, alternating on one box.
TAG=${1:-abf}; shift
mkdir -p gpurun_out/$TAG; : > gpurun_out/$TAG/ab.log
for r in 1 2; do
  for L in "" "$@"; do
    echo "== ${L:-default}" >> gpurun_out/$TAG/ab.log
    HEC_LIB_PATH=$L timeout -k 10 250 python tools/file_stages.py --reps 2 --fresh >> gpurun_out/$TAG/ab.log 2>/dev/null || exit 1
    HEC_LIB_PATH=$L timeout -k 10 250 python tools/file_stages.py --reps 2 >> gpurun_out/$TAG/ab.log 2>/dev/null || exit 1
  done
done
