# A/B of the bench's mixed (ragged) section between an old library build and
# the current one, alternating on one box. Usage: bash tools/ab_mixed.sh OLD_SO TAG
OLD=$1; TAG=${2:-abm}
mkdir -p gpurun_out/$TAG; : > gpurun_out/$TAG/ab.log
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then L=$OLD; else L=""; fi
    echo "== $v" >> gpurun_out/$TAG/ab.log
    HEC_LIB_PATH=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 2>/dev/null \
      | python -c "import json,sys; d=json.load(sys.stdin); print(json.dumps({'value': d['value'], 'mixed_dev': d['mixed']['device_resident_data_GiB_s']}))" >> gpurun_out/$TAG/ab.log || exit 1
  done
done
