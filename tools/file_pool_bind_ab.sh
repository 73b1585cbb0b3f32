# A/B of the file layer's thread placement (HEC_FILE_POOL_BIND=1: I/O and
# writer threads bound to the GPU's NUMA node; 0: inherited affinity, the
# shipped default), alternating processes on one box over the same 12 GiB volume in
# /dev/shm: write_ec_files 3x per process (fresh shard files each time) and a
# 4-shard rebuild. One JSON line per process to stdout.
set -e
DIR=$(mktemp -d -p /dev/shm hec_ab.XXXX)
trap 'rm -rf $DIR' EXIT
python3 - "$DIR" <<'PY'
import sys
from oracle import corc
with open(sys.argv[1] + "/v.dat", "wb") as f:
    for g in range(12):  # 12 GiB, 1 GiB at a time
        f.write(corc.splitmix64_bytes(99 + g, 1 << 30).tobytes())
PY
for round in 1 2 3; do
  for bind in 1 0; do
    HEC_FILE_POOL_BIND=$bind timeout -k 10 120 python3 - "$DIR" $bind $round <<'PY'
import json, os, sys, time
import helyim_amd as H
d, bind, rnd = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
base = d + "/v"
enc = []
for _ in range(3):
    for i in range(14):
        p = base + H.to_ext(i)
        if os.path.exists(p):
            os.remove(p)
    t0 = time.perf_counter(); H.write_ec_files(base); enc.append(time.perf_counter() - t0)
for i in (0, 5, 10, 13):
    os.remove(base + H.to_ext(i))
t0 = time.perf_counter(); H.rebuild_ec_files(base); reb = time.perf_counter() - t0
print(json.dumps({"round": rnd, "bind": bind, "encode_s": [round(x, 4) for x in enc], "rebuild_s": round(reb, 4),
                  "encode_GiB_s_best": round(12 / min(enc), 2)}), flush=True)
PY
  done
done
