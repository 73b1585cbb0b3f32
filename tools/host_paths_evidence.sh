#!/bin/bash
# Host-memory paths at the current HEAD on one box: batched
# degraded-read intervals, needle reads on a mounted EC volume, the file layer
# on a 12 GiB volume in /dev/shm, and pageable host batches. Each step under
# its own time limit; the first failure ends the script.
# usage: tools/host_paths_evidence.sh OUT_DIR
set -o pipefail
out=${1:?out dir}
mkdir -p "$out"
timeout -k 10 120 python tools/bench_intervals.py > "$out/intervals.json" &&
timeout -k 10 180 python tools/bench_reads.py > "$out/reads.json" &&
timeout -k 10 300 python tools/bench_files.py --gib 12 > "$out/files.json" &&
timeout -k 10 180 python tools/pageable_multi_probe.py > "$out/pageable_multi.jsonl"
