"""RS(10,4) encode+decode throughput on MI355X (device-resident), the metric of
BASELINE.json: "RS(10,4) encode+decode GiB/s (device-resident), 1 MiB stripes,
1/2/4/8 GPUs".

One step = one pass of the hot path over one batch: encode every stripe of a
[4096, 14, 1 MiB] HBM-resident batch (10 data shards -> 4 parity, one
hec_gpu_encode_batch launch), then reconstruct every stripe with 4 random
erasures (one hec_gpu_reconstruct_batch launch; each stripe reads its first 10
survivors and rewrites its 4 erased shards). Inputs are synthetic splitmix64
stripes generated in HBM before the timed region.

value = data-payload GiB/s over all ranks: (encode 10*L + decode 10*L bytes
per stripe) * stripes * ranks / max-over-ranks step time. After the timed
region (outside the clock) every rank checks its WHOLE batch against the C
oracle (oracle/corc.py: data, parity and the rebuilt shards of every stripe)
and its mixed leg's stripes; `verified` is the AND over ranks. Multi-GPU: one
process per GPU, independent stripe batches per rank (seed base
0x5EED0000 + rank*2^20), no data-path collective ("scaling": "weak"); the
only cross-rank traffic is the barrier and the max-reduce of the timings
(gloo, host side).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
  Without WORLD_SIZE in the environment and N > 1, this process is only a
  launcher: it makes no GPU call, starts N ranks with torch.distributed.run
  (127.0.0.1 rendezvous) and exits with their status. Under an external
  launcher WORLD_SIZE must equal N. --dry-run runs the launcher and the
  control plane (seeds, barrier, max-over-ranks timing, aggregation) with a
  GPU-free stand-in step (tests/test_bench_launcher.py).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

K_DATA, M_PARITY, N_TOTAL = 10, 4, 14
HBM_PEAK_GBPS = 8000.0  # MI355X spec HBM3E, GB/s (MI355X_MICROARCH.md)
SEED_BASE = 0x5EED0000


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def rank_seed_base(rank: int) -> int:
    return SEED_BASE + rank * (1 << 20)


def erasure_masks(n_stripes: int, rank: int, erasures: int = 4) -> np.ndarray:
    """Per-stripe present masks with `erasures` shards dropped, uniform over the
    C(14, erasures) patterns, seeded per rank."""
    rng = np.random.default_rng(0xEC0000 + rank)
    full = (1 << N_TOTAL) - 1
    masks = np.empty(n_stripes, dtype=np.int32)
    for s in range(n_stripes):
        drop = rng.choice(N_TOTAL, erasures, replace=False)
        m = full
        for i in drop:
            m &= ~(1 << int(i))
        masks[s] = m
    return masks


def reduce_max(x: float, world: int) -> float:
    """Max over ranks of a host scalar (control plane only: gloo all_reduce)."""
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    v = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    return float(v.item())


def gather(obj, world: int) -> list:
    """Every rank's `obj` (control plane only: gloo all_gather_object)."""
    if world == 1:
        return [obj]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def job_throughput(payload_bytes_per_rank_step: float, steps: int, world: int, t_job: float) -> float:
    """Whole-job GiB/s: every rank processes the same payload per step; the
    job's time is the max over ranks."""
    return payload_bytes_per_rank_step * steps * world / t_job / 2**30


def scaling_fields(value: float, world: int, per_rank: list) -> dict:
    """The per-GPU view of a multi-rank line (the
    1/2/4/8-GPU curve read as per-GPU efficiency against the 1-GPU run):
    per_gpu_GiB_s = value / N; rank_spread = slowest / fastest rank's step
    (its own HIP-event encode + decode ms); each rank's encode / decode
    roofline fraction. per_rank entries: {"rank", "step_ms", "encode_frac",
    "decode_frac"} (fractions None in the GPU-free dry run)."""
    steps = [r["step_ms"] for r in per_rank]
    return {"per_gpu_GiB_s": round(value / world, 4),
            "rank_spread": round(max(steps) / min(steps), 4) if min(steps) > 0 else None,
            "per_rank_frac": [{"rank": r["rank"], "step_ms": round(r["step_ms"], 4),
                               "encode_frac": r.get("encode_frac"), "decode_frac": r.get("decode_frac")}
                              for r in per_rank]}


def aggregate_host_path(per_rank: list) -> dict:
    """Whole-node host-path rate from per-rank legs run at the same time:
    bytes of all ranks / the wall-clock window from the first rank's start to
    the last rank's end, per phase (time.time() stamps, one host clock).
    per_rank entries: {"data_bytes", "encode": [t0, t1], "decode": [t0, t1]}."""
    data = sum(r["data_bytes"] for r in per_rank)

    def window(ph):
        return max(r[ph][1] for r in per_rank) - min(r[ph][0] for r in per_rank)

    def rate(b, t):
        return round(b / t / 2**30, 2)

    return {"ranks": len(per_rank),
            "encode_data_GiB_s": rate(data, window("encode")),
            "decode_data_GiB_s": rate(data, window("decode")),
            "per_rank_encode_data_GiB_s": [rate(r["data_bytes"], r["encode"][1] - r["encode"][0]) for r in per_rank],
            "per_rank_decode_data_GiB_s": [rate(r["data_bytes"], r["decode"][1] - r["decode"][0]) for r in per_rank]}


# ---------------------------------------------------------------------------
# launcher (no GPU call in this process)
# ---------------------------------------------------------------------------
def visible_gpu_count() -> int:
    """GPUs a child process could open, counted without initialising HIP:
    the first *_VISIBLE_DEVICES list that is set, else the KFD topology nodes
    that have SIMDs (GPU agents)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() != ""])
    root = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for node in os.listdir(root):
            try:
                with open(os.path.join(root, node, "properties")) as f:
                    for line in f:
                        k, _, v = line.partition(" ")
                        if k == "simd_count" and int(v) > 0:
                            n += 1
            except (OSError, ValueError):
                pass
    except OSError:
        return 0
    return n


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args, argv: list) -> int:
    """Start args.gpus ranks of this script (torch.distributed.run as a child
    process, one rank per GPU) and return their exit status."""
    n = args.gpus
    if not args.dry_run:
        have = visible_gpu_count()
        if n > have and not args.allow_shared_gpu:
            log(f"bench.py: --gpus {n} but {have} GPU(s) visible; refusing "
                f"(--allow-shared-gpu rehearses more ranks than GPUs)")
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def physical_cores() -> dict:
    """lscpu-equivalent counts from sysfs: physical cores (distinct
    (package, core) pairs), logical CPUs, and what this process may use
    (affinity mask, cgroup v2 cpu.max quota)."""
    base = "/sys/devices/system/cpu"
    cores, logical = set(), 0
    try:
        for d in os.listdir(base):
            if not (d.startswith("cpu") and d[3:].isdigit()):
                continue
            try:
                with open(f"{base}/{d}/topology/physical_package_id") as f:
                    pkg = f.read().strip()
                with open(f"{base}/{d}/topology/core_id") as f:
                    core = f.read().strip()
            except OSError:
                continue
            logical += 1
            cores.add((pkg, core))
    except OSError:
        pass
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()
            if q != "max":
                quota = round(int(q) / int(period), 2)
    except (OSError, ValueError):
        pass
    return {"physical_cores": len(cores) or (os.cpu_count() or 1), "logical_cpus": logical or os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": quota}


def cpu_baseline(seconds: float = 10.0) -> dict:
    """helyim-ec's CPU path restated (oracle/rs_oracle.c, AVX2 nibble-pshufb,
    upstream code_some_slices loop order), 1 thread: encode + 4-erasure
    reconstruct of 1 MiB stripes, cycled over 8 distinct stripes for ~seconds."""
    from oracle import corc
    L = 1 << 20
    rs = corc.CReedSolomon(K_DATA, M_PARITY)
    stripes = []
    rng = np.random.default_rng(11)
    for s in range(8):
        d = corc.splitmix64_bytes(SEED_BASE + s, K_DATA * L).reshape(K_DATA, L)
        sh = [d[i].copy() for i in range(K_DATA)] + [np.zeros(L, np.uint8) for _ in range(M_PARITY)]
        drop = sorted(rng.choice(N_TOTAL, 4, replace=False).tolist())
        stripes.append((sh, [i not in drop for i in range(N_TOTAL)]))
    simd = bool(corc.lib().orc_have_avx2())
    n = 0
    t0 = time.perf_counter()
    while True:
        sh, present = stripes[n % len(stripes)]
        rs.encode(sh, simd=simd)
        rs.reconstruct(sh, present, simd=simd)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    gib = n * 2 * K_DATA * L / 2**30
    return {"value": round(gib / el, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{n} stripe encode+decode passes (10 x 1 MiB data, 4 erasures), 8 distinct "
                      f"splitmix64 stripes cycled, {el:.1f} s, 1 thread, "
                      f"{'AVX2 nibble-pshufb' if simd else 'scalar table'} C restatement of "
                      f"helyim-ec/reed-solomon-erasure (oracle/rs_oracle.c)",
            "cpu_model": _cpu_model(), "host_cpus": os.cpu_count()}


def cpu_baseline_threads(seconds: float = 5.0, threads: int = 16) -> dict:
    """the same C restatement, one thread per core over
    independent stripes (ctypes drops the GIL inside the C calls). 16 threads
    = the GPU box's CPU share per GPU."""
    import threading
    from oracle import corc
    L = 1 << 20
    rs = corc.CReedSolomon(K_DATA, M_PARITY)
    simd = bool(corc.lib().orc_have_avx2())
    counts = [0] * threads
    stop = threading.Event()

    def work(t):
        rng = np.random.default_rng(100 + t)
        d = corc.splitmix64_bytes(SEED_BASE + 1000 + t, K_DATA * L).reshape(K_DATA, L)
        sh = [d[i].copy() for i in range(K_DATA)] + [np.zeros(L, np.uint8) for _ in range(M_PARITY)]
        drop = sorted(rng.choice(N_TOTAL, 4, replace=False).tolist())
        present = [i not in drop for i in range(N_TOTAL)]
        while not stop.is_set():
            rs.encode(sh, simd=simd)
            rs.reconstruct(sh, present, simd=simd)
            counts[t] += 1

    th = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    time.sleep(seconds)
    stop.set()
    for x in th:
        x.join()
    el = time.perf_counter() - t0
    n = sum(counts)
    return {"value": round(n * 2 * K_DATA * L / 2**30 / el, 4), "unit": "GiB/s", "cores": threads,
            "kind": "port", "sample": f"{n} stripe encode+decode passes over {threads} threads, one 1 MiB "
                                      f"stripe per thread, {el:.1f} s"}


def cpu_baseline_legs(seconds: float, allowed, stand_in: bool = False) -> dict:
    """The CPU path timed on this box's host cores, in the same run as the GPU
    legs, at ANY world size (north_star: "next to helyim-ec's CPU path timed
    on the GPU box's own host cores in the same run"). Rank 0 runs it after
    the last GPU barrier while the other ranks wait at the closing barrier.

    cpu_baseline: 1 thread. cpu_baseline_threads: 16 threads (the box's CPU
    share per GPU). cpu_baseline_cores: one thread per CPU this process can
    actually run on at once: min(physical cores, affinity mask, cgroup quota);
    "quota_bound" says the quota (or affinity), not the core count, set it.
    stand_in: the same record shapes without running anything (--dry-run)."""
    os.sched_setaffinity(0, allowed)  # the CPU legs get every CPU this process may use
    cores = physical_cores()
    usable = cores["affinity_cpus"]
    if cores["cgroup_cpu_quota"]:
        usable = min(usable, max(1, int(cores["cgroup_cpu_quota"])))
    n_cores = max(1, min(cores["physical_cores"], usable))
    bound = {"quota_bound": cores["physical_cores"] > usable,
             "threads_note": "one thread per usable CPU: min(physical cores, affinity, cgroup quota)"}
    if stand_in:
        rec = {"value": 0.0, "unit": "GiB/s", "kind": "stand_in", "sample": "dry run: nothing timed"}
        return {"cpu_baseline": dict(rec, cores=1), "cpu_baseline_threads": dict(rec, cores=16),
                "cpu_baseline_cores": dict(rec, cores=n_cores, **cores, **bound)}
    out = {"cpu_baseline": cpu_baseline(seconds),
           "cpu_baseline_threads": cpu_baseline_threads(seconds / 2, 16)}
    if n_cores == 16:  # the same measurement as the 16-thread leg: not run twice
        out["cpu_baseline_cores"] = dict(out["cpu_baseline_threads"], **cores, **bound)
    else:
        out["cpu_baseline_cores"] = dict(cpu_baseline_threads(seconds / 2, n_cores), **cores, **bound)
    return out


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


TRAFFIC_FILE = "profiles/pmc_traffic.json"


def load_traffic() -> dict:
    """HBM traffic per launch from the committed rocprofv3 PMC summary
    (tools/pmc_summary.py), if any; "_file" names it for the bench line."""
    p = os.path.join(ROOT, TRAFFIC_FILE)
    if os.path.exists(p):
        with open(p) as f:
            d = json.load(f)
        d["_file"] = TRAFFIC_FILE
        return d
    return {}


def e2e_section(rs, rank: int, S: int = 512, L: int = 1 << 20, reps: int = 3, devices=None) -> dict:
    """End-to-end rate from pinned host memory (the path helyim runs): host
    stripes -> H2D -> kernel -> D2H, pipelined over 3 streams. Encode moves
    10 L H2D + 4 L D2H per stripe; a 4-erasure decode 10 L H2D + 4 L D2H.
    devices: one call spread over these GPUs (hec_host_*_batch_multi)."""
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    dev = torch.empty((S, N_TOTAL, L), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(dev, K_DATA * L, rank_seed_base(rank))
    if devices is None:
        buf = H.HostBuffer(S * N_TOTAL * L)  # pinned, on this GPU's NUMA node
    else:  # one batch, each device's stripe range on that device's node
        buf = H.HostBuffer.for_devices(devices, N_TOTAL * L, S)
    host = buf.tensor((S, N_TOTAL, L))
    host.copy_(dev)
    del dev
    masks = erasure_masks(S, rank)
    B.host_encode_batch(rs, host, devices=devices)  # warm-up (pipeline buffers, tables)
    B.host_reconstruct_batch(rs, host, masks, devices=devices)
    enc0 = time.time()
    for _ in range(reps):
        B.host_encode_batch(rs, host, devices=devices)
    enc1 = dec0 = time.time()
    for _ in range(reps):
        B.host_reconstruct_batch(rs, host, masks, devices=devices)
    dec1 = time.time()
    te, td = (enc1 - enc0) / reps, (dec1 - dec0) / reps
    data = S * K_DATA * L
    node = buf.numa_node()
    del host
    buf.close()
    mem = ("pinned (hec_host_alloc: this GPU's NUMA node)" if devices is None else
           "pinned (hec_host_alloc_multi: each range on its GPU's NUMA node)")
    return {"stripes": S, "shard_len": L, "host_memory": mem,
            "encode_kernel": H.lib.hec_host_encode_kernel_name(L).decode(),
            "host_numa_node": node, "devices": devices if devices is not None else "current",
            "raw": {"data_bytes": data * reps, "encode": [enc0, enc1], "decode": [dec0, dec1]},
            "encode_data_GiB_s": round(data / te / 2**30, 2),
            "decode_data_GiB_s": round(data / td / 2**30, 2),
            "encode_pcie_GB_s": round(S * N_TOTAL * L / te / 1e9, 2),
            "decode_pcie_GB_s": round(S * N_TOTAL * L / td / 1e9, 2)}


MIXED_LENS = [(64 << 10) << i for i in range(7)]  # 64 KiB .. 4 MiB


def mixed_workload(rank: int, n_stripes: int):
    """BASELINE config 5, seeded per rank: shard lengths log-uniform over
    64 KiB..4 MiB, 0..4 erasures per stripe (uniform count, uniform shards).
    Stripes packed back to back (shard stride = length); stripe s's data is
    splitmix64(rank_seed_base(rank) + s). -> (lengths, erasure counts, present
    masks, hec_stripe_desc rows, total bytes)."""
    rng = np.random.default_rng(0x5E + rank)
    Ls = rng.choice(MIXED_LENS, n_stripes)
    es = rng.integers(0, 5, n_stripes)
    full = (1 << N_TOTAL) - 1
    masks = np.empty(n_stripes, dtype=np.int64)
    for s in range(n_stripes):
        drop = rng.choice(N_TOTAL, int(es[s]), replace=False)
        masks[s] = full & ~int(sum(1 << int(i) for i in drop))
    descs, off = [], 0
    for s in range(n_stripes):
        descs.append((off, int(Ls[s]), int(Ls[s]), int(masks[s])))
        off += N_TOTAL * int(Ls[s])
    return Ls, es, masks, descs, off


def mixed_section(rs, rank: int, n_stripes: int = 2048, e2e_stripes: int = 512) -> dict:
    """BASELINE config 5: shard lengths 64 KiB..4 MiB (log-uniform), 0..4
    erasures per stripe. Device-resident: all n_stripes packed in one HBM
    buffer, one ragged encode launch + one ragged reconstruct launch, each
    timed with its own HIP events (2048 stripes: the 512-stripe launch lost
    ~3% to its fixed cost, profiles/r03/sweep_mixed1.jsonl). End to end: the
    first e2e_stripes stripes through the pinned-host pipeline
    (hec_host_*_batch), one call per length group."""
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    lens = MIXED_LENS
    Ls, es, masks, descs, off = mixed_workload(rank, n_stripes)
    full = (1 << N_TOTAL) - 1
    dev = torch.empty(off, dtype=torch.uint8, device="cuda")
    for s, (o, st, L, _) in enumerate(descs):
        B.fill_splitmix(dev[o:o + K_DATA * L].view(1, 1, -1), K_DATA * L, rank_seed_base(rank) + s)
    data = int(sum(K_DATA * d[2] for d in descs))
    # decode payload counts only stripes with an erasure (e = 0 is upstream's no-op)
    dec_data = int(sum(K_DATA * d[2] for d in descs if d[3] != full))
    enc_hbm = int(sum(N_TOTAL * d[2] for d in descs))  # algorithmic bytes: read 10 L + write 4 L
    dec_hbm = int(sum((K_DATA + N_TOTAL - bin(d[3]).count("1")) * d[2] for d in descs if d[3] != full))
    # the descriptors as the C ABI's hec_stripe_desc array, built once (a list
    # is converted on every call, on the host, with the GPU idle the first time)
    darr = np.array(descs, dtype=B.desc_dtype())
    enc_kernel = B.ragged_kernel_name(darr, False)  # the launch's own choice (hec_ragged_kernel_name)
    dec_kernel = B.ragged_kernel_name(darr, True)
    B.encode_ragged(rs, dev, darr)  # warm-up
    B.reconstruct_ragged(rs, dev, darr)
    torch.cuda.synchronize()
    s_ = torch.cuda.current_stream()
    reps = 5
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps + 1)]
    ev[0].record(s_)
    for i in range(reps):
        B.encode_ragged(rs, dev, darr)
        ev[2 * i + 1].record(s_)
        B.reconstruct_ragged(rs, dev, darr)
        ev[2 * i + 2].record(s_)
    torch.cuda.synchronize()
    t_dev = ev[0].elapsed_time(ev[-1]) * 1e-3 / reps
    enc_ms = float(np.median([ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(reps)]))
    dec_ms = float(np.median([ev[2 * i + 1].elapsed_time(ev[2 * i + 2]) for i in range(reps)]))
    verification = mixed_verify(rs, dev, darr, descs, Ls, es, rank)
    groups, bufs = [], []
    sub_idx = range(min(e2e_stripes, n_stripes))
    for L in lens:
        idx = [s for s in sub_idx if Ls[s] == L]
        if not idx:
            continue
        hb = H.HostBuffer(len(idx) * N_TOTAL * L)  # pinned, on this GPU's NUMA node
        bufs.append(hb)
        h = hb.tensor((len(idx), N_TOTAL, L))
        for j, s in enumerate(idx):
            o = descs[s][0]
            h[j].view(-1).copy_(dev[o:o + N_TOTAL * L])
        groups.append((h, masks[idx].astype(np.uint32)))
    del dev
    e2e_payload = int(sum(K_DATA * descs[s][2] * (2 if descs[s][3] != full else 1) for s in sub_idx))
    for h, m in groups:
        B.host_encode_batch(rs, h)
    w0 = time.time()
    for h, m in groups:
        B.host_encode_batch(rs, h)
        B.host_reconstruct_batch(rs, h, m)
    w1 = time.time()
    t_e2e = w1 - w0
    groups.clear()
    h = m = None  # no view of the pinned buffers outlives them
    for hb in bufs:
        hb.close()
    return {"stripes": n_stripes, "shard_lens": "64 KiB..4 MiB log-uniform", "erasures": "0..4 uniform",
            "payload_GiB": round((data + dec_data) / 2**30, 3),
            "payload": "encode 10 L per stripe + decode 10 L per stripe with >= 1 erasure",
            "device_resident_data_GiB_s": round((data + dec_data) / t_dev / 2**30, 2),
            "device_resident": "one ragged encode + one ragged reconstruct launch over all stripes",
            "encode": {"kernel": enc_kernel, "ms_median": round(enc_ms, 4),
                       "algorithmic_bytes": enc_hbm, "GB_s_hbm": round(enc_hbm / enc_ms / 1e6, 1),
                       "frac": round(enc_hbm / enc_ms / 1e6 / HBM_PEAK_GBPS, 4)},
            "decode": {"kernel": dec_kernel, "ms_median": round(dec_ms, 4),
                       "algorithmic_bytes": dec_hbm, "GB_s_hbm": round(dec_hbm / dec_ms / 1e6, 1),
                       "frac": round(dec_hbm / dec_ms / 1e6 / HBM_PEAK_GBPS, 4)},
            "verification": verification,
            "end_to_end_stripes": len(sub_idx),
            "end_to_end_data_GiB_s": round(e2e_payload / t_e2e / 2**30, 2),
            "raw": {"payload_bytes": e2e_payload, "e2e": [w0, w1], "device_s": t_dev}}


def mixed_verify(rs, dev, darr, descs, Ls, es, rank: int) -> dict:
    """After the timed mixed launches (outside their clock): the erased shards
    of EVERY stripe are overwritten, the ragged reconstruct runs over the
    batch again, and every stripe is compared with the C oracle (grouped by
    length, 32 stripes per copy): data = its splitmix64 seed's stream,
    parity = the oracle's encode, every erased shard = the oracle's
    reconstruct from the survivors."""
    import torch
    import helyim_amd.batch as B
    from oracle import corc
    pick = list(range(len(descs)))
    for s in pick:
        o, st, L, m = descs[s]
        for i in range(N_TOTAL):
            if not (m >> i) & 1:
                dev[o + i * st:o + i * st + L].fill_(0xA5)
    B.reconstruct_ragged(rs, dev, darr)
    torch.cuda.synchronize()
    bad = []
    for L in sorted(set(int(Ls[s]) for s in pick)):
        same = [s for s in pick if int(Ls[s]) == L]
        for g in range(0, len(same), 32):
            idx = same[g:g + 32]
            host = np.stack([dev[descs[s][0]:descs[s][0] + N_TOTAL * L].view(N_TOTAL, L).cpu().numpy()
                             for s in idx])
            masks = np.array([descs[s][3] for s in idx], dtype=np.int64)
            seeds = np.array([rank_seed_base(rank) + s for s in idx], dtype=np.uint64)
            bad += [idx[j] for j in corc.check_stripes(host, masks, 16, seeds)]
    return {"stripes_checked": len(pick), "rebuilt_shards_checked": int(sum(int(es[s]) for s in pick)),
            "pairs_covered": len(set((int(Ls[s]), int(es[s])) for s in pick)),
            "erasure_counts": sorted(set(int(es[s]) for s in pick)),
            "shard_lens": sorted(set(int(Ls[s]) for s in pick)),
            "mismatched_stripes": sorted(bad), "ok": not bad,
            "method": "every stripe's erased shards overwritten, ragged reconstruct re-run, every stripe vs "
                      "the C oracle (seeded data, encode, reconstruct from survivors)"}


def multi_gpu_e2e_child(ndev: int, timeout_s: float = 240.0, cmd=None) -> dict:
    """Run e2e_section over devices 0..ndev-1 in a child process (this
    script with --e2e-multi-child) and return its JSON, or a record of the
    failure (time limit, exit status, unparsable output): never an exception,
    so this leg cannot cost the headline line. cmd: override (tests)."""
    if cmd is None:
        cmd = [sys.executable, os.path.abspath(__file__), "--e2e-multi-child",
               ",".join(str(d) for d in range(ndev))]
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s, cwd=ROOT)
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {timeout_s:.0f} s"}
    except OSError as ex:
        return {"error": f"could not start: {ex}"}
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"error": f"exit {p.returncode}", "stderr_tail": p.stderr[-800:]}
    try:
        return json.loads(lines[-1])
    except ValueError as ex:
        return {"error": f"unparsable output: {ex}", "stdout_tail": lines[-1][-400:]}


def assemble_host_legs(e2e_all: list, mixed_all: list, world: int) -> dict:
    """The bench line's end_to_end / mixed sections from every rank's records
    (gathered on rank 0): one rank's record as is, or per-rank records plus
    the node aggregate over one wall-clock window."""
    extras = {"end_to_end": e2e_all[0] if world == 1 else {
        "aggregate": aggregate_host_path([r["raw"] for r in e2e_all]), "per_rank": e2e_all}}
    if world == 1:
        extras["mixed"] = mixed_all[0]
    else:
        extras["mixed"] = {"per_rank": mixed_all,
                           # one wall-clock window over every rank's end-to-end part
                           "aggregate_end_to_end_data_GiB_s": round(
                               sum(m["raw"]["payload_bytes"] for m in mixed_all)
                               / (max(m["raw"]["e2e"][1] for m in mixed_all)
                                  - min(m["raw"]["e2e"][0] for m in mixed_all)) / 2**30, 2)}
    return extras


def e2e_multi_child_main(devices: list) -> int:
    import torch
    import helyim_amd as H
    torch.cuda.set_device(0)
    rs = H.ReedSolomon(K_DATA, M_PARITY)
    out = e2e_section(rs, 0, S=256 * len(devices), devices=devices)
    out.pop("raw", None)
    print(json.dumps(out), flush=True)
    return 0


def packed_layout_pass(rs, S: int, L: int, masks, rank: int, reps: int) -> dict:
    """The same encode + decode on a PACKED [S, 14, L] batch (shard stride =
    L, what hec_gpu_*_batch callers that do not pad get), timed per launch with
    HIP events beside the padded headline batch (after it, untimed by the
    headline clock)."""
    import torch
    import helyim_amd.batch as B
    tp = torch.empty((S, N_TOTAL, L), dtype=torch.uint8, device="cuda")
    B.fill_stripes_splitmix(tp, K_DATA, rank_seed_base(rank))
    B.encode_batch(rs, tp)  # warm-up
    B.reconstruct_batch(rs, tp, masks)
    st = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps + 1)]
    ev[0].record(st)
    for i in range(reps):
        B.encode_batch(rs, tp)
        ev[2 * i + 1].record(st)
        B.reconstruct_batch(rs, tp, masks)
        ev[2 * i + 2].record(st)
    torch.cuda.synchronize()
    enc = float(np.median([ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(reps)]))
    dec = float(np.median([ev[2 * i + 1].elapsed_time(ev[2 * i + 2]) for i in range(reps)]))
    del tp
    torch.cuda.empty_cache()
    b = S * N_TOTAL * L
    return {"shard_stride": L, "reps": reps, "encode_ms_median": round(enc, 4), "decode_ms_median": round(dec, 4),
            "encode_frac": round(b / enc / 1e6 / HBM_PEAK_GBPS, 4), "decode_frac": round(b / dec / 1e6 / HBM_PEAK_GBPS, 4),
            "data_GiB_s": round(2 * S * K_DATA * L / ((enc + dec) * 1e-3) / 2**30, 2)}


def init_control_plane() -> None:
    """gloo process group for the barrier / max-reduce / gather of host
    scalars. gloo prints its connection report on stdout, which carries only
    the bench line: fd 1 points at stderr while it connects."""
    import torch.distributed as dist
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group("gloo", init_method="env://")
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--shard-len", type=int, default=1 << 20)
    ap.add_argument("--shard-pad", type=int, default=64 << 10,
                    help="HBM layout: shard stride = shard_len + this (DESIGN.md 'Data layout in HBM')")
    ap.add_argument("--base-align", type=int, default=0,
                    help="start the batch at a multiple of this many bytes inside an over-allocation "
                         "(power of two; 0 = the allocator's base; measurement, VERDICT r04 item 1(c))")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the end-to-end and mixed-workload sections")
    ap.add_argument("--no-packed", action="store_true", help="skip the packed-layout pass beside the padded batch")
    ap.add_argument("--e2e-multi-child", default="",
                    help="internal: the multi-GPU end-to-end leg in its own process over this device list "
                         "(e.g. 0,1,2,3; 0,0 rehearses it on one GPU)")
    ap.add_argument("--allow-shared-gpu", action="store_true",
                    help="rehearsal: allow more ranks than visible GPUs (ranks share devices round-robin)")
    ap.add_argument("--dry-run", action="store_true",
                    help="GPU-free control-plane rehearsal: launcher, seeds, barrier, max-over-ranks timing")
    ap.add_argument("--dry-step-ms", type=float, default=5.0,
                    help="dry run: rank r's stand-in step sleeps (r + 1) x this")
    ap.add_argument("--dry-fail-rank", type=int, default=-1,
                    help="dry run: this rank's stand-in verification fails (the job must report verified false)")
    return ap.parse_args(argv)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.e2e_multi_child:
        return e2e_multi_child_main([int(d) for d in args.e2e_multi_child.split(",")])
    if args.gpus < 1:
        log("bench.py: --gpus must be >= 1")
        return 2
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return launch_ranks(args, argv)
    world = int(env_world or "1")
    if world != args.gpus:
        log(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; refusing (one rank per GPU)")
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        init_control_plane()
    try:
        if args.dry_run:
            return dry_run(args, world, rank, local_rank)
        return run_rank(args, world, rank, local_rank)
    finally:
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
            dist.destroy_process_group()


def dry_run(args, world: int, rank: int, local_rank: int) -> int:
    """The control plane of run_rank with a GPU-free stand-in step (rank r
    sleeps (r + 1) x dry_step_ms): same barrier, max-over-ranks job time and
    whole-job throughput formula, one JSON line from rank 0."""
    S, L = args.stripes, args.shard_len

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    step = args.dry_step_ms * (rank + 1) / 1e3
    for _ in range(args.warmup):
        time.sleep(step)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(step)
    barrier()
    wall = time.perf_counter() - t0
    chk_ok = rank != args.dry_fail_rank  # stand-in for the rank's oracle verification
    t_job = reduce_max(wall, world)
    per_rank = gather({"rank": rank, "local_rank": local_rank, "world_size": int(os.environ.get("WORLD_SIZE", "1")),
                       "seed_base": rank_seed_base(rank), "wall_s": wall, "pid": os.getpid(),
                       "step_ms": step * 1e3, "masks_head": erasure_masks(4, rank).tolist()}, world)
    # host legs: stand-in records with the real records' shape (rank r moves
    # (r + 1) GiB in (r + 1) x dry_step_ms per phase), assembled as run_rank does
    barrier()
    e0 = time.time()
    time.sleep(step)
    e1 = time.time()
    time.sleep(step)
    e2 = time.time()
    gib = (rank + 1) * 2**30
    e2e = {"stand_in": True, "raw": {"data_bytes": gib, "encode": [e0, e1], "decode": [e1, e2]}}
    barrier()
    w0 = time.time()
    time.sleep(step)
    mixed = {"stand_in": True, "verification": {"ok": chk_ok},
             "raw": {"payload_bytes": gib, "e2e": [w0, time.time()], "device_s": step}}
    e2e_all, mixed_all = gather(e2e, world), gather(mixed, world)
    chk_ok = chk_ok and all(m["verification"]["ok"] for m in mixed_all)
    extras = assemble_host_legs(e2e_all, mixed_all, world)
    chk_ok = reduce_max(0.0 if chk_ok else 1.0, world) == 0.0
    if rank == 0:
        payload = 2 * S * K_DATA * L
        out = {"metric": "dry run (no GPU): launcher and control plane only", "dry_run": True,
               "value": round(job_throughput(payload, args.steps, world, t_job), 4), "unit": "GiB/s",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": round(t_job / args.steps * 1e3, 4), "scaling": "weak", "verified": chk_ok,
               "rank_seed_bases": [r["seed_base"] for r in per_rank], "ranks": per_rank}
        out.update(scaling_fields(out["value"], world, per_rank))
        out.update(extras)
        if not args.no_cpu_baseline:
            out.update(cpu_baseline_legs(args.cpu_seconds, os.sched_getaffinity(0), stand_in=True))
        print(json.dumps(out), flush=True)
    return 0 if chk_ok else 3


def run_rank(args, world: int, rank: int, local_rank: int) -> int:
    import torch
    import torch.distributed as dist
    # one process per GPU; more ranks than visible GPUs (an --allow-shared-gpu
    # rehearsal) share devices round-robin
    ndev = max(1, torch.cuda.device_count())
    if world > ndev and not args.allow_shared_gpu:
        log(f"bench.py: {world} ranks but {ndev} GPU(s) visible; refusing (--allow-shared-gpu to rehearse)")
        return 2
    device = local_rank % ndev
    torch.cuda.set_device(device)

    import helyim_amd as H
    import helyim_amd.batch as B

    allowed = os.sched_getaffinity(0)
    numa = H.bind_host_to_device(device)  # this rank's host threads next to its GPU's pinned buffers

    S, L = args.stripes, args.shard_len
    rs = H.ReedSolomon(K_DATA, M_PARITY)
    t = B.empty_stripes(S, N_TOTAL, L, shard_pad=args.shard_pad, base_align=args.base_align)
    base_alignment = B.address_alignment(t.data_ptr())
    B.fill_stripes_splitmix(t, K_DATA, rank_seed_base(rank))  # same bytes as a packed batch
    masks = torch.from_numpy(erasure_masks(S, rank)).cuda()
    stream = torch.cuda.current_stream()

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        B.encode_batch(rs, t)
        B.reconstruct_batch(rs, t, masks)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        B.encode_batch(rs, t)
        ev[i][1].record(stream)
        B.reconstruct_batch(rs, t, masks)
        ev[i][2].record(stream)
    barrier()
    wall = time.perf_counter() - t0
    enc_steps = [a.elapsed_time(b) for a, b, _ in ev]
    dec_steps = [b.elapsed_time(c) for _, b, c in ev]
    enc_ms, dec_ms = float(np.mean(enc_steps)), float(np.mean(dec_steps))
    # SURVEY §8d configs 2/3 quote the median of the timed launches
    enc_med, dec_med = float(np.median(enc_steps)), float(np.median(dec_steps))
    t_job = reduce_max(wall, world)

    # correctness of what was timed (outside the clock), the WHOLE batch: the
    # erased shards of every stripe are zeroed and rebuilt by one more
    # reconstruct launch, then every stripe is compared with the C oracle
    # (data = its seed's splitmix64 stream, parity = the oracle's encode, the
    # 4 rebuilt shards = the oracle's reconstruct from the same survivors)
    from oracle import corc
    v0 = time.perf_counter()
    er = torch.zeros((S, N_TOTAL), dtype=torch.bool, device="cuda")
    for i in range(N_TOTAL):
        er[:, i] = (masks & (1 << i)) == 0
    t[er] = 0
    B.reconstruct_batch(rs, t, masks)
    torch.cuda.synchronize()
    del er
    # the seeded-data check regenerates splitmix64 words, so it needs whole
    # 8-byte words per shard; other lengths check parity and rebuilt shards only
    seeds = rank_seed_base(rank) + np.arange(S, dtype=np.uint64) if L % 8 == 0 else None
    bad = corc.check_device_batch(t, masks.cpu().numpy(), data_seeds=seeds)
    chk_ok = not bad
    verification = {"stripes_checked": S, "rebuilt_shards_checked": 4 * S, "mismatched_stripes": bad[:16],
                    "data_seeds_checked": seeds is not None,
                    "seconds": round(time.perf_counter() - v0, 2),
                    "method": "erased shards zeroed and rebuilt, every stripe vs the C oracle (seeded data, "
                              "encode, reconstruct from survivors), 16 threads"}
    t_shard_stride = t.stride(1)
    del t
    packed = None
    if args.shard_pad and not args.no_packed:
        torch.cuda.empty_cache()
        packed = packed_layout_pass(rs, S, L, masks, rank, max(3, args.steps // 2))
    enc_bytes = S * N_TOTAL * L                      # read 10 L + write 4 L per stripe
    dec_bytes = S * (K_DATA + 4) * L                 # read 10 survivors + write 4 erased
    per_rank = gather({"rank": rank, "device": device, "seed_base": rank_seed_base(rank), "numa": numa,
                       "verification": verification,
                       "wall_s": round(wall, 6), "encode_ms": round(enc_ms, 4), "decode_ms": round(dec_ms, 4),
                       "encode_ms_median": round(enc_med, 4), "decode_ms_median": round(dec_med, 4),
                       "step_ms": enc_ms + dec_ms,
                       "encode_frac": round(enc_bytes / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                       "decode_frac": round(dec_bytes / (dec_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)},
                      world)
    enc_ms = max(r["encode_ms"] for r in per_rank)
    dec_ms = max(r["decode_ms"] for r in per_rank)

    payload = 2 * S * K_DATA * L                     # data-payload bytes per step (encode + decode)
    value = job_throughput(payload, args.steps, world, t_job)
    enc_gbps = enc_bytes / (enc_ms * 1e-3) / 1e9
    dec_gbps = dec_bytes / (dec_ms * 1e-3) / 1e9
    prof = load_traffic()
    if prof.get("workload", "").split(",")[0] != f"{S} stripes x {L} B":
        prof = {}  # the committed counters are of another batch size: no traffic figure for this one

    extras = {}
    if not args.no_extras:
        # host-path legs on every rank at once (after one barrier), so at N > 1
        # the aggregate shows the shared host-memory / PCIe limit
        barrier()
        e2e = e2e_section(rs, rank)
        barrier()
        mixed = mixed_section(rs, rank)
        e2e_all = gather(e2e, world)
        mixed_all = gather(mixed, world)
        chk_ok = chk_ok and all(m["verification"]["ok"] for m in mixed_all)
        extras = assemble_host_legs(e2e_all, mixed_all, world)

    # every rank's verification counts (headline batch and mixed leg): the job
    # is verified only if all are
    chk_ok = reduce_max(0.0 if chk_ok else 1.0, world) == 0.0

    if world == 1 and not args.no_extras and torch.cuda.device_count() > 1:
        # one process, every visible GPU: one host call split over them
        # (hec_host_*_batch_multi, the in-process multi-GPU host path), run
        # in a child process with a time limit so that it cannot cost the
        # headline line above it
        extras["end_to_end_multi_gpu"] = multi_gpu_e2e_child(torch.cuda.device_count())

    if rank == 0:
        enc_name = H.lib.hec_encode_kernel_name(L).decode()
        dec_name = H.lib.hec_decode_kernel_name(L).decode()
        # roofline of the dominant kernel (the larger share of the step); PMC
        # counters cannot run inside this process, so the HBM bytes per launch
        # come from the committed rocprofv3 passes named in traffic_source
        dom_dec = dec_ms >= enc_ms
        dom_gbps = dec_gbps if dom_dec else enc_gbps
        dominant = {"bound": "hbm", "achieved": round(dom_gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(dom_gbps / HBM_PEAK_GBPS, 4),
                    "traffic": prof.get("decode_hbm_bytes_per_launch" if dom_dec else "encode_hbm_bytes_per_launch"),
                    "traffic_source": prof.get("_file") and f"{prof['_file']} (rocprofv3 FETCH_SIZE/WRITE_SIZE "
                                                            f"passes of run {prof.get('source')}; not this run)",
                    "kernel": dec_name if dom_dec else enc_name,
                    "launch": "decode (4 erasures)" if dom_dec else "encode",
                    "share_of_step": round((dec_ms if dom_dec else enc_ms) / (enc_ms + dec_ms), 4),
                    "algorithmic_bytes_per_launch": dec_bytes if dom_dec else enc_bytes}
        out = {
            "metric": "RS(10,4) encode+decode GiB/s (device-resident), 1 MiB stripes, 1/2/4/8 GPUs",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_job / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 stripes generated in HBM)",
            "config": {"workload": f"RS(10,4) encode + 4-erasure decode, {S} stripes x {L} B shards per GPU "
                                   f"(BASELINE configs 2+3), device-resident",
                       "stripes_per_gpu": S, "shard_len": L, "erasures_per_stripe": 4,
                       "shard_stride": t_shard_stride,
                       "base_alignment": base_alignment,
                       "parallelism": f"independent stripe batches x{world}"},
            # the dominant kernel: the launch with the larger share of the step
            "roofline": dominant,
            "encode": {"kernel": enc_name, "ms_per_launch": round(enc_ms, 4),
                       "ms_per_launch_median": max(r["encode_ms_median"] for r in per_rank),
                       "GB_s_hbm": round(enc_gbps, 1),
                       "data_GiB_s": round(S * K_DATA * L / (enc_ms * 1e-3) / 2**30, 1),
                       "frac": round(enc_gbps / HBM_PEAK_GBPS, 4),
                       "traffic": prof.get("encode_hbm_bytes_per_launch")},
            "decode": {"kernel": dec_name,
                       "ms_per_launch": round(dec_ms, 4),
                       "ms_per_launch_median": max(r["decode_ms_median"] for r in per_rank),
                       "GB_s_hbm": round(dec_gbps, 1),
                       "data_GiB_s": round(S * K_DATA * L / (dec_ms * 1e-3) / 2**30, 1),
                       "frac": round(dec_gbps / HBM_PEAK_GBPS, 4),
                       "traffic": prof.get("decode_hbm_bytes_per_launch")},
            "packed_layout": packed,
            "verified": chk_ok,
            "verification": verification,
            "ranks": per_rank,
        }
        out.update(scaling_fields(out["value"], world, per_rank))
        out.update(extras)
        if not args.no_cpu_baseline:  # every world size; the other ranks wait at main()'s closing barrier
            out.update(cpu_baseline_legs(args.cpu_seconds, allowed))
        print(json.dumps(out), flush=True)
    return 0 if chk_ok else 3


if __name__ == "__main__":
    sys.exit(main())
