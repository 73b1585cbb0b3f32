"""One process = one allocation of the bench batch ([4096][14][1 MiB], 64 KiB
gap after each shard): torch's caching allocator (hipMalloc, what bench.py
uses) or hipExtMallocWithFlags(hipDeviceMallocContiguous); then 2 warm-up and
5 timed encode + 4-erasure decode steps (HIP events), one JSON line.
Run under a rocprofv3 UTCL1 PMC pass by tools/alloc_tlb_probe.sh.

python tools/alloc_tlb_probe.py --kind torch|contiguous"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HIP_DEVICE_MALLOC_CONTIGUOUS = 0x4


class _Dev:
    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="torch")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--precycle", action="store_true",
                    help="allocate, touch and free a buffer of the batch's size first (torch kind)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    import bench
    torch.cuda.set_device(0)
    S, L, pad = 4096, 1 << 20, 64 << 10
    shard = L + pad
    nbytes = S * 14 * shard
    raw = None
    if args.precycle:
        tmp = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        tmp.fill_(0)
        torch.cuda.synchronize()
        del tmp
        torch.cuda.empty_cache()
    if args.kind == "torch":
        buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    else:
        hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
        hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        p = ctypes.c_void_p()
        rc = hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, HIP_DEVICE_MALLOC_CONTIGUOUS)
        if rc != 0:
            print(json.dumps({"kind": args.kind, "error": rc}), flush=True)
            return 1
        raw = p.value
        buf = torch.as_tensor(_Dev(raw, nbytes), device="cuda")
    t = buf.as_strided((S, 14, L), (14 * shard, shard, 1))
    B.fill_stripes_splitmix(t, 10, bench.rank_seed_base(0))
    rs = H.ReedSolomon(10, 4)
    masks = torch.from_numpy(bench.erasure_masks(S, 0)).cuda()
    st = torch.cuda.current_stream()
    for _ in range(2):
        B.encode_batch(rs, t)
        B.reconstruct_batch(rs, t, masks)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    torch.cuda.synchronize()
    for e in ev:
        e[0].record(st)
        B.encode_batch(rs, t)
        e[1].record(st)
        B.reconstruct_batch(rs, t, masks)
        e[2].record(st)
    torch.cuda.synchronize()
    enc = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    dec = float(np.mean([e[1].elapsed_time(e[2]) for e in ev]))
    alg = S * 14 * L
    print(json.dumps({"kind": args.kind, "precycle": args.precycle, "ptr": hex(t.data_ptr()), "enc_ms": round(enc, 4), "dec_ms": round(dec, 4),
                      "encode_frac": round(alg / enc / 1e6 / 8000, 4), "decode_frac": round(alg / dec / 1e6 / 8000, 4)}),
          flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
