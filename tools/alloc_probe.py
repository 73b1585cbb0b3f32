"""Does where the bench batch lives in HBM decide its speed? The bench step
(encode + 4-erasure decode of 4096 x 1 MiB) on several allocations of the
same 56 GiB: torch's caching allocator (hipMalloc), and hipExtMallocWithFlags
with hipDeviceMallocContiguous (one physically contiguous range). Each
allocation is timed for --steps steps, then freed back to the driver.

python tools/alloc_probe.py [--allocs 3] [--steps 20]
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HIP_DEVICE_MALLOC_CONTIGUOUS = 0x4  # hip_runtime_api.h


class _Dev:
    def __init__(self, ptr, shape):
        self.__cuda_array_interface__ = {"shape": shape, "typestr": "|u1", "data": (ptr, False), "version": 3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--allocs", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--kinds", default="torch,contiguous")
    args = ap.parse_args()
    import torch
    import helyim_amd as H
    import helyim_amd.batch as B
    import bench
    hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    S, L = 4096, 1 << 20
    shape = (S, 14, L)
    rs = H.ReedSolomon(10, 4)
    masks = torch.from_numpy(bench.erasure_masks(S, 0)).cuda()
    st = torch.cuda.current_stream()
    for a in range(args.allocs):
        for kind in args.kinds.split(","):
            raw = None
            if kind == "torch":
                t = torch.empty(shape, dtype=torch.uint8, device="cuda")
            else:
                p = ctypes.c_void_p()
                rc = hip.hipExtMallocWithFlags(ctypes.byref(p), S * 14 * L, HIP_DEVICE_MALLOC_CONTIGUOUS)
                if rc != 0:
                    print(json.dumps({"alloc": a, "kind": kind, "error": rc}), flush=True)
                    continue
                raw = p.value
                t = torch.as_tensor(_Dev(raw, shape), device="cuda")
            B.fill_splitmix(t, 10 * L, 0x5EED0000)
            torch.cuda.synchronize()
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            enc = dec = 0.0
            for _ in range(args.steps):
                e[0].record(st)
                B.encode_batch(rs, t)
                e[1].record(st)
                B.reconstruct_batch(rs, t, masks)
                e[2].record(st)
                torch.cuda.synchronize()
                enc += e[0].elapsed_time(e[1]) / args.steps
                dec += e[1].elapsed_time(e[2]) / args.steps
            print(json.dumps({"alloc": a, "kind": kind, "ptr": hex(t.data_ptr()), "enc_ms": round(enc, 3),
                              "dec_ms": round(dec, 3)}), flush=True)
            del t
            torch.cuda.synchronize()
            if raw is not None:
                hip.hipFree(ctypes.c_void_p(raw))
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
