"""Host batch encode from PAGEABLE memory: the copy pipeline as is, vs
registering the buffer (hipHostRegister) for the call so the zero-copy kernel
can address it, registration time included. Measurement only."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import helyim_amd as H
    from oracle import corc
    S, L = 256, 1 << 20
    a = np.zeros((S, 14, L), dtype=np.uint8)
    for s in range(S):
        a[s, :10] = np.frombuffer(os.urandom(10 * L), np.uint8).reshape(10, L) if s < 2 else s
    rs = H.ReedSolomon(10, 4)
    lib = H.lib
    hip = ctypes.CDLL("libamdhip64.so")
    torch.cuda.init()
    p = a.ctypes.data

    def enc():
        assert lib.hec_host_encode_batch(rs.handle, p, 14 * L, L, p + 10 * L, 14 * L, L, L, S) == 0

    rng = np.random.default_rng(1)
    masks = np.array([((1 << 14) - 1) & ~int(sum(1 << int(i) for i in rng.choice(14, 4, replace=False)))
                      for _ in range(S)], dtype=np.uint32)

    def dec():
        assert lib.hec_host_reconstruct_batch(rs.handle, p, 14 * L, L, L, S, masks.ctypes.data, None) == 0

    res = {}
    for zc, name in ((1, "pooled_pinned_staging"), (0, "runtime_copies")):
        lib.hec_set_host_zero_copy(zc)
        enc()
        dec()
        t0 = time.perf_counter(); enc(); res[f"pageable_encode_{name}_s"] = time.perf_counter() - t0
        t0 = time.perf_counter(); dec(); res[f"pageable_decode_{name}_s"] = time.perf_counter() - t0
    lib.hec_set_host_zero_copy(1)
    res["pageable_copy_pipeline_s"] = res["pageable_encode_pooled_pinned_staging_s"]
    for it in range(2):
        t0 = time.perf_counter()
        assert hip.hipHostRegister(ctypes.c_void_p(p), ctypes.c_size_t(a.nbytes), 0) == 0
        t1 = time.perf_counter()
        enc()
        t2 = time.perf_counter()
        assert hip.hipHostUnregister(ctypes.c_void_p(p)) == 0
        t3 = time.perf_counter()
        res["register_s"], res["zero_copy_encode_s"], res["unregister_s"] = t1 - t0, t2 - t1, t3 - t2
        if it == 0:
            res["first_register_s"] = t1 - t0
    data = S * 10 * L
    out = {k: round(v, 6) for k, v in res.items()}
    for k in list(res):
        if k.startswith("pageable_e") or k.startswith("pageable_d"):
            out[k[:-2] + "_GiB_s"] = round(data / res[k] / 2**30, 2)
    out["register_encode_unregister_GiB_s"] = round(
        data / (res["first_register_s"] + res["zero_copy_encode_s"] + res["unregister_s"]) / 2**30, 2)
    ref = corc.encode_stripes(np.ascontiguousarray(a[:, :10]))
    out["identical"] = bool(np.array_equal(a[:, 10:], ref))
    # registration of never-touched pages (np.empty: mapped lazily)
    b = np.empty(1 << 30, dtype=np.uint8)
    t0 = time.perf_counter()
    rc = hip.hipHostRegister(ctypes.c_void_p(b.ctypes.data), ctypes.c_size_t(b.nbytes), 0)
    out["register_1GiB_untouched_s"] = round(time.perf_counter() - t0, 6)
    out["register_rc"] = rc
    if rc == 0:
        t0 = time.perf_counter()
        hip.hipHostUnregister(ctypes.c_void_p(b.ctypes.data))
        out["unregister_1GiB_s"] = round(time.perf_counter() - t0, 6)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
