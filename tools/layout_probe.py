"""Encode HBM rate for three device layouts of the same 4096 x 1 MiB batch
(interleaved rounds, one process): in place [S][14][L]; data [S][10][L] +
parity [S][4][L] in a second buffer; data [S][10][L] + parity [4][S][L]
(each parity shard of all stripes contiguous). Measurement only."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import helyim_amd as H
    import helyim_amd.batch as B
    S, L = 4096, 1 << 20
    rs = H.ReedSolomon(10, 4)
    full = torch.empty((S, 14, L), dtype=torch.uint8, device="cuda")
    B.fill_splitmix(full, 10 * L, 0x5EED0000)
    data = torch.empty((S, 10, L), dtype=torch.uint8, device="cuda")
    data.copy_(full[:, :10])
    par_s = torch.empty((S, 4, L), dtype=torch.uint8, device="cuda")
    par_j = torch.empty((4, S, L), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    lib = H.lib

    def enc_inplace():
        B.encode_batch(rs, full)

    def enc_sep():
        B.encode_batch_sep(rs, data, par_s)

    def enc_jmajor():
        assert lib.hec_gpu_encode_batch(rs.handle, data.data_ptr(), 10 * L, L, par_j.data_ptr(), L, S * L, L, S,
                                        ctypes.c_void_p(st)) == 0

    import ctypes
    cases = {"inplace_S14L": enc_inplace, "sep_S4L": enc_sep, "sep_4SL": enc_jmajor}
    res = {k: [] for k in cases}
    for f in cases.values():
        f()
    torch.cuda.synchronize()
    for _ in range(7):
        for k, f in cases.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f()
            b.record()
            torch.cuda.synchronize()
            res[k].append(a.elapsed_time(b))
    ok = torch.equal(full[:, 10:], par_s) and torch.equal(par_s.transpose(0, 1), par_j)
    out = {k: round(S * 14 * L / (sorted(v)[len(v) // 2] * 1e-3) / 1e9, 1) for k, v in res.items()}
    out["identical"] = bool(ok)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
