import torch, time, json
n = 1 << 30
h = torch.empty(n, dtype=torch.uint8).pin_memory()
h2 = torch.empty(n // 2, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device="cuda")
d2 = torch.empty(n // 2, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
res = {}
for _ in range(2):
    torch.cuda.synchronize(); t = time.perf_counter(); d.copy_(h, non_blocking=True); torch.cuda.synchronize(); res["h2d_GBps"] = n / (time.perf_counter() - t) / 1e9
    torch.cuda.synchronize(); t = time.perf_counter(); h.copy_(d, non_blocking=True); torch.cuda.synchronize(); res["d2h_GBps"] = n / (time.perf_counter() - t) / 1e9
    torch.cuda.synchronize(); t = time.perf_counter()
    with torch.cuda.stream(s1): d.copy_(h, non_blocking=True)
    with torch.cuda.stream(s2): h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize(); dt = time.perf_counter() - t
    res["duplex_h2d_1GiB_plus_d2h_0.5GiB_GBps_total"] = (n + n // 2) / dt / 1e9
print(json.dumps({k: round(v, 2) for k, v in res.items()}))
