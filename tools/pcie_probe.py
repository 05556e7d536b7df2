"""Raw PCIe rates of this box (tools only): pinned host <-> device copies of
the e2e line's chunk size and of the whole 409.6 MB batch, one stream, and
H2D + D2H at once on two streams.  Prints GB/s."""
import json
import time

import torch

dev = torch.device("cuda", 0)
res = {}
for nbytes in (8192 * 4096, 100_000 * 4096):
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)),
                     ("d2h", lambda: h.copy_(d, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        res[f"{name}_{nbytes >> 20}MiB_GBps"] = round(nbytes * reps / (time.perf_counter() - t0) / 1e9, 2)
    h2 = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d2 = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        with torch.cuda.stream(s1):
            d.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize()
    res[f"bidir_{nbytes >> 20}MiB_GBps_each"] = round(nbytes * 10 / (time.perf_counter() - t0) / 1e9, 2)
try:
    res["numa_node"] = open("/sys/class/drm/card1/device/numa_node").read().strip()
except OSError:
    res["numa_node"] = None
print(json.dumps(res))
