"""Measure achievable HBM bandwidth on this box (roofline calibration)."""
import ctypes, json, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbm_probe.so"))
for f in ("probe_read", "probe_read_lds"):
    getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
L.probe_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
n = 2 << 30
x = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
y = torch.empty_like(x)
sink = torch.zeros(4, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
res = {}
def t(fn, nbytes, reps=20):
    for _ in range(3): fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record(s)
    for _ in range(reps): fn()
    e1.record(s); torch.cuda.synchronize()
    return nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
for grid in (2048, 4096, 8192, 16384):
    res[f"read_dwordx4_g{grid}"] = t(lambda: L.probe_read(x.data_ptr(), n, sink.data_ptr(), grid, s.cuda_stream), n)
    res[f"read_lds_dma_g{grid}"] = t(lambda: L.probe_read_lds(x.data_ptr(), n, sink.data_ptr(), grid, s.cuda_stream), n)
    res[f"copy_g{grid}"] = t(lambda: L.probe_copy(x.data_ptr(), y.data_ptr(), n, grid, s.cuda_stream), 2 * n)
print(json.dumps({k: round(v, 1) for k, v in res.items()}))
