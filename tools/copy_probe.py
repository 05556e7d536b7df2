"""Copy-rate calibration (read + write counted): which store / load form gets
closest to the guide's 6.29 TB/s float4 copy on this box."""
import ctypes, json, os
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbm_probe.so"))
L.probe_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
L.probe_copy_var.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
res = {}
s = torch.cuda.current_stream()
def t(fn, nbytes, reps=20):
    for _ in range(3): fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record(s)
    for _ in range(reps): fn()
    e1.record(s); torch.cuda.synchronize()
    return nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
for n in (400 << 20, 2 << 30):
    x = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
    y = torch.empty_like(x)
    tag = f"{n >> 20}M"
    res[f"torch_copy_{tag}"] = t(lambda: y.copy_(x), 2 * n)
    for grid in (1024, 2048, 4096, 8192):
        res[f"copy_g{grid}_{tag}"] = t(lambda: L.probe_copy(x.data_ptr(), y.data_ptr(), n, grid, s.cuda_stream), 2 * n)
        for kind, name in ((0, "u4"), (1, "u4_nts"), (2, "u4_ntls"), (3, "u1_nts")):
            res[f"{name}_g{grid}_{tag}"] = t(lambda: L.probe_copy_var(x.data_ptr(), y.data_ptr(), n, grid, kind, s.cuda_stream), 2 * n)
    res[f"flat_{tag}"] = t(lambda: L.probe_copy_var(x.data_ptr(), y.data_ptr(), n, 0, 4, s.cuda_stream), 2 * n)
    del x, y
print(json.dumps({k: round(v, 1) for k, v in res.items()}))
