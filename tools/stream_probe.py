"""Ceiling of long-block streaming through a per-wave LDS ring (tools only):
GB/s of block bytes for ring depth x waves x block size, no parsing."""
import ctypes, json, os
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbm_probe.so"))
L.probe_stream.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                           ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
total = 400 << 20
x = torch.randint(0, 255, (total + 64,), dtype=torch.uint8, device="cuda")
sink = torch.zeros(4, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
cus = torch.cuda.get_device_properties(0).multi_processor_count
def t(fn, nbytes, reps=20):
    for _ in range(3): fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record(s)
    for _ in range(reps): fn()
    e1.record(s); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return round(nbytes / (ms * 1e-3) / 1e9, 1)
res = {}
for blk in (4096, 16384, 65536):
    nblk = total // blk
    for nch in (2, 4, 8, 16, 108, 116):
        if (nch % 100) * 1024 > blk and nch % 100 > 4:
            continue
        for wpc in (4, 8, 10, 16, 20, 32):
            if (nch % 100) * wpc > 160:
                continue
            g = min(cus * wpc, nblk)
            res[f"blk{blk}_nch{nch}_wpc{wpc}"] = t(lambda: L.probe_stream(nch, x.data_ptr(), nblk, blk, sink.data_ptr(), g, s.cuda_stream), nblk * blk)
print(json.dumps(res))
