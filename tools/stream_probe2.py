"""decode64k's launch shape without the parse (tools only): 6,400 x 64 KiB
blocks, one wave per block (grid = nblk) vs persistent grids."""
import ctypes, json, os
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbm_probe.so"))
L.probe_stream.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                           ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
blk, nblk = 65536, 6400
x = torch.randint(0, 255, (nblk * blk + 64,), dtype=torch.uint8, device="cuda")
sink = torch.zeros(4, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
cus = torch.cuda.get_device_properties(0).multi_processor_count
def t(fn, nbytes, reps=50):
    for _ in range(3): fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record(s)
    for _ in range(reps): fn()
    e1.record(s); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return round(nbytes / (ms * 1e-3) / 1e9, 1), round(ms * 1e3, 1)
res = {}
for nch in (4, 8, 16):
    for g in (nblk, cus * 8, cus * 16, cus * 25, cus * 32):
        if nch * (g // cus if g != nblk else 25) > 160: continue
        res[f"nch{nch}_grid{g}"] = t(lambda: L.probe_stream(nch, x.data_ptr(), nblk, blk, sink.data_ptr(), g, s.cuda_stream), nblk * blk)
print(json.dumps(res))
