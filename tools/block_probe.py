"""Ceiling of decode4k's memory pattern (tools only): 100,000 x 4 KiB blocks
staged by LDS-DMA, 33 x 16 B descriptors written per block, no parsing.
Compares launch shapes; prints GB/s of (block bytes + descriptor bytes)."""
import ctypes, json, os
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbm_probe.so"))
L.probe_blocks.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
for f in ("probe_read", "probe_read_lds"):
    getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
nblk = 100_000
x = torch.randint(0, 255, (nblk * 4096 + 64,), dtype=torch.uint8, device="cuda")
off = torch.arange(nblk, dtype=torch.int64, device="cuda") * 4096
ln = torch.full((nblk,), 4092, dtype=torch.int32, device="cuda")
out = torch.empty((nblk * 33 * 16,), dtype=torch.uint8, device="cuda")
sink = torch.zeros(4, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
alg = nblk * 4096 + nblk * 33 * 16
def t(fn, nbytes, reps=50):
    for _ in range(5): fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record(s)
    for _ in range(reps): fn()
    e1.record(s); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return round(nbytes / (ms * 1e-3) / 1e9, 1), round(ms * 1e3, 1)
res = {}
names = {0: "dma_wpg4_nometa", 1: "dma_wpg4_meta", 2: "dma_wpg1_meta", 3: "dma_wpg8_meta",
         6: "meta_ntstore", 7: "meta_ntload", 8: "meta_ntload_ntstore", 9: "meta_sc0load",
         10: "meta_sc0sc1load_ntstore"}
for m, nm in names.items():
    res[nm] = t(lambda: L.probe_blocks(m, x.data_ptr(), off.data_ptr(), ln.data_ptr(), nblk, out.data_ptr(), 0, s.cuda_stream), alg)
for g in (1024, 1280, 2048):
    res[f"db_wpg4_g{g}"] = t(lambda: L.probe_blocks(4, x.data_ptr(), 0, 0, nblk, out.data_ptr(), g, s.cuda_stream), alg)
for g in (4096, 5120, 8192):
    res[f"db_wpg1_g{g}"] = t(lambda: L.probe_blocks(5, x.data_ptr(), 0, 0, nblk, out.data_ptr(), g, s.cuda_stream), alg)
n = nblk * 4096
for g in (2048, 8192):
    res[f"read_dwordx4_g{g}"] = t(lambda: L.probe_read(x.data_ptr(), n, sink.data_ptr(), g, s.cuda_stream), n)
    res[f"read_lds_dma_g{g}"] = t(lambda: L.probe_read_lds(x.data_ptr(), n, sink.data_ptr(), g, s.cuda_stream), n)
print(json.dumps(res))
