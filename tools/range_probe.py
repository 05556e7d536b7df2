"""Which buffer stores survive the range check (descriptor of nrec bytes,
voffset 4*lane, soffset so): prints the written dword indices per case."""
import ctypes, json, os
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbm_probe.so"))
L.probe_range.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
res = {}
for nrec, so in ((100, 0), (100, 64), (256, 128), (1 << 20, 0)):
    out = torch.zeros(256, dtype=torch.int32, device="cuda")
    L.probe_range(out.data_ptr(), nrec, so, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    w = torch.nonzero(out).flatten().cpu().tolist()
    res[f"nrec{nrec}_so{so}"] = [w[0], w[-1], len(w)] if w else []
print(json.dumps(res))
