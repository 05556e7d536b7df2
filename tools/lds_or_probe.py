"""LDS bit-set throughput per mode of tools/lds_or_probe.hip (see its header).
Prints one JSON line: per mode, µs per launch and ORs retired per clock per CU
(at 2.4 GHz).  Tools only, never the product."""
import ctypes, json, os, sys
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(ROOT, "tools", "liblds_or_probe.so"))
L.lds_or_probe.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                           ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
ncu = torch.cuda.get_device_properties(0).multi_processor_count
grid = int(sys.argv[1]) if len(sys.argv) > 1 else ncu
per = 256
out = torch.zeros(grid * 1024, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
res = {"grid": grid, "per_thread": per, "cus": ncu}
names = {0: "or_all", 1: "or_half", 2: "or_conflict_free", 3: "write_all", 4: "valu_only",
         5: "or_half_compacted", 6: "or64_all", 8: "or_half_oob_dropped", 9: "or_half_branchfree"}
outs = {}
for mode in (0, 1, 2, 3, 4, 5, 6, 8, 9):
    span = 1_600_000 if mode in (1, 5, 8, 9) else 800_000
    f = lambda: L.lds_or_probe(mode, grid, 1024, span, per, out.data_ptr(), s.cuda_stream)
    for _ in range(3):
        assert f() == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    reps = 20
    for _ in range(reps):
        f()
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    outs[mode] = out.clone()
    ops = grid * 1024 * per * (0.5 if mode in (1, 5, 8, 9) else 1.0)
    wgs_per_cu = grid / ncu
    res[names[mode]] = {"us": round(us, 2),
                        "ops_per_clk_per_cu": round(ops / ncu / (us * 1e-6 * 2.4e9), 3)}
# the slice bitmaps of modes 5, 8 and 9 must equal mode 1's (same positions)
for mode in (5, 8, 9):
    res[names[mode]]["bitmap_equals_or_half"] = bool(torch.equal(outs[mode], outs[1]))
# LDS bounds check: a store past the allocation, read back
assert L.lds_or_probe(7, grid, 1024, 800_000, per, out.data_ptr(), s.cuda_stream) == 0
torch.cuda.synchronize()
res["oob_store_readback_nonzero_lanes"] = int((out != 0).sum())
print(json.dumps(res))
