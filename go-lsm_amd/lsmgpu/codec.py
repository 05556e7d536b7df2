"""Python driver of the gfx950 block codec (tests and bench).

Device memory and streams come from PyTorch (plumbing); every computation
runs in liblsm_gpu.so through the C ABI (include/lsm_gpu.h).  Unsigned C
types are carried in signed torch dtypes of the same width (uint64 -> int64,
uint32 -> int32); the bits are what matter.
"""
from dataclasses import dataclass
from typing import Optional

import ctypes
import numpy as np
import torch

from . import _lib

GRAMMAR_V, GRAMMAR_KV, GRAMMAR_IDX = 0, 1, 2

STATUS_NAMES = {
    0: "ok",
    1: "truncated length prefix",
    2: "truncated key",
    3: "key too long",
    4: "truncated value length",
    5: "value too long",
    6: "truncated value",
    7: "index overrun",
    8: "capacity",
}

DESC_DTYPE = np.dtype([("rec_off", "<u8"), ("key_len", "<u4"), ("val_len", "<u4")])

# go-lsm defaults: bloom.go:79-82, sstable.go:21
DEFAULT_BLOOM_M = 1_600_000
DEFAULT_BLOOM_K = 16
MAX_SSTABLE_SIZE = 2 * 1024 * 1024


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream_handle(stream: Optional[torch.cuda.Stream]):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


INPUT_SLACK = _lib.INPUT_SLACK  # LSM_INPUT_SLACK, include/lsm_gpu.h (checked at load)


def pad16(n: int) -> int:
    """Device inputs must be readable to roundup16(n) + LSM_INPUT_SLACK."""
    return ((n + 15) // 16) * 16 + INPUT_SLACK


def _writable(a: np.ndarray) -> np.ndarray:
    """A contiguous array torch.from_numpy may wrap: read-only inputs (e.g.
    np.frombuffer over bytes) are copied first, since torch cannot mark the
    tensor read-only and warns of undefined behaviour."""
    a = np.ascontiguousarray(a)
    return a if a.flags.writeable else a.copy()


def _dev_i64(a: np.ndarray, dev) -> torch.Tensor:
    return torch.from_numpy(_writable(a).view(np.int64)).to(dev)


def to_device_bytes(buf: np.ndarray, device) -> torch.Tensor:
    """Copy a host byte array into a 16-byte padded device buffer."""
    n = int(buf.nbytes)
    t = torch.zeros(pad16(n), dtype=torch.uint8, device=device)
    if n:
        t[:n].copy_(torch.from_numpy(_writable(buf).view(np.uint8).reshape(-1)))
    return t


class Context:
    """One lsm_ctx per device (and per host thread in concurrent use)."""

    def __init__(self, device: int = 0):
        self.lib = _lib.load()
        self.device = device
        h = ctypes.c_void_p()
        _lib.check(self.lib.lsm_ctx_create(device, ctypes.byref(h)), "lsm_ctx_create")
        self.handle = h
        self.torch_device = torch.device("cuda", device)

    def close(self):
        if self.handle:
            self.lib.lsm_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def num_cus(self) -> int:
        return self.lib.lsm_ctx_num_cus(self.handle)


@dataclass
class DecodePlan:
    """Device-side output placement of one batch (lsm_plan_*)."""

    rec_base: torch.Tensor            # int64[nblk+1]
    arena_base: Optional[torch.Tensor]
    workspace: torch.Tensor
    total_records: int                # capacity (rec_base[nblk])


MIN_RECORD = {GRAMMAR_V: 4, GRAMMAR_KV: 8, GRAMMAR_IDX: 12}


@dataclass
class DecodeResult:
    desc: torch.Tensor                # int32[cap, 4] = lsm_rec_desc
    nrec: torch.Tensor                # int32[nblk]
    status: torch.Tensor              # int32[nblk]
    rec_base: Optional[torch.Tensor]  # int64[nblk+1], or None = offset-addressed
    idx_value: Optional[torch.Tensor] = None
    key_arena: Optional[torch.Tensor] = None
    val_arena: Optional[torch.Tensor] = None
    arena_base: Optional[torch.Tensor] = None
    key_arena_off: Optional[torch.Tensor] = None
    val_arena_off: Optional[torch.Tensor] = None

    grammar: int = GRAMMAR_KV

    def desc_numpy(self) -> np.ndarray:
        return self.desc.cpu().numpy().view(np.uint8).view(DESC_DTYPE).reshape(-1)

    def bases(self, blk_off: np.ndarray) -> np.ndarray:
        """Slot of each block's first record (host copy)."""
        if self.rec_base is not None:
            return self.rec_base.cpu().numpy().view(np.uint64)[:-1]
        return np.asarray(blk_off, dtype=np.uint64) // np.uint64(MIN_RECORD[self.grammar])

    def arena_bases(self, blk_off: np.ndarray) -> np.ndarray:
        if self.arena_base is not None:
            return self.arena_base.cpu().numpy().view(np.uint64)[:-1]
        return np.asarray(blk_off, dtype=np.uint64)


def plan(ctx: Context, grammar: int, blk_len: torch.Tensor, arena: bool = False,
         stream=None) -> DecodePlan:
    nblk = int(blk_len.numel())
    dev = ctx.torch_device
    ws = torch.empty(max(int(ctx.lib.lsm_plan_workspace_bytes(nblk)), 16), dtype=torch.uint8,
                     device=dev)
    rec_base = torch.empty(nblk + 1, dtype=torch.int64, device=dev)
    sh = _stream_handle(stream)
    _lib.check(ctx.lib.lsm_plan_rec_base(ctx.handle, grammar, _ptr(blk_len), nblk,
                                         _ptr(rec_base), _ptr(ws), ws.numel(), sh),
               "lsm_plan_rec_base")
    arena_base = None
    if arena:
        arena_base = torch.empty(nblk + 1, dtype=torch.int64, device=dev)
        _lib.check(ctx.lib.lsm_plan_arena_base(ctx.handle, _ptr(blk_len), nblk,
                                               _ptr(arena_base), _ptr(ws), ws.numel(), sh),
                   "lsm_plan_arena_base")
    total = int(rec_base[nblk].item()) if nblk else 0
    return DecodePlan(rec_base, arena_base, ws, total)


def replan(ctx: Context, grammar: int, blk_len: torch.Tensor, p: DecodePlan, stream=None):
    """Recompute rec_base in place (no host sync): the plan step of a timed loop."""
    nblk = int(blk_len.numel())
    _lib.check(ctx.lib.lsm_plan_rec_base(ctx.handle, grammar, _ptr(blk_len), nblk,
                                         _ptr(p.rec_base), _ptr(p.workspace),
                                         p.workspace.numel(), _stream_handle(stream)),
               "lsm_plan_rec_base")
    if p.arena_base is not None:
        _lib.check(ctx.lib.lsm_plan_arena_base(ctx.handle, _ptr(blk_len), nblk, _ptr(p.arena_base),
                                               _ptr(p.workspace), p.workspace.numel(),
                                               _stream_handle(stream)), "lsm_plan_arena_base")


def alloc_decode(ctx: Context, grammar: int, nblk: int, p: DecodePlan,
                 arena: bool = False, arena_offsets: bool = False) -> DecodeResult:
    dev = ctx.torch_device
    cap = max(p.total_records, 1)
    r = DecodeResult(
        desc=torch.empty((cap, 4), dtype=torch.int32, device=dev),
        nrec=torch.empty(max(nblk, 1), dtype=torch.int32, device=dev),
        status=torch.empty(max(nblk, 1), dtype=torch.int32, device=dev),
        rec_base=p.rec_base, grammar=grammar,
    )
    if grammar == GRAMMAR_IDX:
        r.idx_value = torch.empty(cap, dtype=torch.int64, device=dev)
    if arena:
        nbytes = int(p.arena_base[nblk].item()) if nblk else 0
        r.arena_base = p.arena_base
        if grammar != GRAMMAR_V:
            r.key_arena = torch.zeros(pad16(nbytes), dtype=torch.uint8, device=dev)
        if grammar != GRAMMAR_IDX:
            r.val_arena = torch.zeros(pad16(nbytes), dtype=torch.uint8, device=dev)
        if arena_offsets:
            if grammar != GRAMMAR_V:
                r.key_arena_off = torch.empty(cap, dtype=torch.int64, device=dev)
            if grammar != GRAMMAR_IDX:
                r.val_arena_off = torch.empty(cap, dtype=torch.int64, device=dev)
    return r


def alloc_decode_offset(ctx: Context, grammar: int, nblk: int, in_bytes: int,
                        arena: bool = False, arena_offsets: bool = False) -> DecodeResult:
    """Outputs for offset-addressed placement (rec_base = arena_base = NULL):
    block b's records at slots blk_off[b]/R.., its arena bytes at blk_off[b]."""
    dev = ctx.torch_device
    cap = in_bytes // MIN_RECORD[grammar] + 1
    r = DecodeResult(
        desc=torch.empty((cap, 4), dtype=torch.int32, device=dev),
        nrec=torch.empty(max(nblk, 1), dtype=torch.int32, device=dev),
        status=torch.empty(max(nblk, 1), dtype=torch.int32, device=dev),
        rec_base=None, grammar=grammar)
    if grammar == GRAMMAR_IDX:
        r.idx_value = torch.empty(cap, dtype=torch.int64, device=dev)
    if arena:
        if grammar != GRAMMAR_V:
            r.key_arena = torch.zeros(pad16(in_bytes), dtype=torch.uint8, device=dev)
        if grammar != GRAMMAR_IDX:
            r.val_arena = torch.zeros(pad16(in_bytes), dtype=torch.uint8, device=dev)
        if arena_offsets:
            if grammar != GRAMMAR_V:
                r.key_arena_off = torch.empty(cap, dtype=torch.int64, device=dev)
            if grammar != GRAMMAR_IDX:
                r.val_arena_off = torch.empty(cap, dtype=torch.int64, device=dev)
    return r


def _decode_out(r: DecodeResult):
    return _lib.DecodeOut(
        desc=r.desc.data_ptr(),
        rec_base=r.rec_base.data_ptr() if r.rec_base is not None else None,
        nrec=r.nrec.data_ptr(),
        status=r.status.data_ptr(),
        idx_value=r.idx_value.data_ptr() if r.idx_value is not None else None,
        key_arena=r.key_arena.data_ptr() if r.key_arena is not None else None,
        val_arena=r.val_arena.data_ptr() if r.val_arena is not None else None,
        arena_base=r.arena_base.data_ptr() if r.arena_base is not None else None,
        key_arena_off=r.key_arena_off.data_ptr() if r.key_arena_off is not None else None,
        val_arena_off=r.val_arena_off.data_ptr() if r.val_arena_off is not None else None,
    )


def decode_into(ctx: Context, grammar: int, d_in: torch.Tensor, blk_off: torch.Tensor,
                blk_len: torch.Tensor, r: DecodeResult, stream=None,
                schedule: Optional[torch.Tensor] = None, max_blk_len: Optional[int] = None) -> None:
    """lsm_decode_blocks into preallocated outputs (asynchronous).  With a
    `schedule` workspace (schedule_workspace()): lsm_decode_blocks_scheduled,
    the blocks launched largest first (for batches whose sizes vary).  With
    `max_blk_len`: lsm_decode_blocks_hinted (the ring chosen for that bound).
    The two are exclusive: the scheduled path picks its own (2 KiB) ring."""
    if max_blk_len is not None and schedule is not None:
        raise ValueError("decode_into: pass either schedule or max_blk_len, not both")
    out = _decode_out(r)
    if max_blk_len is not None:
        _lib.check(ctx.lib.lsm_decode_blocks_hinted(
            ctx.handle, grammar, _ptr(d_in), _ptr(blk_off), _ptr(blk_len), int(blk_off.numel()),
            int(max_blk_len), ctypes.byref(out), _stream_handle(stream)), "lsm_decode_blocks_hinted")
        return
    if schedule is not None:
        _lib.check(ctx.lib.lsm_decode_blocks_scheduled(
            ctx.handle, grammar, _ptr(d_in), _ptr(blk_off), _ptr(blk_len), int(blk_off.numel()),
            ctypes.byref(out), _ptr(schedule), schedule.numel(), _stream_handle(stream)),
            "lsm_decode_blocks_scheduled")
        return
    _lib.check(ctx.lib.lsm_decode_blocks(ctx.handle, grammar, _ptr(d_in), _ptr(blk_off),
                                         _ptr(blk_len), int(blk_off.numel()), ctypes.byref(out),
                                         _stream_handle(stream)), "lsm_decode_blocks")


def schedule_workspace(ctx: Context, nblk: int) -> torch.Tensor:
    n = int(ctx.lib.lsm_decode_schedule_workspace_bytes(nblk))
    return torch.empty(max(n, 16), dtype=torch.uint8, device=ctx.torch_device)


def decode_blocks(ctx: Context, grammar: int, d_in: torch.Tensor, blk_off: torch.Tensor,
                  blk_len: torch.Tensor, arena: bool = False, arena_offsets: bool = False,
                  placement: str = "plan", stream=None) -> DecodeResult:
    """placement: "plan" (dense CSR capacity via lsm_plan_*) or "offset"
    (offset-addressed, no plan; blocks must not overlap)."""
    nblk = int(blk_off.numel())
    if placement == "offset":
        r = alloc_decode_offset(ctx, grammar, nblk, int(d_in.numel()), arena=arena,
                                arena_offsets=arena_offsets)
    else:
        p = plan(ctx, grammar, blk_len, arena=arena, stream=stream)
        r = alloc_decode(ctx, grammar, nblk, p, arena=arena, arena_offsets=arena_offsets)
    if nblk:
        decode_into(ctx, grammar, d_in, blk_off, blk_len, r, stream=stream)
    return r


@dataclass
class DenseRecords:
    """lsm_compact_records output: block b's records at desc[base[b]:base[b+1]]."""
    desc: torch.Tensor                # int32[cap, 4]
    base: torch.Tensor                # int64[nblk+1]
    idx_value: Optional[torch.Tensor]
    workspace: torch.Tensor


def alloc_dense(ctx: Context, grammar: int, nblk: int, cap: int) -> DenseRecords:
    dev = ctx.torch_device
    return DenseRecords(
        desc=torch.empty((max(cap, 1), 4), dtype=torch.int32, device=dev),
        base=torch.empty(nblk + 1, dtype=torch.int64, device=dev),
        idx_value=torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
        if grammar == GRAMMAR_IDX else None,
        workspace=torch.empty(max(int(ctx.lib.lsm_plan_workspace_bytes(nblk)), 16),
                              dtype=torch.uint8, device=dev))


def compact_into(ctx: Context, grammar: int, blk_off: torch.Tensor, r: DecodeResult,
                 d: DenseRecords, stream=None) -> None:
    """lsm_compact_records (asynchronous): the decode's records, dense."""
    out = _decode_out(r)
    _lib.check(ctx.lib.lsm_compact_records(
        ctx.handle, grammar, _ptr(blk_off), int(blk_off.numel()), ctypes.byref(out),
        _ptr(d.desc), _ptr(d.idx_value), _ptr(d.base), _ptr(d.workspace), d.workspace.numel(),
        _stream_handle(stream)), "lsm_compact_records")


def wal_workspace(ctx: Context, nwal: int, max_len: int) -> torch.Tensor:
    n = int(ctx.lib.lsm_wal_replay_workspace_bytes(nwal, max_len))
    return torch.empty(max(n, 16), dtype=torch.uint8, device=ctx.torch_device)


def wal_replay_into(ctx: Context, d_wal: torch.Tensor, wal_off: torch.Tensor,
                    wal_len: torch.Tensor, max_len: int, r: DecodeResult, ws: torch.Tensor,
                    stream=None) -> None:
    """lsm_wal_replay (wal.Recover, wal/wal.go:95-121) into preallocated outputs."""
    out = _decode_out(r)
    _lib.check(ctx.lib.lsm_wal_replay(ctx.handle, _ptr(d_wal), _ptr(wal_off), _ptr(wal_len),
                                      int(wal_off.numel()), max_len, ctypes.byref(out), _ptr(ws),
                                      ws.numel(), _stream_handle(stream)), "lsm_wal_replay")


def wal_replay(ctx: Context, d_wal: torch.Tensor, wal_off: torch.Tensor, wal_len: torch.Tensor,
               max_len: Optional[int] = None, stream=None) -> DecodeResult:
    """Replay nwal logs; offset-addressed outputs (record slots wal_off/8..)."""
    nwal = int(wal_off.numel())
    if max_len is None:
        max_len = int(wal_len.max().item()) if nwal else 0
    r = alloc_decode_offset(ctx, GRAMMAR_KV, nwal, int(d_wal.numel()))
    if nwal:
        wal_replay_into(ctx, d_wal, wal_off, wal_len, max_len, r,
                        wal_workspace(ctx, nwal, max_len), stream=stream)
    return r


# ---- whole .sst files (lsm_decode_sst) ----------------------------------------

SST_META_DTYPE = np.dtype([
    ("min_key_off", "<u8"), ("min_key_len", "<u8"), ("max_key_off", "<u8"), ("max_key_len", "<u8"),
    ("filter_m", "<u8"), ("filter_k", "<u8"), ("filter_nbits", "<u8"), ("filter_words_off", "<u8"),
    ("data_off", "<i8"), ("data_size", "<i8"), ("idx_off", "<i8"), ("idx_size", "<i8"),
    ("stage", "<i4"), ("status", "<i4"), ("nidx", "<u4"), ("ndata", "<u4")])
assert SST_META_DTYPE.itemsize == 112

SST_STAGE_NAMES = {0: "ok", 1: "header", 2: "filter", 3: "footer", 4: "index", 5: "data",
                   6: "mismatch"}


@dataclass
class SstDecode:
    """lsm_decode_sst outputs: file f's entries at slots base(f).. of the
    per-record arrays (offset addressing: base(f) = file_off[f] // 4)."""
    meta: torch.Tensor        # uint8[nfile * 112] = lsm_sst_meta
    idx_desc: torch.Tensor    # int32[cap, 4]
    idx_value: torch.Tensor   # int64[cap]
    data_desc: torch.Tensor   # int32[cap, 4]
    workspace: torch.Tensor
    d_file_off: torch.Tensor
    d_file_len: torch.Tensor
    file_off: np.ndarray
    nfile: int

    def meta_numpy(self) -> np.ndarray:
        return self.meta.cpu().numpy().view(SST_META_DTYPE).reshape(-1)

    def bases(self) -> np.ndarray:
        return self.file_off // 4


def alloc_sst_decode(ctx: Context, file_off: np.ndarray, file_len: np.ndarray,
                     img_bytes: int) -> SstDecode:
    dev = ctx.torch_device
    file_off = np.ascontiguousarray(file_off, dtype=np.uint64)
    file_len = np.ascontiguousarray(file_len, dtype=np.uint64)
    nf = file_off.size
    cap = img_bytes // 4 + 1
    ws = int(ctx.lib.lsm_decode_sst_workspace_bytes(nf))
    return SstDecode(
        meta=torch.zeros(max(nf, 1) * SST_META_DTYPE.itemsize, dtype=torch.uint8, device=dev),
        idx_desc=torch.zeros((cap, 4), dtype=torch.int32, device=dev),
        idx_value=torch.zeros(cap, dtype=torch.int64, device=dev),
        data_desc=torch.zeros((cap, 4), dtype=torch.int32, device=dev),
        workspace=torch.empty(max(ws, 16), dtype=torch.uint8, device=dev),
        d_file_off=_dev_i64(file_off, dev),
        d_file_len=_dev_i64(file_len, dev),
        file_off=file_off, nfile=nf)


def decode_sst_into(ctx: Context, d_img: torch.Tensor, r: SstDecode, stream=None) -> None:
    _lib.check(ctx.lib.lsm_decode_sst(
        ctx.handle, _ptr(d_img), _ptr(r.d_file_off), _ptr(r.d_file_len), r.nfile, None,
        _ptr(r.meta), _ptr(r.idx_desc), _ptr(r.idx_value), _ptr(r.data_desc), _ptr(r.workspace),
        r.workspace.numel(), _stream_handle(stream)), "lsm_decode_sst")


def decode_sst(ctx: Context, d_img: torch.Tensor, file_off: np.ndarray, file_len: np.ndarray,
               stream=None) -> SstDecode:
    """Decode whole .sst images (SSTable.DecodeFrom + DecodeDataBlock +
    GetKeyValuePairs) held in d_img at file_off[f], file_len[f] bytes each."""
    r = alloc_sst_decode(ctx, file_off, file_len, int(d_img.numel()))
    if r.nfile:
        decode_sst_into(ctx, d_img, r, stream=stream)
    return r


def may_contain_workspace(ctx: Context, nfile: int, nkeys: int) -> torch.Tensor:
    n = int(ctx.lib.lsm_may_contain_workspace_bytes(nfile, nkeys))
    return torch.empty(max(n, 16), dtype=torch.uint8, device=ctx.torch_device)


def may_contain_into(ctx: Context, d_img: torch.Tensor, r: SstDecode, batch: "RecordBatch",
                     hit: torch.Tensor, ws: Optional[torch.Tensor] = None, stream=None) -> None:
    """lsm_may_contain: SSTable.MayContain of every key of `batch` against
    every file decoded into r; hit viewed as uint8[nkeys, nfile]."""
    if ws is None:
        ws = may_contain_workspace(ctx, r.nfile, batch.n)
    _lib.check(ctx.lib.lsm_may_contain(ctx.handle, _ptr(d_img), _ptr(r.d_file_off), _ptr(r.meta),
                                       r.nfile, _ptr(batch.keys), _ptr(batch.koff), batch.n,
                                       _ptr(hit), _ptr(ws), ws.numel(), _stream_handle(stream)),
               "lsm_may_contain")


def may_contain(ctx: Context, d_img: torch.Tensor, r: SstDecode, batch: "RecordBatch",
                stream=None) -> torch.Tensor:
    hit = torch.zeros((max(batch.n, 1), max(r.nfile, 1)), dtype=torch.uint8,
                      device=ctx.torch_device)
    if batch.n and r.nfile:
        may_contain_into(ctx, d_img, r, batch, hit, stream=stream)
    return hit


def level_may_contain_workspace(ctx: Context, nfile: int, nkeys: int) -> torch.Tensor:
    n = int(ctx.lib.lsm_level_may_contain_workspace_bytes(nfile, nkeys))
    return torch.empty(max(n, 16), dtype=torch.uint8, device=ctx.torch_device)


def level_index(ctx: Context, d_img: torch.Tensor, r: SstDecode, stream=None) -> torch.Tensor:
    """lsm_level_index_build: the level's sparse index (Manager.sparseIndexes),
    parsed once from the decoded tables' headers; valid with this d_img."""
    idx = torch.empty(max(int(ctx.lib.lsm_level_index_bytes(r.nfile)), 16), dtype=torch.uint8,
                      device=ctx.torch_device)
    if r.nfile:
        _lib.check(ctx.lib.lsm_level_index_build(
            ctx.handle, _ptr(d_img), _ptr(r.d_file_off), _ptr(r.meta), r.nfile, _ptr(idx),
            _stream_handle(stream)), "lsm_level_index_build")
    return idx


def level_may_contain_into(ctx: Context, d_img: torch.Tensor, r: SstDecode, batch: "RecordBatch",
                           table: torch.Tensor, may: torch.Tensor,
                           ws: Optional[torch.Tensor] = None, stream=None,
                           index: Optional[torch.Tensor] = None) -> None:
    """lsm_level_may_contain: searchFromLevelWithSparseIndex's candidate table
    (int32 per key, -1 for an empty level) and its MayContain (uint8 per key)
    for a level >= 1 whose tables were decoded into r in sparse-index order.
    index (level_index): lsm_level_may_contain_indexed, the headers not parsed
    again."""
    if ws is None:
        ws = level_may_contain_workspace(ctx, r.nfile, batch.n)
    if index is not None:
        _lib.check(ctx.lib.lsm_level_may_contain_indexed(
            ctx.handle, _ptr(d_img) if r.nfile else None, _ptr(index) if r.nfile else None,
            r.nfile, _ptr(batch.keys), _ptr(batch.koff), batch.n, _ptr(table), _ptr(may), _ptr(ws),
            ws.numel(), _stream_handle(stream)), "lsm_level_may_contain_indexed")
        return
    _lib.check(ctx.lib.lsm_level_may_contain(
        ctx.handle, _ptr(d_img) if r.nfile else None, _ptr(r.d_file_off) if r.nfile else None,
        _ptr(r.meta) if r.nfile else None, r.nfile, _ptr(batch.keys), _ptr(batch.koff), batch.n,
        _ptr(table), _ptr(may), _ptr(ws), ws.numel(), _stream_handle(stream)),
        "lsm_level_may_contain")


def level_may_contain(ctx: Context, d_img: torch.Tensor, r: SstDecode, batch: "RecordBatch",
                      stream=None):
    """-> (table int32[nkeys], may uint8[nkeys]) on the device."""
    table = torch.empty(max(batch.n, 1), dtype=torch.int32, device=ctx.torch_device)
    may = torch.empty(max(batch.n, 1), dtype=torch.uint8, device=ctx.torch_device)
    if batch.n:
        level_may_contain_into(ctx, d_img, r, batch, table, may, stream=stream)
    return table[:batch.n], may[:batch.n]


GET_ABSENT, GET_FOUND, GET_SEEK_FAILED, GET_VALUE_LENGTH, GET_VALUE_TOO_LONG, GET_VALUE_SHORT = range(6)


@dataclass
class SeekTree:
    """lsm_level_get_tree_build's output for one level: the tree bytes and the
    max_nidx it was built for (tables above it walk the index)."""
    data: torch.Tensor
    max_nidx: int


def level_get_tree(ctx: Context, d_img: torch.Tensor, r: SstDecode, max_nidx: Optional[int] = None,
                   stream=None) -> SeekTree:
    """The level's Seek tree (lsm_level_get_tree_build), built once per level
    load.  max_nidx None = the largest decoded nidx (read back once)."""
    if max_nidx is None:
        max_nidx = int(r.meta_numpy()[:r.nfile]["nidx"].max()) if r.nfile else 0
    nb = int(ctx.lib.lsm_level_get_tree_bytes(r.nfile, max_nidx))
    data = torch.empty(max(nb, 16), dtype=torch.uint8, device=ctx.torch_device)
    if r.nfile and nb:
        _lib.check(ctx.lib.lsm_level_get_tree_build(
            ctx.handle, _ptr(d_img), _ptr(r.d_file_off), _ptr(r.meta), r.nfile, None,
            _ptr(r.idx_desc), max_nidx, _ptr(data), nb, _stream_handle(stream)),
            "lsm_level_get_tree_build")
    return SeekTree(data, max_nidx)


def level_get_into(ctx: Context, d_img: torch.Tensor, r: SstDecode, batch: "RecordBatch",
                   table: torch.Tensor, may: torch.Tensor, result: torch.Tensor,
                   value: torch.Tensor, tree: Optional[SeekTree] = None, stream=None) -> None:
    """lsm_level_get: searchFromTable past MayContain for each key with
    may = 1 -- Iterator.Seek over its table's decoded index, then the value
    (GetValueByOffset).  result int32 per key (GET_*), value int32[nkeys, 4]
    (a lsm_rec_desc view of the value in d_img on GET_FOUND).  tree
    (level_get_tree) walks the bisection through the Seek tree; None walks
    the index (the same answers)."""
    _lib.check(ctx.lib.lsm_level_get(
        ctx.handle, _ptr(d_img) if r.nfile else None, _ptr(r.d_file_off) if r.nfile else None,
        _ptr(r.d_file_len) if r.nfile else None, _ptr(r.meta) if r.nfile else None, r.nfile, None,
        _ptr(r.idx_desc) if r.nfile else None, _ptr(r.idx_value) if r.nfile else None,
        _ptr(batch.keys), _ptr(batch.koff), batch.n, _ptr(table), _ptr(may), _ptr(result),
        _ptr(value), _ptr(tree.data) if tree is not None else None,
        tree.max_nidx if tree is not None else 0, tree.data.numel() if tree is not None else 0,
        _stream_handle(stream)), "lsm_level_get")


def level_get(ctx: Context, d_img: torch.Tensor, r: SstDecode, batch: "RecordBatch",
              table: torch.Tensor, may: torch.Tensor, tree: Optional[SeekTree] = None,
              stream=None):
    """-> (result int32[nkeys], value int32[nkeys, 4]) on the device."""
    result = torch.empty(max(batch.n, 1), dtype=torch.int32, device=ctx.torch_device)
    value = torch.empty((max(batch.n, 1), 4), dtype=torch.int32, device=ctx.torch_device)
    if batch.n:
        level_get_into(ctx, d_img, r, batch, table, may, result, value, tree=tree, stream=stream)
    return result[:batch.n], value[:batch.n]


def level_search_get_into(ctx: Context, d_img: torch.Tensor, r: SstDecode, batch: "RecordBatch",
                          index: torch.Tensor, table: torch.Tensor, may: torch.Tensor,
                          result: torch.Tensor, value: torch.Tensor, tree: Optional[SeekTree] = None,
                          ws: Optional[torch.Tensor] = None, stream=None) -> None:
    """lsm_level_search_get: a level's whole batched Get in one call --
    searchFromLevelWithSparseIndex then searchFromTable -- the outputs of
    level_may_contain_into (table, may) and level_get_into (result, value)."""
    if ws is None:
        ws = level_may_contain_workspace(ctx, r.nfile, batch.n)
    nf = r.nfile
    _lib.check(ctx.lib.lsm_level_search_get(
        ctx.handle, _ptr(d_img) if nf else None, _ptr(index) if nf else None, nf,
        _ptr(r.d_file_off) if nf else None, _ptr(r.d_file_len) if nf else None, _ptr(r.meta) if nf else None,
        None, _ptr(r.idx_desc) if nf else None, _ptr(r.idx_value) if nf else None,
        _ptr(batch.keys), _ptr(batch.koff), batch.n, _ptr(table), _ptr(may), _ptr(result), _ptr(value),
        _ptr(tree.data) if tree is not None else None, tree.max_nidx if tree is not None else 0,
        tree.data.numel() if tree is not None else 0, _ptr(ws), ws.numel(), _stream_handle(stream)),
        "lsm_level_search_get")


def level_search_get(ctx: Context, d_img: torch.Tensor, r: SstDecode, batch: "RecordBatch",
                     tree: Optional[SeekTree] = None, index: Optional[torch.Tensor] = None, stream=None):
    """-> (table, may, result, value) on the device."""
    dev = ctx.torch_device
    n = max(batch.n, 1)
    table = torch.empty(n, dtype=torch.int32, device=dev)
    may = torch.empty(n, dtype=torch.uint8, device=dev)
    result = torch.empty(n, dtype=torch.int32, device=dev)
    value = torch.empty((n, 4), dtype=torch.int32, device=dev)
    if index is None:
        index = level_index(ctx, d_img, r, stream=stream)
    if batch.n:
        level_search_get_into(ctx, d_img, r, batch, index, table, may, result, value, tree=tree, stream=stream)
    return table[:batch.n], may[:batch.n], result[:batch.n], value[:batch.n]


def level0_get_into(ctx: Context, d_img: torch.Tensor, r: SstDecode, batch: "RecordBatch",
                    table: torch.Tensor, result: torch.Tensor, value: torch.Tensor,
                    tree: Optional[SeekTree] = None, stream=None) -> None:
    """lsm_level0_get: searchFromLevel0 (manager.go:160-176) over r's tables in
    order (newest first): MayContain, Seek and the value per table until the
    first value or error.  table int32 per key (the answering table or -1),
    result / value as level_get_into."""
    _lib.check(ctx.lib.lsm_level0_get(
        ctx.handle, _ptr(d_img) if r.nfile else None, _ptr(r.d_file_off) if r.nfile else None,
        _ptr(r.d_file_len) if r.nfile else None, _ptr(r.meta) if r.nfile else None, r.nfile, None,
        _ptr(r.idx_desc) if r.nfile else None, _ptr(r.idx_value) if r.nfile else None,
        _ptr(batch.keys), _ptr(batch.koff), batch.n, _ptr(table), _ptr(result), _ptr(value),
        _ptr(tree.data) if tree is not None else None, tree.max_nidx if tree is not None else 0,
        tree.data.numel() if tree is not None else 0, _stream_handle(stream)), "lsm_level0_get")


def level0_get(ctx: Context, d_img: torch.Tensor, r: SstDecode, batch: "RecordBatch",
               tree: Optional[SeekTree] = None, stream=None):
    """-> (table int32[nkeys], result int32[nkeys], value int32[nkeys, 4]) on the device."""
    dev = ctx.torch_device
    table = torch.empty(max(batch.n, 1), dtype=torch.int32, device=dev)
    result = torch.empty(max(batch.n, 1), dtype=torch.int32, device=dev)
    value = torch.empty((max(batch.n, 1), 4), dtype=torch.int32, device=dev)
    if batch.n:
        level0_get_into(ctx, d_img, r, batch, table, result, value, tree=tree, stream=stream)
    return table[:batch.n], result[:batch.n], value[:batch.n]


# ---- encode -----------------------------------------------------------------

@dataclass
class RecordBatch:
    """Columnar (CSR) record batch on the device."""

    keys: torch.Tensor   # uint8, 16-byte padded
    koff: torch.Tensor   # int64[n+1]
    vals: torch.Tensor
    voff: torch.Tensor
    n: int
    koff_host: np.ndarray
    voff_host: np.ndarray


def batch_to_device(ctx: Context, keys: np.ndarray, koff: np.ndarray, vals: np.ndarray,
                    voff: np.ndarray) -> RecordBatch:
    dev = ctx.torch_device
    koff = np.ascontiguousarray(koff, dtype=np.uint64)
    voff = np.ascontiguousarray(voff, dtype=np.uint64)
    return RecordBatch(
        keys=to_device_bytes(keys, dev),
        koff=_dev_i64(koff, dev),
        vals=to_device_bytes(vals, dev),
        voff=_dev_i64(voff, dev),
        n=len(koff) - 1, koff_host=koff, voff_host=voff)


def encoded_size(grammar: int, koff: np.ndarray, voff: np.ndarray, r0: int, r1: int) -> int:
    n = r1 - r0
    if grammar == GRAMMAR_V:
        return 4 * n + int(voff[r1] - voff[r0])
    if grammar == GRAMMAR_KV:
        return 8 * n + int(koff[r1] - koff[r0]) + int(voff[r1] - voff[r0])
    return 12 * n + int(koff[r1] - koff[r0])


def encode_blocks(ctx: Context, grammar: int, batch: RecordBatch, rec_start: np.ndarray,
                  out_off: Optional[np.ndarray] = None, out_bytes: Optional[int] = None,
                  idx_off: Optional[np.ndarray] = None, stream=None):
    """Encode block b = records [rec_start[b], rec_start[b+1]) at out_off[b].
    Returns (d_out, out_off)."""
    dev = ctx.torch_device
    rec_start = np.ascontiguousarray(rec_start, dtype=np.uint64)
    nblk = len(rec_start) - 1
    sizes = np.array([encoded_size(grammar, batch.koff_host, batch.voff_host,
                                   int(rec_start[b]), int(rec_start[b + 1]))
                      for b in range(nblk)], dtype=np.uint64)
    if out_off is None:
        out_off = np.zeros(nblk, dtype=np.uint64)
        if nblk:
            out_off[1:] = np.cumsum(sizes)[:-1]
    out_off = np.ascontiguousarray(out_off, dtype=np.uint64)
    if out_bytes is None:
        out_bytes = int((out_off + sizes).max()) if nblk else 0
    d_out = torch.zeros(pad16(out_bytes), dtype=torch.uint8, device=dev)
    d_rs = _dev_i64(rec_start, dev)
    d_oo = _dev_i64(out_off, dev)
    d_io = None
    if grammar == GRAMMAR_IDX:
        d_io = torch.from_numpy(np.ascontiguousarray(idx_off, dtype=np.int64)).to(dev)
    _lib.check(ctx.lib.lsm_encode_blocks(
        ctx.handle, grammar, _ptr(batch.keys), _ptr(batch.koff), _ptr(batch.vals),
        _ptr(batch.voff), _ptr(d_io), _ptr(d_rs), nblk, _ptr(d_out), _ptr(d_oo),
        _stream_handle(stream)), "lsm_encode_blocks")
    return d_out, out_off


# ---- .sst build ---------------------------------------------------------------

def segment_files(ctx: Context, koff: np.ndarray, voff: np.ndarray,
                  threshold: int = MAX_SSTABLE_SIZE) -> np.ndarray:
    koff = np.ascontiguousarray(koff, dtype=np.uint64)
    voff = np.ascontiguousarray(voff, dtype=np.uint64)
    n = len(koff) - 1
    starts = np.zeros(n + 2, dtype=np.uint64)
    nf = ctx.lib.lsm_segment_files_host(koff.ctypes.data, voff.ctypes.data, n, threshold,
                                        starts.ctypes.data)
    return starts[: nf + 1].copy()


class SstBuild:
    """Inputs / outputs of lsm_build_sst for nfile images.  The layout
    (file_start, file_off, file_size) lives on the device; the host copies
    are made on first use (prepare_sst_device computes the layout on the
    device, so nothing is read back before the build)."""

    def __init__(self, out, footer, workspace, d_file_start, d_file_off, max_recs, m, k, nfile,
                 file_start=None, file_off=None, file_size=None, d_file_size=None, stream=None):
        self.out, self.footer, self.workspace = out, footer, workspace
        self.d_file_start, self.d_file_off, self.d_file_size = d_file_start, d_file_off, d_file_size
        self.max_recs, self.m, self.k, self.nfile = max_recs, m, k, nfile
        self._file_start, self._file_off, self._file_size = file_start, file_off, file_size
        self.stream = stream  # the stream the device layout (and the build) run on

    def _host(self, t, n):
        # the layout kernel ran on self.stream, which need not be torch's
        # current stream: wait for it before the first host copy
        if self.stream is not None:
            self.stream.synchronize()
        return t[:n].cpu().numpy().view(np.uint64).copy()

    @property
    def file_start(self) -> np.ndarray:
        if self._file_start is None:
            self._file_start = self._host(self.d_file_start, self.nfile + 1)
        return self._file_start

    @property
    def file_off(self) -> np.ndarray:
        if self._file_off is None:
            self._file_off = self._host(self.d_file_off, self.nfile)
        return self._file_off

    @property
    def file_size(self) -> np.ndarray:
        if self._file_size is None:
            self._file_size = self._host(self.d_file_size, self.nfile)
        return self._file_size


def prepare_sst(ctx: Context, batch: RecordBatch, file_start: np.ndarray,
                m: int = DEFAULT_BLOOM_M, k: int = DEFAULT_BLOOM_K, align: int = 16) -> SstBuild:
    dev = ctx.torch_device
    file_start = np.ascontiguousarray(file_start, dtype=np.uint64)
    nf = len(file_start) - 1
    koff, voff = batch.koff_host, batch.voff_host
    sizes = np.array([ctx.lib.lsm_sst_image_size_host(koff.ctypes.data, voff.ctypes.data,
                                                      int(file_start[f]), int(file_start[f + 1]),
                                                      m) for f in range(nf)], dtype=np.uint64)
    padded = (sizes + (align - 1)) // align * align
    file_off = np.zeros(nf, dtype=np.uint64)
    if nf:
        file_off[1:] = np.cumsum(padded)[:-1]
    total = int(padded.sum())
    max_recs = int(np.diff(file_start.astype(np.int64)).max()) if nf else 0
    ws_bytes = int(ctx.lib.lsm_build_sst_workspace_bytes(nf, max_recs, m, k))
    return SstBuild(
        out=torch.zeros(pad16(total), dtype=torch.uint8, device=dev),
        file_start=file_start, file_off=file_off, file_size=sizes,
        footer=torch.zeros(max(nf, 1) * 4, dtype=torch.int64, device=dev),
        workspace=torch.empty(ws_bytes, dtype=torch.uint8, device=dev),
        d_file_start=_dev_i64(file_start, dev),
        d_file_off=_dev_i64(file_off, dev),
        max_recs=max_recs, m=m, k=k, nfile=nf)


def build_sst_into(ctx: Context, batch: RecordBatch, sb: SstBuild, stream=None) -> None:
    nf = sb.nfile
    _lib.check(ctx.lib.lsm_build_sst(
        ctx.handle, _ptr(batch.keys), _ptr(batch.koff), _ptr(batch.vals), _ptr(batch.voff),
        _ptr(sb.d_file_start), nf, sb.max_recs, sb.m, sb.k, _ptr(sb.out), _ptr(sb.d_file_off),
        _ptr(sb.footer), _ptr(sb.workspace), sb.workspace.numel(), _stream_handle(stream)),
        "lsm_build_sst")


def build_sst(ctx: Context, batch: RecordBatch, file_start: np.ndarray,
              m: int = DEFAULT_BLOOM_M, k: int = DEFAULT_BLOOM_K, stream=None) -> SstBuild:
    sb = prepare_sst(ctx, batch, file_start, m=m, k=k)
    build_sst_into(ctx, batch, sb, stream=stream)
    return sb


class SstStream:
    """lsm_build_sst_stream's buffers for one sorted stream: the rule, the
    layout and the images in one call, sized on lsm_stream_max_files' bound.
    The counts stay on the device ({nfile, most records in a file, image
    bytes, overflow}); result() reads them back after the build."""

    def __init__(self, ctx, batch, threshold, m, k, align):
        dev = ctx.torch_device
        lib = ctx.lib
        n = batch.n
        kb, vb = int(batch.keys.numel()), int(batch.vals.numel())
        self.threshold, self.m, self.k, self.align, self.n = threshold, m, k, align, n
        self.nfile_max = int(lib.lsm_stream_max_files(n, kb, vb, threshold))
        out_bytes = int(lib.lsm_build_sst_stream_out_bytes(n, kb, vb, self.nfile_max, m, align))
        ws = int(lib.lsm_build_sst_stream_workspace_bytes(n, threshold, self.nfile_max, m, k))
        self.out = torch.empty(pad16(max(out_bytes, 1)), dtype=torch.uint8, device=dev)
        self.workspace = torch.empty(max(ws, 16), dtype=torch.uint8, device=dev)
        self.d_file_start = torch.empty(self.nfile_max + 1, dtype=torch.int64, device=dev)
        self.d_file_off = torch.empty(self.nfile_max + 1, dtype=torch.int64, device=dev)
        self.footer = torch.empty(max(self.nfile_max, 1) * 4, dtype=torch.int64, device=dev)
        self.counts = torch.zeros(4, dtype=torch.int64, device=dev)
        self._koff, self._voff = batch.koff, batch.voff
        self._filter = int(lib.lsm_filter_block_size(m))

    def result(self) -> "SstBuild":
        """The build as an SstBuild with host copies of its layout (reads
        back; raises on overflow)."""
        torch.cuda.synchronize(self.out.device)
        c = self.counts.cpu().numpy().view(np.uint64)
        if int(c[3]):
            raise RuntimeError("lsm_build_sst_stream: the stream needs more than nfile_max files")
        nf = int(c[0])
        fs = self.d_file_start[:nf + 1].cpu().numpy().view(np.uint64).copy()
        fo = self.d_file_off[:nf + 1].cpu().numpy().view(np.uint64).copy()
        # image sizes (sstable.go:131-193) from the device offsets
        ko, vo = self._koff, self._voff
        r0, r1 = self.d_file_start[:nf], self.d_file_start[1:nf + 1]
        sz = (8 + (ko[r0 + 1] - ko[r0]) + (ko[r1] - ko[r1 - 1]) + self._filter + 16 * (r1 - r0) +
              (ko[r1] - ko[r0]) + (vo[r1] - vo[r0]) + 32) if nf else torch.zeros(0, dtype=torch.int64)
        return SstBuild(out=self.out, footer=self.footer, workspace=self.workspace,
                        d_file_start=self.d_file_start[:nf + 1], d_file_off=self.d_file_off[:nf + 1],
                        max_recs=int(c[1]), m=self.m, k=self.k, nfile=nf, file_start=fs,
                        file_off=fo[:nf], file_size=sz.cpu().numpy().view(np.uint64).copy(),
                        d_file_size=None)


def prepare_sst_stream(ctx: Context, batch: RecordBatch, threshold: int = MAX_SSTABLE_SIZE,
                       m: int = DEFAULT_BLOOM_M, k: int = DEFAULT_BLOOM_K, align: int = 16) -> SstStream:
    return SstStream(ctx, batch, threshold, m, k, align)


def build_sst_stream_into(ctx: Context, batch: RecordBatch, ss: SstStream, stream=None) -> None:
    """lsm_build_sst_stream: Builder.Add / ShouldFlush / Build over the sorted
    stream (merge.go:106-128) with SSTable.EncodeTo and Filter.Add per file."""
    _lib.check(ctx.lib.lsm_build_sst_stream(
        ctx.handle, _ptr(batch.keys), _ptr(batch.koff), _ptr(batch.vals), _ptr(batch.voff), batch.n,
        ss.threshold, ss.nfile_max, ss.m, ss.k, ss.align, _ptr(ss.out), _ptr(ss.d_file_start),
        _ptr(ss.d_file_off), _ptr(ss.footer), _ptr(ss.counts), _ptr(ss.workspace),
        ss.workspace.numel(), _stream_handle(stream)), "lsm_build_sst_stream")


def build_sst_stream(ctx: Context, batch: RecordBatch, threshold: int = MAX_SSTABLE_SIZE,
                     m: int = DEFAULT_BLOOM_M, k: int = DEFAULT_BLOOM_K, align: int = 16,
                     stream=None) -> SstStream:
    ss = prepare_sst_stream(ctx, batch, threshold, m, k, align)
    build_sst_stream_into(ctx, batch, ss, stream=stream)
    return ss


def segment_files_device(ctx: Context, batch: RecordBatch, threshold: int = MAX_SSTABLE_SIZE,
                         nfile_max: Optional[int] = None, stream=None):
    """lsm_segment_files (the builder rule on the device) -> (file starts as a
    host array, counts {nfile, most records in a file, 0, overflow})."""
    dev = ctx.torch_device
    if nfile_max is None:
        nfile_max = int(ctx.lib.lsm_stream_max_files(batch.n, int(batch.keys.numel()),
                                                     int(batch.vals.numel()), threshold))
    fs = torch.full((nfile_max + 1,), -1, dtype=torch.int64, device=dev)
    counts = torch.full((4,), -1, dtype=torch.int64, device=dev)
    _lib.check(ctx.lib.lsm_segment_files(ctx.handle, _ptr(batch.koff), _ptr(batch.voff), batch.n,
                                         threshold, nfile_max, _ptr(fs), _ptr(counts),
                                         _stream_handle(stream)), "lsm_segment_files")
    torch.cuda.synchronize(dev)
    c = counts.cpu().numpy().view(np.uint64).copy()
    return fs[:int(c[0]) + 1].cpu().numpy().view(np.uint64).copy(), c


def sum256(ctx: Context, batch: RecordBatch, stream=None) -> torch.Tensor:
    out = torch.empty((max(batch.n, 1), 4), dtype=torch.int64, device=ctx.torch_device)
    _lib.check(ctx.lib.lsm_sum256(ctx.handle, _ptr(batch.keys), _ptr(batch.koff), batch.n,
                                  _ptr(out), _stream_handle(stream)), "lsm_sum256")
    return out


def bloom_probe(ctx: Context, words: torch.Tensor, m: int, k: int, batch: RecordBatch,
                stream=None) -> torch.Tensor:
    hit = torch.empty(max(batch.n, 1), dtype=torch.uint8, device=ctx.torch_device)
    _lib.check(ctx.lib.lsm_bloom_probe(ctx.handle, _ptr(words), m, k, _ptr(batch.keys),
                                       _ptr(batch.koff), batch.n, _ptr(hit),
                                       _stream_handle(stream)), "lsm_bloom_probe")
    return hit


# ---- compaction merge ------------------------------------

TOMBSTONE = "～DELETED～".encode()  # kv.DeletedValue (kv/kv.go:29)


@dataclass
class Merge:
    """lsm_merge_kvs outputs: out[:nout] = input indices of the written pairs,
    file_start[:nfiles + 1] = each file's first position in out."""
    out: torch.Tensor         # int32[n] (u32 indices)
    file_start: torch.Tensor  # int64[n + 1]
    workspace: torch.Tensor
    n: int
    nout: int = 0
    nfiles: int = 0
    max_recs: int = 0  # the most pairs in one output file


def alloc_merge(ctx: Context, n: int) -> Merge:
    dev = ctx.torch_device
    ws = int(ctx.lib.lsm_merge_kvs_workspace_bytes(n))
    return Merge(out=torch.empty(max(n, 1), dtype=torch.int32, device=dev),
                 file_start=torch.empty(n + 1, dtype=torch.int64, device=dev),
                 workspace=torch.empty(ws, dtype=torch.uint8, device=dev), n=n)


TIE_INPUT, TIE_GOHEAP = 0, 1  # enum lsm_tie


def merge_kvs_into(ctx: Context, d_bytes: torch.Tensor, key_desc: torch.Tensor,
                   val_desc: Optional[torch.Tensor], r: Merge, level: int = 1,
                   threshold: int = MAX_SSTABLE_SIZE, stream=None, tie: int = TIE_INPUT,
                   d_counts: Optional[torch.Tensor] = None) -> Merge:
    """CompactAndMergeKVs (merge.go:42-94) over pairs given as descriptors
    (key: IDX/KV descriptor, value: V descriptor or None for KV records).
    tie=TIE_GOHEAP: equal keys in container/heap's pop order (exact).
    d_counts (device int64[3]): lsm_merge_kvs_async -- the counts are left
    there, not read back (r.nout / nfiles / max_recs are not set)."""
    if d_counts is not None:
        _lib.check(ctx.lib.lsm_merge_kvs_async(
            ctx.handle, _ptr(d_bytes), _ptr(key_desc), _ptr(val_desc), r.n, level, threshold, tie,
            _ptr(r.out), _ptr(r.file_start), _ptr(d_counts), _ptr(r.workspace),
            r.workspace.numel(), _stream_handle(stream)), "lsm_merge_kvs_async")
        return r
    counts = np.zeros(3, np.uint64)
    _lib.check(ctx.lib.lsm_merge_kvs_tie(
        ctx.handle, _ptr(d_bytes), _ptr(key_desc), _ptr(val_desc), r.n, level, threshold, tie,
        _ptr(r.out), _ptr(r.file_start), counts.ctypes.data, _ptr(r.workspace),
        r.workspace.numel(), _stream_handle(stream)), "lsm_merge_kvs_tie")
    r.nout, r.nfiles, r.max_recs = int(counts[0]), int(counts[1]), int(counts[2])
    return r


def merge_kvs(ctx: Context, d_bytes: torch.Tensor, key_desc: torch.Tensor,
              val_desc: Optional[torch.Tensor], level: int = 1,
              threshold: int = MAX_SSTABLE_SIZE, stream=None, tie: int = TIE_INPUT) -> Merge:
    r = alloc_merge(ctx, int(key_desc.shape[0]))
    return merge_kvs_into(ctx, d_bytes, key_desc, val_desc, r, level, threshold, stream, tie)


def goheap_pop_order(ctx_or_lib, rank: np.ndarray, phases: bool = False):
    """lsm_goheap_pop_order_host: container/heap's pop order over key ranks.
    phases=True -> (order, push_ms, pop_ms)."""
    lib = ctx_or_lib.lib if isinstance(ctx_or_lib, Context) else ctx_or_lib
    rank = np.ascontiguousarray(rank, dtype=np.uint32)
    order = np.zeros(max(rank.size, 1), np.uint32)
    ns = np.zeros(2, np.uint64)
    _lib.check(lib.lsm_goheap_pop_order_host(rank.ctypes.data, rank.size, order.ctypes.data, ns.ctypes.data),
               "lsm_goheap_pop_order_host")
    if phases:
        return order[:rank.size], float(ns[0]) / 1e6, float(ns[1]) / 1e6
    return order[:rank.size]


def gather_kvs(ctx: Context, d_bytes: torch.Tensor, key_desc: torch.Tensor,
               val_desc: Optional[torch.Tensor], idx: torch.Tensor, nout: int,
               key_bytes: int, val_bytes: int, stream=None,
               reuse: Optional[RecordBatch] = None, d_nout: Optional[torch.Tensor] = None) -> RecordBatch:
    """The selected pairs as a device CSR batch (lsm_build_sst's input);
    key_bytes / val_bytes bound the selected bytes.  koff_host / voff_host
    are left None (use sst_layout for the image sizes).  reuse: an earlier
    result whose buffers are large enough is written again (a compaction
    loop allocates once)."""
    dev = ctx.torch_device
    kb, vb = pad16(max(key_bytes, 1)), (pad16(max(val_bytes, 1)) if val_bytes is not None else None)
    wsb = int(ctx.lib.lsm_gather_kvs_workspace_bytes(nout))
    if (reuse is not None and reuse.koff.numel() >= nout + 1 and reuse.keys.numel() >= kb and
            (vb is None) == (reuse.vals is None) and (vb is None or reuse.vals.numel() >= vb) and
            getattr(reuse, "_ws", None) is not None and reuse._ws.numel() >= wsb):
        keys, vals, koff, voff, ws = reuse.keys, reuse.vals, reuse.koff, reuse.voff, reuse._ws
    else:
        keys = torch.empty(kb, dtype=torch.uint8, device=dev)
        vals = torch.empty(vb, dtype=torch.uint8, device=dev) if vb is not None else None
        koff = torch.empty(nout + 1, dtype=torch.int64, device=dev)  # vals None: keys only
        voff = torch.empty(nout + 1, dtype=torch.int64, device=dev)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    if d_nout is not None:  # lsm_gather_kvs_dev: the count on the device, nout its bound
        _lib.check(ctx.lib.lsm_gather_kvs_dev(
            ctx.handle, _ptr(d_bytes), _ptr(key_desc), _ptr(val_desc), _ptr(idx), _ptr(d_nout), nout,
            _ptr(keys), _ptr(koff), _ptr(vals), _ptr(voff), _ptr(ws), ws.numel(),
            _stream_handle(stream)), "lsm_gather_kvs_dev")
    else:
        _lib.check(ctx.lib.lsm_gather_kvs(
            ctx.handle, _ptr(d_bytes), _ptr(key_desc), _ptr(val_desc), _ptr(idx), nout, _ptr(keys),
            _ptr(koff), _ptr(vals), _ptr(voff), _ptr(ws), ws.numel(), _stream_handle(stream)),
            "lsm_gather_kvs")
    out = RecordBatch(keys=keys, koff=koff, vals=vals, voff=voff, n=nout, koff_host=None,
                      voff_host=None)
    out._ws = ws
    return out


def prepare_sst_device(ctx: Context, batch: RecordBatch, d_file_start: torch.Tensor, nfile: int,
                       max_recs: int, val_bytes: Optional[int] = None,
                       m: int = DEFAULT_BLOOM_M, k: int = DEFAULT_BLOOM_K,
                       align: int = 16, stream=None, reuse: Optional["SstBuild"] = None) -> "SstBuild":
    """prepare_sst for a device-resident batch (a merge's output): the layout
    by lsm_sst_layout on the device, nothing read back.  max_recs = the merge's
    most pairs per file (Merge.max_recs); the image buffer is sized from the
    header's bound (batch.keys bounds the key bytes, val_bytes -- or
    batch.vals -- the value bytes)."""
    dev = ctx.torch_device
    if val_bytes is None:
        if batch.vals is None:
            raise ValueError("prepare_sst_device: val_bytes is required for a keys-only batch")
        val_bytes = int(batch.vals.numel())
    fbytes = int(ctx.lib.lsm_filter_block_size(m))
    bound = (nfile * (fbytes + 40 + align - 1) + 16 * batch.n + 3 * int(batch.keys.numel()) +
             int(val_bytes))
    if reuse is not None and reuse.nfile == nfile:
        d_size, d_off = reuse.d_file_size, reuse.d_file_off
    else:
        d_size = torch.empty(max(nfile, 1), dtype=torch.int64, device=dev)
        d_off = torch.empty(nfile + 1, dtype=torch.int64, device=dev)
    _lib.check(ctx.lib.lsm_sst_layout(
        ctx.handle, _ptr(batch.koff), _ptr(batch.voff), _ptr(d_file_start), nfile, m, align,
        _ptr(d_size), _ptr(d_off), _stream_handle(stream)), "lsm_sst_layout")
    ws_bytes = int(ctx.lib.lsm_build_sst_workspace_bytes(nfile, max_recs, m, k))
    if (reuse is not None and reuse.out.numel() >= pad16(bound) and reuse.footer.numel() >= nfile * 4
            and reuse.workspace.numel() >= ws_bytes):  # reuse: an earlier build's buffers
        out, footer, workspace = reuse.out, reuse.footer, reuse.workspace
    else:  # every image byte and every footer word is written by the build: no fill
        out = torch.empty(pad16(bound), dtype=torch.uint8, device=dev)
        footer = torch.empty(max(nfile, 1) * 4, dtype=torch.int64, device=dev)
        workspace = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    return SstBuild(
        out=out, footer=footer, workspace=workspace,
        d_file_start=d_file_start[:nfile + 1], d_file_off=d_off, d_file_size=d_size,
        max_recs=max_recs, m=m, k=k, nfile=nfile,
        stream=stream if stream is not None else torch.cuda.current_stream(dev))


def sst_pairs_into(ctx: Context, r: "SstDecode", key_out: torch.Tensor, val_out: torch.Tensor,
                   prefix: torch.Tensor, stream=None) -> None:
    """lsm_sst_pairs: the positional join of every decoded file, file after
    file (loadLevelData's allPairs), into dense descriptor arrays."""
    _lib.check(ctx.lib.lsm_sst_pairs(
        ctx.handle, _ptr(r.meta), _ptr(r.d_file_off), r.nfile, _ptr(r.idx_desc), _ptr(r.data_desc),
        _ptr(key_out), _ptr(val_out), _ptr(prefix), _stream_handle(stream)), "lsm_sst_pairs")


def sst_pairs(ctx: Context, r: "SstDecode", stream=None) -> tuple:
    """(key descriptors, value descriptors, prefix) of every file's pairs in
    file order; sized from the decoded metadata."""
    dev = r.idx_desc.device
    cap = int(r.idx_desc.shape[0])
    kd = torch.empty((cap, 4), dtype=torch.int32, device=dev)
    vd = torch.empty((cap, 4), dtype=torch.int32, device=dev)
    prefix = torch.zeros(r.nfile + 1, dtype=torch.int64, device=dev)
    sst_pairs_into(ctx, r, kd, vd, prefix, stream=stream)
    n = int(prefix[r.nfile].item())
    return kd[:n], vd[:n], prefix


def compact_merge_into(ctx: Context, d_img: torch.Tensor, r: "SstDecode", key_out: torch.Tensor,
                       val_out: torch.Tensor, prefix: torch.Tensor, mg: Merge, d_counts: torch.Tensor,
                       level: int = 1, threshold: int = MAX_SSTABLE_SIZE, tie: int = TIE_INPUT,
                       stream=None) -> Merge:
    """lsm_compact_merge_async: sst_pairs_into + merge_kvs_into(d_counts=...)
    in one call (the join, then CompactAndMergeKVs, on one stream).  mg.n
    must be the join's pair count; the counts stay on the device in
    d_counts (int64[3])."""
    _lib.check(ctx.lib.lsm_compact_merge_async(
        ctx.handle, _ptr(d_img), _ptr(r.meta), _ptr(r.d_file_off), r.nfile, _ptr(r.idx_desc),
        _ptr(r.data_desc), mg.n, _ptr(key_out), _ptr(val_out), _ptr(prefix), level, threshold, tie,
        _ptr(mg.out), _ptr(mg.file_start), _ptr(d_counts), _ptr(mg.workspace), mg.workspace.numel(),
        _stream_handle(stream)), "lsm_compact_merge_async")
    return mg


def build_sst_views_into(ctx: Context, batch: RecordBatch, sb: "SstBuild", d_bytes: torch.Tensor,
                         key_desc: torch.Tensor, val_desc: Optional[torch.Tensor],
                         idx: torch.Tensor, stream=None) -> None:
    """lsm_build_sst_views: the images of a keys-only gathered batch, values
    read in place from their views (value i = view of pair idx[i])."""
    nf = sb.nfile
    _lib.check(ctx.lib.lsm_build_sst_views(
        ctx.handle, _ptr(batch.keys), _ptr(batch.koff), _ptr(d_bytes), _ptr(key_desc),
        _ptr(val_desc), _ptr(idx), _ptr(batch.voff), _ptr(sb.d_file_start), nf, sb.max_recs, sb.m,
        sb.k, _ptr(sb.out), _ptr(sb.d_file_off), _ptr(sb.footer), _ptr(sb.workspace),
        sb.workspace.numel(), _stream_handle(stream)), "lsm_build_sst_views")
