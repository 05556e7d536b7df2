"""lsmgpu — Python driver of the MI355X (gfx950) go-lsm SSTable block codec.

The codec itself is liblsm_gpu.so (HIP kernels + C ABI, include/lsm_gpu.h).
This package only moves buffers (PyTorch) and calls the C ABI (ctypes).
"""
from . import _lib  # noqa: F401
from .codec import (  # noqa: F401
    DEFAULT_BLOOM_K, DEFAULT_BLOOM_M, DESC_DTYPE, GRAMMAR_IDX, GRAMMAR_KV, GRAMMAR_V,
    MAX_SSTABLE_SIZE, STATUS_NAMES, Context, DenseRecords, alloc_decode, alloc_decode_offset,
    alloc_dense, batch_to_device, bloom_probe, build_sst, build_sst_into, compact_into,
    decode_blocks, decode_into, schedule_workspace, encode_blocks, pad16, plan, prepare_sst, replan, segment_files,
    sum256, to_device_bytes, SST_META_DTYPE, SST_STAGE_NAMES, SstDecode, alloc_sst_decode,
    decode_sst, decode_sst_into, wal_replay, wal_replay_into, wal_workspace,
    may_contain, may_contain_into, may_contain_workspace, level_may_contain,
    level_may_contain_into, level_may_contain_workspace, level_index, level_get, level_get_into,
    level_get_tree, SeekTree, level0_get, level0_get_into, level_search_get, level_search_get_into,
    GET_ABSENT, GET_FOUND, GET_SEEK_FAILED, GET_VALUE_LENGTH, GET_VALUE_TOO_LONG, GET_VALUE_SHORT, Merge, alloc_merge, merge_kvs, merge_kvs_into, gather_kvs,
    prepare_sst_device, sst_pairs, sst_pairs_into, compact_merge_into, TOMBSTONE, build_sst_views_into,
    TIE_INPUT, TIE_GOHEAP, goheap_pop_order,
    SstStream, prepare_sst_stream, build_sst_stream, build_sst_stream_into, segment_files_device)
from . import synth  # noqa: F401
