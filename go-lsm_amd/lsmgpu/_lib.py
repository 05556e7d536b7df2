"""ctypes declarations of the C ABI in include/lsm_gpu.h.

The product path is liblsm_gpu.so, built in-tree by go-lsm_amd/Makefile.  There
is no fallback: if the library is missing, importing this module raises.
"""
import ctypes
import os

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_PKG_DIR), "liblsm_gpu.so")

c_u8p = ctypes.c_void_p
c_u32p = ctypes.c_void_p
c_u64p = ctypes.c_void_p


class DecodeOut(ctypes.Structure):
    """struct lsm_decode_out (include/lsm_gpu.h)."""

    _fields_ = [
        ("desc", ctypes.c_void_p),
        ("rec_base", ctypes.c_void_p),
        ("nrec", ctypes.c_void_p),
        ("status", ctypes.c_void_p),
        ("idx_value", ctypes.c_void_p),
        ("key_arena", ctypes.c_void_p),
        ("val_arena", ctypes.c_void_p),
        ("arena_base", ctypes.c_void_p),
        ("key_arena_off", ctypes.c_void_p),
        ("val_arena_off", ctypes.c_void_p),
    ]


# name -> (restype, argtypes)
SIGNATURES = {
    "lsm_abi_version": (ctypes.c_int, []),
    "lsm_input_slack": (ctypes.c_int, []),
    "lsm_build_id": (ctypes.c_char_p, []),
    "lsm_build_flags": (ctypes.c_char_p, []),
    "lsm_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "lsm_ctx_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "lsm_ctx_num_cus": (ctypes.c_int, [ctypes.c_void_p]),
    "lsm_max_records": (ctypes.c_uint64, [ctypes.c_int, ctypes.c_uint64]),
    "lsm_plan_workspace_bytes": (ctypes.c_size_t, [ctypes.c_uint32]),
    "lsm_plan_rec_base": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, c_u32p, ctypes.c_uint32,
                                         c_u64p, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_void_p]),
    "lsm_plan_arena_base": (ctypes.c_int, [ctypes.c_void_p, c_u32p, ctypes.c_uint32, c_u64p,
                                           ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_decode_blocks": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, c_u8p, c_u64p, c_u32p,
                                         ctypes.c_uint32, ctypes.POINTER(DecodeOut),
                                         ctypes.c_void_p]),
    "lsm_decode_blocks_hinted": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, c_u8p, c_u64p, c_u32p,
                                                ctypes.c_uint32, ctypes.c_uint32,
                                                ctypes.POINTER(DecodeOut), ctypes.c_void_p]),
    "lsm_decode_schedule_workspace_bytes": (ctypes.c_size_t, [ctypes.c_uint32]),
    "lsm_decode_blocks_scheduled": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, c_u8p, c_u64p,
                                                   c_u32p, ctypes.c_uint32,
                                                   ctypes.POINTER(DecodeOut), ctypes.c_void_p,
                                                   ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_compact_records": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, c_u64p, ctypes.c_uint32,
                                           ctypes.POINTER(DecodeOut), ctypes.c_void_p,
                                           ctypes.c_void_p, c_u64p, ctypes.c_void_p,
                                           ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_encoded_size_host": (ctypes.c_uint64, [ctypes.c_int, c_u64p, c_u64p, ctypes.c_uint64,
                                                ctypes.c_uint64]),
    "lsm_encode_blocks": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, c_u8p, c_u64p, c_u8p,
                                         c_u64p, ctypes.c_void_p, c_u64p, ctypes.c_uint32, c_u8p,
                                         c_u64p, ctypes.c_void_p]),
    "lsm_segment_files_host": (ctypes.c_uint64, [c_u64p, c_u64p, ctypes.c_uint64,
                                                 ctypes.c_uint64, c_u64p]),
    "lsm_sst_image_size_host": (ctypes.c_uint64, [c_u64p, c_u64p, ctypes.c_uint64,
                                                  ctypes.c_uint64, ctypes.c_uint64]),
    "lsm_filter_block_size": (ctypes.c_uint64, [ctypes.c_uint64]),
    "lsm_build_sst_workspace_bytes": (ctypes.c_size_t, [ctypes.c_uint32, ctypes.c_uint32,
                                                         ctypes.c_uint64, ctypes.c_uint32]),
    "lsm_build_sst": (ctypes.c_int, [ctypes.c_void_p, c_u8p, c_u64p, c_u8p, c_u64p, c_u64p,
                                     ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
                                     ctypes.c_uint32, c_u8p, c_u64p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_build_sst_views": (ctypes.c_int, [ctypes.c_void_p, c_u8p, c_u64p, c_u8p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p, c_u64p, c_u64p,
                                           ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
                                           ctypes.c_uint32, c_u8p, c_u64p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_bloom_probe": (ctypes.c_int, [ctypes.c_void_p, c_u64p, ctypes.c_uint64, ctypes.c_uint32,
                                       c_u8p, c_u64p, ctypes.c_uint64, c_u8p, ctypes.c_void_p]),
    "lsm_sum256": (ctypes.c_int, [ctypes.c_void_p, c_u8p, c_u64p, ctypes.c_uint64, c_u64p,
                                  ctypes.c_void_p]),
    "lsm_bloom_build": (ctypes.c_int, [ctypes.c_void_p, c_u8p, c_u64p, ctypes.c_uint64,
                                       ctypes.c_uint64, ctypes.c_uint32, c_u64p,
                                       ctypes.c_void_p]),
    "lsm_wal_replay_workspace_bytes": (ctypes.c_size_t, [ctypes.c_uint32, ctypes.c_uint32]),
    "lsm_wal_replay": (ctypes.c_int, [ctypes.c_void_p, c_u8p, c_u64p, c_u32p, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.POINTER(DecodeOut), ctypes.c_void_p,
                                      ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_decode_sst_workspace_bytes": (ctypes.c_size_t, [ctypes.c_uint32]),
    "lsm_decode_sst": (ctypes.c_int, [ctypes.c_void_p, c_u8p, c_u64p, c_u64p, ctypes.c_uint32,
                                      c_u64p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_void_p]),
    "lsm_may_contain_workspace_bytes": (ctypes.c_size_t, [ctypes.c_uint32, ctypes.c_uint64]),
    "lsm_may_contain": (ctypes.c_int, [ctypes.c_void_p, c_u8p, c_u64p, ctypes.c_void_p,
                                       ctypes.c_uint32, c_u8p, c_u64p, ctypes.c_uint64, c_u8p,
                                       ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_level_may_contain_workspace_bytes": (ctypes.c_size_t, [ctypes.c_uint32, ctypes.c_uint64]),
    "lsm_level_may_contain": (ctypes.c_int, [ctypes.c_void_p, c_u8p, c_u64p, ctypes.c_void_p,
                                             ctypes.c_uint32, c_u8p, c_u64p, ctypes.c_uint64,
                                             ctypes.c_void_p, c_u8p, ctypes.c_void_p,
                                             ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_level_index_bytes": (ctypes.c_size_t, [ctypes.c_uint32]),
    "lsm_level_index_build": (ctypes.c_int, [ctypes.c_void_p, c_u8p, c_u64p, ctypes.c_void_p,
                                             ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    "lsm_level_may_contain_indexed": (ctypes.c_int, [ctypes.c_void_p, c_u8p, ctypes.c_void_p,
                                                     ctypes.c_uint32, c_u8p, c_u64p,
                                                     ctypes.c_uint64, ctypes.c_void_p, c_u8p,
                                                     ctypes.c_void_p, ctypes.c_size_t,
                                                     ctypes.c_void_p]),
    "lsm_level_get": (ctypes.c_int, [ctypes.c_void_p, c_u8p, c_u64p, c_u64p, ctypes.c_void_p,
                                     ctypes.c_uint32, c_u64p, ctypes.c_void_p, ctypes.c_void_p,
                                     c_u8p, c_u64p, ctypes.c_uint64, ctypes.c_void_p, c_u8p,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_uint32, ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_level_search_get": (ctypes.c_int, [ctypes.c_void_p, c_u8p, ctypes.c_void_p, ctypes.c_uint32,
                                            c_u64p, c_u64p, ctypes.c_void_p, c_u64p, ctypes.c_void_p,
                                            ctypes.c_void_p, c_u8p, c_u64p, ctypes.c_uint64,
                                            ctypes.c_void_p, c_u8p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t,
                                            ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_level0_get": (ctypes.c_int, [ctypes.c_void_p, c_u8p, c_u64p, c_u64p, ctypes.c_void_p,
                                      ctypes.c_uint32, c_u64p, ctypes.c_void_p, ctypes.c_void_p,
                                      c_u8p, c_u64p, ctypes.c_uint64, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_uint32, ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_level_get_tree_bytes": (ctypes.c_size_t, [ctypes.c_uint32, ctypes.c_uint32]),
    "lsm_level_get_tree_build": (ctypes.c_int, [ctypes.c_void_p, c_u8p, c_u64p, ctypes.c_void_p,
                                                ctypes.c_uint32, c_u64p, ctypes.c_void_p,
                                                ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t,
                                                ctypes.c_void_p]),
    "lsm_merge_kvs_workspace_bytes": (ctypes.c_size_t, [ctypes.c_uint64]),
    "lsm_merge_kvs": (ctypes.c_int, [ctypes.c_void_p, c_u8p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p,
                                     c_u64p, c_u64p, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_void_p]),
    "lsm_merge_kvs_tie": (ctypes.c_int, [ctypes.c_void_p, c_u8p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64,
                                         ctypes.c_int, ctypes.c_void_p, c_u64p, c_u64p,
                                         ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_merge_kvs_async": (ctypes.c_int, [ctypes.c_void_p, c_u8p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64,
                                           ctypes.c_int, ctypes.c_void_p, c_u64p, c_u64p,
                                           ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_compact_merge_async": (ctypes.c_int, [ctypes.c_void_p, c_u8p, ctypes.c_void_p, c_u64p,
                                               ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                               c_u64p, ctypes.c_int, ctypes.c_uint64, ctypes.c_int,
                                               ctypes.c_void_p, c_u64p, c_u64p, ctypes.c_void_p,
                                               ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_goheap_pop_order_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                                 ctypes.c_void_p]),
    "lsm_goheap_replays": (ctypes.c_uint64, [ctypes.c_void_p]),
    "lsm_gather_kvs_workspace_bytes": (ctypes.c_size_t, [ctypes.c_uint64]),
    "lsm_gather_kvs": (ctypes.c_int, [ctypes.c_void_p, c_u8p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_uint64, c_u8p, c_u64p, c_u8p,
                                      c_u64p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_gather_kvs_dev": (ctypes.c_int, [ctypes.c_void_p, c_u8p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, c_u64p, ctypes.c_uint64, c_u8p, c_u64p,
                                          c_u8p, c_u64p, ctypes.c_void_p, ctypes.c_size_t,
                                          ctypes.c_void_p]),
    "lsm_stream_max_files": (ctypes.c_uint32, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                               ctypes.c_uint64]),
    "lsm_segment_files": (ctypes.c_int, [ctypes.c_void_p, c_u64p, c_u64p, ctypes.c_uint64,
                                         ctypes.c_uint64, ctypes.c_uint32, c_u64p, c_u64p,
                                         ctypes.c_void_p]),
    "lsm_build_sst_stream_workspace_bytes": (ctypes.c_size_t, [ctypes.c_uint64, ctypes.c_uint64,
                                                                ctypes.c_uint32, ctypes.c_uint64,
                                                                ctypes.c_uint32]),
    "lsm_build_sst_stream_out_bytes": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64,
                                                          ctypes.c_uint64, ctypes.c_uint32,
                                                          ctypes.c_uint64, ctypes.c_uint32]),
    "lsm_build_sst_stream": (ctypes.c_int, [ctypes.c_void_p, c_u8p, c_u64p, c_u8p, c_u64p,
                                            ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                            ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, c_u8p,
                                            c_u64p, c_u64p, ctypes.c_void_p, c_u64p,
                                            ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_sst_image_sizes": (ctypes.c_int, [ctypes.c_void_p, c_u64p, c_u64p, c_u64p,
                                           ctypes.c_uint32, ctypes.c_uint64, c_u64p,
                                           ctypes.c_void_p]),
    "lsm_sst_layout": (ctypes.c_int, [ctypes.c_void_p, c_u64p, c_u64p, c_u64p, ctypes.c_uint32,
                                      ctypes.c_uint64, ctypes.c_uint32, c_u64p, c_u64p,
                                      ctypes.c_void_p]),
    "lsm_sst_pairs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, c_u64p, ctypes.c_uint32,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, c_u64p, ctypes.c_void_p]),
    "lsm_dev_alloc": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.POINTER(ctypes.c_void_p)]),
    "lsm_dev_free": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "lsm_host_alloc_pinned": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t,
                                             ctypes.POINTER(ctypes.c_void_p)]),
    "lsm_host_free_pinned": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "lsm_memcpy_h2d": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_memcpy_d2h": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_memset_dev": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                      ctypes.c_size_t, ctypes.c_void_p]),
    "lsm_stream_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "lsm_stream_destroy": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "lsm_stream_sync": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
}

ABI_VERSION = 7   # LSM_ABI_VERSION this binding is written against
INPUT_SLACK = 32  # LSM_INPUT_SLACK: device inputs are padded by this much

_lib = None
# scripts/ab_lib.py clears this to load a diagnostic variant built from
# patched sources; the product path always checks
CHECK_BUILD_ID = True


def load():
    """Load liblsm_gpu.so (in-tree).  Raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `make -C go-lsm_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.lsm_abi_version() != ABI_VERSION or lib.lsm_input_slack() != INPUT_SLACK:
        raise RuntimeError(
            f"{LIB_PATH}: ABI {lib.lsm_abi_version()} / input slack {lib.lsm_input_slack()}, "
            f"this binding expects ABI {ABI_VERSION} / slack {INPUT_SLACK}: rebuild")
    # the library must be built from the sources beside it (build_id.py): a
    # stale prebuilt liblsm_gpu.so never stands in for the current tree
    pkg = os.path.dirname(_PKG_DIR)
    if CHECK_BUILD_ID and os.path.isdir(os.path.join(pkg, "csrc")):
        import importlib.util
        spec = importlib.util.spec_from_file_location("_lsm_build_id", os.path.join(pkg, "build_id.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        # hashed with the compiler, target and flags the library records it
        # was built with (a `make ARCH=... HIPFLAGS=...` build is accepted)
        flags = lib.lsm_build_flags().decode().split("|")
        want = mod.source_id(pkg, flags=flags if len(flags) == 3 else None)
        have = lib.lsm_build_id().decode()
        if want != have:
            raise RuntimeError(
                f"{LIB_PATH} was built from other sources (build id {have}, the tree's "
                f"sources hash to {want}): rebuild with `make -C go-lsm_amd`")
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc}")
    return rc
