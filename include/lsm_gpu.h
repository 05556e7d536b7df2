/*
 * lsm_gpu.h — C ABI of the MI355X (gfx950) SSTable block codec.
 *
 * Drop-in boundary for the go-lsm hot path (xmh1011/go-lsm @ 2025-08-24):
 * the Go methods it replaces are cited per entry point.  Plain pointers and
 * sizes only; `stream` is an opaque hipStream_t (NULL = default stream).
 * Every launch entry point is asynchronous on `stream`, performs no device
 * allocation and no host synchronisation (hipGraph-capturable) -- except
 * lsm_merge_kvs, which synchronizes `stream` (its radix passes are chosen
 * from key statistics read back to the host); the caller owns every buffer
 * and the library keeps no pointer after the call returns.  lsm_build_sst
 * and lsm_build_sst_views may run part of their launches on the context's
 * side stream, forked from `stream` by an event and joined back into it
 * before they return (so a context serves one caller thread at a time).
 *
 * Device input buffers (blocks, images, logs, key and value arenas) must be
 * readable up to LSM_INPUT_SLACK bytes past the next multiple of 16 bytes
 * after their last byte: roundup16(n) + 32.  The kernels stream 16-byte
 * aligned chunks, and key hashing / bound prefixes load 8-byte words at any
 * key start (up to key_start + 20 for a key ending the buffer).  Bytes past a
 * block or key are never interpreted.  lsm_dev_alloc pads by this much.
 *
 * Return convention: 0 = ok; negative = LSM_E* (argument error) or
 * -(1000 + hipError_t) for a HIP runtime error.
 */
#ifndef LSM_GPU_H
#define LSM_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* v3: the input slack grew from 16 to 32 bytes (a binding built for v2 pads
 * too little); lsm_input_slack() reports it at run time.
 * v4: lsm_merge_kvs_tie writes 3 h_counts entries; lsm_merge_kvs keeps the
 * v2 / v3 contract of exactly 2 ({nout, nfiles}).
 * v5: lsm_merge_kvs_async and lsm_gather_kvs_dev (the merge's counts stay on
 * the device; the gather reads its pair count there); the level sparse index
 * (lsm_level_index_build, lsm_level_may_contain_indexed).
 * v6: lsm_level_get (the batched Get past MayContain: Seek + the value) and
 * its Seek tree (lsm_level_get_tree_bytes, lsm_level_get_tree_build);
 * lsm_compact_merge_async (the join and the merge as one call).
 * v7: the builder rule on the device (lsm_segment_files) and the builder path
 * over one sorted stream as one call (lsm_build_sst_stream: rule, layout and
 * images with the fused bloom, no host round trip); lsm_level_get takes the
 * Seek tree's size; lsm_level0_get (searchFromLevel0 over every table);
 * lsm_level_search_get (a level's search and Get in one call);
 * lsm_goheap_pop_order_host reports its phases, lsm_goheap_replays;
 * lsm_build_flags. */
#define LSM_ABI_VERSION 7
#define LSM_INPUT_SLACK 32  /* readable bytes past roundup16(n) of any device input */

/* Record grammars (all fixed-width little-endian). */
enum lsm_grammar {
    LSM_GRAMMAR_V = 0,   /* ([u32 vlen][value])*            sstable/block/data.go:26-79   */
    LSM_GRAMMAR_KV = 1,  /* ([u32 klen][key][u32 vlen][v])*  kv/kv.go:46-115, wal/wal.go:107 */
    LSM_GRAMMAR_IDX = 2, /* ([u32 klen][key][i64 offset])*   sstable/block/index.go:30-101 */
};

/* Per-block decode status (d_status[b]); d_nrec[b] always counts the
 * records decoded before the status was raised (data.go:75 keeps them). */
enum lsm_status {
    LSM_OK = 0,
    LSM_ST_TRUNC_LEN_PREFIX = 1, /* 1-3 bytes left for a leading u32 length: data.go:65 "read value length failed", kv.go:80 "decode key length" */
    LSM_ST_TRUNC_KEY = 2,        /* kv.go:90 "decode key"                          */
    LSM_ST_KEY_TOO_LONG = 3,     /* kv.go:84 "invalid key length: %d" (> 1<<20)   */
    LSM_ST_TRUNC_VLEN = 4,       /* kv.go:98 "decode value length"                 */
    LSM_ST_VAL_TOO_LONG = 5,     /* kv.go:102 "invalid value length: %d" (> 1<<30) */
    LSM_ST_TRUNC_VAL = 6,        /* data.go:71 "read value data failed", kv.go:108 "decode value" */
    LSM_ST_IDX_OVERRUN = 7,      /* an index entry crosses the block's end: see below */
    LSM_ST_CAPACITY = 8,         /* record capacity rec_base[b+1]-rec_base[b] exhausted (not a reference error) */
};

/* LSM_ST_IDX_OVERRUN and the reference's three messages.  IndexBlock.DecodeFrom
 * (index.go:61-101) reads an entry whole -- Key.DecodeFrom, then the i64
 * offset -- and only then compares totalRead with the size.  Which error Go
 * returns for an entry that crosses the block's end therefore depends on the
 * bytes its io.Reader holds PAST the block:
 *   - enough bytes (SSTable.DecodeFrom's reader is the whole file, the footer
 *     follows the index, sstable.go:122; index_test.go's reader holds the
 *     whole buffer): "unexpected EOF: size limit reached while reading key
 *     length" (index.go:88-91);
 *   - the reader ends inside the key length or the key (a reader cut at the
 *     block): "decode index key length failed" (index.go:73-76);
 *   - the reader ends inside the offset: "decode index offset failed"
 *     (index.go:81-84).
 * The library never reads past blk_len, so it reports this one status for
 * all three, with d_nrec = the entries before the crossing one -- what Go
 * appended in every case (the oracle, oracle/lsm_oracle.c, follows the first
 * reading: bytes past the block present).  A binding that needs Go's message
 * picks it from the bytes its own reader holds past the block. */

enum lsm_error {
    LSM_EINVAL = -1,  /* bad argument                        */
    LSM_ENODEV = -2,  /* no gfx950 device / device not found  */
    LSM_ENOMEM = -3,  /* host allocation failed              */
    LSM_ESPACE = -4,  /* workspace too small                 */
};

/* One decoded record: a zero-copy view into the input buffer.
 *   KV : key  = d_in[rec_off+4 .. +key_len), value = d_in[rec_off+8+key_len .. +val_len)
 *   V  : key_len = 0, value = d_in[rec_off+4 .. +val_len)
 *   IDX: key  = d_in[rec_off+4 .. +key_len), val_len = 8 (the i64 offset follows the key) */
typedef struct lsm_rec_desc {
    uint64_t rec_off;
    uint32_t key_len;
    uint32_t val_len;
} lsm_rec_desc;

/* Outputs of lsm_decode_blocks.  Record i of block b goes to slot
 * base(b) + i of every per-record array, where
 *   rec_base != NULL : base(b) = rec_base[b], capacity rec_base[b+1]-rec_base[b]
 *                      (lsm_plan_rec_base computes a dense-capacity plan);
 *   rec_base == NULL : offset-addressed, base(b) = blk_off[b] / R and capacity
 *                      (blk_off[b]+blk_len[b]) / R - base(b), R = 4 (V), 8 (KV),
 *                      12 (IDX) -- disjoint for non-overlapping blocks, no plan
 *                      needed; per-record arrays need (input bytes / R) + 1 slots. */
typedef struct lsm_decode_out {
    lsm_rec_desc *desc;         /* required                                         */
    const uint64_t *rec_base;   /* optional, nblk+1 entries (see above)             */
    uint32_t *nrec;             /* required, nblk                                   */
    int32_t *status;            /* required, nblk                                   */
    int64_t *idx_value;         /* IDX only, optional: the entry's i64 offset       */
    /* Materialized ("ARENA") mode, all optional.  Keys / values of block b are
     * packed, in record order, from key_arena + A(b) / val_arena + A(b), where
     * A(b) = arena_base[b] (lsm_plan_arena_base: exclusive scan of blk_len) or,
     * with arena_base == NULL, A(b) = blk_off[b] (arenas mirror the input's
     * addressing; a block's keys or values never exceed blk_len bytes). */
    uint8_t *key_arena;
    uint8_t *val_arena;
    const uint64_t *arena_base; /* optional, nblk+1                                 */
    uint64_t *key_arena_off;    /* optional per record: absolute offset in key_arena */
    uint64_t *val_arena_off;    /* optional per record: absolute offset in val_arena */
} lsm_decode_out;

typedef struct lsm_ctx lsm_ctx;

/* ---- context ------------------------------------------------------------ */

int lsm_abi_version(void);
/* LSM_INPUT_SLACK of the loaded library: a binding checks it at load time. */
int lsm_input_slack(void);
/* Identity of the sources the library was compiled from (16 hex digits,
 * go-lsm_amd/build_id.py): a binding shipped beside the sources compares it
 * and refuses a stale prebuilt library.  Not part of the Go surface. */
const char *lsm_build_id(void);
/* "HIPCC|ARCH|HIPFLAGS" the library was compiled with: the build id hashes
 * these with the sources, so a binding recomputes the id from this string. */
const char *lsm_build_flags(void);
/* One context per goroutine / OS thread (callers are concurrent goroutines,
 * sstable_test.go:379-400); no hidden global mutable state. */
int lsm_ctx_create(int device, lsm_ctx **out);
int lsm_ctx_destroy(lsm_ctx *ctx);
/* Number of compute units of the context's device (grid sizing). */
int lsm_ctx_num_cus(const lsm_ctx *ctx);

/* ---- memory / stream plumbing (so a cgo or C++ host needs no HIP headers) -- */

/* Device allocation, rounded up to 16 bytes plus 16 bytes of slack (the
 * readability contract above).  Not for use inside a timed/captured region. */
int lsm_dev_alloc(lsm_ctx *ctx, size_t bytes, void **out);
int lsm_dev_free(lsm_ctx *ctx, void *p);
/* Pinned (page-locked) host memory for asynchronous H2D/D2H staging. */
int lsm_host_alloc_pinned(lsm_ctx *ctx, size_t bytes, void **out);
int lsm_host_free_pinned(lsm_ctx *ctx, void *p);
int lsm_memcpy_h2d(lsm_ctx *ctx, void *d_dst, const void *h_src, size_t bytes, void *stream);
int lsm_memcpy_d2h(lsm_ctx *ctx, void *h_dst, const void *d_src, size_t bytes, void *stream);
int lsm_memset_dev(lsm_ctx *ctx, void *d_dst, int value, size_t bytes, void *stream);
int lsm_stream_create(lsm_ctx *ctx, void **out);
int lsm_stream_destroy(lsm_ctx *ctx, void *stream);
int lsm_stream_sync(lsm_ctx *ctx, void *stream);

/* ---- planning ------------------------------------------------------------ */

/* Largest record count a block of `len` bytes can hold: KV len/8, V len/4,
 * IDX len/12 (every record carries at least its fixed-width fields). */
uint64_t lsm_max_records(int grammar, uint64_t len);
size_t lsm_plan_workspace_bytes(uint32_t nblk);
/* d_rec_base[0..nblk] = exclusive scan of lsm_max_records(grammar, blk_len[b]). */
int lsm_plan_rec_base(lsm_ctx *ctx, int grammar, const uint32_t *d_blk_len, uint32_t nblk,
                      uint64_t *d_rec_base, void *d_workspace, size_t ws_bytes, void *stream);
/* d_arena_base[0..nblk] = exclusive scan of blk_len[b]. */
int lsm_plan_arena_base(lsm_ctx *ctx, const uint32_t *d_blk_len, uint32_t nblk,
                        uint64_t *d_arena_base, void *d_workspace, size_t ws_bytes, void *stream);

/* ---- decode ---------------------------------------------------------------- */

/* Batch decode of independent blocks [blk_off[b], blk_off[b]+blk_len[b]).
 * Replaces, per block:
 *   V   : block.DataBlock.DecodeFrom(r, size)      sstable/block/data.go:49-79
 *   KV  : kv.KeyValuePair.DecodeFrom loop           kv/kv.go:77-115, wal/wal.go:106-118
 *   IDX : block.IndexBlock.DecodeFrom(r, size)     sstable/block/index.go:61-101
 * and, composed by the host layer, SSTable.DecodeDataBlock/GetDataBlockFromFile
 * (sstable/sstable.go:214-246).  One wavefront owns one block: the block is
 * streamed into an LDS ring and the record boundaries are chased there. */
int lsm_decode_blocks(lsm_ctx *ctx, int grammar, const uint8_t *d_in, const uint64_t *d_blk_off,
                      const uint32_t *d_blk_len, uint32_t nblk, const lsm_decode_out *out,
                      void *stream);

/* lsm_decode_blocks with the caller's upper bound on the block lengths: above
 * 32 KiB a larger per-wave LDS ring is used (more bytes in flight per wave).
 * The hint only selects the ring; results are identical for any input, also
 * when a block is longer than the hint. */
int lsm_decode_blocks_hinted(lsm_ctx *ctx, int grammar, const uint8_t *d_in,
                             const uint64_t *d_blk_off, const uint32_t *d_blk_len, uint32_t nblk,
                             uint32_t max_blk_len, const lsm_decode_out *out, void *stream);

/* lsm_decode_blocks for a batch whose block sizes vary: the blocks are
 * launched largest first (a device-side bucketing of d_blk_len by power-of-
 * two size class, part of this call), so the batch does not end on a tail of
 * large blocks each streamed by a single wave.  Outputs are addressed by
 * block id exactly as in lsm_decode_blocks (identical results).  Workspace:
 * lsm_decode_schedule_workspace_bytes(nblk). */
size_t lsm_decode_schedule_workspace_bytes(uint32_t nblk);
int lsm_decode_blocks_scheduled(lsm_ctx *ctx, int grammar, const uint8_t *d_in,
                                const uint64_t *d_blk_off, const uint32_t *d_blk_len,
                                uint32_t nblk, const lsm_decode_out *out, void *d_workspace,
                                size_t ws_bytes, void *stream);

/* Compact the records of a finished lsm_decode_blocks into one dense array:
 * d_dense_base[0..nblk] = exclusive scan of nrec (d_dense_base[nblk] = total)
 * and block b's records land at d_dense[d_dense_base[b] ..] (and IDX values
 * at d_dense_idx, optional).  `out` is the lsm_decode_out the decode used
 * (its rec_base, or offset addressing with d_blk_off).  Workspace:
 * lsm_plan_workspace_bytes(nblk).  This is the hand-off a host consumer
 * copies back (GetKeyValuePairs' record list, sstable.go:248-268). */
int lsm_compact_records(lsm_ctx *ctx, int grammar, const uint64_t *d_blk_off, uint32_t nblk,
                        const lsm_decode_out *out, lsm_rec_desc *d_dense, int64_t *d_dense_idx,
                        uint64_t *d_dense_base, void *d_workspace, size_t ws_bytes, void *stream);

/* ---- WAL replay ------------------------------------------------------------ */

/* wal.Recover (wal/wal.go:95-121) of nwal write-ahead logs, each read whole
 * into device memory (io.ReadAll, :101) at [wal_off[w], wal_off[w]+wal_len[w]):
 * KeyValuePair.DecodeFrom (kv/kv.go:77-115) looped while bytes remain
 * (:107-118).  The records decoded before an error are delivered (Recover has
 * already called back for them, :117) and status[w] names the error, which
 * Recover returns as "failed to read wal <file>: <err>".  Outputs and
 * placement as lsm_decode_blocks with LSM_GRAMMAR_KV, one block per log
 * (descriptors only; no arenas).  A log is decoded by many waves (16 KiB
 * segments, guessed entry points, an exact stitch), so the records are the
 * serial chase's.  max_wal_len >= every wal_len[w] sizes the grid and the
 * workspace (a longer log is chased by one wave); workspace:
 * lsm_wal_replay_workspace_bytes(nwal, max_wal_len). */
size_t lsm_wal_replay_workspace_bytes(uint32_t nwal, uint32_t max_wal_len);
int lsm_wal_replay(lsm_ctx *ctx, const uint8_t *d_wal, const uint64_t *d_wal_off,
                   const uint32_t *d_wal_len, uint32_t nwal, uint32_t max_wal_len,
                   const lsm_decode_out *out, void *d_workspace, size_t ws_bytes, void *stream);

/* ---- whole .sst files ------------------------------------------------------ */

/* Per-file result of lsm_decode_sst.  Offsets are relative to the file image. */
typedef struct lsm_sst_meta {
    uint64_t min_key_off, min_key_len, max_key_off, max_key_len; /* Header      header.go:40-52 */
    uint64_t filter_m, filter_k, filter_nbits;                   /* Filter      bloom.go:453-469 */
    uint64_t filter_words_off; /* first filter word (u64 big-endian, bitset v1.22.0 WriteTo)   */
    int64_t data_off, data_size, idx_off, idx_size;              /* Footer      footer.go:58-70 */
    int32_t stage;   /* enum lsm_sst_stage: the first step that failed, 0 = none               */
    int32_t status;  /* lsm_status of a failing index (stage 4) or data (stage 5) decode       */
    uint32_t nidx;   /* index entries decoded (those before an error are kept, index.go:94)  */
    uint32_t ndata;  /* values decoded (those before an error are kept, data.go:75)          */
} lsm_sst_meta;

enum lsm_sst_stage {
    LSM_SST_OK = 0,
    LSM_SST_HEADER = 1,   /* sstable.go:101-104 "decode Header failed"                       */
    LSM_SST_FILTER = 2,   /* sstable.go:106-109 "decode FilterBlock failed"                  */
    LSM_SST_FOOTER = 3,   /* sstable.go:112-115 "decode Footer failed" (file < 32 bytes)     */
    LSM_SST_INDEX = 4,    /* sstable.go:118-125 seek / "decode IndexBlock failed"            */
    LSM_SST_DATA = 5,     /* sstable.go:214-225 seek / "decode DataBlock failed"             */
    LSM_SST_MISMATCH = 6, /* sstable.go:254-257 "mismatched DataBlock and IndexBlock entries" */
};

size_t lsm_decode_sst_workspace_bytes(uint32_t nfile);

/* Decode nfile whole .sst images [file_off[f], file_off[f] + file_len[f]) of
 * d_img: SSTable.DecodeFrom (sstable.go:87-128: header, filter, footer, the
 * IndexBlock chase), DecodeDataBlock (:214-225: the DataBlock chase over
 * DataHandle, data.go:49-79) and GetKeyValuePairs (:248-268: the positional
 * join) in one call.  Entry i of file f goes to slot base(f) + i of
 * d_idx_desc / d_idx_value (key view + i64 offset) and of d_data_desc (value
 * view); record i is (key of idx entry i, value i) for
 * i < (stage == 0 && nidx && ndata ? nidx : 0).  base(f) = d_rec_base[f]
 * with capacity d_rec_base[f+1] - base(f), or with d_rec_base == NULL,
 * file_off[f] / 4 with capacity (file_off[f] + file_len[f]) / 4 - base(f).
 * The results equal the reference's serial chases; the index and the values
 * are verified in parallel (stride hypothesis, index offsets) and chased
 * exactly from the first entry the verification cannot vouch for.
 * Workspace: lsm_decode_sst_workspace_bytes(nfile). */
int lsm_decode_sst(lsm_ctx *ctx, const uint8_t *d_img, const uint64_t *d_file_off,
                   const uint64_t *d_file_len, uint32_t nfile, const uint64_t *d_rec_base,
                   lsm_sst_meta *d_meta, lsm_rec_desc *d_idx_desc, int64_t *d_idx_value,
                   lsm_rec_desc *d_data_desc, void *d_workspace, size_t ws_bytes, void *stream);

/* Batched SSTable.MayContain (sstable.go:300-305) of nkeys keys (CSR, as in
 * lsm_bloom_probe) against nfile .sst images: the key range check against
 * the header's MinKey / MaxKey in Go string order, then Filter.Test
 * (bloom.go:371-379) on the filter block as stored in the image.  d_meta is
 * lsm_decode_sst's output for the same images; a file whose header or filter
 * did not decode (stage 1 or 2) reports 0.  d_hit[i * nfile + f] = 1 when
 * key i may be in file f.  Deviations on corrupted filters only: m == 0
 * reports 0 (Go divides by zero) and k is capped at 4096 probes.
 * When every file decoded, the files are in key order with disjoint ranges
 * (a level >= 1 set), nfile <= 2048 and nkeys < 2^32, the probes are grouped
 * by their one candidate file and each filter is tested from LDS; otherwise
 * every key is checked against every file.  The workspace holds the grouping (see
 * lsm_may_contain_workspace_bytes); d_hit is written whole either way. */
size_t lsm_may_contain_workspace_bytes(uint32_t nfile, uint64_t nkeys);
int lsm_may_contain(lsm_ctx *ctx, const uint8_t *d_img, const uint64_t *d_file_off,
                    const lsm_sst_meta *d_meta, uint32_t nfile, const uint8_t *d_keys,
                    const uint64_t *d_koff, uint64_t nkeys, uint8_t *d_hit, void *d_workspace,
                    size_t ws_bytes, void *stream);

/* Batched Manager.searchFromLevelWithSparseIndex (sstable/manager.go:178-207)
 * up to searchFromTable's MayContain (:209-212) for a level >= 1: the nfile
 * images are the level's tables in sparse-index order (sorted by MinKey,
 * manager.go:290-303), d_meta their lsm_decode_sst output.  For key i:
 * sort.Search (Go's exact bisection) for the first table whose MinKey > key
 * (bytes.Compare), index-- when > 0 (:186-192), then SSTable.MayContain
 * (sstable.go:300-305) of that one table: d_table[i] = the candidate (-1 when
 * the level is empty), d_may[i] = 1 when the table may hold the key.
 * Deviation (corrupted tables only): a table whose header did not decode
 * searches as the zero Header (MinKey "") and, like one whose filter did not
 * decode, answers 0 -- go-lsm's Manager.Recover (manager.go:226-275) would
 * have failed on such a file and never listed it in the level, so the
 * reference has no answer to restate; filter deviations as lsm_may_contain.  Level 0 (searchFromLevel0, :160-176, every table in
 * order): lsm_may_contain for the may-bits, lsm_level0_get for the Get.
 * Workspace: lsm_level_may_contain_workspace_bytes. */
size_t lsm_level_may_contain_workspace_bytes(uint32_t nfile, uint64_t nkeys);
int lsm_level_may_contain(lsm_ctx *ctx, const uint8_t *d_img, const uint64_t *d_file_off,
                          const lsm_sst_meta *d_meta, uint32_t nfile, const uint8_t *d_keys,
                          const uint64_t *d_koff, uint64_t nkeys, int32_t *d_table,
                          uint8_t *d_may, void *d_workspace, size_t ws_bytes, void *stream);
/* The level's sparse index (ABI 5) -- Manager's sparseIndexes[level-1]
 * (manager.go:183-187): each table's MinKey / MaxKey prefixes and filter shape,
 * parsed from the images once and kept while the level is unchanged, as the
 * Manager keeps its loaded SSTables.  d_index: lsm_level_index_bytes(nfile)
 * bytes; it refers to offsets inside d_img, so the searches pass the same
 * d_img.  lsm_level_may_contain_indexed = lsm_level_may_contain without
 * parsing the headers again (same outputs, same workspace). */
size_t lsm_level_index_bytes(uint32_t nfile);
int lsm_level_index_build(lsm_ctx *ctx, const uint8_t *d_img, const uint64_t *d_file_off,
                          const lsm_sst_meta *d_meta, uint32_t nfile, void *d_index, void *stream);
int lsm_level_may_contain_indexed(lsm_ctx *ctx, const uint8_t *d_img, const void *d_index,
                                  uint32_t nfile, const uint8_t *d_keys, const uint64_t *d_koff,
                                  uint64_t nkeys, int32_t *d_table, uint8_t *d_may,
                                  void *d_workspace, size_t ws_bytes, void *stream);

/* Batched searchFromTable past its MayContain (sstable/manager.go:209-223):
 * for key i with d_may[i] = 1 (lsm_level_may_contain's answer for table
 * d_table[i]), Iterator.Seek over that table's IndexBlock (sstable/block/
 * index.go:157-181: Go's bisection for the first entry whose key >= the
 * target, valid only on an exact match) and Iterator.Value ->
 * GetValueByOffset (sstable.go:271-296: Value.DecodeFrom, kv.go:181-200, at
 * the entry's offset in the file).  The index is lsm_decode_sst's output for
 * the same images (d_meta, d_idx_desc, d_idx_value, with the same
 * d_rec_base or offset placement); file f is d_img[file_off[f] ..
 * + file_len[f]).  d_result[i] is a lsm_get_result; on LSM_GET_FOUND
 * d_value[i] is a view of the value {rec_off = offset in d_img of its u32
 * length prefix, key_len = 0, val_len}; otherwise d_value[i] is zero.  The
 * Seek runs over the nidx entries the decode kept (a table whose index did
 * not decode is one the Manager would not have loaded, manager.go:226-275).
 * d_tree (or NULL) is the level's Seek tree from lsm_level_get_tree_build
 * over the same decoded tables with max_nidx = tree_nidx; tables with more
 * index entries than that walk the index.  The steps are Go's either way, so
 * the answers are the same with and without the tree.  tree_bytes (ABI 7) is
 * the tree buffer's size: below lsm_level_get_tree_bytes(nfile, tree_nidx) (a
 * tree built for fewer tables) the call returns LSM_ESPACE.  A tree built for
 * an earlier state of the level with the same shape cannot be detected: the
 * caller rebuilds it whenever the level's tables change, as it re-decodes
 * them. */
enum lsm_get_result {
    LSM_GET_ABSENT = 0,         /* (nil, nil): not MayContain, or no entry equals the key        */
    LSM_GET_FOUND = 1,          /* the value, d_value[i]                                          */
    LSM_GET_SEEK_FAILED = 2,    /* negative offset: sstable.go:284-287 "seek to offset failed"  */
    LSM_GET_VALUE_LENGTH = 3,   /* < 4 bytes left: kv.go:183-186 "decode value length"          */
    LSM_GET_VALUE_TOO_LONG = 4, /* kv.go:188-190 "invalid value length: %d" (> 1<<30)           */
    LSM_GET_VALUE_SHORT = 5,    /* kv.go:192-196 "decode value"                                  */
};
int lsm_level_get(lsm_ctx *ctx, const uint8_t *d_img, const uint64_t *d_file_off,
                  const uint64_t *d_file_len, const lsm_sst_meta *d_meta, uint32_t nfile,
                  const uint64_t *d_rec_base, const lsm_rec_desc *d_idx_desc,
                  const int64_t *d_idx_value, const uint8_t *d_keys, const uint64_t *d_koff,
                  uint64_t nkeys, const int32_t *d_table, const uint8_t *d_may, int32_t *d_result,
                  lsm_rec_desc *d_value, const void *d_tree, uint32_t tree_nidx, size_t tree_bytes,
                  void *stream);

/* The whole batched Get of one level >= 1 in one call (ABI 7):
 * Manager.searchFromLevelWithSparseIndex (manager.go:178-207) and
 * searchFromTable (:209-223) -- lsm_level_may_contain_indexed's outputs
 * (d_table, d_may) and lsm_level_get's (d_result, d_value) for the same
 * inputs, queued on one stream.  d_index: lsm_level_index_build; the decode
 * outputs and the tree as lsm_level_get.  Workspace:
 * lsm_level_may_contain_workspace_bytes. */
int lsm_level_search_get(lsm_ctx *ctx, const uint8_t *d_img, const void *d_index, uint32_t nfile,
                         const uint64_t *d_file_off, const uint64_t *d_file_len,
                         const lsm_sst_meta *d_meta, const uint64_t *d_rec_base,
                         const lsm_rec_desc *d_idx_desc, const int64_t *d_idx_value,
                         const uint8_t *d_keys, const uint64_t *d_koff, uint64_t nkeys,
                         int32_t *d_table, uint8_t *d_may, int32_t *d_result, lsm_rec_desc *d_value,
                         const void *d_tree, uint32_t tree_nidx, size_t tree_bytes,
                         void *d_workspace, size_t ws_bytes, void *stream);

/* Batched Manager.searchFromLevel0 (sstable/manager.go:160-176) for level 0,
 * whose tables overlap: the nfile images are the level's tables in the
 * Manager's order (newest first -- addNewSSTables prepends, manager.go:
 * 284-287), with lsm_decode_sst's outputs as for lsm_level_get.  Per key i,
 * searchFromTable (:209-223) on table 0, 1, ...: MayContain (sstable.go:
 * 300-305: the range check, then Filter.Test), Iterator.Seek, the value; a
 * false positive or a Seek miss goes on to the next table, the first value or
 * error ends the search (`return nil, err`).  d_table[i] = the table that
 * answered (LSM_GET_FOUND or an error code in d_result[i], the value's view
 * in d_value[i] as lsm_level_get), -1 with LSM_GET_ABSENT when none did.
 * MayContain's deviations are lsm_may_contain's (corrupted filters only).
 * d_tree / tree_nidx / tree_bytes as lsm_level_get (the level-0 tables'
 * Seek tree, or NULL). */
int lsm_level0_get(lsm_ctx *ctx, const uint8_t *d_img, const uint64_t *d_file_off,
                   const uint64_t *d_file_len, const lsm_sst_meta *d_meta, uint32_t nfile,
                   const uint64_t *d_rec_base, const lsm_rec_desc *d_idx_desc,
                   const int64_t *d_idx_value, const uint8_t *d_keys, const uint64_t *d_koff,
                   uint64_t nkeys, int32_t *d_table, int32_t *d_result, lsm_rec_desc *d_value,
                   const void *d_tree, uint32_t tree_nidx, size_t tree_bytes, void *stream);

/* The Seek tree of a level for lsm_level_get, built once when the level is
 * loaded (the Manager keeps each table's decoded IndexBlock in memory,
 * manager.go:226-275; Seek bisects it, index.go:157-181).  Go's bisection
 * over n entries visits a fixed tree of midpoints whatever the keys hold; the
 * tree stores, per table, each midpoint's 16-byte key prefix and length in
 * 128-byte blocks of three levels, so a Seek reads one line per three steps.
 * Tables with nidx <= max_nidx are built; lsm_level_get_tree_bytes(nfile,
 * max_nidx) bytes (about 18 per entry at max_nidx).  Asynchronous. */
size_t lsm_level_get_tree_bytes(uint32_t nfile, uint32_t max_nidx);
int lsm_level_get_tree_build(lsm_ctx *ctx, const uint8_t *d_img, const uint64_t *d_file_off,
                             const lsm_sst_meta *d_meta, uint32_t nfile, const uint64_t *d_rec_base,
                             const lsm_rec_desc *d_idx_desc, uint32_t max_nidx, void *d_tree,
                             size_t tree_bytes, void *stream);

/* ---- encode ---------------------------------------------------------------- */

/* Batch encode of a columnar record batch (CSR: record i's key is
 * d_keys[d_koff[i] .. d_koff[i+1]), value d_vals[d_voff[i] .. d_voff[i+1])).
 * Block b holds records [rec_start[b], rec_start[b+1]) and is written
 * contiguously at d_out + out_off[b]; bytes between blocks are untouched.
 * Replaces KeyValuePair.EncodeTo (kv.go:46-74), DataBlock.EncodeTo
 * (data.go:26-45 / Value.EncodeTo kv.go:165-178) and IndexBlock.Encode
 * (index.go:47-58; d_idx_off[i] is record i's i64 offset, IDX only). */
uint64_t lsm_encoded_size_host(int grammar, const uint64_t *koff, const uint64_t *voff,
                               uint64_t r0, uint64_t r1);
int lsm_encode_blocks(lsm_ctx *ctx, int grammar, const uint8_t *d_keys, const uint64_t *d_koff,
                      const uint8_t *d_vals, const uint64_t *d_voff, const int64_t *d_idx_off,
                      const uint64_t *d_rec_start, uint32_t nblk, uint8_t *d_out,
                      const uint64_t *d_out_off, void *stream);

/* ---- .sst build (builder path + fused bloom) ------------------------------ */

/* Builder flush rule on host-resident CSR offsets: Builder.Add/ShouldFlush
 * (builder.go:34-42, EstimateSize kv.go:118-121) as driven by
 * CompactAndMergeKVs (merge.go:106-123).  threshold 0 = never flush
 * (BuildSSTableFromIMemTable builder.go:22-31); go-lsm uses 2 MiB
 * (sstable.go:21).  Writes file_start[0..nfile] (file_start[nfile] = n);
 * returns nfile.  file_start must hold n+1 entries. */
uint64_t lsm_segment_files_host(const uint64_t *koff, const uint64_t *voff, uint64_t n,
                                uint64_t threshold, uint64_t *file_start);
/* Exact .sst image size of records [r0, r1) (host-resident CSR offsets). */
uint64_t lsm_sst_image_size_host(const uint64_t *koff, const uint64_t *voff, uint64_t r0,
                                 uint64_t r1, uint64_t m);
/* Filter block bytes for m bits: 8 + 24 + 8*ceil(m/64) (bloom.go:472-491). */
uint64_t lsm_filter_block_size(uint64_t m);
/* Device workspace lsm_build_sst needs for nfile files of at most
 * max_file_records records each: when the filter splits into two LDS slices
 * (go-lsm's default m), a 16-byte hash record per key (k <= 16: the key hash
 * runs inside the region writer) or the slice-1 bit positions (k u32 per
 * record); else a token 16 bytes. */
size_t lsm_build_sst_workspace_bytes(uint32_t nfile, uint32_t max_file_records, uint64_t m,
                                     uint32_t k);

/* Build nfile .sst images: file f holds records [file_start[f], file_start[f+1])
 * and its image (Header | Filter | V data | IDX index | Footer) is written at
 * d_out + file_off[f].  Replaces Builder.Add/Build (builder.go:34-59),
 * SSTable.Add (sstable.go:322-326), bloom Filter.Add (bloom.go:175-181,
 * murmur.go:245-275) and SSTable.EncodeTo (sstable.go:131-193).  The bloom
 * (m bits, k hashes; go-lsm default 1,600,000 / 16, bloom.go:79-82) is
 * built in LDS slices and its words are stored straight into each image;
 * for the default shape each key is hashed by the kernel that writes its
 * index entry.
 * d_footer (optional) gets {dataOff, dataSize, idxOff, idxSize} per file.
 * max_file_records must be >= every file_start[f+1]-file_start[f] (it sizes
 * the grid and the workspace).  Requires m >= 1. */
int lsm_build_sst(lsm_ctx *ctx, const uint8_t *d_keys, const uint64_t *d_koff,
                  const uint8_t *d_vals, const uint64_t *d_voff, const uint64_t *d_file_start,
                  uint32_t nfile, uint32_t max_file_records, uint64_t m, uint32_t k,
                  uint8_t *d_out, const uint64_t *d_file_off, int64_t *d_footer,
                  void *d_workspace, size_t ws_bytes, void *stream);

/* lsm_build_sst with the values read in place: value i of the batch is the
 * value of pair d_idx[i], a view into d_bytes (d_val_desc[d_idx[i]], a V
 * descriptor; or, d_val_desc == NULL, the value of KV descriptor
 * d_key_desc[d_idx[i]]); d_voff is the exclusive scan of those value lengths.
 * The keys come packed (d_keys / d_koff).  That is the output of
 * lsm_merge_kvs + lsm_gather_kvs(..., d_vals = NULL, ...): the values are not
 * copied twice.  Same images as lsm_build_sst. */
int lsm_build_sst_views(lsm_ctx *ctx, const uint8_t *d_keys, const uint64_t *d_koff,
                        const uint8_t *d_bytes, const lsm_rec_desc *d_key_desc,
                        const lsm_rec_desc *d_val_desc, const uint32_t *d_idx,
                        const uint64_t *d_voff, const uint64_t *d_file_start, uint32_t nfile,
                        uint32_t max_file_records, uint64_t m, uint32_t k, uint8_t *d_out,
                        const uint64_t *d_file_off, int64_t *d_footer, void *d_workspace,
                        size_t ws_bytes, void *stream);

/* ---- bloom probe (verification side, Filter.Test bloom.go:371-379) ------- */

/* Standalone bloom build: Filter.Add of every key (bloom.go:175-181) into
 * d_words (ceil(m/64) native u64 words, zeroed by the call). */
int lsm_bloom_build(lsm_ctx *ctx, const uint8_t *d_keys, const uint64_t *d_koff, uint64_t nkeys,
                    uint64_t m, uint32_t k, uint64_t *d_words, void *stream);

/* d_hit[i] = Filter.Test(key i) against the filter words of one .sst
 * (native u64 words, bit p -> word p>>6 bit p&63). */
int lsm_bloom_probe(lsm_ctx *ctx, const uint64_t *d_words, uint64_t m, uint32_t k,
                    const uint8_t *d_keys, const uint64_t *d_koff, uint64_t nkeys,
                    uint8_t *d_hit, void *stream);
/* sum256 (murmur.go:245-275) of each key: d_h[4*i .. 4*i+3]. */
int lsm_sum256(lsm_ctx *ctx, const uint8_t *d_keys, const uint64_t *d_koff, uint64_t nkeys,
               uint64_t *d_h, void *stream);

/* ---- compaction merge ------------------------------- */

/* Replaces CompactAndMergeKVs (sstable/merge.go:42-94) up to the builder:
 * the n pairs are views into d_bytes -- key i at d_key_desc[i].rec_off + 4,
 * d_key_desc[i].key_len bytes (an IDX or KV descriptor); value i at
 * d_val_desc[i].rec_off + 4, d_val_desc[i].val_len bytes (a V descriptor) or,
 * with d_val_desc == NULL, right after the key of a KV descriptor
 * (d_key_desc[i].val_len bytes).  That is the output of lsm_decode_sst (f1)
 * or of a KV decode / WAL replay, with no copy.
 *
 * Pairs leave in key order (Go string order, bytewise); equal keys leave in
 * input order -- merge.go:41's contract, "the newest pair comes first and
 * wins".  lsm_merge_kvs_tie with LSM_TIE_GOHEAP reproduces container/heap's
 * own tie order instead (the reference's exact output; a host replay of the
 * heap over device-computed key ranks).  Per
 * pair, as merge.go:57-85: a key equal to the last written non-empty key is
 * skipped; a tombstone (kv.DeletedValue) is dropped when level >= 6
 * (maxSSTableLevel); otherwise it is written; a file is flushed when the
 * EstimateSize sum (16 + key + value bytes, kv.go:118-121) reaches
 * threshold (maxSSTableSize, 2 MiB; must be > 0) and the last written key is
 * forgotten at each flush.
 *
 * Outputs: d_out[0 .. nout) = input indices of the written pairs, in order;
 * d_file_start[0 .. nfiles] = each file's first position in d_out (optional,
 * n + 1 entries), d_file_start[nfiles] = nout; lsm_merge_kvs_tie's h_counts
 * (host, 3 entries) = {nout, nfiles, the most pairs in one file} (the last
 * sizes lsm_build_sst's max_file_records with no second read-back; ABI 4).
 * Synchronizes the stream (the radix passes are chosen from key statistics). */
size_t lsm_merge_kvs_workspace_bytes(uint64_t n);
enum lsm_tie {
    LSM_TIE_INPUT = 0,   /* equal keys in input order (merge.go:41's contract)              */
    LSM_TIE_GOHEAP = 1,  /* equal keys in container/heap's pop order (merge.go:47-66, exact) */
};
/* lsm_merge_kvs = lsm_merge_kvs_tie(..., LSM_TIE_INPUT, ...) with h_counts
 * holding 2 entries, {nout, nfiles} (unchanged since v2).  Same workspace. */
int lsm_merge_kvs_tie(lsm_ctx *ctx, const uint8_t *d_bytes, const lsm_rec_desc *d_key_desc,
                      const lsm_rec_desc *d_val_desc, uint64_t n, int level, uint64_t threshold,
                      int tie, uint32_t *d_out, uint64_t *d_file_start, uint64_t *h_counts,
                      void *d_ws, size_t ws_bytes, void *stream);
/* container/heap's pop order over dense key ranks (host, no device): Push of
 * 0 .. n-1, then Pop until empty, Less = rank <; order[j] = the j-th popped
 * index.  What LSM_TIE_GOHEAP replays.  phase_ns (optional, 2 entries): the
 * nanoseconds of the push and the pop phases (ABI 7).
 * LSM_TIE_GOHEAP skips the replay when every key is distinct (the device's
 * group count equals n): the heap then pops in key order, which the sort
 * already is -- both tie modes give the same output.  lsm_goheap_replays
 * counts the replays a context has run. */
int lsm_goheap_pop_order_host(const uint32_t *rank, uint64_t n, uint32_t *order, uint64_t *phase_ns);
uint64_t lsm_goheap_replays(const lsm_ctx *ctx);
int lsm_merge_kvs(lsm_ctx *ctx, const uint8_t *d_bytes, const lsm_rec_desc *d_key_desc,
                  const lsm_rec_desc *d_val_desc, uint64_t n, int level, uint64_t threshold,
                  uint32_t *d_out, uint64_t *d_file_start, uint64_t *h_counts, void *d_ws,
                  size_t ws_bytes, void *stream);
/* lsm_merge_kvs_tie without its closing read-back (ABI 5): the counts {nout,
 * nfiles, the most pairs in one file} go to d_counts (device, 3 entries) and
 * the call returns with the file walk and the emit still queued.  The
 * key-statistics read-back that picks the radix passes stays (and, for
 * LSM_TIE_GOHEAP, the host replay).  A compaction reads d_counts while its
 * gather (lsm_gather_kvs_dev) runs: the stream does not idle for the read. */
int lsm_merge_kvs_async(lsm_ctx *ctx, const uint8_t *d_bytes, const lsm_rec_desc *d_key_desc,
                        const lsm_rec_desc *d_val_desc, uint64_t n, int level, uint64_t threshold,
                        int tie, uint32_t *d_out, uint64_t *d_file_start, uint64_t *d_counts,
                        void *d_ws, size_t ws_bytes, void *stream);

/* The selected pairs d_idx[0 .. nout) as a CSR record batch -- the input of
 * lsm_build_sst: keys packed into d_keys with d_koff[0 .. nout], values into
 * d_vals with d_voff[0 .. nout] (the arenas must hold the selected bytes; the
 * input's totals always suffice).  d_vals == NULL packs the keys only (d_voff
 * is still written) for lsm_build_sst_views.  Asynchronous. */
size_t lsm_gather_kvs_workspace_bytes(uint64_t nout);
int lsm_gather_kvs(lsm_ctx *ctx, const uint8_t *d_bytes, const lsm_rec_desc *d_key_desc,
                   const lsm_rec_desc *d_val_desc, const uint32_t *d_idx, uint64_t nout,
                   uint8_t *d_keys, uint64_t *d_koff, uint8_t *d_vals, uint64_t *d_voff,
                   void *d_ws, size_t ws_bytes, void *stream);
/* lsm_gather_kvs with the pair count on the device (ABI 5): nout = *d_nout
 * (lsm_merge_kvs_async's d_counts[0]), at most nout_max, which sizes the
 * launches, the workspace (lsm_gather_kvs_workspace_bytes(nout_max)) and
 * d_koff / d_voff (nout_max + 1 entries).  Asynchronous. */
int lsm_gather_kvs_dev(lsm_ctx *ctx, const uint8_t *d_bytes, const lsm_rec_desc *d_key_desc,
                       const lsm_rec_desc *d_val_desc, const uint32_t *d_idx, const uint64_t *d_nout,
                       uint64_t nout_max, uint8_t *d_keys, uint64_t *d_koff, uint8_t *d_vals,
                       uint64_t *d_voff, void *d_ws, size_t ws_bytes, void *stream);

/* lsm_sst_pairs + lsm_merge_kvs_async in one call (ABI 6): the join of the
 * decoded files and CompactAndMergeKVs over it, queued in that order on
 * `stream` (compaction.go:173-193 then :49-95).  n = the join's pair count
 * (d_prefix[nfile], e.g. the sum of the decoded nidx of the files that
 * decoded), known to the caller; outputs, workspace
 * (lsm_merge_kvs_workspace_bytes(n)) and d_counts exactly as the two calls.
 * Waits on the host for the merge's key statistics, as lsm_merge_kvs_async
 * does; the join's own count d_prefix[nfile] comes back with them, and a call
 * whose n differs returns LSM_EINVAL before any pass indexes past the join
 * (the join's outputs and the statistics pass are then the only work done).  (Statistics taken before the join, to overlap their read-back with
 * it, measured slower and are not used: DESIGN.md section 7.) */
int lsm_compact_merge_async(lsm_ctx *ctx, const uint8_t *d_img, const lsm_sst_meta *d_meta,
                            const uint64_t *d_file_off, uint32_t nfile, const lsm_rec_desc *d_idx_desc,
                            const lsm_rec_desc *d_data_desc, uint64_t n, lsm_rec_desc *d_key_out,
                            lsm_rec_desc *d_val_out, uint64_t *d_prefix, int level, uint64_t threshold,
                            int tie, uint32_t *d_out, uint64_t *d_file_start, uint64_t *d_counts,
                            void *d_ws, size_t ws_bytes, void *stream);

/* The positional join of decoded files in file order -- loadLevelData's
 * allPairs (compaction.go:173-193) over GetKeyValuePairs (sstable.go:248-268):
 * d_key_out / d_val_out = the files' index (key) and data (value) descriptors
 * from lsm_decode_sst's outputs (file f's entries at slot d_file_off[f] / 4),
 * densely, file after file; files that failed (stage != 0) or hold no data or
 * no index entries contribute nothing.  d_prefix[0 .. nfile] = each file's
 * first output slot, d_prefix[nfile] = the total.  Asynchronous. */
int lsm_sst_pairs(lsm_ctx *ctx, const lsm_sst_meta *d_meta, const uint64_t *d_file_off,
                  uint32_t nfile, const lsm_rec_desc *d_idx_desc, const lsm_rec_desc *d_data_desc,
                  lsm_rec_desc *d_key_out, lsm_rec_desc *d_val_out, uint64_t *d_prefix,
                  void *stream);

/* ---- the builder path over one sorted stream (ABI 7) ----------------------- */

/* The builder rule on the device: lsm_segment_files_host's file starts for
 * the device CSR offsets d_koff / d_voff (n + 1 entries each) -- Builder.Add /
 * ShouldFlush (builder.go:34-42, EstimateSize kv.go:118-121) as driven by
 * CompactAndMergeKVs (merge.go:106-128); threshold 0 = never flush.  Writes
 * d_file_start[0 .. nfile] (d_file_start[nfile] = n; nfile_max + 1 entries)
 * and d_counts (device, 4 entries) = {nfile, the most records in one file, 0,
 * overflow}.  nfile_max = lsm_stream_max_files(n, key bytes, value bytes,
 * threshold) always suffices; with a smaller bound a stream needing more files
 * gets nfile = 0 and overflow = 1.  One workgroup; asynchronous. */
uint32_t lsm_stream_max_files(uint64_t n, uint64_t key_bytes, uint64_t val_bytes, uint64_t threshold);
int lsm_segment_files(lsm_ctx *ctx, const uint64_t *d_koff, const uint64_t *d_voff, uint64_t n,
                      uint64_t threshold, uint32_t nfile_max, uint64_t *d_file_start,
                      uint64_t *d_counts, void *stream);

/* Builder.Add / ShouldFlush / Build over one sorted record stream, every file
 * flushed at `threshold` (merge.go:106-128's loop; sstable.go:21's 2 MiB in
 * go-lsm), with SSTable.Add / EncodeTo and Filter.Add for every file -- the
 * rule (lsm_segment_files), the layout (lsm_sst_layout's: each image at a
 * multiple of `align` in d_out) and the images (lsm_build_sst's bytes) in one
 * call, with no host round trip for go-lsm's filter shape (two LDS slices,
 * k <= 16): every launch is sized on nfile_max and the counts stay on the
 * device.  Other filter shapes read the counts back (the call synchronizes).
 * Outputs: d_file_start (nfile_max + 1), d_file_off (nfile_max + 1: the last
 * entry used is the total), d_footer (optional, 4 * nfile_max), d_counts (4:
 * {nfile, most records in a file, image bytes, overflow}); d_out must hold
 * lsm_build_sst_stream_out_bytes(...) bytes, the workspace
 * lsm_build_sst_stream_workspace_bytes(...).  Same images, file for file, as
 * lsm_segment_files_host + lsm_build_sst. */
size_t lsm_build_sst_stream_workspace_bytes(uint64_t n, uint64_t threshold, uint32_t nfile_max,
                                            uint64_t m, uint32_t k);
uint64_t lsm_build_sst_stream_out_bytes(uint64_t n, uint64_t key_bytes, uint64_t val_bytes,
                                        uint32_t nfile_max, uint64_t m, uint32_t align);
int lsm_build_sst_stream(lsm_ctx *ctx, const uint8_t *d_keys, const uint64_t *d_koff,
                         const uint8_t *d_vals, const uint64_t *d_voff, uint64_t n,
                         uint64_t threshold, uint32_t nfile_max, uint64_t m, uint32_t k,
                         uint32_t align, uint8_t *d_out, uint64_t *d_file_start,
                         uint64_t *d_file_off, int64_t *d_footer, uint64_t *d_counts,
                         void *d_workspace, size_t ws_bytes, void *stream);

/* .sst image size of each file f = records [d_file_start[f], d_file_start[f+1])
 * of a device CSR batch (as lsm_sst_image_size_host, sstable.go:131-193). */
int lsm_sst_image_sizes(lsm_ctx *ctx, const uint64_t *d_koff, const uint64_t *d_voff,
                        const uint64_t *d_file_start, uint32_t nfile, uint64_t m,
                        uint64_t *d_size, void *stream);

/* The images' layout without a host round trip: d_size[f] as
 * lsm_sst_image_sizes, d_file_off[f] = the sum of the earlier sizes, each
 * rounded up to `align` (> 0), and d_file_off[nfile] = the total (nfile + 1
 * entries) -- lsm_build_sst's d_file_off, ready on the device.  The output
 * buffer can be sized from host-known bounds: the total is at most
 * nfile * (lsm_filter_block_size(m) + 40 + align - 1) + 16 * nrec
 * + 3 * key bytes + value bytes.  Asynchronous. */
int lsm_sst_layout(lsm_ctx *ctx, const uint64_t *d_koff, const uint64_t *d_voff,
                   const uint64_t *d_file_start, uint32_t nfile, uint64_t m, uint32_t align,
                   uint64_t *d_size, uint64_t *d_file_off, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* LSM_GPU_H */
