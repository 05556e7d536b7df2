/*
 * lsm_oracle.h — CPU restatement of the go-lsm SSTable block-codec path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity oracle and the
 * "port" CPU baseline.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product (liblsm_gpu.so) never links,
 * loads or falls back to it.
 *
 * Every function restates a Go function of xmh1011/go-lsm (snapshot
 * 2025-08-24, /root/reference); the citation is on each declaration.
 * Nothing here is copied: it is re-derived from the Go semantics, including
 * the error ordering and the "partial entries stay appended" behaviour.
 *
 * Pinning: the wire formats are pinned by the
 * reference's own KATs (index_test.go:13-58 exact bytes, footer_test.go
 * sizes, data_test.go / kv_test.go round trips and error cases); sum256 is
 * pinned against an independent SMHasher MurmurHash3_x64_128
 * (mmh3_smhasher.c), itself pinned by SMHasher's published verification
 * value 0x6384BA69, exactly as murmur_test.go:12-70 pins sum256 against
 * twmb/murmur3.  The filter-block word serialization follows
 * bits-and-blooms/bitset v1.22.0 WriteTo (third-party, absent here):
 * parity unpinned by reference tests beyond round trips.
 */
#ifndef LSM_ORACLE_H
#define LSM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Grammars (SURVEY.md §8 wire formats). */
enum {
    ORA_GRAMMAR_V = 0,   /* ([u32 vlen][value])*          data.go:26-79, kv.go:165-200 */
    ORA_GRAMMAR_KV = 1,  /* ([u32 klen][key][u32 vlen][v])* kv.go:46-115               */
    ORA_GRAMMAR_IDX = 2, /* ([u32 klen][key][i64 off])*    index.go:30-101            */
};

/* Per-block status.  Same numbering as include/lsm_gpu.h (the contract). */
enum {
    ORA_OK = 0,
    ORA_TRUNC_LEN_PREFIX = 1, /* 1-3 bytes where a leading u32 length was due (data.go:65, kv.go:80) */
    ORA_TRUNC_KEY = 2,        /* kv.go:90                                      */
    ORA_KEY_TOO_LONG = 3,     /* klen > 1<<20, kv.go:84                       */
    ORA_TRUNC_VLEN = 4,       /* kv.go:98                                      */
    ORA_VAL_TOO_LONG = 5,     /* vlen > 1<<30, kv.go:102                      */
    ORA_TRUNC_VAL = 6,        /* data.go:71, kv.go:108                        */
    ORA_IDX_OVERRUN = 7,      /* index.go:88-91                               */
    ORA_CAPACITY = 8,         /* output capacity exhausted (contract only)    */
};

typedef struct {
    uint64_t rec_off; /* absolute offset of the record's first length prefix */
    uint32_t key_len; /* 0 for the V grammar                                  */
    uint32_t val_len; /* IDX: 8 (the i64 offset that follows the key)        */
} ora_desc;

/* ---- record decode ---------------------------------------------------- */

/* Decode one block [blk_off, blk_off+blk_len) of `base`.
 *   V   : DataBlock.DecodeFrom(r, size)   sstable/block/data.go:49-79
 *   KV  : wal.Recover loop of KeyValuePair.DecodeFrom  wal/wal.go:106-118, kv/kv.go:77-115
 *   IDX : IndexBlock.DecodeFrom(r, size)  sstable/block/index.go:61-101
 * Records decoded before an error stay in `desc` (data.go:75, index.go:94).
 * idx_val (IDX only, may be NULL) receives each entry's i64 offset. */
int ora_decode_block(int grammar, const uint8_t *base, uint64_t blk_off, uint64_t blk_len,
                     ora_desc *desc, int64_t *idx_val, uint64_t cap, uint32_t *nrec);

/* Materialize decoded records into packed key / value arenas (the bytes
 * Go's make()+ReadFull copies produce, kv.go:88-112, data.go:69-75).
 * Returns the number of key bytes; *val_bytes gets value bytes. */
uint64_t ora_materialize(int grammar, const uint8_t *base, const ora_desc *desc, uint64_t n,
                         uint8_t *key_arena, uint8_t *val_arena, uint64_t *val_bytes);

/* ---- record encode ---------------------------------------------------- */

/* Encoded size of records [r0,r1) of a columnar batch (CSR offsets). */
uint64_t ora_encoded_size(int grammar, const uint64_t *koff, const uint64_t *voff, uint64_t r0,
                          uint64_t r1);

/* KV: KeyValuePair.EncodeTo kv.go:46-74;  V: DataBlock.EncodeTo data.go:26-45 +
 * Value.EncodeTo kv.go:165-178;  IDX: IndexBlock.Encode index.go:47-58 with
 * IndexEntry.Encode index.go:30-44 (idx_off[i - r0] is the entry's offset). */
uint64_t ora_encode_records(int grammar, const uint8_t *keys, const uint64_t *koff,
                            const uint8_t *vals, const uint64_t *voff, uint64_t r0, uint64_t r1,
                            const int64_t *idx_off, uint8_t *out);

/* ---- MurmurHash3 / bloom ---------------------------------------------- */

/* digest128.sum256  sstable/bloom/murmur.go:245-275 (bmix :64-71, bmixWords
 * :74-95, sum128 :104-221, fmix64 :223-230). */
void ora_sum256(const uint8_t *data, uint64_t len, uint64_t h[4]);

/* Independent MurmurHash3_x64_128 (SMHasher reference algorithm). */
void ora_mmh3_x64_128(const void *key, uint64_t len, uint32_t seed, uint64_t out[2]);
/* SMHasher VerificationTest for MurmurHash3_x64_128; published value 0x6384BA69. */
uint32_t ora_mmh3_verification(void);

/* location(h, i) before the modulo, bloom.go:133-136. */
uint64_t ora_location(const uint64_t h[4], uint64_t i);
/* Filter.Add bloom.go:175-181 (bit p -> words[p>>6] bit p&63, bitset.Set). */
void ora_bloom_add(uint64_t *words, uint64_t m, uint64_t k, const uint8_t *key, uint64_t len);
/* Filter.Test bloom.go:371-379. */
int ora_bloom_test(const uint64_t *words, uint64_t m, uint64_t k, const uint8_t *key,
                   uint64_t len);
/* Filter.Test bloom.go:371-379 on a DECODED filter (ReadFrom :262-281 keeps
 * m and k as stored, no max(1, .)): k == 0 -> 1; bitset.Test is false at and
 * past the stored bit count nbits; m == 0 < k -> -1 (Go panics: location()'s
 * `% arraySize` divides by zero). */
int ora_filter_test(const uint64_t *words, uint64_t nbits, uint64_t m, uint64_t k,
                    const uint8_t *key, uint64_t len);
/* EstimateParameters bloom.go:145-149. */
void ora_estimate_parameters(uint64_t n, double p, uint64_t *m, uint64_t *k);

/* Filter.EncodeTo bloom.go:472-491 -> MarshalBinary :303-311 -> WriteTo
 * :239-250 -> bitset.WriteTo (v1.22.0: u64be length, words u64be). */
uint64_t ora_filter_block_size(uint64_t m);
uint64_t ora_filter_encode(const uint64_t *words, uint64_t m, uint64_t k, uint8_t *out);
/* Filter.DecodeFrom bloom.go:453-469 -> ReadFrom :262-281.  Returns 0 on
 * success, <0 on error; *consumed = bytes read. */
int ora_filter_decode(const uint8_t *in, uint64_t n, uint64_t *m, uint64_t *k, uint64_t *nbits,
                      uint64_t *words, uint64_t words_cap, uint64_t *consumed);

/* ---- .sst file ---------------------------------------------------------- */

/* Builder flush rule: Builder.Add + ShouldFlush (builder.go:34-42) as driven
 * by CompactAndMergeKVs merge.go:106-123 (EstimateSize kv.go:118-121).
 * threshold==0 disables flushing (BuildSSTableFromIMemTable builder.go:22-31).
 * Writes file start indices to starts[0..nfiles], starts[nfiles] = n. */
uint64_t ora_segment_files(const uint64_t *koff, const uint64_t *voff, uint64_t n,
                           uint64_t threshold, uint64_t *starts);

uint64_t ora_sst_image_size(const uint64_t *koff, const uint64_t *voff, uint64_t r0, uint64_t r1,
                            uint64_t m);

/* Builder.Add/Build (builder.go:34-59) + SSTable.EncodeTo (sstable.go:131-193):
 * Header | Filter | V data | IDX index | Footer.  footer_out = {dataOff,
 * dataSize, idxOff, idxSize}.  Returns bytes written. */
uint64_t ora_build_sst(const uint8_t *keys, const uint64_t *koff, const uint8_t *vals,
                       const uint64_t *voff, uint64_t r0, uint64_t r1, uint64_t m, uint64_t k,
                       uint8_t *out, int64_t footer_out[4]);

typedef struct {
    uint64_t min_key_off, min_key_len, max_key_off, max_key_len; /* Header   */
    uint64_t filter_m, filter_k, filter_nbits, filter_words_off; /* Filter   */
    int64_t data_off, data_size, idx_off, idx_size;              /* Footer   */
    int32_t stage;   /* 0 ok, 1 header, 2 filter, 3 footer, 4 index, 5 data, 6 join mismatch */
    int32_t status;  /* block status of the failing stage (index/data)       */
    uint32_t nidx, ndata;
} ora_sst_meta;

/* SSTable.DecodeFrom (sstable.go:87-128) + DecodeDataBlock (:214-225) +
 * GetKeyValuePairs (:248-268) over an in-memory file image. */
int ora_sst_decode(const uint8_t *file, uint64_t n, ora_sst_meta *meta, ora_desc *idx_desc,
                   int64_t *idx_val, uint64_t idx_cap, ora_desc *data_desc, uint64_t data_cap);

/* Batched SSTable.MayContain (sstable.go:300-305) of keys [k0, k1) against
 * nfile decoded images: hit[(i - k0) * nfile + f].  Each (key, file) test
 * hashes the key again, as Filter.Test does per file. */
void ora_may_contain_batch(const uint8_t *img, const uint64_t *file_off, const ora_sst_meta *meta,
                           uint32_t nfile, const uint8_t *keys, const uint64_t *koff, uint64_t k0,
                           uint64_t k1, uint8_t *hit);

/* Manager.searchFromLevelWithSparseIndex (sstable/manager.go:178-207) up to
 * searchFromTable's MayContain (:209-212), keys [k0, k1) against one level's
 * tables in sparse-index order (sorted by MinKey, manager.go:290-303):
 * Go's sort.Search for the first table whose MinKey > key, index-- when > 0,
 * then SSTable.MayContain of that table.  table[i - k0] = the candidate (-1 for
 * an empty level), may[i - k0] = its MayContain.  A table whose header did not
 * decode searches as the zero Header (MinKey "") and answers 0 -- the ABI's
 * stated deviation: Manager.Recover (manager.go:226-275) would not have
 * listed such a file in the level at all. */
void ora_level_may_contain(const uint8_t *img, const uint64_t *file_off, const ora_sst_meta *meta,
                           uint32_t nfile, const uint8_t *keys, const uint64_t *koff, uint64_t k0,
                           uint64_t k1, int32_t *table, uint8_t *may);

/* searchFromTable past its MayContain (sstable/manager.go:209-223) for keys
 * [k0, k1) with may[i - k0] = 1 in table t = table[i - k0]: Iterator.Seek
 * (sstable/block/index.go:157-181: the first entry whose key >= the target by
 * Go's bisection, valid only on an exact match) over t's decoded index (the
 * ora_sst_decode rows idx_base[t] .. + meta[t].nidx of idx_desc / idx_val,
 * rec_off relative to the file), then GetValueByOffset (sstable.go:271-296):
 * Value.DecodeFrom (kv.go:181-200) at the entry's offset in the file of
 * file_len[t] bytes at img + file_off[t].  res: ORA_GET_*; on ORA_GET_FOUND
 * val_off = offset in img of the value's length prefix, val_len its length. */
enum {
    ORA_GET_ABSENT = 0, ORA_GET_FOUND = 1, ORA_GET_SEEK_FAILED = 2, ORA_GET_VALUE_LENGTH = 3,
    ORA_GET_VALUE_TOO_LONG = 4, ORA_GET_VALUE_SHORT = 5,
};
void ora_level_get(const uint8_t *img, const uint64_t *file_off, const uint64_t *file_len,
                   const ora_sst_meta *meta, const ora_desc *idx_desc, const int64_t *idx_val,
                   const uint64_t *idx_base, const uint8_t *keys, const uint64_t *koff, uint64_t k0,
                   uint64_t k1, const int32_t *table, const uint8_t *may, int32_t *res,
                   uint64_t *val_off, uint32_t *val_len);
/* Manager.searchFromLevel0 (manager.go:160-176): every table in order,
 * searchFromTable on each, the first non-nil value or error wins; table[o] =
 * the answering table or -1. */
void ora_level0_get(const uint8_t *img, const uint64_t *file_off, const uint64_t *file_len,
                    const ora_sst_meta *meta, uint32_t nfile, const ora_desc *idx_desc,
                    const int64_t *idx_val, const uint64_t *idx_base, const uint8_t *keys,
                    const uint64_t *koff, uint64_t k0, uint64_t k1, int32_t *table, int32_t *res,
                    uint64_t *val_off, uint32_t *val_len);

/* ---- compaction merge ----------------------------- */

enum { ORA_TIE_INPUT = 0, ORA_TIE_GOHEAP = 1 };

/* CompactAndMergeKVs (sstable/merge.go:42-94) over n pairs held as views into
 * `bytes`: key i = bytes[koff[i], +klen[i]), value i = bytes[voff[i], +vlen[i]).
 * Pairs are popped in key order (Go string order = bytewise); equal keys
 * leave in input order (tie = ORA_TIE_INPUT, merge.go:41's stated contract)
 * or in container/heap's own order (ORA_TIE_GOHEAP: Push = append + up,
 * Pop = Swap(0, n-1) + down, Less = key <).  The loop is the reference's:
 * skip a key equal to the last written one (non-empty), drop tombstones when
 * level >= maxSSTableLevel (6), flush at size >= threshold (EstimateSize sums,
 * builder.go:34-42), and forget the last written key at each flush.
 * Writes the written pairs' input indices to out[] (returned count) and the
 * files' first positions in out[] to starts[0..*nfiles]; starts[*nfiles] = count. */
uint64_t ora_merge_kvs(const uint8_t *bytes, const uint64_t *koff, const uint32_t *klen,
                       const uint64_t *voff, const uint32_t *vlen, uint64_t n, int level,
                       uint64_t threshold, int tie, uint32_t *out, uint64_t *starts,
                       uint64_t *nfiles);

/* ---- CPU baseline (Go allocation pattern) ------------------------------ */

/* config 1 from a file with the reference's read(2)-per-field pattern -> pairs, < 0 on error */
int64_t ora_sst_decode_file(const char *path);

/* Decode blocks the way the Go path does: a fresh heap buffer per key and
 * per value, append-grown record slices; `threads` pthreads over a static
 * block partition.  Returns total records decoded. */
uint64_t ora_bench_decode_golike(int grammar, const uint8_t *base, const uint64_t *blk_off,
                                 const uint32_t *blk_len, uint64_t nblk, int threads);

#ifdef __cplusplus
}
#endif
#endif
