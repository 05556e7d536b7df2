// golsm.h — C++ host mirror of go-lsm's block-codec surface over the C ABI.
//
// go-lsm is Go and no Go toolchain exists in this image, so the host side
// above include/lsm_gpu.h is C++ mirroring the reference's types and methods
// (names, argument meaning, error text):
//   block.DataBlock   sstable/block/data.go:15-91
//   block.IndexBlock  sstable/block/index.go:12-113
//   block.Header      sstable/block/header.go:12-52
//   block.Footer      sstable/block/footer.go:11-102
//   bloom.Filter      sstable/bloom/bloom.go:74-491
//   sstable.SSTable   sstable/sstable.go:33-326
//   sstable.Builder   sstable/builder.go:9-59
// Every record decode/encode, the bloom build and probe run on the GPU
// (liblsm_gpu.so); only fixed-size framing (header, footer, filter words) is
// parsed on the host.  There is no CPU fallback: without a gfx950 device
// Device() throws.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "lsm_gpu.h"

namespace golsm {

// Go's `error`: an empty message is nil.
class Error {
  public:
    Error() = default;
    explicit Error(std::string m) : msg_(std::move(m)) {}
    explicit operator bool() const { return !msg_.empty(); }
    const std::string &Message() const { return msg_; }
    // fmt.Errorf("prefix: %w", err)
    Error Wrap(const std::string &prefix) const {
        return msg_.empty() ? Error() : Error(prefix + ": " + msg_);
    }

  private:
    std::string msg_;
};

using Bytes = std::vector<uint8_t>;

// io.Reader over an in-memory byte range (bytes.Reader, or a file read whole).
class Reader {
  public:
    Reader(const uint8_t *p, size_t n) : p_(p), n_(n) {}
    explicit Reader(const Bytes &b) : p_(b.data()), n_(b.size()) {}
    size_t Len() const { return n_ - pos_; }
    const uint8_t *Cur() const { return p_ + pos_; }
    void Skip(size_t k) { pos_ += k < Len() ? k : Len(); }
    size_t Pos() const { return pos_; }
    void Seek(size_t pos) { pos_ = pos < n_ ? pos : n_; }
    size_t Size() const { return n_; }
    const uint8_t *Data() const { return p_; }

  private:
    const uint8_t *p_;
    size_t n_;
    size_t pos_ = 0;
};

// io.Writer appending to a byte buffer (bytes.Buffer).
struct Buffer {
    Bytes data;
    void Write(const uint8_t *p, size_t n) { data.insert(data.end(), p, p + n); }
    size_t Len() const { return data.size(); }
};

// One lsm_ctx + HIP stream + grow-only staging buffers.  One per OS thread
// (go-lsm decodes from concurrent goroutines, sstable_test.go:379-400).
class Device {
  public:
    explicit Device(int ordinal = 0);
    ~Device();
    Device(const Device &) = delete;
    Device &operator=(const Device &) = delete;
    static Device &ThisThread();  // device 0, created on first use per thread

    lsm_ctx *ctx() const { return ctx_; }
    void *stream() const { return stream_; }
    void *Dev(int slot, size_t bytes);   // grow-only device buffer
    void *Host(int slot, size_t bytes);  // grow-only pinned host buffer
    void H2D(void *d, const void *h, size_t n);
    void D2H(void *h, const void *d, size_t n);
    void Sync();

  private:
    static constexpr int kSlots = 12;
    lsm_ctx *ctx_ = nullptr;
    void *stream_ = nullptr;
    void *dev_[kSlots] = {};
    size_t dcap_[kSlots] = {};
    void *host_[kSlots] = {};
    size_t hcap_[kSlots] = {};
};

namespace kv {
using Key = std::string;
using Value = Bytes;
extern const std::string kDeletedValue;  // "～DELETED～" kv/kv.go:30

struct KeyValuePair {
    Key key;
    Value value;
    bool IsDeleted() const;        // kv.go:40-43
    uint64_t EstimateSize() const; // kv.go:118-121
};
}  // namespace kv

namespace block {

struct DataBlock {
    std::vector<kv::Value> Entries;
    Error EncodeTo(Buffer &w) const;               // data.go:26-45
    Error DecodeFrom(Reader &r, int64_t size);     // data.go:49-79 (size <= 0: unlimited)
    void Add(kv::Value v) { Entries.push_back(std::move(v)); }
    int Len() const { return (int)Entries.size(); }
};

struct IndexEntry {
    kv::Key Key;
    int64_t Offset;
};

struct IndexBlock {
    std::vector<IndexEntry> Indexes;
    int64_t Encode(Buffer &w, Error *err = nullptr) const;  // index.go:47-58
    Error DecodeFrom(Reader &r, int64_t size);              // index.go:61-101
    void Add(const kv::Key &k, int64_t off) { Indexes.push_back({k, off}); }
    int Len() const { return (int)Indexes.size(); }
    // Iterator.Seek (index.go:157-181): exact-match binary search, -1 if absent
    int Seek(const kv::Key &target) const;
};

struct Header {
    kv::Key MinKey, MaxKey;
    Error EncodeTo(Buffer &w) const;  // header.go:25-37
    Error DecodeFrom(Reader &r);      // header.go:40-52
};

constexpr int kFooterSize = 32;  // footer.go:23
constexpr int kHandleSize = 16;  // footer.go:24

struct Handle {
    int64_t Offset = 0, Size = 0;
    Error EncodeTo(Buffer &w) const;  // footer.go:94-102
    Error DecodeFrom(Reader &r);      // footer.go:73-91
};

struct Footer {
    Handle DataHandle, IndexHandle;
    Error EncodeTo(Buffer &w) const;  // footer.go:43-55
    Error DecodeFrom(Reader &r);      // footer.go:58-70
};

}  // namespace block

namespace bloom {

constexpr uint64_t kDefaultM = 1600000;  // bloom.go:80
constexpr uint64_t kDefaultK = 16;       // bloom.go:81

// Filter over native u64 words (bit p -> word p>>6, bit p&63).  Add() queues
// keys; they are hashed into the words on the GPU (lsm_bloom_build) in one
// batch the next time the words are needed.
class Filter {
  public:
    Filter(uint64_t m, uint64_t k);  // NewBloomFilter bloom.go:95-101 (m, k >= 1)
    static Filter Default() { return Filter(kDefaultM, kDefaultK); }
    Filter &Add(const uint8_t *data, size_t n);  // bloom.go:175-181
    Filter &AddString(const std::string &s) { return Add((const uint8_t *)s.data(), s.size()); }
    bool Test(const uint8_t *data, size_t n);    // bloom.go:371-379 (GPU probe)
    bool TestString(const std::string &s) { return Test((const uint8_t *)s.data(), s.size()); }
    bool MayContain(const kv::Key &k) { return TestString(k); }  // bloom.go:448-450
    Error EncodeTo(Buffer &w);    // bloom.go:472-491
    Error DecodeFrom(Reader &r);  // bloom.go:453-469
    uint64_t Cap() const { return m_; }
    uint64_t K() const { return k_; }
    const std::vector<uint64_t> &Words();
    bool Equal(Filter &g);        // bloom.go:318-321
    bool OnlyPending() const { return !built_; }
    const std::vector<std::string> &Pending() const { return pending_; }

  private:
    void Flush();
    uint64_t m_, k_;
    std::vector<uint64_t> words_;
    std::vector<std::string> pending_;
    bool built_ = false;  // words_ carry bits not derived from pending_
};

}  // namespace bloom

namespace sstable {

constexpr uint64_t kMaxSSTableSize = 2 * 1024 * 1024;  // sstable.go:21

class SSTable {
  public:
    block::Header Header;
    bloom::Filter FilterBlock = bloom::Filter::Default();
    block::IndexBlock IndexBlock;
    block::DataBlock DataBlock;
    block::Footer Footer;

    void Add(const kv::KeyValuePair &p);              // sstable.go:322-326
    Error EncodeImage(Bytes *out);                     // sstable.go:131-193, in memory
    Error EncodeTo(const std::string &path);           // sstable.go:131-193
    Error DecodeImage(const Bytes &img);               // sstable.go:87-128, in memory
    Error DecodeFrom(const std::string &path);         // sstable.go:87-128
    Error DecodeDataBlock(const Bytes &img);           // sstable.go:214-225
    std::vector<kv::KeyValuePair> GetDataBlockFromFile(const std::string &path, Error *err);
    std::vector<kv::KeyValuePair> GetKeyValuePairs(Error *err) const;  // sstable.go:248-268
    kv::Value GetValueByOffset(int64_t offset, Error *err);           // sstable.go:271-296
    bool MayContain(const kv::Key &key);                                // sstable.go:300-305
    const std::string &FilePath() const { return path_; }
    int level = 0;  // sstable.go:46 (set by NewSSTableWithLevel / CompactAndMergeKVs)

  private:
    std::string path_;
    Bytes image_;  // the file bytes once encoded/decoded (GetValueByOffset)
};

class Builder {  // builder.go:9-59
  public:
    void Add(const kv::KeyValuePair &p);
    bool ShouldFlush() const { return size_ >= kMaxSSTableSize; }
    void Finalize();
    SSTable &Build();
    uint64_t Size() const { return size_; }
    void SetSize(uint64_t s) { size_ = s; }
    SSTable &Table() { return table_; }

  private:
    SSTable table_;
    uint64_t size_ = 0;
};

// Batch entry points: the GPU's natural granularity.
// Decode many V-grammar data regions at once (compaction input,
// compaction.go:173-220); errs[i] uses the reference's error text.
std::vector<std::vector<kv::Value>> DecodeDataBlocks(const std::vector<Bytes> &regions,
                                                     std::vector<Error> *errs);
// Whole .sst images -> KV pairs in one launch (lsm_decode_sst): per image
// SSTable.DecodeFrom + DecodeDataBlock + GetKeyValuePairs (sstable.go:87-128,
// 214-268), the batch form of compaction's loadLevelData (compaction.go:
// 173-220).  errs[i] carries the reference's error prefix for the failing
// step ("decode Header failed", ..., "mismatched DataBlock and IndexBlock
// entries").
std::vector<std::vector<kv::KeyValuePair>> DecodeFiles(const std::vector<Bytes> &images,
                                                       std::vector<Error> *errs);
// Builder flush rule + SSTable.EncodeTo for a sorted batch in one launch:
// threshold 0 = one file (memtable flush), kMaxSSTableSize = CompactAndMergeKVs.
std::vector<Bytes> BuildImages(const std::vector<kv::KeyValuePair> &sorted, uint64_t threshold,
                               uint64_t m = bloom::kDefaultM, uint64_t k = bloom::kDefaultK);
// The same for given file boundaries: file f = sorted[starts[f], starts[f+1]).
std::vector<Bytes> BuildImagesAt(const std::vector<kv::KeyValuePair> &sorted,
                                 const std::vector<uint64_t> &starts,
                                 uint64_t m = bloom::kDefaultM, uint64_t k = bloom::kDefaultK);
// CompactAndMergeKVs (merge.go:42-94) over lsm_merge_kvs: pairs in key order,
// a key equal to the last written one skipped, tombstones dropped at level 6,
// a new table at every 2 MiB of EstimateSize, the last written key forgotten
// at each flush.  Pairs with equal keys leave in input order (merge.go:41's
// contract; container/heap's own order is unspecified).  The
// tables are returned as decoded from their built images, level set.
std::vector<SSTable> CompactAndMergeKVs(const std::vector<kv::KeyValuePair> &kvs, int level);

}  // namespace sstable
}  // namespace golsm
