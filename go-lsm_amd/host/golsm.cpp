// golsm.cpp — C++ host mirror of go-lsm's block codec over include/lsm_gpu.h.
// See golsm.h.  Record decode/encode, bloom build and probe are GPU launches;
// the host only packs buffers, parses fixed framing and formats errors with
// the reference's text.
#include "golsm.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <iterator>
#include <memory>
#include <stdexcept>

namespace golsm {

namespace {

uint32_t ld32(const uint8_t *p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}
uint64_t ld64(const uint8_t *p) { return (uint64_t)ld32(p) | (uint64_t)ld32(p + 4) << 32; }
uint64_t ld64be(const uint8_t *p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v = v << 8 | p[i];
    return v;
}
void put32(Buffer &w, uint32_t v) {
    uint8_t b[4] = {(uint8_t)v, (uint8_t)(v >> 8), (uint8_t)(v >> 16), (uint8_t)(v >> 24)};
    w.Write(b, 4);
}
void put64(Buffer &w, uint64_t v) {
    put32(w, (uint32_t)v);
    put32(w, (uint32_t)(v >> 32));
}
void put64be(Buffer &w, uint64_t v) {
    uint8_t b[8];
    for (int i = 0; i < 8; i++) b[i] = (uint8_t)(v >> (8 * (7 - i)));
    w.Write(b, 8);
}

void check(int rc, const char *what) {
    if (rc != 0) throw std::runtime_error(std::string(what) + " failed with code " + std::to_string(rc));
}

const char *eof_or_unexpected(size_t got) { return got == 0 ? "EOF" : "unexpected EOF"; }

size_t pad16(size_t n) { return ((n + 15) & ~(size_t)15) + LSM_INPUT_SLACK; }

// One-launch batch decode of host blocks; descriptors come back per block.
struct Decoded {
    std::vector<int32_t> status;
    std::vector<uint32_t> nrec;
    std::vector<std::vector<lsm_rec_desc>> desc;  // rec_off relative to the block
    std::vector<std::vector<int64_t>> idx;        // IDX offsets
};

Decoded gpu_decode(int grammar, const std::vector<std::pair<const uint8_t *, size_t>> &blocks) {
    Device &d = Device::ThisThread();
    const size_t nb = blocks.size();
    Decoded out;
    out.status.assign(nb, 0);
    out.nrec.assign(nb, 0);
    out.desc.resize(nb);
    out.idx.resize(nb);
    if (nb == 0) return out;
    std::vector<uint64_t> off(nb);
    std::vector<uint32_t> len(nb);
    size_t total = 0;
    for (size_t i = 0; i < nb; i++) {
        off[i] = total;
        len[i] = (uint32_t)blocks[i].second;
        total += (blocks[i].second + 15) & ~(size_t)15;
    }
    uint8_t *h_in = (uint8_t *)d.Host(0, pad16(total));
    std::memset(h_in, 0, pad16(total));
    for (size_t i = 0; i < nb; i++) std::memcpy(h_in + off[i], blocks[i].first, blocks[i].second);
    void *d_in = d.Dev(0, pad16(total));
    void *d_off = d.Dev(1, nb * 8);
    void *d_len = d.Dev(2, nb * 4);
    void *d_nrec = d.Dev(3, nb * 4);
    void *d_st = d.Dev(4, nb * 4);
    const uint64_t R = grammar == LSM_GRAMMAR_V ? 4 : grammar == LSM_GRAMMAR_KV ? 8 : 12;
    const size_t cap = total / R + 1;
    void *d_desc = d.Dev(5, cap * sizeof(lsm_rec_desc));
    void *d_idx = grammar == LSM_GRAMMAR_IDX ? d.Dev(6, cap * 8) : nullptr;
    d.H2D(d_in, h_in, pad16(total));
    d.H2D(d_off, off.data(), nb * 8);
    d.H2D(d_len, len.data(), nb * 4);
    lsm_decode_out o{};
    o.desc = (lsm_rec_desc *)d_desc;
    o.nrec = (uint32_t *)d_nrec;
    o.status = (int32_t *)d_st;
    o.idx_value = (int64_t *)d_idx;
    check(lsm_decode_blocks(d.ctx(), grammar, (const uint8_t *)d_in, (const uint64_t *)d_off,
                            (const uint32_t *)d_len, (uint32_t)nb, &o, d.stream()),
          "lsm_decode_blocks");
    d.D2H(out.nrec.data(), d_nrec, nb * 4);
    d.D2H(out.status.data(), d_st, nb * 4);
    d.Sync();
    for (size_t i = 0; i < nb; i++) {
        const size_t base = off[i] / R, k = out.nrec[i];
        out.desc[i].resize(k);
        if (k) d.D2H(out.desc[i].data(), (lsm_rec_desc *)d_desc + base, k * sizeof(lsm_rec_desc));
        if (d_idx) {
            out.idx[i].resize(k);
            if (k) d.D2H(out.idx[i].data(), (int64_t *)d_idx + base, k * 8);
        }
    }
    d.Sync();
    for (size_t i = 0; i < nb; i++)
        for (auto &x : out.desc[i]) x.rec_off -= off[i];
    return out;
}

// One-launch encode of a CSR batch as one block.
Bytes gpu_encode(int grammar, const Bytes &keys, const std::vector<uint64_t> &koff,
                 const Bytes &vals, const std::vector<uint64_t> &voff,
                 const std::vector<int64_t> &idx_off) {
    Device &d = Device::ThisThread();
    const uint64_t n = (grammar == LSM_GRAMMAR_V ? voff.size() : koff.size()) - 1;
    const uint64_t size = lsm_encoded_size_host(grammar, koff.data(), voff.data(), 0, n);
    Bytes out(size);
    if (n == 0) return out;
    void *d_keys = d.Dev(0, pad16(keys.size()));
    void *d_koff = d.Dev(1, koff.size() * 8);
    void *d_vals = d.Dev(2, pad16(vals.size()));
    void *d_voff = d.Dev(3, voff.size() * 8);
    void *d_io = d.Dev(4, (idx_off.size() + 1) * 8);
    void *d_rs = d.Dev(5, 16);
    void *d_oo = d.Dev(6, 8);
    void *d_out = d.Dev(7, pad16(size));
    if (!keys.empty()) d.H2D(d_keys, keys.data(), keys.size());
    d.H2D(d_koff, koff.data(), koff.size() * 8);
    if (!vals.empty()) d.H2D(d_vals, vals.data(), vals.size());
    d.H2D(d_voff, voff.data(), voff.size() * 8);
    if (!idx_off.empty()) d.H2D(d_io, idx_off.data(), idx_off.size() * 8);
    const uint64_t rs[2] = {0, n}, oo = 0;
    d.H2D(d_rs, rs, 16);
    d.H2D(d_oo, &oo, 8);
    check(lsm_encode_blocks(d.ctx(), grammar, (const uint8_t *)d_keys, (const uint64_t *)d_koff,
                            (const uint8_t *)d_vals, (const uint64_t *)d_voff,
                            grammar == LSM_GRAMMAR_IDX ? (const int64_t *)d_io : nullptr,
                            (const uint64_t *)d_rs, 1, (uint8_t *)d_out, (const uint64_t *)d_oo,
                            d.stream()),
          "lsm_encode_blocks");
    d.D2H(out.data(), d_out, size);
    d.Sync();
    return out;
}

template <class T, class F>
void csr(const std::vector<T> &items, F get, Bytes *data, std::vector<uint64_t> *off) {
    off->assign(items.size() + 1, 0);
    size_t tot = 0;
    for (size_t i = 0; i < items.size(); i++) {
        tot += get(items[i]).size();
        (*off)[i + 1] = tot;
    }
    data->resize(tot);
    size_t p = 0;
    for (auto &it : items) {
        const auto &v = get(it);
        if (!v.empty()) std::memcpy(data->data() + p, v.data(), v.size());
        p += v.size();
    }
}

}  // namespace

// ---- Device -----------------------------------------------------------------

Device::Device(int ordinal) {
    check(lsm_ctx_create(ordinal, &ctx_), "lsm_ctx_create (a gfx950 GPU is required)");
    check(lsm_stream_create(ctx_, &stream_), "lsm_stream_create");
}

Device::~Device() {
    for (int i = 0; i < kSlots; i++) {
        if (dev_[i]) lsm_dev_free(ctx_, dev_[i]);
        if (host_[i]) lsm_host_free_pinned(ctx_, host_[i]);
    }
    if (stream_) lsm_stream_destroy(ctx_, stream_);
    if (ctx_) lsm_ctx_destroy(ctx_);
}

Device &Device::ThisThread() {
    thread_local std::unique_ptr<Device> d;
    if (!d) d.reset(new Device(0));
    return *d;
}

void *Device::Dev(int slot, size_t bytes) {
    if (bytes > dcap_[slot]) {
        if (dev_[slot]) check(lsm_dev_free(ctx_, dev_[slot]), "lsm_dev_free");
        dev_[slot] = nullptr;
        size_t c = bytes < 4096 ? 4096 : bytes + bytes / 4;
        check(lsm_dev_alloc(ctx_, c, &dev_[slot]), "lsm_dev_alloc");
        dcap_[slot] = c;
    }
    return dev_[slot];
}

void *Device::Host(int slot, size_t bytes) {
    if (bytes > hcap_[slot]) {
        if (host_[slot]) check(lsm_host_free_pinned(ctx_, host_[slot]), "lsm_host_free_pinned");
        host_[slot] = nullptr;
        size_t c = bytes < 4096 ? 4096 : bytes + bytes / 4;
        check(lsm_host_alloc_pinned(ctx_, c, &host_[slot]), "lsm_host_alloc_pinned");
        hcap_[slot] = c;
    }
    return host_[slot];
}

void Device::H2D(void *dd, const void *h, size_t n) {
    check(lsm_memcpy_h2d(ctx_, dd, h, n, stream_), "lsm_memcpy_h2d");
}
void Device::D2H(void *h, const void *dd, size_t n) {
    check(lsm_memcpy_d2h(ctx_, h, dd, n, stream_), "lsm_memcpy_d2h");
}
void Device::Sync() { check(lsm_stream_sync(ctx_, stream_), "lsm_stream_sync"); }

// ---- kv -----------------------------------------------------------------------

namespace kv {
const std::string kDeletedValue = "\xef\xbd\x9e" "DELETED" "\xef\xbd\x9e";

bool KeyValuePair::IsDeleted() const {
    return value.size() == kDeletedValue.size() &&
           std::memcmp(value.data(), kDeletedValue.data(), value.size()) == 0;
}
uint64_t KeyValuePair::EstimateSize() const { return 4 + key.size() + 4 + value.size() + 8; }
}  // namespace kv

// ---- block ----------------------------------------------------------------------

namespace block {

Error DataBlock::EncodeTo(Buffer &w) const {
    Bytes vals;
    std::vector<uint64_t> voff;
    csr(Entries, [](const kv::Value &v) -> const kv::Value & { return v; }, &vals, &voff);
    std::vector<uint64_t> koff(voff.size(), 0);
    Bytes enc = gpu_encode(LSM_GRAMMAR_V, Bytes(), koff, vals, voff, {});
    w.Write(enc.data(), enc.size());
    return Error();
}

Error DataBlock::DecodeFrom(Reader &r, int64_t size) {
    // size > 0: io.LimitReader(r, size); otherwise read to EOF (data.go:51-54)
    const size_t n = size > 0 ? std::min((size_t)size, r.Len()) : r.Len();
    const uint8_t *p = r.Cur();
    Decoded dec = gpu_decode(LSM_GRAMMAR_V, {{p, n}});
    size_t end = 0;
    for (auto &ds : dec.desc[0]) {
        Entries.emplace_back(p + ds.rec_off + 4, p + ds.rec_off + 4 + ds.val_len);
        end = ds.rec_off + 4 + ds.val_len;
    }
    r.Skip(n);  // ReadFull/binary.Read drain the limited reader up to the failure
    switch (dec.status[0]) {
    case LSM_OK: return Error();
    case LSM_ST_TRUNC_LEN_PREFIX:
        return Error("read value length failed: unexpected EOF");
    case LSM_ST_TRUNC_VAL:
        return Error(std::string("read value data failed: ") + eof_or_unexpected(n - end - 4));
    default: return Error("decode status " + std::to_string(dec.status[0]));
    }
}

int64_t IndexBlock::Encode(Buffer &w, Error *err) const {
    Bytes keys;
    std::vector<uint64_t> koff;
    csr(Indexes, [](const IndexEntry &e) -> const std::string & { return e.Key; }, &keys, &koff);
    std::vector<int64_t> io;
    for (auto &e : Indexes) io.push_back(e.Offset);
    std::vector<uint64_t> voff(koff.size(), 0);
    Bytes enc = gpu_encode(LSM_GRAMMAR_IDX, keys, koff, Bytes(), voff, io);
    w.Write(enc.data(), enc.size());
    if (err) *err = Error();
    return (int64_t)enc.size();
}

Error IndexBlock::DecodeFrom(Reader &r, int64_t size) {
    Indexes.clear();  // index.go:63
    if (size < 0)
        return Error("invalid size: " + std::to_string(size) + ", must be non-negative");
    // Entries lie inside the size limit; the underlying stream may be shorter.
    const size_t avail = r.Len();
    const size_t n = std::min((size_t)size, avail);
    const uint8_t *p = r.Cur();
    Decoded dec = gpu_decode(LSM_GRAMMAR_IDX, {{p, n}});
    size_t pos = 0;
    for (size_t i = 0; i < dec.desc[0].size(); i++) {
        const auto &ds = dec.desc[0][i];
        Indexes.push_back({kv::Key((const char *)p + ds.rec_off + 4, ds.key_len), dec.idx[0][i]});
        pos = ds.rec_off + 12 + ds.key_len;
    }
    // A limit past the end of the stream can never be reached: the loop keeps
    // reading until a read hits EOF, even when the entries tile the stream.
    if (dec.status[0] == LSM_OK && (size_t)size <= avail) {
        r.Skip(pos);
        return Error();
    }
    // Reproduce the reference's message for the failing entry (index.go:70-91):
    // it reads past the limit from the stream, which may or may not hold the bytes.
    const size_t rem = avail - pos;
    r.Skip(avail);
    if (rem < 4)
        return Error(std::string("decode index key length failed: decode key keyLen: ") +
                     eof_or_unexpected(rem));
    const uint32_t kl = ld32(p + pos);
    if (rem - 4 < kl)
        return Error(std::string("decode index key length failed: decode key bytes: ") +
                     eof_or_unexpected(rem - 4));
    if (rem - 4 - kl < 8)
        return Error(std::string("decode index offset failed: ") + eof_or_unexpected(rem - 4 - kl));
    return Error("unexpected EOF: size limit reached while reading key length");
}

int IndexBlock::Seek(const kv::Key &target) const {
    auto it = std::lower_bound(Indexes.begin(), Indexes.end(), target,
                               [](const IndexEntry &e, const kv::Key &t) { return e.Key < t; });
    if (it == Indexes.end() || it->Key != target) return -1;
    return (int)(it - Indexes.begin());
}

static Error decode_key(Reader &r, kv::Key *k) {  // kv.Key.DecodeFrom kv.go:124-139
    if (r.Len() < 4) {
        Error e(std::string("decode key keyLen: ") + eof_or_unexpected(r.Len()));
        r.Skip(r.Len());
        return e;
    }
    const uint32_t kl = ld32(r.Cur());
    r.Skip(4);
    if (r.Len() < kl) {
        Error e(std::string("decode key bytes: ") + eof_or_unexpected(r.Len()));
        r.Skip(r.Len());
        return e;
    }
    k->assign((const char *)r.Cur(), kl);
    r.Skip(kl);
    return Error();
}

Error Header::EncodeTo(Buffer &w) const {
    put32(w, (uint32_t)MinKey.size());
    w.Write((const uint8_t *)MinKey.data(), MinKey.size());
    put32(w, (uint32_t)MaxKey.size());
    w.Write((const uint8_t *)MaxKey.data(), MaxKey.size());
    return Error();
}

Error Header::DecodeFrom(Reader &r) {
    Error e = decode_key(r, &MinKey);
    if (e) return e.Wrap("decode min key");
    return decode_key(r, &MaxKey);  // header.go:46-49 returns it unwrapped
}

Error Handle::EncodeTo(Buffer &w) const {
    put64(w, (uint64_t)Offset);
    put64(w, (uint64_t)Size);
    return Error();
}

Error Handle::DecodeFrom(Reader &r) {
    if (r.Len() < (size_t)kHandleSize) {
        Error e(std::string("decode footer failed: ") + eof_or_unexpected(r.Len()));
        r.Skip(r.Len());
        return e;
    }
    Offset = (int64_t)ld64(r.Cur());
    Size = (int64_t)ld64(r.Cur() + 8);
    r.Skip(kHandleSize);
    return Error();
}

Error Footer::EncodeTo(Buffer &w) const {
    DataHandle.EncodeTo(w);
    IndexHandle.EncodeTo(w);
    return Error();
}

Error Footer::DecodeFrom(Reader &r) {
    Error e = DataHandle.DecodeFrom(r);
    if (e) return e.Wrap("decode data handle failed");
    e = IndexHandle.DecodeFrom(r);
    if (e) return e.Wrap("decode index handle failed");
    return Error();
}

}  // namespace block

// ---- bloom ----------------------------------------------------------------------

namespace bloom {

Filter::Filter(uint64_t m, uint64_t k)
    : m_(m ? m : 1), k_(k ? k : 1), words_((m_ + 63) / 64, 0) {}

Filter &Filter::Add(const uint8_t *data, size_t n) {
    pending_.emplace_back((const char *)data, n);
    return *this;
}

void Filter::Flush() {
    if (pending_.empty()) return;
    Device &d = Device::ThisThread();
    Bytes keys;
    std::vector<uint64_t> koff;
    csr(pending_, [](const std::string &s) -> const std::string & { return s; }, &keys, &koff);
    const size_t nw = words_.size();
    void *d_keys = d.Dev(0, pad16(keys.size()));
    void *d_koff = d.Dev(1, koff.size() * 8);
    void *d_words = d.Dev(2, nw * 8);
    if (!keys.empty()) d.H2D(d_keys, keys.data(), keys.size());
    d.H2D(d_koff, koff.data(), koff.size() * 8);
    check(lsm_bloom_build(d.ctx(), (const uint8_t *)d_keys, (const uint64_t *)d_koff,
                          pending_.size(), m_, (uint32_t)k_, (uint64_t *)d_words, d.stream()),
          "lsm_bloom_build");
    std::vector<uint64_t> fresh(nw);
    d.D2H(fresh.data(), d_words, nw * 8);
    d.Sync();
    for (size_t i = 0; i < nw; i++) words_[i] |= fresh[i];  // Merge = bitset union
    pending_.clear();
    built_ = true;
}

const std::vector<uint64_t> &Filter::Words() {
    Flush();
    return words_;
}

bool Filter::Test(const uint8_t *data, size_t n) {
    Flush();
    Device &d = Device::ThisThread();
    const size_t nw = words_.size();
    void *d_words = d.Dev(2, nw * 8);
    void *d_key = d.Dev(3, pad16(n));
    void *d_koff = d.Dev(4, 16);
    void *d_hit = d.Dev(5, 16);
    d.H2D(d_words, words_.data(), nw * 8);
    if (n) d.H2D(d_key, data, n);
    const uint64_t ko[2] = {0, n};
    d.H2D(d_koff, ko, 16);
    check(lsm_bloom_probe(d.ctx(), (const uint64_t *)d_words, m_, (uint32_t)k_,
                          (const uint8_t *)d_key, (const uint64_t *)d_koff, 1, (uint8_t *)d_hit,
                          d.stream()),
          "lsm_bloom_probe");
    uint8_t hit = 0;
    d.D2H(&hit, d_hit, 1);
    d.Sync();
    return hit != 0;
}

Error Filter::EncodeTo(Buffer &w) {
    Flush();
    const uint64_t nw = words_.size();
    put64(w, 24 + 8 * nw);  // length prefix, bloom.go:478
    put64be(w, m_);         // WriteTo: arraySize, hashNum, bitset length, words
    put64be(w, k_);
    put64be(w, m_);
    for (uint64_t x : words_) put64be(w, x);
    return Error();
}

Error Filter::DecodeFrom(Reader &r) {
    if (r.Len() < 8) {
        Error e(std::string("decode filter length: ") + eof_or_unexpected(r.Len()));
        r.Skip(r.Len());
        return e;
    }
    const uint64_t L = ld64(r.Cur());
    r.Skip(8);
    if (r.Len() < L) {
        Error e(std::string("decode filter data: ") + eof_or_unexpected(r.Len()));
        r.Skip(r.Len());
        return e;
    }
    const uint8_t *p = r.Cur();
    r.Skip(L);
    if (L < 24) return Error("unexpected EOF");
    const uint64_t m = ld64be(p), k = ld64be(p + 8), nbits = ld64be(p + 16);
    const uint64_t nw = nbits / 64 + ((nbits & 63) != 0);  // no (nbits + 63) overflow
    if (nw > (L - 24) / 8) return Error("unexpected EOF");
    m_ = m;
    k_ = k;
    words_.assign(nw, 0);
    for (uint64_t i = 0; i < nw; i++) words_[i] = ld64be(p + 24 + 8 * i);
    pending_.clear();
    built_ = true;
    return Error();
}

bool Filter::Equal(Filter &g) { return m_ == g.m_ && k_ == g.k_ && Words() == g.Words(); }

}  // namespace bloom

// ---- sstable ----------------------------------------------------------------------

namespace sstable {

void SSTable::Add(const kv::KeyValuePair &p) {
    DataBlock.Add(p.value);
    IndexBlock.Add(p.key, 0);
    FilterBlock.AddString(p.key);
}

Error SSTable::EncodeImage(Bytes *out) {
    const size_t n = DataBlock.Entries.size();
    if (IndexBlock.Indexes.size() < n) return Error("index block shorter than data block");
    bool fused = FilterBlock.OnlyPending() && IndexBlock.Indexes.size() == n &&
                 FilterBlock.Pending().size() == n;
    for (size_t i = 0; fused && i < n; i++) fused = FilterBlock.Pending()[i] == IndexBlock.Indexes[i].Key;
    if (fused) {
        if (n) fused = Header.MinKey == IndexBlock.Indexes[0].Key && Header.MaxKey == IndexBlock.Indexes[n - 1].Key;
        else fused = Header.MinKey.empty() && Header.MaxKey.empty();
    }
    if (fused) {
        // Builder path: one lsm_build_sst launch (bloom fused, sstable.go:131-193)
        Device &d = Device::ThisThread();
        Bytes keys, vals;
        std::vector<uint64_t> koff, voff;
        csr(IndexBlock.Indexes, [](const block::IndexEntry &e) -> const std::string & { return e.Key; }, &keys, &koff);
        csr(DataBlock.Entries, [](const kv::Value &v) -> const kv::Value & { return v; }, &vals, &voff);
        const uint64_t m = FilterBlock.Cap(), k = FilterBlock.K();
        const uint64_t size = lsm_sst_image_size_host(koff.data(), voff.data(), 0, n, m);
        void *d_keys = d.Dev(0, pad16(keys.size()));
        void *d_koff = d.Dev(1, koff.size() * 8);
        void *d_vals = d.Dev(2, pad16(vals.size()));
        void *d_voff = d.Dev(3, voff.size() * 8);
        void *d_fs = d.Dev(4, 16);
        void *d_fo = d.Dev(5, 8);
        void *d_out = d.Dev(6, pad16(size));
        void *d_foot = d.Dev(7, 32);
        const size_t ws = lsm_build_sst_workspace_bytes(1, (uint32_t)n, m, (uint32_t)k);
        void *d_ws = d.Dev(8, ws);
        if (!keys.empty()) d.H2D(d_keys, keys.data(), keys.size());
        d.H2D(d_koff, koff.data(), koff.size() * 8);
        if (!vals.empty()) d.H2D(d_vals, vals.data(), vals.size());
        d.H2D(d_voff, voff.data(), voff.size() * 8);
        const uint64_t fs[2] = {0, n}, fo = 0;
        d.H2D(d_fs, fs, 16);
        d.H2D(d_fo, &fo, 8);
        check(lsm_build_sst(d.ctx(), (const uint8_t *)d_keys, (const uint64_t *)d_koff,
                            (const uint8_t *)d_vals, (const uint64_t *)d_voff,
                            (const uint64_t *)d_fs, 1, (uint32_t)n, m, (uint32_t)k,
                            (uint8_t *)d_out, (const uint64_t *)d_fo, (int64_t *)d_foot, d_ws, ws,
                            d.stream()),
              "lsm_build_sst");
        out->resize(size);
        int64_t foot[4];
        d.D2H(out->data(), d_out, size);
        d.D2H(foot, d_foot, 32);
        d.Sync();
        Footer.DataHandle = {foot[0], foot[1]};
        Footer.IndexHandle = {foot[2], foot[3]};
        for (size_t i = 0; i < n; i++)  // EncodeTo rewrites the offsets (sstable.go:164-169)
            IndexBlock.Indexes[i].Offset = foot[0] + (int64_t)(4 * i + voff[i]);
    } else {
        // General path: framing on the host, both regions encoded on the GPU.
        Buffer w;
        Header.EncodeTo(w);
        FilterBlock.EncodeTo(w);
        const int64_t data_off = (int64_t)w.Len();
        int64_t cur = data_off;
        for (size_t i = 0; i < n; i++) {
            IndexBlock.Indexes[i].Offset = cur;
            cur += 4 + (int64_t)DataBlock.Entries[i].size();
        }
        DataBlock.EncodeTo(w);
        Footer.DataHandle = {data_off, (int64_t)w.Len() - data_off};
        const int64_t idx_off = (int64_t)w.Len();
        Footer.IndexHandle = {idx_off, IndexBlock.Encode(w)};
        Footer.EncodeTo(w);
        *out = std::move(w.data);
    }
    image_ = *out;
    return Error();
}

Error SSTable::EncodeTo(const std::string &path) {
    Bytes img;
    Error e = EncodeImage(&img);
    if (e) return e;
    std::error_code ec;
    const auto dir = std::filesystem::path(path).parent_path();
    if (!dir.empty() && !std::filesystem::create_directories(dir, ec) && ec)
        return Error("create directory failed: mkdir " + dir.string() + ": " + ec.message());
    std::ofstream f(path, std::ios::binary | std::ios::trunc);
    if (!f) return Error("open file error: " + path);
    f.write((const char *)img.data(), (std::streamsize)img.size());
    path_ = path;
    return f ? Error() : Error("encode SSTable failed: write " + path);
}

Error SSTable::DecodeImage(const Bytes &img) {
    Reader r(img);
    Error e = Header.DecodeFrom(r);
    if (e) return e.Wrap("decode Header failed");
    e = FilterBlock.DecodeFrom(r);
    if (e) return e.Wrap("decode FilterBlock failed");
    if (img.size() < (size_t)block::kFooterSize)
        return Error("decode Footer failed: seek to footer position failed: invalid argument");
    Reader fr(img.data() + img.size() - block::kFooterSize, block::kFooterSize);
    e = Footer.DecodeFrom(fr);
    if (e) return e.Wrap("decode Footer failed").Wrap("decode Footer failed");
    const int64_t io = Footer.IndexHandle.Offset;
    if (io < 0) return Error("seek to index block position failed: invalid argument");
    Reader ir(img.data() + std::min((size_t)io, img.size()), img.size() - std::min((size_t)io, img.size()));
    e = IndexBlock.DecodeFrom(ir, Footer.IndexHandle.Size);
    if (e) return e.Wrap("decode IndexBlock failed");
    image_ = img;
    return Error();
}

Error SSTable::DecodeFrom(const std::string &path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return Error("open file error: open " + path + ": no such file or directory");
    Bytes img((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    path_ = path;
    return DecodeImage(img);
}

Error SSTable::DecodeDataBlock(const Bytes &img) {
    const int64_t off = Footer.DataHandle.Offset;
    if (off < 0) return Error("seek to IndexBlock position failed: invalid argument");
    const size_t o = std::min((size_t)off, img.size());
    Reader r(img.data() + o, img.size() - o);
    Error e = DataBlock.DecodeFrom(r, Footer.DataHandle.Size);
    if (e) return e.Wrap("decode DataBlock failed");
    return Error();
}

std::vector<kv::KeyValuePair> SSTable::GetDataBlockFromFile(const std::string &path, Error *err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) {
        *err = Error("open file error: open " + path + ": no such file or directory");
        return {};
    }
    Bytes img((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    Error e = DecodeDataBlock(img);
    if (e) {
        *err = e.Wrap("decode DataBlock failed");
        return {};
    }
    return GetKeyValuePairs(err);
}

std::vector<kv::KeyValuePair> SSTable::GetKeyValuePairs(Error *err) const {
    *err = Error();
    if (DataBlock.Len() == 0 || IndexBlock.Len() == 0) return {};
    if (DataBlock.Len() != IndexBlock.Len()) {
        *err = Error("mismatched DataBlock and IndexBlock entries");
        return {};
    }
    std::vector<kv::KeyValuePair> pairs;
    pairs.reserve(DataBlock.Entries.size());
    for (size_t i = 0; i < DataBlock.Entries.size(); i++)
        pairs.push_back({IndexBlock.Indexes[i].Key, DataBlock.Entries[i]});
    return pairs;
}

kv::Value SSTable::GetValueByOffset(int64_t offset, Error *err) {
    // Point read (not the batched path): Value.DecodeFrom at the offset.
    *err = Error();
    if (offset < 0) {
        *err = Error("seek to offset failed: seek " + path_ + ": invalid argument");
        return {};
    }
    if ((size_t)offset > image_.size()) offset = (int64_t)image_.size();
    Reader r(image_.data() + offset, image_.size() - (size_t)offset);
    if (r.Len() < 4) {
        *err = Error(std::string("decode value failed: decode value length: ") + eof_or_unexpected(r.Len()));
        return {};
    }
    const uint32_t vl = ld32(r.Cur());
    if (vl > (1u << 30)) {
        *err = Error("decode value failed: invalid value length: " + std::to_string(vl));
        return {};
    }
    if (r.Len() - 4 < vl) {
        *err = Error(std::string("decode value failed: decode value: ") + eof_or_unexpected(r.Len() - 4));
        return {};
    }
    return kv::Value(r.Cur() + 4, r.Cur() + 4 + vl);
}

bool SSTable::MayContain(const kv::Key &key) {
    if (Header.MinKey > key || Header.MaxKey < key) return false;
    return FilterBlock.MayContain(key);
}

void Builder::Add(const kv::KeyValuePair &p) {
    table_.Add(p);
    size_ += p.EstimateSize();
}

void Builder::Finalize() {
    if (table_.DataBlock.Len() > 0)
        table_.Header = {table_.IndexBlock.Indexes.front().Key,
                         table_.IndexBlock.Indexes[table_.DataBlock.Len() - 1].Key};
}

SSTable &Builder::Build() {
    Finalize();
    return table_;
}

std::vector<std::vector<kv::Value>> DecodeDataBlocks(const std::vector<Bytes> &regions,
                                                     std::vector<Error> *errs) {
    std::vector<std::pair<const uint8_t *, size_t>> blocks;
    for (auto &r : regions) blocks.push_back({r.data(), r.size()});
    Decoded dec = gpu_decode(LSM_GRAMMAR_V, blocks);
    std::vector<std::vector<kv::Value>> out(regions.size());
    errs->assign(regions.size(), Error());
    for (size_t i = 0; i < regions.size(); i++) {
        const uint8_t *p = regions[i].data();
        size_t end = 0;
        for (auto &ds : dec.desc[i]) {
            out[i].emplace_back(p + ds.rec_off + 4, p + ds.rec_off + 4 + ds.val_len);
            end = ds.rec_off + 4 + ds.val_len;
        }
        if (dec.status[i] == LSM_ST_TRUNC_LEN_PREFIX) (*errs)[i] = Error("read value length failed: unexpected EOF");
        else if (dec.status[i] == LSM_ST_TRUNC_VAL)
            (*errs)[i] = Error(std::string("read value data failed: ") + eof_or_unexpected(regions[i].size() - end - 4));
        else if (dec.status[i] != LSM_OK) (*errs)[i] = Error("decode status " + std::to_string(dec.status[i]));
    }
    return out;
}

static std::string status_text(int grammar, int32_t st) {
    switch (st) {
    case LSM_ST_TRUNC_LEN_PREFIX:
        return grammar == LSM_GRAMMAR_V ? "read value length failed: unexpected EOF"
                                        : "decode key length: unexpected EOF";
    case LSM_ST_TRUNC_VAL: return "read value data failed: unexpected EOF";
    case LSM_ST_IDX_OVERRUN: return "unexpected EOF: size limit reached while reading key length";
    case LSM_ST_CAPACITY: return "record capacity exhausted";
    default: return "decode status " + std::to_string(st);
    }
}

std::vector<std::vector<kv::KeyValuePair>> DecodeFiles(const std::vector<Bytes> &images,
                                                       std::vector<Error> *errs) {
    Device &d = Device::ThisThread();
    const size_t n = images.size();
    std::vector<std::vector<kv::KeyValuePair>> out(n);
    errs->assign(n, Error());
    if (n == 0) return out;
    std::vector<uint64_t> off(n), len(n);
    size_t total = 0;
    for (size_t i = 0; i < n; i++) {
        off[i] = total;
        len[i] = images[i].size();
        total += (images[i].size() + 15) & ~(size_t)15;
    }
    uint8_t *h_in = (uint8_t *)d.Host(0, pad16(total));
    std::memset(h_in, 0, pad16(total));
    for (size_t i = 0; i < n; i++) std::memcpy(h_in + off[i], images[i].data(), images[i].size());
    const size_t cap = total / 4 + 1;
    void *d_in = d.Dev(0, pad16(total));
    void *d_off = d.Dev(1, n * 8);
    void *d_len = d.Dev(2, n * 8);
    void *d_meta = d.Dev(3, n * sizeof(lsm_sst_meta));
    void *d_idesc = d.Dev(4, cap * sizeof(lsm_rec_desc));
    void *d_ival = d.Dev(5, cap * 8);
    void *d_ddesc = d.Dev(6, cap * sizeof(lsm_rec_desc));
    const size_t ws = lsm_decode_sst_workspace_bytes((uint32_t)n);
    void *d_ws = d.Dev(7, ws);
    d.H2D(d_in, h_in, pad16(total));
    d.H2D(d_off, off.data(), n * 8);
    d.H2D(d_len, len.data(), n * 8);
    check(lsm_decode_sst(d.ctx(), (const uint8_t *)d_in, (const uint64_t *)d_off,
                         (const uint64_t *)d_len, (uint32_t)n, nullptr, (lsm_sst_meta *)d_meta,
                         (lsm_rec_desc *)d_idesc, (int64_t *)d_ival, (lsm_rec_desc *)d_ddesc, d_ws,
                         ws, d.stream()),
          "lsm_decode_sst");
    std::vector<lsm_sst_meta> meta(n);
    d.D2H(meta.data(), d_meta, n * sizeof(lsm_sst_meta));
    d.Sync();
    static const char *const kStage[] = {"", "decode Header failed", "decode FilterBlock failed",
                                         "decode Footer failed", "decode IndexBlock failed",
                                         "decode DataBlock failed",
                                         "mismatched DataBlock and IndexBlock entries"};
    for (size_t f = 0; f < n; f++) {
        const lsm_sst_meta &m = meta[f];
        if (m.stage != LSM_SST_OK) {
            // The batch decides THAT file f fails and at which step; the
            // reference's full error text depends on the bytes at the failing
            // read, so it is rendered by the one-file path (also on the GPU),
            // which walks the same steps (sstable.go:87-127, 214-268).
            SSTable t;
            Error e = t.DecodeImage(images[f]);
            if (!e) e = t.DecodeDataBlock(images[f]);
            if (!e) t.GetKeyValuePairs(&e);
            if (!e) {  // cannot happen when the two paths agree; keep the step
                std::string msg = kStage[m.stage];
                if (m.status)
                    msg += ": " + status_text(m.stage == LSM_SST_INDEX ? LSM_GRAMMAR_IDX : LSM_GRAMMAR_V,
                                              m.status);
                e = Error(msg);
            }
            (*errs)[f] = e;
            continue;
        }
        if (m.nidx == 0 || m.ndata == 0) continue;  // GetKeyValuePairs' (nil, nil)
        std::vector<lsm_rec_desc> ki(m.nidx), vi(m.ndata);
        const size_t base = off[f] / 4;
        d.D2H(ki.data(), (lsm_rec_desc *)d_idesc + base, m.nidx * sizeof(lsm_rec_desc));
        d.D2H(vi.data(), (lsm_rec_desc *)d_ddesc + base, m.ndata * sizeof(lsm_rec_desc));
        d.Sync();
        const uint8_t *img = images[f].data();
        out[f].reserve(m.nidx);
        for (uint32_t i = 0; i < m.nidx; i++) {
            const uint64_t ko = ki[i].rec_off - off[f] + 4, vo = vi[i].rec_off - off[f] + 4;
            out[f].push_back({kv::Key((const char *)img + ko, ki[i].key_len),
                              kv::Value(img + vo, img + vo + vi[i].val_len)});
        }
    }
    return out;
}

std::vector<Bytes> BuildImages(const std::vector<kv::KeyValuePair> &sorted, uint64_t threshold,
                               uint64_t m, uint64_t k) {
    std::vector<uint64_t> koff(1, 0), voff(1, 0);
    for (auto &p : sorted) {
        koff.push_back(koff.back() + p.key.size());
        voff.push_back(voff.back() + p.value.size());
    }
    const uint64_t n = sorted.size();
    std::vector<uint64_t> fs(n + 2);
    const uint64_t nf = lsm_segment_files_host(koff.data(), voff.data(), n, threshold, fs.data());
    fs.resize(nf + 1);
    return BuildImagesAt(sorted, fs, m, k);
}

std::vector<Bytes> BuildImagesAt(const std::vector<kv::KeyValuePair> &sorted,
                                 const std::vector<uint64_t> &fs, uint64_t m, uint64_t k) {
    Device &d = Device::ThisThread();
    Bytes keys, vals;
    std::vector<uint64_t> koff, voff;
    csr(sorted, [](const kv::KeyValuePair &p) -> const std::string & { return p.key; }, &keys, &koff);
    csr(sorted, [](const kv::KeyValuePair &p) -> const kv::Value & { return p.value; }, &vals, &voff);
    const uint64_t nf = fs.empty() ? 0 : fs.size() - 1;
    std::vector<uint64_t> fo(nf), sz(nf);
    uint64_t total = 0, maxr = 0;
    for (uint64_t f = 0; f < nf; f++) {
        sz[f] = lsm_sst_image_size_host(koff.data(), voff.data(), fs[f], fs[f + 1], m);
        fo[f] = total;
        total += (sz[f] + 15) & ~(uint64_t)15;
        maxr = std::max(maxr, fs[f + 1] - fs[f]);
    }
    std::vector<Bytes> out(nf);
    if (nf == 0) return out;
    void *d_keys = d.Dev(0, pad16(keys.size()));
    void *d_koff = d.Dev(1, koff.size() * 8);
    void *d_vals = d.Dev(2, pad16(vals.size()));
    void *d_voff = d.Dev(3, voff.size() * 8);
    void *d_fs = d.Dev(4, fs.size() * 8);
    void *d_fo = d.Dev(5, fo.size() * 8);
    void *d_out = d.Dev(6, pad16(total));
    const size_t ws = lsm_build_sst_workspace_bytes((uint32_t)nf, (uint32_t)maxr, m, (uint32_t)k);
    void *d_ws = d.Dev(8, ws);
    if (!keys.empty()) d.H2D(d_keys, keys.data(), keys.size());
    d.H2D(d_koff, koff.data(), koff.size() * 8);
    if (!vals.empty()) d.H2D(d_vals, vals.data(), vals.size());
    d.H2D(d_voff, voff.data(), voff.size() * 8);
    d.H2D(d_fs, fs.data(), fs.size() * 8);
    d.H2D(d_fo, fo.data(), fo.size() * 8);
    check(lsm_build_sst(d.ctx(), (const uint8_t *)d_keys, (const uint64_t *)d_koff,
                        (const uint8_t *)d_vals, (const uint64_t *)d_voff, (const uint64_t *)d_fs,
                        (uint32_t)nf, (uint32_t)maxr, m, (uint32_t)k, (uint8_t *)d_out,
                        (const uint64_t *)d_fo, nullptr, d_ws, ws, d.stream()),
          "lsm_build_sst");
    for (uint64_t f = 0; f < nf; f++) {
        out[f].resize(sz[f]);
        d.D2H(out[f].data(), (uint8_t *)d_out + fo[f], sz[f]);
    }
    d.Sync();
    return out;
}

std::vector<SSTable> CompactAndMergeKVs(const std::vector<kv::KeyValuePair> &kvs, int level) {
    std::vector<SSTable> results;
    const size_t n = kvs.size();
    if (n == 0) return results;  // no builder.size: no table (merge.go:88-91)
    Device &d = Device::ThisThread();
    // the pairs as views: [4 bytes][key] [4 bytes][value], the IDX / V
    // descriptor convention (bytes at rec_off + 4)
    size_t total = 0;
    for (auto &p : kvs) total += 8 + p.key.size() + p.value.size();
    uint8_t *h = (uint8_t *)d.Host(0, pad16(total));
    std::vector<lsm_rec_desc> kd(n), vd(n);
    size_t at = 0;
    for (size_t i = 0; i < n; i++) {
        const kv::KeyValuePair &p = kvs[i];
        kd[i] = lsm_rec_desc{at, (uint32_t)p.key.size(), 0};
        std::memset(h + at, 0, 4);
        std::memcpy(h + at + 4, p.key.data(), p.key.size());
        at += 4 + p.key.size();
        vd[i] = lsm_rec_desc{at, 0, (uint32_t)p.value.size()};
        std::memset(h + at, 0, 4);
        if (!p.value.empty()) std::memcpy(h + at + 4, p.value.data(), p.value.size());
        at += 4 + p.value.size();
    }
    std::memset(h + at, 0, pad16(total) - at);
    void *d_buf = d.Dev(0, pad16(total));
    void *d_kd = d.Dev(1, n * sizeof(lsm_rec_desc));
    void *d_vd = d.Dev(2, n * sizeof(lsm_rec_desc));
    void *d_out = d.Dev(3, n * 4);
    void *d_fs = d.Dev(4, (n + 1) * 8);
    const size_t ws = lsm_merge_kvs_workspace_bytes(n);
    void *d_ws = d.Dev(5, ws);
    d.H2D(d_buf, h, pad16(total));
    d.H2D(d_kd, kd.data(), n * sizeof(lsm_rec_desc));
    d.H2D(d_vd, vd.data(), n * sizeof(lsm_rec_desc));
    uint64_t counts[2] = {0, 0};
    check(lsm_merge_kvs(d.ctx(), (const uint8_t *)d_buf, (const lsm_rec_desc *)d_kd,
                        (const lsm_rec_desc *)d_vd, n, level, kMaxSSTableSize, (uint32_t *)d_out,
                        (uint64_t *)d_fs, counts, d_ws, ws, d.stream()),
          "lsm_merge_kvs");
    std::vector<uint32_t> out(counts[0]);
    std::vector<uint64_t> fs(counts[1] + 1);
    if (counts[0]) d.D2H(out.data(), d_out, counts[0] * 4);
    d.D2H(fs.data(), d_fs, fs.size() * 8);
    d.Sync();
    std::vector<kv::KeyValuePair> written;
    written.reserve(out.size());
    for (uint32_t i : out) written.push_back(kvs[i]);
    const std::vector<Bytes> images = BuildImagesAt(written, fs);
    for (const Bytes &img : images) {
        SSTable t;
        Error e = t.DecodeImage(img);
        if (!e) e = t.DecodeDataBlock(img);
        if (e) throw std::runtime_error("CompactAndMergeKVs: built image does not decode: " + e.Message());
        t.level = level;
        results.push_back(std::move(t));
    }
    return results;
}

}  // namespace sstable
}  // namespace golsm
