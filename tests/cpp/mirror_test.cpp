// mirror_test.cpp — the reference's own block/sstable/bloom tests restated
// against the C++ mirror (go-lsm_amd/host/golsm.h), which runs every codec
// step on the GPU, plus randomized cross-checks against the CPU oracle
// (oracle/lsm_oracle.h, test infrastructure only).  Needs a gfx950 GPU;
// run by tests/test_mirror_gpu.py.  Each case cites the Go test it follows.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <functional>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "golsm.h"
#include "lsm_oracle.h"

using namespace golsm;

static int g_fail = 0, g_checks = 0;
static const char *g_case = "";

#define CHECK(c)                                                                     \
    do {                                                                             \
        g_checks++;                                                                  \
        if (!(c)) {                                                                  \
            g_fail++;                                                                \
            std::fprintf(stderr, "FAIL [%s] %s:%d: %s\n", g_case, __FILE__, __LINE__, #c); \
        }                                                                            \
    } while (0)
#define CHECK_ERR_HAS(e, s)                                                 \
    do {                                                                    \
        const Error e_ = (e);                                               \
        CHECK((bool)e_ && e_.Message().find(s) != std::string::npos);       \
        if (!e_.Message().empty() && e_.Message().find(s) == std::string::npos) \
            std::fprintf(stderr, "  got: %s\n", e_.Message().c_str());     \
    } while (0)

static kv::Value V(const char *s) { return kv::Value(s, s + std::strlen(s)); }
static std::string tmpdir() {
    static std::string d;
    if (d.empty()) {
        char t[] = "/tmp/golsm_mirror_XXXXXX";
        d = mkdtemp(t);
    }
    return d;
}

// ---- sstable/block/data_test.go ---------------------------------------------

static void TestDataBlock_EncodeDecode() {  // data_test.go:13-87
    struct C { std::vector<kv::Value> e; int64_t limit; };
    std::vector<C> cases = {
        {{}, 0},
        {{V("value1")}, 0},
        {{V("value1"), V("value2"), V("value3")}, 0},
        {{V("value1"), V("value2")}, 100},
        {{V("value1"), V("value2")}, 2 * (4 + 6)},
    };
    for (auto &c : cases) {
        block::DataBlock b;
        for (auto &v : c.e) b.Add(v);
        Buffer buf;
        CHECK(!b.EncodeTo(buf));
        block::DataBlock d;
        Reader r(buf.data);
        CHECK(!d.DecodeFrom(r, c.limit));
        CHECK(d.Len() == (int)c.e.size());
        for (size_t i = 0; i < c.e.size() && i < d.Entries.size(); i++) CHECK(d.Entries[i] == c.e[i]);
    }
}

static void TestDataBlock_DecodeWithSizeLimit() {  // data_test.go:89-131
    block::DataBlock b;
    b.Add(V("value1"));
    b.Add(V("value2"));
    b.Add(V("value3"));
    Buffer buf;
    CHECK(!b.EncodeTo(buf));
    {
        block::DataBlock d;
        Reader r(buf.data);
        Error e = d.DecodeFrom(r, 4 + 6 - 1);
        CHECK_ERR_HAS(e, "read value data failed: unexpected EOF");
    }
    {
        block::DataBlock d;
        Reader r(buf.data);
        CHECK(!d.DecodeFrom(r, 2 * (4 + 6)));
        CHECK(d.Len() == 2);
        CHECK(d.Entries[0] == b.Entries[0] && d.Entries[1] == b.Entries[1]);
    }
}

static void TestDataBlock_DecodeCorruptedData() {  // data_test.go:133-162
    {
        Bytes in = {0x3f, 0x42, 0x0f, 0x00};  // u32 999999, no data
        block::DataBlock d;
        Reader r(in);
        Error e = d.DecodeFrom(r, 0);
        CHECK_ERR_HAS(e, "read value data failed: EOF");
    }
    {
        Bytes in = {10, 0, 0, 0, 'i', 'n', 'c', 'o', 'm'};
        block::DataBlock d;
        Reader r(in);
        Error e = d.DecodeFrom(r, 0);
        CHECK_ERR_HAS(e, "read value data failed: unexpected EOF");
    }
    {
        Bytes in = {6, 0, 0, 0, 'v', 'a', 'l', 'u', 'e', '1', 2, 0};  // dangling 2-byte prefix
        block::DataBlock d;
        Reader r(in);
        Error e = d.DecodeFrom(r, 0);
        CHECK_ERR_HAS(e, "read value length failed: unexpected EOF");
        CHECK(d.Len() == 1);  // records before the error are kept
    }
}

static void TestDataBlock_AddAndLen() {  // data_test.go:164-178
    block::DataBlock b;
    CHECK(b.Len() == 0);
    b.Add(V("value1"));
    CHECK(b.Len() == 1);
    b.Add(V("value2"));
    CHECK(b.Len() == 2);
    CHECK(b.Entries[0] == V("value1") && b.Entries[1] == V("value2"));
}

// ---- sstable/block/index_test.go ----------------------------------------------

static void TestIndexBlock_EncodeDecode() {  // index_test.go:60-89
    block::IndexBlock b;
    b.Add("key1", 100);
    b.Add("key2", 200);
    b.Add("key3", 300);
    Buffer buf;
    Error err;
    const int64_t size = b.Encode(buf, &err);
    CHECK(!err);
    CHECK(size == 3 * (4 + 4 + 8));
    block::IndexBlock d;
    {
        Reader r(buf.data);
        Error e = d.DecodeFrom(r, -1);
        CHECK_ERR_HAS(e, "invalid size: -1, must be non-negative");
    }
    Reader r(buf.data);
    CHECK(!d.DecodeFrom(r, size));
    CHECK(d.Len() == 3);
    CHECK(d.Indexes[0].Key == "key1" && d.Indexes[0].Offset == 100);
    CHECK(d.Indexes[1].Key == "key2" && d.Indexes[1].Offset == 200);
    CHECK(d.Indexes[2].Key == "key3" && d.Indexes[2].Offset == 300);
}

static void TestIndexBlock_Iterator() {  // index_test.go:91-126 (Seek exact match)
    block::IndexBlock b;
    b.Add("apple", 10);
    b.Add("banana", 20);
    b.Add("cherry", 30);
    CHECK(b.Seek("banana") == 1);
    CHECK(b.Indexes[b.Seek("banana")].Offset == 20);
    CHECK(b.Seek("orange") == -1);
}

static void TestIndexBlock_DecodeWithSizeLimit() {  // index_test.go:128-153
    block::IndexBlock b;
    b.Add("key1", 100);
    b.Add("key2", 200);
    Buffer buf;
    b.Encode(buf);
    const int64_t first = 4 + 4 + 8;
    {
        block::IndexBlock d;
        Reader r(buf.data);
        CHECK(!d.DecodeFrom(r, first));
        CHECK(d.Len() == 1 && d.Indexes[0].Key == "key1" && d.Indexes[0].Offset == 100);
    }
    {
        Bytes cut(buf.data.begin(), buf.data.begin() + first - 2);
        block::IndexBlock d;
        Reader r(cut);
        Error e = d.DecodeFrom(r, first);
        CHECK_ERR_HAS(e, "decode index offset failed: unexpected EOF");
    }
    {  // an entry straddling the limit reads past it, then trips the size check
        block::IndexBlock d;
        Reader r(buf.data);
        Error e = d.DecodeFrom(r, first + 3);
        CHECK_ERR_HAS(e, "unexpected EOF: size limit reached while reading key length");
        CHECK(d.Len() == 1);
    }
}

// ---- sstable/block/header_test.go, footer_test.go --------------------------------

static void TestHeader_EncodeDecode() {  // header_test.go:14-83
    const std::pair<const char *, const char *> cases[] = {{"key1", "key2"}, {"", "key2"}, {"same", "same"}};
    for (auto &c : cases) {
        block::Header h{c.first, c.second};
        Buffer buf;
        CHECK(!h.EncodeTo(buf));
        block::Header d;
        Reader r(buf.data);
        CHECK(!d.DecodeFrom(r));
        CHECK(d.MinKey == c.first && d.MaxKey == c.second);
    }
    block::Header d;
    Bytes junk = {1, 2};
    Reader r(junk);
    CHECK_ERR_HAS(d.DecodeFrom(r), "decode min key: decode key keyLen: unexpected EOF");
}

static void TestFooter_EncodeDecode() {  // footer_test.go:10-157
    block::Footer f{{100, 200}, {300, 400}};
    Buffer buf;
    CHECK(!f.EncodeTo(buf));
    CHECK(buf.Len() == (size_t)block::kFooterSize);
    block::Footer d;
    Reader r(buf.data);
    CHECK(!d.DecodeFrom(r));
    CHECK(d.DataHandle.Offset == 100 && d.DataHandle.Size == 200);
    CHECK(d.IndexHandle.Offset == 300 && d.IndexHandle.Size == 400);
    Bytes short_(buf.data.begin(), buf.data.begin() + 20);
    Reader rs(short_);
    block::Footer e;
    CHECK_ERR_HAS(e.DecodeFrom(rs), "decode index handle failed: decode footer failed: unexpected EOF");
    Bytes none;
    Reader rn(none);
    CHECK_ERR_HAS(e.DecodeFrom(rn), "decode data handle failed: decode footer failed: EOF");
}

// ---- sstable/bloom/bloom_test.go ----------------------------------------------------

static void TestBloomBasic() {  // bloom_test.go:13-29 (TestAndAdd = Test then Add)
    bloom::Filter f(1000, 4);
    f.AddString("Bess");
    const bool n3a = f.TestString("Emma");
    f.AddString("Emma");
    CHECK(f.TestString("Bess"));
    CHECK(!f.TestString("Jane"));
    CHECK(!n3a);
    CHECK(f.TestString("Emma"));
}

static void TestBloomLowNumbers() {  // bloom_test.go:31-35
    bloom::Filter f(0, 0);
    CHECK(f.K() == 1 && f.Cap() == 1);
}

static void TestBloomVsOracle() {  // GPU words == oracle words; encode/decode round trip
    std::mt19937_64 rng(7);
    for (uint64_t m : {1000ull, 64ull, 65ull, 1600000ull}) {
        bloom::Filter f(m, 16);
        std::vector<uint64_t> ref((m + 63) / 64, 0);
        for (int i = 0; i < 500; i++) {
            std::string k(rng() % 40, '\0');
            for (auto &ch : k) ch = (char)rng();
            f.AddString(k);
            ora_bloom_add(ref.data(), m, 16, (const uint8_t *)k.data(), k.size());
        }
        CHECK(f.Words() == ref);
        Buffer buf;
        CHECK(!f.EncodeTo(buf));
        CHECK(buf.Len() == ora_filter_block_size(m));
        Bytes oenc(ora_filter_block_size(m));
        ora_filter_encode(ref.data(), m, 16, oenc.data());
        CHECK(buf.data == oenc);
        bloom::Filter g(1, 1);
        Reader r(buf.data);
        CHECK(!g.DecodeFrom(r));
        CHECK(g.Equal(f));
    }
}

// ---- sstable/builder_test.go ------------------------------------------------------

static void TestBuilder() {  // builder_test.go:19-116
    sstable::Builder b;
    kv::KeyValuePair p1{"key1", V("value1")}, p2{"key2", V("value2")};
    b.Add(p1);
    b.Add(p2);
    CHECK(b.Table().DataBlock.Len() == 2);
    CHECK(b.Table().IndexBlock.Indexes[0].Key == "key1" && b.Table().IndexBlock.Indexes[1].Key == "key2");
    CHECK(b.Size() == p1.EstimateSize() + p2.EstimateSize());
    for (auto c : {std::make_pair(sstable::kMaxSSTableSize - 1, false),
                   std::make_pair(sstable::kMaxSSTableSize, true),
                   std::make_pair(sstable::kMaxSSTableSize + 1, true)}) {
        sstable::Builder x;
        x.SetSize(c.first);
        CHECK(x.ShouldFlush() == c.second);
    }
    sstable::Builder one;
    one.Add({"testKey", V("testValue")});
    sstable::SSTable &t = one.Build();
    CHECK(t.Header.MinKey == "testKey" && t.Header.MaxKey == "testKey");
}

// ---- sstable/sstable_test.go ------------------------------------------------------

static sstable::SSTable sample() {  // createSampleSSTable sstable_test.go:29-55
    sstable::SSTable t;
    t.DataBlock.Entries = {V("value1"), V("value2")};
    t.IndexBlock.Indexes = {{"key1", 0}, {"key2", 100}};
    t.Header = {"key1", "key2"};
    t.FilterBlock.AddString("key1");
    t.FilterBlock.AddString("key2");
    return t;
}

static void TestSSTableEncodeDecode() {  // sstable_test.go:72-163, 187-198
    const std::string path = tmpdir() + "/0-level/1.sst";
    sstable::SSTable t = sample();
    CHECK(!t.EncodeTo(path));
    CHECK(std::filesystem::exists(path));
    CHECK(t.IndexBlock.Indexes[1].Offset == t.Footer.DataHandle.Offset + 4 + 6);  // rewritten
    sstable::SSTable n;
    CHECK(!n.DecodeFrom(path));
    CHECK(n.Header.MinKey == "key1" && n.Header.MaxKey == "key2");
    CHECK(n.IndexBlock.Len() == 2);
    CHECK(n.IndexBlock.Indexes[0].Offset == t.IndexBlock.Indexes[0].Offset);
    CHECK(n.Footer.IndexHandle.Offset != 0 && n.Footer.IndexHandle.Size != 0);
    CHECK(n.DataBlock.Len() == 0);  // DecodeFrom does not load the data block
    CHECK(n.FilterBlock.Equal(t.FilterBlock));
    Error err;
    auto pairs = n.GetDataBlockFromFile(path, &err);
    CHECK(!err);
    CHECK(pairs.size() == 2 && pairs[0].key == "key1" && pairs[1].key == "key2");
    CHECK(pairs.size() == 2 && pairs[0].value == V("value1") && pairs[1].value == V("value2"));
    kv::Value v = n.GetValueByOffset(n.IndexBlock.Indexes[0].Offset, &err);
    CHECK(!err && v == V("value1"));
    n.GetValueByOffset(999999, &err);
    CHECK_ERR_HAS(err, "decode value length");
    // The general (non-fused) path must produce the same bytes: a filter built
    // from different keys than the index forces it.
    sstable::SSTable g = sample();
    g.FilterBlock = bloom::Filter::Default();
    g.FilterBlock.AddString("key1");
    g.FilterBlock.Words();  // materialize first: no longer "only pending"
    g.FilterBlock.AddString("key2");
    Bytes a, b;
    CHECK(!t.EncodeImage(&a));
    CHECK(!g.EncodeImage(&b));
    CHECK(a == b);
}

static void TestSSTableEdgeCases() {  // sstable_test.go:164-185, 200-206, 238-256, 293-361, 402-415
    sstable::SSTable t = sample();
    Error err;
    auto pairs = t.GetKeyValuePairs(&err);
    CHECK(!err && pairs.size() == 2);
    t.DataBlock.Entries.resize(1);
    t.GetKeyValuePairs(&err);
    CHECK_ERR_HAS(err, "mismatched DataBlock and IndexBlock entries");
    t.DataBlock.Entries.clear();
    pairs = t.GetKeyValuePairs(&err);
    CHECK(!err && pairs.empty());

    sstable::SSTable m = sample();
    CHECK(m.MayContain("key1") && m.MayContain("key2"));
    CHECK(!m.MayContain("nonexistent"));
    CHECK(!m.MayContain("key0") && !m.MayContain("key3") && !m.MayContain(""));

    sstable::SSTable e;  // TestEmptyDataBlock
    const std::string path = tmpdir() + "/empty.sst";
    CHECK(!e.EncodeTo(path));
    sstable::SSTable ed;
    CHECK(!ed.DecodeFrom(path));
    CHECK(ed.DataBlock.Len() == 0 && ed.IndexBlock.Len() == 0);

    sstable::SSTable nf;
    CHECK_ERR_HAS(nf.DecodeFrom("/nonexistent/file.sst"), "open file error");
    CHECK_ERR_HAS(nf.EncodeTo("/proc/nonexistent/path/123.sst"), "create directory failed");

    const std::string bad = tmpdir() + "/corrupted.sst";
    std::ofstream(bad) << "invalid data";
    sstable::SSTable c;
    CHECK_ERR_HAS(c.DecodeFrom(bad), "decode Header failed");
}

static void TestConcurrentAccess() {  // sstable_test.go:379-400: one Device per thread
    const std::string path = tmpdir() + "/concurrent.sst";
    sstable::SSTable t = sample();
    CHECK(!t.EncodeTo(path));
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    for (int i = 0; i < 5; i++)
        th.emplace_back([&] {
            sstable::SSTable n;
            Error e = n.DecodeFrom(path);
            Error e2;
            auto p = n.GetDataBlockFromFile(path, &e2);
            if (e || e2 || p.size() != 2) bad++;
        });
    for (auto &x : th) x.join();
    CHECK(bad == 0);
}

// ---- randomized cross-checks vs the oracle --------------------------------------

static std::vector<kv::KeyValuePair> random_sorted(std::mt19937_64 &rng, size_t n, int maxv) {
    std::vector<kv::KeyValuePair> v(n);
    for (size_t i = 0; i < n; i++) {
        char k[32];
        std::snprintf(k, sizeof k, "k%012zu", i * 3 + (size_t)(rng() % 3));
        v[i].key = k;
        v[i].value.resize(rng() % (maxv + 1));
        for (auto &b : v[i].value) b = (uint8_t)rng();
    }
    return v;
}

static void TestBuildImagesVsOracle() {  // BuildImages == Builder+EncodeTo == oracle, per file
    std::mt19937_64 rng(11);
    auto recs = random_sorted(rng, 6000, 900);
    Bytes keys, vals;
    std::vector<uint64_t> koff{0}, voff{0};
    for (auto &p : recs) {
        keys.insert(keys.end(), p.key.begin(), p.key.end());
        vals.insert(vals.end(), p.value.begin(), p.value.end());
        koff.push_back(keys.size());
        voff.push_back(vals.size());
    }
    const uint64_t thr = 256 * 1024, m = 100000, k = 7;
    auto imgs = sstable::BuildImages(recs, thr, m, k);
    std::vector<uint64_t> starts(recs.size() + 2);
    const uint64_t nf = ora_segment_files(koff.data(), voff.data(), recs.size(), thr, starts.data());
    CHECK(imgs.size() == nf);
    for (uint64_t f = 0; f < nf && f < imgs.size(); f++) {
        Bytes ref(ora_sst_image_size(koff.data(), voff.data(), starts[f], starts[f + 1], m));
        int64_t foot[4];
        ora_build_sst(keys.data(), koff.data(), vals.data(), voff.data(), starts[f], starts[f + 1], m, k,
                      ref.data(), foot);
        CHECK(imgs[f] == ref);
        // Builder path for the same file
        sstable::Builder b;
        b.Table().FilterBlock = bloom::Filter(m, k);
        for (uint64_t i = starts[f]; i < starts[f + 1]; i++) b.Add(recs[i]);
        Bytes img;
        CHECK(!b.Build().EncodeImage(&img));
        CHECK(img == ref);
        // full decode back
        sstable::SSTable d;
        d.FilterBlock = bloom::Filter(1, 1);
        CHECK(!d.DecodeImage(ref));
        CHECK(!d.DecodeDataBlock(ref));
        Error err;
        auto pairs = d.GetKeyValuePairs(&err);
        CHECK(!err && pairs.size() == starts[f + 1] - starts[f]);
        bool same = true;
        for (size_t i = 0; i < pairs.size(); i++)
            same &= pairs[i].key == recs[starts[f] + i].key && pairs[i].value == recs[starts[f] + i].value;
        CHECK(same);
        for (uint64_t i = starts[f]; i < starts[f + 1]; i += 97) CHECK(d.MayContain(recs[i].key));
    }
}

static void TestDecodeDataBlocksVsOracle() {  // batch decode == oracle, incl. truncations
    std::mt19937_64 rng(13);
    std::vector<Bytes> regions;
    for (int b = 0; b < 300; b++) {
        Bytes r;
        const int n = (int)(rng() % 50);
        for (int i = 0; i < n; i++) {
            const uint32_t l = (uint32_t)(rng() % 300);
            for (int s = 0; s < 4; s++) r.push_back((uint8_t)(l >> (8 * s)));
            for (uint32_t j = 0; j < l; j++) r.push_back((uint8_t)rng());
        }
        if (b % 7 == 3 && !r.empty()) r.resize(r.size() - 1 - rng() % std::min<size_t>(r.size(), 9));
        regions.push_back(r);
    }
    std::vector<Error> errs;
    auto out = sstable::DecodeDataBlocks(regions, &errs);
    CHECK(out.size() == regions.size());
    for (size_t b = 0; b < regions.size(); b++) {
        std::vector<ora_desc> d(regions[b].size() / 4 + 1);
        uint32_t n = 0;
        const int st = ora_decode_block(LSM_GRAMMAR_V, regions[b].data(), 0, regions[b].size(), d.data(),
                                        nullptr, d.size(), &n);
        CHECK(out[b].size() == n);
        CHECK((bool)errs[b] == (st != 0));
        bool same = out[b].size() == n;
        for (uint32_t i = 0; same && i < n; i++)
            same = out[b][i] == kv::Value(regions[b].begin() + d[i].rec_off + 4,
                                          regions[b].begin() + d[i].rec_off + 4 + d[i].val_len);
        CHECK(same);
        // single-block DecodeFrom agrees with the batch
        block::DataBlock one;
        Reader r(regions[b]);
        Error e = one.DecodeFrom(r, 0);
        CHECK(one.Entries == out[b]);
        CHECK(e.Message() == errs[b].Message());
    }
}

static void TestDecodeFilesVsSingleFile() {  // lsm_decode_sst batch == per-file DecodeFrom path
    std::mt19937_64 rng(29);
    auto recs = random_sorted(rng, 3000, 400);
    std::vector<Bytes> images = sstable::BuildImages(recs, 64 * 1024, 8192, 4);
    const size_t good = images.size();
    // corrupted variants: truncations and footer fields
    for (size_t i = 0; i < good && i < 6; i++) {
        Bytes t = images[i];
        t.resize(t.size() - 1 - rng() % 200);
        images.push_back(t);
        Bytes u = images[i];
        const size_t at = u.size() - 32 + 8 * (rng() % 4);
        u[at + (rng() % 3)] ^= (uint8_t)(1 + rng() % 255);
        images.push_back(u);
    }
    std::vector<Error> errs;
    auto batch = sstable::DecodeFiles(images, &errs);
    CHECK(batch.size() == images.size());
    for (size_t f = 0; f < images.size(); f++) {
        sstable::SSTable t;
        Error e = t.DecodeImage(images[f]);
        std::vector<kv::KeyValuePair> pairs;
        if (!e) {
            e = t.DecodeDataBlock(images[f]);
            if (!e) pairs = t.GetKeyValuePairs(&e);
        }
        CHECK((bool)e == (bool)errs[f]);
        if (e && errs[f]) {
            const std::string &a = e.Message(), &b = errs[f].Message();
            CHECK(a == b);
            if (a != b) std::fprintf(stderr, "  single: %s\n  batch:  %s\n", a.c_str(), b.c_str());
        }
        // both agree with the oracle's file-level decode on whether and where it fails
        {
            ora_sst_meta om;
            const size_t cap = images[f].size() / 4 + 1;
            std::vector<ora_desc> id(cap), dd(cap);
            std::vector<int64_t> iv(cap);
            ora_sst_decode(images[f].data(), images[f].size(), &om, id.data(), iv.data(), cap,
                           dd.data(), cap);
            CHECK((om.stage != 0) == (bool)errs[f]);
            static const char *const kStep[] = {"", "decode Header", "decode FilterBlock",
                                                "decode Footer", "decode IndexBlock",
                                                "decode DataBlock", "mismatched"};
            const bool seek = (om.stage == 4 && om.idx_off < 0) || (om.stage == 5 && om.data_off < 0);
            if (om.stage > 0 && om.stage < 7 && !seek) {
                CHECK(errs[f].Message().rfind(kStep[om.stage], 0) == 0);
                if (errs[f].Message().rfind(kStep[om.stage], 0) != 0)
                    std::fprintf(stderr, "  oracle stage %d, got: %s\n", om.stage,
                                 errs[f].Message().c_str());
            }
            if (om.stage == 0) CHECK(om.nidx == (om.ndata ? batch[f].size() : om.nidx));
        }
        bool same = batch[f].size() == pairs.size();
        for (size_t i = 0; same && i < pairs.size(); i++)
            same = batch[f][i].key == pairs[i].key && batch[f][i].value == pairs[i].value;
        CHECK(same);
        if (f < good) CHECK(!errs[f] && !batch[f].empty());
    }
}

static void TestCompactAndMergeKVs() {  // merge_test.go:12-60 + the oracle (ORA_TIE_INPUT)
    {
        std::vector<kv::KeyValuePair> in = {{"alpha", kv::Value{'A'}},
                                            {"beta", kv::Value{'B'}},
                                            {"beta", kv::Value{'B', '2'}},
                                            {"carrot", kv::Value{'C'}},
                                            {"delta", kv::Value{'D'}}};
        auto sst = sstable::CompactAndMergeKVs(in, 1);
        CHECK(sst.size() == 1);
        if (sst.size() == 1) {
            CHECK(sst[0].level == 1);
            CHECK(sst[0].DataBlock.Entries.size() == 4);
            std::vector<std::string> keys;
            for (auto &e : sst[0].IndexBlock.Indexes) keys.push_back(e.Key);
            CHECK((keys == std::vector<std::string>{"alpha", "beta", "carrot", "delta"}));
            CHECK(sst[0].DataBlock.Entries.size() > 1 && sst[0].DataBlock.Entries[1] == kv::Value{'B'});
            CHECK(sst[0].MayContain("alpha") && sst[0].MayContain("delta"));
            CHECK(!sst[0].MayContain("nonexistent") && !sst[0].MayContain("deletedKey"));
        }
        CHECK(sstable::CompactAndMergeKVs({}, 1).empty());
    }
    // many pairs, duplicates, tombstones at the last level, several tables
    std::mt19937_64 rng(41);
    const std::string tomb = "\xEF\xBD\x9E" "DELETED" "\xEF\xBD\x9E";
    std::vector<kv::KeyValuePair> in;
    for (int i = 0; i < 40000; i++) {  // ~22k distinct keys, ~3 MB: two or more tables
        std::string k = "key" + std::to_string(rng() % 30000);
        kv::Value v;
        if (rng() % 10 == 0) v.assign(tomb.begin(), tomb.end());
        else v.assign(60 + rng() % 120, (uint8_t)('a' + rng() % 26));
        in.push_back({k, v});
    }
    for (int level : {1, 6}) {
        auto sst = sstable::CompactAndMergeKVs(in, level);
        // the oracle over the same pairs
        std::string blob;
        std::vector<uint64_t> koff, voff;
        std::vector<uint32_t> klen, vlen;
        for (auto &p : in) {
            koff.push_back(blob.size()); klen.push_back((uint32_t)p.key.size()); blob += p.key;
            voff.push_back(blob.size()); vlen.push_back((uint32_t)p.value.size());
            blob.append(p.value.begin(), p.value.end());
        }
        std::vector<uint32_t> out(in.size());
        std::vector<uint64_t> starts(in.size() + 2);
        uint64_t nf = 0;
        const uint64_t cnt = ora_merge_kvs((const uint8_t *)blob.data(), koff.data(), klen.data(),
                                           voff.data(), vlen.data(), in.size(), level,
                                           sstable::kMaxSSTableSize, ORA_TIE_INPUT, out.data(),
                                           starts.data(), &nf);
        CHECK(sst.size() == nf);
        bool same = sst.size() == nf;
        for (uint64_t f = 0; same && f < nf; f++) {
            const auto &E = sst[f].DataBlock.Entries;
            const auto &I = sst[f].IndexBlock.Indexes;
            same = E.size() == starts[f + 1] - starts[f] && I.size() == E.size() && sst[f].level == level;
            for (uint64_t r = 0; same && r < E.size(); r++) {
                const auto &want = in[out[starts[f] + r]];
                same = I[r].Key == want.key && E[r] == want.value;
            }
        }
        CHECK(same);
        CHECK(cnt > 0 && nf >= 2);
    }
}

int main(int argc, char **argv) {
    const std::pair<const char *, std::function<void()>> tests[] = {
        {"TestDataBlock_EncodeDecode", TestDataBlock_EncodeDecode},
        {"TestDataBlock_DecodeWithSizeLimit", TestDataBlock_DecodeWithSizeLimit},
        {"TestDataBlock_DecodeCorruptedData", TestDataBlock_DecodeCorruptedData},
        {"TestDataBlock_AddAndLen", TestDataBlock_AddAndLen},
        {"TestIndexBlock_EncodeDecode", TestIndexBlock_EncodeDecode},
        {"TestIndexBlock_Iterator", TestIndexBlock_Iterator},
        {"TestIndexBlock_DecodeWithSizeLimit", TestIndexBlock_DecodeWithSizeLimit},
        {"TestHeader_EncodeDecode", TestHeader_EncodeDecode},
        {"TestFooter_EncodeDecode", TestFooter_EncodeDecode},
        {"TestBloomBasic", TestBloomBasic},
        {"TestBloomLowNumbers", TestBloomLowNumbers},
        {"TestBloomVsOracle", TestBloomVsOracle},
        {"TestBuilder", TestBuilder},
        {"TestSSTableEncodeDecode", TestSSTableEncodeDecode},
        {"TestSSTableEdgeCases", TestSSTableEdgeCases},
        {"TestConcurrentAccess", TestConcurrentAccess},
        {"TestBuildImagesVsOracle", TestBuildImagesVsOracle},
        {"TestDecodeDataBlocksVsOracle", TestDecodeDataBlocksVsOracle},
        {"TestDecodeFilesVsSingleFile", TestDecodeFilesVsSingleFile},
        {"TestCompactAndMergeKVs", TestCompactAndMergeKVs},
    };
    int failed_cases = 0;
    for (auto &t : tests) {
        if (argc > 1 && std::strcmp(argv[1], t.first) != 0) continue;
        g_case = t.first;
        const int before = g_fail;
        try {
            t.second();
        } catch (const std::exception &e) {
            std::fprintf(stderr, "FAIL [%s] exception: %s\n", t.first, e.what());
            g_fail++;
        }
        const bool ok = g_fail == before;
        failed_cases += !ok;
        std::printf("%s %s\n", ok ? "PASS" : "FAIL", t.first);
    }
    std::filesystem::remove_all(tmpdir());
    std::printf("%d checks, %d failed, %d failing cases\n", g_checks, g_fail, failed_cases);
    return g_fail ? 1 : 0;
}
