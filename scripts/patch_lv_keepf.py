# A/B variant: lv_classify_kernel keeps the candidate table's filter shape (m, its
# reciprocal, k) from the range check's load in registers for the record stores, instead
# of loading the table's fields again after the scan.
s = open('encode.hip').read()
old = '''    uint32_t cand[kLvPer], rank[kLvPer];
    uint64_t hh[kLvPer][4];'''
assert old in s
s = s.replace(old, '''    uint32_t cand[kLvPer], rank[kLvPer], fk[kLvPer];
    uint64_t hh[kLvPer][4], fm[kLvPer], fmr[kLvPer];''')
old = '''        if (lo > 0) {
            const McFile &F = w.files[idx];
            if (F.ok) {'''
assert old in s
s = s.replace(old, '''        if (lo > 0) {
            const McFile &F = w.files[idx];
            fm[p] = F.m; fmr[p] = F.mr; fk[p] = F.k;
            if (F.ok) {''')
old = '''        const McFile &F = w.files[cand[p]];
        if (lv_compact(F)) {
            store_hash_rec(hh[p], (uint32_t)F.m, (uint32_t)F.mr, (uint32_t)(F.mr >> 32),
                           reinterpret_cast<uint32_t *>(w.rec + slot));'''
assert old in s
s = s.replace(old, '''        if (fm[p] != 0 && fm[p] <= (1ull << kHashRecBits) && fk[p] <= kSplitMaxK) {  // lv_compact
            store_hash_rec(hh[p], (uint32_t)fm[p], (uint32_t)fmr[p], (uint32_t)(fmr[p] >> 32),
                           reinterpret_cast<uint32_t *>(w.rec + slot));''')
open('encode.hip', 'w').write(s)
print('ok keepf')
