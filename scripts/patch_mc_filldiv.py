# A/B variant: the hit-row fill's row of a byte offset by a float reciprocal and one
# correction step instead of an integer division per 16-byte chunk.
s = open('encode.hip').read()
old = '''        auto one_at = [&](uint32_t o) -> uint32_t {  // byte o of the rows: the candidate's 1
            const uint32_t row = o / nfile;'''
assert old in s
s = s.replace(old, '''        // row of byte o: o < 2^22 and nfile <= 2^11 are exact in float; the
        // product is within one of o / nfile, one correction step each way
        const float rcp = 1.0f / (float)nfile;
        auto row_of = [&](uint32_t o) -> uint32_t {
            uint32_t r = (uint32_t)((float)o * rcp);
            r = r * nfile > o ? r - 1 : r;
            r = (r + 1) * nfile <= o ? r + 1 : r;
            return r;
        };
        auto one_at = [&](uint32_t o) -> uint32_t {  // byte o of the rows: the candidate's 1
            const uint32_t row = row_of(o);''')
old = '''            for (uint32_t row = o / nfile; row * nfile < o + 16; row++) {'''
assert old in s
s = s.replace(old, '''            for (uint32_t row = row_of(o); row * nfile < o + 16; row++) {''')
open('encode.hip', 'w').write(s)
print('ok filldiv')
