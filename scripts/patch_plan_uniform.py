s=open('encode.hip').read()
old='''    const uint64_t len = lane < cnt ? p1 - p0 : 0;
    uint64_t tot64;
    const uint64_t P64 = wave_excl_scan64(lane < cnt ? pre + len : 0, &tot64);
    tot64 = uni64(tot64);
    R.cnt = cnt;
    R.dst = dst;
    R.base = base;
    R.Sc = lane64(p0, 0);
    R.sbytes = 0;
    if (tot64 + 64 > 4ull * cap) return false;
    R.len = (uint32_t)len;
    {
        const uint32_t l0 = uni((uint32_t)len);
        R.ulen = __ballot(lane < cnt && (uint32_t)len != l0) ? ~0u : l0;
    }
    R.P = (uint32_t)P64;
    R.tot = (uint32_t)tot64;'''
new='''    const uint64_t len = lane < cnt ? p1 - p0 : 0;
    R.cnt = cnt;
    R.dst = dst;
    R.base = base;
    R.Sc = lane64(p0, 0);
    R.sbytes = 0;
    // records of one payload length (fixed-size keys or values): the record
    // starts are lane * (pre + len), no 64-bit scan
    const uint64_t l0 = lane64(len, 0);
    const bool uniform = !__ballot(lane < cnt && len != l0);
    uint64_t P64, tot64;
    if (uniform) {
        P64 = (uint64_t)lane * (pre + l0);
        tot64 = (uint64_t)cnt * (pre + l0);
    } else {
        P64 = wave_excl_scan64(lane < cnt ? pre + len : 0, &tot64);
        tot64 = uni64(tot64);
    }
    if (tot64 + 64 > 4ull * cap) return false;
    R.len = (uint32_t)len;
    R.ulen = uniform && l0 < 0xFFFFFFFFull ? (uint32_t)l0 : ~0u;
    R.P = (uint32_t)P64;
    R.tot = (uint32_t)tot64;'''
assert old in s
s=s.replace(old,new)
open('encode.hip','w').write(s)
