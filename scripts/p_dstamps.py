# build_variant.sh patch: per-iteration stamps in the pipelined region kernel
# {top, issued, landed, finished} x 4 chunks (diagnostics only).
s = open('encode.hip').read()
s = s.replace('namespace lsm {\nnamespace {\n', '''__device__ unsigned long long *g_rstamps;
__device__ __forceinline__ void rstamp(unsigned k) {
    if (g_rstamps && (threadIdx.x & 63) == 0 && k < 16)
        g_rstamps[((blockIdx.y * gridDim.x + blockIdx.x) * 2 + threadIdx.x / 64) * 16 + k] =
            __builtin_amdgcn_s_memrealtime();
}
namespace lsm {
namespace {
''', 1)
rep = [("""    ChunkOffs off = load_offs(a, c0, count(c0));
    for (;;) {""", """    ChunkOffs off = load_offs(a, c0, count(c0));
    uint32_t it = 0;
    for (;;) {
        rstamp(4 * it);"""),
("""            const ChunkOffs nxt = more ? load_offs(a, cn, count(cn)) : off;""",
 """            rstamp(4 * it + 1);
            const ChunkOffs nxt = more ? load_offs(a, cn, count(cn)) : off;"""),
("""            __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
            if (!a.skip_v) region_finish<LSM_GRAMMAR_V>(pv, buf);
            region_finish<LSM_GRAMMAR_IDX>(pi, buf);""",
 """            __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
            rstamp(4 * it + 2);
            if (!a.skip_v) region_finish<LSM_GRAMMAR_V>(pv, buf);
            region_finish<LSM_GRAMMAR_IDX>(pi, buf);
            rstamp(4 * it + 3);"""),
("""        if (!more) break;
        c0 = cn;""", """        if (!more) break;
        c0 = cn;
        it++;""")]
for o, n in rep:
    assert o in s, o
    s = s.replace(o, n)
s += '''
extern "C" int lsm_debug_set_rstamps(void *d_buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_rstamps), &d_buf, sizeof(void *)) == hipSuccess ? 0 : -1;
}
'''
open('encode.hip', 'w').write(s)
