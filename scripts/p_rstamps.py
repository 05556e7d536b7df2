# build_variant.sh patch: s_memrealtime stamps per region wave
# {start, V landed, V stored, IDX landed, end} into g_rstamps (diagnostics only).
s = open('encode.hip').read()
s = s.replace('namespace lsm {\nnamespace {\n', '''__device__ unsigned long long *g_rstamps;
__device__ __forceinline__ void rstamp(unsigned k) {
    if (g_rstamps && (threadIdx.x & 63) == 0)
        g_rstamps[((blockIdx.y * gridDim.x + blockIdx.x) * 4 + threadIdx.x / 64) * 8 + k] =
            __builtin_amdgcn_s_memrealtime();
}
namespace lsm {
namespace {
''', 1)
old = '''    __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");

    // fixed fields of this lane's record'''
assert old in s
s = s.replace(old, '''    __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
    rstamp(G == LSM_GRAMMAR_V ? 1 : 3);

    // fixed fields of this lane's record''')
old = '''    const uint32_t f = blockIdx.x;
    const SstLayout L = sst_layout(a, f);
    const uint32_t wave = uni(threadIdx.x / kWave);
    const uint64_t c0 = L.s + (uint64_t)blockIdx.y * kRegChunkRecs + (uint64_t)wave * kRegWaveRecs;'''
assert old in s
s = s.replace(old, '''    rstamp(0);
    const uint32_t f = blockIdx.x;
    const SstLayout L = sst_layout(a, f);
    const uint32_t wave = uni(threadIdx.x / kWave);
    const uint64_t c0 = L.s + (uint64_t)blockIdx.y * kRegChunkRecs + (uint64_t)wave * kRegWaveRecs;''')
old = '''            &lds[wave].ct);
    encode_chunk_any<LSM_GRAMMAR_IDX, kRegGatherDwords>(
        S, c0, cnt, img + L.idx_off + 12 * (c0 - L.s) + (Kc - Ks), lds[wave].gather, nullptr,
        &lds[wave].ct);'''
assert old in s
s = s.replace(old, '''            &lds[wave].ct);
    rstamp(2);
    encode_chunk_any<LSM_GRAMMAR_IDX, kRegGatherDwords>(
        S, c0, cnt, img + L.idx_off + 12 * (c0 - L.s) + (Kc - Ks), lds[wave].gather, nullptr,
        &lds[wave].ct);
    __asm__ __volatile__("s_waitcnt vmcnt(0)" ::: "memory");
    rstamp(4);''')
s += '''
extern "C" int lsm_debug_set_rstamps(void *d_buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_rstamps), &d_buf, sizeof(void *)) == hipSuccess ? 0 : -1;
}
'''
open('encode.hip', 'w').write(s)
