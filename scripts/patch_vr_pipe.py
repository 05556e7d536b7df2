# Patch: sst_vregion_runs_kernel processes VR_P consecutive 64-record chunks per
# wave with the per-chunk setup loads (index -> descriptor -> source prefix)
# software-pipelined three chunks ahead of the copy.
import os, re
P = int(os.environ.get("VR_P", "4"))
s = open('encode.hip').read()
a = s.index('__global__ __launch_bounds__(256) void sst_vregion_runs_kernel(SstArgs a, VViewArgs v) {')
b = s.index('// Header, filter-block prefix and footer of file f')
new = r'''
constexpr uint32_t kVrChunks = VRP;  // 64-record chunks per wave, setup pipelined

struct VrSetup {
    uint32_t idx;
    uint64_t voff;
    u32x4 d;
    uint32_t pre;
};

__global__ __launch_bounds__(256) void sst_vregion_runs_kernel(SstArgs a, VViewArgs v) {
    constexpr uint32_t W = kSstWaves;
    __shared__ uint64_t s_d[W][kWave + 1];
    __shared__ uint64_t s_in[W][kWave];
    __shared__ uint32_t s_fix[W][kWave];
    __shared__ uint32_t s_slow[W][2 * kWave + 4];
    const uint32_t f = blockIdx.x, w = threadIdx.x / kWave, lane = lane_id();
    const SstLayout L = sst_layout(a, f);
    const uint64_t cw = L.s + ((uint64_t)blockIdx.y * W + w) * kWave * kVrChunks;
    if (cw >= L.e) return;
    const uint64_t Vs = uni64(a.voff[L.s]);
    const uint64_t rbase = uni64(a.file_off[f]) + L.data_off - 4 * L.s - Vs;
    const gptr_t<uint8_t> out = gbl(a.out);
    const gptr_t<const uint8_t> vb = gbl(v.bytes);
    auto cnt_of = [&](uint32_t k) -> uint32_t {
        const uint64_t c0 = cw + (uint64_t)k * kWave;
        return c0 >= L.e ? 0u : (uint32_t)((L.e - c0) < (uint64_t)kWave ? (L.e - c0) : kWave);
    };
    // stage loads of chunk k (lanes past the file's end load nothing)
    auto ld_idx = [&](uint32_t k, VrSetup &S) {
        const uint64_t j = cw + (uint64_t)k * kWave + lane;
        if (lane < cnt_of(k)) { S.idx = v.idx[j]; S.voff = a.voff[j]; }
    };
    auto ld_desc = [&](uint32_t k, VrSetup &S) {
        if (lane < cnt_of(k)) S.d = v.vd[S.idx];
    };
    auto ld_pre = [&](uint32_t k, VrSetup &S) {
        if (lane < cnt_of(k)) {
            const uint64_t in0 = (uint64_t)S.d.y << 32 | S.d.x;
            const gptr_t<const uint8_t> pb = vb + in0;
            S.pre = (uint32_t)pb[0] | (uint32_t)pb[1] << 8 | (uint32_t)pb[2] << 16 | (uint32_t)pb[3] << 24;
        }
    };
    VrSetup S0{}, S1{}, S2{};
    ld_idx(0, S0);
    ld_desc(0, S0);
    ld_idx(1, S1);
    ld_pre(0, S0);
    ld_desc(1, S1);
    ld_idx(2, S2);
#pragma unroll 1
    for (uint32_t k = 0; k < kVrChunks; k++) {
        const uint32_t cnt = cnt_of(k);
        if (cnt == 0) break;
        // next stages in flight during this chunk's copy
        VrSetup S3{};
        if (k + 1 < kVrChunks) ld_pre(k + 1, S1);
        if (k + 2 < kVrChunks) ld_desc(k + 2, S2);
        if (k + 3 < kVrChunks) ld_idx(k + 3, S3);
        const uint64_t c0 = cw + (uint64_t)k * kWave;
        uint64_t d0 = 0, in0 = 0, in1 = 0;
        uint32_t vl = 0;
        bool bad = false;
        if (lane < cnt) {
            const uint64_t j = c0 + lane;
            in0 = (uint64_t)S0.d.y << 32 | S0.d.x;
            vl = S0.d.w;
            in1 = in0 + 4 + vl;
            d0 = rbase + 4 * j + S0.voff;
            bad = S0.pre != vl;
        }
        const uint64_t A = lane64(d0, 0);
        // the chunk's end: the next chunk's first value offset, already loaded
        // when that chunk is this wave's
        const bool nx = cnt == kWave && k + 1 < kVrChunks && cnt_of(k + 1) != 0;
        const uint64_t vend = nx ? lane64(S1.voff, 0) : uni64(a.voff[c0 + cnt]);
        const uint64_t B = uni64(rbase + 4 * (c0 + cnt) + vend);
        const uint64_t prev = __shfl_up(in1, 1);
        const bool prev_bad = __shfl_up((uint32_t)bad, 1) != 0;
        const bool brk = lane < cnt && (lane == 0 || prev != in0 || bad || prev_bad);
        const uint64_t bm = __ballot(brk);
        const uint32_t nrun = (uint32_t)__builtin_popcountll(bm);
        vv_sync();  // the previous chunk's readers of the run table are done
        if (brk) {
            const uint32_t q = mbcnt(bm);
            s_d[w][q] = d0 - A;
            s_in[w][q] = in0;
            s_fix[w][q] = bad ? vl + 1 : 0;
        }
        if (lane == 0) s_d[w][nrun] = B - A;
        vv_sync();
        const uint64_t X = A & ~(uint64_t)15;
        const uint32_t nseg = (uint32_t)((B - X + 15) >> 4);
        const uint32_t head = (uint32_t)(A - X);
        const uint64_t tot = B - A;
        auto run_of = [&](uint64_t r) {
            uint32_t lo = 0, hi = nrun;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_d[w][mid] <= r) lo = mid; else hi = mid;
            }
            return lo;
        };
        uint32_t nslow = 0;
        for (uint32_t eb = 0; eb < nseg; eb += kWave * kVrUnroll) {
            u32x4 x0[kVrUnroll], x1[kVrUnroll];
            uint32_t sh[kVrUnroll];
            bool fast[kVrUnroll];
#pragma unroll
            for (uint32_t u = 0; u < kVrUnroll; u++) {
                const uint32_t e = eb + u * kWave + lane;
                const int64_t r0 = 16 * (int64_t)e - (int64_t)head;
                fast[u] = false;
                sh[u] = 0;
                x0[u] = x1[u] = u32x4{0, 0, 0, 0};
                if (e < nseg && r0 >= 0 && r0 + 16 <= (int64_t)tot) {
                    const uint32_t q = run_of((uint64_t)r0);
                    if ((uint64_t)r0 + 16 <= s_d[w][q + 1] && (!s_fix[w][q] || (uint64_t)r0 >= s_d[w][q] + 4)) {
                        const uint64_t src = s_in[w][q] + ((uint64_t)r0 - s_d[w][q]);
                        const uintptr_t sa = reinterpret_cast<uintptr_t>(v.bytes) + (src & ~(uint64_t)3);
                        x0[u] = *gbl_at<const u32x4a>(sa);
                        x1[u].x = *gbl_at<const uint32_t>(sa + 16);
                        sh[u] = (uint32_t)src & 3;
                        fast[u] = true;
                    }
                }
                const uint64_t sm = __ballot(e < nseg && !fast[u]);
                if (e < nseg && !fast[u]) s_slow[w][nslow + mbcnt(sm)] = e;
                nslow += (uint32_t)__builtin_popcountll(sm);
            }
#pragma unroll
            for (uint32_t u = 0; u < kVrUnroll; u++) {
                if (!fast[u]) continue;
                const uint32_t e = eb + u * kWave + lane;
                const uint32_t w0 = x0[u].x, w1 = x0[u].y, w2 = x0[u].z, w3 = x0[u].w, w4 = x1[u].x;
                __builtin_nontemporal_store(
                    u32x4{funnel(w0, w1, sh[u]), funnel(w1, w2, sh[u]), funnel(w2, w3, sh[u]),
                          funnel(w3, w4, sh[u])}, (gptr_t<u32x4>)(out + X + 16 * (uint64_t)e));
            }
        }
        vv_sync();
        for (uint32_t i = lane; i < nslow; i += kWave) {
            const uint32_t e = s_slow[w][i];
            const int64_t r0 = 16 * (int64_t)e - (int64_t)head;
            const bool whole = r0 >= 0 && r0 + 16 <= (int64_t)tot;
            uint64_t src[16];
            uint32_t fixb = 0, inr = 0;
            uint32_t pre[4] = {0, 0, 0, 0};
            uint32_t q = run_of(r0 > 0 ? (uint64_t)r0 : 0);
#pragma unroll
            for (uint32_t b = 0; b < 16; b++) {
                const int64_t r = r0 + b;
                src[b] = s_in[w][q];
                if (r < 0 || r >= (int64_t)tot) continue;
                inr |= 1u << b;
                while ((uint64_t)r >= s_d[w][q + 1]) q++;
                const uint64_t t = (uint64_t)r - s_d[w][q];
                const uint32_t fx = s_fix[w][q];
                src[b] = s_in[w][q] + t;
                if (fx && t < 4) {
                    fixb |= 1u << b;
                    pre[b >> 2] |= (((fx - 1) >> (8 * t)) & 0xFFu) << (8 * (b & 3));
                }
            }
            uint32_t by[16];
#pragma unroll
            for (uint32_t b = 0; b < 16; b++) by[b] = vb[src[b]];
            uint32_t wd[4] = {pre[0], pre[1], pre[2], pre[3]};
#pragma unroll
            for (uint32_t b = 0; b < 16; b++)
                if (!((fixb >> b) & 1)) wd[b >> 2] |= by[b] << (8 * (b & 3));
            if (whole) {
                *(gptr_t<u32x4>)(out + X + 16 * (uint64_t)e) = u32x4{wd[0], wd[1], wd[2], wd[3]};
            } else {
#pragma unroll
                for (uint32_t b = 0; b < 16; b++)
                    if ((inr >> b) & 1) out[X + 16 * (uint64_t)e + b] = (uint8_t)(wd[b >> 2] >> (8 * (b & 3)));
            }
        }
        S0 = S1;
        S1 = S2;
        S2 = S3;
    }
}

'''.replace('VRP', str(P))
s = s[:a] + new + s[b:]
# grid: chunks of 256 records -> of 256 * P records
s = s.replace('''                hipLaunchKernelGGL(sst_vregion_runs_kernel, dim3(nfile, chunks), dim3(256), 0, vs, a,''',
              '''                hipLaunchKernelGGL(sst_vregion_runs_kernel, dim3(nfile, (chunks + kVrChunks - 1) / kVrChunks), dim3(256), 0, vs, a,''')
assert 'kVrChunks - 1) / kVrChunks' in s
open('encode.hip', 'w').write(s)
