// Token GEMM (nn.Linear over token rows) and weight-gradient GEMM, fp32 MFMA 16x16x4.
//
// mep_gemm : Y[tok, n] = act(alpha * X[tok,:] . W(n,:) + bias[n] + table[tok % T, n]) (+Y)
//            one workgroup = 64 tokens x all N columns; 8 waves; task (m-half, 32-col block)
//            round-robin over waves; A staged through LDS in 128-wide K chunks, W read from
//            L2 with 16-byte loads.  Replaces Unify_Dimension's Linear (cmu-mosei/run.py:210-214),
//            the Conv1d k=1 unify + position add (others/realformer.py:136-152,224-227) and the
//            realformer w_qkv / FFN Linears (others/realformer.py:157,163-168).
// mep_wgrad: dW_i = A^T B_i over token chunks (see the kernel comment below).
#include "common.h"

using namespace mep;

namespace {

// One WAVE = 16 tokens x (up to 128 columns per pass); 4 independent waves per workgroup of 64
// tokens, no block barriers.  v_mfma_f32_16x16x4_f32 with the wave's A rows staged in its own LDS
// slice (128-wide K chunks, zero-padded past K and past the last token) and the weight fragments
// of the next 16-wide k block loaded during the MFMAs of the current one.  Per lane: acc[j] holds
// rows 4g..4g+3 of column block j (c = lane & 15, g = lane >> 4; common.h wgemm16 layout).
constexpr int GEMM_WAVES = 4;
constexpr int GEMM_THREADS = 64 * GEMM_WAVES;
constexpr int GEMM_KC = 128;
constexpr int GEMM_LDA = GEMM_KC + 4;
constexpr int GEMM_NJ = 8;        // 16-column blocks per pass

// weight fragment W(n, k .. k+3) with k clamped into [0, K) and n into [0, N): the clamped
// values meet zero A columns (k >= K) or are never stored (n >= N), so they only need to be finite
MEP_DEV float4 gemm_wfrag(const gfloat* W, int ldw, bool nt, bool vec, int n, int N, int k, int K) {
    n = min(n, N - 1);
    if (nt) {
        const gfloat* p = W + (int64_t)n * ldw;
        if (vec && k + 3 < K) return ldg4(p + k);
        return make_float4(p[min(k, K - 1)], p[min(k + 1, K - 1)], p[min(k + 2, K - 1)], p[min(k + 3, K - 1)]);
    }
    const gfloat* p = W + n;
    return make_float4(p[(int64_t)min(k, K - 1) * ldw], p[(int64_t)min(k + 1, K - 1) * ldw],
                       p[(int64_t)min(k + 2, K - 1) * ldw], p[(int64_t)min(k + 3, K - 1) * ldw]);
}

__global__ __launch_bounds__(GEMM_THREADS) void k_gemm(const mep_gemm_desc* __restrict__ descs) {
    const mep_gemm_desc& d = descs[blockIdx.y];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int r0 = blockIdx.x * 64 + wave * 16;
    if (r0 >= d.ntok) return;   // whole wave; only wave-private LDS below
    __shared__ __attribute__((aligned(16))) float smem[GEMM_WAVES][16 * GEMM_LDA];
    float* As = smem[wave];
    const int K = d.K, N = d.N, ntok = d.ntok;
    const gfloat* W = G<const float>(d.w);
    const bool w_nt = d.w_nt;
    const bool w_vec = w_nt && (d.ldw % 4 == 0) && ((d.w & 15) == 0);
    const bool x_vec = (K % 4 == 0) && ((d.x.ptr & 15) == 0) && (d.x.sB % 4 == 0) && (d.x.sT % 4 == 0);
    const gfloat* bias = G<const float>(d.bias);
    const gfloat* table = G<const float>(d.table);
    // per-lane row offsets of the staging pattern (row = idx / 32 for float4 idx = lane + 64 i)
    const float* arow = As + c * GEMM_LDA + 4 * g;

    for (int cg = 0; cg < N; cg += 16 * GEMM_NJ) {
        const int nj = min(GEMM_NJ, (N - cg + 15) / 16);
        f32x4 acc[GEMM_NJ];
#pragma unroll
        for (int j = 0; j < GEMM_NJ; ++j) acc[j] = zero_f4();
        for (int k0 = 0; k0 < K; k0 += GEMM_KC) {
            const int kc = min(GEMM_KC, K - k0);
            const int kcp = (kc + 15) & ~15;
            // stage A rows [r0, r0+16) x cols [k0, k0 + kcp): zero past K / past ntok
            if (x_vec) {
                const int v4 = kcp >> 2;
                for (int idx = lane; idx < 16 * v4; idx += 64) {
                    const int row = idx / v4, c4 = 4 * (idx - row * v4);
                    const int tok = r0 + row;
                    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (tok < ntok && c4 < kc) v = ldg4(row_ptr(d.x, tok) + k0 + c4);
                    *reinterpret_cast<float4*>(As + row * GEMM_LDA + c4) = v;
                }
            } else {
                for (int idx = lane; idx < 16 * kcp; idx += 64) {
                    const int row = idx / kcp, cc = idx - row * kcp;
                    const int tok = r0 + row;
                    float v = 0.f;
                    if (tok < ntok && cc < kc) v = row_ptr(d.x, tok)[k0 + cc];
                    As[row * GEMM_LDA + cc] = v;
                }
            }
            wave_lds_fence();
            const int nkb = kcp >> 4;
            float4 b[GEMM_NJ];
#pragma unroll
            for (int j = 0; j < GEMM_NJ; ++j)
                if (j < nj) b[j] = gemm_wfrag(W, d.ldw, w_nt, w_vec, cg + 16 * j + c, N, k0 + 4 * g, K);
            for (int kb = 0; kb < nkb; ++kb) {
                float4 cur[GEMM_NJ];
#pragma unroll
                for (int j = 0; j < GEMM_NJ; ++j) cur[j] = b[j];
                if (kb + 1 < nkb) {
#pragma unroll
                    for (int j = 0; j < GEMM_NJ; ++j)
                        if (j < nj) b[j] = gemm_wfrag(W, d.ldw, w_nt, w_vec, cg + 16 * j + c, N, k0 + 16 * (kb + 1) + 4 * g, K);
                }
                const float4 a = *reinterpret_cast<const float4*>(arow + 16 * kb);
#pragma unroll
                for (int j = 0; j < GEMM_NJ; ++j)
                    if (j < nj) {
                        acc[j] = mfma16x4(a.x, cur[j].x, acc[j]);
                        acc[j] = mfma16x4(a.y, cur[j].y, acc[j]);
                        acc[j] = mfma16x4(a.z, cur[j].z, acc[j]);
                        acc[j] = mfma16x4(a.w, cur[j].w, acc[j]);
                    }
            }
            wave_lds_fence();   // every lane is done reading this chunk
        }
        // epilogue: rows 4g + r, column cg + 16 j + c
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int tok = r0 + 4 * g + r;
            if (tok >= ntok) continue;
            gfloat* yrow = row_ptr(d.y, tok);
            const gfloat* trow = table ? table + (int64_t)(tok % d.y.T) * N : nullptr;
#pragma unroll
            for (int j = 0; j < GEMM_NJ; ++j) {
                const int col = cg + 16 * j + c;
                if (j >= nj || col >= N) continue;
                float v = d.alpha * acc[j][r];
                if (bias) v += bias[col];
                if (trow) v += trow[col];
                if (d.relu) v = fmaxf(v, 0.f);
                if (d.accumulate) v += yrow[col];
                yrow[col] = v;
            }
        }
    }
}

// ---------------------------------------------------------------- weight gradient
// dW[n][k] = sum_t A[t][n] B[t][k] on f32 MFMA 16x16x4 with the token axis as the MFMA k.
// One workgroup = (chunk of tok_per_split tokens, group of <= 256 columns of the concatenated K);
// its 8 waves form a 2 x 4 grid over the (N/16) x (kcnt/16) output tiles, each wave a rectangle
// of <= 4 x 4 tiles so A fragments are reused across its k tiles and B fragments across its n
// tiles.  Per 32-token step both operands are staged TRANSPOSED (feature-major) in LDS,
// double-buffered, with the next step's global loads in flight during the current step's MFMAs:
// a thread gathers 8 consecutive tokens of one feature (coalesced across the lanes' features)
// and writes them as two 16-byte LDS stores; a fragment (4 tokens of one feature) is then one
// 16-byte LDS read.
constexpr int WG_THREADS = 512;
constexpr int WG_TT = 32;                      // tokens per step
constexpr int WG_KG = 256;                     // max columns per workgroup
constexpr int WG_NMAX = 128;
constexpr int WG_LD = WG_TT + 4;               // row stride (floats): 16-row fragment reads conflict-free
constexpr int WG_ROWS = WG_NMAX + WG_KG;       // A feature rows, then B column rows
constexpr int WG_STAGE = WG_ROWS * WG_LD;      // floats per stage buffer
constexpr int WG_IPT = (WG_ROWS * (WG_TT / 8) + WG_THREADS - 1) / WG_THREADS;   // items per thread

struct WgItem {        // one (feature row, 8-token group) staging item of a thread
    uint64_t ptr;      // column base (row view ptr + column offset), 0 = none
    int64_t sB, sT;
    int T, lrow, tg;
};

MEP_DEV void wg_load(float (&v)[WG_IPT][8], const WgItem (&it)[WG_IPT], int t0, int t_end) {
#pragma unroll
    for (int m = 0; m < WG_IPT; ++m) {
        const mep_rows r{it[m].ptr, it[m].sB, it[m].sT, it[m].T, 0};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int tok = t0 + 8 * it[m].tg + j;
            v[m][j] = (it[m].ptr && tok < t_end) ? *(G<const float>(r.ptr) + row_off(r, tok)) : 0.f;
        }
    }
}

MEP_DEV void wg_store(lfloat* st, const float (&v)[WG_IPT][8], const WgItem (&it)[WG_IPT]) {
#pragma unroll
    for (int m = 0; m < WG_IPT; ++m) {
        if (!it[m].ptr) continue;
        lfloat* q = st + it[m].lrow * WG_LD + 8 * it[m].tg;
        *reinterpret_cast<lf32x4*>(q) = f32x4{v[m][0], v[m][1], v[m][2], v[m][3]};
        *reinterpret_cast<lf32x4*>(q + 4) = f32x4{v[m][4], v[m][5], v[m][6], v[m][7]};
    }
}

__global__ __launch_bounds__(WG_THREADS) void k_wgrad(const mep_wgrad_desc* __restrict__ descs) {
    const mep_wgrad_desc& d = descs[blockIdx.y];
    const int nkg = (d.Ktot + WG_KG - 1) / WG_KG;
    if ((int)blockIdx.x >= d.n_split * nkg) return;
    const int split = blockIdx.x / nkg, kg = blockIdx.x - split * nkg;
    const int t_begin = split * d.tok_per_split;
    const int t_end = min(d.ntok, t_begin + d.tok_per_split);
    const int kbase = kg * WG_KG, kcnt = min(WG_KG, d.Ktot - kbase);
    const int N = d.N;
    __shared__ __attribute__((aligned(16))) float smem[2 * WG_STAGE];
    lfloat* const stage0 = (lfloat*)&smem[0];   // buffer b at stage0 + b * WG_STAGE

    // staging items of this thread: row f of the (N + kcnt) feature rows, token group tg
    const int nrows = N + kcnt;
    WgItem it[WG_IPT];
#pragma unroll
    for (int m = 0; m < WG_IPT; ++m) {
        const int idx = threadIdx.x + WG_THREADS * m;
        const int tg = idx / nrows, f = idx - tg * nrows;
        it[m] = WgItem{0, 0, 0, 1, 0, 0};
        if (tg < WG_TT / 8) {
            if (f < N) {
                it[m] = WgItem{d.a.ptr + 4ull * f, d.a.sB, d.a.sT, d.a.T, f, tg};
            } else {
                int k = kbase + (f - N), i = 0;
                while (i < d.n_b - 1 && k >= d.kb[i]) { k -= d.kb[i]; ++i; }
                const mep_rows& b = d.b[i];
                it[m] = WgItem{b.ptr + 4ull * k, b.sB, b.sT, b.T, WG_NMAX + (f - N), tg};
            }
        }
    }

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int ntn = (N + 15) >> 4, ntk = (kcnt + 15) >> 4;
    const int wn = wave >> 2, wk = wave & 3;
    const int pn = (ntn + 1) >> 1, pk = (ntk + 3) >> 2;          // tiles per wave (<= 4 each)
    const int tn0 = wn * pn, tk0 = wk * pk;
    const int nn = max(0, min(pn, ntn - tn0)), nk = max(0, min(pk, ntk - tk0));
    f32x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = zero_f4();

    float pre[WG_IPT][8];
    wg_load(pre, it, t_begin, t_end);
    wg_store(stage0, pre, it);
    __syncthreads();
    int cur = 0;
    for (int t0 = t_begin; t0 < t_end; t0 += WG_TT) {
        const bool more = t0 + WG_TT < t_end;
        if (more) wg_load(pre, it, t0 + WG_TT, t_end);
        const lfloat* st = stage0 + cur * WG_STAGE;
#pragma unroll
        for (int kb = 0; kb < WG_TT / 16; ++kb) {
            f32x4 af[4], bf[4];
#pragma unroll
            for (int a = 0; a < 4; ++a)
                if (a < nn) af[a] = ld4w(st + (16 * (tn0 + a) + c) * WG_LD + 16 * kb + 4 * g);
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (b < nk) bf[b] = ld4w(st + (WG_NMAX + 16 * (tk0 + b) + c) * WG_LD + 16 * kb + 4 * g);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        if (a < nn && b < nk)
                            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[a][s], bf[b][s], acc[a][b], 0, 0, 0);
        }
        if (more) wg_store(stage0 + (cur ^ 1) * WG_STAGE, pre, it);
        __syncthreads();
        cur ^= 1;
    }
    // partial[split][n][kbase + k]: lane (c, g) holds rows n = 4g + r, column k = c of each tile
    gfloat* part = G<float>(d.partial) + (int64_t)split * N * d.Ktot;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            if (a >= nn || b >= nk) continue;
            const int k = 16 * (tk0 + b) + c;
            if (k >= kcnt) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = 16 * (tn0 + a) + 4 * g + r;
                if (n < N) part[(int64_t)n * d.Ktot + kbase + k] = acc[a][b][r];
            }
        }
}

__global__ __launch_bounds__(256) void k_wgrad_reduce(const mep_wgrad_desc* __restrict__ descs) {
    const mep_wgrad_desc& d = descs[blockIdx.y];
    const int64_t nk = (int64_t)d.N * d.Ktot;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nk) return;
    const gfloat* part = G<const float>(d.partial);
    float s = 0.f;
    for (int sp = 0; sp < d.n_split; ++sp) s += part[sp * nk + i];
    const int n = (int)(i / d.Ktot);
    int k = (int)(i - (int64_t)n * d.Ktot);
    int j = 0;
    while (j < d.n_b - 1 && k >= d.kb[j]) { k -= d.kb[j]; ++j; }
    gfloat* o = G<float>(d.out[j]) + (d.out_trans ? (int64_t)k * d.ldo[j] + n : (int64_t)n * d.ldo[j] + k);
    *o = d.accumulate ? *o + s : s;
}

}  // namespace

extern "C" int mep_gemm(const mep_gemm_desc* descs, int n_desc, int max_tiles, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    hipLaunchKernelGGL(k_gemm, dim3(max_tiles, n_desc), dim3(GEMM_THREADS), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_gemm");
}

extern "C" int mep_wgrad(const mep_wgrad_desc* descs, int n_desc, int max_tiles, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    hipLaunchKernelGGL(k_wgrad, dim3(max_tiles, n_desc), dim3(WG_THREADS), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_wgrad");
}

extern "C" int mep_wgrad_reduce(const mep_wgrad_desc* descs, int n_desc, int max_tiles, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    hipLaunchKernelGGL(k_wgrad_reduce, dim3(max_tiles, n_desc), dim3(256), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_wgrad_reduce");
}
