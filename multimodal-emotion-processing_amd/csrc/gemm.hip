// Token GEMM (nn.Linear over token rows) and weight-gradient GEMM, fp32 MFMA 32x32x2.
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

constexpr int GEMM_THREADS = 512;
constexpr int GEMM_KC = 128;
constexpr int GEMM_LDA = GEMM_KC + 4;
constexpr int GEMM_MAX_TASKS = 2;  // per wave and column group of 256

__global__ __launch_bounds__(GEMM_THREADS) void k_gemm(const mep_gemm_desc* __restrict__ descs) {
    const mep_gemm_desc& d = descs[blockIdx.y];
    const int tok0 = blockIdx.x * 64;
    if (tok0 >= d.ntok) return;
    __shared__ __attribute__((aligned(16))) float As[64 * GEMM_LDA];

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const gfloat* W = G<const float>(d.w);
    const bool w_vec = d.w_nt && (d.ldw % 4 == 0) && ((d.w & 15) == 0);
    const gfloat* bias = G<const float>(d.bias);
    const gfloat* table = G<const float>(d.table);

    // column groups of 256 (8 waves x 2 tasks x 32 cols / 2 m-halves); A is re-staged per group
    for (int cg = 0; cg < d.N; cg += 256) {
        const int ncg = min(256, d.N - cg);
        const int ntask = 2 * ((ncg + 31) / 32);
        floatx16 acc[GEMM_MAX_TASKS];
#pragma unroll
        for (int t = 0; t < GEMM_MAX_TASKS; ++t) acc[t] = zero16();

        for (int k0 = 0; k0 < d.K; k0 += GEMM_KC) {
            const int kc = min(GEMM_KC, d.K - k0);
            const int kc_pad = (kc + 7) & ~7;
            __syncthreads();
            load_tile(As, GEMM_LDA, d.x, tok0, d.ntok, k0, kc, kc_pad, d.K);
            __syncthreads();
#pragma unroll
            for (int t = 0; t < GEMM_MAX_TASKS; ++t) {
                const int task = wave + 8 * t;
                if (task < ntask) {
                    const int mh = task & 1, n0 = cg + (task >> 1) * 32;
                    if (kc_pad == GEMM_KC) {   // full chunk: unrolled, weight loads issued up front
                        if (d.w_nt)
                            mma_tile<true, GEMM_KC>(acc[t], As, GEMM_LDA, mh * 32, W, d.ldw, n0, d.N, k0, kc_pad, d.K, w_vec);
                        else
                            mma_tile<false, GEMM_KC>(acc[t], As, GEMM_LDA, mh * 32, W, d.ldw, n0, d.N, k0, kc_pad, d.K, false);
                    } else if (d.w_nt) {
                        mma_tile<true>(acc[t], As, GEMM_LDA, mh * 32, W, d.ldw, n0, d.N, k0, kc_pad, d.K, w_vec);
                    } else {
                        mma_tile<false>(acc[t], As, GEMM_LDA, mh * 32, W, d.ldw, n0, d.N, k0, kc_pad, d.K, false);
                    }
                }
            }
        }
#pragma unroll
        for (int t = 0; t < GEMM_MAX_TASKS; ++t) {
            const int task = wave + 8 * t;
            if (task >= ntask) continue;
            const int mh = task & 1;
            const int col = cg + (task >> 1) * 32 + (lane & 31);
            if (col >= d.N) continue;
            const float bcol = bias ? bias[col] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int tok = tok0 + mh * 32 + acc_row(r, lane);
                if (tok >= d.ntok) continue;
                float v = d.alpha * acc[t][r];
                if (bias) v += bcol;
                if (table) v += table[(tok % d.y.T) * d.N + col];
                if (d.relu) v = fmaxf(v, 0.f);
                gfloat* yp = row_ptr(d.y, tok) + col;
                if (d.accumulate) v += *yp;
                *yp = v;
            }
        }
    }
}

// ---------------------------------------------------------------- weight gradient
// One workgroup = (token chunk, 256-column group of the concatenated K).  It stages 32 tokens of
// A [32 x N] and of the B operands [32 x 256] in LDS per step and accumulates the whole
// N x 256 partial (<= 4 x 8 tiles of 32x32, <= 4 per wave) with f32 MFMA, so every input
// element is read from HBM once per column group.
constexpr int WG_THREADS = 512;
constexpr int WG_TT = 32;
constexpr int WG_KG = 256;
constexpr int WG_NMAX = 128;
constexpr int WG_MAXT = 4;

MEP_DEV int wg_koff(const mep_wgrad_desc& d, int i) {
    int o = 0;
    for (int j = 0; j < i; ++j) o += d.kb[j];
    return o;
}

__global__ __launch_bounds__(WG_THREADS) void k_wgrad(const mep_wgrad_desc* __restrict__ descs) {
    const mep_wgrad_desc& d = descs[blockIdx.y];
    const int nkg = (d.Ktot + WG_KG - 1) / WG_KG;
    if ((int)blockIdx.x >= d.n_split * nkg) return;
    const int split = blockIdx.x / nkg, kg = blockIdx.x - (blockIdx.x / nkg) * nkg;
    const int t_begin = split * d.tok_per_split;
    const int t_end = min(d.ntok, t_begin + d.tok_per_split);
    const int kbase = kg * WG_KG, kcnt = min(WG_KG, d.Ktot - kbase);
    const int ntn = (d.N + 31) / 32, ntk = (kcnt + 31) / 32, ntask = ntn * ntk;

    __shared__ __attribute__((aligned(16))) float As[WG_TT * WG_NMAX];
    __shared__ __attribute__((aligned(16))) float Bs[WG_TT * WG_KG];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int h = lane >> 5, r = lane & 31;
    floatx16 acc[WG_MAXT];
#pragma unroll
    for (int t = 0; t < WG_MAXT; ++t) acc[t] = zero16();

    for (int t0 = t_begin; t0 < t_end; t0 += WG_TT) {
        __syncthreads();
        stage_cols<WG_TT>(As, WG_NMAX, d.a, t0, t_end, 0, d.N);
        int koff = 0;
        for (int i = 0; i < d.n_b; ++i) {
            const int lo = max(koff, kbase), hi = min(koff + d.kb[i], kbase + kcnt);
            if (hi > lo) stage_cols<WG_TT>(Bs + (lo - kbase), WG_KG, d.b[i], t0, t_end, lo - koff, hi - lo);
            koff += d.kb[i];
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < WG_MAXT; ++t) {
            const int task = wave + 8 * t;
            if (task < ntask) {
                const int tn = task % ntn, tk = task / ntn;
                const float* ap = As + tn * 32 + r + h * WG_NMAX;
                const float* bp = Bs + tk * 32 + r + h * WG_KG;
#pragma unroll 8
                for (int st = 0; st < WG_TT / 2; ++st)
                    acc[t] = mfma32(ap[2 * st * WG_NMAX], bp[2 * st * WG_KG], acc[t]);
            }
        }
    }
    gfloat* part = G<float>(d.partial) + (int64_t)split * d.N * d.Ktot;
#pragma unroll
    for (int t = 0; t < WG_MAXT; ++t) {
        const int task = wave + 8 * t;
        if (task >= ntask) continue;
        const int tn = task % ntn, tk = task / ntn;
        const int kcol = tk * 32 + (lane & 31);
        if (kcol >= kcnt) continue;
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
            const int n = tn * 32 + acc_row(rr, lane);
            if (n < d.N) part[(int64_t)n * d.Ktot + kbase + kcol] = acc[t][rr];
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
