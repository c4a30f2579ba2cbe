// Token GEMM (nn.Linear over token rows) and weight-gradient GEMM, fp32 MFMA 32x32x2.
//
// mep_gemm : Y[tok, n] = act(alpha * X[tok,:] . W(n,:) + bias[n] + table[tok % T, n]) (+Y)
//            one workgroup = 64 tokens x all N columns; 8 waves; task (m-half, 32-col block)
//            round-robin over waves; A staged through LDS in 128-wide K chunks, W read from
//            L2 with 16-byte loads.  Replaces Unify_Dimension's Linear (cmu-mosei/run.py:210-214),
//            the Conv1d k=1 unify + position add (others/realformer.py:136-152,224-227) and the
//            realformer w_qkv / FFN Linears (others/realformer.py:157,163-168).
// mep_wgrad: partial[split][n][k] = sum_{tok in split} A[tok,n] B[tok,k]; workgroup tile
//            64 x 64 (4 waves of 32x32), tokens streamed through LDS 32 at a time.
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
    const float* W = reinterpret_cast<const float*>(d.w);
    const bool w_vec = d.w_nt && (d.ldw % 4 == 0) && ((d.w & 15) == 0);
    const float* bias = reinterpret_cast<const float*>(d.bias);
    const float* table = reinterpret_cast<const float*>(d.table);

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
                    if (d.w_nt)
                        mma_tile<true>(acc[t], As, GEMM_LDA, mh * 32, W, d.ldw, n0, d.N, k0, kc_pad, d.K, w_vec);
                    else
                        mma_tile<false>(acc[t], As, GEMM_LDA, mh * 32, W, d.ldw, n0, d.N, k0, kc_pad, d.K, false);
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
                float* yp = row_ptr(d.y, tok) + col;
                if (d.accumulate) v += *yp;
                *yp = v;
            }
        }
    }
}

// ---------------------------------------------------------------- weight gradient
constexpr int WG_THREADS = 256;
constexpr int WG_TT = 32;          // tokens per LDS stage
constexpr int WG_LD = 64 + 4;

__global__ __launch_bounds__(WG_THREADS) void k_wgrad(const mep_wgrad_desc* __restrict__ descs) {
    const mep_wgrad_desc& d = descs[blockIdx.y];
    const int ntn = (d.N + 63) / 64, ntk = (d.K + 63) / 64;
    const int tiles = ntn * ntk * d.n_split;
    if ((int)blockIdx.x >= tiles) return;
    const int split = blockIdx.x / (ntn * ntk);
    const int rem = blockIdx.x - split * ntn * ntk;
    const int tn = rem / ntk, tk = rem - (rem / ntk) * ntk;
    const int n0 = tn * 64, kq0 = tk * 64;
    const int t_begin = split * d.tok_per_split;
    const int t_end = min(d.ntok, t_begin + d.tok_per_split);

    __shared__ __attribute__((aligned(16))) float As[WG_TT * WG_LD];
    __shared__ __attribute__((aligned(16))) float Bs[WG_TT * WG_LD];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wm = wave & 1, wn = wave >> 1;
    floatx16 acc = zero16();
    for (int t0 = t_begin; t0 < t_end; t0 += WG_TT) {
        __syncthreads();
        for (int idx = threadIdx.x; idx < WG_TT * 64; idx += WG_THREADS) {
            const int row = idx >> 6, col = idx & 63;
            const int tok = t0 + row;
            float av = 0.f, bv = 0.f;
            if (tok < t_end) {
                if (n0 + col < d.N) av = row_ptr(d.a, tok)[n0 + col];
                if (kq0 + col < d.K) bv = row_ptr(d.b, tok)[kq0 + col];
            }
            As[row * WG_LD + col] = av;
            Bs[row * WG_LD + col] = bv;
        }
        __syncthreads();
        const int h = lane >> 5, r = lane & 31;
#pragma unroll 4
        for (int s = 0; s < WG_TT / 2; ++s) {
            const int tr = 2 * s + h;
            acc = mfma32(As[tr * WG_LD + wm * 32 + r], Bs[tr * WG_LD + wn * 32 + r], acc);
        }
    }
    float* part = reinterpret_cast<float*>(d.partial) + (int64_t)split * d.N * d.K;
    const int kcol = kq0 + wn * 32 + (lane & 31);
    if (kcol < d.K) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int n = n0 + wm * 32 + acc_row(r, lane);
            if (n < d.N) part[(int64_t)n * d.K + kcol] = acc[r];
        }
    }
}

__global__ void k_wgrad_reduce(const mep_wgrad_desc* __restrict__ descs) {
    const mep_wgrad_desc& d = descs[blockIdx.y];
    const int64_t nk = (int64_t)d.N * d.K;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nk) return;
    const float* part = reinterpret_cast<const float*>(d.partial);
    float s = 0.f;
    for (int sp = 0; sp < d.n_split; ++sp) s += part[sp * nk + i];
    const int n = (int)(i / d.K), k = (int)(i - (int64_t)n * d.K);
    float* o = reinterpret_cast<float*>(d.out) + (int64_t)n * d.ldo + k;
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
