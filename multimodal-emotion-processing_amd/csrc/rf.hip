// others/realformer.py: RealFormer block epilogue (forward + backward) and the State_Transfer
// head (fused LayerNorm / classifier / sigmoid-tanh gate recurrence / circle loss, + backward).
//
// Block epilogue (realformer.py:203-209, after the attention core):
//   xp = x Wp^T;  h = LN1(q + a*xp);  f1 = relu(h W1^T + b1);  f = f1 W2^T + b2;  out = LN2(h + b*f)
// One workgroup = 64 tokens, 8 waves.  Each Linear is a chain of f32 MFMA 32x32x2 tasks
// (32 tokens x 32 output columns) over an LDS-resident A tile with the weights streamed from
// L2; the intermediate activations never round-trip through HBM inside the kernel (they are
// written once, for the backward's weight gradients).  LayerNorms are wave-per-row shuffle
// reductions.  D and FD are template parameters so every K loop is fully unrolled.
#include "common.h"
#include "split.h"

using namespace mep;


namespace {

constexpr int THREADS = 512;
constexpr int NWAVE = THREADS / 64;
constexpr float LN_EPS = 1e-5f;

MEP_DEV bool wvec(uint64_t p, int ld) { return ((p & 15) == 0) && (ld % 4 == 0); }

// C[64 x N] = A_lds[64 x K] . W  (NT: W[n*ldw + k], else W[k*ldw + n]); epi(row, col, value)
// for every element of the tile.  Tasks (m-half, 32-column block) round-robin over the waves.
template <int N, int K, bool NT, int MH = 2, typename Epi>
MEP_DEV void tile_gemm(const float* As, int lda, const gfloat* W, int ldw, bool w_vec, Epi&& epi) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int NTASK = MH * ((N + 31) / 32);   // MH 32-row halves of the token tile
    for (int t = wave; t < NTASK; t += NWAVE) {
        const int mh = t % MH, nblk = t / MH;
        floatx16 acc = zero16();
        if constexpr (K <= 128) {
            mma_tile_pf<NT, K>(acc, As, lda, mh * 32, W, ldw, nblk * 32, N, 0, K, w_vec);
        } else {   // two halves: at most 64 prefetch registers per pass
            mma_tile_pf<NT, K / 2>(acc, As, lda, mh * 32, W, ldw, nblk * 32, N, 0, K, w_vec);
            mma_tile_pf<NT, K / 2>(acc, As + K / 2, lda, mh * 32, W, ldw, nblk * 32, N, K / 2, K, w_vec);
        }
        const int col = nblk * 32 + (lane & 31);
        if (col < N) {
#pragma unroll
            for (int r = 0; r < 16; ++r) epi(mh * 32 + acc_row(r, lane), col, acc[r]);
        }
    }
}

// Token rows per workgroup of the forward: 32 (MEP_RF_FWD_ROWS; 64 halves the workgroup count --
// 50 per block at cfg2 -- and measured slower), and 32 always for D = 192 (robot_demo.py,
// inference) so the LDS tiles (x/h, xp/f, f1) stay within 160 KB.
#ifndef MEP_RF_FWD_ROWS
#define MEP_RF_FWD_ROWS 32
#endif
template <int D>
constexpr int rf_fwd_rows() { return D > 128 ? 32 : MEP_RF_FWD_ROWS; }

template <int D, int FD>
__global__ __launch_bounds__(THREADS) void k_rf_epi_fwd(const mep_rf_epi_desc* __restrict__ descs) {
    constexpr int TOK = rf_fwd_rows<D>(), MH = TOK / 32;
    constexpr int NCL = (D + 63) / 64;   // LayerNorm columns per lane (lane + 64 j)
    const mep_rf_epi_desc& d = descs[blockIdx.y];
    const int tok0 = blockIdx.x * TOK;
    const int ntok = d.ntok;
    if (tok0 >= ntok) return;
    constexpr int LD = D + 4, LF = FD + 4;
    __shared__ __attribute__((aligned(16))) float smem[2 * TOK * LD + TOK * LF];
    float* Xs = smem;                 // x, then h
    float* Ps = smem + TOK * LD;      // xp, then f
    float* Fs = smem + 2 * TOK * LD;  // f1
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    bool cv[NCL];
#pragma unroll
    for (int j = 0; j < NCL; ++j) cv[j] = lane + 64 * j < D;
    const float sa = *G<const float>(d.a), sb = *G<const float>(d.b);
    gfloat* stats = G<float>(d.stats);

    stage_cols<TOK>(Xs, LD, d.x, tok0, ntok, 0, D);
    __syncthreads();
    // xp = x Wp^T
    tile_gemm<D, D, true, MH>(Xs, LD, G<const float>(d.wp), D, wvec(d.wp, D), [&](int row, int col, float v) {
        Ps[row * LD + col] = v;
        const int tok = tok0 + row;
        if (tok < ntok) row_ptr(d.xp, tok)[col] = v;
    });
    __syncthreads();
    // LayerNorm of rows z (per lane columns lane + 64 j) into y = w * (z - mean) * rstd + b
    auto layer_norm = [&](const gfloat* w, const gfloat* bb, const float (&z)[NCL], float (&y)[NCL], float& mean,
                          float& rstd) {
        float s1 = 0.f;
#pragma unroll
        for (int j = 0; j < NCL; ++j) s1 += z[j];
        mean = wave_sum(s1) / (float)D;
        float dv[NCL], s2 = 0.f;
#pragma unroll
        for (int j = 0; j < NCL; ++j) { dv[j] = cv[j] ? z[j] - mean : 0.f; s2 += dv[j] * dv[j]; }
        rstd = 1.0f / sqrtf(wave_sum(s2) / (float)D + LN_EPS);
#pragma unroll
        for (int j = 0; j < NCL; ++j) y[j] = cv[j] ? dv[j] * rstd * w[lane + 64 * j] + bb[lane + 64 * j] : 0.f;
    };
    // h = LN1(q + a * xp)
    for (int row = wave; row < TOK; row += NWAVE) {
        const int tok = tok0 + row;
        float* xr = Xs + row * LD;
        if (tok >= ntok) {
#pragma unroll
            for (int j = 0; j < NCL; ++j) if (cv[j]) xr[lane + 64 * j] = 0.f;
            continue;
        }
        const gfloat* qr = row_ptr(d.q, tok);
        float z[NCL], y[NCL], mean, rstd;
#pragma unroll
        for (int j = 0; j < NCL; ++j)
            z[j] = cv[j] ? add_rn(qr[lane + 64 * j], mul_rn(sa, Ps[row * LD + lane + 64 * j])) : 0.f;
        layer_norm(G<const float>(d.ln1_w), G<const float>(d.ln1_b), z, y, mean, rstd);
        gfloat* hr = row_ptr(d.h, tok);
#pragma unroll
        for (int j = 0; j < NCL; ++j) if (cv[j]) { xr[lane + 64 * j] = y[j]; hr[lane + 64 * j] = y[j]; }
        if (lane == 0) { stats[4 * tok] = mean; stats[4 * tok + 1] = rstd; }
    }
    __syncthreads();
    // f1 = relu(h W1^T + b1)
    {
        const gfloat* b1 = G<const float>(d.b1);
        tile_gemm<FD, D, true, MH>(Xs, LD, G<const float>(d.w1), D, wvec(d.w1, D), [&](int row, int col, float v) {
            v = fmaxf(v + b1[col], 0.f);
            Fs[row * LF + col] = v;
            const int tok = tok0 + row;
            if (tok < ntok) row_ptr(d.f1, tok)[col] = v;
        });
    }
    __syncthreads();
    // f = f1 W2^T + b2
    {
        const gfloat* b2 = G<const float>(d.b2);
        tile_gemm<D, FD, true, MH>(Fs, LF, G<const float>(d.w2), FD, wvec(d.w2, FD), [&](int row, int col, float v) {
            v += b2[col];
            Ps[row * LD + col] = v;
            const int tok = tok0 + row;
            if (tok < ntok) row_ptr(d.f, tok)[col] = v;
        });
    }
    __syncthreads();
    // out = LN2(h + b * f)
    for (int row = wave; row < TOK; row += NWAVE) {
        const int tok = tok0 + row;
        if (tok >= ntok) break;
        float z[NCL], y[NCL], mean, rstd;
#pragma unroll
        for (int j = 0; j < NCL; ++j)
            z[j] = cv[j] ? add_rn(Xs[row * LD + lane + 64 * j], mul_rn(sb, Ps[row * LD + lane + 64 * j])) : 0.f;
        layer_norm(G<const float>(d.ln2_w), G<const float>(d.ln2_b), z, y, mean, rstd);
        gfloat* orow = row_ptr(d.out, tok);
#pragma unroll
        for (int j = 0; j < NCL; ++j) if (cv[j]) orow[lane + 64 * j] = y[j];
        if (lane == 0) { stats[4 * tok + 2] = mean; stats[4 * tok + 3] = rstd; }
    }
}

// Token rows per workgroup of the backward (32: twice the workgroups of 64 -- 50 per block at
// cfg2 -- and half the LDS; hosts size the partial rows with _lib.rf_bwd_rows)
#ifndef MEP_RF_BWD_ROWS
#define MEP_RF_BWD_ROWS 32
#endif

template <int D, int FD>
__global__ __launch_bounds__(THREADS) void k_rf_epi_bwd(const mep_rf_epi_bwd_desc* __restrict__ descs) {
    const mep_rf_epi_bwd_desc& bd = descs[blockIdx.y];
    const mep_rf_epi_desc& d = bd.f;
    constexpr int TB = MEP_RF_BWD_ROWS, MH = TB / 32;   // token rows of this workgroup
    const int tok0 = blockIdx.x * TB;
    const int ntok = d.ntok;
    if (tok0 >= ntok) return;
    constexpr int LD = D + 4, LF = FD + 4;
    constexpr int STRIDE = 5 * D + FD + 2;
    __shared__ __attribute__((aligned(16))) float smem[2 * TB * LD + TB * LF];
    __shared__ float red[NWAVE][2][128];
    __shared__ float sred[NWAVE][2];
    float* Gs = smem;                // dout -> dz2 -> dh -> dz1
    float* Ps = smem + TB * LD;      // df, then dxp
    float* Fs = smem + 2 * TB * LD;  // df1
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool c0 = lane < D, c1 = lane + 64 < D;
    const float sa = *G<const float>(d.a), sb = *G<const float>(d.b);
    const gfloat* stats = G<const float>(d.stats);
    gfloat* part = G<float>(bd.partial) + (int64_t)blockIdx.x * STRIDE;

    stage_cols<TB>(Gs, LD, bd.dout, tok0, ntok, 0, D);
    if (bd.dout2.ptr) {
        stage_cols<TB>(Ps, LD, bd.dout2, tok0, ntok, 0, D);
        __syncthreads();
        for (int idx = threadIdx.x; idx < TB * D; idx += THREADS) {
            const int row = idx / D, c = idx - row * D;
            Gs[row * LD + c] += Ps[row * LD + c];
        }
    }
    __syncthreads();
    // LN2 backward -> dz2 (kept in Gs as the residual part of dh); df = b * dz2 -> Ps
    float acc_s = 0.f;
    {
        const gfloat* w = G<const float>(d.ln2_w);
        const float w0 = c0 ? w[lane] : 0.f, w1 = c1 ? w[lane + 64] : 0.f;
        float pw0 = 0.f, pw1 = 0.f, pb0 = 0.f, pb1 = 0.f;
        for (int row = wave; row < TB; row += NWAVE) {
            const int tok = tok0 + row;
            float* gr = Gs + row * LD;
            float* pr = Ps + row * LD;
            if (tok >= ntok) {
                if (c0) { gr[lane] = 0.f; pr[lane] = 0.f; }
                if (c1) { gr[lane + 64] = 0.f; pr[lane + 64] = 0.f; }
                continue;
            }
            const float mean = stats[4 * tok + 2], rstd = stats[4 * tok + 3];
            const gfloat* hr = row_ptr(d.h, tok);
            const gfloat* fr = row_ptr(d.f, tok);
            const float f0 = c0 ? fr[lane] : 0.f, f1 = c1 ? fr[lane + 64] : 0.f;
            const float xh0 = c0 ? (add_rn(hr[lane], mul_rn(sb, f0)) - mean) * rstd : 0.f;
            const float xh1 = c1 ? (add_rn(hr[lane + 64], mul_rn(sb, f1)) - mean) * rstd : 0.f;
            const float g0 = c0 ? gr[lane] : 0.f, g1 = c1 ? gr[lane + 64] : 0.f;
            const float gw0 = g0 * w0, gw1 = g1 * w1;
            const float s1 = wave_sum(gw0 + gw1) / (float)D;
            const float s2 = wave_sum(gw0 * xh0 + gw1 * xh1) / (float)D;
            pw0 += g0 * xh0; pw1 += g1 * xh1; pb0 += g0; pb1 += g1;
            gfloat* dfr = row_ptr(bd.df, tok);
            if (c0) {
                const float dz = rstd * (gw0 - s1 - xh0 * s2);
                gr[lane] = dz; pr[lane] = sb * dz; dfr[lane] = sb * dz;
                acc_s += dz * f0;
            }
            if (c1) {
                const float dz = rstd * (gw1 - s1 - xh1 * s2);
                gr[lane + 64] = dz; pr[lane + 64] = sb * dz; dfr[lane + 64] = sb * dz;
                acc_s += dz * f1;
            }
        }
        red[wave][0][lane] = pw0; red[wave][0][lane + 64] = pw1;
        red[wave][1][lane] = pb0; red[wave][1][lane + 64] = pb1;
        const float s = wave_sum(acc_s);
        if (lane == 0) sred[wave][1] = s;  // db partial
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < 2 * D; idx += THREADS) {
        const int which = idx / D, c = idx - which * D;
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < NWAVE; ++w) s += red[w][which][c];
        part[idx] = s;  // [0, D) dLN2.w, [D, 2D) dLN2.b
    }
    for (int c = threadIdx.x; c < D; c += THREADS) {
        float s = 0.f;
        for (int r = 0; r < TB; ++r) s += Ps[r * LD + c];
        part[4 * D + c] = s;  // db2
    }
    // df1 = relu'(f1) * (df W2)      W2: [D][FD] -> element (k = d, n = f) at W2[d * FD + f]
    tile_gemm<FD, D, false, MH>(Ps, LD, G<const float>(d.w2), FD, false, [&](int row, int col, float v) {
        const int tok = tok0 + row;
        float o = 0.f;
        if (tok < ntok) {
            o = row_ptr(d.f1, tok)[col] > 0.f ? v : 0.f;
            row_ptr(bd.df1, tok)[col] = o;
        }
        Fs[row * LF + col] = o;
    });
    __syncthreads();
    for (int c = threadIdx.x; c < FD; c += THREADS) {
        float s = 0.f;
        for (int r = 0; r < TB; ++r) s += Fs[r * LF + c];
        part[5 * D + c] = s;  // db1
    }
    // dh = dz2 + df1 W1              W1: [FD][D] -> element (k = f, n = d) at W1[f * D + d]
    tile_gemm<D, FD, false, MH>(Fs, LF, G<const float>(d.w1), D, false, [&](int row, int col, float v) {
        Gs[row * LD + col] += v;
    });
    __syncthreads();
    // LN1 backward -> dz1;  dq (+)= dz1;  dxp = a * dz1 -> Ps
    acc_s = 0.f;
    {
        const gfloat* w = G<const float>(d.ln1_w);
        const float w0 = c0 ? w[lane] : 0.f, w1 = c1 ? w[lane + 64] : 0.f;
        float pw0 = 0.f, pw1 = 0.f, pb0 = 0.f, pb1 = 0.f;
        for (int row = wave; row < TB; row += NWAVE) {
            const int tok = tok0 + row;
            float* gr = Gs + row * LD;
            float* pr = Ps + row * LD;
            if (tok >= ntok) {
                if (c0) pr[lane] = 0.f;
                if (c1) pr[lane + 64] = 0.f;
                continue;
            }
            const float mean = stats[4 * tok], rstd = stats[4 * tok + 1];
            const gfloat* qr = row_ptr(d.q, tok);
            const gfloat* xr = row_ptr(d.xp, tok);
            const float x0 = c0 ? xr[lane] : 0.f, x1 = c1 ? xr[lane + 64] : 0.f;
            const float xh0 = c0 ? (add_rn(qr[lane], mul_rn(sa, x0)) - mean) * rstd : 0.f;
            const float xh1 = c1 ? (add_rn(qr[lane + 64], mul_rn(sa, x1)) - mean) * rstd : 0.f;
            const float g0 = c0 ? gr[lane] : 0.f, g1 = c1 ? gr[lane + 64] : 0.f;
            const float gw0 = g0 * w0, gw1 = g1 * w1;
            const float s1 = wave_sum(gw0 + gw1) / (float)D;
            const float s2 = wave_sum(gw0 * xh0 + gw1 * xh1) / (float)D;
            pw0 += g0 * xh0; pw1 += g1 * xh1; pb0 += g0; pb1 += g1;
            gfloat* dqr = row_ptr(bd.dq, tok);
            gfloat* dxr = row_ptr(bd.dxp, tok);
            if (c0) {
                const float dz = rstd * (gw0 - s1 - xh0 * s2);
                dqr[lane] = bd.dq_accumulate ? dqr[lane] + dz : dz;
                pr[lane] = sa * dz; dxr[lane] = sa * dz;
                acc_s += dz * x0;
            }
            if (c1) {
                const float dz = rstd * (gw1 - s1 - xh1 * s2);
                dqr[lane + 64] = bd.dq_accumulate ? dqr[lane + 64] + dz : dz;
                pr[lane + 64] = sa * dz; dxr[lane + 64] = sa * dz;
                acc_s += dz * x1;
            }
        }
        __syncthreads();  // the first reduction above has consumed red
        red[wave][0][lane] = pw0; red[wave][0][lane + 64] = pw1;
        red[wave][1][lane] = pb0; red[wave][1][lane + 64] = pb1;
        const float s = wave_sum(acc_s);
        if (lane == 0) sred[wave][0] = s;  // da partial
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < 2 * D; idx += THREADS) {
        const int which = idx / D, c = idx - which * D;
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < NWAVE; ++w) s += red[w][which][c];
        part[2 * D + idx] = s;  // [2D, 3D) dLN1.w, [3D, 4D) dLN1.b
    }
    if (threadIdx.x < 2) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < NWAVE; ++w) s += sred[w][threadIdx.x];
        part[5 * D + FD + threadIdx.x] = s;  // da, db
    }
    // dx = dxp Wp                   Wp: [D][D] -> element (k = n_out, n = k_in) at Wp[n_out * D + k_in]
    tile_gemm<D, D, false, MH>(Ps, LD, G<const float>(d.wp), D, false, [&](int row, int col, float v) {
        const int tok = tok0 + row;
        if (tok < ntok) row_ptr(bd.dx, tok)[col] = v;
    });
}

// ---------------------------------------------------------------- State_Transfer head
constexpr int RF_PMAX = 16;
constexpr int RF_NC = 6;

MEP_DEV void wave_sync() {
    __threadfence_block();
    __builtin_amdgcn_wave_barrier();
}

MEP_DEV float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

__global__ __launch_bounds__(64) void k_rf_head(mep_rf_head_desc d) {
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    const int P = d.P, D = d.D;
    __shared__ float s_fc[RF_PMAX][128], s_h[RF_PMAX][128];
    __shared__ float s_mean[RF_PMAX], s_rstd[RF_PMAX];
    __shared__ float s_o1[RF_PMAX][RF_NC], s_g[RF_PMAX][RF_NC], s_alpha[RF_PMAX][RF_NC];
    __shared__ float s_t0[RF_PMAX][RF_NC], s_out[RF_PMAX][RF_NC], s_dout[RF_PMAX][RF_NC];
    __shared__ float s_dg[RF_PMAX][RF_NC], s_d12[2 * RF_NC];
    const gfloat* fc = G<const float>(d.fc);
    const gfloat* lnw = G<const float>(d.ln_w);
    const gfloat* lnb = G<const float>(d.ln_b);
    const gfloat* wc = G<const float>(d.wc);
    const gfloat* bc = G<const float>(d.bc);
    const gfloat* trans = G<const float>(d.trans);
    const gfloat* ext = G<const float>(d.ext_dout);
    const bool c0 = lane < D, c1 = lane + 64 < D;
    const float w0 = c0 ? lnw[lane] : 0.f, w1 = c1 ? lnw[lane + 64] : 0.f;
    const float b0 = c0 ? lnb[lane] : 0.f, b1 = c1 ? lnb[lane + 64] : 0.f;
    // the classifier rows (12 x D) in registers for both directions, and each utterance's fc row
    // loaded one utterance ahead: the recurrence is one wave per batch row, so every load the loop
    // waited on was a dependent L2 round trip (72 per direction at P = 6)
    float wc0[2 * RF_NC], wc1[2 * RF_NC];
#pragma unroll
    for (int j = 0; j < 2 * RF_NC; ++j) {
        wc0[j] = c0 ? wc[j * D + lane] : 0.f;
        wc1[j] = c1 ? wc[j * D + lane + 64] : 0.f;
    }
    float loss = 0.f;
    float nx0 = c0 ? fc[(int64_t)(b * P) * D + lane] : 0.f, nx1 = c1 ? fc[(int64_t)(b * P) * D + lane + 64] : 0.f;

    for (int i = 0; i < P; ++i) {
        const int r = b * P + i;
        // h = relu(LN(fc))   (realformer.py:263)
        const float x0 = nx0, x1 = nx1;
        if (i + 1 < P) {
            const gfloat* fn = fc + (int64_t)(r + 1) * D;
            nx0 = c0 ? fn[lane] : 0.f;
            nx1 = c1 ? fn[lane + 64] : 0.f;
        }
        const float mean = wave_sum(x0 + x1) / (float)D;
        const float d0 = c0 ? x0 - mean : 0.f, d1 = c1 ? x1 - mean : 0.f;
        const float rstd = 1.0f / sqrtf(wave_sum(d0 * d0 + d1 * d1) / (float)D + LN_EPS);
        const float h0 = fmaxf(d0 * rstd * w0 + b0, 0.f), h1 = fmaxf(d1 * rstd * w1 + b1, 0.f);
        gfloat* hr = G<float>(d.h) + (int64_t)r * D;
        if (c0) { s_fc[i][lane] = x0; s_h[i][lane] = h0; hr[lane] = h0; }
        if (c1) { s_fc[i][lane + 64] = x1; s_h[i][lane + 64] = h1; hr[lane + 64] = h1; }
        if (lane == 0) { s_mean[i] = mean; s_rstd[i] = rstd; }
        // classifier D -> 12 (realformer.py:276), chunk -> (o, g)
        float z[2 * RF_NC];
#pragma unroll
        for (int j = 0; j < 2 * RF_NC; ++j) {
            float s = (c0 ? wc0[j] * h0 : 0.f) + (c1 ? wc1[j] * h1 : 0.f);
            z[j] = wave_sum(s) + bc[j];
        }
        // gate (realformer.py:278-281), lanes 0..5 own one class each
        const int n = lane < RF_NC ? lane : 0;
        float o1 = z[0], g = z[RF_NC];
#pragma unroll
        for (int j = 1; j < RF_NC; ++j) if (n == j) { o1 = z[j]; g = z[RF_NC + j]; }
        float out = o1, alpha = 0.f, t0 = 0.f;
        if (i > 0) {
            alpha = sigmoidf_(g + s_g[i - 1][n]);
            float s = 0.f;
            for (int m = 0; m < RF_NC; ++m) s = fmaf(s_out[i - 1][m], trans[m * RF_NC + n], s);
            t0 = tanhf(s);
            out = add_rn(mul_rn(1.f - alpha, o1), mul_rn(alpha, t0));
        }
        wave_sync();
        if (lane < RF_NC) {
            s_o1[i][n] = o1; s_g[i][n] = g; s_alpha[i][n] = alpha; s_t0[i][n] = t0; s_out[i][n] = out;
            G<float>(d.out)[(int64_t)r * RF_NC + n] = out;
        }
        wave_sync();
        // circle loss (realformer.py:289-298) * utterance mask, mean over B*P
        if (!ext) {
            const bool ok = lane < RF_NC;
            const float loss_scale = d.scale ? G<const float>(d.scale)[0] : d.loss_scale;
            const float um = (float)G<const int64_t>(d.umask)[r];
            const float t = ok ? (float)G<const int64_t>(d.labels)[(int64_t)r * RF_NC + lane] : 0.f;
            const bool is_pos = ok && t > 0.5f, is_neg = ok && !(t > 0.5f);
            const float vn = is_neg ? out : -INFINITY, vp = is_pos ? -out : -INFINITY;
            const float mn = fmaxf(wave_max(vn), 0.f), mp = fmaxf(wave_max(vp), 0.f);
            const float sn = wave_sum(is_neg ? __expf(vn - mn) : 0.f) + __expf(-mn);
            const float sp = wave_sum(is_pos ? __expf(vp - mp) : 0.f) + __expf(-mp);
            const float ln = mn + logf(sn), lp = mp + logf(sp);
            loss += (ln + lp) * um * loss_scale;
            float gr = 0.f;
            if (is_neg) gr = __expf(out - ln);
            if (is_pos) gr = -__expf(-out - lp);
            if (ok) s_dout[i][lane] = gr * um * loss_scale;
        } else if (lane < RF_NC) {
            s_dout[i][lane] = ext[(int64_t)r * RF_NC + lane];
        }
    }
    if (lane == 0 && !ext) G<float>(d.row_loss)[b] = loss;
    if (!d.compute_grad) return;
    wave_sync();

    // backward through the recurrence, last utterance first
    float pw0 = 0.f, pw1 = 0.f, pb0 = 0.f, pb1 = 0.f;
    float dtr = 0.f;  // lane < 36: dtrans[m = lane / 6][n = lane % 6]
    if (lane < RF_NC) for (int i = 0; i < P; ++i) s_dg[i][lane] = 0.f;
    wave_sync();
    for (int i = P - 1; i >= 0; --i) {
        const int r = b * P + i;
        const int n = lane < RF_NC ? lane : 0;
        const float dO = s_dout[i][n];
        float do1 = dO, dpt = 0.f;
        if (i > 0) {
            const float a = s_alpha[i][n], t0 = s_t0[i][n], o1 = s_o1[i][n];
            do1 = (1.f - a) * dO;
            const float dpre = dO * (t0 - o1) * a * (1.f - a);
            dpt = a * dO * (1.f - t0 * t0);
            if (lane < RF_NC) { s_dg[i][n] += dpre; s_dg[i - 1][n] += dpre; }
        }
        wave_sync();
        if (lane < RF_NC) { s_d12[n] = do1; s_d12[RF_NC + n] = s_dg[i][n]; s_t0[i][n] = dpt; }
        wave_sync();
        if (i > 0) {
            // dtrans[m][n] += out_{i-1}[m] dpt[n];  dout_{i-1}[m] += sum_n trans[m][n] dpt[n]
            if (lane < RF_NC * RF_NC) dtr += s_out[i - 1][lane / RF_NC] * s_t0[i][lane % RF_NC];
            if (lane < RF_NC) {
                float s = 0.f;
                for (int k = 0; k < RF_NC; ++k) s = fmaf(trans[lane * RF_NC + k], s_t0[i][k], s);
                s_dout[i - 1][lane] += s;
            }
        }
        if (lane < 2 * RF_NC) G<float>(d.d12)[(int64_t)r * 2 * RF_NC + lane] = s_d12[lane];
        // dh = d12 Wc;  relu';  LN backward -> dfc
        float dh0 = 0.f, dh1 = 0.f;
#pragma unroll
        for (int j = 0; j < 2 * RF_NC; ++j) {
            const float dz = s_d12[j];
            if (c0) dh0 = fmaf(dz, wc0[j], dh0);
            if (c1) dh1 = fmaf(dz, wc1[j], dh1);
        }
        const float g0 = (c0 && s_h[i][lane] > 0.f) ? dh0 : 0.f;
        const float g1 = (c1 && s_h[i][lane + 64] > 0.f) ? dh1 : 0.f;
        const float mean = s_mean[i], rstd = s_rstd[i];
        const float xh0 = c0 ? (s_fc[i][lane] - mean) * rstd : 0.f;
        const float xh1 = c1 ? (s_fc[i][lane + 64] - mean) * rstd : 0.f;
        const float gw0 = g0 * w0, gw1 = g1 * w1;
        const float s1 = wave_sum(gw0 + gw1) / (float)D;
        const float s2 = wave_sum(gw0 * xh0 + gw1 * xh1) / (float)D;
        pw0 += g0 * xh0; pw1 += g1 * xh1; pb0 += g0; pb1 += g1;
        gfloat* dr = G<float>(d.dfc) + (int64_t)r * D;
        if (c0) dr[lane] = rstd * (gw0 - s1 - xh0 * s2);
        if (c1) dr[lane + 64] = rstd * (gw1 - s1 - xh1 * s2);
        wave_sync();
    }
    gfloat* part = G<float>(d.partial) + (int64_t)b * (2 * D + RF_NC * RF_NC);
    if (c0) { part[lane] = pw0; part[D + lane] = pb0; }
    if (c1) { part[lane + 64] = pw1; part[D + lane + 64] = pb1; }
    if (lane < RF_NC * RF_NC) part[2 * D + lane] = dtr;
}

template <typename F>
int dispatch_rf(int D, int FD, F&& f) {
#define MEP_RF_CASE(DD, FF) \
    if (D == DD && FD == FF) { f(std::integral_constant<int, DD>{}, std::integral_constant<int, FF>{}); return 0; }
    MEP_RF_CASE(32, 32) MEP_RF_CASE(32, 64) MEP_RF_CASE(64, 64) MEP_RF_CASE(64, 128)
    MEP_RF_CASE(96, 96) MEP_RF_CASE(96, 192) MEP_RF_CASE(128, 128) MEP_RF_CASE(128, 256)
#undef MEP_RF_CASE
    return MEP_EINVAL;
}

}  // namespace

extern "C" int mep_rf_epi_fwd(const mep_rf_epi_desc* descs, int n_desc, int max_tiles, int D, int FD,
                              mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    if (D == 192 && FD == 384) {   // robot_demo.py (DIM 192, FFN 2): forward only, 32 rows per workgroup
        hipLaunchKernelGGL((k_rf_epi_fwd<192, 384>), dim3(max_tiles, n_desc), dim3(THREADS), 0, (hipStream_t)stream,
                           descs);
        return mep_check_launch("mep_rf_epi_fwd");
    }
    const int rc = dispatch_rf(D, FD, [&](auto dc, auto fc) {
        hipLaunchKernelGGL((k_rf_epi_fwd<decltype(dc)::value, decltype(fc)::value>), dim3(max_tiles, n_desc),
                           dim3(THREADS), 0, (hipStream_t)stream, descs);
    });
    if (rc) { mep_set_error("mep_rf_epi_fwd: D in {32,64,96,128} and FD in {D, 2D}, or D = 192 / FD = 384"); return rc; }
    return mep_check_launch("mep_rf_epi_fwd");
}

extern "C" int mep_rf_epi_bwd(const mep_rf_epi_bwd_desc* descs, int n_desc, int max_tiles, int D, int FD,
                              mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    const int rc = dispatch_rf(D, FD, [&](auto dc, auto fc) {
        hipLaunchKernelGGL((k_rf_epi_bwd<decltype(dc)::value, decltype(fc)::value>), dim3(max_tiles, n_desc),
                           dim3(THREADS), 0, (hipStream_t)stream, descs);
    });
    if (rc) { mep_set_error("mep_rf_epi_bwd: D in {32,64,96,128} and FD in {D, 2D}"); return rc; }
    return mep_check_launch("mep_rf_epi_bwd");
}

extern "C" int mep_rf_head(const mep_rf_head_desc* d, mep_stream_t stream) {
    if (d->B <= 0) return 0;
    if (d->P < 1 || d->P > RF_PMAX || d->D < 1 || d->D > 128) {
        mep_set_error("mep_rf_head: 1 <= P <= 16 and D <= 128");
        return MEP_EINVAL;
    }
    hipLaunchKernelGGL(k_rf_head, dim3(d->B), dim3(64), 0, (hipStream_t)stream, *d);
    return mep_check_launch("mep_rf_head");
}
