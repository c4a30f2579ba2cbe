// cmu-mosei / Ren-MME Attention_Block epilogue (forward + backward) and row LayerNorm.
//
// Forward (cmu-mosei/run.py:257-261; Ren-MME/run.py:209-213 with dropout and norm2):
//   xp = drop(x Wp^T);  z = [q | xp] Wm^T;  out = drop(LayerNorm(z))
// One workgroup = 64 tokens x D columns (D in {32, 64, 96, 128}, a template parameter so every
// K loop is fully unrolled and hipcc issues the weight loads of a whole chain ahead of its
// MFMAs), 8 waves; each wave owns one 32x32 output block of the (2 x D/32) task grid and runs
// f32 MFMA 32x32x2 over LDS-staged token tiles with the weights read from L2.  The two Linears
// are chained through LDS (xp is consumed before it ever returns from HBM) and the LayerNorm is
// a wave-per-row shuffle reduction.  The concat [q | xp] is never materialised: the minus
// Linear is two accumulating MFMA passes.
#include "common.h"

using namespace mep;

namespace {

constexpr int THREADS = 512;
constexpr float LN_EPS = 1e-5f;

MEP_DEV bool vec_ok(uint64_t p, int ld) { return ((p & 15) == 0) && (ld % 4 == 0); }

// stage 64 token rows x D columns of a row view into LDS [64][D+4]
template <int D>
MEP_DEV void stage(float* dst, const mep_rows& src, int tok0, int ntok) {
    constexpr int LD = D + 4;
    constexpr int V = D / 4;  // float4 per row
    const bool vec = ((src.ptr & 15) == 0) && (src.sB % 4 == 0) && (src.sT % 4 == 0);
    for (int idx = threadIdx.x; idx < 64 * V; idx += THREADS) {
        const int row = idx / V, c4 = idx - row * V;
        const int tok = tok0 + row;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (tok < ntok) {
            const gfloat* p = row_ptr(src, tok) + 4 * c4;
            if (vec) v = ldg4(p);
            else v = make_float4(p[0], p[1], p[2], p[3]);
        }
        *reinterpret_cast<float4*>(dst + row * LD + 4 * c4) = v;
    }
}

template <int D>
__global__ __launch_bounds__(THREADS) void k_epi_fwd(const mep_epi_desc* __restrict__ descs) {
    const mep_epi_desc& d = descs[blockIdx.y];
    const int tok0 = blockIdx.x * 64;
    if (tok0 >= d.ntok) return;
    constexpr int LD = D + 4;
    __shared__ __attribute__((aligned(16))) float smem[3 * 64 * LD];
    float* Xs = smem;                 // x, later z
    float* Qs = smem + 64 * LD;
    float* Ps = smem + 2 * 64 * LD;   // xp (post-dropout)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int NTASK = 2 * (D / 32);
    const int mh = wave & 1, nblk = wave >> 1;
    const bool task = wave < NTASK;
    const int col = nblk * 32 + (lane & 31);
    const gfloat* Wp = G<const float>(d.wp);
    const gfloat* Wm = G<const float>(d.wm);
    const float p = d.drop_p;
    const uint64_t seed = (d.seed && p > 0.f) ? *G<const uint64_t>(d.seed) : 0;

    stage<D>(Xs, d.x, tok0, d.ntok);
    stage<D>(Qs, d.q, tok0, d.ntok);
    __syncthreads();
    floatx16 acc = zero16();
    if (task) {
        mma_tile<true, D>(acc, Xs, LD, mh * 32, Wp, D, nblk * 32, D, 0, D, D, vec_ok(d.wp, D));
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = mh * 32 + acc_row(r, lane);
            const int tok = tok0 + row;
            float v = acc[r];
            if (p > 0.f) v *= drop_scale(seed, 2u * d.drop_stream, (uint64_t)tok * D + col, p);
            Ps[row * LD + col] = v;
            if (tok < d.ntok) row_ptr(d.xp, tok)[col] = v;
        }
    }
    __syncthreads();
    if (task) {
        acc = zero16();
        const bool wv = vec_ok(d.wm, 2 * D);
        mma_tile<true, D>(acc, Qs, LD, mh * 32, Wm, 2 * D, nblk * 32, D, 0, D, D, wv);
        mma_tile<true, D>(acc, Ps, LD, mh * 32, Wm + D, 2 * D, nblk * 32, D, 0, D, D, wv);
    }
    __syncthreads();  // everyone done reading Xs (x) before it becomes z
    if (task) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = mh * 32 + acc_row(r, lane);
            const int tok = tok0 + row;
            Xs[row * LD + col] = acc[r];
            if (tok < d.ntok) row_ptr(d.z, tok)[col] = acc[r];
        }
    }
    __syncthreads();
    // LayerNorm: wave per row, lane covers columns lane and lane+64
    const gfloat* lw = G<const float>(d.ln_w);
    const gfloat* lb = G<const float>(d.ln_b);
    gfloat* stats = G<float>(d.stats);
    const bool c0 = lane < D, c1 = lane + 64 < D;
    const float w0 = c0 ? lw[lane] : 0.f, w1 = c1 ? lw[lane + 64] : 0.f;
    const float b0 = c0 ? lb[lane] : 0.f, b1 = c1 ? lb[lane + 64] : 0.f;
    for (int row = wave; row < 64; row += THREADS / 64) {
        const int tok = tok0 + row;
        if (tok >= d.ntok) break;
        const float x0 = c0 ? Xs[row * LD + lane] : 0.f;
        const float x1 = c1 ? Xs[row * LD + lane + 64] : 0.f;
        const float mean = wave_sum(x0 + x1) / (float)D;
        const float d0 = c0 ? x0 - mean : 0.f, d1 = c1 ? x1 - mean : 0.f;
        const float var = wave_sum(d0 * d0 + d1 * d1) / (float)D;
        const float rstd = 1.0f / sqrtf(var + LN_EPS);
        gfloat* out = row_ptr(d.out, tok);
        if (c0) {
            float y = d0 * rstd * w0 + b0;
            if (p > 0.f) y *= drop_scale(seed, 2u * d.drop_stream + 1u, (uint64_t)tok * D + lane, p);
            out[lane] = y;
        }
        if (c1) {
            float y = d1 * rstd * w1 + b1;
            if (p > 0.f) y *= drop_scale(seed, 2u * d.drop_stream + 1u, (uint64_t)tok * D + lane + 64, p);
            out[lane + 64] = y;
        }
        if (lane == 0) { stats[2 * tok] = mean; stats[2 * tok + 1] = rstd; }
    }
}

template <int D>
__global__ __launch_bounds__(THREADS) void k_epi_bwd(const mep_epi_bwd_desc* __restrict__ descs) {
    const mep_epi_bwd_desc& bd = descs[blockIdx.y];
    const mep_epi_desc& d = bd.f;
    const int tok0 = blockIdx.x * 64;
    if (tok0 >= d.ntok) return;
    constexpr int LD = D + 4;
    __shared__ __attribute__((aligned(16))) float smem[2 * 64 * LD + 8 * 2 * 128];
    float* Gs = smem;                 // dout -> dz
    float* Ps = smem + 64 * LD;       // dxp
    float* red = smem + 2 * 64 * LD;  // [8 waves][2][128]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const float p = d.drop_p;
    const uint64_t seed = (d.seed && p > 0.f) ? *G<const uint64_t>(d.seed) : 0;

    stage<D>(Gs, bd.dout, tok0, d.ntok);
    if (bd.dout2.ptr) {
        __syncthreads();
        stage<D>(Ps, bd.dout2, tok0, d.ntok);
        __syncthreads();
        for (int idx = threadIdx.x; idx < 64 * D; idx += THREADS) {
            const int row = idx / D, c = idx - row * D;
            Gs[row * LD + c] += Ps[row * LD + c];
        }
    }
    __syncthreads();
    // LayerNorm backward, wave per row
    const gfloat* lw = G<const float>(d.ln_w);
    const gfloat* stats = G<const float>(d.stats);
    float pw0 = 0.f, pw1 = 0.f, pb0 = 0.f, pb1 = 0.f;
    const bool c0 = lane < D, c1 = lane + 64 < D;
    const float w0 = c0 ? lw[lane] : 0.f, w1 = c1 ? lw[lane + 64] : 0.f;
    for (int row = wave; row < 64; row += THREADS / 64) {
        const int tok = tok0 + row;
        if (tok >= d.ntok) {
            if (c0) Gs[row * LD + lane] = 0.f;
            if (c1) Gs[row * LD + lane + 64] = 0.f;
            continue;
        }
        const float mean = stats[2 * tok], rstd = stats[2 * tok + 1];
        const gfloat* zr = row_ptr(d.z, tok);
        float g0 = c0 ? Gs[row * LD + lane] : 0.f;
        float g1 = c1 ? Gs[row * LD + lane + 64] : 0.f;
        if (p > 0.f) {
            if (c0) g0 *= drop_scale(seed, 2u * d.drop_stream + 1u, (uint64_t)tok * D + lane, p);
            if (c1) g1 *= drop_scale(seed, 2u * d.drop_stream + 1u, (uint64_t)tok * D + lane + 64, p);
        }
        const float xh0 = c0 ? (zr[lane] - mean) * rstd : 0.f;
        const float xh1 = c1 ? (zr[lane + 64] - mean) * rstd : 0.f;
        const float gw0 = g0 * w0, gw1 = g1 * w1;
        const float s1 = wave_sum(gw0 + gw1) / (float)D;
        const float s2 = wave_sum(gw0 * xh0 + gw1 * xh1) / (float)D;
        pw0 += g0 * xh0; pw1 += g1 * xh1; pb0 += g0; pb1 += g1;
        gfloat* dzr = row_ptr(bd.dz, tok);
        if (c0) { const float v = rstd * (gw0 - s1 - xh0 * s2); Gs[row * LD + lane] = v; dzr[lane] = v; }
        if (c1) { const float v = rstd * (gw1 - s1 - xh1 * s2); Gs[row * LD + lane + 64] = v; dzr[lane + 64] = v; }
    }
    red[(wave * 2 + 0) * 128 + lane] = pw0;
    red[(wave * 2 + 0) * 128 + lane + 64] = pw1;
    red[(wave * 2 + 1) * 128 + lane] = pb0;
    red[(wave * 2 + 1) * 128 + lane + 64] = pb1;
    __syncthreads();
    if (bd.ln_partial) {
        gfloat* lp = G<float>(bd.ln_partial) + (int64_t)blockIdx.x * 2 * D;
        for (int idx = threadIdx.x; idx < 2 * D; idx += THREADS) {
            const int which = idx / D, c = idx - which * D;
            float s = 0.f;
#pragma unroll
            for (int w = 0; w < THREADS / 64; ++w) s += red[(w * 2 + which) * 128 + c];
            lp[idx] = s;
        }
    }
    // dq_direct = dz Wm[:, :D];  dxp = drop'(dz Wm[:, D:])
    constexpr int NTASK = 2 * (D / 32);
    const int mh = wave & 1, nblk = wave >> 1;
    const bool task = wave < NTASK;
    const int col = nblk * 32 + (lane & 31);
    const gfloat* Wm = G<const float>(d.wm);
    const gfloat* Wp = G<const float>(d.wp);
    if (task) {
        floatx16 aq = zero16(), ap = zero16();
        mma_tile<false, D>(aq, Gs, LD, mh * 32, Wm, 2 * D, nblk * 32, D, 0, D, D, false);
        mma_tile<false, D>(ap, Gs, LD, mh * 32, Wm + D, 2 * D, nblk * 32, D, 0, D, D, false);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = mh * 32 + acc_row(r, lane);
            const int tok = tok0 + row;
            float vp = ap[r];
            if (p > 0.f && tok < d.ntok) vp *= drop_scale(seed, 2u * d.drop_stream, (uint64_t)tok * D + col, p);
            Ps[row * LD + col] = (tok < d.ntok) ? vp : 0.f;
            if (tok < d.ntok) {
                gfloat* q = row_ptr(bd.dq, tok) + col;
                *q = bd.dq_accumulate ? *q + aq[r] : aq[r];
                row_ptr(bd.dxp, tok)[col] = vp;
            }
        }
    }
    __syncthreads();
    if (task) {
        floatx16 ax = zero16();
        mma_tile<false, D>(ax, Ps, LD, mh * 32, Wp, D, nblk * 32, D, 0, D, D, false);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int tok = tok0 + mh * 32 + acc_row(r, lane);
            if (tok < d.ntok) row_ptr(bd.dx, tok)[col] = ax[r];
        }
    }
}

// ---------------------------------------------------------------- row LayerNorm (D <= 256)
__global__ __launch_bounds__(256) void k_ln_fwd(const mep_ln_desc* __restrict__ descs) {
    const mep_ln_desc& d = descs[blockIdx.y];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tok = blockIdx.x * 4 + wave;
    if (tok >= d.ntok) return;
    const gfloat* x = row_ptr(d.x, tok);
    float v[4], s = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) { const int c = lane + 64 * j; v[j] = c < d.D ? x[c] : 0.f; s += v[j]; }
    const float mean = wave_sum(s) / (float)d.D;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) { const int c = lane + 64 * j; v[j] = c < d.D ? v[j] - mean : 0.f; q += v[j] * v[j]; }
    const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)d.D + LN_EPS);
    const gfloat* w = G<const float>(d.w);
    const gfloat* b = G<const float>(d.b);
    gfloat* y = row_ptr(d.y, tok);
#pragma unroll
    for (int j = 0; j < 4; ++j) { const int c = lane + 64 * j; if (c < d.D) y[c] = v[j] * rstd * w[c] + b[c]; }
    if (lane == 0) {
        gfloat* st = G<float>(d.stats);
        st[2 * tok] = mean;
        st[2 * tok + 1] = rstd;
    }
}

// backward; partial[blockIdx.x][2][D] = per-workgroup (dgamma, dbeta) over its 64 rows
__global__ __launch_bounds__(256) void k_ln_bwd(const mep_ln_desc* __restrict__ descs) {
    const mep_ln_desc& d = descs[blockIdx.y];
    const int tok0 = blockIdx.x * 64;
    if (tok0 >= d.ntok) return;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __shared__ float red[4][2][256];
    float pw[4] = {0.f, 0.f, 0.f, 0.f}, pb[4] = {0.f, 0.f, 0.f, 0.f};
    const gfloat* w = G<const float>(d.w);
    const gfloat* st = G<const float>(d.stats);
    for (int row = wave; row < 64; row += 4) {
        const int tok = tok0 + row;
        if (tok >= d.ntok) break;
        const float mean = st[2 * tok], rstd = st[2 * tok + 1];
        const gfloat* x = row_ptr(d.x, tok);
        const gfloat* dy = row_ptr(d.dy, tok);
        float xh[4], gw[4], s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = lane + 64 * j;
            const bool ok = c < d.D;
            const float g = ok ? dy[c] : 0.f;
            xh[j] = ok ? (x[c] - mean) * rstd : 0.f;
            gw[j] = ok ? g * w[c] : 0.f;
            pw[j] += g * xh[j];
            pb[j] += g;
            s1 += gw[j];
            s2 += gw[j] * xh[j];
        }
        s1 = wave_sum(s1) / (float)d.D;
        s2 = wave_sum(s2) / (float)d.D;
        gfloat* dx = row_ptr(d.dx, tok);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = lane + 64 * j;
            if (c < d.D) {
                const float v = rstd * (gw[j] - s1 - xh[j] * s2);
                dx[c] = d.dx_accumulate ? dx[c] + v : v;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) { red[wave][0][lane + 64 * j] = pw[j]; red[wave][1][lane + 64 * j] = pb[j]; }
    __syncthreads();
    if (d.partial) {
        gfloat* lp = G<float>(d.partial) + (int64_t)blockIdx.x * 2 * d.D;
        for (int idx = threadIdx.x; idx < 2 * d.D; idx += 256) {
            const int which = idx / d.D, c = idx - which * d.D;
            lp[idx] = red[0][which][c] + red[1][which][c] + red[2][which][c] + red[3][which][c];
        }
    }
}

template <typename F>
int dispatch_D(int D, F&& f) {
    switch (D) {
        case 32: f(std::integral_constant<int, 32>{}); return 0;
        case 64: f(std::integral_constant<int, 64>{}); return 0;
        case 96: f(std::integral_constant<int, 96>{}); return 0;
        case 128: f(std::integral_constant<int, 128>{}); return 0;
        default: return MEP_EINVAL;
    }
}

}  // namespace

extern "C" int mep_block_epi_fwd(const mep_epi_desc* descs, int n_desc, int max_tiles, int D, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    const int rc = dispatch_D(D, [&](auto dc) {
        hipLaunchKernelGGL(k_epi_fwd<decltype(dc)::value>, dim3(max_tiles, n_desc), dim3(THREADS), 0,
                           (hipStream_t)stream, descs);
    });
    if (rc) { mep_set_error("mep_block_epi_fwd: D must be 32, 64, 96 or 128"); return rc; }
    return mep_check_launch("mep_block_epi_fwd");
}

extern "C" int mep_block_epi_bwd(const mep_epi_bwd_desc* descs, int n_desc, int max_tiles, int D, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    const int rc = dispatch_D(D, [&](auto dc) {
        hipLaunchKernelGGL(k_epi_bwd<decltype(dc)::value>, dim3(max_tiles, n_desc), dim3(THREADS), 0,
                           (hipStream_t)stream, descs);
    });
    if (rc) { mep_set_error("mep_block_epi_bwd: D must be 32, 64, 96 or 128"); return rc; }
    return mep_check_launch("mep_block_epi_bwd");
}

// max_tiles: forward = ceil(ntok / 4) (wave per row), backward = ceil(ntok / 64)
extern "C" int mep_layernorm_fwd(const mep_ln_desc* descs, int n_desc, int max_tiles, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    hipLaunchKernelGGL(k_ln_fwd, dim3(max_tiles, n_desc), dim3(256), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_layernorm_fwd");
}

extern "C" int mep_layernorm_bwd(const mep_ln_desc* descs, int n_desc, int max_tiles, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    hipLaunchKernelGGL(k_ln_bwd, dim3(max_tiles, n_desc), dim3(256), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_layernorm_bwd");
}
