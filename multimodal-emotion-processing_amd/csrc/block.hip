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

// MEP_EXP (development A/B builds only; 0 in the product): 1 = no HBM stores, 2 = no MFMA,
// 4 = no staging loads, 8 = no LayerNorm math, 16 = no weight loads (common.h wfrag)
constexpr int EW = 4;               // waves per workgroup of the forward epilogue
constexpr int ETHREADS = 64 * EW;

// One WAVE = 16 tokens x all D columns, four independent waves per workgroup (no block
// barriers).  Both Linears are wave-level 16-row GEMMs (wgemm16: v_mfma_f32_16x16x4_f32, the
// weight fragments of the next k block in flight during the current one); the LayerNorm runs on
// the accumulators in registers (row sums over the D/16 column blocks a lane holds + a 16-lane
// shuffle reduction).  LDS holds this wave's A operands: x (then xp) and q.  Every HBM store is
// issued after the last weight load: s_waitcnt vmcnt counts loads and stores together in issue
// order, so a store in flight would delay every later weight fragment.
template <int D>
__global__ __launch_bounds__(ETHREADS) void k_epi_fwd(const mep_epi_desc* __restrict__ descs) {
    const mep_epi_desc& d = descs[blockIdx.y];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int ntok = d.ntok;
    const int r0 = blockIdx.x * 64 + wave * 16;
    if (r0 >= ntok) return;   // whole wave; only wave-private LDS below
    constexpr int LD = D + 4, NJ = D / 16;
    __shared__ __attribute__((aligned(16))) float smem[EW][2][16 * LD];
    float* As = smem[wave][0];   // x, then xp (post-dropout)
    float* Qs = smem[wave][1];   // q
    const float p = d.drop_p;
    const uint64_t seed = (d.seed && p > 0.f) ? *G<const uint64_t>(d.seed) : 0;
    const gfloat* Wp = G<const float>(d.wp);
    const gfloat* Wm = G<const float>(d.wm);

    if (!(MEP_EXP & 4)) {
        wave_stage16<D>(As, LD, d.x, r0, ntok);
        wave_stage16<D>(Qs, LD, d.q, r0, ntok);
    }
    wave_lds_fence();
    f32x4 acc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = zero_f4();
    if (!(MEP_EXP & 2)) wgemm16<NJ, D, true>(acc, As, LD, Wp, D, 0, vec_ok(d.wp, D));
    wave_lds_fence();   // every lane is done reading x
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int row = 4 * g + r, tok = r0 + row;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int col = 16 * j + c;
            float v = acc[j][r];
            if (p > 0.f) v *= drop_scale(seed, 2u * d.drop_stream, (uint64_t)tok * D + col, p);
            As[row * LD + col] = v;
        }
    }
    wave_lds_fence();
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = zero_f4();
    const bool wv = vec_ok(d.wm, 2 * D);
    if (!(MEP_EXP & 2)) {
        wgemm16<NJ, D, true>(acc, Qs, LD, Wm, 2 * D, 0, wv);       // [q | xp] Wm^T: q half
        wgemm16<NJ, D, true>(acc, As, LD, Wm + D, 2 * D, 0, wv);   //                xp half
    }
    // LayerNorm on the accumulators; then every store
    const gfloat* lw = G<const float>(d.ln_w);
    const gfloat* lb = G<const float>(d.ln_b);
    gfloat* stats = G<float>(d.stats);
    float wj[NJ], bj[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) { wj[j] = lw[16 * j + c]; bj[j] = lb[16 * j + c]; }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int tok = r0 + 4 * g + r;
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < NJ; ++j) s += acc[j][r];
        const float mean = group16_sum(s) / (float)D;
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < NJ; ++j) { const float t = acc[j][r] - mean; q += t * t; }
        const float rstd = (MEP_EXP & 8) ? 1.f : 1.0f / sqrtf(group16_sum(q) / (float)D + LN_EPS);
        if ((MEP_EXP & 1) ? tok < 0 : tok < ntok) {
            gfloat* zr = row_ptr(d.z, tok);
            gfloat* orow = row_ptr(d.out, tok);
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int col = 16 * j + c;
                zr[col] = acc[j][r];
                float y = (acc[j][r] - mean) * rstd * wj[j] + bj[j];
                if (p > 0.f) y *= drop_scale(seed, 2u * d.drop_stream + 1u, (uint64_t)tok * D + col, p);
                orow[col] = y;
            }
            if (c == 0) { stats[2 * tok] = mean; stats[2 * tok + 1] = rstd; }
        }
    }
    if (!(MEP_EXP & 1)) wave_store16<D>(As, LD, d.xp, r0, ntok);
}

// Backward, same mapping (one wave = 16 tokens x D): dout (+dout2) and z are read straight into
// the accumulator layout, the LayerNorm backward runs in registers, dz is staged once in LDS as
// the A operand of dq_direct = dz Wm[:, :D] and dxp = drop'(dz Wm[:, D:]), and dxp (LDS) of
// dx = dxp Wp.  ln_partial gets one [2][D] row per 16-token wave (no block barrier anywhere).
template <int D>
__global__ __launch_bounds__(ETHREADS) __attribute__((amdgpu_waves_per_eu(3))) void k_epi_bwd(const mep_epi_bwd_desc* __restrict__ descs) {
    const mep_epi_bwd_desc& bd = descs[blockIdx.y];
    const mep_epi_desc& d = bd.f;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int ntok = d.ntok;
    const int r0 = blockIdx.x * 64 + wave * 16;
    if (r0 >= ntok) return;
    constexpr int LD = D + 4, NJ = D / 16;
    __shared__ __attribute__((aligned(16))) float smem[EW][2][16 * LD];
    float* Gs = smem[wave][0];   // dz
    float* Ps = smem[wave][1];   // dxp
    const float p = d.drop_p;
    const uint64_t seed = (d.seed && p > 0.f) ? *G<const uint64_t>(d.seed) : 0;
    const gfloat* lw = G<const float>(d.ln_w);
    const gfloat* stats = G<const float>(d.stats);
    float wj[NJ], pw[NJ], pb[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) { wj[j] = lw[16 * j + c]; pw[j] = 0.f; pb[j] = 0.f; }
    // LayerNorm backward per row of this lane (rows 4g + r); not unrolled: bounds live registers
#pragma unroll 1
    for (int r = 0; r < 4; ++r) {
        const int row = 4 * g + r, tok = r0 + row;
        const bool ok = tok < ntok;
        const int tc = min(tok, ntok - 1);
        const gfloat* gr = row_ptr(bd.dout, tc);
        const gfloat* g2 = bd.dout2.ptr ? row_ptr(bd.dout2, tc) : nullptr;
        const gfloat* zr = row_ptr(d.z, tc);
        const float mean = stats[2 * tc], rstd = stats[2 * tc + 1];
        float gv[NJ], xh[NJ], s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int col = 16 * j + c;
            float gg = gr[col];
            if (g2) gg += g2[col];
            if (p > 0.f) gg *= drop_scale(seed, 2u * d.drop_stream + 1u, (uint64_t)tok * D + col, p);
            gg = ok ? gg : 0.f;
            gv[j] = gg;
            xh[j] = (zr[col] - mean) * rstd;
            const float gw = gg * wj[j];
            s1 += gw;
            s2 += gw * xh[j];
            pw[j] += gg * xh[j];
            pb[j] += gg;
        }
        s1 = group16_sum(s1) / (float)D;
        s2 = group16_sum(s2) / (float)D;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int col = 16 * j + c;
            Gs[row * LD + col] = ok ? rstd * (gv[j] * wj[j] - s1 - xh[j] * s2) : 0.f;
        }
    }
    wave_lds_fence();
    const gfloat* Wm = G<const float>(d.wm);
    const gfloat* Wp = G<const float>(d.wp);
    f32x4 acc[NJ], accq[NJ];
    // dxp = drop'(dz Wm[:, D:])  (Wm[k][n] with k the output unit: NT = false) -> LDS
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = zero_f4();
    wgemm16<NJ, D, false>(acc, Gs, LD, Wm + D, 2 * D, 0, false);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int row = 4 * g + r, tok = r0 + row;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int col = 16 * j + c;
            float v = acc[j][r];
            if (p > 0.f) v *= drop_scale(seed, 2u * d.drop_stream, (uint64_t)tok * D + col, p);
            Ps[row * LD + col] = tok < ntok ? v : 0.f;
        }
    }
    // dq_direct = dz Wm[:, :D]
#pragma unroll
    for (int j = 0; j < NJ; ++j) accq[j] = zero_f4();
    wgemm16<NJ, D, false>(accq, Gs, LD, Wm, 2 * D, 0, false);
    wave_lds_fence();
    // dx = dxp Wp
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = zero_f4();
    wgemm16<NJ, D, false>(acc, Ps, LD, Wp, D, 0, false);
    // stores, after the last weight load
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int tok = r0 + 4 * g + r;
        if (tok >= ntok) continue;
        gfloat* q = row_ptr(bd.dq, tok);
        gfloat* xr = row_ptr(bd.dx, tok);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int col = 16 * j + c;
            q[col] = bd.dq_accumulate ? q[col] + accq[j][r] : accq[j][r];
            xr[col] = acc[j][r];
        }
    }
    wave_store16<D>(Gs, LD, bd.dz, r0, ntok);
    wave_store16<D>(Ps, LD, bd.dxp, r0, ntok);    // per-wave LayerNorm parameter partials: reduce the 4 lane groups
    if (bd.ln_partial) {
        gfloat* lp = G<float>(bd.ln_partial) + (int64_t)(blockIdx.x * EW + wave) * 2 * D;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            float a = pw[j], b = pb[j];
            a += __shfl_xor(a, 16, 64); a += __shfl_xor(a, 32, 64);
            b += __shfl_xor(b, 16, 64); b += __shfl_xor(b, 32, 64);
            if (g == 0) { lp[16 * j + c] = a; lp[D + 16 * j + c] = b; }
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
        hipLaunchKernelGGL(k_epi_fwd<decltype(dc)::value>, dim3(max_tiles, n_desc), dim3(ETHREADS), 0,
                           (hipStream_t)stream, descs);
    });
    if (rc) { mep_set_error("mep_block_epi_fwd: D must be 32, 64, 96 or 128"); return rc; }
    return mep_check_launch("mep_block_epi_fwd");
}

extern "C" int mep_block_epi_bwd(const mep_epi_bwd_desc* descs, int n_desc, int max_tiles, int D, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    const int rc = dispatch_D(D, [&](auto dc) {
        hipLaunchKernelGGL(k_epi_bwd<decltype(dc)::value>, dim3(max_tiles, n_desc), dim3(ETHREADS), 0,
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
