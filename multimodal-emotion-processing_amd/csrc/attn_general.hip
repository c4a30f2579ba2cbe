// mep_attn_general_fwd / _bwd: the reference's multi_head_attention for every mask form its
// signature accepts (cmu-mosei/run.py:236-257, Ren-MME/run.py:188-208, others/realformer.py:
// 190-204): no mask, a [B, Tk] key mask or a [B, Tq, Tk] mask (repeated over the heads, run.py:
// 250-252), with or without residual scores, K != V, any head dim up to 64.
//
// This is the standalone Attention_Block.forward surface for the mask forms the model plans never
// pass (their blocks take [B, Tk] key masks and run on mep_attn_fwd / _bwd).  fp32 throughout,
// the score in the reference's op order (one rounding per op, no contraction), exp(s - max) with
// s - max exact.  One workgroup per (b, h): the forward keeps a query's scores in LDS, the backward
// gives every thread one key (its K / V rows and dK / dV accumulators in registers) and walks the
// queries in order, so every sum has a fixed order.
#include "common.h"

namespace {

using namespace mep;

constexpr int GEN_THREADS = 256;           // keys per pass of the backward
constexpr int GEN_MAX_TK = 4096;           // forward: a query's scores in LDS

MEP_DEV float gen_mask_term(const mep_attn_gen_desc& g, int b, int q, int k) {
    // the reference subtracts 1e8 * (1 - mask); without a mask nothing (s - 0 is s)
    if (!g.f.mask) return 0.f;
    const float m = G<const float>(g.f.mask)[(int64_t)b * g.f.mask_sB + (int64_t)q * g.mask_sQ + k];
    return mul_rn(1.0e8f, sub_rn(1.0f, m));
}

MEP_DEV const gfloat* head_row(const mep_rows& r, int b, int T, int t, int hc) {
    return row_ptr(r, b * T + t) + hc;
}

MEP_DEV float gen_score(const mep_attn_gen_desc& g, float dot, float c, const gfloat* sp, int64_t si, int b, int q, int k) {
    float s = __fdiv_rn(dot, g.scale);                      // q k^T / sqrt(hd)
    if (sp) s = add_rn(s, mul_rn(c, sp[si]));               // + c * scores
    return sub_rn(s, gen_mask_term(g, b, q, k));            // -= 1e8 * (1 - mask)
}

// workgroup reductions over the 256 threads (fixed order: waves in order)
template <bool MAX>
MEP_DEV float block_reduce(float v, float* red) {
    const int w = threadIdx.x >> 6;
    v = MAX ? wave_max(v) : wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float r = red[0];
#pragma unroll
    for (int i = 1; i < GEN_THREADS / 64; ++i) r = MAX ? fmaxf(r, red[i]) : r + red[i];
    return r;
}

__global__ __launch_bounds__(GEN_THREADS) void k_attn_gen_fwd(const mep_attn_gen_desc* __restrict__ descs) {
    const mep_attn_gen_desc& g = descs[blockIdx.y];
    const mep_attn_desc& d = g.f;
    if ((int)blockIdx.x >= d.B * d.H) return;
    const int b = blockIdx.x / d.H, h = blockIdx.x % d.H, hd = g.hd, hc = h * hd, tid = threadIdx.x;
    const int Tq = d.Tq, Tk = d.Tk;
    if (Tk > GEN_MAX_TK || g.hd > 64) return;   // outside the contract (mep.h): writes nothing
    __shared__ float sbuf[GEN_MAX_TK];
    __shared__ float qrow[64];
    __shared__ float red[GEN_THREADS / 64];
    const float c = d.s_prev ? *G<const float>(d.c) : 0.f;
    const gfloat* sp = d.s_prev ? G<const float>(d.s_prev) : nullptr;
    gfloat* so = d.s_out ? G<float>(d.s_out) : nullptr;
    gfloat* stats = G<float>(d.stats);
    for (int q = 0; q < Tq; ++q) {
        __syncthreads();
        if (tid < hd) qrow[tid] = head_row(d.q, b, Tq, q, hc)[tid];
        __syncthreads();
        const int64_t srow = ((int64_t)(b * d.H + h) * Tq + q) * Tk;
        float mx = -INFINITY;
        for (int k = tid; k < Tk; k += GEN_THREADS) {
            const gfloat* kr = head_row(d.k, b, Tk, k, hc);
            float dot = 0.f;
            for (int e = 0; e < hd; ++e) dot = fmaf(qrow[e], kr[e], dot);
            const float s = gen_score(g, dot, c, sp, srow + k, b, q, k);
            if (so) so[srow + k] = s;
            sbuf[k] = s;
            mx = fmaxf(mx, s);
        }
        mx = block_reduce<true>(mx, red);
        float sum = 0.f, rs = 0.f;
        for (int k = tid; k < Tk; k += GEN_THREADS) {
            const float p = expf(sbuf[k] - mx);                  // softmax: exp(s - max), s - max exact
            sbuf[k] = p;
            sum += p;
            if (sp) rs = fmaf(p, sp[srow + k], rs);
        }
        sum = block_reduce<false>(sum, red);
        if (sp) rs = block_reduce<false>(rs, red);
        const float inv = 1.0f / sum;
        // att @ v: thread e < hd sums its output column over the keys in order
        if (tid < hd) {
            float o = 0.f;
            for (int k = 0; k < Tk; ++k) o = fmaf(sbuf[k] * inv, head_row(d.v, b, Tk, k, hc)[tid], o);
            row_ptr(d.x, b * Tq + q)[hc + tid] = o;
        }
        if (tid == 0) {
            stats[2 * ((b * d.H + h) * Tq + q)] = mx;            // raw (max, 1/sum)
            stats[2 * ((b * d.H + h) * Tq + q) + 1] = inv;
            // residual scores: the row's P-weighted mean of S_prev in the stats' tail (attn.hip)
            if (sp) stats[2 * d.B * d.H * Tq + (b * d.H + h) * Tq + q] = rs * inv;
        }
    }
}

template <int HDP>
__global__ __launch_bounds__(GEN_THREADS) void k_attn_gen_bwd(const mep_attn_gen_bwd_desc* __restrict__ descs) {
    const mep_attn_gen_bwd_desc& bd = descs[blockIdx.y];
    const mep_attn_gen_desc& g = bd.g;
    const mep_attn_desc& d = g.f;
    if ((int)blockIdx.x >= d.B * d.H) return;
    const int b = blockIdx.x / d.H, h = blockIdx.x % d.H, hd = g.hd, hc = h * hd, tid = threadIdx.x;
    const int Tq = d.Tq, Tk = d.Tk;
    if (hd > HDP) return;
    __shared__ float qrow[64], dorow[64], gbuf[GEN_THREADS];
    __shared__ float red[GEN_THREADS / 64];
    const float c = d.s_prev ? *G<const float>(d.c) : 0.f;
    const gfloat* sp = d.s_prev ? G<const float>(d.s_prev) : nullptr;
    const gfloat* dsn = bd.ds_next ? G<const float>(bd.ds_next) : nullptr;
    gfloat* dsp = bd.ds_prev ? G<float>(bd.ds_prev) : nullptr;
    const gfloat* stats = G<const float>(d.stats);
    const bool kv_same = bd.dk.ptr == bd.dv.ptr;
    float dc_acc = 0.f;
    for (int k0 = 0; k0 < Tk; k0 += GEN_THREADS) {
        const int k = k0 + tid;
        const bool kok = k < Tk;
        const int kc = min(k, Tk - 1);
        float kr[HDP], vr[HDP], dk[HDP], dv[HDP];
        {
            const gfloat* kp = head_row(d.k, b, Tk, kc, hc);
            const gfloat* vp = head_row(d.v, b, Tk, kc, hc);
#pragma unroll
            for (int e = 0; e < HDP; ++e) {
                kr[e] = e < hd ? kp[e] : 0.f;
                vr[e] = e < hd ? vp[e] : 0.f;
                dk[e] = 0.f;
                dv[e] = 0.f;
            }
        }
        for (int q = 0; q < Tq; ++q) {
            __syncthreads();
            float delta_part = 0.f;
            if (tid < 64) {   // dims past hd read 0 (they meet the zeroed rows past hd)
                const bool on = tid < hd;
                qrow[tid] = on ? head_row(d.q, b, Tq, q, hc)[tid] : 0.f;
                const float dov = on ? head_row(bd.dx, b, Tq, q, hc)[tid] : 0.f;
                dorow[tid] = dov;
                delta_part = on ? dov * head_row(d.x, b, Tq, q, hc)[tid] : 0.f;
            }
            // delta = rowsum(dO * O) = sum_k att_k dP_k (the softmax backward's row term)
            const float delta = block_reduce<false>(delta_part, red);
            const int64_t si = ((int64_t)(b * d.H + h) * Tq + q) * Tk + kc;
            const float mx = stats[2 * ((b * d.H + h) * Tq + q)];
            const float inv = stats[2 * ((b * d.H + h) * Tq + q) + 1];
            const float rp = sp ? stats[2 * d.B * d.H * Tq + (b * d.H + h) * Tq + q] : 0.f;
            float dot = 0.f, dp = 0.f;
#pragma unroll
            for (int e = 0; e < HDP; ++e) {
                dot = fmaf(qrow[e], kr[e], dot);
                dp = fmaf(dorow[e], vr[e], dp);
            }
            const float s = gen_score(g, dot, c, sp, si, b, q, kc);
            const float att = kok ? expf(s - mx) * inv : 0.f;
            float ds = att * (dp - delta);
            // d / dc = sum dS * S_prev, the softmax part against S_prev - rp (its row sum is 0:
            // attn.hip Bwd::tile), the gradient on the post-mask scores against S_prev itself
            if (sp && kok) dc_acc = fmaf(ds, sp[si] - rp, dc_acc);
            if (dsn && kok) {
                const float gn = dsn[si];                        // gradient on the post-mask scores output
                ds += gn;
                if (sp) dc_acc = fmaf(gn, sp[si], dc_acc);
            }
            if (dsp && kok) dsp[si] = c * ds;                    // d(c * scores) / d scores
            const float gs = kok ? __fdiv_rn(ds, g.scale) : 0.f; // through q k^T / sqrt(hd)
#pragma unroll
            for (int e = 0; e < HDP; ++e) {
                dv[e] = fmaf(att, dorow[e], dv[e]);
                dk[e] = fmaf(gs, qrow[e], dk[e]);
            }
            gbuf[tid] = gs;
            __syncthreads();
            // dQ row (accumulated onto dq, as mep_attn_bwd): thread e < hd sums this pass's keys in
            // order, passes in order
            if (tid < hd) {
                float acc = 0.f;
                const int kn = min(GEN_THREADS, Tk - k0);
                for (int j = 0; j < kn; ++j) acc = fmaf(gbuf[j], head_row(d.k, b, Tk, k0 + j, hc)[tid], acc);
                gfloat* dq = row_ptr(bd.dq, b * Tq + q) + hc + tid;
                *dq = *dq + acc;
            }
        }
        if (kok) {
            gfloat* dkp = row_ptr(bd.dk, b * Tk + k) + hc;
            gfloat* dvp = row_ptr(bd.dv, b * Tk + k) + hc;
            for (int e = 0; e < hd; ++e) {
                if (kv_same) {
                    dkp[e] = dk[e] + dv[e];                          // k is v: one gradient
                } else {
                    dkp[e] = dk[e];
                    dvp[e] = dv[e];
                }
            }
        }
    }
    if (bd.dc_partial) {
        const float w = block_reduce<false>(dc_acc, red);
        if (tid == 0) G<float>(bd.dc_partial)[blockIdx.x] = w;
    }
}

}  // namespace

extern "C" int mep_attn_general_fwd(const mep_attn_gen_desc* descs, int n_desc, int max_bh, mep_stream_t stream) {
    if (n_desc <= 0 || max_bh <= 0) return 0;
    hipLaunchKernelGGL(k_attn_gen_fwd, dim3(max_bh, n_desc), dim3(GEN_THREADS), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_attn_general_fwd");
}

extern "C" int mep_attn_general_bwd(const mep_attn_gen_bwd_desc* descs, int n_desc, int max_bh, int max_hd,
                                    mep_stream_t stream) {
    if (n_desc <= 0 || max_bh <= 0) return 0;
    const dim3 grid(max_bh, n_desc), block(GEN_THREADS);
    hipStream_t st = (hipStream_t)stream;
    if (max_hd <= 16) hipLaunchKernelGGL(k_attn_gen_bwd<16>, grid, block, 0, st, descs);
    else if (max_hd <= 32) hipLaunchKernelGGL(k_attn_gen_bwd<32>, grid, block, 0, st, descs);
    else if (max_hd <= 64) hipLaunchKernelGGL(k_attn_gen_bwd<64>, grid, block, 0, st, descs);
    else { mep_set_error("mep_attn_general_bwd: head dim <= 64"); return MEP_EINVAL; }
    return mep_check_launch("mep_attn_general_bwd");
}
