// Residual scaled-dot-product attention core, forward and backward (fp32, hd = 16).
//
// Reference: Attention_Block.multi_head_attention, cmu-mosei/run.py:236-256 (identical in
// Ren-MME/run.py:188-208 and, after the w_qkv projections, others/realformer.py:182-204):
//   S = q k^T / sqrt(hd) [+ c * S_prev];  S -= 1e8 (1 - mask);  X = softmax(S) v
// The post-mask S is returned to the caller, which feeds it to the next layer of the chain.
//
// Mapping (CDNA4): one workgroup = 8 waves = (batch row, 64-row tile); wave w owns head w and
// each LANE owns one query row (forward, backward pass A) or one key row (backward pass B), so
// the softmax row max / sum never crosses lanes.  The 64-key K/V tile (or 64-query Q/dX tile)
// is staged in LDS and read by all lanes of a wave at the same address (broadcast, no bank
// conflicts).  hd = 16 operands live in registers; dots are fp32 FMA chains.  Row statistics
// (max, 1/sum) are kept instead of log-sum-exp because masked rows sit at -1e8 where
// max + log(sum) would round the log away (ulp(1e8) = 8).
#include <float.h>

#include "common.h"

using namespace mep;

namespace {

constexpr int HD = 16;
constexpr int THREADS = 512;     // 8 waves -> up to 8 heads
constexpr int TILE = 64;
constexpr int DMAX = 128;        // H*HD <= 128
constexpr float INV_SCALE = 0.25f;  // 1/sqrt(16), exact

struct Score {
    bool has_prev;
    float c;
};

// s = (q.k) * 0.25 [+ c*sp]  - 1e8 * (1 - m)      (op order of cmu-mosei/run.py:244-253)
MEP_DEV float score(const float* q, const float* k, const Score& sc, float sp, float m) {
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < HD; ++i) dot = fmaf(q[i], k[i], dot);
    float s = mul_rn(dot, INV_SCALE);
    if (sc.has_prev) s = add_rn(s, mul_rn(sc.c, sp));
    return sub_rn(s, mul_rn(1.0e8f, sub_rn(1.0f, m)));
}

MEP_DEV void load16(float* dst, const float* src) {
#pragma unroll
    for (int i = 0; i < HD; i += 4) {
        const float4 v = *reinterpret_cast<const float4*>(src + i);
        dst[i] = v.x; dst[i + 1] = v.y; dst[i + 2] = v.z; dst[i + 3] = v.w;
    }
}
MEP_DEV void load16u(float* dst, const float* src) {  // unaligned-safe
#pragma unroll
    for (int i = 0; i < HD; ++i) dst[i] = src[i];
}
MEP_DEV bool aligned16(const mep_rows& r) {
    return ((r.ptr & 15) == 0) && (r.sB % 4 == 0) && (r.sT % 4 == 0);
}

// stage rows [r0, r0+64) of a row view (batch row b, rows per batch T) into LDS [64][D]
MEP_DEV void stage_rows(float* dst, const mep_rows& src, int b, int r0, int nrows, int T, int D) {
    for (int idx = threadIdx.x; idx < TILE * D; idx += THREADS) {
        const int row = idx / D, col = idx - row * D;
        const int r = r0 + row;
        dst[idx] = (r < nrows) ? row_ptr(src, b * T + r)[col] : 0.f;
    }
}

MEP_DEV bool same_rows(const mep_rows& a, const mep_rows& b) {
    return a.ptr == b.ptr && a.sB == b.sB && a.sT == b.sT && a.T == b.T;
}

__global__ __launch_bounds__(THREADS) void k_attn_fwd(const mep_attn_desc* __restrict__ descs) {
    const mep_attn_desc& d = descs[blockIdx.y];
    const int nqt = (d.Tq + TILE - 1) / TILE;
    if ((int)blockIdx.x >= d.B * nqt) return;
    const int b = blockIdx.x / nqt, qt = blockIdx.x - (blockIdx.x / nqt) * nqt;
    const int D = d.H * HD;
    const int h = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int i = qt * TILE + lane;
    const bool active = (h < d.H) && (i < d.Tq);
    const bool kv_same = same_rows(d.k, d.v);

    __shared__ __attribute__((aligned(16))) float Ks[TILE * DMAX];
    __shared__ __attribute__((aligned(16))) float Vs[TILE * DMAX];
    __shared__ float Ms[TILE];

    Score sc{d.s_prev != 0, d.s_prev ? *reinterpret_cast<const float*>(d.c) : 0.f};
    float q[HD], o[HD];
    float m = -FLT_MAX, l = 0.f;
#pragma unroll
    for (int t = 0; t < HD; ++t) o[t] = 0.f;
    const int64_t srow = (((int64_t)b * d.H + h) * d.Tq + i) * d.Tk;
    const float* sprev = reinterpret_cast<const float*>(d.s_prev);
    float* sout = reinterpret_cast<float*>(d.s_out);
    if (active) {
        const float* qp = row_ptr(d.q, b * d.Tq + i) + h * HD;
        if (aligned16(d.q)) load16(q, qp); else load16u(q, qp);
    }
    const float* mask = reinterpret_cast<const float*>(d.mask) + (int64_t)b * d.mask_sB;
    const float* Vsrc = kv_same ? Ks : Vs;

    for (int k0 = 0; k0 < d.Tk; k0 += TILE) {
        __syncthreads();
        stage_rows(Ks, d.k, b, k0, d.Tk, d.Tk, D);
        if (!kv_same) stage_rows(Vs, d.v, b, k0, d.Tk, d.Tk, D);
        if (threadIdx.x < TILE) Ms[threadIdx.x] = (k0 + threadIdx.x < d.Tk) ? mask[k0 + threadIdx.x] : 0.f;
        __syncthreads();
        const int nk = min(TILE, d.Tk - k0);
        if (!active) continue;
        for (int kb = 0; kb < nk; kb += 8) {
            float s[8];
            float cmax = -INFINITY;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = kb + j;
                if (k < nk) {
                    s[j] = score(q, Ks + k * D + h * HD, sc, sc.has_prev ? sprev[srow + k0 + k] : 0.f, Ms[k]);
                    if (sout) sout[srow + k0 + k] = s[j];
                } else {
                    s[j] = -INFINITY;
                }
                cmax = fmaxf(cmax, s[j]);
            }
            const float mnew = fmaxf(m, cmax);
            const float corr = __expf(m - mnew);
            l *= corr;
#pragma unroll
            for (int t = 0; t < HD; ++t) o[t] *= corr;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = kb + j;
                if (k < nk) {
                    const float p = __expf(s[j] - mnew);
                    l += p;
                    const float* vr = Vsrc + k * D + h * HD;
#pragma unroll
                    for (int t = 0; t < HD; ++t) o[t] = fmaf(p, vr[t], o[t]);
                }
            }
            m = mnew;
        }
    }
    if (active) {
        const float inv = 1.0f / l;
        float* xp = row_ptr(d.x, b * d.Tq + i) + h * HD;
#pragma unroll
        for (int t = 0; t < HD; ++t) xp[t] = o[t] * inv;
        float* st = reinterpret_cast<float*>(d.stats) + 2 * ((((int64_t)b * d.H + h) * d.Tq) + i);
        st[0] = m;
        st[1] = inv;
    }
}

__global__ __launch_bounds__(THREADS) void k_attn_bwd(const mep_attn_bwd_desc* __restrict__ descs) {
    const mep_attn_bwd_desc& bd = descs[blockIdx.y];
    const mep_attn_desc& d = bd.f;
    const int nqt = (d.Tq + TILE - 1) / TILE, nkt = (d.Tk + TILE - 1) / TILE;
    if ((int)blockIdx.x >= d.B * (nqt + nkt)) return;
    const int D = d.H * HD;
    const int h = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool kv_same = same_rows(d.k, d.v);
    Score sc{d.s_prev != 0, d.s_prev ? *reinterpret_cast<const float*>(d.c) : 0.f};
    const float* sprev = reinterpret_cast<const float*>(d.s_prev);
    const float* dsn = reinterpret_cast<const float*>(bd.ds_next);
    const float* stats = reinterpret_cast<const float*>(d.stats);

    __shared__ __attribute__((aligned(16))) float S1[TILE * DMAX];
    __shared__ __attribute__((aligned(16))) float S2[TILE * DMAX];
    __shared__ float Sm[TILE * 8 * 3];   // pass B: (max, 1/sum, delta) per (row, head); pass A: mask

    if ((int)blockIdx.x < d.B * nqt) {
        // ------------------------------------------------ pass A: lane = query row -> dQ
        const int b = blockIdx.x / nqt, qt = blockIdx.x - b * nqt;
        const int i = qt * TILE + lane;
        const bool active = (h < d.H) && (i < d.Tq);
        float q[HD], dout[HD], dq[HD];
        float delta = 0.f, m = 0.f, linv = 0.f;
#pragma unroll
        for (int t = 0; t < HD; ++t) dq[t] = 0.f;
        const int64_t srow = (((int64_t)b * d.H + h) * d.Tq + i) * d.Tk;
        if (active) {
            load16u(q, row_ptr(d.q, b * d.Tq + i) + h * HD);
            load16u(dout, row_ptr(bd.dx, b * d.Tq + i) + h * HD);
            const float* xr = row_ptr(d.x, b * d.Tq + i) + h * HD;
#pragma unroll
            for (int t = 0; t < HD; ++t) delta = fmaf(dout[t], xr[t], delta);
            const float* st = stats + 2 * ((((int64_t)b * d.H + h) * d.Tq) + i);
            m = st[0];
            linv = st[1];
        }
        const float* mask = reinterpret_cast<const float*>(d.mask) + (int64_t)b * d.mask_sB;
        float* Ks = S1;
        float* Vs = kv_same ? S1 : S2;
        for (int k0 = 0; k0 < d.Tk; k0 += TILE) {
            __syncthreads();
            stage_rows(Ks, d.k, b, k0, d.Tk, d.Tk, D);
            if (!kv_same) stage_rows(Vs, d.v, b, k0, d.Tk, d.Tk, D);
            if (threadIdx.x < TILE) Sm[threadIdx.x] = (k0 + threadIdx.x < d.Tk) ? mask[k0 + threadIdx.x] : 0.f;
            __syncthreads();
            if (!active) continue;
            const int nk = min(TILE, d.Tk - k0);
            for (int k = 0; k < nk; ++k) {
                const float* kr = Ks + k * D + h * HD;
                const float* vr = Vs + k * D + h * HD;
                const float s = score(q, kr, sc, sc.has_prev ? sprev[srow + k0 + k] : 0.f, Sm[k]);
                const float p = __expf(s - m) * linv;
                float dp = 0.f;
#pragma unroll
                for (int t = 0; t < HD; ++t) dp = fmaf(dout[t], vr[t], dp);
                float ds = p * (dp - delta);
                if (dsn) ds += dsn[srow + k0 + k];
#pragma unroll
                for (int t = 0; t < HD; ++t) dq[t] = fmaf(ds, kr[t], dq[t]);
            }
        }
        if (active) {
            float* dqp = row_ptr(bd.dq, b * d.Tq + i) + h * HD;
#pragma unroll
            for (int t = 0; t < HD; ++t) dqp[t] += dq[t] * INV_SCALE;
        }
        return;
    }
    // ------------------------------------------------ pass B: lane = key row -> dK, dV, dS_prev, dc
    const int tb = blockIdx.x - d.B * nqt;
    const int b = tb / nkt, kt = tb - (tb / nkt) * nkt;
    const int k = kt * TILE + lane;
    const bool active = (h < d.H) && (k < d.Tk);
    float kk[HD], vv[HD], dk[HD], dv[HD];
    float maskv = 0.f, dc_acc = 0.f;
#pragma unroll
    for (int t = 0; t < HD; ++t) { dk[t] = 0.f; dv[t] = 0.f; }
    if (active) {
        load16u(kk, row_ptr(d.k, b * d.Tk + k) + h * HD);
        load16u(vv, row_ptr(d.v, b * d.Tk + k) + h * HD);
        maskv = reinterpret_cast<const float*>(d.mask)[(int64_t)b * d.mask_sB + k];
    }
    float* dsp = reinterpret_cast<float*>(bd.ds_prev);
    float* Qs = S1;
    float* Gs = S2;
    for (int r0 = 0; r0 < d.Tq; r0 += TILE) {
        __syncthreads();
        stage_rows(Qs, d.q, b, r0, d.Tq, d.Tq, D);
        stage_rows(Gs, bd.dx, b, r0, d.Tq, d.Tq, D);
        for (int idx = threadIdx.x; idx < TILE * d.H; idx += THREADS) {
            const int row = idx / d.H, hh = idx - (idx / d.H) * d.H;
            const int r = r0 + row;
            float mm = 0.f, li = 0.f, del = 0.f;
            if (r < d.Tq) {
                const float* st = stats + 2 * ((((int64_t)b * d.H + hh) * d.Tq) + r);
                mm = st[0];
                li = st[1];
                const float* g = row_ptr(bd.dx, b * d.Tq + r) + hh * HD;
                const float* xr = row_ptr(d.x, b * d.Tq + r) + hh * HD;
#pragma unroll
                for (int t = 0; t < HD; ++t) del = fmaf(g[t], xr[t], del);
            }
            Sm[(row * 8 + hh) * 3 + 0] = mm;
            Sm[(row * 8 + hh) * 3 + 1] = li;
            Sm[(row * 8 + hh) * 3 + 2] = del;
        }
        __syncthreads();
        if (!active) continue;
        const int nq = min(TILE, d.Tq - r0);
        for (int rr = 0; rr < nq; ++rr) {
            const int r = r0 + rr;
            const int64_t sidx = (((int64_t)b * d.H + h) * d.Tq + r) * d.Tk + k;
            const float* qr = Qs + rr * D + h * HD;
            const float* gr = Gs + rr * D + h * HD;
            const float spv = sc.has_prev ? sprev[sidx] : 0.f;
            const float s = score(qr, kk, sc, spv, maskv);
            const float* sm = Sm + (rr * 8 + h) * 3;
            const float p = __expf(s - sm[0]) * sm[1];
            float dp = 0.f;
#pragma unroll
            for (int t = 0; t < HD; ++t) dp = fmaf(gr[t], vv[t], dp);
            float ds = p * (dp - sm[2]);
            if (dsn) ds += dsn[sidx];
#pragma unroll
            for (int t = 0; t < HD; ++t) {
                dk[t] = fmaf(ds, qr[t], dk[t]);
                dv[t] = fmaf(p, gr[t], dv[t]);
            }
            if (sc.has_prev) {
                if (dsp) dsp[sidx] = sc.c * ds;
                dc_acc = fmaf(ds, spv, dc_acc);
            }
        }
    }
    if (active) {
        float* dkp = row_ptr(bd.dk, b * d.Tk + k) + h * HD;
        if (same_rows(bd.dk, bd.dv)) {
#pragma unroll
            for (int t = 0; t < HD; ++t) dkp[t] = dk[t] * INV_SCALE + dv[t];
        } else {
            float* dvp = row_ptr(bd.dv, b * d.Tk + k) + h * HD;
#pragma unroll
            for (int t = 0; t < HD; ++t) { dkp[t] = dk[t] * INV_SCALE; dvp[t] = dv[t]; }
        }
    }
    if (bd.dc_partial) {
        // reduce dc over lanes and heads of this workgroup (fixed order -> deterministic)
        __syncthreads();
        const float w = wave_sum(active ? dc_acc : 0.f);
        if (lane == 0) Sm[h] = w;
        __syncthreads();
        if (threadIdx.x == 0) {
            float s = 0.f;
            for (int hh = 0; hh < THREADS / 64; ++hh) s += Sm[hh];
            reinterpret_cast<float*>(bd.dc_partial)[b * nkt + kt] = s;
        }
    }
}

}  // namespace

extern "C" int mep_attn_fwd(const mep_attn_desc* descs, int n_desc, int max_tiles, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    hipLaunchKernelGGL(k_attn_fwd, dim3(max_tiles, n_desc), dim3(THREADS), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_attn_fwd");
}

extern "C" int mep_attn_bwd(const mep_attn_bwd_desc* descs, int n_desc, int max_tiles, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    hipLaunchKernelGGL(k_attn_bwd, dim3(max_tiles, n_desc), dim3(THREADS), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_attn_bwd");
}
