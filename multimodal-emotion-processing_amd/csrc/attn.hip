// Residual scaled-dot-product attention core, forward and backward (fp32, hd = 16).
//
// Reference: Attention_Block.multi_head_attention, cmu-mosei/run.py:236-256 (identical in
// Ren-MME/run.py:188-208 and, after the w_qkv projections, others/realformer.py:182-204):
//   S = q k^T / sqrt(hd) [+ c * S_prev];  S -= 1e8 (1 - mask);  X = softmax(S) v
// The post-mask S is returned to the caller, which feeds it to the next layer of the chain.
//
// Mapping (CDNA4): one workgroup = (batch row, tile of R = 512/H rows); each LANE owns one
// (row, head) pair, lane = row*H + head, so a row's 16-float head slices are contiguous across
// neighbouring lanes (coalesced q / x / dq traffic) and no lane idles on H = 6.  The softmax row
// max / sum never cross lanes.  K/V tiles of 64 keys (or, in pass B, Q/dX tiles of 64 queries)
// are staged in LDS; lanes of one head read the same address (broadcast) and the H heads hit
// disjoint banks.  hd = 16 operands live in registers; dots are split into 4 independent FMA
// chains and keys are processed 4-8 at a time so the VALU pipeline has independent work.
// Row statistics (max, 1/sum) are kept instead of log-sum-exp because fully masked rows sit at
// -1e8 where max + log(sum) would round the log away (ulp(1e8) = 8).
#include <float.h>

#include "common.h"

using namespace mep;

namespace {

constexpr int HD = 16;
constexpr int MAXT = 512;        // threads per workgroup (upper bound; launch uses <= this)
constexpr int TILE = 64;         // staged keys (fwd / pass A) or queries (pass B) per LDS tile
constexpr int DMAX = 128;        // H*HD <= 128
constexpr float INV_SCALE = 0.25f;  // 1/sqrt(16), exact
constexpr int UA = 2;            // keys per step, backward pass A
constexpr int UB = 2;            // queries per step, backward pass B

struct Score {
    bool has_prev;
    float c;
};

// q . k with four independent FMA chains (identical in forward and both backward passes, so
// the recomputed probabilities match the forward bit for bit)
MEP_DEV float dot16(const float* a, const float* b) {
    float d0 = 0.f, d1 = 0.f, d2 = 0.f, d3 = 0.f;
#pragma unroll
    for (int i = 0; i < HD; i += 4) {
        d0 = fmaf(a[i], b[i], d0);
        d1 = fmaf(a[i + 1], b[i + 1], d1);
        d2 = fmaf(a[i + 2], b[i + 2], d2);
        d3 = fmaf(a[i + 3], b[i + 3], d3);
    }
    return (d0 + d1) + (d2 + d3);
}

// s = (q.k) * 0.25 [+ c*sp]  - 1e8 * (1 - m)      (op order of cmu-mosei/run.py:244-253)
MEP_DEV float score(const float* q, const float* k, const Score& sc, float sp, float m) {
    float s = mul_rn(dot16(q, k), INV_SCALE);
    if (sc.has_prev) s = add_rn(s, mul_rn(sc.c, sp));
    return sub_rn(s, mul_rn(1.0e8f, sub_rn(1.0f, m)));
}

MEP_DEV void load16(float* dst, const float* src) {
#pragma unroll
    for (int i = 0; i < HD; ++i) dst[i] = src[i];
}

// stage rows [r0, r0+64) of a row view (batch row b) into LDS [64][D]
MEP_DEV void stage_rows(float* dst, const mep_rows& src, int b, int r0, int nrows, int T, int D) {
    for (int idx = threadIdx.x; idx < TILE * D; idx += blockDim.x) {
        const int row = idx / D, col = idx - row * D;
        const int r = r0 + row;
        dst[idx] = (r < nrows) ? row_ptr(src, b * T + r)[col] : 0.f;
    }
}

MEP_DEV bool same_rows(const mep_rows& a, const mep_rows& b) {
    return a.ptr == b.ptr && a.sB == b.sB && a.sT == b.sT && a.T == b.T;
}

MEP_DEV int rows_per_tile(int H) { return MAXT / H; }

__global__ __launch_bounds__(MAXT) void k_attn_fwd(const mep_attn_desc* __restrict__ descs) {
    const mep_attn_desc& d = descs[blockIdx.y];
    const int R = rows_per_tile(d.H);
    const int nqt = (d.Tq + R - 1) / R;
    if ((int)blockIdx.x >= d.B * nqt) return;
    const int b = blockIdx.x / nqt, qt = blockIdx.x - (blockIdx.x / nqt) * nqt;
    const int D = d.H * HD;
    const int row = threadIdx.x / d.H, h = threadIdx.x - row * d.H;
    const int i = qt * R + row;
    const bool active = (row < R) && (i < d.Tq);
    const bool kv_same = same_rows(d.k, d.v);

    __shared__ __attribute__((aligned(16))) float Ks[TILE * DMAX];
    __shared__ __attribute__((aligned(16))) float Vs[TILE * DMAX];
    __shared__ float Ms[TILE];

    const Score sc{d.s_prev != 0, d.s_prev ? *reinterpret_cast<const float*>(d.c) : 0.f};
    float q[HD], o[HD];
    float m = -FLT_MAX, l = 0.f;
#pragma unroll
    for (int t = 0; t < HD; ++t) o[t] = 0.f;
    const int64_t srow = (((int64_t)b * d.H + h) * d.Tq + i) * d.Tk;
    const float* sprev = reinterpret_cast<const float*>(d.s_prev);
    float* sout = reinterpret_cast<float*>(d.s_out);
    if (active) load16(q, row_ptr(d.q, b * d.Tq + i) + h * HD);
    const float* mask = reinterpret_cast<const float*>(d.mask) + (int64_t)b * d.mask_sB;
    const float* Vsrc = kv_same ? Ks : Vs;

    for (int k0 = 0; k0 < d.Tk; k0 += TILE) {
        __syncthreads();
        stage_rows(Ks, d.k, b, k0, d.Tk, d.Tk, D);
        if (!kv_same) stage_rows(Vs, d.v, b, k0, d.Tk, d.Tk, D);
        if ((int)threadIdx.x < TILE) Ms[threadIdx.x] = (k0 + (int)threadIdx.x < d.Tk) ? mask[k0 + threadIdx.x] : 0.f;
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
                const float p = (k < nk) ? __expf(s[j] - mnew) : 0.f;
                l += p;
                const float* vr = Vsrc + min(k, nk - 1) * D + h * HD;
#pragma unroll
                for (int t = 0; t < HD; ++t) o[t] = fmaf(p, vr[t], o[t]);
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

__global__ __launch_bounds__(MAXT) void k_attn_bwd(const mep_attn_bwd_desc* __restrict__ descs) {
    const mep_attn_bwd_desc& bd = descs[blockIdx.y];
    const mep_attn_desc& d = bd.f;
    const int R = rows_per_tile(d.H);
    const int nqt = (d.Tq + R - 1) / R, nkt = (d.Tk + R - 1) / R;
    if ((int)blockIdx.x >= d.B * (nqt + nkt)) return;
    const int D = d.H * HD;
    const int row = threadIdx.x / d.H, h = threadIdx.x - row * d.H;
    const bool kv_same = same_rows(d.k, d.v);
    const Score sc{d.s_prev != 0, d.s_prev ? *reinterpret_cast<const float*>(d.c) : 0.f};
    const float* sprev = reinterpret_cast<const float*>(d.s_prev);
    const float* dsn = reinterpret_cast<const float*>(bd.ds_next);
    const float* stats = reinterpret_cast<const float*>(d.stats);

    __shared__ __attribute__((aligned(16))) float S1[TILE * DMAX];
    __shared__ __attribute__((aligned(16))) float S2[TILE * DMAX];
    __shared__ float Sm[TILE * 8 * 3];   // pass B: (max, 1/sum, delta) per (row, head); pass A: mask
    __shared__ float Red[MAXT / 64];

    if ((int)blockIdx.x < d.B * nqt) {
        // ------------------------------------------------ pass A: lane = (query row, head) -> dQ
        const int b = blockIdx.x / nqt, qt = blockIdx.x - b * nqt;
        const int i = qt * R + row;
        const bool active = (row < R) && (i < d.Tq);
        float q[HD], dout[HD], dq[HD];
        float delta = 0.f, m = 0.f, linv = 0.f;
#pragma unroll
        for (int t = 0; t < HD; ++t) dq[t] = 0.f;
        const int64_t srow = (((int64_t)b * d.H + h) * d.Tq + i) * d.Tk;
        if (active) {
            load16(q, row_ptr(d.q, b * d.Tq + i) + h * HD);
            load16(dout, row_ptr(bd.dx, b * d.Tq + i) + h * HD);
            delta = dot16(dout, row_ptr(d.x, b * d.Tq + i) + h * HD);
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
            if ((int)threadIdx.x < TILE) Sm[threadIdx.x] = (k0 + (int)threadIdx.x < d.Tk) ? mask[k0 + threadIdx.x] : 0.f;
            __syncthreads();
            if (!active) continue;
            const int nk = min(TILE, d.Tk - k0);
            for (int kb = 0; kb < nk; kb += UA) {
                float ds[UA];
#pragma unroll
                for (int j = 0; j < UA; ++j) {
                    const int k = min(kb + j, nk - 1);
                    const float* kr = Ks + k * D + h * HD;
                    const float* vr = Vs + k * D + h * HD;
                    const float s = score(q, kr, sc, sc.has_prev ? sprev[srow + k0 + k] : 0.f, Sm[k]);
                    const float p = __expf(s - m) * linv;
                    float g = p * (dot16(dout, vr) - delta);
                    if (dsn) g += dsn[srow + k0 + k];
                    ds[j] = (kb + j < nk) ? g : 0.f;
                }
#pragma unroll
                for (int j = 0; j < UA; ++j) {
                    const float* kr = Ks + min(kb + j, nk - 1) * D + h * HD;
#pragma unroll
                    for (int t = 0; t < HD; ++t) dq[t] = fmaf(ds[j], kr[t], dq[t]);
                }
            }
        }
        if (active) {
            float* dqp = row_ptr(bd.dq, b * d.Tq + i) + h * HD;
#pragma unroll
            for (int t = 0; t < HD; ++t) dqp[t] += dq[t] * INV_SCALE;
        }
        return;
    }
    // ------------------------------------------------ pass B: lane = (key row, head) -> dK, dV, dS_prev, dc
    const int tb = blockIdx.x - d.B * nqt;
    const int b = tb / nkt, kt = tb - (tb / nkt) * nkt;
    const int k = kt * R + row;
    const bool active = (row < R) && (k < d.Tk);
    float kk[HD], vv[HD], dk[HD], dv[HD];
    float maskv = 0.f, dc_acc = 0.f;
#pragma unroll
    for (int t = 0; t < HD; ++t) { dk[t] = 0.f; dv[t] = 0.f; }
    if (active) {
        load16(kk, row_ptr(d.k, b * d.Tk + k) + h * HD);
        load16(vv, row_ptr(d.v, b * d.Tk + k) + h * HD);
        maskv = reinterpret_cast<const float*>(d.mask)[(int64_t)b * d.mask_sB + k];
    }
    float* dsp = reinterpret_cast<float*>(bd.ds_prev);
    float* Qs = S1;
    float* Gs = S2;
    for (int r0 = 0; r0 < d.Tq; r0 += TILE) {
        __syncthreads();
        stage_rows(Qs, d.q, b, r0, d.Tq, d.Tq, D);
        stage_rows(Gs, bd.dx, b, r0, d.Tq, d.Tq, D);
        for (int idx = threadIdx.x; idx < TILE * d.H; idx += blockDim.x) {
            const int rr = idx / d.H, hh = idx - (idx / d.H) * d.H;
            const int r = r0 + rr;
            float mm = 0.f, li = 0.f, del = 0.f;
            if (r < d.Tq) {
                const float* st = stats + 2 * ((((int64_t)b * d.H + hh) * d.Tq) + r);
                mm = st[0];
                li = st[1];
                del = dot16(row_ptr(bd.dx, b * d.Tq + r) + hh * HD, row_ptr(d.x, b * d.Tq + r) + hh * HD);
            }
            Sm[(rr * 8 + hh) * 3 + 0] = mm;
            Sm[(rr * 8 + hh) * 3 + 1] = li;
            Sm[(rr * 8 + hh) * 3 + 2] = del;
        }
        __syncthreads();
        if (!active) continue;
        const int nq = min(TILE, d.Tq - r0);
        for (int rb = 0; rb < nq; rb += UB) {
            float ds[UB], p[UB];
#pragma unroll
            for (int j = 0; j < UB; ++j) {
                const int rr = min(rb + j, nq - 1);
                const int r = r0 + rr;
                const int64_t sidx = (((int64_t)b * d.H + h) * d.Tq + r) * d.Tk + k;
                const float* qr = Qs + rr * D + h * HD;
                const float* gr = Gs + rr * D + h * HD;
                const float spv = sc.has_prev ? sprev[sidx] : 0.f;
                const float s = score(qr, kk, sc, spv, maskv);
                const float* sm = Sm + (rr * 8 + h) * 3;
                const bool ok = rb + j < nq;
                const float pj = ok ? __expf(s - sm[0]) * sm[1] : 0.f;
                float g = pj * (dot16(gr, vv) - sm[2]);
                if (dsn) g += ok ? dsn[sidx] : 0.f;
                p[j] = pj;
                ds[j] = ok ? g : 0.f;
                if (sc.has_prev && ok) {
                    if (dsp) dsp[sidx] = sc.c * g;
                    dc_acc = fmaf(g, spv, dc_acc);
                }
            }
#pragma unroll
            for (int j = 0; j < UB; ++j) {
                const int rr = min(rb + j, nq - 1);
                const float* qr = Qs + rr * D + h * HD;
                const float* gr = Gs + rr * D + h * HD;
#pragma unroll
                for (int t = 0; t < HD; ++t) {
                    dk[t] = fmaf(ds[j], qr[t], dk[t]);
                    dv[t] = fmaf(p[j], gr[t], dv[t]);
                }
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
        // reduce dc over the lanes of this workgroup (fixed order -> deterministic)
        const float w = wave_sum(active ? dc_acc : 0.f);
        if ((threadIdx.x & 63) == 0) Red[threadIdx.x >> 6] = w;
        __syncthreads();
        if (threadIdx.x == 0) {
            float s = 0.f;
            for (int ww = 0; ww < (int)(blockDim.x >> 6); ++ww) s += Red[ww];
            reinterpret_cast<float*>(bd.dc_partial)[b * nkt + kt] = s;
        }
    }
}

}  // namespace

// threads: 64 * ceil(H * min(T, 512/H) / 64) of the largest descriptor (the host knows the
// shapes); max_tiles: max over descriptors of B * ceil(Tq / (512/H))  [+ B * ceil(Tk / (512/H))
// for the backward].
extern "C" int mep_attn_fwd(const mep_attn_desc* descs, int n_desc, int max_tiles, int threads, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    if (threads <= 0 || threads > MAXT || threads % 64) { mep_set_error("mep_attn_fwd: threads"); return MEP_EINVAL; }
    hipLaunchKernelGGL(k_attn_fwd, dim3(max_tiles, n_desc), dim3(threads), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_attn_fwd");
}

extern "C" int mep_attn_bwd(const mep_attn_bwd_desc* descs, int n_desc, int max_tiles, int threads,
                            mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    if (threads <= 0 || threads > MAXT || threads % 64) { mep_set_error("mep_attn_bwd: threads"); return MEP_EINVAL; }
    hipLaunchKernelGGL(k_attn_bwd, dim3(max_tiles, n_desc), dim3(threads), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_attn_bwd");
}
