// Residual scaled-dot-product attention core, forward and backward, on f32 MFMA (hd = 16).
//
// Reference: Attention_Block.multi_head_attention, cmu-mosei/run.py:236-256 (identical in
// Ren-MME/run.py:188-208 and, after the w_qkv projections, others/realformer.py:182-204):
//   S = q k^T / sqrt(hd) [+ c * S_prev];  S -= 1e8 (1 - mask);  X = softmax(S) v
// The post-mask S is returned to the caller, which feeds it to the next layer of the chain.
//
// Mapping (CDNA4): one WAVE = one task (batch row b, head h, chunk of 64 queries [forward] or
// 64 keys [backward]); 4 independent waves per workgroup, no LDS staging, no barriers.  All
// products (S, P.V, dP, dV, dK, dQ) are v_mfma_f32_16x16x4_f32 (exact fp32 fma chains), with the
// operand layouts chosen so an accumulator feeds the next product without moving data:
//   forward   S^T = K Q^T  -> lane (query c, group g) holds keys 4g..4g+3 of its query, i.e.
//             exactly the A operand of O = P V.  Online softmax across 16-key tiles; the row
//             max/sum reduce over 4 registers + 2 lane-group shuffles.
//   backward  S = Q K^T and dP = dO V^T -> lane (key c, g) holds queries 4g..4g+3: the A operand
//             of dV += P^T dO and dK += dS^T Q directly; dQ += dS K needs dS with the query on
//             the lane, done by one 16x16 transpose through 1.3 KB of LDS per wave.
// Reduction dims are ordered (step s, lane group g) -> dim 4g+s, so every operand fetch is one
// 16-byte load and the forward and backward S are bitwise identical fma chains.
// Row statistics (max, 1/sum) are kept instead of log-sum-exp because fully masked rows sit at
// -1e8 where max + log(sum) would round the log away (ulp(1e8) = 8).
#include <float.h>

#include "common.h"

using namespace mep;

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int HD = 16;
constexpr int WAVES = 4;
constexpr int THREADS = 64 * WAVES;
constexpr int CH = 64;              // queries (forward) / keys (backward) per wave task
constexpr float INV_SCALE = 0.25f;  // 1/sqrt(16), exact

MEP_DEV floatx4 mfma16(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
MEP_DEV floatx4 zero4() { return floatx4{0.f, 0.f, 0.f, 0.f}; }

struct Score {
    bool has_prev;
    float c;
};

// s = dot * 0.25 [+ c*sp]  - 1e8 * (1 - m)      (op order of cmu-mosei/run.py:244-253)
MEP_DEV float score(float dot, const Score& sc, float sp, float m) {
    float s = mul_rn(dot, INV_SCALE);
    if (sc.has_prev) s = add_rn(s, mul_rn(sc.c, sp));
    return sub_rn(s, mul_rn(1.0e8f, sub_rn(1.0f, m)));
}

MEP_DEV bool aligned16(const mep_rows& r) {
    return ((r.ptr & 15) == 0) && (r.sB % 4 == 0) && (r.sT % 4 == 0);
}

// element (batch b, time t) of a row view whose T is the attention length: no division
MEP_DEV gfloat* at(const mep_rows& v, int b, int t) {
    return G<float>(v.ptr) + (int64_t)b * v.sB + (int64_t)t * v.sT;
}

// four consecutive floats of row t (clamped into [0, n), zeroed when t >= n) at column col;
// branch-free so the loads of a whole tile issue back to back
MEP_DEV void load4(float* dst, const mep_rows& v, int b, int t, int n, int col, bool vec) {
    const bool ok = t < n;
    const gfloat* p = at(v, b, ok ? t : n - 1) + col;
    float4 x;
    if (vec) x = ldg4(p);
    else x = make_float4(p[0], p[1], p[2], p[3]);
    dst[0] = ok ? x.x : 0.f; dst[1] = ok ? x.y : 0.f; dst[2] = ok ? x.z : 0.f; dst[3] = ok ? x.w : 0.f;
}
// one float of row t (clamped / zeroed as load4)
MEP_DEV float load1(const mep_rows& v, int b, int t, int n, int col) {
    const bool ok = t < n;
    const float x = at(v, b, ok ? t : n - 1)[col];
    return ok ? x : 0.f;
}

MEP_DEV float shfl(float v, int src) { return __shfl(v, src, 64); }

__global__ __launch_bounds__(THREADS) void k_attn_fwd(const mep_attn_desc* __restrict__ descs) {
    const mep_attn_desc& d = descs[blockIdx.y];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int nqc = (d.Tq + CH - 1) / CH;
    const int task = blockIdx.x * WAVES + wave;
    if (task >= d.B * d.H * nqc) return;   // whole wave leaves; no barriers below
    const int qc = task % nqc, bh = task / nqc;
    const int h = bh % d.H, b = bh / d.H;
    const int hc = h * HD;
    const Score sc{d.s_prev != 0, d.s_prev ? *G<const float>(d.c) : 0.f};
    const gfloat* sprev = G<const float>(d.s_prev);
    gfloat* sout = G<float>(d.s_out);
    const gfloat* mask = G<const float>(d.mask) + (int64_t)b * d.mask_sB;
    const bool qv = aligned16(d.q), kv4 = aligned16(d.k);
    const int64_t sbase = ((int64_t)b * d.H + h) * d.Tq;

    // B operand of S^T = K Q^T: lane (query c, group g), dims 4g..4g+3 of 4 query tiles
    float qf[4][4];
    const int q_lo = qc * CH;
    const int nqt = min(4, (d.Tq - q_lo + 15) / 16);
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) load4(qf[qt], d.q, b, q_lo + qt * 16 + c, d.Tq, hc + 4 * g, qv);

    floatx4 o[4];
    float m[4], l[4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) { o[qt] = zero4(); m[qt] = -FLT_MAX; l[qt] = 0.f; }

    const int nkt = (d.Tk + 15) / 16;
    for (int kt = 0; kt < nkt; ++kt) {
        const int k0 = kt * 16;
        float kf[4], vf[4], mk[4];
        load4(kf, d.k, b, k0 + c, d.Tk, hc + 4 * g, kv4);               // A: K[k0+c][4g+s]
#pragma unroll
        for (int s = 0; s < 4; ++s) {                                   // B of P.V: V[k0+4g+s][c]
            const int kk = k0 + 4 * g + s;
            vf[s] = load1(d.v, b, kk, d.Tk, hc + c);
            const float mv = mask[min(kk, d.Tk - 1)];
            mk[s] = kk < d.Tk ? mv : 0.f;
        }
#pragma unroll
        for (int qt = 0; qt < 4; ++qt) {
            if (qt >= nqt) break;
            floatx4 st = zero4();
#pragma unroll
            for (int s = 0; s < 4; ++s) st = mfma16(kf[s], qf[qt][s], st);   // C[key 4g+r][query c]
            const int q = q_lo + qt * 16 + c;
            const bool qok = q < d.Tq;
            float sv[4], mx = -INFINITY;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int kk = k0 + 4 * g + r;
                if (kk < d.Tk) {
                    const int64_t si = (sbase + q) * d.Tk + kk;
                    sv[r] = score(st[r], sc, (sc.has_prev && qok) ? sprev[si] : 0.f, mk[r]);
                    if (sout && qok) sout[si] = sv[r];
                } else {
                    sv[r] = -INFINITY;
                }
                mx = fmaxf(mx, sv[r]);
            }
            mx = fmaxf(mx, shfl(mx, lane ^ 16));
            mx = fmaxf(mx, shfl(mx, lane ^ 32));
            const float mnew = fmaxf(m[qt], mx);
            const float corr = __expf(m[qt] - mnew);
            float p[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) p[r] = __expf(sv[r] - mnew);
            l[qt] = l[qt] * corr + ((p[0] + p[1]) + (p[2] + p[3]));
            m[qt] = mnew;
#pragma unroll
            for (int r = 0; r < 4; ++r) o[qt][r] *= shfl(corr, 4 * g + r);  // O row 4g+r <- corr of query 4g+r
#pragma unroll
            for (int s = 0; s < 4; ++s) o[qt] = mfma16(p[s], vf[s], o[qt]);  // C[query 4g+r][dim c]
        }
    }
    gfloat* stats = G<float>(d.stats);
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
        if (qt >= nqt) break;
        float lt = l[qt] + shfl(l[qt], lane ^ 16);
        lt += shfl(lt, lane ^ 32);
        const float inv = 1.0f / lt;
        const int q = q_lo + qt * 16 + c;
        if (g == 0 && q < d.Tq) {
            stats[2 * (sbase + q)] = m[qt];
            stats[2 * (sbase + q) + 1] = inv;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float ir = shfl(inv, 4 * g + r);
            const int qq = q_lo + qt * 16 + 4 * g + r;
            if (qq < d.Tq) (at(d.x, b, qq))[hc + c] = o[qt][r] * ir;
        }
    }
}

MEP_DEV void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(THREADS) void k_attn_bwd(const mep_attn_bwd_desc* __restrict__ descs) {
    const mep_attn_bwd_desc& bd = descs[blockIdx.y];
    const mep_attn_desc& d = bd.f;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int nkc = (d.Tk + CH - 1) / CH;
    const int task = blockIdx.x * WAVES + wave;
    __shared__ __attribute__((aligned(16))) float Tr[WAVES][16 * 20];
    if (task >= d.B * d.H * nkc) return;   // whole wave leaves; only wave-private LDS below
    const int kc = task % nkc, bh = task / nkc;
    const int h = bh % d.H, b = bh / d.H;
    const int hc = h * HD;
    const Score sc{d.s_prev != 0, d.s_prev ? *G<const float>(d.c) : 0.f};
    const gfloat* sprev = G<const float>(d.s_prev);
    const gfloat* dsn = G<const float>(bd.ds_next);
    gfloat* dsp = G<float>(bd.ds_prev);
    const gfloat* stats = G<const float>(d.stats);
    const gfloat* mask = G<const float>(d.mask) + (int64_t)b * d.mask_sB;
    const int64_t sbase = ((int64_t)b * d.H + h) * d.Tq;
    const bool qv = aligned16(d.q), kv4 = aligned16(d.k), vv4 = aligned16(d.v), gv = aligned16(bd.dx);
    float* T = Tr[wave];

    const int k_lo = kc * CH;
    const int nkt = min(4, (d.Tk - k_lo + 15) / 16);
    // per key tile: B operands of S (K) and dP (V) with the key on the lane, the key mask, and
    // the B operand of dQ (K rows 4g+s, dim c); dK / dV accumulators (C[key 4g+r][dim c])
    float kb[4][4], vb[4][4], kq[4][4], mkey[4];
    floatx4 dk[4], dv[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
        const int k0 = k_lo + kt * 16;
        load4(kb[kt], d.k, b, k0 + c, d.Tk, hc + 4 * g, kv4);
        load4(vb[kt], d.v, b, k0 + c, d.Tk, hc + 4 * g, vv4);
        const float mv = mask[min(k0 + c, d.Tk - 1)];
        mkey[kt] = (k0 + c < d.Tk) ? mv : 0.f;
#pragma unroll
        for (int s = 0; s < 4; ++s) kq[kt][s] = load1(d.k, b, k0 + 4 * g + s, d.Tk, hc + c);
        dk[kt] = zero4();
        dv[kt] = zero4();
    }
    float dc_acc = 0.f;
    const int nqt = (d.Tq + 15) / 16;
    for (int qt = 0; qt < nqt; ++qt) {
        const int q0 = qt * 16;
        float qa[4], da[4], db[4], qb[4], mm[4], li[4], del[4];
        load4(qa, d.q, b, q0 + c, d.Tq, hc + 4 * g, qv);                // A of S: Q[q0+c][4g+s]
        load4(da, bd.dx, b, q0 + c, d.Tq, hc + 4 * g, gv);              // A of dP: dO[q0+c][4g+s]
#pragma unroll
        for (int s = 0; s < 4; ++s) {                                  // B of dV / dK: rows 4g+s, dim c
            const int qq = q0 + 4 * g + s;
            const bool ok = qq < d.Tq;
            const int qc2 = ok ? qq : d.Tq - 1;
            db[s] = load1(bd.dx, b, qq, d.Tq, hc + c);
            qb[s] = load1(d.q, b, qq, d.Tq, hc + c);
            const float ov = load1(d.x, b, qq, d.Tq, hc + c);
            float pr = db[s] * ov;                                     // delta = rowsum(dO * O)
            pr += shfl(pr, lane ^ 1);
            pr += shfl(pr, lane ^ 2);
            pr += shfl(pr, lane ^ 4);
            pr += shfl(pr, lane ^ 8);
            del[s] = pr;
            const float m0 = stats[2 * (sbase + qc2)], l0 = stats[2 * (sbase + qc2) + 1];
            mm[s] = ok ? m0 : 0.f;
            li[s] = ok ? l0 : 0.f;
        }
        floatx4 dq = zero4();
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            if (kt >= nkt) break;
            const int kk = k_lo + kt * 16 + c;
            floatx4 st = zero4(), dp = zero4();
#pragma unroll
            for (int s = 0; s < 4; ++s) st = mfma16(qa[s], kb[kt][s], st);   // C[query 4g+r][key c]
#pragma unroll
            for (int s = 0; s < 4; ++s) dp = mfma16(da[s], vb[kt][s], dp);
            float p[4], ds[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int qq = q0 + 4 * g + r;
                const bool ok = (qq < d.Tq) && (kk < d.Tk);
                const int64_t si = (sbase + qq) * d.Tk + kk;
                const float spv = (sc.has_prev && ok) ? sprev[si] : 0.f;
                const float sv = score(st[r], sc, spv, mkey[kt]);
                const float pv = ok ? __expf(sv - mm[r]) * li[r] : 0.f;
                float gsv = pv * (dp[r] - del[r]);
                if (dsn && ok) gsv += dsn[si];
                gsv = ok ? gsv : 0.f;
                if (sc.has_prev && ok) {
                    if (dsp) dsp[si] = sc.c * gsv;
                    dc_acc = fmaf(gsv, spv, dc_acc);
                }
                p[r] = pv;
                ds[r] = gsv;
            }
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                dv[kt] = mfma16(p[s], db[s], dv[kt]);     // dV[key][dim] += P^T dO
                dk[kt] = mfma16(ds[s], qb[s], dk[kt]);    // dK[key][dim] += dS^T Q
            }
            // dQ += dS K: transpose dS (query 4g+r on lane c=key) to the query-on-lane A layout
#pragma unroll
            for (int r = 0; r < 4; ++r) T[(4 * g + r) * 20 + c] = ds[r];
            wave_lds_sync();
            const float4 t4 = *reinterpret_cast<const float4*>(T + c * 20 + 4 * g);
            wave_lds_sync();
            dq = mfma16(t4.x, kq[kt][0], dq);
            dq = mfma16(t4.y, kq[kt][1], dq);
            dq = mfma16(t4.z, kq[kt][2], dq);
            dq = mfma16(t4.w, kq[kt][3], dq);
        }
        // dq rows q0+4g+r, dim c (exclusive owner when the keys fit one chunk; else atomics)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int qq = q0 + 4 * g + r;
            if (qq < d.Tq) {
                gfloat* dqp = at(bd.dq, b, qq) + hc + c;
                if (nkc == 1) *dqp += dq[r] * INV_SCALE;
                else atomicAdd(reinterpret_cast<float*>(reinterpret_cast<uintptr_t>(dqp)), dq[r] * INV_SCALE);
            }
        }
    }
    const bool same_kv = bd.dk.ptr == bd.dv.ptr && bd.dk.sB == bd.dv.sB && bd.dk.sT == bd.dv.sT;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
        if (kt >= nkt) break;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int kk = k_lo + kt * 16 + 4 * g + r;
            if (kk >= d.Tk) continue;
            gfloat* dkp = at(bd.dk, b, kk) + hc + c;
            if (same_kv) {
                *dkp = dk[kt][r] * INV_SCALE + dv[kt][r];
            } else {
                *dkp = dk[kt][r] * INV_SCALE;
                (at(bd.dv, b, kk))[hc + c] = dv[kt][r];
            }
        }
    }
    if (bd.dc_partial) {
        const float w = wave_sum(dc_acc);
        if (lane == 0) G<float>(bd.dc_partial)[task] = w;
    }
}

}  // namespace

// Launch geometry: 256 threads (4 waves, one task each); tasks = B * H * ceil(Tq/64) forward,
// B * H * ceil(Tk/64) backward; max_tiles = ceil(max tasks / 4).  dc_partial (backward) has one
// float per task, task = (b*H + h) * ceil(Tk/64) + key chunk.
extern "C" int mep_attn_fwd(const mep_attn_desc* descs, int n_desc, int max_tiles, int threads, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    if (threads != THREADS) { mep_set_error("mep_attn_fwd: threads must be 256"); return MEP_EINVAL; }
    hipLaunchKernelGGL(k_attn_fwd, dim3(max_tiles, n_desc), dim3(THREADS), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_attn_fwd");
}

extern "C" int mep_attn_bwd(const mep_attn_bwd_desc* descs, int n_desc, int max_tiles, int threads,
                            mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    if (threads != THREADS) { mep_set_error("mep_attn_bwd: threads must be 256"); return MEP_EINVAL; }
    hipLaunchKernelGGL(k_attn_bwd, dim3(max_tiles, n_desc), dim3(THREADS), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_attn_bwd");
}
