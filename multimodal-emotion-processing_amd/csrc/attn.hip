// Residual scaled-dot-product attention core, forward and backward, on f32 MFMA (hd = 16).
//
// Reference: Attention_Block.multi_head_attention, cmu-mosei/run.py:236-256 (identical in
// Ren-MME/run.py:188-208 and, after the w_qkv projections, others/realformer.py:182-204):
//   S = q k^T / sqrt(hd) [+ c * S_prev];  S -= 1e8 (1 - mask);  X = softmax(S) v
// The post-mask S is returned to the caller, which feeds it to the next layer of the chain.
//
// Mapping (CDNA4): one WAVE = one task (batch row b, head h, chunk of 64 queries [forward] or
// 64 keys [backward]); 4 independent waves per workgroup, no barriers.  All products (S, P.V, dP,
// dV, dK, dQ) are v_mfma_f32_16x16x4_f32 (exact fp32 fma chains), with operand layouts chosen so
// an accumulator feeds the next product without moving data:
//   forward   S^T = K Q^T  -> lane (query c, group g) holds keys 4g..4g+3 of each 16-key tile,
//             i.e. exactly the A operand of O = P V.  Keys are processed in chunks of 64 (4 tiles,
//             16 scores per lane per query tile): one row max / rescale per chunk, so for the
//             common T <= 64 the softmax is exact two-pass with no rescaling at all.
//   backward  S = Q K^T and dP = dO V^T -> lane (key c, g) holds queries 4g..4g+3: the A operand
//             of dV += P^T dO and dK += dS^T Q directly; dQ += dS K needs dS with the query on
//             the lane: one 16 x 64 transpose through LDS per query tile.
// Reduction dims are ordered (step s, lane group g) -> dim 4g+s, so every operand fetch is one
// 16-byte load and the forward and backward S are bitwise identical fma chains.  Validity
// (padded rows / keys) is handled with clamped loads and selects, never branches.
// Row statistics (max, 1/sum) are kept instead of log-sum-exp because fully masked rows sit at
// -1e8 where max + log(sum) would round the log away (ulp(1e8) = 8).
#include <float.h>

#include "common.h"

using namespace mep;

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int HD = 16;
constexpr int WAVES = 4;
constexpr int THREADS = 64 * WAVES;
constexpr int CH = 64;              // queries (forward) / keys (backward) per wave task
constexpr int NT = CH / 16;         // 16-row tiles per chunk
constexpr float INV_SCALE = 0.25f;  // 1/sqrt(16), exact
constexpr int TLD = CH + 4;         // LDS row stride of the dS transpose

MEP_DEV floatx4 mfma16(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
MEP_DEV floatx4 zero4() { return floatx4{0.f, 0.f, 0.f, 0.f}; }

MEP_DEV bool aligned16(const mep_rows& r) {
    return ((r.ptr & 15) == 0) && (r.sB % 4 == 0) && (r.sT % 4 == 0);
}

// base of batch row b of a row view (wave-uniform, 64-bit) -- rows are then addressed with
// 32-bit per-lane offsets t * sT
MEP_DEV gfloat* bat(const mep_rows& v, int b) { return G<float>(v.ptr) + (int64_t)b * v.sB; }

// four consecutive floats of row min(t, n-1) at column col.  Rows past the end are never
// zeroed: a padded key's score is -inf (its mask term is +inf), so its P and dS are exactly 0
// whatever K/V hold there, and padded queries are never stored (forward) or carry P = 0
// (backward); clamping keeps every load in bounds and every value finite.
MEP_DEV void load4(float* dst, const gfloat* base, int sT, int t, int n, int col, bool vec) {
    const gfloat* p = base + min(t, n - 1) * sT + col;
    float4 x;
    if (vec) x = ldg4(p);
    else x = make_float4(p[0], p[1], p[2], p[3]);
    dst[0] = x.x; dst[1] = x.y; dst[2] = x.z; dst[3] = x.w;
}
MEP_DEV float load1(const gfloat* base, int sT, int t, int n, int col) {
    return base[min(t, n - 1) * sT + col];
}

// per-key mask term of the score: 1e8 * (1 - mask) (cmu-mosei/run.py:253), +inf for padding keys
// beyond Tk so that s - term = -inf and exp() = 0 without any per-score select
MEP_DEV float mask_term(const gfloat* mask, int k, int Tk) {
    const float m = mask[min(k, Tk - 1)];
    return k < Tk ? mul_rn(1.0e8f, sub_rn(1.0f, m)) : INFINITY;
}

MEP_DEV float shfl(float v, int src) { return __shfl(v, src, 64); }

// s = dot * 0.25 [+ c*sp] - 1e8 * (1 - m)      (op order of cmu-mosei/run.py:244-253)
template <bool PREV>
MEP_DEV float score(float dot, float c, float sp, float mt) {
    float s = mul_rn(dot, INV_SCALE);
    if (PREV) s = add_rn(s, mul_rn(c, sp));
    return sub_rn(s, mt);
}

// One batch row of a row view as a range-checked buffer (csrc/common.h raw buffer ops): row t,
// column col at byte t * sT + 4 col.  Rows t >= n lie past the range (every view has sT >= its
// D used columns), so their loads return 0 and their stores are dropped -- no clamps, no
// branches, 32-bit offsets.  The base is wave-uniform by construction (one (b, h) per wave);
// readfirstlane makes that provable so the descriptor lives in SGPRs.
struct BRow {
    __amdgpu_buffer_rsrc_t rs;
    int sT4;   // row stride in bytes (wave-uniform)
    bool vec;  // 16-byte loads allowed
    // byte offset of (row t, column col); loads / stores take a per-lane part plus a wave-uniform
    // part (SGPR soffset: whole rows ahead), so row steps cost no vector instructions
    MEP_DEV int at(int t, int col) const { return t * sT4 + 4 * col; }
    MEP_DEV float ld1(int voff, int soff = 0) const {
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0));
    }
    MEP_DEV void ld4(float* dst, int voff) const {
        if (vec) {
            const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0));
            dst[0] = v[0]; dst[1] = v[1]; dst[2] = v[2]; dst[3] = v[3];
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) dst[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff + 4 * e, 0, 0));
        }
    }
    MEP_DEV void st1(int voff, int soff, float v) const {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rs, voff, soff, 0);
    }
};

MEP_DEV __amdgpu_buffer_rsrc_t uniform_rsrc(uint64_t base, int64_t bytes) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)base);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(base >> 32));
    const int n = __builtin_amdgcn_readfirstlane((int)min(bytes, (int64_t)0x7fffffff));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}

// rows [0, n) of batch row b of a view whose used columns are [0, D)
MEP_DEV BRow brow(const mep_rows& v, int b, int n, int D) {
    return BRow{uniform_rsrc(v.ptr + 4ull * (uint64_t)((int64_t)b * v.sB), 4 * ((int64_t)(n - 1) * v.sT + D)),
                4 * (int)v.sT, aligned16(v)};
}

// One forward task: batch row b, head h, 64 queries.  PREV: residual scores in; SOUT: post-mask
// scores out; SINGLE: Tk <= 64 (one key chunk: exact two-pass softmax, each query tile is
// finalised right after its P.V, so no running O/max/sum state stays live).
template <bool PREV, bool SOUT, bool SINGLE>
MEP_DEV void attn_fwd_task(const mep_attn_desc& d, int qc, int h, int b, int lane) {
    const int c = lane & 15, g = lane >> 4;
    const int hc = h * HD;
    const int Tq = d.Tq, Tk = d.Tk;
    const float cres = PREV ? *G<const float>(d.c) : 0.f;
    const gfloat* sprev = G<const float>(d.s_prev);
    gfloat* sout = G<float>(d.s_out);
    const gfloat* mask = G<const float>(d.mask) + (int64_t)b * d.mask_sB;
    const int D = d.H * HD;
    const BRow Qb = brow(d.q, b, Tq, D), Kb = brow(d.k, b, Tk, D), Vb = brow(d.v, b, Tk, D), Xb = brow(d.x, b, Tq, D);
    const int sbase = (b * d.H + h) * Tq;        // row of (b, h, query 0) in [B,H,Tq,Tk]
    const int q_lo = qc * CH;
    const int nqt = min(NT, (Tq - q_lo + 15) / 16);
    gfloat* stats = G<float>(d.stats);

    floatx4 o[SINGLE ? 1 : NT];
    float m[SINGLE ? 1 : NT], l[SINGLE ? 1 : NT];
    if (!SINGLE) {
#pragma unroll
        for (int qt = 0; qt < NT; ++qt) { o[qt] = zero4(); m[qt] = -FLT_MAX; l[qt] = 0.f; }
    }
    auto finish = [&](int qt, const floatx4& oq, float mq, float lq) {
        float lt = lq + shfl(lq, lane ^ 16);
        lt += shfl(lt, lane ^ 32);
        const float inv = 1.0f / lt;
        const int q = q_lo + qt * 16 + c;
        if (g == 0 && q < Tq) {
            stats[2 * (sbase + q)] = mq;
            stats[2 * (sbase + q) + 1] = inv;
        }
        const int ox = Xb.at(q_lo + qt * 16 + 4 * g, hc + c);   // rows past Tq: dropped
#pragma unroll
        for (int r = 0; r < 4; ++r) Xb.st1(ox, r * Xb.sT4, oq[r] * shfl(inv, 4 * g + r));
    };

    for (int k_lo = 0; k_lo < Tk; k_lo += CH) {
        // operands of the 4 key tiles of this chunk
        float kf[NT][4], vf[NT][4], mt[NT][4];
#pragma unroll
        for (int kt = 0; kt < NT; ++kt) {
            const int k0 = k_lo + kt * 16;
            Kb.ld4(kf[kt], Kb.at(k0 + c, hc + 4 * g));                    // A: K[k0+c][4g+s]
            const int ov = Vb.at(k0 + 4 * g, hc + c);                       // B of P.V: V[k0+4g+s][c]
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                vf[kt][s] = Vb.ld1(ov, s * Vb.sT4);
                mt[kt][s] = mask_term(mask, k0 + 4 * g + s, Tk);
            }
        }
        float qfa[NT][4];                                                  // B of S^T: Q[q][4g+s]
#pragma unroll
        for (int qt = 0; qt < NT; ++qt) Qb.ld4(qfa[qt], Qb.at(q_lo + qt * 16 + c, hc + 4 * g));   // past Tq: 0
#pragma unroll
        for (int qt = 0; qt < NT; ++qt) {
            if (qt >= nqt) break;
            const int q = q_lo + qt * 16 + c;
            const float* qf = qfa[qt];
            const int srow = (sbase + min(q, Tq - 1)) * Tk;
            float sv[NT][4];
            float mx = -INFINITY;
#pragma unroll
            for (int kt = 0; kt < NT; ++kt) {
                floatx4 st = zero4();
#pragma unroll
                for (int s = 0; s < 4; ++s) st = mfma16(kf[kt][s], qf[s], st);   // C[key 4g+r][query c]
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float spv = 0.f;
                    const int kk = k_lo + kt * 16 + 4 * g + r;
                    if (PREV || SOUT) {
                        const int si = srow + min(kk, Tk - 1);
                        if (PREV) spv = sprev[si];
                        const float v = score<PREV>(st[r], cres, spv, mt[kt][r]);
                        if (SOUT && kk < Tk && q < Tq) sout[si] = v;
                        sv[kt][r] = v;
                    } else {
                        sv[kt][r] = score<false>(st[r], 0.f, 0.f, mt[kt][r]);
                    }
                    mx = fmaxf(mx, sv[kt][r]);
                }
            }
            mx = fmaxf(mx, shfl(mx, lane ^ 16));
            mx = fmaxf(mx, shfl(mx, lane ^ 32));
            const float mnew = SINGLE ? mx : fmaxf(m[qt], mx);
            float lsum = 0.f;
#pragma unroll
            for (int kt = 0; kt < NT; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    sv[kt][r] = __expf(sv[kt][r] - mnew);
                    lsum += sv[kt][r];
                }
            floatx4 oq = SINGLE ? zero4() : o[qt];
            if (!SINGLE && k_lo > 0) {   // rescale the running state
                const float corr = __expf(m[qt] - mnew);
                l[qt] *= corr;
#pragma unroll
                for (int r = 0; r < 4; ++r) oq[r] *= shfl(corr, 4 * g + r);  // O row 4g+r <- query 4g+r
            }
#pragma unroll
            for (int kt = 0; kt < NT; ++kt)
#pragma unroll
                for (int s = 0; s < 4; ++s) oq = mfma16(sv[kt][s], vf[kt][s], oq);  // C[query 4g+r][dim c]
            if (SINGLE) {
                finish(qt, oq, mnew, lsum);
            } else {
                o[qt] = oq;
                l[qt] += lsum;
                m[qt] = mnew;
            }
        }
    }
    if (!SINGLE) {
#pragma unroll
        for (int qt = 0; qt < NT; ++qt) {
            if (qt >= nqt) break;
            finish(qt, o[qt], m[qt], l[qt]);
        }
    }
}

template <bool PREV, bool SOUT, bool SINGLE>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu((SINGLE && !PREV) ? 4 : 1))) void k_attn_fwd(const mep_attn_desc* __restrict__ descs) {
    const mep_attn_desc& d = descs[blockIdx.y];
    if ((d.Tk <= CH) != SINGLE) return;    // the other variant's descriptor
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nqc = (d.Tq + CH - 1) / CH;
    const int task = blockIdx.x * WAVES + wave;
    if (task >= d.B * d.H * nqc) return;   // whole wave leaves; no barriers below
    const int qc = task % nqc, bh = task / nqc;
    attn_fwd_task<PREV, SOUT, SINGLE>(d, qc, bh % d.H, bh / d.H, lane);
}

MEP_DEV void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One backward task: batch row b, head h, 64 keys.  PREV: residual scores (writes dS_prev and the
// dc partial); DSN: a gradient arrives on this layer's post-mask S output.
template <bool PREV, bool DSN>
MEP_DEV void attn_bwd_task(const mep_attn_bwd_desc& bd, int task, int kc, int nkc, int h, int b, int lane, float* T) {
    const mep_attn_desc& d = bd.f;
    const int c = lane & 15, g = lane >> 4;
    const int hc = h * HD;
    const int Tq = d.Tq, Tk = d.Tk, D = d.H * HD;
    const float cres = PREV ? *G<const float>(d.c) : 0.f;
    const gfloat* sprev = G<const float>(d.s_prev);
    const gfloat* dsn = G<const float>(bd.ds_next);
    gfloat* dsp = G<float>(bd.ds_prev);
    const gfloat* mask = G<const float>(d.mask) + (int64_t)b * d.mask_sB;
    const BRow Qb = brow(d.q, b, Tq, D), Kb = brow(d.k, b, Tk, D), Vb = brow(d.v, b, Tk, D);
    const BRow Ob = brow(d.x, b, Tq, D), Gb = brow(bd.dx, b, Tq, D), dQb = brow(bd.dq, b, Tq, D);
    const int sbase = (b * d.H + h) * Tq;
    const auto rsStat = uniform_rsrc(d.stats + 8ull * (uint64_t)sbase, 8 * (int64_t)Tq);

    const int k_lo = kc * CH;
    // per key tile: B operands of S (K) and dP (V) with the key on the lane, the key's mask term,
    // and the B operand of dQ (K rows 4g+s, dim c); dK / dV accumulators (C[key 4g+r][dim c])
    float kb[NT][4], vb[NT][4], kq[NT][4], mtk[NT];
    floatx4 dk[NT], dv[NT];
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
        const int k0 = k_lo + kt * 16;
        Kb.ld4(kb[kt], Kb.at(k0 + c, hc + 4 * g));
        Vb.ld4(vb[kt], Vb.at(k0 + c, hc + 4 * g));
        mtk[kt] = mask_term(mask, k0 + c, Tk);
#pragma unroll
        for (int s = 0; s < 4; ++s) kq[kt][s] = Kb.ld1(Kb.at(k0 + 4 * g, hc + c), s * Kb.sT4);
        dk[kt] = zero4();
        dv[kt] = zero4();
    }
    float dc_acc = 0.f;
    const int nqt = (Tq + 15) / 16;
    // Every global load of a 16-query tile (Q and dO in both layouts, O for delta, the row stats
    // and the dQ rows this tile accumulates onto) is issued one tile ahead, into the other of two
    // register sets, so only the first tile waits for memory.
    struct QIn {
        float qa[4], da[4], db[4], qb[4], ob[4], dqo[4];
        f32x2 st[4];
    };
    auto fetch = [&](QIn& in, int qt) {
        const int q0 = qt * 16;   // tiles past the end read zeros
        Qb.ld4(in.qa, Qb.at(q0 + c, hc + 4 * g));   // A of S: Q[q0+c][4g+s]
        Gb.ld4(in.da, Gb.at(q0 + c, hc + 4 * g));   // A of dP: dO[q0+c][4g+s]
        const int qg = q0 + 4 * g;                  // B of dV / dK: rows qg + s, dim c
        const int og = Gb.at(qg, hc + c), oq = Qb.at(qg, hc + c), oo = Ob.at(qg, hc + c), od = dQb.at(qg, hc + c);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            in.db[s] = Gb.ld1(og, s * Gb.sT4);
            in.qb[s] = Qb.ld1(oq, s * Qb.sT4);
            in.ob[s] = Ob.ld1(oo, s * Ob.sT4);
            in.st[s] = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rsStat, 8 * qg, 8 * s, 0));
            in.dqo[s] = nkc == 1 ? dQb.ld1(od, s * dQb.sT4) : 0.f;
        }
    };
    auto body = [&](const QIn& in, int qt) {
        const int q0 = qt * 16;
        float mm[4], li[4], del[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int qq = q0 + 4 * g + s;
            // delta = rowsum(dO * O): the 16 dims of query qq sit in one DPP row (lanes c)
            del[s] = row16_sum(in.db[s] * in.ob[s]);
            // padded queries: max = +inf, 1/sum = 0 make P = exp(-inf) * 0 = 0 (and with it dS)
            const bool qok = qq < Tq;
            mm[s] = qok ? in.st[s][0] : INFINITY;
            li[s] = qok ? in.st[s][1] : 0.f;
        }
        float ds[NT][4];
#pragma unroll
        for (int kt = 0; kt < NT; ++kt) {
            const int kk = k_lo + kt * 16 + c;
            floatx4 st = zero4(), dp = zero4();
#pragma unroll
            for (int s = 0; s < 4; ++s) st = mfma16(in.qa[s], kb[kt][s], st);   // C[query 4g+r][key c]
#pragma unroll
            for (int s = 0; s < 4; ++s) dp = mfma16(in.da[s], vb[kt][s], dp);
            float p[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int qq = q0 + 4 * g + r;
                float spv = 0.f;
                int si = 0;
                if (PREV || DSN) {
                    si = (sbase + min(qq, Tq - 1)) * Tk + min(kk, Tk - 1);
                    if (PREV) spv = sprev[si];
                }
                const float sv = score<PREV>(st[r], cres, spv, mtk[kt]);
                const float pv = __expf(sv - mm[r]) * li[r];
                float gsv = pv * (dp[r] - del[r]);
                if (DSN || PREV) {
                    const bool ok = (qq < Tq) && (kk < Tk);
                    if (DSN) gsv += ok ? dsn[si] : 0.f;
                    if (PREV) {
                        if (ok) dsp[si] = cres * gsv;
                        dc_acc = fmaf(gsv, spv, dc_acc);
                    }
                }
                p[r] = pv;
                ds[kt][r] = gsv;
            }
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                dv[kt] = mfma16(p[s], in.db[s], dv[kt]);         // dV[key][dim] += P^T dO
                dk[kt] = mfma16(ds[kt][s], in.qb[s], dk[kt]);    // dK[key][dim] += dS^T Q
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) T[(4 * g + r) * TLD + kt * 16 + c] = ds[kt][r];   // T[query][key]
        }
        // dQ += dS K with the query on the lane: read back the transposed 16 x 64 dS tile
        wave_lds_sync();
        floatx4 dq = zero4();
#pragma unroll
        for (int kt = 0; kt < NT; ++kt) {
            const float4 t4 = *reinterpret_cast<const float4*>(T + c * TLD + kt * 16 + 4 * g);
            dq = mfma16(t4.x, kq[kt][0], dq);
            dq = mfma16(t4.y, kq[kt][1], dq);
            dq = mfma16(t4.z, kq[kt][2], dq);
            dq = mfma16(t4.w, kq[kt][3], dq);
        }
        wave_lds_sync();
        // dq rows q0+4g+r, dim c (exclusive owner when the keys fit one chunk; else atomics);
        // rows past Tq are dropped by the range check
        const int od = dQb.at(q0 + 4 * g, hc + c);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int qq = q0 + 4 * g + r;
            if (nkc == 1) {
                dQb.st1(od, r * dQb.sT4, in.dqo[r] + dq[r] * INV_SCALE);
            } else if (qq < Tq) {
                gfloat* dqp = G<float>(bd.dq.ptr) + (int64_t)b * bd.dq.sB + (int64_t)qq * bd.dq.sT + hc + c;
                atomicAdd(reinterpret_cast<float*>(reinterpret_cast<uintptr_t>(dqp)), dq[r] * INV_SCALE);
            }
        }
    };
    QIn bufA, bufB;
    fetch(bufA, 0);
    for (int qt = 0; qt < nqt; qt += 2) {
        fetch(bufB, qt + 1);
        body(bufA, qt);
        if (qt + 1 < nqt) {
            fetch(bufA, qt + 2);
            body(bufB, qt + 1);
        }
    }
    const bool same_kv = bd.dk.ptr == bd.dv.ptr && bd.dk.sB == bd.dv.sB && bd.dk.sT == bd.dv.sT;
    const BRow dKb = brow(bd.dk, b, Tk, D), dVb = brow(bd.dv, b, Tk, D);   // keys past Tk: dropped
    const int ok_ = dKb.at(k_lo + 4 * g, hc + c), ov_ = dVb.at(k_lo + 4 * g, hc + c);
#pragma unroll
    for (int kt = 0; kt < NT; ++kt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (same_kv) {
                dKb.st1(ok_, (16 * kt + r) * dKb.sT4, dk[kt][r] * INV_SCALE + dv[kt][r]);
            } else {
                dKb.st1(ok_, (16 * kt + r) * dKb.sT4, dk[kt][r] * INV_SCALE);
                dVb.st1(ov_, (16 * kt + r) * dVb.sT4, dv[kt][r]);
            }
        }
    }
    if (PREV && bd.dc_partial) {
        const float w = wave_sum(dc_acc);
        if (lane == 0) G<float>(bd.dc_partial)[task] = w;
    }
}

template <bool PREV, bool DSN>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu((PREV || DSN) ? 1 : 2))) void k_attn_bwd(const mep_attn_bwd_desc* __restrict__ descs) {
    const mep_attn_bwd_desc& bd = descs[blockIdx.y];
    const mep_attn_desc& d = bd.f;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nkc = (d.Tk + CH - 1) / CH;
    const int task = blockIdx.x * WAVES + wave;
    __shared__ __attribute__((aligned(16))) float Tr[WAVES][16 * TLD];
    if (task >= d.B * d.H * nkc) return;   // whole wave leaves; only wave-private LDS below
    const int kc = task % nkc, bh = task / nkc;
    attn_bwd_task<PREV, DSN>(bd, task, kc, nkc, bh % d.H, bh / d.H, lane, Tr[wave]);
}

}  // namespace

// Launch geometry: 256 threads (4 waves, one task each); tasks = B * H * ceil(Tq/64) forward,
// B * H * ceil(Tk/64) backward; max_tiles = ceil(max tasks / 4).  dc_partial (backward) has one
// float per task, task = (b*H + h) * ceil(Tk/64) + key chunk.  `flags` (MEP_ATTN_*) select the
// compiled variants: PREV / SOUT (DSN) must hold for every descriptor of the launch; SHORT / LONG
// say whether descriptors with Tk <= 64 / Tk > 64 are present (one kernel launch per class).
extern "C" int mep_attn_fwd(const mep_attn_desc* descs, int n_desc, int max_tiles, int flags, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    if (!(flags & (MEP_ATTN_SHORT | MEP_ATTN_LONG))) { mep_set_error("mep_attn_fwd: flags need SHORT and/or LONG"); return MEP_EINVAL; }
    const bool prev = flags & MEP_ATTN_PREV, sout = flags & MEP_ATTN_SOUT;
    const dim3 grid(max_tiles, n_desc), block(THREADS);
    hipStream_t st = (hipStream_t)stream;
#define MEP_FWD(P, S, SI) hipLaunchKernelGGL((k_attn_fwd<P, S, SI>), grid, block, 0, st, descs)
    for (int single = 1; single >= 0; --single) {
        if (!(flags & (single ? MEP_ATTN_SHORT : MEP_ATTN_LONG))) continue;
        if (single) {
            if (prev) { if (sout) MEP_FWD(true, true, true); else MEP_FWD(true, false, true); }
            else      { if (sout) MEP_FWD(false, true, true); else MEP_FWD(false, false, true); }
        } else {
            if (prev) { if (sout) MEP_FWD(true, true, false); else MEP_FWD(true, false, false); }
            else      { if (sout) MEP_FWD(false, true, false); else MEP_FWD(false, false, false); }
        }
    }
#undef MEP_FWD
    return mep_check_launch("mep_attn_fwd");
}

extern "C" int mep_attn_bwd(const mep_attn_bwd_desc* descs, int n_desc, int max_tiles, int flags,
                            mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    const bool prev = flags & MEP_ATTN_PREV, dsn = flags & MEP_ATTN_SOUT;
    const dim3 grid(max_tiles, n_desc), block(THREADS);
    hipStream_t st = (hipStream_t)stream;
    if (prev) { if (dsn) hipLaunchKernelGGL((k_attn_bwd<true, true>), grid, block, 0, st, descs);
                else hipLaunchKernelGGL((k_attn_bwd<true, false>), grid, block, 0, st, descs); }
    else      { if (dsn) hipLaunchKernelGGL((k_attn_bwd<false, true>), grid, block, 0, st, descs);
                else hipLaunchKernelGGL((k_attn_bwd<false, false>), grid, block, 0, st, descs); }
    return mep_check_launch("mep_attn_bwd");
}
