// Mean+max pooling over time and the fused fusion-head + loss (forward and backward).
//
// Pool: Multi_ATTN's cat(mean_t, max_t) over the time-concatenated block outputs
// (cmu-mosei/run.py:314-318; realformer.py:258-262).  Padded time steps are included, as in
// the reference.  Max keeps the FIRST index on ties (torch.max(dim) semantics), which matters
// for all-zero "no_name" utterances whose rows are identical.
//
// Head: Concat_Trans / Base_model head (cmu-mosei/run.py:319,330-339; Ren-MME/run.py:271,
// 283-292) fused with multi_circle_loss (cmu-mosei/run.py:342-351), the batch mean (run.py:366)
// and, for Ren-MME, the R-Drop KL (Ren-MME/run.py:331-334).  These are latency-bound (7x7x7
// bilinear, 14->7 Linear); one workgroup per row (per row pair with R-Drop) does forward,
// loss and backward in one launch, writing per-row parameter-gradient partials that
// mep_head_reduce sums in a fixed order (deterministic).
#include "common.h"

using namespace mep;

namespace {

// workgroup = (batch row, 32 columns); 8 time groups of 32 lanes stride the time axis and
// combine in a fixed order (first index of the maximum wins across groups, as within one)
constexpr int POOL_COLS = 32, POOL_GROUPS = 8;

__global__ __launch_bounds__(256) void k_pool_fwd(const mep_pool_desc* __restrict__ descs) {
    const mep_pool_desc& d = descs[blockIdx.y];
    const int nct = (d.C + POOL_COLS - 1) / POOL_COLS;
    if ((int)blockIdx.x >= d.B * nct) return;
    const int b = blockIdx.x / nct;
    const int cl = threadIdx.x & (POOL_COLS - 1), g = threadIdx.x / POOL_COLS;
    const int c = (blockIdx.x - b * nct) * POOL_COLS + cl;
    __shared__ float s_sum[POOL_GROUPS][POOL_COLS], s_max[POOL_GROUPS][POOL_COLS];
    __shared__ int s_idx[POOL_GROUPS][POOL_COLS];
    float s = 0.f, mx = -INFINITY;
    int idx = 0x7fffffff;
    if (c < d.C) {
        const gfloat* x = G<const float>(d.x) + (int64_t)b * d.T * d.C + c;
        // 8 time steps of loads in flight, then consumed in time order (ties: first index wins)
        for (int t0 = g; t0 < d.T; t0 += 8 * POOL_GROUPS) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int t = t0 + POOL_GROUPS * u;
                v[u] = t < d.T ? x[(int64_t)t * d.C] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int t = t0 + POOL_GROUPS * u;
                if (t < d.T) {
                    s += v[u];
                    if (v[u] > mx || idx == 0x7fffffff) { mx = v[u]; idx = t; }   // strict >
                }
            }
        }
    }
    s_sum[g][cl] = s;
    s_max[g][cl] = mx;
    s_idx[g][cl] = idx;
    __syncthreads();
    if (g == 0 && c < d.C) {
        float ts = 0.f, tm = s_max[0][cl];
        int ti = s_idx[0][cl];
#pragma unroll
        for (int k = 0; k < POOL_GROUPS; ++k) {
            ts += s_sum[k][cl];
            const float m = s_max[k][cl];
            const int i = s_idx[k][cl];
            if (i != 0x7fffffff && (m > tm || (m == tm && i < ti))) { tm = m; ti = i; }
        }
        gfloat* pooled = G<float>(d.pooled) + (int64_t)b * 2 * d.C;
        pooled[c] = ts / (float)d.T;
        pooled[d.C + c] = tm;
        G<int>(d.argmax)[(int64_t)b * d.C + c] = ti;
    }
}

// dx = dmean / T + onehot(argmax) * dmax over [B, T, C].  Workgroup = (batch row b, 16 time
// steps); each thread keeps the pooled gradients and argmax of its columns in registers and
// writes its columns of the 16 rows (no index division per element).
constexpr int POOLB_T = 16;
__global__ __launch_bounds__(256) void k_pool_bwd(const mep_pool_desc* __restrict__ descs) {
    const mep_pool_desc& d = descs[blockIdx.y];
    const int ntc = (d.T + POOLB_T - 1) / POOLB_T;
    const int b = blockIdx.x / ntc, t0 = (blockIdx.x - b * ntc) * POOLB_T;
    if (b >= d.B) return;
    const int C = d.C;
    const gfloat* dp = G<const float>(d.dpooled) + (int64_t)b * 2 * C;
    const MEP_G int* am = G<const int>(d.argmax) + (int64_t)b * C;
    gfloat* dx = G<float>(d.dx) + (int64_t)b * d.T * C;
    const int t1 = min(d.T, t0 + POOLB_T);
    for (int c = threadIdx.x; c < C; c += 256) {
        const float dmean = dp[c] / (float)d.T;
        const float dmax = dp[C + c];
        const int ta = am[c];
        for (int t = t0; t < t1; ++t) dx[(int64_t)t * C + c] = (ta == t) ? dmean + dmax : dmean;
    }
}

// ---------------------------------------------------------------- fusion head
constexpr int NCMAX = 16;
constexpr int HEAD_KU = 3;   // classifier columns per thread per pass

struct HeadOff {
    int wo, bo, lnw, lnb, trans, dl0, dl1, stride;
};
__host__ __device__ inline HeadOff head_off(int NC) {
    HeadOff o;
    o.wo = 0;
    o.bo = o.wo + 2 * NC * NC;
    o.lnw = o.bo + NC;
    o.lnb = o.lnw + NC;
    o.trans = o.lnb + NC;
    o.dl0 = o.trans + NC * NC * NC;
    o.dl1 = o.dl0 + NC;
    o.stride = o.dl1 + NC;
    return o;
}

MEP_DEV float label_at(const mep_head_desc& d, int b, int n) {
    if (d.labels_are_float) return G<const float>(d.labels)[b * d.NC + n];
    return (float)G<const int64_t>(d.labels)[b * d.NC + n];
}

// make LDS writes of this wave visible to its other lanes
// (wavefront-scope fences: LDS ordering only, no wait on the wave's outstanding global stores)
MEP_DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

MEP_DEV float log_sigmoid(float x) { return fminf(x, 0.f) - log1pf(__expf(-fabsf(x))); }


#define HT(i) do { } while (0)
#define HT_PRINT() do { } while (0)
// NCT: the class count as a compile-time constant (7 cmu-mosei, 9 Ren-MME; 0 = runtime, <= NCMAX):
// exact unrolls, constant index arithmetic and a small code footprint (each workgroup runs the
// kernel body once, so instruction fetch is on the critical path)
template <int NCT>
__global__ __launch_bounds__(256) void k_head(mep_head_desc d) {
    constexpr int NU = NCT ? NCT : NCMAX;
    HT(0);
    const int rows = d.rdrop ? 2 : 1;
    const int r0 = blockIdx.x * rows;
    const int NC = NCT ? NCT : d.NC, F = d.F;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __shared__ float s_last[2][NCMAX], s_this[2][NCMAX], s_logit[2][NCMAX], s_dlog[2][NCMAX];
    __shared__ float s_temp[2][NCMAX * NCMAX];
    __shared__ float s_yhat[2][NCMAX], s_cat[2][2 * NCMAX], s_rstd[2];
    __shared__ float s_dlast[2][NCMAX], s_dthis[2][NCMAX];
    const gfloat* wc0 = G<const float>(d.wc0);
    const gfloat* wc1 = G<const float>(d.wc1);
    // the small head parameters live in LDS for the whole kernel: the serial phases below read
    // them in dependent chains, where a global (L2) latency per step would dominate
    __shared__ float trans[NCMAX * NCMAX * NCMAX], wo[NCMAX * 2 * NCMAX], lnw[NCMAX], lnb[NCMAX], bo[NCMAX];
    __shared__ float s_part[NCMAX * NCMAX];
    // staged with every load in flight at once (registers first, LDS after the classifier loads
    // are issued): trans <= 1024 and wo <= 512 elements in one pass, a plain loop beyond
    const int ntr = NC * NC * NC, nwo = 2 * NC * NC;
    const gfloat* g_trans = G<const float>(d.trans);
    const gfloat* g_wo = G<const float>(d.wo);
    float st_tr[4], st_wo[2], st_ln[3];
#pragma unroll
    for (int j = 0; j < 4; ++j) st_tr[j] = g_trans[min((int)threadIdx.x + 256 * j, ntr - 1)];
#pragma unroll
    for (int j = 0; j < 2; ++j) st_wo[j] = g_wo[min((int)threadIdx.x + 256 * j, nwo - 1)];
    {
        const int c = min((int)threadIdx.x, NC - 1);
        st_ln[0] = G<const float>(d.ln_w)[c];
        st_ln[1] = G<const float>(d.ln_b)[c];
        st_ln[2] = G<const float>(d.bo)[c];
    }
    auto stage_params = [&]() {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if ((int)threadIdx.x + 256 * j < ntr) trans[threadIdx.x + 256 * j] = st_tr[j];
        for (int i = threadIdx.x + 1024; i < ntr; i += 256) trans[i] = g_trans[i];
#pragma unroll
        for (int j = 0; j < 2; ++j)
            if ((int)threadIdx.x + 256 * j < nwo) wo[threadIdx.x + 256 * j] = st_wo[j];
        if ((int)threadIdx.x < NC) {
            lnw[threadIdx.x] = st_ln[0];
            lnb[threadIdx.x] = st_ln[1];
            bo[threadIdx.x] = st_ln[2];
        }
    };

    // the labels of the loss phase, fetched now so their latency hides behind the classifiers
    float lab[2] = {0.f, 0.f};
    if (wave == 0 && lane < NC && !d.ext_dlogits) {
        lab[0] = label_at(d, r0, lane);
        if (rows > 1) lab[1] = label_at(d, r0 + 1, lane);
    }

    // classifiers (Multi_ATTN.classifier, no bias): every thread takes columns k = tid + 256 j
    // of all 2 NC outputs (all loads of a column issued together), then one block reduction
    __shared__ float s_red[2][4][2 * NCMAX];
    // F <= 256 HEAD_KU (one pass, every configuration of the three models): the classifier
    // columns stay in registers from the classifier pass to the dpooled pass (no second L2 read)
    const bool one_pass = F <= 256 * HEAD_KU;
    float kw0[HEAD_KU][NU], kw1[HEAD_KU][NU];
    for (int rr = 0; rr < rows; ++rr) {
        const int b = r0 + rr;
        const gfloat* p0 = G<const float>(d.pooled0) + (int64_t)b * F;
        const gfloat* p1 = G<const float>(d.pooled1) + (int64_t)b * F;
        float acc[2 * NCMAX];
#pragma unroll
        for (int n = 0; n < 2 * NCMAX; ++n) acc[n] = 0.f;   // [0, NU): last, [NCMAX, NCMAX + NU): this
        // HEAD_KU columns per thread per pass (F <= 768 in one pass), every load of the pass
        // issued before the first FMA: rows clamped to NC - 1, columns past F read column F - 1
        // and are weighted by 0
        for (int k0 = 0; k0 < F; k0 += 256 * HEAD_KU) {
            float x0[HEAD_KU], x1[HEAD_KU], w0[HEAD_KU][NCMAX], w1[HEAD_KU][NCMAX];
#pragma unroll
            for (int u = 0; u < HEAD_KU; ++u) {
                const int k = min(k0 + 256 * u + (int)threadIdx.x, F - 1);
                x0[u] = p0[k];
                x1[u] = p1[k];
#pragma unroll
                for (int n = 0; n < NU; ++n) {
                    const int64_t o = (int64_t)min(n, NC - 1) * F + k;
                    w0[u][n] = wc0[o];
                    w1[u][n] = wc1[o];
                }
            }
            if (rr == 0 && k0 == 0) {
#pragma unroll
                for (int u = 0; u < HEAD_KU; ++u)
#pragma unroll
                    for (int n = 0; n < NU; ++n) {
                        kw0[u][n] = w0[u][n];
                        kw1[u][n] = w1[u][n];
                    }
            }
#pragma unroll
            for (int u = 0; u < HEAD_KU; ++u) {
                const bool kin = k0 + 256 * u + (int)threadIdx.x < F;
                const float a = kin ? x0[u] : 0.f, c = kin ? x1[u] : 0.f;
#pragma unroll
                for (int n = 0; n < NU; ++n) {
                    acc[n] = fmaf(w0[u][n], a, acc[n]);
                    acc[NCMAX + n] = fmaf(w1[u][n], c, acc[NCMAX + n]);
                }
            }
        }
#pragma unroll
        for (int n = 0; n < NU; ++n) {
            if (n < NC) {
                const float s0 = wave_sum(acc[n]), s1 = wave_sum(acc[NCMAX + n]);
                if (lane == 0) {
                    s_red[rr][wave][n] = s0;
                    s_red[rr][wave][NCMAX + n] = s1;
                }
            }
        }
    }
    stage_params();
    __syncthreads();
    if (threadIdx.x < 2 * NCMAX * rows) {
        const int rr = threadIdx.x / (2 * NCMAX), n = threadIdx.x % (2 * NCMAX);
        const int nn = n & (NCMAX - 1);
        if (nn < NC) {
            const float s = (s_red[rr][0][n] + s_red[rr][1][n]) + (s_red[rr][2][n] + s_red[rr][3][n]);
            if (n < NCMAX) s_last[rr][nn] = s; else s_this[rr][nn] = s;
        }
    }
    __syncthreads();
    HT(1);
    if (wave == 0) {
        for (int rr = 0; rr < rows; ++rr) {
            // temp[p][n] = sum_m last[m] trans[p][m][n]   (matmul(last[i], trans), run.py:334)
            for (int idx = lane; idx < NC * NC; idx += 64) {
                const int p = idx / NC, n = idx - p * NC;
                float s = 0.f;
                for (int m = 0; m < NC; ++m) s = fmaf(s_last[rr][m], trans[(p * NC + m) * NC + n], s);
                s_temp[rr][idx] = s;
            }
            wave_sync();
            float y = 0.f;
            if (lane < NC)
                for (int p = 0; p < NC; ++p) y = fmaf(s_this[rr][p], s_temp[rr][p * NC + lane], y);
            const float mean = wave_sum(lane < NC ? y : 0.f) / (float)NC;
            const float dv = lane < NC ? y - mean : 0.f;
            const float var = wave_sum(dv * dv) / (float)NC;
            const float rstd = 1.0f / sqrtf(var + 1e-5f);
            if (lane < NC) {
                s_yhat[rr][lane] = dv * rstd;
                s_cat[rr][lane] = s_this[rr][lane];
                s_cat[rr][NC + lane] = dv * rstd * lnw[lane] + lnb[lane];
            }
            if (lane == 0) s_rstd[rr] = rstd;
            wave_sync();
            if (lane < NC) {
                float s = 0.f;
                for (int j = 0; j < 2 * NC; ++j) s = fmaf(wo[lane * 2 * NC + j], s_cat[rr][j], s);
                s_logit[rr][lane] = s + bo[lane];
                G<float>(d.logits)[(r0 + rr) * NC + lane] = s + bo[lane];
            }
            wave_sync();
        }
        HT(2);
        // losses: circle per row, then R-Drop KL for the pair
        gfloat* row_loss = G<float>(d.row_loss);
        const gfloat* ext = G<const float>(d.ext_dlogits);
        if (ext) {
            for (int rr = 0; rr < rows; ++rr)
                if (lane < NC) s_dlog[rr][lane] = ext[(r0 + rr) * NC + lane];
            wave_sync();
        }
        // loss scale and R-Drop divisor: device-resident when d.scale is set (data-parallel
        // shares replayed from one captured graph)
        const gfloat* dscale = G<const float>(d.scale);
        const float loss_scale = dscale ? dscale[0] : d.loss_scale;
        const int rdrop_pairs = dscale ? (int)dscale[1] : d.rdrop_pairs;
        for (int rr = 0; rr < rows && !ext; ++rr) {
            const int b = r0 + rr;
            const bool ok = lane < NC;
            const float x = ok ? s_logit[rr][lane] : 0.f;
            const float t = ok ? (rr ? lab[1] : lab[0]) : 0.f;
            const bool is_pos = ok && t > 0.5f, is_neg = ok && !(t > 0.5f);
            const float vn = is_neg ? x : -INFINITY;   // y = (1-2t) p for t = 0
            const float vp = is_pos ? -x : -INFINITY;  // y = (1-2t) p for t = 1
            const float mn = fmaxf(wave_max(vn), 0.f), mp = fmaxf(wave_max(vp), 0.f);
            const float en = is_neg ? __expf(vn - mn) : 0.f, ep = is_pos ? __expf(vp - mp) : 0.f;
            const float sn = wave_sum(en) + __expf(-mn), sp = wave_sum(ep) + __expf(-mp);
            const float ln = mn + logf(sn), lp = mp + logf(sp);
            float g = 0.f;
            if (is_neg) g = __expf(x - ln);
            if (is_pos) g = -__expf(-x - lp);
            if (ok) s_dlog[rr][lane] = g * loss_scale;
            if (lane == 0) row_loss[b] = (ln + lp) * loss_scale;
        }
        if (d.rdrop && !ext) {
            const float R = (float)(rdrop_pairs > 0 ? rdrop_pairs : d.B / 2);   // global pairs under DP
            const bool ok = lane < NC;
            const float pv = ok ? s_logit[0][lane] : 0.f, qv = ok ? s_logit[1][lane] : 0.f;
            const float sp = 1.f / (1.f + __expf(-pv)), sq = 1.f / (1.f + __expf(-qv));
            const float lsp = log_sigmoid(pv), lsq = log_sigmoid(qv);
            const float lgp = logf(sp), lgq = logf(sq);
            float kl0 = (ok && sq > 0.f) ? sq * (lgq - lsp) : 0.f;
            float kl1 = (ok && sp > 0.f) ? sp * (lgp - lsq) : 0.f;
            const float kl = wave_sum(kl0 + kl1) / R * 0.5f;
            if (ok) {
                const float gp = (-sq * (1.f - sp) + (sp > 0.f ? (lgp + 1.f - lsq) * sp * (1.f - sp) : 0.f)) / R * 0.5f;
                const float gq = (-sp * (1.f - sq) + (sq > 0.f ? (lgq + 1.f - lsp) * sq * (1.f - sq) : 0.f)) / R * 0.5f;
                s_dlog[0][lane] += gp;
                s_dlog[1][lane] += gq;
            }
            if (lane == 0) row_loss[r0] += kl;
        }
        HT(3);
        if (d.compute_grad) {
            const HeadOff o = head_off(NC);
            for (int rr = 0; rr < rows; ++rr) {
                gfloat* part = G<float>(d.partial) + (int64_t)(r0 + rr) * o.stride;
                // out Linear: dWo, dbo, dcat
                for (int idx = lane; idx < NC * 2 * NC; idx += 64) {
                    const int n = idx / (2 * NC), j = idx - n * 2 * NC;
                    part[o.wo + idx] = s_dlog[rr][n] * s_cat[rr][j];
                }
                float dcat_this = 0.f, dyn = 0.f;
                if (lane < NC) {
                    part[o.bo + lane] = s_dlog[rr][lane];
                    for (int n = 0; n < NC; ++n) {
                        dcat_this = fmaf(wo[n * 2 * NC + lane], s_dlog[rr][n], dcat_this);
                        dyn = fmaf(wo[n * 2 * NC + NC + lane], s_dlog[rr][n], dyn);
                    }
                    part[o.lnw + lane] = dyn * s_yhat[rr][lane];
                    part[o.lnb + lane] = dyn;
                }
                HT(7);
                // LayerNorm(7) backward
                const float yh = lane < NC ? s_yhat[rr][lane] : 0.f;
                const float gsc = lane < NC ? dyn * lnw[lane] : 0.f;
                const float s1 = wave_sum(gsc) / (float)NC, s2 = wave_sum(gsc * yh) / (float)NC;
                const float dy = lane < NC ? s_rstd[rr] * (gsc - s1 - yh * s2) : 0.f;
                // bilinear backward
                __shared__ float s_dy[NCMAX];
                if (lane < NC) s_dy[lane] = dy;
                wave_sync();
                HT(8);
                // dlast[m] = sum_p this[p] sum_n dy[n] trans[p][m][n]: lane (m, p) does the n sum
                for (int idx = lane; idx < NC * NC; idx += 64) {
                    const int m = idx / NC, p = idx - m * NC;
                    float s = 0.f;
                    for (int n = 0; n < NC; ++n) s = fmaf(s_dy[n], trans[(p * NC + m) * NC + n], s);
                    s_part[idx] = s_this[rr][p] * s;
                }
                wave_sync();
                HT(9);
                if (lane < NC) {
                    float dt = dcat_this;
                    for (int n = 0; n < NC; ++n) dt = fmaf(s_dy[n], s_temp[rr][lane * NC + n], dt);
                    s_dthis[rr][lane] = dt;
                    float dl = 0.f;
                    for (int p = 0; p < NC; ++p) dl += s_part[lane * NC + p];
                    s_dlast[rr][lane] = dl;
                    part[o.dl0 + lane] = dl;
                    part[o.dl1 + lane] = dt;
                }
                for (int idx = lane; idx < NC * NC * NC; idx += 64) {
                    const int p = idx / (NC * NC), m = (idx / NC) % NC, n = idx % NC;
                    part[o.trans + idx] = s_last[rr][m] * (s_this[rr][p] * s_dy[n]);
                }
                wave_sync();
            }
        }
    }
    if (!d.compute_grad) return;
    HT(4);
    __syncthreads();
    HT(5);
    // dpooled_e = Wc_e^T dlogit_e
    for (int rr = 0; rr < rows; ++rr) {
        const int b = r0 + rr;
        gfloat* dp0 = G<float>(d.dpooled0) + (int64_t)b * F;
        gfloat* dp1 = G<float>(d.dpooled1) + (int64_t)b * F;
        for (int k0 = 0; k0 < F; k0 += 256 * HEAD_KU) {
            float w0[HEAD_KU][NCMAX], w1[HEAD_KU][NCMAX];
            if (one_pass) {
#pragma unroll
                for (int u = 0; u < HEAD_KU; ++u)
#pragma unroll
                    for (int n = 0; n < NU; ++n) {
                        w0[u][n] = kw0[u][n];
                        w1[u][n] = kw1[u][n];
                    }
            } else {
#pragma unroll
                for (int u = 0; u < HEAD_KU; ++u) {   // all loads of the pass in flight at once
                    const int k = min(k0 + 256 * u + (int)threadIdx.x, F - 1);
#pragma unroll
                    for (int n = 0; n < NU; ++n) {
                        const int64_t o = (int64_t)min(n, NC - 1) * F + k;
                        w0[u][n] = wc0[o];
                        w1[u][n] = wc1[o];
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < HEAD_KU; ++u) {
                const int k = k0 + 256 * u + (int)threadIdx.x;
                float a0 = 0.f, a1 = 0.f;
#pragma unroll
                for (int n = 0; n < NU; ++n) {
                    if (n < NC) {
                        a0 = fmaf(w0[u][n], s_dlast[rr][n], a0);
                        a1 = fmaf(w1[u][n], s_dthis[rr][n], a1);
                    }
                }
                if (k < F) {
                    if (d.mean_div > 0 && 2 * k < F) {   // the mean pool's per-step gradient
                        a0 = a0 / (float)d.mean_div;
                        a1 = a1 / (float)d.mean_div;
                    }
                    dp0[k] = a0;
                    dp1[k] = a1;
                }
            }
        }
    }
    HT(6); HT_PRINT();
}

struct HeadGrads {
    float *g_trans, *g_lnw, *g_lnb, *g_wo, *g_bo, *g_wc0, *g_wc1, *loss;
};

// Sum of the per-row head partials.  Workgroups [0, nA32): 32 columns of the small-parameter
// records each, 8 row groups per column (+ the batch loss in workgroup 0); workgroups after
// that: 32 columns k of one classifier e, dWc_e[n][k] = sum_b dlogit_e[b][n] pooled_e[b][k] for
// every n, rows split over 8 groups.  Fixed summation order (deterministic).
MEP_DEV float head_reduce_block(const mep_head_desc& d, const HeadGrads& g, int bx) {
    const int NC = d.NC, F = d.F, B = d.B;
    const HeadOff o = head_off(NC);
    const int nA = o.dl0;                 // everything before the dlogit records
    const int nA32 = (nA + 31) / 32;
    const int cl = threadIdx.x & 31, rg = threadIdx.x >> 5;
    const gfloat* part = G<const float>(d.partial);
    __shared__ float red[8][NCMAX][33];
    if ((int)bx < nA32) {
        const int i = bx * 32 + cl;
        float s = 0.f;
        if (i < nA) {
#pragma unroll 8
            for (int b = rg; b < B; b += 8) s += part[(int64_t)b * o.stride + i];
        }
        red[rg][0][cl] = s;
        float ls = 0.f, sq = 0.f;
        if (bx == 0)
            for (int b = threadIdx.x; b < B; b += 256) ls += G<const float>(d.row_loss)[b];
        __syncthreads();
        if (rg == 0 && i < nA) {
            float t = 0.f;
#pragma unroll
            for (int k = 0; k < 8; ++k) t += red[k][0][cl];
            float* dst;
            if (i < o.bo) dst = g.g_wo + (i - o.wo);
            else if (i < o.lnw) dst = g.g_bo + (i - o.bo);
            else if (i < o.lnb) dst = g.g_lnw + (i - o.lnw);
            else if (i < o.trans) dst = g.g_lnb + (i - o.lnb);
            else dst = g.g_trans + (i - o.trans);
            *G<float>(reinterpret_cast<uint64_t>(dst)) = t;
            sq = t * t;
        }
        if (bx == 0) {
            ls = wave_sum(ls);
            __syncthreads();
            if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][1][0] = ls;
            __syncthreads();
            if (threadIdx.x == 0)
                *G<float>(reinterpret_cast<uint64_t>(g.loss)) = red[0][1][0] + red[1][1][0] + red[2][1][0] + red[3][1][0];
        }
        return sq;   // the loss is not a gradient
    }
    const int wb = bx - nA32;
    const int nkb = (F + 31) / 32;
    const int e = wb / nkb, k = (wb - e * nkb) * 32 + cl;
    const float* pooled = reinterpret_cast<const float*>(e ? d.pooled1 : d.pooled0);
    const int off = e ? o.dl1 : o.dl0;
    float acc[NCMAX];
#pragma unroll
    for (int n = 0; n < NCMAX; ++n) acc[n] = 0.f;
    // rows in chunks of 64: the chunk's dlogit records (64 x NC floats, one or two loads per
    // thread) are staged in LDS while each thread's 8 pooled loads are in flight, then the products
    // run from registers and LDS.  Loading the records per row and class from global memory left
    // these blocks at ~10 us, the long pole of the launch (scripts/wg_trace.py --reduce).  Same
    // products in the same order: rows rg, rg + 8, ... ascending.
    __shared__ float s_dl[64 * NCMAX];
    const int kc = min(k, F - 1);
    for (int b0 = 0; b0 < B; b0 += 64) {
        const int nb = min(64, B - b0);
        for (int t = threadIdx.x; t < nb * NC; t += 256) {
            const int bb = t / NC, n = t - bb * NC;
            s_dl[bb * NCMAX + n] = part[(int64_t)(b0 + bb) * o.stride + off + n];
        }
        float pk[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) pk[u] = pooled[(int64_t)min(b0 + rg + 8 * u, B - 1) * F + kc];
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int bb = rg + 8 * u;
            if (bb < nb) {
#pragma unroll
                for (int n = 0; n < NCMAX; ++n)
                    if (n < NC) acc[n] = fmaf(s_dl[bb * NCMAX + n], pk[u], acc[n]);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int n = 0; n < NCMAX; ++n) if (n < NC) red[rg][n][cl] = acc[n];
    __syncthreads();
    float sq = 0.f;
    if (k < F) {
        float* out = e ? g.g_wc1 : g.g_wc0;
        for (int n = rg; n < NC; n += 8) {
            float t = 0.f;
#pragma unroll
            for (int q = 0; q < 8; ++q) t += red[q][n][cl];
            *G<float>(reinterpret_cast<uint64_t>(out + (int64_t)n * F + k)) = t;
            sq += t * t;
        }
    }
    return sq;
}

__global__ __launch_bounds__(256) void k_head_reduce(mep_head_desc d, HeadGrads g) {
    head_reduce_block(d, g, blockIdx.x);
}

__host__ __device__ inline int head_reduce_blocks(const mep_head_desc& d) {
    return (head_off(d.NC).dl0 + 31) / 32 + 2 * ((d.F + 31) / 32);
}

// MEP_WG_TRACE (development builds, scripts/wg_trace.py --reduce): thread 0 of every block of
// k_reduce_grads stores the real-time counter at its start (0), after its job (1) and at its end
// (2), and its job kind (3: 0 head, 1 split sum, 2 column sum, 3 empty) into g_rg_trace[block]
#ifdef MEP_WG_TRACE
}  // namespace
__device__ unsigned long long g_rg_trace[8192 * 4];
extern "C" int mep_rg_trace_read(void* dst) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_rg_trace), sizeof(g_rg_trace));
}
namespace {
#define MEP_RG_STAMP(k, v) do { if (threadIdx.x == 0 && blockIdx.x < 8192) g_rg_trace[blockIdx.x * 4 + (k)] = (v); } while (0)
#else
#define MEP_RG_STAMP(k, v) ((void)0)
#endif

// Every gradient reduction of a training step in ONE launch: the head-parameter sums (largest
// blocks first), the weight-gradient split sums and the column sums, each block taking one job
// (block bodies in common.h); there are no dependencies between them.
// norm (optional, single-process steps): the clip's gradient-norm pass folded in -- every block
// writes the sum of squares of the gradients it wrote to norm[OPT_EXT0 + block] (fixed-order
// block reduction) and block 0 advances the optimizer step and its scalars (optim.hip
// mep_clip_adam_ext then skips its own norm launch).
// bmap (optional, mep_reduce_grads_mapped): block b runs job bmap[b] = kind << 30 | descriptor << 12
// | block within the descriptor (kind 0 head, 1 split sum, 2 column sum), so only real jobs are
// launched; without it the grid is the rectangle head + descriptors x max tiles.
__global__ __launch_bounds__(256) void k_reduce_grads(const mep_wgrad_desc* __restrict__ wd, int n_wd, int wd_tiles,
                                                      const mep_colsum_desc* __restrict__ cd, int n_cd, int cd_tiles,
                                                      mep_head_desc hd, HeadGrads hg, int head_blocks,
                                                      float* norm, int* step, const float* hyper,
                                                      const unsigned* __restrict__ bmap) {
    int bx = blockIdx.x;
    float sq = 0.f;
    MEP_RG_STAMP(0, __builtin_amdgcn_s_memrealtime());
    if (bmap) {
        const unsigned job = bmap[bx];
        const int kind = (int)(job >> 30), di = (int)((job >> 12) & 0x3ffffu), blk = (int)(job & 0xfffu);
        MEP_RG_STAMP(3, kind);
        if (kind == 0) sq = head_reduce_block(hd, hg, blk);
        else if (kind == 1) sq = wgrad_reduce_block(wd[di], blk);
        else sq = colsum_block(cd[di], blk);
    } else if (bx < head_blocks) {
        MEP_RG_STAMP(3, 0);
        sq = head_reduce_block(hd, hg, bx);
    } else {
        bx -= head_blocks;
        const int wt = wg_red_blocks(wd_tiles);   // blocks of WG_RED_PER entries per descriptor
        if (bx < n_wd * wt) {
            const mep_wgrad_desc& d = wd[bx / wt];
            MEP_RG_STAMP(3, (int64_t)(bx % wt) * WG_RED_PER < (int64_t)d.N * d.Ktot ? 1 : 3);
            sq = wgrad_reduce_block(d, bx % wt);
        } else {
            bx -= n_wd * wt;
            MEP_RG_STAMP(3, 2);
            if (bx < n_cd * cd_tiles) sq = colsum_block(cd[bx / cd_tiles], bx % cd_tiles);
        }
    }
    MEP_RG_STAMP(1, __builtin_amdgcn_s_memrealtime());
    if (!norm) { MEP_RG_STAMP(2, __builtin_amdgcn_s_memrealtime()); return; }
    __shared__ float nred[4];
    sq = wave_sum(sq);
    if ((threadIdx.x & 63) == 0) nred[threadIdx.x >> 6] = sq;
    __syncthreads();
    if (threadIdx.x == 0) {
        norm[OPT_EXT0 + blockIdx.x] = (nred[0] + nred[1]) + (nred[2] + nred[3]);
        if (blockIdx.x == 0 && step) opt_step_scalars(norm, step, hyper);
    }
    MEP_RG_STAMP(2, __builtin_amdgcn_s_memrealtime());
}

__global__ __launch_bounds__(64) void k_circle_fwd(const float* __restrict__ logits, const void* labels, int lf,
                                                   int NC, float* __restrict__ row_loss, float* __restrict__ dunit) {
    const int b = blockIdx.x, lane = threadIdx.x;
    const bool ok = lane < NC;
    const float x = ok ? logits[b * NC + lane] : 0.f;
    float t = 0.f;
    if (ok) t = lf ? reinterpret_cast<const float*>(labels)[b * NC + lane]
                   : (float)reinterpret_cast<const int64_t*>(labels)[b * NC + lane];
    const bool is_pos = ok && t > 0.5f, is_neg = ok && !(t > 0.5f);
    const float vn = is_neg ? x : -INFINITY, vp = is_pos ? -x : -INFINITY;
    const float mn = fmaxf(wave_max(vn), 0.f), mp = fmaxf(wave_max(vp), 0.f);
    const float sn = wave_sum(is_neg ? __expf(vn - mn) : 0.f) + __expf(-mn);
    const float sp = wave_sum(is_pos ? __expf(vp - mp) : 0.f) + __expf(-mp);
    const float ln = mn + logf(sn), lp = mp + logf(sp);
    if (ok) dunit[b * NC + lane] = is_neg ? __expf(x - ln) : -__expf(-x - lp);
    if (lane == 0) row_loss[b] = ln + lp;
}

__global__ void k_circle_bwd(const float* __restrict__ dunit, const float* __restrict__ g, int n, int NC,
                             float* __restrict__ dl) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dl[i] = dunit[i] * g[i / NC];
}

}  // namespace

extern "C" int mep_circle_loss_fwd(const float* logits, const void* labels, int labels_are_float, int B, int NC,
                                   float* row_loss, float* dunit, mep_stream_t stream) {
    if (NC > 64 || B <= 0) { mep_set_error("mep_circle_loss_fwd: NC <= 64"); return MEP_EINVAL; }
    hipLaunchKernelGGL(k_circle_fwd, dim3(B), dim3(64), 0, (hipStream_t)stream, logits, labels, labels_are_float, NC,
                       row_loss, dunit);
    return mep_check_launch("mep_circle_loss_fwd");
}

extern "C" int mep_circle_loss_bwd(const float* dunit, const float* grad_rows, int B, int NC, float* dlogits,
                                   mep_stream_t stream) {
    const int n = B * NC;
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_circle_bwd, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, dunit, grad_rows, n,
                       NC, dlogits);
    return mep_check_launch("mep_circle_loss_bwd");
}

extern "C" int mep_pool_fwd(const mep_pool_desc* descs, int n_desc, int max_tiles, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    hipLaunchKernelGGL(k_pool_fwd, dim3(max_tiles, n_desc), dim3(256), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_pool_fwd");
}

extern "C" int mep_pool_bwd(const mep_pool_desc* descs, int n_desc, int max_tiles, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    hipLaunchKernelGGL(k_pool_bwd, dim3(max_tiles, n_desc), dim3(256), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_pool_bwd");
}

extern "C" int mep_head_partial_stride(int NC) { return head_off(NC).stride; }

extern "C" int mep_head_fwd_bwd(const mep_head_desc* d, mep_stream_t stream) {
    if (!d || d->NC > NCMAX || d->NC <= 0 || d->B <= 0 || (d->rdrop && (d->B % 2))) {
        mep_set_error("mep_head_fwd_bwd: invalid descriptor (NC <= 16, even B with rdrop)");
        return MEP_EINVAL;
    }
    const int groups = d->rdrop ? d->B / 2 : d->B;
    hipStream_t st = (hipStream_t)stream;
    if (d->NC == 7) hipLaunchKernelGGL(k_head<7>, dim3(groups), dim3(256), 0, st, *d);
    else if (d->NC == 9) hipLaunchKernelGGL(k_head<9>, dim3(groups), dim3(256), 0, st, *d);
    else hipLaunchKernelGGL(k_head<0>, dim3(groups), dim3(256), 0, st, *d);
    return mep_check_launch("mep_head_fwd_bwd");
}

extern "C" int mep_reduce_grads_mapped(const mep_wgrad_desc* wgrad, const mep_colsum_desc* colsum,
                                       const mep_head_desc* head, uint64_t g_trans, uint64_t g_ln_w, uint64_t g_ln_b,
                                       uint64_t g_wo, uint64_t g_bo, uint64_t g_wc0, uint64_t g_wc1, uint64_t loss,
                                       float* norm, int* step, const float* hyper, const unsigned* bmap, int n_blocks,
                                       mep_stream_t stream) {
    if (head && head->NC > NCMAX) { mep_set_error("mep_reduce_grads_mapped: invalid head descriptor"); return MEP_EINVAL; }
    if (!bmap || n_blocks < 0) { mep_set_error("mep_reduce_grads_mapped: need the block map"); return MEP_EINVAL; }
    if (n_blocks == 0) return 0;
    mep_head_desc hd{};
    HeadGrads g{};
    if (head) {
        hd = *head;
        g = HeadGrads{(float*)g_trans, (float*)g_ln_w, (float*)g_ln_b, (float*)g_wo, (float*)g_bo,
                      (float*)g_wc0, (float*)g_wc1, (float*)loss};
    }
    hipLaunchKernelGGL(k_reduce_grads, dim3(n_blocks), dim3(256), 0, (hipStream_t)stream, wgrad, 0, 0, colsum, 0, 0,
                       hd, g, 0, norm, step, hyper, bmap);
    return mep_check_launch("mep_reduce_grads_mapped");
}

extern "C" int mep_reduce_grads(const mep_wgrad_desc* wgrad, int n_wgrad, int wgrad_tiles, const mep_colsum_desc* colsum,
                                int n_colsum, int colsum_tiles, const mep_head_desc* head, uint64_t g_trans,
                                uint64_t g_ln_w, uint64_t g_ln_b, uint64_t g_wo, uint64_t g_bo, uint64_t g_wc0,
                                uint64_t g_wc1, uint64_t loss, float* norm, int* step, const float* hyper,
                                mep_stream_t stream) {
    if (head && head->NC > NCMAX) { mep_set_error("mep_reduce_grads: invalid head descriptor"); return MEP_EINVAL; }
    if (n_wgrad < 0 || n_colsum < 0 || (n_wgrad && wgrad_tiles <= 0) || (n_colsum && colsum_tiles <= 0)) {
        mep_set_error("mep_reduce_grads: invalid grid");
        return MEP_EINVAL;
    }
    mep_head_desc hd{};
    HeadGrads g{};
    int hb = 0;
    if (head) {
        hd = *head;
        g = HeadGrads{(float*)g_trans, (float*)g_ln_w, (float*)g_ln_b, (float*)g_wo, (float*)g_bo,
                      (float*)g_wc0, (float*)g_wc1, (float*)loss};
        hb = head_reduce_blocks(hd);
    }
    const int blocks = hb + n_wgrad * wg_red_blocks(wgrad_tiles) + n_colsum * colsum_tiles;
    if (blocks <= 0) return 0;
    hipLaunchKernelGGL(k_reduce_grads, dim3(blocks), dim3(256), 0, (hipStream_t)stream, wgrad, n_wgrad,
                       wgrad_tiles, colsum, n_colsum, colsum_tiles, hd, g, hb, norm, step, hyper, nullptr);
    return mep_check_launch("mep_reduce_grads");
}

extern "C" int mep_reduce_grads_grid(int n_wgrad, int wgrad_tiles, int n_colsum, int colsum_tiles,
                                     const mep_head_desc* head) {
    return (head ? head_reduce_blocks(*head) : 0) + n_wgrad * wg_red_blocks(wgrad_tiles) + n_colsum * colsum_tiles;
}

extern "C" int mep_head_reduce(const mep_head_desc* d, uint64_t g_trans, uint64_t g_ln_w, uint64_t g_ln_b,
                               uint64_t g_wo, uint64_t g_bo, uint64_t g_wc0, uint64_t g_wc1, uint64_t loss,
                               mep_stream_t stream) {
    if (!d || d->NC > NCMAX) { mep_set_error("mep_head_reduce: invalid descriptor"); return MEP_EINVAL; }
    HeadGrads g{(float*)g_trans, (float*)g_ln_w, (float*)g_ln_b, (float*)g_wo, (float*)g_bo,
                (float*)g_wc0, (float*)g_wc1, (float*)loss};
    const HeadOff o = head_off(d->NC);
    const int blocks = (o.dl0 + 31) / 32 + 2 * ((d->F + 31) / 32);
    hipLaunchKernelGGL(k_head_reduce, dim3(blocks), dim3(256), 0, (hipStream_t)stream, *d, g);
    return mep_check_launch("mep_head_reduce");
}
