// cmu-mosei / Ren-MME Attention_Block epilogue (forward + backward) and row LayerNorm.
//
// Forward (cmu-mosei/run.py:257-261; Ren-MME/run.py:209-213 with dropout and norm2):
//   xp = drop(x Wp^T);  z = [q | xp] Wm^T;  out = drop(LayerNorm(z))
// Backward: LayerNorm backward, dq_direct = dz Wm[:, :D], dxp = drop'(dz Wm[:, D:]), dx = dxp Wp.
// Weight-stationary: a workgroup (8 waves) owns a contiguous range of 16-token tiles of ONE
// block and keeps that block's weights in LDS; each wave runs whole tiles through all products in
// the transposed-tile formulation (common.h), so activations never pass through LDS and the
// concat [q | xp] is two accumulating passes.
// Arithmetic, fp32 path (D <= 96): fp32 operands split into three bf16 parts on the bf16 matrix cores (split.h:
// six products per k pair, fp32-level error, 2.7x the fp32-MFMA rate).  The weights are staged in
// LDS already split, once per workgroup.  The split Wp and Wm together would need 184 KB, so a
// workgroup runs its tiles in two phases, one weight resident per phase: forward (1) xp = Wp x,
// stored, (2) z = Wm [q | xp] re-reading its own xp rows (L2-hot) + LayerNorm; backward (1) the
// LayerNorm backward, dxp and dq with Wm^T, (2) dx = Wp^T dxp.  The first tile of each phase is
// loaded while the weight of that phase is staged.  D = 128 (Ren-MME) runs the exact fp32 MFMA
// path (its split Wm alone would need 210 KB of LDS).  bf16 path (MEP_PREC_BF16, every D): the
// same two-phase kernels with one bf16 part per operand -- one MFMA per k pair, fp32 accumulate,
// LayerNorm and dropout in fp32.
#include "common.h"
#include "split.h"

#ifndef MEP_EPI_ONE_BF16_MAXD
#define MEP_EPI_ONE_BF16_MAXD 96
#endif

using namespace mep;

namespace {

constexpr float LN_EPS = 1e-5f;
constexpr int EWAVES = 8;                 // waves per workgroup of the epilogues
constexpr int ETHREADS = 64 * EWAVES;
#ifndef MEP_EPI_WAVES
#define MEP_EPI_WAVES 1    // minimum waves per SIMD the epilogue kernels are register-limited to
#endif

MEP_DEV float4 f4(const f32x4 v) { return make_float4(v[0], v[1], v[2], v[3]); }

// tiles [t_begin, t_end) of 16 tokens owned by this workgroup (contiguous range per workgroup)
// The epilogue grid is (slices, descriptors).  XCD-aware order: workgroups are
// dispatched to the 8 XCDs round-robin by linear id, so id -> (descriptor, slice) is remapped to
// give XCD x a contiguous run of the descriptor-major work list -- every XCD then stages the
// weights of one or two blocks instead of all of them, and its L2 serves the other workgroups'
// staging reads of those weights (the first reads of each block's weights come from MALL / HBM
// once per XCD, not once per workgroup).
MEP_DEV bool epi_slot(int& desc, int& slice) {
    const int G = gridDim.x * gridDim.y, id = blockIdx.x + gridDim.x * blockIdx.y;
    // XCD x = id % 8 holds q + (x < r) of the G workgroups (G = 8 q + r): the x-th run
    const int q = G / 8, r = G % 8, x = id % 8;
    const int unit = x * q + min(x, r) + id / 8;
    desc = unit / (int)gridDim.x;
    slice = unit - desc * (int)gridDim.x;
    return true;
}
MEP_DEV bool tile_range(int ntok, int slice, int& t_begin, int& t_end) {
    const int ntiles = (ntok + 15) >> 4;
    const int per = (ntiles + (int)gridDim.x - 1) / (int)gridDim.x;
    t_begin = slice * per;
    t_end = min(ntiles, t_begin + per);
    return t_begin < t_end;
}

// upstream gradient of token tc (clamped in range), features col .. col+3: the dout row view, or
// with pool_T != 0 the mean+max pool's backward formed in registers -- exactly k_pool_bwd's dx
// (pool_head.hip: dmean = dpooled / T, + dmax at the argmax step), so the pooled tensor's gradient
// [B, T, C] is never written or read (cmu-mosei/run.py:314-318).  pool_T < 0: the head already
// wrote the mean half of dpooled divided by |pool_T| (the same division, done once per column).
// dmean = the mean half / T, IEEE division (pool_T > 0, no plan of this repository): out of line, so
// the compiler cannot evaluate it speculatively on the pool_T < 0 path and select the result (it
// did: ~10 VALU per element of every tile)
__attribute__((noinline)) MEP_DEV f32x4 pool_div(f32x4 m, int T) {
    f32x4 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = m[r] / (float)T;
    return v;
}
struct Upstream {
    const gfloat* dp;      // pool: this block's columns of dpooled (mean part; max part at + C)
    const MEP_G int* am;   // pool: this block's columns of argmax
    int C, T, Tq, t0;
    MEP_DEV explicit Upstream(const mep_epi_bwd_desc& bd)
        : dp(G<const float>(bd.pool_dpooled) + bd.pool_col), am(G<const int>(bd.pool_argmax) + bd.pool_col),
          C(bd.pool_C), T(bd.pool_T), Tq(bd.pool_Tq), t0(bd.pool_t0) {}
    MEP_DEV f32x4 at(const mep_epi_bwd_desc& bd, int tc, int col) const {
        if (T == 0) return ld4w(row_ptr(bd.dout, tc) + col);
        int b, tq;
        tok_split(tc, Tq, b, tq);
        const int tg = t0 + tq;
        const gfloat* p = dp + (int64_t)__umul24((unsigned)b, (unsigned)(2 * C)) + col;
        const f32x4 mean = ld4w(p), mx = ld4w(p + C);
        // the indices as an integer vector: as float bits they would be denormals, which float
        // moves/selects may flush to zero
        typedef MEP_G const u32x4 gu32x4;
        const u32x4 a = *reinterpret_cast<gu32x4*>(am + (int64_t)__umul24((unsigned)b, (unsigned)C) + col);
        const f32x4 dm = T > 0 ? pool_div(mean, T) : mean;   // T < 0: divided by the head
        f32x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = ((int)a[r] == tg) ? dm[r] + mx[r] : dm[r];
        return v;
    }
};

// ---------------------------------------------------------------- forward
// stage W [R][C] (fp32, row stride C) split into LDS: unit (n, p, g) = W[n][32p + 4g ..] and
// W[n][32p + 16 + 4g ..]; every load of the thread is issued before its first LDS write
template <int R, int C, int NPART, int NT = ETHREADS>
MEP_DEV void stage_split_rows(const SplitW<R, C / 32, NPART>& dst, const gfloat* src) {
    constexpr int NU = R * (C / 32) * 4;
    constexpr int PER = (NU + NT - 1) / NT;
    f32x4 v[PER][2];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int u = threadIdx.x + NT * k;
        if (u < NU) {
            const int g = u & 3, pp = (u >> 2) % (C / 32), n = (u >> 2) / (C / 32);
            v[k][0] = ld4w(src + n * C + 32 * pp + 4 * g);
            v[k][1] = ld4w(src + n * C + 32 * pp + 16 + 4 * g);
        }
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int u = threadIdx.x + NT * k;
        if (u < NU) {
            const int g = u & 3, pp = (u >> 2) % (C / 32), n = (u >> 2) / (C / 32);
            dst.put(n, pp, g, v[k][0], v[k][1]);
        }
    }
}

// stage W^T of W [R][C] (fp32, row stride C) split into LDS (rows = the C columns of W, k = the R
// rows): unit (n, p, g) = W[32p + 4g + j][n] and W[32p + 16 + 4g + j][n], j < 4; consecutive
// threads take consecutive n (coalesced), loads issued before the LDS writes
template <int R, int C, int NPART, int NT = ETHREADS>
MEP_DEV void stage_split_cols(const SplitW<C, R / 32, NPART>& dst, const gfloat* src) {
    constexpr int NP = R / 32, NU = C * NP * 4;
    constexpr int PER = (NU + NT - 1) / NT;
    float v[PER][8];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int u = threadIdx.x + NT * k;
        if (u < NU) {
            const int n = u % C, pg = u / C, g = pg & 3, pp = pg >> 2;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                v[k][j] = src[(32 * pp + 4 * g + j) * C + n];
                v[k][4 + j] = src[(32 * pp + 16 + 4 * g + j) * C + n];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int u = threadIdx.x + NT * k;
        if (u < NU) {
            const int n = u % C, pg = u / C, g = pg & 3, pp = pg >> 2;
            dst.put(n, pp, g, f32x4{v[k][0], v[k][1], v[k][2], v[k][3]}, f32x4{v[k][4], v[k][5], v[k][6], v[k][7]});
        }
    }
}

// ---------------------------------------------------------------- split-bf16 epilogues (D <= 96)
// this workgroup's global stores done and visible to its own later loads (the next phase re-reads
// rows the other waves stored)
MEP_DEV void wg_store_barrier() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}


// the LayerNorm weight (and bias) into LDS with the weight staging (published by its barrier): the
// per-tile LayerNorm then reads them from LDS instead of waiting on a global load at every tile's end
template <int D, bool BIAS>
MEP_DEV void stage_ln(lfloat* dst, const mep_epi_desc& d) {
    const int t = threadIdx.x;
    if (t < D) dst[t] = G<const float>(d.ln_w)[t];
    else if (BIAS && t < 2 * D) dst[t] = G<const float>(d.ln_b)[t - D];
}

template <int D, int NPART, int NW, bool DROP>
MEP_DEV void epi_fwd_split(const mep_epi_desc& d, unsigned char* sm, int t_begin, int t_end) {
    constexpr int NI = D / 16, KB = D / 16, NP = D / 32;
    using WP = SplitW<D, NP, NW>;
    using WM = SplitW<D, 2 * NP, NW>;
    using Op = OpN<NPART>;
    constexpr bool HS = NPART == 1;      // bf16 path: bf16 activations (common.h ld4a / st4a)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int ntok = d.ntok;
    const float p = DROP ? d.drop_p : 0.f;
    const uint64_t seed = (d.seed && p > 0.f) ? *G<const uint64_t>(d.seed) : 0;
    // global token offset of this shard's rows (seed[1] = the rank's first global batch row)
    const uint64_t tok0 = (d.seed && p > 0.f) ? G<const uint64_t>(d.seed)[1] * (uint64_t)d.q.T : 0;
    const uint64_t dbits = p > 0.f ? d.drop_bits : 0;   // the forward's keep bits (0: hash)
    const bool have_bits = dbits != 0;
    const float keep_s = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;   // == drop_scale's kept value
    (void)have_bits; (void)keep_s;
    gfloat* stats = G<float>(d.stats);
    typedef __attribute__((address_space(3))) unsigned char lbyte;
    const WP wp{(lbyte*)sm, 0};
    const WM wm{(lbyte*)sm, 0};
    f32x4 ab[KB], bb[KB];            // one tile ahead: phase 1 x rows; phase 2 q and xp rows
    auto rows_of = [&](const mep_rows& v, int tile, f32x4 (&dst)[KB]) {
        const auto r = rowa<HS>(v, min(tile * 16 + c, ntok - 1)) + 4 * g;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) dst[kb] = ld4a(r + 16 * kb);
    };
    // ---- phase 1: xp = drop(x Wp^T)
    if (t_begin + wave < t_end) rows_of(d.x, t_begin + wave, ab);
    stage_split_rows<D, D, NW>(wp, G<const float>(d.wp));
    __syncthreads();
    for (int tile = t_begin + wave; tile < t_end; tile += EWAVES) {
        const int tok = tile * 16 + c;
        Op xs[NP];
#pragma unroll
        for (int pp = 0; pp < NP; ++pp) xs[pp] = opn<NPART>(ab[2 * pp], ab[2 * pp + 1]);
        if (tile + EWAVES < t_end) rows_of(d.x, tile + EWAVES, ab);
        f32x4 xp[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) xp[i] = zero_f4();
        tgemm_n<NI, NP, NPART, NW>(xp, [&](int i, int pp) { return wp.frag(i, pp); }, [&](int pp) { return xs[pp]; });
        if (tok < ntok) {
            const auto pr = rowa<HS>(d.xp, tok);
            uint32_t kb0 = 0;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                if (p > 0.f) {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        xp[i][r] *= drop_rec(seed, 2u * d.drop_stream, (tok0 + (uint64_t)tok) * D + 16 * i + 4 * g + r, p, kb0, 4 * i + r);
                }
                st4a(pr + 16 * i + 4 * g, xp[i]);
            }
            if (p > 0.f) drop_bits_put(drop_bits_ptr(dbits, tok, 0), kb0);
        }
    }
    // ---- phase 2: z = [q | xp] Wm^T, out = drop(LayerNorm(z))
    if (t_begin + wave < t_end) rows_of(d.q, t_begin + wave, ab);
    wg_store_barrier();              // xp rows stored; Wp no longer read
    if (t_begin + wave < t_end) rows_of(d.xp, t_begin + wave, bb);
    stage_split_rows<D, 2 * D, NW>(wm, G<const float>(d.wm));
    __syncthreads();
    for (int tile = t_begin + wave; tile < t_end; tile += EWAVES) {
        const int tok = tile * 16 + c;
        Op qs[NP], ps[NP];
#pragma unroll
        for (int pp = 0; pp < NP; ++pp) { qs[pp] = opn<NPART>(ab[2 * pp], ab[2 * pp + 1]); ps[pp] = opn<NPART>(bb[2 * pp], bb[2 * pp + 1]); }
        if (tile + EWAVES < t_end) { rows_of(d.q, tile + EWAVES, ab); rows_of(d.xp, tile + EWAVES, bb); }
        f32x4 z[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) z[i] = zero_f4();
        tgemm_n<NI, NP, NPART, NW>(z, [&](int i, int pp) { return wm.frag(i, pp); }, [&](int pp) { return qs[pp]; });
        tgemm_n<NI, NP, NPART, NW>(z, [&](int i, int pp) { return wm.frag(i, NP + pp); }, [&](int pp) { return ps[pp]; });
        float sum = 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i) sum += (z[i][0] + z[i][1]) + (z[i][2] + z[i][3]);
        sum += __shfl_xor(sum, 16, 64);
        sum += __shfl_xor(sum, 32, 64);
        const float mean = sum / (float)D;
        float var = 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) { const float t = z[i][r] - mean; var += t * t; }
        var += __shfl_xor(var, 16, 64);
        var += __shfl_xor(var, 32, 64);
        const float rstd = 1.0f / sqrtf(var / (float)D + LN_EPS);
        if (tok < ntok) {
            const auto zr = rowa<HS>(d.z, tok);
            gfloat* orow = row_ptr(d.out, tok);
            const auto hrow = (HS && d.out_h.ptr) ? rowa<true>(d.out_h, tok) : nullptr;   // next layer's q
            uint32_t kb1 = 0;   // keep bits of the out site
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const int col = 16 * i + 4 * g;
                const f32x4 w = ld4w(G<const float>(d.ln_w) + col), b = ld4w(G<const float>(d.ln_b) + col);
                f32x4 y;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    y[r] = (z[i][r] - mean) * rstd * w[r] + b[r];
                    if (p > 0.f) y[r] *= drop_rec(seed, 2u * d.drop_stream + 1u, (tok0 + (uint64_t)tok) * D + col + r, p, kb1, 4 * i + r);
                }
                st4a(zr + col, z[i]);
                stg4(orow + col, f4(y));
                if (HS && d.out_h.ptr) st4a(hrow + col, y);
            }
            if (p > 0.f) drop_bits_put(drop_bits_ptr(dbits, tok, 1), kb1);
            if (g == 0) { stats[2 * tok] = mean; stats[2 * tok + 1] = rstd; }
        }
    }
}

template <int D, int NPART, int NW, bool DROP>
MEP_DEV void epi_bwd_split(const mep_epi_bwd_desc& bd, unsigned char* sm, int t_begin, int t_end) {
    constexpr int NI = D / 16, KB = D / 16, NP = D / 32;
    using WMT = SplitW<2 * D, NP, NW>;
    using WPT = SplitW<D, NP, NW>;
    using Op = OpN<NPART>;
    constexpr bool HS = NPART == 1;      // bf16 path: bf16 activations and their gradients
    const mep_epi_desc& d = bd.f;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int ntok = d.ntok;
    const float p = DROP ? d.drop_p : 0.f;
    const uint64_t seed = (d.seed && p > 0.f) ? *G<const uint64_t>(d.seed) : 0;
    // global token offset of this shard's rows (seed[1] = the rank's first global batch row)
    const uint64_t tok0 = (d.seed && p > 0.f) ? G<const uint64_t>(d.seed)[1] * (uint64_t)d.q.T : 0;
    const uint64_t dbits = p > 0.f ? d.drop_bits : 0;   // the forward's keep bits (0: hash)
    const bool have_bits = dbits != 0;
    const float keep_s = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;   // == drop_scale's kept value
    (void)have_bits; (void)keep_s;
    const gfloat* stats = G<const float>(d.stats);
    gfloat* lpart = G<float>(bd.ln_partial);
    typedef __attribute__((address_space(3))) unsigned char lbyte;
    const WMT wmt{(lbyte*)sm, 0};
    const WMT wmt_x{(lbyte*)sm, D};
    const WPT wpt{(lbyte*)sm, 0};
    f32x4 ga[KB], zb[KB];            // one tile ahead: dout (+ dout2) and z rows
    float mean = 0.f, rstd = 0.f;
    const Upstream up(bd);
    auto fetch1 = [&](int tile) {
        const int tc = min(tile * 16 + c, ntok - 1);
        const auto zr = rowa<HS>(d.z, tc) + 4 * g;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) ga[kb] = up.at(bd, tc, 16 * kb + 4 * g);
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) zb[kb] = ld4a(zr + 16 * kb);
        mean = stats[2 * tc];
        rstd = stats[2 * tc + 1];
    };
    // ---- phase 1: LayerNorm backward, dxp = drop'(dz Wm[:, D:]), dq (+)= dz Wm[:, :D]
    if (t_begin + wave < t_end) fetch1(t_begin + wave);
    stage_split_cols<D, 2 * D, NW>(wmt, G<const float>(d.wm));
    __syncthreads();
    for (int tile = t_begin + wave; tile < t_end; tile += EWAVES) {
        const int tok = tile * 16 + c;
        const uint32_t kbb0 = have_bits ? drop_bits_get(drop_bits_ptr(dbits, tok, 0)) : 0u;   // the forward's keep bits
        const uint32_t kbb1 = have_bits ? drop_bits_get(drop_bits_ptr(dbits, tok, 1)) : 0u;
        const bool ok = tok < ntok;
        const int tc = min(tok, ntok - 1);
        f32x4 dz[NI], zz[NI];
        const float mu = mean, rs = rstd;
#pragma unroll
        for (int i = 0; i < NI; ++i) { dz[i] = ga[i]; zz[i] = zb[i]; }
        if (bd.dout2.ptr) {
            const auto g2 = rowa<HS>(bd.dout2, tc) + 4 * g;
#pragma unroll
            for (int i = 0; i < NI; ++i) dz[i] += ld4a(g2 + 16 * i);
        }
        if (tile + EWAVES < t_end) fetch1(tile + EWAVES);
        float s1 = 0.f, s2 = 0.f;
        gfloat* lp = lpart ? lpart + (int64_t)tile * 2 * D : nullptr;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int col = 16 * i + 4 * g;
            const f32x4 w = ld4w(G<const float>(d.ln_w) + col);
            f32x4 pw, pb;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float gg = dz[i][r];
                if (p > 0.f) gg *= drop_use(have_bits, kbb1, 4 * i + r, keep_s, seed, 2u * d.drop_stream + 1u, (tok0 + (uint64_t)tok) * D + col + r, p);
                gg = ok ? gg : 0.f;
                const float x = (zz[i][r] - mu) * rs;
                const float gw = gg * w[r];
                s1 += gw;
                s2 += gw * x;
                pw[r] = row16_sum(gg * x);
                pb[r] = row16_sum(gg);
                dz[i][r] = gw;
            }
            if (lp && c == 0) {
                stg4(lp + col, f4(pw));
                stg4(lp + D + col, f4(pb));
            }
        }
        s1 += __shfl_xor(s1, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 16, 64);
        s2 += __shfl_xor(s2, 32, 64);
        s1 /= (float)D;
        s2 /= (float)D;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float x = (zz[i][r] - mu) * rs;
                dz[i][r] = ok ? rs * (dz[i][r] - s1 - x * s2) : 0.f;
            }
        Op dzb[NP];
#pragma unroll
        for (int pp = 0; pp < NP; ++pp) dzb[pp] = opn<NPART>(dz[2 * pp], dz[2 * pp + 1]);
        f32x4 acc[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[i] = zero_f4();
        tgemm_n<NI, NP, NPART, NW>(acc, [&](int i, int pp) { return wmt_x.frag(i, pp); }, [&](int pp) { return dzb[pp]; });
        if (ok) {
            const auto dzr = rowa<HS>(bd.dz, tok);
            const auto dpr = rowa<HS>(bd.dxp, tok);
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                if (p > 0.f) {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        acc[i][r] *= drop_use(have_bits, kbb0, 4 * i + r, keep_s, seed, 2u * d.drop_stream, (tok0 + (uint64_t)tok) * D + 16 * i + 4 * g + r, p);
                }
                st4a(dzr + 16 * i + 4 * g, dz[i]);
                st4a(dpr + 16 * i + 4 * g, acc[i]);
            }
        }
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[i] = zero_f4();
        tgemm_n<NI, NP, NPART, NW>(acc, [&](int i, int pp) { return wmt.frag(i, pp); }, [&](int pp) { return dzb[pp]; });
        if (ok) {
            const auto qrw = rowa<HS>(bd.dq, tok);
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                f32x4 v = acc[i];
                if (bd.dq_accumulate) v += ld4a(qrw + 16 * i + 4 * g);
                st4a(qrw + 16 * i + 4 * g, v);
            }
        }
    }
    // ---- phase 2: dx = dxp Wp (this workgroup's own dxp rows, L2-hot)
    wg_store_barrier();
    auto fetch2 = [&](int tile) {
        const auto r = rowa<HS>(bd.dxp, min(tile * 16 + c, ntok - 1)) + 4 * g;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) ga[kb] = ld4a(r + 16 * kb);
    };
    if (t_begin + wave < t_end) fetch2(t_begin + wave);
    stage_split_cols<D, D, NW>(wpt, G<const float>(d.wp));
    __syncthreads();
    for (int tile = t_begin + wave; tile < t_end; tile += EWAVES) {
        const int tok = tile * 16 + c;
        Op xs[NP];
#pragma unroll
        for (int pp = 0; pp < NP; ++pp) xs[pp] = opn<NPART>(ga[2 * pp], ga[2 * pp + 1]);
        if (tile + EWAVES < t_end) fetch2(tile + EWAVES);
        f32x4 acc[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[i] = zero_f4();
        tgemm_n<NI, NP, NPART, NW>(acc, [&](int i, int pp) { return wpt.frag(i, pp); }, [&](int pp) { return xs[pp]; });
        if (tok < ntok) {
            const auto xrw = rowa<HS>(bd.dx, tok);
#pragma unroll
            for (int i = 0; i < NI; ++i) st4a(xrw + 16 * i + 4 * g, acc[i]);
        }
    }
}

// ---------------------------------------------------------------- single-phase split epilogues
// Both weights resident in LDS for the whole workgroup, one pass per tile: the first product's
// accumulators (C[feature 16 i + 4g + r][token c]) are exactly the B fragments of the second
// product's k blocks (lane (token c, g): features 16 i + 4g .. +3), so xp (forward) and dxp
// (backward) go from accumulators to operands in registers -- no store-and-reload of the
// intermediate, one staging, no second phase.  Parts per weight (NWP, NWM) are chosen so both fit
// the 160 KB of LDS: D = 96 keeps Wp as two parts (forward; 43 + 120 KB) and Wm^T as two parts
// (backward; 86 + 65 KB) -- a 2^-18 relative representation error of that weight.
// DROP: a launch with dropout (drop_p > 0); the no-dropout instance has no hash code at all (the
// dropout hash is most of the loop's instructions: a smaller, branch-free body)
template <int D, int NPART, int NWP, int NWM, bool DROP, int NW = EWAVES>
MEP_DEV void epi_fwd_one(const mep_epi_desc& d, unsigned char* sm, int t_begin, int t_end) {
    constexpr int NI = D / 16, KB = D / 16, NP = D / 32;
    using WP = SplitW<D, NP, NWP>;
    using WM = SplitW<D, 2 * NP, NWM>;
    constexpr bool HS = NPART == 1;      // bf16 path: bf16 activations (common.h ld4a / st4a)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int ntok = d.ntok;
    const float p = DROP ? d.drop_p : 0.f;
    const uint64_t seed = (d.seed && p > 0.f) ? *G<const uint64_t>(d.seed) : 0;
    const uint64_t tok0 = (d.seed && p > 0.f) ? G<const uint64_t>(d.seed)[1] * (uint64_t)d.q.T : 0;
    const uint64_t dbits = p > 0.f ? d.drop_bits : 0;   // the forward's keep bits (0: hash)
    const bool have_bits = dbits != 0;
    const float keep_s = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;   // == drop_scale's kept value
    (void)have_bits; (void)keep_s;
    gfloat* stats = G<float>(d.stats);
    typedef __attribute__((address_space(3))) unsigned char lbyte;
    const WP wp{(lbyte*)sm, 0};
    const WM wm{(lbyte*)sm + WP::BYTES, 0};
    f32x4 ab[KB], bb[KB];            // one tile ahead: x and q rows
    auto rows_of = [&](const mep_rows& v, int tile, f32x4 (&dst)[KB]) {
        const auto r = rowa<HS>(v, min(tile * 16 + c, ntok - 1)) + 4 * g;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) dst[kb] = ld4a(r + 16 * kb);
    };
    __shared__ __attribute__((aligned(16))) float lnp[2 * D];   // LayerNorm weight | bias
    stage_ln<D, true>((lfloat*)lnp, d);
    if (t_begin + wave < t_end) { rows_of(d.x, t_begin + wave, ab); rows_of(d.q, t_begin + wave, bb); }
    stage_split_rows<D, D, NWP, 64 * NW>(wp, G<const float>(d.wp));
    stage_split_rows<D, 2 * D, NWM, 64 * NW>(wm, G<const float>(d.wm));
    __syncthreads();
    for (int tile = t_begin + wave; tile < t_end; tile += NW) {
        const int tok = tile * 16 + c;
        f32x4 xp[NI], z[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) { xp[i] = zero_f4(); z[i] = zero_f4(); }
        {
            OpN<NPART> xs[NP];
#pragma unroll
            for (int pp = 0; pp < NP; ++pp) xs[pp] = opn<NPART>(ab[2 * pp], ab[2 * pp + 1]);
            if (tile + NW < t_end) rows_of(d.x, tile + NW, ab);
            tgemm_n<NI, NP, NPART, NWP>(xp, [&](int i, int pp) { return wp.frag(i, pp); }, [&](int pp) { return xs[pp]; });
        }
        OpN<NPART> qs[NP];
#pragma unroll
        for (int pp = 0; pp < NP; ++pp) qs[pp] = opn<NPART>(bb[2 * pp], bb[2 * pp + 1]);
        if (tile + NW < t_end) rows_of(d.q, tile + NW, bb);
        if (p > 0.f) {
            uint32_t kb0 = 0;
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    xp[i][r] *= drop_rec(seed, 2u * d.drop_stream, (tok0 + (uint64_t)tok) * D + 16 * i + 4 * g + r, p, kb0, 4 * i + r);
            drop_bits_put(drop_bits_ptr(dbits, tok, 0), kb0);
        }
        OpN<NPART> ps[NP];
#pragma unroll
        for (int pp = 0; pp < NP; ++pp) ps[pp] = opn<NPART>(xp[2 * pp], xp[2 * pp + 1]);
        tgemm_n<NI, NP, NPART, NWM>(z, [&](int i, int pp) { return wm.frag(i, pp); }, [&](int pp) { return qs[pp]; });
        tgemm_n<NI, NP, NPART, NWM>(z, [&](int i, int pp) { return wm.frag(i, NP + pp); }, [&](int pp) { return ps[pp]; });
        float sum = 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i) sum += (z[i][0] + z[i][1]) + (z[i][2] + z[i][3]);
        sum += __shfl_xor(sum, 16, 64);
        sum += __shfl_xor(sum, 32, 64);
        const float mean = sum / (float)D;
        float var = 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) { const float t = z[i][r] - mean; var += t * t; }
        var += __shfl_xor(var, 16, 64);
        var += __shfl_xor(var, 32, 64);
        const float rstd = 1.0f / sqrtf(var / (float)D + LN_EPS);
        if (tok < ntok) {
            const auto zr = rowa<HS>(d.z, tok);
            gfloat* orow = row_ptr(d.out, tok);
            const auto pr = rowa<HS>(d.xp, tok);
            const auto hrow = (HS && d.out_h.ptr) ? rowa<true>(d.out_h, tok) : nullptr;   // next layer's q
            uint32_t kb1 = 0;   // keep bits of the out site
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const int col = 16 * i + 4 * g;
                const f32x4 w = ld4w((const lfloat*)lnp + col), b = ld4w((const lfloat*)lnp + D + col);
                f32x4 y;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    y[r] = (z[i][r] - mean) * rstd * w[r] + b[r];
                    if (p > 0.f) y[r] *= drop_rec(seed, 2u * d.drop_stream + 1u, (tok0 + (uint64_t)tok) * D + col + r, p, kb1, 4 * i + r);
                }
                st4a(pr + col, xp[i]);
                st4a(zr + col, z[i]);
                stg4(orow + col, f4(y));
                if (HS && d.out_h.ptr) st4a(hrow + col, y);
            }
            if (p > 0.f) drop_bits_put(drop_bits_ptr(dbits, tok, 1), kb1);
            if (g == 0) { stats[2 * tok] = mean; stats[2 * tok + 1] = rstd; }
        }
    }
}

// Single-phase fp32 forward at D = 96 with all six products of the 3-part split on both products
// (fp32-level, like the two-phase kernel).  LDS (unpadded, swizzled SplitWS layouts) holds the
// 3-part Wm (108 KB), Wp's first two parts (36 KB) and Wp's third part for rows 0 .. 16 (NI - 1)
// - 1 (15 KB: 159 KB in all); the third part of the last 16 rows -- used only in the product
// w2 x0 -- is held in registers (each wave splits its NP fragments of the fp32 Wp once, 4 NP
// VGPRs).  Per tile: x (loaded a tile ahead) -> xp = Wp x, stored; the tile's q rows are loaded
// at its start, behind the xp product; z = Wm [q | xp] with xp from the accumulators; LayerNorm.
// Against the two-phase kernel the xp rows are not re-read, the weights are staged once, and no
// phase barrier splits the workgroup's tiles.
template <int D>
struct EpiWp2r {
    static constexpr int NI = D / 16, NP = D / 32, R2 = D - 16;
    using WP01 = SplitWS<D, NP, 2>;
    using WP2 = SplitWS<R2, NP, 1>;
    using WM = SplitWS<D, 2 * NP, 3>;
    static constexpr int BYTES = WP01::BYTES + WP2::BYTES + WM::BYTES;
};

template <int D>
MEP_DEV void epi_fwd_wp2r(const mep_epi_desc& d, unsigned char* sm, int t_begin, int t_end) {
    using E = EpiWp2r<D>;
    constexpr int NI = E::NI, KB = D / 16, NP = E::NP, R2 = E::R2;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int ntok = d.ntok;
    gfloat* stats = G<float>(d.stats);
    typedef __attribute__((address_space(3))) unsigned char lbyte;
    const typename E::WP01 wp{(lbyte*)sm, 0};
    const typename E::WP2 wp2{(lbyte*)sm + E::WP01::BYTES, 0};
    const typename E::WM wm{(lbyte*)sm + E::WP01::BYTES + E::WP2::BYTES, 0};
    auto rows_of = [&](const mep_rows& v, int tile, f32x4 (&dst)[KB]) {
        const gfloat* r = row_ptr(v, min(tile * 16 + c, ntok - 1)) + 4 * g;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) dst[kb] = ld4w(r + 16 * kb);
    };
    __shared__ __attribute__((aligned(16))) float lnp[2 * D];   // LayerNorm weight | bias
    stage_ln<D, true>((lfloat*)lnp, d);
    f32x4 ab[KB], bb[KB];            // x rows and q rows, one tile ahead
    if (t_begin + wave < t_end) { rows_of(d.x, t_begin + wave, ab); rows_of(d.q, t_begin + wave, bb); }
    const gfloat* W = G<const float>(d.wp);
    // the third part of the last 16 rows' fragments: unit (row R2 + c, k pair pp, group g)
    bf16x8 w2r[NP];
#pragma unroll
    for (int pp = 0; pp < NP; ++pp) {
        const gfloat* r = W + (R2 + c) * D + 32 * pp + 4 * g;
        w2r[pp] = opn<3>(ld4w(r), ld4w(r + 16)).p[2];
    }
    {   // Wp: unit (n, pp, g) = Wp[n][32 pp + 4 g ..], [.. + 16 ..] -> parts 0, 1 (and 2 for n < R2)
        constexpr int NU = D * NP * 4, PER = (NU + ETHREADS - 1) / ETHREADS;
        f32x4 v[PER][2];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int u = threadIdx.x + ETHREADS * k;
            if (u < NU) {
                const int gg = u & 3, pp = (u >> 2) % NP, n = (u >> 2) / NP;
                v[k][0] = ld4w(W + n * D + 32 * pp + 4 * gg);
                v[k][1] = ld4w(W + n * D + 32 * pp + 16 + 4 * gg);
            }
        }
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int u = threadIdx.x + ETHREADS * k;
            if (u < NU) {
                const int gg = u & 3, pp = (u >> 2) % NP, n = (u >> 2) / NP;
                const Parts<3> lo = splitv<3>(v[k][0]), hi = splitv<3>(v[k][1]);
                wp.put_part(0, n, pp, gg, lo.p[0], hi.p[0]);
                wp.put_part(1, n, pp, gg, lo.p[1], hi.p[1]);
                if (n < R2) wp2.put_part(0, n, pp, gg, lo.p[2], hi.p[2]);
            }
        }
    }
    {   // Wm [D][2D]: unit (n, pp, g), all three parts
        constexpr int NU = D * 2 * NP * 4, PER = (NU + ETHREADS - 1) / ETHREADS;
        const gfloat* M = G<const float>(d.wm);
        f32x4 v[PER][2];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int u = threadIdx.x + ETHREADS * k;
            if (u < NU) {
                const int gg = u & 3, pp = (u >> 2) % (2 * NP), n = (u >> 2) / (2 * NP);
                v[k][0] = ld4w(M + n * 2 * D + 32 * pp + 4 * gg);
                v[k][1] = ld4w(M + n * 2 * D + 32 * pp + 16 + 4 * gg);
            }
        }
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int u = threadIdx.x + ETHREADS * k;
            if (u < NU) {
                const int gg = u & 3, pp = (u >> 2) % (2 * NP), n = (u >> 2) / (2 * NP);
                const Parts<3> lo = splitv<3>(v[k][0]), hi = splitv<3>(v[k][1]);
#pragma unroll
                for (int t = 0; t < 3; ++t) wm.put_part(t, n, pp, gg, lo.p[t], hi.p[t]);
            }
        }
    }
    __syncthreads();
    for (int tile = t_begin + wave; tile < t_end; tile += EWAVES) {
        const int tok = tile * 16 + c;
        f32x4 xp[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) xp[i] = zero_f4();
        // the six products in mma_nm<3, 3>'s order: w0x0, w1x0, w0x1, w1x1, w2x0, w0x2; operands
        // are split one k pair at a time; the weight fragments of step s + RING (steps (pp, i),
        // pp-major) are read while step s's MFMAs run (MEP_TG_RING, as tgemm_n)
        {
            struct Frag { OpN<2> a; bf16x8 a2; };
            auto frag = [&](int s) {
                const int pp = s / NI, i = s % NI;
                return Frag{wp.frag(i, pp), i < NI - 1 ? wp2.frag(i, pp).p[0] : w2r[pp]};
            };
            constexpr int S = NI * NP, RING = MEP_TG_RING > 0 ? (MEP_TG_RING < S ? MEP_TG_RING : S) : 1;
            Frag ring[RING];
#pragma unroll
            for (int s = 0; s < RING; ++s) ring[s] = frag(s);
            OpN<3> xs;
#pragma unroll
            for (int s = 0; s < S; ++s) {
                const int pp = s / NI, i = s % NI;
                if (i == 0) xs = opn<3>(ab[2 * pp], ab[2 * pp + 1]);
                const Frag f = ring[s % RING];
                if (s + RING < S) ring[s % RING] = frag(s + RING);
                f32x4 acc = xp[i];
                acc = mfma_bf16(f.a.p[0], xs.p[0], acc);
                acc = mfma_bf16(f.a.p[1], xs.p[0], acc);
                acc = mfma_bf16(f.a.p[0], xs.p[1], acc);
                acc = mfma_bf16(f.a.p[1], xs.p[1], acc);
                acc = mfma_bf16(f.a2, xs.p[0], acc);
                xp[i] = mfma_bf16(f.a.p[0], xs.p[2], acc);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (tile + EWAVES < t_end) rows_of(d.x, tile + EWAVES, ab);   // behind the z product
        if (tok < ntok) {
            gfloat* pr = row_ptr(d.xp, tok);
#pragma unroll
            for (int i = 0; i < NI; ++i) stg4(pr + 16 * i + 4 * g, f4(xp[i]));
        }
        f32x4 z[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) z[i] = zero_f4();
        tgemm_n<NI, NP, 3, 3>(z, [&](int i, int pp) { return wm.frag(i, pp); },
                              [&](int pp) { return opn<3>(bb[2 * pp], bb[2 * pp + 1]); });
        tgemm_n<NI, NP, 3, 3>(z, [&](int i, int pp) { return wm.frag(i, NP + pp); },
                              [&](int pp) { return opn<3>(xp[2 * pp], xp[2 * pp + 1]); });
        float sum = 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i) sum += (z[i][0] + z[i][1]) + (z[i][2] + z[i][3]);
        sum += __shfl_xor(sum, 16, 64);
        sum += __shfl_xor(sum, 32, 64);
        const float mean = sum / (float)D;
        float var = 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) { const float t = z[i][r] - mean; var += t * t; }
        var += __shfl_xor(var, 16, 64);
        var += __shfl_xor(var, 32, 64);
        const float rstd = 1.0f / sqrtf(var / (float)D + LN_EPS);
        // the next tile's q rows before this tile's stores: the wait for them (in-order vmcnt)
        // then does not wait for the stores
        if (tile + EWAVES < t_end) rows_of(d.q, tile + EWAVES, bb);
        if (tok < ntok) {
            gfloat* zr = row_ptr(d.z, tok);
            gfloat* orow = row_ptr(d.out, tok);
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const int col = 16 * i + 4 * g;
                const f32x4 w = ld4w((const lfloat*)lnp + col), b = ld4w((const lfloat*)lnp + D + col);
                f32x4 y;
#pragma unroll
                for (int r = 0; r < 4; ++r) y[r] = (z[i][r] - mean) * rstd * w[r] + b[r];
                stg4(zr + col, f4(z[i]));
                stg4(orow + col, f4(y));
            }
            if (g == 0) { stats[2 * tok] = mean; stats[2 * tok + 1] = rstd; }
        }
    }
}

template <int D, int NPART, int NWP, int NWM, bool DROP, int NW = EWAVES>
MEP_DEV void epi_bwd_one(const mep_epi_bwd_desc& bd, unsigned char* sm, int t_begin, int t_end) {
    constexpr int NI = D / 16, KB = D / 16, NP = D / 32;
    using WMT = SplitW<2 * D, NP, NWM>;
    using WPT = SplitW<D, NP, NWP>;
    using Op = OpN<NPART>;
    constexpr bool HS = NPART == 1;      // bf16 path: bf16 activations and their gradients
    const mep_epi_desc& d = bd.f;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int ntok = d.ntok;
    const float p = DROP ? d.drop_p : 0.f;
    const uint64_t seed = (d.seed && p > 0.f) ? *G<const uint64_t>(d.seed) : 0;
    const uint64_t tok0 = (d.seed && p > 0.f) ? G<const uint64_t>(d.seed)[1] * (uint64_t)d.q.T : 0;
    const uint64_t dbits = p > 0.f ? d.drop_bits : 0;   // the forward's keep bits (0: hash)
    const bool have_bits = dbits != 0;
    const float keep_s = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;   // == drop_scale's kept value
    (void)have_bits; (void)keep_s;
    const gfloat* stats = G<const float>(d.stats);
    gfloat* lpart = G<float>(bd.ln_partial);
    typedef __attribute__((address_space(3))) unsigned char lbyte;
    const WMT wmt{(lbyte*)sm, 0};
    const WMT wmt_x{(lbyte*)sm, D};
    const WPT wpt{(lbyte*)sm + WMT::BYTES, 0};
    f32x4 ga[KB], zb[KB];            // one tile ahead: dout (+ dout2) and z rows
    float mean = 0.f, rstd = 0.f;
    const Upstream up(bd);
    auto fetch1 = [&](int tile) {
        const int tc = min(tile * 16 + c, ntok - 1);
        const auto zr = rowa<HS>(d.z, tc) + 4 * g;
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) ga[kb] = up.at(bd, tc, 16 * kb + 4 * g);
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) zb[kb] = ld4a(zr + 16 * kb);
        mean = stats[2 * tc];
        rstd = stats[2 * tc + 1];
    };
    __shared__ __attribute__((aligned(16))) float lnp[D];   // LayerNorm weight
    stage_ln<D, false>((lfloat*)lnp, d);
    if (t_begin + wave < t_end) fetch1(t_begin + wave);
    stage_split_cols<D, 2 * D, NWM, 64 * NW>(wmt, G<const float>(d.wm));
    stage_split_cols<D, D, NWP, 64 * NW>(wpt, G<const float>(d.wp));
    __syncthreads();
    for (int tile = t_begin + wave; tile < t_end; tile += NW) {
        const int tok = tile * 16 + c;
        const uint32_t kbb0 = have_bits ? drop_bits_get(drop_bits_ptr(dbits, tok, 0)) : 0u;   // the forward's keep bits
        const uint32_t kbb1 = have_bits ? drop_bits_get(drop_bits_ptr(dbits, tok, 1)) : 0u;
        const bool ok = tok < ntok;
        const int tc = min(tok, ntok - 1);
        f32x4 dz[NI], zz[NI];
        const float mu = mean, rs = rstd;
#pragma unroll
        for (int i = 0; i < NI; ++i) { dz[i] = ga[i]; zz[i] = zb[i]; }
        if (bd.dout2.ptr) {
            const auto g2 = rowa<HS>(bd.dout2, tc) + 4 * g;
#pragma unroll
            for (int i = 0; i < NI; ++i) dz[i] += ld4a(g2 + 16 * i);
        }
        if (tile + NW < t_end) fetch1(tile + NW);
        float s1 = 0.f, s2 = 0.f;
        gfloat* lp = lpart ? lpart + (int64_t)tile * 2 * D : nullptr;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int col = 16 * i + 4 * g;
            const f32x4 w = ld4w((const lfloat*)lnp + col);
            f32x4 pw, pb;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float gg = dz[i][r];
                if (p > 0.f) gg *= drop_use(have_bits, kbb1, 4 * i + r, keep_s, seed, 2u * d.drop_stream + 1u, (tok0 + (uint64_t)tok) * D + col + r, p);
                gg = ok ? gg : 0.f;
                const float x = (zz[i][r] - mu) * rs;
                const float gw = gg * w[r];
                s1 += gw;
                s2 += gw * x;
                pw[r] = row16_sum(gg * x);
                pb[r] = row16_sum(gg);
                dz[i][r] = gw;
            }
            if (lp && c == 0) {
                stg4(lp + col, f4(pw));
                stg4(lp + D + col, f4(pb));
            }
        }
        s1 += __shfl_xor(s1, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 16, 64);
        s2 += __shfl_xor(s2, 32, 64);
        s1 /= (float)D;
        s2 /= (float)D;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float x = (zz[i][r] - mu) * rs;
                dz[i][r] = ok ? rs * (dz[i][r] - s1 - x * s2) : 0.f;
            }
        Op dzb[NP];
#pragma unroll
        for (int pp = 0; pp < NP; ++pp) dzb[pp] = opn<NPART>(dz[2 * pp], dz[2 * pp + 1]);
        f32x4 acc[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[i] = zero_f4();
        tgemm_n<NI, NP, NPART, NWM>(acc, [&](int i, int pp) { return wmt_x.frag(i, pp); }, [&](int pp) { return dzb[pp]; });
        if (p > 0.f) {
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    acc[i][r] *= drop_use(have_bits, kbb0, 4 * i + r, keep_s, seed, 2u * d.drop_stream, (tok0 + (uint64_t)tok) * D + 16 * i + 4 * g + r, p);
        }
        // dx = dxp Wp from the dxp accumulators (tokens past ntok: dz = 0, so dxp = 0)
        Op xs[NP];
#pragma unroll
        for (int pp = 0; pp < NP; ++pp) xs[pp] = opn<NPART>(acc[2 * pp], acc[2 * pp + 1]);
        if (ok) {
            const auto dzr = rowa<HS>(bd.dz, tok);
            const auto dpr = rowa<HS>(bd.dxp, tok);
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                st4a(dzr + 16 * i + 4 * g, dz[i]);
                st4a(dpr + 16 * i + 4 * g, acc[i]);
            }
        }
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[i] = zero_f4();
        tgemm_n<NI, NP, NPART, NWM>(acc, [&](int i, int pp) { return wmt.frag(i, pp); }, [&](int pp) { return dzb[pp]; });
        if (ok) {
            const auto qrw = rowa<HS>(bd.dq, tok);
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                f32x4 v = acc[i];
                if (bd.dq_accumulate) v += ld4a(qrw + 16 * i + 4 * g);
                st4a(qrw + 16 * i + 4 * g, v);
            }
        }
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[i] = zero_f4();
        tgemm_n<NI, NP, NPART, NWP>(acc, [&](int i, int pp) { return wpt.frag(i, pp); }, [&](int pp) { return xs[pp]; });
        if (ok) {
            const auto xrw = rowa<HS>(bd.dx, tok);
#pragma unroll
            for (int i = 0; i < NI; ++i) st4a(xrw + 16 * i + 4 * g, acc[i]);
        }
    }
}

// parts per weight of the single-phase epilogues (0: the two-phase kernels)
template <int D, bool BF16> struct EpiOne {
    // fp32 forward: single phase at D = 96 with all six products (epi_fwd_wp2r; a 2-part weight moved
    // one cmu_cfg3 logit 5e-4 relative), two phases below; fp32 backward: single phase for
    // D <= 96 (Wm^T as 2 parts); bf16 path: one part per weight, single phase
    static constexpr bool ON_BF = BF16 && D <= MEP_EPI_ONE_BF16_MAXD;
    static constexpr bool FWD = ON_BF || (!BF16 && D == 96), BWD = D <= 96 || ON_BF;
    static constexpr int NPART = BF16 ? 1 : 3;
    static constexpr bool FWD_WP2R = !BF16 && D == 96;
    static constexpr int FWD_WP = BF16 ? 1 : (D == 96 ? 2 : 3);
    static constexpr int FWD_WM = BF16 ? 1 : NPART;
    static constexpr int BWD_WP = NPART, BWD_WM = BF16 ? 1 : (D == 96 ? 2 : 3);
    static constexpr int FWD_BYTES = FWD_WP2R ? EpiWp2r<D>::BYTES : SplitW<D, D / 32, FWD_WP>::BYTES + SplitW<D, D / 16, FWD_WM>::BYTES;
    static constexpr int BWD_BYTES = SplitW<2 * D, D / 32, BWD_WM>::BYTES + SplitW<D, D / 32, BWD_WP>::BYTES;
    static_assert((!FWD || FWD_BYTES <= 163840) && (!BWD || BWD_BYTES <= 163840), "single-phase weights exceed the LDS");
};

// BF16: the bf16 path (one part per operand, every D); otherwise D <= 96 runs the 3-part split
// and D = 128 the fp32 MFMA path
template <int D, bool BF16>
__global__ __launch_bounds__(ETHREADS) __attribute__((amdgpu_waves_per_eu(MEP_EPI_WAVES))) void k_epi_fwd(const mep_epi_desc* __restrict__ descs) {
    int di, slice;
    if (!epi_slot(di, slice)) return;
    const mep_epi_desc& d = descs[di];
    int t_begin, t_end;
    if (!tile_range(d.ntok, slice, t_begin, t_end)) return;   // whole workgroup
    if constexpr (EpiOne<D, BF16>::FWD) {
        using E = EpiOne<D, BF16>;
        __shared__ __attribute__((aligned(16))) unsigned char sm1[E::FWD_BYTES];
        if constexpr (E::FWD_WP2R) {
            // dropout (Ren-MME; no D = 96 configuration runs it): the two-phase kernel
            if (d.drop_p > 0.f) epi_fwd_split<D, 3, 3, true>(d, sm1, t_begin, t_end);
            else epi_fwd_wp2r<D>(d, sm1, t_begin, t_end);
        } else {
            if (d.drop_p > 0.f) epi_fwd_one<D, E::NPART, E::FWD_WP, E::FWD_WM, true>(d, sm1, t_begin, t_end);
            else epi_fwd_one<D, E::NPART, E::FWD_WP, E::FWD_WM, false>(d, sm1, t_begin, t_end);
        }
        return;
    }
    constexpr int NPART = BF16 ? 1 : 3, NW = BF16 ? 1 : (D == 128 ? 2 : 3);
    constexpr int BYTES = SplitW<D, D / 16, NW>::BYTES;   // the larger phase (Wm)
    __shared__ __attribute__((aligned(16))) unsigned char sm6[BYTES];
    if (d.drop_p > 0.f) epi_fwd_split<D, NPART, NW, true>(d, sm6, t_begin, t_end);
    else epi_fwd_split<D, NPART, NW, false>(d, sm6, t_begin, t_end);
}

// ---------------------------------------------------------------- backward
// dout (+dout2) and z are read straight into the accumulator layout, the LayerNorm backward runs
// in registers, and dz^T feeds the products directly: dxp^T = Wm[:, D:]^T dz^T, dq^T =
// Wm[:, :D]^T dz^T and dx^T = Wp^T dxp^T; LayerNorm parameter partials per 16-token tile into its
// ln_partial row [2][D] (epi_bwd_one / epi_bwd_split).
template <int D, bool BF16>
__global__ __launch_bounds__(ETHREADS) __attribute__((amdgpu_waves_per_eu(MEP_EPI_WAVES))) void k_epi_bwd(const mep_epi_bwd_desc* __restrict__ descs) {
    int di, slice;
    if (!epi_slot(di, slice)) return;
    const mep_epi_bwd_desc& bd = descs[di];
    const mep_epi_desc& d = bd.f;
    int t_begin, t_end;
    if (!tile_range(d.ntok, slice, t_begin, t_end)) return;
    if constexpr (EpiOne<D, BF16>::BWD) {
        using E = EpiOne<D, BF16>;
        __shared__ __attribute__((aligned(16))) unsigned char sm1[E::BWD_BYTES];
        if (d.drop_p > 0.f) epi_bwd_one<D, E::NPART, E::BWD_WP, E::BWD_WM, true>(bd, sm1, t_begin, t_end);
        else epi_bwd_one<D, E::NPART, E::BWD_WP, E::BWD_WM, false>(bd, sm1, t_begin, t_end);
        return;
    }
    constexpr int NPART = BF16 ? 1 : 3, NW = BF16 ? 1 : (D == 128 ? 2 : 3);
    constexpr int BYTES = SplitW<2 * D, D / 32, NW>::BYTES;   // the larger phase (Wm^T)
    __shared__ __attribute__((aligned(16))) unsigned char sm6[BYTES];
    if (d.drop_p > 0.f) epi_bwd_split<D, NPART, NW, true>(bd, sm6, t_begin, t_end);
    else epi_bwd_split<D, NPART, NW, false>(bd, sm6, t_begin, t_end);
}

// The bf16 epilogue forward at D = 96 with MEP_EPI_FWD_BF16_NW waves per workgroup (as below;
// 168 VGPRs with 25 spilled; cfg3 bf16 18.2 -> 17.6 us)
#ifndef MEP_EPI_FWD_BF16_NW
#define MEP_EPI_FWD_BF16_NW 12
#endif
constexpr int EPI_FWD_BF16_NW = MEP_EPI_FWD_BF16_NW;
__global__ __launch_bounds__(64 * EPI_FWD_BF16_NW) void k_epi_fwd_bf16w(const mep_epi_desc* __restrict__ descs) {
    using E = EpiOne<96, true>;
    int di, slice;
    if (!epi_slot(di, slice)) return;
    const mep_epi_desc& d = descs[di];
    int t_begin, t_end;
    if (!tile_range(d.ntok, slice, t_begin, t_end)) return;
    __shared__ __attribute__((aligned(16))) unsigned char sm1[E::FWD_BYTES];
    if (d.drop_p > 0.f) epi_fwd_one<96, 1, E::FWD_WP, E::FWD_WM, true, EPI_FWD_BF16_NW>(d, sm1, t_begin, t_end);
    else epi_fwd_one<96, 1, E::FWD_WP, E::FWD_WM, false, EPI_FWD_BF16_NW>(d, sm1, t_begin, t_end);
}

// The bf16 epilogue backward at D = 96 with MEP_EPI_BWD_BF16_NW waves per workgroup (12: one
// 16-token tile per wave at one workgroup per CU over cfg3's 2,400 tiles, instead of two tiles on
// some of 8 waves; 3 waves per SIMD at <= 168 VGPRs, no spills): cfg3 bf16 25.6 -> 23.2 us
#ifndef MEP_EPI_BWD_BF16_NW
#define MEP_EPI_BWD_BF16_NW 12
#endif
constexpr int EPI_BWD_BF16_NW = MEP_EPI_BWD_BF16_NW;
__global__ __launch_bounds__(64 * EPI_BWD_BF16_NW) void k_epi_bwd_bf16w(const mep_epi_bwd_desc* __restrict__ descs) {
    using E = EpiOne<96, true>;
    int di, slice;
    if (!epi_slot(di, slice)) return;
    const mep_epi_bwd_desc& bd = descs[di];
    int t_begin, t_end;
    if (!tile_range(bd.f.ntok, slice, t_begin, t_end)) return;
    __shared__ __attribute__((aligned(16))) unsigned char sm1[E::BWD_BYTES];
    if (bd.f.drop_p > 0.f) epi_bwd_one<96, 1, E::BWD_WP, E::BWD_WM, true, EPI_BWD_BF16_NW>(bd, sm1, t_begin, t_end);
    else epi_bwd_one<96, 1, E::BWD_WP, E::BWD_WM, false, EPI_BWD_BF16_NW>(bd, sm1, t_begin, t_end);
}


// ---------------------------------------------------------------- row LayerNorm (D <= 256)
// forward: a workgroup takes LNF_ROWS x 4 rows (row 4i + wave of its range for wave `wave`), every
// load of a wave's rows issued before the first row's arithmetic (clamped tokens and columns, no
// branches); each row's arithmetic is unchanged.  Host grids stay ceil(ntok / 4) "tiles"; the
// launcher runs ceil(tiles / LNF_ROWS) workgroups.
constexpr int LNF_ROWS = 4;
// HS: bf16 x / y rows (mep_ln_desc.bf16 = MEP_BF16_STORE, the bf16 path); statistics stay fp32
template <bool HS>
MEP_DEV void ln_fwd_rows(const mep_ln_desc& d) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tok0 = blockIdx.x * 4 * LNF_ROWS + wave;
    if (tok0 >= d.ntok) return;
    const gfloat* w = G<const float>(d.w);
    const gfloat* b = G<const float>(d.b);
    float v[LNF_ROWS][4], wv[4], bv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = min(lane + 64 * j, d.D - 1);
        wv[j] = w[c];
        bv[j] = b[c];
    }
#pragma unroll
    for (int i = 0; i < LNF_ROWS; ++i) {
        const auto x = rowa<HS>(d.x, min(tok0 + 4 * i, d.ntok - 1));
#pragma unroll
        for (int j = 0; j < 4; ++j) v[i][j] = ld1a(x + min(lane + 64 * j, d.D - 1));
    }
#pragma unroll
    for (int i = 0; i < LNF_ROWS; ++i) {
        const int tok = tok0 + 4 * i;
        if (tok >= d.ntok) break;
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[i][j] = lane + 64 * j < d.D ? v[i][j] : 0.f; s += v[i][j]; }
        const float mean = wave_sum(s) / (float)d.D;
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) { const int c = lane + 64 * j; v[i][j] = c < d.D ? v[i][j] - mean : 0.f; q += v[i][j] * v[i][j]; }
        const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)d.D + LN_EPS);
        const auto y = rowa<HS>(d.y, tok);
#pragma unroll
        for (int j = 0; j < 4; ++j) { const int c = lane + 64 * j; if (c < d.D) st1a(y + c, v[i][j] * rstd * wv[j] + bv[j]); }
        if (lane == 0) {
            gfloat* st = G<float>(d.stats);
            st[2 * tok] = mean;
            st[2 * tok + 1] = rstd;
        }
    }
}

// 16 lanes per row (D <= 128, D % 8 == 0, 16-byte aligned rows): lane j of a 16-lane
// group holds features 8j .. 8j+7 of its row -- one 16-byte access per row and lane (two on the fp32
// path) instead of one 2- / 4-byte access per feature -- and the row sums are 16-lane DPP sums
// (row16_sum), not wave sums: a wave takes 4 rows at once.  Same workgroup geometry as the rows
// kernels above (forward 16 rows, backward 64 rows and one partial row per workgroup).
typedef unsigned u32x4g __attribute__((ext_vector_type(4)));
template <bool HS>
MEP_DEV void ln_ld8(const mep_rows& r, int tok, int c0, float (&v)[8]) {
    const auto p = rowa<HS>(r, tok) + c0;
    if constexpr (HS) {
        const u32x4g w = *reinterpret_cast<const MEP_G u32x4g*>(p);
#pragma unroll
        for (int e = 0; e < 4; ++e) { v[2 * e] = bf16_word_lo(w[e]); v[2 * e + 1] = bf16_word_hi(w[e]); }
    } else {
        const f32x4 a = ld4a(p), b = ld4a(p + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) { v[e] = a[e]; v[4 + e] = b[e]; }
    }
}
template <bool HS>
MEP_DEV void ln_st8(const mep_rows& r, int tok, int c0, const float (&v)[8]) {
    const auto p = rowa<HS>(r, tok) + c0;
    if constexpr (HS) {
        *reinterpret_cast<MEP_G u32x4g*>(p) = u32x4g{pk_bf16x2(v[0], v[1]), pk_bf16x2(v[2], v[3]),
                                                     pk_bf16x2(v[4], v[5]), pk_bf16x2(v[6], v[7])};
    } else {
        st4a(p, f32x4{v[0], v[1], v[2], v[3]});
        st4a(p + 4, f32x4{v[4], v[5], v[6], v[7]});
    }
}
MEP_DEV void ld8w(const gfloat* p, float (&v)[8]) {
    const f32x4 a = ld4w(p), b = ld4w(p + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[e] = a[e]; v[4 + e] = b[e]; }
}
MEP_DEV bool ln_rows16(const mep_rows& r, bool hs) {
    const int al = hs ? 8 : 4;
    return r.ptr % 16 == 0 && r.sB % al == 0 && r.sT % al == 0;
}
MEP_DEV bool ln_q_ok(const mep_ln_desc& d, bool fwd) {
    const bool hs = d.bf16 & MEP_BF16_STORE;
    if (d.D > 128 || d.D % 8 || d.w % 16 || d.b % 16 || !ln_rows16(d.x, hs)) return false;
    return fwd ? ln_rows16(d.y, hs) : (ln_rows16(d.dy, hs) && ln_rows16(d.dx, hs));
}

template <bool HS>
MEP_DEV void ln_fwd_q(const mep_ln_desc& d) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15;
    if (blockIdx.x * 16 >= d.ntok) return;                 // the whole workgroup
    const int tok = blockIdx.x * 16 + 4 * wave + (lane >> 4);
    const int c0 = 8 * j;
    const bool on = c0 < d.D;
    float v[8];
    ln_ld8<HS>(d.x, min(tok, d.ntok - 1), on ? c0 : 0, v);
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) { v[e] = on ? v[e] : 0.f; s += v[e]; }
    const float mean = row16_sum(s) / (float)d.D;
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) { v[e] = on ? v[e] - mean : 0.f; q += v[e] * v[e]; }
    const float rstd = 1.0f / sqrtf(row16_sum(q) / (float)d.D + LN_EPS);
    if (tok >= d.ntok) return;
    if (on) {
        float w[8], b[8];
        ld8w(G<const float>(d.w) + c0, w);
        ld8w(G<const float>(d.b) + c0, b);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = v[e] * rstd * w[e] + b[e];
        ln_st8<HS>(d.y, tok, c0, v);
    }
    if (j == 0) {
        gfloat* st = G<float>(d.stats);
        st[2 * tok] = mean;
        st[2 * tok + 1] = rstd;
    }
}

template <bool HS>
MEP_DEV void ln_bwd_q(const mep_ln_desc& d) {
    const int tok0 = blockIdx.x * 64;
    if (tok0 >= d.ntok) return;                            // the whole workgroup
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15;
    const int c0 = 8 * j;
    const bool on = c0 < d.D;
    const int cc = on ? c0 : 0;
    __shared__ float red[4][2][128];
    float wv[8], pw[8], pb[8];
    ld8w(G<const float>(d.w) + cc, wv);
#pragma unroll
    for (int e = 0; e < 8; ++e) pw[e] = pb[e] = 0.f;
    const gfloat* st = G<const float>(d.stats);
    constexpr int P = 4;                                   // rows 16 p + 4 wave + group of the 64
    float xv[P][8], gv[P][8], mean[P], rstd[P];
#pragma unroll
    for (int pp = 0; pp < P; ++pp) {
        const int tk = min(tok0 + 16 * pp + 4 * wave + (lane >> 4), d.ntok - 1);
        mean[pp] = st[2 * tk];
        rstd[pp] = st[2 * tk + 1];
        ln_ld8<HS>(d.x, tk, cc, xv[pp]);
        ln_ld8<HS>(d.dy, tk, cc, gv[pp]);
    }
#pragma unroll
    for (int pp = 0; pp < P; ++pp) {
        const int tok = tok0 + 16 * pp + 4 * wave + (lane >> 4);
        const bool ok = on && tok < d.ntok;                // rows past ntok: no contribution
        float xh[8], gw[8], s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float g = ok ? gv[pp][e] : 0.f;
            xh[e] = on ? (xv[pp][e] - mean[pp]) * rstd[pp] : 0.f;
            gw[e] = g * wv[e];
            pw[e] += g * xh[e];
            pb[e] += g;
            s1 += gw[e];
            s2 += gw[e] * xh[e];
        }
        s1 = row16_sum(s1) / (float)d.D;
        s2 = row16_sum(s2) / (float)d.D;
        if (ok) {
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = rstd[pp] * (gw[e] - s1 - xh[e] * s2);
            if (d.dx_accumulate) {
                float o[8];
                ln_ld8<HS>(d.dx, tok, c0, o);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] += o[e];
            }
            ln_st8<HS>(d.dx, tok, c0, v);
        }
    }
    // the wave's four row groups, then the workgroup's four waves, in a fixed order
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        pw[e] += __shfl_xor(pw[e], 16, 64);
        pw[e] += __shfl_xor(pw[e], 32, 64);
        pb[e] += __shfl_xor(pb[e], 16, 64);
        pb[e] += __shfl_xor(pb[e], 32, 64);
    }
    if (lane < 16 && on) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { red[wave][0][c0 + e] = pw[e]; red[wave][1][c0 + e] = pb[e]; }
    }
    __syncthreads();
    if (d.partial) {
        gfloat* lp = G<float>(d.partial) + (int64_t)blockIdx.x * 2 * d.D;
        for (int idx = threadIdx.x; idx < 2 * d.D; idx += 256) {
            const int which = idx / d.D, c = idx - which * d.D;
            lp[idx] = red[0][which][c] + red[1][which][c] + red[2][which][c] + red[3][which][c];
        }
    }
}

__global__ __launch_bounds__(256) void k_ln_fwd(const mep_ln_desc* __restrict__ descs) {
    const mep_ln_desc& d = descs[blockIdx.y];
    const bool hs = d.bf16 & MEP_BF16_STORE;
    if (ln_q_ok(d, true)) {
        if (hs) ln_fwd_q<true>(d);
        else ln_fwd_q<false>(d);
    } else if (hs) {
        ln_fwd_rows<true>(d);
    } else {
        ln_fwd_rows<false>(d);
    }
}

// backward; partial[blockIdx.x][2][D] = per-workgroup (dgamma, dbeta) over its 64 rows.  A wave
// takes rows wave, wave + 4, ... in batches of LNB_ROWS: every load of a batch (clamped columns and
// tokens, no branches) is issued before the batch's arithmetic, which runs row by row in the same
// order as one row at a time (bit-identical sums).
constexpr int LNB_ROWS = 4;
template <bool HS>
MEP_DEV void ln_bwd_rows(const mep_ln_desc& d) {
    const int tok0 = blockIdx.x * 64;
    if (tok0 >= d.ntok) return;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __shared__ float red[4][2][256];
    float pw[4] = {0.f, 0.f, 0.f, 0.f}, pb[4] = {0.f, 0.f, 0.f, 0.f};
    const gfloat* w = G<const float>(d.w);
    const gfloat* st = G<const float>(d.stats);
    float wv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) wv[j] = w[min(lane + 64 * j, d.D - 1)];
    for (int r0 = wave; r0 < 64; r0 += 4 * LNB_ROWS) {
        float gv[LNB_ROWS][4], xv[LNB_ROWS][4], mean[LNB_ROWS], rstd[LNB_ROWS];
#pragma unroll
        for (int i = 0; i < LNB_ROWS; ++i) {
            const int tk = min(tok0 + r0 + 4 * i, d.ntok - 1);
            mean[i] = st[2 * tk];
            rstd[i] = st[2 * tk + 1];
            const auto x = rowa<HS>(d.x, tk);
            const auto dy = rowa<HS>(d.dy, tk);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = min(lane + 64 * j, d.D - 1);
                gv[i][j] = ld1a(dy + c);
                xv[i][j] = ld1a(x + c);
            }
        }
#pragma unroll
        for (int i = 0; i < LNB_ROWS; ++i) {
            const int tok = tok0 + r0 + 4 * i;
            if (r0 + 4 * i >= 64 || tok >= d.ntok) break;
            float xh[4], gw[4], s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool ok = lane + 64 * j < d.D;
                const float g = ok ? gv[i][j] : 0.f;
                xh[j] = ok ? (xv[i][j] - mean[i]) * rstd[i] : 0.f;
                gw[j] = ok ? g * wv[j] : 0.f;
                pw[j] += g * xh[j];
                pb[j] += g;
                s1 += gw[j];
                s2 += gw[j] * xh[j];
            }
            s1 = wave_sum(s1) / (float)d.D;
            s2 = wave_sum(s2) / (float)d.D;
            const auto dx = rowa<HS>(d.dx, tok);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = lane + 64 * j;
                if (c < d.D) {
                    const float v = rstd[i] * (gw[j] - s1 - xh[j] * s2);
                    st1a(dx + c, d.dx_accumulate ? ld1a(dx + c) + v : v);
                }
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

__global__ __launch_bounds__(256) void k_ln_bwd(const mep_ln_desc* __restrict__ descs) {
    const mep_ln_desc& d = descs[blockIdx.y];
    const bool hs = d.bf16 & MEP_BF16_STORE;
    if (ln_q_ok(d, false)) {
        if (hs) ln_bwd_q<true>(d);
        else ln_bwd_q<false>(d);
    } else if (hs) {
        ln_bwd_rows<true>(d);
    } else {
        ln_bwd_rows<false>(d);
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
    const bool bf16 = D & MEP_PREC_BF16;
    if (bf16 && (D & ~MEP_PREC_BF16) == 96 && EPI_FWD_BF16_NW != EWAVES) {
        hipLaunchKernelGGL(k_epi_fwd_bf16w, dim3(max_tiles, n_desc), dim3(64 * EPI_FWD_BF16_NW), 0, (hipStream_t)stream, descs);
        return mep_check_launch("mep_block_epi_fwd");
    }
    const int rc = dispatch_D(D & ~MEP_PREC_BF16, [&](auto dc) {
        if (bf16) hipLaunchKernelGGL((k_epi_fwd<decltype(dc)::value, true>), dim3(max_tiles, n_desc), dim3(ETHREADS), 0,
                                     (hipStream_t)stream, descs);
        else hipLaunchKernelGGL((k_epi_fwd<decltype(dc)::value, false>), dim3(max_tiles, n_desc), dim3(ETHREADS), 0,
                                (hipStream_t)stream, descs);
    });
    if (rc) { mep_set_error("mep_block_epi_fwd: D must be 32, 64, 96 or 128"); return rc; }
    return mep_check_launch("mep_block_epi_fwd");
}

extern "C" int mep_block_epi_bwd(const mep_epi_bwd_desc* descs, int n_desc, int max_tiles, int D, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    const bool bf16 = D & MEP_PREC_BF16;
    if (bf16 && (D & ~MEP_PREC_BF16) == 96 && EPI_BWD_BF16_NW != EWAVES) {
        hipLaunchKernelGGL(k_epi_bwd_bf16w, dim3(max_tiles, n_desc), dim3(64 * EPI_BWD_BF16_NW), 0, (hipStream_t)stream, descs);
        return mep_check_launch("mep_block_epi_bwd");
    }
    const int rc = dispatch_D(D & ~MEP_PREC_BF16, [&](auto dc) {
        if (bf16) hipLaunchKernelGGL((k_epi_bwd<decltype(dc)::value, true>), dim3(max_tiles, n_desc), dim3(ETHREADS), 0,
                                     (hipStream_t)stream, descs);
        else hipLaunchKernelGGL((k_epi_bwd<decltype(dc)::value, false>), dim3(max_tiles, n_desc), dim3(ETHREADS), 0,
                                (hipStream_t)stream, descs);
    });
    if (rc) { mep_set_error("mep_block_epi_bwd: D must be 32, 64, 96 or 128"); return rc; }
    return mep_check_launch("mep_block_epi_bwd");
}


// max_tiles: forward = ceil(ntok / 4) (wave per row), backward = ceil(ntok / 64)
extern "C" int mep_layernorm_fwd(const mep_ln_desc* descs, int n_desc, int max_tiles, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    hipLaunchKernelGGL(k_ln_fwd, dim3((max_tiles + LNF_ROWS - 1) / LNF_ROWS, n_desc), dim3(256), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_layernorm_fwd");
}

extern "C" int mep_layernorm_bwd(const mep_ln_desc* descs, int n_desc, int max_tiles, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    hipLaunchKernelGGL(k_ln_bwd, dim3(max_tiles, n_desc), dim3(256), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_layernorm_bwd");
}
