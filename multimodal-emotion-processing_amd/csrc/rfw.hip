// Wave-tiled realformer path (others/realformer.py:154-209): every Linear of the RealFormer block
// epilogue and the block's token GEMMs on weights pre-split into bf16 parts (mep_wsplit, once per
// step), one wave per 16-token tile.
//
// Transposed-tile layout (split.h): a product Y^T = W X^T leaves lane (token c = lane & 15,
// g = lane >> 4) holding features 16 i + 4 g .. +3 of token c in acc[i] -- exactly the B operand
// of the next product's k pair (features 32 p + 4 g .. +3 in slots 0-3, 32 p + 16 + 4 g .. +3 in
// slots 4-7).  So the whole epilogue chain xp -> LN1 -> FFN -> LN2 (and its backward) stays in one
// wave's registers: no LDS, no barriers, no re-reads of its own intermediates.  LayerNorm row sums
// are the lane's 4 * NI values plus two cross-group shuffles; the LayerNorm / bias parameter
// partials of the backward are DPP row sums over the tile's 16 tokens.
//
// Arithmetic: activations are split into three bf16 parts in registers, weights come pre-split
// (three 16-byte parts per fragment, L2-resident), six products per k pair on
// v_mfma_f32_16x16x32_bf16 -- fp32-level (split.h), no per-fragment split VALU for the weights,
// which feed only 16 tokens each here.  Weight fragments are streamed through a ring of
// MEP_RFW_DEPTH fragments ahead of their MFMAs.
#include <atomic>
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "split.h"

using namespace mep;

// the token rows per workgroup rf.hip was built with (MEP_RF_FWD_ROWS / MEP_RF_BWD_ROWS)
#ifndef MEP_RF_FWD_ROWS
#define MEP_RF_FWD_ROWS 32
#endif
#ifndef MEP_RF_BWD_ROWS
#define MEP_RF_BWD_ROWS 32
#endif
#define MEP_RF_FWD_ROWS_BUILT MEP_RF_FWD_ROWS
#define MEP_RF_BWD_ROWS_BUILT MEP_RF_BWD_ROWS

#ifndef MEP_RFW_DEPTH
#define MEP_RFW_DEPTH 6   // weight fragments (3 x 16 B per lane each) in flight ahead of their MFMAs
#endif

namespace {

#define MEP_RFW_STAMP(k) ((void)0)

constexpr float LN_EPS = 1e-5f;
typedef const MEP_G u32x4* PartPtr;

// ---------------------------------------------------------------- mep_wsplit
__global__ __launch_bounds__(256) void k_wsplit(const mep_wsplit_desc* __restrict__ descs) {
    const mep_wsplit_desc& d = descs[blockIdx.y];
    const int npk = (d.K + 31) >> 5;
    const int u = blockIdx.x * 256 + threadIdx.x;        // unit (n, p, g)
    if (u >= d.R * npk * 4) return;
    const int g = u & 3, np = u >> 2, n = np / npk, p = np - n * npk;
    const gfloat* src = G<const float>(d.src);
    f32x4 lo, hi;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int k0 = 32 * p + 4 * g + e, k1 = k0 + 16;
        const bool nv = n < d.nrows;
        lo[e] = nv && k0 < d.K ? (d.trans ? src[(int64_t)k0 * d.ld + n] : src[(int64_t)n * d.ld + k0]) : 0.f;
        hi[e] = nv && k1 < d.K ? (d.trans ? src[(int64_t)k1 * d.ld + n] : src[(int64_t)n * d.ld + k1]) : 0.f;
    }
    const Parts<3> a = splitv<3>(lo), b = splitv<3>(hi);
    MEP_G u32x4* dst = G<u32x4>(d.dst);
    const int64_t part = (int64_t)d.R * npk * 4;
#pragma unroll
    for (int t = 0; t < 3; ++t) dst[t * part + u] = u32x4{a.p[t][0], a.p[t][1], b.p[t][0], b.p[t][1]};
}

// ---------------------------------------------------------------- products on pre-split weights
// the activation operands of NPK k pairs from NPK * 2 per-lane f32x4 blocks
template <int NPK>
MEP_DEV void split_ops(OpN<3> (&o)[NPK], const f32x4* v) {
#pragma unroll
    for (int p = 0; p < NPK; ++p) o[p] = opn<3>(v[2 * p], v[2 * p + 1]);
}

MEP_DEV PartPtr parts_at(uint64_t base, int off) { return reinterpret_cast<PartPtr>(G<const unsigned char>(base) + off); }

// lane's 4 * NB features (16 kb + 4 g .. +3, kb < NB) of token tc of a row view
template <int NB>
MEP_DEV void load_rows(f32x4 (&v)[NB], const mep_rows& r, int tc) {
    const int g = (threadIdx.x >> 4) & 3;
    const gfloat* p = row_ptr(r, tc) + 4 * g;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) v[kb] = ld4w(p + 16 * kb);
}
template <int NB>
MEP_DEV void store_rows(const mep_rows& r, int tok, const f32x4 (&v)[NB]) {
    const int g = (threadIdx.x >> 4) & 3;
    gfloat* p = row_ptr(r, tok) + 4 * g;
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) *reinterpret_cast<MEP_G f32x4*>(p + 16 * kb) = v[kb];
}

// sum over the row's D features: the lane's values, then the four lane groups of the token
MEP_DEV float feat_sum(float s) {
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    return s;
}

// y = LN(z) * w + b over the D = 16 NI features of the lane's token (realformer.py LayerNorm:
// biased variance, eps 1e-5); mean / rstd returned
template <int NI>
MEP_DEV void layer_norm(const f32x4 (&z)[NI], f32x4 (&y)[NI], const gfloat* w, const gfloat* b, float& mean, float& rstd) {
    constexpr int D = 16 * NI;
    const int g = (threadIdx.x >> 4) & 3;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i) s += (z[i][0] + z[i][1]) + (z[i][2] + z[i][3]);
    mean = feat_sum(s) / (float)D;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) { const float t = z[i][r] - mean; v += t * t; }
    rstd = 1.0f / sqrtf(feat_sum(v) / (float)D + LN_EPS);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const f32x4 ww = ld4w(w + 16 * i + 4 * g), bb = ld4w(b + 16 * i + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) y[i][r] = (z[i][r] - mean) * rstd * ww[r] + bb[r];
    }
}

// ---------------------------------------------------------------- several waves per tile
// W waves share one 16-token tile: the output tiles of every product are dealt round-robin
// (wave w owns tiles w, w + W, ...), each wave streams only its tiles' weight fragments, and the
// full product is exchanged through LDS (one barrier) for the next LayerNorm / product, which
// every wave then evaluates on whole rows.  W = 6 for D = 96 (6 and 12 output tiles split evenly).
template <int D> constexpr int rfw_waves() { return D == 96 ? 6 : D >= 64 ? 4 : 2; }
// Large launches (State_Transfer: B x P x T tokens per block, MEP_RFW_BIG_TILES or more 16-token
// tiles) at D = 96 run the forward with a shallower weight ring (MEP_RFW_BIG_DEPTH fragments) at
// MEP_RFW_BIG_WPE waves per SIMD, so two 6-wave workgroups (two tiles) share a CU and one's
// exchange barriers and weight latency hide behind the other's products; the default kernels fit
// one 6-wave workgroup per CU (their register count leaves 8 wave slots) and run one tile per CU at
// a time, which suits the cfg2 chain's few tiles.
#ifndef MEP_RFW_BIG_TILES
#define MEP_RFW_BIG_TILES 1024   // (round 6: 1024, so the rf_state_ref fixture's 1,350 tiles run these kernels)
#endif
#ifndef MEP_RFW_BIG_WPARTS
#define MEP_RFW_BIG_WPARTS 2     // weight parts of the large-launch kernels (PG NW)
#endif
#ifndef MEP_RFW_BIG_WPE
#define MEP_RFW_BIG_WPE 3
#endif
#ifndef MEP_RFW_BIG_DEPTH
#define MEP_RFW_BIG_DEPTH 4
#endif

// acc[j] += W'(16 i + c, :) . X for the wave's output tiles i = wave + W j < NI, in two halves:
// prime() issues the first DEPTH weight fragments (callers prime the NEXT product before the
// current one's stores / exchange / LayerNorm, so the weight latency hides behind them), run()
// streams the rest through the ring, one fragment's six MFMAs per step.
// NW: weight parts read (3: every product of the six, fp32-level; 2: the large-launch kernels, whose
// weight fragments stream from L2 per 16-token tile and bound them -- the third part feeds only
// w2 x0, and without it the products are split.h's five, weights represented to <= 2^-18
// relative, as the D = 128 tri-modal epilogues; 2/3 of the fragment bytes)
template <int NI, int NPK, int R, int W, int DEP = MEP_RFW_DEPTH, int NW = 3>
struct PG {
    static constexpr int NJ = (NI + W - 1) / W, NS = NJ * NPK;
    static constexpr int DEPTH = DEP < NS ? DEP : NS;
    OpN<NW> ring[DEPTH];
    PartPtr wl;
    int wave;
    MEP_DEV OpN<NW> ld(int s) const {
        const int p = s / NJ, i = wave + W * (s - (s / NJ) * NJ);
        const int ic = i < NI ? i : NI - 1;   // a wave without this tile loads a valid fragment it never uses
        OpN<NW> o;
#pragma unroll
        for (int t = 0; t < NW; ++t) o.p[t] = __builtin_bit_cast(bf16x8, wl[((t * R + 16 * ic) * NPK + p) * 4]);
        return o;
    }
    MEP_DEV void prime(PartPtr w, int wave_) {
        const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
        wl = w + (c * NPK) * 4 + g;
        wave = wave_;
#pragma unroll
        for (int s = 0; s < DEPTH; ++s) ring[s] = ld(s);
    }
    MEP_DEV void run(f32x4 (&acc)[NJ], const OpN<3> (&b)[NPK]) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const OpN<NW> a = ring[s % DEPTH];
            if (s + DEPTH < NS) ring[s % DEPTH] = ld(s + DEPTH);
            const int j = s % NJ;
            if (wave + W * j < NI) acc[j] = mma_nm<NW, 3>(a, b[s / NJ], acc[j]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
};

typedef __attribute__((address_space(3))) f32x4 xf32x4;

// workgroup barrier for LDS hand-offs only: waits for this wave's LDS (and scalar) operations,
// not for its global loads / stores in flight (__syncthreads waits for vmcnt(0), which would drain
// the next product's primed weight loads at every exchange)
MEP_DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// the wave's tiles into the exchange buffer, barrier, every tile back into full[]
template <int NB, int W>
MEP_DEV void xchg(f32x4 (&full)[NB], const f32x4 (&mine)[(NB + W - 1) / W], xf32x4* buf, int wave, int lane) {
#pragma unroll
    for (int j = 0; j < (NB + W - 1) / W; ++j)
        if (wave + W * j < NB) buf[(wave + W * j) * 64 + lane] = mine[j];
    lds_barrier();
#pragma unroll
    for (int i = 0; i < NB; ++i) full[i] = buf[i * 64 + lane];
}

// the wave's tiles of a full row block: store / per-tile transform helpers
template <int NB, int W>
MEP_DEV void store_owned(const mep_rows& r, int tok, const f32x4 (&v)[NB], int wave) {
    const int g = (threadIdx.x >> 4) & 3;
    gfloat* p = row_ptr(r, tok) + 4 * g;
#pragma unroll
    for (int i = 0; i < NB; ++i)
        if (i % W == wave) *reinterpret_cast<MEP_G f32x4*>(p + 16 * i) = v[i];
}
template <int NB, int W>
MEP_DEV void store_mine(const mep_rows& r, int tok, const f32x4 (&v)[(NB + W - 1) / W], int wave) {
    const int g = (threadIdx.x >> 4) & 3;
    gfloat* p = row_ptr(r, tok) + 4 * g;
#pragma unroll
    for (int j = 0; j < (NB + W - 1) / W; ++j)
        if (wave + W * j < NB) *reinterpret_cast<MEP_G f32x4*>(p + 16 * (wave + W * j)) = v[j];
}

// ---------------------------------------------------------------- RealFormer epilogue forward
// Every global load is issued at the top of the kernel (one exposed latency, not one per phase):
// the x rows in every wave (the first product's operand), the q rows of the wave's own blocks into
// a shared LDS stash, and the LayerNorm / bias parameters cooperatively into LDS -- both read after
// the first exchange's barrier.
typedef __attribute__((address_space(3))) float lds_f;

// parameters [n0 | n1 | ...] -> LDS, cooperatively (the caller's next barrier publishes them)
template <int TOTAL, int NT, int NSEG>
MEP_DEV void stage_params(lds_f* dst, const uint64_t (&src)[NSEG], const int (&len)[NSEG]) {
    constexpr int PER = (TOTAL + NT - 1) / NT;
    float v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {   // every load first (one latency), then the LDS writes
        const int idx = threadIdx.x + NT * k;
        int off = idx, sg = 0;
#pragma unroll
        for (int q = 0; q < NSEG - 1; ++q)
            if (sg == q && off >= len[q]) { off -= len[q]; sg = q + 1; }
        v[k] = idx < TOTAL ? G<const float>(src[sg])[off] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k)
        if (threadIdx.x + NT * k < TOTAL) dst[threadIdx.x + NT * k] = v[k];
}

template <int NI, typename P>
MEP_DEV void layer_norm_l(const f32x4 (&z)[NI], f32x4 (&y)[NI], const P* w, const P* b, float& mean, float& rstd) {
    constexpr int D = 16 * NI;
    const int g = (threadIdx.x >> 4) & 3;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i) s += (z[i][0] + z[i][1]) + (z[i][2] + z[i][3]);
    mean = feat_sum(s) / (float)D;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) { const float t = z[i][r] - mean; v += t * t; }
    rstd = 1.0f / sqrtf(feat_sum(v) / (float)D + LN_EPS);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const f32x4 ww = ld4w(w + 16 * i + 4 * g), bb = ld4w(b + 16 * i + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) y[i][r] = (z[i][r] - mean) * rstd * ww[r] + bb[r];
    }
}

// the wave's own blocks (i % W == wave) of a token's row -> a shared [NB][64 lanes] LDS stash
template <int NB, int W>
MEP_DEV void stash_owned(xf32x4* st, const mep_rows& r, int tc, int wave, int lane) {
    const int g = (threadIdx.x >> 4) & 3;
    const gfloat* p = row_ptr(r, tc) + 4 * g;
    f32x4 v[(NB + W - 1) / W];
#pragma unroll
    for (int j = 0; j < (NB + W - 1) / W; ++j)
        if (wave + W * j < NB) v[j] = ld4w(p + 16 * (wave + W * j));
#pragma unroll
    for (int j = 0; j < (NB + W - 1) / W; ++j)
        if (wave + W * j < NB) st[(wave + W * j) * 64 + lane] = v[j];
}

template <int D, int FD, int W = rfw_waves<D>(), int WPE = 1, int DEP = MEP_RFW_DEPTH, int NW = 3>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(WPE))) void k_rfw_fwd(const mep_rf_epi_desc* __restrict__ descs) {
    constexpr int NI = D / 16, NF = FD / 16, NP = D / 32, NPF = FD / 32;
    constexpr int JI = (NI + W - 1) / W, JF = (NF + W - 1) / W;
    __shared__ f32x4 xsm[2][NF * 64];
    __shared__ f32x4 qsm[NI * 64];
    __shared__ float prm[5 * D + FD];   // ln1_w | ln1_b | ln2_w | ln2_b | b2 | b1
    xf32x4* xbuf[2] = {(xf32x4*)&xsm[0][0], (xf32x4*)&xsm[1][0]};
    xf32x4* qst = (xf32x4*)&qsm[0];
    lds_f* P = (lds_f*)&prm[0];
    const mep_rf_epi_desc& d = descs[blockIdx.y];
    const int ntok = d.ntok;
    const int tile = blockIdx.x;
    if (tile * 16 >= ntok) return;   // whole workgroup
    MEP_RFW_STAMP(0);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
    const int tok = tile * 16 + c, tc = min(tok, ntok - 1);
    const bool ok = tok < ntok;
    const float sa = *G<const float>(d.a), sb = *G<const float>(d.b);

    // every load of the kernel's first phase at once: x (every wave), the first product's weight
    // fragments, q (the wave's blocks, shared stash) and the parameters (LDS)
    f32x4 xv[NI];
    load_rows<NI>(xv, d.x, tc);
    PG<NI, NP, D, W, DEP, NW> g1;
    g1.prime(parts_at(d.wparts, MEP_RFW_PART_OFFSET(D, FD, 0)), wave);
    stash_owned<NI, W>(qst, d.q, tc, wave, lane);
    {
        const uint64_t src[6] = {d.ln1_w, d.ln1_b, d.ln2_w, d.ln2_b, d.b2, d.b1};
        const int len[6] = {D, D, D, D, D, FD};
        stage_params<5 * D + FD, 64 * W, 6>(P, src, len);
    }
    MEP_RFW_STAMP(1);
    // xp = Wp x (the wave's tiles), exchanged (the exchange's barrier also publishes q and the parameters)
    f32x4 xp[NI];
    PG<NF, NP, FD, W, DEP, NW> g2;
    {
        f32x4 acc[JI];
#pragma unroll
        for (int j = 0; j < JI; ++j) acc[j] = zero_f4();
        OpN<3> xs[NP];
        split_ops<NP>(xs, xv);
        g1.run(acc, xs);
        MEP_RFW_STAMP(2);
        g2.prime(parts_at(d.wparts, MEP_RFW_PART_OFFSET(D, FD, 1)), wave);
        if (ok) store_mine<NI, W>(d.xp, tok, acc, wave);
        xchg<NI, W>(xp, acc, xbuf[0], wave, lane);
        MEP_RFW_STAMP(3);
    }
    // h = LN1(q + a xp)  (the reference's q + a * xp: two roundings), on whole rows in every wave
    f32x4 h[NI];
    float mean1, rstd1;
    {
        f32x4 z[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const f32x4 qv = qst[i * 64 + lane];
#pragma unroll
            for (int r = 0; r < 4; ++r) z[i][r] = add_rn(qv[r], mul_rn(sa, xp[i][r]));
        }
        layer_norm_l<NI>(z, h, P, P + D, mean1, rstd1);
    }
    if (ok) store_owned<NI, W>(d.h, tok, h, wave);
    MEP_RFW_STAMP(4);
    // f1 = relu(W1 h + b1)
    f32x4 f1[NF];
    PG<NI, NPF, D, W, DEP, NW> g3;
    {
        f32x4 acc[JF];
#pragma unroll
        for (int j = 0; j < JF; ++j) acc[j] = zero_f4();
        OpN<3> hs[NP];
        split_ops<NP>(hs, h);
        g2.run(acc, hs);
        MEP_RFW_STAMP(5);
        g3.prime(parts_at(d.wparts, MEP_RFW_PART_OFFSET(D, FD, 2)), wave);
#pragma unroll
        for (int j = 0; j < JF; ++j) {
            const f32x4 bb = ld4w(P + 5 * D + 16 * min(wave + W * j, NF - 1) + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[j][r] = fmaxf(acc[j][r] + bb[r], 0.f);
        }
        if (ok) store_mine<NF, W>(d.f1, tok, acc, wave);
        xchg<NF, W>(f1, acc, xbuf[1], wave, lane);
    }
    MEP_RFW_STAMP(6);
    // f = W2 f1 + b2
    f32x4 f[NI];
    {
        f32x4 acc[JI];
#pragma unroll
        for (int j = 0; j < JI; ++j) acc[j] = zero_f4();
        OpN<3> fs[NPF];
        split_ops<NPF>(fs, f1);
        g3.run(acc, fs);
        MEP_RFW_STAMP(7);
#pragma unroll
        for (int j = 0; j < JI; ++j) {
            const f32x4 bb = ld4w(P + 4 * D + 16 * min(wave + W * j, NI - 1) + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[j][r] = acc[j][r] + bb[r];
        }
        if (ok) store_mine<NI, W>(d.f, tok, acc, wave);
        xchg<NI, W>(f, acc, xbuf[0], wave, lane);
    }
    MEP_RFW_STAMP(8);
    // out = LN2(h + b f)
    f32x4 out[NI];
    float mean2, rstd2;
    {
        f32x4 z[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) z[i][r] = add_rn(h[i][r], mul_rn(sb, f[i][r]));
        layer_norm_l<NI>(z, out, P + 2 * D, P + 3 * D, mean2, rstd2);
    }
    if (d.wq_next) {   // the next layer's query projection, qp_next = out Wq_next^T (wave's tiles)
        PG<NI, NP, D, W, DEP, NW> g4;
        g4.prime(reinterpret_cast<PartPtr>(G<const unsigned char>(d.wq_next)), wave);
        f32x4 acc[JI];
#pragma unroll
        for (int j = 0; j < JI; ++j) acc[j] = zero_f4();
        OpN<3> os[NP];
        split_ops<NP>(os, out);
        g4.run(acc, os);
        if (ok) store_mine<NI, W>(d.qp_next, tok, acc, wave);
    }
    if (ok) {
        store_owned<NI, W>(d.out, tok, out, wave);
        if (wave == 0 && g == 0)
            *reinterpret_cast<MEP_G f32x4*>(G<float>(d.stats) + 4 * (int64_t)tok) = f32x4{mean1, rstd1, mean2, rstd2};
        if (d.zero.ptr) {   // the backward's accumulated rows of these tokens, cleared for this step
            f32x4 z[JI];
#pragma unroll
            for (int j = 0; j < JI; ++j) z[j] = zero_f4();
            store_mine<NI, W>(d.zero, tok, z, wave);
        }
    }
    MEP_RFW_STAMP(9);
}

// ---------------------------------------------------------------- RealFormer epilogue backward
// column sums over the tile's 16 tokens of the wave's blocks of NB, written by the c == 0 lanes
template <int NB, int W>
MEP_DEV void tile_colsum(gfloat* dst, const f32x4 (&v)[NB], int wave, int c, int g) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        if (i % W != wave) continue;
        f32x4 s;
#pragma unroll
        for (int r = 0; r < 4; ++r) s[r] = row16_sum(v[i][r]);
        if (c == 0) {   // partial rows are 4-byte aligned only (stride 5D + FD + 2)
#pragma unroll
            for (int r = 0; r < 4; ++r) dst[16 * i + 4 * g + r] = s[r];
        }
    }
}

// LayerNorm backward of one token: g (upstream), xh (normalized input), w (LN weight, lane's
// blocks) -> dz = rstd (g w - mean(g w) - xh mean(g w xh))
template <int NI>
MEP_DEV void ln_bwd(f32x4 (&dz)[NI], const f32x4 (&gu)[NI], const f32x4 (&xh)[NI], const f32x4 (&ww)[NI], float rstd) {
    constexpr int D = 16 * NI;
    f32x4 gw[NI];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            gw[i][r] = gu[i][r] * ww[i][r];
            s1 += gw[i][r];
            s2 += gw[i][r] * xh[i][r];
        }
    }
    s1 = feat_sum(s1) / (float)D;
    s2 = feat_sum(s2) / (float)D;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) dz[i][r] = rstd * (gw[i][r] - s1 - xh[i][r] * s2);
}

template <int D, int FD, int W = rfw_waves<D>(), int WPE = 1, int DEP = MEP_RFW_DEPTH, int NW = 3>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(WPE))) void k_rfw_bwd(const mep_rf_epi_bwd_desc* __restrict__ descs) {
    constexpr int NI = D / 16, NF = FD / 16, NP = D / 32, NPF = FD / 32;
    constexpr int JI = (NI + W - 1) / W, JF = (NF + W - 1) / W;
    __shared__ f32x4 xsm[2][NF * 64];
    __shared__ f32x4 ssm[2][NI * 64];   // q | xp rows (shared stash)
    __shared__ float prm[D];            // ln1_w
    xf32x4* xbuf[2] = {(xf32x4*)&xsm[0][0], (xf32x4*)&xsm[1][0]};
    xf32x4* qst = (xf32x4*)&ssm[0][0];
    xf32x4* xpst = (xf32x4*)&ssm[1][0];
    lds_f* P = (lds_f*)&prm[0];
    const mep_rf_epi_bwd_desc& bd = descs[blockIdx.y];
    const mep_rf_epi_desc& d = bd.f;
    const int ntok = d.ntok;
    const int tile = blockIdx.x;
    if (tile * 16 >= ntok) return;   // whole workgroup
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
    const int tok = tile * 16 + c, tc = min(tok, ntok - 1);
    const bool ok = tok < ntok;
    const float sa = *G<const float>(d.a), sb = *G<const float>(d.b);
    gfloat* part = G<float>(bd.partial) + (int64_t)tile * MEP_RF_PARTIAL_STRIDE(D, FD);

    // every load up front: the rows the LN2 backward needs now (registers), the first product's
    // weight fragments, the f1 blocks of the wave's df1 tiles and the old dq blocks (registers),
    // q / xp (shared stash) and ln1_w (LDS)
    const f32x4 st = ld4w(G<const float>(d.stats) + 4 * (int64_t)tc);   // mean1, rstd1, mean2, rstd2
    f32x4 gu[NI], hv[NI], fv[NI], w2v[NI];
    load_rows<NI>(gu, bd.dout, tc);
    load_rows<NI>(hv, d.h, tc);
    load_rows<NI>(fv, d.f, tc);
#pragma unroll
    for (int i = 0; i < NI; ++i) w2v[i] = ld4w(G<const float>(d.ln2_w) + 16 * i + 4 * g);
    PG<NF, NP, FD, W, DEP, NW> g1;
    g1.prime(parts_at(d.wparts, MEP_RFW_PART_OFFSET(D, FD, 5)), wave);
    f32x4 f1v[JF], dqo[JI];
    {
        const gfloat* f1r = row_ptr(d.f1, tc) + 4 * g;
#pragma unroll
        for (int j = 0; j < JF; ++j) f1v[j] = ld4w(f1r + 16 * min(wave + W * j, NF - 1));
        if (bd.dq_accumulate) {
            const gfloat* o = row_ptr(bd.dq, tc) + 4 * g;
#pragma unroll
            for (int j = 0; j < JI; ++j) dqo[j] = ld4w(o + 16 * min(wave + W * j, NI - 1));
        }
    }
    stash_owned<NI, W>(qst, d.q, tc, wave, lane);
    stash_owned<NI, W>(xpst, d.xp, tc, wave, lane);
    {
        const uint64_t src[1] = {d.ln1_w};
        const int len[1] = {D};
        stage_params<D, 64 * W, 1>(P, src, len);
    }
    if (bd.dout2.ptr) {
        f32x4 g2[NI];
        load_rows<NI>(g2, bd.dout2, tc);
#pragma unroll
        for (int i = 0; i < NI; ++i) gu[i] += g2[i];
    }
    if (bd.wq_in) {   // dout += dqp_in Wq: the next layer's query-projection input gradient (exchanged)
        PG<NI, NP, D, W, DEP, NW> g0;
        g0.prime(reinterpret_cast<PartPtr>(G<const unsigned char>(bd.wq_in)), wave);
        f32x4 dv[NI];
        load_rows<NI>(dv, bd.dqp_in, tc);
        f32x4 acc[JI], full[NI];
#pragma unroll
        for (int j = 0; j < JI; ++j) acc[j] = zero_f4();
        OpN<3> ds[NP];
        split_ops<NP>(ds, dv);
        g0.run(acc, ds);
        xchg<NI, W>(full, acc, xbuf[1], wave, lane);
#pragma unroll
        for (int i = 0; i < NI; ++i) gu[i] += full[i];
    }
#pragma unroll
    for (int i = 0; i < NI; ++i)
        if (!ok) gu[i] = zero_f4();
    // LN2 backward -> dz2; df = b dz2 (whole rows in every wave)
    f32x4 dz2[NI], df[NI];
    float db_s = 0.f;
    f32x4 pw2[NI];
    {
        f32x4 xh[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) xh[i][r] = (add_rn(hv[i][r], mul_rn(sb, fv[i][r])) - st[2]) * st[3];
        ln_bwd<NI>(dz2, gu, xh, w2v, st[3]);
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                pw2[i][r] = mul_rn(gu[i][r], xh[i][r]);   // rounded: a product fused into the column sum's first add would depend on the schedule
                df[i][r] = sb * dz2[i][r];
                db_s += dz2[i][r] * fv[i][r];
            }
    }
    // df1 = relu'(f1) (W2^T df)
    f32x4 df1[NF];
    PG<NI, NPF, D, W, DEP, NW> g2;
    {
        f32x4 acc[JF];
#pragma unroll
        for (int j = 0; j < JF; ++j) acc[j] = zero_f4();
        OpN<3> ds[NP];
        split_ops<NP>(ds, df);
        g1.run(acc, ds);
        g2.prime(parts_at(d.wparts, MEP_RFW_PART_OFFSET(D, FD, 4)), wave);
        // the LN2 partials and df after the primed loads (stores count in vmcnt with the loads)
        tile_colsum<NI, W>(part, pw2, wave, c, g);           // dLN2.w
        tile_colsum<NI, W>(part + D, gu, wave, c, g);        // dLN2.b
        tile_colsum<NI, W>(part + 4 * D, df, wave, c, g);    // db2
        if (ok) store_owned<NI, W>(bd.df, tok, df, wave);
#pragma unroll
        for (int j = 0; j < JF; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[j][r] = (ok && f1v[j][r] > 0.f) ? acc[j][r] : 0.f;
        if (ok) store_mine<NF, W>(bd.df1, tok, acc, wave);
        xchg<NF, W>(df1, acc, xbuf[0], wave, lane);
    }
    tile_colsum<NF, W>(part + 5 * D, df1, wave, c, g);       // db1
    // dh = dz2 + W1^T df1
    f32x4 dh[NI];
    PG<NI, NP, D, W, DEP, NW> g3;
    {
        f32x4 acc[JI];
#pragma unroll
        for (int j = 0; j < JI; ++j) acc[j] = zero_f4();
        OpN<3> ds[NPF];
        split_ops<NPF>(ds, df1);
        g2.run(acc, ds);
        g3.prime(parts_at(d.wparts, MEP_RFW_PART_OFFSET(D, FD, 3)), wave);
        xchg<NI, W>(dh, acc, xbuf[1], wave, lane);
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) dh[i] += dz2[i];
    // LN1 backward -> dz1;  dq (+)= dz1;  dxp = a dz1
    f32x4 dxp[NI];
    float da_s = 0.f;
    {
        f32x4 xh[NI], dz1[NI], w1v[NI], xpv[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const f32x4 qv = qst[i * 64 + lane];
            xpv[i] = xpst[i * 64 + lane];
            w1v[i] = ld4w(P + 16 * i + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r) xh[i][r] = (add_rn(qv[r], mul_rn(sa, xpv[i][r])) - st[0]) * st[1];
        }
        ln_bwd<NI>(dz1, dh, xh, w1v, st[1]);
        f32x4 pw[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                pw[i][r] = mul_rn(dh[i][r], xh[i][r]);
                dxp[i][r] = sa * dz1[i][r];
                da_s += dz1[i][r] * xpv[i][r];
            }
        tile_colsum<NI, W>(part + 2 * D, pw, wave, c, g);    // dLN1.w
        tile_colsum<NI, W>(part + 3 * D, dh, wave, c, g);    // dLN1.b
        if (ok) {
            f32x4 mine[JI];
#pragma unroll
            for (int j = 0; j < JI; ++j) {
                const int i = min(wave + W * j, NI - 1);
                mine[j] = bd.dq_accumulate ? dqo[j] + dz1[i] : dz1[i];
            }
            store_mine<NI, W>(bd.dq, tok, mine, wave);
            store_owned<NI, W>(bd.dxp, tok, dxp, wave);
        }
    }
    if (wave == 0) {   // every wave holds the whole rows; wave 0 writes the scalars
        const float da = wave_sum(da_s), db = wave_sum(db_s);
        if (lane == 0) { part[5 * D + FD] = da; part[5 * D + FD + 1] = db; }
    }
    // dx = Wp^T dxp
    {
        f32x4 acc[JI];
#pragma unroll
        for (int j = 0; j < JI; ++j) acc[j] = zero_f4();
        OpN<3> ds[NP];
        split_ops<NP>(ds, dxp);
        g3.run(acc, ds);
        if (ok) store_mine<NI, W>(bd.dx, tok, acc, wave);
    }
}

// ---------------------------------------------------------------- weight-stationary large launches
// (round 6, MEP_RFS) The State_Transfer epilogue launches (>= MEP_RFW_BIG_TILES tiles, D = 96):
// k_rfw_fwd / k_rfw_bwd stream every weight fragment from L2 once per 16-token tile (10,800 tiles
// per launch, ~44 M L2 requests, MFMA busy 0.05-0.08).  Here one 8-wave workgroup per CU walks
// jobs of 8 tiles (128 tokens) of one descriptor: each wave owns one tile for the whole chain
// (every output tile of every product, so the LayerNorms run in-wave and nothing is exchanged),
// and the workgroup copies each product's 2-part weight fragments into one of two 72-KiB LDS
// buffers by LDS-DMA while it multiplies the previous product from the other -- a fragment leaves
// L2 once per 8 tiles.  Per step: barrier -> the previous step's stores -> the next product's DMA
// and the rows this step's epilogue needs -> MFMAs from LDS -> epilogue -> vmcnt(0) + barrier; the
// forward loads the next job's x rows one step ahead (the backward its first rows at the job's
// start: held across a step they cost more registers than the wait).  The products are
// k_rfw_*<..., NW = 2>'s in the same order per accumulator, and every epilogue the same
// arithmetic: results bit-identical to those kernels (test_gpu_rfw.py).
#ifndef MEP_RFS_FWD_W
#define MEP_RFS_FWD_W 8   // waves (16-token tiles) per workgroup: 2 per SIMD (190 VGPRs)
#endif
#ifndef MEP_RFS_BWD_W
#define MEP_RFS_BWD_W 8   // (4: one wave per SIMD with the rows AGPR-spilled, 276 vs 234 us per launch)
#endif
constexpr int RFS_IMG = 1024;            // one part image of a fragment: 64 lanes x 16 B
constexpr int RFS_BUF = 72 * RFS_IMG;    // the largest product's fragments: 12 x 3 or 6 x 6 pairs, 2 parts
typedef __attribute__((address_space(3))) unsigned char lbyte_t;
typedef __attribute__((address_space(3))) void lvoid_t;
typedef __attribute__((address_space(3))) const bf16x8 lcbf8_t;

// every wave's LDS-DMA and loads / stores retired, then the workgroup barrier
MEP_DEV void rfs_sync() { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// parts 0 and 1 of a product's fragments (NO output tiles x NPK k pairs of mep_wsplit parts with R
// rows) -> an LDS buffer: image f = (i * NPK + p) * 2 + t holds lane l's 16-byte unit at 16 l (one
// conflict-free ds_read_b128 per part), the W waves taking every W-th image
template <int NO, int NPK, int R, int W>
MEP_DEV void rfs_stage(lbyte_t* buf, uint64_t w, int wave, int lane) {
    constexpr int NIMG = NO * NPK * 2;
    static_assert(NIMG * RFS_IMG <= RFS_BUF, "rfs buffer");
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, MEP_WSPLIT_BYTES(R, 32 * NPK), 0x00020000);
    const int c = lane & 15, g = lane >> 4;
    for (int f = wave; f < NIMG; f += W) {
        const int t = f & 1, ip = f >> 1, i = ip / NPK, p = ip - i * NPK;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lvoid_t*)(buf + f * RFS_IMG), 16,
                                                 16 * (((t * R + 16 * i + c) * NPK + p) * 4 + g), 0, 0, 0);
    }
}

// acc[i] = sum over the k pairs, in order, of W'(16 i + c, pair p) . X for every output tile i:
// pair-major (each pair's activation operand split once, as split_ops, its NO fragments' MFMAs on
// independent accumulators), the fragments read from LDS through a ring RFS_DEPTH steps ahead
// (a scheduling barrier per step: left alone, the compiler hoists every read of the product and
// spills)
#ifndef MEP_RFS_BWD_PRE
#define MEP_RFS_BWD_PRE 0   // 1: the backward's next-job rows loaded a step ahead (measured slower: 306 vs 279 us, the rows held across the step cost 100 AGPR moves)
#endif
#ifndef MEP_RFS_DEPTH
#define MEP_RFS_DEPTH 3
#endif
template <int NO, int NPK>
MEP_DEV void rfs_mul(f32x4 (&acc)[NO], const lbyte_t* buf, const f32x4* v, int lane) {
    constexpr int NS = NO * NPK, DEP = MEP_RFS_DEPTH < NS ? MEP_RFS_DEPTH : NS;
    const lbyte_t* b = buf + 16 * lane;
    auto ld = [&](int s) {
        const int p = s / NO, i = s - p * NO;
        OpN<2> a;
        a.p[0] = *(lcbf8_t*)(b + ((i * NPK + p) * 2) * RFS_IMG);
        a.p[1] = *(lcbf8_t*)(b + ((i * NPK + p) * 2 + 1) * RFS_IMG);
        return a;
    };
    OpN<2> ring[DEP];
#pragma unroll
    for (int s = 0; s < DEP; ++s) ring[s] = ld(s);
#pragma unroll
    for (int i = 0; i < NO; ++i) acc[i] = zero_f4();
    OpN<3> x;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int p = s / NO, i = s - p * NO;
        if (i == 0) x = opn<3>(v[2 * p], v[2 * p + 1]);
        const OpN<2> a = ring[s % DEP];
        if (s + DEP < NS) ring[s % DEP] = ld(s + DEP);
        acc[i] = mma_nm<2, 3>(a, x, acc[i]);
        __builtin_amdgcn_sched_barrier(0);
    }
}

// a tile's 16-token column sums of NB blocks, packed: lane (c, g) keeps block c's sums of
// features 16 c + 4 g .. +3 (row16_sum leaves the same sum in every lane of a row); stored by the
// lanes c < NB at the partial row (4-byte aligned: scalar stores)
template <int NB>
MEP_DEV f32x4 rfs_colsum(const f32x4 (&v)[NB], int c) {
    f32x4 k = zero_f4();
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        f32x4 s;
#pragma unroll
        for (int r = 0; r < 4; ++r) s[r] = row16_sum(v[i][r]);
        if (c == i) k = s;
    }
    return k;
}
MEP_DEV void rfs_colsum_store(gfloat* dst, const f32x4& k, int nb, int c, int g) {
    if (c < nb) {
#pragma unroll
        for (int r = 0; r < 4; ++r) dst[16 * c + 4 * g + r] = k[r];
    }
}

// the jobs (descriptor, batch of W tiles) a workgroup walks, skipping batches past a descriptor's
// tokens (uniform over the workgroup).  XCD-chunked: workgroup b runs on XCD b % 8 (round-robin
// dispatch), and each XCD takes one contiguous eighth of the job list (descriptor-major), its
// workgroups striding through it -- the 32 CUs of an XCD work on one or two descriptors at a
// time, so their weight fragments stay in that XCD's L2 (the plain stride spread every
// descriptor over every XCD: L2 hit rate 0.57 on the weight DMA)
MEP_DEV int rfs_ntok(const mep_rf_epi_desc& d) { return d.ntok; }
MEP_DEV int rfs_ntok(const mep_rf_epi_bwd_desc& d) { return d.f.ntok; }
template <typename Desc, int W>
struct RfsJobs {
    const Desc* descs;
    int njobs, nbat, lo, hi, stride;
    MEP_DEV RfsJobs(const Desc* d, int nj, int nb) : descs(d), njobs(nj), nbat(nb) {
        const int G = gridDim.x, b = blockIdx.x;
        if (G % 8 == 0) {
            lo = (int)((int64_t)nj * (b % 8) / 8) + b / 8;
            hi = (int)((int64_t)nj * (b % 8 + 1) / 8);
            stride = G / 8;
        } else {
            lo = b;
            hi = nj;
            stride = G;
        }
    }
    MEP_DEV int ntok(int j) const { return rfs_ntok(descs[j / nbat]); }
    MEP_DEV bool valid(int j) const { return j < hi && (j % nbat) * (16 * W) < ntok(j); }
    // (readfirstlane: the job index is workgroup-uniform; without it the compiler keeps it in a
    // VGPR and reads every descriptor field with vector loads and vmcnt(0) waits)
    MEP_DEV int next(int j) const {
        do { j += stride; } while (j < hi && !valid(j));
        return __builtin_amdgcn_readfirstlane(j < hi ? j : njobs);
    }
    MEP_DEV int first() const { return valid(lo) ? lo : next(lo); }
};

// a job's LayerNorm / bias parameters [n0 | n1 | ...] -> the job's LDS parameter slot: loaded into
// registers at the start of the previous job's last step (before its DMA, so the wait for them,
// at the end of that step, is for loads issued a step earlier), written to LDS there, published by
// the step's barrier
template <int TOTAL, int NSEG, int W>
struct RfsParams {
    static constexpr int PER = (TOTAL + 64 * W - 1) / (64 * W);
    float v[PER];
    MEP_DEV void load(const uint64_t (&src)[NSEG], const int (&len)[NSEG]) {
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int idx = threadIdx.x + 64 * W * k;
            int off = idx, sg = 0;
#pragma unroll
            for (int q = 0; q < NSEG - 1; ++q)
                if (sg == q && off >= len[q]) { off -= len[q]; sg = q + 1; }
            v[k] = idx < TOTAL ? G<const float>(src[sg])[off] : 0.f;
        }
    }
    MEP_DEV void write(lds_f* dst) const {
#pragma unroll
        for (int k = 0; k < PER; ++k)
            if (threadIdx.x + 64 * W * k < TOTAL) dst[threadIdx.x + 64 * W * k] = v[k];
    }
};

template <int D, int FD, int W>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(W / 4, W / 4))) void k_rfs_fwd(const mep_rf_epi_desc* __restrict__ descs, int n_desc, int nbat) {
    constexpr int NI = D / 16, NF = FD / 16, NP = D / 32, NPF = FD / 32;
    constexpr int NPRM = 5 * D + FD;   // ln1_w | ln1_b | ln2_w | ln2_b | b2 | b1 (k_rfw_fwd's order)
    // two weight buffers as separate LDS objects, each product's buffer fixed at compile time
    // (job bodies instantiated per first-buffer parity): the compiler then sees that a ds_read of
    // one buffer does not alias the DMA in flight into the other, and does not wait for it
    __shared__ __attribute__((aligned(16))) unsigned char sm0[RFS_BUF], sm1[RFS_BUF];
    __shared__ __attribute__((aligned(16))) float prm[2 * NPRM];
    lbyte_t* const LB[2] = {(lbyte_t*)sm0, (lbyte_t*)sm1};
    lds_f* const PS = (lds_f*)prm;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
    const RfsJobs<mep_rf_epi_desc, W> jobs(descs, n_desc * nbat, nbat);
    auto woff = [](const mep_rf_epi_desc& d, int k) { return d.wparts + MEP_RFW_PART_OFFSET(D, FD, k); };
    auto tok_of = [&](int j) { return ((j % nbat) * W + wave) * 16 + c; };
    auto prm_load = [&](RfsParams<NPRM, 6, W>& pr, const mep_rf_epi_desc& d) {
        const uint64_t src[6] = {d.ln1_w, d.ln1_b, d.ln2_w, d.ln2_b, d.b2, d.b1};
        const int len[6] = {D, D, D, D, D, FD};
        pr.load(src, len);
    };
    int job = jobs.first();
    if (job >= jobs.njobs) return;   // whole workgroup
    int ps = 0;
    f32x4 xv[NI];                     // the job's x rows (Wp's operand), loaded a step ahead
    {
        const mep_rf_epi_desc& d = descs[job / nbat];
        RfsParams<NPRM, 6, W> pr;
        prm_load(pr, d);
        rfs_stage<NI, NP, D, W>(LB[0], woff(d, 0), wave, lane);
        load_rows<NI>(xv, d.x, min(tok_of(job), d.ntok - 1));
        pr.write(PS);
        rfs_sync();
    }
    // one job; P: the buffer of its first product, Q: the next layer's query projection fused.
    // Returns the next job's first buffer
    auto body = [&](auto pc, auto qc) -> int {
        constexpr int P = decltype(pc)::value;
        constexpr bool Q = decltype(qc)::value;
        job = __builtin_amdgcn_readfirstlane(job);
        const int nj = jobs.next(job);
        const mep_rf_epi_desc& d = descs[job / nbat];
        const mep_rf_epi_desc* dn = nj < jobs.njobs ? &descs[nj / nbat] : nullptr;
        const int ntok = d.ntok, tok = tok_of(job), tc = min(tok, ntok - 1);
        const bool ok = tok < ntok;
        const float sa = *G<const float>(d.a), sb = *G<const float>(d.b);
        const lds_f* PR = PS + ps * NPRM;
        // ---- xp = Wp x;  h = LN1(q + a xp)
        rfs_stage<NF, NP, FD, W>(LB[P ^ 1], woff(d, 1), wave, lane);
        f32x4 qv[NI];
        load_rows<NI>(qv, d.q, tc);
        f32x4 xp[NI], h[NI];
        float mean1, rstd1;
        rfs_mul<NI, NP>(xp, LB[P], xv, lane);
        {
            f32x4 z[NI];
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) z[i][r] = add_rn(qv[i][r], mul_rn(sa, xp[i][r]));
            layer_norm_l<NI>(z, h, PR, PR + D, mean1, rstd1);
        }
        rfs_sync();
        // ---- f1 = relu(W1 h + b1)
        if (ok) {
            store_rows<NI>(d.xp, tok, xp);
            store_rows<NI>(d.h, tok, h);
        }
        rfs_stage<NI, NPF, D, W>(LB[P], woff(d, 2), wave, lane);
        f32x4 f1[NF];
        rfs_mul<NF, NP>(f1, LB[P ^ 1], h, lane);
#pragma unroll
        for (int j = 0; j < NF; ++j) {
            const f32x4 bb = ld4w(PR + 5 * D + 16 * j + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r) f1[j][r] = fmaxf(f1[j][r] + bb[r], 0.f);
        }
        rfs_sync();
        // ---- f = W2 f1 + b2;  out = LN2(h + b f)
        if (ok) store_rows<NF>(d.f1, tok, f1);
        RfsParams<NPRM, 6, W> pr;   // the next job's parameters (its slot is free: the job before used it)
        if (!Q && dn) prm_load(pr, *dn);
        if constexpr (Q) rfs_stage<NI, NP, D, W>(LB[P ^ 1], d.wq_next, wave, lane);
        else if (dn) rfs_stage<NI, NP, D, W>(LB[P ^ 1], woff(*dn, 0), wave, lane);
        f32x4 f[NI], out[NI];
        float mean2, rstd2;
        rfs_mul<NI, NPF>(f, LB[P], f1, lane);
#pragma unroll
        for (int j = 0; j < NI; ++j) {
            const f32x4 bb = ld4w(PR + 4 * D + 16 * j + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r) f[j][r] = f[j][r] + bb[r];
        }
        {
            f32x4 z[NI];
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) z[i][r] = add_rn(h[i][r], mul_rn(sb, f[i][r]));
            layer_norm_l<NI>(z, out, PR + 2 * D, PR + 3 * D, mean2, rstd2);
        }
        if (!Q && dn) {
            load_rows<NI>(xv, dn->x, min(tok_of(nj), dn->ntok - 1));
            pr.write(PS + (ps ^ 1) * NPRM);
        }
        rfs_sync();
        if (ok) {
            store_rows<NI>(d.f, tok, f);
            store_rows<NI>(d.out, tok, out);
            if (g == 0)
                *reinterpret_cast<MEP_G f32x4*>(G<float>(d.stats) + 4 * (int64_t)tok) = f32x4{mean1, rstd1, mean2, rstd2};
            if (d.zero.ptr) {   // the backward's accumulated rows of these tokens, cleared for this step
                f32x4 zr[NI];
#pragma unroll
                for (int i = 0; i < NI; ++i) zr[i] = zero_f4();
                store_rows<NI>(d.zero, tok, zr);
            }
        }
        if constexpr (Q) {   // ---- the next layer's query projection, qp_next = out Wq_next^T
            if (dn) {
                prm_load(pr, *dn);
                rfs_stage<NI, NP, D, W>(LB[P], woff(*dn, 0), wave, lane);
                load_rows<NI>(xv, dn->x, min(tok_of(nj), dn->ntok - 1));
            }
            f32x4 qp[NI];
            rfs_mul<NI, NP>(qp, LB[P ^ 1], out, lane);
            if (dn) pr.write(PS + (ps ^ 1) * NPRM);
            rfs_sync();
            if (ok) store_rows<NI>(d.qp_next, tok, qp);
        }
        ps ^= 1;
        job = nj;
        return Q ? P : P ^ 1;
    };
    int par = 0;
    while (job < jobs.njobs) {
        job = __builtin_amdgcn_readfirstlane(job);
        const bool q = descs[job / nbat].wq_next != 0;
        if (par) par = q ? body(std::integral_constant<int, 1>{}, std::true_type{}) : body(std::integral_constant<int, 1>{}, std::false_type{});
        else par = q ? body(std::integral_constant<int, 0>{}, std::true_type{}) : body(std::integral_constant<int, 0>{}, std::false_type{});
    }
}

template <int D, int FD, int W>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(W / 4, W / 4))) void k_rfs_bwd(const mep_rf_epi_bwd_desc* __restrict__ descs, int n_desc, int nbat) {
    constexpr int NI = D / 16, NF = FD / 16, NP = D / 32, NPF = FD / 32;
    constexpr int NPRM = 2 * D;        // ln1_w | ln2_w
    __shared__ __attribute__((aligned(16))) unsigned char sm0[RFS_BUF], sm1[RFS_BUF];   // (as k_rfs_fwd)
    __shared__ __attribute__((aligned(16))) float prm[2 * NPRM];
    lbyte_t* const LB[2] = {(lbyte_t*)sm0, (lbyte_t*)sm1};
    lds_f* const PS = (lds_f*)prm;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
    const RfsJobs<mep_rf_epi_bwd_desc, W> jobs(descs, n_desc * nbat, nbat);
    auto woff = [](const mep_rf_epi_desc& d, int k) { return d.wparts + MEP_RFW_PART_OFFSET(D, FD, k); };
    auto tok_of = [&](int j) { return ((j % nbat) * W + wave) * 16 + c; };
    auto prm_load = [&](RfsParams<NPRM, 2, W>& pr, const mep_rf_epi_desc& d) {
        const uint64_t src[2] = {d.ln1_w, d.ln2_w};
        const int len[2] = {D, D};
        pr.load(src, len);
    };
    // the job's first product (Wq_in: dqp_in Wq, else W2^T) staged a step ahead, and its rows (MEP_RFS_BWD_PRE: a step ahead too):
    // dout, h, f, the stats and (Wq_in) dqp_in
    f32x4 gu[NI], hv[NI], fv[NI], dv[NI], st;
    auto stage_first = [&](const mep_rf_epi_bwd_desc& b, lbyte_t* buf) {
        if (b.wq_in) rfs_stage<NI, NP, D, W>(buf, b.wq_in, wave, lane);
        else rfs_stage<NF, NP, FD, W>(buf, woff(b.f, 5), wave, lane);
    };
    int job = jobs.first();
    if (job >= jobs.njobs) return;   // whole workgroup
    int ps = 0;
    {
        const mep_rf_epi_bwd_desc& b = descs[job / nbat];
        RfsParams<NPRM, 2, W> pr;
        prm_load(pr, b.f);
        stage_first(b, LB[0]);
        const int t = min(tok_of(job), b.f.ntok - 1);
        st = ld4w(G<const float>(b.f.stats) + 4 * (int64_t)t);
        load_rows<NI>(gu, b.dout, t);
        load_rows<NI>(hv, b.f.h, t);
        load_rows<NI>(fv, b.f.f, t);
        if (b.wq_in) load_rows<NI>(dv, b.dqp_in, t);
        pr.write(PS);
        rfs_sync();
    }
    // one job; P: the buffer of its first product, Q: the next layer's query-projection input
    // gradient fused (Wq_in first).  Returns the next job's first buffer
    auto body = [&](auto pc, auto qc) -> int {
        constexpr int P = decltype(pc)::value;
        constexpr bool Q = decltype(qc)::value;
        constexpr int C1 = Q ? P ^ 1 : P;   // W2^T's buffer
        job = __builtin_amdgcn_readfirstlane(job);
        const int nj = jobs.next(job);
        const mep_rf_epi_bwd_desc& bd = descs[job / nbat];
        const mep_rf_epi_desc& d = bd.f;
        const mep_rf_epi_bwd_desc* bn = nj < jobs.njobs ? &descs[nj / nbat] : nullptr;
        const int ntok = d.ntok, tok = tok_of(job), tc = min(tok, ntok - 1);
        const int tile = (job % nbat) * W + wave;
        const bool ok = tok < ntok, part_ok = tile * 16 < ntok;
        const float sa = *G<const float>(d.a), sb = *G<const float>(d.b);
        const lds_f* PR = PS + ps * NPRM;
        gfloat* part = G<float>(bd.partial) + (int64_t)tile * MEP_RF_PARTIAL_STRIDE(D, FD);
        if (!MEP_RFS_BWD_PRE) {   // (the A/B of the step-ahead rows: loaded here, waited for at once)
            st = ld4w(G<const float>(d.stats) + 4 * (int64_t)tc);
            load_rows<NI>(gu, bd.dout, tc);
            load_rows<NI>(hv, d.h, tc);
            load_rows<NI>(fv, d.f, tc);
            if (Q) load_rows<NI>(dv, bd.dqp_in, tc);
        }
        if (bd.dout2.ptr) {
            f32x4 g2[NI];
            load_rows<NI>(g2, bd.dout2, tc);
#pragma unroll
            for (int i = 0; i < NI; ++i) gu[i] += g2[i];
        }
        if constexpr (Q) {   // ---- dout += dqp_in Wq: the next layer's query-projection input gradient
            rfs_stage<NF, NP, FD, W>(LB[P ^ 1], woff(d, 5), wave, lane);
            f32x4 acc[NI];
            rfs_mul<NI, NP>(acc, LB[P], dv, lane);
#pragma unroll
            for (int i = 0; i < NI; ++i) gu[i] += acc[i];
        }
#pragma unroll
        for (int i = 0; i < NI; ++i)
            if (!ok) gu[i] = zero_f4();
        // LN2 backward -> dz2; df = b dz2
        f32x4 dz2[NI], df[NI], k_w2, k_b2, k_db2;
        float db_s = 0.f;
        {
            f32x4 xh[NI], pw2[NI], w2v[NI];
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                w2v[i] = ld4w(PR + D + 16 * i + 4 * g);
#pragma unroll
                for (int r = 0; r < 4; ++r) xh[i][r] = (add_rn(hv[i][r], mul_rn(sb, fv[i][r])) - st[2]) * st[3];
            }
            ln_bwd<NI>(dz2, gu, xh, w2v, st[3]);
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    pw2[i][r] = mul_rn(gu[i][r], xh[i][r]);   // rounded: a product fused into the column sum's first add would depend on the schedule
                    df[i][r] = sb * dz2[i][r];
                    db_s += dz2[i][r] * fv[i][r];
                }
            k_w2 = rfs_colsum<NI>(pw2, c);   // dLN2.w
            k_b2 = rfs_colsum<NI>(gu, c);    // dLN2.b
            k_db2 = rfs_colsum<NI>(df, c);   // db2
        }
        const float st0 = st[0], st1 = st[1];
        if constexpr (Q) rfs_sync();
        // ---- df1 = relu'(f1) (W2^T df)
        if (part_ok) {
            rfs_colsum_store(part, k_w2, NI, c, g);
            rfs_colsum_store(part + D, k_b2, NI, c, g);
            rfs_colsum_store(part + 4 * D, k_db2, NI, c, g);
        }
        if (ok) store_rows<NI>(bd.df, tok, df);
        rfs_stage<NI, NPF, D, W>(LB[C1 ^ 1], woff(d, 4), wave, lane);
        f32x4 f1v[NF];
        load_rows<NF>(f1v, d.f1, tc);
        f32x4 df1[NF];
        rfs_mul<NF, NP>(df1, LB[C1], df, lane);
#pragma unroll
        for (int j = 0; j < NF; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) df1[j][r] = (ok && f1v[j][r] > 0.f) ? df1[j][r] : 0.f;
        const f32x4 k_db1 = rfs_colsum<NF>(df1, c);
        rfs_sync();
        // ---- dh = dz2 + W1^T df1;  LN1 backward -> dz1;  dq (+)= dz1;  dxp = a dz1
        if (part_ok) rfs_colsum_store(part + 5 * D, k_db1, NF, c, g);
        if (ok) store_rows<NF>(bd.df1, tok, df1);
        rfs_stage<NI, NP, D, W>(LB[C1], woff(d, 3), wave, lane);
        f32x4 qv[NI], xpv[NI];
        load_rows<NI>(qv, d.q, tc);
        load_rows<NI>(xpv, d.xp, tc);
        f32x4 dh[NI];
        rfs_mul<NI, NPF>(dh, LB[C1 ^ 1], df1, lane);
#pragma unroll
        for (int i = 0; i < NI; ++i) dh[i] += dz2[i];
        f32x4 dxp[NI], dq[NI], k_w1, k_b1;
        float da_s = 0.f;
        {
            f32x4 xh[NI], dz1[NI], pw[NI], w1v[NI];
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                w1v[i] = ld4w(PR + 16 * i + 4 * g);
#pragma unroll
                for (int r = 0; r < 4; ++r) xh[i][r] = (add_rn(qv[i][r], mul_rn(sa, xpv[i][r])) - st0) * st1;
            }
            ln_bwd<NI>(dz1, dh, xh, w1v, st1);
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    pw[i][r] = mul_rn(dh[i][r], xh[i][r]);
                    dxp[i][r] = sa * dz1[i][r];
                    da_s += dz1[i][r] * xpv[i][r];
                }
            k_w1 = rfs_colsum<NI>(pw, c);   // dLN1.w
            k_b1 = rfs_colsum<NI>(dh, c);   // dLN1.b
            if (bd.dq_accumulate) {   // the old dq rows, loaded here (the plans never accumulate)
                f32x4 dqo[NI];
                load_rows<NI>(dqo, bd.dq, tc);
#pragma unroll
                for (int i = 0; i < NI; ++i) dq[i] = dqo[i] + dz1[i];
            } else {
#pragma unroll
                for (int i = 0; i < NI; ++i) dq[i] = dz1[i];
            }
        }
        const float da = wave_sum(da_s), db = wave_sum(db_s);
        rfs_sync();
        // ---- dx = Wp^T dxp
        if (part_ok) {
            rfs_colsum_store(part + 2 * D, k_w1, NI, c, g);
            rfs_colsum_store(part + 3 * D, k_b1, NI, c, g);
            if (lane == 0) { part[5 * D + FD] = da; part[5 * D + FD + 1] = db; }
        }
        if (ok) {
            store_rows<NI>(bd.dq, tok, dq);
            store_rows<NI>(bd.dxp, tok, dxp);
        }
        RfsParams<NPRM, 2, W> pr;
        if (bn) {   // the next job's parameters, first product and rows
            prm_load(pr, bn->f);
            stage_first(*bn, LB[C1 ^ 1]);
            if (MEP_RFS_BWD_PRE) {
                const int t = min(tok_of(nj), bn->f.ntok - 1);
                st = ld4w(G<const float>(bn->f.stats) + 4 * (int64_t)t);
                load_rows<NI>(gu, bn->dout, t);
                load_rows<NI>(hv, bn->f.h, t);
                load_rows<NI>(fv, bn->f.f, t);
                if (bn->wq_in) load_rows<NI>(dv, bn->dqp_in, t);
            }
        }
        f32x4 dx[NI];
        rfs_mul<NI, NP>(dx, LB[C1], dxp, lane);
        if (bn) pr.write(PS + (ps ^ 1) * NPRM);
        rfs_sync();
        if (ok) store_rows<NI>(bd.dx, tok, dx);
        ps ^= 1;
        job = nj;
        return C1 ^ 1;
    };
    int par = 0;
    while (job < jobs.njobs) {
        job = __builtin_amdgcn_readfirstlane(job);
        const bool q = descs[job / nbat].wq_in != 0;
        if (par) par = q ? body(std::integral_constant<int, 1>{}, std::true_type{}) : body(std::integral_constant<int, 1>{}, std::false_type{});
        else par = q ? body(std::integral_constant<int, 0>{}, std::true_type{}) : body(std::integral_constant<int, 0>{}, std::false_type{});
    }
}

// ---------------------------------------------------------------- token GEMM on pre-split weights
// Y[tok][n] = act(alpha sum_k X[tok][k] W'[n][k] + bias[n] + table[tok % T][n]) (+ Y): one workgroup
// per 16 tokens x 32 columns (grid.z = column groups), its 4 waves splitting the k pairs (wave w
// takes pairs w, w + 4, ...; every X block and weight fragment of a group of 4 pairs is loaded
// before its MFMAs, so a small K costs one memory latency, not one per pair); the 4 partial
// tiles are summed through LDS in wave order (deterministic) and wave 0 runs the epilogue.
#ifndef MEP_WGM_WAVES
#define MEP_WGM_WAVES 1   // waves splitting the k pairs of a workgroup (4: all loads of K <= 512 at once)
#endif
constexpr int WGM_WAVES = MEP_WGM_WAVES;
__global__ __launch_bounds__(64 * WGM_WAVES) void k_wgemm(const mep_gemm_desc* __restrict__ descs) {
    constexpr int NI = 2, GP = 4;   // output tiles per workgroup, pairs per wave per group
    __shared__ f32x4 red[WGM_WAVES][NI][64];
    const mep_gemm_desc& d = descs[blockIdx.y];
    const int tile = blockIdx.x, cg = blockIdx.z;
    const int ntok = d.ntok, N = d.N, K = d.K;
    if (tile * 16 >= ntok || cg * 32 >= N) return;   // whole workgroup
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
    const int tok = tile * 16 + c, tc = min(tok, ntok - 1);
    const int npk = (K + 31) >> 5;
    const bool xvec = (K % 4 == 0) && ((d.x.ptr & 15) == 0) && (d.x.sB % 4 == 0) && (d.x.sT % 4 == 0);
    const gfloat* xr = row_ptr(d.x, tc);
    const int rows = (N + 31) & ~31;   // rows of the parts (mep_wsplit R)
    const PartPtr wl = reinterpret_cast<PartPtr>(G<const unsigned char>(d.w)) + ((32 * cg + c) * npk) * 4 + g;
    const int tstride = rows * npk * 4;   // units per part
    // wave 0: the epilogue's loads (bias, position-table row, accumulated y), issued first
    f32x4 add[NI], yold[NI];
    if (wave == 0) {
        const gfloat* bias = G<const float>(d.bias);
        const gfloat* trow = d.table ? G<const float>(d.table) + (int64_t)(tc % d.y.T) * (d.ldt ? d.ldt : N) : nullptr;
        const gfloat* yr = row_ptr(d.y, tc);
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = min(32 * cg + 16 * i + 4 * g + r, N - 1);
                add[i][r] = (bias ? bias[n] : 0.f) + (trow ? trow[n] : 0.f);
                yold[i][r] = d.accumulate ? yr[n] : 0.f;
            }
    }
    auto xblk = [&](int k) {
        f32x4 v = zero_f4();
        if (xvec) {
            if (k < K) v = ld4w(xr + k);
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = k + e < K ? xr[k + e] : 0.f;
        }
        return v;
    };
    f32x4 acc[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) acc[i] = zero_f4();
    for (int p0 = wave; p0 < npk; p0 += WGM_WAVES * GP) {
        f32x4 x0[GP], x1[GP];
        OpN<3> a[GP][NI];
#pragma unroll
        for (int u = 0; u < GP; ++u) {
            const int p = p0 + WGM_WAVES * u;
            if (p < npk) {
                x0[u] = xblk(32 * p + 4 * g);
                x1[u] = xblk(32 * p + 16 + 4 * g);
#pragma unroll
                for (int i = 0; i < NI; ++i)
#pragma unroll
                    for (int t = 0; t < 3; ++t)
                        a[u][i].p[t] = __builtin_bit_cast(bf16x8, wl[t * tstride + (16 * i * npk + p) * 4]);
            }
        }
#pragma unroll
        for (int u = 0; u < GP; ++u) {
            if (p0 + WGM_WAVES * u < npk) {
                const OpN<3> b = opn<3>(x0[u], x1[u]);
#pragma unroll
                for (int i = 0; i < NI; ++i) acc[i] = mma_n<3>(a[u][i], b, acc[i]);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) red[wave][i][lane] = acc[i];
    __syncthreads();
    if (wave != 0 || tok >= ntok) return;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        f32x4 t = red[0][i][lane];
#pragma unroll
        for (int w = 1; w < WGM_WAVES; ++w) t += red[w][i][lane];
        acc[i] = t;
    }
    gfloat* yr = row_ptr(d.y, tok);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int n = 32 * cg + 16 * i + 4 * g + r;
            if (n >= N) continue;
            float v = d.alpha * acc[i][r] + add[i][r];
            if (d.relu) v = fmaxf(v, 0.f);
            if (d.accumulate) v += yold[i][r];
            yr[n] = v;
        }
    }
}

// ---------------------------------------------------------------- input-gradient GEMMs + their sum
// mep_wgemm_sum: wave s of a workgroup computes source s's output tile with k_wgemm's arithmetic
// (one accumulator chain over the k pairs in order, then alpha, bias + table, relu, + y), parks
// it in LDS, and wave 0 adds the sources in order onto 0 (the k_sum_rows sequence) and writes
// the sum.  The sources' y rows are read, never written.  A workgroup covers 16 tokens x 16 NI
// columns; the fragments of GP k pairs are loaded before their MFMAs (GP = 6: K <= 192 in one
// memory latency).  The group size only schedules loads, so the results match k_wgemm bit for
// bit (test_wgemm_sum_matches_wgemm_and_sum_rows).
#ifndef MEP_WGSUM_NI
#define MEP_WGSUM_NI 1
#endif
#ifndef MEP_WGSUM_GP
#define MEP_WGSUM_GP 6
#endif
__global__ __launch_bounds__(64 * MEP_WGEMM_SUM_MAX) void k_wgemm_sum(const mep_gemm_sum_desc* __restrict__ descs) {
    constexpr int NI = MEP_WGSUM_NI, GP = MEP_WGSUM_GP, CW = 16 * NI;
    __shared__ f32x4 red[MEP_WGEMM_SUM_MAX][NI][64];
    const mep_gemm_sum_desc& sd = descs[blockIdx.y];
    const int tile = blockIdx.x, cg = blockIdx.z;
    const int ntok = sd.src[0].ntok, N = sd.src[0].N, n_src = min(sd.n_src, MEP_WGEMM_SUM_MAX);
    if (tile * 16 >= ntok || cg * CW >= N) return;   // whole workgroup
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int tok = tile * 16 + c, tc = min(tok, ntok - 1);
    if (wave < n_src) {
        const mep_gemm_desc& d = sd.src[wave];
        const int K = d.K, npk = (K + 31) >> 5;
        const bool xvec = (K % 4 == 0) && ((d.x.ptr & 15) == 0) && (d.x.sB % 4 == 0) && (d.x.sT % 4 == 0);
        const gfloat* xr = row_ptr(d.x, tc);
        const int tstride = ((N + 31) & ~31) * npk * 4;
        const PartPtr wl = reinterpret_cast<PartPtr>(G<const unsigned char>(d.w)) + ((CW * cg + c) * npk) * 4 + g;
        f32x4 add[NI], yold[NI];
        {
            const gfloat* bias = G<const float>(d.bias);
            const gfloat* trow = d.table ? G<const float>(d.table) + (int64_t)(tc % d.y.T) * (d.ldt ? d.ldt : N) : nullptr;
            const gfloat* yr = row_ptr(d.y, tc);
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int n = min(CW * cg + 16 * i + 4 * g + r, N - 1);
                    add[i][r] = (bias ? bias[n] : 0.f) + (trow ? trow[n] : 0.f);
                    yold[i][r] = d.accumulate ? yr[n] : 0.f;
                }
        }
        auto xblk = [&](int k) {
            f32x4 v = zero_f4();
            if (xvec) {
                if (k < K) v = ld4w(xr + k);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = k + e < K ? xr[k + e] : 0.f;
            }
            return v;
        };
        f32x4 acc[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[i] = zero_f4();
        for (int p0 = 0; p0 < npk; p0 += GP) {
            f32x4 x0[GP], x1[GP];
            OpN<3> a[GP][NI];
#pragma unroll
            for (int u = 0; u < GP; ++u) {
                const int p = p0 + u;
                if (p < npk) {
                    x0[u] = xblk(32 * p + 4 * g);
                    x1[u] = xblk(32 * p + 16 + 4 * g);
#pragma unroll
                    for (int i = 0; i < NI; ++i)
#pragma unroll
                        for (int t = 0; t < 3; ++t)
                            a[u][i].p[t] = __builtin_bit_cast(bf16x8, wl[t * tstride + (16 * i * npk + p) * 4]);
                }
            }
#pragma unroll
            for (int u = 0; u < GP; ++u) {
                if (p0 + u < npk) {
                    const OpN<3> b = opn<3>(x0[u], x1[u]);
#pragma unroll
                    for (int i = 0; i < NI; ++i) acc[i] = mma_n<3>(a[u][i], b, acc[i]);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            f32x4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float e = d.alpha * acc[i][r] + add[i][r];
                if (d.relu) e = fmaxf(e, 0.f);
                if (d.accumulate) e += yold[i][r];
                v[r] = e;
            }
            red[wave][i][lane] = v;
        }
    }
    __syncthreads();
    if (wave != 0 || tok >= ntok) return;
    gfloat* o = row_ptr(sd.out, tok);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        f32x4 s = zero_f4();
        for (int w = 0; w < n_src; ++w) s += red[w][i][lane];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int n = CW * cg + 16 * i + 4 * g + r;
            if (n < N) o[n] = s[r];
        }
    }
}

// ---------------------------------------------------------------- weight-stationary token GEMM
// mep_wgemm's contract with the weight block resident in LDS.  A workgroup owns the 16 NT output
// columns [16 NT z, 16 NT (z + 1)) of one descriptor (grid (gx, n_desc, z)): it copies their parts
// (every k pair) from the mep_wsplit image into LDS once (SplitWS: conflict-free 16-byte fragment
// reads), then its W waves walk the 16-token tiles (blockIdx.x + gridDim.x j) W + wave, each
// wave holding the next tile's X rows in registers while it multiplies the current one.  A
// fragment read (three ds_read_b128, 12 LDS cycles) feeds six 16-cycle MFMAs, so four SIMDs keep
// the LDS array half busy.  Products and summation order are k_wgemm's (k pairs in order, six
// products each, then alpha, bias + table, relu, + y), so the two agree bit for bit.
// NT * NPK <= 36 (110.6 KB of LDS).
constexpr int WGS_MAX_WAVES = 8;
#ifndef MEP_WGS_RING
#define MEP_WGS_RING 3   // weight fragments (3 x 16 B per lane each) read ahead of their MFMAs
#endif
template <int NT, int NPK, bool XV>
__global__ __launch_bounds__(64 * WGS_MAX_WAVES) void k_wgemm_ws(const mep_gemm_desc* __restrict__ descs) {
    using WS = SplitWS<16 * NT, NPK, 3>;
    __shared__ __attribute__((aligned(16))) unsigned char sm[WS::BYTES];
    const mep_gemm_desc& d = descs[blockIdx.y];
    const int ntok = d.ntok, N = d.N, K = d.K;
    const int W = blockDim.x >> 6;
    const int ntile = (ntok + 15) >> 4;
    const int n0 = (int)blockIdx.z * 16 * NT;
    if (n0 >= N || (int)blockIdx.x * W >= ntile) return;   // the whole workgroup
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
    const int npk = (K + 31) >> 5;
    const int nt = min(NT, (N - n0 + 15) >> 4);
    typedef __attribute__((address_space(3))) unsigned char lbyte;
    const WS ws{(lbyte*)sm, 0};
    const bool yvec = ((d.y.ptr & 15) == 0) && (d.y.sB % 4 == 0) && (d.y.sT % 4 == 0);
    // X blocks of a tile with no branches or selects (either makes the compiler wait for the
    // loads where they are issued): clamped addresses only -- the values loaded for k >= K are
    // finite row data that meet zero weights (mep_wsplit pads K with zeros, pairs past the
    // descriptor's K are zero in LDS).  XV: 16-byte loads of K rounded up to 4 (the host's
    // MEP_WGEMM_XVEC contract), else one float at a time.
    const int KV = XV ? (K + 3) & ~3 : K;
    auto load_x = [&](int tile, f32x4 (&v)[2 * NPK]) {
        const gfloat* xr = row_ptr(d.x, min(min(tile, ntile - 1) * 16 + c, ntok - 1));
#pragma unroll
        for (int h = 0; h < 2 * NPK; ++h) {
            const int k = 16 * h + 4 * g;   // block h = (pair h / 2, half h % 2)
            if constexpr (XV) {
                v[h] = ld4w(xr + min(k, KV - 4));
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[h][e] = xr[min(k + e, K - 1)];
            }
        }
    };
    {
        int tile = (int)blockIdx.x * W + wave;
        const int step = (int)gridDim.x * W;
        f32x4 xc[2 * NPK];
        load_x(tile, xc);   // in flight across the weight copy
        {
            // k pairs past the descriptor's K are stored as zeros and its X blocks there are zeros, so
            // every tile runs all NPK pairs and all NT output tiles with no guards (tiles past N read
            // rows never stored and are never written back); a launch's short-K / narrow descriptors
            // then do the work of its widest, on workgroups of their own
            const PartPtr src = parts_at(d.w, 0);
            const int64_t part = (int64_t)((N + 31) & ~31) * npk * 4;   // units per part (mep_wsplit R)
            constexpr int UNITS = 16 * NT * NPK * 4;                     // per part
            const int units = 16 * nt * NPK * 4;
            // FB units per thread loaded before any is stored: one memory latency per FB rounds
            constexpr int FB = 8;
            for (int u0 = threadIdx.x; u0 < 3 * units; u0 += FB * blockDim.x) {
                u32x4 v[FB];
#pragma unroll
                for (int j = 0; j < FB; ++j) {
                    const int u = min(u0 + j * (int)blockDim.x, 3 * units - 1);
                    const int t = u / units, r = u - t * units;
                    const int np = r >> 2, nl = np / NPK, p = np - nl * NPK;
                    const u32x4 w = src[t * part + ((int64_t)(n0 + nl) * npk + min(p, npk - 1)) * 4 + (r & 3)];
                    v[j] = p < npk ? w : u32x4{0u, 0u, 0u, 0u};
                }
#pragma unroll
                for (int j = 0; j < FB; ++j) {
                    const int u = u0 + j * blockDim.x;
                    const int t = u / units, r = u - t * units;
                    const int np = r >> 2, nl = np / NPK, p = np - nl * NPK;
                    if (u < 3 * units) ws.put_unit(t, nl, p, r & 3, v[j]);
                }
            }
            static_assert(3 * UNITS * 16 == WS::BYTES, "k_wgemm_ws: LDS image size");
        }
        __syncthreads();
        const gfloat* bias = d.bias ? G<const float>(d.bias) : nullptr;
        const gfloat* table = d.table ? G<const float>(d.table) : nullptr;
        const int ldt = d.ldt ? d.ldt : N;
        // the next tile's X blocks prefetched into registers while this one multiplies (PF), or
        // (NPK = 10: 80 more registers) loaded at the top of each tile, behind the other waves
        constexpr bool PF = NPK <= 6;
        // one tile on X blocks xcur (loaded), the next tile's blocks into xnext: the loop runs
        // tiles in pairs with the two buffers swapping roles, so no register copy makes the
        // compiler wait for the prefetch (and, behind it, for the epilogue's stores)
        auto one_tile = [&](f32x4 (&xcur)[2 * NPK], f32x4 (&xnext)[2 * NPK]) {
            if constexpr (PF) {
                load_x(tile + step, xnext);
            } else {
                if (tile != (int)blockIdx.x * W + wave) load_x(tile, xcur);
            }
            f32x4 acc[NT];
#pragma unroll
            for (int i = 0; i < NT; ++i) acc[i] = zero_f4();
            // steps s = (pair p, tile i), p-major; fragments MEP_WGS_RING steps ahead of their MFMAs
            constexpr int S = NPK * NT, RING = MEP_WGS_RING < S ? MEP_WGS_RING : S;
            OpN<3> ring[RING];
#pragma unroll
            for (int s = 0; s < RING; ++s) ring[s] = ws.frag(s % NT, s / NT);
            OpN<3> b;
#pragma unroll
            for (int s = 0; s < S; ++s) {
                const int p = s / NT, i = s % NT;
                if (i == 0) b = opn<3>(xcur[2 * p], xcur[2 * p + 1]);
                const OpN<3> a = ring[s % RING];
                if (s + RING < S) ring[s % RING] = ws.frag((s + RING) % NT, (s + RING) / NT);
                acc[i] = mma_n<3>(a, b, acc[i]);
                __builtin_amdgcn_sched_barrier(0);
            }
            const int tok = tile * 16 + c;
            // the lane's column offset as a loop-variant value: otherwise the compiler hoists the
            // epilogue's NT x 4 column clamps, compare masks and addresses out of the tile loop
            // (~100 registers live across the products, spilled)
            int gcol = 4 * g;
            asm volatile("" : "+v"(gcol));
            if (tok < ntok) {
                gfloat* yr = row_ptr(d.y, tok);
                const gfloat* trow = table ? table + (int64_t)(tok % d.y.T) * ldt : nullptr;
                // three output tiles at a time: the bias / table / y loads of a group in flight
                // together, never all NT groups' (their registers on top of the accumulators)
#pragma unroll
                for (int i0 = 0; i0 < NT; i0 += 3) {
                    f32x4 add[3], yo[3];
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
                        const int nb = n0 + 16 * (i0 + j) + gcol;
                        add[j] = yo[j] = zero_f4();
                        if (i0 + j >= nt) continue;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int n = min(nb + r, N - 1);
                            add[j][r] = (bias ? bias[n] : 0.f) + (trow ? trow[n] : 0.f);
                            if (d.accumulate) yo[j][r] = yr[n];
                        }
                    }
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
                        const int i = i0 + j, nb = n0 + 16 * i + gcol;
                        if (i >= nt) continue;
                        f32x4 v;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            float s = d.alpha * acc[i][r] + add[j][r];
                            if (d.relu) s = fmaxf(s, 0.f);
                            v[r] = d.accumulate ? s + yo[j][r] : s;
                        }
                        if (yvec && nb + 3 < N) {
                            *reinterpret_cast<MEP_G f32x4*>(yr + nb) = v;
                        } else {
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                if (nb + r < N) yr[nb + r] = v[r];
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        };
        if constexpr (PF) {
            f32x4 xn[2 * NPK];
            while (tile < ntile) {
                one_tile(xc, xn);
                tile += step;
                if (tile >= ntile) break;
                one_tile(xn, xc);
                tile += step;
            }
        } else {
            for (; tile < ntile; tile += step) one_tile(xc, xc);
        }
    }
}

// ---------------------------------------------------------------- realformer front
// mep_rfw_front (include/mep.h): the unify of a 16-token tile (wave w: U features 16 w .. +15, its
// K pairs streamed through a fragment ring), U stored and exchanged through LDS, then every
// projection of U with the output tiles dealt round-robin to the six waves, the fragments of a
// wave's next tile in flight while it multiplies the current one (two register sets in turn).
// The products, their order and the unify epilogue are mep_wgemm's, so U, K / V and Q agree with
// the mep_wgemm launches bit for bit.
#ifndef MEP_FRONT_DEPTH
#define MEP_FRONT_DEPTH 4   // unify weight fragments in flight ahead of their MFMAs
#endif
template <int NPKU>
__global__ __launch_bounds__(384) void k_rfw_front(const mep_rf_front_desc* __restrict__ descs) {
    constexpr int NI = 6, W = 6, RU = 96;   // U tiles (D = 96), waves, rows of the unify parts
    __shared__ f32x4 ubuf[NI * 64];
    const mep_rf_front_desc& fd = descs[blockIdx.y];
    const mep_gemm_desc& u = fd.unify;
    const int ntok = u.ntok;
    if ((int)blockIdx.x * 16 >= ntok) return;
    // descriptor bounds (uniform per workgroup): tile_map / out[] are fixed-size arrays
    if (fd.n_tiles < 0 || fd.n_tiles > MEP_RF_FRONT_MAX_TILES || fd.n_out <= 0 || fd.n_out > MEP_RF_FRONT_MAX_OUT) return;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15, g = lane >> 4;
    const int tok = (int)blockIdx.x * 16 + c, tc = min(tok, ntok - 1);
    // X row blocks: 16-byte loads of K rounded up to 4, clamped (values past K meet zero weights)
    const int KV = (u.K + 3) & ~3;
    f32x4 xr[2 * NPKU];
    {
        const gfloat* xp = row_ptr(u.x, tc);
#pragma unroll
        for (int h = 0; h < 2 * NPKU; ++h) xr[h] = ld4w(xp + min(16 * h + 4 * g, KV - 4));
    }
    const int n = 16 * wave + 4 * g;   // the lane's U features n .. n + 3
    f32x4 add;
    {
        const gfloat* bias = u.bias ? G<const float>(u.bias) : nullptr;
        const gfloat* trow = u.table ? G<const float>(u.table) + (int64_t)(tc % u.y.T) * (u.ldt ? u.ldt : RU) : nullptr;
#pragma unroll
        for (int r = 0; r < 4; ++r) add[r] = (bias ? bias[n + r] : 0.f) + (trow ? trow[n + r] : 0.f);
    }
    const PartPtr wu = parts_at(u.w, 0) + ((16 * wave + c) * NPKU) * 4 + g;
    auto fragu = [&](int p) {
        OpN<3> o;
#pragma unroll
        for (int t = 0; t < 3; ++t) o.p[t] = __builtin_bit_cast(bf16x8, wu[(t * RU * NPKU + p) * 4]);
        return o;
    };
    constexpr int DEP = MEP_FRONT_DEPTH < NPKU ? MEP_FRONT_DEPTH : NPKU;
    OpN<3> ring[DEP];
#pragma unroll
    for (int s = 0; s < DEP; ++s) ring[s] = fragu(s);
    // the projections' tiles: wave's j-th tile t = wave + W j; fragment (t, p) of out[o] rows
    // 16 lt + c, three k pairs (K = 96)
    const int nt = fd.n_tiles, nj = (nt - wave + W - 1) / W;
    auto frag2 = [&](int j, OpN<3> (&f)[3]) {
        const int m = fd.tile_map[wave + W * min(j, nj - 1)];
        const mep_rf_front_out& q = fd.out[m >> 8];
        const int R = (q.N + 31) & ~31;
        const PartPtr w = parts_at(q.w, 0) + ((16 * (m & 255) + c) * 3) * 4 + g;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int t = 0; t < 3; ++t) f[p].p[t] = __builtin_bit_cast(bf16x8, w[(t * R * 3 + p) * 4]);
    };
    f32x4 acc = zero_f4();
#pragma unroll
    for (int p = 0; p < NPKU; ++p) {
        const OpN<3> a = ring[p % DEP];
        if (p + DEP < NPKU) ring[p % DEP] = fragu(p + DEP);
        acc = mma_n<3>(a, opn<3>(xr[2 * p], xr[2 * p + 1]), acc);
        __builtin_amdgcn_sched_barrier(0);
    }
    OpN<3> fa[3], fb[3];
    if (nj > 0) frag2(0, fa);   // the first projection tile's weights in flight across the exchange
    f32x4 uv;
#pragma unroll
    for (int r = 0; r < 4; ++r) uv[r] = u.alpha * acc[r] + add[r];
    if (tok < ntok) *reinterpret_cast<MEP_G f32x4*>(row_ptr(u.y, tok) + n) = uv;
    ubuf[wave * 64 + lane] = uv;
    lds_barrier();
    OpN<3> bu[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) bu[p] = opn<3>(ubuf[2 * p * 64 + lane], ubuf[(2 * p + 1) * 64 + lane]);
    auto tile_out = [&](int j, const OpN<3> (&f)[3]) {
        f32x4 o = zero_f4();
#pragma unroll
        for (int p = 0; p < 3; ++p) o = mma_n<3>(f[p], bu[p], o);
        const int m = fd.tile_map[wave + W * j];
        const mep_rf_front_out& q = fd.out[m >> 8];
        if (tok < ntok) *reinterpret_cast<MEP_G f32x4*>(row_ptr(q.y, tok) + 16 * (m & 255) + 4 * g) = o;
    };
    for (int j = 0; j < nj; j += 2) {
        frag2(j + 1, fb);
        tile_out(j, fa);
        if (j + 1 >= nj) break;
        frag2(j + 2, fa);
        tile_out(j + 1, fb);
    }
}

template <typename F>
int dispatch_rfw(int D, int FD, F&& f) {
#define MEP_RFW_CASE(DD, FF) \
    if (D == DD && FD == FF) { f(std::integral_constant<int, DD>{}, std::integral_constant<int, FF>{}); return 0; }
    MEP_RFW_CASE(32, 32) MEP_RFW_CASE(32, 64) MEP_RFW_CASE(64, 64) MEP_RFW_CASE(64, 128)
    MEP_RFW_CASE(96, 96) MEP_RFW_CASE(96, 192) MEP_RFW_CASE(128, 128) MEP_RFW_CASE(128, 256)
#undef MEP_RFW_CASE
    return MEP_EINVAL;
}

}  // namespace


extern "C" int mep_rf_rows(int which, int D) {
    return which == 2 ? 16 : which == 1 ? MEP_RF_BWD_ROWS_BUILT : (D > 128 ? 32 : MEP_RF_FWD_ROWS_BUILT);
}

extern "C" int mep_wsplit(const mep_wsplit_desc* descs, int n_desc, int max_units, mep_stream_t stream) {
    if (n_desc <= 0 || max_units <= 0) return 0;
    hipLaunchKernelGGL(k_wsplit, dim3((max_units + 255) / 256, n_desc), dim3(256), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_wsplit");
}

extern "C" int mep_wgemm(const mep_gemm_desc* descs, int n_desc, int max_tiles, int max_n, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    if (max_n <= 0 || max_n > 256) { mep_set_error("mep_wgemm: 0 < max_n <= 256"); return MEP_EINVAL; }
    // grid.z: the 32-column groups of the widest descriptor
    hipLaunchKernelGGL(k_wgemm, dim3(max_tiles, n_desc, (max_n + 31) / 32), dim3(64 * WGM_WAVES), 0,
                       (hipStream_t)stream, descs);
    return mep_check_launch("mep_wgemm");
}

extern "C" int mep_wgemm_sum(const mep_gemm_sum_desc* descs, int n_desc, int max_tiles, int max_n, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    if (max_n <= 0 || max_n > 256) { mep_set_error("mep_wgemm_sum: 0 < max_n <= 256"); return MEP_EINVAL; }
    hipLaunchKernelGGL(k_wgemm_sum, dim3(max_tiles, n_desc, (max_n + 16 * MEP_WGSUM_NI - 1) / (16 * MEP_WGSUM_NI)),
                       dim3(64 * MEP_WGEMM_SUM_MAX), 0,
                       (hipStream_t)stream, descs);
    return mep_check_launch("mep_wgemm_sum");
}

#ifndef MEP_WGS_MIN_WG
#define MEP_WGS_MIN_WG 256   // column blocks narrow (12 -> 6 -> 3 tiles) until a launch has this many workgroups
#endif
extern "C" int mep_wgemm_ws(const mep_gemm_desc* descs, int n_desc, int max_ntok, int max_n, int max_k,
                            int flags, mep_stream_t stream) {
    if (n_desc <= 0 || max_ntok <= 0) return 0;
    const int npk = (max_k + 31) / 32, ntf = (max_n + 15) / 16;
    if (max_n <= 0 || max_k <= 0 || npk > 10) { mep_set_error("mep_wgemm_ws: 0 < max_n, 0 < max_k <= 320"); return MEP_EINVAL; }
    const int NPK = npk <= 3 ? 3 : npk <= 6 ? 6 : 10;
    int NT = NPK == 3 ? 12 : NPK == 6 ? 6 : 3;          // NT * NPK <= 36
    while (NT > 3 && ntf <= NT / 2) NT /= 2;            // no wider than the widest descriptor needs
    const int tiles = (max_ntok + 15) / 16;
    auto blocks = [&](int nt, int w) { return (int64_t)n_desc * ((ntf + nt - 1) / nt) * ((tiles + w - 1) / w); };
    while (NT > 3 && blocks(NT, WGS_MAX_WAVES) < MEP_WGS_MIN_WG) NT /= 2;
    const int W = blocks(NT, WGS_MAX_WAVES) < MEP_WGS_MIN_WG ? WGS_MAX_WAVES / 2 : WGS_MAX_WAVES;
    const int nz = (ntf + NT - 1) / NT;
    const dim3 block(64 * W);
    hipStream_t st = (hipStream_t)stream;
    // persistent: one resident round of workgroups, each walking its tiles.  The occupancy (by
    // registers and LDS) is cached per instance, block size and device -- any host thread may
    // launch on any device; the cached values are idempotent, so relaxed atomics suffice -- and
    // the CU count is read per call
    auto run = [&](auto kern, int slot) {
        constexpr int MAX_DEV = 64;
        static std::atomic<int> per_cu[MAX_DEV][2][16];
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
        std::atomic<int>& cached = per_cu[dev % MAX_DEV][W == WGS_MAX_WAVES][slot];
        int pc = cached.load(std::memory_order_relaxed);
        if (pc == 0) {
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, kern, 64 * W, 0) != hipSuccess) pc = 1;
            pc = std::max(pc, 1);
            cached.store(pc, std::memory_order_relaxed);
        }
        int n_cu = 0;
        if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0) n_cu = 256;
        const int64_t fit = std::max<int64_t>(1, (int64_t)n_cu * pc / ((int64_t)n_desc * nz));
        const int gx = (int)std::min<int64_t>((tiles + W - 1) / W, fit);
        hipLaunchKernelGGL(kern, dim3(gx, n_desc, nz), block, 0, st, descs);
    };
    const bool xv = flags & MEP_WGEMM_XVEC;
#define MEP_WGS(A, B, S) if (NT == A && NPK == B) { if (xv) run(k_wgemm_ws<A, B, true>, 2 * S); else run(k_wgemm_ws<A, B, false>, 2 * S + 1); }
    MEP_WGS(12, 3, 0); MEP_WGS(6, 3, 1); MEP_WGS(3, 3, 2); MEP_WGS(6, 6, 3); MEP_WGS(3, 6, 4); MEP_WGS(3, 10, 5);
#undef MEP_WGS
    return mep_check_launch("mep_wgemm_ws");
}

extern "C" int mep_rfw_front(const mep_rf_front_desc* descs, int n_desc, int max_tiles, int npk_u, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    const dim3 grid(max_tiles, n_desc), block(384);
    hipStream_t st = (hipStream_t)stream;
    switch (npk_u) {
        case 2: hipLaunchKernelGGL(k_rfw_front<2>, grid, block, 0, st, descs); break;
        case 3: hipLaunchKernelGGL(k_rfw_front<3>, grid, block, 0, st, descs); break;
        case 10: hipLaunchKernelGGL(k_rfw_front<10>, grid, block, 0, st, descs); break;
        default: mep_set_error("mep_rfw_front: npk_u in {2, 3, 10}"); return MEP_EINVAL;
    }
    return mep_check_launch("mep_rfw_front");
}

// the weight-stationary kernels for the large launches: on unless MEP_RFS=0 in the environment
// (read per call: the A/B switch of the tests and benches); one resident workgroup per CU
static bool rfs_on() {
    const char* e = getenv("MEP_RFS");
    return !(e && e[0] == '0');
}
static int rfs_grid(int njobs) {
    int dev = 0, n_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n_cu <= 0)
        n_cu = 256;
    return std::max(1, std::min(njobs, n_cu));
}

extern "C" int mep_rfw_epi_fwd(const mep_rf_epi_desc* descs, int n_desc, int max_tiles, int D, int FD,
                               mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    const bool big = (int64_t)max_tiles * n_desc >= MEP_RFW_BIG_TILES;
    const int rc = dispatch_rfw(D, FD, [&](auto dc, auto fc) {
        constexpr int DD = decltype(dc)::value, FF = decltype(fc)::value;
        if constexpr (DD == 96 && FF == 192) {
            if (big && rfs_on()) {
                const int nbat = (max_tiles + MEP_RFS_FWD_W - 1) / MEP_RFS_FWD_W;
                hipLaunchKernelGGL((k_rfs_fwd<DD, FF, MEP_RFS_FWD_W>), dim3(rfs_grid(n_desc * nbat)), dim3(64 * MEP_RFS_FWD_W), 0,
                                   (hipStream_t)stream, descs, n_desc, nbat);
                return;
            }
        }
        if (DD == 96 && big)
            hipLaunchKernelGGL((k_rfw_fwd<DD, FF, rfw_waves<DD>(), MEP_RFW_BIG_WPE, MEP_RFW_BIG_DEPTH, MEP_RFW_BIG_WPARTS>), dim3(max_tiles, n_desc),
                               dim3(64 * rfw_waves<DD>()), 0, (hipStream_t)stream, descs);
        else
            hipLaunchKernelGGL((k_rfw_fwd<DD, FF>), dim3(max_tiles, n_desc), dim3(64 * rfw_waves<DD>()), 0,
                               (hipStream_t)stream, descs);
    });
    if (rc) { mep_set_error("mep_rfw_epi_fwd: D in {32,64,96,128} and FD in {D, 2D}"); return rc; }
    return mep_check_launch("mep_rfw_epi_fwd");
}

extern "C" int mep_rfw_epi_bwd(const mep_rf_epi_bwd_desc* descs, int n_desc, int max_tiles, int D, int FD,
                               mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    const bool big = (int64_t)max_tiles * n_desc >= MEP_RFW_BIG_TILES;
    const int rc = dispatch_rfw(D, FD, [&](auto dc, auto fc) {
        constexpr int DD = decltype(dc)::value, FF = decltype(fc)::value;
        if constexpr (DD == 96 && FF == 192) {
            if (big && rfs_on()) {
                const int nbat = (max_tiles + MEP_RFS_BWD_W - 1) / MEP_RFS_BWD_W;
                hipLaunchKernelGGL((k_rfs_bwd<DD, FF, MEP_RFS_BWD_W>), dim3(rfs_grid(n_desc * nbat)), dim3(64 * MEP_RFS_BWD_W), 0,
                                   (hipStream_t)stream, descs, n_desc, nbat);
                return;
            }
        }
        if (DD == 96 && big)
            hipLaunchKernelGGL((k_rfw_bwd<DD, FF, rfw_waves<DD>(), 1, MEP_RFW_DEPTH, MEP_RFW_BIG_WPARTS>), dim3(max_tiles, n_desc),
                               dim3(64 * rfw_waves<DD>()), 0, (hipStream_t)stream, descs);
        else
            hipLaunchKernelGGL((k_rfw_bwd<DD, FF>), dim3(max_tiles, n_desc), dim3(64 * rfw_waves<DD>()), 0,
                               (hipStream_t)stream, descs);
    });
    if (rc) { mep_set_error("mep_rfw_epi_bwd: D in {32,64,96,128} and FD in {D, 2D}"); return rc; }
    return mep_check_launch("mep_rfw_epi_bwd");
}
