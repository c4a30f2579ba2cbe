// Residual scaled-dot-product attention core, forward and backward, hd = 16.
//
// Reference: Attention_Block.multi_head_attention, cmu-mosei/run.py:236-256 (identical in
// Ren-MME/run.py:188-208 and, after the w_qkv projections, others/realformer.py:182-204):
//   S = q k^T / sqrt(hd) [+ c * S_prev];  S -= 1e8 (1 - mask);  X = softmax(S) v
// The post-mask S is returned to the caller, which feeds it to the next layer of the chain.
//
// Arithmetic (fp32 path): fp32 storage, fp32 softmax / score sequence, products on the bf16 matrix cores
// with every fp32 operand split into bf16 parts (x = x0 + x1 [+ x2], each part the round-to-
// nearest bf16 of the remainder; products of bf16 parts are exact in the fp32 accumulator):
//   scores q.k (fwd and bwd)   3-way split, the six products x_i y_j with i + j <= 2:
//                              relative error ~2^-24 per product (fp32 level)
//   backward dP, dV, dK, dQ    2-way split, three or four products: relative error <= 2^-16
//   forward P.V                fp32 MFMA (v_mfma_f32_16x16x4_f32) on the raw P and V: exact
// bf16 path (MEP_PREC_BF16): every product takes the bf16 parts only (scores and 16-deep
// contractions on v_mfma_f32_16x16x16_bf16, P.V and dQ on 16x16x32 with P rounded to bf16), fp32
// softmax, scores and storage as above.
// v_mfma_f32_16x16x32_bf16 takes 8 k-slots per lane; the slot -> index assignment is free as long
// as A and B agree, so a lane's 4 consecutive fp32 values of a 16-wide contraction (the index
// layout (step s, lane group g) -> 4g + s of the fp32 16x16x4 form) fill slots 0-3 with one part
// and slots 4-7 with another: a 16-deep fp32 contraction costs 2 (or 3) bf16 MFMAs of 16 cycles
// instead of 4 fp32 MFMAs of 32 cycles, and every operand is still one 16-byte load.  The
// forward and the backward issue the score products in the same slots, so the recomputed
// backward scores equal the forward's bit for bit.
//
// Mapping (CDNA4)
//   forward   one WAVE per (b, h, 64 queries); S^T = K Q^T leaves lane (query c, group g)
//             holding keys 4g..4g+3 of each 16-key tile -- the A operand of O = P V directly.
//             Keys in chunks of 64 (exact two-pass softmax for T <= 64, online rescale above).
//   backward  one WORKGROUP (4 waves) per (b, h).  Key chunks of 64 are the outer loop; wave w
//             takes query tiles w, w+4, ...  S = Q K^T and dP = dO V^T leave lane (key c, g)
//             holding queries 4g..4g+3: the A operand of dV += P^T dO and dK += dS^T Q; dQ += dS K
//             needs dS with the query on the lane (one 16 x 64 LDS transpose per query tile).
//             dK / dV partials of the 4 waves are summed through LDS in wave order; a query
//             tile's dQ is owned by one wave and carried across key chunks in LDS: every sum
//             has a fixed order, so the backward is deterministic for every Tk.
// Row statistics (max, 1/sum) are kept instead of log-sum-exp because fully masked rows sit at
// -1e8 where max + log(sum) would round the log away (ulp(1e8) = 8).
#include <float.h>

#include "common.h"

using namespace mep;

namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#ifndef MEP_BWD_WAVES
#define MEP_BWD_WAVES 3    // waves per SIMD of the short backward
#endif
#ifndef MEP_BWD_WAVES_KV
#define MEP_BWD_WAVES_KV 4 // waves per SIMD of the short backward with MEP_ATTN_KV (<= 128 registers)
#endif
#ifndef MEP_FWD_WAVES
#define MEP_FWD_WAVES 3    // waves per SIMD of the short, non-residual forward
#endif
#ifndef MEP_BWD_WIDE_WAVES
#define MEP_BWD_WIDE_WAVES 0   // waves per SIMD of the wide Tk > 64 backward (0: as the short one)
#endif
#ifndef MEP_FWD_LONG_WAVES
#define MEP_FWD_LONG_WAVES 2   // waves per SIMD of the Tk > 64 forward (hd 16), fp32 split path
#endif
#ifndef MEP_FWD_LONG_WAVES_BF
#define MEP_FWD_LONG_WAVES_BF 2   // the same, bf16 path
#endif

constexpr int HD = 16;
constexpr int WAVES = 4;
constexpr int THREADS = 64 * WAVES;
constexpr int CH = 64;              // queries (forward) / keys (backward) per chunk
constexpr int NT = CH / 16;         // 16-row tiles per chunk
constexpr float INV_SCALE = 0.25f;  // 1/sqrt(16), exact
constexpr int TLD2 = CH + 8;        // LDS row stride (bf16) of the backward's split dS transpose
constexpr int TFL = 2 * 16 * TLD2 / 2;   // floats of one wave's transpose region (hi + lo parts)
constexpr int RED = 2 * WAVES * CH * HD;   // floats of the backward's dK / dV partial buffer

MEP_DEV floatx4 zero4() { return floatx4{0.f, 0.f, 0.f, 0.f}; }

// ------------------------------------------------------------------ bf16 operand splitting
// two fp32 -> one word of two round-to-nearest bf16 (v_cvt_pk_bf16_f32)
MEP_DEV unsigned pk(float a, float b) { return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, bf16x2)); }
MEP_DEV float bf_lo(unsigned p) { return __builtin_bit_cast(float, p << 16); }
MEP_DEV float bf_hi(unsigned p) { return __builtin_bit_cast(float, p & 0xffff0000u); }

// 4 fp32 -> parts as bf16 words: h = x0 (2 words), l = x1 (2-way split)
struct S2 { unsigned h0, h1, l0, l1; };
// 4 fp32 -> parts a = x0, b = x1, c = x2 (3-way split)
struct S3 { unsigned a0, a1, b0, b1, c0, c1; };

MEP_DEV S2 split2(float x0, float x1, float x2, float x3) {
    S2 s;
    s.h0 = pk(x0, x1);
    s.h1 = pk(x2, x3);
    s.l0 = pk(x0 - bf_lo(s.h0), x1 - bf_hi(s.h0));   // exact remainders (Sterbenz)
    s.l1 = pk(x2 - bf_lo(s.h1), x3 - bf_hi(s.h1));
    return s;
}
MEP_DEV S2 split2(const float* x) { return split2(x[0], x[1], x[2], x[3]); }
MEP_DEV S3 split3(const float* x) {
    S3 s;
    s.a0 = pk(x[0], x[1]);
    s.a1 = pk(x[2], x[3]);
    const float r0 = x[0] - bf_lo(s.a0), r1 = x[1] - bf_hi(s.a0);
    const float r2 = x[2] - bf_lo(s.a1), r3 = x[3] - bf_hi(s.a1);
    s.b0 = pk(r0, r1);
    s.b1 = pk(r2, r3);
    s.c0 = pk(r0 - bf_lo(s.b0), r1 - bf_hi(s.b0));
    s.c1 = pk(r2 - bf_lo(s.b1), r3 - bf_hi(s.b1));
    return s;
}

// hi parts of two 4-vectors as one operand quad {x0 x1 | x2 x3 | y0 y1 | y2 y3}, and the lo parts
MEP_DEV u32x4 split_hi(const float* x, const float* y) {
    return u32x4{pk(x[0], x[1]), pk(x[2], x[3]), pk(y[0], y[1]), pk(y[2], y[3])};
}
MEP_DEV u32x4 split_lo(const float* x, const float* y, const u32x4& h) {
    return u32x4{pk(x[0] - bf_lo(h[0]), x[1] - bf_hi(h[0])), pk(x[2] - bf_lo(h[1]), x[3] - bf_hi(h[1])),
                 pk(y[0] - bf_lo(h[2]), y[1] - bf_hi(h[2])), pk(y[2] - bf_lo(h[3]), y[3] - bf_hi(h[3]))};
}
MEP_DEV bf16x8 op(unsigned w0, unsigned w1, unsigned w2, unsigned w3) {
    return __builtin_bit_cast(bf16x8, u32x4{w0, w1, w2, w3});
}
MEP_DEV floatx4 mfma(bf16x8 a, bf16x8 b, floatx4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
// bf16 path: a 16-deep contraction (4 bf16 per lane, k = 4g .. 4g+3) on v_mfma_f32_16x16x16_bf16
typedef short s16x4 __attribute__((ext_vector_type(4)));
MEP_DEV s16x4 op4(unsigned w0, unsigned w1) { return __builtin_bit_cast(s16x4, u32x2{w0, w1}); }
MEP_DEV floatx4 mfma16(s16x4 a, s16x4 b, floatx4 c) { return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0); }

// Score product over the 16 head dims, 3-way split: P = the "packed" operand, U = the
// "duplicated" one; slots (g, j < 4) and (g, j >= 4) carry
//   MFMA 1: p0 u0 | p1 u0     MFMA 2: p0 u1 | p1 u1     MFMA 3: p0 u2 | p2 u0
// P_IS_A selects which MFMA operand P is (forward: K = A; backward: K = B), the products and
// slots are the same either way.  BF (bf16 path): the one product p0 u0.
template <bool P_IS_A, bool BF>
MEP_DEV floatx4 dot_score(const S3& p, const S3& u, floatx4 acc) {
    if (BF) return P_IS_A ? mfma16(op4(p.a0, p.a1), op4(u.a0, u.a1), acc) : mfma16(op4(u.a0, u.a1), op4(p.a0, p.a1), acc);
    const bf16x8 p01 = op(p.a0, p.a1, p.b0, p.b1), p02 = op(p.a0, p.a1, p.c0, p.c1);
    const bf16x8 u00 = op(u.a0, u.a1, u.a0, u.a1), u11 = op(u.b0, u.b1, u.b0, u.b1), u20 = op(u.c0, u.c1, u.a0, u.a1);
    if (P_IS_A) {
        acc = mfma(p01, u00, acc);
        acc = mfma(p01, u11, acc);
        acc = mfma(p02, u20, acc);
    } else {
        acc = mfma(u00, p01, acc);
        acc = mfma(u11, p01, acc);
        acc = mfma(u20, p02, acc);
    }
    return acc;
}

// 16-deep contraction, 2-way split, all four products.  MEP_BWD_MF16: four v_mfma_f32_16x16x16_bf16
// on the parts as they come out of the split (each a register pair: no operand assembly moves);
// else two 16x16x32 with A = [x0 | x1], B = [y0 | y0] then [y1 | y1].  (BF: x0 y0.)
template <bool BF>
MEP_DEV floatx4 dot16(const S2& x, const S2& y, floatx4 acc) {
    if (BF) return mfma16(op4(x.h0, x.h1), op4(y.h0, y.h1), acc);
    acc = mfma16(op4(x.h0, x.h1), op4(y.h0, y.h1), acc);
    acc = mfma16(op4(x.l0, x.l1), op4(y.h0, y.h1), acc);
    acc = mfma16(op4(x.h0, x.h1), op4(y.l0, y.l1), acc);
    acc = mfma16(op4(x.l0, x.l1), op4(y.l0, y.l1), acc);
    return acc;
}

// 32-deep contraction over two 16-row tiles (slots 0-3: tile 0, 4-7: tile 1), 2-way split,
// products x0 y0 + x1 y0 + x0 y1 (BF: x0 y0); MEP_BWD_MF16: per tile on 16x16x16
template <bool BF>
MEP_DEV floatx4 dot32(const S2& xa, const S2& xb, const S2& ya, const S2& yb, floatx4 acc) {
    const bf16x8 x0 = op(xa.h0, xa.h1, xb.h0, xb.h1), y0 = op(ya.h0, ya.h1, yb.h0, yb.h1);
    acc = mfma(x0, y0, acc);
    if (BF) return acc;
    acc = mfma(op(xa.l0, xa.l1, xb.l0, xb.l1), y0, acc);
    acc = mfma(x0, op(ya.l0, ya.l1, yb.l0, yb.l1), acc);
    return acc;
}

// per-key mask term of the score: 1e8 * (1 - mask) (cmu-mosei/run.py:253), +inf for padding keys
// beyond Tk so that s - term = -inf and exp() = 0 without any per-score select
MEP_DEV float mask_term(const gfloat* mask, int k, int Tk) {
    const float m = mask[min(k, Tk - 1)];
    return k < Tk ? mul_rn(1.0e8f, sub_rn(1.0f, m)) : INFINITY;
}

MEP_DEV float shfl(float v, int src) { return __shfl(v, src, 64); }

// max / sum over the four lanes l, l ^ 16, l ^ 32, l ^ 48 (a query's lane groups g), in the order
// x op shfl(x, l ^ 16), then op shfl(., l ^ 32)
MEP_DEV float xg_max(float x) {
    x = fmaxf(x, shfl(x, (int)(threadIdx.x & 63) ^ 16));
    return fmaxf(x, shfl(x, (int)(threadIdx.x & 63) ^ 32));
}
MEP_DEV float xg_sum(float x) {
    x = x + shfl(x, (int)(threadIdx.x & 63) ^ 16);
    return x + shfl(x, (int)(threadIdx.x & 63) ^ 32);
}

// s = dot / sqrt(hd) [+ c*sp] - 1e8 * (1 - m)      (op order of cmu-mosei/run.py:244-253); hd = 16:
// the exact * 0.25; hd = 32 (robot_demo.py:356): a correctly rounded division by float(sqrt(32)),
// as torch divides by the Python scalar
template <bool PREV, int HDIM = HD>
MEP_DEV float score(float dot, float c, float sp, float mt) {
    float s = HDIM == 16 ? mul_rn(dot, INV_SCALE) : __fdiv_rn(dot, 5.65685424949238f);
    if (PREV) s = add_rn(s, mul_rn(c, sp));
    return sub_rn(s, mt);
}

MEP_DEV bool aligned16(const mep_rows& r) {
    return ((r.ptr & 15) == 0) && (r.sB % 4 == 0) && (r.sT % 4 == 0);
}

// One batch row of a row view as a range-checked buffer (csrc/common.h raw buffer ops): row t,
// column col at byte t * sT + ES col (ES = 4, or 2 for the bf16 path's bf16 rows, HS).  Rows
// t >= n lie past the range (every view has sT >= its D used columns), so their loads return 0
// and their stores are dropped -- no clamps, no branches, 32-bit offsets.  The base is
// wave-uniform by construction (one (b, h) per wave or workgroup); readfirstlane makes that
// provable so the descriptor lives in SGPRs.  Values are fp32 in registers either way (bf16 ->
// fp32 exact; fp32 -> bf16 round to nearest even on stores).
template <bool HS>
struct BRowT {
    static constexpr int ES = HS ? 2 : 4;
    __amdgpu_buffer_rsrc_t rs;
    int sT4;   // row stride in bytes (wave-uniform)
    bool vec;  // 4-element loads as one access (16 bytes fp32, 8 bytes bf16)
    // byte offset of (row t, column col); loads / stores take a per-lane part plus a wave-uniform
    // part (SGPR soffset: whole rows ahead), so row steps cost no vector instructions
    MEP_DEV int at(int t, int col) const { return t * sT4 + ES * col; }
    MEP_DEV float ld1(int voff, int soff = 0) const {
        if (HS) return __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_raw_buffer_load_b16(rs, voff, soff, 0) << 16);
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0));
    }
    MEP_DEV void ld4(float* dst, int voff) const {
        if (HS && vec) {
            const u32x2 w = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, 0, 0));
            dst[0] = bf_lo(w[0]); dst[1] = bf_hi(w[0]); dst[2] = bf_lo(w[1]); dst[3] = bf_hi(w[1]);
        } else if (vec) {
            const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0));
            dst[0] = v[0]; dst[1] = v[1]; dst[2] = v[2]; dst[3] = v[3];
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) dst[e] = ld1(voff + ES * e);
        }
    }
    // HS only: 4 bf16 elements as the two operand words {e0 | e1 << 16, e2 | e3 << 16} (no fp32
    // round trip), and one element as a zero-extended word
    MEP_DEV u32x2 ld4raw(int voff) const {
        if (vec) return __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, 0, 0));
        unsigned e[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) e[i] = ld1raw(voff + 2 * i);
        return u32x2{e[0] | (e[1] << 16), e[2] | (e[3] << 16)};
    }
    MEP_DEV unsigned ld1raw(int voff, int soff = 0) const {
        return (unsigned)__builtin_amdgcn_raw_buffer_load_b16(rs, voff, soff, 0);
    }
    MEP_DEV void st1(int voff, int soff, float v) const {
        if (HS) __builtin_amdgcn_raw_buffer_store_b16((unsigned short)pk(v, 0.f), rs, voff, soff, 0);
        else __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rs, voff, soff, 0);
    }
    MEP_DEV void st4(int voff, f32x4 v) const {
        if (HS && vec) {
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, u32x2{pk(v[0], v[1]), pk(v[2], v[3])}), rs, voff, 0, 0);
        } else if (vec) {
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, voff, 0, 0);
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) st1(voff + ES * e, 0, v[e]);
        }
    }
};
typedef BRowT<false> BRow;

MEP_DEV __amdgpu_buffer_rsrc_t uniform_rsrc(uint64_t base, int64_t bytes) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)base);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(base >> 32));
    const int n = __builtin_amdgcn_readfirstlane((int)min(bytes, (int64_t)0x7fffffff));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}

// rows [0, n) of batch row b of a view whose used columns are [0, D) (HS: bf16 elements)
template <bool HS = false>
MEP_DEV BRowT<HS> brow(const mep_rows& v, int b, int n, int D) {
    constexpr int ES = HS ? 2 : 4;
    const bool vec = HS ? (((v.ptr & 7) == 0) && (v.sB % 4 == 0) && (v.sT % 4 == 0)) : aligned16(v);
    return BRowT<HS>{uniform_rsrc(v.ptr + (uint64_t)ES * (uint64_t)((int64_t)b * v.sB), (int64_t)ES * ((int64_t)(n - 1) * v.sT + D)),
                     ES * (int)v.sT, vec};
}

// ================================================================== forward
#ifndef MEP_FWD_SOUT2
#define MEP_FWD_SOUT2 1   // single-chunk forward: score rows out / S_prev in as 8-byte pairs (Tk even)
#endif
// One forward task: batch row b, head h, 64 queries.  PREV: residual scores in; SOUT: post-mask
// scores out; SINGLE: Tk <= 64 (one key chunk: exact two-pass softmax, each query tile is
// finalised right after its P.V, so no running O/max/sum state stays live).  BF: the bf16 path
// (scores on one bf16 product, P.V on bf16 P and V).  HDIM = 16 or 32 (robot_demo, inference):
// NHB = HDIM / 16 head blocks of 16 dims -- the score sums NHB 16-deep products, P.V fills NHB
// output tiles.
template <bool PREV, bool SOUT, bool SINGLE, bool BF, int HDIM = HD, int qch = CH>
MEP_DEV void attn_fwd_task(const mep_attn_desc& d, int qc, int h, int b, int lane) {
    constexpr int NHB = HDIM / 16;
    const int c = lane & 15, g = lane >> 4;
    const int hc = h * HDIM;
    const int Tq = d.Tq, Tk = d.Tk;
    const float cres = PREV ? *G<const float>(d.c) : 0.f;
    const gfloat* sprev = G<const float>(d.s_prev);
    gfloat* sout = G<float>(d.s_out);
    // SOUT with Tk even and an 8-byte aligned score tensor: every row starts 8-byte aligned, so the
    // lane's 4 keys go out as two 8-byte stores (not four scattered 4-byte ones)
    const bool sout2 = MEP_FWD_SOUT2 && SOUT && (Tk % 2 == 0) && ((d.s_out & 7) == 0);
    // PREV likewise: the lane's 4 S_prev values of a key tile as two 8-byte loads (keys past Tk read
    // the row's last pair, finite; their scores are -inf either way)
    const bool sprev2 = MEP_FWD_SOUT2 && PREV && (Tk % 2 == 0) && ((d.s_prev & 7) == 0);
    const gfloat* mask = G<const float>(d.mask) + (int64_t)b * d.mask_sB;
    const uint64_t mrow = d.mask + 4ull * (uint64_t)((int64_t)b * d.mask_sB);
    const auto rsMask = uniform_rsrc(mrow, 4 * (int64_t)Tk);
    const bool mask16 = (mrow & 15) == 0;   // wave-uniform
    (void)mask;
    const int D = d.H * HDIM;
    const BRowT<BF> Qb = brow<BF>(d.q, b, Tq, D), Kb = brow<BF>(d.k, b, Tk, D), Vb = brow<BF>(d.v, b, Tk, D),
                    Xb = brow<BF>(d.x, b, Tq, D);
    const int sbase = (b * d.H + h) * Tq;        // row of (b, h, query 0) in [B,H,Tq,Tk]
    const int q_lo = qc * qch;                   // qch: queries per task (64, or 16 with MEP_ATTN_SPLITQ)
    const int nqt = min(qch / 16, (Tq - q_lo + 15) / 16);
    gfloat* stats = G<float>(d.stats);
    const int stat_rows = d.B * d.H * Tq;        // PREV: the tail of stats holds one float per row

    floatx4 o[SINGLE ? 1 : NT][NHB];
    float m[SINGLE ? 1 : NT], l[SINGLE ? 1 : NT];
    if (!SINGLE) {
#pragma unroll
        for (int qt = 0; qt < NT; ++qt) {
#pragma unroll
            for (int hb = 0; hb < NHB; ++hb) o[qt][hb] = zero4();
            m[qt] = -FLT_MAX;
            l[qt] = 0.f;
        }
    }
    // O^T = V^T P^T: the accumulator lane (c, g) holds query c, dims 4g .. 4g+3 of each head
    // block, so the row's 1/sum is the lane's own and a row's 4 dims are one 16-byte (8-byte bf16)
    // store.  BF: 1/sum as v_rcp_f32 (fp32: the IEEE division)
    // lq: BF -- the row's full sum already (from the ones-row MFMA); fp32 -- this lane's keys
    auto finish = [&](int qt, const floatx4 (&oq)[NHB], float mq, float lq) {
        const float lt = BF ? lq : xg_sum(lq);
        const float inv = BF ? __builtin_amdgcn_rcpf(lt) : 1.0f / lt;
        const int q = q_lo + qt * 16 + c;
        if (g == 0 && q < Tq) {
            // row statistics for the backward: (max log2 e - log2(1/sum), 1/sum) -- the exp2
            // backward's per-row exponent offset, formed once here instead of per backward tile and
            // key-chunk wave.  PREV: (max, 1/sum) -- the backward forms exp(s - max) with s - max
            // exact (F7, Bwd::tile); the stats' tail (S_prev at the row maximum) is written by the
            // key-chunk loop
            stats[2 * (sbase + q)] = !PREV ? mq * 1.4426950408889634f - __builtin_amdgcn_logf(inv) : mq;
            stats[2 * (sbase + q) + 1] = inv;
        }
#pragma unroll
        for (int hb = 0; hb < NHB; ++hb)   // rows past Tq: dropped by the range check
            Xb.st4(Xb.at(q, hc + 16 * hb + 4 * g), f32x4{oq[hb][0] * inv, oq[hb][1] * inv, oq[hb][2] * inv, oq[hb][3] * inv});
    };
    // 4 consecutive row elements (columns 4g ..) as a score operand: the fp32 path's 3-part
    // split, the bf16 path's raw words (no fp32 round trip)
    auto ld_op = [&](const BRowT<BF>& R, int off) -> S3 {
        if constexpr (BF) {
            const u32x2 w = R.ld4raw(off);
            S3 r{};
            r.a0 = w[0];
            r.a1 = w[1];
            return r;
        } else {
            float f[4];
            R.ld4(f, off);
            return split3(f);
        }
    };

    // MI (no residual scores, hd 16): the key's mask term enters as the score accumulator's
    // initial value (-4 mask: the dot is scaled by 1/4 later), the max runs on the raw dot and the
    // 1/4 folds into the exponent's fma -- per score one max, one fma and the exp2 instead of a
    // scale, a mask subtraction, the max, the fma and the exp2.  Kept keys (mask 0) give the same
    // bits: 1/4 is a power of two, so scaling commutes with every rounding on the way
    constexpr bool MI = !PREV && !SOUT && HDIM == 16;
    constexpr bool QH = !SINGLE;
    S3 qsh[QH ? NT : 1][NHB];                  // QH: B of S^T for every query tile of the task
    if (QH) {
#pragma unroll
        for (int qt = 0; qt < NT; ++qt)
#pragma unroll
            for (int hb = 0; hb < NHB; ++hb) {
                S3 z{};
                if (qch == CH || qt < nqt) z = ld_op(Qb, Qb.at(q_lo + qt * 16 + c, hc + 16 * hb + 4 * g));   // past Tq: 0
                qsh[QH ? qt : 0][hb] = z;
            }
    }
    // the raw loads of one key chunk (K rows, V columns, the keys' mask values)
    struct Raw {
        u32x2 kw[NT][NHB];        // BF: K rows as words
        float kf[BF ? 1 : NT][NHB][4];
        unsigned vr[BF ? NT : 1][NHB][4];
        float vf[BF ? 1 : NT][NHB][4];
        f32x4 m4[NT];
    };
    auto fetch = [&](Raw& R, int k_lo) {
#pragma unroll
        for (int kt = 0; kt < NT; ++kt) {
            const int k0 = k_lo + kt * 16;
#pragma unroll
            for (int hb = 0; hb < NHB; ++hb) {
                const int ov = Vb.at(k0 + 4 * g, hc + 16 * hb + c);
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    if constexpr (BF) R.vr[kt][hb][s] = Vb.ld1raw(ov, s * Vb.sT4);
                    else R.vf[BF ? 0 : kt][hb][s] = Vb.ld1(ov, s * Vb.sT4);
                }
                if constexpr (BF) R.kw[kt][hb] = Kb.ld4raw(Kb.at(k0 + c, hc + 16 * hb + 4 * g));
                else Kb.ld4(R.kf[BF ? 0 : kt][hb], Kb.at(k0 + c, hc + 16 * hb + 4 * g));
            }
            // the lane's 4 keys' mask values in one 16-byte load (range-checked: past Tk -> 0, and
            // those keys get +inf below)
            if (mask16) {
                R.m4[kt] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsMask, 4 * (k0 + 4 * g), 0, 0));
            } else {   // a row that is not 16-byte aligned: 4 dword loads
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    R.m4[kt][s] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsMask, 4 * (k0 + 4 * g + s), 0, 0));
            }
        }
    };
    for (int k_lo = 0; k_lo < Tk; k_lo += CH) {
        // operands of the 4 key tiles of this chunk: K rows (A of S^T: K[k0+c][4g+s], split) and V
        // columns (B of P.V: V[k0+4g+s][c]); past Tk they read 0 (P is 0 there)
        Raw cur;
        fetch(cur, k_lo);
        S3 ks[NT][NHB];
        float vf[BF ? 1 : NT][NHB][4], mt[NT][4];
        unsigned vr[BF ? NT : 1][NHB][4];   // BF: raw bf16 V elements
        bf16x8 vbf[NT / 2][NHB];     // BF: V of key-tile pairs (kt, kt+1) in slots 0-3 / 4-7
#pragma unroll
        for (int kt = 0; kt < NT; ++kt) {
            const int k0 = k_lo + kt * 16;
#pragma unroll
            for (int hb = 0; hb < NHB; ++hb) {
                if constexpr (BF) {
                    S3 r{};
                    r.a0 = cur.kw[kt][hb][0];
                    r.a1 = cur.kw[kt][hb][1];
                    ks[kt][hb] = r;
#pragma unroll
                    for (int s = 0; s < 4; ++s) vr[kt][hb][s] = cur.vr[kt][hb][s];
                } else {
                    ks[kt][hb] = split3(cur.kf[BF ? 0 : kt][hb]);
#pragma unroll
                    for (int s = 0; s < 4; ++s) vf[BF ? 0 : kt][hb][s] = cur.vf[BF ? 0 : kt][hb][s];
                }
            }
#pragma unroll
            for (int s = 0; s < 4; ++s)
                mt[kt][s] = k0 + 4 * g + s < Tk ? mul_rn(1.0e8f, sub_rn(1.0f, cur.m4[kt][s])) : INFINITY;
        }
        if constexpr (BF) {
#pragma unroll
            for (int kt = 0; kt < NT; kt += 2)
#pragma unroll
                for (int hb = 0; hb < NHB; ++hb)
                    vbf[kt / 2][hb] = op(vr[kt][hb][0] | (vr[kt][hb][1] << 16), vr[kt][hb][2] | (vr[kt][hb][3] << 16),
                                         vr[kt + 1][hb][0] | (vr[kt + 1][hb][1] << 16),
                                         vr[kt + 1][hb][2] | (vr[kt + 1][hb][3] << 16));
        }
        // V of key-tile pairs split once per chunk (not per query tile): parts [pair][hb][part]
        bf16x8 vsp[NT / 2][NHB][3];
        if constexpr (!BF) {
#pragma unroll
            for (int kt = 0; kt < NT; kt += 2)
#pragma unroll
                for (int hb = 0; hb < NHB; ++hb) {
                    const S3 va = split3(vf[kt][hb]), vb = split3(vf[kt + 1][hb]);
                    vsp[kt / 2][hb][2] = op(va.c0, va.c1, vb.c0, vb.c1);
                    vsp[kt / 2][hb][0] = op(va.a0, va.a1, vb.a0, vb.a1);
                    vsp[kt / 2][hb][1] = op(va.b0, va.b1, vb.b0, vb.b1);
                }
        }
        float qfa[QH || BF ? 1 : NT][NHB][4];                              // B of S^T: Q[q][4g+s]
        S3 qbf[!QH && BF ? NT : 1][NHB];                                   // BF: raw Q words
        if (!QH) {
#pragma unroll
            for (int qt = 0; qt < NT; ++qt)
#pragma unroll
                for (int hb = 0; hb < NHB; ++hb) {
                    const bool in = qch == CH || qt < nqt;                 // past Tq: 0
                    if constexpr (BF) {
                        S3 z{};
                        if (in) z = ld_op(Qb, Qb.at(q_lo + qt * 16 + c, hc + 16 * hb + 4 * g));
                        qbf[!QH && BF ? qt : 0][hb] = z;
                    } else {
                        float* qf = qfa[QH ? 0 : qt][hb];
                        if (in) Qb.ld4(qf, Qb.at(q_lo + qt * 16 + c, hc + 16 * hb + 4 * g));
                        else qf[0] = qf[1] = qf[2] = qf[3] = 0.f;
                    }
                }
        }
#pragma unroll
        for (int qt = 0; qt < NT; ++qt) {
            if (qt >= nqt) break;
            const int q = q_lo + qt * 16 + c;
            S3 qs[NHB];
#pragma unroll
            for (int hb = 0; hb < NHB; ++hb)
                qs[hb] = QH ? qsh[QH ? qt : 0][hb] : BF ? qbf[!QH && BF ? qt : 0][hb] : split3(qfa[QH || BF ? 0 : qt][hb]);
            const int srow = (sbase + min(q, Tq - 1)) * Tk;
            float sv[NT][4];
            float mx = -INFINITY, spm = 0.f;   // PREV: S_prev at the lane's largest score
#pragma unroll
            for (int kt = 0; kt < NT; ++kt) {
                floatx4 st = MI ? floatx4{-4.f * mt[kt][0], -4.f * mt[kt][1], -4.f * mt[kt][2], -4.f * mt[kt][3]}
                                : zero4();                                 // C[key 4g+r][query c]
#pragma unroll
                for (int hb = 0; hb < NHB; ++hb) st = dot_score<true, BF>(ks[kt][hb], qs[hb], st);
                f32x2 spa = f32x2{0.f, 0.f}, spb = spa;
                if (PREV && sprev2) {
                    const int k2 = k_lo + kt * 16 + 4 * g;
                    spa = *reinterpret_cast<const MEP_G f32x2*>(sprev + srow + min(k2, Tk - 2));
                    spb = *reinterpret_cast<const MEP_G f32x2*>(sprev + srow + min(k2 + 2, Tk - 2));
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float spv = 0.f;
                    const int kk = k_lo + kt * 16 + 4 * g + r;
                    if (PREV || SOUT) {
                        const int si = srow + min(kk, Tk - 1);
                        if (PREV) spv = sprev2 ? (r < 2 ? spa[r] : spb[r - 2]) : sprev[si];
                        const float v = score<PREV, HDIM>(st[r], cres, spv, mt[kt][r]);
                        if (PREV) spm = v > mx ? spv : spm;   // mx below: the running max before v
                        if (SOUT && !sout2 && kk < Tk && q < Tq) sout[si] = v;
                        sv[kt][r] = v;
                    } else if (MI) {
                        sv[kt][r] = st[r];                                 // 4 x the score (dot - 4 mask)
                    } else {
                        sv[kt][r] = score<false, HDIM>(st[r], 0.f, 0.f, mt[kt][r]);
                    }
                    mx = fmaxf(mx, sv[kt][r]);
                }
                if (SOUT && sout2) {   // keys 4g .. 4g + 3 of the row as two 8-byte stores (Tk even: a pair is whole or past Tk)
                    const int k2 = k_lo + kt * 16 + 4 * g;
                    if (q < Tq) {
                        if (k2 < Tk) *reinterpret_cast<MEP_G f32x2*>(sout + srow + k2) = f32x2{sv[kt][0], sv[kt][1]};
                        if (k2 + 2 < Tk) *reinterpret_cast<MEP_G f32x2*>(sout + srow + k2 + 2) = f32x2{sv[kt][2], sv[kt][3]};
                    }
                }
            }
            if (PREV) {
                // the stats' tail: S_prev at the row's maximum score (of tied lanes the largest:
                // deterministic), the shift of the backward's dc sum (Bwd::tile); a later key chunk
                // with a larger maximum overwrites it (no register state across chunks)
                const float ml = mx;
                mx = xg_max(mx);
                const float spr = xg_max(ml == mx ? spm : -INFINITY);
                if (g == 0 && q < Tq && (SINGLE || k_lo == 0 || mx > m[SINGLE ? 0 : qt]))
                    stats[2 * stat_rows + sbase + q] = spr;
            } else {
                mx = xg_max(mx);
            }
            const float mnew = SINGLE ? mx : fmaxf(m[qt], mx);
            float lsum = 0.f;
            constexpr float L2E = 1.4426950408889634f;
            constexpr float SL2E = MI ? INV_SCALE * L2E : L2E;            // MI: raw dots
            const float mb = mnew * SL2E;
#pragma unroll
            for (int kt = 0; kt < NT; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    sv[kt][r] = !PREV ? __builtin_amdgcn_exp2f(fmaf(sv[kt][r], SL2E, -mb))
                                                              : __expf(sv[kt][r] - mnew);
                    if (!BF) lsum += sv[kt][r];
                }
            floatx4 oq[NHB];
#pragma unroll
            for (int hb = 0; hb < NHB; ++hb) oq[hb] = SINGLE ? zero4() : o[qt][hb];
            if (!SINGLE && k_lo > 0) {   // rescale the running state (O^T: the lane's own query c)
                const float corr = __expf(MI ? (m[qt] - mnew) * INV_SCALE : m[qt] - mnew);
                l[qt] *= corr;
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int hb = 0; hb < NHB; ++hb) oq[hb][r] *= corr;
            }
            // O^T += V^T P^T over the chunk's 64 keys: key-tile pairs (slots 0-3 / 4-7); V^T is the
            // A operand (row: dim c), P^T the B operand (column: query c).  BF: the row sums of the
            // bf16 P too, as a ones-row A operand against the same P^T (every accumulator row is
            // the query's sum over the chunk's keys: no VALU add per score, no lane reduction)
            floatx4 lacc = zero4();
#pragma unroll
            for (int kt = 0; kt < NT; kt += 2) {
                if (BF) {   // bf16 P (slots: keys 4g+s of tiles kt / kt+1) against bf16 V
                    const bf16x8 pb = op(pk(sv[kt][0], sv[kt][1]), pk(sv[kt][2], sv[kt][3]), pk(sv[kt + 1][0], sv[kt + 1][1]),
                                         pk(sv[kt + 1][2], sv[kt + 1][3]));
#pragma unroll
                    for (int hb = 0; hb < NHB; ++hb) oq[hb] = mfma(vbf[kt / 2][hb], pb, oq[hb]);
                    lacc = mfma(op(0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u), pb, lacc);
                    continue;
                }
                // P and V as 3-part bf16 splits, the six products p_i v_j with i + j <= 2 (the terms
                // dropped are <= 2^-24 relative: fp32-level) on 16x16x32 MFMAs per key-tile pair
                // (slots 0-3: tile kt, 4-7: tile kt + 1); the three smallest on a chain of their own
                {
                    const S3 pa = split3(sv[kt]), pb = split3(sv[kt + 1]);
                    const bf16x8 p0 = op(pa.a0, pa.a1, pb.a0, pb.a1), p1 = op(pa.b0, pa.b1, pb.b0, pb.b1),
                                 p2 = op(pa.c0, pa.c1, pb.c0, pb.c1);
#pragma unroll
                    for (int hb = 0; hb < NHB; ++hb) {
                        const bf16x8 v0 = vsp[kt / 2][hb][0], v1 = vsp[kt / 2][hb][1];
                        floatx4 t = mfma(v0, p2, zero4());          // two independent chains
                        oq[hb] = mfma(v0, p1, oq[hb]);
                        t = mfma(v1, p1, t);
                        oq[hb] = mfma(v1, p0, oq[hb]);
                        t = mfma(vsp[kt / 2][hb][2], p0, t);
                        oq[hb] = mfma(v0, p0, oq[hb]);
#pragma unroll
                        for (int r = 0; r < 4; ++r) oq[hb][r] += t[r];
                    }
                }
            }
            if (BF) lsum = lacc[0];
            if (SINGLE) {
                finish(qt, oq, MI ? mnew * INV_SCALE : mnew, lsum);
            } else {
#pragma unroll
                for (int hb = 0; hb < NHB; ++hb) o[qt][hb] = oq[hb];
                l[qt] += lsum;
                m[qt] = mnew;
            }
        }
    }
    if (!SINGLE) {
#pragma unroll
        for (int qt = 0; qt < NT; ++qt) {
            if (qt >= nqt) break;
            finish(qt, o[qt], MI ? m[qt] * INV_SCALE : m[qt], l[qt]);
        }
    }
}

template <bool PREV, bool SOUT, bool SINGLE, bool BF, int HDIM = HD, int QCH = CH>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu((SINGLE && !PREV && HDIM == 16) ? MEP_FWD_WAVES : (HDIM == 32 && !SINGLE) ? 1 : !SINGLE ? (BF ? MEP_FWD_LONG_WAVES_BF : PREV ? 1 : MEP_FWD_LONG_WAVES) : 2))) void k_attn_fwd(const mep_attn_desc* __restrict__ descs) {
    const mep_attn_desc& d = descs[blockIdx.y];
    if ((d.Tk <= CH) != SINGLE) return;    // the other variant's descriptor
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nqc = (d.Tq + QCH - 1) / QCH;   // QCH: queries per wave task (64, or 16 with MEP_ATTN_SPLITQ)
    const int task = blockIdx.x * WAVES + wave;
    if (task >= d.B * d.H * nqc) return;   // whole wave leaves; no barriers below
    if (!SINGLE && !(d.H & 3)) {
        // Tk > 64, H % 4 == 0: the workgroup's 4 waves take the same queries of heads 4j .. 4j + 3
        // of one row -- the 128-byte line of a bf16 K / V / Q row that each reads a quarter of is
        // fetched once for all four, into the CU they share
        const int m = task & 3, r = task >> 2;
        const int qc = r % nqc, bhq = r / nqc, hq = d.H >> 2;
        attn_fwd_task<PREV, SOUT, SINGLE, BF, HDIM, QCH>(d, qc, 4 * (bhq % hq) + m, bhq / hq, lane);
        return;
    }
    if (!SINGLE && !(d.H & 1)) {
        // Tk > 64: waves 2i and 2i + 1 of a workgroup take the same queries of heads 2j and 2j + 1
        // of one row, so the 128-byte line of K / V / Q rows each needs half of is fetched once
        // for both, into the CU they share (head_pair_order below has the backward's reason)
        const int m = task & 1, r = task >> 1;
        const int qc = r % nqc, bhp = r / nqc, hp = d.H >> 1;
        attn_fwd_task<PREV, SOUT, SINGLE, BF, HDIM, QCH>(d, qc, 2 * (bhp % hp) + m, bhp / hp, lane);
        return;
    }
    const int qc = task % nqc, bh = task / nqc;
    attn_fwd_task<PREV, SOUT, SINGLE, BF, HDIM, QCH>(d, qc, bh % d.H, bh / d.H, lane);
}

MEP_DEV void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ================================================================== backward
// State of one (descriptor, b, h) backward unit: views, the operands of the current 64-key chunk
// (B of S = K rows with the key on the lane, B of dP = V rows, B of dQ = K columns rows 4g+s /
// dim c, the keys' mask terms) and the chunk's dK / dV accumulators (C[key 4g+r][dim c]).
// PREV: residual scores (writes dS_prev, sums the dc partial); DSN: a gradient arrives on this
// layer's post-mask S output; BF: the bf16 path (one bf16 product per contraction); KV: k is v
// and dk is dv (MEP_ATTN_KV: one register set for the K / V rows and ONE accumulator per key tile
// for dK + dV, with Q pre-scaled by the exact 1/sqrt(hd) = 1/4 -- about 32 registers fewer).
#ifndef MEP_BWD_SSTAGE
#define MEP_BWD_SSTAGE 3   // short backward, LDS-DMA path: bit 0 stages S_prev (rfstate layer-1 launch 433 -> ~345 us), bit 1 dS_next (with the DSN kernel at 2 waves per SIMD: at 3 its addressing spilled 22 registers and ran slower; 2 waves: ~10 us faster than unstaged)
#endif
constexpr bool SST_P = MEP_BWD_SSTAGE & 1, SST_D = (MEP_BWD_SSTAGE >> 1) & 1;
template <bool PREV, bool DSN, bool BF, bool KV = false>
struct Bwd {
    // per query tile: A of S (Q rows), A of dP (dO rows), B of dV / dK (dO / Q columns), O
    // columns for delta, row stats and the dq rows this tile accumulates onto
    struct QIn {
        float qa[4], da[4], db[4], qb[4], ob[4], dqo[4];
        f32x2 st[4];
        float rp[4];      // PREV: the rows' P-weighted mean of S_prev (the forward's stats tail)
        u32x2 qaw, daw;   // BF: Q / dO rows as raw bf16 operand words (no fp32 round trip)
        u32x2 oaw;        // BF: O row (delta on the matrix core)
    };
    const mep_attn_bwd_desc& bd;
    int b, h, lane, c, g, hc, Tq, Tk, sbase;
    float cres;
    const gfloat *sprev, *dsn, *mask;
    gfloat* dsp;
    BRowT<BF> Qb, Kb, Vb, Ob, Gb, dQb;   // BF: bf16 rows
    __amdgpu_buffer_rsrc_t rsStat, rsRp, rsSp, rsDn;
    bool same_kv;
    int k_lo;
    S2 kb[NT], vb[NT], kq[NT];
    float mtk[NT], mtl[NT];   // mask term, and the same times log2(e)
    float mts[BF ? NT : 1];   // BF: -4 x the mask term, the score accumulator's initial value (EXP2)
    floatx4 dk[NT], dv[NT];
    float dc_acc;

    MEP_DEV Bwd(const mep_attn_bwd_desc& bd_, int b_, int h_, int lane_) : bd(bd_), b(b_), h(h_), lane(lane_) {
        const mep_attn_desc& d = bd.f;
        c = lane & 15;
        g = lane >> 4;
        hc = h * HD;
        Tq = d.Tq;
        Tk = d.Tk;
        const int D = d.H * HD;
        cres = PREV ? *G<const float>(d.c) : 0.f;
        sprev = G<const float>(d.s_prev);
        dsn = G<const float>(bd.ds_next);
        dsp = G<float>(bd.ds_prev);
        mask = G<const float>(d.mask) + (int64_t)b * d.mask_sB;
        Qb = brow<BF>(d.q, b, Tq, D);
        Kb = brow<BF>(d.k, b, Tk, D);
        Vb = brow<BF>(d.v, b, Tk, D);
        Ob = brow<BF>(d.x, b, Tq, D);
        Gb = brow<BF>(bd.dx, b, Tq, D);
        dQb = brow<BF>(bd.dq, b, Tq, D);
        same_kv = d.k.ptr == d.v.ptr && d.k.sB == d.v.sB && d.k.sT == d.v.sT;
        sbase = (b * d.H + h) * Tq;
        rsStat = uniform_rsrc(d.stats + 8ull * (uint64_t)sbase, 8 * (int64_t)Tq);
        if (PREV) rsRp = uniform_rsrc(d.stats + 4ull * (uint64_t)(2 * d.B * d.H * Tq + sbase), 4 * (int64_t)Tq);
        if (PREV) rsSp = uniform_rsrc(d.s_prev + 4ull * (uint64_t)sbase * Tk, 4 * (int64_t)Tq * Tk);
        if (DSN) rsDn = uniform_rsrc(bd.ds_next + 4ull * (uint64_t)sbase * Tk, 4 * (int64_t)Tq * Tk);
    }

    MEP_DEV void load_chunk(int kc) {
        k_lo = kc * CH;
#pragma unroll
        for (int kt = 0; kt < NT; ++kt) {
            const int k0 = k_lo + kt * 16;
            float kf[4], vf[4], kc4[4];
            Kb.ld4(kf, Kb.at(k0 + c, hc + 4 * g));
            if (!KV && !same_kv) Vb.ld4(vf, Vb.at(k0 + c, hc + 4 * g));
            mtk[kt] = mask_term(mask, k0 + c, Tk);
            mtl[kt] = mtk[kt] * 1.4426950408889634f;
            if (BF) mts[BF ? kt : 0] = -4.0f * mtk[kt];
            const int okq = Kb.at(k0 + 4 * g, hc + c);
#pragma unroll
            for (int s = 0; s < 4; ++s) kc4[s] = Kb.ld1(okq, s * Kb.sT4);
            kb[kt] = split2(kf);
            if (!KV) vb[kt] = same_kv ? kb[kt] : split2(vf);     // k is v (cmu-mosei, Ren-MME)
            kq[kt] = split2(kc4);
            dk[kt] = zero4();
            if (!KV) dv[kt] = zero4();
        }
        dc_acc = 0.f;
    }

    MEP_DEV void fetch(QIn& in, int qt) const {
        const int q0 = qt * 16;   // rows past Tq read zeros
        if constexpr (BF) {
            in.qaw = Qb.ld4raw(Qb.at(q0 + c, hc + 4 * g));
            in.daw = Gb.ld4raw(Gb.at(q0 + c, hc + 4 * g));
            in.oaw = Ob.ld4raw(Ob.at(q0 + c, hc + 4 * g));
        } else {
            Qb.ld4(in.qa, Qb.at(q0 + c, hc + 4 * g));
            Gb.ld4(in.da, Gb.at(q0 + c, hc + 4 * g));
        }
        const int qg = q0 + 4 * g;
        const int og = Gb.at(qg, hc + c), oq = Qb.at(qg, hc + c), oo = Ob.at(qg, hc + c), od = dQb.at(qg, hc + c);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            in.db[s] = Gb.ld1(og, s * Gb.sT4);
            in.qb[s] = Qb.ld1(oq, s * Qb.sT4);
            if (!BF) in.ob[s] = Ob.ld1(oo, s * Ob.sT4);
            in.st[s] = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rsStat, 8 * qg, 8 * s, 0));
            if (PREV) in.rp[s] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsRp, 4 * qg, 4 * s, 0));
            in.dqo[s] = dQb.ld1(od, s * dQb.sT4);
        }
    }

    // ---- staged query tiles (short kernel, MEP_BWD_DMA): the next tile's Q, dO, O and dQ rows
    // (16 rows x 64 B each: one 1-KiB LDS-DMA wave-instruction per operand, lane L = row L / 4,
    // 16-byte piece L % 4) and its row statistics go straight from HBM into the wave's LDS
    // staging area while this tile computes: no VGPRs in flight, 5 load instructions per tile
    // instead of 22.  Rows past Tq fall outside the row views (no data: the area is zeroed at the
    // wave's start and later holds finite rows of earlier tiles, whose products are masked).
    // BF (bf16 rows): 16 rows x 32 B per operand, lanes 0-31 (lane L = row L / 2, 16-byte piece
    // L % 2) into [16][16] bf16 images at the same float offsets (half of each slot used)
    // PREV / DSN: the tile's S_prev / dS_next rows [16 queries][64 keys] too, one 4-byte DMA
    // wave-instruction per query row (lane = key), rows SSTR floats apart (4 SSTR = 16 mod 32: the
    // score reads of lane groups g and g + 1 fall in different banks), read per score from LDS
    // instead of a dependent global load inside the tile's math (keys past Tk and rows past Tq fall
    // outside the range: whatever finite value the slot holds meets P = 0 there).  Two regions per
    // operand by tile parity: tile() reads tile qt's rows while tile qt + 1's are being staged.
    // dS_next is staged only without PREV (both would take the workgroup past half the LDS)
    static constexpr bool STP = PREV && SST_P, STD = DSN && SST_D && !PREV;
    static constexpr int SSTR = 68, SOPS = 16 * SSTR;
    static constexpr int SPO = 4 * 256 + 48, DNO = SPO + (STP ? 2 * SOPS : 0);
    static constexpr int STG = DNO + (STD ? 2 * SOPS : 0);   // floats: Q, dO, O, dQ [16][16], stats [16][2], PREV's rp [16], S_prev, dS_next
    MEP_DEV static bool dma_view(const mep_rows& v) {   // 16-byte aligned pieces of every row
        return BF ? ((v.ptr & 15) == 0 && v.sB % 8 == 0 && v.sT % 8 == 0) : aligned16(v);
    }
    MEP_DEV bool dma_ok() const {
        return dma_view(bd.f.q) && dma_view(bd.dx) && dma_view(bd.f.x) && dma_view(bd.dq);
    }
    MEP_DEV void stage(int qt, float* S) const {
        typedef __attribute__((address_space(3))) void lvoid;
        if (STP || STD) {
            const int oor = 4 * Tq * Tk, par = (qt & 1) * SOPS;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int q = qt * 16 + j;
                const int off = (lane < Tk && q < Tq) ? 4 * (q * Tk + lane) : oor;
                if (STP) __builtin_amdgcn_raw_ptr_buffer_load_lds(rsSp, (lvoid*)(S + SPO + par + SSTR * j), 4, off, 0, 0, 0);
                if (STD) __builtin_amdgcn_raw_ptr_buffer_load_lds(rsDn, (lvoid*)(S + DNO + par + SSTR * j), 4, off, 0, 0, 0);
            }
        }
        if (BF) {
            if (lane < 32) {
                const int row = qt * 16 + (lane >> 1), col = hc + 8 * (lane & 1);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(Qb.rs, (lvoid*)(S), 16, Qb.at(row, col), 0, 0, 0);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(Gb.rs, (lvoid*)(S + 256), 16, Gb.at(row, col), 0, 0, 0);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(Ob.rs, (lvoid*)(S + 512), 16, Ob.at(row, col), 0, 0, 0);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(dQb.rs, (lvoid*)(S + 768), 16, dQb.at(row, col), 0, 0, 0);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsStat, (lvoid*)(S + 1024), 4, 8 * 16 * qt + 4 * lane, 0, 0, 0);
            }
            if (PREV && lane < 16)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsRp, (lvoid*)(S + 1056), 4, 4 * (16 * qt + lane), 0, 0, 0);
            return;
        }
        const int row = qt * 16 + (lane >> 2), col = hc + 4 * (lane & 3);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(Qb.rs, (lvoid*)(S), 16, Qb.at(row, col), 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(Gb.rs, (lvoid*)(S + 256), 16, Gb.at(row, col), 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(Ob.rs, (lvoid*)(S + 512), 16, Ob.at(row, col), 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(dQb.rs, (lvoid*)(S + 768), 16, dQb.at(row, col), 0, 0, 0);
        if (lane < 32)   // dword pieces: the range check drops exactly the rows past Tq
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsStat, (lvoid*)(S + 1024), 4, 8 * 16 * qt + 4 * lane, 0, 0, 0);
        if (PREV && lane < 16)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsRp, (lvoid*)(S + 1056), 4, 4 * (16 * qt + lane), 0, 0, 0);
    }
    // the staged tile in the operand layouts of fetch()
    MEP_DEV void read_staged(QIn& in, const float* S) const {
        typedef __attribute__((address_space(3))) const float lcf;
        typedef __attribute__((address_space(3))) const f32x4 lcf4;
        typedef __attribute__((address_space(3))) const f32x2 lcf2;
        lcf* L = (lcf*)S;
        if (BF) {
            typedef __attribute__((address_space(3))) const unsigned short lcu16;
            typedef __attribute__((address_space(3))) const u32x2 lcu2;
            lcu16* H = (lcu16*)S;                 // operand o at H + 512 o: [16 rows][16] bf16
            in.qaw = *(lcu2*)(H + 16 * c + 4 * g);
            in.daw = *(lcu2*)(H + 512 + 16 * c + 4 * g);
            in.oaw = *(lcu2*)(H + 1024 + 16 * c + 4 * g);
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const int r = (4 * g + s4) * 16 + c;
                in.qb[s4] = __builtin_bit_cast(float, (unsigned)H[r] << 16);
                in.db[s4] = __builtin_bit_cast(float, (unsigned)H[512 + r] << 16);
                in.dqo[s4] = __builtin_bit_cast(float, (unsigned)H[1536 + r] << 16);
                in.st[s4] = *(lcf2*)(L + 1024 + 2 * (4 * g + s4));
                if (PREV) in.rp[s4] = L[1056 + 4 * g + s4];
            }
            return;
        }
        const f32x4 qa = *(lcf4*)(L + 16 * c + 4 * g), da = *(lcf4*)(L + 256 + 16 * c + 4 * g);
#pragma unroll
        for (int e = 0; e < 4; ++e) { in.qa[e] = qa[e]; in.da[e] = da[e]; }
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            const int r = (4 * g + s4) * 16 + c;
            in.qb[s4] = L[r];
            in.db[s4] = L[256 + r];
            in.ob[s4] = L[512 + r];
            in.dqo[s4] = L[768 + r];
            in.st[s4] = *(lcf2*)(L + 1024 + 2 * (4 * g + s4));
            if (PREV) in.rp[s4] = L[1056 + 4 * g + s4];
        }
    }
    MEP_DEV void store_dq_rows(const float (&dqo)[4], int qt, const floatx4& dq) const {
        const int od = dQb.at(qt * 16 + 4 * g, hc + c);
#pragma unroll
        for (int r = 0; r < 4; ++r) dQb.st1(od, r * dQb.sT4, dqo[r] + dq[r] * INV_SCALE);
    }

    // one 16-query tile against the chunk's 64 keys: accumulates dK / dV, returns this chunk's
    // dQ contribution (C[query 4g+r][dim c], before the 1/sqrt(hd) scale).  Tr: the wave's
    // transpose scratch in LDS (TFL floats: the bf16 hi and lo parts of dS, 16 x TLD2 each).
    // SS: the staged tile (LDS-DMA path: S_prev / dS_next read from it), or nullptr (global loads)
    MEP_DEV floatx4 tile(const QIn& in, int qt, float* Tr, const float* SS = nullptr) {
        const int q0 = qt * 16;
        constexpr float LOG2E = 1.4426950408889634f;
        float mm[4], li[4], del[4];
        floatx4 dd = zero4();
        if constexpr (BF) {
            // delta = rowsum(dO * O) as the diagonal of dO O^T: one 16x16x16 MFMA on the row words
            // (lane (c, g) holds C[query 4g + r][query c]; C[q][q] sits in lane q of group q >> 2,
            // register q & 3), gathered below -- instead of 4 products and 4 DPP row sums
            dd = mfma16(op4(in.daw[0], in.daw[1]), op4(in.oaw[0], in.oaw[1]), zero4());
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int qq = q0 + 4 * g + s;
            // delta = rowsum(dO * O): the 16 dims of query qq sit in one DPP row (lanes c) (fp32:
            // exact products; a 2-part matrix-core delta, subtracted from dP, moved one
            // ren_drop_long unify-weight gradient 3.9e-3 relative)
            if constexpr (BF) del[s] = shfl(dd[s], 20 * g + s);
            else del[s] = row16_sum(in.db[s] * in.ob[s]);
            // padded queries: max = +inf, 1/sum = 0 make P = exp(-inf) * 0 = 0 (and with it dS);
            // the max is kept pre-scaled by log2(e) for exp2
            const bool qok = qq < Tq;
            mm[s] = qok ? in.st[s][0] : INFINITY;   // the forward's max log2 e - log2(1/sum) (PREV: max)
            li[s] = qok ? in.st[s][1] : 0.f;
            // 1/sum folded into the exponent by the forward's statistics:
            // P = exp2(.. - (max log2 e - log2(1/sum)))
        }
        const S2 qs = BF ? S2{in.qaw[0], in.qaw[1], 0u, 0u} : split2(in.qa);
        const S2 do2 = BF ? S2{in.daw[0], in.daw[1], 0u, 0u} : split2(in.da);
        S2 qb2;
        if (KV && !BF) {
            qb2 = S2{};   // in the stacked operand B0 / B1
        } else if (KV) {   // dK folded into the dV accumulator: Q columns times the exact 1/sqrt(hd)
            float q4[4];
#pragma unroll
            for (int s = 0; s < 4; ++s) q4[s] = in.qb[s] * INV_SCALE;
            qb2 = split2(q4);
        } else {
            qb2 = split2(in.qb);
        }
        // stacked dKV operand [dO ; Q/4] (slots 0-3 / 4-7), split straight into the operand words
        u32x4 B0 = u32x4{0u, 0u, 0u, 0u}, B1 = B0;
        if (KV && !BF) {
            float q4[4];
#pragma unroll
            for (int s = 0; s < 4; ++s) q4[s] = in.qb[s] * INV_SCALE;
            B0 = split_hi(in.db, q4);
            B1 = split_lo(in.db, q4, B0);
        }
        const S2 db2 = (KV && !BF) ? S2{} : split2(in.db);
        typedef __attribute__((address_space(3))) unsigned short lushort;
        lushort* Th = (lushort*)Tr;                 // [16 queries][TLD2] bf16 parts of dS
        lushort* Tl = Th + 16 * TLD2;
#pragma unroll
        for (int kt = 0; kt < NT; ++kt) {
            const int kk = k_lo + kt * 16 + c;
            // recomputed scores on the 2-way split (the forward's are 3-way): P differs from the
            // forward's by <= ~2^-16 relative, far inside the gradient tolerance
            // C[query 4g+r][key c].  BF + EXP2: the accumulator starts at -4 x the key's mask term,
            // so the exponent below needs no per-score mask add (0 for kept keys: the same bits; a
            // masked or padding key's score stays ~-4e8 / -inf and its P exactly 0).  The fp32
            // instances keep the add (four more live registers spill the 128-register short kernel)
            constexpr bool MI = BF && !PREV;
            const float m0 = MI ? mts[BF ? kt : 0] : 0.f;
            const floatx4 st = dot16<BF>(qs, kb[kt], floatx4{m0, m0, m0, m0});
            // dP - delta: the accumulator starts at -delta (query 4g+r)
            const floatx4 dp = dot16<BF>(do2, KV ? kb[kt] : vb[kt], floatx4{-del[0], -del[1], -del[2], -del[3]});
            float p[4], dsv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int qq = q0 + 4 * g + r;
                float spv = 0.f;
                int si = 0;
                if (PREV || DSN) {
                    si = (sbase + min(qq, Tq - 1)) * Tk + min(kk, Tk - 1);
                    if (PREV) spv = STP && SS ? ((const __attribute__((address_space(3))) float*)SS)[SPO + (qt & 1) * SOPS + SSTR * (4 * g + r) + kt * 16 + c] : sprev[si];
                }
                float pv;
                if constexpr (PREV) {
                    // residual scores (F7): the score in the forward's op order, then exp(s - max) /
                    // sum with s - max exact.  c * S_prev is ~1e8 at masked keys: for c <= -1 those
                    // slots carry the row's maximum (~5e7, c < -1) or a score of ~0 (c = -1), and a
                    // fused (s log2 e - max log2 e) rounds ~1e8-sized terms to whole units of the
                    // exponent
                    const float sv = score<PREV>(st[r], cres, spv, mtk[kt]);
                    pv = __builtin_amdgcn_exp2f((sv - mm[r]) * LOG2E) * li[r];
                } else {
                    // (dot / 4 - mask) log2 e - max log2 e with the mask and max terms combined
                    pv = __builtin_amdgcn_exp2f(fmaf(st[r], INV_SCALE * LOG2E, MI ? -mm[r] : -(mtl[kt] + mm[r])));
                }
                float gsv = pv * dp[r];
                if (DSN || PREV) {
                    const bool ok = (qq < Tq) && (kk < Tk);
                    const float gn = DSN && ok ? (STD && SS ? ((const __attribute__((address_space(3))) float*)SS)[DNO + (qt & 1) * SOPS + SSTR * (4 * g + r) + kt * 16 + c]
                                                     : dsn[si]) : 0.f;
                    // dc = sum dS S_prev.  The softmax part P (dP - delta) sums to 0 over a row, so
                    // its S_prev is taken relative to the row's P-weighted mean rp (exact in real
                    // arithmetic): where c <= -1 puts the row's weight on masked keys, S_prev there is
                    // -1e8 and the unshifted sum cancels ~1e8-sized terms, leaving 1e8 x the rounding
                    // of dP; the shifted terms are small.  The gradient arriving on the scores (DSN)
                    // has no such identity and keeps S_prev itself
                    if (PREV) dc_acc = fmaf(gsv, spv - in.rp[r], dc_acc);
                    gsv += gn;
                    if (PREV) {
                        if (ok) dsp[si] = cres * gsv;
                        if (DSN) dc_acc = fmaf(gn, spv, dc_acc);
                    }
                }
                p[r] = pv;
                dsv[r] = gsv;
            }
            S2 ds2;
            if (KV && !BF) {
                // dKV[key][dim] += P^T dO + dS^T Q / 4 as ONE 32-deep contraction [P | dS] . [dO ; Q/4]
                // (slots 0-3: P / dO of queries 4g..4g+3, slots 4-7: dS / Q/4 of the same queries),
                // products x0 y0 + x1 y0 + x0 y1 of both terms on three 16x16x32 MFMAs; the parts are
                // split straight into the operand words (no register copies)
                const u32x4 A0 = split_hi(p, dsv), A1 = split_lo(p, dsv, A0);
                ds2 = S2{A0[2], A0[3], A1[2], A1[3]};
                dk[kt] = mfma(__builtin_bit_cast(bf16x8, A0), __builtin_bit_cast(bf16x8, B0), dk[kt]);
                dk[kt] = mfma(__builtin_bit_cast(bf16x8, A1), __builtin_bit_cast(bf16x8, B0), dk[kt]);
                dk[kt] = mfma(__builtin_bit_cast(bf16x8, A0), __builtin_bit_cast(bf16x8, B1), dk[kt]);
            } else {
                ds2 = split2(dsv);
            }
            if (KV && !BF) {
            } else if (KV) {                             // dKV[key][dim] += P^T dO + dS^T Q / 4
                dk[kt] = dot16<BF>(split2(p), db2, dk[kt]);
            } else {
                dv[kt] = dot16<BF>(split2(p), db2, dv[kt]);
            }
            if (!(KV && !BF)) dk[kt] = dot16<BF>(ds2, qb2, dk[kt]);   // dK[key][dim] += dS^T Q
            // the split dS, element by element, into Th / Tl[query][key] (bf16).  (A packed
            // [key][query] word per key tile read back by ds_read_b64_tr_b16 measured no faster on
            // the bf16 path: 26.5 vs 26.4 us at cfg3, round 6)
            const unsigned hw[4] = {ds2.h0, ds2.h0 >> 16, ds2.h1, ds2.h1 >> 16};
            const unsigned lw[4] = {ds2.l0, ds2.l0 >> 16, ds2.l1, ds2.l1 >> 16};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                Th[(4 * g + r) * TLD2 + kt * 16 + c] = (unsigned short)hw[r];
                if (!BF) Tl[(4 * g + r) * TLD2 + kt * 16 + c] = (unsigned short)lw[r];
            }
        }
        // dQ += dS K with the query on the lane: the transposed 16 x 64 dS parts, already split,
        // come back as packed words (keys 4g .. 4g+3 of each key tile, one 8-byte read per part)
        wave_lds_sync();
        S2 tq[NT];
        typedef __attribute__((address_space(3))) u32x2 lu32x2;
#pragma unroll
        for (int kt = 0; kt < NT; ++kt) {
            const u32x2 hh = *reinterpret_cast<const lu32x2*>(Th + c * TLD2 + kt * 16 + 4 * g);
            const u32x2 ll = BF ? u32x2{0u, 0u} : *reinterpret_cast<const lu32x2*>(Tl + c * TLD2 + kt * 16 + 4 * g);
            tq[kt] = S2{hh[0], hh[1], ll[0], ll[1]};
        }
        wave_lds_sync();
        floatx4 dq = zero4();
#pragma unroll
        for (int kt = 0; kt < NT; kt += 2) dq = dot32<BF>(tq[kt], tq[kt + 1], kq[kt], kq[kt + 1], dq);
        return dq;
    }

    // final dq rows of a tile: dq_in + total * 1/sqrt(hd) (rows past Tq dropped)
    MEP_DEV void store_dq(const QIn& in, int qt, const floatx4& dq) const {
        const int od = dQb.at(qt * 16 + 4 * g, hc + c);
#pragma unroll
        for (int r = 0; r < 4; ++r) dQb.st1(od, r * dQb.sT4, in.dqo[r] + dq[r] * INV_SCALE);
    }
};

// SHORT (Tk <= 64): one WAVE per (b, h) -- the single key chunk makes the wave the exclusive owner
// of every dQ row and of its dK / dV rows, so no cross-wave sums are needed; the query tiles are
// walked with every load of the next tile issued before this tile's math (two register sets).
// waves per SIMD of the short backward by register need (scripts/resusage.py, fp32 path; the bf16
// instances need fewer): KV frees the V rows and the dV accumulators
template <bool PREV, bool DSN, bool KV>
constexpr int bwd_short_waves() { return PREV || (DSN && SST_D) ? 2 : (KV && !DSN) ? MEP_BWD_WAVES_KV : MEP_BWD_WAVES; }


template <bool PREV, bool DSN, bool BF, bool KV>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(bwd_short_waves<PREV, DSN, KV>()))) void k_attn_bwd_short(const mep_attn_bwd_desc* __restrict__ descs) {
    __shared__ __attribute__((aligned(16))) float Tr[WAVES][TFL];
    __shared__ __attribute__((aligned(16))) float Stg[WAVES][Bwd<PREV, DSN, BF, KV>::STG];
    const mep_attn_bwd_desc& bd = descs[blockIdx.y];
    if (bd.f.Tk > CH) return;                // a LONG descriptor
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int bh = blockIdx.x * WAVES + wave;
    if (bh >= bd.f.B * bd.f.H) return;       // whole wave leaves; only wave-private LDS below
    Bwd<PREV, DSN, BF, KV> u(bd, bh / bd.f.H, bh % bd.f.H, lane);
    const int nqt = (u.Tq + 15) / 16;
    const bool same_out = bd.dk.ptr == bd.dv.ptr && bd.dk.sB == bd.dv.sB && bd.dk.sT == bd.dv.sT;
    if (KV && !(u.same_kv && same_out)) {    // broken MEP_ATTN_KV promise: NaN dq rows, loudly
        for (int qt = 0; qt < nqt; ++qt) {
            const int od = u.dQb.at(qt * 16 + 4 * u.g, u.hc + u.c);
#pragma unroll
            for (int r = 0; r < 4; ++r) u.dQb.st1(od, r * u.dQb.sT4, __builtin_nanf(""));
        }
        return;
    }
    if (u.dma_ok()) {
        float* S = Stg[wave];
        typedef __attribute__((address_space(3))) f32x4 lf4;
        for (int e = lane; e < Bwd<PREV, DSN, BF, KV>::STG / 4; e += 64) ((lf4*)S)[e] = f32x4{0.f, 0.f, 0.f, 0.f};
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        u.stage(0, S);
        u.load_chunk(0);   // (K rows staged by LDS-DMA as well measured slower: 42.2-43.7 vs 41.7 us)
        floatx4 dq_prev = zero4();
        float dqo_prev[4] = {0.f, 0.f, 0.f, 0.f};
        for (int qt = 0; qt < nqt; ++qt) {
            typename Bwd<PREV, DSN, BF, KV>::QIn in;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tile qt landed in S
            u.read_staged(in, S);
            if (qt > 0) u.store_dq_rows(dqo_prev, qt - 1, dq_prev);   // after the wait: stores stay in flight
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // S read before it is refilled
            if (qt + 1 < nqt) u.stage(qt + 1, S);
            dq_prev = u.tile(in, qt, Tr[wave], S);
#pragma unroll
            for (int r = 0; r < 4; ++r) dqo_prev[r] = in.dqo[r];
        }
        if (nqt > 0) u.store_dq_rows(dqo_prev, nqt - 1, dq_prev);
    } else
    {
    u.load_chunk(0);
    for (int qt = 0; qt < nqt; ++qt) {
        typename Bwd<PREV, DSN, BF, KV>::QIn in;
        u.fetch(in, qt);
        u.store_dq(in, qt, u.tile(in, qt, Tr[wave]));
    }
    }
    const BRowT<BF> dKb = brow<BF>(bd.dk, u.b, u.Tk, bd.f.H * HD), dVb = brow<BF>(bd.dv, u.b, u.Tk, bd.f.H * HD);
    const int ok_ = dKb.at(4 * u.g, u.hc + u.c), ov_ = dVb.at(4 * u.g, u.hc + u.c);   // keys past Tk: dropped
#pragma unroll
    for (int kt = 0; kt < NT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (KV) {
                dKb.st1(ok_, (16 * kt + r) * dKb.sT4, u.dk[kt][r]);
            } else if (same_out) {
                dKb.st1(ok_, (16 * kt + r) * dKb.sT4, u.dk[kt][r] * INV_SCALE + u.dv[kt][r]);
            } else {
                dKb.st1(ok_, (16 * kt + r) * dKb.sT4, u.dk[kt][r] * INV_SCALE);
                dVb.st1(ov_, (16 * kt + r) * dVb.sT4, u.dv[kt][r]);
            }
        }
    if (PREV && bd.dc_partial) {
        const float w = wave_sum(u.dc_acc);
        if (lane == 0) G<float>(bd.dc_partial)[bh] = w;
    }
}

// LONG (Tk > 64): one WORKGROUP per (b, h).  Key chunks are the outer loop; wave w takes query
// tiles w, w+4, ...; the waves' dK / dV partials of a chunk are summed in wave order through LDS
// and a tile's dQ is carried across chunks in (wave-private) LDS, so every sum has a fixed order.
// LDS: [RED] dK/dV partials (aliased by the waves' dS transposes during the query loop), [4] dc
// partials, [dq_tiles][256] the carried dQ tiles.
template <bool PREV, bool DSN, bool BF>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(2))) void k_attn_bwd_long(const mep_attn_bwd_desc* __restrict__ descs, int splitq) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const mep_attn_bwd_desc& bd = descs[blockIdx.y];
    const mep_attn_desc& d = bd.f;
    const int bh = blockIdx.x;
    // splitq bit 0: SHORT descriptors run here too; bit 1: LONG ones ran on the wide kernel
    if ((d.Tk <= CH && !(splitq & 1)) || (d.Tk > CH && (splitq & 2)) || bh >= d.B * d.H) return;   // the whole workgroup
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    Bwd<PREV, DSN, BF> u(bd, bh / d.H, bh % d.H, lane);
    const int D = d.H * HD;
    const int nqt = (u.Tq + 15) / 16, nkc = (u.Tk + CH - 1) / CH;
    const int nw = min(WAVES, nqt);          // waves that own query tiles
    const BRowT<BF> dKb = brow<BF>(bd.dk, u.b, u.Tk, D), dVb = brow<BF>(bd.dv, u.b, u.Tk, D);   // keys past Tk: dropped
    const bool same_out = bd.dk.ptr == bd.dv.ptr && bd.dk.sB == bd.dv.sB && bd.dk.sT == bd.dv.sT;
    float* Tr = lds + wave * TFL;            // inside the R region
    float* R = lds;
    float* DC = lds + RED;
    float* DQ = DC + WAVES;
    for (int kc = 0; kc < nkc; ++kc) {
        u.load_chunk(kc);
        for (int qt = wave; qt < nqt; qt += WAVES) {
            typename Bwd<PREV, DSN, BF>::QIn in;
            u.fetch(in, qt);
            floatx4 dq = u.tile(in, qt, Tr);
            floatx4* carry = reinterpret_cast<floatx4*>(DQ + qt * 256) + lane;
            if (kc > 0) dq += *carry;
            if (kc + 1 < nkc) *carry = dq;
            else u.store_dq(in, qt, dq);
        }
        __syncthreads();                      // every wave is done with its transpose region
        if (wave < nw) {
            float* Rw = R + wave * 2 * CH * HD;
#pragma unroll
            for (int kt = 0; kt < NT; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int e = (kt * 16 + 4 * u.g + r) * HD + u.c;
                    if (same_out) {
                        Rw[e] = u.dk[kt][r] * INV_SCALE + u.dv[kt][r];
                    } else {
                        Rw[e] = u.dk[kt][r] * INV_SCALE;
                        Rw[CH * HD + e] = u.dv[kt][r];
                    }
                }
        }
        if (PREV) {
            const float w = wave < nw ? wave_sum(u.dc_acc) : 0.f;
            if (lane == 0) DC[wave] = w;
        }
        __syncthreads();
        {
            const int t = threadIdx.x;               // key t / 4, dims 4 (t % 4) .. + 3
            const int key = t >> 2, col = 4 * (t & 3);
            const int e = key * HD + col;
            f32x4 sk = *reinterpret_cast<const f32x4*>(R + e);
            f32x4 sv = *reinterpret_cast<const f32x4*>(R + CH * HD + e);
            for (int w = 1; w < nw; ++w) {
                sk += *reinterpret_cast<const f32x4*>(R + w * 2 * CH * HD + e);
                if (!same_out) sv += *reinterpret_cast<const f32x4*>(R + w * 2 * CH * HD + CH * HD + e);
            }
            dKb.st4(dKb.at(kc * CH + key, u.hc + col), sk);
            if (!same_out) dVb.st4(dVb.at(kc * CH + key, u.hc + col), sv);
            if (PREV && t == 0 && bd.dc_partial)
                G<float>(bd.dc_partial)[bh * nkc + kc] = ((DC[0] + DC[1]) + DC[2]) + DC[3];
        }
        __syncthreads();                      // R read before the next chunk's transposes
    }
}

// (b, h) of workgroup P of a one-workgroup-per-(b, h) launch.  A head's 16 dims are 64 bytes of a
// row; the HBM / L2 line is 128.  Heads 2i and 2i + 1 of one row go to workgroups P and P + 8,
// which the round-robin dispatch puts on ONE XCD at about the same time, so the line each of them
// needs half of is fetched once into that XCD's L2 (both in the plain order they run on different
// XCDs and each fetches the whole line: 1.87x the algorithmic reads at cfg5).  Needs
// the x extent (gridDim.x) a multiple of 16 -- the linear workgroup id is x + gridDim.x * y, so
// its XCD is x mod 8 -- and H even; otherwise the plain order.  A bijection of [0, gridDim.x).
MEP_DEV int head_pair_order(int P, int H) {
    if (!(gridDim.x & 31) && !(H & 3)) {
        // heads 4j .. 4j + 3 of a row on one XCD, dispatched one after another (its L2 fetches a
        // 128-byte line of bf16 rows once for the four 32-byte head slices)
        const int x = P & 7, j = P >> 3;
        return ((((j >> 2) << 3) + x) << 2) + (j & 3);
    }
    if ((gridDim.x & 15) || (H & 1)) return P;
    const int x = P & 7, j = P >> 3;
    return ((((j >> 1) << 3) + x) << 1) + (j & 1);
}

// WIDE (64 < Tk <= 64 * MEP_ATTN_MAX_KCHUNKS): one WORKGROUP per (b, h) and one WAVE per 64-key
// chunk (blockDim = 64 x the launch's largest chunk count).  A wave keeps its chunk's K / V rows
// and its dK / dV accumulators in registers for the whole kernel and walks every query tile, so
// dK / dV need no cross-wave sum and are stored once from registers.  The query tiles are walked
// in lockstep: tile qt + 1's Q, dO, O, dQ rows and row statistics are staged once per workgroup
// by LDS-DMA (one wave issues it, double-buffered) while tile qt computes; after tile qt each wave
// leaves its 16 x 16 dQ partial in an LDS slot and one wave sums the slots in chunk order
// (fixed order: deterministic) onto the incoming dQ rows.  One barrier per query tile.
// LDS: [2][STG] staging | [2][waves][256] dQ slots | [waves][TFL] dS transposes.
template <bool PREV, bool DSN, bool BF, bool KV>
__global__ __launch_bounds__(64 * MEP_ATTN_MAX_KCHUNKS) __attribute__((amdgpu_waves_per_eu(MEP_BWD_WIDE_WAVES ? MEP_BWD_WIDE_WAVES : bwd_short_waves<PREV, DSN, KV>())))
void k_attn_bwd_wide(const mep_attn_bwd_desc* __restrict__ descs) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    typedef Bwd<PREV, DSN, BF, KV> U;
    const mep_attn_bwd_desc& bd = descs[blockIdx.y];
    const mep_attn_desc& d = bd.f;
    const int bh = head_pair_order(blockIdx.x, d.H);
    if (d.Tk <= CH || bh >= d.B * d.H) return;   // a SHORT descriptor / past the end: the whole workgroup
    const int nwv = blockDim.x >> 6;             // waves = the launch's largest chunk count
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nkc = (d.Tk + CH - 1) / CH;        // <= nwv (host)
    const int D = d.H * HD;
    float* Stg = lds;
    float* Slot = lds + 2 * U::STG;
    float* Tr = Slot + 2 * nwv * 256 + wave * TFL;
    U u(bd, bh / d.H, bh % d.H, lane);
    const int nqt = (u.Tq + 15) / 16;
    const bool same_out = bd.dk.ptr == bd.dv.ptr && bd.dk.sB == bd.dv.sB && bd.dk.sT == bd.dv.sT;
    if (KV && !(u.same_kv && same_out)) {        // broken MEP_ATTN_KV promise: NaN dq rows, loudly
        if (wave == 0)
            for (int qt = 0; qt < nqt; ++qt) {
                const int od = u.dQb.at(qt * 16 + 4 * u.g, u.hc + u.c);
#pragma unroll
                for (int r = 0; r < 4; ++r) u.dQb.st1(od, r * u.dQb.sT4, __builtin_nanf(""));
            }
        return;                                   // descriptor-uniform: every wave leaves here
    }
    const bool active = wave < nkc;
    const bool dma = u.dma_ok();
    // rows past Tq receive no DMA data: start from zeros (later finite rows of earlier tiles)
    for (int e = threadIdx.x; e < 2 * U::STG / 4; e += blockDim.x)
        reinterpret_cast<f32x4*>(Stg)[e] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (active) u.load_chunk(wave);
    __syncthreads();
    if (dma && wave == 0) {
        u.stage(0, Stg);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    for (int qt = 0; qt < nqt; ++qt) {
        typename U::QIn in;
        if (dma) u.read_staged(in, Stg + (qt & 1) * U::STG);
        else u.fetch(in, qt);
        // the other staging buffer held tile qt - 1, read by every wave before the last barrier
        const int iw = (qt + 1) % nwv;
        if (dma && wave == iw && qt + 1 < nqt) u.stage(qt + 1, Stg + ((qt + 1) & 1) * U::STG);
        floatx4 dq = zero4();
        if (active) dq = u.tile(in, qt, Tr);
        reinterpret_cast<floatx4*>(Slot + ((qt & 1) * nwv + wave) * 256)[lane] = dq;
        if (dma && wave == iw) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // tile qt + 1 landed
        __syncthreads();
        if (wave == qt % nwv) {                   // chunk-ordered sum onto the incoming dq rows
            const floatx4* sl = reinterpret_cast<const floatx4*>(Slot + (qt & 1) * nwv * 256) + lane;
            floatx4 tot = sl[0];
            for (int w = 1; w < nkc; ++w) tot += sl[w * 64];
            u.store_dq_rows(in.dqo, qt, tot);
        }
    }
    if (!active) return;
    const BRowT<BF> dKb = brow<BF>(bd.dk, u.b, u.Tk, D), dVb = brow<BF>(bd.dv, u.b, u.Tk, D);   // keys past Tk: dropped
    const int ok_ = dKb.at(u.k_lo + 4 * u.g, u.hc + u.c), ov_ = dVb.at(u.k_lo + 4 * u.g, u.hc + u.c);
#pragma unroll
    for (int kt = 0; kt < NT; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (KV) {
                dKb.st1(ok_, (16 * kt + r) * dKb.sT4, u.dk[kt][r]);
            } else if (same_out) {
                dKb.st1(ok_, (16 * kt + r) * dKb.sT4, u.dk[kt][r] * INV_SCALE + u.dv[kt][r]);
            } else {
                dKb.st1(ok_, (16 * kt + r) * dKb.sT4, u.dk[kt][r] * INV_SCALE);
                dVb.st1(ov_, (16 * kt + r) * dVb.sT4, u.dv[kt][r]);
            }
        }
    if (PREV && bd.dc_partial) {
        const float w = wave_sum(u.dc_acc);
        if (lane == 0) G<float>(bd.dc_partial)[bh * nkc + wave] = w;
    }
}

}  // namespace

// Launch geometry: forward 256 threads (4 waves, one task each), tasks = B * H * ceil(Tq/64),
// max_tiles = ceil(max tasks / 4); backward max_tiles = max B * H: SHORT descriptors (Tk <= 64)
// one wave per (b, h) (ceil(max_tiles / 4) workgroups), LONG ones one workgroup per (b, h).
// dc_partial (backward) has one float per (b, h, key chunk): index (b*H + h) * ceil(Tk/64) +
// chunk.  `flags` (MEP_ATTN_*) select the compiled variants: PREV / SOUT (DSN) must hold for every
// descriptor of the launch; SHORT / LONG say whether descriptors with Tk <= 64 / Tk > 64 are
// present (one kernel launch per class); backward: MEP_ATTN_DQ_TILES(n) in bits 8.. = the
// largest ceil(Tq/16) among descriptors with Tk > 64 (LDS for the carried dQ).
extern "C" int mep_attn_fwd(const mep_attn_desc* descs, int n_desc, int max_tiles, int flags, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    if (!(flags & (MEP_ATTN_SHORT | MEP_ATTN_LONG))) { mep_set_error("mep_attn_fwd: flags need SHORT and/or LONG"); return MEP_EINVAL; }
    const bool prev = flags & MEP_ATTN_PREV, sout = flags & MEP_ATTN_SOUT, bf = flags & MEP_PREC_BF16;
    const bool splitq = flags & MEP_ATTN_SPLITQ;   // 16 queries per wave task instead of 64
    const dim3 grid(max_tiles, n_desc), block(THREADS);
    hipStream_t st = (hipStream_t)stream;
    if (flags & MEP_ATTN_HD32) {   // robot_demo (inference, fp32 path)
        if (bf) { mep_set_error("mep_attn_fwd: hd = 32 runs the fp32 path only"); return MEP_EINVAL; }
#define MEP_FWD32(P, S, SI) hipLaunchKernelGGL((k_attn_fwd<P, S, SI, false, 32>), grid, block, 0, st, descs)
        for (int single = 1; single >= 0; --single) {
            if (!(flags & (single ? MEP_ATTN_SHORT : MEP_ATTN_LONG))) continue;
            if (single) {
                if (prev) { if (sout) MEP_FWD32(true, true, true); else MEP_FWD32(true, false, true); }
                else      { if (sout) MEP_FWD32(false, true, true); else MEP_FWD32(false, false, true); }
            } else {
                if (prev) { if (sout) MEP_FWD32(true, true, false); else MEP_FWD32(true, false, false); }
                else      { if (sout) MEP_FWD32(false, true, false); else MEP_FWD32(false, false, false); }
            }
        }
#undef MEP_FWD32
        return mep_check_launch("mep_attn_fwd");
    }
#define MEP_FWD(P, S, SI) \
    do { if (splitq) { if (bf) hipLaunchKernelGGL((k_attn_fwd<P, S, SI, true, HD, 16>), grid, block, 0, st, descs); \
                       else hipLaunchKernelGGL((k_attn_fwd<P, S, SI, false, HD, 16>), grid, block, 0, st, descs); } \
         else if (bf) hipLaunchKernelGGL((k_attn_fwd<P, S, SI, true>), grid, block, 0, st, descs); \
         else hipLaunchKernelGGL((k_attn_fwd<P, S, SI, false>), grid, block, 0, st, descs); } while (0)
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
    if (!(flags & (MEP_ATTN_SHORT | MEP_ATTN_LONG))) { mep_set_error("mep_attn_bwd: flags need SHORT and/or LONG"); return MEP_EINVAL; }
    const bool prev = flags & MEP_ATTN_PREV, dsn = flags & MEP_ATTN_SOUT, bf = flags & MEP_PREC_BF16;
    const bool kv = flags & MEP_ATTN_KV;
    const int dq_tiles = (flags >> 8) & 0xff;
    if (flags & MEP_ATTN_HD32) { mep_set_error("mep_attn_bwd: hd = 32 is forward-only (robot_demo inference)"); return MEP_EINVAL; }
    const size_t lds = sizeof(float) * ((size_t)RED + WAVES + 256 * (size_t)dq_tiles);
    if (lds > 160 * 1024) { mep_set_error("mep_attn_bwd: Tq too large for the LDS-carried dQ (Tk > 64)"); return MEP_EINVAL; }
    hipStream_t st = (hipStream_t)stream;
    const bool splitq = flags & MEP_ATTN_SPLITQ;
    if ((flags & MEP_ATTN_SHORT) && !splitq) {
        const dim3 grid((max_tiles + WAVES - 1) / WAVES, n_desc), block(THREADS);
#define MEP_BS2(P, S, K) \
    do { if (bf) hipLaunchKernelGGL((k_attn_bwd_short<P, S, true, K>), grid, block, 0, st, descs); else hipLaunchKernelGGL((k_attn_bwd_short<P, S, false, K>), grid, block, 0, st, descs); } while (0)
#define MEP_BS(P, S) do { if (kv) MEP_BS2(P, S, true); else MEP_BS2(P, S, false); } while (0)
        if (prev) { if (dsn) MEP_BS(true, true); else MEP_BS(true, false); }
        else      { if (dsn) MEP_BS(false, true); else MEP_BS(false, false); }
#undef MEP_BS
#undef MEP_BS2
    }
    const int kchunks = (flags >> 20) & 0xf;   // MEP_ATTN_KCHUNKS: the wide kernel for the LONG descriptors
    if ((flags & MEP_ATTN_LONG) && kchunks >= 2) {
        if (kchunks > MEP_ATTN_MAX_KCHUNKS) { mep_set_error("mep_attn_bwd: MEP_ATTN_KCHUNKS above MEP_ATTN_MAX_KCHUNKS"); return MEP_EINVAL; }
        const size_t wl = sizeof(float) * (2 * (size_t)Bwd<false, false, false>::STG + (size_t)kchunks * (2 * 256 + TFL));
        const dim3 grid(max_tiles, n_desc), block(64 * kchunks);
#define MEP_BW2(P, S, K) \
    do { if (bf) hipLaunchKernelGGL((k_attn_bwd_wide<P, S, true, K>), grid, block, wl, st, descs); \
         else hipLaunchKernelGGL((k_attn_bwd_wide<P, S, false, K>), grid, block, wl, st, descs); } while (0)
#define MEP_BW(P, S) do { if (kv) MEP_BW2(P, S, true); else MEP_BW2(P, S, false); } while (0)
        if (prev) { if (dsn) MEP_BW(true, true); else MEP_BW(true, false); }
        else      { if (dsn) MEP_BW(false, true); else MEP_BW(false, false); }
#undef MEP_BW
#undef MEP_BW2
    }
    if (((flags & MEP_ATTN_LONG) && kchunks < 2) || splitq) {
        const int mode = (splitq ? 1 : 0) | ((flags & MEP_ATTN_LONG) && kchunks >= 2 ? 2 : 0);
        static bool lds_attr = false;   // allow more than 64 KB of dynamic LDS (long Tq)
        if (!lds_attr) {
            const int mx = 160 * 1024;
            const void* fns[] = {(const void*)k_attn_bwd_long<true, true, false>, (const void*)k_attn_bwd_long<true, false, false>,
                                 (const void*)k_attn_bwd_long<false, true, false>, (const void*)k_attn_bwd_long<false, false, false>,
                                 (const void*)k_attn_bwd_long<true, true, true>, (const void*)k_attn_bwd_long<true, false, true>,
                                 (const void*)k_attn_bwd_long<false, true, true>, (const void*)k_attn_bwd_long<false, false, true>};
            for (const void* f : fns) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
            lds_attr = true;
        }
        const dim3 grid(max_tiles, n_desc), block(THREADS);
#define MEP_BL(P, S) \
    do { if (bf) hipLaunchKernelGGL((k_attn_bwd_long<P, S, true>), grid, block, lds, st, descs, mode); \
         else hipLaunchKernelGGL((k_attn_bwd_long<P, S, false>), grid, block, lds, st, descs, mode); } while (0)
        if (prev) { if (dsn) MEP_BL(true, true); else MEP_BL(true, false); }
        else      { if (dsn) MEP_BL(false, true); else MEP_BL(false, false); }
#undef MEP_BL
    }
    return mep_check_launch("mep_attn_bwd");
}

// hipcc (ROCm 7.2) leaves the host stubs of k_attn_bwd_wide undefined when they are only named
// inside mep_attn_bwd's launch macros (the device code is emitted); instantiating them explicitly
// here emits them
namespace {
#define MEP_BWI(P, S, B, K) template __global__ void k_attn_bwd_wide<P, S, B, K>(const mep_attn_bwd_desc* __restrict__);
#define MEP_BWI2(P, S) MEP_BWI(P, S, false, false) MEP_BWI(P, S, false, true) MEP_BWI(P, S, true, false) MEP_BWI(P, S, true, true)
MEP_BWI2(false, false) MEP_BWI2(false, true) MEP_BWI2(true, false) MEP_BWI2(true, true)
#undef MEP_BWI2
#undef MEP_BWI
}  // namespace
