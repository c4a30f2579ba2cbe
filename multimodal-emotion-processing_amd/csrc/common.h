// Device helpers shared by the gfx950 kernels of libmep_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mep.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

#define MEP_DEV __device__ __forceinline__
// Device memory is addressed through the GLOBAL address space explicitly: pointers rebuilt from
// the 64-bit integers of a descriptor are otherwise generic and every access becomes a FLAT
// instruction (counted on both vmcnt and lgkmcnt, serialising LDS and VMEM waits).
#define MEP_G __attribute__((address_space(1)))

namespace mep {

typedef MEP_G float gfloat;
template <typename T>
MEP_DEV MEP_G T* G(uint64_t p) { return reinterpret_cast<MEP_G T*>(p); }

typedef float f32x4 __attribute__((ext_vector_type(4)));
// 16-byte global load / store (p must be 16-byte aligned)
MEP_DEV float4 ldg4(const gfloat* p) {
    const f32x4 v = *reinterpret_cast<const MEP_G f32x4*>(p);
    return make_float4(v.x, v.y, v.z, v.w);
}
MEP_DEV void stg4(gfloat* p, float4 v) { *reinterpret_cast<MEP_G f32x4*>(p) = f32x4{v.x, v.y, v.z, v.w}; }

constexpr int kWave = 64;

// ------------------------------------------------------------------ activation storage
// Activations of the bf16 path (MEP_PREC_BF16 plans: features, unified rows, attention outputs,
// epilogue intermediates and their gradients) are stored as bf16, everything else (block outputs,
// scores, statistics, parameters and their gradients) as fp32.  Row views count elements, so
// the same mep_rows addresses either; HS (half storage) selects the element type at compile time.
// 4 consecutive elements are one 16-byte (fp32) or 8-byte (bf16) access; bf16 -> fp32 is exact,
// fp32 -> bf16 rounds to nearest even (v_cvt_pk_bf16_f32).
typedef MEP_G unsigned short ghalf;
typedef unsigned u32x2a __attribute__((ext_vector_type(2)));
template <bool HS> struct AElem { typedef float T; };
template <> struct AElem<true> { typedef unsigned short T; };
template <bool HS> using aelem = MEP_G typename AElem<HS>::T;
MEP_DEV unsigned pk_bf16x2(float a, float b) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef __bf16 b2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(unsigned, __builtin_convertvector(f2{a, b}, b2));
}
MEP_DEV float bf16_word_lo(unsigned w) { return __builtin_bit_cast(float, w << 16); }
MEP_DEV float bf16_word_hi(unsigned w) { return __builtin_bit_cast(float, w & 0xffff0000u); }
MEP_DEV f32x4 ld4a(const gfloat* p) { return *reinterpret_cast<const MEP_G f32x4*>(p); }
MEP_DEV f32x4 ld4a(const ghalf* p) {
    const u32x2a w = *reinterpret_cast<const MEP_G u32x2a*>(p);
    return f32x4{bf16_word_lo(w[0]), bf16_word_hi(w[0]), bf16_word_lo(w[1]), bf16_word_hi(w[1])};
}
MEP_DEV void st4a(gfloat* p, f32x4 v) { *reinterpret_cast<MEP_G f32x4*>(p) = v; }
MEP_DEV void st4a(ghalf* p, f32x4 v) {
    *reinterpret_cast<MEP_G u32x2a*>(p) = u32x2a{pk_bf16x2(v[0], v[1]), pk_bf16x2(v[2], v[3])};
}
MEP_DEV float ld1a(const gfloat* p) { return *p; }
MEP_DEV float ld1a(const ghalf* p) { return __builtin_bit_cast(float, (unsigned)*p << 16); }
MEP_DEV void st1a(gfloat* p, float v) { *p = v; }
MEP_DEV void st1a(ghalf* p, float v) { *p = (unsigned short)pk_bf16x2(v, 0.f); }

// ------------------------------------------------------------------ row views
// tok -> (b, t) = (tok / T, tok % T) without an integer division: the quotient from the f32
// reciprocal (v_rcp_f32, 1 ulp) is off by at most one for tok < 2^22 (relative error of the
// product <= 2^-22), and one correction step each way makes it exact.  Hosts keep every row view
// under 2^22 rows (4M tokens).
//
// MEP_ROW24 (default): the products on the 24-bit multiplier (full rate; v_mul_lo_u32 and the
// 64-bit multiplies are quarter rate, and an epilogue tile addresses ~8 views).  Needs strides
// sB, sT < 2^24 elements and every view's element offsets < 2^32 (mep.h, mep_rows; the Python
// hosts check both when they build a view).
// (b, t) = (tok / T, tok % T), tok < 2^22, T < 2^24
MEP_DEV void tok_split(int tok, int T, int& b, int& t) {
    b = (int)((float)tok * __builtin_amdgcn_rcpf((float)T));
    t = tok - (int)__umul24((unsigned)b, (unsigned)T);
    if (t < 0) { --b; t += T; }
    if (t >= T) { ++b; t -= T; }
}
MEP_DEV int64_t row_off(const mep_rows& r, int tok) {
    const int T = r.T;
    int b, t;
    tok_split(tok, T, b, t);
    return (int64_t)(uint32_t)(__umul24((unsigned)b, (unsigned)r.sB) + __umul24((unsigned)t, (unsigned)r.sT));
}
MEP_DEV gfloat* row_ptr(const mep_rows& r, int tok) { return G<float>(r.ptr) + row_off(r, tok); }
// row of an activation view in HS storage (element pointer: ld4a / st4a / ld1a / st1a)
template <bool HS>
MEP_DEV aelem<HS>* rowa(const mep_rows& r, int tok) {
    return reinterpret_cast<aelem<HS>*>(r.ptr) + row_off(r, tok);
}

// ------------------------------------------------------------------ exact-rounding scalar ops
// The residual-score sequence of the reference ((q.k)/sqrt(d) + c*S_prev - 1e8*(1-m)) is
// evaluated with one rounding per op, no FMA contraction (masked slots sit at ~1e8 where
// ulp = 8).  __fadd_rn / __fmul_rn do not stop hipcc from fusing a product into the
// following sum (v_fmac_f32: one rounding fewer, a different grid value at ~1e8); the operations
// below are compiled with contraction off, so they keep their own rounding after inlining.
MEP_DEV float add_rn(float a, float b) {
#pragma clang fp contract(off)
    return a + b;
}
MEP_DEV float sub_rn(float a, float b) {
#pragma clang fp contract(off)
    return a - b;
}
MEP_DEV float mul_rn(float a, float b) {
#pragma clang fp contract(off)
    return a * b;
}

// ------------------------------------------------------------------ wave reductions (64 lanes)
// DPP within each row of 16 lanes (quad butterflies xor 1 / xor 2, then the half-row and row
// mirrors), then the four row results through readlane, combined as (r0 + r1) + (r2 + r3): no
// LDS round trips (ds_bpermute), result wave-uniform, fixed order.
// update_dpp with old = 0 and bound_ctrl set: the same lanes move (every source lane of these
// row-local patterns is valid), and the form lets the compiler fold the move into the consuming
// add as one v_add_f32_dpp (half the instructions of v_mov_b32_dpp + v_add_f32)
template <int CTRL>
MEP_DEV float dpp_mov(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
MEP_DEV float lane_f(float v, int l) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l)); }
MEP_DEV float wave_sum(float v) {
    v += dpp_mov<0xB1>(v);
    v += dpp_mov<0x4E>(v);
    v += dpp_mov<0x141>(v);
    v += dpp_mov<0x140>(v);
    return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
MEP_DEV float wave_max(float v) {
    v = fmaxf(v, dpp_mov<0xB1>(v));
    v = fmaxf(v, dpp_mov<0x4E>(v));
    v = fmaxf(v, dpp_mov<0x141>(v));
    v = fmaxf(v, dpp_mov<0x140>(v));
    return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}

// ------------------------------------------------------------------ counter-based dropout
MEP_DEV uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27; x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}
// 32-bit avalanche hash (two multiplies): the per-element part of the dropout hash
MEP_DEV uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du;
    x ^= x >> 15; x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
// keep-scale for element `idx` of dropout stream `stream`: 0 (dropped) or 1/(1-p).  The stream's
// 32-bit key is one 64-bit mix of (seed, stream) -- loop-invariant, hoisted out of the element
// loops -- and each element costs two 32-bit hashes of its index halves (four 32-bit multiplies;
// round 3's two 64-bit mixes per element were most of the dropout epilogues' instructions).
// Restated bit for bit by oracle/dropout.py keep_scale.
MEP_DEV float drop_scale(uint64_t seed, uint32_t stream, uint64_t idx, float p) {
    const uint32_t key = (uint32_t)mix64(seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(stream + 1)));
    const uint32_t h = lowbias32((uint32_t)idx ^ lowbias32((uint32_t)(idx >> 32) ^ key));
    const float u = (float)(h >> 8) * (1.0f / 16777216.0f);
    return u >= p ? 1.0f / (1.0f - p) : 0.0f;
}

// The forward's keep bits of a 16-token tile and dropout site (mep_epi_desc.drop_bits): one
// dword per lane, bit 4 i + r = element (feature 16 i + 4 g + r, token 16 tile + c) kept.
MEP_DEV gfloat* drop_bits_ptr(uint64_t base, int tok, int site) {
    return base ? G<float>(base) + ((tok >> 4) * 2 + site) * 64 + (threadIdx.x & 63) : nullptr;
}
// forward: the hash's scale, recording the keep bit
MEP_DEV float drop_rec(uint64_t seed, uint32_t stream, uint64_t idx, float p, uint32_t& bits, int pos) {
    const float s = drop_scale(seed, stream, idx, p);
    bits |= (s != 0.f ? 1u : 0u) << pos;
    return s;
}
MEP_DEV void drop_bits_put(gfloat* bp, uint32_t bits) {
    if (bp) *bp = __builtin_bit_cast(float, bits);
}
MEP_DEV uint32_t drop_bits_get(const gfloat* bp) { return bp ? __builtin_bit_cast(uint32_t, *bp) : 0u; }
// backward: the scale from the forward's bits (the same value as drop_scale: 1/(1-p) or 0), or the
// hash when there are none
MEP_DEV float drop_use(bool have, uint32_t bits, int pos, float keep, uint64_t seed, uint32_t stream, uint64_t idx, float p) {
    return have ? (((bits >> pos) & 1u) ? keep : 0.0f) : drop_scale(seed, stream, idx, p);
}

// ------------------------------------------------------------------ f32 MFMA 32x32x2
// lane l supplies A[l&31][k], B[k][l&31] with k = l>>5 of the 2-wide step; C/D register r of
// lane l is C[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31].
MEP_DEV floatx16 mfma32(float a, float b, floatx16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
MEP_DEV int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// acc += A_lds[m0 .. m0+31][0 .. kc) * W(n0 .. n0+31, k0 .. k0+kc)
// A_lds: row-major [64][lda] tile in LDS, zero beyond the valid K range.
// K is traversed in groups of 8: lane half h covers k = 8g + 4h + j at step 4g + j (the sum
// over k is order-free; this lets each lane fetch 4 consecutive k with one 16-byte read).
// W(n,k): NT -> W[n*ldw + k] (nn.Linear weight), else W[k*ldw + n].
// KC > 0: compile-time chunk width (fully unrolled, so hipcc issues every weight load of the
// chunk ahead of the MFMA chain); KC == 0: runtime width kc.
template <bool NT>
MEP_DEV void mma_step(floatx16& acc, const float* __restrict__ arow, const gfloat* __restrict__ W, int ldw, int n,
                      bool nval, int kk, int kg, int K, bool w_vec) {
    const float4 a = *reinterpret_cast<const float4*>(arow + kk);
    float b0 = 0.f, b1 = 0.f, b2 = 0.f, b3 = 0.f;
    if (NT) {
        const gfloat* wp = W + (int64_t)n * ldw + kg;
        if (nval && w_vec && kg + 3 < K) {
            const float4 b = ldg4(wp);
            b0 = b.x; b1 = b.y; b2 = b.z; b3 = b.w;
        } else if (nval) {
            if (kg < K) b0 = wp[0];
            if (kg + 1 < K) b1 = wp[1];
            if (kg + 2 < K) b2 = wp[2];
            if (kg + 3 < K) b3 = wp[3];
        }
    } else {
        if (nval) {
            const gfloat* wp = W + (int64_t)kg * ldw + n;
            if (kg < K) b0 = wp[0];
            if (kg + 1 < K) b1 = wp[ldw];
            if (kg + 2 < K) b2 = wp[2 * ldw];
            if (kg + 3 < K) b3 = wp[3 * ldw];
        }
    }
    acc = mfma32(a.x, b0, acc);
    acc = mfma32(a.y, b1, acc);
    acc = mfma32(a.z, b2, acc);
    acc = mfma32(a.w, b3, acc);
}

template <bool NT, int KC = 0>
MEP_DEV void mma_tile(floatx16& acc, const float* __restrict__ As, int lda, int m0,
                      const gfloat* __restrict__ W, int ldw, int n0, int N, int k0, int kc, int K,
                      bool w_vec) {
    const int lane = threadIdx.x & 63;
    const int r = lane & 31;
    const int h = lane >> 5;
    const float* arow = As + (m0 + r) * lda + 4 * h;
    const int n = n0 + r;
    const bool nval = n < N;
    if (KC > 0) {
#pragma unroll
        for (int kk = 0; kk < KC; kk += 8) mma_step<NT>(acc, arow, W, ldw, n, nval, kk, k0 + kk + 4 * h, K, w_vec);
    } else {
        for (int kk = 0; kk < kc; kk += 8) mma_step<NT>(acc, arow, W, ldw, n, nval, kk, k0 + kk + 4 * h, K, w_vec);
    }
}

// mma_tile with the weight operand of the whole K range fetched into registers before the first
// MFMA (KC / 8 x 16 bytes per lane): the L2 latency of the weight reads is paid once per tile
// instead of once per k-step (hipcc otherwise sinks each load next to its MFMA).
template <bool NT, int KC>
MEP_DEV void mma_tile_pf(floatx16& acc, const float* __restrict__ As, int lda, int m0,
                         const gfloat* __restrict__ W, int ldw, int n0, int N, int k0, int K, bool w_vec) {
    static_assert(KC % 8 == 0, "KC must be a multiple of 8");
    constexpr int NS = KC / 8;
    const int lane = threadIdx.x & 63;
    const int r = lane & 31;
    const int h = lane >> 5;
    const float* arow = As + (m0 + r) * lda + 4 * h;
    const int n = n0 + r;
    const bool nval = n < N;
    float4 b[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        const int kg = k0 + 8 * i + 4 * h;
        float b0 = 0.f, b1 = 0.f, b2 = 0.f, b3 = 0.f;
        if (NT) {
            const gfloat* wp = W + (int64_t)n * ldw + kg;
            if (nval && w_vec && kg + 3 < K) {
                const float4 v = ldg4(wp);
                b0 = v.x; b1 = v.y; b2 = v.z; b3 = v.w;
            } else if (nval) {
                if (kg < K) b0 = wp[0];
                if (kg + 1 < K) b1 = wp[1];
                if (kg + 2 < K) b2 = wp[2];
                if (kg + 3 < K) b3 = wp[3];
            }
        } else if (nval) {
            const gfloat* wp = W + (int64_t)kg * ldw + n;
            if (kg < K) b0 = wp[0];
            if (kg + 1 < K) b1 = wp[ldw];
            if (kg + 2 < K) b2 = wp[2 * ldw];
            if (kg + 3 < K) b3 = wp[3 * ldw];
        }
        b[i] = make_float4(b0, b1, b2, b3);
    }
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        const float4 a = *reinterpret_cast<const float4*>(arow + 8 * i);
        acc = mfma32(a.x, b[i].x, acc);
        acc = mfma32(a.y, b[i].y, acc);
        acc = mfma32(a.z, b[i].z, acc);
        acc = mfma32(a.w, b[i].w, acc);
    }
}

MEP_DEV floatx16 zero16() {
    floatx16 z;
#pragma unroll
    for (int i = 0; i < 16; ++i) z[i] = 0.f;
    return z;
}

// Cooperative load of rows [tok0, tok0+64) x cols [c0, c0+kc) of a row view into an LDS tile
// [64][lda]; out-of-range rows/cols are zero.  kc_pad (multiple of 8) columns are written.
MEP_DEV void load_tile(float* __restrict__ dst, int lda, const mep_rows& src, int tok0, int ntok,
                       int c0, int kc, int kc_pad, int ncol_total) {
    const int nth = blockDim.x;
    for (int idx = threadIdx.x; idx < 64 * kc_pad; idx += nth) {
        const int row = idx / kc_pad;
        const int col = idx - row * kc_pad;
        const int tok = tok0 + row;
        const int c = c0 + col;
        float v = 0.f;
        if (tok < ntok && col < kc && c < ncol_total) v = row_ptr(src, tok)[c];
        dst[row * lda + col] = v;
    }
}

// Stage rows [t0, t0+TT) x columns [c0, c0+nc) of a row view into LDS (row stride ld floats);
// rows at or beyond t_end are zero.  16-byte loads/stores whenever the view allows it, one
// row-address computation per 4 columns.
template <int TT>
MEP_DEV void stage_cols(float* __restrict__ dst, int ld, const mep_rows& src, int t0, int t_end, int c0, int nc) {
    const bool vec = (nc % 4 == 0) && (c0 % 4 == 0) && (ld % 4 == 0) && ((src.ptr & 15) == 0) &&
                     (src.sB % 4 == 0) && (src.sT % 4 == 0) && ((reinterpret_cast<uintptr_t>(dst) & 15) == 0);
    if (vec) {
        const int nc4 = nc >> 2;
        for (int s = threadIdx.x; s < TT * nc4; s += blockDim.x) {
            const int row = s / nc4, c = 4 * (s - row * nc4);
            const int tok = t0 + row;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (tok < t_end) v = ldg4(row_ptr(src, tok) + c0 + c);
            *reinterpret_cast<float4*>(dst + row * ld + c) = v;
        }
    } else {
        for (int s = threadIdx.x; s < TT * nc; s += blockDim.x) {
            const int row = s / nc, c = s - row * nc;
            const int tok = t0 + row;
            dst[row * ld + c] = tok < t_end ? row_ptr(src, tok)[c0 + c] : 0.f;
        }
    }
}

// ------------------------------------------------------------------ wave-level 16-row GEMM tiles
// v_mfma_f32_16x16x4_f32: lane l = (c = l & 15, g = l >> 4) supplies A[c][k] and B[k][c] for the
// k-slot g of a 4-wide step, and holds C[4g + r][c] (r < 4).  Reduction indices are ordered
// (step s, slot g) -> 4g + s within each 16-wide k block, so every operand fetch is one 16-byte
// read of 4 consecutive k.
MEP_DEV f32x4 mfma16x4(float a, float b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
MEP_DEV f32x4 zero_f4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// LDS writes of this wave visible to all of its lanes (no other wave involved)
MEP_DEV void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// weight operand of k block kb for output column block j:
//   NT: W[n][k] = W[n * ldw + k] (nn.Linear weight, forward);  else W[k][n] = W[k * ldw + n]
template <bool NT>
MEP_DEV float4 wfrag(const gfloat* W, int ldw, int n, int k, bool w_vec) {
    if (NT) {
        const gfloat* p = W + (int64_t)n * ldw + k;
        if (w_vec) return ldg4(p);
        return make_float4(p[0], p[1], p[2], p[3]);
    }
    const gfloat* p = W + (int64_t)k * ldw + n;
    return make_float4(p[0], p[ldw], p[2 * ldw], p[3 * ldw]);
}

// acc[j] += A[16 x K] . W(cols n0 + 16j .. + 15)   for j < NJ.  A: 16 rows in LDS, row c at
// A + c * lda.  Per 16-wide k block all NJ accumulators are advanced (4 NJ MFMAs, 128 NJ cycles
// of MFMA issue), and the NJ weight fragments of the NEXT k block are loaded before them, so
// one k block of MFMA work covers the L2 latency of the next block's weights.
template <int NJ, int K, bool NT>
MEP_DEV void wgemm16(f32x4 (&acc)[NJ], const float* A, int lda, const gfloat* W, int ldw, int n0, bool w_vec) {
    static_assert(K % 16 == 0, "K must be a multiple of 16");
    constexpr int KB = K / 16;
    const int lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const float* arow = A + c * lda + 4 * g;
    float4 b[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) b[j] = wfrag<NT>(W, ldw, n0 + 16 * j + c, 4 * g, w_vec);
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
        float4 cur[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) cur[j] = b[j];
        if (kb + 1 < KB) {
#pragma unroll
            for (int j = 0; j < NJ; ++j) b[j] = wfrag<NT>(W, ldw, n0 + 16 * j + c, 16 * (kb + 1) + 4 * g, w_vec);
        }
        const float4 a = *reinterpret_cast<const float4*>(arow + 16 * kb);
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[j] = mfma16x4(a.x, cur[j].x, acc[j]);
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[j] = mfma16x4(a.y, cur[j].y, acc[j]);
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[j] = mfma16x4(a.z, cur[j].z, acc[j]);
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[j] = mfma16x4(a.w, cur[j].w, acc[j]);
    }
}

// ------------------------------------------------------------------ transposed 16-token tiles
// Products over a tile of 16 tokens are formed TRANSPOSED: Y^T = W X^T with the output features
// on the MFMA rows and the tokens on its columns (v_mfma_f32_16x16x4_f32, exact fp32).  Lane
// (c = lane & 15, g = lane >> 4) then holds features 16i + 4g .. +3 of token c in accumulator i,
// which is exactly the B operand of the next product over those features (k block i, k = 4g + s),
// so chained Linears pass activations in registers; a token's row statistics are an in-lane sum
// plus two shuffles, and its stores are 16-byte stores.  Weights are the A operand, read as one
// float4 (4 consecutive k of row 16i + c) per (output tile, k block) from LDS or global memory.
typedef __attribute__((address_space(3))) float lfloat;
typedef __attribute__((address_space(3))) f32x4 lf32x4;

MEP_DEV f32x4 ld4w(const lfloat* p) { return *reinterpret_cast<const lf32x4*>(p); }
MEP_DEV f32x4 ld4w(const gfloat* p) { return *reinterpret_cast<const MEP_G f32x4*>(p); }

// acc[i] (i < NI) += sum over KB k blocks of A_i,kb[c][4g + s] * B_kb[4g + s][c]:
// afr(i, kb) yields the lane's A values (row 16i + c of the weight operand, k = 16kb + 4g + s),
// bfr(kb) its B values (token c, k = 16kb + 4g + s).  The NI A fragments of a k block are read
// before its 4*NI MFMAs, which are issued s-major so consecutive MFMAs never chain on one
// accumulator.
template <int NI, int KB, typename AF, typename BF>
MEP_DEV void tgemm(f32x4 (&acc)[NI], AF&& afr, BF&& bfr) {
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
        const f32x4 b = bfr(kb);
        f32x4 a[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) a[i] = afr(i, kb);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int i = 0; i < NI; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[s], acc[i], 0, 0, 0);
        // keep the next block's fragment reads behind this block's MFMAs (a fully hoisted,
        // fully unrolled product holds 4 * NI * KB fragment VGPRs)
        __builtin_amdgcn_sched_barrier(0);
    }
}

// A accessors of tgemm over a weight W [R][C] (row stride ld):
//   rows of W     : A row n = W row row0 + n, k = W column pos0 + k        (x W^T)
//   rows of W^T   : A row n = W column row0 + n, k = W row pos0 + k        (dy W)
template <typename T>
struct WRows {
    const T* w;
    int ld, row0, pos0;
    MEP_DEV f32x4 operator()(int i, int kb) const {
        const int lane = threadIdx.x & 63;
        return ld4w(w + (row0 + 16 * i + (lane & 15)) * ld + pos0 + 16 * kb + 4 * (lane >> 4));
    }
};
struct WCols {
    const gfloat* w;
    int ld, row0, pos0;
    MEP_DEV f32x4 operator()(int i, int kb) const {
        const int lane = threadIdx.x & 63;
        const gfloat* p = w + (pos0 + 16 * kb + 4 * (lane >> 4)) * ld + row0 + 16 * i + (lane & 15);
        return f32x4{p[0], p[ld], p[2 * ld], p[3 * ld]};
    }
};

// sum over the 16 lanes of a DPP row (lanes sharing g = lane >> 4), result in every lane: quad
// butterflies (xor 1, xor 2), then the half-row and row mirrors pair the quads
MEP_DEV float row16_sum(float v) {
    v += dpp_mov<0xB1>(v);
    v += dpp_mov<0x4E>(v);
    v += dpp_mov<0x141>(v);
    v += dpp_mov<0x140>(v);
    return v;
}

// sum over the 16 lanes of a lane group (lanes sharing g = lane >> 4)
MEP_DEV float group16_sum(float v) {
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    return v;
}

// stage rows [r0, r0 + 16) of a row view (D columns) into LDS rows of stride lda, one wave;
// rows >= ntok are zero
template <int D>
MEP_DEV void wave_stage16(float* dst, int lda, const mep_rows& src, int r0, int ntok) {
    const int lane = threadIdx.x & 63;
    constexpr int V = D / 4;
    const bool vec = ((src.ptr & 15) == 0) && (src.sB % 4 == 0) && (src.sT % 4 == 0);
    for (int idx = lane; idx < 16 * V; idx += 64) {
        const int row = idx / V, c4 = idx - row * V;
        const int tok = r0 + row;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (tok < ntok) {
            const gfloat* p = row_ptr(src, tok) + 4 * c4;
            v = vec ? ldg4(p) : make_float4(p[0], p[1], p[2], p[3]);
        }
        *reinterpret_cast<float4*>(dst + row * lda + 4 * c4) = v;
    }
}

// store rows [r0, r0 + 16) (those < ntok) of an LDS tile to a row view, one wave, 16-byte stores
template <int D>
MEP_DEV void wave_store16(const float* src, int lda, const mep_rows& dst, int r0, int ntok) {
    const int lane = threadIdx.x & 63;
    constexpr int V = D / 4;
    const bool vec = ((dst.ptr & 15) == 0) && (dst.sB % 4 == 0) && (dst.sT % 4 == 0);
    for (int idx = lane; idx < 16 * V; idx += 64) {
        const int row = idx / V, c4 = idx - row * V;
        const int tok = r0 + row;
        if (tok >= ntok) continue;
        const float4 v = *reinterpret_cast<const float4*>(src + row * lda + 4 * c4);
        gfloat* p = row_ptr(dst, tok) + 4 * c4;
        if (vec) stg4(p, v);
        else { p[0] = v.x; p[1] = v.y; p[2] = v.z; p[3] = v.w; }
    }
}


// ------------------------------------------------------------------ gradient reductions
// Block bodies shared by their own launches and the fused mep_reduce_grads launch (256 threads).
// Weight-gradient split sum (gemm.hip k_wgrad_reduce): block bx of descriptor d sums the
// n_split partials of WG_RED_PER = 1024 consecutive (n, k) entries in a fixed order, 4 per thread
// (one 16-byte load per partial when N * Ktot and the workspace allow it; hosts count tiles of
// 256 entries, the launches run cdiv(tiles, 4) blocks: wg_red_blocks).
// Each returns the sum of squares of the gradient values its thread wrote (the fused gradient-norm
// partials of mep_reduce_grads; ignored by the standalone launches).
constexpr int WG_RED_PER = 1024;
__host__ __device__ inline int wg_red_blocks(int tiles256) { return (tiles256 + 3) / 4; }

// A descriptor's output operands in registers, and dW_i's address of entry (n, k of the
// concatenated K).  Looked up per entry from the descriptor in memory, the operand index made
// every lookup a per-lane load -- and behind the previous entry's store such a load waits for that
// store too (vmcnt counts both), so each entry of a reduction cost a memory round trip.
struct WgOuts {
    uint64_t out[MEP_WG_MAX_B];
    int kb[MEP_WG_MAX_B], ldo[MEP_WG_MAX_B];
    int n_b, trans;
    MEP_DEV explicit WgOuts(const mep_wgrad_desc& d) : n_b(d.n_b), trans(d.out_trans) {
#pragma unroll
        for (int j = 0; j < MEP_WG_MAX_B; ++j) { out[j] = d.out[j]; kb[j] = d.kb[j]; ldo[j] = d.ldo[j]; }
    }
    MEP_DEV gfloat* at(int n, int k) const {
        int j = 0;
#pragma unroll
        for (int q = 0; q < MEP_WG_MAX_B - 1; ++q) {   // the first operand whose columns hold k
            const bool adv = j == q && q < n_b - 1 && k >= kb[q];
            k -= adv ? kb[q] : 0;
            j += adv ? 1 : 0;
        }
        uint64_t o = out[0];
        int ld = ldo[0];
#pragma unroll
        for (int q = 1; q < MEP_WG_MAX_B; ++q) {
            o = j == q ? out[q] : o;
            ld = j == q ? ldo[q] : ld;
        }
        return G<float>(o) + (trans ? (int64_t)k * ld + n : (int64_t)n * ld + k);
    }
};

MEP_DEV float wgrad_reduce_block(const mep_wgrad_desc& d, int bx) {
    const int64_t nk = (int64_t)d.N * d.Ktot;
    const int64_t i0 = (int64_t)bx * WG_RED_PER + 4 * threadIdx.x;
    if (i0 >= nk) return 0.f;
    const gfloat* part = G<const float>(d.partial);
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    const int cnt = (int)min((int64_t)4, nk - i0);
    if (cnt == 4 && (nk & 3) == 0 && (d.partial & 15) == 0) {
#pragma unroll 8
        for (int sp = 0; sp < d.n_split; ++sp) {
            const f32x4 v = *reinterpret_cast<const __attribute__((address_space(1))) f32x4*>(part + sp * nk + i0);
#pragma unroll
            for (int e = 0; e < 4; ++e) s[e] += v[e];
        }
    } else {
        for (int e = 0; e < cnt; ++e) {
            float t = 0.f;
            for (int sp = 0; sp < d.n_split; ++sp) t += part[sp * nk + i0 + e];
            s[e] = t;
        }
    }
    float sq = 0.f;
    const WgOuts wo(d);
    const bool acc = d.accumulate != 0;
    gfloat* o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {   // every address before the first store
        const int64_t i = i0 + min(e, cnt - 1);
        const int n = (int)(i / d.Ktot);
        o[e] = wo.at(n, (int)(i - (int64_t)n * d.Ktot));
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        if (e < cnt) {
            const float v = acc ? *o[e] + s[e] : s[e];
            *o[e] = v;
            sq += v * v;
        }
    }
    return sq;
}

// Column sums of a partial matrix (optim.hip k_colsum): block bx = 32 columns.  16-byte rows
// (ld, n_cols multiples of 4, aligned): 8 lanes x 4 columns x 32 row groups, each thread's rows
// loaded at once, the 32 groups combined in a fixed order; else 32 columns x 8 row groups.
MEP_DEV float colsum_block(const mep_colsum_desc& d, int bx) {
    if (bx * 32 >= d.n_cols) return 0.f;   // whole block
    __shared__ float red[32][33];
    const bool v4 = (d.ld % 4 == 0) && (d.n_cols % 4 == 0) && (d.partial & 15) == 0;
    if (v4) {
        const int q = threadIdx.x & 7, g = threadIdx.x >> 3;
        const int c0 = bx * 32 + 4 * q;
        f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
        if (c0 < d.n_cols) {
            const gfloat* p = G<const float>(d.partial) + c0;
#pragma unroll 16
            for (int r = g; r < d.n_rows; r += 32)
                s += *reinterpret_cast<const __attribute__((address_space(1))) f32x4*>(p + (int64_t)r * d.ld);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) red[g][4 * q + e] = s[e];
    } else {
        const int cl = threadIdx.x & 31, g = threadIdx.x >> 5;
        const int c = bx * 32 + cl;
        float s = 0.f;
        if (c < d.n_cols) {
            const gfloat* p = G<const float>(d.partial) + c;
#pragma unroll 8
            for (int r = g; r < d.n_rows; r += 8) s += p[(int64_t)r * d.ld];
        }
        red[g][cl] = s;
    }
    __syncthreads();
    const int cl = threadIdx.x;
    const int c = bx * 32 + cl;
    if (cl < 32 && c < d.n_cols) {
        float t = 0.f;
        const int ng = v4 ? 32 : 8;
        for (int k = 0; k < ng; ++k) t += red[k][cl];
        gfloat* o = G<float>(d.out) + c;
        const float v = (d.accumulate & 1) ? *o + t : t;
        *o = v;
        return (d.accumulate & MEP_COLSUM_NOT_GRAD) ? 0.f : v * v;
    }
    return 0.f;
}

// clip + optimizer workspace (optim.hip): per-workgroup g^2 partials of the norm pass in
// [0, OPT_NPART), the step's scalars at OPT_SCAL (lr / (1 - b1^t), sqrt(1 - b2^t)), and from
// OPT_EXT0 the partials of a mep_reduce_grads launch that folded the norm pass in
constexpr int OPT_NPART = 1016, OPT_SCAL = OPT_NPART, OPT_EXT0 = 1024;

// the step counter and the bias corrections (double pow) once per step: one thread of one workgroup
MEP_DEV void opt_step_scalars(float* partial, int* step, const float* hyper) {
    const int ts = step[0] + 1;
    step[0] = ts;
    const double lr = hyper[0], b1 = hyper[1], b2 = hyper[2];
    partial[OPT_SCAL] = (float)(lr / (1.0 - pow(b1, (double)ts)));
    partial[OPT_SCAL + 1] = (float)sqrt(1.0 - pow(b2, (double)ts));
}

}  // namespace mep

// error plumbing shared by the launchers (api.cpp)
extern "C" void mep_set_error(const char* msg);
int mep_check_launch(const char* what);

