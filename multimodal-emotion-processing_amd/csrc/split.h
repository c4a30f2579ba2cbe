// fp32 products on the bf16 matrix cores (v_mfma_f32_16x16x32_bf16) with every fp32 operand
// split into bf16 parts: x = x0 + x1 + x2 (+ r), each part the round-to-nearest bf16 of the
// remainder, |r| <= 2^-27 |x|.  Products of bf16 parts are exact in the fp32 accumulator, so the
// six products x_i y_j with i + j <= 2 give an fp32-level result (dropped terms <= ~2^-25
// relative) at 6 x 16 = 96 MFMA cycles per 16 x 16 x 32 step, against 8 x 32 = 256 cycles for
// the same step on v_mfma_f32_16x16x4_f32 (1/16 of the bf16 rate on gfx950).
//
// Slot convention of the 16x16x32 operands: lane (c = lane & 15, g = lane >> 4) supplies
// A[row c][8 slots] and B[8 slots][col c]; the result is C[4g + r][c] (the layout of the fp32
// 16x16x4 form).  Which contraction index a slot carries is free as long as A and B agree: here
// slots 0-3 carry indices 4g..4g+3 of one 16-wide k block and slots 4-7 the same positions of a
// second block (a "k pair"), so each half is the 16-byte fragment the fp32 form would load.
#pragma once
#include "common.h"

namespace mep {

typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// two fp32 -> one word of two round-to-nearest bf16 (v_cvt_pk_bf16_f32)
MEP_DEV unsigned pk_bf16(float a, float b) {
    return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2v{a, b}, bf16x2v));
}
MEP_DEV float bf16_lo(unsigned p) { return __builtin_bit_cast(float, p << 16); }
MEP_DEV float bf16_hi(unsigned p) { return __builtin_bit_cast(float, p & 0xffff0000u); }

// the three parts of 4 fp32 values, two words (4 bf16) per part
struct Parts3 { u32x2 p0, p1, p2; };

MEP_DEV Parts3 split3v(f32x4 x) {
    Parts3 s;
    s.p0 = u32x2{pk_bf16(x[0], x[1]), pk_bf16(x[2], x[3])};
    const float r0 = x[0] - bf16_lo(s.p0[0]), r1 = x[1] - bf16_hi(s.p0[0]);   // exact remainders
    const float r2 = x[2] - bf16_lo(s.p0[1]), r3 = x[3] - bf16_hi(s.p0[1]);
    s.p1 = u32x2{pk_bf16(r0, r1), pk_bf16(r2, r3)};
    s.p2 = u32x2{pk_bf16(r0 - bf16_lo(s.p1[0]), r1 - bf16_hi(s.p1[0])), pk_bf16(r2 - bf16_lo(s.p1[1]), r3 - bf16_hi(s.p1[1]))};
    return s;
}

// operand of a k pair: part words of block 0 in slots 0-3, of block 1 in slots 4-7
MEP_DEV bf16x8 kpair(u32x2 lo, u32x2 hi) { return __builtin_bit_cast(bf16x8, u32x4{lo[0], lo[1], hi[0], hi[1]}); }

struct Op3 { bf16x8 p0, p1, p2; };   // the three parts of a k-pair operand

MEP_DEV Op3 op3(f32x4 blk0, f32x4 blk1) {
    const Parts3 a = split3v(blk0), b = split3v(blk1);
    return Op3{kpair(a.p0, b.p0), kpair(a.p1, b.p1), kpair(a.p2, b.p2)};
}

MEP_DEV f32x4 mfma_bf16(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }

// acc += A B over one k pair, the six products with i + j <= 2
MEP_DEV f32x4 mma6(const Op3& a, const Op3& b, f32x4 acc) {
    acc = mfma_bf16(a.p0, b.p0, acc);
    acc = mfma_bf16(a.p1, b.p0, acc);
    acc = mfma_bf16(a.p0, b.p1, acc);
    acc = mfma_bf16(a.p1, b.p1, acc);
    acc = mfma_bf16(a.p2, b.p0, acc);
    acc = mfma_bf16(a.p0, b.p2, acc);
    return acc;
}

// ---------------------------------------------------------------- split weights in LDS
// A weight operand of R rows (output features) and K = 32 * NP contraction indices kept in LDS
// as its three bf16 parts: part t, row n, k pair p, lane group g is the 16-byte unit at
//   base + t * R * RS + n * RS + (4 p + g) * 16,      RS = 64 NP + 32 bytes (two units of padding:
// with a row stride of 16 NP + 8 dwords every 16-lane group of a ds_read_b128 fragment read --
// rows c, units g -- covers the 64 banks exactly once, for every NP).  A fragment read is one
// ds_read_b128 per part.
template <int R, int NP>
struct SplitW {
    static constexpr int RS = 64 * NP + 32;
    static constexpr int BYTES = 3 * R * RS;
    __attribute__((address_space(3))) unsigned char* base;
    int row0;   // first row of the operand (output tile 0)
    MEP_DEV Op3 frag(int i, int p) const {
        const int lane = threadIdx.x & 63;
        const int off = (row0 + 16 * i + (lane & 15)) * RS + (4 * p + (lane >> 4)) * 16;
        typedef __attribute__((address_space(3))) u32x4 lu32x4;
        const u32x4 a = *reinterpret_cast<const lu32x4*>(base + off);
        const u32x4 b = *reinterpret_cast<const lu32x4*>(base + R * RS + off);
        const u32x4 c = *reinterpret_cast<const lu32x4*>(base + 2 * R * RS + off);
        return Op3{__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), __builtin_bit_cast(bf16x8, c)};
    }
    // write the unit (n, p, g) from the 8 fp32 values of its two k blocks
    MEP_DEV void put(int n, int p, int g, f32x4 blk0, f32x4 blk1) const {
        const Parts3 a = split3v(blk0), b = split3v(blk1);
        typedef __attribute__((address_space(3))) u32x4 lu32x4;
        const int off = n * RS + (4 * p + g) * 16;
        *reinterpret_cast<lu32x4*>(base + off) = u32x4{a.p0[0], a.p0[1], b.p0[0], b.p0[1]};
        *reinterpret_cast<lu32x4*>(base + R * RS + off) = u32x4{a.p1[0], a.p1[1], b.p1[0], b.p1[1]};
        *reinterpret_cast<lu32x4*>(base + 2 * R * RS + off) = u32x4{a.p2[0], a.p2[1], b.p2[0], b.p2[1]};
    }
};

// acc[i] (i < NI) += A_i B over NP k pairs: afr(i, p) -> Op3 (A fragment of output tile i),
// bfr(p) -> Op3 (B fragment, shared by the NI tiles).
#ifndef MEP_TG6
#define MEP_TG6 0
#endif
template <int NI, int NP, typename AF, typename BF>
MEP_DEV void tgemm6(f32x4 (&acc)[NI], AF&& afr, BF&& bfr) {
#if MEP_TG6 == 2
    // output tiles in pairs, the six products of the two tiles interleaved
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const Op3 b = bfr(p);
#pragma unroll
        for (int i = 0; i < NI; i += 2) {
            const Op3 a0 = afr(i, p), a1 = afr(i + 1, p);
            acc[i] = mfma_bf16(a0.p0, b.p0, acc[i]);
            acc[i + 1] = mfma_bf16(a1.p0, b.p0, acc[i + 1]);
            acc[i] = mfma_bf16(a0.p1, b.p0, acc[i]);
            acc[i + 1] = mfma_bf16(a1.p1, b.p0, acc[i + 1]);
            acc[i] = mfma_bf16(a0.p0, b.p1, acc[i]);
            acc[i + 1] = mfma_bf16(a1.p0, b.p1, acc[i + 1]);
            acc[i] = mfma_bf16(a0.p1, b.p1, acc[i]);
            acc[i + 1] = mfma_bf16(a1.p1, b.p1, acc[i + 1]);
            acc[i] = mfma_bf16(a0.p2, b.p0, acc[i]);
            acc[i + 1] = mfma_bf16(a1.p2, b.p0, acc[i + 1]);
            acc[i] = mfma_bf16(a0.p0, b.p2, acc[i]);
            acc[i + 1] = mfma_bf16(a1.p0, b.p2, acc[i + 1]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#else
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const Op3 b = bfr(p);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            acc[i] = mma6(afr(i, p), b, acc[i]);
            // keep the next fragment's reads behind these MFMAs (a fully hoisted, fully unrolled
            // product would hold 12 NI NP fragment VGPRs)
            if (MEP_TG6 == 0 && i % 2 == 1) __builtin_amdgcn_sched_barrier(0);
        }
    }
#endif
}

}  // namespace mep
