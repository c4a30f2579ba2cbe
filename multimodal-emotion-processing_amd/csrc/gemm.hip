// Token GEMM (nn.Linear over token rows, fp32 MFMA 16x16x4) and weight-gradient GEMM (bf16 MFMA
// 32x32x16 on split or plain bf16 operands).
//
// mep_gemm : Y[tok, n] = act(alpha * X[tok,:] . W(n,:) + bias[n] + table[tok % T, n]) (+Y)
//            one workgroup = 64 tokens x all N columns; 8 waves; task (m-half, 32-col block)
//            round-robin over waves; A staged through LDS in 128-wide K chunks, W read from
//            L2 with 16-byte loads.  Replaces Unify_Dimension's Linear (cmu-mosei/run.py:210-214),
//            the Conv1d k=1 unify + position add (others/realformer.py:136-152,224-227) and the
//            realformer w_qkv / FFN Linears (others/realformer.py:157,163-168).
// mep_wgrad: dW_i = A^T B_i over token chunks (see the kernel comment below).
#include "common.h"
#include "split.h"

#include <type_traits>

using namespace mep;

namespace {

// One WAVE = 16 tokens x one pass of 16 * GEMM_NJ columns (passes over grid.z, then strided); 4
// independent waves per workgroup of 64 tokens, no block barriers.  v_mfma_f32_16x16x4_f32 with the wave's A rows staged in its own LDS
// slice (128-wide K chunks, zero-padded past K and past the last token) and the weight fragments
// of the next 16-wide k block loaded during the MFMAs of the current one.  Per lane: acc[j] holds
// rows 4g..4g+3 of column block j (c = lane & 15, g = lane >> 4; common.h wgemm16 layout).
constexpr int GEMM_WAVES = 4;
constexpr int GEMM_THREADS = 64 * GEMM_WAVES;
constexpr int GEMM_KC = 128;
constexpr int GEMM_LDA = GEMM_KC + 4;
#ifndef MEP_GEMM_NJ
#define MEP_GEMM_NJ 1
#endif
constexpr int GEMM_NJ = MEP_GEMM_NJ;   // 16-column blocks per pass
#ifndef MEP_GEMM_ZP
#define MEP_GEMM_ZP 32
#endif
constexpr int GEMM_ZP = MEP_GEMM_ZP;             // column passes spread over grid.z (more waves in flight)

// weight fragment W(n, k .. k+3) with k clamped into [0, K) and n into [0, N): the clamped
// values meet zero A columns (k >= K) or are never stored (n >= N), so they only need to be finite
MEP_DEV float4 gemm_wfrag(const gfloat* W, int ldw, bool nt, bool vec, int n, int N, int k, int K) {
    n = min(n, N - 1);
    if (nt) {
        const gfloat* p = W + (int64_t)n * ldw;
        if (vec && k + 3 < K) return ldg4(p + k);
        return make_float4(p[min(k, K - 1)], p[min(k + 1, K - 1)], p[min(k + 2, K - 1)], p[min(k + 3, K - 1)]);
    }
    const gfloat* p = W + n;
    return make_float4(p[(int64_t)min(k, K - 1) * ldw], p[(int64_t)min(k + 1, K - 1) * ldw],
                       p[(int64_t)min(k + 2, K - 1) * ldw], p[(int64_t)min(k + 3, K - 1) * ldw]);
}

__global__ __launch_bounds__(GEMM_THREADS) void k_gemm(const mep_gemm_desc* __restrict__ descs) {
    const mep_gemm_desc& d = descs[blockIdx.y];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int r0 = blockIdx.x * 64 + wave * 16;
    if (r0 >= d.ntok) return;   // whole wave; only wave-private LDS below
    __shared__ __attribute__((aligned(16))) float smem[GEMM_WAVES][16 * GEMM_LDA];
    float* As = smem[wave];
    const int K = d.K, N = d.N, ntok = d.ntok;
    const gfloat* W = G<const float>(d.w);
    const bool w_nt = d.w_nt;
    const bool w_vec = w_nt && (d.ldw % 4 == 0) && ((d.w & 15) == 0);
    const bool x_vec = (K % 4 == 0) && ((d.x.ptr & 15) == 0) && (d.x.sB % 4 == 0) && (d.x.sT % 4 == 0);
    const gfloat* bias = G<const float>(d.bias);
    const gfloat* table = G<const float>(d.table);
    // per-lane row offsets of the staging pattern (row = idx / 32 for float4 idx = lane + 64 i)
    const float* arow = As + c * GEMM_LDA + 4 * g;

    for (int cg = 16 * GEMM_NJ * (int)blockIdx.z; cg < N; cg += 16 * GEMM_NJ * (int)gridDim.z) {
        const int nj = min(GEMM_NJ, (N - cg + 15) / 16);
        f32x4 acc[GEMM_NJ];
#pragma unroll
        for (int j = 0; j < GEMM_NJ; ++j) acc[j] = zero_f4();
        for (int k0 = 0; k0 < K; k0 += GEMM_KC) {
            const int kc = min(GEMM_KC, K - k0);
            const int kcp = (kc + 15) & ~15;
            // stage A rows [r0, r0+16) x cols [k0, k0 + kcp): zero past K / past ntok
            if (x_vec) {
                const int v4 = kcp >> 2;
                for (int idx = lane; idx < 16 * v4; idx += 64) {
                    const int row = idx / v4, c4 = 4 * (idx - row * v4);
                    const int tok = r0 + row;
                    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (tok < ntok && c4 < kc) v = ldg4(row_ptr(d.x, tok) + k0 + c4);
                    *reinterpret_cast<float4*>(As + row * GEMM_LDA + c4) = v;
                }
            } else {
                for (int idx = lane; idx < 16 * kcp; idx += 64) {
                    const int row = idx / kcp, cc = idx - row * kcp;
                    const int tok = r0 + row;
                    float v = 0.f;
                    if (tok < ntok && cc < kc) v = row_ptr(d.x, tok)[k0 + cc];
                    As[row * GEMM_LDA + cc] = v;
                }
            }
            wave_lds_fence();
            const int nkb = kcp >> 4;
            float4 b[GEMM_NJ];
#pragma unroll
            for (int j = 0; j < GEMM_NJ; ++j)
                if (j < nj) b[j] = gemm_wfrag(W, d.ldw, w_nt, w_vec, cg + 16 * j + c, N, k0 + 4 * g, K);
            for (int kb = 0; kb < nkb; ++kb) {
                float4 cur[GEMM_NJ];
#pragma unroll
                for (int j = 0; j < GEMM_NJ; ++j) cur[j] = b[j];
                if (kb + 1 < nkb) {
#pragma unroll
                    for (int j = 0; j < GEMM_NJ; ++j)
                        if (j < nj) b[j] = gemm_wfrag(W, d.ldw, w_nt, w_vec, cg + 16 * j + c, N, k0 + 16 * (kb + 1) + 4 * g, K);
                }
                const float4 a = *reinterpret_cast<const float4*>(arow + 16 * kb);
#pragma unroll
                for (int j = 0; j < GEMM_NJ; ++j)
                    if (j < nj) {
                        acc[j] = mfma16x4(a.x, cur[j].x, acc[j]);
                        acc[j] = mfma16x4(a.y, cur[j].y, acc[j]);
                        acc[j] = mfma16x4(a.z, cur[j].z, acc[j]);
                        acc[j] = mfma16x4(a.w, cur[j].w, acc[j]);
                    }
            }
            wave_lds_fence();   // every lane is done reading this chunk
        }
        // epilogue: rows 4g + r, column cg + 16 j + c
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int tok = r0 + 4 * g + r;
            if (tok >= ntok) continue;
            gfloat* yrow = row_ptr(d.y, tok);
            const gfloat* trow = table ? table + (int64_t)(tok % d.y.T) * (d.ldt ? d.ldt : N) : nullptr;
#pragma unroll
            for (int j = 0; j < GEMM_NJ; ++j) {
                const int col = cg + 16 * j + c;
                if (j >= nj || col >= N) continue;
                float v = d.alpha * acc[j][r];
                if (bias) v += bias[col];
                if (trow) v += trow[col];
                if (d.relu) v = fmaxf(v, 0.f);
                if (d.accumulate) v += yrow[col];
                yrow[col] = v;
            }
        }
    }
}

// ---------------------------------------------------------------- weight gradient
// dW[n][k] = sum_t A[t][n] B[t][k]: a long token reduction into a small (<= 128-row) output, on
// v_mfma_f32_32x32x16_bf16 with the token axis as the MFMA k.  Lane l (column c = l & 31, half
// h = l >> 5) supplies A[row c][k = 8h + j] and B[k = 8h + j][col c], j < 8: eight tokens of ONE
// operand column, so operands go straight from HBM into registers (dword loads, 32 lanes on 32
// consecutive floats of a row) -- no LDS staging, no block barriers in the main loop.  The lane
// halves walk two halves of the wave's token range one token at a time (one wrap check per step,
// no divisions), eight tokens per MFMA k block.  fp32 path: every 8-token operand is split into
// three bf16 parts (split.h, six products per k block: fp32-level error, 2.7x the f32-MFMA rate);
// bf16 path (desc.bf16): one bf16 part, one product.  A wave keeps a whole MT x KT block of 32x32
// tiles in accumulators (MT = ceil(N/32) covers every output row; KT = 3, 2, 4, 4 for MT = 3, 4,
// 2, 1) and WG_PF k blocks of loads in flight beyond the one being multiplied.  One workgroup = 4
// waves (one per SIMD, ~400 VGPRs each) on consecutive quarters of a tok_per_split chunk and one
// column group; the four accumulator blocks are summed through LDS in a fixed order
// ((w0 + w2) + (w1 + w3)) and written once as partial[split][n][k]; mep_wgrad_reduce sums the
// splits.  Row views are addressed with 32-bit offsets (hosts keep every view under 2^31 floats).
// MEP_WG_OCC: k_wgrad workgroups per CU.  2: two waves per SIMD, each on a 32MT x 64 block (KT = 2
// at MT = 3; <= 256 registers: no operand prefetch slot), so one wave's operand loads and split VALU overlap the other's
// products; the LDS reduction buffers shrink to fit two workgroups.
#ifndef MEP_WG_OCC
#define MEP_WG_OCC 2
#endif
#ifndef MEP_WG_KT4
#define MEP_WG_KT4 1   // occupancy 2: column tiles per block at MT = 4 (D = 128)
#endif
#ifndef MEP_WG_PF
// 2 would need ~300 arch VGPRs (spills): double-buffered operands.  Occupancy 2: none (the other
// wave hides the loads; a slot spills at KT = 2)
#define MEP_WG_PF (MEP_WG_OCC > 1 ? 0 : 1)
#endif
constexpr int WG_WAVES = 4;
constexpr int WG_THREADS = 64 * WG_WAVES;
constexpr int WG_SLOTS_F = MEP_WG_PF + 1;     // k blocks of operand registers, fp32 instance
#ifndef MEP_WG_SLOTS_B
#define MEP_WG_SLOTS_B 3   // bf16 instance: k blocks of operand registers (3: two prefetch slots; cfg3 28.2 -> 25.6 us, 4 slower)
#endif
#ifndef MEP_WG_OCC_BF
#define MEP_WG_OCC_BF 1    // bf16 instance: workgroups per CU (2: the fp32 instance's narrow blocks)
#endif
constexpr int WG_SLOTS_B = MEP_WG_SLOTS_B;
// largest 32MT x (32KT + 8) reduction buffer: MT = KT = 3 (occupancy 1, and the bf16 path); two
// workgroups of 2 x 39 KB fit the CU's 160 KB
constexpr int WG_RED = 96 * (96 + 8);

// bf16 path (one part per operand, no split registers): its own kernel instance at one workgroup
// per CU with the wide blocks (the narrow ones double its operand loads: cfg5 bf16 308 vs 170 us at
// KT = 1; the wide ones spill at 256 registers)
__host__ __device__ constexpr int wg_occ(bool bf) { return bf ? MEP_WG_OCC_BF : MEP_WG_OCC; }
__host__ __device__ constexpr int wg_kt(int mt, bool bf) {
    if (wg_occ(bf) > 1) return mt == 4 ? (bf ? 2 : MEP_WG_KT4) : 2;   // <= 96 accumulators (128 at KT = 2, MT = 4)
    return mt == 4 ? 2 : mt == 3 ? 3 : 4;
}

// byte extent of a row view's first ntok rows, `width` columns wide, es bytes per element (the
// range the raw buffer loads check; hosts keep it under 2^31)
MEP_DEV int wg_extent(const mep_rows& r, int T, int ntok, int width, int es = 4) {
    const int64_t last = (int64_t)((ntok - 1) / T) * r.sB + (int64_t)((ntok - 1) % T) * r.sT + width;
    return (int)min((int64_t)es * last, (int64_t)0x7fffffff);
}

constexpr int WG_INV = (int)0x80000000u;   // byte offset past every view: the buffer load returns 0

// a view whose element offset is linear in the token, tok * step (contiguous rows, or T = 1)
MEP_DEV bool wg_linear(const mep_rows& r) { return r.T == 1 || r.sB == (int64_t)r.T * r.sT; }
MEP_DEV int wg_step(const mep_rows& r) { return (int)(r.T == 1 ? r.sB : r.sT); }

// MEP_WG_TRACE (development builds, scripts/wg_trace.py): thread 0 of every workgroup stores the
// real-time counter at phase k of its (last) segment into g_wg_trace[block][k]:
// 0 start, 1 main loop start, 2 main loop end, 3 slot written
#ifdef MEP_WG_TRACE
}  // namespace
__device__ unsigned long long g_wg_trace[8192 * 8];
extern "C" int mep_wg_trace_read(void* dst) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_wg_trace), sizeof(g_wg_trace));
}
namespace {
#define MEP_WG_STAMP(k) do { if (threadIdx.x == 0 && blockIdx.x < 8192) g_wg_trace[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define MEP_WG_STAMP(k) ((void)0)
#endif

// LIN: every view of the item is linear in the token -- a lane's eight tokens of a k block sit at
// fixed byte distances, so they are ONE per-lane base (VGPR) plus a wave-uniform per-token offset
// (the load's SGPR soffset) and the column tile an immediate: no address arithmetic per token.
template <int MT, int KT, int NPART, bool LIN, int WG_SLOTS>
MEP_DEV void wgrad_task(const mep_wgrad_desc& d, int t_begin, int t_end, int slot, int kbase, lfloat* red) {
    // The bf16 path (one part) reads bf16 operand rows (MEP_BF16_STORE, 2-byte elements) as
    // column PAIRS: per 8-token block and 32-column tile a lane loads 4 dwords -- columns
    // 2(c & 15), +1 of tokens 4(c >> 4) .. +3 of its lane half's 8 -- and one v_permlane16_swap
    // per operand dword trades the odd column of tokens 0-3 (lane c < 16) for the even column of
    // tokens 4-7 (lane c + 16).  Lane c < 16 then holds column 2c, lane c + 16 column 2c + 1, each
    // for all 8 tokens: MFMA row / column m is tensor column sg(m) = 2(m & 15) + (m >> 4) of the
    // tile (undone when the accumulators are written).  Half the load instructions of the fp32
    // path (dword per column), no conversion; LIN views only (the bf16 plans' views all are).
    constexpr bool HS = NPART == 1;
    static_assert(!HS || LIN, "bf16 operand rows need linear views");
    constexpr int ES = HS ? 2 : 4;
    constexpr int NE = HS ? 4 : 8;                         // operand registers per tile and block
    typedef typename AElem<HS>::T RT0;
    typedef std::conditional_t<HS, unsigned, float> RT;
    auto ld = [&](__amdgpu_buffer_rsrc_t rs, int voff, int soff) -> RT {
        if constexpr (HS) return __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0);
        else return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0));
    };
    (void)sizeof(RT0);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 31, h = lane >> 5;
    const int N = d.N;
    t_end = min(d.ntok, t_end);
    const int per_wave = (max(0, t_end - t_begin) + WG_WAVES - 1) / WG_WAVES;
    const int w0 = t_begin + wave * per_wave;
    const int n = max(0, min(t_end, w0 + per_wave) - w0);
    const int half = (n + 1) >> 1;                         // tokens of lane half 0 (half 1: n - half)
    const int nh = h ? n - half : half;
    const int nblk = (half + 7) >> 3;                      // k blocks (wave-uniform)

    const int T = d.a.T;   // every view of the item shares T
    // Operand columns of this lane, clamped in range: a column past N (past Ktot) only feeds
    // output rows (columns) that are never stored.  Tokens past the lane half's range read 0
    // through the buffer range check (offset WG_INV).
    // HS: the range covers whole column pairs (a dword past the range would read as 0 -- the
    // last row's odd last column; rows are padded to even widths, so the pad element is ours)
    const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)d.a.ptr, 0, wg_extent(d.a, T, d.ntok, N + (HS ? N & 1 : 0), ES), 0x00020000);
    int colA[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) colA[i] = ES * min(32 * i + c, N - 1);
    const int asB = (int)d.a.sB, asT = (int)d.a.sT;
    __amdgpu_buffer_rsrc_t rsB[KT];
    int colB[KT], bsB[KT], bsT[KT];
#pragma unroll
    for (int j = 0; j < KT; ++j) {
        // the operand of tile j is wave-uniform (hosts keep operand boundaries on 32-column tiles)
        int k0 = min(kbase + 32 * j, d.Ktot - 1), o = 0;
        while (o < d.n_b - 1 && k0 >= d.kb[o]) { k0 -= d.kb[o]; ++o; }
        const mep_rows& b = d.b[o];
        rsB[j] = __builtin_amdgcn_make_buffer_rsrc((void*)b.ptr, 0, wg_extent(b, T, d.ntok, d.kb[o] + (HS ? d.kb[o] & 1 : 0), ES), 0x00020000);
        colB[j] = ES * min(k0 + c, d.kb[o] - 1);
        bsB[j] = (int)b.sB;
        bsT[j] = (int)b.sT;
    }

    floatx16 acc[MT][KT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < KT; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // load cursor: this lane's next token (b, t) and its element offsets, one token per step
    int idx = 0, t, offA, offB[KT];
    {
        const int tq = min(w0 + h * half, d.ntok - 1);
        const int bq = tq / T, tt = tq - bq * T;
        t = tt;
        offA = bq * asB + tt * asT;
#pragma unroll
        for (int j = 0; j < KT; ++j) offB[j] = bq * bsB[j] + tt * bsT[j];
    }
    const int wA = asB - T * asT;
    int wB[KT];
#pragma unroll
    for (int j = 0; j < KT; ++j) wB[j] = bsB[j] - T * bsT[j];

    RT ra[WG_SLOTS][MT][NE], rb[WG_SLOTS][KT][NE];
    // LIN addressing: half h's tokens start at w0 + h * half; token 8 s + e of the half is at
    // base + (8 s + e) * step (bytes, soffset); columns unclamped (a column past N / Ktot reads
    // neighbouring data or 0 and only feeds output entries that are never stored)
    const int t0 = min(w0 + h * half, d.ntok);
    const int stA = ES * (LIN ? wg_step(d.a) : 0);
    int stB[KT], baseB[KT];
    // HS: column pair 2 (c & 15) of tokens 4 (c >> 4) + e (the lane's token offset in its base)
    const int lcol = HS ? 2 * (c & 15) : c, ltok = HS ? 4 * (c >> 4) : 0;
    const int baseA = LIN ? (t0 + ltok) * stA + ES * lcol : 0;
#pragma unroll
    for (int j = 0; j < KT; ++j) {
        int k0 = min(kbase + 32 * j, d.Ktot - 1), o = 0;
        while (o < d.n_b - 1 && k0 >= d.kb[o]) { k0 -= d.kb[o]; ++o; }
        stB[j] = LIN ? ES * wg_step(d.b[o]) : 0;
        baseB[j] = LIN ? (t0 + ltok) * stB[j] + ES * (k0 + lcol) : 0;
    }
    int blk = 0;   // LIN: next k block to load
    auto load_lin = [&](int p, bool checked) {
#pragma unroll
        for (int e = 0; e < NE; ++e) {
            const int tk = 8 * blk + e;                   // wave-uniform part of the token
            const bool ok = !checked || tk + ltok < nh;
            const int va = ok ? baseA : WG_INV;
            // per-token offsets are wave-uniform: readfirstlane keeps them in SGPRs (a VGPR
            // soffset would turn every load into a waterfall loop)
#pragma unroll
            for (int i = 0; i < MT; ++i)
                ra[p][i][e] = ld(rsA, va + 32 * ES * i, __builtin_amdgcn_readfirstlane(tk * stA));
#pragma unroll
            for (int j = 0; j < KT; ++j)
                rb[p][j][e] = ld(rsB[j], ok ? baseB[j] : WG_INV, __builtin_amdgcn_readfirstlane(tk * stB[j]));
        }
        ++blk;
    };
    auto load = [&](int p) {
        if constexpr (LIN) {
            if (8 * blk + 8 <= n - half) load_lin(p, false);   // every token of both halves valid
            else load_lin(p, true);
            return;
        } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const bool ok = idx < nh;
            const int va = ok ? ES * offA : WG_INV;
#pragma unroll
            for (int i = 0; i < MT; ++i) ra[p][i][e] = ld(rsA, va + colA[i], 0);
#pragma unroll
            for (int j = 0; j < KT; ++j) rb[p][j][e] = ld(rsB[j], (ok ? ES * offB[j] : WG_INV) + colB[j], 0);
            ++idx;
            ++t;
            const bool wrap = t >= T;
            t -= wrap ? T : 0;
            offA += asT + (wrap ? wA : 0);
#pragma unroll
            for (int j = 0; j < KT; ++j) offB[j] += bsT[j] + (wrap ? wB[j] : 0);
        }
        }
    };
    auto mma = [&](int p) {
        OpN<NPART> bo[KT];
        auto op = [&](const RT (&v)[NE]) -> OpN<NPART> {
            if constexpr (HS) {
                // even / odd columns of tokens 0-3 (own) ... then the swap (see above)
                unsigned e0 = (v[0] & 0xffffu) | (v[1] << 16), e1 = (v[2] & 0xffffu) | (v[3] << 16);
                unsigned o0 = (v[0] >> 16) | (v[1] & 0xffff0000u), o1 = (v[2] >> 16) | (v[3] & 0xffff0000u);
                const auto s0 = __builtin_amdgcn_permlane16_swap(e0, o0, false, false);
                const auto s1 = __builtin_amdgcn_permlane16_swap(e1, o1, false, false);
                OpN<NPART> o;
                o.p[0] = __builtin_bit_cast(bf16x8, u32x4{s0[0], s1[0], s0[1], s1[1]});
                return o;
            } else {
                return opn<NPART>(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]});
            }
        };
#pragma unroll
        for (int j = 0; j < KT; ++j) bo[j] = op(rb[p][j]);
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const OpN<NPART> ao = op(ra[p][i]);
#pragma unroll
            for (int j = 0; j < KT; ++j) acc[i][j] = mma_n<NPART>(ao, bo[j], acc[i][j]);
        }
    };
    MEP_WG_STAMP(1);
    if (nblk > 0) {
        // blocks 0 .. S-2 go to slots 0 .. S-2; step s loads block s + S - 1 into the slot that
        // step s - 1 consumed, then runs the MFMAs of block s
#pragma unroll
        for (int p = 0; p < WG_SLOTS - 1; ++p) load(p);
        int s0 = 0;
        if constexpr (LIN) {
            // main loop: every block it loads (s0 + S - 1 .. s0 + 2S - 2) is full in both lane
            // halves -- unchecked loads and a branch-free body, so the wait counts stay exact
            // (the loads of the next block stay in flight across this block's products)
            const int nfast = (n - half) >> 3;
            for (; s0 + WG_SLOTS <= nblk && s0 + 2 * WG_SLOTS - 2 < nfast; s0 += WG_SLOTS) {
#pragma unroll
                for (int p = 0; p < WG_SLOTS; ++p) {
                    load_lin((p + WG_SLOTS - 1) % WG_SLOTS, false);
                    __builtin_amdgcn_sched_barrier(0);
                    mma(p);
                }
            }
        }
        for (; s0 + WG_SLOTS <= nblk; s0 += WG_SLOTS) {
#pragma unroll
            for (int p = 0; p < WG_SLOTS; ++p) {
                load((p + WG_SLOTS - 1) % WG_SLOTS);
                // the next block's loads go out before this block's operand conversion (the
                // scheduler would otherwise hoist the conversion, whose wait then drains them too)
                __builtin_amdgcn_sched_barrier(0);
                mma(p);
            }
        }
        const int rem = nblk - s0;     // slots 0 .. rem-1 (rem < S) hold the last blocks
#pragma unroll
        for (int p = 0; p < WG_SLOTS - 1; ++p)
            if (p < rem) mma(p);
    }

    MEP_WG_STAMP(2);
    // ((w0 + w2) + (w1 + w3)) through two LDS buffers, then one coalesced partial write
    constexpr int LDR = 32 * KT + 8;            // == 8 mod 16: lane halves 32 banks apart
    constexpr int BUF = 32 * MT * LDR;
    lfloat* mine = red + (wave & 1) * BUF;
    // MFMA row / column -> tile column (HS: sg(m) = 2 (m & 15) + (m >> 4), the pair layout)
    auto sg = [](int m) { return HS ? 2 * (m & 15) + (m >> 4) : m; };
    const int cc = sg(c);
    if (wave >= 2) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < KT; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) mine[(32 * i + sg(acc_row(r, lane))) * LDR + 32 * j + cc] = acc[i][j][r];
    }
    __syncthreads();
    if (wave < 2) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < KT; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    lfloat* q = mine + (32 * i + sg(acc_row(r, lane))) * LDR + 32 * j + cc;
                    *q = acc[i][j][r] + *q;
                }
    }
    __syncthreads();
    const int kcnt = min(32 * KT, d.Ktot - kbase);
    gfloat* part = G<float>(d.partial) + (int64_t)slot * N * d.Ktot + kbase;
    for (int e = threadIdx.x; e < N * 32 * KT; e += WG_THREADS) {
        const int nn = e / (32 * KT), k = e - nn * (32 * KT);
        if (k < kcnt) part[(int64_t)nn * d.Ktot + k] = red[nn * LDR + k] + red[BUF + nn * LDR + k];
    }
    MEP_WG_STAMP(3);
}

// a descriptor this instance cannot run: NaN partials (loudly wrong, never silently)
MEP_DEV void wg_nan_partial(const mep_wgrad_desc& d, int slot) {
    gfloat* part = G<float>(d.partial) + (int64_t)slot * d.N * d.Ktot;
    for (int e = threadIdx.x; e < d.N * d.Ktot; e += WG_THREADS) part[e] = __builtin_nanf("");
}

// Flat grid of n_wg workgroups.  The map after the n_desc descriptors: off[n_wg + 1] (CSR), then
// 4-int segments {desc << 8 | column group, t_begin, t_end, slot}.  Workgroup w runs segments
// off[w] .. off[w+1]-1 in order: tokens [t_begin, t_end) of one column group of one descriptor,
// written to partial slot `slot` (slots never written stay zero: hosts zero the workspace once).
// The host cuts the launch's total MFMA work into n_wg equal contiguous ranges, so a workgroup
// may finish one descriptor's token range and start another's.
// BF: the instance for bf16-path descriptors (MEP_PREC_BF16); a descriptor of the other precision
// gets NaN partials (loudly wrong, never silently)
template <bool BF>
__global__ __launch_bounds__(WG_THREADS) __attribute__((amdgpu_waves_per_eu(wg_occ(BF)))) void k_wgrad(const mep_wgrad_desc* __restrict__ descs, int n_desc, int n_wg) {
    const int* map = reinterpret_cast<const int*>(descs + n_desc);
    const int s0 = map[blockIdx.x], s1 = map[blockIdx.x + 1];
    const int* seg = map + n_wg + 1;
    __shared__ __attribute__((aligned(16))) float smem[2 * WG_RED];
    lfloat* red = (lfloat*)&smem[0];
    MEP_WG_STAMP(0);
    for (int si = s0; si < s1; ++si) {
        const int hdr = seg[4 * si], t_begin = seg[4 * si + 1], t_end = seg[4 * si + 2], slot = seg[4 * si + 3];
        const mep_wgrad_desc& d = descs[hdr >> 8];
        const int cg = hdr & 0xff;
        const int mt = (d.N + 31) >> 5, ktm = wg_kt(mt, d.bf16);
        const int ktiles = (d.Ktot + 31) >> 5;
        const int kt = min(ktm, ktiles - cg * ktm);
        const int kbase = 32 * ktm * cg;
        if (si > s0) __syncthreads();   // the previous segment's partial write has read `red`
        bool lin = wg_linear(d.a);
        for (int o = 0; o < d.n_b; ++o) lin = lin && wg_linear(d.b[o]);
#define MEP_WGT(M, K)                                                                          \
        case 8 * M + K:                                                                        \
            if constexpr (K > wg_kt(M, BF)) break;   /* not a tile block of this instance */   \
            if (lin) wgrad_task<M, K, BF ? 1 : 3, true, BF ? WG_SLOTS_B : WG_SLOTS_F>(d, t_begin, t_end, slot, kbase, red);  \
            else if constexpr (!BF) wgrad_task<M, K, 3, false, WG_SLOTS_F>(d, t_begin, t_end, slot, kbase, red);         \
            else wg_nan_partial(d, slot);   /* bf16 rows: linear views only */                                                       \
            break;
        // the bf16-path instance needs bf16 operands AND bf16 operand rows (MEP_BF16_OPS | MEP_BF16_STORE)
        if ((d.bf16 != 0) != BF || (BF && d.bf16 != (MEP_BF16_OPS | MEP_BF16_STORE))) {
            wg_nan_partial(d, slot);
            continue;
        }
        switch (8 * mt + kt) {
            MEP_WGT(1, 1) MEP_WGT(1, 2) MEP_WGT(1, 3) MEP_WGT(1, 4)
            MEP_WGT(2, 1) MEP_WGT(2, 2) MEP_WGT(2, 3) MEP_WGT(2, 4)
            MEP_WGT(3, 1) MEP_WGT(3, 2) MEP_WGT(3, 3)
            MEP_WGT(4, 1) MEP_WGT(4, 2)
            default: break;
        }
#undef MEP_WGT
    }
}


__global__ __launch_bounds__(256) void k_wgrad_reduce(const mep_wgrad_desc* __restrict__ descs) {
    wgrad_reduce_block(descs[blockIdx.y], blockIdx.x);
}

// ---------------------------------------------------------------- unify projection
// Y[tok][n] = X[tok][:K] . W[n][:K] (+ table[tok % T][n]) for N = D <= 128 output features:
// Unify_Dimension's bias-free Linears (cmu-mosei/run.py:210-214, Ren-MME/run.py:161-166).
// Weight-stationary transposed tiles (common.h): a workgroup of 8 waves stages W [N][Kp] (zero
// padded to Kp = 16 * KB) in LDS once -- or, when that does not fit, reads 16-byte W fragments
// from L2 (K % 16 == 0) -- and its waves take (16-token tile, output part) tasks of the
// workgroup's contiguous tile range.  Per task Y^T = W X^T on f32 MFMA 16x16x4: lane (c, g)
// holds features 16 i + 4g .. +3 of token c, X fragments (4 consecutive k of token c) come
// straight from HBM through a range-checked buffer resource (past the view: 0), UN_PF k blocks
// ahead of their MFMAs.  Flat grid: workgroup w runs map[w] = desc << 20 | n_wg << 10 | index.
constexpr int UN_WAVES = 8;
constexpr int UN_THREADS = 64 * UN_WAVES;
constexpr int UN_LDS = 30720;   // floats (120 KB): W [N][Kp + 8] when N * (Kp + 8) fits
constexpr int UN_PF = 8;        // X fragments (k blocks) in flight per lane

template <int NIP, bool WL, bool XV>
MEP_DEV void unify_tasks(const mep_gemm_desc& d, const lfloat* wl, int ldl, int tile_lo, int tile_hi, int np) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int K = d.K, KB = (K + 15) >> 4, ntok = d.ntok;
    const int T = d.x.T;
    const auto rsX = __builtin_amdgcn_make_buffer_rsrc((void*)d.x.ptr, 0, wg_extent(d.x, T, ntok, K), 0x00020000);
    const gfloat* wg = G<const float>(d.w);
    const gfloat* table = G<const float>(d.table);
    const int ntask = (tile_hi - tile_lo) * np;
    for (int task = wave; task < ntask; task += UN_WAVES) {
        const int tile = tile_lo + task / np, part = task - (task / np) * np;
        const int tok = tile * 16 + c;
        const bool ok = tok < ntok;
        int xo = WG_INV;   // byte offset of the lane's X row (k = 4g within each k block)
        if (ok) {
            const int b = tok / T, t = tok - b * T;
            xo = 4 * ((int)(b * d.x.sB + t * d.x.sT) + 4 * g);
        }
        const int n0 = 16 * NIP * part;       // first output feature of this part
        f32x4 acc[NIP];
#pragma unroll
        for (int i = 0; i < NIP; ++i) acc[i] = zero_f4();
        f32x4 xf[UN_PF];
        auto load = [&](int p, int kb) {
            const int o = kb < KB ? xo + 64 * kb : WG_INV;
            if (XV) {
                xf[p] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsX, o, 0, 0));
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    xf[p][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsX, o + 4 * e, 0, 0));
            }
        };
        auto mma = [&](int p, int kb) {
            f32x4 a[NIP];
#pragma unroll
            for (int i = 0; i < NIP; ++i) {
                const int row = n0 + 16 * i + c;
                if (WL) a[i] = ld4w(wl + row * ldl + 16 * kb + 4 * g);
                else a[i] = ld4w(wg + (int64_t)row * d.ldw + 16 * kb + 4 * g);
            }
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int i = 0; i < NIP; ++i) acc[i] = mfma16x4(a[i][s], xf[p][s], acc[i]);
        };
        // k block kb -> slot kb % PF; step kb loads block kb + PF - 1 into the slot step kb - 1
        // consumed, then runs block kb's MFMAs
#pragma unroll
        for (int p = 0; p < UN_PF - 1; ++p) load(p, p);
        int k0 = 0;
        for (; k0 + UN_PF <= KB; k0 += UN_PF) {
#pragma unroll
            for (int p = 0; p < UN_PF; ++p) {
                load((p + UN_PF - 1) % UN_PF, k0 + p + UN_PF - 1);
                mma(p, k0 + p);
            }
        }
#pragma unroll
        for (int p = 0; p < UN_PF - 1; ++p)
            if (k0 + p < KB) mma(p, k0 + p);
        if (ok) {
            gfloat* yr = row_ptr(d.y, tok);
            const gfloat* tr = table ? table + (int64_t)(tok % d.y.T) * (d.ldt ? d.ldt : d.N) : nullptr;
#pragma unroll
            for (int i = 0; i < NIP; ++i) {
                const int col = n0 + 16 * i + 4 * g;
                f32x4 v = acc[i];
                if (tr) v += ld4w(tr + col);
                stg4(yr + col, make_float4(v[0], v[1], v[2], v[3]));
            }
        }
    }
}

// bf16 path (desc.bf16): the same mapping on v_mfma_f32_16x16x32_bf16 with plain bf16 operands,
// one MFMA per k pair (two 16-wide k blocks: slots 0-3 / 4-7, split.h).  The weight is staged in
// LDS already rounded, in 16-byte units (n, pair p, lane group g) at n * RS + (4p + g) * 16,
// RS = 64 NP + 32 bytes (conflict-free fragment reads, split.h SplitW), zero past K; when it does
// not fit, fragments are read from L2 and rounded on the fly (K % 16 == 0).
// HS: bf16 X and Y rows (MEP_BF16_STORE, the bf16 path's features and unified rows): X fragments
// stay raw bf16 words (no fp32 round trip).  A wave's first task issues its first UN_PPB k pairs
// of X loads BEFORE the weight staging, so the staging's L2 round trip and the first X fetch from
// HBM overlap (most waves run one task: the launch is latency-bound).
#ifndef MEP_UN_PPB
#define MEP_UN_PPB 8    // k pairs of X fragments in flight per lane (bf16 path)
#endif
typedef __attribute__((address_space(3))) unsigned char un_lbyte;

MEP_DEV void unify_stage_bf(const mep_gemm_desc& d, un_lbyte* wl) {
    // W [N][K] -> rounded bf16 units in LDS (zero past K): UN_SU units per thread per pass, every
    // load of a pass in flight before the first LDS write (a text weight, N = 96 x K = 300, is one
    // pass)
    constexpr int UN_SU = 8;
    const int N = d.N, K = d.K, NPK = (K + 31) >> 5, RS = 64 * NPK + 32;
    const int units = N * NPK * 4;
    const auto rsW = __builtin_amdgcn_make_buffer_rsrc((void*)d.w, 0, 4 * ((N - 1) * d.ldw + K), 0x00020000);
    // a unit is two runs of 4 consecutive k: one 16-byte load each when the runs are aligned and
    // K splits into whole runs (4 lanes of a unit row cover 64 contiguous bytes; 4x fewer
    // address-unit passes than dword loads), else 8 dword loads
    const bool v4 = K % 4 == 0 && d.ldw % 4 == 0 && (d.w & 15) == 0;
    for (int u0 = 0; u0 < units; u0 += UN_SU * UN_THREADS) {
        float v[UN_SU][8];
#pragma unroll
        for (int q = 0; q < UN_SU; ++q) {
            const int u = u0 + q * UN_THREADS + (int)threadIdx.x;
            const int gg = u & 3, pp = (u >> 2) % NPK, n = (u >> 2) / NPK;
            if (v4) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int k = 32 * pp + 16 * h + 4 * gg;
                    const f32x4 x = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                        rsW, (u < units && k < K) ? 4 * (n * d.ldw + k) : WG_INV, 0, 0));
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[q][4 * h + e] = x[e];
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int k = 32 * pp + (j < 4 ? 0 : 16) + 4 * gg + (j & 3);
                    v[q][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                        rsW, (u < units && k < K) ? 4 * (n * d.ldw + k) : WG_INV, 0, 0));
                }
            }
        }
#pragma unroll
        for (int q = 0; q < UN_SU; ++q) {
            const int u = u0 + q * UN_THREADS + (int)threadIdx.x;
            const int gg = u & 3, pp = (u >> 2) % NPK, n = (u >> 2) / NPK;
            typedef __attribute__((address_space(3))) u32x4 lu32x4;
            if (u < units)
                *reinterpret_cast<lu32x4*>(wl + n * RS + (4 * pp + gg) * 16) =
                    u32x4{pk_bf16(v[q][0], v[q][1]), pk_bf16(v[q][2], v[q][3]),
                          pk_bf16(v[q][4], v[q][5]), pk_bf16(v[q][6], v[q][7])};
        }
    }
}

template <int NIP, bool WL, bool XV, bool HS>
MEP_DEV void unify_tasks_bf(const mep_gemm_desc& d, un_lbyte* wl, int tile_lo, int tile_hi, int np) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int K = d.K, NPK = (K + 31) >> 5, ntok = d.ntok, RS = 64 * NPK + 32;
    const int T = d.x.T;
    constexpr int ES = HS ? 2 : 4;
    const auto rsX = __builtin_amdgcn_make_buffer_rsrc((void*)d.x.ptr, 0, wg_extent(d.x, T, ntok, K, ES), 0x00020000);
    const gfloat* wg = G<const float>(d.w);
    const gfloat* table = G<const float>(d.table);
    const int ntask = (tile_hi - tile_lo) * np;
    constexpr int PP = HS ? MEP_UN_PPB : UN_PF / 2;   // k pairs of X fragments in flight
    // one X fragment (4 consecutive k of the lane's token): raw bf16 words (HS) or fp32
    typedef std::conditional_t<HS, u32x2, f32x4> XF;
    auto ld = [&](int o) -> XF {
        if constexpr (HS) {
            if (XV) return __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rsX, o, 0, 0));
            unsigned e[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) e[i] = (unsigned)__builtin_amdgcn_raw_buffer_load_b16(rsX, o + 2 * i, 0, 0);
            return u32x2{e[0] | (e[1] << 16), e[2] | (e[3] << 16)};
        } else {
            f32x4 v;
            if (XV) {
                v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsX, o, 0, 0));
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsX, o + 4 * e, 0, 0));
            }
            return v;
        }
    };
    XF xf[PP][2];
    int xo = WG_INV;
    auto setup = [&](int task) {   // the lane's X row for this task
        const int tile = tile_lo + task / np;
        const int tok = tile * 16 + c;
        xo = WG_INV;
        if (tok < ntok) {
            const int b = tok / T, t = tok - b * T;
            xo = ES * ((int)(b * d.x.sB + t * d.x.sT) + 4 * g);
        }
    };
    auto load = [&](int s, int pp) {
        const int o = pp < NPK ? xo + 32 * ES * pp : WG_INV;
        xf[s][0] = ld(o);
        xf[s][1] = ld(o == WG_INV || 32 * pp + 16 >= K ? WG_INV : o + 16 * ES);
    };
    auto prologue = [&]() {
#pragma unroll
        for (int s = 0; s < PP - 1; ++s) load(s, s);
    };
    int task = wave;
    if (task < ntask) {
        setup(task);
        prologue();
    }
    if (WL) {   // every wave reaches the barrier, with or without a task
        unify_stage_bf(d, wl);
        __syncthreads();
    }
    for (; task < ntask; task += UN_WAVES) {
        if (task != wave) {
            setup(task);
            prologue();
        }
        const int tile = tile_lo + task / np, part = task - (task / np) * np;
        const int tok = tile * 16 + c;
        const int n0 = 16 * NIP * part;
        f32x4 acc[NIP];
#pragma unroll
        for (int i = 0; i < NIP; ++i) acc[i] = zero_f4();
        auto mma = [&](int s, int pp) {
            OpN<1> xb;
            if constexpr (HS) xb.p[0] = kpair(xf[s][0], xf[s][1]);
            else xb = opn<1>(xf[s][0], xf[s][1]);
#pragma unroll
            for (int i = 0; i < NIP; ++i) {
                const int row = n0 + 16 * i + c;
                OpN<1> a;
                if (WL) {
                    typedef __attribute__((address_space(3))) u32x4 lu32x4;
                    a.p[0] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const lu32x4*>(wl + row * RS + (4 * pp + g) * 16));
                } else {
                    const gfloat* wr = wg + (int64_t)row * d.ldw + 32 * pp + 4 * g;
                    a = opn<1>(ld4w(wr), 32 * pp + 16 < K ? ld4w(wr + 16) : zero_f4());
                }
                acc[i] = mma_n<1>(a, xb, acc[i]);
            }
        };
        int p0 = 0;
        for (; p0 + PP <= NPK; p0 += PP) {
#pragma unroll
            for (int s = 0; s < PP; ++s) {
                load((s + PP - 1) % PP, p0 + s + PP - 1);
                mma(s, p0 + s);
            }
        }
#pragma unroll
        for (int s = 0; s < PP - 1; ++s)
            if (p0 + s < NPK) mma(s, p0 + s);
        if (tok < ntok) {
            const auto yr = rowa<HS>(d.y, tok);
            const gfloat* tr = table ? table + (int64_t)(tok % d.y.T) * (d.ldt ? d.ldt : d.N) : nullptr;
#pragma unroll
            for (int i = 0; i < NIP; ++i) {
                const int col = n0 + 16 * i + 4 * g;
                f32x4 v = acc[i];
                if (tr) v += ld4w(tr + col);
                st4a(yr + col, v);
            }
        }
    }
}

__global__ __launch_bounds__(UN_THREADS) void k_unify(const mep_gemm_desc* __restrict__ descs, int n_desc) {
    const int task = reinterpret_cast<const int*>(descs + n_desc)[blockIdx.x];
    const mep_gemm_desc& d = descs[task >> 20];
    const int n_wg = (task >> 10) & 1023, w = task & 1023;
    const int ntiles = (d.ntok + 15) >> 4;
    const int per = (ntiles + n_wg - 1) / n_wg;
    const int tile_lo = w * per, tile_hi = min(ntiles, tile_lo + per);
    if (tile_lo >= tile_hi) return;   // whole workgroup
    __shared__ __attribute__((aligned(16))) float smem[UN_LDS];
    const bool hs = d.bf16 & MEP_BF16_STORE;   // bf16 X / Y rows
    // bf16 rows: 8-byte loads whenever the rows are 8-byte aligned -- columns past K meet zero
    // weight columns (staged as zeros), and the plans pad their bf16 feature rows with zeros
    const bool xv = (hs || d.K % 4 == 0) && ((d.x.ptr & (hs ? 7 : 15)) == 0) && (d.x.sB % 4 == 0) && (d.x.sT % 4 == 0);
    const int np = d.N >= 64 ? 2 : 1, nip = d.N / (16 * np);
    if (d.bf16) {
        // W [N][K] -> rounded bf16 units in LDS (zero past K) when N * RS fits, staged inside the
        // task function (after each wave's first X loads)
        const int N = d.N, K = d.K, NPK = (K + 31) >> 5, RS = 64 * NPK + 32;
        const bool wlds = N * RS <= 4 * UN_LDS;
        un_lbyte* wl = (un_lbyte*)&smem[0];
#define MEP_UNB2(NIP, HS)                                                                                \
            if (wlds) { if (xv) unify_tasks_bf<NIP, true, true, HS>(d, wl, tile_lo, tile_hi, np);        \
                        else unify_tasks_bf<NIP, true, false, HS>(d, wl, tile_lo, tile_hi, np); }        \
            else unify_tasks_bf<NIP, false, true, HS>(d, wl, tile_lo, tile_hi, np);
#define MEP_UNB(NIP)                                                                                     \
        if (nip == NIP) { if (hs) { MEP_UNB2(NIP, true) } else { MEP_UNB2(NIP, false) } }
        MEP_UNB(1) MEP_UNB(2) MEP_UNB(3) MEP_UNB(4)
#undef MEP_UNB
#undef MEP_UNB2
        return;
    }
    lfloat* wl = (lfloat*)&smem[0];
    // rows of 16 KB + 8 floats: a row stride of 2 mod 4 sixteen-byte units puts every lane group of
    // the fragment reads' ds_read_b128 ({0-3, 12-15, 20-27}, ...: rows c, units g) on 16 distinct
    // bank quads (+ 4 floats: two rows per quad, 2-way conflicts -- 0.41 of the kernel's LDS cycles)
    const int N = d.N, K = d.K, KB = (K + 15) >> 4, ldl = 16 * KB + 8;
    const bool wlds = N * ldl <= UN_LDS;
    if (wlds) {   // W [N][K] -> LDS rows of ldl floats, zero past K
        // wave w stages rows w, w + 8, ... (N <= 128: 16 rows per wave), 320 columns per pass:
        // every load of a pass in flight at once through a range-checked buffer resource (rows
        // past N / columns past K read 0, no branches), then the LDS writes
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, KP = 16 * KB;
        const auto rsW = __builtin_amdgcn_make_buffer_rsrc((void*)d.w, 0, 4 * ((N - 1) * d.ldw + K), 0x00020000);
        for (int k0 = 0; k0 < KP; k0 += 320) {
            float v[16][5];
#pragma unroll
            for (int r = 0; r < 16; ++r)
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const int n = wave + UN_WAVES * r, k = k0 + lane + 64 * j;
                    v[r][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                        rsW, (n < N && k < K) ? 4 * (n * d.ldw + k) : WG_INV, 0, 0));
                }
#pragma unroll
            for (int r = 0; r < 16; ++r)
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const int n = wave + UN_WAVES * r, k = k0 + lane + 64 * j;
                    if (n < N && k < KP) wl[n * ldl + k] = v[r][j];
                }
        }
        __syncthreads();
    }
#define MEP_UN(NIP)                                                                          \
    if (nip == NIP) {                                                                        \
        if (wlds) { if (xv) unify_tasks<NIP, true, true>(d, wl, ldl, tile_lo, tile_hi, np);    \
                    else unify_tasks<NIP, true, false>(d, wl, ldl, tile_lo, tile_hi, np); }     \
        else unify_tasks<NIP, false, true>(d, wl, ldl, tile_lo, tile_hi, np);                   \
    }
    MEP_UN(1) MEP_UN(2) MEP_UN(3) MEP_UN(4)
#undef MEP_UN
}

}  // namespace

extern "C" int mep_gemm(const mep_gemm_desc* descs, int n_desc, int max_tiles, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    // grid.z: column passes of 16 * GEMM_NJ (blocks past a descriptor's N leave at once)
    hipLaunchKernelGGL(k_gemm, dim3(max_tiles, n_desc, GEMM_ZP), dim3(GEMM_THREADS), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_gemm");
}

extern "C" int mep_wgrad_kt(int mt, int bf16) { return wg_kt(mt, bf16 != 0); }
extern "C" int mep_wgrad_occupancy(int bf16) { return wg_occ(bf16 != 0); }

extern "C" int mep_wgrad(const mep_wgrad_desc* descs, int n_desc, int max_tiles, int flags, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    if (flags & MEP_PREC_BF16)
        hipLaunchKernelGGL(k_wgrad<true>, dim3(max_tiles), dim3(WG_THREADS), 0, (hipStream_t)stream, descs, n_desc, max_tiles);
    else
        hipLaunchKernelGGL(k_wgrad<false>, dim3(max_tiles), dim3(WG_THREADS), 0, (hipStream_t)stream, descs, n_desc, max_tiles);
    return mep_check_launch("mep_wgrad");
}

extern "C" int mep_wgrad_reduce(const mep_wgrad_desc* descs, int n_desc, int max_tiles, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    hipLaunchKernelGGL(k_wgrad_reduce, dim3(wg_red_blocks(max_tiles), n_desc), dim3(256), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_wgrad_reduce");
}

extern "C" int mep_unify(const mep_gemm_desc* descs, int n_desc, int n_wg, mep_stream_t stream) {
    if (n_desc <= 0 || n_wg <= 0) return 0;
    hipLaunchKernelGGL(k_unify, dim3(n_wg), dim3(UN_THREADS), 0, (hipStream_t)stream, descs, n_desc);
    return mep_check_launch("mep_unify");
}
