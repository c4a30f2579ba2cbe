// Tiled token GEMM on the bf16 matrix cores:
//   Y[tok, n] = act(alpha * sum_k X[tok, k] W(n, k) + bias[n] + table[tok % T, n]) (+ Y)
// the mep_gemm_desc contract (include/mep.h), for the Linears of Unify_Dimension
// (cmu-mosei/run.py:210-214, Ren-MME/run.py:161-166), the realformer Conv1d unify + position
// table and the w_qkv / input-gradient products (others/realformer.py:136-157,182-188).
//
// Mapping (CDNA4).  Transposed tiles (common.h): Y^T = W X^T on v_mfma_f32_16x16x32_bf16 with
// the k-pair slot convention of split.h, so lane (token c, group g) holds output features
// 16 i + 4g .. +3 of its token in accumulator i and both operands are 16-byte row fragments:
// W(n, k .. k+3) (the A operand, rows = output features) and X(tok, k .. k+3) (the B operand).
// A workgroup (4 waves) owns 128 tokens (two 16-token tiles per wave) and an N tile of up to 128
// output features; the K axis runs in 32-wide chunks.  The W chunk is staged in LDS once per
// workgroup, already split into its bf16 parts (split.h SplitW, conflict-free 16-byte units),
// double-buffered: chunk kc+1's W loads are in flight while chunk kc multiplies, and one barrier
// per chunk.  X fragments go straight from HBM into registers one chunk ahead and are split in
// registers.  fp32 path: three parts per operand, six products (fp32-level, split.h); bf16 path
// (desc.bf16): one part, one product.  W columns past K are staged as zeros, so the X columns past
// K (the next row's data, or zeros past the view through the range-checked buffer loads) never
// contribute.
#include <type_traits>

#include "common.h"
#include "split.h"

using namespace mep;

namespace {

constexpr int TG_WAVES = 4;
constexpr int TG_THREADS = 64 * TG_WAVES;
#ifndef MEP_TG_TT
#define MEP_TG_TT 2
#endif
#ifndef MEP_TG_NI
#define MEP_TG_NI 8        // 16-column tiles of a workgroup's N tile at N >= 128
#endif
constexpr int TG_TT = MEP_TG_TT;                  // 16-token tiles per wave
#ifndef MEP_TG_PF
#define MEP_TG_PF 4        // fp32 path: k chunks of W / X in registers (loads 3 chunks ahead; cfg5 125 -> 104 us)
#endif
#ifndef MEP_TG_PF_BF
#define MEP_TG_PF_BF 2     // bf16 path: one chunk ahead keeps two workgroups per CU (3-6 chunks: one, 92 vs 76 us)
#endif
constexpr int TG_BM = 16 * TG_TT * TG_WAVES;      // tokens per workgroup

// W(n, k .. k+3) of the staged chunk, zero past K / N
template <bool WNT>
MEP_DEV f32x4 tg_wfrag(const gfloat* W, int ldw, bool vec, int n, int N, int k, int K) {
    if (n >= N) return f32x4{0.f, 0.f, 0.f, 0.f};
    if (WNT) {
        const gfloat* p = W + (int64_t)n * ldw;
        if (vec && k + 3 < K) return ld4w(p + k);
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = k + e < K ? p[k + e] : 0.f;
        return v;
    }
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = k + e < K ? W[(int64_t)(k + e) * ldw + n] : 0.f;
    return v;
}

template <int NI, int NPART, bool WNT>
__global__ __launch_bounds__(TG_THREADS) void k_tgemm(const mep_gemm_desc* __restrict__ descs) {
    constexpr int BN = 16 * NI;
    constexpr int TG_PF = NPART == 1 ? MEP_TG_PF_BF : MEP_TG_PF;
    using WS = SplitW<BN, 1, NPART>;                     // one k pair (32 wide) of BN rows
    __shared__ __attribute__((aligned(16))) unsigned char sm[2 * WS::BYTES];
    const mep_gemm_desc& d = descs[blockIdx.y];
    const int n0 = (int)blockIdx.z * BN;
    const int tok0 = (int)blockIdx.x * TG_BM;
    if (n0 >= d.N || tok0 >= d.ntok) return;            // the whole workgroup
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int K = d.K, N = d.N, ntok = d.ntok;
    const int nkc = (K + 31) >> 5;
    typedef __attribute__((address_space(3))) unsigned char lbyte;
    auto wbuf = [&](int b) { return WS{(lbyte*)sm + b * WS::BYTES, 0}; };

    // ---- W chunk staging: unit (n, g) = W(n0 + n, k0 + 4g ..) and W(n0 + n, k0 + 16 + 4g ..);
    // consecutive threads take consecutive n (coalesced for W stored [k][n])
    const gfloat* W = G<const float>(d.w);
    const bool wvec = WNT && (d.ldw % 4 == 0) && ((d.w & 15) == 0);
    constexpr int NU = BN * 4, UPT = (NU + TG_THREADS - 1) / TG_THREADS;
    // TG_PF chunks of W and X in registers: chunk kc + TG_PF - 1's loads go out while chunk kc
    // multiplies, so a chunk's loads have TG_PF - 1 chunks of work to arrive in (one chunk ahead
    // left every chunk waiting a full memory latency: the launch was latency-bound)
    f32x4 wr[TG_PF][UPT][2];
    auto load_w = [&](int s, int kc) {
        const int k0 = 32 * kc;
#pragma unroll
        for (int u = 0; u < UPT; ++u) {
            const int idx = threadIdx.x + TG_THREADS * u;
            const int n = idx % BN, gg = idx / BN;
            if (idx < NU) {
                wr[s][u][0] = tg_wfrag<WNT>(W, d.ldw, wvec, n0 + n, N, k0 + 4 * gg, K);
                wr[s][u][1] = tg_wfrag<WNT>(W, d.ldw, wvec, n0 + n, N, k0 + 16 + 4 * gg, K);
            }
        }
    };
    auto put_w = [&](int s, const WS& ws) {
#pragma unroll
        for (int u = 0; u < UPT; ++u) {
            const int idx = threadIdx.x + TG_THREADS * u;
            if (idx < NU) ws.put(idx % BN, 0, idx / BN, wr[s][u][0], wr[s][u][1]);
        }
    };

    // ---- X rows of this wave's tiles (tokens past ntok: clamped rows, never stored)
    // the bf16 path (one part) reads bf16 X rows and writes bf16 Y rows (MEP_BF16_STORE)
    constexpr bool HS = NPART == 1;
    constexpr int ES = HS ? 2 : 4;
    const int64_t last = row_off(d.x, ntok - 1) + K;
    const auto rsX = __builtin_amdgcn_make_buffer_rsrc((void*)d.x.ptr, 0, (int)min((int64_t)ES * last, (int64_t)0x7fffffff), 0x00020000);
    const bool xvec = ((d.x.ptr & (HS ? 7 : 15)) == 0) && (d.x.sB % 4 == 0) && (d.x.sT % 4 == 0);
    int xoff[TG_TT];
#pragma unroll
    for (int t = 0; t < TG_TT; ++t) {
        const int tok = min(tok0 + 16 * (TG_TT * wave + t) + c, ntok - 1);
        xoff[t] = ES * ((int)row_off(d.x, tok) + 4 * g);
    }
    f32x4 xr[TG_PF][TG_TT][2];
    auto load_x = [&](int s, int kc) {
#pragma unroll
        for (int t = 0; t < TG_TT; ++t)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int o = xoff[t] + 32 * ES * kc + 16 * ES * h;   // bytes: k0 + 16 h + 4g
                if (HS && xvec) {
                    const u32x2a w = __builtin_bit_cast(u32x2a, __builtin_amdgcn_raw_buffer_load_b64(rsX, o, 0, 0));
                    xr[s][t][h] = f32x4{bf16_word_lo(w[0]), bf16_word_hi(w[0]), bf16_word_lo(w[1]), bf16_word_hi(w[1])};
                } else if (HS) {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        xr[s][t][h][e] = __builtin_bit_cast(float, (unsigned)__builtin_amdgcn_raw_buffer_load_b16(rsX, o + 2 * e, 0, 0) << 16);
                } else if (xvec) {
                    xr[s][t][h] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsX, o, 0, 0));
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        xr[s][t][h][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsX, o + 4 * e, 0, 0));
                }
            }
    };

    f32x4 acc[TG_TT][NI];
#pragma unroll
    for (int t = 0; t < TG_TT; ++t)
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[t][i] = zero_f4();

    // chunk kc lives in register slot kc % TG_PF and LDS buffer kc & 1
#pragma unroll
    for (int s = 0; s < TG_PF - 1; ++s)
        if (s < nkc) { load_w(s, s); load_x(s, s); }
    put_w(0, wbuf(0));
    __syncthreads();
    auto step = [&](int kc, int s) {   // s = kc % TG_PF (compile-time in the unrolled loop)
        OpN<NPART> xo[TG_TT];
#pragma unroll
        for (int t = 0; t < TG_TT; ++t) xo[t] = opn<NPART>(xr[s][t][0], xr[s][t][1]);
        const int kn = kc + TG_PF - 1, sn = (s + TG_PF - 1) % TG_PF;
        if (kn < nkc) {                     // TG_PF - 1 chunks ahead, in flight across this chunk's MFMAs
            load_w(sn, kn);
            load_x(sn, kn);
        }
        __builtin_amdgcn_sched_barrier(0);
        const WS ws = wbuf(kc & 1);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const OpN<NPART> w = ws.frag(i, 0);
#pragma unroll
            for (int t = 0; t < TG_TT; ++t) acc[t][i] = mma_n<NPART>(w, xo[t], acc[t][i]);
            if (i & 1) __builtin_amdgcn_sched_barrier(0);
        }
        if (kc + 1 < nkc) put_w((s + 1) % TG_PF, wbuf((kc + 1) & 1));   // its last readers finished before the last barrier
        __syncthreads();
    };
    int kc = 0;
    for (; kc + TG_PF <= nkc; kc += TG_PF) {
#pragma unroll
        for (int s = 0; s < TG_PF; ++s) step(kc + s, s);
    }
#pragma unroll
    for (int s = 0; s < TG_PF - 1; ++s)
        if (kc + s < nkc) step(kc + s, s);

    // ---- epilogue: token c of tile t, features n0 + 16 i + 4g .. +3
    const gfloat* bias = G<const float>(d.bias);
    const gfloat* table = G<const float>(d.table);
    const int ldt = d.ldt ? d.ldt : N;
#pragma unroll
    for (int t = 0; t < TG_TT; ++t) {
        const int tok = tok0 + 16 * (TG_TT * wave + t) + c;
        if (tok >= ntok) continue;
        const auto yrow = rowa<HS>(d.y, tok);
        const gfloat* trow = table ? table + (int64_t)(tok % d.y.T) * ldt : nullptr;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int col = n0 + 16 * i + 4 * g;
            if (col >= N) continue;
            f32x4 v = acc[t][i];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = d.alpha * v[r];
            if (bias) v += ld4w(bias + col);
            if (trow) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += trow[col + r];
            }
            if (d.relu) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
            }
            if (d.accumulate) v += ld4a(yrow + col);
            st4a(yrow + col, v);
        }
    }
}

// Weight staged by LDS-DMA (MEP_TGEMM_DMA: w_nt; both paths).  The fp32 W chunk [BN rows][32 k]
// goes straight from HBM / L2 into a ring of TGB_NS LDS slots (no VGPRs in flight: TGB_NS - 1 chunks
// ahead instead of one), one 1-KiB wave instruction per 8 rows; the fragment read splits it into
// its bf16 parts (one on the bf16 path, three on the fp32 path: the operand the register-staged
// kernel's SplitW::put stores).  X rows stay in registers, TGB_PFX chunks deep (raw bf16 words on
// the bf16 path).  Slot layout: row r, 16-byte unit s holds
// k piece q = s ^ ((r >> 1) & 7) (a ds_read_b128 of 16 rows x one piece covers the 64 banks once).
#ifndef MEP_TGB_NS
#define MEP_TGB_NS 4       // LDS weight-ring slots (4 x 16 KiB at BN = 128)
#endif
#ifndef MEP_TGB_PFX
#define MEP_TGB_PFX 3      // X chunks in registers (bf16 path)
#endif
#ifndef MEP_TGD_PFX
#define MEP_TGD_PFX 2      // X chunks in registers (fp32 path: two workgroups per CU)
#endif
template <int NI, int NPART>
MEP_DEV void tgemm_dma(const mep_gemm_desc* __restrict__ descs) {
    constexpr bool HS = NPART == 1;                  // bf16 path: bf16 X / Y rows
    constexpr int ES = HS ? 2 : 4;
    constexpr int BN = 16 * NI, NS = MEP_TGB_NS, PFX = HS ? MEP_TGB_PFX : MEP_TGD_PFX;
    constexpr int CHB = BN * 128;                    // bytes of one fp32 chunk slot
    constexpr int UPW = BN / (8 * TG_WAVES);         // DMA instructions per wave per chunk
    static_assert(BN % (8 * TG_WAVES) == 0 && NS >= 2 && PFX >= 2, "tgemm_bf geometry");
    __shared__ __attribute__((aligned(16))) unsigned char sm[NS * CHB];
    const mep_gemm_desc& d = descs[blockIdx.y];
    const int n0 = (int)blockIdx.z * BN;
    const int tok0 = (int)blockIdx.x * TG_BM;
    if (n0 >= d.N || tok0 >= d.ntok) return;         // the whole workgroup
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = lane & 15, g = lane >> 4;
    const int K = d.K, N = d.N, ntok = d.ntok;
    const int nkc = (K + 31) >> 5;
    typedef __attribute__((address_space(3))) unsigned char lbyte;
    typedef __attribute__((address_space(3))) void lvoid;
    typedef __attribute__((address_space(3))) const f32x4 lcf4;

    // a lane's 16-byte unit goes by LDS-DMA when it is whole (k + 3 < K) and the weight rows are
    // 16-byte aligned; otherwise (the K tail, unaligned rows) the lane loads what exists, zero-fills
    // the rest and writes the unit with a plain LDS store (a plain load is waited for before its
    // store, so that path is synchronous).  Rows past N take their DMA from row N - 1: every wave
    // then issues exactly UPW DMA instructions per whole chunk, which the steady-state
    // vmcnt(NEWER) below counts on (a wave skipping the DMA of its rows past N would let the wait
    // pass with its chunk-kc DMA still in flight).  Rows past N only feed output columns >= N,
    // which are never stored.
    const gfloat* W = G<const float>(d.w);
    const bool wdma = (d.ldw % 4 == 0) && ((d.w & 15) == 0);
    const auto rsW = __builtin_amdgcn_make_buffer_rsrc((void*)d.w, 0, (int)min((int64_t)4 * N * d.ldw, (int64_t)0x7fffffff), 0x00020000);
    int wrow[UPW], wq[UPW], wsrc[UPW];
#pragma unroll
    for (int u = 0; u < UPW; ++u) {
        wrow[u] = n0 + 8 * (wave * UPW + u) + (lane >> 3);
        wq[u] = 4 * ((lane & 7) ^ (((wrow[u] - n0) >> 1) & 7));
        wsrc[u] = min(wrow[u], N - 1);
    }
    auto issue_w = [&](int kc) {
        lbyte* dst = (lbyte*)sm + (kc % NS) * CHB + wave * UPW * 1024;
#pragma unroll
        for (int u = 0; u < UPW; ++u) {
            const int k = 32 * kc + wq[u];
            if (wdma && k + 3 < K) {
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (lvoid*)(dst + u * 1024), 16, 4 * (wsrc[u] * d.ldw + wq[u]),
                                                         128 * kc, 0, 0);
            } else {
                f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
                if (wrow[u] < N) {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (k + e < K) v[e] = W[(int64_t)wrow[u] * d.ldw + k + e];
                }
                *(__attribute__((address_space(3))) f32x4*)(dst + u * 1024 + 16 * lane) = v;
            }
        }
    };

    // X: bf16 path raw bf16 words (rows not 8-byte aligned: four 2-byte loads per unit); fp32 path
    // fp32 units (rows not 16-byte aligned: four 4-byte loads), split into 3 parts per chunk.  X
    // columns past K (the next row's values, or zeros past the view) meet zero weight units
    const int64_t last = row_off(d.x, ntok - 1) + K;
    const auto rsX = __builtin_amdgcn_make_buffer_rsrc((void*)d.x.ptr, 0, (int)min((int64_t)ES * last, (int64_t)0x7fffffff), 0x00020000);
    const bool xvec = ((d.x.ptr & (HS ? 7 : 15)) == 0) && (d.x.sB % 4 == 0) && (d.x.sT % 4 == 0);
    int xoff[TG_TT];
#pragma unroll
    for (int t = 0; t < TG_TT; ++t) {
        const int tok = min(tok0 + 16 * (TG_TT * wave + t) + c, ntok - 1);
        xoff[t] = ES * ((int)row_off(d.x, tok) + 4 * g);
    }
    typedef typename std::conditional<HS, u32x2, f32x4>::type XU;
    XU xr[PFX][TG_TT][2];
    auto load_x = [&](int s, int kc) {
#pragma unroll
        for (int t = 0; t < TG_TT; ++t)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int o = xoff[t] + 32 * ES * kc + 16 * ES * h;
                if constexpr (HS) {
                    if (xvec) {
                        xr[s][t][h] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(rsX, o, 0, 0));
                    } else {
                        unsigned e[4];
#pragma unroll
                        for (int j = 0; j < 4; ++j) e[j] = (unsigned)__builtin_amdgcn_raw_buffer_load_b16(rsX, o + 2 * j, 0, 0);
                        xr[s][t][h] = u32x2{e[0] | (e[1] << 16), e[2] | (e[3] << 16)};
                    }
                } else {
                    if (xvec) {
                        xr[s][t][h] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsX, o, 0, 0));
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            xr[s][t][h][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsX, o + 4 * j, 0, 0));
                    }
                }
            }
    };

    f32x4 acc[TG_TT][NI];
#pragma unroll
    for (int t = 0; t < TG_TT; ++t)
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[t][i] = zero_f4();

#pragma unroll
    for (int k = 0; k < NS - 1; ++k)
        if (k < nkc) issue_w(k);
#pragma unroll
    for (int k = 0; k < PFX - 1; ++k)
        if (k < nkc) load_x(k, k);
    // vector-memory operations a wave issues after chunk kc's weight in the steady state
    constexpr int XI = 2 * TG_TT;
    constexpr int NEWER = (NS - 2) * UPW + (NS - 1) * XI;
    auto step = [&](int kc, int s) {                  // s = kc % PFX (compile-time in the unrolled loop)
        const bool steady = kc >= NS - 1 && kc + NS - 2 < nkc && kc + PFX - 2 < nkc;
        if (steady) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NEWER) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();                              // chunk kc landed; slot (kc - 1) % NS free
        if (kc + NS - 1 < nkc) issue_w(kc + NS - 1);
        if (kc + PFX - 1 < nkc) load_x((s + PFX - 1) % PFX, kc + PFX - 1);
        const lbyte* ws = (const lbyte*)sm + (kc % NS) * CHB;
        OpN<NPART> xo[TG_TT];
#pragma unroll
        for (int t = 0; t < TG_TT; ++t) {
            if constexpr (HS) xo[t].p[0] = kpair(xr[s][t][0], xr[s][t][1]);
            else xo[t] = opn<NPART>(xr[s][t][0], xr[s][t][1]);
        }
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int r = 16 * i + c, sw = (r >> 1) & 7;
            const f32x4 a0 = *(lcf4*)(ws + r * 128 + 16 * (g ^ sw));
            const f32x4 a1 = *(lcf4*)(ws + r * 128 + 16 * ((4 + g) ^ sw));
            const OpN<NPART> wo = opn<NPART>(a0, a1);     // the parts SplitW::put would store
#pragma unroll
            for (int t = 0; t < TG_TT; ++t) acc[t][i] = mma_n<NPART>(wo, xo[t], acc[t][i]);
        }
    };
    int kc = 0;
    for (; kc + PFX <= nkc; kc += PFX) {
#pragma unroll
        for (int s = 0; s < PFX; ++s) step(kc + s, s);
    }
#pragma unroll
    for (int s = 0; s < PFX - 1; ++s)
        if (kc + s < nkc) step(kc + s, s);

    // ---- epilogue: token c of tile t, features n0 + 16 i + 4g .. +3
    const gfloat* bias = G<const float>(d.bias);
    const gfloat* table = G<const float>(d.table);
    const int ldt = d.ldt ? d.ldt : N;
#pragma unroll
    for (int t = 0; t < TG_TT; ++t) {
        const int tok = tok0 + 16 * (TG_TT * wave + t) + c;
        if (tok >= ntok) continue;
        const auto yrow = rowa<HS>(d.y, tok);
        const gfloat* trow = table ? table + (int64_t)(tok % d.y.T) * ldt : nullptr;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int col = n0 + 16 * i + 4 * g;
            if (col >= N) continue;
            f32x4 v = acc[t][i];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = d.alpha * v[r];
            if (bias) v += ld4w(bias + col);
            if (trow) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += trow[col + r];
            }
            if (d.relu) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
            }
            if (d.accumulate) v += ld4a(yrow + col);
            st4a(yrow + col, v);
        }
    }
}

// one kernel per N tile (plain kernels: hipcc leaves the host stubs of kernel templates named only
// inside a switch undefined)
#define MEP_TGB_K(NI) \
    __global__ __launch_bounds__(TG_THREADS) void k_tgemm_bf##NI(const mep_gemm_desc* __restrict__ descs) { tgemm_dma<NI, 1>(descs); } \
    __global__ __launch_bounds__(TG_THREADS) void k_tgemm_dma##NI(const mep_gemm_desc* __restrict__ descs) { tgemm_dma<NI, 3>(descs); }
MEP_TGB_K(2) MEP_TGB_K(4) MEP_TGB_K(6) MEP_TGB_K(8)
#undef MEP_TGB_K

}  // namespace

// Grid (ceil(max ntok / 128), n_desc, ceil(max N / (16 * NI))): flags = MEP_PREC_BF16 for the bf16
// path; the host guarantees N % 16 == 0, 16-byte aligned y rows / bias (and table rows when
// present) and w_nt shared by every descriptor of the launch (mep_tgemm_ok in the Python binding).
extern "C" int mep_tgemm(const mep_gemm_desc* descs, int n_desc, int max_ntok, int max_n, int flags,
                         mep_stream_t stream) {
    if (n_desc <= 0 || max_ntok <= 0 || max_n <= 0) return 0;
    const bool bf = flags & MEP_PREC_BF16, wnt = !(flags & MEP_TGEMM_WT);
    hipStream_t st = (hipStream_t)stream;
    const int ni = max_n >= 16 * MEP_TG_NI ? MEP_TG_NI : (max_n + 15) / 16;   // 16-col tiles per workgroup N tile
    if (flags & MEP_TGEMM_DMA) {   // w_nt (host)
        if (!wnt) { mep_set_error("mep_tgemm: MEP_TGEMM_DMA needs w_nt"); return MEP_EINVAL; }
        const dim3 grid((max_ntok + TG_BM - 1) / TG_BM, n_desc, (max_n + 16 * ni - 1) / (16 * ni)), block(TG_THREADS);
#define MEP_TGD(NI) do { if (bf) hipLaunchKernelGGL(k_tgemm_bf##NI, grid, block, 0, st, descs); \
                         else hipLaunchKernelGGL(k_tgemm_dma##NI, grid, block, 0, st, descs); } while (0)
        switch (ni) {
            case 2: MEP_TGD(2); break;
            case 4: MEP_TGD(4); break;
            case 6: MEP_TGD(6); break;
            case 8: MEP_TGD(8); break;
            default: mep_set_error("mep_tgemm: N must be 32, 64, 96 or >= 128 (a multiple of 16)"); return MEP_EINVAL;
        }
#undef MEP_TGD
        return mep_check_launch("mep_tgemm");
    }
    const dim3 grid((max_ntok + TG_BM - 1) / TG_BM, n_desc, (max_n + 16 * ni - 1) / (16 * ni)), block(TG_THREADS);
#define MEP_TG3(NI, P, WT) hipLaunchKernelGGL((k_tgemm<NI, P, WT>), grid, block, 0, st, descs)
#define MEP_TG2(NI, P) do { if (wnt) MEP_TG3(NI, P, true); else MEP_TG3(NI, P, false); } while (0)
#define MEP_TG(NI) do { if (bf) MEP_TG2(NI, 1); else MEP_TG2(NI, 3); } while (0)
    switch (ni) {
        case 2: MEP_TG(2); break;
        case 4: MEP_TG(4); break;
        case 6: MEP_TG(6); break;
        case 8: MEP_TG(8); break;
        default: mep_set_error("mep_tgemm: N must be 32, 64, 96 or >= 128 (a multiple of 16)"); return MEP_EINVAL;
    }
#undef MEP_TG
#undef MEP_TG2
#undef MEP_TG3
    return mep_check_launch("mep_tgemm");
}

