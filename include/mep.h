/*
 * mep.h -- C ABI of libmep_hip.so, the MI355X (gfx950) kernels of the tri-modal
 * residual-attention training path (youngzhou97qz/Multimodal-emotion-processing).
 *
 * The reference has no FFI: its hot path is PyTorch ATen called from the model classes in
 * cmu-mosei/run.py, Ren-MME/run.py and others/realformer.py.  Each entry point below replaces
 * the ATen ops of one reference function (file:line cited per entry).
 *
 * Conventions
 *   - Every pointer is a DEVICE pointer owned by the caller (PyTorch caching allocator).  The
 *     library never allocates; workspaces are passed in.  Descriptor arrays live in device
 *     memory too (built once per plan, so a captured hipGraph replays them unchanged).
 *   - All arithmetic is fp32 (the reference has no AMP).  Layouts are row-major.
 *   - Launches are asynchronous on `stream`; no host synchronisation, no allocation, so every
 *     call may be captured into a hipGraph.
 *   - Return 0 on success or a negative code (-(int)hipError_t, or MEP_EINVAL); the text of the
 *     last error of the calling thread is available from mep_last_error().
 *
 * Row views ("mep_rows"): a token-indexed 2-D view.  Row `tok` (0 <= tok < B*T) of the view
 * starts at  ptr + (tok / T) * sB + (tok % T) * sT  (in floats); columns are contiguous.  This
 * addresses slot-strided inputs ([B,2,T,d] slices), strided concatenation slices and plain
 * contiguous [B*T, d] buffers with one descriptor.
 */
#ifndef MEP_H_
#define MEP_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MEP_EINVAL (-1000)
#define MEP_ABI_VERSION 7

typedef void* mep_stream_t; /* a hipStream_t */

/* Arithmetic precision.  Default (fp32 path): fp32 storage and every product at fp32 level --
 * f32 MFMA, or fp32 operands split into bf16 parts on the bf16 matrix cores (3 parts: fp32-level
 * error).  MEP_PREC_BF16 (bf16 path, BASELINE cfg3/cfg5): the matrix products take plain bf16
 * operands with fp32 accumulation -- one MFMA per k block -- and the ACTIVATIONS are stored as
 * bf16 (what torch.autocast(bfloat16) keeps between ops): the features, the unified rows, the
 * attention outputs, the epilogue intermediates xp / z and every gradient of those rows (dx, dq,
 * dk / dv, dz, dxp, the per-modality sums).  Scores, softmax / LayerNorm statistics, the block
 * outputs the pool reads, loss, parameters, their gradients and the optimizer state stay fp32.
 * Row views keep counting ELEMENTS (2 bytes for bf16 rows).  OR-ed into the `flags` of
 * mep_attn_fwd / mep_attn_bwd (q k v x dx dq dk dv bf16) and the `D` argument of
 * mep_block_epi_fwd / mep_block_epi_bwd (q x xp z dout2 dz dxp dx dq out_h bf16; out, dout
 * fp32); the `bf16` field of mep_gemm_desc (mep_unify / mep_tgemm) and mep_wgrad_desc take
 * MEP_BF16_OPS (bf16 operands) | MEP_BF16_STORE (bf16 x / y, or a / b, rows). */
#define MEP_BF16_OPS 1
#define MEP_BF16_STORE 2
#define MEP_PREC_BF16 0x10000

/* A row view: token tok = b * T + t sits at ptr + b * sB + t * sT (elements).  Strides are
 * below 2^24 elements and every element offset of a view below 2^32 (the kernels address rows on
 * the 24-bit multiplier, csrc/common.h row_off). */
typedef struct {
    uint64_t ptr;   /* float* base                                  */
    int64_t  sB;    /* stride (floats) between consecutive batch rows */
    int64_t  sT;    /* stride (floats) between consecutive time steps */
    int32_t  T;     /* time steps per batch row                      */
    int32_t  _pad;
} mep_rows;

/* ---------------------------------------------------------------- token GEMM (MFMA f32)
 * Y[tok, n] = act( alpha * sum_k X[tok, k] * W(n, k) + bias[n] + table[tok % T, n] ) (+ Y if accumulate)
 * (table row stride ldt, default N; T = y.T)
 * W(n,k) = W[n*ldw + k] when w_nt (nn.Linear weight, used by forward), else W[k*ldw + n]
 * (backward dX = dY W).  Replaces the bias-free nn.Linear of Unify_Dimension
 * (cmu-mosei/run.py:210-214, Ren-MME/run.py:161-166), the k=1 Conv1d unify + position
 * embedding (others/realformer.py:136-152,224-227) and the realformer w_qkv / FFN Linears
 * (others/realformer.py:157,163-168,188). */
typedef struct {
    mep_rows x;        /* A operand rows, K columns                      */
    mep_rows y;        /* output rows, N columns                         */
    uint64_t w;        /* weight                                          */
    uint64_t bias;     /* [N] or 0                                        */
    uint64_t table;    /* [T, N] row table added by (tok % y.T) or 0      */
    int32_t  ntok, N, K, ldw;
    int32_t  w_nt;     /* 1: W[n][k] (Linear weight); 0: W[k][n]          */
    int32_t  accumulate;
    int32_t  relu;
    float    alpha;
    int32_t  bf16;     /* mep_unify: 1 = bf16 operands (MEP_PREC_BF16); mep_gemm: must be 0 */
    int32_t  ldt;      /* row stride (floats) of table; 0 = N (a column slice of a wider table) */
} mep_gemm_desc;
int mep_gemm(const mep_gemm_desc* descs, int n_desc, int max_tiles, mep_stream_t stream);

/* Unify projection: the forward bias-free Linear of Unify_Dimension (cmu-mosei/run.py:210-214,
 * Ren-MME/run.py:161-166) on the same descriptor, restricted to w_nt = 1, N in {16, 32, 48, 64,
 * 96, 128}, no bias / relu / accumulate, alpha = 1 (table allowed), 16-byte aligned output rows.
 * The weight is staged in LDS when N * (16 * ceil(K / 16) + 8) <= 30720 floats; otherwise it is
 * read from L2 and needs K % 16 == 0 and 16-byte aligned W and X rows.  `descs` holds the n_desc
 * descriptors FOLLOWED BY n_wg int32 task entries (descriptor << 20 | workgroups of that
 * descriptor << 10 | workgroup index), one per workgroup of the flat grid; a descriptor's
 * workgroups split its 16-token tiles into contiguous ranges.
 * bf16 rows (MEP_BF16_STORE) with 8-byte aligned rows are read 4 elements at a time: when
 * K % 4 != 0 the row's elements K .. 4 ceil(K / 4) - 1 are read too and MUST be finite (they meet
 * zero weight columns; 0 x inf is nan).  The plans zero-pad their bf16 feature rows to a
 * multiple of 8 elements. */
int mep_unify(const mep_gemm_desc* descs, int n_desc, int n_wg, mep_stream_t stream);

/* Tiled token GEMM on the bf16 matrix cores, the mep_gemm contract for N % 16 == 0: a workgroup
 * owns 128 tokens x (up to) 128 output features, the weight is staged in LDS in 32-wide k chunks
 * already split into bf16 parts (double-buffered), X rows go straight into registers.  fp32 path:
 * 3-part splits of both operands (six products, fp32-level error); flags | MEP_PREC_BF16: plain
 * bf16 operands (one product).  Every descriptor of a launch has the same w_nt (MEP_TGEMM_WT:
 * w_nt = 0, W stored [K][N]); y rows (and bias) 16-byte aligned; N in {32, 64, 96} or >= 128.
 * Grid: (ceil(max_ntok / 128), n_desc, N tiles). */
#define MEP_TGEMM_WT 0x1
#define MEP_TGEMM_DMA 0x4        /* w_nt = 1 only: the fp32 weight chunks staged by LDS-DMA into a ring of
                                    4 slots (3 chunks in flight; K tails, rows past N and unaligned rows
                                    by plain loads) and split into the path's bf16 parts on the
                                    fragment read (bit-identical to the register-staged kernel) */
int mep_tgemm(const mep_gemm_desc* descs, int n_desc, int max_ntok, int max_n, int flags, mep_stream_t stream);

/* ---------------------------------------------------------------- weight-gradient GEMM
 * dW_i[n, k] (+)= sum_tok A[tok, n] * B_i[tok, k]   for up to 4 operands B_i sharing one A
 * (dW = dY^T X of every nn.Linear on the path; e.g. minus.weight = dZ^T [q | xp] is one
 * descriptor with two B operands).  Tiling: MT = ceil(N/32) row tiles of 32 x 32
 * (v_mfma_f32_32x32x16_bf16 on 3-part split operands, or plain bf16 with desc.bf16), column
 * groups of KT tiles (KT = 3, 2, 4, 4 for MT = 3, 4, 2, 1).  A workgroup (4 waves) runs token
 * ranges ("segments") of column groups and writes each into a partial slot
 * partial[slot][n][k]; mep_wgrad_reduce sums the n_split slots in a fixed order into out_i
 * (slots a column group never writes must hold zeros: hosts zero the workspace once).
 * N <= 128; partial holds n_split * N * Ktot floats; every row view of a descriptor shares T
 * and spans < 2^31 floats.  tok_per_split: unused (0).
 * mep_wgrad: `descs` holds the n_desc descriptors FOLLOWED BY an int32 map: max_tiles + 1 CSR
 * offsets (workgroup w runs segments off[w] .. off[w+1]-1 in order), then 4 int32 per segment
 * {descriptor << 8 | column group, t_begin, t_end, slot}.  mep_wgrad_reduce: grid (max_tiles,
 * n_desc), max_tiles = max(ceil(N*Ktot/256)). */
#define MEP_WG_MAX_B 4
typedef struct {
    mep_rows a;                  /* [ntok, N]  (dY)                           */
    mep_rows b[MEP_WG_MAX_B];    /* [ntok, K_i]                               */
    uint64_t out[MEP_WG_MAX_B];  /* dW_i: [N][ldo_i]                          */
    int32_t  kb[MEP_WG_MAX_B];   /* K_i                                       */
    int32_t  ldo[MEP_WG_MAX_B];
    uint64_t partial;            /* workspace [n_split][N][Ktot]              */
    int32_t  n_b, ntok, N, Ktot;
    int32_t  tok_per_split, n_split, accumulate;
    int32_t  out_trans;          /* 1: write dW_i transposed, out_i[k * ldo_i + n] (for weights
                                    whose output dim exceeds 128, e.g. realformer ffn.0 /
                                    [w_qkv.1; w_qkv.2])                                         */
    int32_t  bf16;               /* 1: bf16 operands (MEP_PREC_BF16); 0: 3-part split (fp32)   */
    int32_t  _pad;
} mep_wgrad_desc;
/* k_wgrad geometry of this build: column tiles per group for ceil(N / 32) row tiles, and the
 * workgroups per CU the host sizes the launch for (trimodal.wgrad_geometry / wg_target), for the
 * fp32-split instance (bf16 = 0) or the bf16-path instance (bf16 = 1).
 * mep_wgrad flags: MEP_PREC_BF16 selects the bf16-path instance; every descriptor's bf16 field must
 * match it (a mismatched descriptor gets NaN partials). */
int mep_wgrad_kt(int mt, int bf16);
int mep_wgrad_occupancy(int bf16);
int mep_wgrad(const mep_wgrad_desc* descs, int n_desc, int max_tiles, int flags, mep_stream_t stream);
int mep_wgrad_reduce(const mep_wgrad_desc* descs, int n_desc, int max_tiles, mep_stream_t stream);

/* ---------------------------------------------------------------- residual attention core
 * Per (batch row b, head h, query row i):
 *   s_ik = (q_i . k_k) / sqrt(hd)  [+ c * S_prev[b,h,i,k]]  - 1e8 * (1 - mask[b,k])
 *   P = softmax_k(s);  X[b,i,h*hd:(h+1)*hd] = sum_k P_ik v_k
 * cmu-mosei/run.py:236-256 (== Ren-MME/run.py:188-208, realformer.py:182-204 after w_qkv).
 * hd = 16 (hd = 32 with MEP_ATTN_HD32: forward only).  S_out (post-mask scores, needed by a
 * following residual layer, F7) is optional.
 * Row statistics rowmax / 1/rowsum are saved for the backward. */
typedef struct {
    mep_rows q, k, v;   /* [B*Tq, D], [B*Tk, D], [B*Tk, D]  (k may equal v)   */
    mep_rows x;         /* out [B*Tq, D]                                        */
    uint64_t mask;      /* key mask: mask[b*mask_sB + k]                        */
    int64_t  mask_sB;
    uint64_t s_prev;    /* [B,H,Tq,Tk] or 0                                     */
    uint64_t c;         /* residual coefficient (device float*), used iff s_prev */
    uint64_t s_out;     /* [B,H,Tq,Tk] or 0                                     */
    uint64_t stats;     /* [B,H,Tq,2]: (max log2 e - log2(1/sum), 1/sum) per row;
                           with s_prev: (max, 1/sum) per row, then [B,H,Tq] more floats (ABI 6):
                           each row's P-weighted mean of S_prev, sum_k P_ik S_prev_ik, which
                           the backward subtracts from S_prev in the dc sum (its softmax part
                           sums to 0 over a row; F7 rows at c <= -1 would otherwise cancel
                           ~1e8-sized terms) -- 3 B H Tq floats in all */
    int32_t  B, H, Tq, Tk;
} mep_attn_desc;
/* Launch geometry: forward one wave per (b, h, 64-query chunk), 4 waves (256 threads) per
 * workgroup, max_tiles = max ceil(B * H * ceil(Tq / 64) / 4) over descriptors; backward one
 * 256-thread workgroup per (b, h), max_tiles = max B * H.
 * flags select the specialised kernels: PREV = every descriptor has s_prev, SOUT = every
 * descriptor has s_out (backward: ds_next); SHORT / LONG = descriptors with Tk <= 64 / Tk > 64
 * are present (the forward launches one kernel per class present); backward:
 * MEP_ATTN_DQ_TILES(n) = the largest ceil(Tq / 16) among descriptors with Tk > 64 (their dQ
 * tiles are carried across key chunks in LDS; n <= 127).
 * Products run on the bf16 matrix cores with fp32 operands split into bf16 parts: 3 parts for
 * the scores (fp32-level error), 2 parts elsewhere (relative error <= 2^-17 per product). */
#define MEP_ATTN_PREV  1
#define MEP_ATTN_SOUT  2
#define MEP_ATTN_SHORT 4
#define MEP_ATTN_LONG  8
#define MEP_ATTN_DQ_TILES(n) ((n) << 8)
#define MEP_ATTN_HD32  0x20000   /* head dim 32 (robot_demo.py, D = 192 / H = 6): forward only, fp32 path */
#define MEP_ATTN_KV    0x40000   /* backward: every descriptor has k == v and dk == dv (cmu-mosei, Ren-MME:
                                    cmu-mosei/run.py:241-242 attends with k = v): the short kernel keeps one
                                    register set for K / V and one dK + dV accumulator (4 waves per SIMD);
                                    a descriptor that breaks the promise gets NaN dq rows */
#define MEP_ATTN_SPLITQ 0x80000  /* for launches with few (b, h) units: forward tasks of 16 queries instead
                                    of 64 (max_tiles = ceil(B H ceil(Tq / 16) / 4)); backward: descriptors
                                    with Tk <= 64 also run the workgroup-per-(b, h) kernel, its 4 waves on
                                    separate query tiles (4x the waves of the wave-per-(b, h) kernel) */
#define MEP_ATTN_KCHUNKS(n) ((n) << 20)  /* backward: n = the largest ceil(Tk / 64) among the launch's
                                    descriptors with Tk > 64, 2 <= n <= MEP_ATTN_MAX_KCHUNKS: those run the
                                    chunk-parallel kernel (one workgroup of n waves per (b, h), one wave
                                    per 64-key chunk, no Tq limit); without it the key-chunk-serial
                                    kernel with the LDS-carried dQ (MEP_ATTN_DQ_TILES) */
#define MEP_ATTN_MAX_KCHUNKS 8
int mep_attn_fwd(const mep_attn_desc* descs, int n_desc, int max_tiles, int flags, mep_stream_t stream);

/* mep_attn_general_fwd / _bwd: the reference multi_head_attention for every mask form it accepts
 * (cmu-mosei/run.py:236-257): f.mask = 0 (no mask: nothing subtracted), a key mask (mask_sQ = 0) or
 * a [B, Tq, Tk] mask (element mask[b * mask_sB + q * mask_sQ + k], shared by the heads), residual
 * scores as mep_attn_fwd, k != v, head dim hd <= 64, s = (q . k) / scale with scale = float(sqrt(hd))
 * (a correctly rounded division), Tk <= 4096.  fp32, the score in the reference's op order, one
 * workgroup per (b, h) (grid max_bh = max B * H), every sum in a fixed order.  f.stats receives the
 * raw (max, 1/sum) per row.  Backward: dq accumulated (+=), dk / dv written (dk.ptr == dv.ptr: k is v, their
 * sum written), ds_prev = c * dS (0: none), dc_partial one float per (b, h) (0: none), ds_next the
 * gradient on the post-mask scores output (0: none).  The standalone Attention_Block.forward with a
 * 3-D mask runs here; the model plans never pass one. */
typedef struct {
    mep_attn_desc f;
    int64_t  mask_sQ;
    int32_t  hd;
    float    scale;
} mep_attn_gen_desc;
typedef struct {
    mep_attn_gen_desc g;
    mep_rows dx, dq, dk, dv;
    uint64_t ds_next, ds_prev, dc_partial;
} mep_attn_gen_bwd_desc;
int mep_attn_general_fwd(const mep_attn_gen_desc* descs, int n_desc, int max_bh, mep_stream_t stream);
int mep_attn_general_bwd(const mep_attn_gen_bwd_desc* descs, int n_desc, int max_bh, int max_hd, mep_stream_t stream);

/* Backward of the attention core.  Inputs dx (grad of X), the forward's q/k/v/x/stats/s_prev.
 * Outputs: dq += (written with accumulate semantics onto dq_base), dk, dv (dk==dv pointer ->
 * summed, for k is v), ds_prev = c * dS (grad of S_prev) and a per-workgroup partial of
 * dc = sum dS * S_prev.  ds_next: gradient arriving on this layer's S output (c_next * dS_next)
 * or 0.  Deterministic: every sum (over query tiles, waves and key chunks) has a fixed order. */
typedef struct {
    mep_attn_desc f;
    mep_rows dx;
    mep_rows dq;        /* accumulated into                       */
    mep_rows dk, dv;    /* written (summed when dk.ptr == dv.ptr)  */
    uint64_t ds_next;   /* [B,H,Tq,Tk] or 0                        */
    uint64_t ds_prev;   /* [B,H,Tq,Tk] or 0                        */
    uint64_t dc_partial;/* [B * H * ceil(Tk/64)] floats or 0       */
} mep_attn_bwd_desc;
int mep_attn_bwd(const mep_attn_bwd_desc* descs, int n_desc, int max_tiles, int flags, mep_stream_t stream);

/* ---------------------------------------------------------------- cmu / Ren-MME block epilogue
 * xp = drop(x @ Wp^T);  z = [q | xp] @ Wm^T;  out = drop(LayerNorm(z))
 * cmu-mosei/run.py:257-261 (proj, cat, minus, norm1), Ren-MME/run.py:209-213 (norm2, dropout).
 * D in {32, 64, 96, 128}.  Saves xp (post-dropout), z and (mean, rstd) for the backward. */
typedef struct {
    mep_rows q, x, xp, z, out;
    uint64_t wp, wm, ln_w, ln_b;
    uint64_t stats;      /* [ntok][2] */
    uint64_t seed;       /* device uint64[2] {dropout seed, row0} (0: no dropout).  The mask of
                            element (token tok, feature f) hashes ((row0 * q.T + tok) * D + f):
                            row0 = the first GLOBAL batch row of a data-parallel shard, so every
                            rank draws the masks of the full batch's rows (csrc/common.h drop_scale) */
    int32_t  ntok, D;
    float    drop_p;
    int32_t  drop_stream;/* distinct per block */
    mep_rows out_h;      /* MEP_PREC_BF16: optional bf16 copy of out (ptr 0: none) -- the next
                            layer's q of a residual chain, whose out stays fp32 for the pool */
    uint64_t drop_bits;  /* optional (0: none) uint32 [ceil(ntok/16)][2][64], zeroed once: with
                            dropout the forward writes the keep bits of every 16-token tile and
                            site (0: xp, 1: out) -- lane (c, g) of the tile's wave, bit 4 i + r =
                            feature 16 i + 4 g + r of token 16 tile + c -- and the backward reads
                            them instead of re-hashing (the same masks; ABI 3) */
} mep_epi_desc;
/* D (32/64/96/128, shared by every descriptor of the launch) selects the compiled variant.
 * Geometry: max_tiles = workgroups PER DESCRIPTOR; each workgroup (512 threads) stages its block's
 * weights in LDS once and processes a contiguous range of ceil(ceil(ntok/16) / max_tiles)
 * 16-token tiles.  Row views must be 16-byte aligned (ptr, sB, sT multiples of 4 floats). */
int mep_block_epi_fwd(const mep_epi_desc* descs, int n_desc, int max_tiles, int D, mep_stream_t stream);

/* Backward: dout -> (dropout) -> LN backward -> dz;  dq_direct = dz Wm[:, :D];
 * dxp = drop'(dz Wm[:, D:]);  dx = dxp Wp.  Writes dz, dxp, dx, dq and LayerNorm
 * parameter-gradient partials ln_partial[ceil(ntok / 16)][2][D] (one row per 16 tokens). */
typedef struct {
    mep_epi_desc f;
    mep_rows dout;
    mep_rows dout2;      /* optional second upstream gradient (ptr 0: none), e.g. the next
                            layer's dq for residual chains */
    mep_rows dz, dxp, dx, dq;
    uint64_t ln_partial;
    int32_t  dq_accumulate;
    /* pool_T > 0: dout is not read; the upstream gradient is the mean+max pool's backward
     * (mep_pool_bwd's dx, formed in registers: dmean / pool_T, + dmax at the argmax step) for
     * this block's slice of the pooled tensor -- token tok = b * pool_Tq + t sits at time
     * pool_t0 + t and columns pool_col .. pool_col + D - 1 of [B, pool_T, pool_C]
     * (cmu-mosei/run.py:314-318).  dout2 is still added. */
    int32_t  pool_T;         /* < 0: the mean half of dpooled already holds dmean / |pool_T|
                                (mep_head_desc.mean_div) */
    uint64_t pool_dpooled;   /* [B][2 * pool_C] floats (mean part, then max part) */
    uint64_t pool_argmax;    /* [B][pool_C] int32 */
    int32_t  pool_C, pool_Tq, pool_t0, pool_col;
} mep_epi_bwd_desc;
int mep_block_epi_bwd(const mep_epi_bwd_desc* descs, int n_desc, int max_tiles, int D, mep_stream_t stream);

/* ---------------------------------------------------------------- realformer block epilogue
 * others/realformer.py:182-209 after the attention core (x = attention output, q = block input):
 *   xp = x Wp^T;  h = LN1(q + a*xp);  f1 = relu(h W1^T + b1);  f = f1 W2^T + b2;
 *   out = LN2(h + b*f)
 * a, b: the block's ReZero scalars (device float*).  One workgroup = 64 tokens; the three
 * Linears run on f32 MFMA through LDS.  D in {32, 64, 96, 128}, FD = FFN * D with FFN in {1, 2}.
 * Saves xp, h, f1, f and (mean1, rstd1, mean2, rstd2) per token for the backward. */
typedef struct {
    mep_rows q, x;       /* inputs [ntok, D]                        */
    mep_rows xp, h, f1, f, out;  /* outputs; f1 is [ntok, FD]        */
    uint64_t wp, w1, b1, w2, b2;
    uint64_t ln1_w, ln1_b, ln2_w, ln2_b;
    uint64_t a, b;       /* device float* scalars                   */
    uint64_t stats;      /* [ntok][4]                               */
    int32_t  ntok, D, FD, _pad;
    uint64_t wparts;     /* mep_rfw_epi_*: mep_wsplit parts of [Wp | W1 | W2 | Wp^T | W1^T | W2^T]
                            (MEP_RFW_PART_OFFSET); 0 for mep_rf_epi_*                     */
    /* mep_rfw_epi_fwd, optional (wq_next 0: off): the next layer's query projection fused after
     * LN2, qp_next = out Wq_next^T (wq_next = mep_wsplit parts of Wq_next [D][D]) */
    uint64_t wq_next;
    mep_rows qp_next;
    /* mep_rfw_epi_fwd, optional (zero.ptr 0: off): [ntok, D] rows set to zero for the tile's
     * tokens (the realformer plan's accumulated attention dq, cleared in the forward instead of
     * by a separate fill) */
    mep_rows zero;
} mep_rf_epi_desc;
int mep_rf_epi_fwd(const mep_rf_epi_desc* descs, int n_desc, int max_tiles, int D, int FD, mep_stream_t stream);

/* Backward: dout (+dout2) -> LN2' -> dz2;  df = b dz2;  df1 = relu'(f1) (df W2);
 * dh = dz2 + df1 W1 -> LN1' -> dz1;  dq (+)= dz1 (residual);  dxp = a dz1;  dx = dxp Wp.
 * Writes df, df1, dxp (the wgrad operands), dx (the attention core's dO), dq, and per-tile
 * partial sums partial[tile][5D + FD + 2] = [dLN2.w | dLN2.b | dLN1.w | dLN1.b | db2 | db1 | da | db]. */
typedef struct {
    mep_rf_epi_desc f;
    mep_rows dout, dout2;  /* dout2 optional (ptr 0)                 */
    mep_rows df, df1, dxp, dx, dq;
    uint64_t partial;
    int32_t  dq_accumulate, _pad;
    /* mep_rfw_epi_bwd, optional (wq_in 0: off): the next layer's query-projection input gradient
     * fused before the LN2 backward, dout += dqp_in Wq (wq_in = mep_wsplit parts of Wq^T) */
    uint64_t wq_in;
    mep_rows dqp_in;
} mep_rf_epi_bwd_desc;
int mep_rf_epi_bwd(const mep_rf_epi_bwd_desc* descs, int n_desc, int max_tiles, int D, int FD, mep_stream_t stream);
#define MEP_RF_PARTIAL_STRIDE(D, FD) (5 * (D) + (FD) + 2)
/* token rows per workgroup (= rows per partial row of the backward): which 0 = mep_rf_epi_fwd,
 * 1 = mep_rf_epi_bwd, 2 = mep_rfw_epi_fwd / _bwd and mep_wgemm (the compiled values; hosts size
 * their grids and partial buffers from this, never from their own constants) */
int mep_rf_rows(int which, int D);

/* ---------------------------------------------------------------- wave-tiled realformer path
 * (round 3, others/realformer.py:154-209; csrc/rfw.hip).  Every Linear of the realformer block runs
 * on pre-split weights: one wave per 16-token tile keeps the whole chain of products in registers
 * (the transposed-tile layout: a product's accumulators are the next product's operand), six bf16
 * products per k pair on v_mfma_f32_16x16x32_bf16 (fp32-level, split.h).
 *
 * mep_wsplit: W (R x K; element (n, k) = src[n * ld + k], or src[k * ld + n] when trans) -> its
 * three bf16 parts x = x0 + x1 + x2 (each the round-to-nearest of the remainder), bf16
 * [3][R][Kp / 32][4][8] with Kp = K rounded up to 32 (zero past K): unit (n, p, g) holds
 * W(n, 32p + 4g + 0..3) then W(n, 32p + 16 + 4g + 0..3).  One launch per step before the forward:
 * the weights do not change until the optimizer step. */
typedef struct {
    uint64_t src, dst;
    int32_t  R, K, ld, trans;
    int32_t  nrows, _pad;   /* rows of W (<= R); rows nrows .. R-1 of the parts are zero */
} mep_wsplit_desc;
int mep_wsplit(const mep_wsplit_desc* descs, int n_desc, int max_units, mep_stream_t stream);
#define MEP_WSPLIT_BYTES(R, K) (3 * 2 * (R) * (((K) + 31) / 32 * 32))
/* byte offsets of the six parts at mep_rf_epi_desc.wparts: Wp [D][D], W1 [FD][D], W2 [D][FD], then
 * the transposes Wp^T [D][D], W1^T [D][FD], W2^T [FD][D] (the backward's dY W products) */
#define MEP_RFW_PART_OFFSET(D, FD, i)                                                               \
    ((i) <= 0 ? 0 : (i) == 1 ? MEP_WSPLIT_BYTES(D, D) : (i) == 2 ? MEP_WSPLIT_BYTES(D, D) + MEP_WSPLIT_BYTES(FD, D) \
     : (i) == 3 ? MEP_WSPLIT_BYTES(D, D) + MEP_WSPLIT_BYTES(FD, D) + MEP_WSPLIT_BYTES(D, FD)         \
     : (i) == 4 ? 2 * MEP_WSPLIT_BYTES(D, D) + MEP_WSPLIT_BYTES(FD, D) + MEP_WSPLIT_BYTES(D, FD)     \
     : 2 * MEP_WSPLIT_BYTES(D, D) + MEP_WSPLIT_BYTES(FD, D) + 2 * MEP_WSPLIT_BYTES(D, FD))
#define MEP_RFW_PARTS_BYTES(D, FD) (2 * MEP_WSPLIT_BYTES(D, D) + 2 * MEP_WSPLIT_BYTES(FD, D) + 2 * MEP_WSPLIT_BYTES(D, FD))

/* mep_wgemm: mep_gemm's Y = act(alpha X W'^T + bias + table) (+ Y) with desc.w = the mep_wsplit
 * parts of W' [N][K] (a Linear weight as it is; a dY W product takes the parts of W^T); one wave
 * per 16 tokens x 32 columns, grid (max_tiles, n_desc, ceil(max_n / 32)), max_n = the largest N
 * (<= 256).  ldw, w_nt and bf16 are unused. */
int mep_wgemm(const mep_gemm_desc* descs, int n_desc, int max_tiles, int max_n, mep_stream_t stream);
/* mep_wgemm_ws: mep_wgemm's contract (bit-identical results) with each workgroup's column block of
 * the parts resident in LDS and its waves walking 16-token tiles (persistent grid sized from the
 * device's CU count); max_ntok / max_n / max_k = the largest ntok / N / K of the descriptors,
 * max_k <= 320.  The same token GEMMs as mep_wgemm (others/realformer.py:136-157,182-188).
 * flags: MEP_WGEMM_XVEC when every descriptor's X rows are 16-byte aligned (x.ptr, sB, sT
 * multiples of 4 floats) and readable up to K rounded up to 4 (K % 4 == 0, or rows padded): the
 * X rows are then read in 16-byte blocks (values past K are read and multiplied by zero weights:
 * they must be finite), else one float at a time. */
#define MEP_WGEMM_XVEC 0x1
int mep_wgemm_ws(const mep_gemm_desc* descs, int n_desc, int max_ntok, int max_n, int max_k, int flags,
                 mep_stream_t stream);

/* mep_rfw_front: the realformer front of one modality in one launch -- the Conv1d unify + position
 * table (others/realformer.py:136-152,224-227) and every projection that reads its output U: the
 * [K | V] = U [W_k; W_v]^T of the blocks keyed on this modality and the Q = U W_q^T of its
 * layer-0 blocks (realformer.py:157).  One workgroup (6 waves) per 16-token tile: U's six 16-feature
 * tiles (one per wave) are stored and exchanged through LDS, then the products' output tiles are
 * dealt round-robin to the waves.  unify: the mep_wgemm contract on mep_wsplit parts with D = N =
 * 96, alpha / bias / table as mep_gemm, no relu / accumulate, x rows 16-byte aligned and readable
 * up to K rounded up to 4 (MEP_WGEMM_XVEC), ceil(K / 32) = npk_u in {2, 3, 10}; out[o]: parts of a
 * [N_o][96] weight (N_o % 16 == 0), y_o = U W_o^T written; tile_map[t] = o << 8 | (16-column tile
 * of out[o]) for the t < n_tiles output tiles, 0 <= n_tiles <= MEP_RF_FRONT_MAX_TILES,
 * 0 < n_out <= MEP_RF_FRONT_MAX_OUT (a descriptor outside these bounds writes nothing), every
 * tile_map entry naming an o < n_out and a tile < N_o / 16.  Bit-identical to mep_wgemm on the
 * same parts. */
/* mep_wgemm_sum: out = sum over s < n_src, in order, of mep_wgemm(src[s]) -- the input-gradient
 * products of one modality and their per-modality sum (mep_sum_rows) in one launch, bit-identical
 * to those launches (each source's mep_wgemm epilogue: alpha * acc (+ its y rows when accumulate),
 * then ((0 + v_0) + v_1) + ...).  The sources' y views are read (accumulate) but not written; all
 * sources share ntok and N (<= 256).  Grid (max_tiles, n_desc, ceil(max_n / 16)).
 * (others/realformer.py:157,188: the dQ W_q and [dK | dV] [W_k; W_v] input gradients of U.) */
#define MEP_WGEMM_SUM_MAX 4
typedef struct {
    mep_gemm_desc src[MEP_WGEMM_SUM_MAX];
    int32_t n_src, _pad;
    mep_rows out;
} mep_gemm_sum_desc;
int mep_wgemm_sum(const mep_gemm_sum_desc* descs, int n_desc, int max_tiles, int max_n, mep_stream_t stream);

#define MEP_RF_FRONT_MAX_OUT 12
#define MEP_RF_FRONT_MAX_TILES 96
typedef struct {
    uint64_t w;      /* mep_wsplit parts of W_o [N][96] */
    mep_rows y;      /* output rows, N columns          */
    int32_t  N, _pad;
} mep_rf_front_out;
typedef struct {
    mep_gemm_desc unify;
    int32_t n_out, n_tiles;
    mep_rf_front_out out[MEP_RF_FRONT_MAX_OUT];
    int16_t tile_map[MEP_RF_FRONT_MAX_TILES];
} mep_rf_front_desc;
int mep_rfw_front(const mep_rf_front_desc* descs, int n_desc, int max_tiles, int npk_u, mep_stream_t stream);
/* mep_rfw_epi_fwd / _bwd: mep_rf_epi_fwd / _bwd on the parts at desc.wparts; one wave per 16-token
 * tile, one partial row per tile; D in {32, 64, 96, 128}, FD in {D, 2D}. */
int mep_rfw_epi_fwd(const mep_rf_epi_desc* descs, int n_desc, int max_tiles, int D, int FD, mep_stream_t stream);
int mep_rfw_epi_bwd(const mep_rf_epi_bwd_desc* descs, int n_desc, int max_tiles, int D, int FD, mep_stream_t stream);

/* ---------------------------------------------------------------- State_Transfer head
 * others/realformer.py:257-286 after the fully_connected Linear (run by mep_gemm):
 * per batch row b and utterance i < P (rows r = b*P + i):
 *   h = relu(LN(fc[r]));  [o | g] = h Wc^T + bc  (classifier D -> 12, chunk(2));
 *   i > 0: alpha = sigmoid(g + g_prev);  o = (1 - alpha) o + alpha tanh(out_prev @ trans)
 * plus multi_circle_loss(out, labels) * umask, mean over B*P (realformer.py:311-312).
 * compute_grad: also the backward through the whole recurrence, writing d12 [R,12] (grad at the
 * classifier output), dfc [R,D] (grad at the fc output) and partial[b][2D + 36] =
 * [dLN.w | dLN.b | dtrans].  ext_dout != 0: upstream grad [B,P,6] instead of the fused loss.
 * One wave per batch row; P <= 16, D <= 128. */
typedef struct {
    uint64_t fc;         /* [R, D]                                 */
    uint64_t ln_w, ln_b; /* normalization                          */
    uint64_t wc, bc;     /* classifier [12, D], [12]               */
    uint64_t trans;      /* [6, 6]                                 */
    uint64_t labels;     /* int64 [B, P, 6]                        */
    uint64_t umask;      /* int64 [B, P]                           */
    uint64_t out;        /* out [B, P, 6]                          */
    uint64_t h;          /* out [R, D]                             */
    uint64_t d12, dfc;   /* out [R, 12], [R, D]                    */
    uint64_t row_loss;   /* out [B] (already scaled)               */
    uint64_t partial;    /* out [B][2D + 36]                       */
    uint64_t ext_dout;   /* [B, P, 6] or 0                         */
    int32_t  B, P, D, compute_grad;
    float    loss_scale;
    int32_t  _pad;
    uint64_t scale;      /* device float[1] loss scale read in place of loss_scale, or 0 */
} mep_rf_head_desc;
int mep_rf_head(const mep_rf_head_desc* d, mep_stream_t stream);

/* ---------------------------------------------------------------- row LayerNorm (D <= 256)
 * Ren-MME's shared unify LayerNorm (Ren-MME/run.py:164-166).  fwd: y = LN(x); bwd: dx from dy,
 * per-tile partial dgamma/dbeta. */
typedef struct {
    mep_rows x, y, dy, dx;
    uint64_t w, b, stats, partial;
    int32_t  ntok, D;
    int32_t  dx_accumulate;
    int32_t  bf16;       /* MEP_BF16_STORE: x, y, dy, dx rows are bf16 (statistics fp32) */
} mep_ln_desc;
int mep_layernorm_fwd(const mep_ln_desc* descs, int n_desc, int max_tiles, mep_stream_t stream);
int mep_layernorm_bwd(const mep_ln_desc* descs, int n_desc, int max_tiles, mep_stream_t stream);

/* ---------------------------------------------------------------- reductions
 * Column sums over tiles: out[c] (+)= sum_t partial[t*ld + c].  Used for LayerNorm / bias /
 * position-embedding / per-row head gradient partials.  accumulate: bit 0 = add onto out;
 * MEP_COLSUM_NOT_GRAD = out is not a gradient (e.g. the batch loss), left out of the norm that
 * mep_reduce_grads can fold in. */
#define MEP_COLSUM_NOT_GRAD 2
typedef struct {
    uint64_t partial, out;
    int32_t  n_rows, n_cols, ld, accumulate;
} mep_colsum_desc;
int mep_colsum(const mep_colsum_desc* descs, int n_desc, int max_tiles, mep_stream_t stream);

/* out = sum_i src_i (up to 16 sources), elementwise over ntok x D rows.  accumulate: bit 0 = add
 * onto out; MEP_SUM_BF16 = bf16 source and output rows (the bf16 path), summed in fp32. */
#define MEP_SUM_MAX_SRC 16
#define MEP_SUM_BF16 2
typedef struct {
    mep_rows src[MEP_SUM_MAX_SRC];
    mep_rows out;
    int32_t  n_src, ntok, D, accumulate;
} mep_sum_desc;
int mep_sum_rows(const mep_sum_desc* descs, int n_desc, int max_tiles, mep_stream_t stream);

/* ---------------------------------------------------------------- mean+max pooling
 * pooled[b, 0:C] = mean_t x[b,t,:], pooled[b, C:2C] = max_t x[b,t,:] (first index on ties),
 * cmu-mosei/run.py:314-318, realformer.py:258-262.  bwd: dx = dmean/T + onehot(argmax)*dmax. */
typedef struct {
    uint64_t x, dx;       /* [B, T, C] contiguous          */
    uint64_t pooled, dpooled; /* [B, 2C]                   */
    uint64_t argmax;      /* int32 [B, C]                  */
    int32_t  B, T, C, _pad;
} mep_pool_desc;
/* Grids: forward max_tiles = B * ceil(C / 32); backward max_tiles = B * ceil(T / 16). */
int mep_pool_fwd(const mep_pool_desc* descs, int n_desc, int max_tiles, mep_stream_t stream);
int mep_pool_bwd(const mep_pool_desc* descs, int n_desc, int max_tiles, mep_stream_t stream);

/* ---------------------------------------------------------------- fusion head + loss
 * cmu-mosei Concat_Trans head (cmu-mosei/run.py:319,330-339) / Ren-MME Base_model head
 * (Ren-MME/run.py:271,283-292), fused with multi_circle_loss (cmu-mosei/run.py:342-351) and its
 * .mean() (run.py:366) / multi_loss + R-Drop KL (Ren-MME/run.py:295-304,331-334):
 *   last = Wc0 p0, this = Wc1 p1 (classifier, no bias); y = einsum(this,last,trans);
 *   logits = Wo [this | LN(y)] + bo;  loss = mean_b circle(logits_b, labels_b) (+ KL).
 * One workgroup per row (per row pair with R-Drop).  Writes logits, per-row losses, dpooled
 * (grad of both pooled inputs, scaled for the batch mean) and per-row parameter-gradient
 * partials (layout in head_partial_layout()).  compute_grad = 0 runs forward + loss only. */
typedef struct {
    uint64_t pooled0, pooled1;   /* [B, F]                              */
    uint64_t dpooled0, dpooled1; /* [B, F]                              */
    uint64_t wc0, wc1;           /* [NC, F]                             */
    uint64_t trans;              /* [NC, NC, NC]                        */
    uint64_t ln_w, ln_b;         /* [NC]                                */
    uint64_t wo, bo;             /* [NC, 2NC], [NC]                     */
    uint64_t labels;             /* [B, NC] (int64 or float32)          */
    uint64_t logits;             /* [B, NC]                             */
    uint64_t row_loss;           /* [B]                                 */
    uint64_t partial;            /* [B][head_partial_stride]            */
    int32_t  B, F, NC;
    int32_t  labels_are_float;
    int32_t  rdrop;              /* Ren-MME R-Drop pairs (2i, 2i+1)     */
    int32_t  compute_grad;
    float    loss_scale;         /* d(total loss)/d(row loss) = 1/B (1/B_global under data
                                    parallelism: the rank's share of the global-batch mean) */
    int32_t  rdrop_pairs;        /* R-Drop KL batchmean divisor (pairs of the global batch
                                    under data parallelism); 0 = B / 2                */
    uint64_t ext_dlogits;        /* [B, NC] upstream grad of the logits; when set the fused
                                    loss is skipped and this gradient is back-propagated */
    int32_t  mean_div;           /* > 0: the mean halves of dpooled0/1 (entries < F/2) are written
                                    already divided by mean_div (the pool's time length T), i.e.
                                    as the per-step gradient dmean / T of the mean pool */
    int32_t  _pad;
    uint64_t scale;              /* device float[2] {loss_scale, rdrop_pairs} read at run time in place
                                    of the two fields above, or 0: a captured graph then replays any
                                    data-parallel share (1 / B_global changes per batch) unchanged */
} mep_head_desc;
int mep_head_fwd_bwd(const mep_head_desc* d, mep_stream_t stream);
/* Reduce the per-row partials into the gradient buffers and the batch-mean loss:
 * g_trans, g_ln_w, g_ln_b, g_wo, g_bo (each [.] floats), g_wc0/g_wc1 = dlogit^T pooled, loss[1]. */
int mep_head_reduce(const mep_head_desc* d, uint64_t g_trans, uint64_t g_ln_w, uint64_t g_ln_b,
                    uint64_t g_wo, uint64_t g_bo, uint64_t g_wc0, uint64_t g_wc1, uint64_t loss,
                    mep_stream_t stream);
/* Every gradient reduction of a step in one launch (no dependencies between them): the
 * mep_wgrad_reduce split sums (wgrad_tiles per descriptor, as mep_wgrad_reduce's max_tiles), the
 * mep_colsum column sums (colsum_tiles per descriptor) and, when head is not NULL, the
 * mep_head_reduce sums of the fusion head (same arguments).  Results are bitwise identical to the
 * three separate launches. */
int mep_reduce_grads(const mep_wgrad_desc* wgrad, int n_wgrad, int wgrad_tiles, const mep_colsum_desc* colsum,
                     int n_colsum, int colsum_tiles, const mep_head_desc* head, uint64_t g_trans, uint64_t g_ln_w,
                     uint64_t g_ln_b, uint64_t g_wo, uint64_t g_bo, uint64_t g_wc0, uint64_t g_wc1, uint64_t loss,
                     float* norm, int* step, const float* hyper, mep_stream_t stream);
/* norm != 0 (a single-process step): the clip's gradient-norm pass folded in -- block k of the
 * launch writes the sum of squares of the gradients it wrote to norm[1024 + k], block 0 advances
 * *step and writes the step's Adam scalars (norm = the optimizer workspace of mep_clip_adam_ext,
 * >= 1024 + mep_reduce_grads_grid(..) floats; step / hyper as there).  norm = 0: no norm pass. */
int mep_reduce_grads_grid(int n_wgrad, int wgrad_tiles, int n_colsum, int colsum_tiles, const mep_head_desc* head);
/* mep_reduce_grads over a compact block map (ABI 7): block b of the n_blocks runs job bmap[b] (device
 * uint32) = kind << 30 | descriptor << 12 | block within the descriptor -- kind 0: fusion-head block
 * (as mep_head_reduce's blocks), 1: split-sum block of wgrad[descriptor] (1,024 entries each), 2:
 * column-sum tile of colsum[descriptor] (32 columns) -- so the empty blocks of the rectangular grid
 * (every descriptor padded to the largest one's block count) are never launched: State_Transfer's
 * reduction is 29,430 rectangular blocks for a few thousand jobs.  Results are those of
 * mep_reduce_grads; with norm, block b writes norm[1024 + b] (n_ext = n_blocks). */
int mep_reduce_grads_mapped(const mep_wgrad_desc* wgrad, const mep_colsum_desc* colsum, const mep_head_desc* head,
                            uint64_t g_trans, uint64_t g_ln_w, uint64_t g_ln_b, uint64_t g_wo, uint64_t g_bo,
                            uint64_t g_wc0, uint64_t g_wc1, uint64_t loss, float* norm, int* step, const float* hyper,
                            const uint32_t* bmap, int n_blocks, mep_stream_t stream);
int mep_head_partial_stride(int NC);

/* multi_circle_loss per row (cmu-mosei/run.py:342-351) as a standalone op for callers that
 * compute the loss outside the model: row_loss[b] and dunit[b, :] = d row_loss[b] / d logits[b, :].
 * mep_circle_loss_bwd: dlogits[b, n] = grad_rows[b] * dunit[b, n]. */
int mep_circle_loss_fwd(const float* logits, const void* labels, int labels_are_float, int B, int NC,
                        float* row_loss, float* dunit, mep_stream_t stream);
int mep_circle_loss_bwd(const float* dunit, const float* grad_rows, int B, int NC, float* dlogits,
                        mep_stream_t stream);

/* ---------------------------------------------------------------- optimizer
 * clip_grad_norm_(max_norm) (cmu-mosei/run.py:368) + AdamW / Adam step (run.py:369,398;
 * realformer.py:342) over a flat fp32 parameter buffer.  `segs` (host array, <= 16) lists
 * [offset, length) ranges of parameters that HAVE a gradient this step; torch skips grad-None
 * parameters entirely (no decay, no state update) and so does this.  Device-side state so a
 * captured graph replays correctly: hyper = float[7] {lr, beta1, beta2, eps, weight_decay,
 * max_norm, grad_scale (0 = 1; 1/world after a SUM all-reduce)}; step = int[1] (incremented by the call, then used as the 1-based step t).
 * partial: workspace of >= 1024 floats.  decoupled = 1: AdamW; 0: Adam (L2 decay in the grad).
 * gnorm_out (device float*, may be 0) receives the pre-clip global norm.  Grads are clipped in
 * place, as clip_grad_norm_ does. */
typedef struct {
    int64_t offset, length;
} mep_seg;
int mep_clip_adam(float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                  const mep_seg* segs, int n_seg, int64_t total_len, float* partial,
                  float* gnorm_out, const float* hyper, int* step, int decoupled,
                  mep_stream_t stream);
/* n_ext > 0: the norm partials (n_ext of them, at partial[1024 ..]) and the step's scalars were
 * written by a mep_reduce_grads launch with norm = partial, which also advanced *step: the norm
 * launch is skipped.  n_ext = 0: mep_clip_adam. */
int mep_clip_adam_ext(float* params, float* grads, float* exp_avg, float* exp_avg_sq,
                      const mep_seg* segs, int n_seg, int64_t total_len, float* partial,
                      float* gnorm_out, const float* hyper, int* step, int decoupled, int n_ext,
                      mep_stream_t stream);

/* advance the device-side dropout seed (graph-replay safe) */
int mep_seed_advance(uint64_t* seed, mep_stream_t stream);

/* ---------------------------------------------------------------- evaluation
 * Ensemble combine + threshold sweep.  Replaces the test() loops of others/realformer.py:395-477
 * (pred = pred_1 * 0.6 + pred_2 * 0.4; pred > threshold for t/200 - 1, t < 400; a full test-set
 * forward per threshold) and cmu-mosei/run.py:456-498 (mean of 4 models, fixed per-class
 * thresholds): the logits are computed once and every threshold is counted on the GPU.
 *   score[n, c] = (((p_0[n,c] * w_0) + p_1[n,c] * w_1) + ...) / post_div   (fp32, each op rounded:
 *   realformer w = {0.6, 0.4}, post_div 1; cmu-mosei w = 1, post_div = the model count)
 *   pred = score > thr(t, c)  (fp32 compare, as torch compares an fp32 tensor with a scalar);
 *   thr(t, c) = thresholds[t] or, with thr_per_class, thresholds[t * C + c] (run.py:478-483)
 *   counts[t, c, :] += {tp, fp, fn, tn} over the rows n that count.
 * A row counts when row_mask == 0, or when row_mask[i][0..j] are all 1 for n = i * P + j
 * (the `if mask == 1 ... else: break` walk of realformer.py:423-437).  Labels are positive iff
 * != 0.  counts is int32 and accumulated into (the caller zeroes it); exact integer atomics, so
 * the result does not depend on the launch order.  Launch: ceil(N/256) x ceil(n_thr/64)
 * workgroups of 256 threads; the rows of a workgroup are staged in LDS once. */
#define MEP_EVAL_MAX_MODELS 8
#define MEP_EVAL_MAX_CLASSES 16
typedef struct {
    uint64_t preds[MEP_EVAL_MAX_MODELS];   /* model m's scores, [N, C] fp32, row stride ld_pred */
    float    weights[MEP_EVAL_MAX_MODELS];
    uint64_t labels;       /* [N, C] int64, row stride ld_label                          */
    uint64_t row_mask;     /* [N / P, P] int64 utterance mask, or 0 (every row counts)    */
    uint64_t thresholds;   /* [n_thr] fp32, or [n_thr, C] with thr_per_class              */
    uint64_t scores;       /* [N, C] fp32 out (combined scores, every row), or 0          */
    uint64_t counts;       /* [n_thr, C, 4] int32, accumulated: tp, fp, fn, tn            */
    int32_t  n_models, N, C, n_thr, P, ld_pred, ld_label;
    float    post_div;
    int32_t  thr_per_class;
    int32_t  sorted;       /* 1: thr(t, c) is non-decreasing in t for every c (caller's promise):
                              histogram + suffix-sum path, O(N C log n_thr); needs hist and
                              C * (3 n_thr + 2) * 4 <= 65536                                 */
    uint64_t hist;         /* sorted mode: int32 workspace [C, 2, n_thr + 1], zeroed by the caller
                              once; every call leaves it zeroed                                */
} mep_sweep_desc;
int mep_threshold_sweep(const mep_sweep_desc* d, mep_stream_t stream);

/* ---------------------------------------------------------------- batch assembly
 * Windowed, masked feature slots gathered from packed, HBM-resident sequences.  Replaces the
 * host numpy of masking() + data_loader() in cmu-mosei/run.py:104-198 and
 * others/realformer.py:72-82,94-125, and the torch.cuda.FloatTensor(list) copy of the batch
 * (cmu-mosei/run.py:362, realformer.py:307-309).  For output slot i of a descriptor:
 *   seq = sel[i] (-1: an empty 'no_name' slot -> zero features, zero mask)
 *   summary = 1 (cmu): rows 0..2 = max, min, mean over all L frames of seq (in the source dtype,
 *     the mean as sum-in-frame-order / L), rows 3.. = frames start, start+1, ... (zero past L);
 *     mask[t] = 1 for t < 3 + (L - start)
 *   summary = 0 (realformer): rows 0.. = frames start, ...; mask[t] = 1 for t < L - start
 *   clean = 1: inf / nan source values read as -71 (cmu audio, every realformer modality)
 * The host picks each slot's window start (first window 0, last window L - (m_len - 3), realformer
 * max(0, L - m_len)).  Launch: n_out x n_desc workgroups of 256 threads. */
#define MEP_WINDOW_MAX_DESC 4
typedef struct {
    uint64_t src;      /* packed frames [n_frames, d], fp32 (src_f64 = 0) or fp64 (src_f64 = 1) */
    uint64_t segs;     /* mep_seg [n_seq]: first frame and frame count of each sequence          */
    uint64_t sel;      /* int32 [n_out]: sequence of each output slot, -1 = empty slot           */
    uint64_t start;    /* int32 [n_out]: first frame of the slot's window                        */
    uint64_t out;      /* fp32 [n_out, m_len, d]                                                 */
    uint64_t mask;     /* fp32 [n_out, m_len]                                                    */
    int32_t  n_out, m_len, d, src_f64, summary, clean, n_seq, _pad;
} mep_window_desc;
int mep_assemble_windows(const mep_window_desc* descs, int n_desc, mep_stream_t stream);

/* ---------------------------------------------------------------- measurement
 * Not a reference interface: the measured HBM peak bench.py reports beside the 8 TB/s spec
 * ("vendor spec and a measured copy-kernel peak on the box").  Streams n16 16-byte units with
 * n_wg workgroups of 256 threads: mode 0 copies src -> dst (2 x 16 n16 bytes), mode 1 reads src
 * (16 n16 bytes; one xor dword per thread written to dst, so dst holds n_wg * 256 dwords), mode 2
 * zero-fills dst (16 n16 bytes).  Buffers 16-byte aligned.  mode | MEP_PROBE_BLOCKED: each
 * workgroup streams one contiguous span (32 KiB per step) instead of the grid-stride order (mode 1
 * then writes n_wg * 256 dwords too); | MEP_PROBE_NT: nontemporal loads / stores (blocked only). */
#define MEP_PROBE_BLOCKED 4
#define MEP_PROBE_NT 8
int mep_hbm_probe(const void* src, void* dst, int64_t n16, int mode, int n_wg, mep_stream_t stream);

/* Writes the device's 100-MHz real-time counter to slots[i] (uint64) when this one-wave kernel
 * starts (measurement, not a reference interface): stamps placed between the launches of a
 * captured step bracket each launch's device time (bench.py). */
int mep_stamp(void* slots, int i, mep_stream_t stream);
/* The counter's rate in kHz (hipDeviceAttributeWallClockRate of the current device), or < 0. */
int mep_stamp_khz(void);

/* ---------------------------------------------------------------- misc */
int mep_abi_version(void);
int mep_last_error(char* buf, size_t len);
int mep_device_sync(void);

#ifdef __cplusplus
}
#endif
#endif /* MEP_H_ */
