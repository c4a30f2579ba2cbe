// Reductions, clip_grad_norm_ + AdamW/Adam over the flat parameter buffer, dropout seed.
//
// clip + optimizer: cmu-mosei/run.py:368-369 (clip_grad_norm_(model.parameters(), CLIP),
// optimizer.step()), AdamW(lr) at run.py:398, Adam(lr) at others/realformer.py:342.
// Two launches: (1) per-workgroup partial sums of g^2 over the segments that have gradients;
// (2) every workgroup re-reduces the partials in the same fixed order (deterministic, no
// grid barrier), forms coef = min(1, max_norm / (||g|| + 1e-6)) and applies the torch update
//   p *= 1 - lr*wd (AdamW);  m = lerp(m, g, 1-b1);  v = b2 v + (1-b2) g^2;
//   p -= (lr / (1-b1^t)) * m / (sqrt(v) / sqrt(1-b2^t) + eps)
// Hyper-parameters and the step counter live in device memory so a captured graph replays
// with the current values.
#include "common.h"

using namespace mep;

namespace {

constexpr int NPART = OPT_NPART;    // per-workgroup norm partials; partial[NPART ..] holds the step's scalars
constexpr int SCAL = OPT_SCAL;      // partial[SCAL + 0..1]: lr / (1 - b1^t), sqrt(1 - b2^t)
constexpr int OPT_THREADS = 256;
constexpr int MAX_SEG = 16;

struct Segs {
    int64_t off[MAX_SEG];
    int64_t len[MAX_SEG];
    int n;
};

// Segments whose offset is a multiple of 4 floats run as float4 streams (the flat buffers are
// 256-byte aligned), the rest of a segment (tail, or a misaligned segment) element by element.
__global__ __launch_bounds__(OPT_THREADS) void k_sqnorm(const float* __restrict__ g, Segs segs,
                                                        float* __restrict__ partial, int* __restrict__ step,
                                                        const float* __restrict__ hyper) {
    float s = 0.f;
    const int64_t gid = (int64_t)blockIdx.x * OPT_THREADS + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * OPT_THREADS;
    for (int si = 0; si < segs.n; ++si) {
        const float* gs = g + segs.off[si];
        const int64_t n = segs.len[si];
        const int64_t n4 = (segs.off[si] & 3) == 0 ? n >> 2 : 0;
        for (int64_t i = gid; i < n4; i += stride) {
            const float4 v = ldg4(G<const float>(reinterpret_cast<uint64_t>(gs)) + 4 * i);
            s = fmaf(v.x, v.x, s);
            s = fmaf(v.y, v.y, s);
            s = fmaf(v.z, v.z, s);
            s = fmaf(v.w, v.w, s);
        }
        for (int64_t i = 4 * n4 + gid; i < n; i += stride) s = fmaf(gs[i], gs[i], s);
    }
    __shared__ float red[OPT_THREADS / 64];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int w = 0; w < OPT_THREADS / 64; ++w) t += red[w];
        partial[blockIdx.x] = t;
        if (blockIdx.x == 0 && step) opt_step_scalars(partial, step, hyper);
    }
}

struct AdamCoef {
    float gs, step_size, bc2_sqrt, decay, one_m_b1, b2, one_m_b2, wd, eps;
    int decoupled;
};

MEP_DEV void adam_elem(float& pv, float& gv, float& mv, float& vv, const AdamCoef& k) {
    gv = gv * k.gs;
    float ge = gv;
    if (k.decoupled) pv *= k.decay;
    else if (k.wd != 0.f) ge = ge + pv * k.wd;
    mv = mv + (ge - mv) * k.one_m_b1;
    vv = vv * k.b2 + k.one_m_b2 * ge * ge;
    const float denom = sqrtf(vv) / k.bc2_sqrt + k.eps;
    pv = pv - k.step_size * mv / denom;
}

// hyper: [lr, beta1, beta2, eps, weight_decay, max_norm, grad_scale]
__global__ __launch_bounds__(OPT_THREADS) void k_clip_adam(float* __restrict__ p, float* __restrict__ g,
                                                           float* __restrict__ m, float* __restrict__ v, Segs segs,
                                                           const float* __restrict__ partial, int npart, int pbase,
                                                           const float* __restrict__ hyper,
                                                           const int* __restrict__ step, float* gnorm_out,
                                                           int decoupled) {
    const int64_t gid = (int64_t)blockIdx.x * OPT_THREADS + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * OPT_THREADS;
    // the thread's first float4 of segment 0 is loaded before the norm reduction: the update's
    // operands do not depend on the norm, so their latency runs under the partial-sum loads (the
    // launch is sized to about one float4 per thread, so this is most of the update's reads)
    float4 P0 = {}, G0 = {}, M0 = {}, V0 = {};
    const bool pre = segs.n > 0 && (segs.off[0] & 3) == 0 && gid < (segs.len[0] >> 2);
    if (pre) {
        const int64_t j = segs.off[0] + 4 * gid;
        P0 = ldg4(G<float>(reinterpret_cast<uint64_t>(p)) + j);
        G0 = ldg4(G<float>(reinterpret_cast<uint64_t>(g)) + j);
        M0 = ldg4(G<float>(reinterpret_cast<uint64_t>(m)) + j);
        V0 = ldg4(G<float>(reinterpret_cast<uint64_t>(v)) + j);
    }
    // every workgroup sums the partials in the same fixed order (lane-strided, then the wave's
    // DPP tree, then the 4 waves in order): identical totals, no grid barrier
    __shared__ float red[OPT_THREADS / 64];
    float s = 0.f;
    // 16 partials per thread in flight at once (a folded reduction can leave thousands): one
    // memory latency per 4096 partials, fixed order
    for (int i0 = 0; i0 < npart; i0 += 16 * OPT_THREADS) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int i = i0 + (int)threadIdx.x + OPT_THREADS * u;
            const float p = partial[pbase + min(i, npart - 1)];   // clamped: no branch per load
            v[u] = i < npart ? p : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) s += v[u];
    }
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    const float sum = ((red[0] + red[1]) + red[2]) + red[3];
    const float gscale = hyper[6] > 0.f ? hyper[6] : 1.0f;   // 1/world after a SUM all-reduce
    const float total = sqrtf(sum) * gscale;
    const float max_norm = hyper[5];
    const float coef = fminf(max_norm / (total + 1e-6f), 1.0f);
    if (blockIdx.x == 0 && threadIdx.x == 0 && gnorm_out) *gnorm_out = total;
    const float lr = hyper[0], b1 = hyper[1], b2 = hyper[2], wd = hyper[4];
    AdamCoef k;
    k.gs = gscale * coef;
    k.step_size = partial[SCAL];
    k.bc2_sqrt = partial[SCAL + 1];
    k.decay = (float)(1.0 - (double)lr * (double)wd);
    k.one_m_b1 = (float)(1.0 - (double)b1);
    k.b2 = b2;
    k.one_m_b2 = (float)(1.0 - (double)b2);
    k.wd = wd;
    k.eps = hyper[3];
    k.decoupled = decoupled;
    for (int si = 0; si < segs.n; ++si) {
        const int64_t off = segs.off[si], n = segs.len[si];
        const int64_t n4 = (off & 3) == 0 ? n >> 2 : 0;
        for (int64_t i = gid; i < n4; i += stride) {
            const int64_t j = off + 4 * i;
            gfloat* pp = G<float>(reinterpret_cast<uint64_t>(p)) + j;
            gfloat* gp = G<float>(reinterpret_cast<uint64_t>(g)) + j;
            gfloat* mp = G<float>(reinterpret_cast<uint64_t>(m)) + j;
            gfloat* vp = G<float>(reinterpret_cast<uint64_t>(v)) + j;
            float4 P4, G4, M4, V4;
            if (si == 0 && i == gid) {   // prefetched above (pre holds exactly when this runs)
                P4 = P0; G4 = G0; M4 = M0; V4 = V0;
            } else {
                P4 = ldg4(pp); G4 = ldg4(gp); M4 = ldg4(mp); V4 = ldg4(vp);
            }
            adam_elem(P4.x, G4.x, M4.x, V4.x, k);
            adam_elem(P4.y, G4.y, M4.y, V4.y, k);
            adam_elem(P4.z, G4.z, M4.z, V4.z, k);
            adam_elem(P4.w, G4.w, M4.w, V4.w, k);
            stg4(pp, P4);
            stg4(gp, G4);
            stg4(mp, M4);
            stg4(vp, V4);
        }
        for (int64_t i = 4 * n4 + gid; i < n; i += stride) {
            const int64_t j = off + i;
            float pv = p[j], gv = g[j], mv = m[j], vv = v[j];
            adam_elem(pv, gv, mv, vv, k);
            p[j] = pv;
            g[j] = gv;
            m[j] = mv;
            v[j] = vv;
        }
    }
}

__global__ void k_seed(uint64_t* seed) { seed[0] = mix64(seed[0] + 0x9E3779B97F4A7C15ull); }

// ---------------------------------------------------------------- colsum / row sums
// workgroup = 32 columns x 8 row groups; fixed-order combine (deterministic)
__global__ __launch_bounds__(256) void k_colsum(const mep_colsum_desc* __restrict__ descs) {
    colsum_block(descs[blockIdx.y], blockIdx.x);
}

// out = sum of sources, 4 columns per thread (D % 4 == 0 for every model width); HS: bf16 source
// and output rows (MEP_SUM_BF16, the bf16 path), summed in fp32
// Sources in groups of SR_GROUP: every load of a group is issued before its first add (one
// memory round trip per group, not per source); the adds keep source order.
constexpr int SR_GROUP = 8;
template <bool HS>
MEP_DEV void sum_rows(const mep_sum_desc& d) {
    const int D4 = d.D / 4;
    const int64_t total = (int64_t)d.ntok * D4;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
        const int tok = (int)(i / D4), c = 4 * (int)(i - (int64_t)tok * D4);
        f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int k0 = 0; k0 < d.n_src; k0 += SR_GROUP) {
            f32x4 v[SR_GROUP];
#pragma unroll
            for (int k = 0; k < SR_GROUP; ++k)
                if (k0 + k < d.n_src) v[k] = ld4a(rowa<HS>(d.src[k0 + k], tok) + c);
#pragma unroll
            for (int k = 0; k < SR_GROUP; ++k)
                if (k0 + k < d.n_src) s += v[k];
        }
        const auto o = rowa<HS>(d.out, tok) + c;
        if (d.accumulate & 1) s += ld4a(o);
        st4a(o, s);
    }
}
__global__ __launch_bounds__(256) void k_sum_rows(const mep_sum_desc* __restrict__ descs) {
    const mep_sum_desc& d = descs[blockIdx.y];
    if (d.accumulate & MEP_SUM_BF16) sum_rows<true>(d);
    else sum_rows<false>(d);
}

}  // namespace

extern "C" int mep_clip_adam_ext(float* params, float* grads, float* exp_avg, float* exp_avg_sq, const mep_seg* segs,
                                 int n_seg, int64_t total_len, float* partial, float* gnorm_out, const float* hyper,
                                 int* step, int decoupled, int n_ext, mep_stream_t stream) {
    if (n_seg <= 0 || n_seg > MAX_SEG || !partial || !hyper || !step) {
        mep_set_error("mep_clip_adam: need 1..16 segments, partial, hyper and step buffers");
        return MEP_EINVAL;
    }
    Segs s;
    s.n = n_seg;
    int64_t longest = 0;
    for (int i = 0; i < n_seg; ++i) {
        s.off[i] = segs[i].offset;
        s.len[i] = segs[i].length;
        if (segs[i].offset < 0 || segs[i].offset + segs[i].length > total_len) {
            mep_set_error("mep_clip_adam: segment out of range");
            return MEP_EINVAL;
        }
        if (segs[i].length > longest) longest = segs[i].length;
    }
    // one float4 per thread (a single HBM round trip per lane in the update pass; 4 float4 per
    // thread serialised 4 dependent load -> store trips), one partial per workgroup for the norm
    // The norm pass has one partial slot per workgroup (at most NPART); the update pass is not
    // bound by the slots and runs one float4 per thread of the longest segment (at most 65535
    // workgroups), so no thread loops over dependent load -> store trips
    int grid_u = (int)((longest + OPT_THREADS * 4 - 1) / (OPT_THREADS * 4));
    grid_u = grid_u < 1 ? 1 : (grid_u > 65535 ? 65535 : grid_u);
    const int grid_n = grid_u > NPART ? NPART : grid_u;
    if (n_ext <= 0) {
        hipLaunchKernelGGL(k_sqnorm, dim3(grid_n), dim3(OPT_THREADS), 0, (hipStream_t)stream, grads, s, partial, step, hyper);
        int rc = mep_check_launch("mep_clip_adam/sqnorm");
        if (rc) return rc;
    }
    hipLaunchKernelGGL(k_clip_adam, dim3(grid_u), dim3(OPT_THREADS), 0, (hipStream_t)stream, params, grads, exp_avg,
                       exp_avg_sq, s, partial, n_ext > 0 ? n_ext : grid_n, n_ext > 0 ? OPT_EXT0 : 0, hyper, step,
                       gnorm_out, decoupled);
    return mep_check_launch("mep_clip_adam/update");
}

extern "C" int mep_clip_adam(float* params, float* grads, float* exp_avg, float* exp_avg_sq, const mep_seg* segs,
                             int n_seg, int64_t total_len, float* partial, float* gnorm_out, const float* hyper,
                             int* step, int decoupled, mep_stream_t stream) {
    return mep_clip_adam_ext(params, grads, exp_avg, exp_avg_sq, segs, n_seg, total_len, partial, gnorm_out, hyper,
                             step, decoupled, 0, stream);
}

extern "C" int mep_seed_advance(uint64_t* seed, mep_stream_t stream) {
    hipLaunchKernelGGL(k_seed, dim3(1), dim3(1), 0, (hipStream_t)stream, seed);
    return mep_check_launch("mep_seed_advance");
}

extern "C" int mep_colsum(const mep_colsum_desc* descs, int n_desc, int max_tiles, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    hipLaunchKernelGGL(k_colsum, dim3(max_tiles, n_desc), dim3(256), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_colsum");
}

extern "C" int mep_sum_rows(const mep_sum_desc* descs, int n_desc, int max_tiles, mep_stream_t stream) {
    if (n_desc <= 0 || max_tiles <= 0) return 0;
    hipLaunchKernelGGL(k_sum_rows, dim3(max_tiles, n_desc), dim3(256), 0, (hipStream_t)stream, descs);
    return mep_check_launch("mep_sum_rows");
}
