// Batch assembly on the device: windowed, masked feature slots gathered from HBM-resident
// packed sequences (include/mep.h, mep_assemble_windows).
//
// Reference: masking() + data_loader() of cmu-mosei/run.py:104-198 (3 summary rows max / min /
// mean over the whole sequence, then the first or the last m_len - 3 frames; audio inf / nan ->
// -71 before the statistics) and others/realformer.py:72-82,94-125 (the last m_len frames,
// zero-padded, inf / nan -> -71 element by element).  The reference builds every slot with numpy
// on the host and copies the batch with torch.cuda.FloatTensor(list); here the raw sequences stay
// in HBM (the whole CMU-MOSEI feature set is a few GB against 288 GB) and one launch writes the
// [n_out, m_len, d] slots and their masks for every modality.
//
// Mapping: one workgroup per (output slot, modality).  The frame rows are a contiguous span of
// the packed source, copied with coalesced loads.  The summary statistics stage the sequence
// through LDS in chunks (coalesced, all 256 lanes loading), then one lane per column walks the
// chunk in frame order, so the running sum has the reference's order (numpy's axis-0 reduction
// adds row after row): the mean is bit-identical, max / min are order free (NaN propagates as in
// numpy).  HBM-bound: each slot reads its window (and, with summaries, its sequence) once.
#include "common.h"

using namespace mep;

namespace {

constexpr int BA_THREADS = 256;
constexpr int BA_LDS_BYTES = 65536;   // 2 workgroups per CU; larger chunks = fewer exposed HBM round trips
constexpr int BA_MAX_COLS_PER_LANE = 4;   // summary mode: d <= 1024

struct WindowArgs {
    mep_window_desc d[MEP_WINDOW_MAX_DESC];
};

template <typename T>
MEP_DEV T clean_val(T v, int clean) {
    // realformer.py:78-81 / cmu-mosei/run.py:106-109: math.isinf(x) or math.isnan(x) -> -71.
    return (clean && (v != v || v == (T)INFINITY || v == -(T)INFINITY)) ? (T)-71 : v;
}

MEP_DEV float div_rn(float a, float b) { return __fdiv_rn(a, b); }
MEP_DEV double div_rn(double a, double b) { return a / b; }

template <typename T>
MEP_DEV void copy_frames(const mep_window_desc& D, int64_t off, int start, int avail, int P0, MEP_G float* out) {
    const int d = D.d;
    const int rows = D.m_len - P0;
    const int64_t n = (int64_t)rows * d;
    const int64_t n_src = (int64_t)min(avail, rows) * d;
    const MEP_G T* src = G<const T>(D.src) + (off + start) * (int64_t)d;
    MEP_G float* dst = out + (int64_t)P0 * d;
    // 16 elements per lane per pass, every load issued before the first store (dst may alias
    // nothing, but the compiler cannot know that)
    constexpr int U = 16;   // a 47 x 300 text window is 55 elements per lane: 4 round trips, not 14
    for (int64_t i0 = threadIdx.x; i0 < n; i0 += U * BA_THREADS) {
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * BA_THREADS;
            v[u] = i < n_src ? src[i] : (T)0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * BA_THREADS;
            if (i < n) dst[i] = i < n_src ? (float)clean_val<T>(v[u], D.clean) : 0.f;
        }
    }
}

template <typename T>
MEP_DEV void summary_rows(const mep_window_desc& D, int64_t off, int L, MEP_G float* out, unsigned char* lds) {
    // Chunks of ch frames fill the LDS buffer; the next chunk is loaded into registers (E values
    // per lane, coalesced) while the current one is walked, so the frame-order sums wait on LDS
    // only, not on HBM latency.
    constexpr int E = BA_LDS_BYTES / (int)sizeof(T) / BA_THREADS;
    T* buf = reinterpret_cast<T*>(lds);
    const int d = D.d;
    const int ch = max(1, BA_LDS_BYTES / (int)(d * sizeof(T)));
    const bool split = d <= BA_THREADS / 2;
    T mx[BA_MAX_COLS_PER_LANE], mn[BA_MAX_COLS_PER_LANE], sm[BA_MAX_COLS_PER_LANE];
#pragma unroll
    for (int k = 0; k < BA_MAX_COLS_PER_LANE; ++k) { mx[k] = -(T)INFINITY; mn[k] = (T)INFINITY; sm[k] = -(T)0; }   // -0 + x == x, signed zeros included
    const MEP_G T* src = G<const T>(D.src) + off * (int64_t)d;
    T pre[E];
    {
        const int n = min(ch, L) * d;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int i = threadIdx.x + e * BA_THREADS;
            pre[e] = src[min(i, n - 1)];   // clamped, not predicated: the loads issue back to back
        }
    }
    for (int f0 = 0; f0 < L; f0 += ch) {
        const int nf = min(ch, L - f0);
        const int n = nf * d;
        __syncthreads();   // the previous chunk has been walked
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const int i = threadIdx.x + e * BA_THREADS;
            if (i < n) buf[i] = clean_val<T>(pre[e], D.clean);
        }
        __syncthreads();
        const int f1 = f0 + ch;
        if (f1 < L) {
            const int n1 = min(ch, L - f1) * d;
            const MEP_G T* s1 = src + (int64_t)f1 * d;
#pragma unroll
            for (int e = 0; e < E; ++e) {
                const int i = threadIdx.x + e * BA_THREADS;
                pre[e] = s1[min(i, n1 - 1)];   // lanes past the chunk re-read its last element
            }
        }
        if (split) {
            // d <= 128: waves 0-1 carry the serial frame-order sums, waves 2-3 the order-free
            // max / min of the same columns, side by side on other SIMDs
            const int c = threadIdx.x & (BA_THREADS / 2 - 1);
            if (c < d) {
                if (threadIdx.x < BA_THREADS / 2) {
                    T s = sm[0];
#pragma unroll 8
                    for (int f = 0; f < nf; ++f) s = s + buf[f * d + c];
                    sm[0] = s;
                } else {
                    T a = mx[0], b = mn[0];
                    if (D.clean) {
#pragma unroll 8
                        for (int f = 0; f < nf; ++f) {
                            const T v = buf[f * d + c];
                            a = v > a ? v : a;
                            b = v < b ? v : b;
                        }
                    } else {
#pragma unroll 8
                        for (int f = 0; f < nf; ++f) {
                            const T v = buf[f * d + c];
                            a = (v > a || v != v) ? v : a;
                            b = (v < b || v != v) ? v : b;
                        }
                    }
                    mx[0] = a; mn[0] = b;
                }
            }
            continue;
        }
#pragma unroll
        for (int k = 0; k < BA_MAX_COLS_PER_LANE; ++k) {
            const int c = threadIdx.x + k * BA_THREADS;
            if (c < d) {
                T a = mx[k], b = mn[k], s = sm[k];
                if (D.clean) {
                    // cleaned values hold no NaN: two selects per frame (ties keep the earlier
                    // frame, as numpy's reduction does)
#pragma unroll 8
                    for (int f = 0; f < nf; ++f) {
                        const T v = buf[f * d + c];
                        a = v > a ? v : a;
                        b = v < b ? v : b;
                        s = s + v;
                    }
                } else {
#pragma unroll 8
                    for (int f = 0; f < nf; ++f) {
                        const T v = buf[f * d + c];
                        // numpy maximum / minimum: a NaN operand wins, and stays
                        a = (v > a || v != v) ? v : a;
                        b = (v < b || v != v) ? v : b;
                        s = s + v;
                    }
                }
                mx[k] = a; mn[k] = b; sm[k] = s;
            }
        }
    }
    if (split) {
        const int c = threadIdx.x & (BA_THREADS / 2 - 1);
        if (c < d) {
            if (threadIdx.x < BA_THREADS / 2) {
                out[2 * d + c] = (float)div_rn(sm[0], (T)L);
            } else {
                out[c] = (float)mx[0];
                out[d + c] = (float)mn[0];
            }
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < BA_MAX_COLS_PER_LANE; ++k) {
        const int c = threadIdx.x + k * BA_THREADS;
        if (c < d) {
            out[c] = (float)mx[k];
            out[d + c] = (float)mn[k];
            out[2 * d + c] = (float)div_rn(sm[k], (T)L);   // np.mean: sum / count in the input dtype
        }
    }
}

__global__ __launch_bounds__(BA_THREADS) void k_assemble(WindowArgs args) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[BA_LDS_BYTES];
    const mep_window_desc& D = args.d[blockIdx.y];
    const int slot = blockIdx.x;
    if (slot >= D.n_out) return;   // uniform per workgroup
    int seq = G<const int32_t>(D.sel)[slot];
    int64_t off = 0;
    int L = 0;
    if (seq >= 0 && seq < D.n_seq) {
        const MEP_G mep_seg* sg = G<const mep_seg>(D.segs) + seq;
        off = sg->offset;
        L = (int)sg->length;
    } else {
        seq = -1;
    }
    // window start clamped into the sequence: every source read stays inside [off, off + L)
    const int start = seq >= 0 ? max(0, min(G<const int32_t>(D.start)[slot], L)) : 0;
    const int P0 = (D.summary && seq >= 0) ? 3 : 0;
    const int avail = seq >= 0 ? max(0, L - start) : 0;
    MEP_G float* out = G<float>(D.out) + (int64_t)slot * D.m_len * D.d;
    MEP_G float* mask = G<float>(D.mask) + (int64_t)slot * D.m_len;
    for (int t = threadIdx.x; t < D.m_len; t += BA_THREADS) mask[t] = (seq >= 0 && t < P0 + avail) ? 1.f : 0.f;
    if (D.src_f64) {
        copy_frames<double>(D, off, start, avail, P0, out);
        if (P0) summary_rows<double>(D, off, L, out, lds);
    } else {
        copy_frames<float>(D, off, start, avail, P0, out);
        if (P0) summary_rows<float>(D, off, L, out, lds);
    }
}

}  // namespace

extern "C" int mep_assemble_windows(const mep_window_desc* descs, int n_desc, mep_stream_t stream) {
    if (!descs || n_desc < 1 || n_desc > MEP_WINDOW_MAX_DESC) {
        mep_set_error("mep_assemble_windows: 1..MEP_WINDOW_MAX_DESC descriptors");
        return MEP_EINVAL;
    }
    WindowArgs a;
    int max_out = 0;
    for (int i = 0; i < n_desc; ++i) {
        const mep_window_desc& D = descs[i];
        const int min_len = D.summary ? 3 : 0;
        if (D.n_out < 0 || D.d < 1 || D.m_len < min_len || D.n_seq < 0 || (D.n_out > 0 && (!D.sel || !D.start || !D.out || !D.mask)) ||
            (D.n_seq > 0 && (!D.src || !D.segs)) || (D.summary && D.d > BA_MAX_COLS_PER_LANE * BA_THREADS) ||
            (D.src_f64 != 0 && D.src_f64 != 1)) {
            mep_set_error("mep_assemble_windows: invalid descriptor");
            return MEP_EINVAL;
        }
        a.d[i] = D;
        max_out = max(max_out, D.n_out);
    }
    for (int i = n_desc; i < MEP_WINDOW_MAX_DESC; ++i) a.d[i] = a.d[0];
    if (max_out == 0) return 0;
    hipLaunchKernelGGL(k_assemble, dim3(max_out, n_desc), dim3(BA_THREADS), 0, (hipStream_t)stream, a);
    return mep_check_launch("mep_assemble_windows");
}
