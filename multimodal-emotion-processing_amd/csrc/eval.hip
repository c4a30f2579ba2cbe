// Evaluation: ensemble combine + threshold sweep (include/mep.h, mep_threshold_sweep).
//
// Reference: test() of others/realformer.py:395-477 runs the full test set through both models
// once per threshold (400 thresholds t/200 - 1) and thresholds pred_1 * 0.6 + pred_2 * 0.4;
// cmu-mosei/run.py:456-498 averages 4 models and applies fixed per-class thresholds.  Here the
// logits are produced once (one forward per model) and every (threshold, class) confusion count
// is formed on the GPU; the F1 / accuracy arithmetic on the counts is host code
// (mep_amd/evaluate.py), as sklearn's is in the reference.
//
// Mapping: a workgroup stages 256 rows (combined scores + a label/row-valid code per element)
// in LDS once, then each thread owns (threshold, class) pairs of the workgroup's 64-threshold
// slice and walks the 256 rows: every lane of a wave reads the same row at the same time, so the
// LDS reads are broadcasts.  Counts are exact integers added with global atomics (order free).
// Bound: VALU compares (N * C * n_thr of them); the HBM traffic is one read of the model scores.
#include "common.h"

using namespace mep;

namespace {

// realformer.py:423-437: rows j of utterance batch i count while mask[i][j] == 1
MEP_DEV bool row_counts(const mep_sweep_desc& d, int n) {
    if (!d.row_mask) return true;
    const int P = d.P;
    const int i = n / P, j = n - i * P;
    const MEP_G int64_t* m = G<const int64_t>(d.row_mask) + (int64_t)i * P;
    bool ok = true;
    for (int jj = 0; jj <= j; ++jj) ok = ok && (m[jj] == 1);
    return ok;
}

// pred_1 * w_1 + pred_2 * w_2 + ... in model order, then / post_div (correctly rounded IEEE
// division, as torch's `/ 4` of run.py:476)
MEP_DEV float row_score(const mep_sweep_desc& d, int n, int c) {
    float acc = mul_rn(G<const float>(d.preds[0])[(int64_t)n * d.ld_pred + c], d.weights[0]);
    for (int m = 1; m < d.n_models; ++m)
        acc = add_rn(acc, mul_rn(G<const float>(d.preds[m])[(int64_t)n * d.ld_pred + c], d.weights[m]));
    return __fdiv_rn(acc, d.post_div);
}

constexpr int SW_ROWS = 256;     // rows per workgroup (one per thread when staging)
constexpr int SW_THREADS = 256;
constexpr int SW_THR = 64;       // thresholds per workgroup

__global__ __launch_bounds__(SW_THREADS) void k_sweep(mep_sweep_desc d) {
    __shared__ float S[SW_ROWS * MEP_EVAL_MAX_CLASSES];
    __shared__ unsigned char L[SW_ROWS * MEP_EVAL_MAX_CLASSES];   // 0 negative, 1 positive, 2 skip
    const int C = d.C;
    const int r0 = blockIdx.x * SW_ROWS;
    const int nr = min(SW_ROWS, d.N - r0);
    {
        const int r = threadIdx.x;
        const int n = r0 + r;
        if (r < nr) {
            const bool counts = row_counts(d, n);
            const MEP_G int64_t* lab = G<const int64_t>(d.labels) + (int64_t)n * d.ld_label;
            for (int c = 0; c < C; ++c) {
                const float s = row_score(d, n, c);
                if (d.scores && blockIdx.y == 0) G<float>(d.scores)[(int64_t)n * C + c] = s;
                S[r * C + c] = s;
                L[r * C + c] = counts ? (lab[c] != 0 ? 1 : 0) : 2;
            }
        }
    }
    __syncthreads();
    const int t_lo = blockIdx.y * SW_THR;
    const int n_pair = min(SW_THR, d.n_thr - t_lo) * C;
    for (int p = threadIdx.x; p < n_pair; p += SW_THREADS) {
        const int t = t_lo + p / C, c = p - (p / C) * C;
        const float thr = G<const float>(d.thresholds)[d.thr_per_class ? t * C + c : t];
        int tp = 0, fp = 0, fn = 0, tn = 0;
        for (int r = 0; r < nr; ++r) {
            const int l = L[r * C + c];
            const bool pos = S[r * C + c] > thr;   // NaN scores predict 0, as torch.where(pred > t)
            tp += (l == 1) & pos;
            fp += (l == 0) & pos;
            fn += (l == 1) & !pos;
            tn += (l == 0) & !pos;
        }
        MEP_G int* out = G<int>(d.counts) + ((int64_t)t * C + c) * 4;
        if (tp) atomicAdd((int*)(uintptr_t)(out + 0), tp);
        if (fp) atomicAdd((int*)(uintptr_t)(out + 1), fp);
        if (fn) atomicAdd((int*)(uintptr_t)(out + 2), fn);
        if (tn) atomicAdd((int*)(uintptr_t)(out + 3), tn);
    }
}

// ---- sorted thresholds: one binary search per (row, class) instead of n_thr compares.
// With thr(0, c) <= thr(1, c) <= ..., `s > thr(t, c)` holds exactly for t < k, k = #{t : thr(t, c) < s}
// (NaN: k = 0, never positive).  Pass 1 counts every (class, label, k) in an LDS histogram per
// workgroup and flushes it to the workspace; pass 2 turns each class's histograms into suffix
// sums gt[t] = #{rows : k > t}: tp = gt_pos, fn = n_pos - gt_pos, fp = gt_neg, tn = n_neg - gt_neg,
// adds them to counts and re-zeroes the workspace.  Integer counts: identical to the direct pass.
constexpr int SH_ROWS = SW_THREADS;   // rows per workgroup, one per lane
constexpr int SH_LDS_BYTES = 65536;

__global__ __launch_bounds__(SW_THREADS) void k_sweep_hist(mep_sweep_desc d) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int C = d.C, nt = d.n_thr, nb = nt + 1;
    float* T = reinterpret_cast<float*>(smem);                 // [C][n_thr]
    int* H = reinterpret_cast<int*>(smem + (size_t)C * nt * 4); // [C][2][n_thr + 1]
    for (int i = threadIdx.x; i < C * nt; i += SW_THREADS) {
        const int c = i / nt, t = i - c * nt;
        T[i] = G<const float>(d.thresholds)[d.thr_per_class ? t * C + c : t];
    }
    for (int i = threadIdx.x; i < 2 * C * nb; i += SW_THREADS) H[i] = 0;
    __syncthreads();
    // one row per lane: its C scores are independent loads in flight together
    const int r = threadIdx.x;
    const int n = blockIdx.x * SH_ROWS + r;
    if (n < d.N) {
        const bool ok = row_counts(d, n);
        const MEP_G int64_t* lab = G<const int64_t>(d.labels) + (int64_t)n * d.ld_label;
        for (int c = 0; c < C; ++c) {
            const float s = row_score(d, n, c);
            if (d.scores) G<float>(d.scores)[(int64_t)n * C + c] = s;   // every row, as the direct pass
            if (!ok) continue;
            const int pos = lab[c] != 0;
            const float* tc = T + c * nt;
            int lo = 0, hi = nt;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (tc[mid] < s) lo = mid + 1; else hi = mid;
            }
            atomicAdd(&H[(c * 2 + pos) * nb + lo], 1);
        }
    }
    __syncthreads();
    MEP_G int* W = G<int>(d.hist);
    for (int i = threadIdx.x; i < 2 * C * nb; i += SW_THREADS)
        if (H[i]) atomicAdd((int*)(uintptr_t)(W + i), H[i]);
}

__global__ __launch_bounds__(SW_THREADS) void k_sweep_hist_counts(mep_sweep_desc d) {
    __shared__ int part[2][SW_THREADS];
    const int C = d.C, nt = d.n_thr, nb = nt + 1;
    const int c = blockIdx.x;
    MEP_G int* W = G<int>(d.hist) + (int64_t)c * 2 * nb;
    // each lane owns bins [b0, b1) of both histograms
    const int per = (nb + SW_THREADS - 1) / SW_THREADS;
    const int b0 = min(nb, threadIdx.x * per), b1 = min(nb, b0 + per);
    int own[2] = {0, 0};
    for (int k = b0; k < b1; ++k) { own[0] += W[k]; own[1] += W[nb + k]; }
    part[0][threadIdx.x] = own[0];
    part[1][threadIdx.x] = own[1];
    __syncthreads();
    // inclusive suffix scan of the lane totals (Hillis-Steele, fixed order: exact integers anyway)
    for (int off = 1; off < SW_THREADS; off <<= 1) {
        const int a0 = threadIdx.x + off < SW_THREADS ? part[0][threadIdx.x + off] : 0;
        const int a1 = threadIdx.x + off < SW_THREADS ? part[1][threadIdx.x + off] : 0;
        __syncthreads();
        part[0][threadIdx.x] += a0;
        part[1][threadIdx.x] += a1;
        __syncthreads();
    }
    const int n_neg = part[0][0], n_pos = part[1][0];
    // rows with k >= b1 (later lanes)
    int gt_neg = part[0][threadIdx.x] - own[0], gt_pos = part[1][threadIdx.x] - own[1];
    MEP_G int* out = G<int>(d.counts);
    for (int k = b1 - 1; k >= b0; --k) {
        // gt[t] for t = k: rows with bin > k
        if (k < nt) {
            MEP_G int* o = out + ((int64_t)k * C + c) * 4;
            o[0] += gt_pos;
            o[1] += gt_neg;
            o[2] += n_pos - gt_pos;
            o[3] += n_neg - gt_neg;
        }
        gt_neg += W[k];
        gt_pos += W[nb + k];
    }
    __syncthreads();
    for (int k = b0; k < b1; ++k) { W[k] = 0; W[nb + k] = 0; }   // the workspace is left zeroed
}

}  // namespace

extern "C" int mep_threshold_sweep(const mep_sweep_desc* d, mep_stream_t stream) {
    if (!d || d->n_models < 1 || d->n_models > MEP_EVAL_MAX_MODELS || d->C < 1 || d->C > MEP_EVAL_MAX_CLASSES ||
        d->N < 0 || d->n_thr < 0 || d->ld_pred < d->C || d->ld_label < d->C ||
        (d->N > 0 && d->n_thr > 0 && (!d->labels || !d->counts || !d->thresholds)) ||
        (d->row_mask && (d->P < 1 || d->N % d->P))) {
        mep_set_error("mep_threshold_sweep: invalid descriptor");
        return MEP_EINVAL;
    }
    if (d->N == 0 || d->n_thr == 0) return 0;   // empty inputs carry null data pointers
    for (int m = 0; m < d->n_models; ++m)
        if (!d->preds[m]) { mep_set_error("mep_threshold_sweep: null model scores"); return MEP_EINVAL; }
    if (d->sorted) {
        const size_t lds = (size_t)d->C * d->n_thr * 4 + (size_t)2 * d->C * (d->n_thr + 1) * 4;
        if (!d->hist || lds > SH_LDS_BYTES) {
            mep_set_error("mep_threshold_sweep: sorted mode needs the hist workspace and C * (3 n_thr + 2) * 4 <= 65536");
            return MEP_EINVAL;
        }
        hipLaunchKernelGGL(k_sweep_hist, dim3((d->N + SH_ROWS - 1) / SH_ROWS), dim3(SW_THREADS), lds,
                           (hipStream_t)stream, *d);
        int rc = mep_check_launch("mep_threshold_sweep (histogram)");
        if (rc) return rc;
        hipLaunchKernelGGL(k_sweep_hist_counts, dim3(d->C), dim3(SW_THREADS), 0, (hipStream_t)stream, *d);
        return mep_check_launch("mep_threshold_sweep (counts)");
    }
    const dim3 grid((d->N + SW_ROWS - 1) / SW_ROWS, (d->n_thr + SW_THR - 1) / SW_THR);
    hipLaunchKernelGGL(k_sweep, grid, dim3(SW_THREADS), 0, (hipStream_t)stream, *d);
    return mep_check_launch("mep_threshold_sweep");
}
