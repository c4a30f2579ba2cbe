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
            bool counts = true;
            if (d.row_mask) {
                // realformer.py:423-437: rows j of utterance batch i count while mask[i][j] == 1
                const int P = d.P;
                const int i = n / P, j = n - i * P;
                const MEP_G int64_t* m = G<const int64_t>(d.row_mask) + (int64_t)i * P;
                for (int jj = 0; jj <= j; ++jj) counts = counts && (m[jj] == 1);
            }
            const MEP_G int64_t* lab = G<const int64_t>(d.labels) + (int64_t)n * d.ld_label;
            for (int c = 0; c < C; ++c) {
                // pred_1 * w_1 + pred_2 * w_2 + ... in model order, then / post_div (correctly
                // rounded IEEE division, as torch's `/ 4` of run.py:476)
                float acc = mul_rn(G<const float>(d.preds[0])[(int64_t)n * d.ld_pred + c], d.weights[0]);
                for (int m = 1; m < d.n_models; ++m)
                    acc = add_rn(acc, mul_rn(G<const float>(d.preds[m])[(int64_t)n * d.ld_pred + c], d.weights[m]));
                const float s = __fdiv_rn(acc, d.post_div);
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
    const dim3 grid((d->N + SW_ROWS - 1) / SW_ROWS, (d->n_thr + SW_THR - 1) / SW_THR);
    hipLaunchKernelGGL(k_sweep, grid, dim3(SW_THREADS), 0, (hipStream_t)stream, *d);
    return mep_check_launch("mep_threshold_sweep");
}
