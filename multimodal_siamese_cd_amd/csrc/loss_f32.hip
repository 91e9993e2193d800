// Fused multi-term power-Jaccard loss of the dual-task and semi-supervised (MMCR) trainers
// (train_supervised_dualtask.py:73-85, train_semisupervised.py:78-113) on loss_functions.py:141-150.
//
// Every term is power_jaccard_loss(logits[sel], target[sel]) over a sample subset sel (all samples, the labelled
// ones or the unlabelled ones) with a coefficient; a term whose subset is empty is left out, as the reference's
// `if is_labeled.any()` / `if not is_labeled.all()` branches do, but decided on the device (no host sync, no
// boolean-mask gathers).  A soft target is sigmoid(target logits) and receives a gradient too (the MMCR
// consistency target is not detached).  Same per-element expressions as pjaccard_partial / pjaccard_bwd_kernel.
#include "common.h"

namespace scd {

constexpr int JT_MAX = 4;        // terms per call
constexpr int JT_BLOCKS = 256;   // partial-record blocks per term

struct JTerms {
    scd_jaccard_term_t t[JT_MAX];
    int n;
};

__device__ __forceinline__ float jt_sigmoid(float x) { return 1.f / (1.f + expf(-x)); }

__device__ __forceinline__ bool jt_selected(int select, const uint8_t *labeled, int s) {
    return select == 0 || ((labeled[s] != 0) == (select == 1));
}

// rec[term][block] = {sum p*t, sum p^2 + t^2} over this block's selected elements
__global__ __launch_bounds__(256) void jaccard_multi_partial(JTerms terms, const uint8_t *__restrict__ labeled,
                                                             int n_samples, int64_t pixels, float *__restrict__ rec) {
    const scd_jaccard_term_t T = terms.t[blockIdx.y];
    const int64_t n = int64_t(n_samples) * pixels;
    __shared__ float s1[256], s2[256];
    float a = 0.f, b = 0.f;
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
        if (!jt_selected(T.select, labeled, int(i / pixels))) continue;
        const float p = jt_sigmoid(T.logits[i]);
        const float tt = T.soft_target ? jt_sigmoid(T.target[i]) : T.target[i];
        a = fmaf(p, tt, a);
        b += p * p + tt * tt;
    }
    s1[threadIdx.x] = a;
    s2[threadIdx.x] = b;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (threadIdx.x < off) {
            s1[threadIdx.x] += s1[threadIdx.x + off];
            s2[threadIdx.x] += s2[threadIdx.x + off];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        float *r = rec + (size_t(blockIdx.y) * gridDim.x + blockIdx.x) * 2;
        r[0] = s1[0];
        r[1] = s2[0];
    }
}

// sums[term] = {I, sum(p^2 + t^2), D, selected samples}; loss = sum_t coef_t * [selected_t > 0] * (1 - I_t / D_t)
__global__ __launch_bounds__(256) void jaccard_multi_finalize(JTerms terms, const uint8_t *__restrict__ labeled,
                                                              int n_samples, const float *__restrict__ rec, int nrec,
                                                              float *sums, float *loss) {
    __shared__ double sI[256], sA[256];
    __shared__ int cnt[JT_MAX];
    const int t = threadIdx.x;
    float total = 0.f;
    for (int k = 0; k < terms.n; ++k) {
        double I = 0, A = 0;
        for (int j = t; j < nrec; j += 256) {
            I += rec[(size_t(k) * nrec + j) * 2];
            A += rec[(size_t(k) * nrec + j) * 2 + 1];
        }
        sI[t] = I;
        sA[t] = A;
        if (t == 0) {
            int c = 0;
            for (int s = 0; s < n_samples; ++s) c += jt_selected(terms.t[k].select, labeled, s);
            cnt[k] = c;
        }
        __syncthreads();
        for (int off = 128; off > 0; off >>= 1) {
            if (t < off) {
                sI[t] += sI[t + off];
                sA[t] += sA[t + off];
            }
            __syncthreads();
        }
        if (t == 0) {
            const float If = float(sI[0]);
            const float Df = float(sA[0]) - If + 1e-6f;
            sums[k * 4 + 0] = If;
            sums[k * 4 + 1] = float(sA[0]);
            sums[k * 4 + 2] = Df;
            sums[k * 4 + 3] = float(cnt[k]);
            if (cnt[k] > 0) total += terms.t[k].coef * (1.f - If / Df);
        }
        __syncthreads();
    }
    if (t == 0) loss[0] = total;
}

__global__ void jaccard_multi_bwd_kernel(JTerms terms, const uint8_t *__restrict__ labeled, int n_samples,
                                         int64_t pixels, const float *__restrict__ sums,
                                         const float *__restrict__ gloss) {
    const int k = blockIdx.y;
    const scd_jaccard_term_t T = terms.t[k];
    const float I = sums[k * 4 + 0], D = sums[k * 4 + 2];
    const float g = (gloss ? gloss[0] : 1.f) * T.coef;
    const float invD2 = 1.f / (D * D);
    const int64_t n = int64_t(n_samples) * pixels;
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
        if (!jt_selected(T.select, labeled, int(i / pixels))) {
            if (T.glogits && (T.zero_unselected & 1)) T.glogits[i] = 0.f;
            if (T.gtarget && (T.zero_unselected & 2)) T.gtarget[i] = 0.f;
            continue;
        }
        const float p = jt_sigmoid(T.logits[i]);
        const float tt = T.soft_target ? jt_sigmoid(T.target[i]) : T.target[i];
        if (T.glogits) T.glogits[i] = g * (-(tt * D - I * (2.f * p - tt)) * invD2) * (p * (1.f - p));
        if (T.gtarget) T.gtarget[i] = g * (-(p * D - I * (2.f * tt - p)) * invD2) * (tt * (1.f - tt));
    }
}

// The exact-DataParallel loss (utils/networks.py:27 with train_supervised.py:75: ONE loss over the gathered batch):
// each rank's per-term records {I, S = sum(p^2 + t^2), D, count} (stride 4; the single-term form: {I, S, D}, stride
// 3) are summed over the ranks, then D = S - I + 1e-6 and the loss are re-formed from the global sums exactly as
// the finalize kernels form them from one device's partial sums.
__global__ void jaccard_loss_from_sums(JTerms terms, int stride, float *sums, float *loss) {
    if (threadIdx.x != 0) return;
    float total = 0.f;
    for (int k = 0; k < terms.n; ++k) {
        float *r = sums + k * stride;
        const float If = r[0];
        const float Df = r[1] - If + 1e-6f;
        r[2] = Df;
        if (stride < 4 || r[3] > 0.f) total += terms.t[k].coef * (1.f - If / Df);
    }
    loss[0] = total;
}

static int jt_load(const scd_jaccard_term_t *terms, int n_terms, JTerms &jt, const char *what) {
    if (!terms || n_terms < 1 || n_terms > JT_MAX) {
        set_error("%s: 1..%d terms", what, JT_MAX);
        return SCD_ERR_ARG;
    }
    jt.n = n_terms;
    for (int k = 0; k < n_terms; ++k) {
        const scd_jaccard_term_t &T = terms[k];
        if (!T.logits || !T.target || T.select < 0 || T.select > 2 || (T.gtarget && !T.soft_target)) {
            set_error("%s: term %d: bad arguments (gtarget only for a soft target)", what, k);
            return SCD_ERR_ARG;
        }
        jt.t[k] = T;
    }
    return SCD_OK;
}

}  // namespace scd

using namespace scd;

extern "C" size_t scd_jaccard_multi_workspace_bytes(int32_t n_terms) {
    return size_t(n_terms < 1 ? 1 : n_terms) * JT_BLOCKS * 2 * sizeof(float);
}

extern "C" int scd_jaccard_multi_fwd(const scd_jaccard_term_t *terms, int32_t n_terms, const uint8_t *labeled,
                                     int32_t n_samples, int64_t pixels, float *sums, float *loss, void *ws,
                                     size_t ws_bytes, scd_stream_t stream) {
    clear_error();
    JTerms jt;
    SCD_TRY(jt_load(terms, n_terms, jt, "jaccard_multi_fwd"));
    if (!labeled || n_samples < 1 || pixels < 1 || !sums || !loss) {
        set_error("jaccard_multi_fwd: bad arguments");
        return SCD_ERR_ARG;
    }
    if (!ws || ws_bytes < scd_jaccard_multi_workspace_bytes(n_terms)) {
        set_error("jaccard_multi_fwd: workspace too small");
        return SCD_ERR_WORKSPACE;
    }
    hipStream_t s = as_stream(stream);
    float *rec = static_cast<float *>(ws);
    hipLaunchKernelGGL(jaccard_multi_partial, dim3(JT_BLOCKS, n_terms), dim3(256), 0, s, jt, labeled, n_samples, pixels,
                       rec);
    hipLaunchKernelGGL(jaccard_multi_finalize, dim3(1), dim3(256), 0, s, jt, labeled, n_samples, rec, JT_BLOCKS, sums,
                       loss);
    return launch_status("scd_jaccard_multi_fwd");
}

extern "C" int scd_jaccard_multi_bwd(const scd_jaccard_term_t *terms, int32_t n_terms, const uint8_t *labeled,
                                     int32_t n_samples, int64_t pixels, const float *sums, const float *gloss,
                                     scd_stream_t stream) {
    clear_error();
    JTerms jt;
    SCD_TRY(jt_load(terms, n_terms, jt, "jaccard_multi_bwd"));
    if (!labeled || n_samples < 1 || pixels < 1 || !sums) {
        set_error("jaccard_multi_bwd: bad arguments");
        return SCD_ERR_ARG;
    }
    const int64_t n = int64_t(n_samples) * pixels;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(jaccard_multi_bwd_kernel, dim3(unsigned(blocks), n_terms), dim3(256), 0, as_stream(stream), jt,
                       labeled, n_samples, pixels, sums, gloss);
    return launch_status("scd_jaccard_multi_bwd");
}

extern "C" int scd_jaccard_multi_loss_from_sums(const scd_jaccard_term_t *terms, int32_t n_terms, float *sums,
                                                float *loss, scd_stream_t stream) {
    clear_error();
    JTerms jt;
    SCD_TRY(jt_load(terms, n_terms, jt, "jaccard_multi_loss_from_sums"));
    if (!sums || !loss) {
        set_error("jaccard_multi_loss_from_sums: bad arguments");
        return SCD_ERR_ARG;
    }
    hipLaunchKernelGGL(jaccard_loss_from_sums, dim3(1), dim3(64), 0, as_stream(stream), jt, 4, sums, loss);
    return launch_status("scd_jaccard_multi_loss_from_sums");
}

extern "C" int scd_pjaccard_loss_from_sums(float *sums, float *loss, scd_stream_t stream) {
    clear_error();
    if (!sums || !loss) {
        set_error("pjaccard_loss_from_sums: bad arguments");
        return SCD_ERR_ARG;
    }
    JTerms jt;
    jt.n = 1;
    jt.t[0] = scd_jaccard_term_t{};
    jt.t[0].coef = 1.f;
    hipLaunchKernelGGL(jaccard_loss_from_sums, dim3(1), dim3(64), 0, as_stream(stream), jt, 3, sums, loss);
    return launch_status("scd_pjaccard_loss_from_sums");
}
