// On-device training augmentations of the reference's data pipeline (utils/augmentations.py:6-142), batched:
//   - window_label_sums: the change-label sum of every candidate crop of ImportanceRandomCrop (augmentations.py:
//     129-142: 20 uniform candidates, weight = label sum + 5);
//   - augment_apply: crop (augmentations.py:110-122) -> RandomFlip (48-65: horizontal = axis 1, then vertical =
//     axis 0) -> RandomRotate (68-74: np.rot90(k, axes=(0, 1))) -> ColorShift (77-89: x * f, clip [0, 1], in
//     double as numpy promotes float32 * float64) -> GammaCorrection (92-105: x ** g, clip [0, 1], double) ->
//     Numpy2Torch (HWC -> CHW), for one channel group of a batch of tiles of any sizes.
// The random parameters are drawn by the host (the reference draws them with np.random per item).
#include "common.h"

namespace scd {

// sums[b][k] = sum of label[b][y : y + S, x : x + S] (channel 0 of an HW1 tile), one block per (b, k).
__global__ __launch_bounds__(256) void window_label_sums_kernel(const float *const *__restrict__ labels,
                                                                const int *__restrict__ hw, const int *__restrict__ yx,
                                                                int ncand, int S, float *__restrict__ sums) {
    const int b = blockIdx.y, k = blockIdx.x;
    const float *lab = labels[b];
    const int W = hw[2 * b + 1];
    const int y0 = yx[(b * ncand + k) * 2], x0 = yx[(b * ncand + k) * 2 + 1];
    float acc = 0.f;
    for (int e = threadIdx.x; e < S * S; e += blockDim.x) {
        const int i = e / S, j = e - (e / S) * S;
        acc += lab[int64_t(y0 + i) * W + (x0 + j)];
    }
    __shared__ float red[256];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) sums[b * ncand + k] = red[0];  // 0/1 labels: exact integers below 2^24
}

// out[b][c][i][j] for an S x S crop of tile b (H_b x W_b x C, HWC); params[b] = {y0, x0, flip_h, flip_v, rot_k}.
__global__ void augment_apply_kernel(const float *const *__restrict__ src, const int *__restrict__ hw, int C, int S,
                                     const int *__restrict__ params, const double *__restrict__ scale,
                                     const double *__restrict__ gamma, float *__restrict__ out, int64_t total) {
    for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < total; e += int64_t(gridDim.x) * blockDim.x) {
        const int j = int(e % S);
        const int i = int((e / S) % S);
        const int c = int((e / (int64_t(S) * S)) % C);
        const int b = int(e / (int64_t(S) * S * C));
        const int *p = params + 5 * b;
        // invert rot90^k: rot90(m)[i][j] = m[j][S-1-i]
        int y = i, x = j;
        for (int r = 0; r < p[4]; ++r) {
            const int ny = x, nx = S - 1 - y;
            y = ny;
            x = nx;
        }
        if (p[3]) y = S - 1 - y;  // vertical flip (axis 0), applied after the horizontal one
        if (p[2]) x = S - 1 - x;  // horizontal flip (axis 1)
        const int W = hw[2 * b + 1];
        float v = src[b][(int64_t(p[0] + y) * W + (p[1] + x)) * C + c];
        if (scale) v = float(fmin(fmax(double(v) * scale[b * C + c], 0.0), 1.0));
        if (gamma) v = float(fmin(fmax(pow(double(v), gamma[b * C + c]), 0.0), 1.0));
        out[e] = v;
    }
}

}  // namespace scd

using namespace scd;

extern "C" int scd_window_label_sums(const float *const *labels, const int32_t *hw, const int32_t *yx, int32_t batch,
                                     int32_t ncand, int32_t crop, float *sums, scd_stream_t stream) {
    clear_error();
    if (!labels || !hw || !yx || !sums || batch < 1 || ncand < 1 || crop < 1 || batch > 65535) {
        set_error("window_label_sums: bad arguments");
        return SCD_ERR_ARG;
    }
    hipLaunchKernelGGL(window_label_sums_kernel, dim3(ncand, batch), dim3(256), 0, as_stream(stream), labels, hw, yx,
                       ncand, crop, sums);
    return launch_status("scd_window_label_sums");
}

extern "C" int scd_augment_apply(const float *const *src, const int32_t *hw, int32_t batch, int32_t channels,
                                 int32_t crop, const int32_t *params, const double *scale, const double *gamma,
                                 float *out, scd_stream_t stream) {
    clear_error();
    if (!src || !hw || !params || !out || batch < 1 || channels < 1 || crop < 1) {
        set_error("augment_apply: bad arguments");
        return SCD_ERR_ARG;
    }
    const int64_t total = int64_t(batch) * channels * crop * crop;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(augment_apply_kernel, dim3(unsigned(blocks)), dim3(256), 0, as_stream(stream), src, hw,
                       channels, crop, params, scale, gamma, out, total);
    return launch_status("scd_augment_apply");
}
