// Implicit-GEMM convolution kernels on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces aten::convolution / convolution_backward for the reference's Conv2d(3x3, pad 1),
// ConvTranspose2d(2x2, stride 2) (utils/networks.py:392,395,433).  Two kernel families:
//
//   igemm_f32  : out[m, o] = bias + sum_k A[m, k] * Wpk[o, k]  with A gathered on the fly from an NHWC
//                source (k = (tap, c)); used for conv forward, conv data-grad (flipped weights), ConvT
//                forward (1 tap + 2x2 pixel-shuffle store into the concat buffer slice) and ConvT
//                data-grad (4 taps, stride 2).
//   wgrad_f32  : slab[s][r][(tap, c)] = sum_{m in split s} P[m, r] * Q[src(m, tap), c]; split-K over the
//                pixel dimension into fp32 slabs, summed deterministically by wgrad_finalize.
//
// MFMA operand trick (fp32, 32x32x2): instruction s of an 8-deep K chunk takes k = 4h + s from lane
// half h = lane>>5, so every lane reads its 4 k-values for a row with ONE ds_read_b128 from a
// [row][k] LDS image (row stride BK+4 floats: conflict-free b128 reads).
#include <algorithm>

#include "conv_common.h"

namespace scd {

template <int WAVES_M, int WAVES_N, int TM, int TN, int BK>
__global__ __launch_bounds__(64 * WAVES_M *WAVES_N) void igemm_f32(IgemmArgs a) {
    constexpr int NT = 64 * WAVES_M * WAVES_N;
    constexpr int BM = WAVES_M * TM * 32;
    constexpr int BN = WAVES_N * TN * 32;
    constexpr int LS = BK + 4;  // LDS row stride (floats)
    constexpr int KC = BK / 4;  // 16-byte chunks per row
    constexpr int A_CH = BM * KC;
    constexpr int B_CH = BN * KC;
    constexpr int A_PER = (A_CH + NT - 1) / NT;
    constexpr int B_PER = (B_CH + NT - 1) / NT;
    constexpr int STAGE = (BM + BN) * LS;
    __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wm = wid % WAVES_M;
    const int wn = wid / WAVES_M;
    int mt, nt;
    if (a.remap) {  // logical tiles: N fastest, so the N-tiles of one pixel tile run together on one XCD
        const uint32_t L = xcd_swizzle(blockIdx.x, uint32_t(a.grid_m * a.grid_n));
        mt = int(L / uint32_t(a.grid_n));
        nt = int(L - uint32_t(mt) * uint32_t(a.grid_n));
    } else {
        mt = int(blockIdx.x % uint32_t(a.grid_m));
        nt = int(blockIdx.x / uint32_t(a.grid_m));
    }
    const int m0 = mt * BM;
    const int n0 = nt * BN;

    // Per-thread A-chunk bookkeeping (fixed across the K loop): the source pixel (img, oy*s, ox*s) as a
    // base pointer; a tap then only adds the wave-uniform offset (dy*ws + dx)*ldc + c0 after a bounds test.
    const float *a_base[A_PER];
    int a_sy[A_PER], a_sx[A_PER], a_off[A_PER];
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
        const int ch = tid + i * NT;
        const int row = ch / KC, col = ch % KC;
        const int m = m0 + row;
        const bool ok = (ch < A_CH) && (m < a.M);
        const uint32_t mm = ok ? uint32_t(m) : 0u;
        const uint32_t img = fdiv(mm, a.div_hw);
        const uint32_t r = mm - img * uint32_t(a.ho * a.wo);
        const uint32_t oy = fdiv(r, a.div_w);
        const uint32_t ox = r - oy * uint32_t(a.wo);
        // an out-of-range row gets a y coordinate that fails every bounds test
        a_sy[i] = ok ? int(oy) * a.stride : -(1 << 20);
        a_sx[i] = int(ox) * a.stride;
        a_base[i] = a.src + (size_t(int(img) * a.hs + a_sy[i] * ok) * a.ws + a_sx[i]) * a.ldc_s + col * 4;
        a_off[i] = row * LS + col * 4;
    }
    int b_row[B_PER], b_off[B_PER];
    bool b_ok[B_PER], b_in[B_PER];
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
        const int ch = tid + i * NT;
        const int row = ch / KC, col = ch % KC;
        b_in[i] = ch < B_CH;
        b_ok[i] = b_in[i] && (n0 + row < a.n_out);
        b_row[i] = (n0 + row) * a.K + col * 4;
        b_off[i] = BM * LS + row * LS + col * 4;
    }

    f32x4 ra[A_PER], rb[B_PER];
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};

    auto load_stage = [&](int t, int c0) {
        const int dyt = tap_at(a.tdy, t), dxt = tap_at(a.tdx, t);
        const long toff = long(dyt * a.ws + dxt) * a.ldc_s + c0;  // wave-uniform
#pragma unroll
        for (int i = 0; i < A_PER; ++i) {
            const bool v = unsigned(a_sy[i] + dyt) < unsigned(a.hs) && unsigned(a_sx[i] + dxt) < unsigned(a.ws);
            ra[i] = v ? gload4(a_base[i] + toff) : zero4;
        }
        const int k0 = t * a.c + c0;
#pragma unroll
        for (int i = 0; i < B_PER; ++i) {
            rb[i] = b_ok[i] ? gload4(a.w + size_t(b_row[i]) + k0) : zero4;
        }
    };
    auto store_stage = [&](int buf) {
        float *S = smem + buf * STAGE;
#pragma unroll
        for (int i = 0; i < A_PER; ++i)
            if (tid + i * NT < A_CH) lstore4(S + a_off[i], ra[i]);
#pragma unroll
        for (int i = 0; i < B_PER; ++i)
            if (b_in[i]) lstore4(S + b_off[i], rb[i]);
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int csteps = a.c / BK;
    const int nsteps = a.ntaps * csteps;
    const int a_lane = (wm * TM * 32 + (lane & 31)) * LS + 4 * (lane >> 5);
    const int b_lane = BM * LS + (wn * TN * 32 + (lane & 31)) * LS + 4 * (lane >> 5);

    int t = 0, cs = 0;
    load_stage(0, 0);
    store_stage(0);
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
        const bool more = s + 1 < nsteps;
        if (more) {
            if (++cs == csteps) {
                cs = 0;
                ++t;
            }
            load_stage(t, cs * BK);
        }
        const float *S = smem + (s & 1) * STAGE;
#pragma unroll
        for (int q = 0; q < BK / 8; ++q) {
            f32x4 av[TM], bv[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
                av[i] = lload4(S + a_lane + i * 32 * LS + 8 * q);
#pragma unroll
            for (int j = 0; j < TN; ++j)
                bv[j] = lload4(S + b_lane + j * 32 * LS + 8 * q);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][0], bv[j][0], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][1], bv[j][1], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][2], bv[j][2], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][3], bv[j][3], acc[i][j], 0, 0, 0);
                }
        }
        if (more) store_stage((s + 1) & 1);
        __syncthreads();
    }

    // Epilogue: C/D layout of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * TN * 32 + j * 32 + (lane & 31);
        if (n >= a.n_out) continue;
        if (a.store_mode == 0) {
            const float bias = a.bias ? a.bias[n] : 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    if (m < a.M) gstore1(a.dst + size_t(m) * a.ldc_d + n, acc[i][j][r] + bias);
                }
        } else {
            const int ij = n / a.cout, oc = n - ij * a.cout;
            const int di = ij >> 1, dj = ij & 1;
            const float bias = a.bias ? a.bias[oc] : 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    if (m < a.M) {
                        const uint32_t img = fdiv(uint32_t(m), a.div_hw);
                        const uint32_t rr = uint32_t(m) - img * uint32_t(a.ho * a.wo);
                        const uint32_t oy = fdiv(rr, a.div_w);
                        const uint32_t ox = rr - oy * uint32_t(a.wo);
                        const size_t pix = size_t(int(img) * a.dst_h + 2 * int(oy) + di) * a.dst_w + 2 * int(ox) + dj;
                        gstore1(a.dst + pix * a.ldc_d + oc, acc[i][j][r] + bias);
                    }
                }
        }
    }
}

// ------------------------------------------------------------------------------------------------
// wgrad
// ------------------------------------------------------------------------------------------------

template <int WAVES_M, int WAVES_N, int TM, int TN, int BK>
__global__ __launch_bounds__(64 * WAVES_M *WAVES_N) void wgrad_f32(WgradArgs a) {
    constexpr int NT = 64 * WAVES_M * WAVES_N;
    constexpr int BM = WAVES_M * TM * 32;
    constexpr int BN = WAVES_N * TN * 32;
    constexpr int AQ = BM / 4;  // 16-byte chunks per A row (one pixel)
    constexpr int BQ = BN / 4;
    constexpr int A_CH = BK * AQ;
    constexpr int B_CH = BK * BQ;
    constexpr int A_PER = (A_CH + NT - 1) / NT;
    constexpr int B_PER = (B_CH + NT - 1) / NT;
    constexpr int STAGE = BK * (BM + BN);
    __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wm = wid % WAVES_M;
    const int wn = wid / WAVES_M;
    // logical block -> (split, column tile, row tile), row tile fastest: the tiles of one pixel split share
    // their B pixels and run together on one XCD when remapped.
    const uint32_t per_split = uint32_t(a.grid_r * a.grid_j);
    const uint32_t L = a.remap ? xcd_swizzle(blockIdx.x, gridDim.x) : blockIdx.x;
    const int split = int(L / per_split);
    const int rem = int(L - uint32_t(split) * per_split);
    const int jt = rem / a.grid_r;
    const int r0 = (rem - jt * a.grid_r) * BM;
    const int j0 = jt * BN;
    const int kbeg = split * a.kchunk;
    const int kend = min(a.M, kbeg + a.kchunk);

    int a_k[A_PER], a_r[A_PER];
    bool a_in[A_PER], a_ok[A_PER];
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
        const int ch = tid + i * NT;
        a_in[i] = ch < A_CH;
        a_k[i] = ch / AQ;
        a_r[i] = r0 + (ch % AQ) * 4;
        a_ok[i] = a_in[i] && a_r[i] < a.R;
    }
    // B chunks: fixed column (tap, c) per thread; the pixel m = kb + b_k advances by BK per step, so its
    // (img, oy, ox) coordinates are stepped incrementally instead of divided out every step.
    int b_k[B_PER], b_dy[B_PER], b_dx[B_PER], b_c[B_PER];
    int b_img[B_PER], b_oy[B_PER], b_ox[B_PER];
    bool b_in[B_PER], b_ok[B_PER];
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
        const int ch = tid + i * NT;
        b_in[i] = ch < B_CH;
        b_k[i] = ch / BQ;
        const int j = j0 + (ch % BQ) * 4;
        b_ok[i] = b_in[i] && j < a.Ng;
        const int t = b_ok[i] ? int(fdiv(uint32_t(j), a.div_c)) : 0;
        b_c[i] = j - t * a.C;
        b_dy[i] = tap_at(a.tdy, t);
        b_dx[i] = tap_at(a.tdx, t);
        const uint32_t mm = uint32_t(min(kbeg + b_k[i], a.M - 1));
        const uint32_t img = fdiv(mm, a.div_hw);
        const uint32_t rr = mm - img * uint32_t(a.ho * a.wo);
        const uint32_t oy = fdiv(rr, a.div_w);
        b_img[i] = int(img);
        b_oy[i] = int(oy);
        b_ox[i] = int(rr - oy * uint32_t(a.wo));
    }

    f32x4 ra[A_PER], rb[B_PER];
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
    auto load_stage = [&](int kb) {
#pragma unroll
        for (int i = 0; i < A_PER; ++i) {
            const int m = kb + a_k[i];
            ra[i] = (a_ok[i] && m < kend) ? gload4(a.rows + size_t(m) * a.ldc_r + a_r[i]) : zero4;
        }
#pragma unroll
        for (int i = 0; i < B_PER; ++i) {
            const int sy = b_oy[i] * a.stride + b_dy[i];
            const int sx = b_ox[i] * a.stride + b_dx[i];
            const bool v = b_ok[i] && (kb + b_k[i] < kend) && unsigned(sy) < unsigned(a.hs) &&
                           unsigned(sx) < unsigned(a.ws);
            rb[i] = v ? gload4(a.src + (size_t(b_img[i] * a.hs + sy) * a.ws + sx) * a.ldc_s + b_c[i]) : zero4;
        }
    };
    auto advance = [&]() {  // pixel += BK for every B chunk
#pragma unroll
        for (int i = 0; i < B_PER; ++i) {
            int ox = b_ox[i] + BK, oy = b_oy[i], img = b_img[i];
            while (ox >= a.wo) {
                ox -= a.wo;
                if (++oy == a.ho) {
                    oy = 0;
                    ++img;
                }
            }
            b_ox[i] = ox;
            b_oy[i] = oy;
            b_img[i] = img;
        }
    };
    auto store_stage = [&](int buf) {
        float *S = smem + buf * STAGE;
#pragma unroll
        for (int i = 0; i < A_PER; ++i)
            if (a_in[i]) lstore4(S + (tid + i * NT) * 4, ra[i]);
#pragma unroll
        for (int i = 0; i < B_PER; ++i)
            if (b_in[i]) lstore4(S + BK * BM + (tid + i * NT) * 4, rb[i]);
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int h = lane >> 5;
    const int a_lane = h * BM + wm * TM * 32 + (lane & 31);
    const int b_lane = BK * BM + h * BN + wn * TN * 32 + (lane & 31);

    const int nsteps = (kend > kbeg) ? (kend - kbeg + BK - 1) / BK : 0;
    if (nsteps > 0) {
        load_stage(kbeg);
        store_stage(0);
        __syncthreads();
        for (int s = 0; s < nsteps; ++s) {
            const bool more = s + 1 < nsteps;
            if (more) {
                advance();
                load_stage(kbeg + (s + 1) * BK);
            }
            const float *S = smem + (s & 1) * STAGE;
            // Two groups of 4 k-pairs: group 0's fragments are read and waited for, group 1's reads are
            // issued (sched_barrier keeps them ahead) and land while group 0's MFMAs run.
            float av0[4][TM], bv0[4][TN], av1[4][TM], bv1[4][TN];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
#pragma unroll
                for (int i = 0; i < TM; ++i) av0[u][i] = S[a_lane + 2 * u * BM + i * 32];
#pragma unroll
                for (int j = 0; j < TN; ++j) bv0[u][j] = S[b_lane + 2 * u * BN + j * 32];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
#pragma unroll
                for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(av0[u][i]));
#pragma unroll
                for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(bv0[u][j]));
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
#pragma unroll
                for (int i = 0; i < TM; ++i) av1[u][i] = S[a_lane + 2 * (4 + u) * BM + i * 32];
#pragma unroll
                for (int j = 0; j < TN; ++j) bv1[u][j] = S[b_lane + 2 * (4 + u) * BN + j * 32];
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av0[u][i], bv0[u][j], acc[i][j], 0, 0, 0);
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av1[u][i], bv1[u][j], acc[i][j], 0, 0, 0);
            if (more) store_stage((s + 1) & 1);
            __syncthreads();
        }
    }

    float *slab = a.slabs + size_t(split) * a.R * a.Ng;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int col = j0 + wn * TN * 32 + j * 32 + (lane & 31);
        if (col >= a.Ng) continue;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = r0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                if (row < a.R) gstore1(slab + size_t(row) * a.Ng + col, acc[i][j][r]);
            }
    }
}

// Level 1 of the slab reduction: group g sums slabs [g*per, min((g+1)*per, nsplit)) in a fixed order and
// writes the result in place into slab g*per (only this thread reads that element of that slab).
__global__ void wgrad_group_sum(float *__restrict__ slabs, int nsplit, int per, size_t total) {
    const size_t e = blockIdx.x * size_t(blockDim.x) + threadIdx.x;
    if (e >= total) return;
    const int k0 = blockIdx.y * per;
    const int k1 = min(k0 + per, nsplit);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int k = k0;
    for (; k + 3 < k1; k += 4) {
        s0 += slabs[e + size_t(k) * total];
        s1 += slabs[e + size_t(k + 1) * total];
        s2 += slabs[e + size_t(k + 2) * total];
        s3 += slabs[e + size_t(k + 3) * total];
    }
    for (; k < k1; ++k) s0 += slabs[e + size_t(k) * total];
    slabs[e + size_t(k0) * total] = (s0 + s1) + (s2 + s3);
}

// wgrad_group_sum on 16-byte pieces (total % 4 == 0, 16-byte aligned slabs): per element the same sums in the same
// order (bit-identical), four slabs' 16-byte loads in flight per thread instead of 4-byte ones.
__global__ void wgrad_group_sum4(float *__restrict__ slabs, int nsplit, int per, size_t total) {
    const size_t e = (blockIdx.x * size_t(blockDim.x) + threadIdx.x) * 4;
    if (e >= total) return;
    const int k0 = blockIdx.y * per;
    const int k1 = min(k0 + per, nsplit);
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, s2 = s0, s3 = s0;
    int k = k0;
    for (; k + 3 < k1; k += 4) {
        s0 += gload4(slabs + e + size_t(k) * total);
        s1 += gload4(slabs + e + size_t(k + 1) * total);
        s2 += gload4(slabs + e + size_t(k + 2) * total);
        s3 += gload4(slabs + e + size_t(k + 3) * total);
    }
    for (; k < k1; ++k) s0 += gload4(slabs + e + size_t(k) * total);
    *reinterpret_cast<f32x4 *>(slabs + e + size_t(k0) * total) = (s0 + s1) + (s2 + s3);
}

// Level 2, one workgroup per (row r, block of kFinCB channels): sum the (group) slabs of the block's 9 column runs
// [t][c0, c0 + kFinCB) into LDS (coalesced reads; the slab loads of one element issued together, summed in slab
// order), then write the parameter-order run [c0, c0 + kFinCB)[t] (coalesced writes; LDS rows padded by one float
// so the transposed reads do not conflict).
constexpr int kFinCB = 64, kFinMaxTaps = 9;
__global__ __launch_bounds__(256) void wgrad_finalize_rows(const float *__restrict__ slabs, int nsum, int gstride,
                                                           int R, int ntaps, int C, int mode, int c_valid,
                                                           float *__restrict__ out) {
    __shared__ float tile[kFinMaxTaps * (kFinCB + 1)];
    const int r = blockIdx.x, c0 = blockIdx.y * kFinCB;
    const int cb = min(kFinCB, C - c0);
    const int Ng = ntaps * C;
    const size_t total = size_t(R) * Ng, kstride = size_t(gstride) * total;
    const float *row = slabs + size_t(r) * Ng + c0;
    for (int e = threadIdx.x; e < ntaps * cb; e += blockDim.x) {
        const int t = e / cb, c = e - t * cb;
        const float *p = row + t * C + c;
        float s = 0.f;
        int k = 0;
        for (; k + 4 <= nsum; k += 4) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = p[size_t(k + u) * kstride];
#pragma unroll
            for (int u = 0; u < 4; ++u) s += v[u];
        }
        for (; k < nsum; ++k) s += p[size_t(k) * kstride];
        tile[t * (kFinCB + 1) + c] = s;
    }
    __syncthreads();
    // mode 0: OIHW [R][c_valid][taps]; mode 1: ConvT [R][C][taps]
    const int cw = mode == 0 ? c_valid : C, cv = max(0, min(cb, cw - c0));
    float *o = out + (size_t(r) * cw + c0) * ntaps;
    for (int j = threadIdx.x; j < cv * ntaps; j += blockDim.x) {
        const int c = j / ntaps, t = j - c * ntaps;
        o[j] = tile[t * (kFinCB + 1) + c];
    }
}

// Level 2 (more than kFinMaxTaps taps): sum the (group) slabs at stride `gstride` slabs and scatter into the
// parameter layout.
__global__ void wgrad_finalize_kernel(const float *__restrict__ slabs, int nsum, int gstride, int R, int ntaps,
                                      int C, int mode, int c_valid, float *__restrict__ out) {
    const int Ng = ntaps * C;
    const size_t total = size_t(R) * Ng;
    for (size_t e = blockIdx.x * size_t(blockDim.x) + threadIdx.x; e < total; e += size_t(gridDim.x) * blockDim.x) {
        const int r = int(e / Ng);
        const int col = int(e - size_t(r) * Ng);
        const int t = col / C;
        const int c = col - t * C;
        if (c >= c_valid) continue;
        float s = 0.f;
        for (int k = 0; k < nsum; ++k) s += slabs[e + size_t(k) * gstride * total];
        size_t o;
        if (mode == 0)
            o = (size_t(r) * c_valid + c) * ntaps + t;  // OIHW [R][c_valid][3][3], t = ky*3+kx
        else
            o = (size_t(r) * C + c) * ntaps + t;        // ConvT [R][C][2][2], t = i*2+j
        out[o] = s;
    }
}

// ------------------------------------------------------------------------------------------------
// Host launchers
// ------------------------------------------------------------------------------------------------
template <int WM, int WN, int TM, int TN, int BK>
static void launch_igemm(const IgemmArgs &a, hipStream_t s) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    IgemmArgs b = a;
    b.grid_m = (a.M + BM - 1) / BM;
    b.grid_n = (a.n_out + BN - 1) / BN;
    b.remap = xcd_remap_enabled(a.tune);
    hipLaunchKernelGGL((igemm_f32<WM, WN, TM, TN, BK>), dim3(b.grid_m * b.grid_n), dim3(64 * WM * WN), 0, s, b);
}

template <int WM, int WN, int TM, int TN>
static void launch_igemm_bk(const IgemmArgs &a, hipStream_t s) {
    if (a.c % 16 == 0)
        launch_igemm<WM, WN, TM, TN, 16>(a, s);
    else
        launch_igemm<WM, WN, TM, TN, 8>(a, s);
}

static int check_taps(int ntaps, const int8_t *dy, const int8_t *dx) {
    if (ntaps < 1 || ntaps > 9) {
        set_error("ntaps=%d out of range [1,9]", ntaps);
        return SCD_ERR_ARG;
    }
    for (int i = 0; i < ntaps; ++i)
        if (dy[i] < -8 || dy[i] > 7 || dx[i] < -8 || dx[i] > 7) {
            set_error("tap %d offset (%d,%d) out of range", i, dy[i], dx[i]);
            return SCD_ERR_ARG;
        }
    return SCD_OK;
}

}  // namespace scd

using namespace scd;

extern "C" int scd_abi_version(void) { return SCD_ABI_VERSION; }

namespace scd {
// Validate a descriptor and fill the kernel arguments.
static int igemm_prepare(const scd_igemm_t *d, IgemmArgs &a) {
    if (!d) {
        set_error("scd_conv_igemm: null descriptor");
        return SCD_ERR_ARG;
    }
    if (!math_valid(d->math)) {
        set_error("igemm: math %d is not an scd_conv_math value", d->math);
        return SCD_ERR_ARG;
    }
    SCD_TRY(check_view(d->src, "igemm.src"));
    SCD_TRY(check_view(d->dst, "igemm.dst"));
    SCD_TRY(check_taps(d->ntaps, d->dy, d->dx));
    const int dt = common_dtype("igemm", {&d->src, &d->dst, d->bn_bwd ? &d->bn_bwd->y : nullptr});
    if (dt < 0) return SCD_ERR_ARG;
    if (dt == SCD_DT_BF16 && d->math != SCD_MATH_BF16) {
        set_error("igemm: bf16 views need math SCD_MATH_BF16 (got %d)", d->math);
        return SCD_ERR_ARG;
    }
    a.sb = dt == SCD_DT_BF16 ? 1 : 0;
    const int eb = elem_size(a.sb);
    if (d->src.c % 8) {
        set_error("igemm: src.c=%d must be a multiple of 8 (pad channels)", d->src.c);
        return SCD_ERR_ARG;
    }
    if (!d->wpk || !aligned16(d->wpk) || d->n_out <= 0 || d->out_h <= 0 || d->out_w <= 0 || d->stride < 1) {
        set_error("igemm: bad weights/n_out/out grid/stride");
        return SCD_ERR_ARG;
    }
    const int64_t M = int64_t(d->src.n) * d->out_h * d->out_w;
    if (M >= (int64_t(1) << 31) || pixels(d->src) >= (int64_t(1) << 31)) {
        set_error("igemm: problem too large for 32-bit pixel indexing");
        return SCD_ERR_ARG;
    }
    if (d->dst.n != d->src.n) {
        set_error("igemm: dst.n=%d != src.n=%d", d->dst.n, d->src.n);
        return SCD_ERR_ARG;
    }
    if (d->store_mode == 0) {
        if (d->dst.h != d->out_h || d->dst.w != d->out_w || d->dst.c != d->n_out) {
            set_error("igemm: dst view (%d,%d,%d) != out grid (%d,%d,%d)", d->dst.h, d->dst.w, d->dst.c, d->out_h,
                      d->out_w, d->n_out);
            return SCD_ERR_ARG;
        }
    } else if (d->store_mode == 1) {
        if (d->n_out % 4 || d->dst.c != d->n_out / 4 || d->dst.h != 2 * d->out_h || d->dst.w != 2 * d->out_w) {
            set_error("igemm: shuffle store needs dst (2h,2w,n_out/4)");
            return SCD_ERR_ARG;
        }
    } else {
        set_error("igemm: store_mode %d", d->store_mode);
        return SCD_ERR_ARG;
    }
    a.src = static_cast<const float *>(d->src.data);
    a.n_img = d->src.n;
    a.hs = d->src.h;
    a.ws = d->src.w;
    a.c = d->src.c;
    a.ldc_s = d->src.ldc;
    a.ho = d->out_h;
    a.wo = d->out_w;
    a.stride = d->stride;
    a.ntaps = d->ntaps;
    a.tdy = pack_taps(d->dy, d->ntaps);
    a.tdx = pack_taps(d->dx, d->ntaps);
    a.w = d->wpk;
    a.n_out = d->n_out;
    a.K = d->ntaps * d->src.c;
    a.bias = d->bias;
    a.dst = static_cast<float *>(d->dst.data);
    a.ldc_d = d->dst.ldc;
    a.dst_h = d->dst.h;
    a.dst_w = d->dst.w;
    a.store_mode = d->store_mode;
    a.cout = d->store_mode == 1 ? d->n_out / 4 : d->n_out;
    a.M = int(M);
    a.div_hw = make_fastdiv(uint32_t(d->out_h * d->out_w));
    a.div_w = make_fastdiv(uint32_t(d->out_w));
    a.wsplit = d->wsplit;
    a.wplane = int64_t((a.n_out + 31) / 32) * 32 * a.K;  // fragment-major pre-split plane (rows padded to 32)
    a.stat_rec = d->stat_rec;
    a.in_scale = d->in_scale;
    a.in_shift = d->in_shift;
    a.in_seg_imgs = d->src.n;
    if (d->in_scale || d->in_shift) {
        if (!d->in_scale || !d->in_shift || d->in_nseg < 1 || d->src.n % d->in_nseg || !aligned16(d->in_scale) ||
            !aligned16(d->in_shift)) {
            set_error("igemm: input transform needs both 16-byte aligned coefficient arrays and in_nseg | src.n "
                      "(in_nseg=%d, n=%d)", d->in_nseg, d->src.n);
            return SCD_ERR_ARG;
        }
        a.in_seg_imgs = d->src.n / d->in_nseg;
    }
    a.bb_y = nullptr;
    a.bb_rec = nullptr;
    if (const scd_bn_bwd_tiles_t *b = d->bn_bwd) {
        if (!b->y.data || !b->rec || !b->save_mean || !b->save_invstd || !b->scale || !b->shift || b->nseg < 1 ||
            b->y.n != d->dst.n || b->y.h != d->dst.h || b->y.w != d->dst.w || b->y.c != d->n_out ||
            d->dst.n % b->nseg || b->y.ldc % 4 || (reinterpret_cast<uintptr_t>(b->y.data) & (a.sb ? 7 : 15)) ||
            !aligned16(b->save_mean) || !aligned16(b->save_invstd) || !aligned16(b->scale) || !aligned16(b->shift)) {
            set_error("igemm: bn_bwd needs y shaped like dst (c = n_out, aligned, ldc %% 4 == 0), all "
                      "coefficient arrays 16-byte aligned and nseg | n");
            return SCD_ERR_ARG;
        }
        a.bb_y = static_cast<const float *>(b->y.data);
        a.bb_ldy = b->y.ldc;
        a.bb_seg_imgs = d->dst.n / b->nseg;
        a.bb_mean = b->save_mean;
        a.bb_inv = b->save_invstd;
        a.bb_scale = b->scale;
        a.bb_shift = b->shift;
        a.bb_rec = b->rec;
    }
    {
        const int64_t sb = (pixels(d->src) - 1) * d->src.ldc * eb + int64_t(d->src.c) * eb;
        a.src_bytes = sb < (int64_t(1) << 31) ? uint32_t(sb) : 0u;
    }
    a.src_bound = d->src_bound;
    a.dst_bound = d->dst_bound;
    a.dst_bound_seed = d->dst_bound_seed;
    if (d->dst_bound_seed && !d->dst_bound) {
        set_error("igemm: dst_bound_seed needs dst_bound");
        return SCD_ERR_ARG;
    }
    a.math = d->math;
    a.tune = d->tune;
    if (d->wsplit && !aligned16(d->wsplit)) {
        set_error("igemm: wsplit must be 16-byte aligned");
        return SCD_ERR_ALIGN;
    }
    return SCD_OK;
}
}  // namespace scd

namespace scd {
// Image chunking.  The buffer-load kernels address operands with 32-bit byte offsets, so a conv whose
// operands span 2 GiB or more (e.g. the Siamese level-0 maps at bs=64: 128 x 256^2 x 64 fp32) runs as several
// launches over image ranges.  A chunk keeps whole BatchNorm coefficient segments or divides one, so the
// per-segment coefficient pointers are offset instead of the kernels learning an image base; fused
// statistics / BN-backward records are per image tile, so their pointers advance by whole images.
static int64_t img_bytes(const scd_nhwc_t &v) { return int64_t(v.h) * v.w * v.ldc * elem_bytes(v); }
static int image_chunk(int64_t bytes_per_img, int n, int seg) {
    const int64_t lim = ((int64_t(1) << 31) - 1) / std::max<int64_t>(bytes_per_img, 1);
    if (lim >= n) return n;
    if (lim < 1) return 0;
    if (lim >= seg) return int(lim / seg) * seg;
    for (int c = int(lim); c >= 1; --c)
        if (seg % c == 0) return c;
    return 1;
}
static scd_nhwc_t img_slice(scd_nhwc_t v, int img0, int cnt) {
    v.data = static_cast<char *>(v.data) + img0 * img_bytes(v);
    v.n = cnt;
    return v;
}

// Images per launch for `d` (d->src.n = one launch; 0 = cannot chunk, one launch on 64-bit-offset kernels).
static int igemm_chunk(const scd_igemm_t *d) {
    if (d->store_mode != 0 || d->src.n != d->dst.n || d->src.n < 2) return d->src.n;
    const int64_t per = std::max(img_bytes(d->src), std::max(img_bytes(d->dst), d->bn_bwd ? img_bytes(d->bn_bwd->y)
                                                                                          : int64_t(0)));
    if (int64_t(d->src.n) * per < (int64_t(1) << 31)) return d->src.n;
    int seg = 1;  // segment size of the coefficient arrays the launch reads (1 = none)
    if (d->in_scale && d->in_nseg > 0) seg = d->src.n / d->in_nseg;
    if (d->bn_bwd && d->bn_bwd->nseg > 0) {
        const int sb = d->src.n / d->bn_bwd->nseg;
        seg = seg == 1 ? sb : (sb == seg ? seg : 0);
    }
    return seg > 0 ? image_chunk(per, d->src.n, seg) : 0;
}

// Descriptor of images [img0, img0 + cnt) (tiles_per_img: fused-record tiles per image).
static scd_igemm_t igemm_slice(const scd_igemm_t *d, int img0, int cnt, int tiles_per_img, scd_bn_bwd_tiles_t &b) {
    scd_igemm_t c = *d;
    c.src = img_slice(d->src, img0, cnt);
    c.dst = img_slice(d->dst, img0, cnt);
    if (d->stat_rec) c.stat_rec = d->stat_rec + size_t(img0) * tiles_per_img * d->n_out * 2;
    if (d->in_scale && d->in_nseg > 0) {
        const int sg = d->src.n / d->in_nseg;
        c.in_scale = d->in_scale + size_t(img0 / sg) * d->src.c;
        c.in_shift = d->in_shift + size_t(img0 / sg) * d->src.c;
        c.in_nseg = std::max(1, cnt / sg);
    }
    if (d->bn_bwd && d->bn_bwd->nseg > 0) {
        b = *d->bn_bwd;
        const int sg = d->src.n / b.nseg;
        const size_t o = size_t(img0 / sg) * d->n_out;
        b.y = img_slice(b.y, img0, cnt);
        b.save_mean += o;
        b.save_invstd += o;
        b.scale += o;
        b.shift += o;
        b.nseg = std::max(1, cnt / sg);
        b.rec += size_t(img0) * tiles_per_img * 2;
        c.bn_bwd = &b;
    }
    return c;
}

// Kernel arguments as the launches will see them (the first chunk's), with n_img restored to the whole batch:
// what the eligibility and record-tile queries evaluate.
static int igemm_query_prepare(const scd_igemm_t *d, IgemmArgs &a) {
    const int chunk = igemm_chunk(d);
    if (chunk <= 0 || chunk >= d->src.n) return igemm_prepare(d, a);
    scd_bn_bwd_tiles_t b;
    const scd_igemm_t c = igemm_slice(d, 0, chunk, 0, b);
    SCD_TRY(igemm_prepare(&c, a));
    a.n_img = d->src.n;
    return SCD_OK;
}

static int conv_igemm_run(const scd_igemm_t *d, hipStream_t s, int bb_ntiles_total);
}  // namespace scd

extern "C" int scd_igemm_stat_tiles(const scd_igemm_t *d, int32_t *tile_pixels) {
    clear_error();
    IgemmArgs a;
    if (igemm_query_prepare(d, a) != SCD_OK || d->store_mode != 0) return 0;
    int tp = 0;
    const int n = halo_stat_tiles(a, &tp);
    if (tile_pixels) *tile_pixels = tp;
    return n;
}

extern "C" int scd_igemm_bn_bwd_tiles(const scd_igemm_t *d, int32_t *tile_pixels) {
    clear_error();
    IgemmArgs a;
    if (igemm_query_prepare(d, a) != SCD_OK || d->store_mode != 0 || !igemm_takes_halo16(a)) return 0;
    int tp = 0;
    const int n = halo_stat_tiles(a, &tp);
    if (tile_pixels) *tile_pixels = tp;
    return n;
}

extern "C" int scd_igemm_input_bn_supported(const scd_igemm_t *d) {
    clear_error();
    IgemmArgs a;
    if (igemm_query_prepare(d, a) != SCD_OK) return 0;
    return igemm_takes_halo16(a) ? 1 : 0;
}

extern "C" int scd_igemm_arith(const scd_igemm_t *d) {
    clear_error();
    IgemmArgs a;
    SCD_TRY(igemm_query_prepare(d, a));
    if (!math_split(a.math)) return SCD_MATH_F32;
    if (igemm_takes_halo16(a)) return a.math;  // under SCD_MATH_H2 only bounded h2-split convs take it
    if (igemm_takes_gather16(a)) return a.math;  // h2 (bounded, h2 split) or bf16
    if (igemm_takes_c16(a)) return a.math;  // under SCD_MATH_H2 only bounded h2-split input layers take it
    if (a.sb) {
        set_error("igemm: no bf16-storage kernel takes this shape");
        return SCD_ERR_ARG;
    }
    return a.c % 16 == 0 ? SCD_MATH_X3 : SCD_MATH_F32;  // launch_igemm_x3's eligibility
}


extern "C" int scd_conv_igemm(const scd_igemm_t *d, scd_stream_t stream) {
    clear_error();
    if (!d) {
        set_error("igemm: null descriptor");
        return SCD_ERR_ARG;
    }
    hipStream_t s = as_stream(stream);
    const int chunk = igemm_chunk(d);
    if (chunk <= 0 || chunk >= d->src.n) return conv_igemm_run(d, s, 0);
    int tiles = 0, tile_pixels = 0;
    if (d->stat_rec || d->bn_bwd) {
        IgemmArgs a;
        SCD_TRY(igemm_query_prepare(d, a));
        tiles = halo_stat_tiles(a, &tile_pixels);
    }
    const int tiles_per_img = tiles / d->src.n;
    for (int img0 = 0; img0 < d->src.n; img0 += chunk) {
        scd_bn_bwd_tiles_t b;
        const scd_igemm_t c = igemm_slice(d, img0, std::min(chunk, d->src.n - img0), tiles_per_img, b);
        SCD_TRY(conv_igemm_run(&c, s, d->bn_bwd ? tiles : 0));
    }
    return SCD_OK;
}

namespace scd {
static int conv_igemm_run(const scd_igemm_t *d, hipStream_t s, int bb_ntiles_total) {
    IgemmArgs a;
    SCD_TRY(igemm_prepare(d, a));
    if (d->stat_rec) {
        int tp = 0;
        if (halo_stat_tiles(a, &tp) == 0) {
            set_error("igemm: fused statistics requested for a shape without them (check scd_igemm_stat_tiles)");
            return SCD_ERR_ARG;
        }
    }
    if (a.bb_rec) {
        int tp = 0;
        if (!igemm_takes_halo16(a) || d->stat_rec || (a.bb_ntiles = halo_stat_tiles(a, &tp)) == 0) {
            set_error("igemm: fused BatchNorm-backward sums are not supported for this descriptor "
                      "(check scd_igemm_bn_bwd_tiles)");
            return SCD_ERR_ARG;
        }
        if (bb_ntiles_total) a.bb_ntiles = bb_ntiles_total;  // record row stride of the whole batch (chunks)
    }
    if (a.in_scale && !igemm_takes_halo16(a)) {
        set_error("igemm: the fused input transform is not supported for this shape/arithmetic "
                  "(check scd_igemm_input_bn_supported)");
        return SCD_ERR_ARG;
    }
    if (a.dst_bound && a.store_mode != 1 && !igemm_takes_halo16(a) && !igemm_takes_gather16(a) &&
        !igemm_takes_c16(a)) {
        set_error("igemm: dst_bound of a store_mode 0 conv needs the halo16, c16 or gather16 kernel "
                  "(ConvTranspose store_mode 1 convs take it on every split-bf16 kernel)");
        return SCD_ERR_ARG;
    }
    if (math_split(a.math) && launch_igemm_x3(a, s)) return launch_status("scd_conv_igemm");
    if (a.sb) {
        set_error("igemm: bf16 views need the bf16 halo16 / c16 / gather16 kernels; this shape takes none "
                  "(check scd_igemm_arith): n=%d c=%d %dx%d -> %dx%d n_out=%d ldc=%d taps=%d stride=%d store=%d "
                  "K=%d wsplit=%d src_bytes=%u dst%%16=%d bias%%16=%d in_bn=%d bn_bwd=%d math=%d",
                  a.n_img, a.c, a.hs, a.ws, a.ho, a.wo, a.n_out, a.ldc_d, a.ntaps, a.stride, a.store_mode, a.K,
                  a.wsplit ? 1 : 0, a.src_bytes, int(reinterpret_cast<uintptr_t>(a.dst) & 15),
                  a.bias ? int(reinterpret_cast<uintptr_t>(a.bias) & 15) : -1, a.in_scale ? 1 : 0, a.bb_rec ? 1 : 0,
                  a.math);
        return SCD_ERR_ARG;
    }
    if (a.dst_bound) {
        set_error("igemm: dst_bound needs the split-bf16 kernels (math x3 / h2 and src.c %% 16 == 0)");
        return SCD_ERR_ARG;
    }
    if (d->n_out >= 128)
        launch_igemm_bk<2, 2, 2, 2>(a, s);  // 128 x 128
    else if (d->n_out >= 64)
        launch_igemm_bk<4, 1, 2, 2>(a, s);  // 256 x 64
    else
        launch_igemm_bk<4, 1, 2, 1>(a, s);  // 256 x 32
    return launch_status("scd_conv_igemm");
}
}  // namespace scd

namespace scd {
struct WgradTile {
    int id, bm, bn, threads;
};
// Tile shapes of the wgrad instantiations; per call the one with the least padded MFMA work wins
// (ties: the larger tile).  E.g. R=64, Ng=576 (9x64): 64x192 is exact where 64x256 computes 33% waste.
static const WgradTile kWgradTiles[] = {
    {0, 128, 128, 256},  // wgrad_f32<2,2,2,2>
    {1, 64, 256, 256},   // wgrad_f32<1,4,2,2>
    {2, 64, 192, 256},   // wgrad_f32<2,2,1,3>
    {3, 64, 96, 128},    // wgrad_f32<2,1,1,3>   (first layer: Ng = 9*8 = 72)
    {4, 32, 128, 256},   // wgrad_f32<1,4,1,1>
};
static WgradTile wgrad_tile(int R, int Ng) {
    WgradTile best = kWgradTiles[0];
    int64_t best_work = -1;
    for (const WgradTile &t : kWgradTiles) {
        const int64_t work = int64_t((R + t.bm - 1) / t.bm) * t.bm * (int64_t((Ng + t.bn - 1) / t.bn) * t.bn);
        if (best_work < 0 || work < best_work || (work == best_work && t.bm * t.bn > best.bm * best.bn)) {
            best = t;
            best_work = work;
        }
    }
    return best;
}
static int wgrad_validate(const scd_wgrad_t *d) {
    if (!d) {
        set_error("wgrad: null descriptor");
        return SCD_ERR_ARG;
    }
    SCD_TRY(check_view(d->rows, "wgrad.rows"));
    SCD_TRY(check_view(d->src, "wgrad.src"));
    SCD_TRY(check_taps(d->ntaps, d->dy, d->dx));
    if (!math_valid(d->math)) {
        set_error("wgrad: math %d is not an scd_conv_math value", d->math);
        return SCD_ERR_ARG;
    }
    if (d->rows.n != d->src.n || d->stride < 1) {
        set_error("wgrad: rows.n=%d src.n=%d stride=%d", d->rows.n, d->src.n, d->stride);
        return SCD_ERR_ARG;
    }
    if (pixels(d->rows) >= (int64_t(1) << 31) || pixels(d->src) >= (int64_t(1) << 31)) {
        set_error("wgrad: problem too large for 32-bit pixel indexing");
        return SCD_ERR_ARG;
    }
    const int dt = common_dtype("wgrad", {&d->rows, &d->src, d->rows_y.data ? &d->rows_y : nullptr});
    if (dt < 0) return SCD_ERR_ARG;
    if (dt == SCD_DT_BF16 && d->math != SCD_MATH_BF16) {
        set_error("wgrad: bf16 views need math SCD_MATH_BF16 (got %d)", d->math);
        return SCD_ERR_ARG;
    }
    return SCD_OK;
}
static bool wgrad_sb(const scd_wgrad_t *d) { return is_bf16(d->rows); }
// Workgroups of one wgrad instantiation that the whole chip holds at once (occupancy API x CUs), cached.
static int wgrad_resident_blocks(const WgradTile &t, int math) {
    const int x3 = math_split(math);
    static int cache[2][8] = {{0}};
    if (cache[x3][t.id] > 0) return cache[x3][t.id];
    int per_cu = 0, cus = 0, dev = 0;
    const void *fn = nullptr;
    if (x3) {
        fn = wgrad_x3_fn(t.id);
    } else {
        switch (t.id) {
            case 0: fn = reinterpret_cast<const void *>(&wgrad_f32<2, 2, 2, 2, 16>); break;
            case 1: fn = reinterpret_cast<const void *>(&wgrad_f32<1, 4, 2, 2, 16>); break;
            case 2: fn = reinterpret_cast<const void *>(&wgrad_f32<2, 2, 1, 3, 16>); break;
            case 3: fn = reinterpret_cast<const void *>(&wgrad_f32<2, 1, 1, 3, 16>); break;
            default: fn = reinterpret_cast<const void *>(&wgrad_f32<1, 4, 1, 1, 16>); break;
        }
    }
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, t.threads, 0) != hipSuccess || per_cu < 1 ||
        cus < 1) {
        (void)hipGetLastError();
        // MI355X: 256 CUs, >= 2 resident 256-thread blocks; cached like a successful query so the split plan
        // (scd_wgrad_plan) and the launch never disagree
        cache[x3][t.id] = 2 * 256;
        return cache[x3][t.id];
    }
    cache[x3][t.id] = per_cu * cus;
    return cache[x3][t.id];
}

// Split-K factor: the block count tiles*nsplit is quantised against the chip's resident capacity so the
// last round is not a handful of lone workgroups (one wave per SIMD cannot keep the MFMA pipe busy):
// maximise blocks / (rounds * capacity), ties (within 2%) to fewer splits (less slab traffic).
// Split factor over K units (pixels, or 2x16 patches for the halo kernel): the block count tiles*nsplit is
// quantised against the chip's resident capacity so the last round is not a handful of lone workgroups.
// Maximise blocks / (rounds * capacity); ties (within 2%) go to fewer splits (less slab traffic).
static void split_units(int64_t M, int64_t tiles, int64_t cap, int64_t min_units, int64_t gran, int *nsplit,
                        int *kchunk) {
    int64_t maxsplit = (M + min_units - 1) / min_units;
    const int64_t lim = (8 * cap + tiles - 1) / tiles;
    if (maxsplit > lim) maxsplit = lim;
    if (maxsplit < 1) maxsplit = 1;
    int64_t best_kc = (M + gran - 1) / gran * gran;
    double best_eff = -1.0;
    for (int64_t want = 1; want <= maxsplit; ++want) {
        int64_t kc = (M + want - 1) / want;
        kc = (kc + gran - 1) / gran * gran;
        const int64_t n = (M + kc - 1) / kc;
        const int64_t blocks = tiles * n;
        const int64_t rounds = (blocks + cap - 1) / cap;
        const double eff = double(blocks) / double(rounds * cap);
        if (eff > best_eff + 0.02) {
            best_eff = eff;
            best_kc = kc;
        }
    }
    *kchunk = int(best_kc);
    *nsplit = int((M + best_kc - 1) / best_kc);
}

// Halo weight grad eligibility: x3 math, 3x3 taps in standard order, stride 1, same-size maps,
// R and C multiples of 64, maps tiled by 2x16 patches.
static bool wgrad_halo_shape(const scd_wgrad_t *d) {
    if (!math_split(d->math) || d->stride != 1 || d->ntaps != 9) return false;
    for (int t = 0; t < 9; ++t)
        if (d->dy[t] != t / 3 - 1 || d->dx[t] != t % 3 - 1) return false;
    return d->rows.h == d->src.h && d->rows.w == d->src.w && d->rows.c % 64 == 0 && d->rows.h % 2 == 0 &&
           d->rows.w % 16 == 0 && halo_enabled(d->tune);
}
static bool wgrad_halo_ok(const scd_wgrad_t *d) { return wgrad_halo_shape(d) && d->src.c % 64 == 0; }
// The 16-channel-source halo kernel (the padded input layer).  SCD_TUNE_NO_WGRAD_C16 sends it back to the generic x3
// weight grad (A/B).
static bool wgrad_c16_ok(const scd_wgrad_t *d) {
    return wgrad_halo_shape(d) && d->src.c == 16 && !(d->tune & SCD_TUNE_NO_WGRAD_C16);
}

// Both operands bounded: the h2 weight grad under SCD_MATH_H2 (x3 otherwise).
static bool wgrad_bounded(const scd_wgrad_t *d) { return d->rows_bound && d->src_bound; }
// The halo weight grad with the rows' BatchNorm backward (rows_y) and the dY store (rows_out): its bf16 and h2 along-c
// variants; h2 in 128-row blocks only (the 64-row h2 block would spill), at most two rows segments per launch.
static bool wgrad_halo_rbn_ok(const scd_wgrad_t *d) {
    if (!wgrad_halo_ok(d) || !wgrad16_rows_bn_ok(d->math, d->tune, wgrad_bounded(d))) return false;
    if (d->math == SCD_MATH_H2 && wgrad_halo_rblock(d->math, d->tune, d->rows.c, true) != 128) return false;
    return !d->rows_y.data || (d->rows_nseg >= 1 && d->rows_nseg <= 2);
}
// The generic (non-halo) weight grad in h2: bounded, SCD_MATH_H2, a tile with an h2 instantiation.
// SCD_TUNE_NO_WGRAD_H2 keeps it on x3 (A/B).
static bool wgrad_generic_h2(const scd_wgrad_t *d) {
    return wgrad_bounded(d) && d->math == SCD_MATH_H2 && !(d->tune & SCD_TUNE_NO_WGRAD_H2) &&
           wgrad_x3_h2_tile(wgrad_tile(d->rows.c, d->ntaps * d->src.c).id);
}

// The generic weight grad in bf16: the ConvTranspose weight grad (4 taps) under SCD_MATH_BF16; the 3x3 weight grads
// the halo kernels do not take keep x3.
static bool wgrad_generic_bf16(const scd_wgrad_t *d) { return d->math == SCD_MATH_BF16 && d->ntaps == 4; }

static int wgrad_halo_resident(const scd_wgrad_t *d, bool c16, bool bounded, int rblock) {
    // per halo weight-grad kernel: 16x16x32 x3 / x5 / bf16 / h2 (x layout); 16-channel x3 / x5 / bf16; the 128-row
    // bf16 / h2 blocks
    static int caches[2][12] = {{0}};
    const int m = math_planes(d->math);
    const int planes = m == 1 ? 0 : m == 5 ? 1
                       : (m == 2 && bounded && (!c16 || wgrad_c16_planes(d->math, d->tune, bounded) == 4)) ? 3
                                                                                                      : 2;
    const bool r128 = !c16 && rblock == 128;
    const int lay = (d->tune & SCD_TUNE_W16_LAYOUT_2X2) ? 1 : 0;
    int &cache = caches[lay][r128 ? 9 + (planes == 3) : c16 ? 5 + planes : 1 + planes];
    if (cache > 0) return cache;
    int per_cu = 0, cus = 0, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu,
                                                     c16 ? wgrad_halo16_c16_fn(d->math, d->tune, bounded)
                                                         : wgrad_halo_fn(d->math, d->tune, bounded, rblock),
                                                     r128 ? 512 : 256, 0) !=
            hipSuccess ||
        per_cu < 1 ||
        cus < 1) {
        (void)hipGetLastError();
        cache = (r128 ? 1 : 2) * 256;  // cached: plan and launch must see the same capacity
        return cache;
    }
    cache = per_cu * cus;
    return cache;
}

static void wgrad_split(const scd_wgrad_t *d, int *nsplit, int *kchunk) {
    if (wgrad_halo_ok(d) || wgrad_c16_ok(d)) {
        const bool c16 = !wgrad_halo_ok(d);
        const int rb = c16 ? 64 : wgrad_halo_rblock(d->math, d->tune, d->rows.c, wgrad_bounded(d));
        const int64_t patches = pixels(d->rows) / 32;
        const int64_t tiles = int64_t(d->rows.c / rb) * (c16 ? 1 : d->src.c / 64);
        split_units(patches, tiles, wgrad_halo_resident(d, c16, wgrad_bounded(d), rb), 8, 1, nsplit, kchunk);
        return;
    }
    const int Ng = d->ntaps * d->src.c;
    const WgradTile t = wgrad_tile(d->rows.c, Ng);
    const int64_t tiles = int64_t((d->rows.c + t.bm - 1) / t.bm) * ((Ng + t.bn - 1) / t.bn);
    split_units(pixels(d->rows), tiles, wgrad_resident_blocks(t, d->math), 256, 16, nsplit, kchunk);
}
}  // namespace scd

namespace scd {
static bool wgrad_src_bn_ok(const scd_wgrad_t *d) { return wgrad_halo_ok(d) || wgrad_c16_ok(d); }
// The generic split-arithmetic weight grad (wgrad_x3: the ConvTranspose weight grad) also writes src column sums.
static bool wgrad_colsum_ok(const scd_wgrad_t *d) {
    return math_split(d->math) && !wgrad_halo_ok(d) && !wgrad_c16_ok(d) && d->src.c % 4 == 0;
}
}  // namespace scd

extern "C" int scd_wgrad_colsum_supported(const scd_wgrad_t *d) {
    clear_error();
    if (wgrad_validate(d) != SCD_OK) return 0;
    return wgrad_colsum_ok(d) ? 1 : 0;
}

extern "C" int scd_wgrad_src_bn_supported(const scd_wgrad_t *d) {
    clear_error();
    if (wgrad_validate(d) != SCD_OK) return 0;
    return wgrad_src_bn_ok(d) ? 1 : 0;
}

extern "C" int scd_wgrad_rows_bn_supported(const scd_wgrad_t *d) {
    clear_error();
    if (wgrad_validate(d) != SCD_OK) return 0;
    return wgrad_c16_ok(d) || wgrad_halo_rbn_ok(d) ? 1 : 0;
}

extern "C" int scd_wgrad_arith(const scd_wgrad_t *d) {
    clear_error();
    SCD_TRY(wgrad_validate(d));
    if (!math_split(d->math)) return SCD_MATH_F32;
    if (wgrad_sb(d) && !wgrad_halo_ok(d) && !wgrad_c16_ok(d) && !wgrad_generic_bf16(d)) {
        set_error("wgrad: no bf16-storage kernel takes this shape");
        return SCD_ERR_ARG;
    }
    if (wgrad_halo_ok(d)) return d->math == SCD_MATH_H2 && !wgrad_bounded(d) ? SCD_MATH_X3 : d->math;
    if (wgrad_c16_ok(d))
        return d->math != SCD_MATH_H2 ? d->math
               : wgrad_c16_planes(d->math, d->tune, wgrad_bounded(d)) == 4 ? SCD_MATH_H2
                                                                          : SCD_MATH_X3;
    return wgrad_generic_h2(d) ? SCD_MATH_H2 : wgrad_generic_bf16(d) ? SCD_MATH_BF16 : SCD_MATH_X3;
}

extern "C" int scd_wgrad_rows_per_block(const scd_wgrad_t *d) {
    clear_error();
    SCD_TRY(wgrad_validate(d));
    if (wgrad_halo_ok(d)) return wgrad_halo_rblock(d->math, d->tune, d->rows.c, wgrad_bounded(d));
    return wgrad_c16_ok(d) ? 64 : 0;
}

namespace scd {
// Images per weight-grad launch (rows.n = one launch; 0 = one image alone exceeds 2 GiB), see image_chunk.
static int wgrad_chunk(const scd_wgrad_t *d) {
    int64_t per = std::max(img_bytes(d->rows), img_bytes(d->src));
    if (d->rows_y.data) per = std::max(per, img_bytes(d->rows_y));
    if (int64_t(d->rows.n) * per < (int64_t(1) << 31)) return d->rows.n;
    int seg = (d->src_scale && d->src_nseg > 0) ? d->src.n / d->src_nseg : 1;
    if (d->rows_y.data && d->rows_nseg > 0) seg = std::max(seg, d->rows.n / d->rows_nseg);
    return image_chunk(per, d->rows.n, seg);
}
static scd_wgrad_t wgrad_slice(const scd_wgrad_t *d, int img0, int cnt) {
    scd_wgrad_t c = *d;
    c.rows = img_slice(d->rows, img0, cnt);
    c.src = img_slice(d->src, img0, cnt);
    if (d->src_scale && d->src_nseg > 0) {
        const int sg = d->src.n / d->src_nseg;
        c.src_scale = d->src_scale + size_t(img0 / sg) * d->src.c;
        c.src_shift = d->src_shift + size_t(img0 / sg) * d->src.c;
        c.src_nseg = std::max(1, cnt / sg);
    }
    if (d->rows_y.data && d->rows_nseg > 0) {
        const int sg = d->rows.n / d->rows_nseg;
        const size_t o = size_t(img0 / sg) * d->rows.c;
        c.rows_y = img_slice(d->rows_y, img0, cnt);
        c.rows_mean = d->rows_mean + o;
        c.rows_invstd = d->rows_invstd + o;
        c.rows_scale = d->rows_scale + o;
        c.rows_shift = d->rows_shift + o;
        c.rows_coef = d->rows_coef + 2 * o;
        c.rows_nseg = std::max(1, cnt / sg);
    }
    if (d->rows_out.data) c.rows_out = img_slice(d->rows_out, img0, cnt);
    return c;
}
// Total K-splits over the image chunks (each chunk writes its own slab range; the finalize sums them all).
static int wgrad_total_splits(const scd_wgrad_t *d) {
    const int chunk = wgrad_chunk(d);
    int total = 0;
    for (int img0 = 0; img0 < d->rows.n; img0 += std::max(chunk, 1)) {
        const scd_wgrad_t c = wgrad_slice(d, img0, std::min(std::max(chunk, 1), d->rows.n - img0));
        int ns, kc;
        wgrad_split(&c, &ns, &kc);
        total += ns;
    }
    return total;
}
static int conv_wgrad_run(const scd_wgrad_t *d, float *slabs, size_t slab_bytes, hipStream_t s);
}  // namespace scd

extern "C" int scd_wgrad_plan(const scd_wgrad_t *d, int32_t *nsplit, size_t *slab_bytes) {
    clear_error();
    SCD_TRY(wgrad_validate(d));
    if (wgrad_chunk(d) < 1) {
        set_error("wgrad: one image of the operands spans 2 GiB or more (32-bit buffer offsets)");
        return SCD_ERR_ARG;
    }
    const int ns = wgrad_total_splits(d);
    if (nsplit) *nsplit = ns;
    if (slab_bytes) *slab_bytes = size_t(ns) * d->rows.c * d->ntaps * d->src.c * sizeof(float);
    return SCD_OK;
}

extern "C" int scd_conv_wgrad(const scd_wgrad_t *d, float *slabs, size_t slab_bytes, scd_stream_t stream) {
    clear_error();
    SCD_TRY(wgrad_validate(d));
    const int chunk = wgrad_chunk(d);
    if (chunk < 1) {
        set_error("wgrad: one image of the operands spans 2 GiB or more (32-bit buffer offsets)");
        return SCD_ERR_ARG;
    }
    if (chunk >= d->rows.n) return conv_wgrad_run(d, slabs, slab_bytes, as_stream(stream));
    const size_t slab = size_t(d->rows.c) * d->ntaps * d->src.c;
    const size_t need = size_t(wgrad_total_splits(d)) * slab * sizeof(float);
    if (!slabs || slab_bytes < need) {
        set_error("wgrad: slab workspace %zu < %zu bytes", slab_bytes, need);
        return SCD_ERR_WORKSPACE;
    }
    size_t used = 0;  // slabs written by the previous chunks
    for (int img0 = 0; img0 < d->rows.n; img0 += chunk) {
        scd_wgrad_t c = wgrad_slice(d, img0, std::min(chunk, d->rows.n - img0));
        if (d->src_colsum) c.src_colsum = d->src_colsum + used * size_t(d->ntaps) * d->src.c;
        int ns, kc;
        wgrad_split(&c, &ns, &kc);
        SCD_TRY(conv_wgrad_run(&c, slabs + used * slab, (size_t(ns)) * slab * sizeof(float), as_stream(stream)));
        used += size_t(ns);
    }
    return SCD_OK;
}

namespace scd {
static int conv_wgrad_run(const scd_wgrad_t *d, float *slabs, size_t slab_bytes, hipStream_t s) {
    int ns, kc;
    wgrad_split(d, &ns, &kc);
    const int Ng = d->ntaps * d->src.c;
    const size_t need = size_t(ns) * d->rows.c * Ng * sizeof(float);
    if (!slabs || slab_bytes < need) {
        set_error("wgrad: slab workspace %zu < %zu bytes", slab_bytes, need);
        return SCD_ERR_WORKSPACE;
    }
    WgradArgs a;
    a.sb = wgrad_sb(d) ? 1 : 0;
    const int eb = elem_size(a.sb);
    if (d->src_colsum && !wgrad_colsum_ok(d)) {
        set_error("wgrad: src_colsum needs the generic split-arithmetic weight grad (check scd_wgrad_colsum_supported)");
        return SCD_ERR_ARG;
    }
    a.colsum = d->src_colsum;
    if (a.sb && !wgrad_halo_ok(d) && !wgrad_c16_ok(d) && !wgrad_generic_bf16(d)) {
        set_error("wgrad: bf16 views need the bf16 halo16 / c16 / ConvTranspose weight-grad kernels; this shape takes "
                  "none (check scd_wgrad_arith)");
        return SCD_ERR_ARG;
    }
    a.rows = static_cast<const float *>(d->rows.data);
    a.ho = d->rows.h;
    a.wo = d->rows.w;
    a.R = d->rows.c;
    a.ldc_r = d->rows.ldc;
    a.src = static_cast<const float *>(d->src.data);
    a.hs = d->src.h;
    a.ws = d->src.w;
    a.C = d->src.c;
    a.ldc_s = d->src.ldc;
    a.stride = d->stride;
    a.ntaps = d->ntaps;
    a.tdy = pack_taps(d->dy, d->ntaps);
    a.tdx = pack_taps(d->dx, d->ntaps);
    a.Ng = Ng;
    a.M = int(pixels(d->rows));
    a.kchunk = kc;
    a.slabs = slabs;
    a.div_hw = make_fastdiv(uint32_t(d->rows.h * d->rows.w));
    a.div_w = make_fastdiv(uint32_t(d->rows.w));
    a.div_c = make_fastdiv(uint32_t(d->src.c));
    // byte extents for the x3 kernel's buffer loads (32-bit offsets)
    const int64_t rb = (pixels(d->rows) - 1) * d->rows.ldc * eb + int64_t(d->rows.c) * eb;
    const int64_t sb = (pixels(d->src) - 1) * d->src.ldc * eb + int64_t(d->src.c) * eb;
    if (rb >= (int64_t(1) << 31) || sb >= (int64_t(1) << 31)) {
        set_error("wgrad: operands above 2 GiB are not supported (32-bit buffer offsets)");
        return SCD_ERR_ARG;
    }
    a.rows_bytes = uint32_t(rb);
    a.src_bytes = uint32_t(sb);
    a.src_scale = d->src_scale;
    a.src_shift = d->src_shift;
    a.src_seg_imgs = d->src.n;
    a.rows_bound = d->rows_bound;
    a.src_bound = d->src_bound;
    a.math = d->math;
    a.tune = d->tune;
    a.rows_y = nullptr;
    a.ldc_y = 0;
    a.y_bytes = 0;
    a.rbn_mean = a.rbn_inv = a.rbn_gamma = a.rbn_scale = a.rbn_shift = a.rbn_coef = nullptr;
    a.rows_seg_imgs = d->rows.n;
    if (d->rows_y.data) {
        const scd_nhwc_t &y = d->rows_y;
        const int64_t yb = (pixels(y) - 1) * y.ldc * eb + int64_t(y.c) * eb;
        if (check_view(y, "wgrad.rows_y") != SCD_OK || y.n != d->rows.n || y.h != d->rows.h || y.w != d->rows.w ||
            y.c != d->rows.c || y.ldc % 4 || d->rows_nseg < 1 || d->rows.n % d->rows_nseg || !d->rows_mean ||
            !d->rows_invstd || !d->rows_scale || !d->rows_shift || !d->rows_coef || !aligned16(d->rows_mean) ||
            !aligned16(d->rows_invstd) || !aligned16(d->rows_scale) || !aligned16(d->rows_shift) ||
            !aligned16(d->rows_coef) || (d->rows_gamma && !aligned16(d->rows_gamma)) ||
            !(wgrad_c16_ok(d) || wgrad_halo_rbn_ok(d)) || yb >= (int64_t(1) << 31)) {
            set_error("wgrad: the rows BatchNorm backward needs y shaped as rows, rows_nseg | rows.n, 16-byte "
                      "aligned coefficient arrays and a supported shape (check scd_wgrad_rows_bn_supported)");
            return SCD_ERR_ARG;
        }
        a.rows_y = static_cast<const float *>(y.data);
        a.ldc_y = y.ldc;
        a.y_bytes = uint32_t(yb);
        a.rbn_mean = d->rows_mean;
        a.rbn_inv = d->rows_invstd;
        a.rbn_gamma = d->rows_gamma;
        a.rbn_scale = d->rows_scale;
        a.rbn_shift = d->rows_shift;
        a.rbn_coef = d->rows_coef;
        a.rows_seg_imgs = d->rows.n / d->rows_nseg;
    }
    a.rows_out = nullptr;
    a.ldc_o = 0;
    a.rows_out_bound = nullptr;
    if (d->rows_out.data) {
        const scd_nhwc_t &o = d->rows_out;
        if (!d->rows_y.data || !wgrad_halo_rbn_ok(d) || check_view(o, "wgrad.rows_out") != SCD_OK || o.n != d->rows.n ||
            o.h != d->rows.h || o.w != d->rows.w || o.c != d->rows.c || o.dtype != d->rows.dtype || o.ldc % 4 ||
            (reinterpret_cast<uintptr_t>(o.data) & (a.sb ? 7 : 15))) {
            set_error("wgrad: rows_out needs rows_y on the halo weight grad (scd_wgrad_rows_bn_supported) and a view "
                      "shaped and typed as rows, ldc %% 4 == 0, aligned");
            return SCD_ERR_ARG;
        }
        a.rows_out = o.data;
        a.ldc_o = o.ldc;
        a.rows_out_bound = d->rows_out_bound;
    }
    if (d->src_scale || d->src_shift) {
        if (!d->src_scale || !d->src_shift || d->src_nseg < 1 || d->src.n % d->src_nseg ||
            !aligned16(d->src_scale) || !aligned16(d->src_shift) || !wgrad_src_bn_ok(d)) {
            set_error("wgrad: src transform needs both 16-byte aligned coefficient arrays, src_nseg | src.n and a "
                      "supported shape (check scd_wgrad_src_bn_supported)");
            return SCD_ERR_ARG;
        }
        a.src_seg_imgs = d->src.n / d->src_nseg;
    }
    if (wgrad_halo_ok(d)) {
        a.n_img_w = d->rows.n;
        a.grid_r = a.R / wgrad_halo_rblock(a.math, a.tune, a.R, wgrad_bounded(d));
        a.grid_j = a.C / 64;
        a.remap = xcd_remap_enabled(a.tune);
        launch_wgrad_halo16_x3(a, dim3(a.grid_r * a.grid_j * ns), s);
        return launch_status("scd_conv_wgrad");
    }
    if (wgrad_c16_ok(d)) {
        a.n_img_w = d->rows.n;
        a.grid_r = a.R / 64;
        a.grid_j = 1;
        a.remap = xcd_remap_enabled(a.tune);
        launch_wgrad_halo16_c16(a, dim3(a.grid_r * ns), s);
        return launch_status("scd_conv_wgrad");
    }
    const WgradTile t = wgrad_tile(a.R, Ng);
    a.grid_r = (a.R + t.bm - 1) / t.bm;
    a.grid_j = (Ng + t.bn - 1) / t.bn;
    a.remap = xcd_remap_enabled(a.tune);
    dim3 grid(a.grid_r * a.grid_j * ns);
    dim3 block(t.threads);
    if (math_split(a.math)) {
        if (wgrad_generic_h2(d))
            launch_wgrad_x3_h2(a, t.id, grid, block, s);
        else if (wgrad_generic_bf16(d))
            launch_wgrad_x3_bf16(a, t.id, grid, block, s);
        else
            launch_wgrad_x3(a, t.id, grid, block, s);
        return launch_status("scd_conv_wgrad");
    }
    switch (t.id) {
        case 0: hipLaunchKernelGGL((wgrad_f32<2, 2, 2, 2, 16>), grid, block, 0, s, a); break;
        case 1: hipLaunchKernelGGL((wgrad_f32<1, 4, 2, 2, 16>), grid, block, 0, s, a); break;
        case 2: hipLaunchKernelGGL((wgrad_f32<2, 2, 1, 3, 16>), grid, block, 0, s, a); break;
        case 3: hipLaunchKernelGGL((wgrad_f32<2, 1, 1, 3, 16>), grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL((wgrad_f32<1, 4, 1, 1, 16>), grid, block, 0, s, a); break;
    }
    return launch_status("scd_conv_wgrad");
}
}  // namespace scd

namespace scd {
// scd_wgrad_colsum_finalize, two fixed-order stages: (1) in place, split group g's 16 rows summed in split order into
// its first row, one thread per column (coalesced); (2) per channel, the group rows in order, then the taps in order.
constexpr int kColsumGroup = 16;
__global__ __launch_bounds__(256) void colsum_group_kernel(float *__restrict__ colsum, int nsplit, int Ng) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= Ng) return;
    const int s0 = blockIdx.y * kColsumGroup, s1 = min(s0 + kColsumGroup, nsplit);
    float v[kColsumGroup];
#pragma unroll
    for (int u = 0; u < kColsumGroup; ++u) v[u] = s0 + u < s1 ? colsum[size_t(s0 + u) * Ng + j] : 0.f;
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < kColsumGroup; ++u) acc += v[u];
    colsum[size_t(s0) * Ng + j] = acc;
}
__global__ __launch_bounds__(256) void colsum_final_kernel(const float *__restrict__ colsum, int nsplit, int ntaps,
                                                           int C, float *__restrict__ out) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    const int Ng = ntaps * C;
    float tap[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) tap[t] = 0.f;
#pragma unroll 4
    for (int s = 0; s < nsplit; s += kColsumGroup)
#pragma unroll
        for (int t = 0; t < 9; ++t)
            if (t < ntaps) tap[t] += colsum[size_t(s) * Ng + t * C + c];
    float acc = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t)
        if (t < ntaps) acc += tap[t];
    out[c] = acc;
}
}  // namespace scd

extern "C" int scd_wgrad_colsum_finalize(float *colsum, int32_t nsplit, int32_t ntaps, int32_t C, float *out,
                                         scd_stream_t stream) {
    clear_error();
    if (!colsum || !out || nsplit < 1 || ntaps < 1 || ntaps > 9 || C < 1) {
        set_error("wgrad_colsum_finalize: colsum/out non-null, nsplit=%d >= 1, ntaps=%d in [1, 9], C=%d >= 1", nsplit,
                  ntaps, C);
        return SCD_ERR_ARG;
    }
    const hipStream_t s = as_stream(stream);
    const int Ng = ntaps * C;
    hipLaunchKernelGGL(colsum_group_kernel, dim3((Ng + 255) / 256, (nsplit + kColsumGroup - 1) / kColsumGroup),
                       dim3(256), 0, s, colsum, nsplit, Ng);
    hipLaunchKernelGGL(colsum_final_kernel, dim3((C + 255) / 256), dim3(256), 0, s, colsum, nsplit, ntaps, C, out);
    return launch_status("scd_wgrad_colsum_finalize");
}

extern "C" int scd_wgrad_finalize(float *slabs, int32_t nsplit, int32_t R, int32_t ntaps, int32_t C,
                                  int32_t mode, int32_t c_valid, float *out, scd_stream_t stream) {
    clear_error();
    if (!slabs || !out || nsplit < 1 || R < 1 || ntaps < 1 || C < 1 || (mode != 0 && mode != 1) || c_valid < 1 ||
        c_valid > C) {
        set_error("wgrad_finalize: bad arguments");
        return SCD_ERR_ARG;
    }
    const size_t total = size_t(R) * ntaps * C;
    const int base_blocks = int((total + 255) / 256);
    hipStream_t s = as_stream(stream);
    // enough parallelism for long split lists: G groups of `per` slabs summed first (in place)
    int G = (2048 + base_blocks - 1) / base_blocks;
    if (G > (nsplit + 3) / 4) G = (nsplit + 3) / 4;
    if (G < 1) G = 1;
    int nsum = nsplit, gstride = 1;
    if (G > 1) {
        const int per = (nsplit + G - 1) / G;
        G = (nsplit + per - 1) / per;
        if (total % 4 == 0 && aligned16(slabs))
            hipLaunchKernelGGL(wgrad_group_sum4, dim3(unsigned((total / 4 + 255) / 256), G), dim3(256), 0, s, slabs,
                               nsplit, per, total);
        else
            hipLaunchKernelGGL(wgrad_group_sum, dim3(base_blocks, G), dim3(256), 0, s, slabs, nsplit, per, total);
        nsum = G;
        gstride = per;
    }
    if (ntaps <= kFinMaxTaps) {
        hipLaunchKernelGGL(wgrad_finalize_rows, dim3(R, (C + kFinCB - 1) / kFinCB), dim3(256), 0, s, slabs, nsum,
                           gstride, R, ntaps, C, mode, c_valid, out);
        return launch_status("scd_wgrad_finalize");
    }
    const int blocks = base_blocks > 4096 ? 4096 : base_blocks;
    hipLaunchKernelGGL(wgrad_finalize_kernel, dim3(blocks), dim3(256), 0, s, slabs, nsum, gstride, R, ntaps, C, mode,
                       c_valid, out);
    return launch_status("scd_wgrad_finalize");
}
