// Halo-tiled 3x3 implicit-GEMM convolution on v_mfma_f32_16x16x32_bf16 with the exact split-bf16 ("x3")
// arithmetic of conv_x3.hip.
//
// Why a second halo kernel: on random operands the chip holds a higher clock under the 16x16x32 MFMA than
// under 32x32x16 at equal FLOPs per cycle (MI355X_MICROARCH.md 'DVFS give-back' item 7).  Measured with
// tools/mfma_shape_bench.hip in this loop's shape (A from LDS, B from L2, six split products): 1693 vs
// 1573 TFLOP/s.
//
// Structure (same as igemm_halo_x3, conv_x3.hip):
//   - a block owns a TR x TW patch of output pixels of one image and BN output channels;
//   - per 32-channel chunk it stages the (TR+2) x (TW+2) input halo once, split into its three bf16
//     planes ([row][32 bf16], 64-byte rows), and serves all 9 taps from LDS by shifting the row index;
//   - the pre-split weights (scd_split_bf16x3_frag layout) are loaded straight into registers one step
//     ahead; barriers only at chunk ends.
// Roles: the MFMA A operand is the weights (rows = output channels), B is the pixels.  The 16x16 result
// then holds 4 consecutive channels of one pixel per lane, stored as one 16-byte store.
//
// LDS image: the 16-byte segment s of halo row r sits at r*64 + 16*(s ^ ((r >> 1) & 3)).  A fragment read
// (16 consecutive rows from any start, segment = lane >> 4) is then conflict-free in every ds_read_b128
// lane group (checked exhaustively over row offsets).
#include "x3_common.h"

namespace scd {

// Sum over the 16 lanes of a DPP row; every lane of the row receives the total.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float row16_sum(float x) {
    x += dpp_mov<0x140>(x);  // row_mirror:      i <-> 15 - i
    x += dpp_mov<0x141>(x);  // row_half_mirror: i <-> 7 - i within each half
    x += dpp_mov<0xB1>(x);   // quad_perm [1,0,3,2]
    x += dpp_mov<0x4E>(x);   // quad_perm [2,3,0,1]
    return x;
}

__device__ __forceinline__ void gstore4(float *p, f32x4 v) { *(__attribute__((address_space(1))) f32x4 *)(p) = v; }

// WAVES_M x WAVES_N waves; a wave computes TM*16 pixels x TN*16 channels (TM x TN MFMA tiles).
template <int WAVES_M, int WAVES_N, int TM, int TN, int TW, int OCC>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N, OCC) void igemm_halo16_x3(IgemmArgs a) {
    constexpr int NT = 64 * WAVES_M * WAVES_N;
    constexpr int WPX = TM * 16, WCH = TN * 16;
    constexpr int BM = WAVES_M * WPX, BN = WAVES_N * WCH;
    constexpr int TR = BM / TW;
    constexpr int HWD = TW + 2;
    constexpr int HR = (TR + 2) * HWD;
    constexpr int A_CH = HR * 8;  // 16-byte (4-channel) pieces of one 32-channel chunk
    constexpr int A_PER = (A_CH + NT - 1) / NT;
    constexpr int PA = HR * 64;
    constexpr int RED = 2 * WAVES_M * BN * 4;
    __shared__ __attribute__((aligned(16))) unsigned char smem[3 * PA > RED ? 3 * PA : RED];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wm = wid % WAVES_M;
    const int wn = wid / WAVES_M;
    const int g = lane >> 4, l16 = lane & 15;
    int mt, nt;
    if (a.remap == 2) {  // N slowest: each XCD's blocks share one n-tile of weights (L2-resident)
        const uint32_t L = xcd_swizzle(blockIdx.x, uint32_t(a.grid_m * a.grid_n));
        nt = int(L / uint32_t(a.grid_m));
        mt = int(L - uint32_t(nt) * uint32_t(a.grid_m));
    } else if (a.remap) {
        const uint32_t L = xcd_swizzle(blockIdx.x, uint32_t(a.grid_m * a.grid_n));
        mt = int(L / uint32_t(a.grid_n));
        nt = int(L - uint32_t(mt) * uint32_t(a.grid_n));
    } else {
        mt = int(blockIdx.x % uint32_t(a.grid_m));
        nt = int(blockIdx.x / uint32_t(a.grid_m));
    }
    const int tiles_x = a.wo / TW, tiles_y = a.ho / TR;
    const int img = mt / (tiles_x * tiles_y);
    const int trem = mt - img * tiles_x * tiles_y;
    const int ty = trem / tiles_x;
    const int y0 = ty * TR, x0 = (trem - ty * tiles_x) * TW;
    const int n0 = nt * BN;

    auto soff = [](int row, int col) { return row * 64 + ((((col >> 1) ^ (row >> 1)) & 3) << 4) + ((col & 1) << 3); };

    uint32_t a_boff[A_PER];
    int a_off[A_PER];
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
        const int e = tid + i * NT;
        const bool in = e < A_CH;
        const int hp = in ? (e >> 3) : 0, col = e & 7;
        const int hy = hp / HWD, hx = hp - (hp / HWD) * HWD;
        const int sy = y0 - 1 + hy, sx = x0 - 1 + hx;
        const bool ok = in && unsigned(sy) < unsigned(a.hs) && unsigned(sx) < unsigned(a.ws);
        a_boff[i] = ok ? uint32_t(((img * a.hs + sy) * a.ws + sx) * a.ldc_s + col * 4) * 4u : kOOB;
        a_off[i] = in ? soff(hp, col) : -1;
    }
    // Weight fragments from the 32-row fragment-major split (scd_split_bf16x3_frag): the 16 rows x 8 k of
    // one 16-lane group are 256 contiguous bytes of a 1 KB 32x16 fragment.
    const int KS16 = a.K / 16, NB32 = (a.n_out + 31) / 32;
    const uint32_t wplane_b = uint32_t(a.wplane) * 2u;
    uint32_t w_base[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int cb = (n0 >> 4) + wn * TN + j;  // 16-channel block
        const int nb = cb >> 1;
        w_base[j] = nb < NB32 ? uint32_t(nb * KS16 + (g >> 1)) * 1024u + uint32_t(16 * (cb & 1) + l16 + 32 * (g & 1)) * 16u
                              : kOOB;
    }

    f32x4 ra[A_PER];
    const __amdgpu_buffer_rsrc_t rs_src = make_rsrc(a.src, a.src_bytes);
    const __amdgpu_buffer_rsrc_t rs_w = make_rsrc(a.wsplit, 3u * wplane_b);
    auto load_A = [&](int cc) {
#pragma unroll
        for (int i = 0; i < A_PER; ++i) ra[i] = bload4(rs_src, a_boff[i] == kOOB ? kOOB : a_boff[i] + cc * 128u);
    };
    auto store_A = [&]() {
#pragma unroll
        for (int i = 0; i < A_PER; ++i)
            if ((A_CH % NT == 0) || a_off[i] >= 0) {
                u32x2 h, m, l;
                split3(ra[i], h, m, l);
                *reinterpret_cast<u32x2 *>(smem + a_off[i]) = h;
                *reinterpret_cast<u32x2 *>(smem + PA + a_off[i]) = m;
                *reinterpret_cast<u32x2 *>(smem + 2 * PA + a_off[i]) = l;
            }
    };
    const int cpk = a.c / 32;
    auto load_W = [&](int cc, int t, u32x4 (&wq)[3][TN]) {
        const uint32_t ko = uint32_t(t * cpk + cc) * 2048u;  // 32-deep step = two 16-deep fragments
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                wq[p][j] = bload4u(rs_w, w_base[j] == kOOB ? kOOB : w_base[j] + ko + uint32_t(p) * wplane_b);
    };

    f32x4 acc[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

    int a_hr[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int p = wm * WPX + i * 16 + l16;
        a_hr[i] = (p / TW + 1) * HWD + (p % TW) + 1;
    }

    const int nsteps = cpk * a.ntaps;
    u32x4 wq[3][TN];
    load_A(0);
    load_W(0, 0, wq);
    store_A();
    __syncthreads();
    int cc = 0, t = 0;
    for (int s = 0; s < nsteps; ++s) {
        int t1 = t + 1, cc1 = cc;
        if (t1 == a.ntaps) {
            t1 = 0;
            cc1 = cc + 1;
        }
        const bool more = s + 1 < nsteps;
        if (more && t1 == 0) load_A(cc1);
        const int toff = tap_at(a.tdy, t) * HWD + tap_at(a.tdx, t);
        bf16x8 xv[3][TM], wv[3][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int hr = a_hr[i] + toff;
            const int ad = hr * 64 + (((g ^ (hr >> 1)) & 3) << 4);
#pragma unroll
            for (int p = 0; p < 3; ++p)
                xv[p][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4 *>(smem + p * PA + ad));
        }
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int j = 0; j < TN; ++j) wv[p][j] = __builtin_bit_cast(bf16x8, wq[p][j]);
        constexpr int QW[6] = {1, 0, 2, 0, 1, 0};
        constexpr int QX[6] = {1, 2, 0, 1, 0, 0};
#pragma unroll
        for (int q = 0; q < 6; ++q)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[QW[q]][j], xv[QX[q]][i], acc[j][i], 0, 0, 0);
        if (more) load_W(cc1, t1, wq);
        if (more && t1 == 0) {  // chunk end: every wave is done with this halo; overwrite it with the next one
            __syncthreads();
            store_A();
            __syncthreads();
        }
        t = t1;
        cc = cc1;
    }
    __syncthreads();  // the epilogue reuses smem for the statistics reduction

    // acc[j][i][r]: channel n0 + wn*WCH + 16j + 4g + r, pixel wm*WPX + 16i + l16
    f32x4 bias4[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WCH + j * 16 + 4 * g;
        bias4[j] = (a.bias && n < a.n_out) ? *reinterpret_cast<const f32x4 *>(a.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int p = wm * WPX + i * 16 + l16;
        const size_t pix = size_t(img * a.ho + y0 + p / TW) * a.wo + x0 + (p % TW);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * WCH + j * 16 + 4 * g;
            if (n < a.n_out) gstore4(a.dst + pix * a.ldc_d + n, acc[j][i] + bias4[j]);
        }
    }

    // Fused BatchNorm statistics of this tile (BM pixels of one image) per channel: mean, then M2 about it.
    if (a.stat_rec) {
        float *red1 = reinterpret_cast<float *>(smem);  // [WAVES_M][BN] sums
        float *red2 = red1 + WAVES_M * BN;              // [WAVES_M][BN] M2
        float mean[TN][4];
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float s = 0.f;
#pragma unroll
                for (int i = 0; i < TM; ++i) s += acc[j][i][r] + bias4[j][r];
                s = row16_sum(s);
                if (l16 == 0) red1[wm * BN + wn * WCH + j * 16 + 4 * g + r] = s;
            }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int nl = wn * WCH + j * 16 + 4 * g + r;
                float s = 0.f;
#pragma unroll
                for (int w = 0; w < WAVES_M; ++w) s += red1[w * BN + nl];
                mean[j][r] = s * (1.f / float(BM));
                float q = 0.f;
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const float d = (acc[j][i][r] + bias4[j][r]) - mean[j][r];
                    q = fmaf(d, d, q);
                }
                q = row16_sum(q);
                if (l16 == 0) red2[wm * BN + nl] = q;
            }
        __syncthreads();
        for (int nl = tid; nl < BN; nl += NT) {
            if (n0 + nl >= a.n_out) continue;
            float s = 0.f, m2 = 0.f;
#pragma unroll
            for (int w = 0; w < WAVES_M; ++w) {
                s += red1[w * BN + nl];
                m2 += red2[w * BN + nl];
            }
            float *rec = a.stat_rec + (size_t(mt) * a.n_out + n0 + nl) * 2;
            rec[0] = s * (1.f / float(BM));
            rec[1] = m2;
        }
    }
}

namespace {

struct H16Cfg {
    int id, bm, bn;
};

// 0 = off, 1 = automatic tile choice, 2 + id = force tile config id (scd_set_halo16; initial value from
// SCD_HALO16=0 and SCD_HALO16_CFG=<id>).
int g_halo16 = -2;
int halo16_mode() {
    if (g_halo16 == -2) {
        const char *e = getenv("SCD_HALO16");
        g_halo16 = (e && e[0] == '0') ? 0 : 1;
        const char *c = getenv("SCD_HALO16_CFG");
        if (g_halo16 && c) g_halo16 = 2 + atoi(c);
    }
    return g_halo16;
}

template <int WM, int WN, int TM, int TN, int OCC>
void launch16(const IgemmArgs &a, int tw, hipStream_t s) {
    constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
    IgemmArgs b = a;
    b.grid_m = a.n_img * (a.ho / (BM / tw)) * (a.wo / tw);
    b.grid_n = (a.n_out + BN - 1) / BN;
    b.remap = xcd_remap_enabled();
    {
        const char *o = getenv("SCD_HALO_ORDER");
        if (b.remap && !(o && o[0] == 'm')) b.remap = 2;
    }
    const dim3 grid(b.grid_m * b.grid_n), block(64 * WM * WN);
    if (tw == 64)
        hipLaunchKernelGGL((igemm_halo16_x3<WM, WN, TM, TN, 64, OCC>), grid, block, 0, s, b);
    else if (tw == 32)
        hipLaunchKernelGGL((igemm_halo16_x3<WM, WN, TM, TN, 32, OCC>), grid, block, 0, s, b);
    else
        hipLaunchKernelGGL((igemm_halo16_x3<WM, WN, TM, TN, 16, OCC>), grid, block, 0, s, b);
}

// Tile configurations: id -> (pixels, channels) per block.
//   0: 2x2 waves of 64 px x 64 ch  (128 x 128), 2 waves/SIMD
//   1: 2x2 waves of 64 px x 32 ch  (128 x 64),  3 waves/SIMD
//   2: 2x2 waves of 32 px x 64 ch  (64 x 128),  3 waves/SIMD
constexpr H16Cfg kCfg[] = {{0, 128, 128}, {1, 128, 64}, {2, 64, 128}};

}  // namespace

// 0 when `a` does not take this kernel, else 1 + config id; *bm = pixels per tile, *tw = tile width.
int halo16_pick(const IgemmArgs &a, bool eligible, int *bm, int *tw) {
    const int mode = halo16_mode();
    if (!mode || !eligible || a.c % 32 || a.n_out % 4 || a.ldc_d % 4 || (reinterpret_cast<uintptr_t>(a.dst) & 15) ||
        (a.bias && (reinterpret_cast<uintptr_t>(a.bias) & 15)))
        return 0;
    int id;
    if (mode >= 2)
        id = mode - 2;
    else if (a.n_out >= 128)
        id = 0;  // 128 x 128 at 2 waves/SIMD: +4..17% over the 32x32x16 halo kernel on the 128..512-channel layers
    else if (a.n_out >= 64)
        id = 1;  // 128 x 64 at 3 waves/SIMD: +3..9% on the 64-channel layers
    else
        return 0;
    if (id < 0 || id > 2) return 0;
    *bm = kCfg[id].bm;
    for (int cand : {64, 32, 16})
        if (a.wo % cand == 0 && a.ho % (*bm / cand) == 0 && *bm / cand >= 1 && *bm % cand == 0) {
            *tw = cand;
            return 1 + id;
        }
    return 0;
}

void launch_halo16(const IgemmArgs &a, int cfg, int tw, hipStream_t s) {
    switch (cfg - 1) {
        case 0: launch16<2, 2, 4, 4, 2>(a, tw, s); break;
        case 1: launch16<2, 2, 4, 2, 3>(a, tw, s); break;
        default: launch16<2, 2, 2, 4, 3>(a, tw, s); break;
    }
}

}  // namespace scd

using namespace scd;

extern "C" int scd_set_halo16(int32_t mode) {
    clear_error();
    const int prev = scd::halo16_mode();
    if (mode >= 0 && mode <= 4) {
        scd::g_halo16 = mode;
    } else if (mode != -1) {
        set_error("scd_set_halo16: mode %d", mode);
        return SCD_ERR_ARG;
    }
    return prev;
}
