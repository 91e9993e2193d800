// Implicit-GEMM convolution on gfx950 bf16 MFMA with exact three-way operand splitting ("x3").
//
// Every fp32 operand x is split into three bf16 terms, each rounded to nearest:
//   h = bf16(x), m = bf16(x - h), l = bf16(x - h - m).
// The subtractions are exact in fp32, so h + m + l reproduces x to within 2^-27 |x|.
//
// A product of two split operands is accumulated from the six terms whose magnitudes reach fp32's
// precision: hh + hm + mh + mm + hl + lh.  The dropped terms ml, lm, ll are at most ~2^-26 relative.
// Each bf16 x bf16 product is exact in the fp32 accumulator.  The result is therefore an fp32 GEMM with
// a rounding error of the same order as the fp32-MFMA kernel (conv_f32.hip); it differs only in
// summation order.
//
// Cost: 6 x v_mfma_f32_32x32x16_bf16 (32 cycles each) per 16-deep k step of a 32x32 tile, against
// 8 x v_mfma_f32_32x32x2_f32 (64 cycles each), i.e. 2.67x less matrix-core time per FLOP.
//
// Same GEMM view as igemm_f32: out[m, o] = bias + sum_k A[m, k] * Wpk[o, k], where A is gathered on the
// fly from an NHWC source and k = (tap, c).  This kernel requires c % 16 == 0, so a 16-deep k step never
// straddles two taps.
//
// LDS image: per stage and per operand, three planes (h, m, l) of [row][16 bf16] with 32-byte rows.  The
// 16-byte half of a row is XOR-swizzled with row bit 3, which makes the ds_read_b128 operand reads
// conflict-free; see the bank analysis in DESIGN.md.
#include <algorithm>

#include "x3_common.h"

namespace scd {

// PRE: B (weights) come pre-split in a.wsplit planes and are staged by copy (8 k per chunk, 3 x 16 B).
template <int WAVES_M, int WAVES_N, int TM, int TN, bool PRE>
__global__ __launch_bounds__(64 * WAVES_M *WAVES_N) void igemm_x3(IgemmArgs a) {
    constexpr int BK = 16;
    constexpr int NT = 64 * WAVES_M * WAVES_N;
    constexpr int BM = WAVES_M * TM * 32;
    constexpr int BN = WAVES_N * TN * 32;
    constexpr int ROWS = BM + BN;
    constexpr int KC = BK / 4;            // 4-float chunks per row and stage
    constexpr int A_CH = BM * KC;
    constexpr int B_CH = PRE ? BN * 2 : BN * KC;  // PRE: 8-k chunks
    constexpr int A_PER = (A_CH + NT - 1) / NT;
    constexpr int B_PER = (B_CH + NT - 1) / NT;
    constexpr int PLANE = ROWS * 32;      // bytes of one plane: ROWS x 16 bf16
    constexpr int STAGE = 3 * PLANE;
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wm = wid % WAVES_M;
    const int wn = wid / WAVES_M;
    int mt, nt;
    if (a.remap) {
        const uint32_t L = xcd_swizzle(blockIdx.x, uint32_t(a.grid_m * a.grid_n));
        mt = int(L / uint32_t(a.grid_n));
        nt = int(L - uint32_t(mt) * uint32_t(a.grid_n));
    } else {
        mt = int(blockIdx.x % uint32_t(a.grid_m));
        nt = int(blockIdx.x / uint32_t(a.grid_m));
    }
    const int m0 = mt * BM;
    const int n0 = nt * BN;

    // byte offset of (row, 4-float chunk col) inside a plane: 32-byte rows, 16-byte half swizzled by row bit 3
    auto soff = [](int row, int col) { return row * 32 + ((((col >> 1) ^ (row >> 3)) & 1) << 4) + ((col & 1) << 3); };

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
        a_sy[i] = ok ? int(oy) * a.stride : -(1 << 20);
        a_sx[i] = int(ox) * a.stride;
        a_base[i] = a.src + (size_t(int(img) * a.hs + a_sy[i] * ok) * a.ws + a_sx[i]) * a.ldc_s + col * 4;
        a_off[i] = soff(row, col);
    }
    int b_row[B_PER], b_off[B_PER];
    bool b_ok[B_PER], b_in[B_PER];
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
        const int ch = tid + i * NT;
        const int row = ch / KC, col = ch % KC;
        b_in[i] = ch < B_CH;
        b_ok[i] = b_in[i] && (n0 + row < a.n_out);
        if (PRE) {  // fragment-major pre-split weights: the 16-byte piece (n, 8 k) sits in lane (n&31) + 32*half
            const int r8 = ch >> 1, half = ch & 1;
            const int n = n0 + r8;
            b_ok[i] = b_in[i] && (n < a.n_out);
            b_row[i] = ((n >> 5) * (a.K / 16)) * 512 + ((n & 31) + 32 * half) * 8;
            b_off[i] = (BM + r8) * 32 + (((half ^ ((BM + r8) >> 3)) & 1) << 4);
        } else {
            b_row[i] = (n0 + row) * a.K + col * 4;
            b_off[i] = soff(BM + row, col);
        }
    }

    f32x4 ra[A_PER], rb[B_PER];
    u32x4 pb[B_PER][3];
    const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};

    auto load_stage = [&](int t, int c0) {
        const int dyt = tap_at(a.tdy, t), dxt = tap_at(a.tdx, t);
        const long toff = long(dyt * a.ws + dxt) * a.ldc_s + c0;
#pragma unroll
        for (int i = 0; i < A_PER; ++i) {
            const bool v = unsigned(a_sy[i] + dyt) < unsigned(a.hs) && unsigned(a_sx[i] + dxt) < unsigned(a.ws);
            ra[i] = v ? gload4(a_base[i] + toff) : zero4;
        }
        const int k0 = t * a.c + c0;
        if (PRE) {
            const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int i = 0; i < B_PER; ++i)
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    pb[i][p] = b_ok[i] ? *(const __attribute__((address_space(1))) u32x4 *)(a.wsplit + p * a.wplane +
                                                                                          size_t(b_row[i]) + (k0 / 16) * 512)
                                       : z;
        } else {
#pragma unroll
            for (int i = 0; i < B_PER; ++i) rb[i] = b_ok[i] ? gload4(a.w + size_t(b_row[i]) + k0) : zero4;
        }
    };
    auto store_stage = [&](int buf) {
        unsigned char *S = smem + buf * STAGE;
#pragma unroll
        for (int i = 0; i < A_PER; ++i)
            if (tid + i * NT < A_CH) {
                u32x2 h, m, l;
                split3(ra[i], h, m, l);
                *reinterpret_cast<u32x2 *>(S + a_off[i]) = h;
                *reinterpret_cast<u32x2 *>(S + PLANE + a_off[i]) = m;
                *reinterpret_cast<u32x2 *>(S + 2 * PLANE + a_off[i]) = l;
            }
        if (PRE) {
#pragma unroll
            for (int i = 0; i < B_PER; ++i)
                if (b_in[i]) {
#pragma unroll
                    for (int p = 0; p < 3; ++p) *reinterpret_cast<u32x4 *>(S + p * PLANE + b_off[i]) = pb[i][p];
                }
            return;
        }
#pragma unroll
        for (int i = 0; i < B_PER; ++i)
            if (b_in[i]) {
                u32x2 h, m, l;
                split3(rb[i], h, m, l);
                *reinterpret_cast<u32x2 *>(S + b_off[i]) = h;
                *reinterpret_cast<u32x2 *>(S + PLANE + b_off[i]) = m;
                *reinterpret_cast<u32x2 *>(S + 2 * PLANE + b_off[i]) = l;
            }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // operand reads: lane (r = lane&31, h = lane>>5) takes row r, k = 8h..8h+7 -> 16-byte half h of the row
    const int h = lane >> 5;
    int a_rd[TM], b_rd[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int row = wm * TM * 32 + i * 32 + (lane & 31);
        a_rd[i] = row * 32 + (((h ^ (row >> 3)) & 1) << 4);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int row = BM + wn * TN * 32 + j * 32 + (lane & 31);
        b_rd[j] = row * 32 + (((h ^ (row >> 3)) & 1) << 4);
    }

    const int csteps = a.c / BK;
    const int nsteps = a.ntaps * csteps;
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
        const unsigned char *S = smem + (s & 1) * STAGE;
        bf16x8 av[3][TM], bv[3][TN];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
                av[p][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4 *>(S + p * PLANE + a_rd[i]));
#pragma unroll
            for (int j = 0; j < TN; ++j)
                bv[p][j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4 *>(S + p * PLANE + b_rd[j]));
        }
        // small terms first: mm, hl, lh, hm, mh, hh
        constexpr int PA[6] = {1, 0, 2, 0, 1, 0};
        constexpr int PB[6] = {1, 2, 0, 1, 0, 0};
#pragma unroll
        for (int q = 0; q < 6; ++q)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[PA[q]][i], bv[PB[q]][j], acc[i][j], 0, 0, 0);
        if (more) store_stage((s + 1) & 1);
        __syncthreads();
    }

    float omax = 0.f;  // max |stored value| of this lane (dst_bound)
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
            for (int i = 0; i < TM; ++i) {
                // (img, oy, ox) of the tile's first row once; the 16 rows of a lane are at offsets < 32, walked
                // by carrying ox into oy (and oy into img) instead of two divisions per element
                const int mb = m0 + wm * TM * 32 + i * 32 + 4 * (lane >> 5);
                const uint32_t ib = fdiv(uint32_t(mb), a.div_hw);
                const uint32_t rb = uint32_t(mb) - ib * uint32_t(a.ho * a.wo);
                const uint32_t yb = fdiv(rb, a.div_w);
                const int img0 = int(ib), oy0 = int(yb), ox0 = int(rb - yb * uint32_t(a.wo));
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int d = (r & 3) + 8 * (r >> 2);
                    if (mb + d >= a.M) continue;
                    int ox = ox0 + d, oy = oy0, img = img0;
                    while (ox >= a.wo) {
                        ox -= a.wo;
                        if (++oy == a.ho) {
                            oy = 0;
                            ++img;
                        }
                    }
                    const size_t pix = size_t(img * a.dst_h + 2 * oy + di) * a.dst_w + 2 * ox + dj;
                    const float v = acc[i][j][r] + bias;
                    gstore1(a.dst + pix * a.ldc_d + oc, v);
                    omax = fmaxf(omax, fabsf(v));
                }
            }
        }
    }
    if (a.dst_bound) wave_max_bound(a.dst_bound, fmaxf(omax, bound_seed(a)));  // uniform: every lane of the wave takes part
}

template <int WM, int WN, int TM, int TN>
static void launch_x3(const IgemmArgs &a, hipStream_t s) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    IgemmArgs b = a;
    b.grid_m = (a.M + BM - 1) / BM;
    b.grid_n = (a.n_out + BN - 1) / BN;
    b.remap = xcd_remap_enabled(a.tune);
    const dim3 grid(b.grid_m * b.grid_n), block(64 * WM * WN);
    if (a.wsplit)
        hipLaunchKernelGGL((igemm_x3<WM, WN, TM, TN, true>), grid, block, 0, s, b);
    else
        hipLaunchKernelGGL((igemm_x3<WM, WN, TM, TN, false>), grid, block, 0, s, b);
}

// ------------------------------------------------------------------------------------------------
// Halo-tiled 3x3 igemm (stride 1, "same" padding).  A block owns a TR x TW patch of output pixels of one
// image and BN output channels.  For every 16-channel chunk it stages the (TR+2) x (TW+2) input halo
// once, split into its three bf16 planes, and serves all 9 taps from LDS by shifting the row index.  The
// per-tap path above re-loads and re-splits every input element 9 times.
// B (pre-split weight planes) is streamed per (chunk, tap), double-buffered.  A is single-buffered: the
// next chunk's halo is loaded into registers at tap 0 and written behind an extra barrier after tap 8.
// ------------------------------------------------------------------------------------------------
template <int WAVES_M, int WAVES_N, int TM, int TN, int TW>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N, 3) void igemm_halo_x3(IgemmArgs a) {
    constexpr int NT = 64 * WAVES_M * WAVES_N;
    constexpr int BM = WAVES_M * TM * 32;
    constexpr int BN = WAVES_N * TN * 32;
    constexpr int TR = BM / TW;
    constexpr int HWD = TW + 2;
    constexpr int HR = (TR + 2) * HWD;
    constexpr int A_CH = HR * 4;
    constexpr int A_PER = (A_CH + NT - 1) / NT;
    constexpr int PA = HR * 32;
    __shared__ __attribute__((aligned(16))) unsigned char smem[3 * PA > 2 * WAVES_M * BN * 4 ? 3 * PA : 2 * WAVES_M * BN * 4];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wm = wid % WAVES_M;
    const int wn = wid / WAVES_M;
    int mt, nt;
    if (a.remap == 2) {  // N slowest: each XCD's blocks share one n-tile of weights (L2-resident)
        const uint32_t L = xcd_swizzle(blockIdx.x, uint32_t(a.grid_m * a.grid_n));
        nt = int(L / uint32_t(a.grid_m));
        mt = int(L - uint32_t(nt) * uint32_t(a.grid_m));
    } else if (a.remap) {  // N fastest: each XCD's blocks share input halos
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

    auto soff = [](int row, int col) { return row * 32 + ((((col >> 1) ^ (row >> 3)) & 1) << 4) + ((col & 1) << 3); };

    uint32_t a_boff[A_PER];  // byte offset of the chunk's source (kOOB when outside the image: reads 0)
    int a_off[A_PER];
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
        const int e = tid + i * NT;
        const bool in = e < A_CH;
        const int hp = in ? (e >> 2) : 0, col = e & 3;
        const int hy = hp / HWD, hx = hp - (hp / HWD) * HWD;
        const int sy = y0 - 1 + hy, sx = x0 - 1 + hx;
        const bool ok = in && unsigned(sy) < unsigned(a.hs) && unsigned(sx) < unsigned(a.ws);
        a_boff[i] = ok ? uint32_t(((img * a.hs + sy) * a.ws + sx) * a.ldc_s + col * 4) * 4u : kOOB;
        a_off[i] = in ? soff(hp, col) : -1;
    }
    // B fragments straight from the fragment-major pre-split weights into registers: fragment (plane p,
    // 32-row block nb, k step ks) of this wave's tile j is 1 KB at ((p*NB + nb)*KS + ks)*1024 + lane*16.
    const int KS = a.K / 16, NB = (a.n_out + 31) / 32;
    const uint32_t wplane_b = uint32_t(a.wplane) * 2u;
    uint32_t b_base[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int nb = (n0 >> 5) + wn * TN + j;
        b_base[j] = nb < NB ? uint32_t(nb * KS) * 1024u + uint32_t(lane) * 16u : kOOB;
    }

    f32x4 ra[A_PER];
    const __amdgpu_buffer_rsrc_t rs_src = make_rsrc(a.src, a.src_bytes);
    const __amdgpu_buffer_rsrc_t rs_w = make_rsrc(a.wsplit, 3u * wplane_b);
    auto load_A = [&](int cc) {
#pragma unroll
        for (int i = 0; i < A_PER; ++i) ra[i] = bload4(rs_src, a_boff[i] == kOOB ? kOOB : a_boff[i] + cc * 64u);
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
    auto load_B = [&](int cc, int t, u32x4 (&bq)[3][TN]) {
        const uint32_t ko = uint32_t(t * (a.c / 16) + cc) * 1024u;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                bq[p][j] = bload4u(rs_w, b_base[j] == kOOB ? kOOB : b_base[j] + ko + uint32_t(p) * wplane_b);
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int h = lane >> 5;
    int a_hr[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int p = wm * TM * 32 + i * 32 + (lane & 31);
        a_hr[i] = (p / TW + 1) * HWD + (p % TW) + 1;
    }

    const int nc = a.c / 16;
    const int nsteps = nc * a.ntaps;
    u32x4 bq[3][TN];
    load_A(0);
    load_B(0, 0, bq);
    store_A();
    __syncthreads();
    int cc = 0, t = 0;
    // B(s) in registers; B(s+1) is loaded into the same registers once the step's MFMAs are issued (they
    // still execute for several hundred cycles, hiding most of the latency).  One B register set keeps the
    // kernel at 3 waves per SIMD.  Barriers only at 16-channel chunk ends (halo rewrite).
    for (int s = 0; s < nsteps; ++s) {
        int t1 = t + 1, cc1 = cc;
        if (t1 == a.ntaps) {
            t1 = 0;
            cc1 = cc + 1;
        }
        const bool more = s + 1 < nsteps;
        if (more && t1 == 0) load_A(cc1);
        const int toff = tap_at(a.tdy, t) * HWD + tap_at(a.tdx, t);
        bf16x8 av[3][TM], bv[3][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int hr = a_hr[i] + toff;
            const int ad = hr * 32 + (((h ^ (hr >> 3)) & 1) << 4);
#pragma unroll
            for (int p = 0; p < 3; ++p)
                av[p][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4 *>(smem + p * PA + ad));
        }
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int j = 0; j < TN; ++j) bv[p][j] = __builtin_bit_cast(bf16x8, bq[p][j]);
        constexpr int QA[6] = {1, 0, 2, 0, 1, 0};
        constexpr int QB[6] = {1, 2, 0, 1, 0, 0};
#pragma unroll
        for (int q = 0; q < 6; ++q)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[QA[q]][i], bv[QB[q]][j], acc[i][j], 0, 0, 0);
        if (more) load_B(cc1, t1, bq);
        if (more && t1 == 0) {  // chunk end: every wave is done with this halo; overwrite it with the next one
            __syncthreads();
            store_A();
            __syncthreads();
        }
        t = t1;
        cc = cc1;
    }
    __syncthreads();  // the epilogue reuses smem for the statistics reduction

#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * TN * 32 + j * 32 + (lane & 31);
        if (n >= a.n_out) continue;
        const float bias = a.bias ? a.bias[n] : 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int p = wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                const size_t pix = size_t(img * a.ho + y0 + p / TW) * a.wo + x0 + (p % TW);
                gstore1(a.dst + pix * a.ldc_d + n, acc[i][j][r] + bias);
            }
    }

    // Fused BatchNorm statistics of this tile (BM pixels of one image) per channel: two passes over the
    // stored values (mean, then M2 about it), lane halves combined by shuffle, waves through LDS.
    if (a.stat_rec) {
        float *red = reinterpret_cast<float *>(smem);  // [WAVES_M][BN]; the main loop ended on a barrier
        float bias_j[TN], mean_j[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int nl = wn * TN * 32 + j * 32 + (lane & 31);
            bias_j[j] = (a.bias && n0 + nl < a.n_out) ? a.bias[n0 + nl] : 0.f;
            float sum = 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) sum += acc[i][j][r] + bias_j[j];
            sum += __shfl_xor(sum, 32);
            if (lane < 32) red[wm * BN + nl] = sum;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int nl = wn * TN * 32 + j * 32 + (lane & 31);
            float t = 0.f;
#pragma unroll
            for (int w = 0; w < WAVES_M; ++w) t += red[w * BN + nl];
            mean_j[j] = t * (1.f / float(BM));
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int nl = wn * TN * 32 + j * 32 + (lane & 31);
            float q = 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float d = (acc[i][j][r] + bias_j[j]) - mean_j[j];
                    q = fmaf(d, d, q);
                }
            q += __shfl_xor(q, 32);
            if (lane < 32) red[wm * BN + nl] = q;
        }
        __syncthreads();
        if (wm == 0 && lane < 32) {
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int nl = wn * TN * 32 + j * 32 + lane;
                if (n0 + nl >= a.n_out) continue;
                float m2 = 0.f;
#pragma unroll
                for (int w = 0; w < WAVES_M; ++w) m2 += red[w * BN + nl];
                float *rec = a.stat_rec + (size_t(mt) * a.n_out + n0 + nl) * 2;
                rec[0] = mean_j[j];
                rec[1] = m2;
            }
        }
    }
}

template <int WM, int WN, int TM, int TN>
static void launch_halo(const IgemmArgs &a, int tw, hipStream_t s) {
    constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
    IgemmArgs b = a;
    b.grid_m = a.n_img * (a.ho / (BM / tw)) * (a.wo / tw);
    b.grid_n = (a.n_out + BN - 1) / BN;
    // N-slowest XCD order by default (keeps one n-tile of weights per XCD L2: -4..13% on the 512/1024-channel
    // layers, neutral elsewhere); SCD_TUNE_HALO_ORDER_M selects the N-fastest order.
    b.remap = halo_remap(a.tune);
    const dim3 grid(b.grid_m * b.grid_n), block(64 * WM * WN);
    if (tw == 64)
        hipLaunchKernelGGL((igemm_halo_x3<WM, WN, TM, TN, 64>), grid, block, 0, s, b);
    else if (tw == 32)
        hipLaunchKernelGGL((igemm_halo_x3<WM, WN, TM, TN, 32>), grid, block, 0, s, b);
    else
        hipLaunchKernelGGL((igemm_halo_x3<WM, WN, TM, TN, 16>), grid, block, 0, s, b);
}

// 3x3 / stride 1 / same-size convs with pre-split weights take the halo path.
static bool halo_eligible(const IgemmArgs &a) {
    if (!a.wsplit || !a.src_bytes || a.store_mode != 0 || a.stride != 1 || a.ntaps != 9 || a.ho != a.hs ||
        a.wo != a.ws || 3 * a.wplane * 2 >= (int64_t(1) << 31))
        return false;
    for (int t = 0; t < 9; ++t) {
        const int dy = int((a.tdy >> (4 * t)) & 15ull), dx = int((a.tdx >> (4 * t)) & 15ull);
        const int sdy = dy >= 8 ? dy - 16 : dy, sdx = dx >= 8 ? dx - 16 : dx;
        if (sdy < -1 || sdy > 1 || sdx < -1 || sdx > 1) return false;
    }
    return halo_enabled(a.tune);
}

// Halo configuration of `a`: 0 = not eligible, 1 = <2,2,2,2> (128 px x 128), 2 = <4,1,2,2> (256 x 64),
// 3 = <4,1,2,1> (256 x 32); *bm = pixels per tile, *tw = tile width (tile = bm/tw rows of one image).
static int halo_pick(const IgemmArgs &a, int *bm, int *tw) {
    if (a.c % 16 || !halo_eligible(a)) return 0;
    const int cfg = a.n_out >= 128 ? 1 : (a.n_out >= 64 ? 2 : 3);
    *bm = cfg == 1 ? 128 : 256;
    for (int cand : {64, 32, 16})
        if (a.wo % cand == 0 && a.ho % (*bm / cand) == 0) {
            *tw = cand;
            return cfg;
        }
    return 0;
}

// SCD_MATH_H2: a conv whose weight split is in the h2 format runs the h2 halo16 kernel (3x3) or the h2 gather16
// kernel (ConvTranspose forward / data grad) when the descriptor bounds its source and the kernel takes the shape;
// otherwise the x3 kernels split the fp32 weights on the fly (the h2 split is ignored).
static IgemmArgs x3_view(const IgemmArgs &a) {
    IgemmArgs b = a;
    int bm = 0, tw = 0;
    const bool h2_kernel = a.ntaps != 9 ? gather16_pick(a) != 0
                           : a.c == 16 ? halo16_c16_pick(a, halo_eligible(a), &bm, &tw) != 0
                                       : halo16_pick(a, halo_eligible(a), &bm, &tw) != 0;
    if (h2_weight_format(a.math, a.ntaps, a.c) && (!a.src_bound || !h2_kernel)) b.wsplit = nullptr;
    return b;
}

bool igemm_takes_gather16(const IgemmArgs &a) { return math_split(a.math) && a.c % 16 == 0 && gather16_pick(a) != 0; }

bool igemm_takes_halo16(const IgemmArgs &a0) {
    int bm = 0, tw = 0;
    const IgemmArgs a = x3_view(a0);
    return math_split(a.math) && a.c % 16 == 0 && halo16_pick(a, halo_eligible(a), &bm, &tw) != 0;
}

bool igemm_takes_c16(const IgemmArgs &a0) {
    int bm = 0, tw = 0;
    const IgemmArgs a = x3_view(a0);
    return math_split(a.math) && halo16_c16_pick(a, halo_eligible(a), &bm, &tw) != 0;
}

int halo_stat_tiles(const IgemmArgs &a0, int *tile_pixels) {
    int bm = 0, tw = 0;
    const IgemmArgs a = x3_view(a0);
    if (!math_split(a.math)) return 0;
    if (!halo16_pick(a, halo_eligible(a), &bm, &tw) && !halo16_c16_pick(a, halo_eligible(a), &bm, &tw) &&
        (a.sb || !halo_pick(a, &bm, &tw)))
        return 0;
    *tile_pixels = bm;
    return a.n_img * (a.ho * a.wo / bm);
}

bool launch_igemm_x3(const IgemmArgs &a0, hipStream_t s) {
    if (a0.c % 16) return false;
    const IgemmArgs a = x3_view(a0);
    int bm = 0, tw = 0;
    if (const int c16 = halo16_pick(a, halo_eligible(a), &bm, &tw)) {
        launch_halo16(a, c16, tw, s);
        return true;
    }
    if (const int g16 = gather16_pick(a)) {
        launch_gather16(a, g16, s);
        return true;
    }
    if (halo16_c16_pick(a, halo_eligible(a), &bm, &tw)) {
        launch_halo16_c16(a, tw, s);
        return true;
    }
    if (a.sb) return false;  // bf16 storage: only the bf16 kernels above (the caller reports the unsupported shape)
    switch (halo_pick(a, &bm, &tw)) {
        case 1: launch_halo<2, 2, 2, 2>(a, tw, s); return true;
        case 2: launch_halo<4, 1, 2, 2>(a, tw, s); return true;
        case 3: launch_halo<4, 1, 2, 1>(a, tw, s); return true;
        default: break;
    }
    // SCD_TUNE_X3_TILE (tile study, tools/perf_convT.py): 1 128x128, 2 256x64, 3 256x32, 4 128x64, 5 256x128
    switch ((a.tune & SCD_TUNE_X3_TILE_MASK) >> 12) {
        case 1: launch_x3<2, 2, 2, 2>(a, s); return true;
        case 2: launch_x3<4, 1, 2, 2>(a, s); return true;
        case 3: launch_x3<4, 1, 2, 1>(a, s); return true;
        case 4: launch_x3<2, 2, 2, 1>(a, s); return true;
        case 5: launch_x3<4, 2, 2, 2>(a, s); return true;
        default: break;
    }
    if (a.n_out >= 128)
        launch_x3<2, 2, 2, 2>(a, s);  // 128 x 128
    else if (a.n_out >= 64)
        launch_x3<2, 2, 2, 1>(a, s);  // 128 x 64 (tools/perf_convT.py: up1 ConvT data grad 177 -> 155 us vs 256 x 64)
    else
        launch_x3<4, 1, 2, 1>(a, s);  // 256 x 32
    return true;
}

// ------------------------------------------------------------------------------------------------
// Weight gradient, split-K over pixels (same decomposition as wgrad_f32):
//   slab[s][r][j] = sum_{m in split s} P[m, r] * Q[src(m, t), c],  j = (t, c)
// Both MFMA operands need 8 consecutive pixels (k) per lane, but global memory is pixel-major.  The
// stage is therefore written as it arrives, as [16 px][W ch] bf16 planes, and each fragment is read
// with two ds_read_b64_tr_b16 (hardware 4x16 transpose).
// Row stride = 2W bytes padded to = 64 (mod 128), so the 4 rows a 16-lane group reads fall in four
// different 64-byte bank groups: conflict-free per 32-lane half.
// ------------------------------------------------------------------------------------------------
// [16 px][W ch] bf16 plane addressing for the transposed reads.  W % 128 == 0: unpadded 2W-byte rows with the
// 64-byte segments of each 256-byte bank row XOR-permuted by (k & 3), so the 4 rows a 16-lane group reads
// land in 4 different segments (conflict-free, and 25% less LDS than padding -> one more workgroup per CU).
// Other widths: rows padded to tr_stride.
template <int W>
struct TrPlane {
    static constexpr bool XOR = (W % 128) == 0;
    static constexpr int RS = XOR ? 2 * W : tr_stride(W);
    static constexpr int BYTES = 16 * RS;
    __device__ static __forceinline__ int off(int k, int colbyte) {
        return XOR ? k * RS + (colbyte ^ ((k & 3) << 6)) : k * RS + colbyte;
    }
};

// NP = 4: the h2 arithmetic (x3_common.h) for convs outside the halo kernels (the ConvTranspose weight grad): both
// operands scaled by the powers of two of *rows_bound / *src_bound and split into fp16 h and pre-scaled m' planes,
// three v_mfma_f32_32x32x16_f16 products (a_h 2^-11) b_m' + a_m' (b_h 2^-11) + a_h b_h, scales undone in the
// epilogue.  NP = 1: bf16 (the ConvTranspose weight grad of the bf16 configs), both operands rounded to bf16 (RNE),
// one v_mfma_f32_32x32x16_bf16 product.
// SB: bf16 storage of rows and src (the bf16 configs' ConvTranspose weight grad; bf16 arithmetic only).
template <int WAVES_M, int WAVES_N, int TM, int TN, int NP = 3, bool SB = false>
__global__ __launch_bounds__(64 * WAVES_M *WAVES_N) void wgrad_x3(WgradArgs a) {
    static_assert(NP == 1 || NP == 3 || NP == 4, "bf16, x3 or h2");
    static_assert(!SB || NP == 1, "bf16 storage runs the bf16 arithmetic");
    constexpr uint32_t EB = SB ? 2u : 4u;
    constexpr bool H2 = NP == 4;
    constexpr int NPL = H2 ? 2 : NP == 1 ? 1 : 3;  // planes per operand
    constexpr int BK = 16;
    constexpr int NT = 64 * WAVES_M * WAVES_N;
    constexpr int BM = WAVES_M * TM * 32;
    constexpr int BN = WAVES_N * TN * 32;
    constexpr int AQ = BM / 4, BQ = BN / 4;
    constexpr int A_CH = BK * AQ, B_CH = BK * BQ;
    constexpr int A_PER = (A_CH + NT - 1) / NT;
    constexpr int B_PER = (B_CH + NT - 1) / NT;
    constexpr bool A_FULL = A_CH % NT == 0, B_FULL = B_CH % NT == 0;
    using LA = TrPlane<BM>;
    using LB = TrPlane<BN>;
    constexpr int PA = LA::BYTES, PB = LB::BYTES;  // plane bytes
    constexpr int STAGE = NPL * (PA + PB);
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE];
    float rsc = 1.f, rsc_inv = 1.f, ssc = 1.f, ssc_inv = 1.f;  // h2 operand scales
    if constexpr (H2) {
        h2_scale(*a.rows_bound, rsc, rsc_inv);
        h2_scale(*a.src_bound, ssc, ssc_inv);
    }

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wm = wid % WAVES_M;
    const int wn = wid / WAVES_M;
    const uint32_t per_split = uint32_t(a.grid_r * a.grid_j);
    const uint32_t L = a.remap ? xcd_swizzle(blockIdx.x, gridDim.x) : blockIdx.x;
    const int split = int(L / per_split);
    const int rem = int(L - uint32_t(split) * per_split);
    const int jt = rem / a.grid_r;
    const int r0 = (rem - jt * a.grid_r) * BM;
    const int j0 = jt * BN;
    const int kbeg = split * a.kchunk;
    const int kend = min(a.M, kbeg + a.kchunk);

    int a_k[A_PER], a_r[A_PER], a_off[A_PER];
    bool a_in[A_PER], a_ok[A_PER];
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
        const int ch = tid + i * NT;
        a_in[i] = ch < A_CH;
        a_k[i] = ch / AQ;
        const int q = ch % AQ;
        a_r[i] = r0 + q * 4;
        a_ok[i] = a_in[i] && a_r[i] < a.R;
        a_off[i] = LA::off(a_k[i], q * 8);
    }
    int b_k[B_PER], b_dy[B_PER], b_dx[B_PER], b_c[B_PER], b_off[B_PER];
    int b_img[B_PER], b_oy[B_PER], b_ox[B_PER];
    bool b_in[B_PER], b_ok[B_PER];
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
        const int ch = tid + i * NT;
        b_in[i] = ch < B_CH;
        b_k[i] = ch / BQ;
        const int q = ch % BQ;
        const int j = j0 + q * 4;
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
        b_off[i] = NPL * PA + LB::off(b_k[i], q * 8);
    }

    StageT<SB> ra[A_PER], rb[B_PER];
    // colsum: the blocks of row tile 0 also sum every src element they stage, per column (as loaded: before the
    // split and the h2 scale), so the ConvTranspose bias grad needs no pass of its own over dOut
    const bool col_sums = a.colsum != nullptr && r0 == 0;
    f32x4 cs[B_PER];
#pragma unroll
    for (int i = 0; i < B_PER; ++i) cs[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const __amdgpu_buffer_rsrc_t rs_rows = make_rsrc(a.rows, a.rows_bytes);
    const __amdgpu_buffer_rsrc_t rs_src = make_rsrc(a.src, a.src_bytes);
    auto load_stage = [&](int kb) {
#pragma unroll
        for (int i = 0; i < A_PER; ++i) {
            const int m = kb + a_k[i];
            ra[i] = bload_q<SB>(rs_rows, (a_ok[i] && m < kend) ? uint32_t(m * a.ldc_r + a_r[i]) * EB : kOOB);
        }
#pragma unroll
        for (int i = 0; i < B_PER; ++i) {
            const int sy = b_oy[i] * a.stride + b_dy[i];
            const int sx = b_ox[i] * a.stride + b_dx[i];
            const bool v = b_ok[i] && (kb + b_k[i] < kend) && unsigned(sy) < unsigned(a.hs) &&
                           unsigned(sx) < unsigned(a.ws);
            rb[i] = bload_q<SB>(rs_src, v ? uint32_t(((b_img[i] * a.hs + sy) * a.ws + sx) * a.ldc_s + b_c[i]) * EB : kOOB);
        }
    };
    auto advance = [&]() {
#pragma unroll
        for (int i = 0; i < B_PER; ++i) {
            b_ox[i] += BK;
            if (b_ox[i] >= a.wo) {  // row wrap (rare: once per wo/16 steps)
                int ox = b_ox[i], oy = b_oy[i], img = b_img[i];
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
        }
    };
    auto store_stage = [&](int buf) {
        unsigned char *S = smem + buf * STAGE;
#pragma unroll
        for (int i = 0; i < A_PER; ++i)
            if (A_FULL || a_in[i]) {
                u32x2 h, m, l;
                if constexpr (H2) {
                    split2h_pre(ra[i] * rsc, h, m);
                } else if constexpr (NP == 1) {
                    h = stage_bits<SB>(ra[i]);
                } else {
                    split3(ra[i], h, m, l);
                    *reinterpret_cast<u32x2 *>(S + 2 * PA + a_off[i]) = l;
                }
                *reinterpret_cast<u32x2 *>(S + a_off[i]) = h;
                if constexpr (NPL > 1) *reinterpret_cast<u32x2 *>(S + PA + a_off[i]) = m;
            }
#pragma unroll
        for (int i = 0; i < B_PER; ++i)
            if (B_FULL || b_in[i]) {
                if (col_sums) cs[i] += stage_f32<SB>(rb[i]);
                u32x2 h, m, l;
                if constexpr (H2) {
                    split2h_pre(rb[i] * ssc, h, m);
                } else if constexpr (NP == 1) {
                    h = stage_bits<SB>(rb[i]);
                } else {
                    split3(rb[i], h, m, l);
                    *reinterpret_cast<u32x2 *>(S + 2 * PB + b_off[i]) = l;
                }
                *reinterpret_cast<u32x2 *>(S + b_off[i]) = h;
                if constexpr (NPL > 1) *reinterpret_cast<u32x2 *>(S + PB + b_off[i]) = m;
            }
    };

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // transposed-read addresses: 16-lane group g reads rows k0 = 8*(g>>1) (+4), columns 16*(g&1) + 4*(w&3)
    const int g = lane >> 4, w = lane & 15;
    const int trk = 8 * (g >> 1) + (w >> 2);
    const int trc = 16 * (g & 1) + 4 * (w & 3);
    int a_rd[TM], a_rd4[TM], b_rd[TN], b_rd4[TN];  // rows trk and trk + 4
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        a_rd[i] = LA::off(trk, (wm * TM * 32 + i * 32 + trc) * 2);
        a_rd4[i] = LA::off(trk + 4, (wm * TM * 32 + i * 32 + trc) * 2);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        b_rd[j] = NPL * PA + LB::off(trk, (wn * TN * 32 + j * 32 + trc) * 2);
        b_rd4[j] = NPL * PA + LB::off(trk + 4, (wn * TN * 32 + j * 32 + trc) * 2);
    }

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
            const unsigned char *S = smem + (s & 1) * STAGE;
            bf16x8 av[NPL][TM], bv[NPL][TN];
#pragma unroll
            for (int p = 0; p < NPL; ++p) {
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const s16x4 lo = lds_tr16(S + p * PA + a_rd[i]);
                    const s16x4 hi = lds_tr16(S + p * PA + a_rd4[i]);
                    av[p][i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const s16x4 lo = lds_tr16(S + p * PB + b_rd[j]);
                    const s16x4 hi = lds_tr16(S + p * PB + b_rd4[j]);
                    bv[p][j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
                }
            }
            if constexpr (H2) {
                auto f16 = [](u32x4 v) { return __builtin_bit_cast(f16x8, v); };
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const u32x4 ah = __builtin_bit_cast(u32x4, av[0][i]), am = __builtin_bit_cast(u32x4, av[1][i]);
                    const u32x4 ahl = f16_down11(ah);
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        const u32x4 bh = __builtin_bit_cast(u32x4, bv[0][j]), bm = __builtin_bit_cast(u32x4, bv[1][j]);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f16(ahl), f16(bm), acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f16(am), f16(f16_down11(bh)), acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f16(ah), f16(bh), acc[i][j], 0, 0, 0);
                    }
                }
            } else {
                constexpr int QA[6] = {1, 0, 2, 0, 1, 0};
                constexpr int QB[6] = {1, 2, 0, 1, 0, 0};
#pragma unroll
                for (int q = NP == 1 ? 5 : 0; q < 6; ++q)  // bf16: the hh product only
#pragma unroll
                    for (int i = 0; i < TM; ++i)
#pragma unroll
                        for (int j = 0; j < TN; ++j)
                            acc[i][j] =
                                __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[QA[q]][i], bv[QB[q]][j], acc[i][j], 0, 0, 0);
            }
            if (more) store_stage((s + 1) & 1);
            __syncthreads();
        }
    }

    if (col_sums) {  // uniform per block; the loop's last barrier has released the stage buffers
        // piece ch = tid + i * NT is (pixel row b_k, column quad ch % BQ): each quad's 16 rows summed in row order
        static_assert(B_CH * 16 <= 2 * STAGE, "column-sum rows fit the stage buffers");
        f32x4 *red = reinterpret_cast<f32x4 *>(smem);
#pragma unroll
        for (int i = 0; i < B_PER; ++i)
            if (B_FULL || b_in[i]) red[tid + i * NT] = cs[i];
        __syncthreads();
        for (int q = tid; q < BQ; q += NT) {
            f32x4 v = red[q];
#pragma unroll
            for (int k = 1; k < BK; ++k) v += red[k * BQ + q];
            const int j = j0 + q * 4;
            float *o = a.colsum + size_t(split) * a.Ng + j;
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (j + e < a.Ng) o[e] = v[e];
        }
    }

    float *slab = a.slabs + size_t(split) * a.R * a.Ng;
    const float osc = rsc_inv * ssc_inv;  // h2: both operand scales (powers of two: exact); 1 otherwise
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int col = j0 + wn * TN * 32 + j * 32 + (lane & 31);
        if (col >= a.Ng) continue;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = r0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                if (row < a.R) gstore1(slab + size_t(row) * a.Ng + col, H2 ? acc[i][j][r] * osc : acc[i][j][r]);
            }
    }
}


const void *wgrad_x3_fn(int tile_id) {
    switch (tile_id) {
        case 0: return reinterpret_cast<const void *>(&wgrad_x3<2, 2, 2, 2>);
        case 1: return reinterpret_cast<const void *>(&wgrad_x3<1, 4, 2, 2>);
        case 2: return reinterpret_cast<const void *>(&wgrad_x3<2, 2, 1, 3>);
        case 3: return reinterpret_cast<const void *>(&wgrad_x3<2, 1, 1, 3>);
        default: return reinterpret_cast<const void *>(&wgrad_x3<1, 4, 1, 1>);
    }
}

void launch_wgrad_x3(const WgradArgs &a, int tile_id, dim3 grid, dim3 block, hipStream_t s) {
    switch (tile_id) {
        case 0: hipLaunchKernelGGL((wgrad_x3<2, 2, 2, 2>), grid, block, 0, s, a); break;
        case 1: hipLaunchKernelGGL((wgrad_x3<1, 4, 2, 2>), grid, block, 0, s, a); break;
        case 2: hipLaunchKernelGGL((wgrad_x3<2, 2, 1, 3>), grid, block, 0, s, a); break;
        case 3: hipLaunchKernelGGL((wgrad_x3<2, 1, 1, 3>), grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL((wgrad_x3<1, 4, 1, 1>), grid, block, 0, s, a); break;
    }
}

// h2 (both operand bounds given, SCD_MATH_H2): every tile of the generic weight grad (the ConvTranspose weight grads
// and the 3x3 weight grads outside the halo kernels, e.g. a 32-channel source).
bool wgrad_x3_h2_tile(int tile_id) { return tile_id >= 0 && tile_id <= 4; }
void launch_wgrad_x3_h2(const WgradArgs &a, int tile_id, dim3 grid, dim3 block, hipStream_t s) {
    switch (tile_id) {
        case 0: hipLaunchKernelGGL((wgrad_x3<2, 2, 2, 2, 4>), grid, block, 0, s, a); break;
        case 1: hipLaunchKernelGGL((wgrad_x3<1, 4, 2, 2, 4>), grid, block, 0, s, a); break;
        case 2: hipLaunchKernelGGL((wgrad_x3<2, 2, 1, 3, 4>), grid, block, 0, s, a); break;
        case 3: hipLaunchKernelGGL((wgrad_x3<2, 1, 1, 3, 4>), grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL((wgrad_x3<1, 4, 1, 1, 4>), grid, block, 0, s, a); break;
    }
}

// bf16 (SCD_MATH_BF16): the ConvTranspose weight grad (4 taps), every tile.
template <bool SB>
static void launch_wgrad_x3_bf16_sb(const WgradArgs &a, int tile_id, dim3 grid, dim3 block, hipStream_t s) {
    switch (tile_id) {
        case 0: hipLaunchKernelGGL((wgrad_x3<2, 2, 2, 2, 1, SB>), grid, block, 0, s, a); break;
        case 1: hipLaunchKernelGGL((wgrad_x3<1, 4, 2, 2, 1, SB>), grid, block, 0, s, a); break;
        case 2: hipLaunchKernelGGL((wgrad_x3<2, 2, 1, 3, 1, SB>), grid, block, 0, s, a); break;
        case 3: hipLaunchKernelGGL((wgrad_x3<2, 1, 1, 3, 1, SB>), grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL((wgrad_x3<1, 4, 1, 1, 1, SB>), grid, block, 0, s, a); break;
    }
}
void launch_wgrad_x3_bf16(const WgradArgs &a, int tile_id, dim3 grid, dim3 block, hipStream_t s) {
    if (a.sb) {
        launch_wgrad_x3_bf16_sb<true>(a, tile_id, grid, block, s);
        return;
    }
    switch (tile_id) {
        case 0: hipLaunchKernelGGL((wgrad_x3<2, 2, 2, 2, 1>), grid, block, 0, s, a); break;
        case 1: hipLaunchKernelGGL((wgrad_x3<1, 4, 2, 2, 1>), grid, block, 0, s, a); break;
        case 2: hipLaunchKernelGGL((wgrad_x3<2, 2, 1, 3, 1>), grid, block, 0, s, a); break;
        case 3: hipLaunchKernelGGL((wgrad_x3<2, 1, 1, 3, 1>), grid, block, 0, s, a); break;
        default: hipLaunchKernelGGL((wgrad_x3<1, 4, 1, 1, 1>), grid, block, 0, s, a); break;
    }
}

// Fragment-major pre-split weights: dst[p][nb][ks][lane][8] (bf16 bits of term p), the B-operand fragment of
// rows n = 32*nb + (lane & 31), k = 16*ks + 8*(lane >> 5) + j of a [n_out][K] fp32 matrix (zero for n >= n_out).
// One wave's fragment for (p, nb, ks) is 1 KB contiguous: a single coalesced load straight into registers.
__global__ void split_frag_kernel(const float *__restrict__ w, int n_out, int K, int NB, uint16_t *__restrict__ dst) {
    const int KS = K / 16;
    const int64_t total = int64_t(NB) * KS * 64;
    const int64_t plane = total * 8;
    for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < total; e += int64_t(gridDim.x) * blockDim.x) {
        const int lane = int(e & 63);
        const int64_t fk = e >> 6;  // nb * KS + ks
        const int nb = int(fk / KS), ks = int(fk - int64_t(nb) * KS);
        const int n = nb * 32 + (lane & 31), k0 = ks * 16 + 8 * (lane >> 5);
        f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = v0;
        if (n < n_out) {
            v0 = gload4(w + size_t(n) * K + k0);
            v1 = gload4(w + size_t(n) * K + k0 + 4);
        }
        u32x2 h0, m0, l0, h1, m1, l1;
        split3(v0, h0, m0, l0);
        split3(v1, h1, m1, l1);
        uint16_t *o = dst + e * 8;
        *reinterpret_cast<u32x4 *>(o) = u32x4{h0[0], h0[1], h1[0], h1[1]};
        *reinterpret_cast<u32x4 *>(o + plane) = u32x4{m0[0], m0[1], m1[0], m1[1]};
        *reinterpret_cast<u32x4 *>(o + 2 * plane) = u32x4{l0[0], l0[1], l1[0], l1[1]};
    }
}

__global__ void split_bf16x3_kernel(const float *__restrict__ src, int64_t n4, uint16_t *__restrict__ dst, int64_t n) {
    for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < n4; e += int64_t(gridDim.x) * blockDim.x) {
        u32x2 h, m, l;
        split3(gload4(src + 4 * e), h, m, l);
        *reinterpret_cast<u32x2 *>(dst + 4 * e) = h;
        *reinterpret_cast<u32x2 *>(dst + n + 4 * e) = m;
        *reinterpret_cast<u32x2 *>(dst + 2 * n + 4 * e) = l;
    }
}

// ------------------------------------------------------------------------------------------------
// Batched weight preparation: for up to kPackJobs conv3x3 weights per launch, the packed fp32 layout of
// scd_pack_conv3x3 and (optionally) its fragment-major bf16x3 split of scd_split_bf16x3_frag, both read straight
// from the OIHW parameter (one launch per training step instead of two per conv).
// ------------------------------------------------------------------------------------------------
constexpr int kPackJobs = 48;
constexpr int kPackCW = 64;  // inner columns (mode 0: input channels, mode 1: output channels) per tile
constexpr int kPackLD = kPackCW + 1;  // LDS row stride: the strided fills hit distinct banks
struct PackJobs {
    scd_pack_job_t j[kPackJobs];
    int first_block[kPackJobs + 1];  // tiles (32 rows x kPackCW inner columns x 9 taps), prefix sums
    int first_rs[kPackJobs + 1];     // h2 jobs: padded split rows (NB * 32) of the row-scale pass, prefix sums
    int h2[kPackJobs];               // split in the SCD_MATH_H2 format (fp16 h, m planes + per-row inverse scales)
    int n;
};

// Per-row inverse scales of an h2 split: float [NB * 32] after the two fp16 planes.
__device__ __forceinline__ float *h2_row_inv(uint16_t *split, int64_t plane) {
    return reinterpret_cast<float *>(split + 2 * plane);
}

// Rows, inner width and K of a job's packed layout: mode 0 [co][9][ci_pad], mode 1 [ci][9][co] (taps flipped).
__device__ __forceinline__ void pack_dims(const scd_pack_job_t &J, int &rows, int &kin, int &K) {
    rows = J.mode == 0 ? J.co : J.ci;
    kin = J.mode == 0 ? J.ci_pad : J.co;
    K = 9 * kin;
}

// One wave per padded split row of every h2 job: the row's max |w| -> its power-of-two inverse scale (the tile pass
// below scales the row by the reciprocal).  Rows of the packed layout are output channels (mode 0) or input channels
// (mode 1, the data-grad layout); the max is read from the OIHW parameter directly.  (A block per 32-row group reading
// the mode-1 rows as contiguous runs w[o][r0 .. r0+31][*] walked the output channels serially: 9x slower.)
__global__ __launch_bounds__(256) void pack_rowscale_kernel(PackJobs jobs) {
    const int wave = int(blockIdx.x) * 4 + int(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (wave >= jobs.first_rs[jobs.n]) return;
    int q = 0;
    while (q + 1 < jobs.n && wave >= jobs.first_rs[q + 1]) ++q;
    const scd_pack_job_t J = jobs.j[q];
    int rows, kin, K;
    pack_dims(J, rows, kin, K);
    const int r = wave - jobs.first_rs[q];
    float mx = 0.f;
    if (r < rows) {
        if (J.mode == 0) {
            const int n = J.ci * 9;
            for (int e = lane; e < n; e += 64) mx = fmaxf(mx, fabsf(J.w[size_t(r) * n + e]));
        } else {
            const int n = J.co * 9;
            for (int e = lane; e < n; e += 64) {
                const int o = e / 9, t = e - o * 9;
                mx = fmaxf(mx, fabsf(J.w[(size_t(o) * J.ci + r) * 9 + t]));
            }
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
    if (lane == 0) {
        float sc, inv;
        h2_scale(mx, sc, inv);
        h2_row_inv(J.split, int64_t((rows + 31) / 32) * 32 * K)[r] = inv;
    }
}

// One block per tile of 32 rows x kPackCW inner columns x 9 taps of a job's packed layout.  The tile's OIHW values
// are read in contiguous runs into LDS (mode 0: w[r][c0 ..][*] per row; mode 1: w[o][r0 .. r0+31][*] per output
// channel), then written as coalesced packed rows and, with a split, as whole 1 KB fragment slots (fragment order of
// scd_split_bf16x3_frag / scd_split_h2_frag).  The same values and split arithmetic as the element-wise pack.
__global__ __launch_bounds__(256) void pack_multi_kernel(PackJobs jobs) {
    __shared__ float T[32 * 9 * kPackLD];  // [row][tap][inner column]
    const int b = blockIdx.x, tid = threadIdx.x;
    int q = 0;
    while (q + 1 < jobs.n && b >= jobs.first_block[q + 1]) ++q;
    const scd_pack_job_t J = jobs.j[q];
    int rows, kin, K;
    pack_dims(J, rows, kin, K);
    const int nchunk = (kin + kPackCW - 1) / kPackCW;
    const int tile = b - jobs.first_block[q];
    const int nb = tile / nchunk, c0 = (tile - nb * nchunk) * kPackCW;
    const int cw = min(kPackCW, kin - c0);
    const int r0 = nb * 32;
    // 8 loads in flight per thread: unconditional (an element outside the weight reads w[0]), selected afterwards
    constexpr int U = 8;
    auto fill = [&](auto at) {  // at(e, ok, src, dst): element e of the tile's OIHW run
        const int total = J.mode == 0 ? 32 * cw * 9 : cw * 288;
        for (int e0 = tid; e0 < total; e0 += 256 * U) {
            float v[U];
            int dst[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = e0 + u * 256;
                bool ok;
                size_t src;
                at(e, ok, src, dst[u]);
                ok = ok && e < total;
                v[u] = J.w[ok ? src : 0];
                v[u] = ok ? v[u] : 0.f;
                dst[u] = e < total ? dst[u] : -1;
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (dst[u] >= 0) T[dst[u]] = v[u];
        }
    };
    if (J.mode == 0) {  // T[rr][t][j] = w[r0 + rr][c0 + j][t] (zero for padded channels and rows)
        const int run = cw * 9;
        fill([&](int e, bool &ok, size_t &src, int &dst) {
            const int rr = e / run, f = e - rr * run, j = f / 9, t = f - j * 9;
            ok = r0 + rr < rows && c0 + j < J.ci;
            src = (size_t(r0 + rr) * J.ci + c0 + j) * 9 + t;
            dst = (rr * 9 + t) * kPackLD + j;
        });
    } else {  // T[rr][t][j] = w[c0 + j][r0 + rr][8 - t]
        fill([&](int e, bool &ok, size_t &src, int &dst) {
            const int j = e / 288, f = e - j * 288, rr = f / 9, t = f - rr * 9;
            ok = r0 + rr < rows;
            src = (size_t(c0 + j) * J.ci + r0 + rr) * 9 + t;
            dst = (rr * 9 + (8 - t)) * kPackLD + j;
        });
    }
    __syncthreads();
    for (int e = tid; e < 32 * 9 * cw; e += 256) {  // packed rows: out[r][t * kin + c0 + j]
        const int rr = e / (9 * cw), f = e - rr * 9 * cw, t = f / cw, j = f - t * cw;
        if (r0 + rr < rows) J.out[size_t(r0 + rr) * K + t * kin + c0 + j] = T[(rr * 9 + t) * kPackLD + j];
    }
    if (!J.split) return;
    const int KS = K / 16, NB = (rows + 31) / 32;
    const int64_t plane = int64_t(NB) * KS * 64 * 8;
    const int nkb = cw / 16;  // 16-column fragment blocks per tap in this tile (kin % 16 == 0 with a split)
    for (int e = tid; e < 9 * nkb * 64; e += 256) {
        const int lane = e & 63, tk = e >> 6, t = tk / nkb, kb = tk - t * nkb;
        const int rr = lane & 31, j0 = kb * 16 + 8 * (lane >> 5);
        const int ks = (t * kin + c0) / 16 + kb;
        const float *src = T + (rr * 9 + t) * kPackLD + j0;
        f32x4 v0 = {src[0], src[1], src[2], src[3]}, v1 = {src[4], src[5], src[6], src[7]};
        uint16_t *o = J.split + ((int64_t(nb) * KS + ks) * 64 + lane) * 8;
        u32x2 h0, m0, l0, h1, m1, l1;
        if (jobs.h2[q]) {
            const float sc = 1.f / h2_row_inv(J.split, plane)[r0 + rr];  // exact: a power of two
            split2h(v0 * sc, h0, m0);
            split2h(v1 * sc, h1, m1);
            *reinterpret_cast<u32x4 *>(o) = u32x4{h0[0], h0[1], h1[0], h1[1]};
            *reinterpret_cast<u32x4 *>(o + plane) = u32x4{m0[0], m0[1], m1[0], m1[1]};
            continue;
        }
        split3(v0, h0, m0, l0);
        split3(v1, h1, m1, l1);
        *reinterpret_cast<u32x4 *>(o) = u32x4{h0[0], h0[1], h1[0], h1[1]};
        *reinterpret_cast<u32x4 *>(o + plane) = u32x4{m0[0], m0[1], m1[0], m1[1]};
        *reinterpret_cast<u32x4 *>(o + 2 * plane) = u32x4{l0[0], l0[1], l1[0], l1[1]};
    }
}

}  // namespace scd

using namespace scd;

extern "C" int scd_pack_conv3x3_multi(const scd_pack_job_t *jobs, int32_t n, scd_stream_t stream) {
    clear_error();
    if (!jobs || n < 0) {
        set_error("pack_conv3x3_multi: bad arguments");
        return SCD_ERR_ARG;
    }
    for (int base = 0; base < n; base += kPackJobs) {
        PackJobs pj;
        pj.n = std::min(kPackJobs, n - base);
        pj.first_block[0] = 0;
        pj.first_rs[0] = 0;
        for (int i = 0; i < pj.n; ++i) {
            const scd_pack_job_t &J = jobs[base + i];
            const int rows = J.mode == 0 ? J.co : J.ci, kin = J.mode == 0 ? J.ci_pad : J.co, K = 9 * kin;
            if (!J.w || !J.out || J.co < 1 || J.ci < 1 || J.ci_pad < J.ci || (J.mode != 0 && J.mode != 1) ||
                (J.split && (K % 16 || !aligned16(J.split)))) {
                set_error("pack_conv3x3_multi: job %d: bad arguments (split needs K %% 16 == 0, 16-byte alignment)",
                          base + i);
                return SCD_ERR_ARG;
            }
            pj.h2[i] = J.split && h2_weight_format(J.math, 9, kin);
            const int groups = (rows + 31) / 32;
            pj.first_rs[i + 1] = pj.first_rs[i] + (pj.h2[i] ? groups * 32 : 0);
            pj.j[i] = J;
            pj.first_block[i + 1] = pj.first_block[i] + groups * ((kin + kPackCW - 1) / kPackCW);
        }
        if (pj.n == 0) break;
        if (pj.first_rs[pj.n] > 0)
            hipLaunchKernelGGL(pack_rowscale_kernel, dim3((pj.first_rs[pj.n] + 3) / 4), dim3(256), 0, as_stream(stream),
                               pj);
        hipLaunchKernelGGL(pack_multi_kernel, dim3(pj.first_block[pj.n]), dim3(256), 0, as_stream(stream), pj);
        SCD_TRY(launch_status("scd_pack_conv3x3_multi"));
    }
    return SCD_OK;
}

extern "C" size_t scd_split_frag_bytes(int32_t n_out, int32_t K) {
    if (n_out < 1 || K < 16 || K % 16) return 0;
    return size_t(3) * ((n_out + 31) / 32) * 32 * size_t(K) * sizeof(uint16_t);
}

extern "C" int scd_split_bf16x3_frag(const float *w, int32_t n_out, int32_t K, uint16_t *dst, scd_stream_t stream) {
    clear_error();
    if (!w || !dst || n_out < 1 || K < 16 || K % 16 || !aligned16(w) || !aligned16(dst)) {
        set_error("split_bf16x3_frag: need K %% 16 == 0 and 16-byte aligned w/dst (n_out=%d K=%d)", n_out, K);
        return SCD_ERR_ARG;
    }
    const int NB = (n_out + 31) / 32;
    const int64_t total = int64_t(NB) * (K / 16) * 64;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(split_frag_kernel, dim3(unsigned(blocks)), dim3(256), 0, as_stream(stream), w, n_out, K, NB, dst);
    return launch_status("scd_split_bf16x3_frag");
}

namespace scd {
// h2 split of a packed [n_out][K] matrix in fragment order: per-row inverse scales (one wave per padded row), then
// the two fp16 planes of the scaled rows (scd_split_h2_frag).
__global__ __launch_bounds__(256) void h2_rowscale_kernel(const float *__restrict__ w, int n_out, int K, int NB,
                                                          uint16_t *__restrict__ dst) {
    const int r = int(blockIdx.x) * 4 + int(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (r >= NB * 32) return;
    float mx = 0.f;
    if (r < n_out)
        for (int k = lane; k < K; k += 64) mx = fmaxf(mx, fabsf(w[size_t(r) * K + k]));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
    if (lane == 0) {
        float sc, inv;
        h2_scale(mx, sc, inv);
        h2_row_inv(dst, int64_t(NB) * 32 * K)[r] = inv;
    }
}
__global__ void h2_split_frag_kernel(const float *__restrict__ w, int n_out, int K, int NB, uint16_t *__restrict__ dst) {
    const int KS = K / 16;
    const int64_t total = int64_t(NB) * KS * 64;
    const int64_t plane = total * 8;
    const float *inv = h2_row_inv(dst, plane);
    for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < total; e += int64_t(gridDim.x) * blockDim.x) {
        const int lane = int(e & 63);
        const int64_t fk = e >> 6;
        const int nb = int(fk / KS), ks = int(fk - int64_t(nb) * KS);
        const int n = nb * 32 + (lane & 31), k0 = ks * 16 + 8 * (lane >> 5);
        f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = v0;
        if (n < n_out) {
            const float sc = 1.f / inv[n];
            v0 = gload4(w + size_t(n) * K + k0) * sc;
            v1 = gload4(w + size_t(n) * K + k0 + 4) * sc;
        }
        u32x2 h0, m0, h1, m1;
        split2h(v0, h0, m0);
        split2h(v1, h1, m1);
        uint16_t *o = dst + e * 8;
        *reinterpret_cast<u32x4 *>(o) = u32x4{h0[0], h0[1], h1[0], h1[1]};
        *reinterpret_cast<u32x4 *>(o + plane) = u32x4{m0[0], m0[1], m1[0], m1[1]};
    }
}
}  // namespace scd

namespace scd {
// ------------------------------------------------------------------------------------------------
// Batched ConvTranspose2d(2, s2) weight preparation (scd_pack_convT2x2_multi): the packed layouts of
// scd_pack_convT2x2 and their fragment-order splits (h2 or bf16x3) for up to kConvTJobs weights in three launches
// (pack, h2 row scales, split) instead of three per weight.  Same index maps and split arithmetic as the one-weight
// path (pack_convT_kernel, h2_rowscale_kernel, h2_split_frag_kernel / split_frag_kernel).
// ------------------------------------------------------------------------------------------------
constexpr int kConvTJobs = 8;
struct ConvTJobs {
    const float *w[kConvTJobs];
    float *out[kConvTJobs];
    uint16_t *split[kConvTJobs];
    int ci[kConvTJobs], co[kConvTJobs], mode[kConvTJobs];
    int fmt[kConvTJobs];                // 0 no split, 1 bf16x3, 2 h2
    int64_t first_e[kConvTJobs + 1];    // packed elements (ci * co * 4), prefix sums
    int first_rs[kConvTJobs + 1];       // h2 jobs: padded split rows, prefix sums
    int64_t first_f[kConvTJobs + 1];    // split jobs: fragment lanes (NB * K/16 * 64), prefix sums
    int n;
};
__device__ __forceinline__ int convT_job(const int64_t *first, int n, int64_t e) {
    int q = 0;
    while (q + 1 < n && e >= first[q + 1]) ++q;
    return q;
}
__device__ __forceinline__ void convT_dims(const ConvTJobs &J, int q, int &n_out, int &K) {
    n_out = J.mode[q] == 0 ? 4 * J.co[q] : J.ci[q];
    K = J.mode[q] == 0 ? J.ci[q] : 4 * J.co[q];
}
__global__ void convT_pack_multi_kernel(ConvTJobs J) {
    const int64_t total = J.first_e[J.n];
    for (int64_t g = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; g < total; g += int64_t(gridDim.x) * blockDim.x) {
        const int q = convT_job(J.first_e, J.n, g);
        const int64_t e = g - J.first_e[q];
        const int ci = J.ci[q], co = J.co[q];
        if (J.mode[q] == 0) {  // out[(t*co + o)][c]
            const int c = int(e % ci);
            const int r = int(e / ci);
            const int t = r / co, o = r % co;
            J.out[q][e] = J.w[q][(int64_t(c) * co + o) * 4 + t];
        } else {  // out[c][t*co + o]
            const int col = int(e % (4 * co));
            const int c = int(e / (4 * co));
            const int t = col / co, o = col % co;
            J.out[q][e] = J.w[q][(int64_t(c) * co + o) * 4 + t];
        }
    }
}
__global__ __launch_bounds__(256) void convT_rowscale_multi_kernel(ConvTJobs J) {
    const int wave = int(blockIdx.x) * 4 + int(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (wave >= J.first_rs[J.n]) return;
    int q = 0;
    while (q + 1 < J.n && wave >= J.first_rs[q + 1]) ++q;
    int n_out, K;
    convT_dims(J, q, n_out, K);
    const int r = wave - J.first_rs[q];
    float mx = 0.f;
    if (r < n_out)
        for (int k = lane; k < K; k += 64) mx = fmaxf(mx, fabsf(J.out[q][size_t(r) * K + k]));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off));
    if (lane == 0) {
        float sc, inv;
        h2_scale(mx, sc, inv);
        h2_row_inv(J.split[q], int64_t((n_out + 31) / 32) * 32 * K)[r] = inv;
    }
}
__global__ void convT_split_multi_kernel(ConvTJobs J) {
    const int64_t total = J.first_f[J.n];
    for (int64_t g = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; g < total; g += int64_t(gridDim.x) * blockDim.x) {
        const int q = convT_job(J.first_f, J.n, g);
        if (!J.fmt[q]) continue;
        const int64_t e = g - J.first_f[q];
        int n_out, K;
        convT_dims(J, q, n_out, K);
        const int KS = K / 16, NB = (n_out + 31) / 32;
        const int64_t plane = int64_t(NB) * KS * 64 * 8;
        const int lane = int(e & 63);
        const int64_t fk = e >> 6;
        const int nb = int(fk / KS), ks = int(fk - int64_t(nb) * KS);
        const int n = nb * 32 + (lane & 31), k0 = ks * 16 + 8 * (lane >> 5);
        const float *w = J.out[q];
        uint16_t *o = J.split[q] + e * 8;
        f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = v0;
        if (J.fmt[q] == 2) {
            if (n < n_out) {
                const float sc = 1.f / h2_row_inv(J.split[q], plane)[n];
                v0 = gload4(w + size_t(n) * K + k0) * sc;
                v1 = gload4(w + size_t(n) * K + k0 + 4) * sc;
            }
            u32x2 h0, m0, h1, m1;
            split2h(v0, h0, m0);
            split2h(v1, h1, m1);
            *reinterpret_cast<u32x4 *>(o) = u32x4{h0[0], h0[1], h1[0], h1[1]};
            *reinterpret_cast<u32x4 *>(o + plane) = u32x4{m0[0], m0[1], m1[0], m1[1]};
        } else {
            if (n < n_out) {
                v0 = gload4(w + size_t(n) * K + k0);
                v1 = gload4(w + size_t(n) * K + k0 + 4);
            }
            u32x2 h0, m0, l0, h1, m1, l1;
            split3(v0, h0, m0, l0);
            split3(v1, h1, m1, l1);
            *reinterpret_cast<u32x4 *>(o) = u32x4{h0[0], h0[1], h1[0], h1[1]};
            *reinterpret_cast<u32x4 *>(o + plane) = u32x4{m0[0], m0[1], m1[0], m1[1]};
            *reinterpret_cast<u32x4 *>(o + 2 * plane) = u32x4{l0[0], l0[1], l1[0], l1[1]};
        }
    }
}
}  // namespace scd

extern "C" int scd_pack_convT2x2_multi(const scd_pack_job_t *jobs, int32_t n, scd_stream_t stream) {
    clear_error();
    if (!jobs || n < 0) {
        set_error("pack_convT2x2_multi: bad arguments");
        return SCD_ERR_ARG;
    }
    const hipStream_t s = as_stream(stream);
    auto grid = [](int64_t total) { return dim3(unsigned(std::min<int64_t>((total + 255) / 256, 8192))); };
    for (int base = 0; base < n; base += kConvTJobs) {
        ConvTJobs J;
        J.n = std::min(kConvTJobs, n - base);
        J.first_e[0] = 0;
        J.first_rs[0] = 0;
        J.first_f[0] = 0;
        for (int i = 0; i < J.n; ++i) {
            const scd_pack_job_t &P = jobs[base + i];
            const int n_out = P.mode == 0 ? 4 * P.co : P.ci, K = P.mode == 0 ? P.ci : 4 * P.co;
            if (!P.w || !P.out || P.co < 1 || P.ci < 1 || (P.mode != 0 && P.mode != 1) ||
                (P.split && (K % 16 || !aligned16(P.split) || !aligned16(P.out)))) {
                set_error("pack_convT2x2_multi: job %d: bad arguments (split needs K %% 16 == 0, 16-byte alignment)",
                          base + i);
                return SCD_ERR_ARG;
            }
            J.w[i] = P.w;
            J.out[i] = P.out;
            J.split[i] = P.split;
            J.ci[i] = P.ci;
            J.co[i] = P.co;
            J.mode[i] = P.mode;
            const int c = P.mode == 0 ? P.ci : P.co;  // source channels of the conv reading this layout
            J.fmt[i] = !P.split ? 0 : h2_weight_format(P.math, P.mode == 0 ? 1 : 4, c) ? 2 : 1;
            const int NB = (n_out + 31) / 32;
            J.first_e[i + 1] = J.first_e[i] + int64_t(P.ci) * P.co * 4;
            J.first_rs[i + 1] = J.first_rs[i] + (J.fmt[i] == 2 ? NB * 32 : 0);
            J.first_f[i + 1] = J.first_f[i] + (J.fmt[i] ? int64_t(NB) * (K / 16) * 64 : 0);
        }
        hipLaunchKernelGGL(convT_pack_multi_kernel, grid(J.first_e[J.n]), dim3(256), 0, s, J);
        if (J.first_rs[J.n] > 0)
            hipLaunchKernelGGL(convT_rowscale_multi_kernel, dim3((J.first_rs[J.n] + 3) / 4), dim3(256), 0, s, J);
        if (J.first_f[J.n] > 0) hipLaunchKernelGGL(convT_split_multi_kernel, grid(J.first_f[J.n]), dim3(256), 0, s, J);
        SCD_TRY(launch_status("scd_pack_convT2x2_multi"));
    }
    return SCD_OK;
}

extern "C" int scd_split_h2_frag(const float *w, int32_t n_out, int32_t K, uint16_t *dst, scd_stream_t stream) {
    clear_error();
    if (!w || !dst || n_out < 1 || K < 16 || K % 16 || !aligned16(w) || !aligned16(dst)) {
        set_error("split_h2_frag: need K %% 16 == 0 and 16-byte aligned w/dst (n_out=%d K=%d)", n_out, K);
        return SCD_ERR_ARG;
    }
    const int NB = (n_out + 31) / 32;
    hipStream_t s = as_stream(stream);
    hipLaunchKernelGGL(h2_rowscale_kernel, dim3(NB * 8), dim3(256), 0, s, w, n_out, K, NB, dst);
    const int64_t total = int64_t(NB) * (K / 16) * 64;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(h2_split_frag_kernel, dim3(unsigned(blocks)), dim3(256), 0, s, w, n_out, K, NB, dst);
    return launch_status("scd_split_h2_frag");
}

extern "C" int scd_split_bf16x3(const float *src, int64_t n, uint16_t *dst, scd_stream_t stream) {
    clear_error();
    if (!src || !dst || n <= 0 || (n & 7) || !aligned16(src) || !aligned16(dst)) {
        set_error("split_bf16x3: need n %% 8 == 0 and 16-byte aligned src/dst (n=%lld)", (long long)n);
        return SCD_ERR_ARG;
    }
    const int64_t n4 = n / 4;
    int64_t blocks = (n4 + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(split_bf16x3_kernel, dim3(unsigned(blocks)), dim3(256), 0, as_stream(stream), src, n4, dst, n);
    return launch_status("scd_split_bf16x3");
}
