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

// row16_sum of the four components of v, bit-identical to four row16_sum calls (x + perm(x) is perm(x) + x).  The
// four chains are interleaved in one asm block so each DPP add reads a value written four VALU instructions earlier
// (the DPP read-after-VALU-write hazard needs two wait states; the leading s_nop covers the producers of v).  Written
// out because, on vector inputs, the compiler packs the four chains' adds into v_pk_add_f32 and can then no longer
// fold each DPP move into its add: 2.5 instructions per step instead of one.
__device__ __forceinline__ f32x4 row16_sum4(f32x4 v) {
    float a, b, c, d;
    asm volatile(
        "s_nop 1\n\t"
        "v_add_f32_dpp %0, %4, %4 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %1, %5, %5 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %2, %6, %6 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %3, %7, %7 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %1, %1, %1 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %2, %2, %2 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %3, %3, %3 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %1, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %2, %2, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %3, %3, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %1, %1, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %2, %2, %2 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %3, %3, %3 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1"
        : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d)
        : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
    return f32x4{a, b, c, d};
}

__device__ __forceinline__ void gstore4(float *p, f32x4 v) { *(__attribute__((address_space(1))) f32x4 *)(p) = v; }

// WAVES_M x WAVES_N waves; a wave computes TM*16 pixels x TN*16 channels (TM x TN MFMA tiles).
// IN_BN: the source is a conv output y of the previous layer; its BatchNorm-apply + ReLU,
// max(fma(y, scale, shift), 0) with the exact expression of bn_relu_apply_kernel, is applied while the halo
// is staged (in-range pixels only: the zero padding belongs to the activation).
// DB: double-buffered halo.  The next chunk's halo is written into the other buffer in the middle of the
// current chunk (its loads were issued at the chunk's first tap), so a chunk end costs one barrier and the
// split/store work overlaps the MFMAs instead of stalling between two barriers.
// NP selects the arithmetic: 3 = the exact x3 split (six products per step), 5 = x3 without the w_l * x_h product
// (SCD_MATH_X5: weights in two planes, five products), 1 = bf16 operands (SCD_MATH_BF16: the h terms, one product),
// 2 = the two-term fp16 split (SCD_MATH_H2, x3_common.h: three v_mfma_f32_16x16x32_f16 products; the halo is
// scaled by the power of two of *src_bound while staged, the weights come pre-scaled per output channel, and the
// epilogue multiplies both inverse scales back out -- exact, powers of two).
// SB: bf16 storage of src / dst / the BatchNorm-backward y (bf16 arithmetic only, StageT in x3_common.h).
// WL (SCD_TUNE_HALO16_WRING, h2 single-buffered 3x3 only): the weight fragments go through a 3-slot LDS ring instead of
// straight into registers.  Each k-step's BN x 32 x 2-plane weights (8 or 16 KB) are copied global -> LDS by LDS-DMA
// (global_load_lds_dwordx4, 1 KB per wave-instruction, split over the block's waves) two steps ahead; a step starts with
// a counted vmcnt wait for this wave's pieces of the step plus one barrier, then reads its fragments with ds_read_b128.
// What it changes: (1) a weight fragment shared by two waves (the 2 x 2 tile) is fetched once; (2) the next chunk's
// halo loads, issued after the DMA of step T+2, are waited for only at step T+3 (vmcnt counts them as younger than the
// DMA pieces of steps T+1 and T+2), two k-steps later than when every wave waited for its own next-step weight loads
// behind them.  Same products in the same order: bit-identical to WL = false.
template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ void lds_barrier() {  // a barrier that leaves LDS-DMA pieces in flight (no vmcnt(0))
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// The bf16 1 x N double-buffered tiles load their weight fragments two k-steps ahead (W2 below): dual-stream bs=64
// 40.65 -> 40.10 ms per step, alternating processes (profiles/r05_bf16_w2_ab.txt); -DSCD_HALO16_W2=0 builds the
// one-step lead for A/B.
#ifndef SCD_HALO16_W2
#define SCD_HALO16_W2 1
#endif
template <int WAVES_M, int WAVES_N, int TM, int TN, int TW, int OCC, bool IN_BN, bool DB, int NP, bool SB = false,
          bool WL = false>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N, OCC) void igemm_halo16_x3(IgemmArgs a) {
    static_assert(!SB || NP == 1, "bf16 storage runs the bf16 arithmetic");
    static_assert(!WL || (NP == 4 && !DB && !SB), "the weight ring: single-buffered h2 only");
    constexpr uint32_t EB = SB ? 2u : 4u;  // bytes per element
    constexpr int NT = 64 * WAVES_M * WAVES_N;
    constexpr int WPX = TM * 16, WCH = TN * 16;
    constexpr int BM = WAVES_M * WPX, BN = WAVES_N * WCH;
    constexpr int TR = BM / TW;
    constexpr int HWD = TW + 2;
    // LDS row pitch of the halo.  16-wide tiles on one buffer: 24 rows per halo row instead of 18, so the 16-pixel
    // groups of a wave (one halo row apart) sit 24 rows apart, and 24 / 2 = 12 = 0 mod 4 leaves the row swizzle
    // unchanged between them: one swizzled address per k-step, the groups at immediate offsets (8 VALU per step
    // instead of ~50).  The 6 pad rows per halo row are never staged or read.
    // (double-buffered tiles too where both padded buffers of every resident block fit the CU's LDS: the bf16 tiles)
    constexpr bool PADP = TW == 16 && !WL &&
                          (!DB || OCC * 2 * (NP == 1 ? 1 : (NP == 2 || NP == 4) ? 2 : 3) * (TR + 2) * 24 * 64 <= 160 * 1024);
    constexpr int HWP = PADP ? 24 : HWD;
    constexpr int HR = (TR + 2) * HWP;           // LDS rows of one plane
    constexpr int A_CH = (TR + 2) * HWD * 8;     // 16-byte (4-channel) pieces of one 32-channel chunk
    constexpr int A_PER = (A_CH + NT - 1) / NT;
    constexpr int PA = HR * 64;
    // Epilogue reductions run over groups of 4 pixel tiles (64 pixels) per wave, so a 1 x N wave layout (TM = 8) sums
    // in the order of the 2 x N layout (TM = 4) and both give bit-identical statistics records.
    constexpr int RG = TM >= 8 ? TM / 4 : 1;  // reduction groups per wave
    constexpr int TMG = TM / RG;              // pixel tiles per group
    constexpr int WME = WAVES_M * RG;         // reduction rows of the block
    constexpr int RED = 2 * WME * BN * 4;
    constexpr int NBUF = DB ? 2 : 1;
    static_assert(NP == 1 || NP == 2 || NP == 3 || NP == 4 || NP == 5, "x3, x5, bf16 or h2");
    constexpr bool H2 = NP == 2 || NP == 4;  // 4: h2 with the activations' low term pre-scaled (x3_common.h)
    constexpr int XP = NP == 1 ? 1 : H2 ? 2 : 3;               // activation planes (LDS)
    constexpr int WP = NP == 1 ? 1 : (NP == 5 || H2) ? 2 : 3;  // weight planes (registers)
    constexpr int NBB = BN / 32;                               // 32-channel weight blocks of the tile
    constexpr int WSLOT = WL ? WP * NBB * 2048 : 0;            // WL: bytes of one k-step's weights (one ring slot)
    constexpr int WG = WSLOT / (1024 * WAVES_M * WAVES_N);     // WL: 1 KB DMA pieces per wave per step
    static_assert(!WL || WG * 1024 * WAVES_M * WAVES_N == WSLOT, "ring slot splits evenly over the waves");
    constexpr int HALO_B = NBUF * XP * PA;
    constexpr int SMEM = HALO_B + 3 * WSLOT > RED ? HALO_B + 3 * WSLOT : RED;
    __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
    float xs = 1.f, xs_inv = 1.f;  // h2: power-of-two scale of the staged activations and its inverse
    if constexpr (H2) h2_scale(*a.src_bound, xs, xs_inv);

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
    {
        // this thread's pieces: halo pixel (tid >> 3) + i NT / 8, channel piece tid & 7 (NT % 8 == 0).  The halo
        // position and byte offset advance by a constant step per piece (one compare for the row wrap), instead of
        // a division and three 32-bit products per piece
        static_assert(NT % 8 == 0, "a thread's pieces share one channel piece");
        constexpr int S = NT / 8, DQ = S / HWD, DR = S % HWD;
        const int col = tid & 7;
        int hy = (tid >> 3) / HWD, hx = (tid >> 3) - ((tid >> 3) / HWD) * HWD;
        const int pix_b = a.ldc_s * int(EB), row_b = a.ws * pix_b;
        // byte offset of halo pixel (0, 0) = source pixel (y0 - 1, x0 - 1), channel piece col (may wrap below zero:
        // only in-range pieces use the sum, whose true value fits)
        const uint32_t base = uint32_t(((img * a.hs + y0 - 1) * a.ws + x0 - 1) * a.ldc_s + col * 4) * EB;
        int off = hy * row_b + hx * pix_b;
        const int step = DQ * row_b + DR * pix_b, wrap = row_b - HWD * pix_b;
#pragma unroll
        for (int i = 0; i < A_PER; ++i) {
            const bool in = tid + i * NT < A_CH;
            const int sy = y0 - 1 + hy, sx = x0 - 1 + hx;
            const bool ok = in && unsigned(sy) < unsigned(a.hs) && unsigned(sx) < unsigned(a.ws);
            a_boff[i] = ok ? base + uint32_t(off) : kOOB;
            a_off[i] = in ? soff(hy * HWP + hx, col) : -1;
            hx += DR;
            const bool w = hx >= HWD;  // selects, not a branch
            hx = w ? hx - HWD : hx;
            hy += DQ + int(w);
            off += step + (w ? wrap : 0);
        }
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

    StageT<SB> ra[A_PER];
    f32x4 in_sc, in_sh;  // IN_BN coefficients of this thread's 4 channels (col = tid & 7 for every piece)
    const __amdgpu_buffer_rsrc_t rs_src = make_rsrc(a.src, a.src_bytes);
    const __amdgpu_buffer_rsrc_t rs_w = make_rsrc(a.wsplit, uint32_t(WP) * wplane_b);
    auto load_A = [&](int cc) {
#pragma unroll
        for (int i = 0; i < A_PER; ++i) ra[i] = bload_q<SB>(rs_src, a_boff[i] == kOOB ? kOOB : a_boff[i] + cc * 32u * EB);
        if constexpr (IN_BN) {
            const int ch = (img / a.in_seg_imgs) * a.c + cc * 32 + (tid & 7) * 4;
            in_sc = gload4(a.in_scale + ch);
            in_sh = gload4(a.in_shift + ch);
        }
    };
    auto store_A = [&](int buf) {
        unsigned char *const sb = smem + buf * (XP * PA);
        // h2: fma(y, sc * s, sh * s) == s * fma(y, sc, sh) exactly (s a power of two).  Scaled here, where the halo
        // is consumed, not where its coefficients are loaded: a use right behind the loads made the compiler wait for
        // them there, and vmcnt retires in order, so that wait drained the whole halo prefetch at issue.
        const f32x4 sc = H2 ? in_sc * xs : in_sc, sh = H2 ? in_sh * xs : in_sh;
#pragma unroll
        for (int i = 0; i < A_PER; ++i)
            if ((A_CH % NT == 0) || a_off[i] >= 0) {
                u32x2 h, m, l;
                f32x4 x = stage_f32<SB>(ra[i]);
                if constexpr (IN_BN) {
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        x[q] = a_boff[i] == kOOB ? 0.f : fmaxf(fmaf(x[q], sc[q], sh[q]), 0.f);
                }
                if constexpr (H2) {
                    if constexpr (!IN_BN) x *= xs;
                    if constexpr (NP == 4)
                        split2h_pre(x, h, m);
                    else
                        split2h(x, h, m);
                    *reinterpret_cast<u32x2 *>(sb + a_off[i]) = h;
                    *reinterpret_cast<u32x2 *>(sb + PA + a_off[i]) = m;
                } else if constexpr (XP == 3) {
                    split3(x, h, m, l);
                    *reinterpret_cast<u32x2 *>(sb + a_off[i]) = h;
                    *reinterpret_cast<u32x2 *>(sb + PA + a_off[i]) = m;
                    *reinterpret_cast<u32x2 *>(sb + 2 * PA + a_off[i]) = l;
                } else {
                    if constexpr (SB && !IN_BN)
                        h = ra[i];  // the stored bf16 is the operand
                    else
                        h = u32x2{cvt_pk_bf16(x[0], x[1]), cvt_pk_bf16(x[2], x[3])};
                    *reinterpret_cast<u32x2 *>(sb + a_off[i]) = h;
                }
            }
    };
    const int cpk = a.c / 32;
    auto load_W = [&](int cc, int t, u32x4 (&wq)[WP][TN]) {
        const uint32_t ko = uint32_t(t * cpk + cc) * 2048u;  // 32-deep step = two 16-deep fragments
#pragma unroll
        for (int p = 0; p < WP; ++p)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                wq[p][j] = bload4u(rs_w, w_base[j] == kOOB ? kOOB : w_base[j] + ko + uint32_t(p) * wplane_b);
    };
    // WL: step s2's weights -> ring slot s2 % 3.  Piece q (1 KB) = plane q / (2 NBB), 32-channel block (q / 2) % NBB,
    // 16-deep half q % 2: the slot holds [plane][block][2 KB] in the global fragment order, so a lane reads its fragment
    // at the same offset within the block's 2 KB as the register path's w_base.
    const int wave_u = __builtin_amdgcn_readfirstlane(wid);
    auto issue_W = [&](int s2) {
        const int c2 = s2 / a.ntaps, t2 = s2 - c2 * a.ntaps;
        const uint32_t ko = uint32_t(t2 * cpk + c2) * 2048u;
        unsigned char *const slot = smem + HALO_B + (s2 % 3) * WSLOT;
#pragma unroll
        for (int u = 0; u < WG; ++u) {
            const int q = wave_u * WG + u;
            const int p = q / (2 * NBB), r = q - p * (2 * NBB);
            const uint32_t goff = uint32_t(p) * wplane_b + uint32_t(((n0 >> 5) + (r >> 1)) * KS16) * 1024u + ko +
                                  uint32_t(r & 1) * 1024u + uint32_t(lane) * 16u;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(reinterpret_cast<const unsigned char *>(a.wsplit) + goff),
                (__attribute__((address_space(3))) void *)(slot + q * 1024), 16, 0, 0);
        }
        asm volatile("" ::: "memory");  // the DMA pieces stay older than the halo loads issued after them
    };
    int w_lds[TN];  // WL: this lane's fragment offset within a ring slot (plane 0)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int cb = (n0 >> 4) + wn * TN + j;
        w_lds[j] = ((cb >> 1) - (n0 >> 5)) * 2048 + (g >> 1) * 1024 + (16 * (cb & 1) + l16 + 32 * (g & 1)) * 16;
    }

    f32x4 acc[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

    int a_hr[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int p = wm * WPX + i * 16 + l16;
        a_hr[i] = (p / TW + 1) * HWP + (p % TW) + 1;
    }

    const int nsteps = cpk * a.ntaps;
    constexpr int T_STORE = 4;  // DB: tap at which the prefetched halo is written to the other buffer
    // single buffer: the tap at which the next chunk's halo loads are issued into registers (stored at the chunk end),
    // 4 taps ahead so HBM latency hides behind 4 taps of MFMAs; SCD_TUNE_HALO16_LATE_LOAD: the last tap (A/B)
    // (WL: always 4 taps ahead; the launcher takes WL for 9-tap convs only)
    const int t_load = !WL && ((a.tune & SCD_TUNE_HALO16_LATE_LOAD) || a.ntaps < 5) ? a.ntaps - 1 : a.ntaps - 5;
    u32x4 wq[WP][TN];
    if constexpr (WL) {
        issue_W(0);
        if (nsteps > 1) issue_W(1);
    }
    load_A(0);
    if constexpr (!WL) load_W(0, 0, wq);
    // W2 (the bf16 double-buffered tiles, SCD_HALO16_W2): the weight fragments two k-steps ahead in two register sets.
    // A bf16 k-step is 16 MFMAs per wave, a third of an h2 one, and one step of lead left the L2 latency of the next
    // step's fragments exposed.
    constexpr bool W2 = SCD_HALO16_W2 && NP == 1 && DB && !WL && WAVES_M == 1;  // (2 x 2 tiles: spills)
    u32x4 wq2[W2 ? WP : 1][W2 ? TN : 1];
    if constexpr (W2) {
        if (nsteps > 1) load_W(a.ntaps > 1 ? 0 : 1, a.ntaps > 1 ? 1 : 0, wq2);
    }
    store_A(0);
    __syncthreads();
    int cc = 0, t = 0;
    if constexpr (W2) {
        // one k-step: MFMAs on wcur, then wcur refilled with step s + 2 (same sums and order as the loop below)
        auto step = [&](int s, u32x4 (&wcur)[W2 ? WP : 1][W2 ? TN : 1]) {
            int t1 = t + 1, cc1 = cc;
            if (t1 == a.ntaps) {
                t1 = 0;
                cc1 = cc + 1;
            }
            int t2 = t1 + 1, cc2 = cc1;
            if (t2 == a.ntaps) {
                t2 = 0;
                cc2 = cc1 + 1;
            }
            const bool more = s + 1 < nsteps;
            if (t == 0 && cc + 1 < cpk) load_A(cc + 1);
            const unsigned char *const sbuf = smem + (cc & 1) * (XP * PA);
            const int toff = tap_at(a.tdy, t) * HWP + tap_at(a.tdx, t);
            bf16x8 xv[TM];
            if constexpr (PADP) {
                const int hr = a_hr[0] + toff;
                const unsigned char *const sb0 = sbuf + hr * 64 + (((g ^ (hr >> 1)) & 3) << 4);
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    xv[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4 *>(sb0 + i * (HWP * 64)));
            } else {
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int hr = a_hr[i] + toff;
                    const int ad = hr * 64 + (((g ^ (hr >> 1)) & 3) << 4);
                    xv[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4 *>(sbuf + ad));
                }
            }
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int i = 0; i < TM; ++i)
                    acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wcur[0][j]), xv[i],
                                                                        acc[j][i], 0, 0, 0);
            if (s + 2 < nsteps) load_W(cc2, t2, wcur);
            if (t == T_STORE && cc + 1 < cpk) store_A((cc + 1) & 1);
            if (more && t1 == 0) __syncthreads();
            t = t1;
            cc = cc1;
        };
        for (int s = 0; s < nsteps; s += 2) {
            step(s, wq);
            if (s + 1 < nsteps) step(s + 1, wq2);
        }
    }
    for (int s = 0; s < (W2 ? 0 : nsteps); ++s) {
        int t1 = t + 1, cc1 = cc;
        if (t1 == a.ntaps) {
            t1 = 0;
            cc1 = cc + 1;
        }
        const bool more = s + 1 < nsteps;
        if constexpr (WL) {
            // Retire this wave's DMA pieces of step s: younger than them are step s+1's pieces (WG) and, at the step after
            // the next chunk's halo loads were issued (ahead of step t_load+2's pieces), those loads (HL); then every
            // wave's pieces.  The halo loads go first at step t_load: the compiler drains vmcnt before reissuing into
            // their registers, and what is in flight then is only step t_load+1's pieces, issued a step earlier.
            constexpr int HL = A_PER + (IN_BN ? 2 : 0);
            if (!more)
                wait_vm_barrier<0>();
            else if (cc + 1 < cpk && t == t_load + 1)
                wait_vm_barrier<WG + HL>();
            else
                wait_vm_barrier<WG>();
            if (t == t_load && cc + 1 < cpk) load_A(cc + 1);
            asm volatile("" ::: "memory");
            if (s + 2 < nsteps) issue_W(s + 2);  // into the slot of step s-1, which every wave has left
        } else if constexpr (DB) {
            if (t == 0 && cc + 1 < cpk) load_A(cc + 1);
        }
        const unsigned char *const sbuf = smem + (DB ? (cc & 1) * (XP * PA) : 0);
        const int toff = tap_at(a.tdy, t) * HWP + tap_at(a.tdx, t);
        bf16x8 xv[XP][TM], wv[WP][TN];
        if constexpr (PADP) {  // a_hr[i] = a_hr[0] + 24 i: same swizzle, rows 24 i further
            const int hr = a_hr[0] + toff;
            const unsigned char *const sb0 = sbuf + hr * 64 + (((g ^ (hr >> 1)) & 3) << 4);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int p = 0; p < XP; ++p)
                    xv[p][i] = __builtin_bit_cast(bf16x8,
                                                  *reinterpret_cast<const u32x4 *>(sb0 + p * PA + i * (HWP * 64)));
        } else {
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int hr = a_hr[i] + toff;
                const int ad = hr * 64 + (((g ^ (hr >> 1)) & 3) << 4);
#pragma unroll
                for (int p = 0; p < XP; ++p)
                    xv[p][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4 *>(sbuf + p * PA + ad));
            }
        }
        if constexpr (WL) {
            const unsigned char *const wslot = smem + HALO_B + (s % 3) * WSLOT;
#pragma unroll
            for (int p = 0; p < WP; ++p)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    wv[p][j] = __builtin_bit_cast(
                        bf16x8, *reinterpret_cast<const u32x4 *>(wslot + p * (NBB * 2048) + w_lds[j]));
        } else {
#pragma unroll
            for (int p = 0; p < WP; ++p)
#pragma unroll
                for (int j = 0; j < TN; ++j) wv[p][j] = __builtin_bit_cast(bf16x8, wq[p][j]);
        }
        if constexpr (H2) {
            // h2: w_h x_m (NP 4: (w_h 2^-11) x_m', x_m' pre-scaled by 2^11), w_m x_h, w_h x_h on the fp16 planes
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const u32x4 wh = __builtin_bit_cast(u32x4, wv[0][j]), wm = __builtin_bit_cast(u32x4, wv[1][j]);
                const u32x4 wh_lo = NP == 4 ? f16_down11(wh) : wh;
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const u32x4 xh = __builtin_bit_cast(u32x4, xv[0][i]), xm = __builtin_bit_cast(u32x4, xv[1][i]);
                    acc[j][i] = mfma16_f16(wh_lo, xm, acc[j][i]);
                    acc[j][i] = mfma16_f16(wm, xh, acc[j][i]);
                    acc[j][i] = mfma16_f16(wh, xh, acc[j][i]);
                }
            }
        } else {
            // (w, x) term pairs smallest first: mm, hl, lh, hm, mh, hh; x5 drops lh (w_l * x_h), bf16 runs hh only
            constexpr int QW[6] = {1, 0, 2, 0, 1, 0};
            constexpr int QX[6] = {1, 2, 0, 1, 0, 0};
#pragma unroll
            for (int q = NP == 1 ? 5 : 0; q < 6; ++q)
                if (NP != 5 || QW[q] != 2)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
#pragma unroll
                        for (int i = 0; i < TM; ++i)
                            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[QW[q]][j], xv[QX[q]][i], acc[j][i],
                                                                                0, 0, 0);
        }
        if constexpr (!WL) {
            if (more) load_W(cc1, t1, wq);
            // single buffer: the next chunk's halo loads go out BEHIND the next step's weight loads.  vmcnt retires in
            // order, so halo loads issued ahead of them (at the top of the step, as before round 4) were drained by the
            // very next weight wait: the prefetch ran synchronously.  Behind them, the first wait that drains the halo
            // is the weight wait one step later.
            if constexpr (!DB) {
                asm volatile("" ::: "memory");
                if (t == t_load && cc + 1 < cpk) load_A(cc + 1);
            }
        }
        if constexpr (DB) {
            // the other buffer was last read in the previous chunk, which every wave has left (barrier below)
            if (t == T_STORE && cc + 1 < cpk) store_A((cc + 1) & 1);
            if (more && t1 == 0) __syncthreads();  // chunk end: the next halo is complete
        } else if constexpr (WL) {
            if (more && t1 == 0) {  // as below, with barriers that leave the next two steps' DMA pieces in flight
                lds_barrier();
                store_A(0);
                lds_barrier();
            }
        } else {
            if (more && t1 == 0) {  // chunk end: every wave is done with this halo; overwrite it with the next one
                __syncthreads();
                store_A(0);
                __syncthreads();
            }
        }
        t = t1;
        cc = cc1;
    }
    __syncthreads();  // the epilogue reuses smem for the statistics reduction

    if constexpr (H2) {  // undo the operand scales: per-channel weight inverse scales after the planes
        const float *winv = reinterpret_cast<const float *>(reinterpret_cast<const unsigned char *>(a.wsplit) +
                                                            2u * wplane_b);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * WCH + j * 16 + 4 * g;
            const f32x4 sc = (n < NB32 * 32 ? gload4(winv + n) : f32x4{0.f, 0.f, 0.f, 0.f}) * xs_inv;
#pragma unroll
            for (int i = 0; i < TM; ++i) acc[j][i] *= sc;
        }
    }

    // acc[j][i][r]: channel n0 + wn*WCH + 16j + 4g + r, pixel wm*WPX + 16i + l16
    f32x4 bias4[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WCH + j * 16 + 4 * g;
        bias4[j] = (a.bias && n < a.n_out) ? *reinterpret_cast<const f32x4 *>(a.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // 16-wide tiles: pixel tile i of the wave is output row y0 + (wm WPX) / 16 + i, column x0 + l16, so a lane's
    // addresses are one base plus i rows plus 16 j channels (one 64-bit multiply per lane instead of one per tile;
    // the 64-bit index products had made the epilogue the kernel's largest VALU block on the K = 576 layers)
    const int nq = n0 + wn * WCH + 4 * g;  // the lane's first channel (tile j adds 16 j)
    auto row_pix = [&](int i) -> size_t {  // output pixel of pixel tile i of this lane
        const int p = wm * WPX + i * 16 + l16;
        return size_t(img * a.ho + y0 + p / TW) * a.wo + x0 + (p % TW);
    };
    unsigned char *const dst_b = reinterpret_cast<unsigned char *>(a.dst);
    const size_t d_row = size_t(a.wo) * a.ldc_d * EB;  // TW == 16: bytes from pixel tile i to i + 1
    unsigned char *d_p = dst_b + (row_pix(0) * a.ldc_d + nq) * EB;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        if constexpr (TW != 16) d_p = dst_b + (row_pix(i) * a.ldc_d + nq) * EB;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            if (nq + j * 16 < a.n_out) {
                const f32x4 v = store_qb<SB>(d_p + j * 16 * EB, acc[j][i] + bias4[j]);
                if constexpr (SB) acc[j][i] = v;  // the statistics / BN-backward sums see the stored values
            }
        }
        if constexpr (TW == 16) d_p += d_row;
    }
    if constexpr (SB) {
#pragma unroll
        for (int j = 0; j < TN; ++j) bias4[j] = f32x4{0.f, 0.f, 0.f, 0.f};  // already in acc
    }
    // The stored value of tile (j, i): acc + bias (bf16 storage: acc already holds it, and x + 0 would only turn -0
    // into +0, which neither a sum, a squared deviation nor a magnitude can see).
    auto stored = [&](int j, int i) -> f32x4 {
        if constexpr (SB)
            return acc[j][i];
        else
            return acc[j][i] + bias4[j];
    };
    if (a.dst_bound) {  // uniform: every lane of the wave takes part; skipped where no consumer needs a bound (bf16)
        float omax = 0.f;  // max |stored value| of this lane
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                if (nq + j * 16 < a.n_out) {
                    const f32x4 v = stored(j, i);
                    omax = fmaxf(omax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
                }
        wave_max_bound(a.dst_bound, fmaxf(omax, bound_seed(a)));
    }

    // The epilogue reductions below run on channel quads (f32x4: the adds, multiplies and fmas issue as packed
    // two-float instructions); every component follows the scalar order of bn_bwd_partial / the statistics merge, so
    // the records are unchanged.
    // Fused BatchNorm statistics of this tile (BM pixels of one image) per channel: mean, then M2 about it.
    if (a.stat_rec) {
        float *red1 = reinterpret_cast<float *>(smem);  // [WME][BN] sums
        float *red2 = red1 + WME * BN;                  // [WME][BN] M2
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int q = 0; q < RG; ++q) {
                f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int i = q * TMG; i < (q + 1) * TMG; ++i) s4 += stored(j, i);
                const f32x4 t = row16_sum4(s4);
                if (l16 == 0) *reinterpret_cast<f32x4 *>(&red1[(wm * RG + q) * BN + wn * WCH + j * 16 + 4 * g]) = t;
            }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int nl = wn * WCH + j * 16 + 4 * g;
            f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int w = 0; w < WME; ++w) s4 += *reinterpret_cast<const f32x4 *>(&red1[w * BN + nl]);
            const f32x4 mean4 = s4 * (1.f / float(BM));
#pragma unroll
            for (int qg = 0; qg < RG; ++qg) {
                f32x4 q4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int i = qg * TMG; i < (qg + 1) * TMG; ++i) {
                    const f32x4 d = stored(j, i) - mean4;
                    q4 = __builtin_elementwise_fma(d, d, q4);
                }
                const f32x4 t = row16_sum4(q4);
                if (l16 == 0) *reinterpret_cast<f32x4 *>(&red2[(wm * RG + qg) * BN + nl]) = t;
            }
        }
        __syncthreads();
        for (int nl = tid; nl < BN; nl += NT) {
            if (n0 + nl >= a.n_out) continue;
            float s = 0.f, m2 = 0.f;
#pragma unroll
            for (int w = 0; w < WME; ++w) {
                s += red1[w * BN + nl];
                m2 += red2[w * BN + nl];
            }
            float *rec = a.stat_rec + (size_t(mt) * a.n_out + n0 + nl) * 2;
            rec[0] = s * (1.f / float(BM));
            rec[1] = m2;
        }
    }

    // Fused BatchNorm + ReLU backward partial sums of the stored g over this tile (exclusive with stat_rec):
    // {sum dz, sum dz * xhat} with the expressions of bn_bwd_partial (bn_f32.hip) -> bb_rec[c][tile][2].
    if (a.bb_rec) {
        float *red1 = reinterpret_cast<float *>(smem);  // [WME][BN]
        float *red2 = red1 + WME * BN;
        const int co = (img / a.bb_seg_imgs) * a.n_out;
        const unsigned char *const y_b = reinterpret_cast<const unsigned char *>(a.bb_y);
        const size_t y_row = size_t(a.wo) * a.bb_ldy * EB;  // TW == 16: as the stores above
        const unsigned char *const y_p0 = y_b + (row_pix(0) * a.bb_ldy + nq) * EB;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = nq + j * 16;
            const bool nok = n < a.n_out;
            const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
            const f32x4 mu = nok ? gload4(a.bb_mean + co + n) : z4, iv = nok ? gload4(a.bb_inv + co + n) : z4;
            const f32x4 sc = nok ? gload4(a.bb_scale + co + n) : z4, sf = nok ? gload4(a.bb_shift + co + n) : z4;
#pragma unroll
            for (int qg = 0; qg < RG; ++qg) {
                f32x4 s1 = z4, s2 = z4;
#pragma unroll
                for (int i = qg * TMG; i < (qg + 1) * TMG; ++i) {
                    const unsigned char *const yp = TW == 16 ? y_p0 + size_t(i) * y_row + j * 16 * EB
                                                             : y_b + (row_pix(i) * a.bb_ldy + n) * EB;
                    const f32x4 y4 = nok ? load_qb<SB>(yp) : z4;
                    const f32x4 t = __builtin_elementwise_fma(y4, sc, sf);  // the forward's exact ReLU test
                    const f32x4 dz = {t[0] > 0.f ? acc[j][i][0] : 0.f, t[1] > 0.f ? acc[j][i][1] : 0.f,
                                      t[2] > 0.f ? acc[j][i][2] : 0.f, t[3] > 0.f ? acc[j][i][3] : 0.f};
                    s1 += dz;
                    s2 = __builtin_elementwise_fma(dz, (y4 - mu) * iv, s2);  // s2 += dz * xhat, contracted
                }
                const f32x4 t1 = row16_sum4(s1);
                const f32x4 t2 = row16_sum4(s2);
                if (l16 == 0) {
                    *reinterpret_cast<f32x4 *>(&red1[(wm * RG + qg) * BN + wn * WCH + j * 16 + 4 * g]) = t1;
                    *reinterpret_cast<f32x4 *>(&red2[(wm * RG + qg) * BN + wn * WCH + j * 16 + 4 * g]) = t2;
                }
            }
        }
        __syncthreads();
        for (int nl = tid; nl < BN; nl += NT) {
            if (n0 + nl >= a.n_out) continue;
            float t1 = 0.f, t2 = 0.f;
#pragma unroll
            for (int w = 0; w < WME; ++w) {
                t1 += red1[w * BN + nl];
                t2 += red2[w * BN + nl];
            }
            float *rec = a.bb_rec + (size_t(n0 + nl) * a.bb_ntiles + mt) * 2;
            rec[0] = t1;
            rec[1] = t2;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Warp-specialized h2 halo forward / data grad (SCD_TUNE_HALO16_WS): WAVES_N compute waves of 128 px x 32 ch (the
// 1 x N wave tiles of igemm_halo16_x3) plus one producer wave per block.  The producer alone loads each 32-channel
// chunk's halo, applies the input transform, splits it into the fp16 h / pre-scaled m planes and writes them into the
// other of two LDS buffers while the compute waves run the current chunk.  The compute waves' only vector-memory stream
// is their own weight fragments, one k-step ahead: vmcnt retires in order per wave, so in igemm_halo16_x3 every weight
// wait also drained the next chunk's halo loads (about one k-step of MFMAs to hide an HBM latency); here those loads
// belong to a wave that waits for nothing else.  One barrier per chunk.  Same products, reduction order and epilogue as
// igemm_halo16_x3<..., NP = 4> (bit-identical outputs and records).
// ------------------------------------------------------------------------------------------------
template <int WAVES_N, int TM, int TN, int TW, int OCC, bool IN_BN>
__global__ __launch_bounds__(64 * (WAVES_N + 1), OCC) void igemm_halo16_ws(IgemmArgs a) {
    constexpr int NT = 64 * (WAVES_N + 1);
    constexpr int WPX = TM * 16, WCH = TN * 16;
    constexpr int BM = WPX, BN = WAVES_N * WCH;
    constexpr int TR = BM / TW;
    constexpr int HWD = TW + 2;
    constexpr int HR = (TR + 2) * HWD;
    constexpr int A_CH = HR * 8;               // 16-byte (4-channel) pieces of one 32-channel chunk
    constexpr int P_PER = (A_CH + 63) / 64;    // per producer lane
    constexpr int PA = HR * 64;                // one plane
    constexpr int BUF = 2 * PA;                // h and m planes
    constexpr int RG = TM >= 8 ? TM / 4 : 1;   // reduction groups per wave (igemm_halo16_x3's order)
    constexpr int TMG = TM / RG;
    constexpr int WME = RG;                    // reduction rows of the block (one wave row)
    constexpr int RED = 2 * WME * BN * 4;
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BUF > RED ? 2 * BUF : RED];
    float xs = 1.f, xs_inv = 1.f;
    h2_scale(*a.src_bound, xs, xs_inv);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: the role branch is scalar
    const bool producer = wid == WAVES_N;
    const int wn = producer ? 0 : wid;
    const int g = lane >> 4, l16 = lane & 15;
    int mt, nt;
    if (a.remap == 2) {
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
    const int cpk = a.c / 32;
    const int nsteps = cpk * a.ntaps;

    f32x4 acc[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (producer) {
        // ---- the producer: halo of chunk cc + 1 while the compute waves run chunk cc
        auto soff = [](int row, int col) { return row * 64 + ((((col >> 1) ^ (row >> 1)) & 3) << 4) + ((col & 1) << 3); };
        const int col = lane & 7;  // the channel piece of every piece of this lane (e = lane + 64 i)
        uint32_t p_boff[P_PER];
        int p_off[P_PER];
#pragma unroll
        for (int i = 0; i < P_PER; ++i) {
            const int e = lane + i * 64;
            const bool in = e < A_CH;
            const int hp = in ? (e >> 3) : 0;
            const int hy = hp / HWD, hx = hp - (hp / HWD) * HWD;
            const int sy = y0 - 1 + hy, sx = x0 - 1 + hx;
            const bool ok = in && unsigned(sy) < unsigned(a.hs) && unsigned(sx) < unsigned(a.ws);
            p_boff[i] = ok ? uint32_t(((img * a.hs + sy) * a.ws + sx) * a.ldc_s + col * 4) * 4u : kOOB;
            p_off[i] = in ? soff(hp, col) : -1;
        }
        const __amdgpu_buffer_rsrc_t rs_src = make_rsrc(a.src, a.src_bytes);
        f32x4 ra[P_PER];
        f32x4 in_sc, in_sh;
        auto pload = [&](int cc) {
#pragma unroll
            for (int i = 0; i < P_PER; ++i) ra[i] = bload4(rs_src, p_boff[i] == kOOB ? kOOB : p_boff[i] + cc * 128u);
            if constexpr (IN_BN) {
                const int ch = (img / a.in_seg_imgs) * a.c + cc * 32 + col * 4;
                in_sc = gload4(a.in_scale + ch) * xs;  // fma(y, sc s, sh s) == s fma(y, sc, sh): s a power of two
                in_sh = gload4(a.in_shift + ch) * xs;
            }
        };
        auto pstore = [&](int buf) {
            unsigned char *const sb = smem + buf * BUF;
#pragma unroll
            for (int i = 0; i < P_PER; ++i)
                if ((A_CH % 64 == 0) || p_off[i] >= 0) {
                    f32x4 x = ra[i];
                    if constexpr (IN_BN) {
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            x[q] = p_boff[i] == kOOB ? 0.f : fmaxf(fmaf(x[q], in_sc[q], in_sh[q]), 0.f);
                    } else {
                        x *= xs;
                    }
                    u32x2 h, m;
                    split2h_pre(x, h, m);
                    *reinterpret_cast<u32x2 *>(sb + p_off[i]) = h;
                    *reinterpret_cast<u32x2 *>(sb + PA + p_off[i]) = m;
                }
        };
        pload(0);
        pstore(0);
        __syncthreads();  // buffer 0 holds chunk 0
        for (int cc = 0; cc < cpk; ++cc) {
            if (cc + 1 < cpk) {
                pload(cc + 1);
                pstore((cc + 1) & 1);  // the buffer chunk cc - 1 used: every compute wave left it (last barrier)
            }
            __syncthreads();  // end of chunk cc
        }
    } else {
        // ---- a compute wave: 128 px x 32 ch, weights one k-step ahead in registers
        const int KS16 = a.K / 16, NB32 = (a.n_out + 31) / 32;
        const uint32_t wplane_b = uint32_t(a.wplane) * 2u;
        uint32_t w_base[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int cb = (n0 >> 4) + wn * TN + j;
            const int nb = cb >> 1;
            w_base[j] = nb < NB32 ? uint32_t(nb * KS16 + (g >> 1)) * 1024u +
                                        uint32_t(16 * (cb & 1) + l16 + 32 * (g & 1)) * 16u
                                  : kOOB;
        }
        const __amdgpu_buffer_rsrc_t rs_w = make_rsrc(a.wsplit, 2u * wplane_b);
        auto load_W = [&](int cc, int t, u32x4 (&wq)[2][TN]) {
            const uint32_t ko = uint32_t(t * cpk + cc) * 2048u;
#pragma unroll
            for (int p = 0; p < 2; ++p)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    wq[p][j] = bload4u(rs_w, w_base[j] == kOOB ? kOOB : w_base[j] + ko + uint32_t(p) * wplane_b);
        };
        int a_hr[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int p = i * 16 + l16;
            a_hr[i] = (p / TW + 1) * HWD + (p % TW) + 1;
        }
        u32x4 wq[2][TN];
        load_W(0, 0, wq);
        __syncthreads();  // buffer 0 holds chunk 0
        int cc = 0, t = 0;
        for (int s = 0; s < nsteps; ++s) {
            int t1 = t + 1, cc1 = cc;
            if (t1 == a.ntaps) {
                t1 = 0;
                cc1 = cc + 1;
            }
            const unsigned char *const sbuf = smem + (cc & 1) * BUF;
            const int toff = tap_at(a.tdy, t) * HWD + tap_at(a.tdx, t);
            u32x4 wh[TN], wm_[TN], wl[TN];
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                wh[j] = wq[0][j];
                wm_[j] = wq[1][j];
                wl[j] = f16_down11(wh[j]);
            }
            if (s + 1 < nsteps) load_W(cc1, t1, wq);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int hr = a_hr[i] + toff;
                const int ad = hr * 64 + (((g ^ (hr >> 1)) & 3) << 4);
                const u32x4 xh = *reinterpret_cast<const u32x4 *>(sbuf + ad);
                const u32x4 xm = *reinterpret_cast<const u32x4 *>(sbuf + PA + ad);
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[j][i] = mfma16_f16(wl[j], xm, acc[j][i]);
                    acc[j][i] = mfma16_f16(wm_[j], xh, acc[j][i]);
                    acc[j][i] = mfma16_f16(wh[j], xh, acc[j][i]);
                }
            }
            if (t1 == 0) __syncthreads();  // end of chunk cc: the producer has written chunk cc + 1
            t = t1;
            cc = cc1;
        }
        // undo the operand scales: per-channel weight inverse scales after the planes
        const float *winv = reinterpret_cast<const float *>(reinterpret_cast<const unsigned char *>(a.wsplit) +
                                                            2u * wplane_b);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * WCH + j * 16 + 4 * g;
            const f32x4 sc = (n < NB32 * 32 ? gload4(winv + n) : f32x4{0.f, 0.f, 0.f, 0.f}) * xs_inv;
#pragma unroll
            for (int i = 0; i < TM; ++i) acc[j][i] *= sc;
        }
    }

    // ---- epilogue (igemm_halo16_x3's, the producer joining its barriers only)
    f32x4 bias4[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WCH + j * 16 + 4 * g;
        bias4[j] = (!producer && a.bias && n < a.n_out) ? *reinterpret_cast<const f32x4 *>(a.bias + n)
                                                        : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    float omax = 0.f;
    if (!producer) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int p = i * 16 + l16;
            const size_t pix = size_t(img * a.ho + y0 + p / TW) * a.wo + x0 + (p % TW);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int n = n0 + wn * WCH + j * 16 + 4 * g;
                if (n < a.n_out) {
                    const f32x4 v = acc[j][i] + bias4[j];
                    gstore4(a.dst + pix * a.ldc_d + n, v);
                    omax = fmaxf(omax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
                }
            }
        }
    }
    if (a.dst_bound) wave_max_bound(a.dst_bound, fmaxf(omax, bound_seed(a)));  // uniform per wave; the producer adds 0

    if (a.stat_rec) {
        float *red1 = reinterpret_cast<float *>(smem);  // [WME][BN] sums
        float *red2 = red1 + WME * BN;                  // [WME][BN] M2
        if (!producer) {
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int q = 0; q < RG; ++q) {
                        float sm = 0.f;
#pragma unroll
                        for (int i = q * TMG; i < (q + 1) * TMG; ++i) sm += acc[j][i][r] + bias4[j][r];
                        sm = row16_sum(sm);
                        if (l16 == 0) red1[q * BN + wn * WCH + j * 16 + 4 * g + r] = sm;
                    }
        }
        __syncthreads();
        if (!producer) {
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int nl = wn * WCH + j * 16 + 4 * g + r;
                    float sm = 0.f;
#pragma unroll
                    for (int w = 0; w < WME; ++w) sm += red1[w * BN + nl];
                    const float mean = sm * (1.f / float(BM));
#pragma unroll
                    for (int qg = 0; qg < RG; ++qg) {
                        float q = 0.f;
#pragma unroll
                        for (int i = qg * TMG; i < (qg + 1) * TMG; ++i) {
                            const float d = (acc[j][i][r] + bias4[j][r]) - mean;
                            q = fmaf(d, d, q);
                        }
                        q = row16_sum(q);
                        if (l16 == 0) red2[qg * BN + nl] = q;
                    }
                }
        }
        __syncthreads();
        for (int nl = tid; nl < BN; nl += NT) {
            if (n0 + nl >= a.n_out) continue;
            float sm = 0.f, m2 = 0.f;
#pragma unroll
            for (int w = 0; w < WME; ++w) {
                sm += red1[w * BN + nl];
                m2 += red2[w * BN + nl];
            }
            float *rec = a.stat_rec + (size_t(mt) * a.n_out + n0 + nl) * 2;
            rec[0] = sm * (1.f / float(BM));
            rec[1] = m2;
        }
    }

    if (a.bb_rec) {
        float *red1 = reinterpret_cast<float *>(smem);
        float *red2 = red1 + WME * BN;
        if (!producer) {
            const int co = (img / a.bb_seg_imgs) * a.n_out;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int n = n0 + wn * WCH + j * 16 + 4 * g;
                const bool nok = n < a.n_out;
                const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
                const f32x4 mu = nok ? gload4(a.bb_mean + co + n) : z4, iv = nok ? gload4(a.bb_inv + co + n) : z4;
                const f32x4 sc = nok ? gload4(a.bb_scale + co + n) : z4, sf = nok ? gload4(a.bb_shift + co + n) : z4;
#pragma unroll
                for (int qg = 0; qg < RG; ++qg) {
                    f32x4 s1 = z4, s2 = z4;
#pragma unroll
                    for (int i = qg * TMG; i < (qg + 1) * TMG; ++i) {
                        const int p = i * 16 + l16;
                        const size_t pix = size_t(img * a.ho + y0 + p / TW) * a.wo + x0 + (p % TW);
                        const f32x4 y4 = nok ? gload4(a.bb_y + pix * a.bb_ldy + n) : z4;
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const float dz = fmaf(y4[r], sc[r], sf[r]) > 0.f ? acc[j][i][r] : 0.f;
                            s1[r] += dz;
                            s2[r] += dz * ((y4[r] - mu[r]) * iv[r]);
                        }
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float t1 = row16_sum(s1[r]), t2 = row16_sum(s2[r]);
                        if (l16 == 0) {
                            red1[qg * BN + wn * WCH + j * 16 + 4 * g + r] = t1;
                            red2[qg * BN + wn * WCH + j * 16 + 4 * g + r] = t2;
                        }
                    }
                }
            }
        }
        __syncthreads();
        for (int nl = tid; nl < BN; nl += NT) {
            if (n0 + nl >= a.n_out) continue;
            float t1 = 0.f, t2 = 0.f;
#pragma unroll
            for (int w = 0; w < WME; ++w) {
                t1 += red1[w * BN + nl];
                t2 += red2[w * BN + nl];
            }
            float *rec = a.bb_rec + (size_t(n0 + nl) * a.bb_ntiles + mt) * 2;
            rec[0] = t1;
            rec[1] = t2;
        }
    }
}

namespace {

struct H16Cfg {
    int id, bm, bn;
};

// 0 = off (the 32x32x16 halo kernel), 1 = automatic tile choice, 2 + id = force tile config id
// (SCD_TUNE_HALO16_* bits of the launch).
int halo16_mode(uint32_t tune) {
    const uint32_t v = tune & SCD_TUNE_HALO16_MASK;
    return v == SCD_TUNE_HALO16_OFF ? 0 : (v == 0 || v == SCD_TUNE_HALO16_WRING) ? 1 : int(v) + 1;
}
// SCD_TUNE_HALO16_WRING: automatic tiles, h2 weights through the LDS ring (igemm_halo16_x3's WL).
bool halo16_wring(uint32_t tune) { return (tune & SCD_TUNE_HALO16_MASK) == SCD_TUNE_HALO16_WRING; }

template <int WM, int WN, int TM, int TN, int OCC, bool IN_BN, bool DB, int NP, bool SB = false, bool WL = false>
void launch16b(const IgemmArgs &a, int tw, hipStream_t s) {
    constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
    IgemmArgs b = a;
    b.grid_m = a.n_img * (a.ho / (BM / tw)) * (a.wo / tw);
    b.grid_n = (a.n_out + BN - 1) / BN;
    b.remap = halo_remap(a.tune);
    const dim3 grid(b.grid_m * b.grid_n), block(64 * WM * WN);
    if (tw == 64) {
        if constexpr (!WL)  // (the launcher keeps the weight ring off 64-wide tiles)
            hipLaunchKernelGGL((igemm_halo16_x3<WM, WN, TM, TN, 64, OCC, IN_BN, DB, NP, SB>), grid, block, 0, s, b);
    } else if (tw == 32)
        hipLaunchKernelGGL((igemm_halo16_x3<WM, WN, TM, TN, 32, OCC, IN_BN, DB, NP, SB, WL>), grid, block, 0, s, b);
    else
        hipLaunchKernelGGL((igemm_halo16_x3<WM, WN, TM, TN, 16, OCC, IN_BN, DB, NP, SB, WL>), grid, block, 0, s, b);
}

// h2: the activation / gradient operand's low term pre-scaled by 2^11 (x3_common.h; floor 2^-36 instead of 2^-25
// of the scaled bound): h2_prescale(tune), conv_common.h (SCD_TUNE_H2_NO_PRESCALE drops it).

// h2, >= 128 output channels: the 1 x 4 wave layout of the 128 x 128 tile (SCD_TUNE_H2_TILE_2X2: 2 x 2).
int h2_wide_tile(uint32_t tune) { return (tune & SCD_TUNE_H2_TILE_2X2) ? 0 : 1; }

// h2, 64..127 output channels: the 1 x 2 wave layout of the 128 x 64 tile (config 4: no weight fragment loaded by two
// waves; same-box A/B 31.81 -> 31.49 ms per step); SCD_TUNE_H2_TILE64_2X2: 2 x 2 waves (config 1).
int h2_tile64(uint32_t tune) { return (tune & SCD_TUNE_H2_TILE64_2X2) ? 0 : 1; }

// Double buffering where two halo buffers of every resident block still fit the CU's 160 KB of LDS: for x3 / x5 /
// bf16; h2 runs single-buffered (same-box A/B: data grad -2.3%, step +0.5%).  SCD_TUNE_HALO16_DB_ON / _OFF force it.
int halo16_db(uint32_t tune, bool h2) {
    if (tune & SCD_TUNE_HALO16_DB_OFF) return 0;
    if (tune & SCD_TUNE_HALO16_DB_ON) return 1;
    return h2 ? 0 : 1;
}

template <int WM, int WN, int TM, int TN, int OCC, bool DB, int NP, bool WL = false>
void launch16c(const IgemmArgs &a, int tw, hipStream_t s) {
    if constexpr (NP == 1) {  // the bf16 arithmetic: fp32 or bf16 storage
        if (a.sb) {
            if (a.in_scale)
                launch16b<WM, WN, TM, TN, OCC, true, DB, NP, true>(a, tw, s);
            else
                launch16b<WM, WN, TM, TN, OCC, false, DB, NP, true>(a, tw, s);
            return;
        }
    }
    if (a.in_scale)
        launch16b<WM, WN, TM, TN, OCC, true, DB, NP, false, WL>(a, tw, s);
    else
        launch16b<WM, WN, TM, TN, OCC, false, DB, NP, false, WL>(a, tw, s);
}

template <int WM, int WN, int TM, int TN, int OCC>
void launch16(const IgemmArgs &a, int tw, hipStream_t s) {
    constexpr int BM = WM * TM * 16;
    const int hr = (BM / tw + 2) * (tw + 2);
    const bool db3 = tw != 64 && halo16_db(a.tune, false) && OCC * 2 * 3 * hr * 64 <= 160 * 1024;
    const bool db_h2 = tw != 64 && halo16_db(a.tune, true) && OCC * 2 * 2 * hr * 64 <= 160 * 1024;
    // h2 needs the h2 weight split and a bound (igemm_takes_halo16); otherwise x3 (h2 mode: other shapes)
    const int planes = a.src_bound && h2_weight_format(a.math, a.ntaps, a.c) ? (h2_prescale(a.tune) ? 4 : 2)
                       : math_planes(a.math) == 2                            ? 3
                                                                             : math_planes(a.math);
    switch (planes) {
        case 1:  // one plane: double buffering always fits
            if (halo16_db(a.tune, false))
                launch16c<WM, WN, TM, TN, OCC, true, 1>(a, tw, s);
            else
                launch16c<WM, WN, TM, TN, OCC, false, 1>(a, tw, s);
            break;
        case 2:
            if (db_h2)
                launch16c<WM, WN, TM, TN, OCC, true, 2>(a, tw, s);
            else
                launch16c<WM, WN, TM, TN, OCC, false, 2>(a, tw, s);
            break;
        case 4:
            if (db_h2)
                launch16c<WM, WN, TM, TN, OCC, true, 4>(a, tw, s);
            else
                launch16c<WM, WN, TM, TN, OCC, false, 4>(a, tw, s);
            break;
        case 5:
            if (db3)
                launch16c<WM, WN, TM, TN, OCC, true, 5>(a, tw, s);
            else
                launch16c<WM, WN, TM, TN, OCC, false, 5>(a, tw, s);
            break;
        default:
            if (db3)
                launch16c<WM, WN, TM, TN, OCC, true, 3>(a, tw, s);
            else
                launch16c<WM, WN, TM, TN, OCC, false, 3>(a, tw, s);
    }
}

// Tile configurations: id -> (pixels, channels) per block.
//   0: 2x2 waves of 64 px x 64 ch  (128 x 128), 2 waves/SIMD
//   1: 2x2 waves of 64 px x 32 ch  (128 x 64),  3 waves/SIMD
//   2: 2x2 waves of 32 px x 64 ch  (64 x 128),  3 waves/SIMD
//   3: 1x4 waves of 128 px x 32 ch (128 x 128), 2 waves/SIMD, h2 only (no duplicated weight loads)
//   4: 1x2 waves of 128 px x 32 ch (128 x 64),  2 waves/SIMD, h2 only (the same wave tile on 64-channel outputs)
//   5: 2x2 waves of 128 px x 32 ch (256 x 64),  2 waves/SIMD, h2 only (the wave tile of config 4 on a 16 x 16 pixel
//      patch, whose halo is 1.27 rows per pixel instead of 1.41: 64-channel sources; SCD_TUNE_H2_TILE64_128 keeps 4)
constexpr H16Cfg kCfg[] = {{0, 128, 128}, {1, 128, 64}, {2, 64, 128}, {3, 128, 128}, {4, 128, 64}, {5, 256, 64}};

// The 1 x N wave tiles: the h2 arithmetic only (bf16 on them measured slower: 21.38 vs 21.05 ms per bf16 step,
// the 64-channel layers -5..-15%, same-box A/B, round 3; not kept).
template <int WM, int WN, int TM, int TN, int OCC>
void launch16_1xn(const IgemmArgs &a, int tw, hipStream_t s) {
    constexpr int BM = WM * TM * 16;
    const int hr = (BM / tw + 2) * (tw + 2);
    const bool db2 = tw != 64 && halo16_db(a.tune, true) && OCC * 2 * 2 * hr * 64 <= 160 * 1024;
    if (db2)
        launch16c<WM, WN, TM, TN, OCC, true, 4>(a, tw, s);
    else if (halo16_wring(a.tune) && a.ntaps == 9 && tw != 64 && a.n_out % (WN * TN * 16) == 0)  // pieces in the split;
        // 64-wide tiles: halo + ring would leave one block per CU
        launch16c<WM, WN, TM, TN, OCC, false, 4, true>(a, tw, s);
    else
        launch16c<WM, WN, TM, TN, OCC, false, 4>(a, tw, s);
}

// Whether the 1 x N wave tiles (ids 3, 4) may run: h2 with its weight split, a bound and the pre-scaled low term.
bool wide_1xn_ok(const IgemmArgs &a) {
    return a.src_bound && h2_weight_format(a.math, a.ntaps, a.c) && h2_prescale(a.tune);
}
// The bf16 arithmetic on the 1 x N tiles: one wave per weight fragment, no fragment loaded by two waves.  The default
// with bf16 storage (round 5: baseline_dualstream bs=64 42.23 -> 41.77 ms per step, same-process A/B,
// profiles/r05_bf16_tiles_ab.txt; round 4: +0.45%); the 2 x 2 tiles with fp32 storage (round 3: the 1 x N tiles 1.6%
// slower there).  SCD_TUNE_BF16_1XN flips the choice (A/B).
bool bf16_1xn(const IgemmArgs &a) {
    return a.math == SCD_MATH_BF16 && (bool(a.sb) != bool(a.tune & SCD_TUNE_BF16_1XN));
}

// The 1 x N tiles in the bf16 arithmetic (fp32 or bf16 storage).  Double-buffered halo on the tiles of 128 and more
// channels; the 64-channel tiles (256 x 64, 128 x 64) single-buffered: there the second buffer cost resident blocks
// (256 x 64: 41 KB per block, 3 blocks per CU; 5 single-buffered) and every block covers only two to eight 32-channel
// chunks.  Round 6, tools/perf_conv.py bf16 storage: enc0b fwd 0.516 -> 0.459 ms, up1b 0.236 -> 0.203, enc1a data grad
// 0.231 -> 0.198 single-buffered, while the 128-channel up3a forward lost 6% (profiles/r06_bf16_halo_db_study.txt).
// Steps (one process, profiles/r06_bf16_halo_db_ab.txt): dual-stream bs=64 40.29 -> 39.75 ms, MMCR 56.94 -> 56.28,
// bf16 Siamese 15.17 -> 15.02 (every tile single-buffered: 40.00, 56.49, 15.18).
// SCD_TUNE_HALO16_DB_ON / _OFF force one choice for every tile.
template <int WM, int WN, int TM, int TN, int OCC>
void launch16_1xn_bf16(const IgemmArgs &a, int tw, hipStream_t s) {
    const bool db = (a.tune & (SCD_TUNE_HALO16_DB_ON | SCD_TUNE_HALO16_DB_OFF)) ? halo16_db(a.tune, false) != 0
                                                                                  : WN * TN * 16 >= 128;
    if (db)
        launch16c<WM, WN, TM, TN, OCC, true, 1>(a, tw, s);
    else
        launch16c<WM, WN, TM, TN, OCC, false, 1>(a, tw, s);
}

// The warp-specialized form of the 1 x N tiles (igemm_halo16_ws): WN compute waves + one producer wave per block.
template <int WN, int TM, int TN, int OCC, bool IN_BN>
void launch_ws_b(const IgemmArgs &a, int tw, hipStream_t s) {
    constexpr int BM = TM * 16, BN = WN * TN * 16;
    IgemmArgs b = a;
    b.grid_m = a.n_img * (a.ho / (BM / tw)) * (a.wo / tw);
    b.grid_n = (a.n_out + BN - 1) / BN;
    b.remap = halo_remap(a.tune);
    const dim3 grid(b.grid_m * b.grid_n), block(64 * (WN + 1));
    (void)tw;  // 16: halo16_ws only takes maps tiled by 16-wide tiles (halo16_pick's first choice)
    hipLaunchKernelGGL((igemm_halo16_ws<WN, TM, TN, 16, OCC, IN_BN>), grid, block, 0, s, b);
}
template <int WN, int TM, int TN, int OCC>
void launch_ws(const IgemmArgs &a, int tw, hipStream_t s) {
    if (a.in_scale)
        launch_ws_b<WN, TM, TN, OCC, true>(a, tw, s);
    else
        launch_ws_b<WN, TM, TN, OCC, false>(a, tw, s);
}
bool halo16_ws(const IgemmArgs &a) {
    return (a.tune & SCD_TUNE_HALO16_WS) && wide_1xn_ok(a) && !a.sb && a.wo % 16 == 0 && a.ho % 8 == 0;
}

}  // namespace

// 0 when `a` does not take this kernel, else 1 + config id; *bm = pixels per tile, *tw = tile width.
int halo16_pick(const IgemmArgs &a, bool eligible, int *bm, int *tw) {
    const int mode = halo16_mode(a.tune);
    if (!mode || !eligible || a.c % 32 || a.n_out % 4 || a.ldc_d % 4 ||
        (reinterpret_cast<uintptr_t>(a.dst) & (a.sb ? 7 : 15)) || (a.bias && (reinterpret_cast<uintptr_t>(a.bias) & 15)) ||
        (a.sb && a.math != SCD_MATH_BF16))
        return 0;
    int id;
    if (mode >= 2)
        id = mode - 2;
    else if (a.n_out >= 128)
        // 128 x 128 at 2 waves/SIMD: +4..17% over the 32x32x16 halo kernel on the 128..512-channel layers; under h2
        // as 1 x 4 waves of 128 px x 32 ch (no weight fragment loaded by two waves; SCD_H2_TILE=0: 2 x 2)
        id = ((wide_1xn_ok(a) && h2_wide_tile(a.tune)) || bf16_1xn(a)) ? 3 : 0;
    else if (a.n_out >= 64)
        // 128 x 64 at 3 waves/SIMD: +3..9% on the 64-channel layers
        // h2 on 1 x 2 waves; 64-channel sources (K = 576, two 32-channel chunks) on the 256 x 64 tile of 2 x 2 such
        // waves (enc0b fwd / dgrad -4..-5%, up2b -2%; 128- and 256-channel sources measured neutral or slower)
        // (bf16 storage too: the 128 x 64 tile ran its layers 10-14% faster in isolation but the step 0.6% slower,
        // profiles/r06_bf16_tile64_study.txt)
        id = ((wide_1xn_ok(a) && h2_tile64(a.tune)) || bf16_1xn(a))
                 ? ((a.c == 64 && !(a.tune & SCD_TUNE_H2_TILE64_128)) ? 5 : 4)
                 : 1;
    else
        return 0;
    if (id < 0 || id > 5 || (id > 2 && !wide_1xn_ok(a) && !bf16_1xn(a))) return 0;
    if (id == 5 && halo16_ws(a)) id = 4;  // the warp-specialized blocks tile 128 pixels
    for (;;) {
        *bm = kCfg[id].bm;
        const int pref = 16;  // preferred tile width, the smallest halo per pixel (180 rows for 128 px)
        for (int cand : {pref, 64, 32, 16})
            if (a.wo % cand == 0 && a.ho % (*bm / cand) == 0 && *bm / cand >= 1 && *bm % cand == 0) {
                *tw = cand;
                return 1 + id;
            }
        if (id != 5) return 0;
        id = 4;  // the 256-pixel patch does not tile this map: the 128-pixel one
    }
}

// bf16 outputs of 256 channels and more on 1 x 4 waves of 128 px x 64 ch (128 x 256 per block, two blocks per CU) when
// that grid has at least SCD_HALO16_BF16_TN4 blocks: a pixel fragment read from LDS feeds four weight fragments instead
// of two, and the block's fixed prologue / epilogue cost covers twice the MFMAs.  Same products in the same order
// (bit-identical).  Alternating processes (profiles/r05_bf16_tn4_ab.txt): dual-stream bs=64 40.59 -> 40.25 ms, MMCR
// 57.71 -> 56.97 ms, bf16 Siamese bs=32 15.33 -> 15.21 ms; a 256- or 1-block threshold measured slightly less.
// -DSCD_HALO16_BF16_TN4=0 builds the 128 x 128 tiles only.
#ifndef SCD_HALO16_BF16_TN4
#define SCD_HALO16_BF16_TN4 512
#endif
void launch_halo16(const IgemmArgs &a, int cfg, int tw, hipStream_t s) {
    if (cfg >= 4 && bf16_1xn(a)) {
        switch (cfg - 1) {
            case 3:
                // (automatic tiles only: SCD_TUNE_HALO16_CFG(3) keeps the 128 x 128 tile, the bit-identity tests' A/B)
                if (SCD_HALO16_BF16_TN4 > 0 && halo16_mode(a.tune) == 1 && a.n_out % 256 == 0 &&
                    int64_t(a.n_img) * a.ho * a.wo / 128 * (a.n_out / 256) >= SCD_HALO16_BF16_TN4) {
                    launch16_1xn_bf16<1, 4, 8, 4, 2>(a, tw, s);
                    return;
                }
                launch16_1xn_bf16<1, 4, 8, 2, 3>(a, tw, s);
                return;
            case 4: launch16_1xn_bf16<1, 2, 8, 2, 3>(a, tw, s); return;
            default: launch16_1xn_bf16<2, 2, 8, 2, 3>(a, tw, s); return;
        }
    }
    switch (cfg - 1) {
        case 0: launch16<2, 2, 4, 4, 2>(a, tw, s); break;
        case 1: launch16<2, 2, 4, 2, 3>(a, tw, s); break;
        case 3:
            if (halo16_ws(a))
                launch_ws<4, 8, 2, 2>(a, tw, s);
            else
                launch16_1xn<1, 4, 8, 2, 2>(a, tw, s);
            break;
        case 4:
            if (halo16_ws(a))
                launch_ws<2, 8, 2, 3>(a, tw, s);
            else
                launch16_1xn<1, 2, 8, 2, 2>(a, tw, s);
            break;
        case 5: launch16_1xn<2, 2, 8, 2, 2>(a, tw, s); break;
        default: launch16<2, 2, 2, 4, 3>(a, tw, s); break;
    }
}


// ------------------------------------------------------------------------------------------------
// Halo forward conv of a 16-channel source (the input layer: 5 bands padded to 16).  The 32-deep MFMA step
// of igemm_halo16_x3 would be half padding here, so one step covers two taps instead: lane group g supplies
// k = 8g..8g+7 = tap 2s + (g >> 1), channels 8(g & 1)..+7, and the fragment-major weights (K = tap * 16 + c)
// already hold the two taps' 16-deep fragments back to back.  9 taps = 5 steps; the second tap of the last
// step is masked to zero on both operands.  One 16-channel halo per block ([row][16 bf16], 32-byte rows,
// 16-byte halves swapped by bit 3 of the row: the 16 rows a lane group reads hit 16 distinct bank groups);
// same epilogue (bias, 16-byte stores, fused BatchNorm statistics) as igemm_halo16_x3.
// 2 x 2 waves of 64 px x 32 ch: 128 px x 64 ch per block.
// ------------------------------------------------------------------------------------------------
template <int TW, int NP, bool SB = false>
__global__ __launch_bounds__(256, 2) void igemm_halo16_c16(IgemmArgs a) {
    static_assert(!SB || NP == 1, "bf16 storage runs the bf16 arithmetic");
    constexpr uint32_t EB = SB ? 2u : 4u;
    constexpr int WAVES_M = 2, TM = 4, TN = 2, NT = 256;
    constexpr int WPX = TM * 16, WCH = TN * 16;
    constexpr int BM = WAVES_M * WPX, BN = 2 * WCH;
    constexpr int TR = BM / TW;
    constexpr int HWD = TW + 2;
    constexpr int HR = (TR + 2) * HWD;
    constexpr int A_CH = HR * 4;  // 16-byte (4-channel) pieces
    constexpr int A_PER = (A_CH + NT - 1) / NT;
    constexpr int PA = HR * 32;
    static_assert(NP == 1 || NP == 3 || NP == 4 || NP == 5, "x3, x5, bf16 or h2");
    // NP 4: h2 as in igemm_halo16_x3 (fp16 h and pre-scaled m' planes of the halo scaled by the power of two of
    // *src_bound, the weights' h2 split with its per-channel inverse scales, three f16 products per term pair)
    constexpr bool H2 = NP == 4;
    constexpr int XP = NP == 1 ? 1 : H2 ? 2 : 3;
    constexpr int WP = NP == 1 ? 1 : (NP == 5 || H2) ? 2 : 3;
    // halo planes, then the statistics reduction ([2][WAVES_M][BN] floats) in a region of its own, so the next
    // tile's halo can be written while no wave is still reducing
    __shared__ __attribute__((aligned(16))) unsigned char smem[XP * PA + 2 * WAVES_M * BN * 4];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid % WAVES_M, wn = wid / WAVES_M;
    const int g = lane >> 4, l16 = lane & 15;
    const int tiles_x = a.wo / TW, tiles_y = a.ho / TR;
    const int ntile = a.grid_m * a.grid_n;
    float xs = 1.f, xs_inv = 1.f;  // h2: power-of-two scale of the staged halo and its inverse
    if constexpr (H2) h2_scale(*a.src_bound, xs, xs_inv);

    auto soff = [](int row, int col) { return row * 32 + ((((col >> 1) ^ (row >> 3)) & 1) << 4) + ((col & 1) << 3); };
    // tile -> (m-tile, n-tile): n slowest, so a block's consecutive tiles (stride gridDim.x) keep one weight tile
    auto coords = [&](int tile, int &mt, int &img, int &y0, int &x0, int &n0) {
        const int nt = tile / a.grid_m;
        mt = tile - nt * a.grid_m;
        img = mt / (tiles_x * tiles_y);
        const int trem = mt - img * tiles_x * tiles_y;
        const int ty = trem / tiles_x;
        y0 = ty * TR;
        x0 = (trem - ty * tiles_x) * TW;
        n0 = nt * BN;
    };

    const __amdgpu_buffer_rsrc_t rs_src = make_rsrc(a.src, a.src_bytes);
    StageT<SB> ra[A_PER];
    auto load_halo = [&](int tile) {
        int mt, img, y0, x0, n0;
        coords(tile, mt, img, y0, x0, n0);
#pragma unroll
        for (int i = 0; i < A_PER; ++i) {
            const int e = tid + i * NT;
            const int hp = e < A_CH ? (e >> 2) : 0, col = e & 3;
            const int hy = hp / HWD, hx = hp - (hp / HWD) * HWD;
            const int sy = y0 - 1 + hy, sx = x0 - 1 + hx;
            const bool ok = e < A_CH && unsigned(sy) < unsigned(a.hs) && unsigned(sx) < unsigned(a.ws);
            ra[i] = bload_q<SB>(rs_src, ok ? uint32_t(((img * a.hs + sy) * a.ws + sx) * a.ldc_s + col * 4) * EB : kOOB);
        }
    };
    // weights: the 16 rows x 8 k of lane group g are 256 contiguous bytes of a 1 KB 32x16 fragment; fragment
    // 2s + (g >> 1) of step s
    const int KS16 = a.K / 16, NB32 = (a.n_out + 31) / 32;
    const uint32_t wplane_b = uint32_t(a.wplane) * 2u;
    const __amdgpu_buffer_rsrc_t rs_w = make_rsrc(a.wsplit, uint32_t(WP) * wplane_b);
    uint32_t w_base[TN];
    auto load_W = [&](int st, u32x4 (&wq)[WP][TN]) {
        const bool pad = st == 4 && g >= 2;  // tap 9 does not exist
#pragma unroll
        for (int p = 0; p < WP; ++p)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                wq[p][j] = bload4u(rs_w, (w_base[j] == kOOB || pad) ? kOOB : w_base[j] + uint32_t(st) * 2048u +
                                                                         uint32_t(p) * wplane_b);
    };
    int a_hr[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int p = wm * WPX + i * 16 + l16;
        a_hr[i] = (p / TW + 1) * HWD + (p % TW) + 1;
    }
    float *red1 = reinterpret_cast<float *>(smem + XP * PA);  // [WAVES_M][BN] sums
    float *red2 = red1 + WAVES_M * BN;                         // [WAVES_M][BN] M2

    // Persistent blocks: each walks tiles blockIdx.x, + gridDim.x, ...; the next tile's halo is loaded into
    // registers during this tile's last MFMA step and epilogue.  Every wave of a block runs the same trip count.
    int tile = blockIdx.x;
    if (tile >= ntile) return;
    float omax = 0.f;  // max |stored value| of this lane over its tiles (dst_bound)
    load_halo(tile);
    for (; tile < ntile; tile += gridDim.x) {
        int mt, img, y0, x0, n0;
        coords(tile, mt, img, y0, x0, n0);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int cb = (n0 >> 4) + wn * TN + j;
            const int nb = cb >> 1;
            w_base[j] = nb < NB32 ? uint32_t(nb * KS16 + (g >> 1)) * 1024u +
                                        uint32_t(16 * (cb & 1) + l16 + 32 * (g & 1)) * 16u
                                  : kOOB;
        }
        u32x4 wq[WP][TN];
        load_W(0, wq);
        f32x4 bias4[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * WCH + j * 16 + 4 * g;
            bias4[j] = (a.bias && n < a.n_out) ? *reinterpret_cast<const f32x4 *>(a.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        __syncthreads();  // every wave is done reading the previous tile's halo
#pragma unroll
        for (int i = 0; i < A_PER; ++i) {
            const int e = tid + i * NT;
            if ((A_CH % NT == 0) || e < A_CH) {
                const int o = soff(e >> 2, e & 3);
                u32x2 h, m, l;
                if constexpr (H2) {
                    split2h_pre(ra[i] * xs, h, m);
                    *reinterpret_cast<u32x2 *>(smem + PA + o) = m;
                } else if constexpr (XP == 3) {
                    split3(ra[i], h, m, l);
                    *reinterpret_cast<u32x2 *>(smem + PA + o) = m;
                    *reinterpret_cast<u32x2 *>(smem + 2 * PA + o) = l;
                } else {
                    h = stage_bits<SB>(ra[i]);
                }
                *reinterpret_cast<u32x2 *>(smem + o) = h;
            }
        }
        __syncthreads();
        const bool more = tile + int(gridDim.x) < ntile;

        f32x4 acc[TN][TM];
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int st = 0; st < 5; ++st) {
            const int t = 2 * st + (g >> 1) < 9 ? 2 * st + (g >> 1) : 8;  // the masked lanes read tap 8 again
            const int toff = (t / 3 - 1) * HWD + (t % 3 - 1);
            bf16x8 xv[XP][TM], wv[WP][TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int hr = a_hr[i] + toff;
                const int ad = hr * 32 + ((((g & 1) ^ (hr >> 3)) & 1) << 4);
#pragma unroll
                for (int p = 0; p < XP; ++p) {
                    u32x4 v = *reinterpret_cast<const u32x4 *>(smem + p * PA + ad);
                    if (st == 4 && g >= 2) v = u32x4{0u, 0u, 0u, 0u};
                    xv[p][i] = __builtin_bit_cast(bf16x8, v);
                }
            }
#pragma unroll
            for (int p = 0; p < WP; ++p)
#pragma unroll
                for (int j = 0; j < TN; ++j) wv[p][j] = __builtin_bit_cast(bf16x8, wq[p][j]);
            if constexpr (H2) {
                // (w_h 2^-11) x_m', w_m x_h, w_h x_h on the fp16 planes (igemm_halo16_x3's NP 4)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const u32x4 wh = __builtin_bit_cast(u32x4, wv[0][j]), wmv = __builtin_bit_cast(u32x4, wv[1][j]);
                    const u32x4 wh_lo = f16_down11(wh);
#pragma unroll
                    for (int i = 0; i < TM; ++i) {
                        const u32x4 xh = __builtin_bit_cast(u32x4, xv[0][i]), xm = __builtin_bit_cast(u32x4, xv[1][i]);
                        acc[j][i] = mfma16_f16(wh_lo, xm, acc[j][i]);
                        acc[j][i] = mfma16_f16(wmv, xh, acc[j][i]);
                        acc[j][i] = mfma16_f16(wh, xh, acc[j][i]);
                    }
                }
            } else {
                constexpr int QW[6] = {1, 0, 2, 0, 1, 0};
                constexpr int QX[6] = {1, 2, 0, 1, 0, 0};
#pragma unroll
                for (int q = NP == 1 ? 5 : 0; q < 6; ++q)
                    if (NP != 5 || QW[q] != 2)
#pragma unroll
                        for (int j = 0; j < TN; ++j)
#pragma unroll
                            for (int i = 0; i < TM; ++i)
                                acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[QW[q]][j], xv[QX[q]][i],
                                                                                    acc[j][i], 0, 0, 0);
            }
            if (st < 4) load_W(st + 1, wq);
            if (st == 3 && more) load_halo(tile + gridDim.x);  // issued after the last weight step's loads
        }

        if constexpr (H2) {  // undo the operand scales: per-channel weight inverse scales after the planes
            const float *winv =
                reinterpret_cast<const float *>(reinterpret_cast<const unsigned char *>(a.wsplit) + 2u * wplane_b);
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int n = n0 + wn * WCH + j * 16 + 4 * g;
                const f32x4 sc = (n < NB32 * 32 ? gload4(winv + n) : f32x4{0.f, 0.f, 0.f, 0.f}) * xs_inv;
#pragma unroll
                for (int i = 0; i < TM; ++i) acc[j][i] *= sc;
            }
        }
        // acc[j][i][r]: channel n0 + wn*WCH + 16j + 4g + r, pixel wm*WPX + 16i + l16 (igemm_halo16_x3's epilogue:
        // 16-wide tiles address pixel tile i as one base plus i rows; channel-quad reductions, same order)
        const int nq = n0 + wn * WCH + 4 * g;
        auto row_pix = [&](int i) -> size_t {
            const int p = wm * WPX + i * 16 + l16;
            return size_t(img * a.ho + y0 + p / TW) * a.wo + x0 + (p % TW);
        };
        unsigned char *const dst_b = reinterpret_cast<unsigned char *>(a.dst);
        const size_t d_row = size_t(a.wo) * a.ldc_d * EB;
        unsigned char *d_p = dst_b + (row_pix(0) * a.ldc_d + nq) * EB;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            if constexpr (TW != 16) d_p = dst_b + (row_pix(i) * a.ldc_d + nq) * EB;
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                if (nq + j * 16 < a.n_out) {
                    const f32x4 v = store_qb<SB>(d_p + j * 16 * EB, acc[j][i] + bias4[j]);
                    if constexpr (SB) acc[j][i] = v;  // statistics of the stored values
                    omax = fmaxf(omax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
                }
            }
            if constexpr (TW == 16) d_p += d_row;
        }
        auto stored = [&](int j, int i) -> f32x4 {  // bf16 storage: acc holds the stored value (see igemm_halo16_x3)
            if constexpr (SB)
                return acc[j][i];
            else
                return acc[j][i] + bias4[j];
        };
        if (a.stat_rec) {  // as igemm_halo16_x3: tile mean, then M2 about it
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int i = 0; i < TM; ++i) s4 += stored(j, i);
                const f32x4 t = row16_sum4(s4);
                if (l16 == 0) *reinterpret_cast<f32x4 *>(&red1[wm * BN + wn * WCH + j * 16 + 4 * g]) = t;
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int nl = wn * WCH + j * 16 + 4 * g;
                f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int w = 0; w < WAVES_M; ++w) s4 += *reinterpret_cast<const f32x4 *>(&red1[w * BN + nl]);
                const f32x4 mean4 = s4 * (1.f / float(BM));
                f32x4 q4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const f32x4 d = stored(j, i) - mean4;
                    q4 = __builtin_elementwise_fma(d, d, q4);
                }
                const f32x4 t = row16_sum4(q4);
                if (l16 == 0) *reinterpret_cast<f32x4 *>(&red2[wm * BN + nl]) = t;
            }
            __syncthreads();
            for (int nl = tid; nl < BN; nl += NT) {
                if (n0 + nl >= a.n_out) continue;
                float sm = 0.f, m2 = 0.f;
#pragma unroll
                for (int w = 0; w < WAVES_M; ++w) {
                    sm += red1[w * BN + nl];
                    m2 += red2[w * BN + nl];
                }
                float *rec = a.stat_rec + (size_t(mt) * a.n_out + n0 + nl) * 2;
                rec[0] = sm * (1.f / float(BM));
                rec[1] = m2;
            }
            // the next tile's first barrier orders these red1/red2 reads before the next writes
        }
    }
    if (a.dst_bound) wave_max_bound(a.dst_bound, fmaxf(omax, bound_seed(a)));  // uniform: every lane of the block ran every tile
}

// 0 when `a` does not take igemm_halo16_c16, else 1; *bm = 128 pixels per tile, *tw = tile width.
// SCD_TUNE_NO_HALO16_C16 switches it off (A/B).
int halo16_c16_pick(const IgemmArgs &a, bool eligible, int *bm, int *tw) {
    if (!halo16_mode(a.tune) || !eligible || (a.tune & SCD_TUNE_NO_HALO16_C16) || a.c != 16 || a.K != 144 ||
        a.in_scale || a.bb_rec ||
        a.n_out % 4 || a.ldc_d % 4 || (reinterpret_cast<uintptr_t>(a.dst) & (a.sb ? 7 : 15)) ||
        (a.bias && (reinterpret_cast<uintptr_t>(a.bias) & 15)) || (a.sb && a.math != SCD_MATH_BF16))
        return 0;
    for (int cand : {16, 32, 64})
        if (a.wo % cand == 0 && a.ho % (128 / cand) == 0) {
            *bm = 128;
            *tw = cand;
            return 1;
        }
    return 0;
}

// Arithmetic of the input-layer kernel: the mode's own; h2 with its weight split and a bound of the input (the
// descriptors the x3 view keeps the split for), else x3.
static int c16_planes(const IgemmArgs &b) {
    if (math_planes(b.math) == 2) return b.src_bound && h2_weight_format(b.math, 9, 16) ? 4 : 3;
    return math_planes(b.math);
}

template <int TW>
static void launch_c16_tw(const IgemmArgs &b, dim3 grid, hipStream_t s) {
    switch (c16_planes(b)) {
        case 1:
            if (b.sb)
                hipLaunchKernelGGL((igemm_halo16_c16<TW, 1, true>), grid, dim3(256), 0, s, b);
            else
                hipLaunchKernelGGL((igemm_halo16_c16<TW, 1>), grid, dim3(256), 0, s, b);
            break;
        case 4: hipLaunchKernelGGL((igemm_halo16_c16<TW, 4>), grid, dim3(256), 0, s, b); break;
        case 5: hipLaunchKernelGGL((igemm_halo16_c16<TW, 5>), grid, dim3(256), 0, s, b); break;
        default: hipLaunchKernelGGL((igemm_halo16_c16<TW, 3>), grid, dim3(256), 0, s, b);
    }
}

template <int TW>
static int c16_resident(const IgemmArgs &b) {
    static int cache[4] = {0, 0, 0, 0};  // per arithmetic: bf16, x5, x3, h2
    const int pl = c16_planes(b);
    const int k = pl == 1 ? 0 : pl == 5 ? 1 : pl == 4 ? 3 : 2;
    if (cache[k] > 0) return cache[k];
    const void *fn = k == 0   ? reinterpret_cast<const void *>(&igemm_halo16_c16<TW, 1>)
                     : k == 1 ? reinterpret_cast<const void *>(&igemm_halo16_c16<TW, 5>)
                     : k == 3 ? reinterpret_cast<const void *>(&igemm_halo16_c16<TW, 4>)
                              : reinterpret_cast<const void *>(&igemm_halo16_c16<TW, 3>);
    int per_cu = 0, cus = 0, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, 0) != hipSuccess || per_cu < 1 || cus < 1) {
        (void)hipGetLastError();
        cache[k] = 2 * 256;  // cached: every launch of a shape sees the same capacity
        return cache[k];
    }
    cache[k] = per_cu * cus;
    return cache[k];
}

// Each block walks 4 tiles (measured on the 256^2 input layer, x3 / bf16: 1 tile 0.62 / 0.35 ms, 4 tiles 0.50 /
// 0.31, as many as the resident capacity allows 0.53 / 0.32); SCD_TUNE_C16_TILES(k) overrides, 15 = one resident
// round.
void launch_halo16_c16(const IgemmArgs &a, int tw, hipStream_t s) {
    IgemmArgs b = a;
    b.grid_m = a.n_img * (a.ho / (128 / tw)) * (a.wo / tw);
    b.grid_n = (a.n_out + 63) / 64;
    b.remap = 0;
    const int64_t ntile = int64_t(b.grid_m) * b.grid_n;
    const int cap = tw == 64 ? c16_resident<64>(a) : tw == 32 ? c16_resident<32>(a) : c16_resident<16>(a);
    const int kt = int((a.tune & SCD_TUNE_C16_TILES_MASK) >> 16);
    const int k = kt == 0 ? 4 : kt == 15 ? 0 : kt;
    const int64_t blocks = k >= 1 ? (ntile + k - 1) / k : (ntile < cap ? ntile : cap);
    const dim3 grid(static_cast<unsigned>(blocks));
    if (tw == 64)
        launch_c16_tw<64>(b, grid, s);
    else if (tw == 32)
        launch_c16_tw<32>(b, grid, s);
    else
        launch_c16_tw<16>(b, grid, s);
}

// ------------------------------------------------------------------------------------------------
// Halo weight gradient on v_mfma_f32_16x16x32_bf16 (3x3 / stride 1 / same size, R and C multiples of 64).
//   dW[r][t][c] = sum_p dY[p][r] * X[p + off_t][c]
// Same decomposition as wgrad_halo_x3 (conv_x3.hip): a block owns 64 rows r x 64 channels c x 9 taps and
// walks a range of 2x16-pixel patches (split-K); per patch the dY patch (32 px x 64 r) and the X halo
// (4 x 18 px x 64 c) are staged once, split into bf16 planes, and every tap is a shifted read.
// One MFMA consumes the whole 32-pixel patch as its k.  k = 8g + j of lane group g is pixel
// (g >> 1, 4(g & 1) + (j & 3) + 8(j >> 2)): each 32-lane half of a transposed read then touches 8
// consecutive staged rows, which the 160-byte row stride spreads over the 8 distinct 32-byte bank slots
// (conflict-free for every tap shift).
// Roles: A = X (rows = channels c), B = dY (columns = r), so a lane's result is 4 consecutive c of one r:
// one 16-byte slab store per tile.
// ------------------------------------------------------------------------------------------------
namespace {
constexpr int kW16RS = 160;

// Patch walk of a split (a contiguous range of patch indices): DOWN each 16-pixel column strip of an image, so two
// consecutive patches share two of their four halo rows -- a re-read the L2 still holds one patch later.  The row walk
// (-DSCD_WGRAD_ROW_WALK=1, the round-4 order) re-read those rows a whole strip row (w / 16 patches) later, past the L2
// with ~64 blocks per XCD streaming: the 256^2 weight grads fetched 1.5-1.7x their algorithmic bytes
// (profiles/r05_traffic_table.txt).  Same patches per split, so only the order of the split's accumulation changes.
#ifndef SCD_WGRAD_ROW_WALK
#define SCD_WGRAD_ROW_WALK 0
#endif
__device__ __forceinline__ int patch_y0(int pr, int pw_n, int ph_n, int ph) {
    return SCD_WGRAD_ROW_WALK ? (pr / pw_n) * ph : (pr - (pr / ph_n) * ph_n) * ph;
}
__device__ __forceinline__ int patch_x0(int pr, int pw_n, int ph_n, int pw) {
    return SCD_WGRAD_ROW_WALK ? (pr - (pr / pw_n) * pw_n) * pw : (pr / ph_n) * pw;
}

// X planes of the weight-grad kernel per arithmetic: x3 3, x5 2 (its l term is the dropped product's), bf16 1,
// h2 2 (fp16 h, m).  dY planes: x3 / x5 3, bf16 1, h2 2.
template <int NP>
constexpr int w16_xp() { return NP == 1 ? 1 : (NP == 5 || NP == 2 || NP == 4) ? 2 : 3; }
template <int NP>
constexpr int w16_dp() { return NP == 1 ? 1 : (NP == 2 || NP == 4) ? 2 : 3; }

// Wave layouts of the halo weight grad's 64 r x 64 c block: LC 0 = 2 x 2 waves of 32 r x 32 c (two 16-channel X
// blocks, two 16-row dY blocks per wave); LC 1 = 4 waves of 64 r x 16 c along c (one X block, four dY blocks per wave):
// the X fragments, re-read for every tap, are then read by one wave instead of two (-35% LDS bytes per patch) at the
// same accumulator count.
template <int LC>
struct W16L {
    static constexpr int CB = LC ? 1 : 2;  // 16-channel X blocks per wave
    static constexpr int RB = LC ? 4 : 2;  // 16-row dY blocks per wave
    static constexpr int NH = 9 * CB;      // half taps (tap, channel block) per patch
};

// X fragments of half tap (T, CB): two transposed reads per X plane.
template <int T, int CB, int PB, int HW_, int NP>
__device__ __forceinline__ void w16_read_x(s16x4 (&f)[6], uint32_t xbase) {
    constexpr int toff = (T / 3) * HW_ + (T % 3);  // (1 + dy) * HW_ + (1 + dx)
    tr_read<0 * PB + toff * kW16RS + CB * 32>(f[0], xbase);
    tr_read<0 * PB + (toff + 8) * kW16RS + CB * 32>(f[1], xbase);
    if constexpr (w16_xp<NP>() >= 2) {
        tr_read<1 * PB + toff * kW16RS + CB * 32>(f[2], xbase);
        tr_read<1 * PB + (toff + 8) * kW16RS + CB * 32>(f[3], xbase);
    }
    if constexpr (w16_xp<NP>() == 3) {
        tr_read<2 * PB + toff * kW16RS + CB * 32>(f[4], xbase);
        tr_read<2 * PB + (toff + 8) * kW16RS + CB * 32>(f[5], xbase);
    }
}

// dY fragments of a patch, I = plane * NRB + rb: two transposed reads of 16 rows r (32 bytes) each; RSD = the
// staged dY row stride.
template <int I, int PA, int NRB, int DP, int RSD>
__device__ __forceinline__ void w16_read_dy(bf16x8 (&dv)[3][NRB], uint32_t dbase) {
    if constexpr (I < DP * NRB) {
        constexpr int p = I / NRB, rb = I % NRB;
        s16x4 lo, hi;
        tr_read<p * PA + rb * 32>(lo, dbase);
        tr_read<p * PA + 8 * RSD + rb * 32>(hi, dbase);
        dv[p][rb] = cat8(lo, hi);
        w16_read_dy<I + 1, PA, NRB, DP, RSD>(dv, dbase);
    }
}

// One half tap (tap T, channel block CB): wait for its X fragments, then the split products (six for x3, hh
// for bf16) x 2 r-blocks.
template <int T, int CB, int WAIT, int NP, int LC>
__device__ __forceinline__ void w16_half(f32x4 (&acc)[9][W16L<LC>::CB][W16L<LC>::RB],
                                         bf16x8 (&dv)[3][W16L<LC>::RB], s16x4 (&f)[6]) {
    bf16x8 x0 = cat8(f[0], f[1]), x1 = cat8(f[2], f[3]), x2 = cat8(f[4], f[5]);
    if constexpr (NP == 2 || NP == 4) {  // fp16 planes: x_m dy_h, x_h dy_m (NP 4: (x_h 2^-11) dy_m', dY's low
                                         // term pre-scaled), x_h dy_h
        lds_wait<WAIT>(x0, x1);
        if (T == 0 && CB == 0) {
#pragma unroll
            for (int rb = 0; rb < W16L<LC>::RB; ++rb) lds_wait<WAIT>(dv[0][rb], dv[1][rb]);
        }
        const u32x4 xh = __builtin_bit_cast(u32x4, x0), xm = __builtin_bit_cast(u32x4, x1);
        const u32x4 xh_lo = NP == 4 ? f16_down11(xh) : xh;
#pragma unroll
        for (int rb = 0; rb < W16L<LC>::RB; ++rb) {
            const u32x4 dh = __builtin_bit_cast(u32x4, dv[0][rb]), dm = __builtin_bit_cast(u32x4, dv[1][rb]);
            acc[T][CB][rb] = mfma16_f16(xm, dh, acc[T][CB][rb]);
            acc[T][CB][rb] = mfma16_f16(xh_lo, dm, acc[T][CB][rb]);
            acc[T][CB][rb] = mfma16_f16(xh, dh, acc[T][CB][rb]);
        }
        return;
    }
    if constexpr (NP != 1) {
        if constexpr (NP == 3)
            lds_wait<WAIT>(x0, x1, x2);
        else
            lds_wait<WAIT>(x0, x1);
        if (T == 0 && CB == 0) {
#pragma unroll
            for (int rb = 0; rb < W16L<LC>::RB; ++rb) lds_wait<WAIT>(dv[0][rb], dv[1][rb], dv[2][rb]);
        }
    } else {
        lds_wait<WAIT>(x0);
        if (T == 0 && CB == 0) {
#pragma unroll
            for (int rb = 0; rb < W16L<LC>::RB; ++rb) lds_wait<WAIT>(dv[0][rb]);
        }
    }
#pragma unroll
    for (int rb = 0; rb < W16L<LC>::RB; ++rb) {
        if constexpr (NP != 1) {
            acc[T][CB][rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, dv[1][rb], acc[T][CB][rb], 0, 0, 0);
            acc[T][CB][rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, dv[2][rb], acc[T][CB][rb], 0, 0, 0);
            if constexpr (NP == 3)  // x5 drops x_l * dy_h
                acc[T][CB][rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x2, dv[0][rb], acc[T][CB][rb], 0, 0, 0);
            acc[T][CB][rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, dv[1][rb], acc[T][CB][rb], 0, 0, 0);
            acc[T][CB][rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, dv[0][rb], acc[T][CB][rb], 0, 0, 0);
        }
        acc[T][CB][rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, dv[0][rb], acc[T][CB][rb], 0, 0, 0);
    }
}

// Half taps H = CB_per_wave * T + CB, one ahead: compute H from buffer H & 1, then refill that buffer with H + 2.
// The counted wait leaves the reads of the other buffer (2 per X plane, issued one half tap earlier) in flight.
template <int H, int PB, int HW_, int NP, int LC>
__device__ __forceinline__ void w16_chain(f32x4 (&acc)[9][W16L<LC>::CB][W16L<LC>::RB], bf16x8 (&dv)[3][W16L<LC>::RB],
                                          s16x4 (&f0)[6], s16x4 (&f1)[6], uint32_t xbase) {
    constexpr int NCB = W16L<LC>::CB, NH = W16L<LC>::NH;
    if constexpr (H < NH) {
        s16x4 (&f)[6] = (H & 1) ? f1 : f0;
        w16_half<H / NCB, H % NCB, (H == NH - 1 ? 0 : 2 * w16_xp<NP>()), NP, LC>(acc, dv, f);
        if constexpr (H + 2 < NH) w16_read_x<(H + 2) / NCB, (H + 2) % NCB, PB, HW_, NP>(f, xbase);
        w16_chain<H + 1, PB, HW_, NP, LC>(acc, dv, f0, f1, xbase);
    }
}
}  // namespace

// RG = 2 (LC 1 only): a block of 8 waves owns 128 rows r x 64 channels c; the two 4-wave groups share the
// staged X halo, which is then split and stored once per 128 rows instead of per 64 (the staging per MFMA,
// a third of the kernel's time at RG 1, drops by ~35%).
// DB (SCD_TUNE_WGRAD16_DB): two patch buffers, one barrier per patch; with RG 2 the second 4-wave group (waves 4-7,
// the partners of waves 0-3 on their SIMDs) stores the next patch BEFORE its MFMAs while the first group stores it
// after them, so one wave of each SIMD pair stages while the other computes (a stagger: without it both reach
// their split + LDS writes, and the matrix cores idle, together).
// RBN: the rows are dL/da of a = relu(BN(y)) and every dY element is formed while staging (bn_bwd_dy4, the expression
// of bn_bwd_apply: bit-identical values), with the BatchNorm coefficients of the block's rows held in LDS for both
// segments; the blocks of channel tile 0 also store the formed dY (a.rows_out) for the data grad, which then reads
// it as before: the separate BatchNorm-backward apply pass (read y and da, write dy) and this kernel's read of dy
// become this kernel's read of y and da.
template <int NP, int LC, int RG, bool SB = false, bool DB = false, bool RBN = false>
__global__ __launch_bounds__(256 * RG, 2 / RG) void wgrad_halo16_x3(WgradArgs a) {
    static_assert(!SB || NP == 1, "bf16 storage runs the bf16 arithmetic");
    static_assert(!RBN || (LC == 1 && !DB && (NP == 1 || NP == 4)), "rows transform: h2 / bf16, along-c layout");
    constexpr uint32_t EB = SB ? 2u : 4u;
    constexpr int NT = 256 * RG;
    constexpr int PH = 2, PW = 16, P = PH * PW;
    constexpr int HW_ = PW + 2, HP = (PH + 2) * HW_;  // halo: 4 x 18
    constexpr int RS = kW16RS;                        // X row stride (64 channels + 32 bytes)
    constexpr int RSD = 128 * RG + 32;                // dY row stride (64 RG rows + 32 bytes: conflict-free reads)
    constexpr int CQ = 16 * RG;                       // 4-row pieces per dY pixel
    constexpr int PA = P * RSD, PB = HP * RS;         // plane bytes
    constexpr int A_CH = P * CQ, B_CH = HP * 16;      // 4-channel pieces
    constexpr int A_PER = A_CH / NT, B_PER = (B_CH + NT - 1) / NT;
    static_assert(RG == 1 || (RG == 2 && LC == 1), "128-row blocks use the along-c wave layout");
    static_assert(NP == 1 || NP == 2 || NP == 3 || NP == 4 || NP == 5, "x3, x5, bf16 or h2");
    constexpr bool H2 = NP == 2 || NP == 4;
    constexpr int DP = w16_dp<NP>();  // dY planes
    constexpr int XP = w16_xp<NP>();  // X planes
    constexpr int STAGE = DP * PA + XP * PB;
    constexpr int RBLK = 64 * RG;                      // dY rows of the block
    constexpr int COEF = RBN ? 2 * 7 * RBLK * 4 : 0;   // RBN: [segment 2][7 coefficients][RBLK] floats
    // RBN under h2: the y pieces come by LDS-DMA (16 B per lane) into a staging area instead of registers (the h2
    // kernels sit at 256 VGPRs; eight more for y spilled the 64-row block)
    constexpr bool YDMA = RBN && H2;
    constexpr int YST = YDMA ? A_PER * NT * 16 : 0;
    __shared__ __attribute__((aligned(16))) unsigned char smem[(DB ? 2 : 1) * STAGE + COEF + YST];
    float ds = 1.f, ds_inv = 1.f, xs = 1.f, xs_inv = 1.f;  // h2: power-of-two operand scales
    if constexpr (H2) {
        h2_scale(*a.rows_bound, ds, ds_inv);
        h2_scale(*a.src_bound, xs, xs_inv);
    }

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    constexpr int NCB = W16L<LC>::CB, NRB = W16L<LC>::RB;
    // wave's dY / X block (in units of its width)
    const int wi = LC ? (RG == 1 ? 0 : wid >> 2) : wid >> 1, wj = LC ? (RG == 1 ? wid : wid & 3) : wid & 1;
    const uint32_t per_split = uint32_t(a.grid_r * a.grid_j);
    const uint32_t L = a.remap ? xcd_swizzle(blockIdx.x, gridDim.x) : blockIdx.x;
    const int split = int(L / per_split);
    const int rem = int(L - uint32_t(split) * per_split);
    const int ct = rem / a.grid_r;
    const int r0 = (rem - ct * a.grid_r) * 64 * RG, c0 = ct * 64;
    const int pw_n = a.wo / PW, ph_n = a.ho / PH, pimg = pw_n * ph_n;
    const int npatch = a.n_img_w * pimg;
    const int pbeg = split * a.kchunk, pend = min(npatch, pbeg + a.kchunk);

    const __amdgpu_buffer_rsrc_t rs_rows = make_rsrc(a.rows, a.rows_bytes);
    const __amdgpu_buffer_rsrc_t rs_src = make_rsrc(a.src, a.src_bytes);
    const __amdgpu_buffer_rsrc_t rs_y = make_rsrc(RBN ? a.rows_y : a.rows, RBN ? a.y_bytes : 0u);
    const bool writer = RBN && a.rows_out && ct == 0;  // block-uniform: this block stores its dY pieces
    float omax = 0.f;                                  // RBN writer: max |dY| stored by this lane

    StageT<SB> ra[A_PER], rb[B_PER], ya[RBN && !YDMA ? A_PER : 1];
    unsigned char *const ystage = smem + (DB ? 2 : 1) * STAGE + COEF;  // YDMA: piece e of the patch at e * 16
    const int wave_u = __builtin_amdgcn_readfirstlane(wid);
    f32x4 x_sc, x_sh;      // src transform coefficients of this thread's 4 channels (cq = tid & 15)
    uint32_t x_valid = 0;  // bit i: halo piece i is inside the image (the padding stays zero)
    int st_img = 0, st_y0 = 0, st_x0 = 0;  // the patch whose pieces the staging registers hold
    auto load_patch = [&](int pi) {
        const int img = pi / pimg, pr = pi - img * pimg;
        if (a.src_scale) {
            const int ch = (img / a.src_seg_imgs) * a.C + c0 + (tid & 15) * 4;
            x_sc = gload4(a.src_scale + ch);  // h2: times xs where consumed (store_patch)
            x_sh = gload4(a.src_shift + ch);
        }
        x_valid = 0;
        const int y0 = patch_y0(pr, pw_n, ph_n, PH), x0 = patch_x0(pr, pw_n, ph_n, PW);
        st_img = img;
        st_y0 = y0;
        st_x0 = x0;
#pragma unroll
        for (int i = 0; i < A_PER; ++i) {
            const int e = tid + i * NT, q = e / CQ, cq = e % CQ;
            const int py = q >> 4, px = q & 15;
            const int pix = (img * a.ho + y0 + py) * a.wo + x0 + px;
            if constexpr (YDMA)  // issued before the rows loads: waiting for those (in order) retires it too
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(a.rows_y + size_t(pix) * a.ldc_y + r0 + cq * 4),
                    (__attribute__((address_space(3))) void *)(ystage + (i * NT + wave_u * 64) * 16), 16, 0, 0);
            ra[i] = bload_q<SB>(rs_rows, uint32_t(pix * a.ldc_r + r0 + cq * 4) * EB);
            if constexpr (RBN && !YDMA) ya[i] = bload_q<SB>(rs_y, uint32_t(pix * a.ldc_y + r0 + cq * 4) * EB);
        }
#pragma unroll
        for (int i = 0; i < B_PER; ++i) {
            const int e = tid + i * NT, hp = e >> 4, cq = e & 15;
            const int hy = hp / HW_, hx = hp - (hp / HW_) * HW_;
            const int sy = y0 - 1 + hy, sx = x0 - 1 + hx;
            const bool v = e < B_CH && unsigned(sy) < unsigned(a.hs) && unsigned(sx) < unsigned(a.ws);
            x_valid |= uint32_t(v) << i;
            rb[i] = bload_q<SB>(rs_src, v ? uint32_t(((img * a.hs + sy) * a.ws + sx) * a.ldc_s + c0 + cq * 4) * EB : kOOB);
        }
    };
    auto store_patch = [&](int buf) {
        unsigned char *const smem_b = smem + buf * STAGE;
        // h2: the scale folds into the transform exactly; applied here, not behind the coefficient loads, where the
        // compiler waited for them (vmcnt in order: the wave stalled at issue)
        const f32x4 sc = H2 ? x_sc * xs : x_sc, sh = H2 ? x_sh * xs : x_sh;
        if constexpr (YDMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this patch's y pieces have landed
#pragma unroll
        for (int i = 0; i < A_PER; ++i) {
            const int e = tid + i * NT;
            const int o = (e / CQ) * RSD + (e % CQ) * 8;
            u32x2 h, m, l;
            if constexpr (RBN) {
                // dY of this piece from y and dL/da: bn_bwd_apply's expression (stored4: one rounding to the storage
                // type), the writer blocks store it, then it is staged as a plain dY piece
                const int cq = e % CQ, q = e / CQ;
                const float *cf = reinterpret_cast<const float *>(smem + (DB ? 2 : 1) * STAGE) +
                                  (st_img / a.rows_seg_imgs) * 7 * RBLK + cq * 4;
                const f32x4 mu = *reinterpret_cast<const f32x4 *>(cf), iv = *reinterpret_cast<const f32x4 *>(cf + RBLK);
                const f32x4 sc = *reinterpret_cast<const f32x4 *>(cf + 2 * RBLK);
                const f32x4 sf = *reinterpret_cast<const f32x4 *>(cf + 3 * RBLK);
                const f32x4 k1 = *reinterpret_cast<const f32x4 *>(cf + 4 * RBLK);
                const f32x4 k2 = *reinterpret_cast<const f32x4 *>(cf + 5 * RBLK);
                const f32x4 mul = *reinterpret_cast<const f32x4 *>(cf + 6 * RBLK);
                f32x4 yv;
                if constexpr (YDMA)
                    yv = *reinterpret_cast<const f32x4 *>(ystage + e * 16);
                else
                    yv = stage_f32<SB>(ya[i]);
                f32x4 dv = bn_bwd_dy4(yv, stage_f32<SB>(ra[i]), mu, iv, sc, sf, k1, k2, mul);
                if constexpr (SB) {
                    const u32x2 bits = pk_bf16x4(dv);
                    ra[i] = bits;
                    dv = unpk_bf16x4(bits);
                } else {
                    ra[i] = dv;
                }
                if (writer) {
                    const int pix = (st_img * a.ho + st_y0 + (q >> 4)) * a.wo + st_x0 + (q & 15);
                    const size_t idx = size_t(pix) * a.ldc_o + r0 + cq * 4;
                    if constexpr (SB)
                        *reinterpret_cast<u32x2 *>(static_cast<unsigned short *>(a.rows_out) + idx) = ra[i];
                    else
                        gstore4(static_cast<float *>(a.rows_out) + idx, dv);
                    omax = fmaxf(omax, fmaxf(fmaxf(fabsf(dv[0]), fabsf(dv[1])), fmaxf(fabsf(dv[2]), fabsf(dv[3]))));
                }
            }
            if constexpr (H2) {
                if constexpr (NP == 4)
                    split2h_pre(ra[i] * ds, h, m);
                else
                    split2h(ra[i] * ds, h, m);
                *reinterpret_cast<u32x2 *>(smem_b + PA + o) = m;
            } else if constexpr (DP == 3) {
                split3(ra[i], h, m, l);
                *reinterpret_cast<u32x2 *>(smem_b + PA + o) = m;
                *reinterpret_cast<u32x2 *>(smem_b + 2 * PA + o) = l;
            } else {
                h = stage_bits<SB>(ra[i]);
            }
            *reinterpret_cast<u32x2 *>(smem_b + o) = h;
        }
#pragma unroll
        for (int i = 0; i < B_PER; ++i)
            if constexpr (SB) {
                if (tid + i * NT < B_CH) {
                    u32x2 h = rb[i];
                    if (a.src_scale) {  // bf16 -> the BatchNorm + ReLU transform in fp32 -> the bf16 operand
                        const bool v = (x_valid >> i) & 1u;
                        f32x4 x = unpk_bf16x4(rb[i]);
#pragma unroll
                        for (int q = 0; q < 4; ++q) x[q] = v ? fmaxf(fmaf(x[q], sc[q], sh[q]), 0.f) : 0.f;
                        h = pk_bf16x4(x);
                    }
                    const int e = tid + i * NT;
                    *reinterpret_cast<u32x2 *>(smem_b + DP * PA + (e >> 4) * RS + (e & 15) * 8) = h;
                }
            } else if (tid + i * NT < B_CH) {
                u32x2 h, m, l;
                if (a.src_scale) {
                    const bool v = (x_valid >> i) & 1u;
#pragma unroll
                    for (int q = 0; q < 4; ++q) rb[i][q] = v ? fmaxf(fmaf(rb[i][q], sc[q], sh[q]), 0.f) : 0.f;
                } else if constexpr (H2) {
                    rb[i] *= xs;
                }
                const int e = tid + i * NT;
                const int o = DP * PA + (e >> 4) * RS + (e & 15) * 8;
                if constexpr (H2) {
                    split2h(rb[i], h, m);
                    *reinterpret_cast<u32x2 *>(smem_b + PB + o) = m;
                } else if constexpr (XP >= 2) {
                    split3(rb[i], h, m, l);  // x5: the l term is not needed (dead code)
                    *reinterpret_cast<u32x2 *>(smem_b + PB + o) = m;
                    if constexpr (XP == 3) *reinterpret_cast<u32x2 *>(smem_b + 2 * PB + o) = l;
                } else {
                    h[0] = cvt_pk_bf16(rb[i][0], rb[i][1]);
                    h[1] = cvt_pk_bf16(rb[i][2], rb[i][3]);
                }
                *reinterpret_cast<u32x2 *>(smem_b + o) = h;
            }
    };

    f32x4 acc[9][NCB][NRB];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < NCB; ++i)
#pragma unroll
            for (int j = 0; j < NRB; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // transposed-read lane roles: 16-lane group g supplies patch pixels (g >> 1, 4(g & 1) + (w16 >> 2)) (+8
    // for the second read of a fragment) and channel columns 4(w16 & 3)..+3 of a 16-channel block
    const int g = lane >> 4, w16 = lane & 15;
    const int py = g >> 1, pxq = 4 * (g & 1) + (w16 >> 2);
    const uint32_t dbase = lds_addr(smem) + (py * PW + pxq) * RSD + (16 * NRB * wi + 4 * (w16 & 3)) * 2;
    const uint32_t xbase = lds_addr(smem) + DP * PA + (py * HW_ + pxq) * RS + (16 * NCB * wj + 4 * (w16 & 3)) * 2;

    if constexpr (RBN) {  // the block's rows' BatchNorm coefficients, both segments (launcher: at most 2 per launch)
        float *cf = reinterpret_cast<float *>(smem + (DB ? 2 : 1) * STAGE);
        const int nsl = a.n_img_w / a.rows_seg_imgs;
        for (int e = tid; e < nsl * RBLK; e += NT) {
            const int sg = e / RBLK, r = e - sg * RBLK, o = sg * a.R + r0 + r;
            const float iv = a.rbn_inv[o];
            float *c = cf + sg * 7 * RBLK + r;
            c[0] = a.rbn_mean[o];
            c[RBLK] = iv;
            c[2 * RBLK] = a.rbn_scale[o];
            c[3 * RBLK] = a.rbn_shift[o];
            c[4 * RBLK] = a.rbn_coef[2 * o];
            c[5 * RBLK] = a.rbn_coef[2 * o + 1];
            c[6 * RBLK] = (a.rbn_gamma ? a.rbn_gamma[r0 + r] : 1.f) * iv;  // bn_bwd_apply's mul = gamma * invstd
        }
        __syncthreads();
    }
    if (pbeg < pend) {
        // DB, RG 2: waves 4-7 stage the next patch before their MFMAs (loads two patches ahead), waves 0-3 after
        const bool early = DB && RG == 2 && __builtin_amdgcn_readfirstlane(wid) >= 4;
        load_patch(pbeg);
        store_patch(0);
        if (early && pbeg + 1 < pend) load_patch(pbeg + 1);
        __syncthreads();
        int buf = 0;
        for (int pi = pbeg; pi < pend; ++pi) {
            const bool more = pi + 1 < pend;
            if (early) {
                // the buffer of patch pi + 1 was last read in the previous patch, which the barrier closed
                if (more) store_patch(buf ^ 1);
                if (pi + 2 < pend) load_patch(pi + 2);
            } else if (more) {
                load_patch(pi + 1);
            }
            const uint32_t bo = uint32_t(buf * STAGE);
            bf16x8 dv[3][NRB];
            w16_read_dy<0, PA, NRB, DP, RSD>(dv, dbase + bo);
            s16x4 f0[6], f1[6];
            w16_read_x<0 / NCB, 0 % NCB, PB, HW_, NP>(f0, xbase + bo);
            w16_read_x<1 / NCB, 1 % NCB, PB, HW_, NP>(f1, xbase + bo);
            w16_chain<0, PB, HW_, NP, LC>(acc, dv, f0, f1, xbase + bo);
            if constexpr (DB) {
                if (!early && more) store_patch(buf ^ 1);
                __syncthreads();  // patch pi + 1 is staged; every wave is done with patch pi
                buf ^= 1;
            } else if (more) {
                __syncthreads();  // every wave is done with this patch
                store_patch(0);
                __syncthreads();
            }
        }
    }

    if constexpr (H2) {
        const float k = ds_inv * xs_inv;  // exact: a power of two
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
                for (int r = 0; r < NRB; ++r) acc[t][cb][r] *= k;
    }
    if (writer && a.rows_out_bound) wave_max_bound(a.rows_out_bound, omax);  // uniform: the whole block takes part
    // acc[t][cb][rb][q]: r = r0 + 16 NRB wi + 16rb + (lane & 15), c = c0 + 16 NCB wj + 16cb + 4g + q
    float *slab = a.slabs + size_t(split) * a.R * a.Ng;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
            for (int r = 0; r < NRB; ++r) {
                const int row = r0 + 16 * NRB * wi + 16 * r + w16;
                const int col = c0 + 16 * NCB * wj + 16 * cb + 4 * g;
                gstore4(slab + size_t(row) * a.Ng + t * a.C + col, acc[t][cb][r]);
            }
}

// ------------------------------------------------------------------------------------------------
// The bf16-storage halo weight grad with its patches brought into LDS by LDS-DMA (buffer_load ... lds), NB - 1
// patches ahead.  wgrad_halo16_x3<1, 1, RG, true> holds ONE patch in flight (its next patch in staging registers):
// at ~0.5 us of MFMAs per 32-pixel patch against an HBM latency of 1-2 us under load, every patch waited for its own
// loads (MFMA busy 0.25-0.34 at 2.3 GHz, profiles/r05_pmc_dualstream_last).  Here a ring of NB patch buffers keeps NB - 1
// patches in flight with no staging registers: with bf16 storage and no operand transform the staged planes are the
// stored bits, so the global pieces land in the kernel's LDS image unchanged (the same [pixel][row] / [halo pixel]
// [channel] planes with 32-byte row pads as wgrad_halo16_x3, filled 16 bytes per lane; pad lanes and halo pixels
// outside the image read out of the buffer range, which returns zeros).  One barrier per patch: it retires every
// wave's pieces of the patch about to be read and closes the reads of the buffer the next DMA overwrites.
// Same products in the same order as wgrad_halo16_x3<1, 1, RG, true> (bit-identical slabs).
// XT: the source is read through its BatchNorm + ReLU (src_scale / src_shift, at most two segments): the raw bf16 y
// lands by DMA as above and each X plane is transformed in place one patch ahead of its use -- max(fma(y, sc, sh), 0)
// rounded to bf16, zero outside the image, wgrad_halo16_x3's expressions (bit-identical) -- so a patch is waited for one
// iteration earlier (NB - 2 patches in flight) and the transform's LDS pass overlaps the current patch's MFMAs.
// RBN: the rows are dL/da of a plain BatchNorm + ReLU (wgrad_halo16_x3's RBN, ABI 8): y and dL/da both land by DMA (y in a
// third plane with dY's layout) and dY is formed in place in the same pass, with the writer blocks (channel tile 0)
// storing it for the data grad; their stores are counted in the loop's vmcnt waits.
// ------------------------------------------------------------------------------------------------
namespace {
// dummy destination of the padding DMA pieces that even out the per-wave piece count (zeros, never read)
constexpr int kDmaSink = 1024;
}  // namespace
#ifndef SCD_WGRAD16_DMA_NB
#define SCD_WGRAD16_DMA_NB 4  // ring depth: 3 patches in flight while one is computed
#endif
#ifndef SCD_WGRAD16_DMA_TRANSFORMS
#define SCD_WGRAD16_DMA_TRANSFORMS 1  // 0: the ring for untransformed operands only (A/B build)
#endif
#ifndef SCD_WGRAD16_DMA_NB_XT
#define SCD_WGRAD16_DMA_NB_XT 5  // 128-row blocks with the source transform: 3 patches in flight (64-row: NB above)
#endif

template <int RG, int NB, bool XT = false, bool RBN = false>
__global__ __launch_bounds__(256 * RG, 2 / RG) void wgrad_halo16_dma(WgradArgs a) {
    constexpr int NT = 256 * RG, NW = NT / 64;
    constexpr int PH = 2, PW = 16, P = PH * PW;
    constexpr int HW_ = PW + 2, HP = (PH + 2) * HW_;  // halo: 4 x 18
    constexpr int RS = kW16RS;                        // X row stride (64 channels + 32 bytes)
    constexpr int RSD = 128 * RG + 32;                // dY row stride (64 RG rows + 32 bytes)
    constexpr int PA = P * RSD, PB = HP * RS;         // plane bytes
    constexpr int PA_K = (PA + 1023) / 1024, PB_K = (PB + 1023) / 1024;  // 1 KB DMA pieces per plane
    constexpr int NPC = PA_K + PB_K + (RBN ? PA_K : 0);  // pieces per patch (RBN: y in its own plane, dY's layout)
    constexpr int PPW = (NPC + NW - 1) / NW;          // pieces per wave and patch (padded with sink pieces)
    constexpr int STAGE = NPC * 1024;
    constexpr int DCH = 8 * RG;                       // 16-byte dY chunks per staged pixel (64 RG rows)
    constexpr int RBLK = 64 * RG;                     // dY rows of the block
    constexpr int NCB = W16L<1>::CB, NRB = W16L<1>::RB;
    constexpr bool TR = XT || RBN;                    // a transform pass one patch ahead
    static_assert(NB >= (TR ? 3 : 2) && NB <= 6, "ring depth");
    static_assert(!RBN || (P * DCH) % NT == 0, "rows transform: whole 16-byte chunks per thread");
    constexpr int RCH = RBN ? P * DCH / NT : 0;       // RBN: dY chunks each thread forms (and the writer stores) per patch
    constexpr int CFX = XT ? 2 * 2 * 64 * 4 : 0;      // XT: [segment 2][sc, sh][64 channels] floats
    constexpr int CFR = RBN ? 2 * 7 * RBLK * 4 : 0;   // RBN: [segment 2][7 coefficients][RBLK] (wgrad_halo16_x3's)
    __shared__ __attribute__((aligned(16))) unsigned char smem[NB * STAGE + kDmaSink + CFX + CFR];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wave_u = __builtin_amdgcn_readfirstlane(wid);
    const int wi = RG == 1 ? 0 : wid >> 2, wj = RG == 1 ? wid : wid & 3;
    const uint32_t per_split = uint32_t(a.grid_r * a.grid_j);
    const uint32_t L = a.remap ? xcd_swizzle(blockIdx.x, gridDim.x) : blockIdx.x;
    const int split = int(L / per_split);
    const int rem = int(L - uint32_t(split) * per_split);
    const int ct = rem / a.grid_r;
    const int r0 = (rem - ct * a.grid_r) * 64 * RG, c0 = ct * 64;
    const int pw_n = a.wo / PW, ph_n = a.ho / PH, pimg = pw_n * ph_n;
    const int npatch = a.n_img_w * pimg;
    const int pbeg = split * a.kchunk, pend = min(npatch, pbeg + a.kchunk);
    const bool writer = RBN && a.rows_out && ct == 0;  // block-uniform: this block stores the formed dY
    float omax = 0.f;                                  // writer: max |dY| stored by this thread

    const __amdgpu_buffer_rsrc_t rs_rows = make_rsrc(a.rows, a.rows_bytes);
    const __amdgpu_buffer_rsrc_t rs_src = make_rsrc(a.src, a.src_bytes);
    const __amdgpu_buffer_rsrc_t rs_y = make_rsrc(RBN ? a.rows_y : a.rows, RBN ? a.y_bytes : 0u);
    // This lane's 16-byte chunk of each of the wave's pieces: piece k of a patch is the block's piece u = k * NW + wave
    // (u < PA_K: dY plane bytes [1024 u, +1024); then the X plane; RBN: then the y plane; else a sink piece).  Position
    // within its plane: row = byte / stride, chunk = (byte % stride) / 16; chunks past the data (the row pads, the tail)
    // read out of range.
    // Per piece, precomputed once: rel = its element offset relative to the patch's first pixel (dY / y: that pixel's
    // row start; X: the halo's, one row and column up-left, so the validity test per patch is two compares) -- issue()
    // then adds one patch base per plane and tests the halo piece's bounds: a few VALU per piece instead of the index
    // arithmetic that made the first DMA ring (round 6, profiles/r06_wgrad_dma_pmc) 2.3 VALU per MFMA.
    int rel[PPW], x_hy[PPW], x_hx[PPW], kind[PPW];  // kind 0 dY / y, 1 X, 2 sink / pad
#pragma unroll
    for (int k = 0; k < PPW; ++k) {
        const int u = k * NW + wave_u;
        kind[k] = 2;
        rel[k] = x_hy[k] = x_hx[k] = 0;
        const bool is_y = RBN && u >= PA_K + PB_K && u < NPC;
        if (u < PA_K || is_y) {
            const int b = (is_y ? u - PA_K - PB_K : u) * 1024 + lane * 16;
            const int row = b / RSD, ch = (b - row * RSD) / 16;
            if (row < P && ch < DCH) {
                kind[k] = 0;
                rel[k] = ((row >> 4) * a.wo + (row & 15)) * (is_y ? a.ldc_y : a.ldc_r) + r0 + 8 * ch;
            }
        } else if (u < PA_K + PB_K) {
            const int b = (u - PA_K) * 1024 + lane * 16;
            const int row = b / RS, ch = (b - row * RS) / 16;
            if (row < HP && ch < 8) {
                kind[k] = 1;
                x_hy[k] = row / HW_;
                x_hx[k] = row - (row / HW_) * HW_;
                rel[k] = ((x_hy[k] - 1) * a.ws + (x_hx[k] - 1)) * a.ldc_s + c0 + 8 * ch;
            }
        }
    }
    // The patch walk as a cursor (image, first row, first column): down each 16-pixel column strip (patch_y0 / x0's
    // order), advanced by compares instead of divisions.
    struct Cursor {
        int img, y0, x0;
    };
    auto cursor_at = [&](int pi) {
        const int img = pi / pimg, pr = pi - img * pimg;
        return Cursor{img, patch_y0(pr, pw_n, ph_n, PH), patch_x0(pr, pw_n, ph_n, PW)};
    };
    auto advance = [&](Cursor &c) {
        if constexpr (SCD_WGRAD_ROW_WALK) {
            if ((c.x0 += PW) == a.wo) {
                c.x0 = 0;
                if ((c.y0 += PH) == a.ho) c.y0 = 0, ++c.img;
            }
        } else if ((c.y0 += PH) == a.ho) {
            c.y0 = 0;
            if ((c.x0 += PW) == a.wo) c.x0 = 0, ++c.img;
        }
    };
    // Issue the pieces of the patch at cursor `c` into ring slot `slot` (wave-uniform LDS base per piece: M0 + lane * 16).
    auto issue = [&](const Cursor &c, int slot) {
        const int img = c.img, y0 = c.y0, x0 = c.x0;
        const int pix0 = (img * a.ho + y0) * a.wo + x0;  // the patch's first pixel (rows and src share h, w)
        const int br = pix0 * a.ldc_r, by = RBN ? pix0 * a.ldc_y : 0, bs = pix0 * a.ldc_s;
#pragma unroll
        for (int k = 0; k < PPW; ++k) {
            const int u = k * NW + wave_u;
            const bool is_y = RBN && u >= PA_K + PB_K && u < NPC;
            const int base = u < PA_K ? br : is_y ? by : bs;  // wave-uniform: the piece's plane
            // branch-free: dY / y pieces always load, halo pieces inside the image, pads and sinks never
            const bool ok = kind[k] == 0 || (kind[k] == 1 && unsigned(y0 - 1 + x_hy[k]) < unsigned(a.hs) &&
                                             unsigned(x0 - 1 + x_hx[k]) < unsigned(a.ws));
            const uint32_t off = ok ? uint32_t(base + rel[k]) * 2u : kOOB;
            unsigned char *dst = u < NPC ? smem + slot * STAGE + u * 1024 : smem + NB * STAGE;
            if (u < PA_K)  // wave-uniform
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_rows, (__attribute__((address_space(3))) void *)dst, 16, off,
                                                         0, 0, 0);
            else if (is_y)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_y, (__attribute__((address_space(3))) void *)dst, 16, off, 0,
                                                         0, 0);
            else
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_src, (__attribute__((address_space(3))) void *)dst, 16, off,
                                                         0, 0, 0);
        }
        asm volatile("" ::: "memory");
    };

    f32x4 acc[9][NCB][NRB];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < NCB; ++i)
#pragma unroll
            for (int j = 0; j < NRB; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // transposed-read lane roles of wgrad_halo16_x3
    const int g = lane >> 4, w16 = lane & 15;
    const int py = g >> 1, pxq = 4 * (g & 1) + (w16 >> 2);
    const uint32_t dbase = lds_addr(smem) + (py * PW + pxq) * RSD + (16 * NRB * wi + 4 * (w16 & 3)) * 2;
    const uint32_t xbase = lds_addr(smem) + PA_K * 1024 + (py * HW_ + pxq) * RS + (16 * NCB * wj + 4 * (w16 & 3)) * 2;

    // The transforms of patch pi in ring slot `slot_`, in place, one patch ahead of its MFMAs:
    //   XT  this thread's X chunks q = tid + i NT (halo pixel q >> 3, channels c0 + 8 (q & 7) ..+7): the source's
    //       BatchNorm + ReLU, rounded to bf16; out-of-image chunks stay the DMA's zeros;
    //   RBN this thread's dY chunks q = tid + i NT (pixel q / DCH, rows r0 + 8 (q % DCH) ..+7): dY = the BatchNorm
    //       backward of (y, dL/da) (bn_bwd_dy4, rounded once to bf16 as bn_bwd_apply stores it), which the writer blocks
    //       also store for the data grad.
    float *const cfx = reinterpret_cast<float *>(smem + NB * STAGE + kDmaSink);         // [seg][sc | sh][64]
    // XT: this thread's 16-byte chunks of the X plane, by linear LDS position (chunk tid + i NT: consecutive lanes read
    // and write consecutive 16 bytes, no bank conflicts): halo row / column and channel octet (-1: a row pad or past the
    // plane), fixed for the kernel
    constexpr int XTI = XT ? (PB / 16 + NT - 1) / NT : 1;
    int xt_hy[XTI], xt_hx[XTI], xt_j[XTI];
#pragma unroll
    for (int i = 0; i < XTI; ++i) {
        const int L = tid + i * NT, row = L / (RS / 16), col = L - row * (RS / 16);
        xt_j[i] = (XT && L < PB / 16 && col < 8) ? col : -1;
        xt_hy[i] = row / HW_;
        xt_hx[i] = row - (row / HW_) * HW_;
    }
    float *const cfr = reinterpret_cast<float *>(smem + NB * STAGE + kDmaSink + CFX);   // [seg][7][RBLK]
    auto transform = [&](const Cursor &cur, int slot_) {
        const int img = cur.img, y0 = cur.y0, x0 = cur.x0;
        if constexpr (XT) {
            const float *c_sc = cfx + (img / a.src_seg_imgs) * 128, *c_sh = c_sc + 64;
            unsigned char *const xp = smem + slot_ * STAGE + PA_K * 1024;
#pragma unroll
            for (int i = 0; i < XTI; ++i) {
                if (xt_j[i] < 0 || unsigned(y0 - 1 + xt_hy[i]) >= unsigned(a.hs) ||
                    unsigned(x0 - 1 + xt_hx[i]) >= unsigned(a.ws))
                    continue;  // a row pad, past the plane, or outside the image (the DMA's zeros stay)
                const int j = xt_j[i];
                u32x4 *const ptr = reinterpret_cast<u32x4 *>(xp + (tid + i * NT) * 16);
                const u32x4 raw = *ptr;
                u32x4 out;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    f32x4 x = unpk_bf16x4(u32x2{raw[2 * h], raw[2 * h + 1]});
                    const f32x4 sc = *reinterpret_cast<const f32x4 *>(c_sc + 8 * j + 4 * h);
                    const f32x4 sh = *reinterpret_cast<const f32x4 *>(c_sh + 8 * j + 4 * h);
#pragma unroll
                    for (int e = 0; e < 4; ++e) x[e] = fmaxf(fmaf(x[e], sc[e], sh[e]), 0.f);
                    const u32x2 pk = pk_bf16x4(x);
                    out[2 * h] = pk[0];
                    out[2 * h + 1] = pk[1];
                }
                *ptr = out;
            }
        }
        if constexpr (RBN) {
            const float *cs = cfr + (img / a.rows_seg_imgs) * 7 * RBLK;
            unsigned char *const dp = smem + slot_ * STAGE;
            const unsigned char *const yp = smem + slot_ * STAGE + (PA_K + PB_K) * 1024;
#pragma unroll
            for (int i = 0; i < RCH; ++i) {
                const int q = tid + i * NT;
                const int px = q / DCH, j = q - px * DCH;
                u32x4 *const ptr = reinterpret_cast<u32x4 *>(dp + px * RSD + j * 16);
                const u32x4 raw = *ptr, yr = *reinterpret_cast<const u32x4 *>(yp + px * RSD + j * 16);
                u32x4 out;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const float *c = cs + 8 * j + 4 * h;
                    const f32x4 mu = *reinterpret_cast<const f32x4 *>(c), iv = *reinterpret_cast<const f32x4 *>(c + RBLK);
                    const f32x4 sc = *reinterpret_cast<const f32x4 *>(c + 2 * RBLK);
                    const f32x4 sf = *reinterpret_cast<const f32x4 *>(c + 3 * RBLK);
                    const f32x4 k1 = *reinterpret_cast<const f32x4 *>(c + 4 * RBLK);
                    const f32x4 k2 = *reinterpret_cast<const f32x4 *>(c + 5 * RBLK);
                    const f32x4 mul = *reinterpret_cast<const f32x4 *>(c + 6 * RBLK);
                    const f32x4 dv = bn_bwd_dy4(unpk_bf16x4(u32x2{yr[2 * h], yr[2 * h + 1]}),
                                                unpk_bf16x4(u32x2{raw[2 * h], raw[2 * h + 1]}), mu, iv, sc, sf, k1, k2, mul);
                    const u32x2 pk = pk_bf16x4(dv);
                    out[2 * h] = pk[0];
                    out[2 * h + 1] = pk[1];
                    if (writer && a.rows_out_bound) {  // (no bound in the bf16 arithmetic)
                        const f32x4 r = unpk_bf16x4(pk);
                        omax = fmaxf(omax, fmaxf(fmaxf(fabsf(r[0]), fabsf(r[1])), fmaxf(fabsf(r[2]), fabsf(r[3]))));
                    }
                }
                *ptr = out;
                if (writer) {  // one 16-byte store per chunk (vmcnt: counted in the loop's waits)
                    const int pix = (img * a.ho + y0 + (px >> 4)) * a.wo + x0 + (px & 15);
                    *reinterpret_cast<u32x4 *>(static_cast<unsigned short *>(a.rows_out) + size_t(pix) * a.ldc_o + r0 +
                                               8 * j) = out;
                }
            }
        }
    };
    if constexpr (XT) {  // both segments' coefficients of the block's 64 channels (launcher: at most two)
        const int nsl = a.n_img_w / a.src_seg_imgs;
        for (int e = tid; e < nsl * 64; e += NT) {
            const int sg = e / 64, c = e - sg * 64;
            cfx[sg * 128 + c] = a.src_scale[sg * a.C + c0 + c];
            cfx[sg * 128 + 64 + c] = a.src_shift[sg * a.C + c0 + c];
        }
    }
    if constexpr (RBN) {  // the block's rows' BatchNorm coefficients (wgrad_halo16_x3's table; at most two segments)
        const int nsl = a.n_img_w / a.rows_seg_imgs;
        for (int e = tid; e < nsl * RBLK; e += NT) {
            const int sg = e / RBLK, r = e - sg * RBLK, o = sg * a.R + r0 + r;
            const float iv = a.rbn_inv[o];
            float *c = cfr + sg * 7 * RBLK + r;
            c[0] = a.rbn_mean[o];
            c[RBLK] = iv;
            c[2 * RBLK] = a.rbn_scale[o];
            c[3 * RBLK] = a.rbn_shift[o];
            c[4 * RBLK] = a.rbn_coef[2 * o];
            c[5 * RBLK] = a.rbn_coef[2 * o + 1];
            c[6 * RBLK] = (a.rbn_gamma ? a.rbn_gamma[r0 + r] : 1.f) * iv;  // bn_bwd_apply's mul = gamma * invstd
        }
    }

    // the writer's dY stores of the previous transform are the youngest vector-memory operations at each wait
    const int wst = writer ? RCH : 0;
    Cursor ci = cursor_at(pbeg), ct1 = ci;  // the next patch to issue; the patch the next transform forms
#pragma unroll
    for (int k = 0; k < NB - 1; ++k)
        if (pbeg + k < pend) {
            issue(ci, k);
            advance(ci);
        }
    if constexpr (TR) {  // patch pbeg transformed before the loop (its first barrier publishes it)
        if (pbeg < pend) {
            const int ahead = min(NB - 2, pend - 1 - pbeg);
            if (ahead >= 3)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PPW) : "memory");
            else if (ahead == 2)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW) : "memory");
            else if (ahead == 1)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            lds_barrier();  // every wave's pieces of patch pbeg (and the coefficients) are in LDS
            transform(ct1, 0);
            advance(ct1);
        }
    }
    int slot = 0;
    for (int pi = pbeg; pi < pend; ++pi) {
        // this wave's pieces of patch pi (with a transform: pi + 1, transformed during this iteration): younger in
        // flight are those of the patches after it up to min(pi + NB - 2, pend - 1), and the writer's stores
        const int ahead = TR ? (pi + 1 < pend ? min(NB - 3, pend - 2 - pi) : -1) : min(NB - 2, pend - 1 - pi);
        if (wst == 0) {
            if (ahead >= 4)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * PPW) : "memory");
            else if (ahead == 3)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PPW) : "memory");
            else if (ahead == 2)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW) : "memory");
            else if (ahead == 1)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
            else if (ahead == 0)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if constexpr (RBN) {  // RCH stores of the last transform behind the pieces
            if (ahead >= 3)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PPW + RCH) : "memory");
            else if (ahead == 2)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW + RCH) : "memory");
            else if (ahead == 1)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW + RCH) : "memory");
            else if (ahead == 0)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RCH) : "memory");
        }
        lds_barrier();  // every wave's pieces of patch pi landed; every wave left the slot of patch pi - 1
        if (pi + NB - 1 < pend) {
            issue(ci, slot == 0 ? NB - 1 : slot - 1);
            advance(ci);
        }
        if constexpr (TR) {
            if (pi + 1 < pend) {
                transform(ct1, slot == NB - 1 ? 0 : slot + 1);
                advance(ct1);
            }
        }
        const uint32_t bo = uint32_t(slot * STAGE);
        bf16x8 dv[3][NRB];
        w16_read_dy<0, PA_K * 1024, NRB, 1, RSD>(dv, dbase + bo);
        s16x4 f0[6], f1[6];
        w16_read_x<0, 0, PB_K * 1024, HW_, 1>(f0, xbase + bo);
        w16_read_x<1, 0, PB_K * 1024, HW_, 1>(f1, xbase + bo);
        w16_chain<0, PB_K * 1024, HW_, 1, 1>(acc, dv, f0, f1, xbase + bo);
        slot = slot == NB - 1 ? 0 : slot + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (writer && a.rows_out_bound) wave_max_bound(a.rows_out_bound, omax);  // uniform: the whole block takes part

    float *slab = a.slabs + size_t(split) * a.R * a.Ng;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
            for (int r = 0; r < NRB; ++r) {
                const int row = r0 + 16 * NRB * wi + 16 * r + w16;
                const int col = c0 + 16 * NCB * wj + 16 * cb + 4 * g;
                gstore4(slab + size_t(row) * a.Ng + t * a.C + col, acc[t][cb][r]);
            }
}

// ------------------------------------------------------------------------------------------------
// Halo weight gradient of a 16-channel source (the input layer: 5 bands padded to the bf16 K granule of 16).
// Same patch walk, tap shifts and transposed-read lane roles as wgrad_halo16_x3, with the channel block cut to
// the 16 channels that exist: a block owns 64 rows r x 16 c x 9 taps and each wave 16 r, so a patch costs
// 9 taps x (6 | 4 | 1) MFMAs per wave and the X halo staged per patch is a quarter of the 64-channel kernel's.
// The X plane rows are 32 bytes (16 channels, unpadded): a 32-lane half of a transposed read then covers 256
// contiguous bytes, conflict-free.
// ------------------------------------------------------------------------------------------------
namespace {
constexpr int kC16RS = 32;

template <int T, int PB, int HW_, int NP>
__device__ __forceinline__ void c16_read_x(s16x4 (&f)[6], uint32_t xbase) {
    constexpr int toff = (T / 3) * HW_ + (T % 3);
    tr_read<0 * PB + toff * kC16RS>(f[0], xbase);
    tr_read<0 * PB + (toff + 8) * kC16RS>(f[1], xbase);
    if constexpr (w16_xp<NP>() >= 2) {
        tr_read<1 * PB + toff * kC16RS>(f[2], xbase);
        tr_read<1 * PB + (toff + 8) * kC16RS>(f[3], xbase);
    }
    if constexpr (w16_xp<NP>() == 3) {
        tr_read<2 * PB + toff * kC16RS>(f[4], xbase);
        tr_read<2 * PB + (toff + 8) * kC16RS>(f[5], xbase);
    }
}

template <int T, int WAIT, int NP>
__device__ __forceinline__ void c16_tap(f32x4 (&acc)[9], bf16x8 (&dv)[3], s16x4 (&f)[6]) {
    bf16x8 x0 = cat8(f[0], f[1]), x1 = cat8(f[2], f[3]), x2 = cat8(f[4], f[5]);
    if constexpr (NP == 4) {  // h2 (as w16_half): x_m dy_h, (x_h 2^-11) dy_m', x_h dy_h on the fp16 planes
        lds_wait<WAIT>(x0, x1);
        if (T == 0) lds_wait<WAIT>(dv[0], dv[1]);
        const u32x4 xh = __builtin_bit_cast(u32x4, x0), xm = __builtin_bit_cast(u32x4, x1);
        const u32x4 dh = __builtin_bit_cast(u32x4, dv[0]), dm = __builtin_bit_cast(u32x4, dv[1]);
        acc[T] = mfma16_f16(xm, dh, acc[T]);
        acc[T] = mfma16_f16(f16_down11(xh), dm, acc[T]);
        acc[T] = mfma16_f16(xh, dh, acc[T]);
        return;
    }
    if constexpr (NP != 1) {
        if constexpr (NP == 3)
            lds_wait<WAIT>(x0, x1, x2);
        else
            lds_wait<WAIT>(x0, x1);
        if (T == 0) lds_wait<WAIT>(dv[0], dv[1], dv[2]);
    } else {
        lds_wait<WAIT>(x0, dv[0]);
    }
    if constexpr (NP != 1) {
        acc[T] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, dv[1], acc[T], 0, 0, 0);
        acc[T] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, dv[2], acc[T], 0, 0, 0);
        if constexpr (NP == 3) acc[T] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x2, dv[0], acc[T], 0, 0, 0);
        acc[T] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, dv[1], acc[T], 0, 0, 0);
        acc[T] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, dv[0], acc[T], 0, 0, 0);
    }
    acc[T] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, dv[0], acc[T], 0, 0, 0);
}

// taps T = 0..8, one ahead: compute T from buffer T & 1, then refill it with tap T + 2
template <int T, int PB, int HW_, int NP>
__device__ __forceinline__ void c16_chain(f32x4 (&acc)[9], bf16x8 (&dv)[3], s16x4 (&f0)[6], s16x4 (&f1)[6],
                                          uint32_t xbase) {
    if constexpr (T < 9) {
        s16x4 (&f)[6] = (T & 1) ? f1 : f0;
        c16_tap<T, (T == 8 ? 0 : 2 * w16_xp<NP>()), NP>(acc, dv, f);
        if constexpr (T + 2 < 9) c16_read_x<T + 2, PB, HW_, NP>(f, xbase);
        c16_chain<T + 1, PB, HW_, NP>(acc, dv, f0, f1, xbase);
    }
}
}  // namespace

// RBN: the rows are dL/da of a = relu(BN(y)) and each staged dY piece is formed as the BatchNorm backward's apply
// would write it (bn_bwd_dy4, the same bits), so that gradient is never written or re-read (the input layer's).
// NP 4: h2 (as wgrad_halo16_x3<4, ...>): dY scaled by the power of two of *rows_bound (with RBN a bound of the formed
// dY, scd_bn_relu_backward_coef's dy_bound) and split with its low term pre-scaled, X by that of *src_bound.
template <int NP, bool RBN, bool SB = false>
__global__ __launch_bounds__(256, 2) void wgrad_halo16_c16(WgradArgs a) {
    static_assert(!SB || NP == 1, "bf16 storage runs the bf16 arithmetic");
    constexpr uint32_t EB = SB ? 2u : 4u;
    constexpr int PH = 2, PW = 16, P = PH * PW;
    constexpr int HW_ = PW + 2, HP = (PH + 2) * HW_;  // halo: 4 x 18
    constexpr int RS = kW16RS, RSX = kC16RS;
    constexpr int PA = P * RS, PB = HP * RSX;           // plane bytes
    constexpr int A_CH = P * 16, B_CH = HP * 4;         // 4-channel pieces: dY 32 px x 64 r, X 72 px x 16 c
    constexpr int A_PER = A_CH / 256, B_PER = (B_CH + 255) / 256;
    static_assert(NP == 1 || NP == 3 || NP == 4 || NP == 5, "x3, x5, bf16 or h2");
    constexpr bool H2 = NP == 4;
    constexpr int DP = w16_dp<NP>();
    constexpr int XP = w16_xp<NP>();
    __shared__ __attribute__((aligned(16))) unsigned char smem[DP * PA + XP * PB];
    float ds = 1.f, ds_inv = 1.f, xs = 1.f, xs_inv = 1.f;  // h2: power-of-two operand scales
    if constexpr (H2) {
        h2_scale(*a.rows_bound, ds, ds_inv);
        h2_scale(*a.src_bound, xs, xs_inv);
    }

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t L = a.remap ? xcd_swizzle(blockIdx.x, gridDim.x) : blockIdx.x;
    const int split = int(L / uint32_t(a.grid_r));
    const int r0 = int(L - uint32_t(split) * uint32_t(a.grid_r)) * 64;
    const int pw_n = a.wo / PW, ph_n = a.ho / PH, pimg = pw_n * ph_n;
    const int npatch = a.n_img_w * pimg;
    const int pbeg = split * a.kchunk, pend = min(npatch, pbeg + a.kchunk);

    const __amdgpu_buffer_rsrc_t rs_rows = make_rsrc(a.rows, a.rows_bytes);
    const __amdgpu_buffer_rsrc_t rs_src = make_rsrc(a.src, a.src_bytes);
    const __amdgpu_buffer_rsrc_t rs_y = make_rsrc(RBN ? a.rows_y : a.rows, RBN ? a.y_bytes : 0u);

    StageT<SB> ra[A_PER], rb[B_PER], ya[RBN ? A_PER : 1];
    f32x4 x_sc, x_sh;      // src transform coefficients of this thread's 4 channels (cq = tid & 3)
    f32x4 r_mu, r_iv, r_sc, r_sf, r_k1, r_k2, r_mul;  // RBN: this thread's 4 rows r0 + 4 (tid & 15) + 0..3
    uint32_t x_valid = 0;  // bit i: halo piece i is inside the image (the padding stays zero)
    auto load_patch = [&](int pi) {
        const int img = pi / pimg, pr = pi - img * pimg;
        if (a.src_scale) {
            const int ch = (img / a.src_seg_imgs) * a.C + (tid & 3) * 4;
            x_sc = gload4(a.src_scale + ch);  // h2: times xs where consumed (store_patch)
            x_sh = gload4(a.src_shift + ch);
        }
        if constexpr (RBN) {
            const int c = r0 + (tid & 15) * 4, o = (img / a.rows_seg_imgs) * a.R + c;
            r_mu = gload4(a.rbn_mean + o);
            r_iv = gload4(a.rbn_inv + o);
            r_sc = gload4(a.rbn_scale + o);
            r_sf = gload4(a.rbn_shift + o);
            const f32x4 c0 = gload4(a.rbn_coef + 2 * o), c1 = gload4(a.rbn_coef + 2 * o + 4);
            r_k1 = f32x4{c0[0], c0[2], c1[0], c1[2]};
            r_k2 = f32x4{c0[1], c0[3], c1[1], c1[3]};
            r_mul = (a.rbn_gamma ? gload4(a.rbn_gamma + c) : f32x4{1.f, 1.f, 1.f, 1.f}) * r_iv;
        }
        x_valid = 0;
        const int y0 = patch_y0(pr, pw_n, ph_n, PH), x0 = patch_x0(pr, pw_n, ph_n, PW);
#pragma unroll
        for (int i = 0; i < A_PER; ++i) {
            const int e = tid + i * 256, q = e >> 4, cq = e & 15;
            const int py = q >> 4, px = q & 15;
            const int pix = (img * a.ho + y0 + py) * a.wo + x0 + px;
            ra[i] = bload_q<SB>(rs_rows, uint32_t(pix * a.ldc_r + r0 + cq * 4) * EB);
            if constexpr (RBN) ya[i] = bload_q<SB>(rs_y, uint32_t(pix * a.ldc_y + r0 + cq * 4) * EB);
        }
#pragma unroll
        for (int i = 0; i < B_PER; ++i) {
            const int e = tid + i * 256, hp = e >> 2, cq = e & 3;
            const int hy = hp / HW_, hx = hp - (hp / HW_) * HW_;
            const int sy = y0 - 1 + hy, sx = x0 - 1 + hx;
            const bool v = e < B_CH && unsigned(sy) < unsigned(a.hs) && unsigned(sx) < unsigned(a.ws);
            x_valid |= uint32_t(v) << i;
            rb[i] = bload_q<SB>(rs_src, v ? uint32_t(((img * a.hs + sy) * a.ws + sx) * a.ldc_s + cq * 4) * EB : kOOB);
        }
    };
    auto store_patch = [&]() {
        const f32x4 sc = H2 ? x_sc * xs : x_sc, sh = H2 ? x_sh * xs : x_sh;  // as in wgrad_halo16_x3
#pragma unroll
        for (int i = 0; i < A_PER; ++i) {
            const int e = tid + i * 256;
            const int o = (e >> 4) * RS + (e & 15) * 8;
            u32x2 h, m, l;
            if constexpr (SB) {  // dY formed in fp32 from the bf16 da and y, rounded once (as bn_bwd_apply stores it)
                if constexpr (RBN)
                    h = pk_bf16x4(bn_bwd_dy4(unpk_bf16x4(ya[i]), unpk_bf16x4(ra[i]), r_mu, r_iv, r_sc, r_sf, r_k1,
                                             r_k2, r_mul));
                else
                    h = ra[i];
                *reinterpret_cast<u32x2 *>(smem + o) = h;
                continue;
            } else {
                if constexpr (RBN) ra[i] = bn_bwd_dy4(ya[i], ra[i], r_mu, r_iv, r_sc, r_sf, r_k1, r_k2, r_mul);
            }
            if constexpr (H2) {
                split2h_pre(ra[i] * ds, h, m);
                *reinterpret_cast<u32x2 *>(smem + PA + o) = m;
            } else if constexpr (DP == 3) {
                split3(ra[i], h, m, l);
                *reinterpret_cast<u32x2 *>(smem + PA + o) = m;
                *reinterpret_cast<u32x2 *>(smem + 2 * PA + o) = l;
            } else {
                h = stage_bits<SB>(ra[i]);
            }
            *reinterpret_cast<u32x2 *>(smem + o) = h;
        }
#pragma unroll
        for (int i = 0; i < B_PER; ++i)
            if constexpr (SB) {
                if (tid + i * 256 < B_CH) {
                    u32x2 h = rb[i];
                    if (a.src_scale) {
                        const bool v = (x_valid >> i) & 1u;
                        f32x4 x = unpk_bf16x4(rb[i]);
#pragma unroll
                        for (int q = 0; q < 4; ++q) x[q] = v ? fmaxf(fmaf(x[q], sc[q], sh[q]), 0.f) : 0.f;
                        h = pk_bf16x4(x);
                    }
                    const int e = tid + i * 256;
                    *reinterpret_cast<u32x2 *>(smem + DP * PA + (e >> 2) * RSX + (e & 3) * 8) = h;
                }
            } else if (tid + i * 256 < B_CH) {
                u32x2 h, m, l;
                if (a.src_scale) {
                    const bool v = (x_valid >> i) & 1u;
#pragma unroll
                    for (int q = 0; q < 4; ++q) rb[i][q] = v ? fmaxf(fmaf(rb[i][q], sc[q], sh[q]), 0.f) : 0.f;
                } else if constexpr (H2) {
                    rb[i] *= xs;
                }
                const int e = tid + i * 256;
                const int o = DP * PA + (e >> 2) * RSX + (e & 3) * 8;
                if constexpr (H2) {
                    split2h(rb[i], h, m);
                    *reinterpret_cast<u32x2 *>(smem + PB + o) = m;
                } else if constexpr (XP >= 2) {
                    split3(rb[i], h, m, l);
                    *reinterpret_cast<u32x2 *>(smem + PB + o) = m;
                    if constexpr (XP == 3) *reinterpret_cast<u32x2 *>(smem + 2 * PB + o) = l;
                } else {
                    h[0] = cvt_pk_bf16(rb[i][0], rb[i][1]);
                    h[1] = cvt_pk_bf16(rb[i][2], rb[i][3]);
                }
                *reinterpret_cast<u32x2 *>(smem + o) = h;
            }
    };

    f32x4 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

    // lane roles as wgrad_halo16_x3: group g supplies patch pixels (g >> 1, 4(g & 1) + (w16 >> 2)) (+8 for the
    // second read of a fragment) and columns 4(w16 & 3)..+3 of the wave's 16 r / the 16 channels
    const int g = lane >> 4, w16 = lane & 15;
    const int py = g >> 1, pxq = 4 * (g & 1) + (w16 >> 2);
    const uint32_t dbase = lds_addr(smem) + (py * PW + pxq) * RS + (16 * wid + 4 * (w16 & 3)) * 2;
    const uint32_t xbase = lds_addr(smem) + DP * PA + (py * HW_ + pxq) * RSX + (4 * (w16 & 3)) * 2;

    if (pbeg < pend) {
        load_patch(pbeg);
        store_patch();
        __syncthreads();
        for (int pi = pbeg; pi < pend; ++pi) {
            const bool more = pi + 1 < pend;
            if (more) load_patch(pi + 1);
            s16x4 fa[6];
            tr_read<0 * PA + 0>(fa[0], dbase);
            tr_read<0 * PA + 8 * RS>(fa[1], dbase);
            if constexpr (DP >= 2) {
                tr_read<1 * PA + 0>(fa[2], dbase);
                tr_read<1 * PA + 8 * RS>(fa[3], dbase);
            }
            if constexpr (DP == 3) {
                tr_read<2 * PA + 0>(fa[4], dbase);
                tr_read<2 * PA + 8 * RS>(fa[5], dbase);
            }
            bf16x8 dv[3];
#pragma unroll
            for (int p = 0; p < DP; ++p) dv[p] = cat8(fa[2 * p], fa[2 * p + 1]);
            s16x4 f0[6], f1[6];
            c16_read_x<0, PB, HW_, NP>(f0, xbase);
            c16_read_x<1, PB, HW_, NP>(f1, xbase);
            c16_chain<0, PB, HW_, NP>(acc, dv, f0, f1, xbase);
            if (more) {
                __syncthreads();  // every wave is done with this patch
                store_patch();
                __syncthreads();
            }
        }
    }

    if constexpr (H2) {
        const float k = ds_inv * xs_inv;  // exact: a power of two
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[t] *= k;
    }
    // acc[t][q]: r = r0 + 16 wid + (lane & 15), c = 4g + q
    float *slab = a.slabs + size_t(split) * a.R * a.Ng;
    const int row = r0 + 16 * wid + w16;
#pragma unroll
    for (int t = 0; t < 9; ++t) gstore4(slab + size_t(row) * a.Ng + t * 16 + 4 * g, acc[t]);
}

// h2 runs where both operands are bounded, x3 otherwise.
static int wgrad16_planes(int math, uint32_t tune, bool bounded) {
    return math_planes(math) == 2 ? (bounded ? (h2_prescale(tune) ? 4 : 2) : 3) : math_planes(math);
}
// The 16-channel kernel's arithmetic: h2 with the pre-scaled low term only (SCD_TUNE_H2_NO_PRESCALE keeps it on x3).
int wgrad_c16_planes(int math, uint32_t tune, bool bounded) {
    const int np = wgrad16_planes(math, tune, bounded);
    return np == 2 ? 3 : np;
}
const void *wgrad_halo16_c16_fn(int math, uint32_t tune, bool bounded) {
    switch (wgrad_c16_planes(math, tune, bounded)) {
        case 1: return reinterpret_cast<const void *>(&wgrad_halo16_c16<1, false>);
        case 4: return reinterpret_cast<const void *>(&wgrad_halo16_c16<4, false>);
        case 5: return reinterpret_cast<const void *>(&wgrad_halo16_c16<5, false>);
        default: return reinterpret_cast<const void *>(&wgrad_halo16_c16<3, false>);
    }
}
template <bool RBN>
static void launch_c16(const WgradArgs &a, dim3 grid, hipStream_t s) {
    switch (wgrad_c16_planes(a.math, a.tune, a.rows_bound && a.src_bound)) {
        case 1:
            if (a.sb)
                hipLaunchKernelGGL((wgrad_halo16_c16<1, RBN, true>), grid, dim3(256), 0, s, a);
            else
                hipLaunchKernelGGL((wgrad_halo16_c16<1, RBN>), grid, dim3(256), 0, s, a);
            break;
        case 4: hipLaunchKernelGGL((wgrad_halo16_c16<4, RBN>), grid, dim3(256), 0, s, a); break;
        case 5: hipLaunchKernelGGL((wgrad_halo16_c16<5, RBN>), grid, dim3(256), 0, s, a); break;
        default: hipLaunchKernelGGL((wgrad_halo16_c16<3, RBN>), grid, dim3(256), 0, s, a);
    }
}
void launch_wgrad_halo16_c16(const WgradArgs &a, dim3 grid, hipStream_t s) {
    if (a.rows_y)
        launch_c16<true>(a, grid, s);
    else
        launch_c16<false>(a, grid, s);
}
// Wave layout of the h2 and bf16 variants (W16L): SCD_TUNE_W16_LAYOUT_2X2 keeps the 2x2 layout, default along c.
// x3 / x5 keep 2x2: their third dY plane does not fit four r blocks in registers.
static int w16_layout(uint32_t tune) { return (tune & SCD_TUNE_W16_LAYOUT_2X2) ? 0 : 1; }
// Rows of dY per block: 128 (RG 2) for the h2 / bf16 variants in the along-c layout when R % 128 == 0, else 64
// (SCD_TUNE_WGRAD_R64: always 64; plan and launch see the same descriptor bits).
int wgrad16_rblock(int math, uint32_t tune, int R, bool bounded) {
    const int np = wgrad16_planes(math, tune, bounded);
    if (!(np == 1 || np == 2 || np == 4) || !w16_layout(tune) || R % 128) return 64;
    return (tune & SCD_TUNE_WGRAD_R64) ? 64 : 128;
}
template <int NP>
static const void *w16_kernel(int lc, int rb) {
    return rb == 128 ? reinterpret_cast<const void *>(&wgrad_halo16_x3<NP, 1, 2>)
           : lc      ? reinterpret_cast<const void *>(&wgrad_halo16_x3<NP, 1, 1>)
                     : reinterpret_cast<const void *>(&wgrad_halo16_x3<NP, 0, 1>);
}
template <int NP, bool SB = false>
static void w16_launch(int lc, int rb, const WgradArgs &a, dim3 grid, hipStream_t s) {
    if constexpr (NP == 4 && !SB) {
        if ((a.tune & SCD_TUNE_WGRAD16_DB) && lc) {
            if (rb == 128)
                hipLaunchKernelGGL((wgrad_halo16_x3<NP, 1, 2, false, true>), grid, dim3(512), 0, s, a);
            else
                hipLaunchKernelGGL((wgrad_halo16_x3<NP, 1, 1, false, true>), grid, dim3(256), 0, s, a);
            return;
        }
    }
    if (rb == 128)
        hipLaunchKernelGGL((wgrad_halo16_x3<NP, 1, 2, SB>), grid, dim3(512), 0, s, a);
    else if (lc)
        hipLaunchKernelGGL((wgrad_halo16_x3<NP, 1, 1, SB>), grid, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((wgrad_halo16_x3<NP, 0, 1, SB>), grid, dim3(256), 0, s, a);
}
const void *wgrad_halo16_fn(int math, uint32_t tune, bool bounded, int rblock) {
    switch (wgrad16_planes(math, tune, bounded)) {
        case 1: return w16_kernel<1>(w16_layout(tune), rblock);
        case 2: return w16_kernel<2>(w16_layout(tune), rblock);
        case 4: return w16_kernel<4>(w16_layout(tune), rblock);
        case 5: return reinterpret_cast<const void *>(&wgrad_halo16_x3<5, 0, 1>);
        default: return reinterpret_cast<const void *>(&wgrad_halo16_x3<3, 0, 1>);
    }
}
// The rows transform (a.rows_y): h2 with the pre-scaled low term, or bf16, in the along-c layout
// (wgrad16_rows_bn_ok); both row-block sizes.
template <int NP, bool SB>
static void w16_launch_rbn(int rb, const WgradArgs &a, dim3 grid, hipStream_t s) {
    if (rb == 128)
        hipLaunchKernelGGL((wgrad_halo16_x3<NP, 1, 2, SB, false, true>), grid, dim3(512), 0, s, a);
    else
        hipLaunchKernelGGL((wgrad_halo16_x3<NP, 1, 1, SB, false, true>), grid, dim3(256), 0, s, a);
}
bool wgrad16_rows_bn_ok(int math, uint32_t tune, bool bounded) {
    const int np = wgrad16_planes(math, tune, bounded);
    return (np == 1 || np == 4) && w16_layout(tune) && !(tune & SCD_TUNE_WGRAD16_DB);
}
// a.grid_r = R / wgrad16_rblock(...) (the caller plans with the same choice).
void launch_wgrad_halo16_x3(const WgradArgs &a, dim3 grid, hipStream_t s) {
    const bool bounded = a.rows_bound && a.src_bound;
    const int lc = w16_layout(a.tune), rb = wgrad16_rblock(a.math, a.tune, a.R, bounded);
    if (a.rows_y) {  // the caller checked wgrad16_rows_bn_ok
        if (wgrad16_planes(a.math, a.tune, bounded) == 4)
            w16_launch_rbn<4, false>(rb, a, grid, s);
        else if (SCD_WGRAD16_DMA_TRANSFORMS && a.sb && !(a.tune & SCD_TUNE_WGRAD16_REGSTAGE) &&
                 (!a.src_scale || a.n_img_w / a.src_seg_imgs <= 2)) {
            // bf16 storage: the LDS-DMA ring with y and dL/da landed raw and dY formed in place (+ the source transform)
            if (rb == 128) {
                if (a.src_scale)
                    hipLaunchKernelGGL((wgrad_halo16_dma<2, 5, true, true>), grid, dim3(512), 0, s, a);
                else
                    hipLaunchKernelGGL((wgrad_halo16_dma<2, 5, false, true>), grid, dim3(512), 0, s, a);
            } else if (a.src_scale)
                hipLaunchKernelGGL((wgrad_halo16_dma<1, 3, true, true>), grid, dim3(256), 0, s, a);
            else
                hipLaunchKernelGGL((wgrad_halo16_dma<1, 3, false, true>), grid, dim3(256), 0, s, a);
        } else if (a.sb)
            w16_launch_rbn<1, true>(rb, a, grid, s);
        else
            w16_launch_rbn<1, false>(rb, a, grid, s);
        return;
    }
    switch (wgrad16_planes(a.math, a.tune, bounded)) {
        case 1:
            if (a.sb && lc && !(a.tune & SCD_TUNE_WGRAD16_REGSTAGE) &&
                (!a.src_scale || (SCD_WGRAD16_DMA_TRANSFORMS && a.n_img_w / a.src_seg_imgs <= 2))) {
                // bf16 storage: the LDS-DMA ring (same residency as the register-staged kernel: one 512-thread block /
                // two 256-thread blocks per CU, so the split plan is unchanged); a source transform in place
                if (a.src_scale) {
                    if (rb == 128)
                        hipLaunchKernelGGL((wgrad_halo16_dma<2, SCD_WGRAD16_DMA_NB_XT, true>), grid, dim3(512), 0, s, a);
                    else
                        hipLaunchKernelGGL((wgrad_halo16_dma<1, SCD_WGRAD16_DMA_NB, true>), grid, dim3(256), 0, s, a);
                } else if (rb == 128)
                    hipLaunchKernelGGL((wgrad_halo16_dma<2, SCD_WGRAD16_DMA_NB>), grid, dim3(512), 0, s, a);
                else
                    hipLaunchKernelGGL((wgrad_halo16_dma<1, SCD_WGRAD16_DMA_NB>), grid, dim3(256), 0, s, a);
            } else if (a.sb)
                w16_launch<1, true>(lc, rb, a, grid, s);
            else
                w16_launch<1>(lc, rb, a, grid, s);
            break;
        case 2: w16_launch<2>(lc, rb, a, grid, s); break;
        case 4: w16_launch<4>(lc, rb, a, grid, s); break;
        case 5: hipLaunchKernelGGL((wgrad_halo16_x3<5, 0, 1>), grid, dim3(256), 0, s, a); break;
        default: hipLaunchKernelGGL((wgrad_halo16_x3<3, 0, 1>), grid, dim3(256), 0, s, a);
    }
}

}  // namespace scd

using namespace scd;
