// Gather igemm in the h2 arithmetic (x3_common.h; v_mfma_f32_16x16x32_f16) or in bf16 (v_mfma_f32_16x16x32_bf16):
// the ConvTranspose2d(k=2, s=2) forward (one tap, pixel-shuffle store, networks.py:433) and its data grad (four taps
// gathered with stride 2).
//
// These convs have no tap reuse (every source pixel feeds one k-step of one output pixel), so the halo16 kernel's
// shape does not apply; they ran on the generic per-tap x3 kernel (igemm_x3: six 32x32x16 bf16 products per
// 16-deep step, one barrier per step, scalar stores) at 80-100 TFLOP/s.  Here:
//   - a block owns BM pixels x BN output channels; a stage holds SK 32-channel k-steps of the gathered pixel rows,
//     scaled by the power of two of *src_bound and split into the fp16 h / pre-scaled m planes ([row][32 fp16],
//     64-byte rows, the halo16 LDS swizzle: 16 consecutive rows from any start are conflict-free);
//   - two stage buffers: the next stage's global loads are issued before the current stage's MFMAs and written
//     to the other buffer after them, one barrier per stage;
//   - weights (scd_split_h2_frag layout, per-row inverse scales after the planes) go straight into registers one
//     k-step ahead, exactly as in igemm_halo16_x3;
//   - roles as in the halo16 kernel: A = weights (rows = output channels), B = pixels, so a lane's accumulator
//     holds 4 consecutive channels of one pixel and leaves as one 16-byte store (store_mode 1: to the pixel
//     (2y + di, 2x + dj) of the upsampled map, with dst_bound raised to the max |stored value|).
// The products (w_h 2^-11) x_m', w_m x_h, w_h x_h are the halo16 kernel's NP = 4 expressions; NP = 1 (bf16) stages
// one bf16 plane (RNE) and runs w_h x_h on plane 0 of the bf16 weight split, the bf16 halo16 kernel's product.
#include "x3_common.h"

namespace scd {

// SB: bf16 storage of src and dst (bf16 arithmetic only).
// (Persistent blocks walking several tiles with the next tile's first stage loaded early were measured slower in round
// 4, step 30.07 -> 30.29 ms, profiles/r04_variants_ab.txt, and removed in round 6; the tile loop below keeps one tile.)
template <int WM, int WN, int TM, int TN, int SK, int OCC, int NP, bool SB = false>
__global__ __launch_bounds__(64 * WM * WN, OCC) void igemm_gather16(IgemmArgs a) {
    static_assert(NP == 1 || NP == 4, "bf16 or h2");
    static_assert(!SB || NP == 1, "bf16 storage runs the bf16 arithmetic");
    using ST = typename std::conditional<SB, bf16_t, float>::type;
    constexpr bool H2 = NP == 4;
    constexpr int XP = H2 ? 2 : 1;  // activation planes (LDS) = weight planes (registers)
    constexpr int NT = 64 * WM * WN;
    constexpr int WPX = TM * 16, WCH = TN * 16;
    constexpr int BM = WM * WPX, BN = WN * WCH;
    constexpr int PL = BM * 64;          // one fp16 plane of one 32-channel k-step
    constexpr int STG = SK * XP * PL;    // one stage: SK k-steps x (h, m) / (h)
    constexpr int A_PER = BM * 8 / NT;   // 16-byte (4-channel) pieces per thread and k-step
    static_assert((BM * 8) % NT == 0 && NT % 8 == 0, "pieces tile the block");
    __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STG];
    // the epilogue's per-channel scale and bias of the block's BN channels, per tile parity (P: a tile's are written
    // at its start, while the other half may still be read by the previous tile's epilogue)
    __shared__ __attribute__((aligned(16))) float ep_sc[2][BN], ep_b[2][BN];
    float xs = 1.f, xs_inv = 1.f;
    if constexpr (H2) h2_scale(*a.src_bound, xs, xs_inv);

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid % WM, wn = wid / WM;
    const int g = lane >> 4, l16 = lane & 15;
    const uint32_t ntile = uint32_t(a.grid_m * a.grid_n);
    auto tile_of = [&](uint32_t q, int &m0_, int &n0_) {
        int mt, nt;
        if (a.remap) {  // N fastest: the n-tiles of one pixel tile (sharing its gathered rows) under one L2
            const uint32_t L = xcd_swizzle(q, ntile);
            mt = int(L / uint32_t(a.grid_n));
            nt = int(L - uint32_t(mt) * uint32_t(a.grid_n));
        } else {
            mt = int(q % uint32_t(a.grid_m));
            nt = int(q / uint32_t(a.grid_m));
        }
        m0_ = mt * BM;
        n0_ = nt * BN;
    };
    uint32_t q = blockIdx.x;
    int m0, n0;
    tile_of(q, m0, n0);

    auto soff = [](int row, int col) { return row * 64 + ((((col >> 1) ^ (row >> 1)) & 3) << 4) + ((col & 1) << 3); };

    // this thread's pieces: pixel rows (tid >> 3) + i * NT / 8, channel piece tid & 7 of every k-step
    const int col = tid & 7;
    const ST *a_base[A_PER];
    int a_sy[A_PER], a_sx[A_PER], a_off[A_PER];
#pragma unroll
    for (int i = 0; i < A_PER; ++i) a_off[i] = soff((tid >> 3) + i * (NT / 8), col);
    auto set_rows = [&](int m0_) {
#pragma unroll
        for (int i = 0; i < A_PER; ++i) {
            const int m = m0_ + (tid >> 3) + i * (NT / 8);
            const bool ok = m < a.M;
            const uint32_t mm = ok ? uint32_t(m) : 0u;
            const uint32_t img = fdiv(mm, a.div_hw);
            const uint32_t r = mm - img * uint32_t(a.ho * a.wo);
            const uint32_t oy = fdiv(r, a.div_w);
            const uint32_t ox = r - oy * uint32_t(a.wo);
            a_sy[i] = ok ? int(oy) * a.stride : -(1 << 20);
            a_sx[i] = int(ox) * a.stride;
            a_base[i] = reinterpret_cast<const ST *>(a.src) +
                        (size_t(int(img) * a.hs + (ok ? a_sy[i] : 0)) * a.ws + a_sx[i]) * a.ldc_s + col * 4;
        }
    };
    set_rows(m0);
    const int KS16 = a.K / 16, NB32 = (a.n_out + 31) / 32;
    const uint32_t wplane_b = uint32_t(a.wplane) * 2u;
    uint32_t w_base[TN];
    auto set_wbase = [&](int n0_) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int cb = (n0_ >> 4) + wn * TN + j;  // 16-channel block
            const int nb = cb >> 1;
            w_base[j] = nb < NB32 ? uint32_t(nb * KS16 + (g >> 1)) * 1024u +
                                        uint32_t(16 * (cb & 1) + l16 + 32 * (g & 1)) * 16u
                                  : kOOB;
        }
    };
    set_wbase(n0);
    const __amdgpu_buffer_rsrc_t rs_w = make_rsrc(a.wsplit, uint32_t(XP) * wplane_b);

    const int cpk = a.c / 32;
    const int nk = a.ntaps * cpk;  // k-steps (a multiple of SK: gather16_pick)
    StageT<SB> ra[SK][A_PER];
    auto load_stage = [&](int st) {
#pragma unroll
        for (int s = 0; s < SK; ++s) {
            const int q = st * SK + s;
            const int t = q / cpk, cc = q - t * cpk;
            const int dyt = tap_at(a.tdy, t), dxt = tap_at(a.tdx, t);
            const long toff = long(dyt * a.ws + dxt) * a.ldc_s + cc * 32;
#pragma unroll
            for (int i = 0; i < A_PER; ++i) {
                const bool v = unsigned(a_sy[i] + dyt) < unsigned(a.hs) && unsigned(a_sx[i] + dxt) < unsigned(a.ws);
                if constexpr (SB)
                    ra[s][i] = v ? *(const __attribute__((address_space(1))) u32x2 *)(a_base[i] + toff) : u32x2{0u, 0u};
                else
                    ra[s][i] = v ? gload4(a_base[i] + toff) : f32x4{0.f, 0.f, 0.f, 0.f};
            }
        }
    };
    auto store_stage = [&](int buf) {
        unsigned char *const sb = smem + buf * STG;
#pragma unroll
        for (int s = 0; s < SK; ++s)
#pragma unroll
            for (int i = 0; i < A_PER; ++i) {
                u32x2 h, m;
                if constexpr (H2) {
                    split2h_pre(ra[s][i] * xs, h, m);
                    *reinterpret_cast<u32x2 *>(sb + s * XP * PL + PL + a_off[i]) = m;
                } else {
                    h = stage_bits<SB>(ra[s][i]);
                }
                *reinterpret_cast<u32x2 *>(sb + s * XP * PL + a_off[i]) = h;
            }
    };
    u32x4 wq[XP][TN];
    auto load_W = [&](int q) {
        const uint32_t ko = uint32_t(q) * 2048u;  // 32-deep step = two 16-deep fragments
#pragma unroll
        for (int p = 0; p < XP; ++p)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                wq[p][j] = bload4u(rs_w, w_base[j] == kOOB ? kOOB : w_base[j] + ko + uint32_t(p) * wplane_b);
    };

    f32x4 acc[TN][TM];
    int x_rd[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int p = wm * WPX + i * 16 + l16;
        x_rd[i] = p * 64 + (((g ^ (p >> 1)) & 3) << 4);
    }

    const int nst = nk / SK;
    const float *winv = reinterpret_cast<const float *>(reinterpret_cast<const unsigned char *>(a.wsplit) + 2u * wplane_b);
    float omax = 0.f;
    load_stage(0);
    load_W(0);
    store_stage(0);
    __syncthreads();
    int buf = 0;   // stage buffer of the current stage (stages run on across the tiles of a persistent block)
    int tpar = 0;  // tile parity (epilogue constants)
    for (;;) {
    const uint32_t qn = q + gridDim.x;
    const bool has_next = false && qn < ntile;
    int nm0 = 0, nn0 = 0;
    if (has_next) tile_of(qn, nm0, nn0);
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the epilogue's per-channel scale and bias into LDS now, before any of the next tile's stage loads (vmcnt retires
    // in order: loaded in the epilogue they would wait for those); read after at least one stage barrier
    for (int c = tid; c < BN; c += NT) {
        const int n = n0 + c;
        const int oc = a.store_mode == 1 ? n - (n / a.cout) * a.cout : n;
        const bool nok = n < a.n_out;
        ep_sc[tpar][c] = H2 && nok ? winv[n] * xs_inv : 1.f;
        ep_b[tpar][c] = a.bias && nok ? a.bias[oc] : 0.f;
    }
    for (int st = 0; st < nst; ++st) {
        const bool more = st + 1 < nst;
        if (more) {
            load_stage(st + 1);
        } else if (has_next) {  // the next tile's first stage, behind this tile's last MFMAs and its epilogue
            set_rows(nm0);
            load_stage(0);
        }
        const unsigned char *const sb = smem + buf * STG;
#pragma unroll
        for (int s = 0; s < SK; ++s) {
            u32x4 xh[TM], xm[TM];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                xh[i] = *reinterpret_cast<const u32x4 *>(sb + s * XP * PL + x_rd[i]);
                if constexpr (H2) xm[i] = *reinterpret_cast<const u32x4 *>(sb + s * XP * PL + PL + x_rd[i]);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                if constexpr (H2) {
                    const u32x4 wl = f16_down11(wq[0][j]);
#pragma unroll
                    for (int i = 0; i < TM; ++i) {
                        acc[j][i] = mfma16_f16(wl, xm[i], acc[j][i]);
                        acc[j][i] = mfma16_f16(wq[XP - 1][j], xh[i], acc[j][i]);
                        acc[j][i] = mfma16_f16(wq[0][j], xh[i], acc[j][i]);
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < TM; ++i)
                        acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wq[0][j]),
                                                                            __builtin_bit_cast(bf16x8, xh[i]),
                                                                            acc[j][i], 0, 0, 0);
                }
            }
            if (st * SK + s + 1 < nk) {
                load_W(st * SK + s + 1);  // next k-step's fragments (L2), one step ahead
            } else if (has_next) {
                set_wbase(nn0);
                load_W(0);
            }
        }
        // the other buffer was last read in stage st - 1, which every wave has left (barrier below)
        if (more || has_next) store_stage(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }

    // h2: undo the operand scales (powers of two: exact); add the bias, store 4 channels per lane.  A lane's pixel
    // addresses depend on i only (store_mode 1: the upsampled pixel (2y, 2x); tap (di, dj) of channel tile j adds
    // di rows + dj pixels), so they are formed once per i, not once per (i, j).
    constexpr uint32_t EB = SB ? 2u : 4u;
    size_t e_pix[TM];  // element offset of pixel tile i's pixel (store_mode 1: of its (2y, 2x) pixel)
    bool m_ok[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm * WPX + i * 16 + l16;
        m_ok[i] = m < a.M;
        size_t pix = size_t(m);
        if (a.store_mode == 1) {
            const uint32_t mm = m_ok[i] ? uint32_t(m) : 0u;
            const uint32_t img = fdiv(mm, a.div_hw);
            const uint32_t r = mm - img * uint32_t(a.ho * a.wo);
            const uint32_t oy = fdiv(r, a.div_w);
            const uint32_t ox = r - oy * uint32_t(a.wo);
            pix = size_t(int(img) * a.dst_h + 2 * int(oy)) * a.dst_w + 2 * int(ox);
        }
        e_pix[i] = pix * a.ldc_d;
    }
    unsigned char *const dst_b = reinterpret_cast<unsigned char *>(a.dst);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WCH + j * 16 + 4 * g;
        if (n >= a.n_out) continue;  // n_out % 4 == 0: a lane's 4 channels are all in or all out
        const int nl = wn * WCH + j * 16 + 4 * g;
        const f32x4 sc = *reinterpret_cast<const f32x4 *>(&ep_sc[tpar][nl]);
        size_t e_j = size_t(n);  // element offset of channel tile j within a pixel tile's row
        if (a.store_mode == 1) {
            const int ij = n / a.cout;
            const int oc = n - ij * a.cout, di = ij >> 1, dj = ij & 1;
            e_j = size_t(di * a.dst_w + dj) * a.ldc_d + oc;
        }
        const f32x4 b4 = *reinterpret_cast<const f32x4 *>(&ep_b[tpar][nl]);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            if (!m_ok[i]) continue;
            const f32x4 v = acc[j][i] * sc + b4;
            store_qb<SB>(dst_b + (e_pix[i] + e_j) * EB, v);
            if (a.dst_bound)  // uniform; no bound in the bf16 arithmetic
                omax = fmaxf(omax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
        }
    }
    if (!has_next) break;
    q = qn;
    m0 = nm0;
    n0 = nn0;
    tpar ^= 1;
    }
    if (a.dst_bound) wave_max_bound(a.dst_bound, fmaxf(omax, bound_seed(a)));  // uniform: every lane of the wave takes part
}

namespace {
// Tiles: 0 = 128 px x 128 ch (2x2 waves of 64 x 64), 1 = 128 x 64 (2x2 of 64 x 32), 2 = 64 x 128 (2x2 of 32 x 64)
constexpr int kSK = 2;  // 32-channel k-steps per stage

int gather16_enabled(uint32_t tune) { return (tune & SCD_TUNE_NO_GATHER16) ? 0 : 1; }

template <int WM, int WN, int TM, int TN, int OCC, int NP, bool SB = false>
void launch_g16(const IgemmArgs &a, hipStream_t s) {
    constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
    IgemmArgs b = a;
    b.grid_m = (a.M + BM - 1) / BM;
    b.grid_n = (a.n_out + BN - 1) / BN;
    b.remap = xcd_remap_enabled(a.tune);
    const uint32_t ntile = uint32_t(b.grid_m * b.grid_n);
    hipLaunchKernelGGL((igemm_gather16<WM, WN, TM, TN, kSK, OCC, NP, SB>), dim3(ntile), dim3(64 * WM * WN), 0, s, b);
}

// h2 with the h2 weight split and a source bound; bf16 on plane 0 of the bf16 weight split (no bound needed)
bool gather16_h2(const IgemmArgs &a) { return a.src_bound && h2_weight_format(a.math, a.ntaps, a.c); }

template <int WM, int WN, int TM, int TN, int OCC>
void launch_g16_math(const IgemmArgs &a, hipStream_t s) {
    if (gather16_h2(a))
        launch_g16<WM, WN, TM, TN, OCC, 4>(a, s);
    else if (a.sb)
        launch_g16<WM, WN, TM, TN, OCC, 1, true>(a, s);
    else
        launch_g16<WM, WN, TM, TN, OCC, 1>(a, s);
}
}  // namespace

// 1 + tile id when `a` takes the gather kernel (h2-split weights and a bound of the source, or the bf16 arithmetic;
// the shape constraints below), else 0.  Convs with 9 taps go to the halo kernels instead.
int gather16_pick(const IgemmArgs &a) {
    if (!a.wsplit || a.ntaps == 9 || !(gather16_h2(a) || a.math == SCD_MATH_BF16) || !gather16_enabled(a.tune))
        return 0;
    if (a.c % 32 || (a.ntaps * (a.c / 32)) % kSK || a.n_out % 64 || a.ldc_s % 4 || a.ldc_d % 4 || a.K != a.ntaps * a.c ||
        (reinterpret_cast<uintptr_t>(a.src) & (a.sb ? 7 : 15)) || (reinterpret_cast<uintptr_t>(a.dst) & (a.sb ? 7 : 15)) ||
        (a.sb && a.math != SCD_MATH_BF16) ||
        (a.bias && (reinterpret_cast<uintptr_t>(a.bias) & 15)) || (a.store_mode != 0 && a.store_mode != 1) ||
        (a.store_mode == 1 && (a.cout % 4 || a.n_out != 4 * a.cout)) || 2 * a.wplane * 2 >= (int64_t(1) << 31))
        return 0;
    // SCD_TUNE_X3_TILE(1..3) forces tile 0..2 here (tile study, tools/perf_convT.py --math h2)
    const int forced = int((a.tune & SCD_TUNE_X3_TILE_MASK) >> 12);
    if (forced >= 1 && forced <= 3) return forced;
    if (a.n_out % 128) return 2;  // 128 x 64
    const int64_t big = int64_t((a.M + 127) / 128) * (a.n_out / 128);
    return big >= 512 ? 1 : 3;  // 64 x 128 when 128 x 128 tiles leave CUs idle (two blocks per CU)
}

void launch_gather16(const IgemmArgs &a, int cfg, hipStream_t s) {
    switch (cfg - 1) {
        case 0: launch_g16_math<2, 2, 4, 4, 2>(a, s); break;
        case 1: launch_g16_math<2, 2, 4, 2, 2>(a, s); break;
        default: launch_g16_math<2, 2, 2, 4, 2>(a, s); break;
    }
}

}  // namespace scd
