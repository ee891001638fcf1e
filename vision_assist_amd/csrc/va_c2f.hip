// va_c2f.hip -- one YOLOv8 C2f block (n = 1, shortcut, 64 -> 64 channels, hidden 32) as ONE kernel:
// block.py C2f.forward (cv1 -> chunk -> Bottleneck(m.0.cv1, m.0.cv2, + residual) -> cat -> cv2), the
// stride-4 backbone stage (model.2) of YOLOv8s-seg, run inside YOLO.predict (FrameProcessor.py:322).
//
// Unfused, the block is four launches moving ~1.4 GB per 64 frames at 640 x 640 through HBM (the
// 96-channel concat buffer is written, re-read in slices and re-read whole).  Here a workgroup owns a
// 16 x 16 output tile and every intermediate stays on the chip:
//
//   stage 1  cv1 (1x1, 64 -> 64) on the 20 x 20 tile + halo 2, B fragments straight from HBM.
//            Centre pixels keep both halves (a, b) in registers; the b half of every pixel goes to
//            LDS S1 (the 3x3 below needs neighbours).  Pixels outside the image are zero in S1
//            (the next conv's zero padding).
//   stage 2  m.0.cv1 (3x3, 32 -> 32) on the 18 x 18 tile + halo 1 from S1 -> LDS S2 (zero outside).
//   stage 3  m.0.cv2 (3x3, 32 -> 32) on the centre from S2, + residual b from registers -> b'.
//   stage 4  cv2 (1x1, 96 -> 64) over [a | b | b'] straight from registers -> HBM, 16-byte stores.
//
// Register hand-offs work because a 16x16x32 MFMA's C fragment (lane: 4 consecutive rows of one
// column) holds, over two 16-row groups, 8 channels of one pixel -- exactly one lane's share of a
// B fragment once the consumer's K order is permuted the same way (P32 below); the weight blob is
// pre-permuted and pre-arranged in fragment order by the host (seg.py SegNet._pack_c2f).
//
// Persistent: one 512-thread workgroup per CU walks its tiles; the 3x3 weights live in LDS, the
// 1x1 weights in registers, and the next tile's stage-1 input is loaded while the current tile's
// stages 2-4 run.  Tiles are dealt to XCDs in contiguous runs so neighbouring tiles' halo reads
// hit the same L2.  Rounding matches the unfused layers: each intermediate is bias + SiLU (+
// residual) in f32, rounded to bf16 as a stored layer would be.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "../../include/va355.h"
#include "va_dev.h"
#include "va_fuse.h"
#include "va_switch.h"

namespace {

using fz::mma;

constexpr int CF_T = 16;      // tile width (a row segment = one 16-pixel MFMA column group)
constexpr int CF_R1W = CF_T + 4, CF_R2W = CF_T + 2;  // stage-1 / stage-2 region widths (halo 2 / 1)
constexpr int CF_FRAG = fz::FRAG;
constexpr int CF_PS = 96;     // LDS bytes per pixel of S1 / S2 (32 bf16 channels + 32 bytes of padding)
// weight blob (bf16, fragment order): F1 cv1 [4 groups][2 k-steps], F2 m.0.cv1 [9 taps][2 groups],
// F3 m.0.cv2 [9][2], F4 cv2 [4 groups][3 k-steps]
constexpr int CF_F1 = 0, CF_F2 = 8 * CF_FRAG, CF_F3 = CF_F2 + 18 * CF_FRAG, CF_F4 = CF_F3 + 18 * CF_FRAG;
constexpr int CF_WBLOB = CF_F4 + 12 * CF_FRAG;  // 28672 bf16 = 56 KiB
static_assert(CF_WBLOB == 28672, "blob size (seg.py SegNet._pack_c2f)");
constexpr int CF_OOB = fz::OOB, CF_RSRC = fz::RSRC;

// Tile geometry and LDS map of one configuration: TH output rows x 16 columns per tile, NW waves,
// WPC workgroups per CU, the 1x1 weights in registers (WREG) or in LDS.
//   LDS: S1 [R1H*20 px][64 B], S2 [R2H*18 px][64 B], the weights (fragment order: one conflict-free
//   ds_read_b128 per fragment; F2/F3 only with WREG), the biases (kept out of global memory: a global
//   bias load behind the next tile's prefetch would wait for it, vmcnt is in order), 16-byte sink
//   slots that masked lanes write instead of branching.
template <int TH_, int NW_, int WPC_, bool WREG_>
struct CfCfg {
    static constexpr int TH = TH_, NW = NW_, WPC = WPC_;
    static constexpr bool WREG = WREG_;
    static constexpr int R1H = TH + 4, R2H = TH + 2;
    static constexpr int RPW = TH / NW;                         // centre rows per wave
    static constexpr int NRING = (R1H * CF_R1W - TH * CF_T) / 16;  // 16-pixel groups of the stage-1 ring
    static constexpr int NG2T = R2H + (2 * R2H + 15) / 16;       // stage-2 groups: row segments + columns 16..17
    static constexpr int NRG = (NRING + NW - 1) / NW, NG2 = (NG2T + NW - 1) / NW;
    static constexpr int S1 = 0, S2 = R1H * CF_R1W * CF_PS, WB = S2 + R2H * CF_R2W * CF_PS;
    static constexpr int W2 = WB, W3 = W2 + 18 * 1024;  // F2, F3 (, F4, F1 without WREG: blob order from F2)
    static constexpr int W4 = W3 + 18 * 1024, W1 = W4 + 12 * 1024;
    static constexpr int BIAS = WREG ? W4 : W1 + 8 * 1024;
    static constexpr int SINK = BIAS + 192 * 4;
    static constexpr int LDS = SINK + 64 * 16;
    static_assert(TH % NW == 0 && (TH * CF_T) % 16 == 0, "rows per wave");
    static_assert((LDS + 16) * WPC <= 160 * 1024, "LDS per CU (+ the work-queue slots)");
};

// 16-byte chunk c (0..3) of pixel p: pixels padded to 96 bytes, so a 3x3 tap is a constant offset
// (the ds_read immediate: one base address per pixel group instead of one per tap), and the B-fragment
// reads (16 consecutive pixels of a row per lane group) are bank-conflict free; the 16-byte writes are
// 2-way, which the write's own transfer time hides
__device__ __forceinline__ int cf_addr(int p, int c) { return p * CF_PS + 16 * c; }

struct CfGeom {
    int N, H, W, ldx, ldy, tx, tpf, ntiles;
    unsigned long long* trace;  // debug (va_c2f_trace): [grid][NW waves][CF_TR_TILES][CF_TR_PTS] clocks, or null
    int* wq;                    // the plan's work counter (va_fuse.h fz::wq_claim), or null: fz::tile's static schedule
};
constexpr int CF_TR_TILES = 32, CF_TR_PTS = 6;

// ring pixel q of the R1H x 20 stage-1 region minus its TH x 16 centre: rows 0-1, rows R1H-2..R1H-1,
// then columns 0, 1, 18, 19 of rows 2 .. R1H-3
template <int R1H>
__device__ __forceinline__ void cf_ring(int q, int& y, int& x) {
    if (q < 2 * CF_R1W) {
        y = q / CF_R1W;
        x = q % CF_R1W;
    } else if (q < 4 * CF_R1W) {
        y = R1H - 2 + (q - 2 * CF_R1W) / CF_R1W;
        x = (q - 2 * CF_R1W) % CF_R1W;
    } else {
        const int r = q - 4 * CF_R1W, c = r & 3;
        y = 2 + (r >> 2);
        x = c < 2 ? c : CF_T + c;
    }
}

// wave w owns centre rows RPW*w .. RPW*w + RPW - 1, stage-1 ring groups w + NW*i (< NRING) and
// stage-2 groups w + NW*j (< NG2T)
template <class C>
__global__ __launch_bounds__(C::NW * 64, C::WPC) void c2f_kernel(const __bf16* __restrict__ X,
                                                                const __bf16* __restrict__ wf,
                                                                const float* __restrict__ bias,
                                                                __bf16* __restrict__ Y, CfGeom g) {
    constexpr int NW = C::NW, RPW = C::RPW, NRG = C::NRG, NG2 = C::NG2, R1H = C::R1H, R2H = C::R2H;
    extern __shared__ __attribute__((aligned(16))) unsigned char cf_smem[];
    const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const float* b1 = (const float*)(cf_smem + C::BIAS);  // cv1 [64]
    const float* b2 = b1 + 64;                              // m.0.cv1 [32]
    const float* b3 = b1 + 96;                              // m.0.cv2 [32]
    const float* b4 = b1 + 128;                             // cv2 [64]

    // work queue: tile j's index in LDS slot j & 1, claimed by thread 0 in tile j - 2 as its stage 2 starts, published after that stage
    volatile int* slot = (volatile int*)(cf_smem + C::LDS);
    int t, nx;  // this tile, the next
    if (g.wq) {
        if (tid == 0) {
            slot[0] = fz::wq_claim(g.wq, g.ntiles);
            slot[1] = fz::wq_claim(g.wq, g.ntiles);
        }
        __syncthreads();
        t = __builtin_amdgcn_readfirstlane(slot[0]);
        nx = __builtin_amdgcn_readfirstlane(slot[1]);
    } else {
        t = fz::tile(g.ntiles, 0);
        nx = fz::tile(g.ntiles, 1);
    }
    if (t < 0) {
        if (g.wq && tid == 0) fz::wq_release(g.wq);
        return;
    }
    // weights and biases -> LDS (once per workgroup); with WREG the 1x1 weights -> registers
    {
        constexpr int nv = (C::WREG ? 36 : 48) * CF_FRAG / 8;
        for (int i = tid; i < nv; i += NW * 64) {
            const u32x4 v = *(const u32x4*)(wf + CF_F2 + 8 * i);  // F2, F3 (, F4)
            *(u32x4*)(cf_smem + C::W2 + 16 * i) = v;
        }
        if constexpr (!C::WREG) {
            for (int i = tid; i < 8 * CF_FRAG / 8; i += NW * 64) {
                const u32x4 v = *(const u32x4*)(wf + CF_F1 + 8 * i);
                *(u32x4*)(cf_smem + C::W1 + 16 * i) = v;
            }
        }
    }
    if (tid < 48) *(float4*)(cf_smem + C::BIAS + 16 * tid) = *(const float4*)(bias + 4 * tid);
    bf16x8 f1r[8], f4r[12];
    if constexpr (C::WREG) {
        const int l = tid & 63;
#pragma unroll
        for (int f = 0; f < 8; ++f) f1r[f] = *(const bf16x8*)(wf + CF_F1 + f * CF_FRAG + 8 * l);
#pragma unroll
        for (int f = 0; f < 12; ++f) f4r[f] = *(const bf16x8*)(wf + CF_F4 + f * CF_FRAG + 8 * l);
    }

    // stage-1 input of tile t: centre rows (pc), ring groups (pr).  Buffer loads over one frame: pixels
    // outside the image read 0 with no branch, and every load / store of the loop is unconditional, so
    // the compiler's vmcnt before stage 1 counts the stores issued after the prefetch instead of
    // waiting for them
    u32x4 pc[RPW][2], pr[NRG][2];
    const int fbytes = g.H * g.W * g.ldx * 2;
    auto load_tile = [&](int tt) {
        const int l = tid & 63, fr = l & 15, fq = l >> 4;
        const int n = tt / g.tpf, rr = tt % g.tpf, y0 = (rr / g.tx) * C::TH, x0 = (rr % g.tx) * CF_T;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(X + (int64_t)n * g.H * g.W * g.ldx), (short)0, fbytes, CF_RSRC);
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
            const int y = y0 + RPW * wid + i, x = x0 + fr;
            const int off = (y < g.H && x < g.W) ? ((y * g.W + x) * g.ldx + 8 * fq) * 2 : CF_OOB;
#pragma unroll
            for (int s = 0; s < 2; ++s) pc[i][s] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 64 * s, 0);
        }
#pragma unroll
        for (int i = 0; i < NRG; ++i) {
            if (wid + NW * i >= C::NRING) break;
            int ry, rx;
            cf_ring<R1H>(16 * (wid + NW * i) + fr, ry, rx);
            const int y = y0 - 2 + ry, x = x0 - 2 + rx;
            const bool ok = (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W;
            const int off = ok ? ((y * g.W + x) * g.ldx + 8 * fq) * 2 : CF_OOB;
#pragma unroll
            for (int s = 0; s < 2; ++s) pr[i][s] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 64 * s, 0);
        }
    };
    load_tile(t);
    __syncthreads();

    // stage boundary clocks of the first CF_TR_TILES tiles (debug only; one vector store per point)
    auto mark = [&](int k, int pt) {
        if (g.trace && k <= CF_TR_TILES && (tid & 63) == 0)
            g.trace[((blockIdx.x * NW + wid) * CF_TR_TILES + k - 1) * CF_TR_PTS + pt] = __builtin_amdgcn_s_memtime();
    };
    for (int k = 1; t >= 0; ++k) {
        mark(k, 0);
        // at 16 waves (128 VGPRs) and with the 1x1 weights in registers the lane id is re-read each tile
        // (opaque to the compiler): otherwise it
        // hoists every per-lane LDS address of the body out of the loop and spills them to scratch, whose
        // reloads then wait on the in-flight prefetch (vmcnt is in order)
        const int lane = (NW == 16 || C::WREG) ? fz::lane_id() : tid & 63, fr = lane & 15, fq = lane >> 4;
        auto frag = [&](int base, int f) { return *(const bf16x8*)(cf_smem + base + f * 1024 + 16 * lane); };
        auto bvec = [&](const float* b) {  // bias rows of a C fragment: the accumulators start from the bias
            const float4 v = *(const float4*)b;
            return (f32x4){v.x, v.y, v.z, v.w};
        };
        const int n = t / g.tpf, rr = t % g.tpf, y0 = (rr / g.tx) * C::TH, x0 = (rr % g.tx) * CF_T;
        // tile and halo inside the image: no zero masking
        const bool interior = y0 >= 2 && x0 >= 2 && y0 + R1H - 2 <= g.H && x0 + CF_R1W - 2 <= g.W;

        // ---- stage 1: cv1
        bf16x8 ra[RPW], rb[RPW];  // centre rows: a and b halves (P32 channel order)
        {
            f32x4 acc1[RPW][4], accr[NRG][2];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const f32x4 bq = bvec(b1 + 16 * q + 4 * fq);
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    bf16x8 w;
                    if constexpr (C::WREG) w = f1r[2 * q + s];
                    else w = frag(C::W1, 2 * q + s);
#pragma unroll
                    for (int i = 0; i < RPW; ++i) acc1[i][q] = mma(w, (bf16x8)pc[i][s], s ? acc1[i][q] : bq);
                    if (q >= 2) {
#pragma unroll
                        for (int i = 0; i < NRG; ++i)
                            if (wid + NW * i < C::NRING)
                                accr[i][q - 2] = mma(w, (bf16x8)pr[i][s], s ? accr[i][q - 2] : bq);
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < RPW; ++i) {
                const int y = RPW * wid + i;
                ra[i] = fz::pack(fz::act(acc1[i][0]), fz::act(acc1[i][1]));
                rb[i] = fz::pack(fz::act(acc1[i][2]), fz::act(acc1[i][3]));
                if (!interior) {
                    const bool out = y0 + y >= g.H || x0 + fr >= g.W;
                    ra[i] = fz::zero_if(ra[i], out);
                    rb[i] = fz::zero_if(rb[i], out);
                }
                *(bf16x8*)(cf_smem + C::S1 + cf_addr((y + 2) * CF_R1W + fr + 2, fq)) = rb[i];
            }
#pragma unroll
            for (int i = 0; i < NRG; ++i) {
                if (wid + NW * i >= C::NRING) break;
                int ry, rx;
                cf_ring<R1H>(16 * (wid + NW * i) + fr, ry, rx);
                bf16x8 v = fz::pack(fz::act(accr[i][0]), fz::act(accr[i][1]));
                if (!interior) {
                    const int y = y0 - 2 + ry, x = x0 - 2 + rx;
                    v = fz::zero_if(v, (unsigned)y >= (unsigned)g.H || (unsigned)x >= (unsigned)g.W);
                }
                *(bf16x8*)(cf_smem + C::S1 + cf_addr(ry * CF_R1W + rx, fq)) = v;
            }
        }
        mark(k, 1);
        const int tn = nx;
        if (tn >= 0) load_tile(tn);  // lands during stages 2-4
        int cl = 0;  // the tile after next: claimed here, published after stage 2 (va_fuse.h wq_claim_raw)
        if (g.wq && tid == 0) cl = fz::wq_claim_raw(g.wq);
        __syncthreads();
        mark(k, 2);

        // ---- stage 2: m.0.cv1 on the R2H x 18 region: rows as 16-pixel row segments (columns 0..15,
        // groups 0 .. R2H-1), then the 2*R2H pixels of columns 16..17.  Two copies (the wave's group
        // count, uniform) keep the tap loop branch-free; its fragment reads run one tap ahead.
        auto stage2 = [&](auto ngc) {
            constexpr int NGJ = decltype(ngc)::value;
            int py[NGJ], px[NGJ], bj[NGJ];  // bj: S1 address of the group's tap (0, 0)
            bool pv[NGJ];
#pragma unroll
            for (int j = 0; j < NGJ; ++j) {
                const int gi = wid + NW * j;
                if (gi < R2H) {
                    py[j] = gi;
                    px[j] = fr;
                    pv[j] = true;
                } else {
                    const int q = 16 * (gi - R2H) + fr;
                    pv[j] = q < 2 * R2H;
                    const int qc = pv[j] ? q : 2 * R2H - 1;
                    py[j] = qc >> 1;
                    px[j] = CF_T + (qc & 1);
                }
                bj[j] = C::S1 + cf_addr(py[j] * CF_R1W + px[j], fq);
            }
            f32x4 acc[NGJ][2];
            const f32x4 c0 = bvec(b2 + 4 * fq), c1 = bvec(b2 + 16 + 4 * fq);
#pragma unroll
            for (int j = 0; j < NGJ; ++j) {
                acc[j][0] = c0;
                acc[j][1] = c1;
            }
            bf16x8 wa[2][2], bv[2][NGJ];
            auto fetch = [&](int tap, int sl) {
                const int off = ((tap / 3) * CF_R1W + tap % 3) * CF_PS;
                wa[sl][0] = frag(C::W2, 2 * tap);
                wa[sl][1] = frag(C::W2, 2 * tap + 1);
#pragma unroll
                for (int j = 0; j < NGJ; ++j) bv[sl][j] = *(const bf16x8*)(cf_smem + bj[j] + off);
            };
            fetch(0, 0);
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                if (tap < 8) fetch(tap + 1, (tap + 1) & 1);
#pragma unroll
                for (int j = 0; j < NGJ; ++j) {
                    acc[j][0] = mma(wa[tap & 1][0], bv[tap & 1][j], acc[j][0]);
                    acc[j][1] = mma(wa[tap & 1][1], bv[tap & 1][j], acc[j][1]);
                }
            }
#pragma unroll
            for (int j = 0; j < NGJ; ++j) {
                bf16x8 v = fz::pack(fz::act(acc[j][0]), fz::act(acc[j][1]));
                if (!interior) {
                    const int y = y0 - 1 + py[j], x = x0 - 1 + px[j];
                    v = fz::zero_if(v, (unsigned)y >= (unsigned)g.H || (unsigned)x >= (unsigned)g.W);
                }
                const int ad = pv[j] ? C::S2 + cf_addr(py[j] * CF_R2W + px[j], fq) : C::SINK + 16 * lane;
                *(bf16x8*)(cf_smem + ad) = v;
            }
        };
        if (wid + NW * (NG2 - 1) < C::NG2T)
            stage2(std::integral_constant<int, NG2>{});
        else
            stage2(std::integral_constant<int, NG2 - 1>{});
        mark(k, 3);
        if (g.wq && tid == 0) slot[(k + 1) & 1] = cl < g.ntiles ? cl : -1;
        __syncthreads();
        mark(k, 4);
        nx = g.wq ? __builtin_amdgcn_readfirstlane(slot[(k + 1) & 1]) : fz::tile(g.ntiles, k + 1);

        // ---- stage 3: m.0.cv2 (+ b) on the wave's centre rows; stage 4: cv2 -> HBM
        {
            const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(Y + (int64_t)n * g.H * g.W * g.ldy), (short)0, g.H * g.W * g.ldy * 2, CF_RSRC);
            f32x4 acc[RPW][2];
            const int bi = C::S2 + cf_addr(RPW * wid * CF_R2W + fr, fq);  // row RPW * wid, tap (0, 0)
            const f32x4 c0 = bvec(b3 + 4 * fq), c1 = bvec(b3 + 16 + 4 * fq);
#pragma unroll
            for (int i = 0; i < RPW; ++i) {
                acc[i][0] = c0;
                acc[i][1] = c1;
            }
            bf16x8 wa[2][2], bv[2][RPW];  // fragment reads one tap ahead
            auto fetch = [&](int tap, int sl) {
                wa[sl][0] = frag(C::W3, 2 * tap);
                wa[sl][1] = frag(C::W3, 2 * tap + 1);
#pragma unroll
                for (int i = 0; i < RPW; ++i)
                    bv[sl][i] = *(const bf16x8*)(cf_smem + bi + ((i + tap / 3) * CF_R2W + tap % 3) * CF_PS);
            };
            fetch(0, 0);
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                if (tap < 8) fetch(tap + 1, (tap + 1) & 1);
#pragma unroll
                for (int i = 0; i < RPW; ++i) {
                    acc[i][0] = mma(wa[tap & 1][0], bv[tap & 1][i], acc[i][0]);
                    acc[i][1] = mma(wa[tap & 1][1], bv[tap & 1][i], acc[i][1]);
                }
            }
            bf16x8 rbp[RPW];
#pragma unroll
            for (int i = 0; i < RPW; ++i) {
                f32x4 v[2];
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    v[q] = fz::act(acc[i][q]);
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[q][r] += (float)rb[i][4 * q + r];
                }
                rbp[i] = fz::pack(v[0], v[1]);
            }
            f32x4 o4[RPW][4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const f32x4 bq = bvec(b4 + 32 * (q >> 1) + 8 * fq + 4 * (q & 1));
#pragma unroll
                for (int s = 0; s < 3; ++s) {
                    bf16x8 w;
                    if constexpr (C::WREG) w = f4r[3 * q + s];
                    else w = frag(C::W4, 3 * q + s);
#pragma unroll
                    for (int i = 0; i < RPW; ++i)
                        o4[i][q] = mma(w, s == 0 ? ra[i] : s == 1 ? rb[i] : rbp[i], s ? o4[i][q] : bq);
                }
            }
#pragma unroll
            for (int i = 0; i < RPW; ++i) {
                const int y = y0 + RPW * wid + i, x = x0 + fr;
                const int off = (y < g.H && x < g.W) ? ((y * g.W + x) * g.ldy + 8 * fq) * 2 : CF_OOB;
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    __builtin_amdgcn_raw_buffer_store_b128(
                        (u32x4)fz::pack(fz::act(o4[i][2 * h]), fz::act(o4[i][2 * h + 1])), ry, off, 64 * h, 0);
            }
        }
        mark(k, 5);
        t = tn;
    }
    if (g.wq && tid == 0) fz::wq_release(g.wq);  // after this workgroup's last (failed) claim
}

// the configuration: 8 x 16 tiles, 4 waves, two workgroups per CU (their phases drift apart, so one's SiLU
// epilogues overlap the other's MFMAs), 1x1 weights in registers -- measured best in round 1 against 16 x 16
// tiles with all weights in LDS and 8 or 16 waves per workgroup (one workgroup per CU), which were removed
using CfC = CfCfg<8, 4, 2, true>;

int g_cus = 0;
unsigned long long* g_trace = nullptr;

template <class C>
hipError_t cf_launch(const va_conv_args* a, CfGeom g, int cus, hipStream_t st) {
    static DevFlag attr;
    if (!attr()) {
        if (hipFuncSetAttribute((const void*)c2f_kernel<C>, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS + 16) !=
            hipSuccess)
            return hipErrorInvalidValue;
        attr() = true;
    }
    g.tx = (a->W + CF_T - 1) / CF_T;
    g.tpf = g.tx * ((a->H + C::TH - 1) / C::TH);
    const int64_t nt = (int64_t)g.tpf * a->N;
    if (nt > INT32_MAX) return hipErrorInvalidValue;
    g.ntiles = (int)nt;
    int grid = C::WPC * (cus > 0 ? cus : 256);
    if (grid > g.ntiles) grid = g.ntiles;
    if (g.ntiles < fz::WQ_MIN_TILES_PER_WG * grid) g.wq = nullptr;  // one or two tiles per workgroup: static
    hipLaunchKernelGGL(c2f_kernel<C>, dim3(grid), dim3(C::NW * 64), C::LDS + 16, st, (const __bf16*)a->x,
                       (const __bf16*)a->w, a->bias, (__bf16*)a->y, g);
    return hipGetLastError();
}

}  // namespace

extern "C" int va_seg_c2f(void* stream, const va_conv_args* a) {
    if (!a || !a->x || !a->w || !a->bias || !a->y || a->dtype != VA_DTYPE_BF16 || a->Cin != 64 || a->Cout != 64 ||
        a->N <= 0 || a->H <= 0 || a->W <= 0 || a->ldx < 64 || a->ldy < 64 || a->ldx % 8 || a->ldy % 8 ||
        ((uintptr_t)a->x & 15) || ((uintptr_t)a->y & 15) || ((uintptr_t)a->w & 15) || ((uintptr_t)a->bias & 15))
        return VA_ERR_ARG;
    // per-frame buffer descriptors: a frame's bytes (and the OOB sentinel above them) must fit 31 bits
    if ((int64_t)a->H * a->W * (a->ldx > a->ldy ? a->ldx : a->ldy) * 2 >= 0x80000000LL) return VA_ERR_ARG;
    if (g_cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return VA_ERR_HIP;
    }
    CfGeom g;
    g.trace = g_trace;
    g.N = a->N;
    g.H = a->H;
    g.W = a->W;
    g.ldx = a->ldx;
    g.ldy = a->ldy;
    g.wq = a->wcnt && a->ncnt >= 2 && va_sw().conv3q != 2 ? a->wcnt : nullptr;
    hipStream_t st = (hipStream_t)stream;
    const hipError_t rc = cf_launch<CfC>(a, g, g_cus, st);
    return rc == hipSuccess ? VA_OK : VA_ERR_HIP;
}

// Debug: stage clocks of the next launches into buf (device memory of grid * 8 * 32 * 6 uint64; the
// launch's grid is the CU count, capped by the tile count), or stop with NULL.
extern "C" int va_c2f_trace(void* buf) {
    g_trace = (unsigned long long*)buf;
    return VA_OK;
}
