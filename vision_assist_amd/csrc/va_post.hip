// va_post.hip -- segmentation post-processing on MI355X: Detect decode, NMS, process_mask, mask choice.
//
// Restates (Ultralytics is external; vendored spec copy testing/old/segmenting_using_tflite/ops.py):
//   post_decode_kernel   Detect inference tail (DFL softmax expectation, dist2bbox, class sigmoid) and
//                        the candidate filter of non_max_suppression (ops.py:281-317): one thread per anchor
//   post_nms_kernel      class-offset greedy NMS (torchvision.ops.nms: IoU > thr suppresses, float32 IoU),
//                        max_det cap (ops.py:318-330): one 1024-thread workgroup per frame, repeated
//                        "highest remaining score (lowest anchor on ties) -> keep -> suppress" == the
//                        sorted greedy scan
//   post_mask_kernel     process_mask(upsample=True) (ops.py:707-737): coef . proto over the cropped
//                        low-res box region into LDS, bilinear x4 (align_corners=False), > 0; per
//                        instance pixel count and pixel bounding box.  One workgroup per detection.
//   post_select_kernel   FrameProcessor.py:67-97 restated (cv2 absent, parity unpinned): the instance
//                        with the most mask pixels (first wins), its pixel bbox as boundingRect, its
//                        mask sampled at the 20-px cell centres -> the nav stage's (cells, rect);
//                        optional planted masks (bench / tests) when the network yields none.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/va355.h"

namespace {

constexpr int REG_MAX = 16;
constexpr int NMC = 32;
constexpr float MAX_WH = 7680.0f;

struct Level {
    const float* p;
    int h, w, stride, a0;
};

__device__ inline Level level_of(const float* const* lv, int H, int W, int a, int* local) {
    int h0 = H / 8, w0 = W / 8, h1 = H / 16, w1 = W / 16, h2 = H / 32, w2 = W / 32;
    int n0 = h0 * w0, n1 = h1 * w1;
    Level L;
    if (a < n0) {
        L = {lv[0], h0, w0, 8, 0};
    } else if (a < n0 + n1) {
        L = {lv[1], h1, w1, 16, n0};
    } else {
        L = {lv[2], h2, w2, 32, n0 + n1};
    }
    *local = a - L.a0;
    return L;
}

__device__ inline float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

struct LevelPtrs {
    const float* p[3];
};

// One 16-lane group per anchor: the group reads the anchor's class logits as consecutive 16-byte
// chunks (one 320-byte run per anchor at nc = 80, coalesced across the group) and reduces the maximum
// with xor shuffles inside the group.  Sigmoid is monotone, so an anchor whose best logit does not
// clear the threshold -- nearly every anchor -- is done after that one coalesced read; the rare
// candidate is decoded by the group's first lane.
constexpr int DEC_GROUP = 16;

__global__ __launch_bounds__(256) void post_decode_kernel(LevelPtrs lv, int B, int H, int W, int nc, int A,
                                                          float conf, va_cand* cand, int32_t* count) {
    const int no = 4 * REG_MAX + nc + NMC;
    const int64_t gid = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / DEC_GROUP;
    const int gl = threadIdx.x % DEC_GROUP;
    if (gid >= (int64_t)B * A) return;  // whole groups leave together
    int b = (int)(gid / A), a = (int)(gid % A);
    int local;
    Level L = level_of(lv.p, H, W, a, &local);
    const float* row = L.p + ((int64_t)b * L.h * L.w + local) * no;
    const float* cl = row + 4 * REG_MAX;
    float mx = -INFINITY;
    if ((nc & 3) == 0 && (no & 3) == 0) {
        for (int c = 4 * gl; c < nc; c += 4 * DEC_GROUP) {
            const float4 v = *(const float4*)(cl + c);
            mx = fmaxf(mx, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
        }
    } else {
        for (int c = gl; c < nc; c += DEC_GROUP) mx = fmaxf(mx, cl[c]);
    }
#pragma unroll
    for (int o = DEC_GROUP / 2; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, DEC_GROUP));
    if (gl != 0 || !(sigmoidf_(mx) > conf)) return;
    // class scores: sigmoid, first maximum (cls.max(1) on sigmoid values: saturated ties -> lowest class)
    float best = -1.0f;
    int bc = 0;
    for (int c = 0; c < nc; ++c) {
        float s = sigmoidf_(cl[c]);
        if (s > best) {
            best = s;
            bc = c;
        }
    }
    if (!(best > conf)) return;
    // DFL: softmax over 16 bins, expectation
    float d[4];
    for (int side = 0; side < 4; ++side) {
        const float* v = row + side * REG_MAX;
        float m = v[0];
        for (int i = 1; i < REG_MAX; ++i) m = fmaxf(m, v[i]);
        float e[REG_MAX], s = 0.f;
        for (int i = 0; i < REG_MAX; ++i) {
            e[i] = expf(v[i] - m);
            s += e[i];
        }
        float acc = 0.f;
        for (int i = 0; i < REG_MAX; ++i) acc += (e[i] / s) * (float)i;
        d[side] = acc;
    }
    int x = local % L.w, y = local / L.w;
    float ax = (float)x + 0.5f, ay = (float)y + 0.5f;
    float x1 = ax - d[0], y1 = ay - d[1], x2 = ax + d[2], y2 = ay + d[3];
    float st = (float)L.stride;
    float cx = (x1 + x2) / 2.0f * st, cy = (y1 + y2) / 2.0f * st;
    float bw = (x2 - x1) * st, bh = (y2 - y1) * st;
    va_cand c;
    c.x1 = cx - bw / 2.0f;  // xywh2xyxy (ops.py: y[...,0] = x - w/2)
    c.y1 = cy - bh / 2.0f;
    c.x2 = cx + bw / 2.0f;
    c.y2 = cy + bh / 2.0f;
    c.score = best;
    c.cls = bc;
    c.anchor = a;
    c.pad = 0;
    int slot = atomicAdd(&count[b], 1);
    cand[(int64_t)b * A + slot] = c;
}

// ------------------------------------------------------------------------------------------- NMS
constexpr int NMS_THREADS = 1024;

constexpr int NMS_LDS_KEYS = 12288;  // keys kept in LDS up to this many candidates (96 KiB)

__global__ __launch_bounds__(NMS_THREADS) void post_nms_kernel(const va_cand* cand, const int32_t* count, int A,
                                                               float iou, int max_det, va_det* dets,
                                                               int32_t* ndet, unsigned long long* gkeys) {
    const int b = blockIdx.x, tid = threadIdx.x;
    const int n = count[b];
    const va_cand* C = cand + (int64_t)b * A;
    __shared__ __align__(16) unsigned long long lkeys[NMS_LDS_KEYS];
    __shared__ unsigned long long red[NMS_THREADS / 64];
    // (score bits << 32 | ~anchor): max = highest score, lowest anchor on ties; 0 = kept or suppressed
    unsigned long long* key = n <= NMS_LDS_KEYS ? lkeys : gkeys + (int64_t)b * A;
    for (int i = tid; i < n; i += NMS_THREADS) {
        unsigned sb = __float_as_uint(C[i].score);
        key[i] = ((unsigned long long)sb << 32) | (unsigned long long)(0xFFFFFFFFu - (unsigned)C[i].anchor);
    }
    __syncthreads();
    int kept = 0;
    while (kept < max_det) {
        unsigned long long best = 0;
        int bi = -1;
        for (int i = tid; i < n; i += NMS_THREADS) {
            if (key[i] > best) {
                best = key[i];
                bi = i;
            }
        }
        // block argmax: pack index into the low bits is impossible (64-bit key), so reduce pairs
        for (int o = 32; o > 0; o >>= 1) {
            unsigned long long ob = __shfl_xor(best, o, 64);
            int oi = __shfl_xor(bi, o, 64);
            if (ob > best) {
                best = ob;
                bi = oi;
            }
        }
        __shared__ int red_i[NMS_THREADS / 64];
        if ((tid & 63) == 0) {
            red[tid >> 6] = best;
            red_i[tid >> 6] = bi;
        }
        __syncthreads();
        best = red[0];
        bi = red_i[0];
        for (int w = 1; w < NMS_THREADS / 64; ++w)
            if (red[w] > best) {
                best = red[w];
                bi = red_i[w];
            }
        __syncthreads();
        if (best == 0) break;
        const va_cand k = C[bi];
        if (tid == 0) {
            va_det d;
            d.x1 = k.x1;
            d.y1 = k.y1;
            d.x2 = k.x2;
            d.y2 = k.y2;
            d.score = k.score;
            d.cls = k.cls;
            d.anchor = k.anchor;
            d.pad = 0;
            dets[(int64_t)b * max_det + kept] = d;
            key[bi] = 0;
        }
        // suppress IoU > thr among the remaining (class-offset boxes, torchvision float math)
        const float off = (float)k.cls * MAX_WH;
        const float kx1 = k.x1 + off, ky1 = k.y1 + off, kx2 = k.x2 + off, ky2 = k.y2 + off;
        const float karea = (kx2 - kx1) * (ky2 - ky1);
        for (int i = tid; i < n; i += NMS_THREADS) {
            if (key[i] == 0 || i == bi) continue;
            const va_cand c = C[i];
            const float o2 = (float)c.cls * MAX_WH;
            const float x1 = c.x1 + o2, y1 = c.y1 + o2, x2 = c.x2 + o2, y2 = c.y2 + o2;
            const float area = (x2 - x1) * (y2 - y1);
            const float w = fmaxf(0.f, fminf(kx2, x2) - fmaxf(kx1, x1));
            const float h = fmaxf(0.f, fminf(ky2, y2) - fmaxf(ky1, y1));
            const float inter = w * h;
            const float ovr = inter / (karea + area - inter);
            if ((double)ovr > (double)iou) key[i] = 0;
        }
        ++kept;
        __syncthreads();
    }
    if (tid == 0) ndet[b] = kept;
}

// ------------------------------------------------------------------------------------------- masks
struct MaskArgs {
    const float* proto;  // [B][mh][mw][32]
    const float* lv[3];
    int B, H, W, nc, max_det, mh, mw;
    const va_det* dets;
    const int32_t* ndet;
    va_mask_stat* stats;  // [B][max_det]
};

__device__ inline const float* coef_of(const MaskArgs& a, int b, int anchor) {
    int local;
    Level L = level_of(a.lv, a.H, a.W, anchor, &local);
    const int no = 4 * REG_MAX + a.nc + NMC;
    return L.p + ((int64_t)b * L.h * L.w + local) * no + 4 * REG_MAX + a.nc;
}

// low-res crop window of a detection: r >= x1*mw/W && r < x2*mw/W (crop_mask), clipped to the map
__device__ inline void crop_window(const va_det& d, int W, int H, int mw, int mh, int* rx0, int* rx1, int* ry0,
                                   int* ry1) {
    float fx1 = d.x1 * ((float)mw / (float)W), fx2 = d.x2 * ((float)mw / (float)W);
    float fy1 = d.y1 * ((float)mh / (float)H), fy2 = d.y2 * ((float)mh / (float)H);
    int a0 = (int)ceilf(fx1), a1 = (int)ceilf(fx2) - 1;  // integer r with fx1 <= r < fx2
    int b0 = (int)ceilf(fy1), b1 = (int)ceilf(fy2) - 1;
    *rx0 = max(a0, 0);
    *rx1 = min(a1, mw - 1);
    *ry0 = max(b0, 0);
    *ry1 = min(b1, mh - 1);
}

// bilinear tap positions of F.interpolate(align_corners=False) for output index o (scale in/out)
__device__ inline void taps(int o, float scale, int in, int* i0, int* i1, float* l0, float* l1) {
    float src = scale * ((float)o + 0.5f) - 0.5f;
    if (src < 0.f) src = 0.f;
    int x0 = (int)src;
    int p = x0 < in - 1 ? 1 : 0;
    *l1 = src - (float)x0;
    *l0 = 1.0f - *l1;
    *i0 = x0;
    *i1 = x0 + p;
}

constexpr int MASK_THREADS = 256;
constexpr int MASK_LDS_MAX = 160 * 160;

__global__ __launch_bounds__(MASK_THREADS) void post_mask_kernel(MaskArgs a) {
    const int k = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    if (k >= a.ndet[b]) return;
    const va_det d = a.dets[(int64_t)b * a.max_det + k];
    int rx0, rx1, ry0, ry1;
    crop_window(d, a.W, a.H, a.mw, a.mh, &rx0, &rx1, &ry0, &ry1);
    va_mask_stat* st = a.stats + (int64_t)b * a.max_det + k;
    __shared__ float coef[NMC];
    __shared__ int s_cnt, s_x0, s_x1, s_y0, s_y1;
    extern __shared__ __align__(16) float tile[];  // [(ry1-ry0+1)][(rx1-rx0+1)]
    if (tid < NMC) coef[tid] = coef_of(a, b, d.anchor)[tid];
    if (tid == 0) {
        s_cnt = 0;
        s_x0 = a.W;
        s_x1 = -1;
        s_y0 = a.H;
        s_y1 = -1;
    }
    __syncthreads();
    if (rx1 < rx0 || ry1 < ry0) {
        if (tid == 0) *st = va_mask_stat{0, 0, 0, -1, -1, {0, 0, 0}};
        return;
    }
    const int tw = rx1 - rx0 + 1, th = ry1 - ry0 + 1;
    const bool in_lds = tw * th <= MASK_LDS_MAX;
    for (int i = tid; in_lds && i < tw * th; i += MASK_THREADS) {
        int y = ry0 + i / tw, x = rx0 + i % tw;
        const float* p = a.proto + (((int64_t)b * a.mh + y) * a.mw + x) * NMC;
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < NMC; ++c) s += coef[c] * p[c];
        tile[i] = s;
    }
    __syncthreads();
    const float sx = (float)a.mw / (float)a.W, sy = (float)a.mh / (float)a.H;
    // full-res pixels whose taps can touch the window
    const int X0 = max(0, (int)((rx0 - 1) / sx) - 2), X1 = min(a.W - 1, (int)((rx1 + 1) / sx) + 2);
    const int Y0 = max(0, (int)((ry0 - 1) / sy) - 2), Y1 = min(a.H - 1, (int)((ry1 + 1) / sy) + 2);
    const int ow = X1 - X0 + 1, oh = Y1 - Y0 + 1;
    int cnt = 0, bx0 = a.W, bx1 = -1, by0 = a.H, by1 = -1;
    for (int i = tid; i < ow * oh; i += MASK_THREADS) {
        int X = X0 + i % ow, Y = Y0 + i / ow;
        int xa, xb, ya, yb;
        float wx0, wx1, wy0, wy1;
        taps(X, sx, a.mw, &xa, &xb, &wx0, &wx1);
        taps(Y, sy, a.mh, &ya, &yb, &wy0, &wy1);
        auto val = [&](int yy, int xx) -> float {
            if (xx < rx0 || xx > rx1 || yy < ry0 || yy > ry1) return 0.f;
            if (in_lds) return tile[(yy - ry0) * tw + (xx - rx0)];
            const float* p = a.proto + (((int64_t)b * a.mh + yy) * a.mw + xx) * NMC;
            float s = 0.f;
            for (int c = 0; c < NMC; ++c) s += coef[c] * p[c];
            return s;
        };
        float v = wy0 * (wx0 * val(ya, xa) + wx1 * val(ya, xb)) + wy1 * (wx0 * val(yb, xa) + wx1 * val(yb, xb));
        if (v > 0.f) {
            ++cnt;
            bx0 = min(bx0, X);
            bx1 = max(bx1, X);
            by0 = min(by0, Y);
            by1 = max(by1, Y);
        }
    }
    atomicAdd(&s_cnt, cnt);
    if (bx1 >= 0) {
        atomicMin(&s_x0, bx0);
        atomicMax(&s_x1, bx1);
        atomicMin(&s_y0, by0);
        atomicMax(&s_y1, by1);
    }
    __syncthreads();
    if (tid == 0) *st = va_mask_stat{s_cnt, s_x0, s_y0, s_x1, s_y1, {0, 0, 0}};
}

__device__ float mask_value_at(const MaskArgs& a, int b, const va_det& d, const float* coef, int X, int Y) {
    int rx0, rx1, ry0, ry1;
    crop_window(d, a.W, a.H, a.mw, a.mh, &rx0, &rx1, &ry0, &ry1);
    const float sx = (float)a.mw / (float)a.W, sy = (float)a.mh / (float)a.H;
    int xa, xb, ya, yb;
    float wx0, wx1, wy0, wy1;
    taps(X, sx, a.mw, &xa, &xb, &wx0, &wx1);
    taps(Y, sy, a.mh, &ya, &yb, &wy0, &wy1);
    auto val = [&](int yy, int xx) -> float {
        if (xx < rx0 || xx > rx1 || yy < ry0 || yy > ry1) return 0.f;
        const float* p = a.proto + (((int64_t)b * a.mh + yy) * a.mw + xx) * NMC;
        float s = 0.f;
        for (int c = 0; c < NMC; ++c) s += coef[c] * p[c];
        return s;
    };
    return wy0 * (wx0 * val(ya, xa) + wx1 * val(ya, xb)) + wy1 * (wx0 * val(yb, xa) + wx1 * val(yb, xb));
}

__global__ void post_select_kernel(MaskArgs a, const uint8_t* plant_cells, const int32_t* plant_rects,
                                   int plant_mode, uint8_t* cells, int32_t* rects, int32_t* chosen) {
    const int b = blockIdx.x, tid = threadIdx.x;
    const int LR = a.H / VA_GRID, LC = a.W / VA_GRID;
    __shared__ int s_k;
    __shared__ float coef[NMC];
    if (tid == 0) {
        int best = -1;
        long long bc = 0;
        int n = a.ndet[b];
        for (int k = 0; k < n; ++k) {
            int c = a.stats[(int64_t)b * a.max_det + k].count;
            if (c > bc) {  // strict: the first maximum wins
                bc = c;
                best = k;
            }
        }
        if (plant_mode == 2 || (best < 0 && plant_mode == 1)) best = -2;  // planted
        s_k = best;
        chosen[b] = best;
    }
    __syncthreads();
    const int k = s_k;
    uint8_t* out = cells + (int64_t)b * LR * LC;
    if (k == -2) {
        for (int i = tid; i < LR * LC; i += blockDim.x) out[i] = plant_cells[(int64_t)b * LR * LC + i];
        if (tid < 4) rects[4 * b + tid] = plant_rects[4 * b + tid];
        return;
    }
    if (k < 0) {
        for (int i = tid; i < LR * LC; i += blockDim.x) out[i] = 0;
        if (tid < 4) rects[4 * b + tid] = 0;  // no mask: w = h = 0
        return;
    }
    const va_det d = a.dets[(int64_t)b * a.max_det + k];
    if (tid < NMC) coef[tid] = coef_of(a, b, d.anchor)[tid];
    __syncthreads();
    for (int i = tid; i < LR * LC; i += blockDim.x) {
        int r = i / LC, c = i % LC;
        out[i] = mask_value_at(a, b, d, coef, VA_GRID * c + VA_GRID / 2, VA_GRID * r + VA_GRID / 2) > 0.f;
    }
    if (tid == 0) {
        const va_mask_stat s = a.stats[(int64_t)b * a.max_det + k];
        rects[4 * b + 0] = s.x0;
        rects[4 * b + 1] = s.y0;
        rects[4 * b + 2] = s.x1 - s.x0 + 1;
        rects[4 * b + 3] = s.y1 - s.y0 + 1;
    }
}

int grid1(int64_t n, int t) { return (int)((n + t - 1) / t); }

}  // namespace

extern "C" {

int va_post_anchors(int32_t H, int32_t W) {
    if (H % 32 || W % 32 || H <= 0 || W <= 0) return VA_ERR_ARG;
    return (H / 8) * (W / 8) + (H / 16) * (W / 16) + (H / 32) * (W / 32);
}

int va_post_run(void* stream, const va_post_args* p) {
    if (!p || p->B <= 0 || p->max_det <= 0 || p->max_det > 65535) return VA_ERR_ARG;
    const int A = va_post_anchors(p->H, p->W);
    if (A <= 0 || p->nc <= 0 || !p->levels[0] || !p->levels[1] || !p->levels[2] || !p->proto || !p->cand ||
        !p->cand_count || !p->keys || !p->dets || !p->ndet || !p->stats)
        return VA_ERR_ARG;
    if (p->cells && (!p->rects || !p->chosen || (p->plant_mode && (!p->plant_cells || !p->plant_rects))))
        return VA_ERR_ARG;
    hipStream_t st = (hipStream_t)stream;
    const int B = p->B;
    if (hipMemsetAsync(p->cand_count, 0, sizeof(int32_t) * B, st) != hipSuccess) return VA_ERR_HIP;
    LevelPtrs lv{{p->levels[0], p->levels[1], p->levels[2]}};
    hipLaunchKernelGGL(post_decode_kernel, dim3(grid1((int64_t)B * A * DEC_GROUP, 256)), dim3(256), 0, st, lv, B, p->H,
                       p->W, p->nc, A, p->conf, p->cand, p->cand_count);
    if (hipGetLastError() != hipSuccess) return VA_ERR_HIP;
    static bool mask_attr = false;
    if (!mask_attr) {
        if (hipFuncSetAttribute((const void*)post_mask_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                MASK_LDS_MAX * 4) != hipSuccess)
            return VA_ERR_HIP;
        mask_attr = true;
    }
    hipLaunchKernelGGL(post_nms_kernel, dim3(B), dim3(NMS_THREADS), 0, st, p->cand, p->cand_count, A, p->iou,
                       p->max_det, p->dets, p->ndet, p->keys);
    if (hipGetLastError() != hipSuccess) return VA_ERR_HIP;
    MaskArgs ma;
    ma.proto = p->proto;
    ma.lv[0] = p->levels[0];
    ma.lv[1] = p->levels[1];
    ma.lv[2] = p->levels[2];
    ma.B = B;
    ma.H = p->H;
    ma.W = p->W;
    ma.nc = p->nc;
    ma.max_det = p->max_det;
    ma.mh = p->H / 4;
    ma.mw = p->W / 4;
    ma.dets = p->dets;
    ma.ndet = p->ndet;
    ma.stats = p->stats;
    const int tile = ma.mh * ma.mw < MASK_LDS_MAX ? ma.mh * ma.mw : MASK_LDS_MAX;
    hipLaunchKernelGGL(post_mask_kernel, dim3(p->max_det, B), dim3(MASK_THREADS), (size_t)tile * 4, st, ma);
    if (hipGetLastError() != hipSuccess) return VA_ERR_HIP;
    if (p->cells) {
        if (p->H % VA_GRID || p->W % VA_GRID) return VA_ERR_ARG;
        hipLaunchKernelGGL(post_select_kernel, dim3(B), dim3(256), 0, st, ma, p->plant_cells, p->plant_rects,
                           p->plant_mode, p->cells, p->rects, p->chosen);
        if (hipGetLastError() != hipSuccess) return VA_ERR_HIP;
    }
    return VA_OK;
}

}  // extern "C"
