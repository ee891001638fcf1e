// va_post.hip -- segmentation post-processing on MI355X: Detect decode, NMS, process_mask, mask choice.
//
// Restates (Ultralytics is external; vendored spec copy testing/old/segmenting_using_tflite/ops.py):
//   post_decode_kernel   Detect inference tail (DFL softmax expectation, dist2bbox, class sigmoid) and
//                        the candidate filter of non_max_suppression (ops.py:281-317): one 16-lane group
//                        per anchor, one candidate-list atomic per workgroup
//   post_nms_kernel      class-offset greedy NMS (torchvision.ops.nms: IoU > thr suppresses, float32 IoU),
//                        max_det cap (ops.py:318-330): one 1024-thread workgroup per frame, candidates
//                        bitonic-sorted in LDS and scanned greedily in 64-candidate chunks (fallback for
//                        lists that do not fit: repeated "highest remaining -> keep -> suppress")
//   masks + choice       process_mask (ops.py:707-737: coef . proto over the cropped low-res box region,
//                        bilinear x4, > 0) with each instance's pixel count / bbox, and FrameProcessor.py:67-97
//                        with OpenCV's findContours / contourArea / boundingRect / fillPoly restated
//                        (va_contour.hip, checked against oracle/contours.py; cv2 parity unpinned) -> the nav
//                        stage's (cells, rect); optional planted masks (bench / tests) when the network yields
//                        no detection.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/va355.h"
#include "va_contour.h"
#include "va_dev.h"
#include "va_diag.h"

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

// One workgroup per (frame, run of DEC_APB anchors); one 16-lane group per anchor: the group reads the
// anchor's class logits as consecutive 16-byte chunks (one 320-byte run per anchor at nc = 80, coalesced
// across the group) and reduces the maximum with xor shuffles inside the group.  Sigmoid is monotone, so
// an anchor whose best logit does not clear the threshold -- nearly every anchor of a trained network --
// is done after that one coalesced read.  A candidate is decoded by the whole group (class argmax across
// the lanes, one DFL side per lane 0-3, each in the reference's sequential order) and staged in LDS; the
// workgroup then reserves its run of the frame's candidate list with ONE global atomic.  (One atomic per
// candidate serialises on the frame counters' cache lines: 13.8 ms per 256-frame batch when every anchor
// is a candidate, the synthetic n-seg weights' case.)  NMS orders candidates by (score, anchor), so the
// list order is free.
constexpr int DEC_GROUP = 16;
constexpr int DEC_THREADS = 256;
constexpr int DEC_APB = 256;  // anchors per workgroup (at most; small batches take fewer, see va_post_run)

__global__ __launch_bounds__(DEC_THREADS) void post_decode_kernel(LevelPtrs lv, int B, int H, int W, int nc, int A,
                                                                  float conf, va_cand* cand, int32_t* count, int apb) {
    const int no = 4 * REG_MAX + nc + NMC;
    const int b = blockIdx.y, a_base = blockIdx.x * apb;
    const int grp = threadIdx.x / DEC_GROUP, gl = threadIdx.x % DEC_GROUP;
    __shared__ va_cand s_c[DEC_APB];
    __shared__ int s_n, s_base;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    for (int ai = grp; ai < apb; ai += DEC_THREADS / DEC_GROUP) {
        const int a = a_base + ai;
        if (a >= A) break;  // whole group
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
        if (!(sigmoidf_(mx) > conf)) continue;  // group-uniform
        // class scores: sigmoid, first maximum (cls.max(1) on sigmoid values: saturated ties -> lowest class)
        float best = -1.0f;
        int bc = 0;
        for (int c = gl; c < nc; c += DEC_GROUP) {
            const float sc = sigmoidf_(cl[c]);
            if (sc > best) {
                best = sc;
                bc = c;
            }
        }
#pragma unroll
        for (int o = DEC_GROUP / 2; o > 0; o >>= 1) {
            const float ob = __shfl_xor(best, o, DEC_GROUP);
            const int oc = __shfl_xor(bc, o, DEC_GROUP);
            if (ob > best || (ob == best && oc < bc)) {
                best = ob;
                bc = oc;
            }
        }
        if (!(best > conf)) continue;  // group-uniform
        // DFL: softmax over 16 bins, expectation -- lane `side` of the group, bins in order
        float dside = 0.f;
        if (gl < 4) {
            const float* v = row + gl * REG_MAX;
            float m = v[0];
            for (int i = 1; i < REG_MAX; ++i) m = fmaxf(m, v[i]);
            float e[REG_MAX], sum = 0.f;
            for (int i = 0; i < REG_MAX; ++i) {
                e[i] = expf(v[i] - m);
                sum += e[i];
            }
            for (int i = 0; i < REG_MAX; ++i) dside += (e[i] / sum) * (float)i;
        }
        const float d0 = __shfl(dside, 0, DEC_GROUP), d1 = __shfl(dside, 1, DEC_GROUP),
                    d2 = __shfl(dside, 2, DEC_GROUP), d3 = __shfl(dside, 3, DEC_GROUP);
        if (gl == 0) {
            int x = local % L.w, y = local / L.w;
            float ax = (float)x + 0.5f, ay = (float)y + 0.5f;
            float x1 = ax - d0, y1 = ay - d1, x2 = ax + d2, y2 = ay + d3;
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
            s_c[atomicAdd(&s_n, 1)] = c;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) s_base = s_n ? atomicAdd(&count[b], s_n) : 0;
    __syncthreads();
    // A frame holds at most A candidates; a count past A can only come from a second decode racing this one on
    // the same buffers (count not reset in between) -- drop, never write past the frame's region (the NMS kernel
    // clamps its count the same way)
    const int lim = A - s_base < s_n ? A - s_base : s_n;
    if (threadIdx.x == 0) (void)VA_DIAG_OK(lim == s_n, 11, s_base, s_n);
    for (int i = threadIdx.x; i < lim; i += DEC_THREADS) cand[(int64_t)b * A + s_base + i] = s_c[i];
}

// ------------------------------------------------------------------------------------------- NMS
constexpr int NMS_THREADS = 1024;
constexpr int NMS_CAP = 16384;       // candidates whose keys fit LDS (128 KiB)
constexpr int NMS_BATCH = 2048;      // longer lists: sorted and scanned in batches of their largest keys
constexpr int NMS_KEPT_MAX = 1024;   // max_det of the sorted path (kept boxes in LDS)
constexpr int NMS_CH = 64;           // candidates per greedy-scan chunk (one ballot per row)
constexpr size_t NMS_LDS = (size_t)NMS_CAP * 8 + (size_t)NMS_KEPT_MAX * 20 + NMS_CH * 32;

// torchvision's suppression test for kept box k against c (class-offset boxes, float32 IoU, > thr)
__device__ inline bool iou_over(float4 k, float karea, float4 c, float area, float thr) {
    const float w = fmaxf(0.f, fminf(k.z, c.z) - fmaxf(k.x, c.x));
    const float h = fmaxf(0.f, fminf(k.w, c.w) - fmaxf(k.y, c.y));
    const float inter = w * h;
    const float ovr = inter / (karea + area - inter);
    return (double)ovr > (double)thr;
}

__device__ inline float4 offset_box(const va_cand& c) {
    const float off = (float)c.cls * MAX_WH;
    return make_float4(c.x1 + off, c.y1 + off, c.x2 + off, c.y2 + off);
}

__device__ inline va_det to_det(const va_cand& k) {
    va_det d;
    d.x1 = k.x1;
    d.y1 = k.y1;
    d.x2 = k.x2;
    d.y2 = k.y2;
    d.score = k.score;
    d.cls = k.cls;
    d.anchor = k.anchor;
    d.pad = 0;
    return d;
}

// The k-th largest (1-based) of the keys below `hi` (keys unique, at least k of them below hi): an exact
// 8-pass radix select, one byte per pass, block-wide histograms in LDS.  Every thread of the block calls it.
__device__ unsigned long long nms_select(const unsigned long long* keys, int n, unsigned long long hi, int k,
                                         unsigned* s_hist, unsigned long long* s_T, int* s_k) {
    const int tid = threadIdx.x, nt = blockDim.x;
    if (tid == 0) {
        *s_k = k;
        *s_T = 0;
    }
    for (int i = tid; i < 256; i += nt) s_hist[i] = 0;
    __syncthreads();
    unsigned long long prefix = 0, mask = 0;
    for (int shift = 56; shift >= 0; shift -= 8) {
        for (int i = tid; i < n; i += nt) {
            const unsigned long long kk = keys[i];
            if (kk < hi && (kk & mask) == prefix) atomicAdd(&s_hist[(kk >> shift) & 255], 1u);
        }
        __syncthreads();
        if (tid < 64) {  // the digit: suffix sums over the 256 bins, 4 per lane, on wave 0
            const int need = *s_k;
            const unsigned h0 = s_hist[4 * tid], h1 = s_hist[4 * tid + 1], h2 = s_hist[4 * tid + 2],
                           h3 = s_hist[4 * tid + 3];
            const unsigned own = h0 + h1 + h2 + h3;
            unsigned suf = own;  // this lane's bins and every higher lane's
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned t = __shfl_down(suf, o, 64);
                if (tid + o < 64) suf += t;
            }
            const unsigned above = suf - own;
            if (suf >= (unsigned)need && above < (unsigned)need) {  // exactly one lane
                int left = need - (int)above, dsel = 4 * tid;
                if ((int)h3 >= left) {
                    dsel += 3;
                } else if ((int)(h3 + h2) >= left) {
                    dsel += 2, left -= (int)h3;
                } else if ((int)(h3 + h2 + h1) >= left) {
                    dsel += 1, left -= (int)(h3 + h2);
                } else {
                    left -= (int)(h3 + h2 + h1);
                }
                *s_k = left;
                *s_T = prefix | ((unsigned long long)dsel << shift);
            }
        }
        __syncthreads();
        prefix = *s_T;
        mask |= 0xFFull << shift;
        for (int i = tid; i < 256; i += nt) s_hist[i] = 0;
        __syncthreads();
    }
    return prefix;
}

// One 1024-thread workgroup per frame.  Sorted path (A <= 65536, max_det <= NMS_KEPT_MAX; lists longer than
// NMS_BATCH in batches of their largest keys, so a frame sorts 2048 keys at a time, not all of them):
// keys (score bits | ~anchor | list index) bitonic-sorted descending in LDS -- the order the greedy scan
// visits candidates in (highest score, lowest anchor on ties) -- then 64-candidate chunks: each candidate
// tested against every box kept so far (16 threads per candidate), the chunk's own pairwise suppression
// as one 64-bit ballot per row, and the chunk scanned in order on one wave (take the lowest live candidate,
// drop the candidates its row suppresses: one iteration per kept box, the kept boxes written in parallel).  Same kept set and order as
// the repeated "highest remaining -> keep -> suppress" loop of the fallback path, which keeps the
// candidates that do not fit (keys in LDS up to NMS_CAP, else in global scratch).
// max_nms (ops.py:332-333, 30000): a list longer than that is first cut to its max_nms highest-scoring
// candidates (ties: lowest anchor first, the order the scan uses) -- the sorted path simply stops taking
// batches after max_nms keys, the fallback zeroes every key below the max_nms-th.
__global__ __launch_bounds__(NMS_THREADS) void post_nms_kernel(const va_cand* cand, const int32_t* count, int A,
                                                               float iou, int max_det, int max_nms, va_det* dets,
                                                               int32_t* ndet, unsigned long long* gkeys) {
    extern __shared__ __align__(16) unsigned long long nms_smem[];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int n = min(max(count[b], 0), A);  // clamped: see post_decode_kernel
    if (tid == 0) (void)VA_DIAG_OK(n == count[b], 12, count[b], A);
    const va_cand* C = cand + (int64_t)b * A;
    va_det* D = dets + (int64_t)b * max_det;
    __shared__ int s_kept;
    if (A <= 65536 && max_det <= NMS_KEPT_MAX) {
        unsigned long long* sk = nms_smem;
        float4* kb = (float4*)(sk + NMS_CAP);     // kept boxes, class-offset
        float* ka = (float*)(kb + NMS_KEPT_MAX);   // their areas
        float4* cb = (float4*)(ka + NMS_KEPT_MAX); // chunk boxes
        float* ca = (float*)(cb + NMS_CH);
        unsigned long long* cm = (unsigned long long*)(ca + NMS_CH);  // chunk row masks
        int* sup = (int*)(cm + NMS_CH);
        __shared__ unsigned s_hist[256];
        __shared__ unsigned long long s_T;
        __shared__ int s_m, s_k;
        auto key_of = [&](int i) {
            return ((unsigned long long)__float_as_uint(C[i].score) << 32) |
                   ((unsigned long long)(0xFFFFu - (unsigned)C[i].anchor) << 16) | (unsigned long long)i;
        };
        // lists longer than NMS_BATCH run in batches: the NMS_BATCH largest keys below the previous batch's
        // smallest (an exact radix select over the keys in global scratch, keys are unique), sorted and
        // scanned like a short list, until max_det boxes are kept or the list is exhausted
        const bool big = n > NMS_BATCH || n > max_nms;  // batches (or the max_nms cut) through global keys
        unsigned long long* gk = gkeys + (int64_t)b * A;
        if (big) {
            for (int i = tid; i < n; i += NMS_THREADS) gk[i] = key_of(i);
        }
        if (tid == 0) s_kept = 0;
        unsigned long long hi = ~0ull;  // exclusive bound of the remaining keys
        int taken = 0;                  // keys handed to the scan so far (max_nms cap)
        __syncthreads();
        while (true) {
            int nb = n;  // this batch's candidates
            if (big) {
                const int want = min(NMS_BATCH, max_nms - taken);
                if (tid == 0) s_m = 0;
                __syncthreads();
                for (int i0 = 0; i0 < n; i0 += NMS_THREADS) {  // one LDS atomic per wave
                    const int i = i0 + tid;
                    const unsigned long long bal = __ballot(i < n && gk[i] < hi);
                    if ((tid & 63) == 0 && bal) atomicAdd(&s_m, __popcll(bal));
                }
                __syncthreads();
                const int rem = s_m;
                __syncthreads();  // everyone has read s_m before it is reused
                // T = the want-th largest remaining key
                const unsigned long long T = rem > want ? nms_select(gk, n, hi, want, s_hist, &s_T, &s_k) : 0ull;
                if (tid == 0) s_m = 0;
                __syncthreads();
                for (int i0 = 0; i0 < n; i0 += NMS_THREADS) {  // wave-aggregated compaction (sorted below)
                    const int i = i0 + tid, lane = tid & 63;
                    const unsigned long long kk = i < n ? gk[i] : 0ull;
                    const bool in = i < n && kk >= T && kk < hi;
                    const unsigned long long bal = __ballot(in);
                    int base = 0;
                    if (lane == 0 && bal) base = atomicAdd(&s_m, __popcll(bal));
                    base = __shfl(base, 0, 64);
                    if (in) sk[base + __popcll(bal & ((1ull << lane) - 1ull))] = kk;
                }
                __syncthreads();
                nb = s_m;
                hi = T;
                taken += nb;
            }
            int P = 2;
            while (P < nb) P <<= 1;
            for (int i = tid; i < P; i += NMS_THREADS)
                if (big ? i >= nb : true) sk[i] = i < nb ? key_of(i) : 0ull;
            __syncthreads();
            for (int k = 2; k <= P; k <<= 1)
                for (int j = k >> 1; j > 0; j >>= 1) {
                    for (int t = tid; t < P / 2; t += NMS_THREADS) {
                        const int i = 2 * j * (t / j) + (t % j), l = i + j;
                        const unsigned long long x = sk[i], y = sk[l];
                        if ((i & k) == 0 ? x < y : x > y) {
                            sk[i] = y;
                            sk[l] = x;
                        }
                    }
                    __syncthreads();
                }
        for (int c0 = 0; c0 < nb; c0 += NMS_CH) {
            const int kept = s_kept;
            if (kept >= max_det) break;  // uniform
            const int m = min(NMS_CH, nb - c0);
            if (tid < NMS_CH) {
                sup[tid] = tid < m ? 0 : 1;
                if (tid < m) {
                    const float4 bx = offset_box(C[sk[c0 + tid] & 0xFFFF]);
                    cb[tid] = bx;
                    ca[tid] = (bx.z - bx.x) * (bx.w - bx.y);
                }
            }
            __syncthreads();
            {  // suppressed by a box kept in an earlier chunk
                const int t = tid % NMS_CH, part = tid / NMS_CH;
                if (t < m) {
                    const float4 c = cb[t];
                    const float a = ca[t];
                    bool sp = false;
                    for (int q = part; q < kept && !sp; q += NMS_THREADS / NMS_CH) sp = iou_over(kb[q], ka[q], c, a, iou);
                    if (sp) sup[t] = 1;
                }
            }
            {  // chunk-internal: row r = the later candidates r suppresses if kept
                const int w = tid >> 6, lane = tid & 63;
                for (int r = w; r < NMS_CH; r += NMS_THREADS / 64) {
                    const bool pr = r < m && lane < m && lane > r && iou_over(cb[r], ca[r], cb[lane], ca[lane], iou);
                    const unsigned long long bal = __ballot(pr);
                    if (lane == 0) cm[r] = bal;
                }
            }
            __syncthreads();
            if (tid < 64) {  // the in-order scan on wave 0: lowest live candidate -> keep -> drop the rows it hits
                const unsigned long long row = cm[tid];
                unsigned long long live = __ballot(tid < m && !sup[tid]), keep = 0;
                int kk = kept;
                while (live && kk < max_det) {  // wave-uniform
                    const int t = __builtin_ctzll(live);
                    keep |= 1ull << t;
                    ++kk;
                    const unsigned long long rt =
                        ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(row >> 32), t) << 32) |
                        (unsigned)__builtin_amdgcn_readlane((int)(unsigned)row, t);
                    live &= ~(rt | (1ull << t));
                }
                if ((keep >> tid) & 1ull) {
                    const int r = kept + __popcll(keep & ((1ull << tid) - 1ull));
                    kb[r] = cb[tid];
                    ka[r] = ca[tid];
                    D[r] = to_det(C[sk[c0 + tid] & 0xFFFF]);
                }
                if (tid == 0) s_kept = kk;
            }
            __syncthreads();
        }
            if (!big || s_kept >= max_det || hi == 0ull || taken >= max_nms) break;  // uniform
        }
        if (tid == 0) ndet[b] = s_kept;
        return;
    }
    __shared__ unsigned long long red[NMS_THREADS / 64];
    __shared__ int red_i[NMS_THREADS / 64];
    __shared__ unsigned f_hist[256];
    __shared__ unsigned long long f_T;
    __shared__ int f_k;
    // (score bits << 32 | ~anchor): max = highest score, lowest anchor on ties; 0 = kept or suppressed
    unsigned long long* key = n <= NMS_CAP ? nms_smem : gkeys + (int64_t)b * A;
    for (int i = tid; i < n; i += NMS_THREADS) {
        unsigned sb = __float_as_uint(C[i].score);
        key[i] = ((unsigned long long)sb << 32) | (unsigned long long)(0xFFFFFFFFu - (unsigned)C[i].anchor);
    }
    __syncthreads();
    if (n > max_nms) {  // keep the max_nms largest keys (scores > conf > 0, so no key is 0 yet)
        const unsigned long long T = nms_select(key, n, ~0ull, max_nms, f_hist, &f_T, &f_k);
        for (int i = tid; i < n; i += NMS_THREADS)
            if (key[i] < T) key[i] = 0;
        __syncthreads();
    }
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
        for (int o = 32; o > 0; o >>= 1) {
            unsigned long long ob = __shfl_xor(best, o, 64);
            int oi = __shfl_xor(bi, o, 64);
            if (ob > best) {
                best = ob;
                bi = oi;
            }
        }
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
            D[kept] = to_det(k);
            key[bi] = 0;
        }
        const float4 kbx = offset_box(k);
        const float karea = (kbx.z - kbx.x) * (kbx.w - kbx.y);
        for (int i = tid; i < n; i += NMS_THREADS) {
            if (key[i] == 0 || i == bi) continue;
            const float4 c = offset_box(C[i]);
            if (iou_over(kbx, karea, c, (c.z - c.x) * (c.w - c.y), iou)) key[i] = 0;
        }
        ++kept;
        __syncthreads();
    }
    if (tid == 0) ndet[b] = kept;
}

// LetterBox: one thread per destination pixel (3 bytes).  Resize = cv2.INTER_LINEAR on uint8 in its
// fixed-point form: per axis src = (d + 0.5) / scale - 0.5, clamped at the borders, weights rounded to
// 11 bits (w0 = round((1 - f) * 2048), w1 = 2048 - w0); the two passes combine as
// (sum of w_y * w_x * pixel + 2^21) >> 22.  (OpenCV is absent here: parity with cv2.resize is unpinned.)
__device__ inline void lin_coef(int d, float inv, int n, int* i0, int* i1, int* w0) {
    float f = ((float)d + 0.5f) * inv - 0.5f;
    int s = (int)floorf(f);
    f -= (float)s;
    if (s < 0) {
        s = 0;
        f = 0.f;
    }
    if (s >= n - 1) {
        s = n - 1;
        f = 0.f;
    }
    *i0 = s;
    *i1 = min(s + 1, n - 1);
    *w0 = (int)lrintf((1.0f - f) * 2048.0f);
}

__global__ void letterbox_kernel(const uint8_t* __restrict__ src, int H, int W, uint8_t* __restrict__ dst, int Hn,
                                 int Wn, int top, int left, int newh, int neww, int64_t total) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int x = (int)(i % Wn), y = (int)((i / Wn) % Hn), b = (int)(i / ((int64_t)Wn * Hn));
    uint8_t* o = dst + i * 3;
    const int ry = y - top, rx = x - left;
    if (ry < 0 || ry >= newh || rx < 0 || rx >= neww) {
        o[0] = o[1] = o[2] = 114;
        return;
    }
    const uint8_t* f = src + (int64_t)b * H * W * 3;
    if (newh == H && neww == W) {
        const uint8_t* p = f + ((int64_t)ry * W + rx) * 3;
        o[0] = p[0];
        o[1] = p[1];
        o[2] = p[2];
        return;
    }
    int x0, x1, wx0, y0, y1, wy0;
    lin_coef(rx, (float)W / (float)neww, W, &x0, &x1, &wx0);
    lin_coef(ry, (float)H / (float)newh, H, &y0, &y1, &wy0);
    const int wx1 = 2048 - wx0, wy1 = 2048 - wy0;
    const uint8_t* r0 = f + (int64_t)y0 * W * 3;
    const uint8_t* r1 = f + (int64_t)y1 * W * 3;
    for (int c = 0; c < 3; ++c) {
        const int h0 = r0[x0 * 3 + c] * wx0 + r0[x1 * 3 + c] * wx1;
        const int h1 = r1[x0 * 3 + c] * wx0 + r1[x1 * 3 + c] * wx1;
        const int v = (h0 * wy0 + h1 * wy1 + (1 << 21)) >> 22;
        o[c] = (uint8_t)min(max(v, 0), 255);
    }
}

int grid1(int64_t n, int t) { return (int)((n + t - 1) / t); }

// The mask choice of FrameProcessor.py:67-97 (cells != NULL) and / or Results.masks.xy (polys) for the detections
// of the post-processing buffers p: va_contour.hip.
int contours(hipStream_t st, const va_post_args* p, float* polys, int32_t* poly_n, int poly_cap, bool fill) {
    const bool lb = p->H0 > 0;
    const int H0 = lb ? p->H0 : p->H, W0 = lb ? p->W0 : p->W;
    if (!p->cscratch || p->cslots <= 0 || p->ccap <= 0 || !p->cstats || H0 % VA_GRID || W0 % VA_GRID ||
        H0 / VA_GRID > 64 || W0 / VA_GRID > 64 || p->H > 65535 || p->W > 65535 || (lb && !(p->sc_gain > 0.0f)) ||
        !p->cpts || p->cpts_cap <= 0 || p->cpts_cap > p->ccap)
        return VA_ERR_ARG;
    if (fill && (!p->cells || !p->rects || !p->chosen || (p->plant_mode && (!p->plant_cells || !p->plant_rects))))
        return VA_ERR_ARG;
    CtSrc src{};
    src.proto = p->proto;
    for (int l = 0; l < 3; ++l) src.lv[l] = p->levels[l];
    src.dets = p->dets;
    src.nc = p->nc;
    src.max_det = p->max_det;
    src.ndet = p->ndet;
    src.B = p->B;
    src.Hn = p->H;
    src.Wn = p->W;
    src.mh = p->H / 4;
    src.mw = p->W / 4;
    src.stats = p->stats;
    CtFrame f{H0, W0, lb ? p->sc_gain : 1.0f, lb ? p->sc_padx : 0.0f, lb ? p->sc_pady : 0.0f};
    CtScratch sc{(unsigned char*)p->cscratch, 0, 0, 0, p->cslots, p->ccap, p->cpts, p->cpts_cap};
    if (va_contour_scratch_bytes(p->H, p->W, p->cslots, p->ccap, &sc.slot_bytes, &sc.img_off, &sc.pts_off) != VA_OK)
        return VA_ERR_ARG;
    const hipError_t e = va_contour_launch(src, f, sc, p->cstats, p->max_det, p->plant_cells, p->plant_rects,
                                           p->plant_mode, fill ? p->cells : nullptr, p->rects, p->chosen, p->cstatus,
                                           polys, poly_n, poly_cap, st);
    return e == hipSuccess ? VA_OK : VA_ERR_HIP;
}

}  // namespace

extern "C" {

int va_letterbox(void* stream, const uint8_t* src, int32_t B, int32_t H, int32_t W, uint8_t* dst, int32_t Hn,
                 int32_t Wn, int32_t top, int32_t left, int32_t newh, int32_t neww) {
    if (!src || !dst || B <= 0 || H <= 0 || W <= 0 || Hn <= 0 || Wn <= 0 || newh <= 0 || neww <= 0 || top < 0 ||
        left < 0 || top + newh > Hn || left + neww > Wn)
        return VA_ERR_ARG;
    const int64_t total = (int64_t)B * Hn * Wn;
    hipLaunchKernelGGL(letterbox_kernel, dim3(grid1(total, 256)), dim3(256), 0, (hipStream_t)stream, src, H, W, dst,
                       Hn, Wn, top, left, newh, neww, total);
    return hipGetLastError() == hipSuccess ? VA_OK : VA_ERR_HIP;
}

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
    if (B > 65535) return VA_ERR_ARG;
    // anchors per workgroup: 256, halved (down to one per 16-lane group) while the launch has under 2048
    // workgroups -- at batch 1 a group's 16 anchors in a row were 16 dependent loads (23 us for the n-seg frame)
    int apb = DEC_APB;
    while (apb > DEC_THREADS / DEC_GROUP && (int64_t)B * grid1(A, apb) < 2048) apb /= 2;
    hipLaunchKernelGGL(post_decode_kernel, dim3(grid1(A, apb), B), dim3(DEC_THREADS), 0, st, lv, B, p->H, p->W,
                       p->nc, A, p->conf, p->cand, p->cand_count, apb);
    if (hipGetLastError() != hipSuccess) return VA_ERR_HIP;
    static DevFlag nms_attr;  // post_nms_kernel's 150 KiB of dynamic LDS (set explicitly: graph kernel nodes too)
    if (!nms_attr()) {
        if (hipFuncSetAttribute((const void*)post_nms_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)NMS_LDS) != hipSuccess)
            return VA_ERR_HIP;
        nms_attr() = true;
    }
    const int max_nms = p->max_nms > 0 ? p->max_nms : VA_MAX_NMS;
    hipLaunchKernelGGL(post_nms_kernel, dim3(B), dim3(NMS_THREADS), NMS_LDS, st, p->cand, p->cand_count, A, p->iou,
                       p->max_det, max_nms, p->dets, p->ndet, p->keys);
    if (hipGetLastError() != hipSuccess) return VA_ERR_HIP;
    // detections only (no mask choice, no per-detection contour stats asked for): the contour pass is skipped,
    // and so are its buffer checks
    if (!p->cells && !p->cstats) return VA_OK;
    return contours(st, p, nullptr, nullptr, 0, p->cells != nullptr);
}

int va_post_polygons(void* stream, const va_post_args* p, float* polys, int32_t* poly_n, int32_t poly_cap) {
    if (!p || !polys || !poly_n || poly_cap <= 0) return VA_ERR_ARG;
    return contours((hipStream_t)stream, p, polys, poly_n, poly_cap, false);
}

}  // extern "C"

int va_diag_post(unsigned int* out4, int clear) { return diag_read_tu(out4, clear); }
