// va_contour.h -- shared between va_post.hip (the pipeline's post-processing) and va_contour.hip (the mask ->
// polygon -> cells boundary): where the instance masks come from, the frame mapping and the scratch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/va355.h"

struct CtSrc {  // where the instance masks come from
    // head (the pipeline): proto [B][mh][mw][32], coefficient rows of the three level tensors, kept detections
    const float* proto;
    const float* lv[3];
    const va_det* dets;
    int nc, max_det;
    // given binary masks (tests / the C-ABI): [B][maxn][Hn][Wn] uint8
    const uint8_t* masks;
    int maxn;
    const int32_t* ndet;  // detections (masks) per frame
    int B, Hn, Wn, mh, mw;
    va_mask_stat* stats;  // out [B][max_det] or NULL: pixel count / bbox of each mask (head source)
};

struct CtFrame {  // scale_coords of the network's Hn x Wn onto the H0 x W0 frame (float32, as numpy computes it)
    int H0, W0;
    float gain, padx, pady;
};

struct CtScratch {
    unsigned char* base;  // nslots slots: low-res strip | framed 2-bit image | int32 point pairs
    int64_t slot_bytes, img_off, pts_off;
    int nslots, cap;      // cap: int32 point pairs per slot (post_fill_kernel)
    uint32_t* cpts;       // [B][max_det][2][capd] packed contour points
    int capd;
};

// Launch the contour kernels for every detection (stats, cstats, optional polygons) and, with cells, the
// per-frame choice + fill (va_contour.hip).
hipError_t va_contour_launch(const CtSrc& src, const CtFrame& f, const CtScratch& sc, va_contour_stat* cstats,
                             int max_det, const uint8_t* plant_cells, const int32_t* plant_rects, int plant_mode,
                             uint8_t* cells, int32_t* rects, int32_t* chosen, int32_t* status, float* polys,
                             int32_t* poly_n, int poly_cap, hipStream_t st);
