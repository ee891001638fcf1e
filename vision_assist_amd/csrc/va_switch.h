// va_switch.h -- the library's A/B switches.  Every default is the measured-best form; the other
// settings are kept for same-box comparisons and for the parity tests that hold two forms against each other.
// They are read from the environment ONCE per process, at the first launch that consults them, never per launch;
// va_switches_reload() (va355.h) re-reads them, for a test that changes one inside a process.
#pragma once

struct VaSwitches {
    int f32_split;   // VA_F32_SPLIT: bf16 term products per f32 product, 6 (default) or 9; 0 = the f32 MFMA
    int conv3h;      // VA_CONV3H=0: the stride-1 multi-tap f32 layers on conv3t instead of the halo-staged kernel
    int conv3t;      // VA_CONV3T=0: the wide f32 layers on conv2's three-term form; default (2): conv3t takes the
                     // batch-1 layers conv2 would split over K too, split over K itself; "nosplit" (1): those stay on
                     // conv2's split-K
    int conv3q;      // VA_CONV3Q=0: the 32 -> 32 stride-1 3x3 f32 layers on conv2's three-term form instead of conv3q;
                     // 2 = "static": the persistent kernels (conv3q, the f32 and bf16 stems, the bf16 C2f) on
                     // fz::tile's static schedule instead of the plan's work counter (va_fuse.h fz::wq_claim)
    int splitk;      // VA_SPLITK=0: no split-K for launches of few tiles; "ticket" (2): the slices' sum and epilogue
                     // in the last-arriving workgroup of each tile instead of conv2_reduce_kernel (the default, 1)
    int splitk_ks;   // VA_SPLITK_KS=<n> (diagnostic sweeps only): the slice count of every split launch forced to n
                     // (within the workspace and two workgroups per CU); 0 = the cost model
    bool patch;      // VA_CONV_PATCH=0: the narrow bf16 3x3 layers on conv_dn instead of the patch kernel
    int conv4_min;   // VA_CONV4: 0 = conv4 off (-1 here), "all" = every eligible layer (1), default 256 tiles
    bool pw;         // VA_PW=0: the bf16 128-channel 1x1 layers on conv2 instead of pw_kernel
    bool ct_runs;    // VA_CT_RUNS=0: border following pixel by pixel (no straight-run probe)
    bool ct_wgp;     // VA_CT_WGP=0: large-batch contours on the pool form instead of the persistent workgroups
};

const VaSwitches& va_sw();
