// va_dev.h -- per-device one-time state of the launchers.  One process may drive several GPUs (e.g. two
// FramePipelines on different devices), so a "done once" flag such as the dynamic-LDS attribute of a kernel
// or the upload of a __constant__ table is kept per HIP device, never process-global.
#pragma once
#include <hip/hip_runtime.h>

constexpr int VA_MAX_DEV = 64;

inline int va_cur_dev() {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0) d = 0;
    return d < VA_MAX_DEV ? d : VA_MAX_DEV - 1;
}

// flag() -> this device's flag (zero-initialised static storage)
struct DevFlag {
    bool on[VA_MAX_DEV];
    bool& operator()() { return on[va_cur_dev()]; }
};

// per-device value (e.g. the largest dynamic LDS size set so far)
template <typename T>
struct DevVal {
    T v[VA_MAX_DEV];
    T& operator()() { return v[va_cur_dev()]; }
};
