// va_handle.hip -- the device-bound handle of the C ABI (va_create / va_destroy and a fused
// per-batch entry point, va_frame).  The kernels' entry points are stateless (caller-owned buffers, the stream as
// an argument); the handle binds a caller to one HIP device -- the library is built for gfx950 only, so
// va_create refuses any other -- and va_frame runs one batch through the whole hot path (forward -> decode / NMS /
// contours / mask choice -> grid / penalty / protrusion / A*) on that device in one call, with the device made
// current for the call and restored after it (a process may drive several GPUs).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>

#include "../../include/va355.h"
#include "va_diag.h"
#include "va_switch.h"

struct va_handle_s {
    int32_t device;
    uint32_t flags;
};

namespace {
// the handle's device current for the call, the caller's restored after it
struct DeviceScope {
    int prev = -1;
    bool ok = false;
    explicit DeviceScope(int d) {
        ok = hipGetDevice(&prev) == hipSuccess && hipSetDevice(d) == hipSuccess;
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};
VaSwitches g_sw;
std::once_flag g_sw_once;

bool env_off(const char* name) {
    const char* e = getenv(name);
    return e && e[0] == '0';
}

void read_switches(VaSwitches& s) {
    const char* e = getenv("VA_F32_SPLIT");
    s.f32_split = !e ? 6 : e[0] == '9' ? 9 : e[0] == '6' ? 6 : 0;
    e = getenv("VA_CONV3H");
    s.conv3h = !e ? 1 : e[0] == '0' ? 0 : 1;
    e = getenv("VA_CONV3T");
    s.conv3t = !e ? 2 : e[0] == '0' ? 0 : strcmp(e, "nosplit") == 0 ? 1 : 2;
    e = getenv("VA_CONV3Q");
    s.conv3q = !e ? 1 : e[0] == '0' ? 0 : strcmp(e, "static") == 0 ? 2 : 1;
    e = getenv("VA_SPLITK");
    s.splitk = !e ? 1 : e[0] == '0' ? 0 : strcmp(e, "ticket") == 0 ? 2 : 1;
    e = getenv("VA_SPLITK_KS");
    s.splitk_ks = e ? atoi(e) : 0;
    s.patch = !env_off("VA_CONV_PATCH");
    e = getenv("VA_CONV4");
    s.conv4_min = !e ? 256 : e[0] == '0' ? -1 : strcmp(e, "all") == 0 ? 1 : 256;
    s.pw = !env_off("VA_PW");
    s.ct_runs = !env_off("VA_CT_RUNS");
    s.ct_wgp = !env_off("VA_CT_WGP");
}
}  // namespace

const VaSwitches& va_sw() {
    std::call_once(g_sw_once, [] { read_switches(g_sw); });
    return g_sw;
}

extern "C" {

int va_switches_reload(void) {
    va_sw();
    read_switches(g_sw);
    return VA_OK;
}

int va_create(int32_t device, uint32_t flags, va_handle* out) {
    if (!out || flags != 0) return VA_ERR_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return VA_ERR_HIP;
    if (device < 0 || device >= n) return VA_ERR_ARG;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess) return VA_ERR_HIP;
    if (strncmp(p.gcnArchName, "gfx950", 6) != 0) return VA_ERR_ARG;  // the code objects are gfx950 only
    *out = new va_handle_s{device, flags};
    return VA_OK;
}

int va_destroy(va_handle h) {
    delete h;
    return VA_OK;
}

int va_handle_device(va_handle h, int32_t* device) {
    if (!h || !device) return VA_ERR_ARG;
    *device = h->device;
    return VA_OK;
}

int va_frame(va_handle h, void* stream, const va_seg_op* ops, int32_t nops, const va_post_args* post, int32_t H0,
             int32_t W0, uint64_t* seen, void* nav_work, int32_t* rounds) {
    return va_frame_rb(h, stream, ops, nops, post, H0, W0, seen, nav_work, rounds, nullptr, 0);
}

int va_frame_rb(va_handle h, void* stream, const va_seg_op* ops, int32_t nops, const va_post_args* post, int32_t H0,
                int32_t W0, uint64_t* seen, void* nav_work, int32_t* rounds, void* host_records,
                int64_t host_bytes) {
    if (!h || !ops || nops <= 0 || !post || !post->cells || !post->rects || !seen || !nav_work) return VA_ERR_ARG;
    if (host_records && host_bytes < va_nav_records_bytes(post->B, H0, W0)) return VA_ERR_ARG;
    DeviceScope scope(h->device);
    if (!scope.ok) return VA_ERR_HIP;
    int rc = va_seg_run(stream, ops, nops);
    if (rc != VA_OK) return rc;
    rc = va_post_run(stream, post);
    if (rc != VA_OK) return rc;
    return va_nav_run_rb(stream, post->cells, post->rects, post->B, H0, W0, seen, nav_work, rounds, host_records,
                         host_bytes);
}

int va_diag(uint32_t* out, int32_t n, int32_t clear) {
    if (!out || n < 12) return VA_ERR_ARG;
    int (*const tu[3])(unsigned int*, int) = {va_diag_post, va_diag_contour, va_diag_nav};
    for (int i = 0; i < 3; ++i)
        if (tu[i](out + 4 * i, clear) != 0) return VA_ERR_HIP;
    return VA_OK;
}

}  // extern "C"
