// Issue cost of the e4m3 -> bf16 conversions on gfx950 (tools/micro/cvt_rate.py): one wave per SIMD runs N
// independent conversions per iteration; s_memtime around the loop.  hipcc --offload-arch=gfx950 -O3 -shared -fPIC
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef __attribute__((ext_vector_type(2))) __bf16 b2;
typedef __attribute__((ext_vector_type(2))) float f2;

template <int MODE>
__global__ void k(const unsigned* in, unsigned* out, int iters, unsigned long long* clk) {
    unsigned v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = in[threadIdx.x * 8 + i];
    unsigned acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            unsigned r;
            if constexpr (MODE == 0) {
                r = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)v[i], 1.0f, false));
            } else if constexpr (MODE == 1) {
                const f2 f = __builtin_amdgcn_cvt_pk_f32_fp8((int)v[i], false);
                r = __builtin_amdgcn_perm(__float_as_uint(f[1]), __float_as_uint(f[0]), 0x07060302u);
            } else {
                r = v[i] + 0x01010101u;
            }
            acc ^= r;
            v[i] = v[i] * 3u + r;  // a dependency chain per register, 8 independent chains
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

extern "C" int run(int mode, const unsigned* in, unsigned* out, int iters, unsigned long long* clk, int blocks) {
    if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, in, out, iters, clk);
    else if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64), 0, 0, in, out, iters, clk);
    else hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(64), 0, 0, in, out, iters, clk);
    return hipDeviceSynchronize();
}
