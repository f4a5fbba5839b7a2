#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __bf16 b2 __attribute__((ext_vector_type(2)));
__global__ void k(const unsigned* w, float* out) {
    const unsigned x = w[threadIdx.x];
    const b2 p = __builtin_bit_cast(b2, x);
    const b2 lo1 = __builtin_bit_cast(b2, 0x00003f80u);
    const b2 hi1 = __builtin_bit_cast(b2, 0x3f800000u);
    out[threadIdx.x * 4 + 0] = __builtin_amdgcn_fdot2_f32_bf16(p, lo1, 0.5f, false);
    out[threadIdx.x * 4 + 1] = __builtin_amdgcn_fdot2_f32_bf16(p, hi1, 0.5f, false);
    out[threadIdx.x * 4 + 2] = __uint_as_float(x << 16) + 0.5f;
    out[threadIdx.x * 4 + 3] = __uint_as_float(x & 0xffff0000u) + 0.5f;
}
int main() {
    unsigned h[4] = {0x40003f80u, 0xbf804040u, 0x3e004120u, 0x12345678u};
    unsigned* d; float* o; float ho[16];
    hipMalloc(&d, 16); hipMalloc(&o, 64);
    hipMemcpy(d, h, 16, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(4), 0, 0, d, o);
    hipMemcpy(ho, o, 64, hipMemcpyDeviceToHost);
    for (int i = 0; i < 4; ++i) printf("%08x: dot_lo %g dot_hi %g | ref_lo %g ref_hi %g\n", h[i], ho[4*i], ho[4*i+1], ho[4*i+2], ho[4*i+3]);
    return 0;
}
