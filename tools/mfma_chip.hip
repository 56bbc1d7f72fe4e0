// mfma_chip.hip — chip-wide v_mfma_f32_32x32x16_bf16 rate at two waves per SIMD (512-thread
// workgroups, one per CU), operands in registers: the effective MFMA clock under full load.
//   hipcc -O3 --offload-arch=gfx950 -o tools/mfma_chip tools/mfma_chip.hip && tools/mfma_chip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__global__ __launch_bounds__(512) void k(const bf16x8* in, f32x16* out, int iters) {
    const int lane = threadIdx.x & 63;
    bf16x8 a = in[lane], b = in[64 + lane];
    f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * 512 + threadIdx.x] = c0 + c1 + c2 + c3;
}

int main() {
    bf16x8* in;
    f32x16* out;
    hipMalloc(&in, 128 * sizeof(bf16x8));
    hipMemset(in, 0, 128 * sizeof(bf16x8));
    hipMalloc(&out, 256 * 512 * sizeof(f32x16));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int iters : {2000, 8000, 32000}) {
        k<<<256, 512>>>(in, out, iters);
        hipEventRecord(e0);
        k<<<256, 512>>>(in, out, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        // per SIMD: 2 waves x 4 x iters MFMAs
        const double mfma_per_simd = 2.0 * 4 * iters;
        printf("{\"iters\": %d, \"ms\": %.4f, \"ns_per_mfma_per_simd\": %.3f, \"eff_ghz_at_32cyc\": %.3f}\n", iters, ms,
               ms * 1e6 / mfma_per_simd, 32.0 * mfma_per_simd / (ms * 1e6));
    }
    return 0;
}
