// Back-to-back launch period of simple kernels on one stream (diagnostic):
// what a dependent-dispatch boundary costs on gfx950, with and without a data
// stream behind it. hipcc --offload-arch=gfx950 -O3 tools/launchbench.hip -o tools/launchbench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void empty_kernel(int* p) {
    if (p && threadIdx.x == 1024) p[0] = 1;  // never true: keeps the argument live
}

template <bool kNt>
__global__ void copy_kernel(const uint4* __restrict__ in, uint4* __restrict__ out, int64_t n16) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
        uint4 v = in[i];
        if (kNt) __builtin_nontemporal_store(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v),
                                             reinterpret_cast<__attribute__((ext_vector_type(4))) uint32_t*>(out + i));
        else out[i] = v;
    }
}

template <typename F>
static float period_us(F launch, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 50; ++i) launch();
    hipDeviceSynchronize();
    hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1e3f / reps;
}

int main() {
    const int reps = 2000;
    printf("{\"empty_1024x256_us\": %.3f", period_us([] { empty_kernel<<<1024, 256>>>(nullptr); }, reps));
    printf(", \"empty_1x64_us\": %.3f", period_us([] { empty_kernel<<<1, 64>>>(nullptr); }, reps));
    for (int64_t mb : {22, 44, 700}) {
        const int64_t bytes = mb << 20, n16 = bytes / 16;
        uint4 *in, *out;
        hipMalloc(&in, bytes);
        hipMalloc(&out, bytes);
        hipMemset(in, 1, bytes);
        const int grid = 2048;
        const float t0 = period_us([&] { copy_kernel<false><<<grid, 256>>>(in, out, n16); }, mb > 100 ? 100 : reps);
        const float t1 = period_us([&] { copy_kernel<true><<<grid, 256>>>(in, out, n16); }, mb > 100 ? 100 : reps);
        printf(", \"copy_%ldMB_us\": %.3f, \"copy_%ldMB_nt_us\": %.3f, \"copy_%ldMB_GBps\": %.0f, \"copy_%ldMB_nt_GBps\": %.0f",
               (long)mb, t0, (long)mb, t1, (long)mb, 2.0 * bytes / t0 / 1e3, (long)mb, 2.0 * bytes / t1 / 1e3);
        hipFree(in);
        hipFree(out);
    }
    printf("}\n");
    return 0;
}
