// rmwbench.hip — in-place read-modify-write streaming floor vs N and cache policy.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/rmwbench tools/rmwbench.hip && tools/rmwbench
//
// Each thread reads K float4 and writes them back in place (what a step kernel
// does to its state every launch). Policies: plain, nontemporal stores,
// nontemporal loads+stores. Reported: us per launch and GB/s of bytes moved.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>

constexpr int K = 5;
typedef float f4 __attribute__((ext_vector_type(4)));

template <int kPolicy>
__global__ __launch_bounds__(256) void rmw(f4* buf, int64_t groups) {
    for (int64_t g = blockIdx.x * 256ll + threadIdx.x; g < groups; g += (int64_t)gridDim.x * 256) {
        f4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (kPolicy == 2) v[k] = __builtin_nontemporal_load(&buf[k * groups + g]);
            else v[k] = buf[k * groups + g];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            v[k].x += 1.0f;
            if (kPolicy >= 1) __builtin_nontemporal_store(v[k], &buf[k * groups + g]);
            else buf[k * groups + g] = v[k];
        }
    }
}

// write-through (sc1) stores: drop the line from L2 as it is written
__global__ __launch_bounds__(256) void rmw_sc1(f4* buf, int64_t groups) {
    for (int64_t g = blockIdx.x * 256ll + threadIdx.x; g < groups; g += (int64_t)gridDim.x * 256) {
        f4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = buf[k * groups + g];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            v[k].x += 1.0f;
            f4* p = &buf[k * groups + g];
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v[k]) : "memory");
        }
    }
}

template <typename F>
float time_it(F launch, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 10; ++i) launch();
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) launch();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1000.0f / reps;
}

int main() {
    for (int lg = 16; lg <= 22; ++lg) {
        const int64_t groups = (int64_t)1 << lg;  // threads' worth of work
        f4* buf = nullptr;
        if (hipMalloc(&buf, K * groups * sizeof(f4)) != hipSuccess) return 1;
        (void)hipMemset(buf, 0, K * groups * sizeof(f4));
        const int blocks = (int)((groups + 255) / 256 < 2048 ? (groups + 255) / 256 : 2048);
        const int reps = lg < 20 ? 500 : 100;
        const double bytes = 2.0 * K * 16.0 * groups;
        float t0 = time_it([&] { rmw<0><<<blocks, 256>>>(buf, groups); }, reps);
        float t1 = time_it([&] { rmw<1><<<blocks, 256>>>(buf, groups); }, reps);
        float t2 = time_it([&] { rmw<2><<<blocks, 256>>>(buf, groups); }, reps);
        float t3 = time_it([&] { rmw_sc1<<<blocks, 256>>>(buf, groups); }, reps);
        printf("{\"MB_moved\": %.1f, \"plain_us\": %.2f, \"nt_store_us\": %.2f, \"nt_both_us\": %.2f, "
               "\"sc1_store_us\": %.2f, \"plain_GBps\": %.0f, \"nt_store_GBps\": %.0f, "
               "\"nt_both_GBps\": %.0f, \"sc1_GBps\": %.0f}\n",
               bytes / 1e6, t0, t1, t2, t3, bytes / t0 / 1e3, bytes / t1 / 1e3, bytes / t2 / 1e3,
               bytes / t3 / 1e3);
        (void)hipFree(buf);
    }
    return 0;
}
