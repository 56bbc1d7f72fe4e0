// hbmcopy.hip — the achievable HBM streaming rate on this part (tuning tool, VERDICT r02
// item 3): a float4 copy of a buffer far beyond the 256 MiB Infinity Cache, in the
// shapes that decide what a streaming kernel reaches.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/hbmcopy tools/hbmcopy.hip && tools/hbmcopy
//
// Rate = (bytes read + bytes written) / kernel time (HIP events over 20 back-to-back
// launches after 3 warm-ups). Variants, one JSON line each:
//   unroll U     each thread copies U float4 per pass (U loads in flight, then U stores),
//                grid-stride over the buffer with G workgroups of 256
//   onepass      one float4 per thread, grid = bytes / 16 / 256 (no loop)
//   store flavour plain / nt (__builtin_nontemporal_store); loads plain / nt
// The MI355X guide quotes 6.29 TB/s for a float4 copy (MI355X_MICROARCH.md chip table).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool kNtLoad, bool kNtStore>
__global__ __launch_bounds__(256) void copy_loop(const u32x4* __restrict__ in, u32x4* __restrict__ out, int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += stride * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + (int64_t)u * 256;
            if (i < n4) v[u] = kNtLoad ? __builtin_nontemporal_load(in + i) : in[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + (int64_t)u * 256;
            if (i < n4) {
                if (kNtStore) __builtin_nontemporal_store(v[u], out + i);
                else out[i] = v[u];
            }
        }
    }
}

template <bool kNtLoad, bool kNtStore>
__global__ __launch_bounds__(256) void copy_onepass(const u32x4* __restrict__ in, u32x4* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const u32x4 v = kNtLoad ? __builtin_nontemporal_load(in + i) : in[i];
    if (kNtStore) __builtin_nontemporal_store(v, out + i);
    else out[i] = v;
}

template <typename F>
static float time_us(F launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) launch();
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < 20; ++i) launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.0f / 20;
}

template <int U, bool L, bool S>
static void run_loop(const u32x4* in, u32x4* out, int64_t n4, int grid, double bytes) {
    const float us = time_us([&] { copy_loop<U, L, S><<<grid, 256>>>(in, out, n4); });
    printf("{\"variant\": \"loop\", \"unroll\": %d, \"grid\": %d, \"nt_load\": %d, \"nt_store\": %d, "
           "\"us\": %.2f, \"TBps\": %.3f}\n", U, grid, (int)L, (int)S, us, bytes / (us * 1e-6) / 1e12);
}

int main() {
    const size_t bytes = (size_t)1 << 31;  // 2 GiB in, 2 GiB out
    const int64_t n4 = (int64_t)(bytes / 16);
    u32x4 *in, *out;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&out, bytes));
    CK(hipMemset(in, 1, bytes));
    CK(hipMemset(out, 0, bytes));
    const double moved = 2.0 * (double)bytes;
    {
        const int grid = (int)(n4 / 256);
        float us = time_us([&] { copy_onepass<false, false><<<grid, 256>>>(in, out); });
        printf("{\"variant\": \"onepass\", \"nt_load\": 0, \"nt_store\": 0, \"us\": %.2f, \"TBps\": %.3f}\n", us,
               moved / (us * 1e-6) / 1e12);
        us = time_us([&] { copy_onepass<false, true><<<grid, 256>>>(in, out); });
        printf("{\"variant\": \"onepass\", \"nt_load\": 0, \"nt_store\": 1, \"us\": %.2f, \"TBps\": %.3f}\n", us,
               moved / (us * 1e-6) / 1e12);
        us = time_us([&] { copy_onepass<true, true><<<grid, 256>>>(in, out); });
        printf("{\"variant\": \"onepass\", \"nt_load\": 1, \"nt_store\": 1, \"us\": %.2f, \"TBps\": %.3f}\n", us,
               moved / (us * 1e-6) / 1e12);
    }
    for (int grid : {1024, 2048, 4096, 8192, 16384}) {
        run_loop<1, false, false>(in, out, n4, grid, moved);
        run_loop<2, false, false>(in, out, n4, grid, moved);
        run_loop<4, false, false>(in, out, n4, grid, moved);
        run_loop<8, false, false>(in, out, n4, grid, moved);
        run_loop<4, false, true>(in, out, n4, grid, moved);
        run_loop<8, false, true>(in, out, n4, grid, moved);
    }
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
}
