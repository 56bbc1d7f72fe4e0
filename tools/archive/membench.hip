// membench.hip — streaming floors for candidate step-kernel layouts (tuning tool).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/membench tools/membench.hip && tools/membench
//
// Moves the same algorithmic bytes per env as the step kernel (20 B read,
// 22 B written) with trivial arithmetic, in three layouts:
//   A  current: x,y,origin,dest u8 + cargo i32 + fuel f64 + action i32 in;
//      x,y,origin,dest,cargo,fuel,reward,done,err out (4 envs per thread)
//   B  hybrid: ship word u32 {x,y,origin,dest} + cargo + fuel + action in;
//      ship, cargo, fuel, reward, done, err out (4 envs per thread)
//   C  float4 copy of 20 B in / 22 B out per env equivalent (floor)
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            printf("%s: %s\n", #x, hipGetErrorString(e));                       \
            return 1;                                                           \
        }                                                                       \
    } while (0)

struct BufA {
    uint8_t *x, *y, *o, *d, *done, *err;
    int32_t *cargo, *act;
    double* fuel;
    float* reward;
};

__global__ __launch_bounds__(256) void kA(BufA b, int64_t groups) {
    for (int64_t g = blockIdx.x * 256ll + threadIdx.x; g < groups; g += (int64_t)gridDim.x * 256) {
        uint32_t x = ((uint32_t*)b.x)[g], y = ((uint32_t*)b.y)[g], o = ((uint32_t*)b.o)[g],
                 d = ((uint32_t*)b.d)[g];
        int4 c = ((int4*)b.cargo)[g], a = ((int4*)b.act)[g];
        double2 f0 = ((double2*)b.fuel)[2 * g], f1 = ((double2*)b.fuel)[2 * g + 1];
        x ^= (uint32_t)a.x;
        y ^= (uint32_t)a.y;
        c.x += a.z;
        f0.x -= 1.0;
        f1.y -= 1.0;
        ((uint32_t*)b.x)[g] = x;
        ((uint32_t*)b.y)[g] = y;
        ((uint32_t*)b.o)[g] = o + 1;
        ((uint32_t*)b.d)[g] = d + 1;
        ((int4*)b.cargo)[g] = c;
        ((double2*)b.fuel)[2 * g] = f0;
        ((double2*)b.fuel)[2 * g + 1] = f1;
        ((float4*)b.reward)[g] = make_float4((float)a.x, (float)a.y, (float)a.z, (float)a.w);
        ((uint32_t*)b.done)[g] = x & 0x01010101u;
        ((uint32_t*)b.err)[g] = y & 0x03030303u;
    }
}

struct BufB {
    uint32_t* ship;
    uint8_t *done, *err;
    int32_t *cargo, *act;
    double* fuel;
    float* reward;
};

__global__ __launch_bounds__(256) void kB(BufB b, int64_t groups) {
    for (int64_t g = blockIdx.x * 256ll + threadIdx.x; g < groups; g += (int64_t)gridDim.x * 256) {
        uint4 s = ((uint4*)b.ship)[g];
        int4 c = ((int4*)b.cargo)[g], a = ((int4*)b.act)[g];
        double2 f0 = ((double2*)b.fuel)[2 * g], f1 = ((double2*)b.fuel)[2 * g + 1];
        s.x ^= (uint32_t)a.x;
        s.y ^= (uint32_t)a.y;
        c.x += a.z;
        f0.x -= 1.0;
        f1.y -= 1.0;
        ((uint4*)b.ship)[g] = s;
        ((int4*)b.cargo)[g] = c;
        ((double2*)b.fuel)[2 * g] = f0;
        ((double2*)b.fuel)[2 * g + 1] = f1;
        ((float4*)b.reward)[g] = make_float4((float)a.x, (float)a.y, (float)a.z, (float)a.w);
        ((uint32_t*)b.done)[g] = s.x & 0x01010101u;
        ((uint32_t*)b.err)[g] = s.y & 0x03030303u;
    }
}

// 4 envs per thread: 80 B in (5 x 16 B), 88 B out (5.5 x 16 B): read 5 float4, write 5 float4 + 1 float2
__global__ __launch_bounds__(256) void kC(const float4* in, float4* out,
                                          float2* __restrict__ out2, int64_t groups) {
    for (int64_t g = blockIdx.x * 256ll + threadIdx.x; g < groups; g += (int64_t)gridDim.x * 256) {
        float4 v[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) v[k] = in[k * groups + g];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            v[k].x += 1.0f;
            out[k * groups + g] = v[k];
        }
        out2[g] = make_float2(v[0].y, v[1].z);
    }
}

template <typename F>
float time_it(F launch, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 5; ++i) launch();
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) launch();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1000.0f / reps;
}

int main() {
    const int blocks_opts[] = {1024, 2048, 4096, 8192};
    for (int64_t n : {(int64_t)1 << 20, (int64_t)1 << 24}) {
        const int64_t groups = n / 4;
        BufA A;
        BufB B;
        // one arena, every buffer 2 MiB aligned (ARENA=1) or separate hipMallocs (ARENA=0)
        const bool arena = getenv("ARENA") && atoi(getenv("ARENA"));
        char* base = nullptr;
        size_t off = 0;
        const size_t align = 2u << 20;
        if (arena) CK(hipMalloc(&base, 40 * (size_t)n + 16 * align));
        auto get = [&](size_t bytes) -> void* {
            if (!arena) {
                void* p = nullptr;
                (void)hipMalloc(&p, bytes);
                return p;
            }
            void* p = base + off;
            off += (bytes + align - 1) / align * align;
            return p;
        };
        A.x = (uint8_t*)get(n);
        A.y = (uint8_t*)get(n);
        A.o = (uint8_t*)get(n);
        A.d = (uint8_t*)get(n);
        A.done = (uint8_t*)get(n);
        A.err = (uint8_t*)get(n);
        A.cargo = (int32_t*)get(4 * n);
        A.act = (int32_t*)get(4 * n);
        A.fuel = (double*)get(8 * n);
        A.reward = (float*)get(4 * n);
        B.ship = (uint32_t*)get(4 * n);
        CK(hipMemset(A.x, 0, n));
        B.done = A.done;
        B.err = A.err;
        B.cargo = A.cargo;
        B.act = A.act;
        B.fuel = A.fuel;
        B.reward = A.reward;
        float4 *cin, *cout;
        float2* cout2;
        CK(hipMalloc(&cin, 5 * groups * sizeof(float4)));
        CK(hipMalloc(&cout, 5 * groups * sizeof(float4)));
        CK(hipMalloc(&cout2, groups * sizeof(float2)));
        const double bytes = 42.0 * n;
        for (int blocks : blocks_opts) {
            const int reps = n > (1 << 20) ? 50 : 300;
            float ta = time_it([&] { kA<<<blocks, 256>>>(A, groups); }, reps);
            float tb = time_it([&] { kB<<<blocks, 256>>>(B, groups); }, reps);
            float tc = time_it([&] { kC<<<blocks, 256>>>(cin, cout, cout2, groups); }, reps);
            float td = time_it([&] { kC<<<blocks, 256>>>(cin, cin, cout2, groups); }, reps);
            int flip = 0;
            float te = time_it([&] {
                flip ^= 1;
                if (flip) kC<<<blocks, 256>>>(cin, cout, cout2, groups);
                else kC<<<blocks, 256>>>(cout, cin, cout2, groups);
            }, reps);
            printf("{\"D_inplace_us\": %.2f, \"E_pingpong_us\": %.2f}\n", td, te);
            printf("{\"arena\": %d, \"n\": %lld, \"blocks\": %d, \"A_us\": %.2f, \"B_us\": %.2f, \"C_us\": %.2f, "
                   "\"A_GBps\": %.0f, \"B_GBps\": %.0f, \"C_GBps\": %.0f}\n",
                   (int)arena, (long long)n, blocks, ta, tb, tc, bytes / ta / 1e3, bytes / tb / 1e3,
                   bytes / tc / 1e3);
        }
        if (!arena) {
            (void)hipFree(A.x); (void)hipFree(A.y); (void)hipFree(A.o); (void)hipFree(A.d);
            (void)hipFree(A.done); (void)hipFree(A.err); (void)hipFree(A.cargo);
            (void)hipFree(A.act); (void)hipFree(A.fuel); (void)hipFree(A.reward);
            (void)hipFree(B.ship);
        } else {
            (void)hipFree(base);
        }
        (void)hipFree(cin); (void)hipFree(cout); (void)hipFree(cout2);
    }
    return 0;
}
