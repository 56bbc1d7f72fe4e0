// layoutbench.hip — in-place streaming floors of candidate state layouts (tuning tool).
//   hipcc --offload-arch=gfx950 -O3 -o tools/layoutbench tools/layoutbench.hip
// K1: the step kernel's streams: x,y,origin,dest u8 (4 B/lane per 4 envs), cargo i32,
//     fuel f64, action i32 in; same + reward f32, done u8, err i8 out.
// K2: K1 + the per-workgroup LDS world staging (730 words) and barrier.
// K3: x,y,origin,dest packed in one u32 "ship word" per env (16 B/lane).
// Scalar variables only (no private arrays: hipcc promotes those to LDS).
// Every kernel also has a nontemporal-store variant (the step kernel's stores).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

struct S {
    uint32_t *x, *y, *o, *d, *done, *err, *ship;  // u8 x4 packed words / ship words
    int4 *cargo, *act;
    double2* fuel;
    float4* reward;
    const uint32_t* world;
};

template <typename T>
__device__ __forceinline__ void st(T* p, T v, bool nt) {
    if (nt) {
        if constexpr (sizeof(T) == 16) {
            typedef uint32_t u4 __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(__builtin_bit_cast(u4, v), reinterpret_cast<u4*>(p));
        } else {
            __builtin_nontemporal_store(v, p);
        }
    } else {
        *p = v;
    }
}

template <bool kStage, bool kNt>
__global__ __launch_bounds__(256) void k1(S s, int64_t groups) {
    extern __shared__ uint32_t lds[];
    int64_t g = blockIdx.x * 256ll + threadIdx.x;
    uint32_t salt = 0;
    if (kStage) {
        for (int i = threadIdx.x; i < 730; i += 256) lds[i] = s.world[i];
        __syncthreads();
        salt = lds[threadIdx.x & 511];
    }
    for (; g < groups; g += (int64_t)gridDim.x * 256) {
        uint32_t x = s.x[g], y = s.y[g], o = s.o[g], d = s.d[g];
        int4 c = s.cargo[g], a = s.act[g];
        double2 f0 = s.fuel[2 * g], f1 = s.fuel[2 * g + 1];
        x ^= (uint32_t)a.x ^ salt;
        y ^= (uint32_t)a.y;
        c.x += a.z;
        f0.x -= 1.0;
        f1.y -= 1.0;
        st(&s.x[g], x, kNt);
        st(&s.y[g], y, kNt);
        st(&s.o[g], o + 1, kNt);
        st(&s.d[g], d + 1, kNt);
        st(&s.cargo[g], c, kNt);
        st(&s.fuel[2 * g], f0, kNt);
        st(&s.fuel[2 * g + 1], f1, kNt);
        st(&s.reward[g], make_float4((float)a.x, (float)a.y, (float)a.z, (float)a.w), kNt);
        st(&s.done[g], x & 0x01010101u, kNt);
        st(&s.err[g], y & 0x03030303u, kNt);
    }
}

template <bool kNt>
__global__ __launch_bounds__(256) void k3(S s, int64_t groups) {
    for (int64_t g = blockIdx.x * 256ll + threadIdx.x; g < groups; g += (int64_t)gridDim.x * 256) {
        uint4 sh = ((uint4*)s.ship)[g];
        int4 c = s.cargo[g], a = s.act[g];
        double2 f0 = s.fuel[2 * g], f1 = s.fuel[2 * g + 1];
        sh.x ^= (uint32_t)a.x;
        sh.y ^= (uint32_t)a.y;
        c.x += a.z;
        f0.x -= 1.0;
        f1.y -= 1.0;
        st(&((uint4*)s.ship)[g], sh, kNt);
        st(&s.cargo[g], c, kNt);
        st(&s.fuel[2 * g], f0, kNt);
        st(&s.fuel[2 * g + 1], f1, kNt);
        st(&s.reward[g], make_float4((float)a.x, (float)a.y, (float)a.z, (float)a.w), kNt);
        st(&s.done[g], sh.x & 0x01010101u, kNt);
        st(&s.err[g], sh.y & 0x03030303u, kNt);
    }
}

template <typename F> float time_it(F launch, int reps) {
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

template <typename T> T* alloc(size_t bytes) {
    void* p = nullptr;
    (void)hipMalloc(&p, bytes);
    (void)hipMemset(p, 0, bytes);
    return (T*)p;
}

int main() {
    for (int64_t n : {(int64_t)1 << 20, (int64_t)1 << 22, (int64_t)1 << 24}) {
        const int64_t groups = n / 4;
        S s;
        s.x = alloc<uint32_t>(n); s.y = alloc<uint32_t>(n); s.o = alloc<uint32_t>(n);
        s.d = alloc<uint32_t>(n); s.done = alloc<uint32_t>(n); s.err = alloc<uint32_t>(n);
        s.ship = alloc<uint32_t>(4 * n);
        s.cargo = alloc<int4>(4 * n); s.act = alloc<int4>(4 * n);
        s.fuel = alloc<double2>(8 * n); s.reward = alloc<float4>(4 * n);
        s.world = alloc<uint32_t>(4096);
        const double bytes = 42.0 * n;
        const int reps = n > (1 << 20) ? 100 : 400;
        // 2048 workgroups (grid-stride) and one group per thread (the step kernel's grid)
        for (int blocks : {2048, (int)(groups / 256)}) {
            float t1 = time_it([&] { k1<false, false><<<blocks, 256, 0>>>(s, groups); }, reps);
            float t2 = time_it([&] { k1<true, false><<<blocks, 256, 4096>>>(s, groups); }, reps);
            float t3 = time_it([&] { k3<false><<<blocks, 256>>>(s, groups); }, reps);
            float t4 = time_it([&] { k1<false, true><<<blocks, 256, 0>>>(s, groups); }, reps);
            float t5 = time_it([&] { k1<true, true><<<blocks, 256, 4096>>>(s, groups); }, reps);
            float t6 = time_it([&] { k3<true><<<blocks, 256>>>(s, groups); }, reps);
            printf("{\"n\": %lld, \"blocks\": %d, \"k1_us\": %.2f, \"k1_lds_us\": %.2f, \"k3_ship_us\": %.2f, "
                   "\"k1_nt_us\": %.2f, \"k1_lds_nt_us\": %.2f, \"k3_ship_nt_us\": %.2f, \"k1_nt_GBps\": %.0f}\n",
                   (long long)n, blocks, t1, t2, t3, t4, t5, t6, bytes / t4 / 1e3);
        }
    }
    return 0;
}
