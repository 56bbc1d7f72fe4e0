// floorbench.hip — what separates the step kernel's no-logic floor (SHIPENV_ABLATE=2,
// 7.5-8.4 us at N = 2^20) from a bare kernel with the same streams (layoutbench K1,
// 6.5 us). Each variant changes one thing against K1 (tuning tool):
//   base     K1: the step's streams, 4 envs per lane, 1024 x 256 threads
//   karg     the arguments padded to the size of StepArgs (~300 B)
//   ntload   nontemporal loads (the product's choice at N = 2^20)
//   lds      5 KB of dynamic LDS per workgroup (the world image's allocation)
//   cold     a fresh action row per launch (1000 rows, read from HBM like bench.py)
//   wpe      __attribute__((amdgpu_waves_per_eu(4))) as on step_kernel
//   hipcc --offload-arch=gfx950 -O3 -o tools/floorbench tools/floorbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

struct S {
    uint32_t *x, *y, *o, *d, *done, *err;
    int4* cargo;
    const int4* act;
    double2* fuel;
    float4* reward;
};
struct SPad {
    S s;
    char pad[200];
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <bool kNt, typename T>
__device__ __forceinline__ T ld(const T* p) {
    if constexpr (kNt) {
        if constexpr (sizeof(T) == 16)
            return __builtin_bit_cast(T, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)));
        else
            return __builtin_nontemporal_load(p);
    } else {
        return *p;
    }
}
template <typename T>
__device__ __forceinline__ void st(T* p, T v) {
    if constexpr (sizeof(T) == 16)
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, v), reinterpret_cast<u32x4*>(p));
    else
        __builtin_nontemporal_store(v, p);
}

template <bool kNt>
__device__ __forceinline__ void body(const S& s, int64_t g) {
    uint32_t x = ld<kNt>(&s.x[g]), y = ld<kNt>(&s.y[g]), o = ld<kNt>(&s.o[g]), d = ld<kNt>(&s.d[g]);
    int4 c = ld<kNt>(&s.cargo[g]);
    const int4 a = ld<kNt>(&s.act[g]);
    double2 f0 = ld<kNt>(&s.fuel[2 * g]), f1 = ld<kNt>(&s.fuel[2 * g + 1]);
    x ^= (uint32_t)a.x;
    y ^= (uint32_t)a.y;
    c.x += a.z;
    f0.x -= 1.0;
    f1.y -= 1.0;
    st(&s.x[g], x);
    st(&s.y[g], y);
    st(&s.fuel[2 * g], f0);
    st(&s.fuel[2 * g + 1], f1);
    st(&s.done[g], x & 0x01010101u);
    st(&s.err[g], y & 0x03030303u);
    st(&s.o[g], o + 1);
    st(&s.d[g], d + 1);
    st(&s.cargo[g], c);
    st(&s.reward[g], make_float4((float)a.x, (float)a.y, (float)a.z, (float)a.w));
}

template <bool kNt>
__global__ __launch_bounds__(256) void k_base(S s, int64_t groups) {
    const int64_t g = blockIdx.x * 256ll + threadIdx.x;
    if (g < groups) body<kNt>(s, g);
}
__global__ __launch_bounds__(256) void k_karg(SPad p, int64_t groups) {
    const int64_t g = blockIdx.x * 256ll + threadIdx.x;
    if (g < groups) body<false>(p.s, g);
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_wpe(S s, int64_t groups) {
    const int64_t g = blockIdx.x * 256ll + threadIdx.x;
    if (g < groups) body<false>(s, g);
}

template <typename F>
float time_it(F launch, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 20; ++i) launch(i);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) launch(i);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1000.0f / reps;
}

template <typename T>
T* alloc(size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        exit(1);
    }
    (void)hipMemset(p, 0, bytes);
    return (T*)p;
}

int main() {
    const int64_t n = 1 << 20, groups = n / 4;
    const int rows = 1000, reps = 1000, blocks = (int)(groups / 256);
    S s;
    s.x = alloc<uint32_t>(n);
    s.y = alloc<uint32_t>(n);
    s.o = alloc<uint32_t>(n);
    s.d = alloc<uint32_t>(n);
    s.done = alloc<uint32_t>(n);
    s.err = alloc<uint32_t>(n);
    s.cargo = alloc<int4>(4 * n);
    s.fuel = alloc<double2>(8 * n);
    s.reward = alloc<float4>(4 * n);
    int4* acts = alloc<int4>((size_t)rows * 4 * n);
    s.act = acts;
    SPad p;
    p.s = s;
    for (int rep = 0; rep < 2; ++rep) {
        const float base = time_it([&](int) { k_base<false><<<blocks, 256>>>(s, groups); }, reps);
        const float karg = time_it([&](int) { k_karg<<<blocks, 256>>>(p, groups); }, reps);
        const float ntl = time_it([&](int) { k_base<true><<<blocks, 256>>>(s, groups); }, reps);
        const float lds = time_it([&](int) { k_base<false><<<blocks, 256, 5120>>>(s, groups); }, reps);
        const float cold = time_it([&](int i) {
            S c = s;
            c.act = acts + (size_t)(i % rows) * groups;
            k_base<false><<<blocks, 256>>>(c, groups);
        }, reps);
        const float wpe = time_it([&](int) { k_wpe<<<blocks, 256>>>(s, groups); }, reps);
        printf("{\"n\": %lld, \"base_us\": %.2f, \"karg_us\": %.2f, \"ntload_us\": %.2f, \"lds_us\": %.2f, "
               "\"cold_us\": %.2f, \"wpe_us\": %.2f}\n",
               (long long)n, base, karg, ntl, lds, cold, wpe);
        fflush(stdout);
    }
    return 0;
}
