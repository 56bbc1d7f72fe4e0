// mfmarate.hip — issue rate of v_mfma_f32_32x32x2_f32 per SIMD (tuning tool): one workgroup
// per CU, W waves per SIMD, each running C independent accumulation chains of K MFMAs
// (operands in registers, no memory in the loop). Prints cycles per MFMA per SIMD and per
// wave, from s_memtime around the loop (median over the grid's workgroups, wave 0 of each).
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfmarate tools/mfmarate.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

typedef __attribute__((ext_vector_type(16))) float f32x16;

template <int C>
__global__ void chains(int k, float seed, uint64_t* cyc, float* sink) {
    f32x16 acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[c][i] = 0.0f;
    const float a = seed + (float)(threadIdx.x & 7), b = seed * 0.5f + (float)(threadIdx.x >> 6);
    __syncthreads();
    const uint64_t t0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int j = 0; j < k; ++j)
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
    float s = 0.0f;
#pragma unroll
    for (int c = 0; c < C; ++c) s += acc[c][0];
    const uint64_t t1 = __builtin_readcyclecounter(), r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        cyc[(blockIdx.x * 64 + (threadIdx.x >> 6)) * 2] = t0;
        cyc[(blockIdx.x * 64 + (threadIdx.x >> 6)) * 2 + 1] = t1;
        if (threadIdx.x == 0) reinterpret_cast<float*>(sink)[1024 + blockIdx.x] = (float)(t1 - t0) / (float)(r1 - r0) * 0.1f;
    }
    if (s == 12345.0f) sink[threadIdx.x] = s;  // keeps the chains live
}

// the same chain with its B operands read from an LDS [k][33] tile 8 k-steps ahead, as T1's
// gemm_lds does (the tile is 64 k-steps, re-read each pass)
__global__ void lds_chain(int k, float seed, uint64_t* cyc, float* sink) {
    __shared__ float tile[128 * 33 * 4];
    const int lane = threadIdx.x & 63, h = lane >> 5, c = lane & 31, w = threadIdx.x >> 6;
    float* src = tile + (w & 3) * 128 * 33;
    for (int i = threadIdx.x; i < 128 * 33 * 4; i += blockDim.x) tile[i] = seed + (float)(i & 15);
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
    const float a = seed + (float)(threadIdx.x & 7);
    __syncthreads();
    const uint64_t t0 = __builtin_readcyclecounter();
    for (int j = 0; j < k; j += 64) {
        float b[64];
#pragma unroll
        for (int s = 0; s < 8; ++s) b[s] = src[(2 * s + h) * 33 + c];
#pragma unroll
        for (int s = 0; s < 64; ++s) {
            if (s + 8 < 64) b[s + 8] = src[(2 * (s + 8) + h) * 33 + c];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b[s], acc, 0, 0, 0);
        }
#pragma unroll
        for (int s = 0; s < 8; ++s) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
        for (int s = 0; s < 64; ++s) {
            if (s + 8 < 64) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
    }
    const float sum = acc[0];
    const uint64_t t1 = __builtin_readcyclecounter();
    if ((threadIdx.x & 63) == 0) {
        cyc[(blockIdx.x * 64 + (threadIdx.x >> 6)) * 2] = t0;
        cyc[(blockIdx.x * 64 + (threadIdx.x >> 6)) * 2 + 1] = t1;
    }
    if (sum == 12345.0f) sink[threadIdx.x] = sum;
}

template <int C>
void run(int waves_per_simd, int cus) {
    const int k = 1024, threads = 4 * 64 * waves_per_simd;
    uint64_t* cyc;
    float* sink;
    (void)hipMalloc(&cyc, (size_t)cus * 128 * sizeof(uint64_t));
    (void)hipMalloc(&sink, 4096 * sizeof(float));
    (void)hipMemset(sink, 0, 4096 * sizeof(float));
    if (C == 0) {  // C = 0: lds_chain, one chain with LDS B operands
        lds_chain<<<cus, threads>>>(k, 1.0f, cyc, sink);
        lds_chain<<<cus, threads>>>(k, 1.0f, cyc, sink);
    } else {
        chains<(C > 0 ? C : 1)><<<cus, threads>>>(k, 1.0f, cyc, sink);  // warm-up
        chains<(C > 0 ? C : 1)><<<cus, threads>>>(k, 1.0f, cyc, sink);
    }
    (void)hipDeviceSynchronize();
    std::vector<uint64_t> h((size_t)cus * 128);
    (void)hipMemcpy(h.data(), cyc, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost);
    // per workgroup: the span from the first wave's start to the last wave's end, and wave
    // 0's own span (s_memtime counts the shader clock); per SIMD the MFMAs are W * C * k
    std::vector<uint64_t> span, own;
    const int nw = threads / 64;
    for (int b = 0; b < cus; ++b) {
        uint64_t lo = ~0ull, hi = 0;
        for (int w = 0; w < nw; ++w) {
            lo = std::min(lo, h[((size_t)b * 64 + w) * 2]);
            hi = std::max(hi, h[((size_t)b * 64 + w) * 2 + 1]);
        }
        span.push_back(hi - lo);
        own.push_back(h[(size_t)b * 128 + 1] - h[(size_t)b * 128]);
    }
    std::vector<float> ghz(cus);
    (void)hipMemcpy(ghz.data(), sink + 1024, cus * sizeof(float), hipMemcpyDeviceToHost);
    std::sort(ghz.begin(), ghz.end());
    std::sort(span.begin(), span.end());
    std::sort(own.begin(), own.end());
    const double med = (double)span[span.size() / 2], med0 = (double)own[own.size() / 2];
    printf("{\"waves_per_simd\": %d, \"chains_per_wave\": %d, \"mfma_per_wave\": %d, "
           "\"cycles_per_mfma_per_simd\": %.1f, \"wave0_cycles_per_mfma\": %.1f, \"ghz_wave0\": %.2f}\n",
           waves_per_simd, C, (C ? C : 1) * k, med / (waves_per_simd * (C ? C : 1) * k), med0 / ((C ? C : 1) * k), ghz[cus / 2]);
    (void)hipFree(cyc);
    (void)hipFree(sink);
}

int main() {
    const int cus = 256;
    for (int w : {1, 2, 4}) {
        run<1>(w, cus);
        run<2>(w, cus);
        run<4>(w, cus);
        run<0>(w, cus);
    }
    return 0;
}
