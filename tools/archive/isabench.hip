// isabench.hip — issue cost (cycles per wave-instruction) of the VALU ops the step
// kernel leans on, one wave per SIMD, 8 independent chains per loop body.
//   hipcc -O3 --offload-arch=gfx950 -o tools/isabench tools/isabench.hip && ./tools/isabench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define REP 256

#define BODY8(S) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)

template <int OP>
__global__ void bench(uint64_t* out, uint32_t seed) {
    uint32_t a[8], b[8];
    double d[8];
    for (int i = 0; i < 8; ++i) {
        a[i] = seed * (threadIdx.x + 1) + i;
        b[i] = a[i] ^ 0x1234567u;
        d[i] = (double)a[i];
    }
    uint64_t t0 = __builtin_readcyclecounter();
    for (int r = 0; r < REP; ++r) {
        if constexpr (OP == 0) {  // v_mad_u64_u32
#define S(i) { uint64_t p_; asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, 0" : "=v"(p_) : "v"(a[i]), "v"(b[i]) : "s0", "s1"); a[i] = (uint32_t)(p_ >> 32); }
            BODY8(S)
#undef S
        } else if constexpr (OP == 1) {  // v_mul_hi_u32
#define S(i) asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "v"(b[i]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 2) {  // v_mul_lo_u32
#define S(i) asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "v"(b[i]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 3) {  // v_xor3_b32
#define S(i) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a[i]) : "v"(b[i]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 4) {  // v_fma_f64
#define S(i) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(d[i]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 5) {  // v_add_f64
#define S(i) asm volatile("v_add_f64 %0, %0, %0" : "+v"(d[i]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 6) {  // v_cvt_f64_u32
#define S(i) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d[i]) : "v"(a[i]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 7) {  // v_sqrt_f64
#define S(i) asm volatile("v_sqrt_f64 %0, %0" : "+v"(d[i]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 8) {  // v_mul_u32_u24
#define S(i) asm volatile("v_mul_u32_u24 %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "v"(b[i]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 9) {  // v_cndmask_b32 (vcc)
#define S(i) asm volatile("v_cndmask_b32 %0, %1, %2, vcc" : "=v"(a[i]) : "v"(a[i]), "v"(b[i]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 10) {  // v_add_u32
#define S(i) asm volatile("v_add_u32 %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "v"(b[i]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 11) {  // v_mul_f64
#define S(i) asm volatile("v_mul_f64 %0, %0, %0" : "+v"(d[i]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 12) {  // v_cmp_lt_f64 -> vcc
#define S(i) asm volatile("v_cmp_lt_f64 vcc, %0, %1" : : "v"(d[i]), "v"(d[(i + 1) & 7]) : "vcc");
            BODY8(S)
#undef S
        } else if constexpr (OP == 13) {  // v_mul_hi_u32_u24
#define S(i) asm volatile("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "v"(b[i]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 14) {  // v_bfe_u32
#define S(i) asm volatile("v_bfe_u32 %0, %1, 8, 8" : "=v"(a[i]) : "v"(b[i]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 16) {  // v_bitop3_b32 (xor3, gfx950)
#define S(i) asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96" : "+v"(a[i]) : "v"(b[i]), "v"(a[(i + 1) & 7]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 17) {  // v_ldexp_f64
#define S(i) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d[i]) : "v"(b[i]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 18) {  // v_cvt_f32_f64
#define S(i) { float f_; asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f_) : "v"(d[i])); a[i] = __float_as_uint(f_); }
            BODY8(S)
#undef S
        } else if constexpr (OP == 19) {  // v_cvt_i32_f64
#define S(i) asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(a[i]) : "v"(d[i]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 20) {  // v_cndmask_b32 e64 with sgpr-pair condition
#define S(i) asm volatile("v_cndmask_b32_e64 %0, %1, %2, s[4:5]" : "=v"(a[i]) : "v"(a[i]), "v"(b[i]));
            BODY8(S)
#undef S
        } else if constexpr (OP == 15) {  // v_pk_mul_f32 (packed, reference for dual rate)
#define S(i) asm volatile("v_pk_mul_f32 %0, %0, %0" : "+v"(d[i]));
            BODY8(S)
#undef S
        }
    }
    uint64_t t1 = __builtin_readcyclecounter();
    uint32_t acc = 0;
    for (int i = 0; i < 8; ++i) acc ^= a[i] ^ b[i] ^ (uint32_t)__double_as_longlong(d[i]);
    if (threadIdx.x == 0) out[blockIdx.x * 2] = t1 - t0;
    if (acc == 0x12345678u) out[blockIdx.x * 2 + 1] = acc;
}

template <int OP>
double run(const char* name, uint64_t* dout) {
    hipLaunchKernelGGL(bench<OP>, dim3(1), dim3(64), 0, 0, dout, 7u);  // warm
    hipDeviceSynchronize();
    hipLaunchKernelGGL(bench<OP>, dim3(1), dim3(64), 0, 0, dout, 7u);
    hipDeviceSynchronize();
    uint64_t h[2];
    hipMemcpy(h, dout, sizeof(h), hipMemcpyDeviceToHost);
    const double c = (double)h[0] / (REP * 8.0);
    printf("%-20s %6.2f cycles/wave-instr (s_memtime units)\n", name, c);
    return c;
}

int main() {
    uint64_t* d;
    hipMalloc(&d, 1 << 16);
    run<10>("v_add_u32", d);
    run<0>("v_mad_u64_u32", d);
    run<1>("v_mul_hi_u32", d);
    run<2>("v_mul_lo_u32", d);
    run<8>("v_mul_u32_u24", d);
    run<13>("v_mul_hi_u32_u24", d);
    run<3>("v_xor_b32", d);
    run<14>("v_bfe_u32", d);
    run<9>("v_cndmask_b32", d);
    run<4>("v_fma_f64", d);
    run<5>("v_add_f64", d);
    run<11>("v_mul_f64", d);
    run<12>("v_cmp_lt_f64", d);
    run<6>("v_cvt_f64_u32", d);
    run<7>("v_sqrt_f64", d);
    run<15>("v_pk_mul_f32", d);
    run<16>("v_bitop3_b32", d);
    run<17>("v_ldexp_f64", d);
    run<18>("v_cvt_f32_f64", d);
    run<19>("v_cvt_i32_f64", d);
    run<20>("v_cndmask_b32_e64", d);
    hipFree(d);
    return 0;
}
