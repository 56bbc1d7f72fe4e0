// philox.h — device-side counter-based RNG for the step kernels (gfx950).
//
// Philox4x32-10 (Salmon et al., SC'11; constants of Random123's philox4x32),
// keyed by the 64-bit seed and indexed by (global env id, step counter, slot):
// no RNG state lives in HBM. The draw conventions below are the "RNG contract"
// of DESIGN.md; oracle/shipenv_oracle.c states the same contract independently
// on the CPU, and tests compare the two bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace shipenv {

// Step draws (contract v5) are keyed by the quad k = env / 4: quad blocks, where word
// j belongs to env 4k+j (a 32-bit uniform u = w * 2^-32 or an integer draw), and the
// LOSS_r / RESET_r blocks, which belong whole to the r-th env of the quad whose gate
// fired / that auto-resets.
// The reset kernel and the synthetic agent draw one block per env.
enum Slot : uint32_t {
    kSlotFuel = 0,           // u_fuel (fuel-cost noise, every step)
    kSlotLoss0 = 1,          // LOSS_r, r = 0..3 at slots 1, 2, 8, 9 (kSlotLoss[r]): the r-th env
    kSlotLoss1 = 2,          // of the quad whose gate fired takes the whole block: word 0
                             // u_type, words 1-3 the Beta(2,2) uniforms
    kSlotArrive = 3,         // new destination != origin on arrival
    kSlotReset = 4,          // RESET_r, r = 0..3 at slots 4, 10, 16, 17 (reset_slot(r)): the
                             // r-th env of the quad auto-reset in step t: word 0 origin, 1 dest
    kSlotExplicitReset = 5,  // se_reset, per env, epoch in the t word: words 0 origin, 1 dest
    kSlotAction = 6,         // synthetic bench agent, per env
    kSlotGate = 7,           // u_gate (cargo-loss gate)
    kSlotLoss2 = 8,
    kSlotLoss3 = 9,
    kSlotReset1 = 10,
    kSlotSample = 11,        // se_sample_actions, per env: word 0
    kSlotRollout = 12,       // rollout attempt, per rollout: sample word, u_fuel, u_gate, u_type
    kSlotRolloutB = 13,      // rollout attempt (partial loss / arrival): 3 beta uniforms, dest
    kSlotPolicy = 14,        // se_policy, per env: explore draw, random.choice index
    kSlotReplay = 15,        // se_replay_sample, key (seed, 2^64 - 1), t = update: Feistel round keys
    kSlotReset2 = 16,
    kSlotReset3 = 17,
};

// RESET_r slot of the r-th auto-reset env of a quad
__host__ __device__ constexpr uint32_t reset_slot(uint32_t r) {
    return r == 0 ? kSlotReset : r == 1 ? kSlotReset1 : r == 2 ? kSlotReset2 : kSlotReset3;
}

// LOSS_r slot of the r-th firing env of a quad
__host__ __device__ constexpr uint32_t loss_slot(uint32_t r) {
    return r == 0 ? kSlotLoss0 : r == 1 ? kSlotLoss1 : r == 2 ? kSlotLoss2 : kSlotLoss3;
}

struct U4 {
    uint32_t v[4];
};

// One 32x32 -> 64-bit product per multiplier (v_mad_u64_u32) instead of a
// separate mul_hi / mul_lo pair; the key schedule is wave-uniform (scalar).
__device__ __forceinline__ U4 philox10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                       uint32_t k0, uint32_t k1) {
    // The key is opaque here, so each block recomputes its 18 scalar key adds
    // instead of the compiler hoisting every block's schedule out of the step
    // loop: ~20 live SGPRs per block spilled to VGPR lanes (v_readlane + s_nop).
    asm volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        // three-way xor in one v_bitop3_b32 (truth table 0x96, gfx950)
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return U4{{c0, c1, c2, c3}};
}

// (seed, env, t, slot) -> 4 words
struct Key {
    uint32_t k0, k1;  // seed
    uint32_t e0, e1;  // global env id
};

__device__ __forceinline__ U4 draw(const Key& k, uint32_t t, uint32_t slot) {
    return philox10(k.e0, k.e1, t, slot, k.k0, k.k1);
}

// integer uniform on [0, m): high word of r * m (bias < m / 2^32)
__device__ __forceinline__ int32_t uniform_int(uint32_t r, uint32_t m) {
    return (int32_t)__umulhi(r, m);
}

// port index uniform over the P-1 ports other than `other`
__device__ __forceinline__ int32_t pick_other(uint32_t r, int32_t P, int32_t other) {
    const int32_t k = uniform_int(r, (uint32_t)(P - 1));
    return k + (k >= other ? 1 : 0);
}

}  // namespace shipenv
