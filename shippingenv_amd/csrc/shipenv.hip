// shipenv.hip — MI355X (gfx950) batched ShippingEnv: step / reset / observe kernels
// and the C-ABI of include/shipenv.h.
//
// What one step does per environment is shipping/environment.py:359-376 (step)
// and :273-339 (_move_ship) of the reference; DESIGN.md walks through the
// mapping. The shape of the work is what drives the design:
//   * the path is HBM-streaming integer/f64 work, ~0 useful FLOPs: no MFMA;
//   * state is SoA with narrow fields (u8 positions/indices, i32 cargo,
//     f64 fuel) so each field of 4 consecutive envs is one 4-/16-byte lane
//     access: every wave instruction is a fully coalesced 256 B - 1 KiB access;
//   * the static world (ground bitmap, port bitmap, ports table) is staged once
//     per workgroup into LDS; the per-env map lookups are LDS reads;
//   * RNG is counter-based Philox keyed by (seed, global env id): 0 bytes of RNG
//     state in HBM and shard-invariant results;
//   * auto-reset compacts finished envs into a done list with one wave ballot
//     prefix and one atomic per wave, and reduces episode statistics per
//     workgroup into a fixed slab (deterministic sums, no float atomics).
//
// Built with -ffp-contract=off: the reference's f64 arithmetic (CPython float,
// np.sqrt) is unfused, and an FMA in -0.1 + 0.2*u changes fuel bits.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/shipenv.h"
#include "philox.h"

#ifndef SHIPENV_ABLATE
#define SHIPENV_ABLATE 0  // 0 = the product; 1, 2 = timing-only ablations (tools/ablate.py)
#endif

using namespace shipenv;

namespace {

constexpr int kBlock = 256;       // 4 waves
constexpr int kEnvsPerThread = 4; // one 4-byte / 16-byte lane access per field
constexpr int kMaxBlocks = 2048;  // 256 CUs x 8; grid-stride beyond
constexpr int kStepBlocks = 2048; // step kernel default cap (SHIPENV_STEP_BLOCKS overrides)

// se_tape.used bits (replay): which of the reference's draws this step consumed
constexpr uint32_t kUsedFuelGate = SE_USED_FUEL_GATE, kUsedLossType = SE_USED_LOSS_TYPE,
                   kUsedBeta = SE_USED_BETA, kUsedArrive = SE_USED_ARRIVE, kUsedMoved = SE_USED_MOVED;

// reference constants, shipping/environment.py:8-26
constexpr double kFuelInit = 200.0;
constexpr double kMaxCargo = 50.0;

// ------------------------------------------------------------------ world image
// One device buffer of 32-bit words, staged as-is into LDS by every workgroup:
//   [0, w)          ground bitmap  (bit = 1: np_game[x, y] == GROUND)
//   [w, 2w)         port bitmap    (bit = 1: some port sits on the cell)
//   [2w, 3w)        port-bit prefix counts (set bits in the words before)
//   [3w, 3w+P)      port position  (x | y << 8)
//   [+P)            port fuel stock
//   [+P)            port cargo stock
//   [+P+1)          rank -> port: the FIRST port on the rank-th occupied cell
//                   (_get_current_port_idx returns the first match, :150-152)
//   [frac, +100)    f64 table fl(c / 50) for c in [0, 50) (8-byte aligned)
// For the 100x100 map with 5 ports that is 4.2 KB.
struct WorldDims {
    int32_t H, W, P, words;
    __host__ __device__ int pos() const { return 3 * words; }
    __host__ __device__ int rank2port() const { return 3 * words + 3 * P; }
    __host__ __device__ int frac() const { return (rank2port() + P + 1 + 1) & ~1; }
    __host__ __device__ int total() const { return frac() + 2 * 50; }
};

struct LdsWorld {
    const uint32_t* ground;
    const uint32_t* portbit;
    const uint32_t* prefix;
    const uint32_t* pos;
    const int32_t* pfuel;
    const int32_t* pcargo;
    const int32_t* rank2port;
    const double* frac;
    int32_t H, W, P;

    __device__ bool is_ground(int x, int y) const {
        const uint32_t c = (uint32_t)(x * W + y);
        return (ground[c >> 5] >> (c & 31)) & 1u;
    }
    // _get_current_port_idx (:145-153): first port on the ship's cell, -1 if none.
    // O(1): rank of the cell among occupied cells -> first port index.
    __device__ int port_at(int x, int y) const {
        const uint32_t c = (uint32_t)(x * W + y);
        const uint32_t word = portbit[c >> 5], bit = c & 31;
        const int rank = (int)prefix[c >> 5] + __popc(word & ((1u << bit) - 1u));
        return ((word >> bit) & 1u) ? rank2port[rank] : -1;
    }
    __device__ int px(int i) const { return (int)(pos[i] & 0xffu); }
    __device__ int py(int i) const { return (int)((pos[i] >> 8) & 0xffu); }
    // normalize(cargo, 50, 0) (util.py:6-8), only read for 0 < cargo < 50
    __device__ double likelihood(int cargo) const { return frac[cargo]; }
};

__device__ __forceinline__ LdsWorld stage_world(const uint32_t* __restrict__ g, WorldDims d,
                                                uint32_t* lds) {
    const int total = d.total();
    for (int i = threadIdx.x; i < total; i += blockDim.x) lds[i] = g[i];
    __syncthreads();
    LdsWorld w;
    w.ground = lds;
    w.portbit = lds + d.words;
    w.prefix = lds + 2 * d.words;
    w.pos = lds + d.pos();
    w.pfuel = (const int32_t*)(lds + d.pos() + d.P);
    w.pcargo = (const int32_t*)(lds + d.pos() + 2 * d.P);
    w.rank2port = (const int32_t*)(lds + d.rank2port());
    w.frac = (const double*)(lds + d.frac());
    w.H = d.H;
    w.W = d.W;
    w.P = d.P;
    return w;
}

// ------------------------------------------------------------------ one env
struct Ship {
    int x, y;
    double fuel;
    int cargo, origin, dest;  // origin/dest: SE_NONE = None
};

__device__ __forceinline__ Key env_key(uint64_t seed, int64_t env) {
    Key k;
    k.k0 = (uint32_t)seed;
    k.k1 = (uint32_t)(seed >> 32);
    k.e0 = (uint32_t)(uint64_t)env;
    k.e1 = (uint32_t)((uint64_t)env >> 32);
    return k;
}

// The rare per-env draws of one MOVE (loss type, beta, arrival redraw): Philox
// (production) or a replay tape. u_fuel / u_gate come from the quad blocks drawn
// for a whole group of 4 envs.
template <bool kReplay>
struct Draws;

template <>
struct Draws<false> {
    Key key;
    uint32_t t;
    __device__ double loss_type() const {  // words 0,1 of slot LOSS
        const U4 a = draw(key, t, kSlotLoss);
        return u53(a.v[0], a.v[1]);
    }
    // Beta(2,2) as the median of three uniforms (words 2,3 of LOSS and 0..3 of
    // BETA) — exact in distribution, a fixed number of draws.
    __device__ double beta() const {
        const U4 a = draw(key, t, kSlotLoss), b = draw(key, t, kSlotBeta);
        const double u1 = u53(a.v[2], a.v[3]), u2 = u53(b.v[0], b.v[1]), u3 = u53(b.v[2], b.v[3]);
        return fmax(fmin(u1, u2), fmin(fmax(u1, u2), u3));
    }
    __device__ int arrive(int P, int origin) const {
        const U4 o = draw(key, t, kSlotArrive);
        return pick_other(o.v[0], P, origin);
    }
};

// Replay: the variates the reference drew through `random`. A missing one (NaN,
// or arrive_dest < 0) makes the step report SE_ERR_NEED_DRAW without effect.
template <>
struct Draws<true> {
    const se_tape* rec;
    __device__ double loss_type() const { return rec->u_type; }
    __device__ double beta() const { return rec->beta; }
    __device__ int arrive(int, int) const { return rec->arrive_dest; }
};

// sqrt of a non-negative integer, correctly rounded (np.sqrt on the int sum of
// squares, shipping/util.py:4). Unit moves take the exact fast path.
__device__ __forceinline__ double int_sqrt_rn(int v) {
    return v == 1 ? 1.0 : __dsqrt_rn((double)v);
}

// Does this env's step draw a gate that can change anything? (a MOVE that passes
// its checks with 0 < cargo < 50; cargo 0 never loses, cargo >= 50 always fires)
template <bool kUnitMoves>
__device__ __forceinline__ bool needs_gate(const LdsWorld& w, const Ship& s, int type, int a, int b) {
    if (kUnitMoves) {
        const int nx = s.x + a, ny = s.y + b;
        return type == 1 && s.dest != SE_NONE && (unsigned)nx < (unsigned)w.H &&
               (unsigned)ny < (unsigned)w.W && s.cargo > 0 && s.cargo < 50;
    }
    return type == 1 && s.cargo > 0 && s.cargo < 50;  // typed form: draw whenever possible
}

// One env's step (:359-376) for a typed action (shipping/type.py:1-5), written as
// selects over the three action families so a wave runs one straight path; only
// cargo loss and arrival branch. Returns SE_ERR_*; an error leaves s untouched
// (the reference raises before mutating: :284 before :287, :266-269, :342-346).
template <bool kUnitMoves, bool kReplay>
__device__ __forceinline__ int env_step(const LdsWorld& w, Ship& s, int e_in, int type, int a, int b,
                                        double u_fuel, double u_gate,
                                        const Draws<kReplay>& dr, double& reward, int& done,
                                        uint32_t& used) {
    // --- MOVE (_move_ship :273-339)
    const bool no_dest = s.dest == SE_NONE;                                      // :276
    const bool big = !kUnitMoves && (a < -256 || a > 256 || b < -256 || b > 256);  // surely OOB
    const int nx = s.x + (big ? 0 : a), ny = s.y + (big ? 0 : b);
    const bool oob = big || (unsigned)nx >= (unsigned)w.H || (unsigned)ny >= (unsigned)w.W;  // :284
    const bool mv_ok = !no_dest && !oob;
    const int cx = mv_ok ? nx : s.x, cy = mv_ok ? ny : s.y;  // in-range cell for the lookups
    // fuel cost (:103-104): dist * (1 + uniform(-0.1, 0.1)), uniform = -0.1 + 0.2*u, unfused
    const double scale = 1.0 + (-0.1 + 0.2 * u_fuel);
    const double cost = kUnitMoves ? scale : int_sqrt_rn(big ? 1 : a * a + b * b) * scale;
    const bool out_of_fuel = s.fuel < cost;  // :288-290
    const double r0 = out_of_fuel ? -10.0 : 0.0;
    const bool ground = w.is_ground(cx, cy);  // :293
    // :294 blocked (-5) or :296-300 moved (-0.0001 then -1), in the reference's add order
    double rm = ground ? r0 + -5.0 : (r0 + -0.0001) + -1.0;
    const int mx = ground ? s.x : cx, my = ground ? s.y : cy;
    const double fuel_m = ground ? s.fuel : s.fuel - cost;
    // :307-315 old cell vs ATTEMPTED cell; sqrt is monotone and the squared
    // distances are small integers, so comparing them is exact
    const int dcl = no_dest ? 0 : s.dest;
    const int px = w.px(dcl), py = w.py(dcl);
    const int d_old = (s.x - px) * (s.x - px) + (s.y - py) * (s.y - py);
    const int d_new = (cx - px) * (cx - px) + (cy - py) * (cy - py);
    rm += d_old > d_new ? 2.0 : -2.0;

    // --- SELECT_PORT (_select_port :265-271)
    const int e_sel = (a < 0 || a >= w.P) ? SE_ERR_PORT_RANGE
                                          : (s.origin == a ? SE_ERR_SAME_PORT : SE_ERR_OK);
    // --- TAKE_FUEL / TAKE_CARGO (:341-357)
    const int idx = w.port_at(s.x, s.y);
    const int sidx = idx < 0 ? 0 : idx;
    const int stock = type == 4 ? w.pcargo[sidx] : w.pfuel[sidx];
    const int e_take = idx < 0 ? SE_ERR_NOT_AT_PORT : ((a <= 0 || a > stock) ? SE_ERR_AMOUNT : SE_ERR_OK);

    const int e = e_in != SE_ERR_OK ? e_in  // the decode runs before env.step (agents/dqn.py:286-287)
                : w.P == 0 ? SE_ERR_NO_PORTS  // :360
                : type == 1 ? (no_dest ? SE_ERR_NO_DEST : (oob ? SE_ERR_OOB : SE_ERR_OK))
                : type == 2 ? e_sel
                : (type == 3 || type == 4) ? e_take
                : SE_ERR_BAD_CATEGORY;  // :373-374
    const bool ok = e == SE_ERR_OK;
    const bool do_move = ok && type == 1;

    int cargo_m = s.cargo, origin_m = s.origin, dest_m = s.dest;
    bool need = false;  // replay only: a variate the reference drew here is missing
    used = do_move ? (kUsedFuelGate | (ground ? 0u : kUsedMoved)) : 0u;
    if (kReplay) need = do_move && (u_fuel != u_fuel || u_gate != u_gate);
    // :318-323 the gate random() <= cargo/50. Production skips the cargo-0 case (a
    // firing gate then loses nothing, :180-181); replay keeps it, because the
    // reference still draws the loss type there (:177) and replay tracks every draw.
    // From cargo 50 on it always fires (random() < 1 <= cargo/50).
    const int ci = (s.cargo > 0 && s.cargo < 50) ? s.cargo : 0;
    const bool fires = s.cargo >= 50 || ((kReplay || s.cargo > 0) && u_gate <= w.likelihood(ci));
    if (do_move && fires) {  // _calculate_cargo_loss :169-200
        used |= kUsedLossType;
        const double lt = dr.loss_type();
        const bool partial = cargo_m != 0 && lt >= 0.1 && lt <= 0.9;  // :180, :184, :188
        double beta = 0.0;
        if (partial) {
            used |= kUsedBeta;
            beta = dr.beta();
        }
        if (kReplay) need = need || lt != lt || (partial && beta != beta);
        const int loss = lt < 0.1 ? 0 : (lt > 0.9 ? cargo_m : (int)(beta * (double)cargo_m));
        cargo_m -= loss;
        rm += (double)(-3 * loss);
    }
    if (do_move && mx == px && my == py) {  // :325-337 arrival
        used |= kUsedArrive;
        rm += (double)(2 * cargo_m);
        cargo_m = 0;
        origin_m = dest_m;
        dest_m = dr.arrive(w.P, origin_m);
        if (kReplay) need = need || dest_m < 0;
        rm += 10.0;
    }
    if (kReplay && need) {  // ask the caller for the next variate; change nothing
        reward = 0.0;
        done = 0;
        return SE_ERR_NEED_DRAW;
    }

    const bool take_fuel = ok && type == 3, take_cargo = ok && type == 4;
    s.x = do_move ? mx : s.x;
    s.y = do_move ? my : s.y;
    s.fuel = do_move ? fuel_m : (take_fuel ? s.fuel + (double)a : s.fuel);
    s.cargo = do_move ? cargo_m : (take_cargo ? s.cargo + a : s.cargo);
    s.origin = do_move ? origin_m : s.origin;
    s.dest = do_move ? dest_m : ((ok && type == 2) ? a : s.dest);
    reward = do_move ? rm : ((take_fuel || take_cargo) ? 0.05 : 0.0);
    done = (do_move && out_of_fuel) ? 1 : 0;
    return e;
}

// utils/preprocessing.py:111-137 (moves N, E, S, W; Python wraps -4..-1)
__device__ __forceinline__ int decode_agent(int P, int act, int& type, int& a, int& b) {
    const int k = act & 3;  // -4..-1 -> 0..3 like Python's negative list index
    const bool move = act < 4;
    type = move ? 1 : (act < 4 + P ? 2 : (act < 4 + P + 50 ? 4 : 3));
    const int val = act - (type == 2 ? 4 : (type == 4 ? 4 + P : 4 + P + 50));
    a = move ? (k == 1 ? -1 : (k == 3 ? 1 : 0)) : val;  // EAST = (-1, 0), WEST = (1, 0)
    b = move ? (k == 0 ? -1 : (k == 2 ? 1 : 0)) : 0;    // NORTH = (0, -1), SOUTH = (0, 1)
    return act < -4 ? SE_ERR_BAD_INDEX : SE_ERR_OK;
}

// reset (:227-243) from two Philox words
__device__ __forceinline__ void reset_ship(const LdsWorld& w, Ship& s, uint32_t r0, uint32_t r1) {
    s.origin = uniform_int(r0, (uint32_t)w.P);
    s.dest = pick_other(r1, w.P, s.origin);
    s.cargo = 0;
    s.fuel = kFuelInit;
    s.x = w.px(s.origin);
    s.y = w.py(s.origin);
}

__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
// number of set bits of `mask` below this lane
__device__ __forceinline__ uint32_t count_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// ------------------------------------------------------------------ step kernel
struct StepArgs {
    const uint32_t* world;
    WorldDims dims;
    int64_t n;
    int64_t env_base;  // multiple of 4 (a quad of envs shares its fuel / gate blocks)
    uint64_t seed;
    uint32_t t;
    se_state st;
    const int32_t* act;   // agent index (kTyped = false) or type (kTyped = true)
    const int32_t* act_a;
    const int32_t* act_b;
    se_tape* tape;           // replay: variates in, used flags out
    se_done_rec* done_recs;  // this step's done list: per-block segments of `seg` records
    int32_t* done_count;     // this step's per-block record counts
    int64_t seg;             // segment stride (records) of one workgroup
    int64_t iters;           // groups per thread (each workgroup owns iters * 256 groups)
    double* slab;            // per-block {sum_ret, n_eps, sum_len, pad}
};

// 4 consecutive elements: one 16-byte lane access (kFull) or guarded scalars (tail)
template <bool kFull, typename T>
__device__ __forceinline__ void ld4(const T* __restrict__ p, int64_t base, int64_t n, T& v0, T& v1,
                                    T& v2, T& v3) {
    if constexpr (kFull) {
        if constexpr (sizeof(T) == 4) {
            const uint4 w = *reinterpret_cast<const uint4*>(p + base);
            v0 = __builtin_bit_cast(T, w.x);
            v1 = __builtin_bit_cast(T, w.y);
            v2 = __builtin_bit_cast(T, w.z);
            v3 = __builtin_bit_cast(T, w.w);
        } else {
            const double2 a = *reinterpret_cast<const double2*>(p + base);
            const double2 b = *reinterpret_cast<const double2*>(p + base + 2);
            v0 = a.x;
            v1 = a.y;
            v2 = b.x;
            v3 = b.y;
        }
    } else {
        v0 = base + 0 < n ? p[base + 0] : T(0);
        v1 = base + 1 < n ? p[base + 1] : T(0);
        v2 = base + 2 < n ? p[base + 2] : T(0);
        v3 = base + 3 < n ? p[base + 3] : T(0);
    }
}

template <bool kFull, typename T>
__device__ __forceinline__ void st4(T* __restrict__ p, int64_t base, int64_t n, T v0, T v1, T v2,
                                    T v3) {
    if constexpr (kFull) {
        if constexpr (sizeof(T) == 4) {
            uint4 w;
            w.x = __builtin_bit_cast(uint32_t, v0);
            w.y = __builtin_bit_cast(uint32_t, v1);
            w.z = __builtin_bit_cast(uint32_t, v2);
            w.w = __builtin_bit_cast(uint32_t, v3);
            *reinterpret_cast<uint4*>(p + base) = w;
        } else {
            *reinterpret_cast<double2*>(p + base) = make_double2(v0, v1);
            *reinterpret_cast<double2*>(p + base + 2) = make_double2(v2, v3);
        }
    } else {
        if (base + 0 < n) p[base + 0] = v0;
        if (base + 1 < n) p[base + 1] = v1;
        if (base + 2 < n) p[base + 2] = v2;
        if (base + 3 < n) p[base + 3] = v3;
    }
}

// 4 u8 fields of consecutive envs as one packed word
template <bool kFull>
__device__ __forceinline__ uint32_t ld4u8(const uint8_t* __restrict__ p, int64_t base, int64_t n) {
    if constexpr (kFull) {
        return *reinterpret_cast<const uint32_t*>(p + base);
    } else {
        uint32_t w = 0;
        for (int j = 0; j < 4; ++j)
            if (base + j < n) w |= (uint32_t)p[base + j] << (8 * j);
        return w;
    }
}

template <bool kFull>
__device__ __forceinline__ void st4u8(uint8_t* __restrict__ p, int64_t base, int64_t n, uint32_t w) {
    if constexpr (kFull) {
        *reinterpret_cast<uint32_t*>(p + base) = w;
    } else {
        for (int j = 0; j < 4; ++j)
            if (base + j < n) p[base + j] = (uint8_t)(w >> (8 * j));
    }
}

__device__ __forceinline__ int byte_of(uint32_t w, int j) { return (int)((w >> (8 * j)) & 0xffu); }

// The inputs of 4 consecutive envs (one lane access per field when kFull).
template <bool kTyped, bool kAuto>
struct Group {
    uint32_t x, y, org, dst;  // packed u8 x4
    int32_t c0, c1, c2, c3;   // cargo
    double f0, f1, f2, f3;    // fuel
    int32_t a0, a1, a2, a3;   // agent index / action type
    int32_t p0, p1, p2, p3;   // typed: value a
    int32_t q0, q1, q2, q3;   // typed: value b
    float e0, e1, e2, e3;     // ep_return
    int32_t l0, l1, l2, l3;   // ep_len

    template <bool kFull>
    __device__ __forceinline__ void load(const StepArgs& A, int64_t base) {
        const se_state& S = A.st;
        x = ld4u8<kFull>(S.x, base, A.n);
        y = ld4u8<kFull>(S.y, base, A.n);
        org = ld4u8<kFull>(S.origin, base, A.n);
        dst = ld4u8<kFull>(S.dest, base, A.n);
        ld4<kFull>(S.cargo, base, A.n, c0, c1, c2, c3);
        ld4<kFull>(S.fuel, base, A.n, f0, f1, f2, f3);
        ld4<kFull>(A.act, base, A.n, a0, a1, a2, a3);
        if (kTyped) {
            ld4<kFull>(A.act_a, base, A.n, p0, p1, p2, p3);
            ld4<kFull>(A.act_b, base, A.n, q0, q1, q2, q3);
        }
        if (kAuto) {
            ld4<kFull>(S.ep_return, base, A.n, e0, e1, e2, e3);
            ld4<kFull>(S.ep_len, base, A.n, l0, l1, l2, l3);
        }
    }
};

struct BlockStats {
    double ret = 0.0, eps = 0.0, len = 0.0;
};

// 32-bit uniform in [0, 1): u = w * 2^-32 (exact in f64)
__device__ __forceinline__ double u32(uint32_t w) { return (double)w * (1.0 / 4294967296.0); }

// Step the 4 envs of one group (base = 4k). u_fuel / u_gate of env 4k+j are word j
// of the quad's FUEL / GATE Philox blocks; the GATE block is only drawn when some
// env of the group can observe its gate.
// Finished episodes of one group (auto-reset): bit j of `mask` for env base+j.
struct Finished {
    uint32_t mask = 0;
    float ret[4];
    int32_t len[4];
};

template <bool kTyped, bool kReplay, bool kAuto, bool kFull>
__device__ __forceinline__ void step_group(const StepArgs& A, const LdsWorld& w,
                                           Group<kTyped, kAuto>& G, int64_t base, BlockStats& bs,
                                           Finished& F) {
    const se_state& S = A.st;
    const int64_t n = A.n;
    int32_t act[4] = {G.a0, G.a1, G.a2, G.a3};
    int32_t pa[4] = {G.p0, G.p1, G.p2, G.p3};
    int32_t qb[4] = {G.q0, G.q1, G.q2, G.q3};
    int32_t cargo[4] = {G.c0, G.c1, G.c2, G.c3};
    double fuel[4] = {G.f0, G.f1, G.f2, G.f3};
    float epr[4] = {G.e0, G.e1, G.e2, G.e3};
    int32_t epl[4] = {G.l0, G.l1, G.l2, G.l3};

    // pass 1 (registers only): can any env of the group observe its gate draw?
    bool gate_needed = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        int ty, va, vb, er = SE_ERR_OK;
        if (kTyped) {
            ty = act[j];
            va = pa[j];
            vb = qb[j];
        } else {
            er = decode_agent(w.P, act[j], ty, va, vb);
        }
        const Ship s{byte_of(G.x, j), byte_of(G.y, j), 0.0, cargo[j], 0, byte_of(G.dst, j)};
        gate_needed |= er == SE_ERR_OK && needs_gate<!kTyped>(w, s, ty, va, vb);
    }

    double uf[4], ug[4];
    if constexpr (kReplay) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool in = kFull || base + j < n;
            uf[j] = in ? A.tape[base + j].u_fuel : 0.0;
            ug[j] = in ? A.tape[base + j].u_gate : 0.0;
        }
    } else {
        const int64_t quad = (A.env_base + base) >> 2;
        const Key qk = env_key(A.seed, quad);
#if SHIPENV_ABLATE == 1 || SHIPENV_ABLATE == 3  // timing-only builds: a trivial hash, no Philox
        const uint32_t h = (uint32_t)base * 0x9E3779B9u ^ A.t;
        const U4 fb = U4{{h, h * 3u, h ^ 0x55u, h + 7u}};
        const U4 gb = fb;
        (void)qk;
        (void)gate_needed;
#else
        const U4 fb = draw(qk, A.t, kSlotFuel);
        U4 gb = U4{{0u, 0u, 0u, 0u}};
        if (gate_needed) gb = draw(qk, A.t, kSlotGate);
#endif
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uf[j] = u32(fb.v[j]);
            ug[j] = u32(gb.v[j]);
        }
    }

    // pass 2: step the 4 envs (unrolled: measured ~5 % faster than a rolled loop
    // despite the higher register count, tools/ablate.sh)
    uint32_t ox = 0, oy = 0, oo = 0, od = 0, dn = 0, ee = 0, fin = 0;
    float rw[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t i = base + j;
        const bool live = kFull || i < n;
        Ship s{byte_of(G.x, j), byte_of(G.y, j), fuel[j], cargo[j], byte_of(G.org, j),
               byte_of(G.dst, j)};
        int ty, va, vb, e = SE_ERR_OK;
        if (kTyped) {
            ty = act[j];
            va = pa[j];
            vb = qb[j];
        } else {
            e = decode_agent(w.P, act[j], ty, va, vb);
        }
        double r = 0.0;
        int d = 0;
        const Key key = env_key(A.seed, A.env_base + i);
#if SHIPENV_ABLATE >= 2  // timing-only builds: no game logic (memory traffic kept)
        if (true) {
            s.x ^= ty & 1;
            s.fuel -= uf[j];
            r = ug[j] + (double)va + (double)vb;
        } else
#endif
        uint32_t used = 0;
        if constexpr (kReplay) {
            const Draws<true> dr{A.tape + (live ? i : 0)};
            e = env_step<false, true>(w, s, e, ty, va, vb, uf[j], ug[j], dr, r, d, used);
            if (live) A.tape[i].used = (int32_t)used;
        } else {
            const Draws<false> dr{key, A.t};
            e = env_step<!kTyped, false>(w, s, e, ty, va, vb, uf[j], ug[j], dr, r, d, used);
        }
        rw[j] = (float)r;  // one rounding of the reference's f64 reward
        if (kReplay && live && S.reward64) S.reward64[i] = r;
        if (kAuto && live) {
            epr[j] += rw[j];
            epl[j] += 1;
            if (d) {
                fin |= 1u << j;
                bs.ret += (double)epr[j];
                bs.eps += 1.0;
                bs.len += (double)epl[j];
                const U4 o = draw(key, A.t, kSlotReset);
                reset_ship(w, s, o.v[0], o.v[1]);
            }
        }
        fuel[j] = s.fuel;
        cargo[j] = s.cargo;
        const uint32_t sh = 8u * (uint32_t)j;
        ox |= (uint32_t)(s.x & 0xff) << sh;
        oy |= (uint32_t)(s.y & 0xff) << sh;
        oo |= (uint32_t)(s.origin & 0xff) << sh;
        od |= (uint32_t)(s.dest & 0xff) << sh;
        dn |= (uint32_t)d << sh;
        ee |= (uint32_t)(e & 0xff) << sh;
    }

    if constexpr (kAuto) {
        F.mask = fin;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            F.ret[j] = epr[j];
            F.len[j] = epl[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            epr[j] = ((fin >> j) & 1u) ? 0.0f : epr[j];
            epl[j] = ((fin >> j) & 1u) ? 0 : epl[j];
        }
        st4<kFull>(S.ep_return, base, n, epr[0], epr[1], epr[2], epr[3]);
        st4<kFull>(S.ep_len, base, n, epl[0], epl[1], epl[2], epl[3]);
    }
    st4u8<kFull>(S.x, base, n, ox);
    st4u8<kFull>(S.y, base, n, oy);
    st4u8<kFull>(S.origin, base, n, oo);
    st4u8<kFull>(S.dest, base, n, od);
    st4<kFull>(S.fuel, base, n, fuel[0], fuel[1], fuel[2], fuel[3]);
    st4<kFull>(S.cargo, base, n, cargo[0], cargo[1], cargo[2], cargo[3]);
    st4<kFull>(S.reward, base, n, rw[0], rw[1], rw[2], rw[3]);
    st4u8<kFull>(S.done, base, n, dn);
    st4u8<kFull>(reinterpret_cast<uint8_t*>(S.err), base, n, ee);
}

// Done-list compaction of one grid-stride iteration (auto-reset), no global
// atomics: a wave-exclusive prefix of the per-lane counts (0..4) from three
// ballots, a block prefix over the 4 wave totals in LDS, and the records go to
// this workgroup's own segment of the list in env order (deterministic).
// All threads of the block call it (it holds two barriers).
__device__ __forceinline__ void block_compact(const StepArgs& A, const Finished& F, int64_t base,
                                              int32_t* wtot, int32_t& running, bool last) {
    const int nd = __popc(F.mask);
    const uint64_t b0 = __ballot(nd & 1), b1 = __ballot(nd & 2), b2 = __ballot(nd & 4);
    const uint32_t wave_total = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) wtot[wave] = (int32_t)wave_total;
    if (!__syncthreads_or(nd)) return;  // nothing finished in the block: no second barrier
    int32_t before = 0, block_total = 0;
#pragma unroll
    for (int k = 0; k < kBlock / 64; ++k) {
        const int32_t v = wtot[k];
        before += k < wave ? v : 0;
        block_total += v;
    }
    if (nd) {
        int64_t slot = (int64_t)blockIdx.x * A.seg + running + before +
                       (int32_t)(count_below(b0) + 2 * count_below(b1) + 4 * count_below(b2));
        const int32_t t = (int32_t)A.t;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if ((F.mask >> j) & 1u) A.done_recs[slot++] = se_done_rec{(int32_t)(base + j), F.ret[j], F.len[j], t};
    }
    running += block_total;
    if (!last) __syncthreads();  // wtot is rewritten by the next iteration
}

// Workgroup b owns the contiguous groups [b*iters*256, (b+1)*iters*256) (a group is
// 4 consecutive envs, one thread per group per iteration), so its done-list
// segment follows env order and the concatenated segments are globally sorted.
// A full group's fields are single 4- or 16-byte lane accesses; the one partial
// group at the end (n % 4 envs) is stepped in place by its owner with guarded
// scalar accesses. The first group's loads are issued before the world is staged
// into LDS so the staging hides under them; each iteration loads the next group
// before storing the current one. The trip count is uniform over the block (the
// auto-reset compaction holds barriers).
template <bool kTyped, bool kReplay, bool kAuto>
__global__ __launch_bounds__(kBlock) void step_kernel(StepArgs A) {
    extern __shared__ uint32_t lds[];
    __shared__ double red[kBlock / 64][3];
    __shared__ int32_t wtot[kBlock / 64];
    const int64_t full = A.n >> 2, groups = (A.n + 3) >> 2;
    const int64_t first = (int64_t)blockIdx.x * A.iters * kBlock + threadIdx.x;

    Group<kTyped, kAuto> G;
    if (first < full) G.template load<true>(A, first * 4);
    const LdsWorld w = stage_world(A.world, A.dims, lds);

    BlockStats bs;
    int32_t running = 0;  // this block's done records so far (block-uniform)
    for (int64_t k = 0; k < A.iters; ++k) {
        const int64_t g = first + k * kBlock;
        Finished F;
        if (g < full) {
            step_group<kTyped, kReplay, kAuto, true>(A, w, G, g * 4, bs, F);
            if (k + 1 < A.iters && g + kBlock < full) G.template load<true>(A, (g + kBlock) * 4);
        } else if (g < groups) {  // the partial last group
            G.template load<false>(A, g * 4);
            step_group<kTyped, kReplay, kAuto, false>(A, w, G, g * 4, bs, F);
        }
        if constexpr (kAuto) block_compact(A, F, g * 4, wtot, running, k + 1 == A.iters);
    }

    if (kAuto) {
        if (threadIdx.x == 0) A.done_count[blockIdx.x] = running;
        // per-block statistics: fixed-order wave butterfly, then waves in order
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            bs.ret += __shfl_xor(bs.ret, off);
            bs.eps += __shfl_xor(bs.eps, off);
            bs.len += __shfl_xor(bs.len, off);
        }
        const int wave = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) {
            red[wave][0] = bs.ret;
            red[wave][1] = bs.eps;
            red[wave][2] = bs.len;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double a = 0.0, b = 0.0, c = 0.0;
            for (int k = 0; k < kBlock / 64; ++k) {
                a += red[k][0];
                b += red[k][1];
                c += red[k][2];
            }
            if (b != 0.0) {
                double* sl = A.slab + 4 * blockIdx.x;
                sl[0] += a;
                sl[1] += b;
                sl[2] += c;
            }
        }
    }
}

// Contiguous copy of the last step's per-block done lists (se_done_compact): block
// b sums the counts before it (grid <= 2048 entries) and copies its segment.
__global__ __launch_bounds__(kBlock) void done_compact_kernel(const se_done_rec* __restrict__ recs,
                                                              const int32_t* __restrict__ counts,
                                                              int64_t seg, se_done_rec* __restrict__ out,
                                                              int32_t* __restrict__ out_count) {
    __shared__ int32_t part[kBlock];
    int32_t acc = 0;
    for (int i = threadIdx.x; i < (int)blockIdx.x; i += kBlock) acc += counts[i];
    part[threadIdx.x] = acc;
    __syncthreads();
    for (int off = kBlock / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) part[threadIdx.x] += part[threadIdx.x + off];
        __syncthreads();
    }
    const int32_t start = part[0], cnt = counts[blockIdx.x];
    for (int i = threadIdx.x; i < cnt; i += kBlock) out[start + i] = recs[(int64_t)blockIdx.x * seg + i];
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *out_count = start + cnt;
}

// ------------------------------------------------------------------ reset kernel
struct ResetArgs {
    const uint32_t* world;
    WorldDims dims;
    int64_t n, env_base;
    uint64_t seed;
    uint32_t epoch;
    se_state st;
    const uint8_t* mask;
    const int32_t* origin_in;  // explicit values (se_reset_to) or NULL
    const int32_t* dest_in;
};

__global__ __launch_bounds__(kBlock) void reset_kernel(ResetArgs A) {
    extern __shared__ uint32_t lds[];
    const LdsWorld w = stage_world(A.world, A.dims, lds);
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < A.n;
         i += (int64_t)gridDim.x * kBlock) {
        if (A.mask && !A.mask[i]) continue;
        Ship s;
        if (A.origin_in) {
            s.origin = A.origin_in[i];
            s.dest = A.dest_in[i];
            s.cargo = 0;
            s.fuel = kFuelInit;
            s.x = w.px(s.origin);
            s.y = w.py(s.origin);
        } else {
            const U4 o = draw(env_key(A.seed, A.env_base + i), A.epoch, kSlotExplicitReset);
            reset_ship(w, s, o.v[0], o.v[1]);
        }
        A.st.x[i] = (uint8_t)s.x;
        A.st.y[i] = (uint8_t)s.y;
        A.st.fuel[i] = s.fuel;
        A.st.cargo[i] = s.cargo;
        A.st.origin[i] = (uint8_t)s.origin;
        A.st.dest[i] = (uint8_t)s.dest;
        if (A.st.ep_return) A.st.ep_return[i] = 0.0f;
        if (A.st.ep_len) A.st.ep_len[i] = 0;
        A.st.done[i] = 0;
        A.st.err[i] = 0;
        A.st.reward[i] = 0.0f;
    }
}

// ------------------------------------------------------------------ observation
// preprocess_state rows (utils/preprocessing.py:25-62): one thread per output
// element so the f32 row writes are coalesced; the port block comes from LDS.
struct ObsArgs {
    const uint32_t* world;
    WorldDims dims;
    int64_t n, ld;
    se_state st;
    float* obs;
};

__global__ __launch_bounds__(kBlock) void observe_kernel(ObsArgs A) {
    extern __shared__ uint32_t lds[];
    const LdsWorld w = stage_world(A.world, A.dims, lds);
    const int64_t width = 6 + 4 * (int64_t)w.P;
    const int64_t total = A.n * width;
    for (int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * kBlock) {
        const int64_t i = k / width;
        const int c = (int)(k - i * width);
        float v;
        if (c < 6) {
            switch (c) {
            case 0: v = (float)A.st.x[i]; break;
            case 1: v = (float)A.st.y[i]; break;
            case 2:
            case 3: v = (float)A.st.fuel[i]; break;  // "cargo" is self.fuel (environment.py:206)
            case 4: v = A.st.origin[i] == SE_NONE ? -1.0f : (float)A.st.origin[i]; break;
            default: v = A.st.dest[i] == SE_NONE ? -1.0f : (float)A.st.dest[i]; break;
            }
        } else {
            const int p = (c - 6) >> 2, f = (c - 6) & 3;
            v = f == 0 ? (float)w.px(p) : f == 1 ? (float)w.py(p) : f == 2 ? (float)w.pfuel[p] : (float)w.pcargo[p];
        }
        A.obs[i * A.ld + c] = v;
    }
}

// ------------------------------------------------------------------ DQN validity mask
// agents/dqn.py:125-175, one thread per output byte (8 agent indices).
struct MaskArgs {
    const uint32_t* world;
    WorldDims dims;
    int64_t n;
    int32_t stride;
    se_state st;
    uint8_t* bits;
};

__global__ __launch_bounds__(kBlock) void valid_mask_kernel(MaskArgs A) {
    extern __shared__ uint32_t lds[];
    const LdsWorld w = stage_world(A.world, A.dims, lds);
    const int P = w.P, nact = 4 + P + 250;
    const int64_t total = A.n * A.stride;
    for (int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * kBlock) {
        const int64_t i = k / A.stride;
        const int byte = (int)(k - i * A.stride);
        const int x = A.st.x[i], y = A.st.y[i];
        const int origin = A.st.origin[i] == SE_NONE ? -1 : A.st.origin[i];
        const int cur = w.port_at(x, y);
        uint32_t out = 0;
        for (int bit = 0; bit < 8; ++bit) {
            const int a = byte * 8 + bit;
            bool v;
            if (a >= nact) v = false;
            else if (a < 4) v = true;
            else if (a < 4 + P) {
                const int p = a - 4;
                v = p != origin && w.px(p) == x && w.py(p) == y;
            } else if (a < 4 + P + 50) {
                const int amt = a - (4 + P);
                v = cur >= 0 && amt > 0 && amt <= w.pcargo[cur];
            } else {
                const int amt = a - (4 + P + 50);
                v = cur >= 0 && amt > 0 && amt <= w.pfuel[cur];
            }
            out |= (uint32_t)v << (7 - bit);
        }
        A.bits[k] = (uint8_t)out;
    }
}

// ------------------------------------------------------------------ synthetic agent
__global__ __launch_bounds__(kBlock) void gen_actions_kernel(int64_t n, int64_t env_base,
                                                             uint64_t seed, uint32_t t, int32_t P,
                                                             int32_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kBlock) {
        const U4 o = draw(env_key(seed, env_base + i), t, kSlotAction);
        const int32_t c = uniform_int(o.v[0], 100);
        int32_t a;
        if (c < 90) a = (int32_t)(o.v[1] & 3u);
        else if (c < 95) a = 4 + P + 1 + uniform_int(o.v[1], 20);
        else if (c < 98) a = 4 + P + 50 + 1 + uniform_int(o.v[1], 20);
        else a = 4 + uniform_int(o.v[2], (uint32_t)P);
        out[i] = a;
    }
}

// ------------------------------------------------------------------ stats reduce
__global__ __launch_bounds__(64) void stats_kernel(const double* __restrict__ slab, int blocks,
                                                   double* __restrict__ out) {
    double a = 0.0, b = 0.0, c = 0.0;
    for (int i = threadIdx.x; i < blocks; i += 64) {
        a += slab[4 * i];
        b += slab[4 * i + 1];
        c += slab[4 * i + 2];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_xor(a, off);
        b += __shfl_xor(b, off);
        c += __shfl_xor(c, off);
    }
    if (threadIdx.x == 0) {
        out[0] = a;
        out[1] = b;
        out[2] = c;
    }
}

}  // namespace

// ====================================================================== host side
struct se_env {
    int device = 0;
    int64_t n = 0, env_base = 0;
    WorldDims dims{};
    uint64_t seed = 0;
    uint32_t flags = 0;
    uint64_t step_t = 0, epoch = 0;
    std::vector<uint8_t> water;  // H*W, 0 = ground
    uint32_t* d_world = nullptr;
    int64_t seg = 0;    // done-list segment stride (records per workgroup)
    int64_t iters = 1;  // groups per thread of the step kernel
    int world_cap = 0;  // words allocated
    se_state st{};
    bool bound = false;
    double* d_slab = nullptr;       // [grid][4]
    int grid = 0;
};

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail(SE_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));        \
    } while (0)

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

int grid_for(int64_t items, int cap = kMaxBlocks) {
    int64_t b = (items + kBlock - 1) / kBlock;
    if (b < 1) b = 1;
    if (b > cap) b = cap;
    return (int)b;
}

// Workgroup cap of the step kernel: each thread then walks ceil(groups / (cap*256))
// groups with the next group's loads in flight while it computes the current one.
int step_block_cap() {
    const char* v = getenv("SHIPENV_STEP_BLOCKS");
    const int c = v ? atoi(v) : 0;
    return c > 0 ? c : kStepBlocks;
}

size_t lds_bytes(const se_env* env) { return (size_t)env->dims.total() * 4; }

int upload_world(se_env* env, int32_t P, const int32_t* px, const int32_t* py, const int32_t* pf,
                 const int32_t* pc) {
    if (P < 0 || P > SE_MAX_PORTS) return fail(SE_EINVAL, "P must be in [0, 254]");
    const int H = env->dims.H, W = env->dims.W;
    for (int i = 0; i < P; ++i) {
        if (px[i] < 0 || px[i] >= H || py[i] < 0 || py[i] >= W)
            return fail(SE_EINVAL, "Coordinates not within map");  // add_port, environment.py:59-60
        if (pf[i] < 0 || pc[i] < 0) return fail(SE_EINVAL, "port stocks must be >= 0");
    }
    const int words = (H * W + 31) / 32;
    WorldDims d{H, W, P, words};
    std::vector<uint32_t> img((size_t)d.total(), 0u);
    std::vector<uint8_t> nonground(env->water);
    for (int i = 0; i < P; ++i) nonground[(size_t)px[i] * W + py[i]] = 1;  // Entity.PORT (:65)
    for (int c = 0; c < H * W; ++c)
        if (!nonground[c]) img[c >> 5] |= 1u << (c & 31);
    for (int i = 0; i < P; ++i) {
        const int c = px[i] * W + py[i];
        img[words + (c >> 5)] |= 1u << (c & 31);
        img[d.pos() + i] = (uint32_t)px[i] | ((uint32_t)py[i] << 8);
        img[d.pos() + P + i] = (uint32_t)pf[i];
        img[d.pos() + 2 * P + i] = (uint32_t)pc[i];
    }
    uint32_t run = 0;
    for (int k = 0; k < words; ++k) {
        img[2 * words + k] = run;
        run += (uint32_t)__builtin_popcount(img[words + k]);
    }
    // rank -> first port (in port order) on that cell
    for (int i = P - 1; i >= 0; --i) {
        const uint32_t c = (uint32_t)(px[i] * W + py[i]);
        const uint32_t word = img[words + (c >> 5)];
        const uint32_t rank = img[2 * words + (c >> 5)] + (uint32_t)__builtin_popcount(word & ((1u << (c & 31)) - 1u));
        img[d.rank2port() + rank] = (uint32_t)i;
    }
    // normalize(cargo, 50, 0) = cargo / 50 (util.py:6-8): Python's int / int true
    // division is the correctly rounded quotient, which IEEE f64 division gives here.
    for (int c = 0; c < 50; ++c) {
        const double q = (double)c / kMaxCargo;
        memcpy(&img[d.frac() + 2 * c], &q, sizeof q);
    }
    if (d.total() > env->world_cap) {
        if (env->d_world) HIP_TRY(hipFree(env->d_world));
        env->d_world = nullptr;
        HIP_TRY(hipMalloc(&env->d_world, (size_t)d.total() * 4));
        env->world_cap = d.total();
    }
    HIP_TRY(hipMemcpy(env->d_world, img.data(), (size_t)d.total() * 4, hipMemcpyHostToDevice));
    env->dims = d;
    return SE_OK;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

int check_ready(se_env* env) {
    if (!env) return fail(SE_EINVAL, "null env");
    if (!env->bound) return fail(SE_ESTATE, "se_bind has not been called");
    return SE_OK;
}

int launch_step(se_env* env, bool typed, bool replay, const int32_t* act, const int32_t* a,
                const int32_t* b, se_tape* tape, void* stream) {
    int rc = check_ready(env);
    if (rc) return rc;
    if (!act || (typed && (!a || !b)) || (replay && !tape))
        return fail(SE_EINVAL, "null action/tape pointer");
    if (!aligned16(act) || (typed && (!aligned16(a) || !aligned16(b))))
        return fail(SE_EINVAL, "action buffers must be 16-byte aligned");
    const bool autoreset = (env->flags & SE_FLAG_AUTO_RESET) && !replay;
    if (autoreset && env->dims.P < 2) return fail(SE_EINVAL, "auto-reset needs at least two ports");
    DeviceGuard g(env->device);
    StepArgs A{};
    A.world = env->d_world;
    A.dims = env->dims;
    A.n = env->n;
    A.env_base = env->env_base;
    A.seed = env->seed;
    A.t = (uint32_t)env->step_t;
    A.st = env->st;
    A.act = act;
    A.act_a = a;
    A.act_b = b;
    A.tape = tape;
    // done lists double-buffered by step parity: the list of step t-1 stays
    // readable while step t runs; every block rewrites its own count each step.
    if (autoreset) {
        const size_t par = (size_t)(env->step_t & 1u);
        A.done_recs = env->st.done_recs + par * (size_t)env->grid * (size_t)env->seg;
        A.done_count = env->st.done_count + par * (size_t)env->grid;
    }
    A.seg = env->seg;
    A.iters = env->iters;
    A.slab = env->d_slab;
    const hipStream_t s = (hipStream_t)stream;
    const size_t lds = lds_bytes(env);
    const int grid = env->grid;
    if (env->n > 0) {
        if (!typed && !autoreset) step_kernel<false, false, false><<<grid, kBlock, lds, s>>>(A);
        else if (!typed && autoreset) step_kernel<false, false, true><<<grid, kBlock, lds, s>>>(A);
        else if (typed && replay) step_kernel<true, true, false><<<grid, kBlock, lds, s>>>(A);
        else if (typed && !autoreset) step_kernel<true, false, false><<<grid, kBlock, lds, s>>>(A);
        else step_kernel<true, false, true><<<grid, kBlock, lds, s>>>(A);
        HIP_TRY(hipGetLastError());
    }
    if (!replay) env->step_t += 1;
    return SE_OK;
}

}  // namespace

extern "C" {

int se_abi_version(void) { return SHIPENV_ABI_VERSION; }

const char* se_last_error(void) { return g_err.c_str(); }

int se_create(se_env** out, int device, int64_t n, int64_t env_id_base, int32_t H, int32_t W,
              const uint8_t* water, int32_t P, const int32_t* port_x, const int32_t* port_y,
              const int32_t* port_fuel, const int32_t* port_cargo, uint64_t seed, uint32_t flags) {
    if (!out) return fail(SE_EINVAL, "null out");
    *out = nullptr;
    if (n < 0) return fail(SE_EINVAL, "n must be >= 0");
    if (env_id_base < 0 || (env_id_base & 3))
        return fail(SE_EINVAL, "env_id_base must be a multiple of 4 (envs 4k..4k+3 share draw blocks)");
    if (H < 1 || W < 1 || H > SE_MAX_SIDE || W > SE_MAX_SIDE)
        return fail(SE_EINVAL, "map sides must be in [1, 256]");
    if (!water) return fail(SE_EINVAL, "null water map");
    if (P > 0 && (!port_x || !port_y || !port_fuel || !port_cargo))
        return fail(SE_EINVAL, "null port arrays");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(SE_EINVAL, "bad device ordinal");
    DeviceGuard g(device);
    se_env* env = new se_env();
    env->device = device;
    env->n = n;
    env->env_base = env_id_base;
    env->seed = seed;
    env->flags = flags;
    env->dims.H = H;
    env->dims.W = W;
    env->water.assign(water, water + (size_t)H * W);
    for (auto& v : env->water) v = v ? 1 : 0;
    int rc = upload_world(env, P, port_x, port_y, port_fuel, port_cargo);
    if (rc) {
        se_destroy(env);
        return rc;
    }
    {
        // workgroup b owns iters * 256 consecutive groups of 4 envs
        const int64_t groups = (n + kEnvsPerThread - 1) / kEnvsPerThread;
        const int64_t cap = step_block_cap();
        env->iters = groups > 0 ? (groups + cap * kBlock - 1) / (cap * kBlock) : 1;
        env->grid = (int)(groups > 0 ? (groups + env->iters * kBlock - 1) / (env->iters * kBlock) : 1);
        env->seg = env->iters * kBlock * kEnvsPerThread;
    }
    hipError_t e = hipMalloc(&env->d_slab, (size_t)env->grid * 4 * sizeof(double));
    if (e == hipSuccess) e = hipMemset(env->d_slab, 0, (size_t)env->grid * 4 * sizeof(double));
    if (e != hipSuccess) {
        se_destroy(env);
        return fail(SE_EHIP, std::string("se_create allocation: ") + hipGetErrorString(e));
    }
    *out = env;
    return SE_OK;
}

int se_set_ports(se_env* env, int32_t P, const int32_t* port_x, const int32_t* port_y,
                 const int32_t* port_fuel, const int32_t* port_cargo) {
    if (!env) return fail(SE_EINVAL, "null env");
    if (P > 0 && (!port_x || !port_y || !port_fuel || !port_cargo))
        return fail(SE_EINVAL, "null port arrays");
    DeviceGuard g(env->device);
    HIP_TRY(hipDeviceSynchronize());  // the old image may still be read by queued work
    return upload_world(env, P, port_x, port_y, port_fuel, port_cargo);
}

int se_bind(se_env* env, const se_state* st) {
    if (!env || !st) return fail(SE_EINVAL, "null argument");
    const void* req[] = {st->x, st->y, st->fuel, st->cargo, st->origin, st->dest,
                         st->reward, st->done, st->err};
    for (const void* p : req) {
        if (!p && env->n > 0) return fail(SE_EINVAL, "null state buffer");
        if (!aligned16(p)) return fail(SE_EINVAL, "state buffers must be 16-byte aligned");
    }
    if (env->flags & SE_FLAG_AUTO_RESET) {
        if (!st->ep_return || !st->ep_len || !st->done_recs || !st->done_count)
            return fail(SE_EINVAL, "auto-reset needs ep_return, ep_len, done_recs and done_count");
        if (!aligned16(st->ep_return) || !aligned16(st->ep_len) || !aligned16(st->done_recs))
            return fail(SE_EINVAL, "state buffers must be 16-byte aligned");
        DeviceGuard g(env->device);
        HIP_TRY(hipMemset(st->done_count, 0, 2 * (size_t)env->grid * sizeof(int32_t)));
    }
    env->st = *st;
    env->bound = true;
    return SE_OK;
}

int se_reset(se_env* env, const uint8_t* mask, void* stream) {
    int rc = check_ready(env);
    if (rc) return rc;
    if (env->dims.P < 2) return fail(SE_EINVAL, "reset needs at least two ports");
    DeviceGuard g(env->device);
    ResetArgs A{env->d_world, env->dims, env->n, env->env_base, env->seed,
                (uint32_t)env->epoch, env->st, mask, nullptr, nullptr};
    if (env->n > 0) {
        reset_kernel<<<grid_for(env->n), kBlock, lds_bytes(env), (hipStream_t)stream>>>(A);
        HIP_TRY(hipGetLastError());
    }
    env->epoch += 1;
    return SE_OK;
}

int se_reset_to(se_env* env, const uint8_t* mask, const int32_t* origin, const int32_t* dest,
                void* stream) {
    int rc = check_ready(env);
    if (rc) return rc;
    if (!origin || !dest) return fail(SE_EINVAL, "null origin/dest");
    DeviceGuard g(env->device);
    ResetArgs A{env->d_world, env->dims, env->n, env->env_base, env->seed,
                (uint32_t)env->epoch, env->st, mask, origin, dest};
    if (env->n > 0) {
        reset_kernel<<<grid_for(env->n), kBlock, lds_bytes(env), (hipStream_t)stream>>>(A);
        HIP_TRY(hipGetLastError());
    }
    return SE_OK;
}

int se_step(se_env* env, const int32_t* actions, void* stream) {
    return launch_step(env, false, false, actions, nullptr, nullptr, nullptr, stream);
}

int se_step_typed(se_env* env, const int32_t* type, const int32_t* a, const int32_t* b,
                  void* stream) {
    return launch_step(env, true, false, type, a, b, nullptr, stream);
}

int se_step_replay(se_env* env, const int32_t* type, const int32_t* a, const int32_t* b,
                   se_tape* tape, void* stream) {
    return launch_step(env, true, true, type, a, b, tape, stream);
}

int se_observe(se_env* env, float* obs, int64_t ld, void* stream) {
    int rc = check_ready(env);
    if (rc) return rc;
    if (!obs || ld < 6 + 4 * (int64_t)env->dims.P) return fail(SE_EINVAL, "bad obs buffer / ld");
    DeviceGuard g(env->device);
    ObsArgs A{env->d_world, env->dims, env->n, ld, env->st, obs};
    const int64_t total = env->n * (6 + 4 * (int64_t)env->dims.P);
    if (total > 0) {
        observe_kernel<<<grid_for(total), kBlock, lds_bytes(env), (hipStream_t)stream>>>(A);
        HIP_TRY(hipGetLastError());
    }
    return SE_OK;
}

int se_valid_mask(se_env* env, uint8_t* bits, void* stream) {
    int rc = check_ready(env);
    if (rc) return rc;
    if (!bits) return fail(SE_EINVAL, "null bits");
    DeviceGuard g(env->device);
    const int32_t stride = (4 + env->dims.P + 250 + 7) / 8;
    MaskArgs A{env->d_world, env->dims, env->n, stride, env->st, bits};
    const int64_t total = env->n * stride;
    if (total > 0) {
        valid_mask_kernel<<<grid_for(total), kBlock, lds_bytes(env), (hipStream_t)stream>>>(A);
        HIP_TRY(hipGetLastError());
    }
    return SE_OK;
}

int se_gen_actions(se_env* env, int32_t* actions, uint32_t t, void* stream) {
    if (!env || !actions) return fail(SE_EINVAL, "null argument");
    if (!aligned16(actions)) return fail(SE_EINVAL, "actions must be 16-byte aligned");
    if (env->dims.P < 1) return fail(SE_EINVAL, "the synthetic agent needs ports");
    DeviceGuard g(env->device);
    if (env->n > 0) {
        gen_actions_kernel<<<grid_for(env->n), kBlock, 0, (hipStream_t)stream>>>(
            env->n, env->env_base, env->seed, t, env->dims.P, actions);
        HIP_TRY(hipGetLastError());
    }
    return SE_OK;
}

int se_episode_stats(se_env* env, double* out, void* stream) {
    if (!env || !out) return fail(SE_EINVAL, "null argument");
    DeviceGuard g(env->device);
    stats_kernel<<<1, 64, 0, (hipStream_t)stream>>>(env->d_slab, env->grid, out);
    HIP_TRY(hipGetLastError());
    return SE_OK;
}

int se_clear_stats(se_env* env, void* stream) {
    if (!env) return fail(SE_EINVAL, "null env");
    DeviceGuard g(env->device);
    HIP_TRY(hipMemsetAsync(env->d_slab, 0, (size_t)env->grid * 4 * sizeof(double),
                           (hipStream_t)stream));
    return SE_OK;
}

int se_done_layout(se_env* env, int64_t* seg_stride, int32_t* segments) {
    if (!env) return fail(SE_EINVAL, "null env");
    if (seg_stride) *seg_stride = env->seg;
    if (segments) *segments = env->grid;
    return SE_OK;
}

int se_done_list(se_env* env, int64_t* rec_offset, int64_t* count_offset) {
    if (!env || !rec_offset || !count_offset) return fail(SE_EINVAL, "null argument");
    if (!(env->flags & SE_FLAG_AUTO_RESET)) return fail(SE_ESTATE, "no done list without auto-reset");
    if (env->step_t == 0) return fail(SE_ESTATE, "no step has run");
    const int64_t par = (int64_t)((env->step_t - 1) & 1u);
    *rec_offset = par * (int64_t)env->grid * env->seg;
    *count_offset = par * (int64_t)env->grid;
    return SE_OK;
}

int se_done_compact(se_env* env, se_done_rec* out, int32_t* out_count, void* stream) {
    int64_t ro = 0, co = 0;
    int rc = se_done_list(env, &ro, &co);
    if (rc) return rc;
    if (!out || !out_count) return fail(SE_EINVAL, "null output");
    DeviceGuard g(env->device);
    done_compact_kernel<<<env->grid, kBlock, 0, (hipStream_t)stream>>>(
        env->st.done_recs + ro, env->st.done_count + co, env->seg, out, out_count);
    HIP_TRY(hipGetLastError());
    return SE_OK;
}

int se_get_counters(se_env* env, uint64_t* step, uint64_t* epoch) {
    if (!env) return fail(SE_EINVAL, "null env");
    if (step) *step = env->step_t;
    if (epoch) *epoch = env->epoch;
    return SE_OK;
}

int se_set_counters(se_env* env, uint64_t step, uint64_t epoch) {
    if (!env) return fail(SE_EINVAL, "null env");
    DeviceGuard g(env->device);
    HIP_TRY(hipDeviceSynchronize());
    if (env->bound && env->st.done_count)
        HIP_TRY(hipMemset(env->st.done_count, 0, 2 * (size_t)env->grid * sizeof(int32_t)));
    env->step_t = step;
    env->epoch = epoch;
    return SE_OK;
}

int se_destroy(se_env* env) {
    if (!env) return SE_OK;
    DeviceGuard g(env->device);
    if (env->d_world) (void)hipFree(env->d_world);
    if (env->d_slab) (void)hipFree(env->d_slab);
    delete env;
    return SE_OK;
}

}  // extern "C"
