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
//   * auto-reset compacts finished envs into a done list with a wave ballot
//     prefix into per-(iteration, wave) segments (no atomics, no barrier), and
//     reduces episode statistics per wave into a fixed slab (deterministic sums,
//     no float atomics).
//
// Built with -ffp-contract=off: the reference's f64 arithmetic (CPython float,
// np.sqrt) is unfused, and an FMA in -0.1 + 0.2*u changes fuel bits.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <vector>

#include "../../include/shipenv.h"
#include "philox.h"

#ifndef SHIPENV_TRACE
#define SHIPENV_TRACE 0  // 1 = diagnostic build: per-wave phase timestamps (tools/archive/wave_trace.py)
#endif

using namespace shipenv;

namespace {

constexpr int kBlock = 256;       // 4 waves
constexpr int kStepBlock = 256;  // step kernel workgroup (one LDS world copy each)
constexpr int kEnvsPerThread = 4; // one 4-byte / 16-byte lane access per field
constexpr int kMaxBlocks = 2048;  // 256 CUs x 8; grid-stride beyond
// step kernel default workgroup cap (SHIPENV_STEP_BLOCKS overrides): one group of 4 envs per
// thread up to 2^25 envs. Measured against 2048 (iters = 8 at 2^24; tools/archive/blk_sweep.sh,
// profiles/r02h/blk_sweep): 2^24 129 -> 123 us, 2^25 293 -> 253 us, config 4 at 2^24
// 200 -> 182 us; 2^20 (grid 1024 either way) unchanged
constexpr int kStepBlocks = 32768;

// se_tape.used bits (replay): which of the reference's draws this step consumed
constexpr uint32_t kUsedFuelGate = SE_USED_FUEL_GATE, kUsedLossType = SE_USED_LOSS_TYPE,
                   kUsedBeta = SE_USED_BETA, kUsedArrive = SE_USED_ARRIVE, kUsedMoved = SE_USED_MOVED;

// reference constants, shipping/environment.py:8-26
constexpr double kFuelInit = 200.0;
constexpr double kMaxCargo = 50.0;

// ------------------------------------------------------------------ world image
// One device buffer of 32-bit words, staged as-is into LDS by every workgroup:
//   [0, cw)         cell codes, one byte per cell c = x * W + y (x = map row, :65,
//                   :293): 0 water, kCellGround ground (np_game[x, y] == GROUND),
//                   k + 1 the FIRST port k on the cell (a port is never ground, :65;
//                   _get_current_port_idx returns the first match, :150-152).
//                   cw = H*W bytes rounded up to whole 16-byte units
//   [pos, +P)       port position  x | y << 16 (the packed form of a ship position)
//   [stk, +2P)      port stocks, (fuel, cargo) per port (8-byte aligned pairs)
//   [gate, +51)     u32 table floor(fl(c / 50) * 2^32) for c in [0, 50), and
//                   0xffffffff at 50: the gate on a Philox word (cargo >= 50 fires)
//   [frac, +100)    f64 table fl(c / 50) for c in [0, 50) (8-byte aligned; replay)
//   [rtab, +20)     f64 step rewards before cargo loss / arrival (8-byte aligned):
//                   [0, 8) a move, index out_of_fuel*4 + ground*2 + closer, summed in
//                   the reference's order (:288-315); [8] a take (0.05); [9] else 0
//   [moves, +4)     packed (dx, dy) of N, E, S, W (utils/preprocessing.py:126) as two
//                   16-bit halves: v_pk_add_u16 moves a packed position
// For the 100x100 map with 5 ports that is 10.8 KB: one byte lookup answers both
// "is the target cell ground" (:293) and "which port is the ship on" (:145-153),
// where bitmaps took a word read, bit arithmetic and a 3-read rank chain.
constexpr int kCellGround = 255;
// kStepBlock x 4-dword rows of the world image the step kernel stages unguarded
// (one 16-byte load per thread and row), at least 12 KB: the 100x100 image with up
// to 130 ports
constexpr int kStageRows = (3072 + 4 * kStepBlock - 1) / (4 * kStepBlock);
constexpr int kStageWords = kStageRows * 4 * kStepBlock;

struct WorldDims {
    int32_t H, W, P, cw;  // cw: words of cell codes (a multiple of 4)
    __host__ __device__ int pos() const { return cw; }
    __host__ __device__ int stk() const { return (pos() + P + 1) & ~1; }
    __host__ __device__ int gate() const { return stk() + 2 * P; }
    __host__ __device__ int frac() const { return (gate() + 51 + 1) & ~1; }
    __host__ __device__ int rtab() const { return frac() + 2 * 50; }
    __host__ __device__ int moves() const { return rtab() + 2 * 10; }
    __host__ __device__ int total() const { return moves() + 4; }
    // device image / LDS size: whole 1024-dword rows, at least the step kernel's
    // unguarded staging window
    __host__ __device__ int padded() const {
        const int t = (total() + 1023) / 1024 * 1024;
        return t > kStageWords ? t : kStageWords;
    }
};

// The per-env step core (env_begin / env_finish, the replayed step) is compiled for the
// host too: se_host_step_replay steps host-resident envs with the same source (the N = 1
// drop-in). The two helpers below are the only operations that differ between the
// targets; both are exact for the operand ranges used (< 2^24, correctly rounded sqrt).
__host__ __device__ inline uint32_t mul24u(uint32_t a, uint32_t b) {
#ifdef __HIP_DEVICE_COMPILE__
    return __umul24(a, b);
#else
    return a * b;
#endif
}
__host__ __device__ inline int mul24i(int a, int b) {
#ifdef __HIP_DEVICE_COMPILE__
    return __mul24(a, b);
#else
    return a * b;
#endif
}
// IEEE square root, correctly rounded on both targets (np.sqrt, shipping/util.py:4)
__host__ __device__ inline double sqrt_rn(double v) {
#ifdef __HIP_DEVICE_COMPILE__
    return __dsqrt_rn(v);
#else
    return sqrt(v);
#endif
}

struct LdsWorld {
    const uint8_t* cell;
    const uint32_t* pos;
    const int2* stock;
    const uint32_t* gate_thr;
    const double* frac;
    const double* rtab;
    const uint32_t* moves;
    int32_t H, W, P;

    // cell index x * W + y: coordinates and W are below 256, so 24-bit multiplies
    // (full rate) are exact where a 32-bit one would be a 64-bit-product op
    __host__ __device__ int code(int x, int y) const { return cell[mul24u((uint32_t)x, (uint32_t)W) + (uint32_t)y]; }
    __host__ __device__ bool is_ground(int x, int y) const { return code(x, y) == kCellGround; }
    // _get_current_port_idx (:145-153): first port on the ship's cell, -1 if none
    // (water 0 -> -1, ground 255 -> 254 >= P)
    __host__ __device__ int port_at(int x, int y) const { return port_of_code(code(x, y)); }
    __host__ __device__ int port_of_code(int c) const {
        const int k = c - 1;
        return (unsigned)k < (unsigned)P ? k : -1;
    }
    __host__ __device__ int px(int i) const { return (int)(pos[i] & 0xffffu); }
    __host__ __device__ int py(int i) const { return (int)(pos[i] >> 16); }
    __host__ __device__ int pfuel(int i) const { return stock[i].x; }
    __host__ __device__ int pcargo(int i) const { return stock[i].y; }
    // normalize(cargo, 50, 0) (util.py:6-8), only read for 0 < cargo < 50
    __host__ __device__ double likelihood(int cargo) const { return frac[cargo]; }
};

__host__ __device__ inline LdsWorld world_view(WorldDims d, const uint32_t* img) {
    LdsWorld w;
    w.cell = reinterpret_cast<const uint8_t*>(img);
    w.pos = img + d.pos();
    w.stock = reinterpret_cast<const int2*>(img + d.stk());
    w.gate_thr = img + d.gate();
    w.frac = reinterpret_cast<const double*>(img + d.frac());
    w.rtab = reinterpret_cast<const double*>(img + d.rtab());
    w.moves = img + d.moves();
    w.H = d.H;
    w.W = d.W;
    w.P = d.P;
    return w;
}

// Staging in two halves. stage_issue puts every thread's share of the image in
// flight at once (independent 16-byte loads into registers); stage_finish writes it
// to LDS and holds the barrier. A load -> wait -> ds_write loop would make each
// round a full L2 round trip behind whatever the wave loaded before it (its
// s_waitcnt vmcnt(0) also waits for those). The step kernel issues its first
// group's loads between the halves, so the image (first in the in-order vmcnt
// queue) is written while the group's data is still on its way.
struct Staged {
    uint4 r[kStageRows];
};

// The step kernel's half (kStepBlock threads): the image is padded to at least
// kStageWords (WorldDims::padded), so these loads need no guard and no branch.
__device__ __forceinline__ Staged stage_issue(const uint32_t* __restrict__ g) {
    Staged st;
    const uint4* g4 = reinterpret_cast<const uint4*>(g);
#pragma unroll
    for (int k = 0; k < kStageRows; ++k) st.r[k] = g4[threadIdx.x + kStepBlock * k];
    return st;
}

__device__ __forceinline__ void stage_write(const uint32_t* __restrict__ g, WorldDims d, uint32_t* lds,
                                            const Staged& st) {
    uint4* l4 = reinterpret_cast<uint4*>(lds);
#pragma unroll
    for (int k = 0; k < kStageRows; ++k) l4[threadIdx.x + kStepBlock * k] = st.r[k];
    for (int i = (int)threadIdx.x + kStepBlock * kStageRows; i < (d.total() + 3) / 4; i += kStepBlock)
        l4[i] = reinterpret_cast<const uint4*>(g)[i];  // larger maps / port tables: the remainder
}
__device__ __forceinline__ LdsWorld stage_finish(const uint32_t* __restrict__ g, WorldDims d,
                                                 uint32_t* lds, const Staged& st) {
    stage_write(g, d, lds, st);
    __syncthreads();
    return world_view(d, lds);
}

// Any block size (the other kernels): every thread's 16-byte loads issued before any
// store (the image is padded to whole 1024-dword rows).
__device__ __forceinline__ LdsWorld stage_world(const uint32_t* __restrict__ g, WorldDims d,
                                                uint32_t* lds) {
    const int total = (d.total() + 3) / 4;
    const uint4* g4 = reinterpret_cast<const uint4*>(g);
    uint4* l4 = reinterpret_cast<uint4*>(lds);
    constexpr int kR = 4;
    for (int i0 = 0; i0 < total; i0 += kR * (int)blockDim.x) {
        // unconditional loads (past the end: the last word again), so r stays in VGPRs: a
        // conditionally assigned array was placed in scratch
        uint4 r[kR];
#pragma unroll
        for (int k = 0; k < kR; ++k) r[k] = g4[min(i0 + (int)threadIdx.x + k * (int)blockDim.x, total - 1)];
#pragma unroll
        for (int k = 0; k < kR; ++k) {
            const int i = i0 + (int)threadIdx.x + k * (int)blockDim.x;
            if (i < total) l4[i] = r[k];
        }
    }
    __syncthreads();
    return world_view(d, lds);
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

// 32-bit uniform in [0, 1): u = w * 2^-32 (exact in f64)
__device__ __forceinline__ double u32(uint32_t w) { return (double)w * (1.0 / 4294967296.0); }

// Loss type on the LOSS word w (u = w * 2^-32, :180-188): u < 0.1 <=> w < kTypeLo,
// u > 0.9 <=> w > kTypeHi. Both products by 2^32 are exact and not integers.
constexpr uint32_t kTypeLo = (uint32_t)(0.1 * 4294967296.0) + 1u;  // 429496730
constexpr uint32_t kTypeHi = (uint32_t)(0.9 * 4294967296.0);       // 3865470566
static_assert(0.1 * 4294967296.0 != (double)(uint32_t)(0.1 * 4294967296.0), "bound is an integer");
static_assert(0.9 * 4294967296.0 != (double)(uint32_t)(0.9 * 4294967296.0), "bound is an integer");
enum LossKind : int { kLossNone = 0, kLossPartial = 1, kLossTotal = 2 };

// sqrt of a non-negative integer, correctly rounded (np.sqrt on the int sum of
// squares, shipping/util.py:4). Unit moves take the exact fast path.
__host__ __device__ __forceinline__ double int_sqrt_rn(int v) {
    return v == 1 ? 1.0 : sqrt_rn((double)v);
}

// Does this env's step draw a gate that can change anything? (a MOVE that passes
// its checks with 0 < cargo < 50; cargo 0 never loses, cargo >= 50 always fires)
template <bool kUnitMoves>
__device__ __forceinline__ bool needs_gate(const LdsWorld& w, const Ship& s, int type, int a, int b) {
    if (kUnitMoves) {
        const int nx = s.x + a, ny = s.y + b;
        return (type == 1) & (s.dest != SE_NONE) & ((unsigned)nx < (unsigned)w.H) &
               ((unsigned)ny < (unsigned)w.W) & (s.cargo > 0) & (s.cargo < 50);
    }
    return (type == 1) & (s.cargo > 0) & (s.cargo < 50);  // typed form: draw whenever possible
}

// One env's step between its two halves.
struct Pending {
    double r;     // reward so far, in the reference's add order
    int e;        // SE_ERR_*
    bool mv;      // a MOVE that passed its checks (:276-284)
    bool moved;   // ... and left its cell (not blocked by ground, :293-300)
    bool fires;   // the cargo-loss gate fired (:318-323)
    bool arrive;  // the move ends on the destination port (:325)
    bool dead;    // out of fuel: the step returns done (:288-290)
};

// First half of one env's step (:359-376) for a typed action (shipping/type.py:1-5):
// everything that needs no optional draw, as selects over the three action
// families so a wave runs one straight path. On return `s` holds the state after
// the move / select / take; env_finish applies cargo loss and arrival. An error
// leaves s untouched (the reference raises before mutating: :284 before :287,
// :266-269, :342-346). The gate (:318-323, random() <= cargo/50) tests the tape's
// f64 u_gate in replay and the Philox word gw in production: w <= floor(fl(c/50)
// * 2^32) is the same test on u = w * 2^-32. Production skips the cargo-0 case (a
// firing gate then loses nothing, :180-181); replay keeps it because the reference
// still draws the loss type there (:177) and replay tracks every draw. From cargo
// 50 on the gate always fires (random() < 1 <= cargo/50).
// u_fuel: replay, the tape's f64 uniform; production, the Philox word w as a double
// (u = w * 2^-32), so 0.2 * u is one product with 0.2 * 2^-32: scaling by a power of
// two is exact, so fl(w * fl(0.2) * 2^-32) == fl(fl(0.2) * u) bit for bit.
constexpr double kFifthPerWord = 0x1.999999999999ap-35;  // fl(0.2) * 2^-32
static_assert(kFifthPerWord * 4294967296.0 == 0.2, "0.2 * 2^-32 must be exact");

template <bool kUnitMoves, bool kReplay>
__host__ __device__ __forceinline__ Pending env_begin(const LdsWorld& w, Ship& s, int e_in, int type, int a,
                                             int b, double u_fuel, double u_gate, uint32_t gw) {
    // --- MOVE (_move_ship :273-339)
    const bool no_dest = s.dest == SE_NONE;                                      // :276
    const bool big = !kUnitMoves & ((a < -256) | (a > 256) | (b < -256) | (b > 256));  // surely OOB
    const int nx = s.x + (big ? 0 : a), ny = s.y + (big ? 0 : b);
    const bool oob = big | ((unsigned)nx >= (unsigned)w.H) | ((unsigned)ny >= (unsigned)w.W);  // :284
    const bool mv_ok = !no_dest & !oob;
    const int cx = mv_ok ? nx : s.x, cy = mv_ok ? ny : s.y;  // in-range cell for the lookups
    // fuel cost (:103-104): dist * (1 + uniform(-0.1, 0.1)), uniform = -0.1 + 0.2*u, unfused
    const double fifth_u = kReplay ? 0.2 * u_fuel : u_fuel * kFifthPerWord;
    const double scale = 1.0 + (-0.1 + fifth_u);
    const double cost = kUnitMoves ? scale : int_sqrt_rn(big ? 1 : a * a + b * b) * scale;
    const bool out_of_fuel = s.fuel < cost;  // :288-290
    const bool ground = w.is_ground(cx, cy);  // :293: blocked (-5) or moved (-0.0001 then -1)
    const int mx = ground ? s.x : cx, my = ground ? s.y : cy;
    // :307-315 old cell vs ATTEMPTED cell; sqrt is monotone and the squared
    // distances are small integers, so comparing them is exact
    const int dcl = no_dest ? 0 : s.dest;
    const int px = w.px(dcl), py = w.py(dcl);
    const int d_old = mul24i(s.x - px, s.x - px) + mul24i(s.y - py, s.y - py);  // |d| < 256
    const int d_new = mul24i(cx - px, cx - px) + mul24i(cy - py, cy - py);
    const bool closer = d_old > d_new;

    // --- SELECT_PORT (_select_port :265-271); an agent index always names a port in range
    const int e_same = s.origin == a ? SE_ERR_SAME_PORT : SE_ERR_OK;
    const int e_sel = (!kUnitMoves & ((a < 0) | (a >= w.P))) ? SE_ERR_PORT_RANGE : e_same;
    // --- TAKE_FUEL / TAKE_CARGO (:341-357)
    const int idx = w.port_at(s.x, s.y);
    const int sidx = idx < 0 ? 0 : idx;
    const int2 st2 = w.stock[sidx];
    const int stock = type == 4 ? st2.y : st2.x;
    const int e_amount = ((a <= 0) | (a > stock)) ? SE_ERR_AMOUNT : SE_ERR_OK;
    const int e_take = idx < 0 ? SE_ERR_NOT_AT_PORT : e_amount;
    const int e_oob = oob ? SE_ERR_OOB : SE_ERR_OK;
    const int e_move = no_dest ? SE_ERR_NO_DEST : e_oob;

    // Every ternary below has named values as arms: clang emits a nested or
    // computing arm as control flow, which becomes a divergent branch.
    // :373-374; an agent index always decodes to a category in 1..4
    const int e4 = (kUnitMoves | (type == 3) | (type == 4)) ? e_take : SE_ERR_BAD_CATEGORY;
    const int e3 = type == 2 ? e_sel : e4;
    const int e2 = type == 1 ? e_move : e3;
    const int e1 = w.P == 0 ? SE_ERR_NO_PORTS : e2;  // :360
    Pending p;
    p.e = e_in != SE_ERR_OK ? e_in : e1;  // the decode runs before env.step (agents/dqn.py:286-287)
    const bool ok = p.e == SE_ERR_OK;
    const bool do_move = ok & (type == 1);

    const int ci = ((s.cargo > 0) & (s.cargo < 50)) ? s.cargo : 0;
    bool fires;
    if constexpr (kReplay) {
        const double lk = w.likelihood(ci);
        fires = (s.cargo >= 50) | (u_gate <= lk);
    } else {
        const uint32_t thr = w.gate_thr[ci];
        fires = (s.cargo >= 50) | ((s.cargo > 0) & (gw <= thr));
    }

    p.mv = do_move;
    p.moved = do_move & !ground;
    p.fires = do_move & fires;
    p.arrive = do_move & (mx == px) & (my == py);
    p.dead = do_move & out_of_fuel;
    const bool take_fuel = ok & (type == 3), take_cargo = ok & (type == 4);
    // reward before loss / arrival from the table the host summed in the reference's order
    const int r_move = ((int)out_of_fuel << 2) | ((int)ground << 1) | (int)closer;
    const int r_other = (take_fuel | take_cargo) ? 8 : 9;
    p.r = w.rtab[do_move ? r_move : r_other];
    s.x = do_move ? mx : s.x;
    s.y = do_move ? my : s.y;
    const double burnt = s.fuel - cost, filled = s.fuel + (double)a;
    const double fuel_mv = (do_move & !ground) ? burnt : s.fuel;  // moves and takes exclude
    s.fuel = take_fuel ? filled : fuel_mv;
    const int loaded = s.cargo + a;
    s.cargo = take_cargo ? loaded : s.cargo;
    s.dest = (ok & (type == 2)) ? a : s.dest;
    return p;
}

// int(beta * cargo) (:195-197) for beta = m * 2^-32 (production: m the median word).
// While m * cargo < 2^53 the f64 product is exact, and scaling by 2^-32 is too, so
// the truncation is the high word of the 64-bit product: one v_mul_hi_u32 in place
// of three conversions and a multiply. Larger cargo takes the f64 path.
__device__ __forceinline__ int beta_part(uint32_t m, int cargo) {
    const int hi = (int)__umulhi(m, (uint32_t)cargo);
    const int f = (int)(((double)m * (1.0 / 4294967296.0)) * (double)cargo);
    return cargo < (1 << 21) ? hi : f;
}

// Second half: cargo loss (_calculate_cargo_loss :169-200) of kind none / partial
// (part = int(beta * cargo), :195-197) / total, then arrival (:325-337) with the
// redrawn destination. Selects only.
__host__ __device__ __forceinline__ void env_finish(Ship& s, Pending& p, int kind, int part, int new_dest,
                                           bool fires, bool arrive) {
    const int some = kind == kLossTotal ? s.cargo : part;
    const int loss = kind == kLossNone ? 0 : some;
    const double rl = p.r + (double)(-3 * loss);
    const int kept = s.cargo - loss;
    p.r = fires ? rl : p.r;
    s.cargo = fires ? kept : s.cargo;
    const double ra = (p.r + (double)(2 * s.cargo)) + 10.0;
    p.r = arrive ? ra : p.r;
    s.cargo = arrive ? 0 : s.cargo;
    const int dest = s.dest;
    s.dest = arrive ? new_dest : dest;
    s.origin = arrive ? dest : s.origin;
}

// utils/preprocessing.py:111-137 (moves N, E, S, W; Python wraps -4..-1), in
// integer arithmetic: the compiler turns nested ternaries into divergent branches.
//   act < 4: MOVE k = act & 3, N (0,-1) E (-1,0) S (0,1) W (1,0)
//   [4, 4+P): SELECT_PORT act-4   [4+P, 54+P): TAKE_CARGO   [54+P, ...): TAKE_FUEL
__device__ __forceinline__ int decode_agent(int P, int act, int& type, int& a, int& b) {
    const int k = act & 3;  // -4..-1 -> 0..3 like Python's negative list index
    const int move = act < 4, sel = act < 4 + P, cargo = act < 54 + P;
    type = move ? 1 : 3 + cargo - 2 * sel;
    const int val = act - 4 - (1 - sel) * P - (1 - cargo) * 50;
    const int odd = k & 1;
    const int dx = odd * (k - 2);   // EAST = (-1, 0), WEST = (1, 0)
    a = move ? dx : val;
    b = move * (1 - odd) * (k - 1);  // NORTH = (0, -1), SOUTH = (0, 1)
    return act < -4 ? SE_ERR_BAD_INDEX : SE_ERR_OK;
}

// One env's replayed step (se_step_replay; se_host_step_replay runs the same code on the
// host): the reference's draws come from the tape record tp (uf / ug its u_fuel / u_gate,
// read by the caller). Returns the SE_USED_* bits of the draws the reference made. A
// variate the step needs but the record lacks (NaN, arrive_dest < 0) leaves the env
// untouched with SE_ERR_NEED_DRAW, reward 0 and done 0.
__host__ __device__ __forceinline__ uint32_t replay_env(const LdsWorld& w, Ship& s, Pending& p, int er, int ty,
                                                        int va, int vb, double uf, double ug,
                                                        const se_tape* tp) {
    const Ship s0 = s;
    p = env_begin<false, true>(w, s, er, ty, va, vb, uf, ug, 0u);
    uint32_t used = p.mv ? (kUsedFuelGate | (p.moved ? kUsedMoved : 0u)) : 0u;
    bool need = p.mv && (uf != uf || ug != ug);
    int kind = kLossNone, nd = 0;
    double beta = 0.0;
    if (p.fires) {
        used |= kUsedLossType;
        const double lt = tp->u_type;
        const bool partial = s.cargo != 0 && lt >= 0.1 && lt <= 0.9;
        if (partial) {
            used |= kUsedBeta;
            beta = tp->beta;
        }
        need = need || lt != lt || (partial && beta != beta);
        kind = lt < 0.1 ? kLossNone : (lt > 0.9 ? kLossTotal : kLossPartial);
    }
    if (p.arrive) {
        used |= kUsedArrive;
        nd = tp->arrive_dest;
        need = need || nd < 0;
    }
    env_finish(s, p, kind, (int)(beta * (double)s.cargo), nd, p.fires, p.arrive);
    if (need) {  // ask the caller for the next variate; change nothing
        s = s0;
        p.r = 0.0;
        p.dead = false;
        p.e = SE_ERR_NEED_DRAW;
    }
    return used;
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

// number of set bits of `mask` below this lane
__device__ __forceinline__ uint32_t count_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// ------------------------------------------------------------------ step kernel
#if SHIPENV_TRACE
// [step parity][wave][8] s_memrealtime stamps (100 MHz): start, staged, stepped, end
constexpr int kTraceWaves = 1 << 16;
__device__ uint64_t g_trace[kTraceWaves * 8];
#define TRACE_STAMP(k)                                                                        \
    do {                                                                                      \
        const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                                 \
        const uint32_t w_ = blockIdx.x * (kStepBlock / 64) + (threadIdx.x >> 6);                  \
        if ((threadIdx.x & 63) == 0 && w_ < kTraceWaves / 2)                                  \
            g_trace[((A.t & 1u) * (kTraceWaves / 2) + w_) * 8 + (k)] = t_;                    \
    } while (0)
#else
#define TRACE_STAMP(k) \
    do {               \
    } while (0)
#endif

constexpr uint8_t kRecDone = 1, kRecInvalid = 2;  // replay ring flags byte (csrc/replay.h)

constexpr int64_t kRecMaxIters = 8;  // se_step_record's cut bits: 4 per group, <= 32 per thread

// se_step_record: the replay ring's end-of-step record (replay_end4_kernel's stores,
// csrc/replay.h) written by the step kernel from the state it holds in registers, and
// the cut envs restarted there (se_replay_end_reset). Null rew outside se_step_record.
struct StepRecord {
    float* rew;
    uint8_t* flags;
    uint32_t* n_pos;
    float* n_fuel;
    int64_t* d_size;
    int64_t head, cap, new_size;  // head, cap multiples of 4 (a group's slots are consecutive)
    uint8_t* cut;
    int32_t max_steps;
    uint32_t epoch;
};

struct StepArgs {
    const uint32_t* world;
    WorldDims dims;
    int64_t n;
    int64_t env_base;  // multiple of 4 (a quad of envs shares its draw blocks)
    uint64_t seed;
    uint32_t t;
    se_state st;
    const int32_t* act;   // agent index (kTyped = false) or type (kTyped = true)
    const int32_t* act_a;
    const int32_t* act_b;
    se_tape* tape;           // replay: variates in, used flags out
    se_done_rec* done_recs;  // this step's done list: per-(iteration, wave) segments of `seg` records
    int32_t* done_count;     // this step's per-segment record counts
    int64_t seg;             // segment stride (records) of one workgroup
    int32_t done_pad;        // done-list records padded to runs of this many (1: none; wave_compact)
    int64_t iters;           // groups per thread (each workgroup owns iters * 256 groups)
    double* slab;            // per-wave {sum_ret, n_eps, sum_len, pad}
    StepRecord rec;          // step_kernel<..., kRec = true> only
};

// The kernel's StepArgs re-read from the kernarg segment where a late phase needs
// them. The empty asm makes the compiler forget its SGPR copies, so pointers used
// only after the Philox / select stretch (store_rest, the episode counters, the done
// list, the slab) are fetched with s_load where they are used instead of staying
// live in SGPRs across it (the config-4 kernel spilled 44 SGPRs to VGPR lanes:
// ~135 v_writelane / v_readlane). StepArgs is the kernels' only argument, so it
// starts the kernarg segment.
typedef const __attribute__((address_space(4))) StepArgs* StepArgsK;
__device__ __forceinline__ const StepArgs& late_args() {
    StepArgsK p = (StepArgsK)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const StepArgs*)p;
}

// Field access for the 4 envs of one group. Full groups: the pointer advanced to
// the block-uniform first group g0 stays scalar and the lane offset is
// loop-invariant, so no per-access 64-bit address arithmetic runs on the VALU; each
// field is one 4-byte (u8 x4), 16-byte (32-bit x4) or 2 x 16-byte (f64 x4) lane
// access. The partial last group uses guarded scalar accesses at env index base.
template <typename T>
__device__ __forceinline__ T* slab_of(T* p, int64_t g0) {
    return p + g0 * 4;
}

// Streaming accesses: state is touched once per step, so stores carry the
// nontemporal hint (written lines do not linger dirty in L2 until the end-of-kernel
// writeback). Loads take it only when the step's working set is cache-resident
// (kNt, chosen per launch by step_nt_loads): measured faster at N = 2^20, slower
// at 2^24.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <bool kNt = false, typename V>
__device__ __forceinline__ V ld_stream(const V* p) {
    if constexpr (kNt) {
        if constexpr (sizeof(V) == 16)
            return __builtin_bit_cast(V, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)));
        else
            return __builtin_nontemporal_load(p);
    } else {
        return *p;
    }
}
template <typename V>
__device__ __forceinline__ void st_stream(V* p, V v) {
    if constexpr (sizeof(V) == 16)
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, v), reinterpret_cast<u32x4*>(p));
    else
        __builtin_nontemporal_store(v, p);
}

// the full-group stores: st_stream above at a byte offset
template <typename V>
__device__ __forceinline__ void st_at(void* base, uint32_t byte_off, V v) {
    st_stream(reinterpret_cast<V*>(reinterpret_cast<char*>(base) + byte_off), v);
}

template <bool kNt = false, typename T>
__device__ __forceinline__ void ld4_full(const T* __restrict__ p, int64_t g0, T (&v)[4],
                                         uint32_t lane = threadIdx.x) {
    if constexpr (sizeof(T) == 4) {
        const uint4 w = ld_stream<kNt>(reinterpret_cast<const uint4*>(slab_of(p, g0)) + lane);
        v[0] = __builtin_bit_cast(T, w.x);
        v[1] = __builtin_bit_cast(T, w.y);
        v[2] = __builtin_bit_cast(T, w.z);
        v[3] = __builtin_bit_cast(T, w.w);
    } else {
        const double2* q = reinterpret_cast<const double2*>(slab_of(p, g0)) + 2 * lane;
        const double2 a = ld_stream<kNt>(q), b = ld_stream<kNt>(q + 1);
        v[0] = a.x;
        v[1] = a.y;
        v[2] = b.x;
        v[3] = b.y;
    }
}

template <typename T>
__device__ __forceinline__ void st4_full(T* __restrict__ p, int64_t g0, const T (&v)[4]) {
    if constexpr (sizeof(T) == 4) {
        uint4 w;
        w.x = __builtin_bit_cast(uint32_t, v[0]);
        w.y = __builtin_bit_cast(uint32_t, v[1]);
        w.z = __builtin_bit_cast(uint32_t, v[2]);
        w.w = __builtin_bit_cast(uint32_t, v[3]);
        st_at(slab_of(p, g0), 16u * threadIdx.x, w);
    } else {
        st_at(slab_of(p, g0), 32u * threadIdx.x, make_double2(v[0], v[1]));
        st_at(slab_of(p, g0), 32u * threadIdx.x + 16u, make_double2(v[2], v[3]));
    }
}

template <typename T>
__device__ __forceinline__ void ld4_tail(const T* __restrict__ p, int64_t base, int64_t n, T (&v)[4]) {
    for (int j = 0; j < 4; ++j) v[j] = base + j < n ? p[base + j] : T(0);
}

template <typename T>
__device__ __forceinline__ void st4_tail(T* __restrict__ p, int64_t base, int64_t n, const T (&v)[4]) {
    for (int j = 0; j < 4; ++j)
        if (base + j < n) p[base + j] = v[j];
}

template <bool kNt = false>
__device__ __forceinline__ uint32_t ld4u8_full(const uint8_t* __restrict__ p, int64_t g0,
                                               uint32_t lane = threadIdx.x) {
    return ld_stream<kNt>(reinterpret_cast<const uint32_t*>(slab_of(p, g0)) + lane);
}
__device__ __forceinline__ void st4u8_full(uint8_t* __restrict__ p, int64_t g0, uint32_t w) {
    st_at(slab_of(p, g0), 4u * threadIdx.x, w);
}
__device__ __forceinline__ uint32_t ld4u8_tail(const uint8_t* __restrict__ p, int64_t base, int64_t n) {
    uint32_t w = 0;
    for (int j = 0; j < 4; ++j)
        if (base + j < n) w |= (uint32_t)p[base + j] << (8 * j);
    return w;
}
__device__ __forceinline__ void st4u8_tail(uint8_t* __restrict__ p, int64_t base, int64_t n, uint32_t w) {
    for (int j = 0; j < 4; ++j)
        if (base + j < n) p[base + j] = (uint8_t)(w >> (8 * j));
}

__device__ __forceinline__ int byte_of(uint32_t w, int j) { return (int)((w >> (8 * j)) & 0xffu); }

// Where one group's fields live: g0 (block-uniform) for a full group, whose envs
// are 4 * (g0 + threadIdx.x) + j; base = the group's first env in both cases.
template <bool kFull>
struct At {
    int64_t g0, base, n;
};

// The inputs of the 4 envs of one group.
template <bool kTyped, bool kAuto, bool kNt = false>
struct Group {
    uint32_t x, y, org, dst;  // packed u8 x4
    int32_t c[4];             // cargo
    double f[4];              // fuel
    int32_t a[4];             // agent index / action type
    int32_t p[4], q[4];       // typed: values a, b
    float e[4];               // ep_return
    uint32_t l[4];            // ep_start: the step counter when the episode began

    // lane: the group within the block's row (threadIdx.x; the kernel's first load
    // clamps it into range instead of branching around the load)
    template <bool kFull>
    __device__ __forceinline__ void load(const StepArgs& A, At<kFull> at, uint32_t lane = threadIdx.x) {
        const se_state& S = A.st;
        if constexpr (kFull) {
            x = ld4u8_full<kNt>(S.x, at.g0, lane);
            y = ld4u8_full<kNt>(S.y, at.g0, lane);
            org = ld4u8_full<kNt>(S.origin, at.g0, lane);
            dst = ld4u8_full<kNt>(S.dest, at.g0, lane);
            ld4_full<kNt>(S.cargo, at.g0, c, lane);
            ld4_full<kNt>(S.fuel, at.g0, f, lane);
            ld4_full<kNt>(A.act, at.g0, a, lane);
            if (kTyped) {
                ld4_full<kNt>(A.act_a, at.g0, p, lane);
                ld4_full<kNt>(A.act_b, at.g0, q, lane);
            }
        } else {
            x = ld4u8_tail(S.x, at.base, at.n);
            y = ld4u8_tail(S.y, at.base, at.n);
            org = ld4u8_tail(S.origin, at.base, at.n);
            dst = ld4u8_tail(S.dest, at.base, at.n);
            ld4_tail(S.cargo, at.base, at.n, c);
            ld4_tail(S.fuel, at.base, at.n, f);
            ld4_tail(A.act, at.base, at.n, a);
            if (kTyped) {
                ld4_tail(A.act_a, at.base, at.n, p);
                ld4_tail(A.act_b, at.base, at.n, q);
            }
            if (kAuto) {
                ld4_tail(S.ep_return, at.base, at.n, e);
                ld4_tail(reinterpret_cast<const uint32_t*>(S.ep_start), at.base, at.n, l);
            }
        }
    }
    // episode counters of a full group, loaded late (step_group), where they would
    // otherwise hold 8 registers across the whole step: the running return of every
    // env, and the episode-start stamps only where they are needed, i.e. in the lanes
    // with an env that finishes in this step (`any`; about 1 env in 240 per step) or
    // for every env (kAll: se_step_record's max_steps cut). The stamps of other lanes
    // are never read or written, so a running length costs no traffic per step.
    template <bool kAll = false>
    __device__ __forceinline__ void load_episode(const StepArgs& A, At<true> at, bool any) {
        ld4_full<kNt>(A.st.ep_return, at.g0, e);
#pragma unroll
        for (int j = 0; j < 4; ++j) l[j] = 0u;
        if (kAll || any)
            ld4_full<kNt>(reinterpret_cast<const uint32_t*>(A.st.ep_start), at.g0, l);
    }
    template <bool kAll = false>
    __device__ __forceinline__ void load_episode(const StepArgs&, At<false>, bool) {}  // loaded with the rest
};

// Whether this lane's stamps move: one of its envs finished.
__device__ __forceinline__ bool stamp_lane(uint32_t fin) { return fin != 0; }

// ep_start of a group after a step at counter t: t + 1 for the envs that finished (the
// next step starts their new episode), unchanged for the others. A full group stores
// its lane's 16 bytes only when one of its envs finished; the partial last group
// stores its live envs.
template <bool kFull>
__device__ __forceinline__ void store_stamps(const se_state& S, At<kFull> at, const uint32_t (&l)[4],
                                             uint32_t fin, uint32_t t, bool any) {
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = ((fin >> j) & 1u) ? t + 1u : l[j];
    if constexpr (kFull) {
        if (any) st4_full(reinterpret_cast<uint32_t*>(S.ep_start), at.g0, v);
    } else {
        st4_tail(reinterpret_cast<uint32_t*>(S.ep_start), at.base, at.n, v);
    }
}

template <bool kFull, typename T>
__device__ __forceinline__ void store4(T* p, At<kFull> at, const T (&v)[4]) {
    if constexpr (kFull) st4_full(p, at.g0, v);
    else st4_tail(p, at.base, at.n, v);
}
template <bool kFull>
__device__ __forceinline__ void store4u8(uint8_t* p, At<kFull> at, uint32_t w) {
    if constexpr (kFull) st4u8_full(p, at.g0, w);
    else st4u8_tail(p, at.base, at.n, w);
}

// Per-thread episode statistics of the finished episodes. Counts are integers:
// summed as doubles they were exact anyway, and they hold two fewer registers.
struct BlockStats {
    double ret = 0.0;
    int32_t eps = 0;
    int64_t len = 0;
};

// Finished episodes of one group (auto-reset): bit j of `mask` for env base+j.
struct Finished {
    uint32_t mask = 0;
    float ret[4];
    int32_t len[4];
    uint32_t cut = 0;  // se_step_record: bit j = env j of the group restarts (cut)
};

// x, y, fuel, done, err of a group's 4 envs: final once the first half has run
// (cargo loss and arrival change none of them).
template <bool kFull>
__device__ __forceinline__ void store_moved(const se_state& S, At<kFull> at, const Ship (&s)[4],
                                            const Pending (&p)[4]) {
    uint32_t ox = 0, oy = 0, dn = 0, ee = 0;
    double fuel[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t sh = 8u * (uint32_t)j;
        ox |= (uint32_t)(s[j].x & 0xff) << sh;
        oy |= (uint32_t)(s[j].y & 0xff) << sh;
        dn |= (uint32_t)p[j].dead << sh;
        ee |= (uint32_t)(p[j].e & 0xff) << sh;
        fuel[j] = s[j].fuel;
    }
    // The two 16-byte halves of a lane's 32 bytes of fuel are two store
    // instructions, each writing every other 16 bytes of the wave's span. Issued
    // apart, the nontemporal halves reach memory as separate partial-line writes
    // (measured: +4.5 MB per launch at N = 2^20); the scheduling barriers keep the
    // pair, and the whole group of stores, back to back.
    __builtin_amdgcn_sched_barrier(0);
    store4u8(S.x, at, ox);
    store4u8(S.y, at, oy);
    store4(S.fuel, at, fuel);
    store4u8(S.done, at, dn);
    store4u8(reinterpret_cast<uint8_t*>(S.err), at, ee);
    __builtin_amdgcn_sched_barrier(0);
}

// cargo, origin, dest, reward (+ the running returns): final after the second half.
template <bool kAuto, bool kFull>
__device__ __forceinline__ void store_rest(const se_state& S, At<kFull> at, const Ship (&s)[4],
                                           const float (&rw)[4], const float (&epr)[4]) {
    uint32_t oo = 0, od = 0;
    int32_t cargo[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t sh = 8u * (uint32_t)j;
        oo |= (uint32_t)(s[j].origin & 0xff) << sh;
        od |= (uint32_t)(s[j].dest & 0xff) << sh;
        cargo[j] = s[j].cargo;
    }
    store4u8(S.origin, at, oo);
    store4u8(S.dest, at, od);
    store4(S.cargo, at, cargo);
    store4(S.reward, at, rw);
    if constexpr (kAuto) store4(S.ep_return, at, epr);
}

// Step the 4 envs 4k..4k+3 of one group (base = 4k). Production draws are Philox
// quad blocks at counter (k, t, slot): word j belongs to env 4k+j (RNG contract,
// DESIGN.md). Each block is drawn only when some env of the quad consumes it, so
// the draws are lane-uniform branches instead of a branch per env and draw:
//   FUEL   every step           GATE    a move with 0 < cargo < 50
//   LOSS   the gate fired       BETA1-3 a partial loss (Beta(2,2) = median of 3)
//   ARRIVE an arrival           RESET, RESET_DEST  an auto-reset
// Replay takes every variate from the env's tape record instead.
// Registers: x, y, fuel, done and err are stored as soon as the first half has
// run (and auto-reset has replaced the finished envs' positions), so only cargo,
// origin, dest and the reward stay live across the loss / arrival blocks.
template <bool kTyped, bool kReplay, bool kAuto, bool kFull, bool kNt = false>
__device__ __forceinline__ void step_group(const StepArgs& A, const LdsWorld& w,
                                           Group<kTyped, kAuto, kNt>& G, At<kFull> at, BlockStats& bs,
                                           Finished& F) {
    const se_state& S = A.st;
    const int64_t n = A.n, base = at.base;
    int ty[4], va[4], vb[4], er[4];
    Ship s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (kTyped) {
            ty[j] = G.a[j];
            va[j] = G.p[j];
            vb[j] = G.q[j];
            er[j] = SE_ERR_OK;
        } else {
            er[j] = decode_agent(w.P, G.a[j], ty[j], va[j], vb[j]);
        }
        s[j] = Ship{byte_of(G.x, j), byte_of(G.y, j), G.f[j], G.c[j], byte_of(G.org, j), byte_of(G.dst, j)};
    }
    const Key qk = env_key(A.seed, (A.env_base + base) >> 2);
    const uint32_t t = A.t;
    Pending p[4];

    if constexpr (kReplay) {
        // one env at a time; a missing variate (NEED_DRAW) leaves its env untouched
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t i = base + j;
            const bool live = kFull || i < n;
            se_tape* tp = A.tape + (live ? i : 0);
            const double uf = live ? tp->u_fuel : 0.0, ug = live ? tp->u_gate : 0.0;
            const uint32_t used = replay_env(w, s[j], p[j], er[j], ty[j], va[j], vb[j], uf, ug, tp);
            if (live) {
                tp->used = (int32_t)used;
                if (S.reward64) S.reward64[i] = p[j].r;
            }
        }
        store_moved(S, at, s, p);
        float rw[4], none[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) rw[j] = (float)p[j].r;
        store_rest<false>(S, at, s, rw, none);
        (void)bs;
        (void)F;
    } else {
        bool gate_needed = false;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            gate_needed |= (er[j] == SE_ERR_OK) & needs_gate<!kTyped>(w, s[j], ty[j], va[j], vb[j]);
        const U4 fb = draw(qk, t, kSlotFuel);
        U4 gb{{0u, 0u, 0u, 0u}};
        if (gate_needed) gb = draw(qk, t, kSlotGate);
        uint32_t fire = 0, arrive = 0, fin = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            p[j] = env_begin<!kTyped, false>(w, s[j], er[j], ty[j], va[j], vb[j], (double)fb.v[j], 0.0, gb.v[j]);
            fire |= (uint32_t)p[j].fires << j;
            arrive |= (uint32_t)p[j].arrive << j;
            fin |= (uint32_t)((kFull || base + j < n) & p[j].dead) << j;
        }
        // The per-env flags travel as these VGPR bit masks from here on: opaque to
        // the compiler, so it does not keep 4 x 3 lane masks (SGPR pairs) live
        // across the draw blocks below, which spilled them to VGPR lanes.
        asm volatile("" : "+v"(fire), "+v"(arrive), "+v"(fin));
        // auto-reset (:227-243) of the envs that ran out of fuel: their position and
        // fuel now, cargo / origin / dest after the second half (whose reward the
        // finished episode still collects). Contract v5: the r-th finishing env of the
        // quad takes block RESET_r (word 0 origin, word 1 destination), as LOSS_r.
        uint32_t reset_o = 0, reset_d = 0;  // reset origin / dest bytes of the 4 envs
        if constexpr (kAuto) {
            if (fin) {
                uint32_t ow[4], dw[4];
                {
                    const uint32_t rk[4] = {0u, fin & 1u, (uint32_t)__popc(fin & 3u), (uint32_t)__popc(fin & 7u)};
                    U4 r = draw(qk, t, reset_slot(0));
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        ow[j] = r.v[0];
                        dw[j] = r.v[1];
                    }
#pragma unroll
                    for (uint32_t q = 1; q < 4; ++q) {
                        if (__popc(fin) > q) {
                            r = draw(qk, t, reset_slot(q));
#pragma unroll
                            for (int j = (int)q; j < 4; ++j) {
                                ow[j] = rk[j] >= q ? r.v[0] : ow[j];
                                dw[j] = rk[j] >= q ? r.v[1] : dw[j];
                            }
                        }
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    Ship r;
                    reset_ship(w, r, ow[j], dw[j]);
                    reset_o |= (uint32_t)r.origin << (8 * j);
                    reset_d |= (uint32_t)r.dest << (8 * j);
                    const bool f = (fin >> j) & 1u;
                    s[j].x = f ? r.x : s[j].x;
                    s[j].y = f ? r.y : s[j].y;
                    s[j].fuel = f ? r.fuel : s[j].fuel;
                }
            }
            G.load_episode(late_args(), at, stamp_lane(fin));
        }
        store_moved(S, at, s, p);

        // Cargo loss (contract v5): the r-th env of the quad whose gate fired takes
        // the whole block LOSS_r: word 0 the loss type, words 1-3 the Beta(2, 2)
        // uniforms. LOSS_0 runs whenever any env of the wave fired; LOSS_1..3 only
        // where a quad had two or more (a few percent of waves). Envs take the
        // words of the block matching their rank; non-firing envs ignore theirs.
        uint32_t lt[4], v1[4], v2[4], v3[4];
        {
            const uint32_t f1 = fire & 1u, f2 = __popc(fire & 3u), f3 = __popc(fire & 7u);
            const uint32_t rk[4] = {0u, f1, f2, f3};
            U4 r{{0u, 0u, 0u, 0u}};
            if (fire) r = draw(qk, t, loss_slot(0));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                lt[j] = r.v[0];
                v1[j] = r.v[1];
                v2[j] = r.v[2];
                v3[j] = r.v[3];
            }
#pragma unroll
            for (uint32_t q = 1; q < 4; ++q) {
                if (fire >> q) {  // some env after the first fired too: rank q exists
                    if (__popc(fire) > q) {
                        r = draw(qk, t, loss_slot(q));
#pragma unroll
                        for (int j = (int)q; j < 4; ++j) {
                            const bool take = rk[j] >= q;
                            lt[j] = take ? r.v[0] : lt[j];
                            v1[j] = take ? r.v[1] : v1[j];
                            v2[j] = take ? r.v[2] : v2[j];
                            v3[j] = take ? r.v[3] : v3[j];
                        }
                    }
                }
            }
        }
        int kind[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int total = lt[j] > kTypeHi ? kLossTotal : kLossPartial;
            kind[j] = lt[j] < kTypeLo ? kLossNone : total;
        }
        U4 ab{{0u, 0u, 0u, 0u}};
        if (arrive) ab = draw(qk, t, kSlotArrive);
        float rw[4], epr[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            // beta = the median of the three words * 2^-32 (the conversion is monotone)
            const uint32_t lo = min(v1[j], v2[j]), hi = max(v1[j], v2[j]);
            const uint32_t med = max(lo, min(hi, v3[j]));  // v_med3_u32
            env_finish(s[j], p[j], kind[j], beta_part(med, s[j].cargo), pick_other(ab.v[j], w.P, s[j].dest),
                       (fire >> j) & 1u, (arrive >> j) & 1u);
            rw[j] = (float)p[j].r;  // one rounding of the reference's f64 reward
            epr[j] = 0.0f;
            if constexpr (kAuto) {
                const bool f = (fin >> j) & 1u;
                F.ret[j] = G.e[j] + rw[j];
                F.len[j] = (int32_t)(t + 1u - G.l[j]);  // stamps are loaded where fin
                if (f) {
                    bs.ret += (double)F.ret[j];
                    bs.eps += 1;
                    bs.len += F.len[j];
                }
                epr[j] = f ? 0.0f : F.ret[j];
                s[j].cargo = f ? 0 : s[j].cargo;
                s[j].origin = f ? byte_of(reset_o, j) : s[j].origin;
                s[j].dest = f ? byte_of(reset_d, j) : s[j].dest;
            }
        }
        if constexpr (kAuto) F.mask = fin;
        store_rest<kAuto>(late_args().st, at, s, rw, epr);
        if constexpr (kAuto) store_stamps(late_args().st, at, G.l, fin, t, stamp_lane(fin));
    }
}

// ------------------------------------------------------------------ agent-index path
// The production step for agent-index actions (se_step), written for VALU issue,
// the bound at N = 2^20: the same semantics as env_begin +
// env_finish with kUnitMoves (tests compare it bit for bit with the
// oracle), in a packed form.
//   * A ship position is one register x | y << 16: a move is one v_pk_add_u16 of
//     the action's packed (dx, dy) from the world image, the bounds test one
//     v_pk_min_u16 against (H-1, W-1), a cell index one v_dot2_u32_u16 with (W, 1),
//     the squared distances of the closer/farther test (:307-315) one v_pk_sub_i16
//     and one v_dot2_i32_i16 each, and the arrival test (:325) one compare.
//   * One cell-code byte answers "ground?" for the target cell (:293) and "which
//     port?" for the ship's cell (:145-153).
//   * Fuel changes by one f64 add of a selected delta (-cost, +amount or -0.0, which
//     leaves every fuel value as it is, -0.0 included).
//   * Cargo loss and arrival arithmetic run inside the branches that draw their
//     blocks, so waves without a firing gate / an arrival skip them.
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
typedef int16_t i16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_add_u16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) + __builtin_bit_cast(u16x2, b));
}
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
}
// squared euclidean distance of two packed positions (halves < 256)
__device__ __forceinline__ int dist2(uint32_t a, uint32_t b) {
    const i16x2 d = __builtin_bit_cast(i16x2, a) - __builtin_bit_cast(i16x2, b);
    return __builtin_amdgcn_sdot2(d, d, 0, false);
}
// cell index x * W + y of a packed position; wh = W | 1 << 16
__device__ __forceinline__ uint32_t cell_of(uint32_t p, uint32_t wh) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, p), __builtin_bit_cast(u16x2, wh), 0u, false);
}

// The Philox blocks of a group that depend on no state (contract v5: FUEL every step;
// GATE, whose words are the same whether or not an env consumes them; LOSS_0, the
// block of the quad's first firing env, used by most waves): drawn right after the
// group's loads are issued, so their VALU work overlaps the wait for the data
// instead of following it.
// LOSS_0 is drawn early with auto-reset (config 4 measured 12.71 -> 12.44 us at
// 2^20) and on demand without (config 3: 8.48 vs 8.56 us).
struct Draws {
    U4 fuel, gate, loss0, arrive;
};
template <bool kSpecLoss>
__device__ __forceinline__ Draws early_draws(const StepArgs& A, int64_t base) {
    const Key qk = env_key(A.seed, (A.env_base + base) >> 2);
    Draws d;
    d.fuel = draw(qk, A.t, kSlotFuel);
    d.gate = draw(qk, A.t, kSlotGate);
    d.loss0 = kSpecLoss ? draw(qk, A.t, loss_slot(0)) : U4{{0u, 0u, 0u, 0u}};
    d.arrive = U4{{0u, 0u, 0u, 0u}};
    return d;
}

template <bool kAuto>
constexpr bool spec_loss() { return kAuto; }

// se_step_record, per group of 4 envs at env index base (a full group; head and cap
// multiples of 4, so its ring slots are consecutive): the stores of replay_end4_kernel
// (csrc/replay.h) from the post-step values this thread just computed. After the
// thread's last group, record_restart runs se_replay_end_reset's restart of the cut envs
// (reset_kernel's body, at most one bit per env of the thread's <= 8 groups). Their
// fields were stored by this thread earlier in program order; the restart stores the same
// addresses again, as the separate replay-end launch would after the step. Deferred past
// the loop, the restart's registers do not overlap the group's (inline there it spilled).
__device__ __forceinline__ void record_restart(const StepArgs& A, const LdsWorld& w, uint32_t cuts) {
    const se_state& S = A.st;
    const int64_t first = (int64_t)blockIdx.x * A.iters * kStepBlock;  // step_kernel's first group
    while (cuts) {
        const int b = __builtin_ctz(cuts);
        cuts &= cuts - 1;
        const int64_t i = (first + (int64_t)(b >> 2) * kStepBlock + threadIdx.x) * 4 + (b & 3);
        const U4 o = draw(env_key(A.seed, A.env_base + i), A.rec.epoch, kSlotExplicitReset);
        Ship sh;
        reset_ship(w, sh, o.v[0], o.v[1]);
        S.x[i] = (uint8_t)sh.x;
        S.y[i] = (uint8_t)sh.y;
        S.fuel[i] = sh.fuel;
        S.cargo[i] = sh.cargo;
        S.origin[i] = (uint8_t)sh.origin;
        S.dest[i] = (uint8_t)sh.dest;
        S.ep_return[i] = 0.0f;
        S.ep_start[i] = (int32_t)(A.t + 1u);  // its first step is the next one
        S.done[i] = 0;
        S.err[i] = 0;
        S.reward[i] = 0.0f;
    }
}

__device__ __forceinline__ int64_t record_slot(const StepRecord& R, int64_t base) {
    const int64_t slot = R.head + base;
    return slot - (slot >= R.cap ? R.cap : 0);
}

__device__ __forceinline__ void record_early(const StepArgs& A, int64_t base, uint32_t flags4, const float (&fuel)[4]) {
    const StepRecord& R = A.rec;
    const int64_t slot = record_slot(R, base);
    *reinterpret_cast<uint32_t*>(R.flags + slot) = flags4;
    *reinterpret_cast<float4*>(R.n_fuel + slot) = make_float4(fuel[0], fuel[1], fuel[2], fuel[3]);
}

// returns the cut envs as bits 0-3
__device__ __forceinline__ uint32_t record_group(const StepArgs& A, int64_t base, const float (&rw)[4],
                                                 uint32_t x4, uint32_t y4, uint32_t o4, uint32_t d4,
                                                 uint32_t cut4, const int32_t (&len)[4]) {
    const StepRecord& R = A.rec;
    const int64_t slot = record_slot(R, base);
    uint4 pos;
    uint32_t* pw = &pos.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        pw[j] = ((x4 >> (8 * j)) & 0xffu) | ((y4 >> (8 * j)) & 0xffu) << 8 | ((o4 >> (8 * j)) & 0xffu) << 16 |
                ((d4 >> (8 * j)) & 0xffu) << 24;
        if (R.max_steps > 0) cut4 |= (uint32_t)(len[j] >= R.max_steps) << (8 * j);
    }
    *reinterpret_cast<float4*>(R.rew + slot) = make_float4(rw[0], rw[1], rw[2], rw[3]);
    *reinterpret_cast<uint4*>(R.n_pos + slot) = pos;
    *reinterpret_cast<uint32_t*>(R.cut + base) = cut4;
    return (cut4 & 1u) | ((cut4 >> 7) & 2u) | ((cut4 >> 14) & 4u) | ((cut4 >> 21) & 8u);
}

// kReplay (se_step_agent_replay; parity only): the same code with the reference's draws
// from the tape instead of Philox words: u_fuel and u_gate as f64 uniforms (the gate
// tested against fl(c/50) as env_begin<.., kReplay> does, so a cargo-0 ship's gate can
// fire, lose nothing, and still consume the loss-type draw), the loss type, beta and
// the arrival's new destination; SE_USED_* bits back in the tape, and a step that needs
// a variate the tape lacks leaves its env untouched with SE_ERR_NEED_DRAW.
template <bool kAuto, bool kFull, bool kNt, bool kRec = false, bool kReplay = false>
__device__ __forceinline__ void step_group_agent(const StepArgs& A, const LdsWorld& w,
                                                 Group<false, kAuto, kNt>& G, At<kFull> at,
                                                 BlockStats& bs, Finished& F, const Draws& D) {
    static_assert(!kReplay || (!kAuto && !kRec), "agent replay: no auto-reset, no ring record");
    const int64_t n = A.n, base = at.base;
    const int P = w.P;
    const uint32_t lim = (uint32_t)(w.H - 1) | ((uint32_t)(w.W - 1) << 16);
    const uint32_t wh = (uint32_t)w.W | (1u << 16);
    const uint32_t pm1 = P > 0 ? (uint32_t)(P - 1) : 0u;  // clamp for table reads whose value an error discards
    const Key qk = env_key(A.seed, (A.env_base + base) >> 2);
    const uint32_t t = A.t;
    constexpr bool kSpecLoss = spec_loss<kAuto>();
#if SHIPENV_TRACE
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the group's data has arrived
    TRACE_STAMP(4);
#endif
    // --- first half: everything that needs no optional draw (:359-376, :273-315)
    uint32_t pos[4], pd16[4];
    int val[4], dst[4], cg[4], err[4], ridx[4];
    bool do_move[4], moved[4], tf_ok[4];
    bool gate_needed = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        // utils/preprocessing.py:111-137: [0,4) moves N, E, S, W (-4..-1 wrap like a
        // Python index), [4, 4+P) SELECT, [4+P, 54+P) TAKE_CARGO, then TAKE_FUEL
        const int act = G.a[j];
        const bool bad = act < -4, is_mv = act < 4, lt_sel = act < 4 + P, lt_tc = act < 54 + P;
        val[j] = act - 4 - (lt_sel ? 0 : P) - (lt_tc ? 0 : 50);
        const uint32_t dxy = w.moves[act & 3];
        // packed position x | y << 16 from the group's x and y bytes
        const uint32_t p = __builtin_amdgcn_perm(G.y, G.x, (uint32_t)j | 0x0c000c00u | ((uint32_t)(4 + j) << 16));
        dst[j] = byte_of(G.dst, j);
        cg[j] = G.c[j];
        // MOVE (_move_ship :273-339)
        const uint32_t np = pk_add_u16(p, dxy);
        const bool inb = pk_min_u16(np, lim) == np;  // _is_within_map (:284); -1 wraps to 0xffff
        const bool nodest = dst[j] == SE_NONE;       // :276
        const uint32_t cp = (!nodest & inb) ? np : p;  // in-range cell for the lookups
        const bool ground = w.cell[cell_of(cp, wh)] == kCellGround;  // :293
        pd16[j] = w.pos[min((uint32_t)dst[j], pm1)];
        const bool closer = dist2(p, pd16[j]) > dist2(cp, pd16[j]);  // old vs ATTEMPTED cell (:307-315)
        // TAKE_* (:341-357) at the port on the ship's cell; SELECT_PORT (:265-271)
        const int k = (int)w.cell[cell_of(p, wh)] - 1;
        const bool atport = (uint32_t)k < (uint32_t)P;
        const int2 st2 = w.stock[min((uint32_t)k, pm1)];
        const int stock = lt_tc ? st2.y : st2.x;
        const bool amount_bad = (val[j] <= 0) | (val[j] > stock);
        const bool same = byte_of(G.org, j) == val[j];
        const int e_move = nodest ? SE_ERR_NO_DEST : (inb ? SE_ERR_OK : SE_ERR_OOB);
        const int e_sel = same ? SE_ERR_SAME_PORT : SE_ERR_OK;
        const int e_amt = amount_bad ? SE_ERR_AMOUNT : SE_ERR_OK;
        const int e_take = atport ? e_amt : SE_ERR_NOT_AT_PORT;
        const int e_ns = lt_sel ? e_sel : e_take;
        const int e_ty = is_mv ? e_move : e_ns;
        const int e_p = P == 0 ? SE_ERR_NO_PORTS : e_ty;  // :360
        err[j] = bad ? SE_ERR_BAD_INDEX : e_p;            // the decode runs before env.step
        const bool ok = err[j] == SE_ERR_OK;
        do_move[j] = ok & is_mv;
        moved[j] = do_move[j] & !ground;
        const bool take_ok = ok & !lt_sel;
        tf_ok[j] = take_ok & !lt_tc;
        const bool tc_ok = take_ok & lt_tc;
        const bool sel_ok = ok & !is_mv & lt_sel;
        pos[j] = moved[j] ? cp : p;
        cg[j] = tc_ok ? cg[j] + val[j] : cg[j];
        dst[j] = sel_ok ? val[j] : dst[j];
        // reward row before loss / arrival: a move by (out_of_fuel, ground, closer),
        // filled in once fuel is known; a take 0.05; anything else 0
        const int r_rest = take_ok ? 8 : 9;
        ridx[j] = do_move[j] ? (((int)ground << 1) | (int)closer) : r_rest;
        gate_needed |= !bad & is_mv & !nodest & inb & (G.c[j] > 0) & (G.c[j] < 50);
    }
    TRACE_STAMP(5);
    (void)gate_needed;  // drawn early (early_draws) whether or not an env needs it
    const U4 fb = D.fuel;
    const U4 gb = D.gate;
    uint32_t fire = 0, arrive = 0, fin = 0, dead = 0;
    double f[4], r[4];
    // kReplay: the group's tape records (the partial last group's missing envs read none)
    [[maybe_unused]] double tu[4], tg[4], tt[4], tb[4];
    [[maybe_unused]] int td[4];
    [[maybe_unused]] uint32_t need = 0;  // kReplay: envs whose step needs a variate the tape lacks
    if constexpr (kReplay) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool live = kFull || base + j < n;
            const se_tape* tp = A.tape + (live ? base + j : 0);
            tu[j] = tp->u_fuel;
            tg[j] = tp->u_gate;
            tt[j] = tp->u_type;
            tb[j] = tp->beta;
            td[j] = tp->arrive_dest;
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        // fuel cost (:103-104): 1 * (1 + uniform(-0.1, 0.1)), uniform = -0.1 + 0.2 u
        double scale;
        if constexpr (kReplay) scale = 1.0 + (-0.1 + 0.2 * tu[j]);
        else scale = 1.0 + (-0.1 + (double)fb.v[j] * kFifthPerWord);
        const bool oof = G.f[j] < scale;  // :288-290 (the ship still moves)
        const double take = tf_ok[j] ? (double)val[j] : -0.0;
        f[j] = G.f[j] + (moved[j] ? -scale : take);
        // the gate random() <= cargo / 50 (:318-323) as w <= floor(fl(c/50) 2^32); the
        // table's entry 50 is all ones (cargo >= 50 always fires); cargo 0 loses nothing
        bool fires;
        if constexpr (kReplay) {
            const double ug = tg[j];
            const int ci = ((cg[j] > 0) & (cg[j] < 50)) ? cg[j] : 0;
            fires = do_move[j] & ((cg[j] >= 50) | (ug <= w.likelihood(ci)));
            need |= (uint32_t)(do_move[j] & ((tu[j] != tu[j]) | (ug != ug))) << j;
        } else {
            const uint32_t thr = w.gate_thr[min(max(cg[j], 0), 50)];
            fires = do_move[j] & (cg[j] > 0) & (gb.v[j] <= thr);
        }
        r[j] = w.rtab[ridx[j] | ((int)(do_move[j] & oof) << 2)];
        fire |= (uint32_t)fires << j;
        arrive |= (uint32_t)(do_move[j] & (pos[j] == pd16[j])) << j;  // :325
        dead |= (uint32_t)(do_move[j] & oof) << j;
        fin |= (uint32_t)((kFull || base + j < n) & do_move[j] & oof) << j;
    }
    // the flags travel as opaque VGPR bit masks (no lane masks live in SGPR pairs
    // across the draw blocks below)
    asm volatile("" : "+v"(fire), "+v"(arrive), "+v"(fin), "+v"(dead));
    int org[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) org[j] = byte_of(G.org, j);

    // auto-reset (:227-243) of the envs that ran out of fuel: position and fuel now,
    // cargo / origin / dest after the second half (whose reward the finished episode
    // still collects). Contract v5: the r-th finishing env of the quad takes RESET_r.
    uint32_t reset_o = 0, reset_d = 0;
    if constexpr (kAuto) {
        if (fin) {
            uint32_t ow[4], dw[4];
            const uint32_t rk[4] = {0u, fin & 1u, (uint32_t)__popc(fin & 3u), (uint32_t)__popc(fin & 7u)};
            U4 rr = draw(qk, t, reset_slot(0));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                ow[j] = rr.v[0];
                dw[j] = rr.v[1];
            }
#pragma unroll
            for (uint32_t q = 1; q < 4; ++q) {
                if (__popc(fin) > q) {
                    rr = draw(qk, t, reset_slot(q));
#pragma unroll
                    for (int j = (int)q; j < 4; ++j) {
                        ow[j] = rk[j] >= q ? rr.v[0] : ow[j];
                        dw[j] = rk[j] >= q ? rr.v[1] : dw[j];
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int o = uniform_int(ow[j], (uint32_t)P);
                const int d = pick_other(dw[j], P, o);
                reset_o |= (uint32_t)o << (8 * j);
                reset_d |= (uint32_t)d << (8 * j);
                const bool fj = (fin >> j) & 1u;
                pos[j] = fj ? w.pos[o] : pos[j];
                f[j] = fj ? kFuelInit : f[j];
            }
        }
        G.template load_episode<kRec>(late_args(), at, stamp_lane(fin));
    }
    // x, y, fuel, done and err are final here (cargo loss and arrival change none)
    uint32_t rec_x = 0, rec_y = 0, rec_cut = 0;
    {
        const uint32_t t01 = __builtin_amdgcn_perm(pos[1], pos[0], 0x06020400u);  // x0 x1 y0 y1
        const uint32_t t23 = __builtin_amdgcn_perm(pos[3], pos[2], 0x06020400u);  // x2 x3 y2 y3
        const uint32_t ox = __builtin_amdgcn_perm(t23, t01, 0x05040100u);
        const uint32_t oy = __builtin_amdgcn_perm(t23, t01, 0x07060302u);
        uint32_t dn = 0, ee = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            dn |= ((dead >> j) & 1u) << (8 * j);
            ee |= (uint32_t)(err[j] & 0xff) << (8 * j);
        }
        if constexpr (kRec) {  // replay_end4_kernel's flags and s' fuel now; x / y held to the end
            rec_x = ox;
            rec_y = oy;
            uint32_t flags4 = 0;
            float nf[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool raised = err[j] != SE_ERR_OK;
                nf[j] = (float)f[j];
                flags4 |= (((dead >> j) & 1u ? (uint32_t)kRecDone : 0u) | (raised ? (uint32_t)kRecInvalid : 0u)) << (8 * j);
                rec_cut |= (uint32_t)raised << (8 * j);
            }
            record_early(late_args(), base, flags4, nf);
        }
        const se_state& S = A.st;
        __builtin_amdgcn_sched_barrier(0);  // the fuel halves back to back (store_moved)
        store4u8(S.x, at, ox);
        store4u8(S.y, at, oy);
        store4(S.fuel, at, f);
        store4u8(S.done, at, dn);
        store4u8(reinterpret_cast<uint8_t*>(S.err), at, ee);
        __builtin_amdgcn_sched_barrier(0);
    }
    TRACE_STAMP(6);

    // --- second half: cargo loss (_calculate_cargo_loss :169-200), contract v5: the
    // r-th env of the quad whose gate fired takes block LOSS_r (word 0 the loss type,
    // words 1-3 the Beta(2, 2) uniforms); only waves with a firing gate run it
    [[maybe_unused]] uint32_t used_loss = 0, used_beta = 0;
    if constexpr (kReplay) {
        if (fire) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool fj = (fire >> j) & 1u;
                const double lt = tt[j], beta = tb[j];
                const bool partial = (cg[j] != 0) & (lt >= 0.1) & (lt <= 0.9);
                const int part = (int)(beta * (double)cg[j]);  // int(betavariate(2,2) * cargo) (:195-197)
                const int some = lt > 0.9 ? cg[j] : part;
                const int loss = ((lt < 0.1) | (cg[j] == 0)) ? 0 : some;
                const double rl = r[j] + (double)loss * -3.0;
                r[j] = fj ? rl : r[j];
                cg[j] = fj ? cg[j] - loss : cg[j];
                used_loss |= (uint32_t)fj << j;
                used_beta |= (uint32_t)(fj & partial) << j;
                need |= (uint32_t)(fj & ((lt != lt) | (partial & (beta != beta)))) << j;
            }
        }
    } else if (fire) {
        uint32_t lt[4], v1[4], v2[4], v3[4];
        const uint32_t rk[4] = {0u, fire & 1u, (uint32_t)__popc(fire & 3u), (uint32_t)__popc(fire & 7u)};
        U4 rr = kSpecLoss ? D.loss0 : draw(qk, t, loss_slot(0));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            lt[j] = rr.v[0];
            v1[j] = rr.v[1];
            v2[j] = rr.v[2];
            v3[j] = rr.v[3];
        }
#pragma unroll
        for (uint32_t q = 1; q < 4; ++q) {
            if (__popc(fire) > q) {
                rr = draw(qk, t, loss_slot(q));
#pragma unroll
                for (int j = (int)q; j < 4; ++j) {
                    const bool take = rk[j] >= q;
                    lt[j] = take ? rr.v[0] : lt[j];
                    v1[j] = take ? rr.v[1] : v1[j];
                    v2[j] = take ? rr.v[2] : v2[j];
                    v3[j] = take ? rr.v[3] : v3[j];
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            // beta = the median of the three words * 2^-32 (the conversion is monotone)
            const uint32_t lo = min(v1[j], v2[j]), hi = max(v1[j], v2[j]);
            const uint32_t med = max(lo, min(hi, v3[j]));  // v_med3_u32
            const int part = beta_part(med, cg[j]);
            const int some = lt[j] > kTypeHi ? cg[j] : part;
            const int loss = lt[j] < kTypeLo ? 0 : some;
            const bool fj = (fire >> j) & 1u;
            const double rl = r[j] + (double)loss * -3.0;  // int(loss * -3) exactly, then += (:323)
            r[j] = fj ? rl : r[j];
            cg[j] = fj ? cg[j] - loss : cg[j];
        }
    }
    // arrival (:325-337): +2 cargo, cargo 0, origin = dest, a new destination != origin
    if (arrive) {
        [[maybe_unused]] U4 ab{{0u, 0u, 0u, 0u}};
        if constexpr (!kReplay) ab = draw(qk, t, kSlotArrive);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool aj = (arrive >> j) & 1u;
            const double ra = (r[j] + (double)(2 * cg[j])) + 10.0;
            int nd;
            if constexpr (kReplay) {
                nd = td[j];
                need |= (uint32_t)(aj & (nd < 0)) << j;
            } else {
                nd = pick_other(ab.v[j], P, dst[j]);
            }
            r[j] = aj ? ra : r[j];
            cg[j] = aj ? 0 : cg[j];
            org[j] = aj ? dst[j] : org[j];
            dst[j] = aj ? nd : dst[j];
        }
    }
    float rw[4], epr[4];
    int32_t epl[4];  // kRec: the running length after this step (0 for a finished episode)
    uint32_t oo = 0, od = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        rw[j] = (float)r[j];  // one rounding of the reference's f64 reward
        epr[j] = 0.0f;
        epl[j] = 0;
        if constexpr (kAuto) {
            const bool fj = (fin >> j) & 1u;
            F.ret[j] = G.e[j] + rw[j];
            F.len[j] = (int32_t)(t + 1u - G.l[j]);  // stamps are loaded where fin (kRec: everywhere)
            if (fj) {
                bs.ret += (double)F.ret[j];
                bs.eps += 1;
                bs.len += F.len[j];
            }
            epr[j] = fj ? 0.0f : F.ret[j];
            epl[j] = fj ? 0 : F.len[j];
            cg[j] = fj ? 0 : cg[j];
            org[j] = fj ? byte_of(reset_o, j) : org[j];
            dst[j] = fj ? byte_of(reset_d, j) : dst[j];
        }
        oo |= (uint32_t)(org[j] & 0xff) << (8 * j);
        od |= (uint32_t)(dst[j] & 0xff) << (8 * j);
    }
    if constexpr (kAuto) F.mask = fin;
    const se_state& S = late_args().st;
    store4u8(S.origin, at, oo);
    store4u8(S.dest, at, od);
    store4(S.cargo, at, cg);
    store4(S.reward, at, rw);
    if constexpr (kAuto) {
        store4(S.ep_return, at, epr);
        store_stamps(S, at, G.l, fin, t, stamp_lane(fin));
    }
    if constexpr (kRec) F.cut = record_group(late_args(), base, rw, rec_x, rec_y, oo, od, rec_cut, epl);
    if constexpr (kReplay) {
        se_tape* tp = A.tape + base;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (!(kFull || base + j < n)) continue;
            const bool mv = do_move[j];
            tp[j].used = (int32_t)((mv ? (uint32_t)kUsedFuelGate : 0u) | (moved[j] ? (uint32_t)kUsedMoved : 0u) |
                                   (((used_loss >> j) & 1u) ? (uint32_t)kUsedLossType : 0u) |
                                   (((used_beta >> j) & 1u) ? (uint32_t)kUsedBeta : 0u) |
                                   (((arrive >> j) & 1u) ? (uint32_t)kUsedArrive : 0u));
            if ((need >> j) & 1u) {  // the env as it was: later stores of this thread win
                const int64_t i = base + j;
                S.x[i] = (uint8_t)byte_of(G.x, j);
                S.y[i] = (uint8_t)byte_of(G.y, j);
                S.fuel[i] = G.f[j];
                S.cargo[i] = G.c[j];
                S.origin[i] = (uint8_t)byte_of(G.org, j);
                S.dest[i] = (uint8_t)byte_of(G.dst, j);
                S.reward[i] = 0.0f;
                S.done[i] = 0;
                S.err[i] = (int8_t)SE_ERR_NEED_DRAW;
            }
        }
    }
}

// Sum over the wave's 64 lanes in a fixed tree, so the result does not depend on
// timing: within each row of 16 lanes, DPP exchanges with lane^1, lane^2, the
// mirrored lane of the half row and of the row (every lane then holds its row's
// sum; each exchange pairs two lanes symmetrically and f64 addition commutes, so
// both hold identical bits), then the four row sums as (r0 + r1) + (r2 + r3).
// No LDS round trips (a shuffle butterfly cost 36 ds_bpermute and 6 dependent
// waits at the end of every wave).
template <int kCtrl>
__device__ __forceinline__ double dpp_f64(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)b, kCtrl, 0xf, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), kCtrl, 0xf, 0xf, false);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
constexpr int kDppXor1 = 0xb1;        // quad_perm [1, 0, 3, 2]
constexpr int kDppXor2 = 0x4e;        // quad_perm [2, 3, 0, 1]
constexpr int kDppHalfMirror = 0x141; // row_half_mirror
constexpr int kDppMirror = 0x140;     // row_mirror
__device__ __forceinline__ double wave_sum(double v) {
    v += dpp_f64<kDppXor1>(v);
    v += dpp_f64<kDppXor2>(v);
    v += dpp_f64<kDppHalfMirror>(v);
    v += dpp_f64<kDppMirror>(v);
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    double r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, 16 * k);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), 16 * k);
        r[k] = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
    }
    return (r[0] + r[1]) + (r[2] + r[3]);
}
__device__ __forceinline__ int wave_sum_int(int v) {
    v += __builtin_amdgcn_mov_dpp(v, kDppXor1, 0xf, 0xf, false);
    v += __builtin_amdgcn_mov_dpp(v, kDppXor2, 0xf, 0xf, false);
    v += __builtin_amdgcn_mov_dpp(v, kDppHalfMirror, 0xf, 0xf, false);
    v += __builtin_amdgcn_mov_dpp(v, kDppMirror, 0xf, 0xf, false);
    return (__builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16)) +
           (__builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48));
}

// Statistics slab update: lanes 0-2 of each wave load the
// wave's entry at the kernel's start and store old + sum at its end (plain loads and stores;
// the entry is this wave's alone during a launch). At N = 2^24 the three no-return f64
// atomics per wave (memory-side 64-B requests) cost config 4 ~16 us of ~190
// (a timing-only ablation, profiles/r04/c4split.jsonl).
// slab[i] += v without reading it back into the wave: the add runs in L2 and the
// wave does not wait for it. Only this wave's lane 0 adds to its own entry during
// a launch (step_tail_kernel adds in a later launch), so the order of additions is
// fixed and the sums are deterministic.
__device__ __forceinline__ void slab_add(double* p, double v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Done-list compaction of one iteration (auto-reset): no atomics, no LDS and no
// barrier. A wave-exclusive prefix of the per-lane counts (0..4) comes from three
// ballot bit-planes; the records go to this wave's own segment of the list in env
// order (deterministic). An earlier version ranked the waves of a workgroup through
// LDS behind two barriers: 1.4 us of a 15.4 us config-4 step.
__device__ __forceinline__ void wave_compact(const StepArgs& A, const Finished& F, int64_t base,
                                             int64_t segment) {
    const int nd = __popc(F.mask);
    const uint64_t b0 = __ballot(nd & 1), b1 = __ballot(nd & 2), b2 = __ballot(nd & 4);
    if (nd) {
        int64_t slot = segment * A.seg + (int32_t)(count_below(b0) + 2 * count_below(b1) + 4 * count_below(b2));
        const int32_t t = (int32_t)A.t;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if ((F.mask >> j) & 1u) A.done_recs[slot++] = se_done_rec{(int32_t)(base + j), F.ret[j], F.len[j], t};
    }
    const int32_t total = (int32_t)(__popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2));
    if (A.done_pad > 1) {  // launch-uniform (done_pad_records)
        // the wave's records padded to whole lines with filler records (env -1) past the
        // count: a line of the list written in part by one wave leaves L2 as a partial-line
        // write, and at N = 2^24 the ~1 record per wave cost config 4 ~11 us of ~192
        // (a timing-only ablation, profiles/r04/ab_c4parts.jsonl). A segment holds 256
        // records, a multiple of the pad, so the filler stays inside it.
        const int32_t pad = (-total) & (A.done_pad - 1), l = (int32_t)(threadIdx.x & 63);
        if (total != 0 && l < pad)
            A.done_recs[segment * A.seg + total + l] = se_done_rec{-1, 0.0f, 0, (int32_t)A.t};
    }
    if ((threadIdx.x & 63) == 0) A.done_count[segment] = total;
}

// Workgroup b owns the contiguous groups [b*iters*256, (b+1)*iters*256) (a group is
// 4 consecutive envs, one lane per group per iteration). In iteration k, wave w
// steps the 64 groups from b*iters*256 + k*256 + w*64: its done-list segment
// (segment = global group / 64) covers them in env order, so the concatenated
// segments are globally sorted. Every field of a group is one 4- or
// 16-byte lane access. The partial last group (n % 4 envs) is left to
// step_tail_kernel, so this loop carries no guarded scalar path. The world image's
// loads, then the first group's, are all in flight before the LDS writes; each
// iteration loads the next group after storing the current one.
// kSeq: the same code, instantiated apart for se_step_seq's launches (the agent path without
// auto-reset), so a kernel trace lists them under a name of their own: bench.py's headline leg
// issues its timed steps that way, and its trace row then holds exactly those launches.
template <bool kTyped, bool kReplay, bool kAuto, bool kNt = false, bool kRec = false, bool kSeq = false>
__global__ __launch_bounds__(kStepBlock) __attribute__((amdgpu_waves_per_eu(4))) void step_kernel(StepArgs A) {
    static_assert(!kRec || (kAuto && !kTyped && !kReplay), "se_step_record: agent actions, auto-reset");
    extern __shared__ uint32_t lds[];
    const int64_t full = A.n >> 2;
    const int64_t first = (int64_t)blockIdx.x * A.iters * kStepBlock;  // block-uniform first group

    TRACE_STAMP(0);
    const Staged st = stage_issue(A.world);
    // the image's loads first: the staging writes then wait for them alone
    __builtin_amdgcn_sched_barrier(0);
    // first group: an unconditional load (lanes past the end re-read the last full
    // group; the host launches this kernel only when there is one), so the staging
    // writes below wait for exactly the image's loads
    Group<kTyped, kAuto, kNt> G;
    {
        const int64_t last = full - 1 - first;  // block-uniform
        const uint32_t lane = last < (int64_t)threadIdx.x ? (uint32_t)(last < 0 ? 0 : last) : threadIdx.x;
        G.template load<true>(A, At<true>{last < 0 ? full - 1 : first, 0, A.n}, lane);
    }
    __builtin_amdgcn_sched_barrier(0);
    // auto-reset: this wave's statistics so far ({sum ret, episodes, sum len} on lanes 0-2),
    // loaded now so the end of the wave adds to them without waiting
    // (kRec keeps the atomics: two more registers there spilled)
    constexpr bool kSlabRmw = kAuto && !kRec;
    [[maybe_unused]] double slab_prev = 0.0;
    if constexpr (kSlabRmw) {
        const uint32_t l = threadIdx.x & 63;
        const double* sl = late_args().slab + 4 * (blockIdx.x * (kStepBlock / 64) + (threadIdx.x >> 6));
        slab_prev = sl[l < 3 ? l : 0];
    }
    // agent-index actions: the production step, or its replay-tape form (parity)
    constexpr bool kAgent = !kTyped;
    constexpr bool kDraws = kAgent && !kReplay;
    Draws D{};
    if constexpr (kDraws) {
        D = early_draws<spec_loss<kAuto>()>(A, (first + threadIdx.x) * 4);
        // keep the draws ahead of the staging wait: they overlap the loads in flight
        asm volatile("" : "+v"(D.fuel.v[0]), "+v"(D.gate.v[0]), "+v"(D.loss0.v[0]), "+v"(D.arrive.v[0]));
    }
    const LdsWorld w = stage_finish(A.world, A.dims, lds, st);
    TRACE_STAMP(1);

    BlockStats bs;
    uint32_t cuts = 0;  // kRec: bit 4k + j = env j of this thread's group k restarts
    for (int64_t k = 0; k < A.iters; ++k) {
        const int64_t g0 = first + k * kStepBlock, g = g0 + threadIdx.x;
        Finished F;
        const bool more = k + 1 < A.iters && g + kStepBlock < full;
        if (g < full) {
            if constexpr (kAgent) {
                if constexpr (kDraws) {
                    if (k > 0) D = early_draws<spec_loss<kAuto>()>(A, g * 4);
                }
                step_group_agent<kAuto, true, kNt, kRec, kReplay>(A, w, G, At<true>{g0, g * 4, A.n}, bs, F, D);
                if constexpr (kRec) cuts |= F.cut << (4 * k);
            } else
                step_group<kTyped, kReplay, kAuto, true, kNt>(A, w, G, At<true>{g0, g * 4, A.n}, bs, F);
            if (k == 0) TRACE_STAMP(2);
            if (more) G.template load<true>(A, At<true>{g0 + kStepBlock, 0, A.n});
        }
        // done-list segment of this (iteration, wave): 64 groups, in env order
        if constexpr (kAuto) wave_compact(late_args(), F, g * 4, __builtin_amdgcn_readfirstlane((int32_t)(g >> 6)));
    }

#if SHIPENV_TRACE
    __builtin_amdgcn_s_waitcnt(0);  // stores acknowledged
    TRACE_STAMP(3);
#endif
    if constexpr (kRec) {  // the ring's stored count, read by the sampler (replay_end4_kernel)
        if (blockIdx.x == 0 && threadIdx.x == 0) *late_args().rec.d_size = late_args().rec.new_size;
        if (cuts) record_restart(late_args(), w, cuts);
    }
    if (kAuto) {
        // per-wave statistics: a fixed-order tree (wave_sum), added to this wave's own
        // slab entry. With episodes ending about once per 240 steps, most waves have one
        // lane with a finished episode or none: then that lane's values are the sums
        // (every other lane adds +0.0, which the tree's f64 adds leave exact), read
        // with three readlanes instead of three trees.
        const uint64_t ended = __ballot(bs.eps != 0);
        if (ended == 0) return;
        double ret, len;
        int eps;
        if ((ended & (ended - 1)) == 0) {
            const int src = __builtin_ctzll(ended);
            const uint64_t rb = __builtin_bit_cast(uint64_t, bs.ret);
            ret = __builtin_bit_cast(double, (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(rb >> 32), src) << 32 |
                                                 (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)rb, src));
            len = (double)__builtin_amdgcn_readlane(bs.len, src);
            eps = __builtin_amdgcn_readlane(bs.eps, src);
        } else {
            ret = wave_sum(bs.ret);
            len = wave_sum((double)bs.len);
            eps = wave_sum_int(bs.eps);
        }
        if constexpr (!kSlabRmw) {
            if (eps != 0 && (threadIdx.x & 63) == 0) {
                double* sl = late_args().slab + 4 * (blockIdx.x * (kStepBlock / 64) + (threadIdx.x >> 6));
                slab_add(sl + 0, ret);
                slab_add(sl + 1, (double)eps);
                slab_add(sl + 2, len);
            }
        } else if (eps != 0 && (threadIdx.x & 63) < 3) {
            // the same additions in the same order as a read-modify-write from registers:
            // lanes 0-2 hold the entry's old values (loaded at the kernel's start), and no
            // other wave touches this entry during the launch
            const uint32_t l = threadIdx.x & 63;
            double* sl = late_args().slab + 4 * (blockIdx.x * (kStepBlock / 64) + (threadIdx.x >> 6));
            sl[l] = slab_prev + (l == 0 ? ret : l == 1 ? (double)eps : len);
        }
    }
}

// The partial last group (n % 4 envs), launched after step_kernel on the same
// stream when n % 4 != 0: one thread steps it with guarded scalar accesses. Its
// envs come last in env order, so auto-reset appends their records to the done
// segment of group n/4 after step_kernel's and adds their statistics to the slab
// entry of the wave that owns that group (env order and a fixed summation order,
// as in the main kernel).
template <bool kTyped, bool kReplay, bool kAuto>
__device__ __forceinline__ void step_tail_envs(const StepArgs& A, const LdsWorld& w) {
    // at most 3 envs: step_tail_kernel reads the world in place (L2), not staged, so the step
    // starts without the staging round trips (the N = 1 launch path is this kernel alone)
    const int64_t g = A.n >> 2;
    const At<false> at{0, g * 4, A.n};
    Group<kTyped, kAuto> G;
    G.template load<false>(A, at);
    BlockStats bs;
    Finished F;
    if constexpr (!kTyped && !kReplay)
        step_group_agent<kAuto, false, false>(A, w, G, at, bs, F, early_draws<spec_loss<kAuto>()>(A, at.base));
    else if constexpr (!kTyped && kReplay)
        step_group_agent<kAuto, false, false, false, true>(A, w, G, at, bs, F, Draws{});
    else
        step_group<kTyped, kReplay, kAuto, false>(A, w, G, at, bs, F);
    if constexpr (kAuto) {
        const int64_t b = g >> 6;  // the (iteration, wave) segment that owns group g
        int32_t c = (g & 63) == 0 ? 0 : A.done_count[b];  // a fresh segment: step_kernel wrote none
        for (int j = 0; j < 4; ++j)
            if ((F.mask >> j) & 1u)
                A.done_recs[b * A.seg + c++] = se_done_rec{(int32_t)(at.base + j), F.ret[j], F.len[j], (int32_t)A.t};
        A.done_count[b] = c;
        if (bs.eps != 0) {
            // the slab entry of the wave that owns group g
            const int64_t bl = g / (A.iters * kStepBlock), wv = (g % kStepBlock) >> 6;
            double* sl = A.slab + 4 * (bl * (kStepBlock / 64) + wv);
            sl[0] += bs.ret;
            sl[1] += (double)bs.eps;
            sl[2] += (double)bs.len;
        }
    }
}

template <bool kTyped, bool kReplay, bool kAuto>
__global__ __launch_bounds__(64) void step_tail_kernel(StepArgs A) {
    if (threadIdx.x != 0) return;
    step_tail_envs<kTyped, kReplay, kAuto>(A, world_view(A.dims, A.world));
}

// Contiguous copy of the last step's done lists (se_done_compact), in two launches:
// done_scan_kernel (one workgroup) turns the per-segment counts into exclusive
// offsets, chunk by chunk in segment order; done_copy_kernel copies segment s to
// out[offsets[s]...], one wave per segment.
__global__ __launch_bounds__(1024) void done_scan_kernel(const int32_t* __restrict__ counts, int64_t nseg,
                                                         int32_t* __restrict__ offsets,
                                                         int32_t* __restrict__ out_count) {
    __shared__ int32_t part[1024];
    const int64_t chunk = (nseg + 1023) / 1024;
    const int64_t lo = (int64_t)threadIdx.x * chunk, hi = lo + chunk < nseg ? lo + chunk : nseg;
    int32_t sum = 0;
    for (int64_t i = lo; i < hi; ++i) sum += counts[i];
    part[threadIdx.x] = sum;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // inclusive Hillis-Steele scan of the chunk sums
        const int32_t v = threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    int32_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
    for (int64_t i = lo; i < hi; ++i) {
        offsets[i] = run;
        run += counts[i];
    }
    if (threadIdx.x == 1023) *out_count = part[1023];
}

__global__ __launch_bounds__(kBlock) void done_copy_kernel(const se_done_rec* __restrict__ recs,
                                                           const int32_t* __restrict__ counts,
                                                           const int32_t* __restrict__ offsets, int64_t nseg,
                                                           int64_t seg, se_done_rec* __restrict__ out) {
    const int64_t s = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if (s >= nseg) return;
    const int32_t cnt = counts[s], start = offsets[s];
    for (int i = threadIdx.x & 63; i < cnt; i += 64) out[start + i] = recs[s * seg + i];
}

// ------------------------------------------------------------------ reset kernel
struct ResetArgs {
    const uint32_t* world;
    WorldDims dims;
    int64_t n, env_base;
    uint64_t seed;
    uint32_t epoch;
    uint32_t t;  // the step counter: the first step of the new episodes
    se_state st;
    const uint8_t* mask;
    const int32_t* origin_in;  // explicit values (se_reset_to) or NULL
    const int32_t* dest_in;
};

// The world is read in place (only the port positions, for the envs being reset): staged
// per workgroup as the other kernels do, it cost 2048 x 10.8 KB of L2 reads per launch,
// the whole launch when a mask selects a few envs (the training loop's episode cuts).
__device__ __forceinline__ void reset_env(const ResetArgs& A, const LdsWorld& w, int64_t i) {
    {
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
        if (A.st.ep_start) A.st.ep_start[i] = (int32_t)A.t;
        A.st.done[i] = 0;
        A.st.err[i] = 0;
        A.st.reward[i] = 0.0f;
    }
}

__global__ __launch_bounds__(kBlock) void reset_kernel(ResetArgs A) {
    const LdsWorld w = world_view(A.dims, A.world);
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < A.n;
         i += (int64_t)gridDim.x * kBlock) {
        if (A.mask && !A.mask[i]) continue;
        reset_env(A, w, i);
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
            v = f == 0 ? (float)w.px(p) : f == 1 ? (float)w.py(p) : f == 2 ? (float)w.pfuel(p) : (float)w.pcargo(p);
        }
        A.obs[i * A.ld + c] = v;
    }
}

// Rows of a 256-row tile are contiguous in a dense [n][W] output, so a workgroup
// builds its tile's values once and writes them with 16-byte stores in address order
// (every wave store a full 1 KB run). The generic kernels above / below (one thread per
// output element or byte) serve any other row stride; they measured 117 us (observe,
// P = 5) and 321 us (mask) at 2^20 envs against 22 us and 7 us of HBM writes.
constexpr int kTileRows = 256;  // = kBlock: one row per thread in the per-row phase

// x / W for x < kTileRows * W, W <= 1022, as one multiply-high (exact: checked for every
// such x and W)
__device__ __forceinline__ uint32_t div_tile(uint32_t x, uint32_t magic) { return __umulhi(x, magic); }

// preprocess_state rows, dense ld == W = 6 + 4P: the tile's ship columns (6 floats a row)
// and the constant port block (4P floats) in LDS, then float4 stores
__global__ __launch_bounds__(kBlock) void observe_tiled_kernel(ObsArgs A, uint32_t magic) {
    extern __shared__ float olds[];
    const LdsWorld w = world_view(A.dims, A.world);  // only the port table is read
    const int W = 6 + 4 * w.P;
    float* ship = olds;                  // [kTileRows][6]
    float* pblk = olds + kTileRows * 6;  // [4P]
    for (int c = threadIdx.x; c < 4 * w.P; c += kBlock) {
        const int p = c >> 2, f = c & 3;
        pblk[c] = f == 0 ? (float)w.px(p) : f == 1 ? (float)w.py(p) : f == 2 ? (float)w.pfuel(p) : (float)w.pcargo(p);
    }
    for (int64_t r0 = (int64_t)blockIdx.x * kTileRows; r0 < A.n; r0 += (int64_t)gridDim.x * kTileRows) {
        const int rows = (int)min((int64_t)kTileRows, A.n - r0);
        __syncthreads();  // the previous tile's reads of `ship` are done
        if ((int)threadIdx.x < rows) {
            const int64_t i = r0 + threadIdx.x;
            const float fuel = (float)A.st.fuel[i];  // "cargo" is self.fuel (environment.py:206)
            const uint8_t o = A.st.origin[i], d = A.st.dest[i];
            float* sr = ship + threadIdx.x * 6;
            sr[0] = (float)A.st.x[i];
            sr[1] = (float)A.st.y[i];
            sr[2] = fuel;
            sr[3] = fuel;
            sr[4] = o == SE_NONE ? -1.0f : (float)o;
            sr[5] = d == SE_NONE ? -1.0f : (float)d;
        }
        __syncthreads();
        const uint32_t nf = (uint32_t)(rows * W);  // W is even: whole float4 runs when rows is
        float4* out = reinterpret_cast<float4*>(A.obs + r0 * W);
        for (uint32_t q = threadIdx.x; 4 * q < nf; q += kBlock) {
            const uint32_t j = 4 * q;
            uint32_t r = div_tile(j, magic);
            int c = (int)(j - r * W);
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[e] = c < 6 ? ship[r * 6 + c] : pblk[c - 6];
                if (++c == W) {
                    c = 0;
                    ++r;
                }
            }
            if (j + 4 <= nf) {
                out[q] = make_float4(v[0], v[1], v[2], v[3]);
            } else {  // the last run of a ragged tile: 2 floats (rows * W is even)
                A.obs[r0 * W + j] = v[0];
                A.obs[r0 * W + j + 1] = v[1];
            }
        }
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
                v = cur >= 0 && amt > 0 && amt <= w.pcargo(cur);
            } else {
                const int amt = a - (4 + P + 50);
                v = cur >= 0 && amt > 0 && amt <= w.pfuel(cur);
            }
            out |= (uint32_t)v << (7 - bit);
        }
        A.bits[k] = (uint8_t)out;
    }
}

// bits i of [0, 32) with lo <= i <= hi (lo, hi any ints)
__device__ __forceinline__ uint32_t bits_in(int lo, int hi) {
    lo = max(lo, 0);
    hi = min(hi, 31);
    if (lo > hi) return 0u;
    const uint32_t top = hi >= 31 ? 0xffffffffu : ((1u << (hi + 1)) - 1u);
    return top & ~((1u << lo) - 1u);
}

// is_valid_action bits, dense rows of S bytes: each thread builds its row 32 actions at a
// time (a word whose bit o is action 32k + o, then bit-reversed and byte-swapped into the
// MSB-first byte order of np.packbits), writes its S bytes into the LDS tile, then the
// workgroup stores the tile with 16-byte writes.
__global__ __launch_bounds__(kBlock) void valid_mask_tiled_kernel(MaskArgs A) {
    extern __shared__ uint8_t mlds[];  // [kTileRows][S] (+ pad to 16 bytes)
    __shared__ uint64_t same[64];  // P <= 64: bit q of same[p] = port q stands on port p's cell
    const LdsWorld w = world_view(A.dims, A.world);
    const int P = w.P, S = A.stride, nw = (S + 3) / 4;
    const int c_lo = 5 + P, f_lo = 55 + P;  // TAKE_CARGO / TAKE_FUEL amount 1
    const bool masks = P <= 64;  // the SELECT rows as one shifted mask per env (else a scan)
    if (masks && (int)threadIdx.x < P) {
        uint64_t m = 0;
        for (int q = 0; q < P; ++q) m |= (uint64_t)(w.pos[q] == w.pos[threadIdx.x]) << q;
        same[threadIdx.x] = m;
    }
    for (int64_t r0 = (int64_t)blockIdx.x * kTileRows; r0 < A.n; r0 += (int64_t)gridDim.x * kTileRows) {
        const int rows = (int)min((int64_t)kTileRows, A.n - r0);
        __syncthreads();  // the previous tile's stores have read the LDS tile
        if ((int)threadIdx.x < rows) {
            const int64_t i = r0 + threadIdx.x;
            const int x = A.st.x[i], y = A.st.y[i];
            const int origin = A.st.origin[i] == SE_NONE ? -1 : A.st.origin[i];
            const int cur = w.port_at(x, y);  // the first port on the ship's cell
            const int cst = cur >= 0 ? w.pcargo(cur) : 0, fst = cur >= 0 ? w.pfuel(cur) : 0;
            const uint32_t spos = (uint32_t)x | ((uint32_t)y << 16);
            // SELECT p: every port on the ship's cell but the origin (dqn.py:152-161)
            const uint64_t sel = masks && cur >= 0 ? same[cur] & ~(origin >= 0 ? 1ull << origin : 0ull) : 0ull;
            uint8_t* row = mlds + threadIdx.x * S;
            for (int k = 0; k < nw; ++k) {
                const int b = 32 * k;
                uint32_t m = bits_in(-b, 3 - b);  // moves: always
                if (cur >= 0) {
                    m |= bits_in(c_lo - b, c_lo + min(cst, 49) - 1 - b) | bits_in(f_lo - b, f_lo + min(fst, 199) - 1 - b);
                    if (masks) {  // rows 4 + p: sel shifted by 4 - b
                        const int sh = b - 4;
                        m |= (uint32_t)(sh < 0 ? sel << -sh : (sh < 64 ? sel >> sh : 0ull));
                    } else {
                        const int p0 = max(cur, b - 4), p1 = min(P, b + 28);
                        for (int p = p0; p < p1; ++p)
                            if (w.pos[p] == spos && p != origin) m |= 1u << (4 + p - b);
                    }
                }
                const uint32_t word = __builtin_amdgcn_perm(0u, __builtin_bitreverse32(m), 0x00010203u);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (4 * k + j < S) row[4 * k + j] = (uint8_t)(word >> (8 * j));
            }
        }
        __syncthreads();
        const uint32_t nb = (uint32_t)(rows * S);
        uint8_t* out = A.bits + r0 * S;
        const uint4* src = reinterpret_cast<const uint4*>(mlds);
        for (uint32_t q = threadIdx.x; 16 * q < nb; q += kBlock) {
            if (16 * q + 16 <= nb) {
                reinterpret_cast<uint4*>(out)[q] = src[q];
            } else {
                for (uint32_t b = 16 * q; b < nb; ++b) out[b] = mlds[b];
            }
        }
    }
}

// Row templates (round 5). A row of is_valid_action bits depends on the ship's state only
// through (cur, origin): cur = the first port on the ship's cell (-1 at sea) fixes the
// TAKE_* amounts (its stocks) and the SELECT rows (every port on its cell), and the origin
// clears its own SELECT bit when it stands on that cell (dqn.py:152-161). So every row is
// one of 1 + P + sum_p |same[p]| templates: template 0 the moves alone, 1 + p port p's
// cell with no origin on it, and 1 + P + pbase[p] + rank(o) port p's cell with origin o
// cleared. mask_tmpl_kernel builds them once per world image into a device buffer:
//   [0, 512)    same[64]: bit q of same[p] = port q stands on port p's cell
//   [512, 772)  pbase[65]: prefix counts of |same[p]|
//   [1024, ...) ntmpl blocks of TB bytes: 16 zero bytes, the S row bytes in np.packbits
//               order, then zeros to the block's end (TB = round16(S + 35))
// so that a 16-byte window read at any byte offset of [0, 16 + S) of a block holds the
// row's bytes from that offset on, zeros before the row and after it.
constexpr int kMaskHdr = 1024;
__host__ __device__ constexpr int mask_tb(int S) { return (S + 35 + 15) & ~15; }
constexpr int kMaskTmplMax = 320;  // templates held in LDS (P = 64 on distinct cells: 129)

// the bits of actions [b, b + 32) of a row (bit o = action b + o), in packbits byte order
__device__ __forceinline__ uint32_t mask_word(int b, int cur, int cst, int fst, uint64_t sel, int P) {
    uint32_t m = bits_in(-b, 3 - b);  // moves: always
    if (cur >= 0) {
        const int c_lo = 5 + P, f_lo = 55 + P;  // TAKE_CARGO / TAKE_FUEL amount 1
        m |= bits_in(c_lo - b, c_lo + min(cst, 49) - 1 - b) | bits_in(f_lo - b, f_lo + min(fst, 199) - 1 - b);
        const int sh = b - 4;  // rows 4 + p: sel shifted by 4 - b
        m |= (uint32_t)(sh < 0 ? (-sh < 64 ? sel << -sh : 0ull) : (sh < 64 ? sel >> sh : 0ull));
    }
    return __builtin_amdgcn_perm(0u, __builtin_bitreverse32(m), 0x00010203u);
}

__global__ __launch_bounds__(kBlock) void mask_tmpl_kernel(const uint32_t* world, WorldDims d, int S,
                                                           uint8_t* buf) {
    const LdsWorld w = world_view(d, world);
    const int P = w.P, TB = mask_tb(S);
    __shared__ uint64_t same[64];
    __shared__ uint32_t pbase[65];
    if ((int)threadIdx.x < P) {
        uint64_t m = 0;
        for (int q = 0; q < P; ++q) m |= (uint64_t)(w.pos[q] == w.pos[threadIdx.x]) << q;
        same[threadIdx.x] = m;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        pbase[0] = 0;
        for (int p = 0; p < P; ++p) pbase[p + 1] = pbase[p] + (uint32_t)__popcll(same[p]);
    }
    __syncthreads();
    if ((int)threadIdx.x < 64) reinterpret_cast<uint64_t*>(buf)[threadIdx.x] = (int)threadIdx.x < P ? same[threadIdx.x] : 0ull;
    if ((int)threadIdx.x <= 64) reinterpret_cast<uint32_t*>(buf + 512)[threadIdx.x] = (int)threadIdx.x <= P ? pbase[threadIdx.x] : 0u;
    const int ntmpl = 1 + P + (int)pbase[P], wpt = TB / 4;
    uint32_t* out = reinterpret_cast<uint32_t*>(buf + kMaskHdr);
    for (int k = threadIdx.x; k < ntmpl * wpt; k += kBlock) {
        const int t = k / wpt, c = 4 * (k - t * wpt) - 16;  // the word's first row byte
        int cur = -1;
        uint64_t sel = 0;
        if (t >= 1 && t <= P) {
            cur = t - 1;
            sel = same[cur];
        } else if (t > P) {
            const uint32_t j = (uint32_t)(t - 1 - P);
            int p = 0;
            while (pbase[p + 1] <= j) ++p;
            uint64_t m = same[p];
            for (uint32_t r = j - pbase[p]; r > 0; --r) m &= m - 1;  // the rank-th port of the cell
            cur = p;
            sel = same[p] & ~(m & (~m + 1));
        }
        uint32_t word = 0;
        if (c >= 0 && c < S) {
            word = mask_word(8 * c, cur, cur >= 0 ? w.pcargo(cur) : 0, cur >= 0 ? w.pfuel(cur) : 0, sel, P);
            const int keep = S - c;  // bytes of the word inside the row
            if (keep < 4) word &= (1u << (8 * keep)) - 1u;
        }
        out[k] = word;
    }
}

// 16 bytes of LDS from any byte offset (the blocks leave 4 spare bytes past every window)
__device__ __forceinline__ uint4 lds_window(const uint32_t* l, uint32_t off) {
    const uint32_t a = off >> 2, sh = off & 3u;
    const uint32_t w0 = l[a], w1 = l[a + 1], w2 = l[a + 2], w3 = l[a + 3], w4 = l[a + 4];
    return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                      __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
}

// is_valid_action bits from the row templates: per 256-row tile, one thread per row looks up
// its template (desc: the block's byte offset in LDS), then one thread per 16-byte chunk of
// the tile's dense output ORs the windows of the (at most two) rows the chunk covers and
// stores it: S and 256 * S are such that a chunk never spans three rows or two tiles.
__global__ __launch_bounds__(kBlock) void valid_mask_tmpl_kernel(MaskArgs A, const uint8_t* __restrict__ buf,
                                                                 int ntmpl, uint32_t magic) {
    extern __shared__ uint32_t tl[];  // [ntmpl * TB / 4] templates
    __shared__ uint64_t same[64];
    __shared__ uint32_t pbase[64];
    __shared__ uint32_t desc[kTileRows + 1];
    const LdsWorld w = world_view(A.dims, A.world);
    const int P = w.P, S = A.stride, TB = mask_tb(S);
    {
        const uint4* src = reinterpret_cast<const uint4*>(buf + kMaskHdr);
        uint4* dst = reinterpret_cast<uint4*>(tl);
        for (int k = threadIdx.x; k < ntmpl * TB / 16; k += kBlock) dst[k] = src[k];
        if (threadIdx.x < 64) {
            same[threadIdx.x] = reinterpret_cast<const uint64_t*>(buf)[threadIdx.x];
            pbase[threadIdx.x] = reinterpret_cast<const uint32_t*>(buf + 512)[threadIdx.x];
        }
    }
    for (int64_t r0 = (int64_t)blockIdx.x * kTileRows; r0 < A.n; r0 += (int64_t)gridDim.x * kTileRows) {
        const int rows = (int)min((int64_t)kTileRows, A.n - r0);
        __syncthreads();  // the templates are in; the previous tile's chunks have read desc
        {
            uint32_t id = 0;
            if ((int)threadIdx.x < rows) {
                const int64_t i = r0 + threadIdx.x;
                const int cur = w.port_at(A.st.x[i], A.st.y[i]);
                const int o = A.st.origin[i];  // SE_NONE (255) is never on a cell
                if (cur >= 0) {
                    const uint64_t sm = same[cur];
                    const bool on = o < 64 && ((sm >> o) & 1ull);
                    id = on ? 1u + (uint32_t)P + pbase[cur] + (uint32_t)__popcll(sm & ((1ull << o) - 1ull))
                            : 1u + (uint32_t)cur;
                }
            }
            desc[threadIdx.x] = id * (uint32_t)TB;
            if (threadIdx.x == 0) desc[kTileRows] = 0;
        }
        __syncthreads();
        const uint32_t nb = (uint32_t)(rows * S);
        uint8_t* out = A.bits + r0 * S;
        for (uint32_t q = threadIdx.x; 16 * q < nb; q += kBlock) {
            const uint32_t c = 16 * q, r = div_tile(c, magic), c0 = c - r * (uint32_t)S;
            const uint4 a = lds_window(tl, desc[r] + 16u + c0);
            // the next row's bytes land at chunk offset S - c0; a window from before that
            // row's start reads its zero prefix (-16 at most: otherwise the chunk ends first)
            const int nx = max((int)c0 - S, -16);
            const uint4 b = lds_window(tl, desc[r + 1] + (uint32_t)(16 + nx));
            const uint4 v = make_uint4(a.x | b.x, a.y | b.y, a.z | b.z, a.w | b.w);
            if (c + 16 <= nb) {
                st_stream(reinterpret_cast<uint4*>(out + c), v);
            } else {  // the ragged tail of the last tile
                const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
                for (uint32_t k = 0; c + k < nb; ++k) out[c + k] = (uint8_t)(vv[k >> 2] >> (8 * (k & 3)));
            }
        }
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

// ------------------------------------------------------------------ random policy
// sample_action() (environment.py:245-263) on one env from one Philox word r.
__device__ __forceinline__ void sample_action(const LdsWorld& w, const Ship& s, uint32_t r, int& type,
                                              int& a, int& b) {
    const int cur = w.port_at(s.x, s.y);  // _get_current_port_idx (:145-153)
    a = 0;
    b = 0;
    if (s.dest == SE_NONE && cur >= 0) {  // :247-253, redraw while == current port
        type = w.P < 2 ? SE_SAMPLE_NO_OTHER_PORT : 2;
        a = pick_other(r, w.P, cur);
    } else if (s.cargo == 0 && cur >= 0) {  // :255-257, randint(1, port_cargo[idx]) :160
        const int stock = w.pcargo(cur);
        type = stock < 1 ? SE_SAMPLE_RAISES : 4;  // randint(1, 0): ValueError
        a = 1 + uniform_int(r, (uint32_t)max(stock, 1));
    } else if (s.fuel == 0.0 && cur >= 0) {  // :258-260: self.fuel[idx] raises TypeError (:163)
        type = SE_SAMPLE_RAISES;
    } else {  // random.choice([NORTH, EAST, SOUTH, WEST]) (:165-167, shipping/type.py:8-16)
        const int k = (int)(r & 3u), odd = k & 1;
        type = 1;
        a = odd * (k - 2);
        b = (1 - odd) * (k - 1);
    }
    if (type < 0) {  // no action: the reference raises / never returns
        a = 0;
        b = 0;
    }
}

struct SampleArgs {
    const uint32_t* world;
    WorldDims dims;
    int64_t n, env_base;
    uint64_t seed;
    uint32_t t;
    se_state st;
    int32_t* type;
    int32_t* a;
    int32_t* b;
};

// One cell-code byte and one stock per env: read in place through L1 / L2 instead of
// staging the 10.8 KB image into every one of up to 2048 workgroups.
__global__ __launch_bounds__(kBlock) void sample_kernel(SampleArgs A) {
    const LdsWorld w = world_view(A.dims, A.world);
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < A.n;
         i += (int64_t)gridDim.x * kBlock) {
        const Ship s{A.st.x[i], A.st.y[i], A.st.fuel[i], A.st.cargo[i], A.st.origin[i], A.st.dest[i]};
        const U4 d = draw(env_key(A.seed, A.env_base + i), A.t, kSlotSample);
        int ty, va, vb;
        sample_action(w, s, d.v[0], ty, va, vb);
        A.type[i] = ty;
        A.a[i] = va;
        A.b[i] = vb;
    }
}

// MCTS rollouts (agents/mcts.py:211-238), one per thread: a private copy of env
// src[r], then sample_action + step until done / max_steps counted steps /
// max_attempts attempts. A raising step is retried without counting (:231-233);
// a raising sample_action ends the rollout (it sits outside the try, :227).
struct RolloutArgs {
    const uint32_t* world;
    WorldDims dims;
    int64_t n, m, rollout_base;
    uint64_t seed;
    int32_t max_steps, max_attempts;
    se_state st;
    const int32_t* src;
    double* ret;
    int32_t* steps;
    int32_t* status;
};

__global__ __launch_bounds__(kBlock) void rollout_kernel(RolloutArgs A) {
    extern __shared__ uint32_t lds[];
    const LdsWorld w = stage_world(A.world, A.dims, lds);
    for (int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x; r < A.m;
         r += (int64_t)gridDim.x * kBlock) {
        const int64_t i = A.src[r];
        if (i < 0 || i >= A.n) {
            A.ret[r] = 0.0;
            A.steps[r] = 0;
            A.status[r] = SE_ROLL_BAD_SRC;
            continue;
        }
        Ship s{A.st.x[i], A.st.y[i], A.st.fuel[i], A.st.cargo[i], A.st.origin[i], A.st.dest[i]};
        const Key key = env_key(A.seed, A.rollout_base + r);
        double total = 0.0;
        int32_t steps = 0, status = SE_ROLL_ATTEMPTS;
        for (int32_t k = 0; k < A.max_attempts; ++k) {
            if (steps >= A.max_steps) {  // while not done and steps < max_rollout_steps (:225)
                status = SE_ROLL_MAX_STEPS;
                break;
            }
            const U4 d = draw(key, (uint32_t)k, kSlotRollout);
            int ty, va, vb;
            sample_action(w, s, d.v[0], ty, va, vb);
            if (ty < 0) {
                status = SE_ROLL_RAISED;
                break;
            }
            Pending p = env_begin<true, false>(w, s, SE_ERR_OK, ty, va, vb, (double)d.v[1], 0.0, d.v[2]);
            if (p.e != SE_ERR_OK) continue;  // except Exception: continue (state untouched)
            const int total_kind = d.v[3] > kTypeHi ? kLossTotal : kLossPartial;
            const int kind = d.v[3] < kTypeLo ? kLossNone : total_kind;
            uint32_t med = 0u;
            int nd = 0;
            if ((p.fires & (kind == kLossPartial)) | p.arrive) {
                const U4 e = draw(key, (uint32_t)k, kSlotRolloutB);
                const uint32_t lo = min(e.v[0], e.v[1]), hi = max(e.v[0], e.v[1]);
                med = max(lo, min(hi, e.v[2]));
                nd = pick_other(e.v[3], w.P, s.dest);
            }
            env_finish(s, p, kind, beta_part(med, s.cargo), nd, p.fires, p.arrive);
            total += p.r;  // total_reward += reward (:229)
            steps += 1;
            if (p.dead) {
                status = SE_ROLL_DONE;
                break;
            }
        }
        if (status == SE_ROLL_ATTEMPTS && steps >= A.max_steps) status = SE_ROLL_MAX_STEPS;
        A.ret[r] = total;
        A.steps[r] = steps;
        A.status[r] = status;
    }
}

// ------------------------------------------------------------------ stats reduce
// One workgroup sums the per-wave slab entries in a fixed order (thread t takes entries
// t, t + 1024, ... in turn; then a shuffle butterfly per wave and the 16 wave sums in
// wave order), so the result does not depend on timing. The slab has one entry per wave
// of the step grid: 4096 at 2^20 envs, 131072 at 2^25 with one group per thread.
constexpr int kStatsBlock = 1024;
__global__ __launch_bounds__(kStatsBlock) void stats_kernel(const double* __restrict__ slab, int blocks,
                                                            double* __restrict__ out) {
    __shared__ double part[3][kStatsBlock / 64];
    double a = 0.0, b = 0.0, c = 0.0;
    for (int i = threadIdx.x; i < blocks; i += kStatsBlock) {
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
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        part[0][w] = a;
        part[1][w] = b;
        part[2][w] = c;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        double s = 0.0;
        for (int k = 0; k < kStatsBlock / 64; ++k) s += part[threadIdx.x][k];
        out[threadIdx.x] = s;
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
    int64_t seg = 0;    // done-list segment stride (records per wave-iteration: 256)
    int64_t iters = 1;  // groups per thread of the step kernel
    int world_cap = 0;  // words allocated
    uint64_t world_version = 0;  // bumped by every world upload (se_qnet folds the ports)
    int32_t cmax = 0, fmax = 0;  // largest TAKE_CARGO / TAKE_FUEL amount any port allows (se_qnet)
    se_state st{};
    bool bound = false;
    double* d_slab = nullptr;       // [nslab][4]
    int32_t* d_offsets = nullptr;   // [nseg] se_done_compact scratch
    int grid = 0;
    int64_t nseg = 0;   // done-list segments: one per (iteration, wave) of the step kernel
    int64_t nslab = 0;  // stats slab entries: one per step-kernel wave
    uint8_t* d_mask_tmpl = nullptr;  // se_valid_mask's row templates (mask_tmpl_kernel), lazily built
    size_t mask_tmpl_cap = 0;
    uint64_t mask_tmpl_version = 0;  // world_version they were built from (0: none)
    int mask_ntmpl = 0;              // 1 + P + sum_p |ports on p's cell| (upload_world)
    bool mask_tiled = false;         // SHIPENV_MASK_TILED=1 at se_create: the round-4 tiled kernel
    int32_t done_pad = 1;   // done-list records padded to runs of this many (done_pad_records)
    bool nt_loads = false;  // nontemporal state loads in the step kernel (step_nt_loads)
};

// A host-resident world (se_host_*): no device, no HIP call. It steps envs whose SoA
// state lives in host memory with the kernels' own per-env code (replay_env).
struct se_host {
    WorldDims dims{};
    std::vector<uint8_t> water;  // H*W, 0 = ground
    std::vector<uint32_t> img;   // the world image, as staged into LDS on the device
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

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) is per device: `done` holds, for one
// kernel, a bit per device it has been set on (devices >= 64 set it on every call).
int allow_dynamic_lds(std::atomic<uint64_t>& done, const void* kernel, int bytes, int device) {
    const uint64_t bit = device >= 0 && device < 64 ? 1ull << device : 0ull;
    if (bit && (done.load(std::memory_order_acquire) & bit)) return SE_OK;
    HIP_TRY(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    done.fetch_or(bit, std::memory_order_acq_rel);
    return SE_OK;
}

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
// groups, loading the next group after storing the current one.
int step_block_cap() {
    const char* v = getenv("SHIPENV_STEP_BLOCKS");
    const int c = v ? atoi(v) : 0;
    return c > 0 ? c : kStepBlocks;
}

// Nontemporal state loads for the kernels without auto-reset while one step's traffic
// (~42 B per env) stays inside or near the 256 MiB Infinity Cache. Forced on vs off at
// the 32768-workgroup cap (profiles/r02h/nt_sweep, two runs each): config 3 at 2^20
// 8.5-8.8 vs 9.1-9.2 us, at 2^24 131-134 vs 123 us. The auto-reset kernels are faster
// without them up to 2^21 envs (config 4 at 2^20 11.6 vs 12.5 us; the training loop's step
// + record 16.0-16.3 vs 17.5-17.9 us) and with them beyond (below).
// The done list's records padded to whole 128-B lines (wave_compact) once the step's traffic
// is beyond the Infinity Cache: config 4 at 2^24 -2.7 us per step (median of five alternating
// rounds), at 2^20 +0.17 us (profiles/r04/ab_donepad.jsonl). SHIPENV_DONE_PAD overrides.
// Both settings are resolved once, by se_create (se_env::done_pad / nt_loads): a launch
// reads no environment variable, and the layout cannot change between two steps.
int32_t done_pad_records(const se_env* env) {
    const char* v = getenv("SHIPENV_DONE_PAD");
    if (v) return atoi(v) == 0 ? 1 : 8;
    return env->n > (int64_t)1 << 23 ? 8 : 1;
}

// Round 5 (episode-start stamps): the auto-reset kernel's few scattered stamp accesses per
// wave are cheap while the state streams do not evict them from the Infinity Cache, which
// the streams' nontemporal loads achieve. Config 4, alternating (profiles/r05/nt_sweep_c4.jsonl):
// 2^20 11.6 (temporal) vs 12.5 us (nontemporal), 2^22 43.6 vs 43.3, 2^23 83.0 vs 80.4,
// 2^24 173.4 vs 157.3, 2^25 339.5 vs 310.6; so nontemporal above 2^21 envs.
bool step_nt_loads(const se_env* env) {
    const char* v = getenv("SHIPENV_NT_LOADS");
    if (v) return atoi(v) != 0;
    if (env->flags & SE_FLAG_AUTO_RESET) return env->n > (int64_t)1 << 21;
    return env->n <= (int64_t)1 << 23;
}

size_t lds_bytes(const se_env* env) { return (size_t)env->dims.padded() * 4; }

// The world image (layout above WorldDims) of an H x W map and P ports, built on the
// host: uploaded by se_create / se_set_ports, kept as is by the host handles.
int build_world_image(int H, int W, const std::vector<uint8_t>& water, int32_t P, const int32_t* px,
                      const int32_t* py, const int32_t* pf, const int32_t* pc, WorldDims& dims,
                      std::vector<uint32_t>& img) {
    if (P < 0 || P > SE_MAX_PORTS) return fail(SE_EINVAL, "P must be in [0, 254]");
    for (int i = 0; i < P; ++i) {
        if (px[i] < 0 || px[i] >= H || py[i] < 0 || py[i] >= W)
            return fail(SE_EINVAL, "Coordinates not within map");  // add_port, environment.py:59-60
        if (pf[i] < 0 || pc[i] < 0) return fail(SE_EINVAL, "port stocks must be >= 0");
    }
    const int cw = (H * W + 15) / 16 * 4;  // cell-code bytes in whole 16-byte units
    WorldDims d{H, W, P, cw};
    img.assign((size_t)d.padded(), 0u);
    uint8_t* cell = reinterpret_cast<uint8_t*>(img.data());
    for (int c = 0; c < H * W; ++c) cell[c] = water[c] ? 0 : (uint8_t)kCellGround;
    for (int i = P - 1; i >= 0; --i)  // Entity.PORT (:65); the first port on a cell wins
        cell[(size_t)px[i] * W + py[i]] = (uint8_t)(i + 1);
    for (int i = 0; i < P; ++i) {
        img[d.pos() + i] = (uint32_t)px[i] | ((uint32_t)py[i] << 16);
        img[d.stk() + 2 * i] = (uint32_t)pf[i];
        img[d.stk() + 2 * i + 1] = (uint32_t)pc[i];
    }
    // normalize(cargo, 50, 0) = cargo / 50 (util.py:6-8): Python's int / int true
    // division is the correctly rounded quotient, which IEEE f64 division gives here.
    for (int c = 0; c < 50; ++c) {
        const double q = (double)c / kMaxCargo;
        memcpy(&img[d.frac() + 2 * c], &q, sizeof q);
        img[d.gate() + c] = (uint32_t)floor(ldexp(q, 32));  // exact product, q < 1
    }
    img[d.gate() + 50] = 0xffffffffu;  // cargo >= 50: random() < 1 <= cargo / 50
    // N, E, S, W as packed 16-bit (dx, dy) (shipping/type.py:8-16)
    const int mdx[4] = {0, -1, 0, 1}, mdy[4] = {-1, 0, 1, 0};
    for (int k = 0; k < 4; ++k)
        img[d.moves() + k] = ((uint32_t)mdx[k] & 0xffffu) | (((uint32_t)mdy[k] & 0xffffu) << 16);
    // step rewards before cargo loss / arrival, added in the reference's order:
    // out of fuel (:288-290), ground (:293-294) or fuel + water (:296-300), closer (:307-315)
    double rtab[10];
    for (int k = 0; k < 8; ++k) {
        double r = 0.0;
        if (k & 4) r += -10.0;
        if (k & 2) {
            r += -5.0;
        } else {
            r += -0.0001;
            r += -1.0;
        }
        r += (k & 1) ? 2.0 : -2.0;
        rtab[k] = r;
    }
    rtab[8] = 0.05;  // TAKE_FUEL / TAKE_CARGO (:349, :357)
    rtab[9] = 0.0;
    memcpy(&img[d.rtab()], rtab, sizeof rtab);
    dims = d;
    return SE_OK;
}

int upload_world(se_env* env, int32_t P, const int32_t* px, const int32_t* py, const int32_t* pf,
                 const int32_t* pc) {
    WorldDims d{};
    std::vector<uint32_t> img;
    int rc = build_world_image(env->dims.H, env->dims.W, env->water, P, px, py, pf, pc, d, img);
    if (rc) return rc;
    if (d.padded() > env->world_cap) {
        if (env->d_world) HIP_TRY(hipFree(env->d_world));
        env->d_world = nullptr;
        HIP_TRY(hipMalloc(&env->d_world, (size_t)d.padded() * 4));
        env->world_cap = d.padded();
    }
    HIP_TRY(hipMemcpy(env->d_world, img.data(), (size_t)d.padded() * 4, hipMemcpyHostToDevice));
    env->dims = d;
    env->cmax = env->fmax = 0;
    for (int i = 0; i < P; ++i) {  // amounts 1..49 / 1..199 exist (utils/preprocessing.py:93-108)
        env->cmax = std::max(env->cmax, std::min(pc[i], 49));
        env->fmax = std::max(env->fmax, std::min(pf[i], 199));
    }
    env->world_version += 1;
    env->mask_ntmpl = 1 + P;  // se_valid_mask's row templates (mask_tmpl_kernel)
    for (int p = 0; p < P; ++p)
        for (int q = 0; q < P; ++q) env->mask_ntmpl += (px[p] == px[q] && py[p] == py[q]) ? 1 : 0;
    return SE_OK;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

int check_ready(se_env* env) {
    if (!env) return fail(SE_EINVAL, "null env");
    if (!env->bound) return fail(SE_ESTATE, "se_bind has not been called");
    return SE_OK;
}

int launch_step(se_env* env, bool typed, bool replay, const int32_t* act, const int32_t* a,
                const int32_t* b, se_tape* tape, void* stream, const StepRecord* rec = nullptr,
                bool seq = false) {
    int rc = check_ready(env);
    if (rc) return rc;
    if (env->n > 0 && (!act || (typed && (!a || !b)) || (replay && !tape)))  // n = 0: an empty batch
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
        A.done_recs = env->st.done_recs + par * (size_t)env->nseg * (size_t)env->seg;
        A.done_count = env->st.done_count + par * (size_t)env->nseg;
    }
    A.seg = env->seg;
    A.done_pad = env->done_pad;
    A.iters = env->iters;
    A.slab = env->d_slab;
    const hipStream_t s = (hipStream_t)stream;
    const size_t lds = lds_bytes(env);
    const int grid = env->grid;
    const bool ntl = env->nt_loads;
    if (rec) {  // se_step_record: the caller checked agent actions, auto-reset, n % 4 == 0, n > 0
        A.rec = *rec;
        if (ntl) step_kernel<false, false, true, true, true><<<grid, kStepBlock, lds, s>>>(A);
        else step_kernel<false, false, true, false, true><<<grid, kStepBlock, lds, s>>>(A);
        HIP_TRY(hipGetLastError());
    } else if (env->n >= kEnvsPerThread) {  // at least one full group (step_kernel's first load assumes it)
        if (!typed && replay) step_kernel<false, true, false><<<grid, kStepBlock, lds, s>>>(A);  // agent replay
        else if (seq && !typed && !autoreset && ntl)
            step_kernel<false, false, false, true, false, true><<<grid, kStepBlock, lds, s>>>(A);
        else if (seq && !typed && !autoreset)
            step_kernel<false, false, false, false, false, true><<<grid, kStepBlock, lds, s>>>(A);
        else if (!typed && !autoreset && ntl) step_kernel<false, false, false, true><<<grid, kStepBlock, lds, s>>>(A);
        else if (!typed && autoreset && ntl) step_kernel<false, false, true, true><<<grid, kStepBlock, lds, s>>>(A);
        else if (!typed && !autoreset) step_kernel<false, false, false><<<grid, kStepBlock, lds, s>>>(A);
        else if (!typed && autoreset) step_kernel<false, false, true><<<grid, kStepBlock, lds, s>>>(A);
        else if (typed && replay) step_kernel<true, true, false><<<grid, kStepBlock, lds, s>>>(A);
        else if (typed && !autoreset) step_kernel<true, false, false><<<grid, kStepBlock, lds, s>>>(A);
        else step_kernel<true, false, true><<<grid, kStepBlock, lds, s>>>(A);
        HIP_TRY(hipGetLastError());
    }
    if (env->n & 3) {
        if (!typed && replay) step_tail_kernel<false, true, false><<<1, 64, 0, s>>>(A);
        else if (!typed && !autoreset) step_tail_kernel<false, false, false><<<1, 64, 0, s>>>(A);
        else if (!typed && autoreset) step_tail_kernel<false, false, true><<<1, 64, 0, s>>>(A);
        else if (typed && replay) step_tail_kernel<true, true, false><<<1, 64, 0, s>>>(A);
        else if (typed && !autoreset) step_tail_kernel<true, false, false><<<1, 64, 0, s>>>(A);
        else step_tail_kernel<true, false, true><<<1, 64, 0, s>>>(A);
        HIP_TRY(hipGetLastError());
    }
    if (!replay) env->step_t += 1;
    return SE_OK;
}

}  // namespace

// error text for se_last_error from the host-only sources (mapload.cpp)
void shipenv_set_error(const std::string& msg) { g_err = msg; }

extern "C" {

#if SHIPENV_TRACE
extern "C" int se_trace_read(void* host, size_t bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_trace), bytes) == hipSuccess ? 0 : -1;
}
#endif

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
        env->iters = groups > 0 ? (groups + cap * kStepBlock - 1) / (cap * kStepBlock) : 1;
        env->grid = (int)(groups > 0 ? (groups + env->iters * kStepBlock - 1) / (env->iters * kStepBlock) : 1);
        env->seg = 64 * kEnvsPerThread;  // one done-list segment per (iteration, wave)
        env->nseg = (int64_t)env->grid * env->iters * (kStepBlock / 64);
        env->nslab = (int64_t)env->grid * (kStepBlock / 64);  // stats: one entry per wave
        env->done_pad = done_pad_records(env);
        env->nt_loads = step_nt_loads(env);
        const char* mv = getenv("SHIPENV_MASK_TILED");
        env->mask_tiled = mv && atoi(mv) != 0;
    }
    hipError_t e = hipMalloc(&env->d_slab, (size_t)env->nslab * 4 * sizeof(double));
    if (e == hipSuccess) e = hipMemset(env->d_slab, 0, (size_t)env->nslab * 4 * sizeof(double));
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
        if ((env->n > 0 && (!st->ep_return || !st->ep_start)) || !st->done_recs || !st->done_count)
            return fail(SE_EINVAL, "auto-reset needs ep_return, ep_start, done_recs and done_count");
        if (!aligned16(st->ep_return) || !aligned16(st->ep_start) || !aligned16(st->done_recs))
            return fail(SE_EINVAL, "state buffers must be 16-byte aligned");
        DeviceGuard g(env->device);
        HIP_TRY(hipMemset(st->done_count, 0, 2 * (size_t)env->nseg * sizeof(int32_t)));
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
                (uint32_t)env->epoch, (uint32_t)env->step_t, env->st, mask, nullptr, nullptr};
    if (env->n > 0) {
        reset_kernel<<<grid_for(env->n), kBlock, 0, (hipStream_t)stream>>>(A);
        HIP_TRY(hipGetLastError());
    }
    env->epoch += 1;
    return SE_OK;
}

int se_reset_to(se_env* env, const uint8_t* mask, const int32_t* origin, const int32_t* dest,
                void* stream) {
    int rc = check_ready(env);
    if (rc) return rc;
    if (env->n > 0 && (!origin || !dest)) return fail(SE_EINVAL, "null origin/dest");
    DeviceGuard g(env->device);
    ResetArgs A{env->d_world, env->dims, env->n, env->env_base, env->seed,
                (uint32_t)env->epoch, (uint32_t)env->step_t, env->st, mask, origin, dest};
    if (env->n > 0) {
        reset_kernel<<<grid_for(env->n), kBlock, 0, (hipStream_t)stream>>>(A);
        HIP_TRY(hipGetLastError());
    }
    return SE_OK;
}

int se_step(se_env* env, const int32_t* actions, void* stream) {
    return launch_step(env, false, false, actions, nullptr, nullptr, nullptr, stream);
}

int se_step_seq_mark(se_env* env, const int32_t* actions, int64_t ld, int32_t steps, void* stream,
                     void* event, int32_t mark_after) {
    int rc = check_ready(env);
    if (rc) return rc;
    if (steps < 0) return fail(SE_EINVAL, "negative step count");
    if (steps > 1 && (ld < env->n || (ld & 3))) return fail(SE_EINVAL, "row stride must be >= n and a multiple of 4");
    if (event && (mark_after < 0 || mark_after > steps)) return fail(SE_EINVAL, "mark_after must be in [0, steps]");
    for (int32_t k = 0; k <= steps; ++k) {
        if (event && k == mark_after) {
            DeviceGuard g(env->device);
            HIP_TRY(hipEventRecord((hipEvent_t)event, (hipStream_t)stream));
        }
        if (k == steps) break;
        rc = launch_step(env, false, false, actions + (int64_t)k * ld, nullptr, nullptr, nullptr, stream, nullptr, true);
        if (rc) return rc;
    }
    return SE_OK;
}

int se_step_seq(se_env* env, const int32_t* actions, int64_t ld, int32_t steps, void* stream) {
    return se_step_seq_mark(env, actions, ld, steps, stream, nullptr, 0);
}

int se_step_typed(se_env* env, const int32_t* type, const int32_t* a, const int32_t* b,
                  void* stream) {
    return launch_step(env, true, false, type, a, b, nullptr, stream);
}

int se_step_replay(se_env* env, const int32_t* type, const int32_t* a, const int32_t* b,
                   se_tape* tape, void* stream) {
    return launch_step(env, true, true, type, a, b, tape, stream);
}

int se_step_agent_replay(se_env* env, const int32_t* actions, se_tape* tape, void* stream) {
    return launch_step(env, false, true, actions, nullptr, nullptr, tape, stream);
}

int se_observe(se_env* env, float* obs, int64_t ld, void* stream) {
    int rc = check_ready(env);
    if (rc) return rc;
    if ((env->n > 0 && !obs) || ld < 6 + 4 * (int64_t)env->dims.P) return fail(SE_EINVAL, "bad obs buffer / ld");
    DeviceGuard g(env->device);
    ObsArgs A{env->d_world, env->dims, env->n, ld, env->st, obs};
    const int64_t W = 6 + 4 * (int64_t)env->dims.P;
    const int64_t total = env->n * W;
    if (total == 0) return SE_OK;
    if (ld == W && aligned16(obs) && W <= 1022) {  // dense rows: the tiled kernel
        const uint32_t magic = (uint32_t)((((uint64_t)1 << 32) + (uint64_t)W - 1) / (uint64_t)W);
        const size_t lds = (size_t)(kTileRows * 6 + 4 * env->dims.P) * sizeof(float);
        observe_tiled_kernel<<<grid_for(env->n), kBlock, lds, (hipStream_t)stream>>>(A, magic);
    } else {
        observe_kernel<<<grid_for(total), kBlock, lds_bytes(env), (hipStream_t)stream>>>(A);
    }
    HIP_TRY(hipGetLastError());
    return SE_OK;
}

int se_valid_mask(se_env* env, uint8_t* bits, void* stream) {
    int rc = check_ready(env);
    if (rc) return rc;
    if (env->n > 0 && !bits) return fail(SE_EINVAL, "null bits");
    DeviceGuard g(env->device);
    const int32_t stride = (4 + env->dims.P + 250 + 7) / 8;
    MaskArgs A{env->d_world, env->dims, env->n, stride, env->st, bits};
    const int64_t total = env->n * stride;
    if (total == 0) return SE_OK;
    const hipStream_t s = (hipStream_t)stream;
    const int tb = mask_tb(stride);
    if (aligned16(bits) && env->dims.P <= 64 && env->mask_ntmpl <= kMaskTmplMax && !env->mask_tiled) {
        // the row templates, rebuilt when the world image changed
        const size_t need = (size_t)kMaskHdr + (size_t)env->mask_ntmpl * tb;
        if (need > env->mask_tmpl_cap) {
            if (env->d_mask_tmpl) HIP_TRY(hipFree(env->d_mask_tmpl));
            env->d_mask_tmpl = nullptr;
            env->mask_tmpl_cap = 0;
            HIP_TRY(hipMalloc(&env->d_mask_tmpl, need));
            env->mask_tmpl_cap = need;
            env->mask_tmpl_version = 0;
        }
        if (env->mask_tmpl_version != env->world_version) {
            mask_tmpl_kernel<<<1, kBlock, 0, s>>>(env->d_world, env->dims, stride, env->d_mask_tmpl);
            HIP_TRY(hipGetLastError());
            env->mask_tmpl_version = env->world_version;
        }
        const uint32_t magic = (uint32_t)((((uint64_t)1 << 32) + (uint64_t)stride - 1) / (uint64_t)stride);
        const size_t lds = (size_t)env->mask_ntmpl * tb;
        valid_mask_tmpl_kernel<<<grid_for(env->n, lds > 4096 ? 1024 : kMaxBlocks), kBlock, lds, s>>>(
            A, env->d_mask_tmpl, env->mask_ntmpl, magic);
    } else if (aligned16(bits)) {  // the tiled kernel (rows are always dense here)
        const size_t lds = ((size_t)kTileRows * stride + 15) & ~(size_t)15;
        valid_mask_tiled_kernel<<<grid_for(env->n), kBlock, lds, s>>>(A);
    } else {
        valid_mask_kernel<<<grid_for(total), kBlock, lds_bytes(env), (hipStream_t)stream>>>(A);
    }
    HIP_TRY(hipGetLastError());
    return SE_OK;
}

int se_gen_actions(se_env* env, int32_t* actions, uint32_t t, void* stream) {
    if (!env || (!actions && env->n > 0)) return fail(SE_EINVAL, "null argument");
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

int se_sample_actions(se_env* env, int32_t* type, int32_t* a, int32_t* b, uint32_t t, void* stream) {
    int rc = check_ready(env);
    if (rc) return rc;
    if (env->n == 0) return SE_OK;
    if (!type || !a || !b) return fail(SE_EINVAL, "null output pointer");
    DeviceGuard g(env->device);
    SampleArgs A{env->d_world, env->dims, env->n, env->env_base, env->seed, t, env->st, type, a, b};
    sample_kernel<<<grid_for(env->n), kBlock, 0, (hipStream_t)stream>>>(A);
    HIP_TRY(hipGetLastError());
    return SE_OK;
}

int se_rollout(se_env* env, const int32_t* src, int64_t m, int32_t max_steps, int32_t max_attempts,
               int64_t rollout_base, double* ret, int32_t* steps, int32_t* status, void* stream) {
    int rc = check_ready(env);
    if (rc) return rc;
    if (m < 0 || max_steps < 0 || max_attempts < 0 || rollout_base < 0)
        return fail(SE_EINVAL, "m, max_steps, max_attempts and rollout_base must be >= 0");
    if (m > 0 && (!src || !ret || !steps || !status)) return fail(SE_EINVAL, "null rollout buffer");
    if (m == 0) return SE_OK;
    DeviceGuard g(env->device);
    RolloutArgs A{};
    A.world = env->d_world;
    A.dims = env->dims;
    A.n = env->n;
    A.m = m;
    A.rollout_base = rollout_base;
    A.seed = env->seed;
    A.max_steps = max_steps;
    A.max_attempts = max_attempts;
    A.st = env->st;
    A.src = src;
    A.ret = ret;
    A.steps = steps;
    A.status = status;
    rollout_kernel<<<grid_for(m), kBlock, lds_bytes(env), (hipStream_t)stream>>>(A);
    HIP_TRY(hipGetLastError());
    return SE_OK;
}

int se_episode_stats(se_env* env, double* out, void* stream) {
    if (!env || !out) return fail(SE_EINVAL, "null argument");
    DeviceGuard g(env->device);
    stats_kernel<<<1, kStatsBlock, 0, (hipStream_t)stream>>>(env->d_slab, (int)env->nslab, out);
    HIP_TRY(hipGetLastError());
    return SE_OK;
}

int se_clear_stats(se_env* env, void* stream) {
    if (!env) return fail(SE_EINVAL, "null env");
    DeviceGuard g(env->device);
    HIP_TRY(hipMemsetAsync(env->d_slab, 0, (size_t)env->nslab * 4 * sizeof(double),
                           (hipStream_t)stream));
    return SE_OK;
}

int se_done_layout(se_env* env, int64_t* seg_stride, int32_t* segments) {
    if (!env) return fail(SE_EINVAL, "null env");
    if (seg_stride) *seg_stride = env->seg;
    if (segments) *segments = (int32_t)env->nseg;
    return SE_OK;
}

int se_done_list(se_env* env, int64_t* rec_offset, int64_t* count_offset) {
    if (!env || !rec_offset || !count_offset) return fail(SE_EINVAL, "null argument");
    if (!(env->flags & SE_FLAG_AUTO_RESET)) return fail(SE_ESTATE, "no done list without auto-reset");
    if (env->step_t == 0) return fail(SE_ESTATE, "no step has run");
    const int64_t par = (int64_t)((env->step_t - 1) & 1u);
    *rec_offset = par * (int64_t)env->nseg * env->seg;
    *count_offset = par * (int64_t)env->nseg;
    return SE_OK;
}

int se_done_compact(se_env* env, se_done_rec* out, int32_t* out_count, void* stream) {
    int64_t ro = 0, co = 0;
    int rc = se_done_list(env, &ro, &co);
    if (rc) return rc;
    if (!out || !out_count) return fail(SE_EINVAL, "null output");
    DeviceGuard g(env->device);
    if (!env->d_offsets) HIP_TRY(hipMalloc(&env->d_offsets, (size_t)env->nseg * sizeof(int32_t)));
    const hipStream_t s = (hipStream_t)stream;
    done_scan_kernel<<<1, 1024, 0, s>>>(env->st.done_count + co, env->nseg, env->d_offsets, out_count);
    const int64_t blocks = (env->nseg + kBlock / 64 - 1) / (kBlock / 64);
    done_copy_kernel<<<(int)blocks, kBlock, 0, s>>>(env->st.done_recs + ro, env->st.done_count + co,
                                                    env->d_offsets, env->nseg, env->seg, out);
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
        HIP_TRY(hipMemset(env->st.done_count, 0, 2 * (size_t)env->nseg * sizeof(int32_t)));
    env->step_t = step;
    env->epoch = epoch;
    return SE_OK;
}

int se_destroy(se_env* env) {
    if (!env) return SE_OK;
    DeviceGuard g(env->device);
    if (env->d_world) (void)hipFree(env->d_world);
    if (env->d_slab) (void)hipFree(env->d_slab);
    if (env->d_offsets) (void)hipFree(env->d_offsets);
    if (env->d_mask_tmpl) (void)hipFree(env->d_mask_tmpl);
    delete env;
    return SE_OK;
}

// ---------------------------------------------------------------- host-resident envs
int se_host_create(se_host** out, int32_t H, int32_t W, const uint8_t* water, int32_t P,
                   const int32_t* port_x, const int32_t* port_y, const int32_t* port_fuel,
                   const int32_t* port_cargo) {
    if (!out) return fail(SE_EINVAL, "null out");
    *out = nullptr;
    if (H < 1 || W < 1 || H > SE_MAX_SIDE || W > SE_MAX_SIDE)
        return fail(SE_EINVAL, "map sides must be in [1, 256]");
    if (!water) return fail(SE_EINVAL, "null water map");
    if (P > 0 && (!port_x || !port_y || !port_fuel || !port_cargo)) return fail(SE_EINVAL, "null port arrays");
    se_host* h = new se_host();
    h->dims.H = H;
    h->dims.W = W;
    h->water.assign(water, water + (size_t)H * W);
    for (auto& v : h->water) v = v ? 1 : 0;
    const int rc = build_world_image(H, W, h->water, P, port_x, port_y, port_fuel, port_cargo, h->dims, h->img);
    if (rc) {
        delete h;
        return rc;
    }
    *out = h;
    return SE_OK;
}

int se_host_set_ports(se_host* h, int32_t P, const int32_t* port_x, const int32_t* port_y,
                      const int32_t* port_fuel, const int32_t* port_cargo) {
    if (!h) return fail(SE_EINVAL, "null host world");
    if (P > 0 && (!port_x || !port_y || !port_fuel || !port_cargo)) return fail(SE_EINVAL, "null port arrays");
    return build_world_image(h->dims.H, h->dims.W, h->water, P, port_x, port_y, port_fuel, port_cargo, h->dims,
                             h->img);
}

int se_host_step_replay(se_host* h, int64_t n, const se_state* st, const int32_t* type, const int32_t* a,
                        const int32_t* b, se_tape* tape) {
    if (!h || !st || n < 0) return fail(SE_EINVAL, "null argument or n < 0");
    if (n == 0) return SE_OK;
    if (!type || !a || !b || !tape || !st->x || !st->y || !st->fuel || !st->cargo || !st->origin || !st->dest ||
        !st->reward || !st->done || !st->err)
        return fail(SE_EINVAL, "null state, action or tape buffer");
    const LdsWorld w = world_view(h->dims, h->img.data());
    for (int64_t i = 0; i < n; ++i) {
        Ship s{st->x[i], st->y[i], st->fuel[i], st->cargo[i], st->origin[i], st->dest[i]};
        Pending p;
        se_tape* tp = tape + i;
        tp->used = (int32_t)replay_env(w, s, p, SE_ERR_OK, type[i], a[i], b[i], tp->u_fuel, tp->u_gate, tp);
        st->x[i] = (uint8_t)s.x;
        st->y[i] = (uint8_t)s.y;
        st->fuel[i] = s.fuel;
        st->cargo[i] = s.cargo;
        st->origin[i] = (uint8_t)s.origin;
        st->dest[i] = (uint8_t)s.dest;
        st->reward[i] = (float)p.r;  // one rounding of the reference's f64 reward
        st->done[i] = (uint8_t)p.dead;
        st->err[i] = (int8_t)p.e;
        if (st->reward64) st->reward64[i] = p.r;
    }
    return SE_OK;
}

int se_host_reset_to(se_host* h, int64_t n, const se_state* st, const uint8_t* mask, const int32_t* origin,
                     const int32_t* dest) {
    if (!h || !st || n < 0 || (n > 0 && (!origin || !dest))) return fail(SE_EINVAL, "null argument or n < 0");
    const LdsWorld w = world_view(h->dims, h->img.data());
    for (int64_t i = 0; i < n; ++i)
        if ((!mask || mask[i]) && (origin[i] < 0 || origin[i] >= w.P || dest[i] < 0 || dest[i] >= w.P))
            return fail(SE_EINVAL, "origin / dest must name ports");
    for (int64_t i = 0; i < n; ++i) {  // reset_kernel's explicit form (reset() :227-243)
        if (mask && !mask[i]) continue;
        st->x[i] = (uint8_t)w.px(origin[i]);
        st->y[i] = (uint8_t)w.py(origin[i]);
        st->fuel[i] = kFuelInit;
        st->cargo[i] = 0;
        st->origin[i] = (uint8_t)origin[i];
        st->dest[i] = (uint8_t)dest[i];
        if (st->ep_return) st->ep_return[i] = 0.0f;
        if (st->ep_start) st->ep_start[i] = 0;  // a host world has no step counter
        st->done[i] = 0;
        st->err[i] = 0;
        st->reward[i] = 0.0f;
    }
    return SE_OK;
}

int se_host_destroy(se_host* h) {
    delete h;
    return SE_OK;
}

}  // extern "C"

// the fused DQN policy step (same translation unit: world image, env handle, Philox)
#include "qpolicy.h"
#include "replay.h"
#include "qtrain.h"
#include "server.h"
