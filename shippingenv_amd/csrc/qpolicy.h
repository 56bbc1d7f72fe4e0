// qpolicy.h — the DQN policy step fused on MFMA.
//
// Part of shipenv.hip's translation unit (included at its end): it shares the
// world image, the env handle and Philox. Reference: agents/dqn.py DQNNetwork
// (:21-33: fc1 6+4P -> 128, relu, fc2 128 -> 128, relu, fc3 128 -> A = 4+P+250)
// and choose_action (:177-203), on preprocess_state rows (utils/preprocessing.py:25-62).
//
// Shape of the work: per env ~50 K MACs (fc2 + fc3) against 16 bytes of state, so
// the step is MFMA-bound, not HBM-bound. One wave takes 32 envs at a time with
// the batch on the MFMA's column (N) dimension: every layer is D = W·X with the
// weights W as the A operand (bf16 fragments pre-permuted into LDS, lane-linear,
// one ds_read_b128 per MFMA) and the activations X as the B operand in registers.
// A v_mfma_f32_32x32x16_bf16 result keeps the env on the lane and the feature rows
// in its 16 registers, so relu + bf16 packing of registers 8s..8s+7 is directly
// the next layer's k-step s (cdna_hip_programming.md §3, "accumulator tile as the
// next MFMA's operand"); the weights are stored in that step's permuted k order.
// fc1 has 6 live inputs (the port block is constant: folded into the bias) and
// runs as one k-step per row tile, with fuel split into bf16 hi + lo parts. Biases
// are the accumulators' initial values (f32). fc3's epilogue is the masked
// argmax: each lane keeps the first maximum over the valid rows it holds, and the
// two lane halves that share an env merge with one shuffle. Q never reaches HBM.
//
// fc3 runs over the compact row layout (QnetDims): only the actions some env can
// ever take, so at P = 5 two 32-row tiles where the full layout has three with a valid
// row (of nine); the full layout serves q_out (every row's Q, for tests / inspection).
//
// LDS: the packed network (113 KB at P = 5) plus the world image, one 1024-thread
// workgroup (16 waves, 4 per SIMD, <= 128 VGPRs) per CU for the whole launch. It fits
// 128 VGPRs with no spills and no scratch: check (-Rpass-analysis=kernel-resource-usage)
// after any edit that adds register pressure.

#ifndef SHIPENV_POLICY_ABL
#define SHIPENV_POLICY_ABL 0  // timing-only ablations of the policy kernel (1: plain max epilogue, 2: no fc3,
                              // 4: no bias reads, 8: fc2 reads one fragment)
#endif
#if SHIPENV_POLICY_ABL == 4
#define PBIAS(b) (f32x16{})
#else
#define PBIAS(b) bias_frag(b)
#endif

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int kQHidden = 128;     // DQNNetwork hidden_size (dqn.py:24, default 128)
// 16 waves (4 per SIMD, <= 128 VGPRs, no scratch) share one LDS copy of the network.
// Measured per launch at 2^20 envs when it was chosen (round 1 kernel): 512 threads
// 108.8 us, 768 (3 waves per SIMD, 165 VGPRs) 92.5 us, 1024 87.2 us: the fourth wave
// covers the others' MFMA -> relu -> MFMA stalls.
#ifndef SHIPENV_POLICY_BLOCK
#define SHIPENV_POLICY_BLOCK 1024
#endif
#ifndef SHIPENV_POLICY_WG_PER_CU
#define SHIPENV_POLICY_WG_PER_CU 1  // resident workgroups per CU (each stages its own network copy)
#endif
#ifndef SHIPENV_POLICY_WAVES_PER_EU
#define SHIPENV_POLICY_WAVES_PER_EU 0  // 0: the compiler's choice from the block size
#endif
constexpr int kPolicyBlock = SHIPENV_POLICY_BLOCK;
constexpr int kPolicyWgPerCu = SHIPENV_POLICY_WG_PER_CU;
constexpr int kPolicyWaves = kPolicyBlock / 64;

// Packed network image (bytes). Fragments are 64 lanes x 8 bf16 = 1 KB.
// Two layouts of fc3's rows:
// * full: row r is action r (A = 4 + P + 250 rows), for the Q output (q_out);
// * compact: only the actions some env can ever take, in ascending order: the moves and
//   SELECT rows [0, 4 + P), then TAKE_CARGO amounts 1..cmax and TAKE_FUEL amounts
//   1..fmax, cmax / fmax the largest stocks of the world's ports (add_port draws 5..20,
//   so 49 rows and 2 tiles at P = 5 instead of 3 of the 9 full tiles with a valid row).
//   The first maximum in compact rows is the first in actions (the map is increasing).
struct QnetDims {
    int32_t P, A, rows, mt3;  // ports, actions, fc3 rows of this layout, its row tiles
    int32_t compact, cmax;    // the layout; TAKE_CARGO rows in the compact one
    __host__ __device__ int in1() const { return 6 + 4 * P; }
    // action of fc3 row r (utils/preprocessing.py:111-137)
    __host__ __device__ int action_of_row(int r) const {
        if (!compact || r < 4 + P) return r;
        return r < 4 + P + cmax ? r + 1 : r + 51 - cmax;
    }
    // row of TAKE_CARGO amount 1 and of TAKE_FUEL amount 1
    __host__ __device__ int cargo_row1() const { return compact ? 4 + P : 5 + P; }
    __host__ __device__ int fuel_row1() const { return compact ? 4 + P + cmax : 55 + P; }
    __host__ __device__ int w1() const { return 0; }                    // 4 fc1 tiles
    __host__ __device__ int w2() const { return 4 * 1024; }              // 4 x 4 x 2 fc2 fragments
    __host__ __device__ int w3() const { return w2() + 32 * 1024; }      // mt3 x 4 x 2 fc3 fragments
    __host__ __device__ int b1() const { return w3() + mt3 * 8 * 1024; } // 128 f32, port block folded
    __host__ __device__ int b2() const { return b1() + 4 * kQHidden; }
    __host__ __device__ int b3() const { return b2() + 4 * kQHidden; }   // mt3 * 32 f32 (0 beyond A)
    __host__ __device__ int same() const { return b3() + mt3 * 128; }    // P uint64: ports on port p's cell
    __host__ __device__ int regm() const { return same() + 8 * P; }      // mt3 uint32: fc3 epilogue regs
    __host__ __device__ int bytes() const { return (regm() + 4 * mt3 + 15) & ~15; }
};

QnetDims qnet_dims(int P, bool compact = false, int cmax = 0, int fmax = 0) {
    QnetDims q;
    q.P = P;
    q.A = 4 + P + 250;  // utils/preprocessing.py:93-108
    q.compact = compact ? 1 : 0;
    q.cmax = compact ? cmax : 49;
    q.rows = compact ? 4 + P + cmax + fmax : q.A;
    q.mt3 = (q.rows + 31) / 32;
    return q;
}

// ------------------------------------------------------------------ packing
// One thread per 16-byte fragment slot / bias entry. Fragment (tile, step) lane
// (r = lane & 31, h = lane >> 5) element j holds W[tile*32 + r][k] with
//   fc1: k = column map of j (h = 0 only; the obs fragment below uses the same map)
//   fc2, fc3: k = kt*32 + 16s + 8(j >> 2) + 4h + (j & 3), the row of the previous
//   layer's accumulator that register 8s + j of lane half h holds.
struct PackArgs {
    const float *w1, *b1, *w2, *b2, *w3, *b3;
    const uint32_t* world;
    WorldDims dims;
    QnetDims q[2];  // blockIdx.y: the full layout, the compact one
    uint8_t* img[2];
    int32_t* bump;  // se_qnet_repack: a device counter advanced once, or null
};

// fc1 input column of fragment element j: x, y, fuel (hi), fuel (lo), "cargo" = fuel
// (hi, lo; environment.py:206), origin, dest (utils/preprocessing.py:51-58)
__device__ __forceinline__ int fc1_col(int j) {
    return j < 2 ? j : (j < 4 ? 2 : (j < 6 ? 3 : j - 2));
}

__device__ __forceinline__ int acc_row(int s, int j, int h) { return 16 * s + 8 * (j >> 2) + 4 * h + (j & 3); }

__global__ __launch_bounds__(256) void qnet_pack_kernel(PackArgs A) {
    const QnetDims q = A.q[blockIdx.y];
    uint8_t* const img = A.img[blockIdx.y];
    if (A.bump && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *A.bump += 1;
    const int in1 = q.in1();
    const int n_w1 = 4 * 64, n_w2 = 32 * 64, n_w3 = q.mt3 * 8 * 64;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x;
         t < n_w1 + n_w2 + n_w3 + 2 * kQHidden + q.mt3 * 32 + q.P + q.mt3; t += gridDim.x * blockDim.x) {
        if (t < n_w1 + n_w2 + n_w3) {
            int f = t >> 6;
            const int lane = t & 63, r = lane & 31, h = lane >> 5;
            bf16x8 v;
            uint8_t* dst;
            if (t < n_w1) {  // fc1 tile f
                const int row = f * 32 + r;
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = h == 0 ? (__bf16)A.w1[row * in1 + fc1_col(j)] : (__bf16)0.0f;
                dst = img + q.w1() + f * 1024 + lane * 16;
            } else {
                const bool second = t < n_w1 + n_w2;
                f -= second ? 4 : 4 + 32;  // fragment index ((mt*4 + kt)*2 + s)
                const int s = f & 1, kt = (f >> 1) & 3, mt = f >> 3;
                const int row = mt * 32 + r;
                const float* W = second ? A.w2 : A.w3;
                const bool in = second || row < q.rows;
                const int wrow = second ? row : q.action_of_row(row);
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    v[j] = in ? (__bf16)W[wrow * kQHidden + kt * 32 + acc_row(s, j, h)] : (__bf16)0.0f;
                dst = img + (second ? q.w2() : q.w3()) + f * 1024 + lane * 16;
            }
            *reinterpret_cast<bf16x8*>(dst) = v;
            continue;
        }
        int u = t - (n_w1 + n_w2 + n_w3);
        const LdsWorld wv = world_view(A.dims, A.world);  // the device image, read in place
        const uint32_t* pos = wv.pos;
        const int P = q.P;
        if (u < kQHidden) {  // b1 + fc1 over the constant port block (x, y, fuel, cargo per port)
            double acc = (double)A.b1[u];
            for (int p = 0; p < P; ++p) {
                const float* w = A.w1 + u * in1 + 6 + 4 * p;
                acc += (double)w[0] * (double)wv.px(p) + (double)w[1] * (double)wv.py(p) +
                       (double)w[2] * (double)wv.pfuel(p) + (double)w[3] * (double)wv.pcargo(p);
            }
            reinterpret_cast<float*>(img + q.b1())[u] = (float)acc;
        } else if ((u -= kQHidden) < kQHidden) {
            reinterpret_cast<float*>(img + q.b2())[u] = A.b2[u];
        } else if ((u -= kQHidden) < q.mt3 * 32) {
            reinterpret_cast<float*>(img + q.b3())[u] = u < q.rows ? A.b3[q.action_of_row(u)] : 0.0f;
        } else if ((u -= q.mt3 * 32) < P) {  // bit p: port p stands on port u's cell (u included)
            uint64_t same = 0;
            for (int p = 0; p < P; ++p)
                if (pos[p] == pos[u]) same |= 1ull << p;
            reinterpret_cast<uint64_t*>(img + q.same())[u] = same;
        } else {
            // fc3 tile mt = u - P: bit reg set when accumulator register reg (rows
            // base + (reg & 3) + 8 (reg >> 2) + 4h, h = 0, 1) can hold a valid action of
            // ANY env: a move or SELECT (row < 4 + P), or an amount within the largest
            // stock (is_valid_action, dqn.py:125-175). The epilogue skips the others.
            const int mt = u - P, base = mt * 32;
            int cmax = 0, fmax = 0;
            for (int p = 0; p < P; ++p) {
                cmax = max(cmax, min(wv.pcargo(p), 49));
                fmax = max(fmax, min(wv.pfuel(p), 199));
            }
            const int c_lo = 5 + P, c_hi = 4 + P + cmax, f_lo = 55 + P, f_hi = 54 + P + fmax;
            uint32_t rm = 0;
            for (int reg = 0; reg < 16; ++reg)
                for (int h = 0; h < 2; ++h) {
                    const int row = base + (reg & 3) + 8 * (reg >> 2) + 4 * h;
                    const int a = q.action_of_row(row);
                    const bool ok = row < q.rows && (a < 4 + P || (a >= c_lo && a <= c_hi) ||
                                                     (a >= f_lo && a <= f_hi));
                    rm |= (uint32_t)ok << reg;
                }
            reinterpret_cast<uint32_t*>(img + q.regm())[mt] = rm;
        }
    }
}

// ------------------------------------------------------------------ the policy step
struct PolicyArgs {
    const uint32_t* world;
    WorldDims dims;
    const uint4* qimg;
    QnetDims q;
    int64_t n, env_base;
    uint64_t seed;
    uint32_t t;
    double eps;
    se_state st;
    int32_t* actions;
    float* q_out;
    int64_t ldq;
    // remember's state and action (se_policy_record): the replay ring's s / a columns
    // at slot (rec_head + env) mod rec_cap, or null
    uint32_t* rec_pos;
    float* rec_fuel;
    int32_t* rec_act;
    int64_t rec_head, rec_cap;
};

// v = p0 + p1 + p2, each the bf16 rounding of the remainder (exact f32 subtractions)
__device__ __forceinline__ void split3(float v, __bf16& p0, __bf16& p1, __bf16& p2) {
    p0 = (__bf16)v;
    const float r1 = v - (float)p0;
    p1 = (__bf16)r1;
    p2 = (__bf16)(r1 - (float)p1);
}

// accumulator initial value: bias rows (reg & 3) + 8 (reg >> 2) + 4h of a 32-row tile
__device__ __forceinline__ f32x16 bias_frag(const float* b) {
    const float4 a = *reinterpret_cast<const float4*>(b), c = *reinterpret_cast<const float4*>(b + 8),
                 d = *reinterpret_cast<const float4*>(b + 16), e = *reinterpret_cast<const float4*>(b + 24);
    return f32x16{a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w, e.x, e.y, e.z, e.w};
}

// registers 8s..8s+7 -> the bf16 B fragment of k-step s, then relu. Rounding to bf16
// keeps the sign (a small negative value rounds to -0), so relu after the rounding
// gives the bits relu before it did. The relu is a signed integer max with 0 on each
// bf16 pattern (a non-negative value orders like its int16 pattern, a negative one has
// the sign bit), two lanes per op: v_cvt_pk_bf16_f32 + v_pk_max_i16, 16 ops per
// 32-row tile where an f32 max per register took 24.
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(2))) float f32x2;
// a - b on two f32 lanes as two v_sub_f32 (SHIPENV_SCALAR_SUB): the vector form compiles to
// v_pk_add_f32, whose issue beside MFMAs costs more than two scalar subtractions
// (MI355X_MICROARCH.md, per-instruction constants). Exact either way.
#ifndef SHIPENV_SCALAR_SUB
#define SHIPENV_SCALAR_SUB 1  // fp32 policy 0.2617 -> 0.2605 ms, update 0.03685 -> 0.0368 ms (profiles/r05/ab_policy_f32_scalarsub.jsonl, ab_update_scalarsub.jsonl): about even
#endif
__device__ __forceinline__ f32x2 sub2(f32x2 a, f32x2 b) {
#if SHIPENV_SCALAR_SUB
    float r0, r1;
    asm("v_sub_f32 %0, %1, %2" : "=v"(r0) : "v"(a[0]), "v"(b[0]));
    asm("v_sub_f32 %0, %1, %2" : "=v"(r1) : "v"(a[1]), "v"(b[1]));
    return f32x2{r0, r1};
#else
    return a - b;
#endif
}
typedef __attribute__((ext_vector_type(2))) short i16x2;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
__device__ __forceinline__ void relu_pack(const f32x16& c, bf16x8 (&out)[2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        u32x4 w;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const bf16x2 b = __builtin_convertvector(f32x2{c[8 * s + 2 * p], c[8 * s + 2 * p + 1]}, bf16x2);
            const i16x2 i = __builtin_elementwise_max(__builtin_bit_cast(i16x2, b), i16x2{0, 0});
            w[p] = __builtin_bit_cast(uint32_t, i);
        }
        out[s] = __builtin_bit_cast(bf16x8, w);
    }
}

// bits i of [0, 32) with lo <= i <= hi
__device__ __forceinline__ uint32_t range_bits(int lo, int hi) {
    lo = max(lo, 0);
    hi = min(hi, 31);
    const uint32_t top = hi >= 31 ? 0xffffffffu : ((1u << (hi + 1)) - 1u);
    const uint32_t low = lo >= 32 ? 0xffffffffu : ((1u << lo) - 1u);
    return lo > hi ? 0u : (top & ~low);
}

// is_valid_action (dqn.py:125-175) of one env, as row ranges of a fc3 layout: moves
// always; SELECT p at the ship's cell and != origin; TAKE_CARGO / TAKE_FUEL at a port
// with 0 < amount <= stock. These helpers are the f32 policy kernel's form of the bf16
// kernel's inline epilogue (policy_kernel below keeps it inline: in helper form the
// compiler unrolled its fc3 loop and spilled SGPRs at its 128-VGPR budget); the GPU tests
// require both kernels to choose the same first maximum from the same Q rows.
struct EnvValid {
    int cur, cst, fst;       // port on the ship's cell (-1), its stocks capped to the amounts
    int c_lo, c_hi, f_lo, f_hi;
    uint64_t sel;            // SELECT: bit p for each port on the ship's cell other than the origin
};
__device__ __forceinline__ EnvValid env_valid(const LdsWorld& w, const QnetDims& q, const uint64_t* SAME, int x,
                                              int y, int origin) {
    EnvValid v;
    v.cur = w.port_at(x, y);
    v.cst = v.cur >= 0 ? min(w.pcargo(max(v.cur, 0)), 49) : 0;
    v.fst = v.cur >= 0 ? min(w.pfuel(max(v.cur, 0)), 199) : 0;
    v.c_lo = q.cargo_row1();
    v.c_hi = v.c_lo + v.cst - 1;
    v.f_lo = q.fuel_row1();
    v.f_hi = v.f_lo + v.fst - 1;
    v.sel = v.cur >= 0 ? SAME[max(v.cur, 0)] & ~(origin >= 0 ? 1ull << origin : 0ull) : 0ull;
    return v;
}

// env_valid from the ship's cell code and the stocks of its first port (read earlier, so
// the two dependent world reads are in flight during MFMA work)
__device__ __forceinline__ EnvValid env_valid_from(const LdsWorld& w, const QnetDims& q, const uint64_t* SAME, int code,
                                                   int2 stock, int origin) {
    EnvValid v;
    v.cur = w.port_of_code(code);
    v.cst = v.cur >= 0 ? min(stock.y, 49) : 0;
    v.fst = v.cur >= 0 ? min(stock.x, 199) : 0;
    v.c_lo = q.cargo_row1();
    v.c_hi = v.c_lo + v.cst - 1;
    v.f_lo = q.fuel_row1();
    v.f_hi = v.f_lo + v.fst - 1;
    v.sel = v.cur >= 0 ? SAME[max(v.cur, 0)] & ~(origin >= 0 ? 1ull << origin : 0ull) : 0ull;
    return v;
}

// can any row of tile mt be valid for this env (a tile no env of the wave can choose from
// is skipped, MFMAs included)
__device__ __forceinline__ bool tile_maybe(const EnvValid& v, int mt, int P) {
    const int base = mt * 32, top = base + 31;
    return (mt == 0) | ((v.cur >= 0) & (base < 4 + P)) | ((v.cst > 0) & (v.c_lo <= top) & (v.c_hi >= base)) |
           ((v.fst > 0) & (v.f_lo <= top) & (v.f_hi >= base));
}

// valid rows of tile mt as bits of the tile
__device__ __forceinline__ uint32_t tile_mask(const EnvValid& v, int mt, int P) {
    const int base = mt * 32;
    uint32_t m = range_bits(-base, 3 - base) | range_bits(v.c_lo - base, v.c_hi - base) |
                 range_bits(v.f_lo - base, v.f_hi - base);
    if (base < 4 + P) {  // SELECT rows 4 + p live in this tile (uniform): sel shifted by 4 - base
        const int sh = base - 4;
        m |= (uint32_t)(sh < 0 ? v.sel << -sh : (sh < 64 ? v.sel >> sh : 0ull));
    }
    return m;
}

// all of an env's valid rows (layouts of at most 64 rows) as one word: bit r = row r
__device__ __forceinline__ uint64_t valid_rows64(const EnvValid& v) {
    auto range64 = [](int lo, int hi) {  // bits lo..hi, 0 <= lo, hi <= 63; empty if hi < lo
        const uint64_t top = hi >= 63 ? ~0ull : ((2ull << (hi & 63)) - 1ull);
        const uint64_t low = (1ull << (lo & 63)) - 1ull;
        return hi < lo ? 0ull : (top & ~low);
    };
    return 0xfull | (v.sel << 4) | range64(v.c_lo, v.c_hi) | range64(v.f_lo, v.f_hi);
}

// the masked first maximum over one fc3 tile's accumulator (ascending rows), registers
// outside the wave-uniform mask rm skipped
__device__ __forceinline__ void tile_argmax(const f32x16& c, uint32_t m, uint32_t rm, int base, int h, float& best,
                                            int& bidx) {
    m >>= 4 * h;  // register reg holds row base + 4h + (reg & 3) + 8 (reg >> 2)
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        if (!((rm >> reg) & 1u)) continue;
        const int i = (reg & 3) + 8 * (reg >> 2);
        const bool better = ((m >> i) & 1u) && c[reg] > best;  // ascending rows: first max
        best = better ? c[reg] : best;
        bidx = better ? base + 4 * h + i : bidx;
    }
}

// bias rows of a fc3 tile, -inf where bit (reg & 3) + 8 (reg >> 2) of m is clear (the row
// is invalid for this env): its Q stays -inf through the MFMAs and never wins the argmax
__device__ __forceinline__ f32x16 masked_bias(const float* b, uint32_t m) {
    f32x16 c = bias_frag(b);
    uint32_t x = m & 0x0f0f0f0fu;  // register reg's bit to bit reg
    x = (x | (x >> 4)) & 0x00ff00ffu;
    x = (x | (x >> 8)) & 0x0000ffffu;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) c[reg] = ((x >> reg) & 1u) ? c[reg] : -INFINITY;
    return c;
}

// the first maximum over registers 4j..4j+3 of a masked tile (invalid rows are -inf), the
// row recorded without the lane half's 4h (added once at the end): one compare and two
// selects per register, no validity test and no per-register branch
__device__ __forceinline__ void argmax_masked_part(const f32x16& c, int base, float& best, int& bidx, int j) {
#pragma unroll
    for (int reg = 4 * j; reg < 4 * j + 4; ++reg) {
        const bool better = c[reg] > best;
        best = better ? c[reg] : best;
        bidx = better ? base + (reg & 3) + 8 * (reg >> 2) : bidx;
    }
}

// argmax_masked_part with the winner's tile-local row kept as an inline constant (bt); after
// part 3 the caller adds the tile's base once if the tile raised the maximum (best != best0)
__device__ __forceinline__ void argmax_local_part(const f32x16& c, float& best, int& bt, int j) {
#pragma unroll
    for (int reg = 4 * j; reg < 4 * j + 4; ++reg) {
        const bool better = c[reg] > best;
        best = better ? c[reg] : best;
        bt = better ? (reg & 3) + 8 * (reg >> 2) : bt;
    }
}

__device__ __forceinline__ void tile_q_out(float* q_out, int64_t ldq, int rows, const f32x16& c, int64_t e, int base,
                                           int h) {
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {  // the full layout: row = action
        const int row = base + 4 * h + (reg & 3) + 8 * (reg >> 2);
        if (row < rows) q_out[e * ldq + row] = c[reg];
    }
}

// the two lane halves of an env merged (larger value, then lower index), then
// epsilon-greedy (choose_action :186-203) and the action / replay record stores
#define FINISH_ENV(v, e, live, h, best, bidx, x8, y8, o8, d8, ff)                                             \
    finish_env(q, v, e, live, h, best, bidx, x8, y8, o8, d8, ff, A.actions, A.eps, A.seed, A.env_base, A.t,       \
               A.rec_pos, A.rec_fuel, A.rec_act, A.rec_head, A.rec_cap)
// the same with the env's epsilon draw words 0 and 1 already drawn (PairedDraws)
#define FINISH_ENV_D(v, e, live, h, best, bidx, x8, y8, o8, d8, ff, dw)                                        \
    finish_env(q, v, e, live, h, best, bidx, x8, y8, o8, d8, ff, A.actions, A.eps, A.seed, A.env_base, A.t,       \
               A.rec_pos, A.rec_fuel, A.rec_act, A.rec_head, A.rec_cap, &(dw))

// the epsilon draws of two tiles from one Philox pass: on even iterations lanes 0-31 draw
// for this tile's envs and lanes 32-63 for the next tile's (tile + stride), whose words
// move to lanes 0-31 and are kept for the odd iteration (a draw depends only on the env
// id, t and the slot, so the words are the same as drawing them one tile at a time)
// (the kept words wait in the wave's 32 x 8-byte LDS slot, not in registers)
constexpr int kPairedDrawBytes = 32 * 8;  // per wave
struct PairedDraws {
    uint2* slot;  // this wave's
    int it = 0;   // iteration parity (uniform)
    __device__ __forceinline__ U4 next(bool on, int64_t e, int64_t stride, int h, int r, uint64_t seed,
                                       int64_t env_base, uint32_t t) {
        U4 d{{0u, 0u, 0u, 0u}};
        if (on) {
            if ((it & 1) == 0) {
                const int64_t de = h ? e + stride * 32 : e;  // the env of this lane in tile + stride
                const U4 w = draw(env_key(seed, env_base + de), t, kSlotPolicy);
                d.v[0] = w.v[0];
                d.v[1] = w.v[1];
                if (h) slot[r] = make_uint2(w.v[0], w.v[1]);
            } else if (!h) {
                const uint2 w = slot[r];
                d.v[0] = w.x;
                d.v[1] = w.y;
            }
        }
        ++it;
        return d;
    }
};

__device__ __forceinline__ void finish_env(const QnetDims& q, const EnvValid& v, int64_t e, bool live, int h, float best,
                                           int bidx, uint32_t x8, uint32_t y8, uint32_t o8, uint32_t d8, float ff,
                                           int32_t* actions, double eps, uint64_t seed, int64_t env_base, uint32_t t,
                                           uint32_t* rec_pos, float* rec_fuel, int32_t* rec_act, int64_t rec_head,
                                           int64_t rec_cap, const U4* drawn = nullptr) {
    const float ob2 = __shfl_xor(best, 32);
    const int oi = __shfl_xor(bidx, 32);
    if (ob2 > best || (ob2 == best && oi < bidx)) {
        best = ob2;
        bidx = oi;
    }
    if (h == 0 && live) {
        const int P = q.P;
        int act = bidx == 0x7fffffff ? 0 : q.action_of_row(bidx);  // no valid action: 0 (:188-189)
        if (eps > 0.0) {
            const U4 d = drawn ? *drawn : draw(env_key(seed, env_base + e), t, kSlotPolicy);
            if (u32(d.v[0]) <= eps) {  // np.random.rand() <= epsilon (:191)
                // random.choice(valid_actions) (:192): the k-th valid action, ascending
                const int nsel = __popcll(v.sel);
                int k = uniform_int(d.v[1], (uint32_t)(4 + nsel + v.cst + v.fst));
                if (k < 4) {
                    act = k;
                } else if ((k -= 4) < nsel) {  // the k-th port of sel, ascending
                    uint64_t b = v.sel;
                    for (; k > 0; --k) b &= b - 1;
                    act = 4 + __builtin_ctzll(b);
                } else {
                    k -= nsel;
                    act = k < v.cst ? 5 + P + k : 55 + P + (k - v.cst);  // amounts k + 1 (action space)
                }
            }
        }
        actions[e] = act;
        if (rec_pos) {  // replay_begin_kernel's record, from the state already in registers
            int64_t slot = rec_head + e;
            slot -= slot >= rec_cap ? rec_cap : 0;
            rec_pos[slot] = x8 | y8 << 8 | o8 << 16 | d8 << 24;
            rec_fuel[slot] = ff;
            rec_act[slot] = act;
        }
    }
}

#ifndef SHIPENV_POLICY_B1FOLD
#define SHIPENV_POLICY_B1FOLD 1
#endif
// fc2 / fc3's biases by one extra MFMA per row tile against the fc1 input's ones, from
// fragments staged past the world (1 LDS read instead of 4): 63.95 vs 62.45 us with the fc1
// fold alone (profiles/r05/ab_policy_bf16_bias_fold.jsonl), not kept; the fc1 fold alone
// 63.05 -> 62.45 (and 63.1 -> 61.75 in a first A/B), kept
#ifndef SHIPENV_POLICY_BFOLD23
#define SHIPENV_POLICY_BFOLD23 0
#endif
#if SHIPENV_POLICY_BFOLD23 && !SHIPENV_POLICY_B1FOLD
#error "SHIPENV_POLICY_BFOLD23 needs SHIPENV_POLICY_B1FOLD (the input's k = 8..10 ones)"
#endif
#ifndef SHIPENV_POLICY_LOCAL_IDX
#define SHIPENV_POLICY_LOCAL_IDX 1
#endif
#ifndef SHIPENV_POLICY_VALID64
#define SHIPENV_POLICY_VALID64 1  // 63.1 -> 61.0 us (profiles/r05/ab_policy_bf16_valid64.jsonl, five alternating rounds); 0: per-tile masks
#endif
#ifndef SHIPENV_POLICY_EARLY_ENV
#define SHIPENV_POLICY_EARLY_ENV 0  // 1: the first tile's env loads before the image / world staging: 64.9 vs 64.45 us (profiles/r05/ab_policy_bf16_early_env.jsonl), not kept
#endif
#ifndef SHIPENV_POLICY_DRAW_PAIR
#define SHIPENV_POLICY_DRAW_PAIR 0  // 1: one Philox pass per two tiles' epsilon draws (PairedDraws): within noise in three alternating A/Bs (bf16 0.0602 -> 0.0595, 0.0597 -> 0.0599, 0.0604 -> 0.0602 ms; fp32 0.2668 -> 0.2641 and, words held in registers, 0.2591 -> 0.261; profiles/r05/ab_policy_*_drawpair*.jsonl), one or three VGPRs spilled: not kept
#endif
#ifndef SHIPENV_POLICY_STAGE_BATCH
#define SHIPENV_POLICY_STAGE_BATCH 0  // 1: policy_kernel's image copy as four loads per thread before one wait: 0.0598 -> 0.0602 and 0.0593 -> 0.0600 ms (profiles/r05/ab_policy_bf16_stage.jsonl), not kept
#endif
// n 16-byte words global -> LDS by a block of `block` threads: four loads per thread issued
// (past the end: the last word again), one wait, four guarded stores
__device__ __forceinline__ void copy_to_lds(const uint4* __restrict__ g, uint4* l, int n, int block) {
    for (int i0 = 0; i0 < n; i0 += 4 * block) {
        uint4 r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = g[min(i0 + (int)threadIdx.x + k * block, n - 1)];
        // the loads stay ahead of the guarded stores (not sunk into them, one wait each)
        for (int k = 0; k < 4; ++k) asm volatile("" ::"v"(r[k].x), "v"(r[k].y), "v"(r[k].z), "v"(r[k].w));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = i0 + (int)threadIdx.x + k * block;
            if (i < n) l[i] = r[k];
        }
    }
}
#ifndef SHIPENV_POLICY_EPS_INT
#define SHIPENV_POLICY_EPS_INT 0  // 1: policy_kernel's explore test as an integer compare with eps_threshold: 0.05985 -> 0.0607 ms (profiles/r05/ab_policy_bf16_epsint.jsonl), not kept
#endif
// u32(w) <= eps (w * 2^-32 in double, exact) as an integer test w <= eps_threshold(eps), for
// 0 < eps: w <= eps * 2^32 (exact: a power-of-two scaling) <=> w <= floor(eps * 2^32) for an
// integer w, and every w passes once eps >= 1 (u32(w) < 1)
__device__ __forceinline__ uint32_t eps_threshold(double eps) {
    return eps >= 1.0 ? 0xFFFFFFFFu : (uint32_t)floor(eps * 4294967296.0);
}
#ifndef SHIPENV_POLICY_RM_SKIP
#define SHIPENV_POLICY_RM_SKIP 1  // 0: every register of an fc3 tile tested: 0.0591 -> 0.0603 ms (profiles/r05/ab_policy_bf16_rmskip.jsonl), not kept
#endif
#ifndef SHIPENV_POLICY_WAVE_SKIP
#define SHIPENV_POLICY_WAVE_SKIP 0  // 1: fc3 tiles / registers also skipped by the wave's union of valid rows (DPP OR per env tile): 0.0592 -> 0.0615 ms, and 0.0595 -> 0.0618 in config 5's state (profiles/r05/ab_policy_bf16_waveskip*.jsonl; 99.9 % of waves hold an env at a port), not kept
#endif
// OR over the 64 lanes of a wave, wave-uniform: a prefix OR within each 16-lane row (DPP
// row_shr 1, 2, 4, 8), then the four rows' last lanes
__device__ __forceinline__ uint32_t wave_or32(uint32_t x) {
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
    return (uint32_t)(__builtin_amdgcn_readlane((int)x, 15) | __builtin_amdgcn_readlane((int)x, 31) |
                      __builtin_amdgcn_readlane((int)x, 47) | __builtin_amdgcn_readlane((int)x, 63));
}
__device__ __forceinline__ uint64_t wave_or64(uint64_t x) {
    return (uint64_t)wave_or32((uint32_t)x) | (uint64_t)wave_or32((uint32_t)(x >> 32)) << 32;
}
#ifndef SHIPENV_POLICY_NXT_WAIT
#define SHIPENV_POLICY_NXT_WAIT 1  // the next tile's loads waited for before the stores (policy_kernel): 0.0598 -> 0.0593 ms (profiles/r05/ab_policy_bf16_stage.jsonl)
#endif
#ifndef SHIPENV_POLICY_PRIO
#define SHIPENV_POLICY_PRIO 3  // static issue priorities of each SIMD's waves (see policy_kernel): 3 (the youngest wave at 1) 0.0602 -> 0.05955 ms (profiles/r05/ab_policy_bf16_prio.jsonl), 1 and 2 0.0599
#endif
#ifndef SHIPENV_POLICY_MASKED
#define SHIPENV_POLICY_MASKED 0  // 1: masked -inf fc3 bias + branch-free argmax (63.5 vs 63.4 us, profiles/r05/ab_policy_bf16_masked.jsonl: not kept); 0: the round-4 epilogue
#endif
template <bool kQout>
__global__ __launch_bounds__(kPolicyBlock)
#if SHIPENV_POLICY_WAVES_PER_EU
__attribute__((amdgpu_waves_per_eu(SHIPENV_POLICY_WAVES_PER_EU)))
#endif
void policy_kernel(PolicyArgs A) {
    extern __shared__ uint4 smem[];
    const QnetDims q = A.q;
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const int64_t tiles = (A.n + 31) >> 5;
    // env state of one tile (lane & 31 = env); the next tile's is loaded while this one
    // computes, so the wave does not wait on HBM at the top of every tile. The first tile's
    // loads go out before the network image and the world are staged, so they overlap.
    struct EnvIn {
        double fuel;
        uint32_t x, y, o8, d8;
    };
    auto load_env = [&](int64_t tile) {
        const int64_t e = tile * 32 + r;
        const int64_t ei = e < A.n ? e : A.n - 1;
        return EnvIn{A.st.fuel[ei], A.st.x[ei], A.st.y[ei], A.st.origin[ei], A.st.dest[ei]};
    };
    int64_t tile = (int64_t)blockIdx.x * kPolicyWaves + (threadIdx.x >> 6);
#if SHIPENV_POLICY_PRIO == 1  // each SIMD's waves at static issue priorities 0..3 (wave >> 2)
    {
        const int pw = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >> 2;  // the immediate is a constant
        if (pw == 1) __builtin_amdgcn_s_setprio(1);
        else if (pw == 2) __builtin_amdgcn_s_setprio(2);
        else if (pw == 3) __builtin_amdgcn_s_setprio(3);
    }
#elif SHIPENV_POLICY_PRIO == 2  // each SIMD's younger two waves at priority 1
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= 8) __builtin_amdgcn_s_setprio(1);
#elif SHIPENV_POLICY_PRIO == 3  // each SIMD's youngest wave at priority 1
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= 12) __builtin_amdgcn_s_setprio(1);
#endif
#if SHIPENV_POLICY_EARLY_ENV
    EnvIn nxt = load_env(tile < tiles ? tile : 0);
#endif
    const int qwords = q.bytes() / 16;
#if SHIPENV_POLICY_B1FOLD
    // fc1's bias rides in the padding half of its single k-step: lanes 32-63 of each W1
    // fragment (k = 8..15, zero in the packed image) get the three bf16 parts of their row's
    // b1 at elements 0-2, and the input's k = 8..10 are 1.0, so the chain starts at 0 and the
    // bias is not read per tile (4 x 16-byte LDS reads per row tile)
    const int w1w = q.w1() / 16, b1f = q.b1() / 4;
#if SHIPENV_POLICY_STAGE_BATCH
    // the image in batches of four 16-byte loads per thread, all issued before one wait
    // (left to itself the compiler sank each load into its guarded store and waited on
    // every one); then each patched W1 fragment lane by the thread that copied it
    copy_to_lds(A.qimg, smem, qwords, kPolicyBlock);
    {
        int k = (int)threadIdx.x - w1w % kPolicyBlock;  // W1 fragment (mt, lane) = k: mt = k >> 6, lane = k & 63
        k += k < 0 ? kPolicyBlock : 0;                  // w1w + k == threadIdx.x (mod the block)
        if (k < 4 * 64 && (k & 32)) {
            const float b = reinterpret_cast<const float*>(A.qimg)[b1f + (k >> 6) * 32 + (k & 31)];
            __bf16 p0, p1, p2;
            split3(b, p0, p1, p2);
            bf16x8 v{};
            v[0] = p0;
            v[1] = p1;
            v[2] = p2;
            smem[w1w + k] = __builtin_bit_cast(uint4, v);
        }
    }
#else
    for (int i = threadIdx.x; i < qwords; i += kPolicyBlock) {
        const int k = i - w1w;  // W1 fragment (mt, lane) = k: mt = k >> 6, lane = k & 63
        if ((unsigned)k < 4u * 64u && (k & 32)) {
            const float b = reinterpret_cast<const float*>(A.qimg)[b1f + (k >> 6) * 32 + (k & 31)];
            __bf16 p0, p1, p2;
            split3(b, p0, p1, p2);
            bf16x8 v{};
            v[0] = p0;
            v[1] = p1;
            v[2] = p2;
            smem[i] = __builtin_bit_cast(uint4, v);
        } else {
            smem[i] = A.qimg[i];
        }
    }
#endif
#else
    for (int i = threadIdx.x; i < qwords; i += kPolicyBlock) smem[i] = A.qimg[i];
#endif
#if SHIPENV_POLICY_BFOLD23
    // fc2 / fc3's bias fragments past the world image: (tile, lane) = the three bf16 parts of
    // the tile row's bias at elements 0-2 of lanes 32-63 (k = 8..10), zero elsewhere. One
    // MFMA of a fragment against the fc1 input (1.0 at k = 8..10, SHIPENV_POLICY_B1FOLD) starts
    // a chain at its bias: one 16-byte LDS read per row tile instead of four.
    uint4* BFw = smem + qwords + A.dims.padded() / 4;
    {
        const int nb = (4 + q.mt3) * 64, b2f = q.b2() / 4, b3f = q.b3() / 4;
        for (int i = threadIdx.x; i < nb; i += kPolicyBlock) {
            const int tl = i >> 6, l = i & 63;
            bf16x8 v{};
            if (l & 32) {
                const int row = (tl < 4 ? tl : tl - 4) * 32 + (l & 31);
                const float b = reinterpret_cast<const float*>(A.qimg)[(tl < 4 ? b2f : b3f) + row];
                __bf16 p0, p1, p2;
                split3(b, p0, p1, p2);
                v[0] = p0;
                v[1] = p1;
                v[2] = p2;
            }
            BFw[i] = __builtin_bit_cast(uint4, v);
        }
    }
    const bf16x8* BF = reinterpret_cast<const bf16x8*>(BFw);
#endif
    const LdsWorld w = stage_world(A.world, A.dims, reinterpret_cast<uint32_t*>(smem + qwords));
    const uint8_t* qb = reinterpret_cast<const uint8_t*>(smem);
    const bf16x8* W1f = reinterpret_cast<const bf16x8*>(qb + q.w1());
    const bf16x8* W2f = reinterpret_cast<const bf16x8*>(qb + q.w2());
    const bf16x8* W3f = reinterpret_cast<const bf16x8*>(qb + q.w3());
    [[maybe_unused]] const float* B1 = reinterpret_cast<const float*>(qb + q.b1());
    [[maybe_unused]] const float* B2 = reinterpret_cast<const float*>(qb + q.b2());
    const float* B3 = reinterpret_cast<const float*>(qb + q.b3());
    const uint64_t* SAME = reinterpret_cast<const uint64_t*>(qb + q.same());
    const uint32_t* REGM = reinterpret_cast<const uint32_t*>(qb + q.regm());

    const int P = q.P;
    const int64_t stride = (int64_t)gridDim.x * kPolicyWaves;
#if !SHIPENV_POLICY_EARLY_ENV
    EnvIn nxt = load_env(tile < tiles ? tile : 0);
#endif
#if SHIPENV_POLICY_EPS_INT
    const uint32_t eps_thr = eps_threshold(A.eps);
#endif
#if SHIPENV_POLICY_DRAW_PAIR
    // past the world image (and the bias fragments of SHIPENV_POLICY_BFOLD23)
    PairedDraws pd{reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(smem + qwords + A.dims.padded() / 4) +
                                            (SHIPENV_POLICY_BFOLD23 ? (4 + q.mt3) * 1024 : 0) +
                                            __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * kPairedDrawBytes)};
#endif
    for (; tile < tiles; tile += stride) {
        const EnvIn cur_in = nxt;
        if (tile + stride < tiles) nxt = load_env(tile + stride);
        const int64_t e = tile * 32 + r;
        const bool live = e < A.n;
        const int x = (int)cur_in.x, y = (int)cur_in.y;
        const int origin = cur_in.o8 == SE_NONE ? -1 : (int)cur_in.o8;
        const int dest = cur_in.d8 == SE_NONE ? -1 : (int)cur_in.d8;
        // the observation row (preprocess_state): torch's .float() of the f64 fuel,
        // as bf16 hi + lo so fc1 sees ~16 bits of it
        const float ff = (float)cur_in.fuel;
        const __bf16 fh = (__bf16)ff, fl = (__bf16)(ff - (float)fh);
        bf16x8 ob;
        ob[0] = (__bf16)(float)x;
        ob[1] = (__bf16)(float)y;
        ob[2] = fh;
        ob[3] = fl;
        ob[4] = fh;
        ob[5] = fl;
        ob[6] = (__bf16)(float)origin;
        ob[7] = (__bf16)(float)dest;
#if SHIPENV_POLICY_B1FOLD
        if (h) {  // k = 8..10: 1.0 against the bias parts, 11..15 padding
            ob = bf16x8{};
            ob[0] = ob[1] = ob[2] = (__bf16)1.0f;
        }
#else
        if (h) ob = bf16x8{};  // k = 8..15 of the single fc1 step are padding
#endif

        bf16x8 h1[4][2], h2[4][2];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {  // fc1 + relu
#if SHIPENV_POLICY_B1FOLD
            f32x16 c = {};
#else
            f32x16 c = PBIAS(B1 + mt * 32 + 4 * h);
#endif
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(W1f[mt * 64 + lane], ob, c, 0, 0, 0);
            relu_pack(c, h1[mt]);
        }
#ifndef SHIPENV_FC2_SPLIT
#define SHIPENV_FC2_SPLIT 4  // one pass per row tile: no spills at 128 VGPRs (2 passes spill 7, 1 spills 14)
#endif
#ifndef SHIPENV_POLICY_LOOKAHEAD
#define SHIPENV_POLICY_LOOKAHEAD 1  // fc2 fragments read this many k-steps ahead (0: as needed); 2 and 3 now fit 128 VGPRs and measure even (0.0603 / 0.0601 / 0.061 ms, profiles/r05/ab_policy_bf16_la.jsonl)
#endif
        // fc2 + relu in SHIPENV_FC2_SPLIT passes over the 4 row tiles: the tiles of a pass
        // advance together (consecutive MFMAs independent, a k-step's fragments read in one
        // batch); with two passes the accumulators take 32 VGPRs instead of 64 and the
        // first pass's relu can issue in the shadow of the second pass's MFMAs
        constexpr int kFc2Tiles = 4 / SHIPENV_FC2_SPLIT;
#pragma unroll
        for (int pass = 0; pass < SHIPENV_FC2_SPLIT; ++pass) {
            f32x16 c2[kFc2Tiles];
#pragma unroll
            for (int i = 0; i < kFc2Tiles; ++i)
#if SHIPENV_POLICY_BFOLD23
                c2[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(BF[(pass * kFc2Tiles + i) * 64 + lane], ob, f32x16{}, 0, 0, 0);
#else
                c2[i] = PBIAS(B2 + (pass * kFc2Tiles + i) * 32 + 4 * h);
#endif
#if SHIPENV_POLICY_LOOKAHEAD > 0
            static_assert(kFc2Tiles == 1, "the fragment lookahead is written for one tile per pass");
            // the tile's 8 fragments read SHIPENV_POLICY_LOOKAHEAD k-steps ahead of their MFMA,
            // pinned in that order (one LDS read, one MFMA): left to itself the compiler read
            // each fragment right before its MFMA and waited out the LDS round trip every time
            constexpr int L = SHIPENV_POLICY_LOOKAHEAD;
            bf16x8 wf[8];
#pragma unroll
            for (int k = 0; k < L; ++k) wf[k] = W2f[(SHIPENV_POLICY_ABL == 8 ? 0 : (pass * 8 + k)) * 64 + lane];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (k + L < 8) wf[k + L] = W2f[(SHIPENV_POLICY_ABL == 8 ? 0 : (pass * 8 + k + L)) * 64 + lane];
                c2[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[k], h1[k >> 1][k & 1], c2[0], 0, 0, 0);
            }
#pragma unroll
            for (int k = 0; k < L; ++k) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (k + L < 8) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            }
#else
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    bf16x8 wf[kFc2Tiles];
#pragma unroll
                    for (int i = 0; i < kFc2Tiles; ++i)
                        wf[i] = W2f[(((pass * kFc2Tiles + i) * 4 + kt) * 2 + s) * 64 + lane];
#pragma unroll
                    for (int i = 0; i < kFc2Tiles; ++i)
                        c2[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i], h1[kt][s], c2[i], 0, 0, 0);
                }
#endif
#pragma unroll
            for (int i = 0; i < kFc2Tiles; ++i) relu_pack(c2[i], h2[pass * kFc2Tiles + i]);
        }

        // is_valid_action (dqn.py:125-175): moves always; SELECT p at the ship's cell
        // and != origin; TAKE_CARGO / TAKE_FUEL at a port with 0 < amount <= stock
        const int cur = w.port_at(x, y);
        const int cst = cur >= 0 ? min(w.pcargo(max(cur, 0)), 49) : 0;
        const int fst = cur >= 0 ? min(w.pfuel(max(cur, 0)), 199) : 0;
        // valid TAKE rows of this env in the layout's row space
        const int c_lo = q.cargo_row1(), c_hi = c_lo + cst - 1, f_lo = q.fuel_row1(), f_hi = f_lo + fst - 1;
        // SELECT: bit p for each port on the ship's cell other than the origin (P <= 64)
        const uint64_t sel = cur >= 0 ? SAME[max(cur, 0)] & ~(origin >= 0 ? 1ull << origin : 0ull) : 0ull;
#if SHIPENV_POLICY_VALID64
        // (compact layouts of at most 64 rows, every greedy call of the bench) the env's valid
        // rows as one 64-bit word, built once per env tile: a fc3 tile's mask is then a shift
        // of it and "any row of this tile valid" its being nonzero, where the per-tile form
        // rebuilt three ranges and the SELECT shift for each fc3 tile
        const bool use64 = !kQout && q.mt3 <= 2;  // uniform
        uint64_t v64 = 0;
        if (use64) {
            auto range64 = [](int lo, int hi) {  // bits lo..hi, 0 <= lo, hi <= 63; empty if hi < lo
                const uint64_t top = hi >= 63 ? ~0ull : ((2ull << (hi & 63)) - 1ull);
                const uint64_t low = (1ull << (lo & 63)) - 1ull;
                return hi < lo ? 0ull : (top & ~low);
            };
            v64 = 0xfull | (sel << 4) | range64(c_lo, c_hi) | range64(f_lo, f_hi);
        }
#if SHIPENV_POLICY_WAVE_SKIP
        // the rows any env of the wave can take (wave-uniform): an fc3 tile's registers that
        // hold none of them are skipped, the moves-only registers of a wave at sea included
        const uint64_t u64 = use64 ? wave_or64(v64) : ~0ull;
#endif
#endif
        float best = -INFINITY;
        int bidx = 0x7fffffff;
#if SHIPENV_POLICY_ABL == 2  // timing-only: no fc3
        for (int mt = 0; mt < 0; ++mt) {
#else
        for (int mt = 0; mt < q.mt3; ++mt) {  // fc3 + the masked first-maximum argmax
#endif
            const int base = mt * 32, top = base + 31;
            // a tile no env of the wave can choose from is skipped, MFMAs included
            // (exact: its rows are invalid for all 32 envs); with port stocks <= 20
            // (add_port's randint(5, 20)) the valid rows sit in the first few tiles
            uint32_t m;
#if SHIPENV_POLICY_VALID64
            if (use64) {
                m = (uint32_t)(v64 >> (base & 63));
#if SHIPENV_POLICY_WAVE_SKIP
                if ((uint32_t)(u64 >> (base & 63)) == 0u) continue;
#else
                if (!__any(m != 0u)) continue;
#endif
            } else
#endif
            {
                const bool maybe = (mt == 0) | ((cur >= 0) & (base < 4 + P)) |
                                   ((cst > 0) & (c_lo <= top) & (c_hi >= base)) |
                                   ((fst > 0) & (f_lo <= top) & (f_hi >= base));
                if (!kQout && !__any(maybe)) continue;
                m = range_bits(-base, 3 - base) | range_bits(c_lo - base, c_hi - base) |
                    range_bits(f_lo - base, f_hi - base);
                if (base < 4 + P) {  // SELECT rows 4 + p live in this tile (uniform): sel shifted by 4 - base
                    const int sh = base - 4;
                    m |= (uint32_t)(sh < 0 ? sel << -sh : (sh < 64 ? sel >> sh : 0ull));
                }
            }
            // registers that hold no valid action for any env are skipped (wave-uniform)
#if SHIPENV_POLICY_VALID64 && SHIPENV_POLICY_WAVE_SKIP
            uint32_t rm = __builtin_amdgcn_readfirstlane(REGM[mt]);
            if (use64) {  // ... and those that hold none for this wave's envs
                uint32_t u2 = (uint32_t)(u64 >> (base & 63));
                u2 |= u2 >> 4;  // lane half h holds rows 4h + (reg & 3) + 8 (reg >> 2)
                rm &= (u2 & 0xFu) | ((u2 >> 4) & 0xF0u) | ((u2 >> 8) & 0xF00u) | ((u2 >> 12) & 0xF000u);
            }
#else
            const uint32_t rm = __builtin_amdgcn_readfirstlane(REGM[mt]);
#endif
            bf16x8 wf[8];  // the tile's 8 fragments, read before the chain consumes them
#pragma unroll
            for (int k = 0; k < 8; ++k) wf[k] = W3f[(mt * 8 + k) * 64 + lane];
            // without q_out (round 5): rows this env cannot take start at -inf (masked_bias), so
            // the first maximum below needs no validity test and no per-register branch
            constexpr bool kMasked = !kQout && SHIPENV_POLICY_MASKED;
#if SHIPENV_POLICY_BFOLD23
            f32x16 c = kMasked ? masked_bias(B3 + mt * 32 + 4 * h, m >> (4 * h))
                               : __builtin_amdgcn_mfma_f32_32x32x16_bf16(BF[(4 + mt) * 64 + lane], ob, f32x16{}, 0, 0, 0);
#else
            f32x16 c = kMasked ? masked_bias(B3 + mt * 32 + 4 * h, m >> (4 * h)) : PBIAS(B3 + mt * 32 + 4 * h);
#endif
#pragma unroll
            for (int k = 0; k < 8; ++k)
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[k], h2[k >> 1][k & 1], c, 0, 0, 0);
            m >>= 4 * h;  // register reg holds row base + 4h + (reg & 3) + 8 (reg >> 2)
#if SHIPENV_POLICY_ABL == 1  // timing-only: the epilogue without masks or indices
            (void)m;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) best = fmaxf(best, c[reg]);
            bidx = base;
#else
            if constexpr (kMasked) {
#pragma unroll
                for (int j = 0; j < 4; ++j) argmax_masked_part(c, base, best, bidx, j);  // rows without 4h
            } else {
#if SHIPENV_POLICY_LOCAL_IDX
                // the winning register's tile-local row as an inline constant, the tile's base
                // added once if the tile raised the maximum (strict >: the first maximum stays)
                const float best0 = best;
                int bt = 0;
#pragma unroll
                for (int reg = 0; reg < 16; ++reg) {
                    // (SHIPENV_POLICY_RM_SKIP 0: no per-register skip; the row masks already
                    // exclude every row no env can take, and the skip's branches were laid out
                    // with the common case taken twice per register)
                    if (SHIPENV_POLICY_RM_SKIP && !((rm >> reg) & 1u)) continue;
                    const int i = (reg & 3) + 8 * (reg >> 2);
                    const bool better = ((m >> i) & 1u) && c[reg] > best;  // ascending rows: first max
                    best = better ? c[reg] : best;
                    bt = better ? i : bt;
                }
                bidx = best != best0 ? base + 4 * h + bt : bidx;
#else
#pragma unroll
                for (int reg = 0; reg < 16; ++reg) {
                    if (!((rm >> reg) & 1u)) continue;
                    const int i = (reg & 3) + 8 * (reg >> 2);
                    const bool better = ((m >> i) & 1u) && c[reg] > best;  // ascending rows: first max
                    best = better ? c[reg] : best;
                    bidx = better ? base + 4 * h + i : bidx;
                }
#endif
            }
#endif
            if (kQout && live) {
#pragma unroll
                for (int reg = 0; reg < 16; ++reg) {  // the full layout: row = action
                    const int row = base + 4 * h + (reg & 3) + 8 * (reg >> 2);
                    if (row < q.rows) A.q_out[e * A.ldq + row] = c[reg];
                }
            }
        }
        if (!kQout && SHIPENV_POLICY_MASKED) bidx += bidx == 0x7fffffff ? 0 : 4 * h;  // the lane half's rows
#if SHIPENV_POLICY_NXT_WAIT
        // the next tile's env loads (issued a tile ago) are waited for here, before this
        // tile's stores: stores count in vmcnt too, so a wait at the loop's back edge would
        // wait out the action / record stores' round trip as well
        asm volatile("" ::"v"(nxt.fuel), "v"(nxt.x), "v"(nxt.y), "v"(nxt.o8), "v"(nxt.d8));
#endif
        // the two lane halves hold the same env: larger value, then lower index
        const float ob2 = __shfl_xor(best, 32);
        const int oi = __shfl_xor(bidx, 32);
        if (ob2 > best || (ob2 == best && oi < bidx)) {
            best = ob2;
            bidx = oi;
        }
#if SHIPENV_POLICY_DRAW_PAIR
        const U4 dw = pd.next(A.eps > 0.0, e, stride, h, lane & 31, A.seed, A.env_base, A.t);
#endif
        if (h == 0 && live) {
            int act = bidx == 0x7fffffff ? 0 : q.action_of_row(bidx);  // no valid action: 0 (:188-189)
            if (A.eps > 0.0) {
#if SHIPENV_POLICY_DRAW_PAIR
                const U4 d = dw;
#else
                const U4 d = draw(env_key(A.seed, A.env_base + e), A.t, kSlotPolicy);
#endif
#if SHIPENV_POLICY_EPS_INT
                if (d.v[0] <= eps_thr) {  // np.random.rand() <= epsilon (:191), as an integer compare
#else
                if (u32(d.v[0]) <= A.eps) {  // np.random.rand() <= epsilon (:191)
#endif
                    // random.choice(valid_actions) (:192): the k-th valid action, ascending
                    const int nsel = __popcll(sel);
                    int k = uniform_int(d.v[1], (uint32_t)(4 + nsel + cst + fst));
                    if (k < 4) {
                        act = k;
                    } else if ((k -= 4) < nsel) {  // the k-th port of sel, ascending
                        uint64_t b = sel;
                        for (; k > 0; --k) b &= b - 1;
                        act = 4 + __builtin_ctzll(b);
                    } else {
                        k -= nsel;
                        act = k < cst ? 5 + P + k : 55 + P + (k - cst);  // amounts k + 1 (action space)
                    }
                }
            }
            A.actions[e] = act;
            if (A.rec_pos) {  // replay_begin_kernel's record, from the state already in registers
                int64_t slot = A.rec_head + e;
                slot -= slot >= A.rec_cap ? A.rec_cap : 0;
                A.rec_pos[slot] = cur_in.x | cur_in.y << 8 | cur_in.o8 << 16 | cur_in.d8 << 24;
                A.rec_fuel[slot] = ff;
                A.rec_act[slot] = act;
            }
        }
        (void)dest;
    }
}

// ------------------------------------------------------------------ the paired-tile form
// (SHIPENV_POLICY_PAIR, compact layouts of at most 64 rows, no q_out) The same step with two
// 32-env tiles per wave iteration: every fragment read from LDS feeds two MFMAs (one per
// tile), so a wave reads the network half as often per env and has two independent
// accumulation chains in flight; 512-thread workgroups, two waves per SIMD at up to 256
// VGPRs (the two tiles' activations). Results are those of policy_kernel<false>: the same
// bf16 products in the same order per env, the same masked first maximum and draws.
// Measured slower: 0.0603 -> 0.0723 ms per call in config 5's state (226 VGPRs, two waves per
// SIMD; profiles/r05/ab_policy_bf16_pair.jsonl), so halving the fragment reads does not pay for
// the halved occupancy; off by default (the policy tests pass on it: SHIPENV_POLICY_PAIR=1)
#ifndef SHIPENV_POLICY_PAIR
#define SHIPENV_POLICY_PAIR 0
#endif
constexpr int kPairBlock = 512;
constexpr int kPairWaves = kPairBlock / 64;
__global__ __launch_bounds__(kPairBlock) void policy_pair_kernel(PolicyArgs A) {
    extern __shared__ uint4 smem[];
    const QnetDims q = A.q;
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const int64_t tiles = (A.n + 31) >> 5, pairs = (tiles + 1) >> 1;
    struct EnvIn {
        double fuel;
        uint32_t x, y, o8, d8;
    };
    auto load_env = [&](int64_t tile) {
        const int64_t e = tile * 32 + r;
        const int64_t ei = e < A.n ? e : A.n - 1;
        return EnvIn{A.st.fuel[ei], A.st.x[ei], A.st.y[ei], A.st.origin[ei], A.st.dest[ei]};
    };
    int64_t pair = (int64_t)blockIdx.x * kPairWaves + (threadIdx.x >> 6);
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= 4) __builtin_amdgcn_s_setprio(1);  // each SIMD's second wave
    const int qwords = q.bytes() / 16;
    {  // the image, fc1's bias in the padding half of its k-step (policy_kernel, SHIPENV_POLICY_B1FOLD)
        const int w1w = q.w1() / 16, b1f = q.b1() / 4;
        for (int i = threadIdx.x; i < qwords; i += kPairBlock) {
            const int k = i - w1w;
            if ((unsigned)k < 4u * 64u && (k & 32)) {
                const float b = reinterpret_cast<const float*>(A.qimg)[b1f + (k >> 6) * 32 + (k & 31)];
                __bf16 p0, p1, p2;
                split3(b, p0, p1, p2);
                bf16x8 v{};
                v[0] = p0;
                v[1] = p1;
                v[2] = p2;
                smem[i] = __builtin_bit_cast(uint4, v);
            } else {
                smem[i] = A.qimg[i];
            }
        }
    }
    const LdsWorld w = stage_world(A.world, A.dims, reinterpret_cast<uint32_t*>(smem + qwords));
    const uint8_t* qb = reinterpret_cast<const uint8_t*>(smem);
    const bf16x8* W1f = reinterpret_cast<const bf16x8*>(qb + q.w1());
    const bf16x8* W2f = reinterpret_cast<const bf16x8*>(qb + q.w2());
    const bf16x8* W3f = reinterpret_cast<const bf16x8*>(qb + q.w3());
    const float* B2 = reinterpret_cast<const float*>(qb + q.b2());
    const float* B3 = reinterpret_cast<const float*>(qb + q.b3());
    const uint64_t* SAME = reinterpret_cast<const uint64_t*>(qb + q.same());
    const uint32_t* REGM = reinterpret_cast<const uint32_t*>(qb + q.regm());
    const int64_t stride = (int64_t)gridDim.x * kPairWaves;
    EnvIn nxt[2];
    {
        const int64_t p0 = pair < pairs ? pair : 0;
        nxt[0] = load_env(2 * p0);
        nxt[1] = load_env(2 * p0 + 1);
    }
    for (; pair < pairs; pair += stride) {
        EnvIn cur[2] = {nxt[0], nxt[1]};
        if (pair + stride < pairs) {
            nxt[0] = load_env(2 * (pair + stride));
            nxt[1] = load_env(2 * (pair + stride) + 1);
        }
        bf16x8 ob[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {  // the observation rows (policy_kernel)
            const float ff = (float)cur[t].fuel;
            const __bf16 fh = (__bf16)ff, fl = (__bf16)(ff - (float)fh);
            const int origin = cur[t].o8 == SE_NONE ? -1 : (int)cur[t].o8;
            const int dest = cur[t].d8 == SE_NONE ? -1 : (int)cur[t].d8;
            bf16x8 o;
            o[0] = (__bf16)(float)(int)cur[t].x;
            o[1] = (__bf16)(float)(int)cur[t].y;
            o[2] = fh;
            o[3] = fl;
            o[4] = fh;
            o[5] = fl;
            o[6] = (__bf16)(float)origin;
            o[7] = (__bf16)(float)dest;
            if (h) {  // k = 8..10: 1.0 against fc1's bias parts
                o = bf16x8{};
                o[0] = o[1] = o[2] = (__bf16)1.0f;
            }
            ob[t] = o;
        }
        bf16x8 h1[2][4][2], h2[2][4][2];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {  // fc1 + relu
            const bf16x8 f = W1f[mt * 64 + lane];
#pragma unroll
            for (int t = 0; t < 2; ++t)
                relu_pack(__builtin_amdgcn_mfma_f32_32x32x16_bf16(f, ob[t], f32x16{}, 0, 0, 0), h1[t][mt]);
        }
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {  // fc2 + relu, one row tile at a time, the two tiles' chains side by side
            const f32x16 b = bias_frag(B2 + mt * 32 + 4 * h);
            f32x16 c2[2] = {b, b};
            bf16x8 wf[2];
            wf[0] = W2f[(mt * 8) * 64 + lane];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (k + 1 < 8) wf[(k + 1) & 1] = W2f[(mt * 8 + k + 1) * 64 + lane];
#pragma unroll
                for (int t = 0; t < 2; ++t)
                    c2[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[k & 1], h1[t][k >> 1][k & 1], c2[t], 0, 0, 0);
            }
#pragma unroll
            for (int t = 0; t < 2; ++t) relu_pack(c2[t], h2[t][mt]);
        }
        EnvValid v[2];
        uint64_t v64[2];
        float best[2];
        int bidx[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            v[t] = env_valid(w, q, SAME, (int)cur[t].x, (int)cur[t].y, cur[t].o8 == SE_NONE ? -1 : (int)cur[t].o8);
            v64[t] = valid_rows64(v[t]);
            best[t] = -INFINITY;
            bidx[t] = 0x7fffffff;
        }
        for (int mt = 0; mt < q.mt3; ++mt) {  // fc3 + the masked first maximum (policy_kernel)
            const int base = mt * 32;
            const uint32_t m0 = (uint32_t)(v64[0] >> (base & 63)), m1 = (uint32_t)(v64[1] >> (base & 63));
            if (!__any((m0 | m1) != 0u)) continue;
            const uint32_t rm = __builtin_amdgcn_readfirstlane(REGM[mt]);
            const f32x16 b = bias_frag(B3 + mt * 32 + 4 * h);
            f32x16 c[2] = {b, b};
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const bf16x8 f = W3f[(mt * 8 + k) * 64 + lane];
#pragma unroll
                for (int t = 0; t < 2; ++t)
                    c[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f, h2[t][k >> 1][k & 1], c[t], 0, 0, 0);
            }
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const uint32_t m = (t ? m1 : m0) >> (4 * h);  // register reg holds row base + 4h + (reg & 3) + 8 (reg >> 2)
                const float best0 = best[t];
                int bt = 0;
#pragma unroll
                for (int reg = 0; reg < 16; ++reg) {
                    if (!((rm >> reg) & 1u)) continue;
                    const int i = (reg & 3) + 8 * (reg >> 2);
                    const bool better = ((m >> i) & 1u) && c[t][reg] > best[t];  // ascending rows: first max
                    best[t] = better ? c[t][reg] : best[t];
                    bt = better ? i : bt;
                }
                bidx[t] = best[t] != best0 ? base + 4 * h + bt : bidx[t];
            }
        }
        // the next pair's env loads waited for before the stores (policy_kernel, SHIPENV_POLICY_NXT_WAIT)
        asm volatile("" ::"v"(nxt[0].fuel), "v"(nxt[0].x), "v"(nxt[0].y), "v"(nxt[0].o8), "v"(nxt[0].d8),
                     "v"(nxt[1].fuel), "v"(nxt[1].x), "v"(nxt[1].y), "v"(nxt[1].o8), "v"(nxt[1].d8));
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int64_t e = (2 * pair + t) * 32 + r;
            FINISH_ENV(v[t], e, e < A.n, h, best[t], bidx[t], cur[t].x, cur[t].y, cur[t].o8, cur[t].d8,
                       (float)cur[t].fuel);
        }
    }
}

// ------------------------------------------------------------------ the f32 policy step
// The fp32-faithful form of the same step (se_policy_f32): DQNNetwork evaluated in f32 as
// agents/dqn.py:198-200 runs it (fp32 weights, fp32 activations), on
// v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulation; gfx950 has no xf32). Its
// result D has the bf16 instruction's 32 x 32 layout (env on the lane, rows
// (reg & 3) + 8 (reg >> 2) + 4h in 16 registers), so a layer's accumulator register s is
// directly the next layer's B operand of k-step s, with the weights' columns permuted to
// match (fragment element (tile, kt, s, lane) = W[tile*32 + (lane & 31)][kt*32 + acc_row(s)]).
// One 32-env tile per wave: fc1 (6 live inputs, 3 k-steps of 2), fc2 (64 k-steps per row
// tile), fc3 over the compact rows, then the bf16 kernel's masked first maximum and
// epsilon-greedy (the helpers above). 512-thread workgroups (2 waves per SIMD: h1, h2 and
// an accumulator in f32 need ~160 registers), one per CU with the image in LDS; fc3's
// fragments are read from global memory (L2) when the layout does not fit beside it (the
// full layout of q_out).
struct QnetF32Dims {
    QnetDims q;  // fc3's row layout (full or compact)
    __host__ __device__ int w1() const { return 0; }                  // 4 x 3 x 64 f32 (3 KB)
    __host__ __device__ int w2() const { return 4096; }               // [mt][kt][s/4][lane][s%4]: 64 KB
    __host__ __device__ int b1() const { return w2() + 65536; }       // 128 f32, port block folded
    __host__ __device__ int b2() const { return b1() + 4 * kQHidden; }
    __host__ __device__ int b3() const { return b2() + 4 * kQHidden; }  // mt3 * 32 f32
    __host__ __device__ int same() const { return b3() + q.mt3 * 128; }
    __host__ __device__ int regm() const { return same() + 8 * q.P; }
    __host__ __device__ int w3() const { return (regm() + 4 * q.mt3 + 15) & ~15; }  // mt3 x 16 KB, last
    __host__ __device__ int bytes() const { return w3() + q.mt3 * 16384; }
};

struct PackF32Args {
    const float *w1, *b1, *w2, *b2, *w3, *b3;
    const uint32_t* world;
    WorldDims dims;
    QnetF32Dims d;
    uint8_t* img;
};

__global__ __launch_bounds__(256) void qnet_pack_f32_kernel(PackF32Args A) {
    const QnetF32Dims d = A.d;
    const QnetDims q = d.q;
    uint8_t* const img = A.img;
    const int in1 = q.in1();
    const int n_w1 = 4 * 3 * 64, n_w2 = 4 * 4 * 16 * 64, n_w3 = q.mt3 * 4 * 16 * 64;
    const int total = n_w1 + n_w2 + n_w3 + 2 * kQHidden + q.mt3 * 32 + q.P + q.mt3;
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        if (t < n_w1) {  // fc1: (mt, s, lane) = W1[mt*32 + r][2s + h] over the 6 dynamic columns
            const int lane = t & 63, st = t >> 6, s = st % 3, mt = st / 3;
            const int col = 2 * s + (lane >> 5);  // x, y, fuel, "cargo" = fuel (:206), origin, dest
            reinterpret_cast<float*>(img + d.w1())[t] = A.w1[(mt * 32 + (lane & 31)) * in1 + col];
            continue;
        }
        if (t < n_w1 + n_w2 + n_w3) {  // fc2 / fc3: float index ((mt*4 + kt)*4 + s4)*256 + lane*4 + i
            const bool second = t < n_w1 + n_w2;
            const int u = t - (second ? n_w1 : n_w1 + n_w2);
            const int i = u & 3, lane = (u >> 2) & 63, s4 = (u >> 8) & 3, kt = (u >> 10) & 3, mt = u >> 12;
            const int s = 4 * s4 + i, h = lane >> 5;
            const int col = kt * 32 + (s & 3) + 8 * (s >> 2) + 4 * h;  // the previous layer's acc row
            const int row = mt * 32 + (lane & 31);
            float v;
            if (second) {
                v = A.w2[row * kQHidden + col];
            } else {
                v = row < q.rows ? A.w3[q.action_of_row(row) * kQHidden + col] : 0.0f;
            }
            reinterpret_cast<float*>(img + (second ? d.w2() : d.w3()))[u] = v;
            continue;
        }
        int u = t - (n_w1 + n_w2 + n_w3);
        const LdsWorld wv = world_view(A.dims, A.world);  // the device image, read in place
        const int P = q.P;
        if (u < kQHidden) {  // b1 + fc1 over the constant port block, in f64 then f32 (as qnet_pack_kernel)
            double acc = (double)A.b1[u];
            for (int p = 0; p < P; ++p) {
                const float* w = A.w1 + u * in1 + 6 + 4 * p;
                acc += (double)w[0] * (double)wv.px(p) + (double)w[1] * (double)wv.py(p) +
                       (double)w[2] * (double)wv.pfuel(p) + (double)w[3] * (double)wv.pcargo(p);
            }
            reinterpret_cast<float*>(img + d.b1())[u] = (float)acc;
        } else if ((u -= kQHidden) < kQHidden) {
            reinterpret_cast<float*>(img + d.b2())[u] = A.b2[u];
        } else if ((u -= kQHidden) < q.mt3 * 32) {
            reinterpret_cast<float*>(img + d.b3())[u] = u < q.rows ? A.b3[q.action_of_row(u)] : 0.0f;
        } else if ((u -= q.mt3 * 32) < P) {  // bit p: port p stands on port u's cell (u included)
            uint64_t same = 0;
            for (int p = 0; p < P; ++p)
                if (wv.pos[p] == wv.pos[u]) same |= 1ull << p;
            reinterpret_cast<uint64_t*>(img + d.same())[u] = same;
        } else {  // fc3 tile mt's epilogue registers, as qnet_pack_kernel
            const int mt = u - P, base = mt * 32;
            int cmax = 0, fmax = 0;
            for (int p = 0; p < P; ++p) {
                cmax = max(cmax, min(wv.pcargo(p), 49));
                fmax = max(fmax, min(wv.pfuel(p), 199));
            }
            const int c_lo = 5 + P, c_hi = 4 + P + cmax, f_lo = 55 + P, f_hi = 54 + P + fmax;
            uint32_t rm = 0;
            for (int reg = 0; reg < 16; ++reg)
                for (int h = 0; h < 2; ++h) {
                    const int row = base + (reg & 3) + 8 * (reg >> 2) + 4 * h;
                    const int a = q.action_of_row(row);
                    const bool ok = row < q.rows && (a < 4 + P || (a >= c_lo && a <= c_hi) || (a >= f_lo && a <= f_hi));
                    rm |= (uint32_t)ok << reg;
                }
            reinterpret_cast<uint32_t*>(img + d.regm())[mt] = rm;
        }
    }
}

constexpr int kPolicyF32Block = 512;
constexpr int kPolicyF32Waves = kPolicyF32Block / 64;

struct PolicyF32Args {
    PolicyArgs p;  // qimg: the f32 image
    QnetF32Dims d;
};

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void relu16(f32x16& c) {
#pragma unroll
    for (int r = 0; r < 16; ++r) c[r] = fmaxf(c[r], 0.0f);
}

// acc + W x H for one 32-row tile over K = 128: W the tile's [kt][s4][lane] float4 fragments
__device__ __forceinline__ f32x16 gemm128(const float4* W, const f32x16 (&H)[4], f32x16 c, int lane) {
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            const float4 a = W[(kt * 4 + s4) * 64 + lane];
            c = mfma32(a.x, H[kt][4 * s4 + 0], c);
            c = mfma32(a.y, H[kt][4 * s4 + 1], c);
            c = mfma32(a.z, H[kt][4 * s4 + 2], c);
            c = mfma32(a.w, H[kt][4 * s4 + 3], c);
        }
    return c;
}

template <bool kW3Global>
__global__ __launch_bounds__(kPolicyF32Block) void policy_f32_kernel(PolicyF32Args F) {
    extern __shared__ uint4 smem[];
    const PolicyArgs& A = F.p;
    const QnetF32Dims D = F.d;
    const QnetDims q = D.q;
    const int staged = (kW3Global ? D.w3() : D.bytes()) / 16;
    for (int i = threadIdx.x; i < staged; i += kPolicyF32Block) smem[i] = A.qimg[i];
    const LdsWorld w = stage_world(A.world, A.dims, reinterpret_cast<uint32_t*>(smem + staged));
    const uint8_t* qb = reinterpret_cast<const uint8_t*>(smem);
    const float* W1 = reinterpret_cast<const float*>(qb + D.w1());
    const float4* W2 = reinterpret_cast<const float4*>(qb + D.w2());
    const float4* W3 = reinterpret_cast<const float4*>(
        (kW3Global ? reinterpret_cast<const uint8_t*>(A.qimg) : qb) + D.w3());
    const float* B1 = reinterpret_cast<const float*>(qb + D.b1());
    const float* B2 = reinterpret_cast<const float*>(qb + D.b2());
    const float* B3 = reinterpret_cast<const float*>(qb + D.b3());
    const uint64_t* SAME = reinterpret_cast<const uint64_t*>(qb + D.same());
    const uint32_t* REGM = reinterpret_cast<const uint32_t*>(qb + D.regm());

    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const int P = q.P;
    const int64_t tiles = (A.n + 31) >> 5;
    const int64_t stride = (int64_t)gridDim.x * kPolicyF32Waves;
    for (int64_t tile = (int64_t)blockIdx.x * kPolicyF32Waves + (threadIdx.x >> 6); tile < tiles; tile += stride) {
        const int64_t e = tile * 32 + r;
        const bool live = e < A.n;
        const int64_t ei = live ? e : A.n - 1;
        const double fuel = A.st.fuel[ei];
        const uint32_t x8 = A.st.x[ei], y8 = A.st.y[ei], o8 = A.st.origin[ei], d8 = A.st.dest[ei];
        const int origin = o8 == SE_NONE ? -1 : (int)o8, dest = d8 == SE_NONE ? -1 : (int)d8;
        // the preprocess_state row as torch's FloatTensor holds it: fuel rounded to f32
        const float ff = (float)fuel;
        const float in0 = h ? (float)y8 : (float)x8, in2 = h ? (float)dest : (float)origin;
        f32x16 h1[4], h2[4];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {  // fc1 over x, y | fuel, fuel | origin, dest, + relu
            f32x16 c = bias_frag(B1 + mt * 32 + 4 * h);
            c = mfma32(W1[(mt * 3 + 0) * 64 + lane], in0, c);
            c = mfma32(W1[(mt * 3 + 1) * 64 + lane], ff, c);
            c = mfma32(W1[(mt * 3 + 2) * 64 + lane], in2, c);
            relu16(c);
            h1[mt] = c;
        }
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {  // fc2 + relu
            h2[mt] = gemm128(W2 + mt * 16 * 64, h1, bias_frag(B2 + mt * 32 + 4 * h), lane);
            relu16(h2[mt]);
        }
        const EnvValid v = env_valid(w, q, SAME, (int)x8, (int)y8, origin);
        float best = -INFINITY;
        int bidx = 0x7fffffff;
#pragma nounroll
        for (int mt = 0; mt < q.mt3; ++mt) {  // fc3 + the masked first-maximum argmax
            const int base = mt * 32;
            if (!A.q_out && !__any(tile_maybe(v, mt, P))) continue;
            const uint32_t m = tile_mask(v, mt, P);
            const uint32_t rm = __builtin_amdgcn_readfirstlane(REGM[mt]);
            const f32x16 c = gemm128(W3 + mt * 16 * 64, h2, bias_frag(B3 + mt * 32 + 4 * h), lane);
            tile_argmax(c, m, rm, base, h, best, bidx);
            if (A.q_out && live) tile_q_out(A.q_out, A.ldq, q.rows, c, e, base, h);
        }
        FINISH_ENV(v, e, live, h, best, bidx, x8, y8, o8, d8, ff);
    }
}

// ------------------------------------------------------------------ the split-bf16 f32 step
// The fp32-faithful step on bf16 MFMA (round 5; se_policy_f32's default). fc2 and fc3 run
// on v_mfma_f32_32x32x16_bf16 with every f32 operand split into three bf16 parts,
// w = w0 + w1 + w2 and x = x0 + x1 + x2 (each part the round-to-nearest bf16 of what the
// parts before it leave; three 8-bit significands hold an f32's 24 bits), and the six
// products whose parts sum to at most 2, w0x2 + w1x1 + w2x0 + w0x1 + w1x0 + w0x0, smallest
// first, into one f32 accumulator. The dropped products (w1x2, w2x1, w2x2) are below
// 2^-23 of |w x|: a simulation of this datapath against float64 (MFMA = one f32 rounding
// per instruction) errs like the f32 MFMA path and torch's fp32 GEMM.
// Six bf16 MFMAs (32 cycles each) per 16-deep k-step where the f32 datapath runs eight
// v_mfma_f32_32x32x2_f32 (64 cycles each): 2.7x fewer MFMA cycles. fc1 (6 live inputs)
// stays on f32 MFMA. Relu'd activations are split once per layer (registers 8s..8s+7 of
// tile kt are k-step (kt, s)'s B operand, as in the bf16 kernel) and held as 24 bf16x8
// parts. Image: the f32 image's fc1 and biases, fc2 and fc3 as three bf16 fragments per
// (tile, kt, s): 96 KB + 24 KB per fc3 tile, so the world is read in place (L2), not
// staged, and fc3 comes from global memory when it does not fit (the full layout).
#ifndef SHIPENV_X3_FC1
#define SHIPENV_X3_FC1 1  // 1: fc1 as two split-bf16 MFMAs per row tile (x3_fc1_slot); 0: f32 MFMA
#endif
struct QnetX3Dims {
    QnetDims q;
    __host__ __device__ int w1() const { return 0; }  // fc1: bf16 fragments [mt][2 steps][lane] (8 KB), or f32 (3 KB)
    __host__ __device__ int w2() const { return 8192; }                 // [mt][kt][s][part] bf16 fragments: 96 KB
    __host__ __device__ int b1() const { return w2() + 96 * 1024; }
    __host__ __device__ int b2() const { return b1() + 4 * kQHidden; }
    __host__ __device__ int b3() const { return b2() + 4 * kQHidden; }  // mt3 * 32 f32
    __host__ __device__ int same() const { return b3() + q.mt3 * 128; }
    __host__ __device__ int regm() const { return same() + 8 * q.P; }
    __host__ __device__ int w3() const { return (regm() + 4 * q.mt3 + 15) & ~15; }  // mt3 x 24 KB, last
    __host__ __device__ int bytes() const { return w3() + q.mt3 * 24 * 1024; }
};


// fc1 on bf16 MFMA (SHIPENV_X3_FC1): the six dynamic columns' products as 24 of the 32 k
// slots of two v_mfma_f32_32x32x16_bf16 per row tile. Slot k (step k >> 4, lane half
// (k >> 3) & 1, element k & 7) holds weight part wp of column col times input part xp:
// x, y, origin, dest are exact in bf16 (|v| <= 255), so they take w0 x + w1 x + w2 x; the
// fuel column (2) and the "cargo" = fuel column (3, environment.py:206) take the six split
// products of w and the fuel f32. Columns: 0 x, 1 y, 2 fuel, 3 cargo, 4 origin, 5 dest.
struct Fc1Slot {
    int8_t col, wp, xp;  // xp: -1 = the exact input, else the fuel part
};
// SHIPENV_X3_BFOLD = 1: slots 24-26 hold the three bf16 parts of fc1's bias (b1 with the port
// block folded, the image's f32 b1) times an input of 1.0 (col -2), so the chains start at 0 and
// no bias is read from LDS (4 x 16-byte reads per row tile and env tile). Measured even or
// slower (0.2776 vs 0.2751 ms per call, medians of 4 alternating runs,
// profiles/r05/ab_policy_f32_bias_fold.jsonl): not kept.
#ifndef SHIPENV_X3_PACK_UNROLL
#define SHIPENV_X3_PACK_UNROLL 6  // fc2 / fc3 pack items whose loads go out together (6 items a thread at P = 5): 0.2646 -> 0.2613 ms per call against 2 (profiles/r05/ab_policy_f32_pack_unroll.jsonl)
#endif
#ifndef SHIPENV_X3_FOLD_UNROLL
#define SHIPENV_X3_FOLD_UNROLL 1  // 8: 0.2699 vs 0.2687 ms per call (profiles/r05/ab_policy_f32_fold_unroll.jsonl), not kept
#endif
// the bf16 kernel's 64-bit valid-row masks (SHIPENV_POLICY_VALID64) in this kernel: 0.2724 vs
// 0.2630 ms per call (profiles/r05/ab_policy_f32_valid64.jsonl; 256 VGPRs and more SGPR
// spills), not kept
#ifndef SHIPENV_X3_VALID64
#define SHIPENV_X3_VALID64 0
#endif
#ifndef SHIPENV_X3_PTAB
#define SHIPENV_X3_PTAB 1  // policy_x3_kernel stages the port table in LDS before its pack: 0.2652 -> 0.2629 ms per call (profiles/r05/ab_policy_f32_ptab.jsonl); 0: the pack reads L2
#endif
constexpr int kX3PtabBytes = SHIPENV_X3_PTAB ? 3 * 64 * 4 + 16 : 0;  // the staged port table, past the image
#ifndef SHIPENV_X3_PACK_VEC
#define SHIPENV_X3_PACK_VEC 1  // pack_x3_items: fc2 / fc3 items with float4 loads and paired splits (0: per element)
#endif
#ifndef SHIPENV_X3_BFOLD
#define SHIPENV_X3_BFOLD 0
#endif
__host__ __device__ constexpr Fc1Slot x3_fc1_slot(int k) {
    constexpr Fc1Slot t[24] = {{0, 0, -1}, {1, 0, -1}, {4, 0, -1}, {5, 0, -1}, {0, 1, -1}, {1, 1, -1}, {4, 1, -1}, {5, 1, -1},
                               {0, 2, -1}, {1, 2, -1}, {4, 2, -1}, {5, 2, -1}, {2, 0, 0},  {2, 0, 1},  {2, 1, 0},  {2, 0, 2},
                               {2, 1, 1},  {2, 2, 0},  {3, 0, 0},  {3, 0, 1},  {3, 1, 0},  {3, 0, 2},  {3, 1, 1},  {3, 2, 0}};
    return k < 24 ? t[k] : (SHIPENV_X3_BFOLD && k < 27 ? Fc1Slot{-2, (int8_t)(k - 24), -1} : Fc1Slot{-1, 0, 0});
}

struct PackX3Args {
    const float *w1, *b1, *w2, *b2, *w3, *b3;
    const uint32_t* world;
    WorldDims dims;
    QnetX3Dims d;
    uint8_t* img;
    // policy_x3_kernel's own pack (SHIPENV_X3_PTAB): the port table (P positions, then P
    // stock pairs) staged in LDS, so the b1 folds and the same-cell / register masks read it
    // there instead of looping over L2 loads; null: the world image in place
    const uint32_t* ptab = nullptr;
};

// the world view the pack reads the ports through
__device__ __forceinline__ LdsWorld pack_world(const PackX3Args& A) {
    LdsWorld wv = world_view(A.dims, A.world);
    if (A.ptab) {
        wv.pos = A.ptab;
        wv.stock = reinterpret_cast<const int2*>(A.ptab + 64);
    }
    return wv;
}

// One thread per (fragment, lane) of fc2 / fc3 (its 8 elements' three parts), per fc1 float,
// bias entry, same-cell mask and epilogue register mask (the latter as qnet_pack_f32_kernel).
// items [first, total) step `stride` of the split image into img (global memory for
// qnet_pack_x3_kernel, the workgroup's LDS for policy_x3_kernel's own prologue)
// b1[f] + W1[f, 6:] . the port block, in f64 then f32 (qnet_pack_kernel's fold)
__device__ __forceinline__ float x3_fold_b1(const PackX3Args& A, int f) {
    const LdsWorld wv = pack_world(A);
    const int in1 = A.d.q.in1();
    double acc = (double)A.b1[f];
    // unrolled so that several ports' weight loads go out before the adds wait on them (the
    // adds stay in port order)
#pragma unroll SHIPENV_X3_FOLD_UNROLL
    for (int p = 0; p < A.d.q.P; ++p) {
        const float* w = A.w1 + f * in1 + 6 + 4 * p;
        acc += (double)w[0] * (double)wv.px(p) + (double)w[1] * (double)wv.py(p) + (double)w[2] * (double)wv.pfuel(p) +
               (double)w[3] * (double)wv.pcargo(p);
    }
    return (float)acc;
}

__device__ __forceinline__ void pack_x3_items(const PackX3Args& A, uint8_t* img, int first, int stride) {
    const QnetX3Dims d = A.d;
    const QnetDims q = d.q;
    const int in1 = q.in1();
    const int n_w1 = SHIPENV_X3_FC1 ? 4 * 2 * 64 : 4 * 3 * 64, n_w2 = 32 * 64, n_w3 = q.mt3 * 8 * 64;
    const int total = n_w1 + n_w2 + n_w3 + 2 * kQHidden + q.mt3 * 32 + q.P + q.mt3;
    // (SHIPENV_X3_PACK_VEC) fc2 / fc3 fragments first, in a loop of their own: an item's 8
    // weights are two float4 loads (elements 0-3 and 4-7 are consecutive columns), split as
    // pairs, and SHIPENV_X3_PACK_UNROLL items' loads go out together. Same bits as the
    // per-element split3 below. Taken when both weight matrices are 16-byte aligned (torch's
    // allocations are); otherwise the element-wise loop below packs them.
    const bool vec = SHIPENV_X3_PACK_VEC &&
                     ((reinterpret_cast<uintptr_t>(A.w2) | reinterpret_cast<uintptr_t>(A.w3)) & 15) == 0;
#if SHIPENV_X3_PACK_VEC
#pragma unroll SHIPENV_X3_PACK_UNROLL
    for (int u0 = vec ? first : n_w2 + n_w3; u0 < n_w2 + n_w3; u0 += stride) {
        const bool second = u0 < n_w2;
        const int u = second ? u0 : u0 - n_w2;
        const int f = u >> 6, lane = u & 63, r = lane & 31, h = lane >> 5;
        const int s = f & 1, kt = (f >> 1) & 3, mt = f >> 3;
        const int row = mt * 32 + r;
        const bool in = second || row < q.rows;
        const float* W = second ? A.w2 : A.w3;
        const int wrow = second ? row : (in ? q.action_of_row(row) : 0);
        const float4* src = reinterpret_cast<const float4*>(W + wrow * kQHidden + kt * 32 + acc_row(s, 0, h));
        float4 a = src[0], b = src[2];  // columns acc_row(s, 0..3, h) and acc_row(s, 4..7, h) = +8
        if (!in) a = b = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        u32x4 w[3];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const f32x2 x{v[2 * k], v[2 * k + 1]};  // (the pack, not beside MFMAs: packed subtractions)
            const bf16x2 p0 = __builtin_convertvector(x, bf16x2);
            const f32x2 r1 = x - __builtin_convertvector(p0, f32x2);
            const bf16x2 p1 = __builtin_convertvector(r1, bf16x2);
            const bf16x2 p2 = __builtin_convertvector(r1 - __builtin_convertvector(p1, f32x2), bf16x2);
            w[0][k] = __builtin_bit_cast(uint32_t, p0);
            w[1][k] = __builtin_bit_cast(uint32_t, p1);
            w[2][k] = __builtin_bit_cast(uint32_t, p2);
        }
        uint8_t* dst = img + (second ? d.w2() : d.w3()) + f * 3 * 1024 + lane * 16;
#pragma unroll
        for (int k = 0; k < 3; ++k) *reinterpret_cast<u32x4*>(dst + k * 1024) = w[k];
    }
#endif
    for (int t = first; t < total; t += stride) {
        if (vec && t >= n_w1 && t < n_w1 + n_w2 + n_w3) continue;  // packed above
        if (t < n_w1) {
            const int lane = t & 63;
            if (SHIPENV_X3_FC1) {  // fc1 fragment (mt, step, lane): element j = slot 16 step + 8h + j
                const int st = (t >> 6) & 1, mt = t >> 7, row = mt * 32 + (lane & 31);
                bf16x8 v;
                float b1f = 0.0f;  // the row's fc1 bias (as the image's b1 below), for the folded slots
                if (SHIPENV_X3_BFOLD && st == 1 && (lane >> 5)) b1f = x3_fold_b1(A, row);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const Fc1Slot sl = x3_fc1_slot(16 * st + 8 * (lane >> 5) + j);
                    __bf16 p0 = (__bf16)0.0f, p1 = p0, p2 = p0;
                    if (sl.col >= 0) split3(A.w1[row * in1 + sl.col], p0, p1, p2);
                    else if (sl.col == -2) split3(b1f, p0, p1, p2);
                    v[j] = sl.wp == 0 ? p0 : (sl.wp == 1 ? p1 : p2);
                }
                reinterpret_cast<bf16x8*>(img + d.w1())[t] = v;
            } else {  // fc1 in f32: (mt, s, lane) = W1[mt*32 + r][2s + h] (qnet_pack_f32_kernel)
                const int st = t >> 6, s = st % 3, mt = st / 3;
                reinterpret_cast<float*>(img + d.w1())[t] = A.w1[(mt * 32 + (lane & 31)) * in1 + 2 * s + (lane >> 5)];
            }
            continue;
        }
        if (t < n_w1 + n_w2 + n_w3) {  // fragment f = (mt*4 + kt)*2 + s, lane: W[row][kt*32 + acc_row(s, j, h)]
            const bool second = t < n_w1 + n_w2;
            const int u = t - (second ? n_w1 : n_w1 + n_w2);
            const int f = u >> 6, lane = u & 63, r = lane & 31, h = lane >> 5;
            const int s = f & 1, kt = (f >> 1) & 3, mt = f >> 3;
            const int row = mt * 32 + r;
            const bool in = second || row < q.rows;
            const float* W = second ? A.w2 : A.w3;
            const int wrow = second ? row : q.action_of_row(row);
            bf16x8 p[3];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = in ? W[wrow * kQHidden + kt * 32 + acc_row(s, j, h)] : 0.0f;
                __bf16 a, b, c;
                split3(v, a, b, c);
                p[0][j] = a;
                p[1][j] = b;
                p[2][j] = c;
            }
            uint8_t* dst = img + (second ? d.w2() : d.w3()) + f * 3 * 1024 + lane * 16;
#pragma unroll
            for (int k = 0; k < 3; ++k) *reinterpret_cast<bf16x8*>(dst + k * 1024) = p[k];
            continue;
        }
        int u = t - (n_w1 + n_w2 + n_w3);
        const LdsWorld wv = pack_world(A);
        const int P = q.P;
        if (u < kQHidden) {  // b1 + fc1 over the constant port block, in f64 then f32
            reinterpret_cast<float*>(img + d.b1())[u] = x3_fold_b1(A, u);
        } else if ((u -= kQHidden) < kQHidden) {
            reinterpret_cast<float*>(img + d.b2())[u] = A.b2[u];
        } else if ((u -= kQHidden) < q.mt3 * 32) {
            reinterpret_cast<float*>(img + d.b3())[u] = u < q.rows ? A.b3[q.action_of_row(u)] : 0.0f;
        } else if ((u -= q.mt3 * 32) < P) {
            uint64_t same = 0;
            for (int p = 0; p < P; ++p)
                if (wv.pos[p] == wv.pos[u]) same |= 1ull << p;
            reinterpret_cast<uint64_t*>(img + d.same())[u] = same;
        } else {
            const int mt = u - P, base = mt * 32;
            int cmax = 0, fmax = 0;
            for (int p = 0; p < P; ++p) {
                cmax = max(cmax, min(wv.pcargo(p), 49));
                fmax = max(fmax, min(wv.pfuel(p), 199));
            }
            const int c_lo = 5 + P, c_hi = 4 + P + cmax, f_lo = 55 + P, f_hi = 54 + P + fmax;
            uint32_t rm = 0;
            for (int reg = 0; reg < 16; ++reg)
                for (int h = 0; h < 2; ++h) {
                    const int row = base + (reg & 3) + 8 * (reg >> 2) + 4 * h;
                    const int a = q.action_of_row(row);
                    const bool ok = row < q.rows && (a < 4 + P || (a >= c_lo && a <= c_hi) || (a >= f_lo && a <= f_hi));
                    rm |= (uint32_t)ok << reg;
                }
            reinterpret_cast<uint32_t*>(img + d.regm())[mt] = rm;
        }
    }
}

__global__ __launch_bounds__(256) void qnet_pack_x3_kernel(PackX3Args A) {
    pack_x3_items(A, A.img, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
}

// relu as a signed integer max with 0 on the f32 pattern (a non-negative float orders like
// its int pattern; a negative one, -0 included, becomes +0): one v_max_i32, where fmaxf
// also canonicalised its operand (two v_max_f32 per element)
__device__ __forceinline__ float relu_bits(float x) {
    return __builtin_bit_cast(float, max(__builtin_bit_cast(int, x), 0));
}

// relu of one 32-row f32 tile, split into the three bf16 B fragments of its two k-steps
__device__ __forceinline__ void relu_split3(const f32x16& c, bf16x8 (&out)[2][3]) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const f32x2 v{relu_bits(c[8 * s + 2 * p]), relu_bits(c[8 * s + 2 * p + 1])};
            const bf16x2 a = __builtin_convertvector(v, bf16x2);
            const f32x2 r1 = sub2(v, __builtin_convertvector(a, f32x2));
            const bf16x2 b = __builtin_convertvector(r1, bf16x2);
            const bf16x2 e = __builtin_convertvector(sub2(r1, __builtin_convertvector(b, f32x2)), bf16x2);
            out[s][0][2 * p] = a[0];
            out[s][0][2 * p + 1] = a[1];
            out[s][1][2 * p] = b[0];
            out[s][1][2 * p + 1] = b[1];
            out[s][2][2 * p] = e[0];
            out[s][2][2 * p + 1] = e[1];
        }
}

__device__ __forceinline__ f32x16 mfma_bf16(const bf16x8& a, const bf16x8& b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// c + W x over one k-step: the six part products, smallest first
__device__ __forceinline__ f32x16 kstep_x3(const bf16x8* Wf, int lane, const bf16x8 (&x)[3], f32x16 c) {
    const bf16x8 w0 = Wf[lane], w1 = Wf[64 + lane], w2 = Wf[128 + lane];
    c = mfma_bf16(w0, x[2], c);
    c = mfma_bf16(w1, x[1], c);
    c = mfma_bf16(w2, x[0], c);
    c = mfma_bf16(w0, x[1], c);
    c = mfma_bf16(w1, x[0], c);
    c = mfma_bf16(w0, x[0], c);
    return c;
}

#ifndef SHIPENV_X3_ABL
#define SHIPENV_X3_ABL 0  // timing-only ablations of policy_x3_kernel: 1 no epilogue, 2 fc3 tile 0 only,
                          // 4 no fragment re-reads, 8 no splits
#endif
#ifndef SHIPENV_X3_LOOKAHEAD
#define SHIPENV_X3_LOOKAHEAD 2  // k-steps ahead that fc2 / fc3's fragments are read; 1 / 3: 0.2582 / 0.2569 vs 0.2549 ms (profiles/r05/ab_policy_f32_la.jsonl)
#endif
#ifndef SHIPENV_X3_STAGGER
#define SHIPENV_X3_STAGGER 0  // experiment: waves 4-7 sleep this many x 6400 cycles first
#endif
#ifndef SHIPENV_X3_WORLD_PIN
#define SHIPENV_X3_WORLD_PIN 1  // the next tile's world reads waited for at their uses, not at their loads: 0.2573 (0) -> 0.2551 ms at k-step groups 8 / 24 (0.259 at 4 / 20, 0.2581 at 12 / 28; profiles/r05/ab_policy_f32_worldpin.jsonl, within the box's noise)
#endif
#ifndef SHIPENV_X3_CODE_AT
#define SHIPENV_X3_CODE_AT 8  // fc2 k-step group at which the next tile's cell code is read (SHIPENV_X3_WORLD_PIN)
#endif
#ifndef SHIPENV_X3_STOCK_AT
#define SHIPENV_X3_STOCK_AT 24  // ... and that port's stocks
#endif
#ifndef SHIPENV_X3_PRIO
#define SHIPENV_X3_PRIO 1  // waves 4-7 (each SIMD's second wave) at issue priority 1: 0.3-1.6 % faster in three alternating A/Bs (profiles/r05/ab_policy_f32_fused_fc1.jsonl, _bias_fold.jsonl, _pack_vec.jsonl); even in round 5's first (ab_policy_r05m.jsonl); 0: off
#endif
#ifndef SHIPENV_X3_SCHED
#define SHIPENV_X3_SCHED 1  // 0: the layers in plain order (the scheduler's own interleave)
#endif
#if !SHIPENV_X3_SCHED && SHIPENV_X3_FC1
#error "SHIPENV_X3_SCHED=0 is written for the f32 fc1 image: build it with SHIPENV_X3_FC1=0"
#endif
// chunk q (0..15) of the relu + 3-way split of tile c into out (relu_split3 in 16 pieces of
// about five VALU): pair q >> 1 (elements 2p, 2p + 1 of k-step s), stage q & 1 (the bf16
// rounding x0 and the remainder, then x1 and x2); r holds the remainders between stages
__device__ __forceinline__ void split_chunk(const f32x16& c, bf16x8 (&out)[2][3], f32x2 (&r)[8], int q) {
    const int pr = q >> 1, s = pr >> 2, p = pr & 3;
#if SHIPENV_X3_ABL & 8  // timing only: the splits dropped (stage 0 keeps x0 = bf16(c))
    if (q & 1) return;
    out[s][0][2 * p] = (__bf16)c[8 * s + 2 * p];
    out[s][0][2 * p + 1] = (__bf16)c[8 * s + 2 * p + 1];
    out[s][1] = out[s][2] = out[s][0];
    return;
#endif
    if ((q & 1) == 0) {
        const f32x2 v{relu_bits(c[8 * s + 2 * p]), relu_bits(c[8 * s + 2 * p + 1])};
        const bf16x2 a = __builtin_convertvector(v, bf16x2);
        out[s][0][2 * p] = a[0];
        out[s][0][2 * p + 1] = a[1];
        r[pr] = sub2(v, __builtin_convertvector(a, f32x2));
    } else {
        const bf16x2 b = __builtin_convertvector(r[pr], bf16x2);
        const bf16x2 e = __builtin_convertvector(sub2(r[pr], __builtin_convertvector(b, f32x2)), bf16x2);
        out[s][1][2 * p] = b[0];
        out[s][1][2 * p + 1] = b[1];
        out[s][2][2 * p] = e[0];
        out[s][2][2 * p + 1] = e[1];
    }
}

// pair q (0..7) of the relu + 3-way split of tile c into out: elements 2p, 2p + 1 of
// k-step s (q = 4s + p), both stages (relu_split3 in 8 pieces of about 11 VALU)
__device__ __forceinline__ void split_pair(const f32x16& c, bf16x8 (&out)[2][3], int q) {
    const int s = q >> 2, p = q & 3;
#if SHIPENV_X3_ABL & 8  // timing only: the splits dropped (x0 = bf16(c) for every part)
    out[s][0][2 * p] = (__bf16)c[8 * s + 2 * p];
    out[s][0][2 * p + 1] = (__bf16)c[8 * s + 2 * p + 1];
    if (p == 3) out[s][1] = out[s][2] = out[s][0];
    return;
#endif
    const f32x2 v{relu_bits(c[8 * s + 2 * p]), relu_bits(c[8 * s + 2 * p + 1])};
    const bf16x2 a = __builtin_convertvector(v, bf16x2);
    const f32x2 r1 = sub2(v, __builtin_convertvector(a, f32x2));
    const bf16x2 b = __builtin_convertvector(r1, bf16x2);
    const bf16x2 e = __builtin_convertvector(sub2(r1, __builtin_convertvector(b, f32x2)), bf16x2);
    out[s][0][2 * p] = a[0];
    out[s][0][2 * p + 1] = a[1];
    out[s][1][2 * p] = b[0];
    out[s][1][2 * p + 1] = b[1];
    out[s][2][2 * p] = e[0];
    out[s][2][2 * p + 1] = e[1];
}

// the three part fragments of fragment f (image order [f][part][lane])
__device__ __forceinline__ void x3_frags(const bf16x8* W, int f, int lane, bf16x8 (&wf)[3]) {
#if SHIPENV_X3_ABL & 4  // timing only: fragment reads after the first k-step dropped
    if (f != 0) return;
#endif
    wf[0] = W[f * 192 + lane];
    wf[1] = W[f * 192 + 64 + lane];
    wf[2] = W[f * 192 + 128 + lane];
}

// half of one k-step's six part products, in kstep_x3's order
__device__ __forceinline__ f32x16 khalf_x3(const bf16x8 (&w)[3], const bf16x8 (&x)[3], f32x16 c, int half) {
    if (half == 0) {
        c = mfma_bf16(w[0], x[2], c);
        c = mfma_bf16(w[1], x[1], c);
        c = mfma_bf16(w[2], x[0], c);
    } else {
        c = mfma_bf16(w[0], x[1], c);
        c = mfma_bf16(w[1], x[0], c);
        c = mfma_bf16(w[0], x[0], c);
    }
    return c;
}

// tile_argmax over registers 4j..4j+3 only (j = 0..3 in order is tile_argmax)
__device__ __forceinline__ void tile_argmax_part(const f32x16& c, uint32_t m, uint32_t rm, int base, int h,
                                                 float& best, int& bidx, int j) {
    m >>= 4 * h;
#pragma unroll
    for (int reg = 4 * j; reg < 4 * j + 4; ++reg) {
        if (!((rm >> reg) & 1u)) continue;
        const int i = (reg & 3) + 8 * (reg >> 2);
        const bool better = ((m >> i) & 1u) && c[reg] > best;
        best = better ? c[reg] : best;
        bidx = better ? base + 4 * h + i : bidx;
    }
}

constexpr int kPolicyX3Block = 512;
constexpr int kPolicyX3Waves = kPolicyX3Block / 64;

template <bool kW3Global, bool kQout = false>
__global__ __launch_bounds__(kPolicyX3Block) void policy_x3_kernel(PolicyF32Args F, QnetX3Dims D, PackX3Args PK) {
    extern __shared__ uint4 smem[];
    const PolicyArgs& A = F.p;
    const QnetDims q = D.q;
    // the first tile's env state (an HBM round trip) is requested before the image is built,
    // so the two overlap
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const int64_t tiles = (A.n + 31) >> 5;
    struct EnvIn {
        double fuel;
        uint32_t x8, y8, o8, d8;
    };
    auto load_env = [&](int64_t t) {
        const int64_t ei = min(t * 32 + (lane & 31), A.n - 1);
        return EnvIn{A.st.fuel[ei], A.st.x[ei], A.st.y[ei], A.st.origin[ei], A.st.dest[ei]};
    };
    int64_t tile = (int64_t)blockIdx.x * kPolicyX3Waves + (threadIdx.x >> 6);
    EnvIn nxt = load_env(tile < tiles ? tile : 0);
    if constexpr (kW3Global) {  // fc3 stays in the packed global image: copy the rest
        const int staged = D.w3() / 16;
        for (int i = threadIdx.x; i < staged; i += kPolicyX3Block) smem[i] = A.qimg[i];
    } else {
        // the whole image fits: each workgroup splits the f32 weights into its own LDS copy
        // (about 93 KB of f32 reads per workgroup at P = 5 where the packed image is 152 KB),
        // so no pack kernel runs before the policy and in-place weight updates are seen
#if SHIPENV_X3_PTAB
        uint32_t* ptab = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(smem) + ((D.bytes() + 15) & ~15));
        {
            const LdsWorld wg = world_view(A.dims, A.world);
            const int t = threadIdx.x, P0 = A.dims.P;
            if (t < P0) ptab[t] = wg.pos[t];
            else if (t >= 64 && t < 64 + 2 * P0) ptab[t] = reinterpret_cast<const uint32_t*>(wg.stock)[t - 64];
        }
        __syncthreads();
        PackX3Args pk = PK;
        pk.ptab = ptab;
        pack_x3_items(pk, reinterpret_cast<uint8_t*>(smem), threadIdx.x, kPolicyX3Block);
#else
        pack_x3_items(PK, reinterpret_cast<uint8_t*>(smem), threadIdx.x, kPolicyX3Block);
#endif
    }
    __syncthreads();
    const LdsWorld w = world_view(A.dims, A.world);  // port_at / stocks read in place (L2)
    const uint8_t* qb = reinterpret_cast<const uint8_t*>(smem);
    const float* W1 = reinterpret_cast<const float*>(qb + D.w1());
    const bf16x8* W2 = reinterpret_cast<const bf16x8*>(qb + D.w2());
    const bf16x8* W3 = reinterpret_cast<const bf16x8*>((kW3Global ? reinterpret_cast<const uint8_t*>(A.qimg) : qb) + D.w3());
    [[maybe_unused]] const float* B1 = reinterpret_cast<const float*>(qb + D.b1());
    const float* B2 = reinterpret_cast<const float*>(qb + D.b2());
    const float* B3 = reinterpret_cast<const float*>(qb + D.b3());
    const uint64_t* SAME = reinterpret_cast<const uint64_t*>(qb + D.same());
    const uint32_t* REGM = reinterpret_cast<const uint32_t*>(qb + D.regm());

    const int P = q.P;
    const int64_t stride = (int64_t)gridDim.x * kPolicyX3Waves;
    // the env state of the wave's next tile is loaded while this one computes (no HBM round
    // trip at the top of a tile), and its validity (the port on the ship's cell and that
    // port's stocks, two dependent L2 reads of the world image) resolved during fc3
#if SHIPENV_X3_PRIO
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= 4) __builtin_amdgcn_s_setprio(1);
#endif
#if SHIPENV_X3_STAGGER
    // waves 4-7 (each SIMD's second wave) start later, so the two waves' VALU-only
    // stretches (the per-tile epilogue) fall beside the partner's MFMA phases
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= 4) {
#pragma unroll
        for (int i = 0; i < SHIPENV_X3_STAGGER; ++i) __builtin_amdgcn_s_sleep(100);
    }
#endif
    EnvValid vnxt = env_valid(w, q, SAME, (int)nxt.x8, (int)nxt.y8, nxt.o8 == SE_NONE ? -1 : (int)nxt.o8);
#if SHIPENV_POLICY_DRAW_PAIR
    // past the image (kW3Global: past the staged part) and the port table
    PairedDraws pd{reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(smem) +
                                            (kW3Global ? D.w3() : ((D.bytes() + 15) & ~15) + kX3PtabBytes) +
                                            __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * kPairedDrawBytes)};
#endif
    for (; tile < tiles; tile += stride) {
        const EnvIn in = nxt;
        const EnvValid v = vnxt;
        const bool more = tile + stride < tiles;
        if (more) nxt = load_env(tile + stride);
        const int64_t e = tile * 32 + (lane & 31);
        const bool live = e < A.n;
        const double fuel = in.fuel;
        const uint32_t x8 = in.x8, y8 = in.y8, o8 = in.o8, d8 = in.d8;
        const int origin = o8 == SE_NONE ? -1 : (int)o8, dest = d8 == SE_NONE ? -1 : (int)d8;
        const float ff = (float)fuel;  // the preprocess_state row as torch's FloatTensor holds it
#if !SHIPENV_X3_FC1
        const float in0 = h ? (float)y8 : (float)x8, in2 = h ? (float)dest : (float)origin;
#endif
        bf16x8 X1[4][2][3], X2[4][2][3];
        float best = -INFINITY;
        int bidx = 0x7fffffff;
#if SHIPENV_X3_SCHED
        // The same arithmetic, hand-interleaved: the MFMAs go in groups of three (half a
        // k-step), and beside each group, fenced by sched_barrier so the compiler cannot
        // cluster them again, about five VALU of work that does not feed those MFMAs (a
        // chunk of a split of the layer's other tiles, or of the previous fc3 tile's
        // argmax). A wave's VALU then issues while its own MFMAs occupy the matrix pipe
        // (32 cycles each) instead of between MFMA phases. fc2 runs k-tile by k-tile over
        // its four row tiles (four accumulators), so k-tile kt + 1 is split during k-tile kt;
        // its last k-tile runs row tile by row tile, so the finished row tiles split beside
        // the rest; fc3's first tile splits fc2's last one. Fragments are read one k-step
        // ahead. Bit-identical to the plain order (the same operations on the same values).
        f32x16 c1[4], acc[4];
#if SHIPENV_X3_FC1
        bf16x8 xin[2];  // fc1's B operands: slot 16 step + 8h + j of x3_fc1_slot
        {
            __bf16 f0, f1, f2;
            split3(ff, f0, f1, f2);
            const __bf16 fp[3] = {f0, f1, f2};
            const __bf16 ex[6] = {(__bf16)(float)x8, (__bf16)(float)y8, f0, f0, (__bf16)(float)origin,
                                  (__bf16)(float)dest};  // exact inputs by column (2, 3 unused)
#pragma unroll
            for (int st = 0; st < 2; ++st)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const Fc1Slot a = x3_fc1_slot(16 * st + j), b = x3_fc1_slot(16 * st + 8 + j);
                    const __bf16 va = a.col == -2 ? (__bf16)1.0f : a.col < 0 ? (__bf16)0.0f : (a.xp < 0 ? ex[a.col] : fp[a.xp]);
                    const __bf16 vb = b.col == -2 ? (__bf16)1.0f : b.col < 0 ? (__bf16)0.0f : (b.xp < 0 ? ex[b.col] : fp[b.xp]);
                    xin[st][j] = h ? vb : va;
                }
        }
        const bf16x8* W1b = reinterpret_cast<const bf16x8*>(W1);
#endif
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {  // fc1 (x, y | fuel, fuel | origin, dest)
#if SHIPENV_X3_FC1 && SHIPENV_X3_BFOLD
            c1[mt] = f32x16{};  // the bias is in the fragments (slots 24-26)
#else
            c1[mt] = bias_frag(B1 + mt * 32 + 4 * h);
#endif
#if SHIPENV_X3_FC1
            c1[mt] = mfma_bf16(W1b[(mt * 2 + 0) * 64 + lane], xin[0], c1[mt]);
            c1[mt] = mfma_bf16(W1b[(mt * 2 + 1) * 64 + lane], xin[1], c1[mt]);
#else
            c1[mt] = mfma32(W1[(mt * 3 + 0) * 64 + lane], in0, c1[mt]);
            c1[mt] = mfma32(W1[(mt * 3 + 1) * 64 + lane], ff, c1[mt]);
            c1[mt] = mfma32(W1[(mt * 3 + 2) * 64 + lane], in2, c1[mt]);
#endif
            if (mt == 0) {
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[i] = bias_frag(B2 + i * 32 + 4 * h);
            } else {  // X1[0]'s 8 pairs beside fc1's other row tiles: 3, 3, 2
#pragma unroll
                for (int j = 0; j < 3; ++j)
                    if ((mt - 1) * 3 + j < 8) split_pair(c1[0], X1[0], (mt - 1) * 3 + j);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // fragments read kLa k-steps ahead over the flat k-step sequence: fc2's 32 (k-tile
        // kt, row tile mt, step s2), then fc3 tile 0's 8
        constexpr int kLa = SHIPENV_X3_LOOKAHEAD;
        bf16x8 wf[kLa + 1][3];
        auto frag_of = [&](int j, bf16x8 (&dst)[3]) {
            if (j < 32) x3_frags(W2, (((j >> 1) & 3) * 4 + (j >> 3)) * 2 + (j & 1), lane, dst);
            else x3_frags(W3, j - 32, lane, dst);
        };
#pragma unroll
        for (int j = 0; j < kLa; ++j) frag_of(j, wf[j]);
        // the next tile's two dependent world reads (its cell code, then that port's stocks)
        // go out during fc2, so their round trips overlap the MFMAs
        int ncode = 0;
        int2 nstock = make_int2(0, 0);
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            const int kt = i >> 3, mt = (i >> 1) & 3, s2 = i & 1;
            if (i == SHIPENV_X3_CODE_AT && (more || SHIPENV_X3_WORLD_PIN)) ncode = w.code((int)nxt.x8, (int)nxt.y8);
#if SHIPENV_X3_WORLD_PIN
            // unconditional (past the last tile nxt is tile 0's state, a valid address) and
            // opaque until their uses: under `if (more)` the compiler merged the arithmetic on
            // each into its load's block and waited out the round trip right there
            if (i == SHIPENV_X3_STOCK_AT) {
                asm volatile("" : "+v"(ncode));
                nstock = w.stock[max(w.port_of_code(ncode), 0)];
            }
#else
            if (i == 20 && more) nstock = w.stock[max(w.port_of_code(ncode), 0)];
#endif
            frag_of(i + kLa, wf[(i + kLa) % (kLa + 1)]);
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                acc[mt] = khalf_x3(wf[i % (kLa + 1)], X1[kt][s2], acc[mt], half);
                const int g = 2 * (i & 7) + half;  // group within the k-tile, 0..15
                if (kt < 3) {
                    if (half == 0) split_pair(c1[kt + 1], X1[kt + 1], g >> 1);  // 8 pairs over 16 groups
                } else if (mt > 0) {  // the previous row tile's 8 pairs over this row tile's 4 groups
                    split_pair(acc[mt - 1], X2[mt - 1], 2 * (g - 4 * mt));
                    split_pair(acc[mt - 1], X2[mt - 1], 2 * (g - 4 * mt) + 1);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // fc3 tile 0 (the moves: every env can choose from it), fc2's last row tile split
        // beside its first 8 groups (done before k-step 6 reads it). Without q_out, a row
        // no action of this env can take starts at -inf (masked_bias), so the argmax needs
        // no validity test and never picks it.
        // (SHIPENV_POLICY_VALID64, compact layouts of at most 64 rows) the fc3 tiles' masks as
        // shifts of one 64-bit word of the env's valid rows
        const bool use64 = SHIPENV_X3_VALID64 && !kQout && q.mt3 <= 2;  // uniform
        const uint64_t v64 = use64 ? valid_rows64(v) : 0ull;
        auto mask_of = [&](int mt) { return use64 ? (uint32_t)(v64 >> ((32 * mt) & 63)) : tile_mask(v, mt, P); };
        f32x16 c = kQout ? bias_frag(B3 + 4 * h) : masked_bias(B3 + 4 * h, mask_of(0) >> (4 * h));
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (32 + k + kLa < 40) frag_of(32 + k + kLa, wf[(32 + k + kLa) % (kLa + 1)]);
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                c = khalf_x3(wf[(32 + k) % (kLa + 1)], X2[k >> 1][k & 1], c, half);
                const int g = 2 * k + half;
                if (g < 8) split_pair(acc[3], X2[3], g);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // the next tile's validity from the world reads issued during fc2 (ncode, nstock)
#if SHIPENV_X3_WORLD_PIN
        // waited for here on every path: a wait only inside env_valid_from's port branch left
        // the load outstanding into the next tile, whose first write of its registers then
        // waited out the new env loads as well
        asm volatile("" ::"v"(nstock.x), "v"(nstock.y));
        vnxt = env_valid_from(w, q, SAME, ncode, nstock, nxt.o8 == SE_NONE ? -1 : (int)nxt.o8);
#else
        if (more) vnxt = env_valid_from(w, q, SAME, ncode, nstock, nxt.o8 == SE_NONE ? -1 : (int)nxt.o8);
#endif
        // fc3 tiles 1..: the previous tile's argmax beside each chain, 4 registers a group
        int pbase = 0;
        [[maybe_unused]] float best0 = best;
        [[maybe_unused]] int bt = 0;
        uint32_t pm = kQout ? tile_mask(v, 0, P) : 0u, prm = __builtin_amdgcn_readfirstlane(REGM[0]);
        if (kQout && live) tile_q_out(A.q_out, A.ldq, q.rows, c, e, 0, h);
#pragma nounroll
        for (int mt = 1; mt < ((SHIPENV_X3_ABL & 2) ? 1 : q.mt3); ++mt) {  // (ABL & 2: timing only, fc3 tile 0 alone)
            const int base = mt * 32;
            const uint32_t m3 = kQout ? 0u : mask_of(mt);
            if (!kQout && !__any(use64 ? m3 != 0u : tile_maybe(v, mt, P))) continue;
            const bf16x8* W3t = W3 + mt * 8 * 192;
            f32x16 c3 = kQout ? bias_frag(B3 + mt * 32 + 4 * h) : masked_bias(B3 + mt * 32 + 4 * h, m3 >> (4 * h));
#pragma unroll
            for (int j = 0; j < kLa; ++j) x3_frags(W3t, j, lane, wf[j]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (k + kLa < 8) x3_frags(W3t, k + kLa, lane, wf[(k + kLa) % (kLa + 1)]);
#pragma unroll
                for (int half = 0; half < 2; ++half) {
                    c3 = khalf_x3(wf[k % (kLa + 1)], X2[k >> 1][k & 1], c3, half);
                    const int g = 2 * k + half;
                    if (g < 4) {
                        if (kQout) {
                            tile_argmax_part(c, pm, prm, pbase, h, best, bidx, g);
                        } else {
#if SHIPENV_POLICY_LOCAL_IDX
                            if (g == 0) best0 = best;
                            argmax_local_part(c, best, bt, g);
                            if (g == 3) bidx = best != best0 ? pbase + bt : bidx;
#else
                            argmax_masked_part(c, pbase, best, bidx, g);
#endif
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            c = c3;
            pbase = base;
            if (kQout) pm = tile_mask(v, mt, P);
            prm = __builtin_amdgcn_readfirstlane(REGM[mt]);
            if (kQout && live) tile_q_out(A.q_out, A.ldq, q.rows, c, e, base, h);
        }
        if (kQout) {
            tile_argmax(c, pm, prm, pbase, h, best, bidx);
        } else {
#if SHIPENV_POLICY_LOCAL_IDX
            best0 = best;
#pragma unroll
            for (int g = 0; g < 4; ++g) argmax_local_part(c, best, bt, g);
            bidx = best != best0 ? pbase + bt : bidx;
#else
#pragma unroll
            for (int g = 0; g < 4; ++g) argmax_masked_part(c, pbase, best, bidx, g);
#endif
            bidx += bidx == 0x7fffffff ? 0 : 4 * h;  // the lane half's rows (argmax_masked_part omits 4h)
        }
#else
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {  // fc1 on f32 MFMA (x, y | fuel, fuel | origin, dest), relu, split
            f32x16 c = bias_frag(B1 + mt * 32 + 4 * h);
            c = mfma32(W1[(mt * 3 + 0) * 64 + lane], in0, c);
            c = mfma32(W1[(mt * 3 + 1) * 64 + lane], ff, c);
            c = mfma32(W1[(mt * 3 + 2) * 64 + lane], in2, c);
            relu_split3(c, X1[mt]);
        }
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {  // fc2 row tile mt = fc3's k-tile mt
            f32x16 c = bias_frag(B2 + mt * 32 + 4 * h);
#pragma unroll
            for (int k = 0; k < 8; ++k) c = kstep_x3(W2 + ((mt * 4 + (k >> 1)) * 2 + (k & 1)) * 192, lane, X1[k >> 1][k & 1], c);
            relu_split3(c, X2[mt]);
        }
        if (more) vnxt = env_valid(w, q, SAME, (int)nxt.x8, (int)nxt.y8, nxt.o8 == SE_NONE ? -1 : (int)nxt.o8);
#pragma nounroll
        for (int mt = 0; mt < q.mt3; ++mt) {  // fc3 + the masked first-maximum argmax
            const int base = mt * 32;
            if (!A.q_out && !__any(tile_maybe(v, mt, P))) continue;
            const uint32_t m = tile_mask(v, mt, P);
            const uint32_t rm = __builtin_amdgcn_readfirstlane(REGM[mt]);
            f32x16 c = bias_frag(B3 + mt * 32 + 4 * h);
#pragma unroll
            for (int k = 0; k < 8; ++k) c = kstep_x3(W3 + ((mt * 4 + (k >> 1)) * 2 + (k & 1)) * 192, lane, X2[k >> 1][k & 1], c);
            tile_argmax(c, m, rm, base, h, best, bidx);
            if (A.q_out && live) tile_q_out(A.q_out, A.ldq, q.rows, c, e, base, h);
        }
#endif
#if SHIPENV_X3_ABL & 1  // timing only: no epilogue (the chosen row stored as the action)
        if (h == 0 && live) A.actions[e] = bidx;
#elif SHIPENV_POLICY_DRAW_PAIR
        const U4 dw = pd.next(A.eps > 0.0, e, stride, h, lane & 31, A.seed, A.env_base, A.t);
        FINISH_ENV_D(v, e, live, h, best, bidx, x8, y8, o8, d8, ff, dw);
#else
        FINISH_ENV(v, e, live, h, best, bidx, x8, y8, o8, d8, ff);
#endif
    }
}

}  // namespace

struct se_qnet {
    se_env* env = nullptr;  // must outlive the qnet (destroy the qnet first)
    int device = 0;
    QnetDims q{}, qc{};  // the full layout (q_out) and the compact one, whose image follows
    const float* w[6] = {};  // the device weights of the last se_qnet_set_weights (se_qnet_repack)
    size_t c_off = 0;    // byte offset of the compact image
    uint8_t* d_img = nullptr;
    int img_bytes = 0;
    uint64_t world_version = 0;
    bool packed = false;
    uint8_t* d_img32 = nullptr;  // se_policy_f32's image, repacked from w[] at every call
    int img32_bytes = 0;
    bool f32_mfma = false;  // SHIPENV_POLICY_F32=mfma at se_qnet_create: the f32-MFMA datapath
                            // (policy_f32_kernel) instead of the split-bf16 one (policy_x3_kernel)
};

extern "C" {

int se_qnet_create(se_qnet** out, se_env* env) {
    if (!out) return fail(SE_EINVAL, "null out");
    *out = nullptr;
    int rc = check_ready(env);
    if (rc) return rc;
    se_qnet* qn = new se_qnet;
    qn->env = env;
    qn->device = env->device;
    const char* mode = getenv("SHIPENV_POLICY_F32");
    qn->f32_mfma = mode && std::string(mode) == "mfma";
    *out = qn;
    return SE_OK;
}

int se_qnet_set_weights(se_qnet* qn, const float* w1, const float* b1, const float* w2, const float* b2,
                        const float* w3, const float* b3, void* stream) {
    if (!qn) return fail(SE_EINVAL, "null qnet");
    if (!w1 || !b1 || !w2 || !b2 || !w3 || !b3) return fail(SE_EINVAL, "null weight pointer");
    se_env* env = qn->env;
    if (env->dims.P < 1) return fail(SE_EINVAL, "the policy needs at least one port");
    DeviceGuard g(env->device);
    const QnetDims q = qnet_dims(env->dims.P);
    const QnetDims qc = qnet_dims(env->dims.P, true, env->cmax, env->fmax);
    const size_t c_off = ((size_t)q.bytes() + 255) & ~(size_t)255;
    const int total = (int)(c_off + (size_t)qc.bytes());
    if (total > qn->img_bytes) {
        if (qn->d_img) HIP_TRY(hipFree(qn->d_img));
        qn->d_img = nullptr;
        HIP_TRY(hipMalloc(&qn->d_img, (size_t)total));
        qn->img_bytes = total;
    }
    qn->q = q;
    qn->qc = qc;
    qn->c_off = c_off;
    PackArgs A{w1, b1, w2, b2, w3, b3, env->d_world, env->dims, {q, qc}, {qn->d_img, qn->d_img + c_off},
               nullptr};
    qnet_pack_kernel<<<dim3(64, 2), 256, 0, (hipStream_t)stream>>>(A);  // both layouts, one launch
    HIP_TRY(hipGetLastError());
    const float* wp[6] = {w1, b1, w2, b2, w3, b3};
    for (int i = 0; i < 6; ++i) qn->w[i] = wp[i];
    qn->world_version = env->world_version;
    qn->packed = true;
    return SE_OK;
}

}  // extern "C"

namespace {
struct PolicyRecord {
    uint32_t* pos;
    float* fuel;
    int32_t* act;
    int64_t head, cap;
};

int launch_policy(se_qnet* qn, int32_t* actions, double epsilon, uint32_t t, float* q_out, int64_t ldq,
                  const PolicyRecord* rec, void* stream) {
    if (!qn) return fail(SE_EINVAL, "null qnet");
    se_env* env = qn->env;
    int rc = check_ready(env);
    if (rc) return rc;
    if (!qn->packed) return fail(SE_ESTATE, "se_qnet_set_weights has not been called");
    if (qn->world_version != env->world_version)
        return fail(SE_ESTATE, "ports changed since se_qnet_set_weights (the port block is folded into fc1)");
    if (!actions && env->n > 0) return fail(SE_EINVAL, "null actions");
    if (q_out && ldq < qn->q.A) return fail(SE_EINVAL, "ldq < number of actions");
    if (!(epsilon >= 0.0)) return fail(SE_EINVAL, "epsilon must be >= 0");
    if (env->n == 0) return SE_OK;
    DeviceGuard g(env->device);
    // the compact layout unless every row's Q is wanted
    const QnetDims& q = q_out ? qn->q : qn->qc;
    const size_t lds = (size_t)q.bytes() + lds_bytes(env) + (SHIPENV_POLICY_BFOLD23 ? (size_t)(4 + q.mt3) * 1024 : 0) +
                       (SHIPENV_POLICY_DRAW_PAIR ? (size_t)kPolicyWaves * kPairedDrawBytes : 0);
    static std::atomic<uint64_t> lds_set{0};
    static std::atomic<uint64_t> lds_set_q{0};
    rc = allow_dynamic_lds(lds_set, reinterpret_cast<const void*>(policy_kernel<false>), 160 * 1024, env->device);
    if (!rc) rc = allow_dynamic_lds(lds_set_q, reinterpret_cast<const void*>(policy_kernel<true>), 160 * 1024, env->device);
    if (rc) return rc;
    if (lds > 160 * 1024) return fail(SE_EINVAL, "network + world image exceed the 160 KB LDS");
    int dev_cus = 256;
    if (hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, env->device) != hipSuccess)
        dev_cus = 256;
    const int64_t tiles = (env->n + 31) / 32;
    const int64_t want = (tiles + kPolicyWaves - 1) / kPolicyWaves;
    const int64_t resident = (int64_t)dev_cus * kPolicyWgPerCu;  // workgroups resident at once
    const int grid = (int)(want < resident ? want : resident);
    PolicyArgs A{};
    A.world = env->d_world;
    A.dims = env->dims;
    A.qimg = reinterpret_cast<const uint4*>(qn->d_img + (q_out ? 0 : qn->c_off));
    A.q = q;
    A.n = env->n;
    A.env_base = env->env_base;
    A.seed = env->seed;
    A.t = t;
    A.eps = epsilon;
    A.st = env->st;
    A.actions = actions;
    A.q_out = q_out;
    A.ldq = ldq;
    if (rec) {
        A.rec_pos = rec->pos;
        A.rec_fuel = rec->fuel;
        A.rec_act = rec->act;
        A.rec_head = rec->head;
        A.rec_cap = rec->cap;
    }
    if (SHIPENV_POLICY_PAIR && !q_out && q.mt3 <= 2) {
        static std::atomic<uint64_t> lds_set_p{0};
        rc = allow_dynamic_lds(lds_set_p, reinterpret_cast<const void*>(policy_pair_kernel), 160 * 1024, env->device);
        if (rc) return rc;
        const int64_t pairs = (tiles + 1) / 2, wantp = (pairs + kPairWaves - 1) / kPairWaves;
        const int gridp = (int)(wantp < dev_cus ? wantp : dev_cus);
        policy_pair_kernel<<<gridp, kPairBlock, q.bytes() + lds_bytes(env), (hipStream_t)stream>>>(A);
    } else if (q_out) {
        policy_kernel<true><<<grid, kPolicyBlock, lds, (hipStream_t)stream>>>(A);
    } else {
        policy_kernel<false><<<grid, kPolicyBlock, lds, (hipStream_t)stream>>>(A);
    }
    HIP_TRY(hipGetLastError());
    return SE_OK;
}
// the split-bf16 datapath (policy_x3_kernel); the caller checked the arguments
int launch_policy_x3(se_qnet* qn, int32_t* actions, double epsilon, uint32_t t, float* q_out, int64_t ldq,
                     const PolicyRecord* rec, void* stream) {
    se_env* env = qn->env;
    QnetX3Dims d;
    d.q = q_out ? qn->q : qn->qc;  // the compact rows unless every row's Q is wanted
    if (d.bytes() > qn->img32_bytes) {
        if (qn->d_img32) HIP_TRY(hipFree(qn->d_img32));
        qn->d_img32 = nullptr;
        HIP_TRY(hipMalloc(&qn->d_img32, (size_t)d.bytes()));
        qn->img32_bytes = d.bytes();
    }
    const hipStream_t s = (hipStream_t)stream;
    // the image from the current weights (in place updates by an optimizer or T2 included)
    PackX3Args pk{qn->w[0], qn->w[1], qn->w[2], qn->w[3], qn->w[4], qn->w[5], env->d_world, env->dims, d,
                  qn->d_img32};
    constexpr int kPtabBytes = kX3PtabBytes + (SHIPENV_POLICY_DRAW_PAIR ? kPolicyX3Waves * kPairedDrawBytes : 0);
    const bool w3_global = d.bytes() + kPtabBytes > 160 * 1024;
    if (w3_global) {  // fc3's fragments are read from a packed global image
        qnet_pack_x3_kernel<<<128, 256, 0, s>>>(pk);
        HIP_TRY(hipGetLastError());
    }
    const size_t lds = (size_t)(w3_global ? d.w3() + (SHIPENV_POLICY_DRAW_PAIR ? kPolicyX3Waves * kPairedDrawBytes : 0)
                                          : ((d.bytes() + 15) & ~15) + kPtabBytes);
    if (lds > 160 * 1024) return fail(SE_EINVAL, "split-bf16 network exceeds the 160 KB LDS");
    static std::atomic<uint64_t> lds_set0{0}, lds_set1{0};
    static std::atomic<uint64_t> lds_set2{0};
    int rc = allow_dynamic_lds(lds_set0, reinterpret_cast<const void*>(policy_x3_kernel<false>), 160 * 1024, env->device);
    if (!rc) rc = allow_dynamic_lds(lds_set1, reinterpret_cast<const void*>(policy_x3_kernel<true>), 160 * 1024, env->device);
    if (!rc) rc = allow_dynamic_lds(lds_set2, reinterpret_cast<const void*>(policy_x3_kernel<true, true>), 160 * 1024, env->device);
    if (rc) return rc;
    int dev_cus = 256;
    if (hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, env->device) != hipSuccess)
        dev_cus = 256;
    const int64_t tiles = (env->n + 31) / 32;
    const int64_t want = (tiles + kPolicyX3Waves - 1) / kPolicyX3Waves;
    const int grid = (int)(want < dev_cus ? want : dev_cus);
    PolicyF32Args F{};
    PolicyArgs& A = F.p;
    A.world = env->d_world;
    A.dims = env->dims;
    A.qimg = reinterpret_cast<const uint4*>(qn->d_img32);
    A.q = d.q;
    A.n = env->n;
    A.env_base = env->env_base;
    A.seed = env->seed;
    A.t = t;
    A.eps = epsilon;
    A.st = env->st;
    A.actions = actions;
    A.q_out = q_out;
    A.ldq = ldq;
    if (rec) {
        A.rec_pos = rec->pos;
        A.rec_fuel = rec->fuel;
        A.rec_act = rec->act;
        A.rec_head = rec->head;
        A.rec_cap = rec->cap;
    }
    if (q_out) {  // the full layout (fc3 from global memory): unmasked Q rows for q_out
        if (!w3_global) return fail(SE_EINVAL, "q_out: the full fc3 layout is expected in global memory");
        policy_x3_kernel<true, true><<<grid, kPolicyX3Block, lds, s>>>(F, d, pk);
    } else if (w3_global) {
        policy_x3_kernel<true><<<grid, kPolicyX3Block, lds, s>>>(F, d, pk);
    } else {
        policy_x3_kernel<false><<<grid, kPolicyX3Block, lds, s>>>(F, d, pk);
    }
    HIP_TRY(hipGetLastError());
    return SE_OK;
}

int launch_policy_f32(se_qnet* qn, int32_t* actions, double epsilon, uint32_t t, float* q_out, int64_t ldq,
                      const PolicyRecord* rec, void* stream) {
    if (!qn) return fail(SE_EINVAL, "null qnet");
    se_env* env = qn->env;
    int rc = check_ready(env);
    if (rc) return rc;
    if (!qn->packed) return fail(SE_ESTATE, "se_qnet_set_weights has not been called");
    if (qn->world_version != env->world_version)
        return fail(SE_ESTATE, "ports changed since se_qnet_set_weights (the port block is folded into fc1)");
    if (!actions && env->n > 0) return fail(SE_EINVAL, "null actions");
    if (q_out && ldq < qn->q.A) return fail(SE_EINVAL, "ldq < number of actions");
    if (!(epsilon >= 0.0)) return fail(SE_EINVAL, "epsilon must be >= 0");
    if (env->n == 0) return SE_OK;
    DeviceGuard g(env->device);
    if (!qn->f32_mfma) return launch_policy_x3(qn, actions, epsilon, t, q_out, ldq, rec, stream);
    QnetF32Dims d;
    d.q = q_out ? qn->q : qn->qc;  // the compact rows unless every row's Q is wanted
    if (d.bytes() > qn->img32_bytes) {
        if (qn->d_img32) HIP_TRY(hipFree(qn->d_img32));
        qn->d_img32 = nullptr;
        HIP_TRY(hipMalloc(&qn->d_img32, (size_t)d.bytes()));
        qn->img32_bytes = d.bytes();
    }
    const hipStream_t s = (hipStream_t)stream;
    // the image from the current weights (in place updates by an optimizer or T2 included)
    PackF32Args pk{qn->w[0], qn->w[1], qn->w[2], qn->w[3], qn->w[4], qn->w[5], env->d_world, env->dims, d,
                   qn->d_img32};
    qnet_pack_f32_kernel<<<128, 256, 0, s>>>(pk);
    HIP_TRY(hipGetLastError());
    const size_t world = lds_bytes(env);
    const bool w3_global = (size_t)d.bytes() + world > 160 * 1024;
    const size_t lds = (size_t)(w3_global ? d.w3() : d.bytes()) + world;
    if (lds > 160 * 1024) return fail(SE_EINVAL, "f32 network + world image exceed the 160 KB LDS");
    static std::atomic<uint64_t> lds_set0{0}, lds_set1{0};
    rc = allow_dynamic_lds(lds_set0, reinterpret_cast<const void*>(policy_f32_kernel<false>), 160 * 1024, env->device);
    if (!rc) rc = allow_dynamic_lds(lds_set1, reinterpret_cast<const void*>(policy_f32_kernel<true>), 160 * 1024, env->device);
    if (rc) return rc;
    int dev_cus = 256;
    if (hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, env->device) != hipSuccess)
        dev_cus = 256;
    const int64_t tiles = (env->n + 31) / 32;
    const int64_t want = (tiles + kPolicyF32Waves - 1) / kPolicyF32Waves;
    const int grid = (int)(want < dev_cus ? want : dev_cus);
    PolicyF32Args F{};
    F.d = d;
    PolicyArgs& A = F.p;
    A.world = env->d_world;
    A.dims = env->dims;
    A.qimg = reinterpret_cast<const uint4*>(qn->d_img32);
    A.q = d.q;
    A.n = env->n;
    A.env_base = env->env_base;
    A.seed = env->seed;
    A.t = t;
    A.eps = epsilon;
    A.st = env->st;
    A.actions = actions;
    A.q_out = q_out;
    A.ldq = ldq;
    if (rec) {
        A.rec_pos = rec->pos;
        A.rec_fuel = rec->fuel;
        A.rec_act = rec->act;
        A.rec_head = rec->head;
        A.rec_cap = rec->cap;
    }
    if (w3_global) policy_f32_kernel<true><<<grid, kPolicyF32Block, lds, s>>>(F);
    else policy_f32_kernel<false><<<grid, kPolicyF32Block, lds, s>>>(F);
    HIP_TRY(hipGetLastError());
    return SE_OK;
}

}  // namespace

extern "C" {

int se_policy(se_qnet* qn, int32_t* actions, double epsilon, uint32_t t, float* q_out, int64_t ldq,
              void* stream) {
    return launch_policy(qn, actions, epsilon, t, q_out, ldq, nullptr, stream);
}

int se_policy_f32(se_qnet* qn, int32_t* actions, double epsilon, uint32_t t, float* q_out, int64_t ldq,
                  void* stream) {
    return launch_policy_f32(qn, actions, epsilon, t, q_out, ldq, nullptr, stream);
}

int se_qnet_repack(se_qnet* qn, int32_t* bump, void* stream) {
    if (!qn) return fail(SE_EINVAL, "null qnet");
    if (!qn->packed) return fail(SE_ESTATE, "se_qnet_set_weights has not been called");
    se_env* env = qn->env;
    if (qn->world_version != env->world_version)
        return fail(SE_ESTATE, "ports changed: call se_qnet_set_weights (the port block is folded into fc1)");
    DeviceGuard g(env->device);
    PackArgs A{qn->w[0], qn->w[1], qn->w[2], qn->w[3], qn->w[4], qn->w[5], env->d_world, env->dims,
               {qn->q, qn->qc}, {qn->d_img, qn->d_img + qn->c_off}, bump};
    qnet_pack_kernel<<<dim3(64, 2), 256, 0, (hipStream_t)stream>>>(A);
    HIP_TRY(hipGetLastError());
    return SE_OK;
}


int se_qnet_destroy(se_qnet* qn) {
    if (!qn) return SE_OK;
    if (qn->d_img || qn->d_img32) {  // does not touch the env, which may be gone already
        DeviceGuard g(qn->device);
        (void)hipDeviceSynchronize();
        if (qn->d_img) (void)hipFree(qn->d_img);
        if (qn->d_img32) (void)hipFree(qn->d_img32);
    }
    delete qn;
    return SE_OK;
}

}  // extern "C"
