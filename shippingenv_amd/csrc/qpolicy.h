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

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int kQHidden = 128;     // DQNNetwork hidden_size (dqn.py:24, default 128)
// 16 waves (4 per SIMD, <= 128 VGPRs, no scratch) share one LDS copy of the network.
// Measured per launch at 2^20 envs when it was chosen (round 1 kernel): 512 threads
// 108.8 us, 768 (3 waves per SIMD, 165 VGPRs) 92.5 us, 1024 87.2 us: the fourth wave
// covers the others' MFMA -> relu -> MFMA stalls.
constexpr int kPolicyBlock = 1024;
constexpr int kPolicyWgPerCu = 1;  // resident workgroups per CU (each stages its own network copy)
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
    // the visiting order (order_chunk): null = position order; else workgroup b visits the
    // envs [b * chunk, (b + 1) * chunk) in the order it writes to order[b * chunk ...]
    uint32_t* order;
    int64_t chunk;
    int32_t lds_list;  // >= 0: the bf16 kernel keeps the list in LDS at this byte offset (u16 per env)
};

// ------------------------------------------------------------------ visiting order
// Only a ship on a port's cell can take anything but the 4 moves (is_valid_action,
// agents/dqn.py:125-175): its valid rows reach fc3's second 32-row tile (the TAKE_FUEL
// amounts), while a ship at sea needs rows 0-3 of tile 0. The policy kernels skip a
// tile no env of the wave can use, but with ~1 ship in 5 in port hardly a 32-env tile
// is all at sea (0.8^32). So from 2^16 envs each workgroup takes a contiguous chunk of envs
// and first lists them in an order where they are: its ships at sea first, then those in
// port, each group in ascending env order (order_chunk, written to a scratch list the
// workgroup alone reads); its waves then take the chunk's 32-env tiles round robin, so
// ~3 in 4 of the tiles skip fc3's second tile and every wave meets its share of in-port
// tiles. The order changes only which lane computes which env: every output is keyed by the
// env (actions, Philox draws, replay slots), so results are identical to position order.
// (Round 6 first built the order in a kernel of its own: 5.6 us per call in the trace.)
// In two halves, so that a kernel can stage its image between them (the counting half's
// loads then overlap the staging): count() walks thread t's own run [b, e) of the chunk and
// counts its ships in port; place() scans the counts over the workgroup (wsum: kBlock / 64 u64
// of LDS) and writes the list. place() ends with a barrier.
constexpr uint32_t kOrderNone = 0xffffffffu;
struct OrderRun {
    int b = 0, e = 0;
    uint32_t port = 0u, bits = 0u;  // bits: the first 32 envs' in-port flags, for place()
    // load(): a run of 4, 8, 12 or 16 envs on a 4-byte boundary (2^20 envs: 4 per thread in the
    // bf16 kernel, 8 in the fp32 one) is loaded as whole words, issued before the image is
    // staged and used after it, so the loads overlap the staging; other runs go byte by byte
    // in count() (the first form issued a dependent load chain per env: +3.3 / +8.6 us on the
    // two kernels' prologues, profiles/r06/order/trace_prologue.jsonl)
    static constexpr int kWords = 4;
    uint32_t xw[kWords] = {}, yw[kWords] = {};
    bool words = false;

    template <int kBlock>
    __device__ __forceinline__ void load(const uint8_t* xs, const uint8_t* ys, int64_t c0, int len) {
        const int per = (len + kBlock - 1) / kBlock;
        b = (int)threadIdx.x * per;
        e = min(b + per, len);
        // uniform; with len a multiple of 4 every run is whole words, none reads past the chunk
        words = (per & 3) == 0 && per <= 4 * kWords && (c0 & 3) == 0 && (len & 3) == 0;
        if (words) {
            const uint32_t* x4 = reinterpret_cast<const uint32_t*>(xs + c0 + b);
            const uint32_t* y4 = reinterpret_cast<const uint32_t*>(ys + c0 + b);
#pragma unroll
            for (int k = 0; k < kWords; ++k) {
                if (4 * k < e - b) {  // e - b: per, or a shorter multiple of 4 for the chunk's last runs
                    xw[k] = x4[k];
                    yw[k] = y4[k];
                }
            }
        }
    }

    template <int kBlock>
    __device__ __forceinline__ void count(const LdsWorld& w, const uint8_t* xs, const uint8_t* ys, int64_t c0) {
        if (words) {
#pragma unroll
            for (int k = 0; k < 4 * kWords; ++k) {
                if (k < e - b) {
                    const int x = (int)((xw[k >> 2] >> (8 * (k & 3))) & 0xffu), y = (int)((yw[k >> 2] >> (8 * (k & 3))) & 0xffu);
                    const uint32_t f = w.port_at(x, y) >= 0 ? 1u : 0u;
                    port += f;
                    bits |= f << k;
                }
            }
            return;
        }
        for (int i = b; i < e; ++i) {
            const uint32_t f = w.port_at(xs[c0 + i], ys[c0 + i]) >= 0 ? 1u : 0u;
            port += f;
            bits |= i - b < 32 ? f << (i - b) : 0u;
        }
    }

    // the list's tail up to a whole tile reads all ones (an idle lane). T = uint32_t: the envs
    // (a global scratch list); T = uint16_t: their indices in the chunk (an LDS list)
    template <int kBlock, typename T>
    __device__ __forceinline__ void place(const LdsWorld& w, const uint8_t* xs, const uint8_t* ys, int64_t c0,
                                          int len, T* out, uint64_t* wsum) const {
        constexpr bool kLocal = sizeof(T) == 2;
        if ((int)threadIdx.x < ((-len) & 31)) out[len + threadIdx.x] = (T)~(T)0;
        const uint32_t sea = (uint32_t)max(e - b, 0) - port;
        // exclusive prefix of (at sea, in port) over the threads, as two 32-bit halves
        const uint64_t mine = (uint64_t)sea | (uint64_t)port << 32;
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        uint64_t inc = mine;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t u = __shfl_up(inc, d);
            inc += lane >= d ? u : 0ull;
        }
        if (lane == 63) wsum[wv] = inc;
        __syncthreads();
        uint64_t off = 0ull, total = 0ull;
#pragma unroll
        for (int i = 0; i < kBlock / 64; ++i) {
            off += i < wv ? wsum[i] : 0ull;
            total += wsum[i];
        }
        const uint64_t ex = inc - mine + off;
        uint32_t at_sea = (uint32_t)ex, in_port = (uint32_t)total + (uint32_t)(ex >> 32);
        for (int i = b; i < e; ++i) {
            const bool p = i - b < 32 ? ((bits >> (i - b)) & 1u) != 0u : w.port_at(xs[c0 + i], ys[c0 + i]) >= 0;
            out[p ? in_port : at_sea] = kLocal ? (T)i : (T)(c0 + i);
            in_port += p ? 1u : 0u;
            at_sea += p ? 0u : 1u;
        }
        __threadfence_block();  // the list is complete before any wave of the workgroup reads it
        __syncthreads();
    }
};
constexpr int kOrderScanBytes = 16 * 8;  // place()'s wsum, past the policy's LDS (<= 16 waves)

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
// a - b on two f32 lanes as two v_sub_f32: the vector form compiles to v_pk_add_f32, whose
// issue beside MFMAs costs more than two scalar subtractions (MI355X_MICROARCH.md,
// per-instruction constants; measured about even, profiles/r05/ab_policy_f32_scalarsub.jsonl).
__device__ __forceinline__ f32x2 sub2(f32x2 a, f32x2 b) {
    float r0, r1;
    asm("v_sub_f32 %0, %1, %2" : "=v"(r0) : "v"(a[0]), "v"(b[0]));
    asm("v_sub_f32 %0, %1, %2" : "=v"(r1) : "v"(a[1]), "v"(b[1]));
    return f32x2{r0, r1};
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
    int c_lo, f_lo;          // the layout's first TAKE_CARGO / TAKE_FUEL rows (wave-uniform)
    __device__ __forceinline__ int c_hi() const { return c_lo + cst - 1; }
    __device__ __forceinline__ int f_hi() const { return f_lo + fst - 1; }
    uint64_t sel;            // SELECT: bit p for each port on the ship's cell other than the origin
};
__device__ __forceinline__ EnvValid env_valid(const LdsWorld& w, const QnetDims& q, const uint64_t* SAME, int x,
                                              int y, int origin) {
    EnvValid v;
    v.cur = w.port_at(x, y);
    v.cst = v.cur >= 0 ? min(w.pcargo(max(v.cur, 0)), 49) : 0;
    v.fst = v.cur >= 0 ? min(w.pfuel(max(v.cur, 0)), 199) : 0;
    v.c_lo = q.cargo_row1();
    v.f_lo = q.fuel_row1();
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
    v.f_lo = q.fuel_row1();
    v.sel = v.cur >= 0 ? SAME[max(v.cur, 0)] & ~(origin >= 0 ? 1ull << origin : 0ull) : 0ull;
    return v;
}

// can any row of tile mt be valid for this env (a tile no env of the wave can choose from
// is skipped, MFMAs included)
__device__ __forceinline__ bool tile_maybe(const EnvValid& v, int mt, int P) {
    const int base = mt * 32, top = base + 31;
    return (int)(mt == 0) | (int)((v.cur >= 0) & (base < 4 + P)) |
           (int)((v.cst > 0) & (v.c_lo <= top) & (v.c_hi() >= base)) | (int)((v.fst > 0) & (v.f_lo <= top) & (v.f_hi() >= base));
}

// valid rows of tile mt as bits of the tile
__device__ __forceinline__ uint32_t tile_mask(const EnvValid& v, int mt, int P) {
    const int base = mt * 32;
    uint32_t m = range_bits(-base, 3 - base) | range_bits(v.c_lo - base, v.c_hi() - base) |
                 range_bits(v.f_lo - base, v.f_hi() - base);
    if (base < 4 + P) {  // SELECT rows 4 + p live in this tile (uniform): sel shifted by 4 - base
        const int sh = base - 4;
        m |= (uint32_t)(sh < 0 ? v.sel << -sh : (sh < 64 ? v.sel >> sh : 0ull));
    }
    return m;
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
// is invalid for this env): its Q stays -inf through the MFMAs and never wins the argmax.
// Two VALU per register, a sign-extended one-bit field (v_bfe_i32) and a bitwise select
// (v_bfi_b32): no compare, so no VALU-written lane mask and none of the wait states a
// compare -> v_cndmask pair costs. The select is inline asm: written as (c & t) | (~t & -inf)
// in C, ROCm 7.2's hipcc folds it into v_bitop3_b32 chains that read ONE bias dword for all 16
// registers (a miscompile, reproduced in a 20-line kernel; tests/test_gpu_policy.py catches it).
__device__ __forceinline__ f32x16 masked_bias(const float* b, uint32_t m) {
    f32x16 c = bias_frag(b);
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int i = (reg & 3) + 8 * (reg >> 2);
        const uint32_t t = (uint32_t)((int32_t)(m << (31 - i)) >> 31);  // all ones: row valid
        float r;
        asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(t), "v"(c[reg]), "v"(0xff800000u));
        c[reg] = r;
    }
    return c;
}

// the first maximum over registers 4j..4j+3 of a masked tile (invalid rows are -inf: one
// compare and two selects per register, no validity test and no per-register branch), the
// winner's tile-local row kept as an inline constant (bt); after part 3 the caller adds the
// tile's base once if the tile raised the maximum (best != best0)
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
__device__ __forceinline__ void finish_env(const QnetDims& q, const EnvValid& v, int64_t e, bool live, int h, float best,
                                           int bidx, uint32_t x8, uint32_t y8, uint32_t o8, uint32_t d8, float ff,
                                           int32_t* actions, double eps, uint64_t seed, int64_t env_base, uint32_t t,
                                           uint32_t* rec_pos, float* rec_fuel, int32_t* rec_act, int64_t rec_head,
                                           int64_t rec_cap) {
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
            const U4 d = draw(env_key(seed, env_base + e), t, kSlotPolicy);
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

#ifndef SHIPENV_X3_TRACE
#define SHIPENV_X3_TRACE 0  // 1 = diagnostic build: per-wave s_memtime phase stamps of the fp32 policy
#endif                      // kernels' 4th tile (se_policy_trace_read, tools/time_policy.py --trace)
#if SHIPENV_X3_TRACE
__device__ uint64_t g_ptrace[4096 * 16];
#define X3STAMP(k)                                                                                          \
    do {                                                                                                    \
        if (tile_iter == 3 && (threadIdx.x & 63) == 0)                                                      \
            g_ptrace[(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % 4096 * 16 + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#define X3STAMP_ANY(k)                                                                                      \
    do {                                                                                                    \
        if ((threadIdx.x & 63) == 0) {                                                                      \
            uint64_t* p_ = g_ptrace + (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % 4096 * 16;       \
            p_[(k)] = __builtin_amdgcn_s_memrealtime();                                                     \
            p_[(k) + 3] = __builtin_amdgcn_s_memtime();                                                     \
        }                                                                                                   \
    } while (0)
#else
#define X3STAMP(k) \
    do {           \
    } while (0)
#define X3STAMP_ANY(k) X3STAMP(k)
#endif
template <bool kQout>
__global__ __launch_bounds__(kPolicyBlock)
void policy_kernel(PolicyArgs A) {
    extern __shared__ uint4 smem[];
    X3STAMP_ANY(9);
    const QnetDims q = A.q;
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const int64_t tiles = (A.n + 31) >> 5;
    // env state of one tile (lane & 31 = env); the next tile's is loaded while this one
    // computes, so the wave does not wait on HBM at the top of every tile. The first tile's
    // loads go out before the network image and the world are staged, so they overlap.
    struct EnvIn {
        double fuel;
        uint32_t x, y, o8, d8;
        int64_t e;  // the env (A.order), past A.n for the last tile's idle lanes
    };
    // the visiting order: this workgroup's chunk and its list (null: position order)
    const uint16_t* ord16 = nullptr;  // or in LDS (chunk indices)
    const uint32_t* ord = nullptr;
    int64_t c0 = 0;
    int len = 0;
    OrderRun orun;
    if (A.order) {  // loaded here, counted and placed once the image and the world are staged
        c0 = (int64_t)blockIdx.x * A.chunk;
        len = __builtin_amdgcn_readfirstlane((int)min(A.chunk, A.n - c0));  // uniform: an SGPR
        orun.load<kPolicyBlock>(A.st.x, A.st.y, c0, len);
    }
    auto load_env = [&](int64_t tile) {
        const int64_t p = tile * 32 + r;
        int64_t ei;
        bool live;
        if (ord16) {  // p < the chunk's whole tiles: its tail reads 0xffff
            const uint32_t v = ord16[p];
            live = v != 0xffffu;
            ei = live ? c0 + (int64_t)v : A.n - 1;
        } else if (ord) {  // the same in global memory, kOrderNone
            const uint32_t v = ord[p];
            live = v != kOrderNone;
            ei = live ? (int64_t)v : A.n - 1;
        } else {
            live = p < A.n;
            ei = live ? p : A.n - 1;
        }
        return EnvIn{A.st.fuel[ei], A.st.x[ei], A.st.y[ei], A.st.origin[ei], A.st.dest[ei], live ? ei : A.n};
    };
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= 12) __builtin_amdgcn_s_setprio(1);
    const int qwords = q.bytes() / 16;
    // fc1's bias rides in the padding half of its single k-step: lanes 32-63 of each W1
    // fragment (k = 8..15, zero in the packed image) get the three bf16 parts of their row's
    // b1 at elements 0-2, and the input's k = 8..10 are 1.0, so the chain starts at 0 and the
    // bias is not read per tile (4 x 16-byte LDS reads per row tile)
    const int w1w = q.w1() / 16, b1f = q.b1() / 4;
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
    const LdsWorld w = stage_world(A.world, A.dims, reinterpret_cast<uint32_t*>(smem + qwords));
    if (A.order) {
        uint32_t* list = A.order + c0;
        uint64_t* wsum = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(smem) +
                                                     ((q.bytes() + 4 * A.dims.padded() + 7) & ~7));
        orun.count<kPolicyBlock>(w, A.st.x, A.st.y, c0);  // the cell codes from LDS
        if (A.lds_list >= 0) {  // the list in LDS: no global stores, fence or list reads from L2
            uint16_t* list16 = reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(smem) + A.lds_list);
            orun.place<kPolicyBlock>(w, A.st.x, A.st.y, c0, len, list16, wsum);
            ord16 = list16;
        } else {
            orun.place<kPolicyBlock>(w, A.st.x, A.st.y, c0, len, list, wsum);
            ord = list;
        }
    }
    X3STAMP_ANY(10);
    [[maybe_unused]] int tile_iter = 0;  // SHIPENV_X3_TRACE: the wave's 4th tile is stamped
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
    // tiles: the chunk's (waves round robin) or all of them (striding over the grid); after
    // the order is placed (A.order: the tile loop reads the list)
    const bool ordered = A.order != nullptr;
    const int64_t my_tiles = ordered ? (len + 31) >> 5 : tiles;
    int64_t tile = ordered ? (threadIdx.x >> 6) : (int64_t)blockIdx.x * kPolicyWaves + (threadIdx.x >> 6);
    const int64_t stride = ordered ? kPolicyWaves : (int64_t)gridDim.x * kPolicyWaves;
    EnvIn nxt = load_env(tile < my_tiles ? tile : 0);
    for (; tile < my_tiles; tile += stride, ++tile_iter) {
        X3STAMP(0);
        const EnvIn cur_in = nxt;
        if (tile + stride < my_tiles) nxt = load_env(tile + stride);
        const int64_t e = cur_in.e;
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
        if (h) {  // k = 8..10: 1.0 against the bias parts, 11..15 padding
            ob = bf16x8{};
            ob[0] = ob[1] = ob[2] = (__bf16)1.0f;
        }

        bf16x8 h1[4][2], h2[4][2];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {  // fc1 + relu
            f32x16 c = {};
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(W1f[mt * 64 + lane], ob, c, 0, 0, 0);
            relu_pack(c, h1[mt]);
        }
        X3STAMP(1);
        // fc2 + relu one row tile per pass: no spills at 128 VGPRs (2 tiles a pass spill 7
        // registers, 4 spill 14); a pass's relu issues in the shadow of the next pass's MFMAs
        constexpr int kFc2Passes = 4, kFc2Tiles = 4 / kFc2Passes;
#pragma unroll
        for (int pass = 0; pass < kFc2Passes; ++pass) {
            f32x16 c2[kFc2Tiles];
#pragma unroll
            for (int i = 0; i < kFc2Tiles; ++i)
                c2[i] = bias_frag(B2 + (pass * kFc2Tiles + i) * 32 + 4 * h);
            static_assert(kFc2Tiles == 1, "the fragment lookahead is written for one tile per pass");
            // the tile's 8 fragments read L k-steps ahead of their MFMA, pinned in that order
            // (one LDS read, one MFMA): left to itself the compiler read each fragment right
            // before its MFMA and waited out the LDS round trip every time (L = 2 and 3
            // measure even, profiles/r05/ab_policy_bf16_la.jsonl)
            constexpr int L = 1;
            bf16x8 wf[8];
#pragma unroll
            for (int k = 0; k < L; ++k) wf[k] = W2f[(pass * 8 + k) * 64 + lane];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (k + L < 8) wf[k + L] = W2f[(pass * 8 + k + L) * 64 + lane];
                c2[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[k], h1[k >> 1][k & 1], c2[0], 0, 0, 0);
            }
#pragma unroll
            for (int k = 0; k < L; ++k) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (k + L < 8) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            }
#pragma unroll
            for (int i = 0; i < kFc2Tiles; ++i) relu_pack(c2[i], h2[pass * kFc2Tiles + i]);
        }

        X3STAMP(2);
        // is_valid_action (dqn.py:125-175): moves always; SELECT p at the ship's cell
        // and != origin; TAKE_CARGO / TAKE_FUEL at a port with 0 < amount <= stock
        const int cur = w.port_at(x, y);
        const int cst = cur >= 0 ? min(w.pcargo(max(cur, 0)), 49) : 0;
        const int fst = cur >= 0 ? min(w.pfuel(max(cur, 0)), 199) : 0;
        // valid TAKE rows of this env in the layout's row space
        const int c_lo = q.cargo_row1(), c_hi = c_lo + cst - 1, f_lo = q.fuel_row1(), f_hi = f_lo + fst - 1;
        // SELECT: bit p for each port on the ship's cell other than the origin (P <= 64)
        const uint64_t sel = cur >= 0 ? SAME[max(cur, 0)] & ~(origin >= 0 ? 1ull << origin : 0ull) : 0ull;
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
        float best = -INFINITY;
        int bidx = 0x7fffffff;
        if (use64) {
            // compact layouts of at most 64 rows (the bench's greedy and epsilon calls): rows
            // this env cannot take start at -inf (masked_bias, two VALU per register), so the
            // first maximum is a compare and two selects per register with no validity test and
            // no per-register branch, and fc3 tile 0's argmax runs beside tile 1's MFMAs
            constexpr int L3 = 2;  // fragments read L3 k-steps ahead (a 3-slot ring: 12 VGPRs)
            bf16x8 wf[L3 + 1];
#pragma unroll
            for (int k = 0; k < L3; ++k) wf[k] = W3f[k * 64 + lane];
            // a tile of ships at sea only (uniform; the visiting order makes them ~3 in 4):
            // rows 0-3, the moves, are each env's valid rows, registers 0-3 of lane half 0
            const bool sea = !__any(cur >= 0);
            f32x16 c = sea ? bias_frag(B3 + 4 * h) : masked_bias(B3 + 4 * h, (uint32_t)v64 >> (4 * h));
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (k + L3 < 8) wf[(k + L3) % (L3 + 1)] = W3f[(k + L3) * 64 + lane];
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[k % (L3 + 1)], h2[k >> 1][k & 1], c, 0, 0, 0);
            }
            int bt = 0, pbase = 0;
            if (sea) {
                argmax_local_part(c, best, bt, 0);
                best = h ? -INFINITY : best;  // lane half 1 holds rows 4-7
                bidx = best != -INFINITY ? bt : bidx;
            } else if (q.mt3 > 1 && __any((uint32_t)(v64 >> 32) != 0u)) {  // fc3 tile 1 (uniform)
#pragma unroll
                for (int k = 0; k < L3; ++k) wf[k] = W3f[(8 + k) * 64 + lane];
                f32x16 c1 = masked_bias(B3 + 32 + 4 * h, (uint32_t)(v64 >> 32) >> (4 * h));
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    if (k + L3 < 8) wf[(k + L3) % (L3 + 1)] = W3f[(8 + k + L3) * 64 + lane];
                    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[k % (L3 + 1)], h2[k >> 1][k & 1], c1, 0, 0, 0);
                    if (k < 4) argmax_local_part(c, best, bt, k);  // tile 0's, beside tile 1's chain
                    __builtin_amdgcn_sched_barrier(0);
                }
                bidx = best != -INFINITY ? bt : bidx;
                c = c1;
                pbase = 32;
            }
            if (!sea) {
                const float best0 = best;
#pragma unroll
                for (int g = 0; g < 4; ++g) argmax_local_part(c, best, bt, g);
                bidx = best != best0 ? pbase + bt : bidx;
                bidx += bidx == 0x7fffffff ? 0 : 4 * h;  // the lane half's rows (argmax_local_part omits 4h)
            }
        }
        for (int mt = 0; mt < (use64 ? 0 : q.mt3); ++mt) {  // fc3 + the masked first-maximum argmax (other layouts)
            const int base = mt * 32, top = base + 31;
            // a tile no env of the wave can choose from is skipped, MFMAs included
            // (exact: its rows are invalid for all 32 envs); with port stocks <= 20
            // (add_port's randint(5, 20)) the valid rows sit in the first few tiles
            const bool maybe = (mt == 0) | ((cur >= 0) & (base < 4 + P)) |
                               ((cst > 0) & (c_lo <= top) & (c_hi >= base)) |
                               ((fst > 0) & (f_lo <= top) & (f_hi >= base));
            if (!kQout && !__any(maybe)) continue;
            uint32_t m = range_bits(-base, 3 - base) | range_bits(c_lo - base, c_hi - base) |
                         range_bits(f_lo - base, f_hi - base);
            if (base < 4 + P) {  // SELECT rows 4 + p live in this tile (uniform): sel shifted by 4 - base
                const int sh = base - 4;
                m |= (uint32_t)(sh < 0 ? sel << -sh : (sh < 64 ? sel >> sh : 0ull));
            }
            // registers that hold no valid action for any env are skipped (wave-uniform)
            const uint32_t rm = __builtin_amdgcn_readfirstlane(REGM[mt]);
            bf16x8 wf[8];  // the tile's 8 fragments, read before the chain consumes them
#pragma unroll
            for (int k = 0; k < 8; ++k) wf[k] = W3f[(mt * 8 + k) * 64 + lane];
            f32x16 c = bias_frag(B3 + mt * 32 + 4 * h);
#pragma unroll
            for (int k = 0; k < 8; ++k)
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[k], h2[k >> 1][k & 1], c, 0, 0, 0);
            m >>= 4 * h;  // register reg holds row base + 4h + (reg & 3) + 8 (reg >> 2)
            {
                // the winning register's tile-local row as an inline constant, the tile's base
                // added once if the tile raised the maximum (strict >: the first maximum stays)
                const float best0 = best;
                int bt = 0;
#pragma unroll
                for (int reg = 0; reg < 16; ++reg) {
                    if (!((rm >> reg) & 1u)) continue;
                    const int i = (reg & 3) + 8 * (reg >> 2);
                    const bool better = ((m >> i) & 1u) && c[reg] > best;  // ascending rows: first max
                    best = better ? c[reg] : best;
                    bt = better ? i : bt;
                }
                bidx = best != best0 ? base + 4 * h + bt : bidx;
            }
            if (kQout && live) {
#pragma unroll
                for (int reg = 0; reg < 16; ++reg) {  // the full layout: row = action
                    const int row = base + 4 * h + (reg & 3) + 8 * (reg >> 2);
                    if (row < q.rows) A.q_out[e * A.ldq + row] = c[reg];
                }
            }
        }
        X3STAMP(3);
        // the next tile's env loads (issued a tile ago) are waited for here, before this
        // tile's stores: stores count in vmcnt too, so a wait at the loop's back edge would
        // wait out the action / record stores' round trip as well
        asm volatile("" ::"v"(nxt.fuel), "v"(nxt.x), "v"(nxt.y), "v"(nxt.o8), "v"(nxt.d8));
        // the two lane halves hold the same env: larger value, then lower index
        const float ob2 = __shfl_xor(best, 32);
        const int oi = __shfl_xor(bidx, 32);
        if (ob2 > best || (ob2 == best && oi < bidx)) {
            best = ob2;
            bidx = oi;
        }
        if (h == 0 && live) {
            int act = bidx == 0x7fffffff ? 0 : q.action_of_row(bidx);  // no valid action: 0 (:188-189)
            if (A.eps > 0.0) {
                const U4 d = draw(env_key(A.seed, A.env_base + e), A.t, kSlotPolicy);
                if (u32(d.v[0]) <= A.eps) {  // np.random.rand() <= epsilon (:191)
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
        X3STAMP(4);
    }
    X3STAMP_ANY(11);
}

// ------------------------------------------------------------------ the split-bf16 f32 step
// The fp32-faithful form of the step (se_policy_f32): DQNNetwork evaluated as agents/dqn.py:198-200
// runs it (fp32 weights, fp32 activations), on bf16 MFMA (round 5; gfx950 has no xf32, and the
// round-4 form on v_mfma_f32_32x32x2_f32 took 0.43 ms per call at 2^20). fc1, fc2 and fc3 run
// on v_mfma_f32_32x32x16_bf16 with every f32 operand split into three bf16 parts,
// w = w0 + w1 + w2 and x = x0 + x1 + x2 (each part the round-to-nearest bf16 of what the
// parts before it leave; three 8-bit significands hold an f32's 24 bits), and the six
// products whose parts sum to at most 2, w0x2 + w1x1 + w2x0 + w0x1 + w1x0 + w0x0, smallest
// first, into one f32 accumulator. The dropped products (w1x2, w2x1, w2x2) are below
// 2^-23 of |w x|: a simulation of this datapath against float64 (MFMA = one f32 rounding
// per instruction) errs like the f32 MFMA path and torch's fp32 GEMM.
// Six bf16 MFMAs (32 cycles each) per 16-deep k-step where the f32 datapath runs eight
// v_mfma_f32_32x32x2_f32 (64 cycles each): 2.7x fewer MFMA cycles. fc1 (6 live inputs)
// runs as two split-bf16 MFMAs per row tile (x3_fc1_slot). Relu'd activations are split
// once per layer (registers 8s..8s+7 of tile kt are k-step (kt, s)'s B operand, as in the
// bf16 kernel) and held as 24 bf16x8 parts. Image: fc1 fragments, f32 biases, fc2 and fc3
// as three bf16 fragments per (tile, kt, s): 96 KB + 24 KB per fc3 tile, so the world is
// read in place (L2), not staged, and fc3 comes from global memory when it does not fit
// (the full layout). One 32-env tile per wave; 512-thread workgroups, one per CU.
struct QnetX3Dims {
    QnetDims q;
    int32_t zrow;  // bf16x8 index, at k-step 0 and part 0, of a zero row of fc3's last tile (lane 31 of it), or -1
    __host__ __device__ int w1() const { return 0; }  // fc1: bf16 fragments [mt][2 steps][lane] (8 KB)
    __host__ __device__ int w2() const { return 8192; }                 // [mt][kt][s][part] bf16 fragments: 96 KB
    __host__ __device__ int b1() const { return w2() + 96 * 1024; }
    __host__ __device__ int b2() const { return b1() + 4 * kQHidden; }
    __host__ __device__ int b3() const { return b2() + 4 * kQHidden; }  // mt3 * 32 f32
    __host__ __device__ int same() const { return b3() + q.mt3 * 128; }
    __host__ __device__ int regm() const { return same() + 8 * q.P; }
    __host__ __device__ int w3() const { return (regm() + 4 * q.mt3 + 15) & ~15; }  // mt3 x 24 KB, last
    __host__ __device__ int bytes() const { return w3() + q.mt3 * 24 * 1024; }
};


// fc1 on bf16 MFMA: the six dynamic columns' products as 24 of the 32 k
// slots of two v_mfma_f32_32x32x16_bf16 per row tile. Slot k (step k >> 4, lane half
// (k >> 3) & 1, element k & 7) holds weight part wp of column col times input part xp:
// x, y, origin, dest are exact in bf16 (|v| <= 255), so they take w0 x + w1 x + w2 x; the
// fuel column (2) and the "cargo" = fuel column (3, environment.py:206) take the six split
// products of w and the fuel f32. Columns: 0 x, 1 y, 2 fuel, 3 cargo, 4 origin, 5 dest.
struct Fc1Slot {
    int8_t col, wp, xp;  // xp: -1 = the exact input, else the fuel part
};
// Slots 24-31 are zero. (fc1's bias folded into slots 24-26 against inputs of 1.0 measured even
// or slower, profiles/r05/ab_policy_f32_bias_fold.jsonl; the bf16 kernel's 64-bit valid-row
// masks here 0.2724 vs 0.2630 ms per call, profiles/r05/ab_policy_f32_valid64.jsonl.)
constexpr int kX3PtabBytes = 3 * 64 * 4 + 16;  // the staged port table, past the image
__host__ __device__ constexpr Fc1Slot x3_fc1_slot(int k) {
    constexpr Fc1Slot t[24] = {{0, 0, -1}, {1, 0, -1}, {4, 0, -1}, {5, 0, -1}, {0, 1, -1}, {1, 1, -1}, {4, 1, -1}, {5, 1, -1},
                               {0, 2, -1}, {1, 2, -1}, {4, 2, -1}, {5, 2, -1}, {2, 0, 0},  {2, 0, 1},  {2, 1, 0},  {2, 0, 2},
                               {2, 1, 1},  {2, 2, 0},  {3, 0, 0},  {3, 0, 1},  {3, 1, 0},  {3, 0, 2},  {3, 1, 1},  {3, 2, 0}};
    return k < 24 ? t[k] : Fc1Slot{-1, 0, 0};
}

struct PackX3Args {
    const float *w1, *b1, *w2, *b2, *w3, *b3;
    const uint32_t* world;
    WorldDims dims;
    QnetX3Dims d;
    uint8_t* img;
    // policy_x3_kernel's own pack: the port table (P positions, then P
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
// bias entry, same-cell mask and epilogue register mask (the latter as qnet_pack_kernel).
// items [first, total) step `stride` of the split image into img (global memory for
// qnet_pack_x3_kernel, the workgroup's LDS for policy_x3_kernel's own prologue)
// b1[f] + W1[f, 6:] . the port block, in f64 then f32 (qnet_pack_kernel's fold)
__device__ __forceinline__ float x3_fold_b1(const PackX3Args& A, int f) {
    const LdsWorld wv = pack_world(A);
    const int in1 = A.d.q.in1();
    double acc = (double)A.b1[f];
    // unrolled so that several ports' weight loads go out before the adds wait on them (the
    // adds stay in port order; unroll 8 measured even, profiles/r05/ab_policy_f32_fold_unroll.jsonl;
    // all 8 ports' loads issued before the adds measured even too, profiles/r06/order/ab_x3_fold.jsonl)
#pragma unroll 1
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
    const int n_w1 = 4 * 2 * 64, n_w2 = 32 * 64, n_w3 = q.mt3 * 8 * 64;
    const int total = n_w1 + n_w2 + n_w3 + 2 * kQHidden + q.mt3 * 32 + q.P + q.mt3;
    // fc2 / fc3 fragments first, in a loop of their own: an item's 8 weights are two float4
    // loads (elements 0-3 and 4-7 are consecutive columns), split as pairs, and 6 items' loads
    // go out together (0.2646 -> 0.2613 ms per call against 2,
    // profiles/r05/ab_policy_f32_pack_unroll.jsonl). Same bits as the
    // per-element split3 below. Taken when both weight matrices are 16-byte aligned (torch's
    // allocations are); otherwise the element-wise loop below packs them.
    const bool vec = ((reinterpret_cast<uintptr_t>(A.w2) | reinterpret_cast<uintptr_t>(A.w3)) & 15) == 0;
#pragma unroll 6
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
    for (int t = first; t < total; t += stride) {
        if (vec && t >= n_w1 && t < n_w1 + n_w2 + n_w3) continue;  // packed above
        if (t < n_w1) {
            const int lane = t & 63;
            // fc1 fragment (mt, step, lane): element j = slot 16 step + 8h + j
            const int st = (t >> 6) & 1, mt = t >> 7, row = mt * 32 + (lane & 31);
            bf16x8 v;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const Fc1Slot sl = x3_fc1_slot(16 * st + 8 * (lane >> 5) + j);
                __bf16 p0 = (__bf16)0.0f, p1 = p0, p2 = p0;
                if (sl.col >= 0) split3(A.w1[row * in1 + sl.col], p0, p1, p2);
                v[j] = sl.wp == 0 ? p0 : (sl.wp == 1 ? p1 : p2);
            }
            reinterpret_cast<bf16x8*>(img + d.w1())[t] = v;
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

// chunk q (0..15) of the relu + 3-way split of tile c into out (relu_split3 in 16 pieces of
// about five VALU): pair q >> 1 (elements 2p, 2p + 1 of k-step s), stage q & 1 (the bf16
// rounding x0 and the remainder, then x1 and x2); r holds the remainders between stages
__device__ __forceinline__ void split_chunk(const f32x16& c, bf16x8 (&out)[2][3], f32x2 (&r)[8], int q) {
    const int pr = q >> 1, s = pr >> 2, p = pr & 3;
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
__global__ __launch_bounds__(kPolicyX3Block) void policy_x3_kernel(PolicyArgs A, QnetX3Dims D, PackX3Args PK) {
    extern __shared__ uint4 smem[];
    X3STAMP_ANY(9);
    const QnetDims q = D.q;
    // the first tile's env state (an HBM round trip) is requested before the image is built,
    // so the two overlap
    const int lane = threadIdx.x & 63, h = lane >> 5;
    const int64_t tiles = (A.n + 31) >> 5;
    struct EnvIn {  // the four state bytes packed (x | y << 8 | origin << 16 | dest << 24): 2 VGPRs fewer
        double fuel;
        uint32_t pk;
        uint32_t e;  // the env (A.order), A.n for the last tile's idle lanes (n < 2^32: the order is u32)
        __device__ uint32_t x8() const { return pk & 0xffu; }
        __device__ uint32_t y8() const { return (pk >> 8) & 0xffu; }
        __device__ uint32_t o8() const { return (pk >> 16) & 0xffu; }
        __device__ uint32_t d8() const { return pk >> 24; }
    };
    // the visiting order: this workgroup's chunk and its list (null: position order)
    const uint32_t* ord = nullptr;
    int64_t c0 = 0;
    int len = 0;
    OrderRun orun;
    if (A.order) {  // loaded here, counted and placed once the image is built (the loads overlap it)
        c0 = (int64_t)blockIdx.x * A.chunk;
        len = __builtin_amdgcn_readfirstlane((int)min(A.chunk, A.n - c0));  // uniform: an SGPR
        orun.load<kPolicyX3Block>(A.st.x, A.st.y, c0, len);
    }
    auto load_env = [&](int64_t t) {
        const int64_t p = t * 32 + (lane & 31);
        int64_t ei;
        bool live;
        if (ord) {  // p < the chunk's whole tiles: its tail reads kOrderNone
            const uint32_t v = ord[p];
            live = v != kOrderNone;
            ei = live ? (int64_t)v : A.n - 1;
        } else {
            live = p < A.n;
            ei = live ? p : A.n - 1;
        }
        const uint32_t pk = (uint32_t)A.st.x[ei] | (uint32_t)A.st.y[ei] << 8 | (uint32_t)A.st.origin[ei] << 16 |
                            (uint32_t)A.st.dest[ei] << 24;
        return EnvIn{A.st.fuel[ei], pk, (uint32_t)(live ? ei : A.n)};
    };
    // tiles: the chunk's (waves round robin) or all of them (striding over the grid); in
    // position order the first tile's env state is requested before the image is built
    const bool ordered = A.order != nullptr;
    const int64_t my_tiles = ordered ? (len + 31) >> 5 : tiles;
    int64_t tile = ordered ? (threadIdx.x >> 6) : (int64_t)blockIdx.x * kPolicyX3Waves + (threadIdx.x >> 6);
    const int64_t stride = ordered ? kPolicyX3Waves : (int64_t)gridDim.x * kPolicyX3Waves;
    EnvIn nxt{};
    if (!ordered) nxt = load_env(tile < my_tiles ? tile : 0);
    if constexpr (kW3Global) {  // fc3 stays in the packed global image: copy the rest
        const int staged = D.w3() / 16;
        for (int i = threadIdx.x; i < staged; i += kPolicyX3Block) smem[i] = A.qimg[i];
    } else {
        // the whole image fits: each workgroup splits the f32 weights into its own LDS copy
        // (about 93 KB of f32 reads per workgroup at P = 5 where the packed image is 152 KB),
        // so no pack kernel runs before the policy and in-place weight updates are seen
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
    }
#if SHIPENV_X3_TRACE
    if ((threadIdx.x & 63) == 0)  // slot 15: the wave's part of the image built
        g_ptrace[(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % 4096 * 16 + 15] = __builtin_amdgcn_s_memrealtime();
#endif
    __syncthreads();
    if (ordered) {
        uint32_t* list = A.order + c0;
        const int wo = kW3Global ? ((D.w3() + 7) & ~7) : (((D.bytes() + 15) & ~15) + kX3PtabBytes);
        const LdsWorld wg = world_view(A.dims, A.world);
        orun.count<kPolicyX3Block>(wg, A.st.x, A.st.y, c0);
        orun.place<kPolicyX3Block>(wg, A.st.x, A.st.y, c0, len, list,
                                   reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(smem) + wo));
        ord = list;
        nxt = load_env(tile < my_tiles ? tile : 0);
    }
    X3STAMP_ANY(10);
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
    // the env state of the wave's next tile is loaded while this one computes (no HBM round
    // trip at the top of a tile), and its validity (the port on the ship's cell and that
    // port's stocks, two dependent L2 reads of the world image) resolved during fc3
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= 4) __builtin_amdgcn_s_setprio(1);
    EnvValid vnxt = env_valid(w, q, SAME, (int)nxt.x8(), (int)nxt.y8(), nxt.o8() == SE_NONE ? -1 : (int)nxt.o8());
    [[maybe_unused]] int tile_iter = 0;  // SHIPENV_X3_TRACE: the wave's 4th tile is stamped
    while (tile < my_tiles) {
        X3STAMP(0);
        const EnvIn in = nxt;
        const EnvValid v = vnxt;
        const int64_t tnext = tile + stride;
        const bool more = tnext < my_tiles;
        if (more) nxt = load_env(tnext);
        const int64_t e = in.e;
        const bool live = e < A.n;
        const double fuel = in.fuel;
        const uint32_t x8 = in.x8(), y8 = in.y8(), o8 = in.o8(), d8 = in.d8();
        const int origin = o8 == SE_NONE ? -1 : (int)o8, dest = d8 == SE_NONE ? -1 : (int)d8;
        const float ff = (float)fuel;  // the preprocess_state row as torch's FloatTensor holds it
        bf16x8 X1[4][2][3], X2[4][2][3];
        float best = -INFINITY;
        int bidx = 0x7fffffff;
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
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {  // fc1 (x, y | fuel, fuel | origin, dest)
            c1[mt] = bias_frag(B1 + mt * 32 + 4 * h);
            c1[mt] = mfma_bf16(W1b[(mt * 2 + 0) * 64 + lane], xin[0], c1[mt]);
            c1[mt] = mfma_bf16(W1b[(mt * 2 + 1) * 64 + lane], xin[1], c1[mt]);
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
        X3STAMP(1);
        // fragments read kLa k-steps ahead over the flat k-step sequence: fc2's 32 (k-tile
        // kt, row tile mt, step s2), then fc3 tile 0's 8
        constexpr int kLa = 2;  // 1 / 3: 0.2582 / 0.2569 vs 0.2549 ms (profiles/r05/ab_policy_f32_la.jsonl)
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
            if (i == 8) ncode = w.code((int)nxt.x8(), (int)nxt.y8());
            // unconditional (past the last tile nxt is tile 0's state, a valid address) and
            // opaque until their uses: under `if (more)` the compiler merged the arithmetic on
            // each into its load's block and waited out the round trip right there
            if (i == 24) {
                asm volatile("" : "+v"(ncode));
                nstock = w.stock[max(w.port_of_code(ncode), 0)];
            }
            if (i == 8) X3STAMP(2);
            if (i == 16) X3STAMP(3);
            if (i == 24) X3STAMP(4);
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
        X3STAMP(5);
        auto mask_of = [&](int mt) { return tile_mask(v, mt, P); };
        // a tile of ships at sea only (uniform; ~3 in 4 under the visiting order) needs rows 0-3
        // (the moves) of fc3 tile 0: its six part products go as three chains, one per
        // activation part x_j, each over the weight parts w_p with p + j <= 2 stacked in the
        // MFMA's rows (x0: w0, w1, w2 in rows 0-3, 4-7, 8-11; x1: w0, w1; x2: w0; the other
        // rows read a zero row of the image), 24 MFMAs where the tile takes 48. Q(row r) = rows
        // r + (4 + r) + (8 + r): the same six products per k-step, summed by chain (an fp32
        // rounding per MFMA as before, in another order: not the same bits as the full tile).
        // 0.2409 -> 0.2275 ms per call at 2^20 (profiles/r06/order/ab_x3_stack.jsonl); the LDS
        // image only (the global-image variant would spill).
        const bool stack = !kW3Global && !kQout && D.zrow >= 0 && !__any(v.cur >= 0);
        f32x16 c;
        if (stack) {
            c = f32x16{};
            if (h == 0) {
#pragma unroll
                for (int i = 0; i < 4; ++i) c[i] = B3[i];
            }
            const int r = lane & 31;
            // bf16x8 index of k-step 0's operand for chain j (k-step k adds 192)
            const int zero = D.zrow + 32 * h;
            const int src = (r >> 2) * 64 + (r & 3) + 32 * h;
            const int o0 = r < 12 ? src : zero, o1 = r < 8 ? src : zero, o2 = r < 4 ? src : zero;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const bf16x8 a2 = W3[k * 192 + o2], a1 = W3[k * 192 + o1], a0 = W3[k * 192 + o0];
                c = mfma_bf16(a2, X2[k >> 1][k & 1][2], c);
                c = mfma_bf16(a1, X2[k >> 1][k & 1][1], c);
                c = mfma_bf16(a0, X2[k >> 1][k & 1][0], c);
                if (k < 4) {  // X2[3] complete before k-step 6 reads it
                    split_pair(acc[3], X2[3], 2 * k);
                    split_pair(acc[3], X2[3], 2 * k + 1);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
            c = kQout ? bias_frag(B3 + 4 * h) : masked_bias(B3 + 4 * h, mask_of(0) >> (4 * h));
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
        }
        X3STAMP(6);
        // the next tile's validity from the world reads issued during fc2 (ncode, nstock)
        // waited for here on every path: a wait only inside env_valid_from's port branch left
        // the load outstanding into the next tile, whose first write of its registers then
        // waited out the new env loads as well
        asm volatile("" ::"v"(nstock.x), "v"(nstock.y));
        vnxt = env_valid_from(w, q, SAME, ncode, nstock, nxt.o8() == SE_NONE ? -1 : (int)nxt.o8());
        // fc3 tiles 1..: the previous tile's argmax beside each chain, 4 registers a group
        int pbase = 0;
        [[maybe_unused]] float best0 = best;
        [[maybe_unused]] int bt = 0;
        uint32_t pm = kQout ? tile_mask(v, 0, P) : 0u, prm = __builtin_amdgcn_readfirstlane(REGM[0]);
        if (kQout && live) tile_q_out(A.q_out, A.ldq, q.rows, c, e, 0, h);
#pragma nounroll
        for (int mt = 1; mt < q.mt3; ++mt) {
            const int base = mt * 32;
            const uint32_t m3 = kQout ? 0u : mask_of(mt);
            if (!kQout && !__any(tile_maybe(v, mt, P))) continue;
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
                            if (g == 0) best0 = best;
                            argmax_local_part(c, best, bt, g);
                            if (g == 3) bidx = best != best0 ? pbase + bt : bidx;
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
        X3STAMP(7);
        if (kQout) {
            tile_argmax(c, pm, prm, pbase, h, best, bidx);
        } else if (stack) {  // rows 0-3 from the three chains' partial rows
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float qi = (c[i] + __shfl_xor(c[i], 32)) + c[4 + i];
                const bool better = qi > best;  // ascending rows: the first maximum
                best = better ? qi : best;
                bidx = better ? i : bidx;
            }
            best = h ? -INFINITY : best;  // lane half 1 holds no row of its own
            bidx = h ? 0x7fffffff : bidx;
        } else {
            best0 = best;
#pragma unroll
            for (int g = 0; g < 4; ++g) argmax_local_part(c, best, bt, g);
            bidx = best != best0 ? pbase + bt : bidx;
            bidx += bidx == 0x7fffffff ? 0 : 4 * h;  // the lane half's rows (argmax_local_part omits 4h)
        }
        FINISH_ENV(v, e, live, h, best, bidx, x8, y8, o8, d8, ff);
        X3STAMP(8);
        tile = more ? tnext : my_tiles;
        ++tile_iter;
    }
    X3STAMP_ANY(11);
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
    uint8_t* d_img32 = nullptr;  // se_policy_f32's split image (the full layout's fc3, global)
    int img32_bytes = 0;
    // the visiting order's scratch list (order_chunk): used when n >= order_min_envs, resolved once
    // by se_qnet_create (SHIPENV_POLICY_ORDER: 0 never, 1 always; unset: from 2^16 envs; 2 always,
    // with the bf16 kernel's list in this global scratch as when it does not fit the LDS, which
    // otherwise happens only past ~10M envs)
    uint32_t* d_order = nullptr;
    int64_t order_cap = 0, order_min_envs = (int64_t)1 << 16;
    bool order_lds = true;
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
    if (const char* v = getenv("SHIPENV_POLICY_ORDER")) {
        qn->order_min_envs = atoi(v) != 0 ? 0 : INT64_MAX;
        qn->order_lds = atoi(v) != 2;
    }
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
// the visiting order's chunk per workgroup (a multiple of 32) and the grid that covers n with
// it, and the scratch list (A.order, A.chunk); position order below order_min_envs
int policy_order(se_qnet* qn, int* grid, PolicyArgs& A) {
    se_env* env = qn->env;
    A.order = nullptr;
    A.chunk = 0;
    if (env->n < qn->order_min_envs) return SE_OK;
    const int64_t per = (env->n + *grid - 1) / *grid;
    const int64_t chunk = (per + 31) & ~(int64_t)31;
    const int64_t g = (env->n + chunk - 1) / chunk;
    if (g * chunk > qn->order_cap) {
        if (qn->d_order) HIP_TRY(hipFree(qn->d_order));
        qn->d_order = nullptr;
        HIP_TRY(hipMalloc(&qn->d_order, (size_t)(g * chunk) * sizeof(uint32_t)));
        qn->order_cap = g * chunk;
    }
    *grid = (int)g;
    A.order = qn->d_order;
    A.chunk = chunk;
    return SE_OK;
}

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
    size_t lds = (((size_t)q.bytes() + lds_bytes(env) + 7) & ~(size_t)7) + kOrderScanBytes;
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
    int grid = (int)(want < resident ? want : resident);
    PolicyArgs A{};
    rc = policy_order(qn, &grid, A);
    if (rc) return rc;
    A.lds_list = -1;
    if (A.order && qn->order_lds && A.chunk <= 0xffff && lds + (size_t)A.chunk * 2 <= 160 * 1024) {  // the list in LDS
        A.lds_list = (int32_t)lds;
        lds += (size_t)A.chunk * 2;
    }
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
    if (q_out) {
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
    // a zero row of fc3's last tile (row 32 mt3 - 1, past the layout's rows), or none
    d.zrow = d.q.rows < 32 * d.q.mt3 ? (d.q.mt3 - 1) * 8 * 192 + 31 : -1;
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
    constexpr int kPtabBytes = kX3PtabBytes;
    const bool w3_global = d.bytes() + kPtabBytes + kOrderScanBytes > 160 * 1024;
    if (w3_global) {  // fc3's fragments are read from a packed global image
        qnet_pack_x3_kernel<<<128, 256, 0, s>>>(pk);
        HIP_TRY(hipGetLastError());
    }
    const size_t lds = (size_t)(w3_global ? ((d.w3() + 7) & ~7) : ((d.bytes() + 15) & ~15) + kPtabBytes) +
                       kOrderScanBytes;
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
    int grid = (int)(want < dev_cus ? want : dev_cus);
    PolicyArgs A{};
    rc = policy_order(qn, &grid, A);
    if (rc) return rc;
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
        policy_x3_kernel<true, true><<<grid, kPolicyX3Block, lds, s>>>(A, d, pk);
    } else if (w3_global) {
        policy_x3_kernel<true><<<grid, kPolicyX3Block, lds, s>>>(A, d, pk);
    } else {
        policy_x3_kernel<false><<<grid, kPolicyX3Block, lds, s>>>(A, d, pk);
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
    return launch_policy_x3(qn, actions, epsilon, t, q_out, ldq, rec, stream);
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

#if SHIPENV_X3_TRACE
int se_policy_trace_read(void* host, size_t bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ptrace), bytes) == hipSuccess ? 0 : -1;
}
#endif

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
    if (qn->d_img || qn->d_img32 || qn->d_order) {  // does not touch the env, which may be gone already
        DeviceGuard g(qn->device);
        (void)hipDeviceSynchronize();
        if (qn->d_img) (void)hipFree(qn->d_img);
        if (qn->d_img32) (void)hipFree(qn->d_img32);
        if (qn->d_order) (void)hipFree(qn->d_order);
    }
    delete qn;
    return SE_OK;
}

}  // extern "C"
