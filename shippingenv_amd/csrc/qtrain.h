// qtrain.h — the DQN update fused on MFMA in f32 arithmetic.
//
// Part of shipenv.hip's translation unit (included at its end, after replay.h).
// Reference: agents/dqn.py DQNAgent.update (:206-245) on a sampled minibatch.
// It computes q = DQNNetwork(states)[a] and y = r + gamma * max target(next_states) * (1 - done),
// then nn.MSELoss and backward, then Adam (lr, betas (0.9, 0.999), eps 1e-8).
//
// The torch version is about 50 small kernels per update, launch-bound below B = 2^13.
// Here it is two kernels, all in f32 arithmetic, deterministic (fixed summation orders, no
// atomics). The forward GEMMs (fc2 of both nets, the target's fc3) run on bf16 MFMA with
// every f32 operand split into three bf16 parts (x3_index, below); fc1 and the
// backward on v_mfma_f32_32x32x2_f32 (an exact f32 fma chain; gfx950 has no xf32):
//
// T1, qtrain_tile_kernel (one workgroup per 32 samples, 8 waves: the online and the
// target net's four 32-row feature tiles side by side):
// * Target net forward: fc1, fc2, then fc3 over all A rows, with a per-sample max.
// * Online net forward: fc1, fc2.
// * q_j = W3[a_j] . h2_j + b3[a_j]. Only the chosen action's Q gets a gradient, so fc3
//   is a row gather here, not a GEMM.
// * g_j = 2 w_j (q_j - y_j), then dH2 = g_j W3[a_j] (a gather too) and dZ2 = dH2 (h2 > 0).
// * dH1 = W2^T dZ2 on MFMA, then dZ1 = dH1 (h1 > 0).
// * Per-tile partial gradients: dW2 = dZ2 H1^T (MFMA, K = 32 samples), dW1 of the six
//   dynamic columns, db1, db2, the loss sum and the weight sum.
// * Per-tile partial dW3 over the tile's distinct actions: row r of a 32 x 128 partial is
//   sum_j [first(j) = r] g_j h2_j, first(j) the first sample of the tile with a_j's action
//   (one G H2^T on MFMA, K = 32), and a slot map names row r's action. A tile's 32 samples
//   hold at most 32 actions, so this is 4 MFMA chains whatever the actions are; the
//   action-tile layout it replaces ran 4 chains per 32-action tile present (up to 36).
// * The port block of every observation row is the same, so fc1 runs on the six
//   dynamic columns with W1[:, 6:] . port + b1 folded into its bias. dW1[:, 6:] is then
//   db1 (x) port.
//
// T2, qtrain_adam_kernel (256-thread workgroups over 64-element parameter blocks, and one
// per W1 row):
// * Sums the tile partials with the threads spread over the tiles: 16 tile groups x 16
//   float4 columns, then a fixed tree. Every load is independent, so the reduction
//   streams instead of walking one dependent load per tile. A W3 workgroup owns one action
//   row: it finds the tiles whose slot map holds the action (one slot at most per tile) and
//   sums those rows in tile order.
// * Divides by sum(w): the MSE mean, since w = 1 on a full batch.
// * Takes one Adam step on the parameters in place (torch nn.Linear layout).
// * Rewrites the online net's MFMA fragment images, and refolds fc1's bias for the
//   next update.
// * Data parallel (se_qtrain_grad / se_qtrain_apply): mode 1 stops after the sums and
//   stores them in a flat gradient vector (struct Grad); the ranks all-reduce it; mode 2
//   reads the summed vector instead of the partials and runs the rest unchanged, so one
//   rank's grad + apply gives the bits of mode 0.
//
// The weight operands are pre-permuted into A-fragment order, [row tile][k step][lane],
// one coalesced 256-byte load per MFMA per wave. Activations are [feature][sample]
// LDS tiles with a 33-float row stride, so both operand orientations read
// conflict-free.

namespace {

constexpr int kQT = 32;       // samples per T1 workgroup
constexpr int kLS = 33;       // LDS row stride (floats) of a [feature][sample] tile
constexpr int kQTBlock = 512; // T1: 8 waves
constexpr int kQABlock = 128; // fold / pack workgroups
constexpr int kQRBlock = 256; // T2 workgroups

typedef __attribute__((ext_vector_type(4))) float f32x4;

struct QtDims {
    int32_t P, in, A, mt3;  // in = 6 + 4P; mt3 = fc3 row tiles (A rounded up to 32)
};

struct Mlp {
    float *w1, *b1, *w2, *b2, *w3, *b3;  // DQNNetwork, torch nn.Linear layout
};

struct QtWork {
    float* pw1[2];   // [4 tiles][3 steps][64]: fc1 over the dynamic columns (online, target)
    float* pw2[2];   // [4][64][64]: fc2
    float* pw2t;     // [4][64][64]: online fc2 transposed (backward)
    float* pw3t;     // [mt3][64][64]: target fc3
    float* c1[2];    // [128]: b1 + W1[:, 6:] . port
    float* portvec;  // [in - 6]: the preprocess_state port block
    float* part_w2;  // [tiles][128][128]
    float* part_w1d; // [tiles][128][6]
    float* part_b1;  // [tiles][128]
    float* part_b2;  // [tiles][128]
    float* part_lw;  // [tiles][2]: sum w d^2, sum w
    // dW3 / db3 per distinct action of a tile: slot r sums the samples whose action first
    // occurs at sample r of the tile; part_map[t][r] is that action, or -1 (no such slot)
    float* part_w3;  // [tiles][32][128]: only the rows of live slots are stored
    float* part_b3;  // [tiles][32]
    int32_t* part_map; // [tiles][32]
    // part_slot[a][t] = the slot of action a in tile t (0..31), 0xff when
    // the tile has none; row stride slot_ld (the workspace's tile capacity)
    uint8_t* part_slot;
    int64_t slot_ld;
};

__device__ __forceinline__ void st_part(float* p, float v) { *p = v; }
// T1's dW2 / dW3 partials as 16-byte stores (4 consecutive f1 / feature columns of one
// row: the MFMAs take H1 / H2 as their A operand, so a lane's accumulator registers 4q..4q+3
// are 4 adjacent columns), write-through (buffer-store aux 16 = sc1), so the 12.6-16.8 MB of
// partials are not left dirty in the XCDs' L2s for the kernel boundary to flush before T2
// (MI355X_MICROARCH.md price list, "boundary" and "publish-large"). Update at B = 8192: 42.2
// (4-byte plain stores) -> 41.3 (16-byte plain) -> 39.65 us (16-byte write-through)
// (profiles/r04/ab_update_t1_wt.jsonl); other aux bits 17 (sc0 + sc1) 39.25, 2 (nt) 40.8,
// 18 (sc1 + nt) 46.35 against 16's 39.3 us (profiles/r04/ab_update_t1_aux.jsonl); the small
// partials write-through too: +9.7 us (profiles/r04/ab_update_t1_wt_small.jsonl).
template <typename T>
__device__ __forceinline__ void st_part1(T* p, T v) {
    static_assert(sizeof(T) == 4, "4-byte partials");
    *p = v;
}
__device__ __forceinline__ void st_part4(float* base, uint32_t idx, float a, float b, float c, float d) {
    const uint4 w = make_uint4(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b),
                               __builtin_bit_cast(uint32_t, c), __builtin_bit_cast(uint32_t, d));
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, w), r, 4u * idx, 0, 16);  // aux 16: sc1
}

__device__ __forceinline__ int acc_r(int reg, int lane) { return (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5); }

__device__ __forceinline__ f32x16 mfma_f32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// The A operands of one row tile (packed fragments, kSteps k-pairs) in registers; loaded
// ahead of the MFMAs that use them, so the L2 round trip hides under the previous layer.
template <int kSteps>
struct Frags {
    float v[kSteps];
    __device__ __forceinline__ void load(const float* __restrict__ pa, int lane) {
#pragma unroll
        for (int s = 0; s < kSteps; ++s) v[s] = pa[s * 64 + lane];
    }
};

// acc += A (fragments in registers) x B (an LDS [k][kLS] tile), k-steps [S0, S1). The B
// operands are read kQtLookahead k-steps ahead of the MFMA that uses them, pinned in that
// order by scheduling groups (one LDS read, one MFMA): left to itself the compiler read
// each pair just before its two MFMAs, so every pair waited out an LDS round trip.
constexpr int kQtLookahead = 8;
template <int kSteps, int S0 = 0, int S1 = kSteps>
__device__ __forceinline__ f32x16 gemm_lds(const Frags<kSteps>& a, const float* src, f32x16 acc, int lane) {
    const int h = lane >> 5, c = lane & 31;
    constexpr int N = S1 - S0;
    constexpr int L = kQtLookahead < N ? kQtLookahead : N;
    if constexpr (L == 0) {
#pragma unroll
        for (int s = S0; s < S1; ++s) acc = mfma_f32(a.v[s], src[(2 * s + h) * kLS + c], acc);
    } else {
        float b[N];
#pragma unroll
        for (int i = 0; i < L; ++i) b[i] = src[(2 * (S0 + i) + h) * kLS + c];
#pragma unroll
        for (int i = 0; i < N; ++i) {
            if (i + L < N) b[i + L] = src[(2 * (S0 + i + L) + h) * kLS + c];
            acc = mfma_f32(a.v[S0 + i], b[i], acc);
        }
#pragma unroll
        for (int i = 0; i < L; ++i) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // the prologue reads
#pragma unroll
        for (int i = 0; i < N; ++i) {
            if (i + L < N) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // read k-step i + L
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                 // MFMA k-step i
        }
    }
    return acc;
}

__device__ __forceinline__ f32x16 bias_init(const float* bias, int tile, int lane, int rows) {
    f32x16 a;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int row = tile * 32 + acc_r(r, lane);
        a[r] = row < rows ? bias[row] : 0.0f;
    }
    return a;
}

__device__ __forceinline__ void store_relu(float* dst, int tile, const f32x16& acc, int lane) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const float x = acc[r];
        dst[(tile * 32 + acc_r(r, lane)) * kLS + (lane & 31)] = x > 0.0f ? x : 0.0f;
    }
}

// T1's forward GEMMs (fc2 of both nets, the target's fc3) on v_mfma_f32_32x32x16_bf16 with
// every f32 operand split into three bf16 parts (split3 in qpolicy.h: round to nearest, exact
// remainders) and the six part products of order <= 2, smallest first: the policy's
// fp32-faithful datapath (§10), at 6 x 32 MFMA cycles per K = 16 where the f32 MFMA takes
// 8 x 64. fc2 / fc3's weights are stored pre-split in global memory (three bf16 parts,
// [tile][k-step][part][lane] bf16x8, kstep_x3's layout; 6 B per weight instead of 4), so T1
// runs no weight splits; the activations are split once, by the wave that produced them, into
// LDS B fragments. The backward stays on f32 MFMA: split-bf16 backward forms measured slower
// (dH1 / dW2 / dW3 split in registers: update 38.8 -> 41.1 us, profiles/r05/ab_update_x3_backward.jsonl;
// dW2 / dW3 from sample-major split tiles: 34.0 -> 37.3 us, profiles/r05/time_update_x3bt.jsonl):
// the splits of operands that are read once cost more than the MFMA cycles they save.
// T1 also writes each tile's action -> slot table column, so a W3 block of T2 reads one
// coalesced 256-byte row of it instead of scanning every tile's 32-entry slot map (9.4 MB of
// map lines across the W3 blocks at B = 8192); 0: the scan

// f32 image index of W[row][k] (128 columns) for the split-bf16 A operand: [row tile][k-step
// g][lane][8], element j of lane (r, h) = W[32 tile + r][32 (g >> 1) + acc_row(g & 1, j, h)],
// the column order in which a 32 x 32 accumulator's registers 8s..8s+7 are the B fragment of
// k-step s (qnet_pack_kernel's acc_row)
__host__ __device__ __forceinline__ int x3_index(int row, int k) {
    const int kk = k & 31, g = 2 * (k >> 5) + (kk >> 4), h = (kk >> 2) & 1, j = 4 * ((kk >> 3) & 1) + (kk & 3);
    return (((row >> 5) * 8 + g) * 64 + (row & 31) + 32 * h) * 8 + j;
}

// bf16 index of part 0 of W[row][k] in a pre-split image: [row tile][k-step g]
// [part][lane][8], elements as x3_index; part p is 512 p further
__host__ __device__ __forceinline__ int x3w_index(int row, int k) {
    const int kk = k & 31, g = 2 * (k >> 5) + (kk >> 4), h = (kk >> 2) & 1, j = 4 * ((kk >> 3) & 1) + (kk & 3);
    return (((row >> 5) * 8 + g) * 3 * 64 + (row & 31) + 32 * h) * 8 + j;
}

// acc + W X over k-steps [g0, g0 + G) with pre-split weights w[i][part] and the LDS B fragments
// S[g][part][lane] (the next k-step's read while this one's MFMAs run)
template <int G>
__device__ __forceinline__ f32x16 gemm_x3w(const bf16x8 (*w)[3], const bf16x8* S, int g0, f32x16 acc, int lane) {
    bf16x8 x[2][3];
#pragma unroll
    for (int p = 0; p < 3; ++p) x[0][p] = S[(g0 * 3 + p) * 64 + lane];
#pragma unroll
    for (int i = 0; i < G; ++i) {
        const int c = i & 1, n = c ^ 1;
        if (i + 1 < G)
#pragma unroll
            for (int p = 0; p < 3; ++p) x[n][p] = S[((g0 + i + 1) * 3 + p) * 64 + lane];
        acc = mfma_bf16(w[i][0], x[c][2], acc);
        acc = mfma_bf16(w[i][1], x[c][1], acc);
        acc = mfma_bf16(w[i][2], x[c][0], acc);
        acc = mfma_bf16(w[i][0], x[c][1], acc);
        acc = mfma_bf16(w[i][1], x[c][0], acc);
        acc = mfma_bf16(w[i][0], x[c][0], acc);
    }
    return acc;
}

// parts p0 .. p1 - 1 of eight f32 weights (a, b) -> their bf16 splits w[0..2] (split3)
__device__ __forceinline__ void split8_half(const float4& a, const float4& b, bf16x8 (&w)[3], int half) {
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int q = 2 * half; q < 2 * half + 2; ++q) {
        const f32x2 x{v[2 * q], v[2 * q + 1]};
        const bf16x2 p0 = __builtin_convertvector(x, bf16x2);
        const f32x2 r1 = sub2(x, __builtin_convertvector(p0, f32x2));
        const bf16x2 p1 = __builtin_convertvector(r1, bf16x2);
        const bf16x2 p2 = __builtin_convertvector(sub2(r1, __builtin_convertvector(p1, f32x2)), bf16x2);
        w[0][2 * q] = p0[0];
        w[0][2 * q + 1] = p0[1];
        w[1][2 * q] = p1[0];
        w[1][2 * q + 1] = p1[1];
        w[2][2 * q] = p2[0];
        w[2][2 * q + 1] = p2[1];
    }
}

// sample-major split tiles: [part][feature][32 samples] bf16, 64-byte rows of four 16-byte chunks
// (8 samples each), chunk k of row r stored at chunk slot k ^ ((r >> 2) & 3), so that 16
// consecutive rows' chunk k (one 16-lane pass of a fragment read) fall in 16 distinct bank groups
__device__ __forceinline__ int tslot(int row, int chunk) { return row * 4 + (chunk ^ ((row >> 2) & 3)); }
constexpr int kTS = 32;
// eight f32 values -> their three bf16 parts, stored as chunk slot `slot` of the three parts'
// sample-major split tiles (parts 128 x 32 elements apart)
__device__ __forceinline__ void t_split8(const float (&v)[8], __bf16* T, int slot) {
    __bf16* dst = T + 8 * slot;
    bf16x8 w[3];
    const float4 x = make_float4(v[0], v[1], v[2], v[3]), y = make_float4(v[4], v[5], v[6], v[7]);
    split8_half(x, y, w, 0);
    split8_half(x, y, w, 1);
#pragma unroll
    for (int p = 0; p < 3; ++p) *reinterpret_cast<bf16x8*>(dst + p * 128 * kTS) = w[p];
}
// the same from eight consecutive floats of an f32 LDS tile row
__device__ __forceinline__ void t_split_row(const float* src, __bf16* T, int slot) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = src[i];
    t_split8(v, T, slot);
}

// acc + W X over k-steps [g0, g0 + G): W from f32 registers wa[2 (g - g0)], [2 (g - g0) + 1]
// (split here), X the LDS B fragments S[g][part][lane]. Step g + 1's splits and LDS reads are
// issued between step g's MFMAs (sched_barrier fences: left alone the scheduler
// clustered the VALU ahead of the chain, as in the policy's x3 kernel).
template <int G>
__device__ __forceinline__ f32x16 gemm_x3(const float4* wa, const bf16x8* S, int g0, f32x16 acc, int lane) {
    bf16x8 w[2][3], x[2][3];
    split8_half(wa[0], wa[1], w[0], 0);
    split8_half(wa[0], wa[1], w[0], 1);
#pragma unroll
    for (int p = 0; p < 3; ++p) x[0][p] = S[(g0 * 3 + p) * 64 + lane];
#pragma unroll
    for (int i = 0; i < G; ++i) {
        const int c = i & 1, n = c ^ 1;
        if (i + 1 < G)
#pragma unroll
            for (int p = 0; p < 3; ++p) x[n][p] = S[((g0 + i + 1) * 3 + p) * 64 + lane];
        acc = mfma_bf16(w[c][0], x[c][2], acc);
        acc = mfma_bf16(w[c][1], x[c][1], acc);
        acc = mfma_bf16(w[c][2], x[c][0], acc);
        __builtin_amdgcn_sched_barrier(0);
        if (i + 1 < G) split8_half(wa[2 * i + 2], wa[2 * i + 3], w[n], 0);
        __builtin_amdgcn_sched_barrier(0);
        acc = mfma_bf16(w[c][0], x[c][1], acc);
        acc = mfma_bf16(w[c][1], x[c][0], acc);
        acc = mfma_bf16(w[c][0], x[c][0], acc);
        __builtin_amdgcn_sched_barrier(0);
        if (i + 1 < G) split8_half(wa[2 * i + 2], wa[2 * i + 3], w[n], 1);
        __builtin_amdgcn_sched_barrier(0);
    }
    return acc;
}

// relu of a 32-row accumulator tile `tile` of a layer's output, split into the LDS B
// fragments of k-steps 2 tile, 2 tile + 1 (each lane its own slots: see x3_index)
__device__ __forceinline__ void store_split(bf16x8* S, int tile, const f32x16& acc, int lane) {
    bf16x8 sp[2][3];
    relu_split3(acc, sp);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int p = 0; p < 3; ++p) S[((2 * tile + s) * 3 + p) * 64 + lane] = sp[s][p];
}

// Sum over a wave in a fixed butterfly of __shfl_xor: lane i and lane i^m add the same
// two values, so every lane ends with the same bits.
__device__ __forceinline__ float wave_sum_f32(float x) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m);
    return x;
}

// fc1 row f's port block folded into its bias: thread t < 128 sums the columns c = 6 + t,
// 6 + t + 128, ... in order, then waves 0 and 1 each reduce (wave_sum_f32) and the
// result is w0 + w1. Called by every thread of a 128- or 256-thread workgroup, so the
// pack and the Adam kernel compute identical bits. `red` holds 2 floats.
__device__ __forceinline__ float fold_row(const float* w1row, int in, const float* portvec, float* red) {
    float x = 0.0f;
    if (threadIdx.x < kQABlock)
        for (int c = 6 + (int)threadIdx.x; c < in; c += kQABlock) x += w1row[c] * portvec[c - 6];
    x = wave_sum_f32(x);
    if ((threadIdx.x & 63) == 0 && threadIdx.x < kQABlock) red[threadIdx.x >> 6] = x;
    __syncthreads();
    const float r = red[0] + red[1];
    __syncthreads();
    return r;
}

__device__ __forceinline__ int frag_index(int row, int k) {  // [row tile][k step][lane]
    return ((row >> 5) * 64 + (k >> 1)) * 64 + (row & 31) + 32 * (k & 1);
}

struct QtPackArgs {
    Mlp net;
    int which;  // 0 online, 1 target
    QtDims d;
    QtWork W;
    const uint32_t* world;
    WorldDims wd;
};

// workgroup f < 128: the port vector (workgroup 0 stores it) and row f's fold; every
// workgroup then packs a strided share of the fragments
__global__ __launch_bounds__(kQABlock) void qtrain_pack_kernel(QtPackArgs A) {
    __shared__ float red[kQABlock];
    __shared__ float port[4 * SE_MAX_PORTS];
    const int P = A.d.P, in = A.d.in;
    const LdsWorld wv = world_view(A.wd, A.world);  // the device image, read in place
    for (int c = threadIdx.x; c < 4 * P; c += kQABlock) {
        const int p = c >> 2, f = c & 3;
        port[c] = f == 0 ? (float)wv.px(p) : f == 1 ? (float)wv.py(p) : f == 2 ? (float)wv.pfuel(p) : (float)wv.pcargo(p);
        if (blockIdx.x == 0) A.W.portvec[c] = port[c];
    }
    __syncthreads();
    const int f = blockIdx.x;
    if (f < 128) {
        const float fold = fold_row(A.net.w1 + (int64_t)f * in, in, port, red);
        if (threadIdx.x == 0) A.W.c1[A.which][f] = A.net.b1[f] + fold;
    }
    const int n1 = 4 * 3 * 64, n2 = 4 * 64 * 64, n3 = A.which ? A.d.mt3 * 64 * 64 : 0;
    const int total = n1 + 2 * n2 + n3;
    for (int e = blockIdx.x * kQABlock + threadIdx.x; e < total; e += gridDim.x * kQABlock) {
        if (e < n1) {
            const int lane = e & 63, s = (e >> 6) % 3, tile = e / (3 * 64);
            const int row = tile * 32 + (lane & 31), k = 2 * s + (lane >> 5);
            A.W.pw1[A.which][e] = A.net.w1[(int64_t)row * in + k];
        } else if (e < n1 + n2) {
            continue;  // fc2's split image: below
        } else if (e < n1 + 2 * n2) {
            if (A.which) continue;  // the transposed image is the online net's (backward)
            const int i = e - n1 - n2, lane = i & 63, s = (i >> 6) & 63, tile = i >> 12;
            A.W.pw2t[i] = A.net.w2[(2 * s + (lane >> 5)) * 128 + tile * 32 + (lane & 31)];
        } else {
            continue;  // fc3's split image: below
        }
    }
    // fc2 (and the target's fc3) pre-split: one item per (tile, k-step, lane), its 8 weights'
    // three parts
    const int m2 = 4 * 8 * 64, m3 = A.which ? A.d.mt3 * 8 * 64 : 0;
    for (int e = blockIdx.x * kQABlock + threadIdx.x; e < m2 + m3; e += gridDim.x * kQABlock) {
        const bool two = e < m2;
        const int i = two ? e : e - m2, lane = i & 63, g = (i >> 6) & 7, tile = i >> 9;
        const int row = tile * 32 + (lane & 31);
        bf16x8 p[3];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 32 * (g >> 1) + acc_row(g & 1, j, lane >> 5);
            const float v = two ? A.net.w2[row * 128 + k] : (row < A.d.A ? A.net.w3[row * 128 + k] : 0.0f);
            __bf16 a, b, c;
            split3(v, a, b, c);
            p[0][j] = a;
            p[1][j] = b;
            p[2][j] = c;
        }
        bf16x8* dst = reinterpret_cast<bf16x8*>(two ? A.W.pw2[A.which] : A.W.pw3t) + (tile * 8 + g) * 3 * 64 + lane;
#pragma unroll
        for (int q = 0; q < 3; ++q) dst[q * 64] = p[q];
    }
}

struct QtStepArgs {
    QtWork W;
    Mlp on, tg;
    QtDims d;
    int64_t B;
    const float *obs, *next_obs;
    const int64_t* act;
    const float *rew, *done, *weight;
    float gamma;
    int32_t* bump;  // se_qtrain_step_policy: the update counter, advanced once here (T2 reads it after)
    // se_qtrain_step_replay: the minibatch drawn here from the ring (the sampler's picks, key
    // t = ctr[0]) instead of read from obs ... weight; block 0 sets ctr[1] = t + 1 (T2's count)
    int32_t from_ring;  // 0: the minibatch buffers above
    Ring ring;
    uint64_t seed;
    int32_t* ctr;
    // the sampler key and the ring's size as the host knows them at enqueue (eager calls), so
    // the picks do not wait on a device load first; -1: read ctr[0] / the ring's size word
    int64_t t_host, size_host;
};

#ifndef SHIPENV_QTRACE
#define SHIPENV_QTRACE 0  // 1 = diagnostic build: per-wave phase stamps of T1 (tools/qtrain_trace.py);
                          // 2 = the same, slots 14 / 15 inside the input staging instead (wave 0:
                          // picks issued, picks in LDS; tools/qtrain_trace.py --inputs)
#endif
#if SHIPENV_QTRACE == 2
#define QSTAMP_IN(k) QSTAMP(k)
#define QSTAMP_MFMA(k) \
    do {               \
    } while (0)
#else
#define QSTAMP_IN(k) \
    do {             \
    } while (0)
#define QSTAMP_MFMA(k) QSTAMP(k)
#endif
#if SHIPENV_QTRACE
constexpr int kQTraceWg = 1024, kQTraceStamps = 16;
__device__ uint64_t g_qtrace[kQTraceWg * 8 * kQTraceStamps];
#define QSTAMP(k)                                                                              \
    do {                                                                                       \
        const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                                  \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < kQTraceWg)                                 \
            g_qtrace[(blockIdx.x * 8 + (threadIdx.x >> 6)) * kQTraceStamps + (k)] = t_;        \
    } while (0)
#else
#define QSTAMP(k) \
    do {          \
    } while (0)
#endif

// 8 waves: 0-3 the online net's feature tiles, 4-7 the target net's, concurrently; fc3
// of the target net and the dW3 tiles over all 8; then dH1 (waves 0-3) beside dW2 (4-7).
__global__ __launch_bounds__(kQTBlock) void qtrain_tile_kernel(QtStepArgs A) {
    extern __shared__ float sm[];
    float* X = sm;                  // [8][kLS] obs, dynamic columns (rows 6, 7 zero)
    float* XN = X + 8 * kLS;        // next obs
    float* HA = XN + 8 * kLS;       // [128][kLS] online h1
    float* HB = HA + 128 * kLS;     // online h2
    float* TA = HB + 128 * kLS;     // target h1, then dZ2
    float* TB = TA + 128 * kLS;     // target h2, then dZ1
    float* DZ2 = TA;
    float* DZ1 = TB;
    float* QM = TB + 128 * kLS;     // [8][32] per-wave max of the target Q
    float* Y = QM + 8 * 32;         // [32] targets
    float* G = Y + 32;              // [32] g_j
    float* LW = G + 32;             // [32] w_j d_j^2
    float* WT = LW + 32;            // [32] w_j
    int* ACT = reinterpret_cast<int*>(WT + 32);
    float* RW = WT + 64;            // [32] r_j
    float* DN = RW + 32;            // [32] done_j
    int* FST = reinterpret_cast<int*>(DN + 32);  // [32] first(j): the dW3 slot of sample j
    // split-bf16 B fragments [k-step][part][lane]: h1 of both nets, the target's h2; fc3's
    // partial accumulators of the tiles past the eighth ([tile - 8][wt][reg][lane] f32) reuse
    // the h1 fragments once fc2 is done
    bf16x8* SH1 = reinterpret_cast<bf16x8*>(FST + 32);  // [2][8][3][64]
    bf16x8* SH2 = SH1 + 2 * 8 * 3 * 64;                  // [8][3][64]
    float* XP = reinterpret_cast<float*>(SH1);
    int* MAPL = reinterpret_cast<int*>(SH2 + 8 * 3 * 64);  // [32] the tile's slot map
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wt = wave & 3;
    const bool tgt = wave >= 4;
    const int64_t r0 = (int64_t)blockIdx.x * kQT;
    const int in = A.d.in;
    QSTAMP(0);
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= kQTBlock / 2) __builtin_amdgcn_s_setprio(1);
    if (A.bump && blockIdx.x == 0 && tid == 0)  // no return value: the wave does not wait on it
        __hip_atomic_fetch_add(A.bump, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    // fc1's operands and fc2's fragments do not depend on the batch: their loads are in
    // flight while the inputs are staged
    const int net = tgt ? 1 : 0;
    // fc1's operands first: behind the fragment loads, fc1 waited for all of them
    Frags<3> f1;
    f1.load(A.W.pw1[net] + wt * 3 * 64, lane);
    f32x16 acc1 = bias_init(A.W.c1[net], wt, lane, 128);
    // the first try of wave 0's minibatch picks: its ring loads go out ahead of the weights'
    // (the vector memory counter is in order: behind ~24 KB of fragments per wave they waited)
    PickFirst pf{{-1, 0u, 0u, 0.0f, 0.0f, 0.0f, 0, 0}, -1};
    U4 pkey{};
    int64_t psize = 0;
    uint32_t pt = 0;
    if (A.from_ring && tid < 32) {
        psize = A.size_host >= 0 ? A.size_host : *A.ring.d_size;
        pt = A.t_host >= 0 ? (uint32_t)A.t_host : (uint32_t)A.ctr[0];
        pkey = draw(env_key(A.seed, kReplayKeyId), pt, kSlotReplay);
        if (r0 + tid < A.B) pf = pick_issue(A.ring, psize, pkey, feistel_half((uint32_t)psize), r0 + tid);
    }
    QSTAMP_IN(14);  // (wave 0: the picks' loads issued)
    Frags<64> fb;   // W2^T (dH1), loaded during fc3
    bf16x8 wa[8][3];  // fc2's pre-split A operands
    {
        const bf16x8* p = reinterpret_cast<const bf16x8*>(A.W.pw2[net]) + wt * 8 * 3 * 64;
#pragma unroll
        for (int g = 0; g < 8; ++g)
#pragma unroll
            for (int q = 0; q < 3; ++q) wa[g][q] = p[(g * 3 + q) * 64 + lane];
    }

    if (A.from_ring) {  // the sampler's pick of row r0 + tid, straight into the tiles
        if (tid < 32) {
            const Ring& ring = A.ring;
            const int64_t row = r0 + tid;
            Pick pk{-1, 0u, 0u, 0.0f, 0.0f, 0.0f, 0, 0};
            const uint32_t t = pt;
            if (row < A.B) pk = pick_resolve(pf, ring, psize, pkey, feistel_half((uint32_t)psize), row, A.B);
            const bool ok = pk.slot >= 0;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                X[c * kLS + tid] = c < 6 && ok ? ship_col(pk.sp, pk.sf, c) : 0.0f;
                XN[c * kLS + tid] = c < 6 && ok ? ship_col(pk.np, pk.nf, c) : 0.0f;
            }
            // as the sampler's act / weight rows read below: act = ok ? a : 0, weight = ok
            const int64_t a = row < A.B ? (ok ? (int64_t)pk.ac : 0) : -1;
            const bool live = a >= 0 && a < A.d.A;
            ACT[tid] = live ? (int)a : 0;
            WT[tid] = live && ok ? 1.0f : 0.0f;
            RW[tid] = ok ? pk.rw : 0.0f;
            DN[tid] = ok && (pk.fl & kRecDone) ? 1.0f : 0.0f;
            if (blockIdx.x == 0 && tid == 0) A.ctr[1] = (int32_t)(t + 1u);  // T2's Adam count
            QSTAMP_IN(15);  // (the picked transitions arrived and are in LDS)
        }
    } else {
        for (int e = tid; e < 2 * 8 * 32; e += kQTBlock) {
            const int which = e >> 8, c = (e >> 5) & 7, j = e & 31;
            const int64_t row = r0 + j;
            float v = 0.0f;
            if (c < 6 && row < A.B) v = (which ? A.next_obs : A.obs)[row * in + c];
            (which ? XN : X)[c * kLS + j] = v;
        }
        if (tid < 32) {
            // an action outside [0, A) (the reference's gather would raise) takes no part in the
            // update (weight 0), and its W3 row gather reads row 0 instead of past the matrix
            const int64_t row = r0 + tid;
            const int64_t a = row < A.B ? A.act[row] : -1;
            const bool live = a >= 0 && a < A.d.A;
            ACT[tid] = live ? (int)a : 0;
            WT[tid] = live ? A.weight[row] : 0.0f;
            RW[tid] = row < A.B ? A.rew[row] : 0.0f;
            DN[tid] = row < A.B ? A.done[row] : 0.0f;
        }
    }
    __syncthreads(); QSTAMP(1);

    // this thread's slice of W3[a_j] (q_j and dZ2 below): sample j = tid >> 4, features
    // 8 (tid & 15) .. + 7
    const int qj = tid >> 4, qpart = tid & 15;
    auto qfeat = [&](int k) { return qpart * 8 + k; };
    float w3s[8];
    {
        const float* w3r = A.on.w3 + (int64_t)ACT[qj] * 128 + qpart * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) w3s[k] = w3r[k];
    }

    // fc1 (f32 MFMA, K = 6), then its relu split into the h1 fragments (the online net's
    // f32 h1 is kept too, for the backward)
    {
        const f32x16 a1 = gemm_lds(f1, tgt ? XN : X, acc1, lane);
        if (!tgt) store_relu(HA, wt, a1, lane);
        store_split(SH1 + net * 8 * 3 * 64, wt, a1, lane);
    }
    __syncthreads(); QSTAMP(2);
    // fc2 of row tile wt; fc3's A operands (tile `wave`) load behind its first k-step,
    // into the registers fc2's consumed k-steps free
    // fc3's pre-split A operands of k-step g load once fc2's k-step g has consumed its own
    // (fenced, so that at most one k-step's worth more is live)
    bf16x8 wb[8][3];
    // the chain starts at 0 and the bias is added after it, so its loads' round trip hides
    // under the chain instead of holding its first MFMA
    const f32x16 bias2 = bias_init(tgt ? A.tg.b2 : A.on.b2, wt, lane, 128);
    f32x16 acc = {};
    {
        const bf16x8* S = SH1 + net * 8 * 3 * 64;
        const bf16x8* P3 = reinterpret_cast<const bf16x8*>(A.W.pw3t) + wave * 8 * 3 * 64;
        bf16x8 x[2][3];
#pragma unroll
        for (int q = 0; q < 3; ++q) x[0][q] = S[q * 64 + lane];
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            const int c = g & 1;
            if (g + 1 < 8)
#pragma unroll
                for (int q = 0; q < 3; ++q) x[c ^ 1][q] = S[((g + 1) * 3 + q) * 64 + lane];
            acc = mfma_bf16(wa[g][0], x[c][2], acc);
            acc = mfma_bf16(wa[g][1], x[c][1], acc);
            acc = mfma_bf16(wa[g][2], x[c][0], acc);
            acc = mfma_bf16(wa[g][0], x[c][1], acc);
            acc = mfma_bf16(wa[g][1], x[c][0], acc);
            acc = mfma_bf16(wa[g][0], x[c][0], acc);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 3; ++q) wb[g][q] = P3[(g * 3 + q) * 64 + lane];
            __builtin_amdgcn_sched_barrier(0);
        }
        acc += bias2;
        if (tgt) store_split(SH2, wt, acc, lane);
        else store_relu(HB, wt, acc, lane);
    }
    QSTAMP_MFMA(14);
    __syncthreads(); QSTAMP(3);
    // target fc3: tile `wave` on each wave (mt3 >= 9), and the mt3 - 8 (at most 2) tiles past
    // the eighth split over K: tile 8 on waves 4-7, tile 9 on waves 0-3, two k-steps each, so
    // every SIMD runs the same MFMA cycles; their partial accumulators meet in LDS (XP) and
    // wave 0 sums them in a fixed order below
    {
        const int xt = tgt ? 8 : 9;
        const bool extra = xt < A.d.mt3;  // wave-uniform
        bf16x8 wx[2][3];
        f32x16 accx = {};
        if (extra) {
            const bf16x8* p = reinterpret_cast<const bf16x8*>(A.W.pw3t) + xt * 8 * 3 * 64;
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int q = 0; q < 3; ++q) wx[u][q] = p[((2 * wt + u) * 3 + q) * 64 + lane];
            if (wt == 0) accx = bias_init(A.tg.b3, xt, lane, A.d.A);
        }
        const f32x16 bias3 = bias_init(A.tg.b3, wave, lane, A.d.A);
        f32x16 acc3 = gemm_x3w<8>(wb, SH2, 0, f32x16{}, lane) + bias3;
        if (!tgt) fb.load(A.W.pw2t + wt * 64 * 64, lane);  // dH1's operands
        float m = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (wave * 32 + acc_r(r, lane) < A.d.A) m = fmaxf(m, acc3[r]);
        m = fmaxf(m, __shfl_xor(m, 32));  // lane & 31 = sample
        if (lane < 32) QM[wave * 32 + lane] = m;
        if (extra) {
            accx = gemm_x3w<2>(wx, SH2, 2 * wt, accx, lane);
            float* o = XP + ((xt - 8) * 4 + wt) * 16 * 64;
#pragma unroll
            for (int r = 0; r < 16; ++r) o[r * 64 + lane] = accx[r];
        }
    }
    QSTAMP_MFMA(15);
    __syncthreads(); QSTAMP(4);
    if (tid < 64) {
        float mx = -INFINITY;
        // the tiles past the eighth: the four K-partials of each in a fixed order
        for (int xt = 8; xt < A.d.mt3; ++xt) {
            const float* o = XP + (xt - 8) * 4 * 16 * 64;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float v = (o[r * 64 + lane] + o[(16 + r) * 64 + lane]) +
                                (o[(32 + r) * 64 + lane] + o[(48 + r) * 64 + lane]);
                if (xt * 32 + acc_r(r, lane) < A.d.A) mx = fmaxf(mx, v);
            }
        }
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        if (tid < 32) {
            const int64_t row = r0 + tid;
            for (int w = 0; w < 8; ++w) mx = fmaxf(mx, QM[w * 32 + tid]);
            Y[tid] = row < A.B ? RW[tid] + (A.gamma * mx) * (1.0f - DN[tid]) : 0.0f;
        }
    }
    __syncthreads(); QSTAMP(5);

    // q_j = W3[a_j] . h2_j + b3[a_j]; g_j = 2 w_j (q_j - y_j): 16 threads per sample
    {
        float s = 0.0f;
#pragma unroll
        for (int k = 0; k < 8; ++k) s += w3s[k] * HB[qfeat(k) * kLS + qj];
        s += __shfl_xor(s, 1);
        s += __shfl_xor(s, 2);
        s += __shfl_xor(s, 4);
        s += __shfl_xor(s, 8);
        // the first sample of the tile with sample qj's action (its dW3 slot): this thread
        // tests samples 2 qpart and 2 qpart + 1, then a min over the 16 threads. Spread over
        // the workgroup it is free; on wave 0's 32 lanes alone it cost 0.45 us (readlanes)
        // and 2 us (a loop of dependent LDS reads).
        {
            const int aq = ACT[qj], k0 = 2 * qpart;
            int fk = ACT[k0 + 1] == aq ? k0 + 1 : 32;
            fk = ACT[k0] == aq ? k0 : fk;
            fk = min(fk, __shfl_xor(fk, 1));
            fk = min(fk, __shfl_xor(fk, 2));
            fk = min(fk, __shfl_xor(fk, 4));
            fk = min(fk, __shfl_xor(fk, 8));
            if (qpart == 0) FST[qj] = fk;
        }
        if (qpart == 0) {
            const float d = (s + A.on.b3[ACT[qj]]) - Y[qj];
            G[qj] = 2.0f * WT[qj] * d;
            LW[qj] = WT[qj] * d * d;
        }
    }
    __syncthreads(); QSTAMP(6);
    // dZ2 = (h2 > 0) g_j W3[a_j] (into the target's dead h1 buffer)
    {
        const float g = G[qj];
        float d[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int f = qfeat(k);
            d[k] = HB[f * kLS + qj] > 0.0f ? g * w3s[k] : 0.0f;
            DZ2[f * kLS + qj] = d[k];
        }
    }
    __syncthreads(); QSTAMP(7);

    const int h = lane >> 5, c = lane & 31;
    if (!tgt) {  // dH1 = W2^T dZ2 -> dZ1 = (h1 > 0) dH1
        f32x16 acc = {};
        acc = gemm_lds(fb, DZ2, acc, lane);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int f = wt * 32 + acc_r(r, lane);
            DZ1[f * kLS + c] = HA[f * kLS + c] > 0.0f ? acc[r] : 0.0f;
        }
    } else {
  // partial dW2[f2][f1] = sum_j dZ2[f2][j] h1[f1][j]: f1 tile wt, 4 f2 tiles
        // computed as its transpose H1 dZ2^T (A operands: f1 rows wt*32.. of h1, once; each
        // f2 tile's B operands read while the previous tile's chain runs), so a lane's
        // registers 4q..4q+3 are dW2[f2 = 32 ct + c][4 adjacent f1]: one 16-byte store each
        float* out = A.W.part_w2 + (int64_t)blockIdx.x * 128 * 128;
        float a2[16], b2[2][16];
#pragma unroll
        for (int s = 0; s < 16; ++s) a2[s] = HA[(wt * 32 + c) * kLS + 2 * s + h];
#pragma unroll
        for (int s = 0; s < 16; ++s) b2[0][s] = DZ2[c * kLS + 2 * s + h];
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
            f32x16 acc = {};
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                if (ct < 3) b2[(ct + 1) & 1][s] = DZ2[((ct + 1) * 32 + c) * kLS + 2 * s + h];
                acc = mfma_f32(a2[s], b2[ct & 1][s], acc);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)  // f1 = 32 wt + acc_r(4q + m, lane) = 32 wt + 8q + 4h + m
                st_part4(out, (uint32_t)((ct * 32 + c) * 128 + wt * 32 + 8 * q + 4 * h), acc[4 * q], acc[4 * q + 1],
                         acc[4 * q + 2], acc[4 * q + 3]);
        }
        // pinned order: the operands of tile 0, then per tile its chain with the next tile's
        // reads interleaved, then its stores (the compiler otherwise read each pair just
        // before its two MFMAs)
        __builtin_amdgcn_sched_group_barrier(0x100, 32, 0);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                if (ct < 3) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x040, 4, 0);
        }
        // partial dW3 over the tile's distinct actions, column tile wt: row r (slot r) =
        // sum_j [first(j) = r] g_j h2[f][j]. A lane holds its 16 k-step samples' slots and g
        // (j = 2s + h), so an A operand is a compare and a select; the 16 B operands are read
        // from LDS in one batch ahead of the chain. Only the live slots' rows are stored.
        const bool live_slot = FST[c] == c && r0 + c < A.B;
        const uint32_t slots = (uint32_t)__ballot(live_slot);  // lanes 0-31 = slots 0-31
        float bv[16], av[16];
#pragma unroll
        for (int s = 0; s < 16; ++s) bv[s] = HB[(wt * 32 + c) * kLS + 2 * s + h];
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const int j = 2 * s + h;
            av[s] = FST[j] == c ? G[j] : 0.0f;
        }
        // as its transpose H2 G^T: lane (c, h) holds slot c's features 32 wt + acc_r(r, lane),
        // 4 adjacent per register quad (16-byte stores, only a live slot's lanes)
        f32x16 acc = {};
#pragma unroll
        for (int s = 0; s < 16; ++s) acc = mfma_f32(bv[s], av[s], acc);
        float* o3 = A.W.part_w3 + (int64_t)blockIdx.x * 32 * 128;
        if ((slots >> c) & 1u)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                st_part4(o3, (uint32_t)(c * 128 + wt * 32 + 8 * q + 4 * h), acc[4 * q], acc[4 * q + 1], acc[4 * q + 2],
                         acc[4 * q + 3]);
        if (wt == 0) {  // db3 of slot c: the even samples' sum plus the odd samples' sum
            float s3 = 0.0f;
#pragma unroll
            for (int s = 0; s < 16; ++s) s3 += av[s];
            const float x3 = __shfl_xor(s3, 32);
            if (h == 0) {
                st_part1(A.W.part_b3 + (int64_t)blockIdx.x * 32 + c, s3 + x3);
                st_part1(A.W.part_map + (int64_t)blockIdx.x * 32 + c, live_slot ? (int32_t)ACT[c] : (int32_t)-1);
                MAPL[c] = live_slot ? (int32_t)ACT[c] : (int32_t)-1;
            }
        }
    }
    __syncthreads(); QSTAMP(8);  // dZ1 complete
    // partial dW1 (dynamic columns), db1, db2, loss and weight sums
    if (tid < 256) {
        // the three columns side by side: each dZ1 value is read once and the three sums
        // are independent chains (each still sums j = 0..31 in order)
        const int f = tid >> 1, c0 = (tid & 1) * 3;
        float* o = A.W.part_w1d + ((int64_t)blockIdx.x * 128 + f) * 6 + c0;
        float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f;
#pragma unroll 8
        for (int j = 0; j < 32; ++j) {
            const float d = DZ1[f * kLS + j];
            s0 += d * X[c0 * kLS + j];
            s1 += d * X[(c0 + 1) * kLS + j];
            s2 += d * X[(c0 + 2) * kLS + j];
        }
        st_part1(o, s0);
        st_part1(o + 1, s1);
        st_part1(o + 2, s2);
    } else {
        const int t = tid - 256;
        const float* src = t < 128 ? DZ2 + t * kLS : DZ1 + (t - 128) * kLS;
        float s = 0.0f;
        for (int j = 0; j < 32; ++j) s += src[j];
        st_part1((t < 128 ? A.W.part_b2 : A.W.part_b1) + (int64_t)blockIdx.x * 128 + (t & 127), s);
        if (t == 0) {
            float l = 0.0f, w = 0.0f;
            for (int j = 0; j < 32; ++j) {
                l += LW[j];
                w += WT[j];
            }
            st_part1(A.W.part_lw + 2 * blockIdx.x, l);
            st_part1(A.W.part_lw + 2 * blockIdx.x + 1, w);
        }
    }
    if (tid < 32 * A.d.mt3) {  // this tile's column of the action -> slot table
        const int4* m4 = reinterpret_cast<const int4*>(MAPL);
        int sl = 0xff;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int4 v = m4[i];
            sl = v.x == tid ? 4 * i : sl;
            sl = v.y == tid ? 4 * i + 1 : sl;
            sl = v.z == tid ? 4 * i + 2 : sl;
            sl = v.w == tid ? 4 * i + 3 : sl;
        }
        A.W.part_slot[(int64_t)tid * A.W.slot_ld + blockIdx.x] = (uint8_t)sl;
    }
    QSTAMP(9);
}

// sum over t = tid, tid + kQRBlock, ... < tiles of p[t * stride]: the first load issued with no
// wait (its value is added where the sum is used), the rest (more than kQRBlock tiles) looped
struct StridedSum {
    float first = 0.0f, rest = 0.0f;
    __device__ __forceinline__ void issue(const float* p, int64_t stride, int64_t tiles) {
        const int64_t t = threadIdx.x;
        first = t < tiles ? p[t * stride] : 0.0f;
        for (int64_t u = t + kQRBlock; u < tiles; u += kQRBlock) rest += p[u * stride];
    }
    __device__ __forceinline__ float value() const { return first + rest; }
};
// a pointer materialised in SGPRs and opaque to the optimiser (no select-of-loads rewrite into
// a per-lane load of the kernel argument)
template <typename T>
__device__ __forceinline__ T* sgpr_ptr(T* p) {
    asm volatile("" : "+s"(p));
    return p;
}
// a 4-byte load through the vector memory path (a VGPR offset the compiler cannot fold)
__device__ __forceinline__ int32_t vload_i32(const int32_t* p) {
    int z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(p), (short)0, 4, 0x00020000);
    return (int32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (uint32_t)z, 0, 0);
}

struct QtAdamArgs {
    QtWork W;
    Mlp on, m, v;
    QtDims d;
    int64_t B, tiles;
    const int64_t* act;
    float lr, beta1, beta2, eps;
    const int32_t* step_dev;  // Adam steps taken before this one (this one included when bumped)
    float* loss_out;
    // se_qtrain_step_policy: the policy's bf16 images (full, compact), rewritten from the new
    // parameters as qnet_pack_kernel would write them; img[0] null otherwise
    uint8_t* img[2];
    QnetDims q[2];
    int32_t bumped;  // T1 advanced step_dev already
    // data-parallel split (se_qtrain_grad / se_qtrain_apply): mode 0 sums the tile partials
    // and steps Adam; mode 1 stores the sums (unscaled) in grad and stops; mode 2 steps Adam
    // from grad (summed over the ranks in between) instead of the partials
    int32_t mode;
    float* grad;  // [grad_floats(d)], layout of the Grad offsets below
    int32_t* ctr_sync;  // se_qtrain_step_replay: block 0 sets *ctr_sync = *step_dev (ctr[0] = ctr[1])
};

// The data-parallel gradient: the sums T2 forms before dividing by sum(w), in a flat f32
// vector that an all-reduce(SUM) over the ranks turns into the global minibatch's sums.
// dW1's port columns are db1 (x) port (the port block is the same on every rank), so only
// the six dynamic columns travel. [128][6] dW1 dynamic, [128] db1, [128][128] dW2, [128] db2,
// [mt3 * 32][128] dW3, [mt3 * 32] db3, then {sum w d^2, sum w}.
struct Grad {
    static constexpr int64_t w1d = 0, b1 = 768, w2 = 896, b2 = 896 + 128 * 128, w3 = b2 + 128;
    __host__ __device__ static int64_t b3(const QtDims& d) { return w3 + (int64_t)d.mt3 * 32 * 128; }
    __host__ __device__ static int64_t lw(const QtDims& d) { return b3(d) + (int64_t)d.mt3 * 32; }
    __host__ __device__ static int64_t size(const QtDims& d) { return lw(d) + 2; }
};

// byte offset of W[row][k] within a packed policy image's fc2 / fc3 fragments: fragment
// ((row / 32) * 4 + k / 32) * 2 + s, lane row % 32 + 32 h, element j, where
// k % 32 = 16 s + 8 (j >> 2) + 4 h + (j & 3) (qnet_pack_kernel's acc_row map)
__device__ __forceinline__ int pol_offset(int row, int k) {
    const int kk = k & 31, s = kk >> 4, h = (kk >> 2) & 1, j = 4 * ((kk >> 3) & 1) + (kk & 3);
    return ((((row >> 5) * 4 + (k >> 5)) * 2 + s) * 64 + (row & 31) + 32 * h) * 16 + 2 * j;
}

__device__ __forceinline__ void put_bf16(uint8_t* p, float v) { *reinterpret_cast<__bf16*>(p) = (__bf16)v; }

// the row of action a in a layout (QnetDims::action_of_row inverted), -1 if it has none
__device__ __forceinline__ int row_of_action(const QnetDims& q, int a) {
    if (!q.compact || a < 4 + q.P) return a < q.rows ? a : -1;
    if (a >= 5 + q.P && a <= 4 + q.P + q.cmax) return a - 1;
    const int r = a - 51 + q.cmax;
    return a >= 55 + q.P && r < q.rows ? r : -1;
}

// torch.optim.Adam (foreach, capturable) for one element: m lerps to g, v = v b2 + (1 - b2) g g,
// p += m / ((sqrt(v) / sqrt(1 - b2^t) + eps) / (-lr / (1 - b1^t)))
struct AdamStep {
    float b1, b2, eps, step_size, bc2_sqrt;
    // steps: *A.step_dev, loaded by the caller (no counter in mode 1, which stops before any
    // Adam step)
    __device__ AdamStep(const QtAdamArgs& A, int32_t steps) : b1(A.beta1), b2(A.beta2), eps(A.eps) {
        const float t = A.step_dev ? (float)(steps + (A.bumped ? 0 : 1)) : 1.0f;
        step_size = 1.0f / ((powf(A.beta1, t) - 1.0f) / A.lr);
        bc2_sqrt = sqrtf(-(powf(A.beta2, t) - 1.0f));
    }
    __device__ float operator()(float p, float g, float& m, float& v) const {
        m = m + (1.0f - b1) * (g - m);
        v = v * b2;
        v = v + ((1.0f - b2) * g) * g;
        const float denom = ((sqrtf(v) / bc2_sqrt) + eps) / step_size;
        return p + m / denom;
    }
};

// Sums over the 256 threads of a workgroup in a fixed order, so every launch (eager or
// graph replay) gives the same bits: a butterfly of __shfl_xor within each wave (lane i
// and lane i^m add the same two values, so the lanes stay identical), then the four
// wave sums as (w0 + w1) + (w2 + w3) through LDS behind one barrier. K values reduce
// side by side behind that one barrier: the W1 blocks' seven sums used to take seven
// tree reductions of nine barriers each. `red` holds 4 * K floats.
template <int K>
__device__ __forceinline__ void block_sum(float (&x)[K], float* red) {
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = wave_sum_f32(x[k]);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) red[w * K + k] = x[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = (red[k] + red[K + k]) + (red[2 * K + k] + red[3 * K + k]);
    __syncthreads();  // red may be reused
}

__device__ __forceinline__ float block_sum256(float x, float* red) {
    float v[1] = {x};
    block_sum<1>(v, red);
    return v[0];
}

// sum over the tiles of 64 consecutive floats (src + t * stride + e0): thread (grp, q) adds
// float4 q of tiles grp, grp + 16, ...; the 16 groups then combine in a fixed order (xor 16
// and 32 inside a wave, then the four waves). Thread t < 64 returns element t of the 64.
template <int kU>  // tiles per group and round (a round: kU independent loads)
__device__ __forceinline__ float tile_sum64(const float* src, int64_t stride, int64_t e0, int64_t tiles, float4* red) {
    const int t = threadIdx.x, q = t & 15, grp = t >> 4;
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    for (int64_t k0 = grp; k0 < tiles; k0 += 16 * kU) {  // kU tiles per round, loads independent
        float4 v[kU];
#pragma unroll
        for (int i = 0; i < kU; ++i) {
            const int64_t k = k0 + 16 * i;
            v[i] = k < tiles ? *reinterpret_cast<const float4*>(src + k * stride + e0 + 4 * q)
                             : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
#pragma unroll
        for (int i = 0; i < kU; ++i) {
            acc.x += v[i].x;
            acc.y += v[i].y;
            acc.z += v[i].z;
            acc.w += v[i].w;
        }
    }
#pragma unroll
    for (int m = 16; m <= 32; m <<= 1) {
        acc.x += __shfl_xor(acc.x, m);
        acc.y += __shfl_xor(acc.y, m);
        acc.z += __shfl_xor(acc.z, m);
        acc.w += __shfl_xor(acc.w, m);
    }
    if ((t & 63) < 16) red[(t >> 6) * 16 + q] = acc;
    __syncthreads();
    float r = 0.0f;
    if (t < 64) {
        const int j = t >> 2, c = t & 3;
        const float* f = reinterpret_cast<const float*>(red);
        r = (f[4 * j + c] + f[4 * (16 + j) + c]) + (f[4 * (32 + j) + c] + f[4 * (48 + j) + c]);
    }
    __syncthreads();  // red may be reused
    return r;
}

// dW3 row a (or its half: the columns from w3's offset) and db3[a] summed over the tiles in
// tile order. A tile holds action a in at most one slot (its slot map, T1). Chunk by chunk of
// 256 tiles, thread t reads row a of the action -> slot table for tile c0 + t (or scans that
// tile's 32 map entries, 8 int4 loads, for a); the tiles that hold it are listed in tile order
// (wave ballot prefix, then the four wave offsets); thread (grp, q) then adds float4 q (of kQ
// per row part) of the rows of list entries grp, grp + 256 / kQ, ... with kU independent loads
// per round, and the groups combine in a fixed pairwise tree. However the actions are spread,
// a row sums at most one partial per tile. Thread t < 4 kQ returns column t of the part,
// thread 4 kQ db3[a].
template <int kU, int kQ>
__device__ __forceinline__ float slot_row_sum(const float* w3, const float* b3, const int32_t* map, int64_t tiles,
                                              int a, float4* red, int* list, int* wtot, const uint8_t* slot_row) {
    constexpr int kG = kQRBlock / kQ;  // groups
    const int t = threadIdx.x, q = t % kQ, grp = t / kQ, lane = t & 63, w = t >> 6;
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float accb = 0.0f;
    for (int64_t c0 = 0; c0 < tiles; c0 += kQRBlock) {
        const int64_t tt = c0 + t;
        int slot = -1;
        if (slot_row) {  // row a of the action -> slot table
            const int v = tt < tiles ? (int)slot_row[tt] : 0xff;
            slot = v == 0xff ? -1 : v;
        } else if (tt < tiles) {
            const int4* mp = reinterpret_cast<const int4*>(map + tt * 32);
            int4 v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = mp[i];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                slot = v[i].x == a ? 4 * i : slot;
                slot = v[i].y == a ? 4 * i + 1 : slot;
                slot = v[i].z == a ? 4 * i + 2 : slot;
                slot = v[i].w == a ? 4 * i + 3 : slot;
            }
        }
        const uint64_t bal = __ballot(slot >= 0);
        const int pre = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wtot[w] = __popcll(bal);
        __syncthreads();
        int off = 0, total = 0;
#pragma unroll
        for (int v = 0; v < kQRBlock / 64; ++v) {
            off += v < w ? wtot[v] : 0;
            total += wtot[v];
        }
        if (slot >= 0) list[off + pre] = t * 32 + slot;  // the row within the chunk
        __syncthreads();
        for (int i0 = grp; i0 < total; i0 += kG * kU) {
            float4 v[kU];
            float vb[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int i = i0 + kG * u;
                const bool ok = i < total;
                const int64_t row = c0 * 32 + (ok ? list[i] : 0);
                v[u] = *reinterpret_cast<const float4*>(w3 + row * 128 + 4 * q);
                vb[u] = b3[row];
                if (!ok) {
                    v[u] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                    vb[u] = 0.0f;
                }
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                acc.x += v[u].x;
                acc.y += v[u].y;
                acc.z += v[u].z;
                acc.w += v[u].w;
                accb += vb[u];
            }
        }
        __syncthreads();  // list and wtot are rewritten by the next chunk
    }
    red[grp * kQ + q] = acc;
    float* rb = reinterpret_cast<float*>(list);  // free after the last chunk's barrier
    if (q == 0) rb[grp] = accb;
    __syncthreads();
    float r = 0.0f;
    if (t <= 4 * kQ) {
        float e[kG];
        if (t < 4 * kQ) {
            const int qq = t >> 2, c = t & 3;
            const float* f = reinterpret_cast<const float*>(red);
#pragma unroll
            for (int g = 0; g < kG; ++g) e[g] = f[4 * (g * kQ + qq) + c];
        } else {
#pragma unroll
            for (int g = 0; g < kG; ++g) e[g] = rb[g];
        }
#pragma unroll
        for (int n = kG; n > 1; n >>= 1)  // ((e0 + e1) + (e2 + e3)) + ...
#pragma unroll
            for (int g = 0; g < n / 2; ++g) e[g] = e[2 * g] + e[2 * g + 1];
        r = e[0];
    }
    __syncthreads();  // red and list may be reused
    return r;
}

__device__ __forceinline__ float comp(const float4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }

// Workgroups: [0, 128) W1 row f (+ b1, the fold, the loss at f = 0); [128, 384) W2 64-element
// blocks (+ b2 on a row's first block); then mt3 x 32 W3 rows in two halves (+ b3 of the row).
__global__ __launch_bounds__(kQRBlock) void qtrain_adam_kernel(QtAdamArgs A) {
    __shared__ float red[kQRBlock];
    __shared__ float4 red4[kQRBlock];
    __shared__ float sums[8];
    __shared__ float rowbuf[6 + 4 * SE_MAX_PORTS];  // W1 blocks: the updated row, for the folds
    __shared__ float portbuf[4 * SE_MAX_PORTS];     // W1 blocks: the port block, for the folds
    __shared__ int list[kQRBlock];                  // W3 rows: the tiles of a chunk that hold the row
    __shared__ int wtot[kQRBlock / 64];
    const int tid = threadIdx.x, in = A.d.in;
    QSTAMP(10);  // T2's stamps: slots 10-13 of the same rows (4 waves)
    // the Adam count: its load is in flight while the sums' loads are issued; the step's
    // constants (two powf) are formed where the first Adam step needs them, after the
    // sums (-0.35 us against the kernel's start, profiles/r04/ab_update_late_adam.jsonl)
    // a vector load (vmcnt): as a scalar load of a line T1 has just written, its wait
    // (lgkmcnt(0), which every later kernel-argument load shares) held each block ~1.4 us
    // before its first partial-sum load
    const int32_t steps_dev = A.step_dev ? vload_i32(A.step_dev) : 0;
#define QT_ADAM() AdamStep(A, steps_dev)
    // every block has read the count; ctr[0] is read by the next update's T1 only
    // sum(w): this thread's share loads now, and the workgroup reduces it after its own
    // sum (inv is first needed by the Adam step), so the two round trips overlap
    const int mode = A.mode;  // block-uniform
    float* G = A.grad;
    // (the first load of each strided sum is not waited for here: in a loop its s_waitcnt held
    // the block one round trip before its partial sums' loads were issued)
    StridedSum ws, ls;  // ls: the loss sum, W1 block 0 (mode 0) only
    if (mode == 0 || (mode == 1 && blockIdx.x == 0)) {
        ws.issue(A.W.part_lw + 1, 2, A.tiles);
        if (mode == 0 && blockIdx.x == 0) ls.issue(A.W.part_lw, 2, A.tiles);
    }
    auto weight_inv = [&]() {
        return 1.0f / fmaxf(mode == 2 ? G[Grad::lw(A.d) + 1] : block_sum256(ws.value(), red), 1.0f);
    };
    QSTAMP(11);
    const int b = blockIdx.x;
    if (b < 128) {  // W1 row f: 6 dynamic columns + db1 reduced over the tiles, the port columns
        // row f = 16 (b % 8) + b / 8: workgroups go round robin over the 8 XCDs, so each XCD
        // sums 16 adjacent rows and the lines of [tiles][128][6] / [tiles][128] that they share
        // (24 and 4 bytes per row and tile) are fetched into its L2 once, not by every block
        const int f = ((b & 7) << 4) | (b >> 3);
        float* w1row = A.on.w1 + (int64_t)f * in;
        // the Adam operands of this thread's columns (tid, tid + 256: in <= 262) and of b1, loaded
        // now so their round trip overlaps the sums
        float pw[2] = {0.f, 0.f}, pm[2] = {0.f, 0.f}, pv[2] = {0.f, 0.f}, bw = 0.f, bm = 0.f, bv = 0.f;
        // the port block (in - 6 <= 256 values): one per thread, into LDS before the sums'
        // barrier, so the Adam step and the folds read it there (they waited on a global load)
        const float port_c = mode != 1 && tid < in - 6 ? A.W.portvec[tid] : 0.0f;
        if (mode != 1) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int c = tid + u * kQRBlock;
                if (c < in) {
                    const int64_t i = (int64_t)f * in + c;
                    pw[u] = w1row[c];
                    pm[u] = A.m.w1[i];
                    pv[u] = A.v.w1[i];
                }
            }
            if (tid == 0) {
                bw = A.on.b1[f];
                bm = A.m.b1[f];
                bv = A.v.b1[f];
            }
        }
        float x[7] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (mode == 2) {
#pragma unroll
            for (int c = 0; c < 6; ++c) x[c] = G[Grad::w1d + f * 6 + c];
            x[6] = G[Grad::b1 + f];
            if (tid < in - 6) portbuf[tid] = port_c;  // visible after the barrier below
        } else {
            for (int64_t t = tid; t < A.tiles; t += kQRBlock) {
                const float* p = A.W.part_w1d + (t * 128 + f) * 6;
#pragma unroll
                for (int c = 0; c < 6; ++c) x[c] += p[c];
                x[6] += A.W.part_b1[t * 128 + f];
            }
            if (mode == 0 && tid < in - 6) portbuf[tid] = port_c;  // visible after block_sum's barrier
            block_sum<7>(x, red);
            if (mode == 1) {
                if (tid == 0) {
#pragma unroll
                    for (int c = 0; c < 6; ++c) G[Grad::w1d + f * 6 + c] = x[c];
                    G[Grad::b1 + f] = x[6];
                }
                if (f == 0) {  // the loss and weight sums
                    float l = 0.0f;
                    for (int64_t t = tid; t < A.tiles; t += kQRBlock) l += A.W.part_lw[2 * t];
                    const float lsm = block_sum256(l, red);
                    const float wsm = block_sum256(ws.value(), red);
                    if (tid == 0) {
                        G[Grad::lw(A.d)] = lsm;
                        G[Grad::lw(A.d) + 1] = wsm;
                    }
                }
                return;
            }
        }
        const float inv = weight_inv();
        const AdamStep adam = QT_ADAM();
        if (A.ctr_sync && f == 0 && tid == 0) *A.ctr_sync = steps_dev;  // the next update's T1 reads it
        QSTAMP(12);
        if (tid == 0)  // every thread holds the sums; the row loop below indexes them by column
#pragma unroll
            for (int c = 0; c < 7; ++c) sums[c] = x[c];
        __syncthreads();
        const float s1 = sums[6];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int c = tid + u * kQRBlock;
            if (c >= in) continue;
            const float g = (c < 6 ? sums[c] : s1 * portbuf[c - 6]) * inv;
            const int64_t i = (int64_t)f * in + c;
            float mm = pm[u], vv = pv[u];
            const float p = adam(pw[u], g, mm, vv);
            A.m.w1[i] = mm;
            A.v.w1[i] = vv;
            w1row[c] = p;
            rowbuf[c] = p;
            if (c < 6) {
                A.W.pw1[0][((f >> 5) * 3 + (c >> 1)) * 64 + (f & 31) + 32 * (c & 1)] = p;
                if (A.img[0])  // the policy's fc1 fragment: element j holds column fc1_col(j)
#pragma unroll
                    for (int l = 0; l < 2; ++l)
#pragma unroll
                        for (int j = 0; j < 8; ++j)
                            if (fc1_col(j) == c) put_bf16(A.img[l] + A.q[l].w1() + ((f >> 5) * 64 + (f & 31)) * 16 + 2 * j, p);
            }
        }
        if (tid == 0) {
            sums[7] = adam(bw, s1 * inv, bm, bv);
            A.m.b1[f] = bm;
            A.v.b1[f] = bv;
        }
        __syncthreads();  // the new row (rowbuf) and b1 are complete before the folds read them
        const float b1 = sums[7];
        if (tid == 0) A.on.b1[f] = b1;
        const float xf = fold_row(rowbuf, in, portbuf, red);  // the pack kernel's bits
        if (tid == 0) A.W.c1[0][f] = b1 + xf;
        if (A.img[0] && tid == 0) {  // the policy's b1: qnet_pack_kernel's f64 fold, same order
            double acc = (double)b1;
            for (int p = 0; p < A.d.P; ++p) {
                const float* wp = rowbuf + 6 + 4 * p;
                const float* pv = portbuf + 4 * p;
                acc += (double)wp[0] * (double)pv[0] + (double)wp[1] * (double)pv[1] +
                       (double)wp[2] * (double)pv[2] + (double)wp[3] * (double)pv[3];
            }
#pragma unroll
            for (int l = 0; l < 2; ++l) reinterpret_cast<float*>(A.img[l] + A.q[l].b1())[f] = (float)acc;
        }
        if (f == 0) {  // the loss: sum w d^2 / sum w
            float loss;
            // (mode 0: this thread's share was loaded at the start, with the weight sum)
            loss = mode == 2 ? G[Grad::lw(A.d)] : block_sum256(ls.value(), red);
            if (tid == 0) *A.loss_out = loss * inv;
        }
    } else if (b < 384) {  // W2 elements e0 .. e0 + 63 (row-major [f2][f1])
        const int64_t e0 = (int64_t)(b - 128) * 64;
        const int f2 = (int)(e0 >> 7);
        // the Adam operands, loaded ahead of the sums (as in the W1 blocks)
        float pw = 0.f, pm = 0.f, pv = 0.f, bw = 0.f, bm = 0.f, bv = 0.f;
        if (mode != 1) {
            if (tid < 64) {
                const int64_t e = e0 + tid;
                pw = A.on.w2[e];
                pm = A.m.w2[e];
                pv = A.v.w2[e];
            }
            if ((e0 & 127) == 0 && tid == 0) {
                bw = A.on.b2[f2];
                bm = A.m.b2[f2];
                bv = A.v.b2[f2];
            }
        }
        float g;
        StridedSum b2s;  // a row's first block: its db2 partials, issued ahead of dW2's
        if (mode != 2 && (e0 & 127) == 0) b2s.issue(A.W.part_b2 + f2, 128, A.tiles);
        if (mode == 2) {
            g = tid < 64 ? G[Grad::w2 + e0 + tid] : 0.0f;
        } else {
            g = tile_sum64<16>(A.W.part_w2, 128 * 128, e0, A.tiles, red4);
            if (mode == 1) {
                if (tid < 64) G[Grad::w2 + e0 + tid] = g;
                if ((e0 & 127) == 0) {
                    const float x = b2s.value();
                    const float s2 = block_sum256(x, red);
                    if (tid == 0) G[Grad::b2 + f2] = s2;
                }
                return;
            }
        }
        const float inv = weight_inv();
        const AdamStep adam = QT_ADAM();
        QSTAMP(12);
        if (tid < 64) {
            const int e = (int)e0 + tid, f1 = e & 127;
            const float p = adam(pw, g * inv, pm, pv);
            A.m.w2[e] = pm;
            A.v.w2[e] = pv;
            A.on.w2[e] = p;
            {
                __bf16 p0, p1, p2;
                split3(p, p0, p1, p2);
                __bf16* img = reinterpret_cast<__bf16*>(A.W.pw2[0]) + x3w_index(f2, f1);
                img[0] = p0;
                img[512] = p1;
                img[1024] = p2;
            }
            A.W.pw2t[frag_index(f1, f2)] = p;
            if (A.img[0])
#pragma unroll
                for (int l = 0; l < 2; ++l) put_bf16(A.img[l] + A.q[l].w2() + pol_offset(f2, f1), p);
        }
        if ((e0 & 127) == 0) {
            float s2;
            if (mode == 2) {
                s2 = G[Grad::b2 + f2];
            } else {
                const float x = b2s.value();
                s2 = block_sum256(x, red);
            }
            if (tid == 0) {
                const float p = adam(bw, s2 * inv, bm, bv);
                A.m.b2[f2] = bm;
                A.v.b2[f2] = bv;
                A.on.b2[f2] = p;
                if (A.img[0])
#pragma unroll
                    for (int l = 0; l < 2; ++l) reinterpret_cast<float*>(A.img[l] + A.q[l].b2())[f2] = p;
            }
        }
    } else {  // W3 row a3's half h (64 columns) and, in half 0, b3[a3] (rows up to mt3 x 32: the padding rows' sums are 0)
        const int a3 = (b - 384) >> 1, h = (b - 384) & 1;
        const bool row_live = a3 < A.d.A;
        const bool mine = tid < 64 || (tid == 64 && h == 0);  // thread 64 of half 0: b3
        const int f3 = 64 * h + (tid & 63);
        const int64_t i3 = (int64_t)a3 * 128 + f3;
        float pw = 0.f, pm = 0.f, pv = 0.f;  // the Adam operands, loaded ahead of the sums
        // the six pointers held in SGPRs (opaque), and every thread loads both candidates: the
        // compiler otherwise merged the two branches' loads (and the stores below) into one
        // through a pointer it re-read from the kernel arguments per lane, a dependent round trip
        float *ow3 = sgpr_ptr(A.on.w3), *ob3 = sgpr_ptr(A.on.b3), *mw3 = sgpr_ptr(A.m.w3), *mb3 = sgpr_ptr(A.m.b3),
              *vw3 = sgpr_ptr(A.v.w3), *vb3 = sgpr_ptr(A.v.b3);
        if (mode != 1 && row_live) {
            const float w_ = ow3[i3], m_ = mw3[i3], v_ = vw3[i3], bw_ = ob3[a3], bm_ = mb3[a3], bv_ = vb3[a3];
            pw = tid < 64 ? w_ : bw_;
            pm = tid < 64 ? m_ : bm_;
            pv = tid < 64 ? v_ : bv_;
        }
        float g = 0.0f;  // dW3[a3][f3] (tid < 64) or db3[a3] (tid = 64)
        if (mode == 2) {
            if (tid < 64) g = G[Grad::w3 + i3];
            else if (tid == 64) g = G[Grad::b3(A.d) + a3];
        } else {
            g = slot_row_sum<16, 16>(A.W.part_w3 + 64 * h, A.W.part_b3, A.W.part_map, A.tiles, a3, red4, list, wtot,
                                     A.W.part_slot + (int64_t)a3 * A.W.slot_ld);
            if (mode == 1) {
                if (tid < 64) G[Grad::w3 + i3] = g;
                else if (tid == 64 && h == 0) G[Grad::b3(A.d) + a3] = g;
                return;
            }
        }
        const float inv = weight_inv();
        const AdamStep adam = QT_ADAM();
        QSTAMP(12);
        if (row_live && mine) {
            const float p = adam(pw, g * inv, pm, pv);
            float* dm = tid < 64 ? mw3 + i3 : mb3 + a3;
            float* dv = tid < 64 ? vw3 + i3 : vb3 + a3;
            float* dp = tid < 64 ? ow3 + i3 : ob3 + a3;
            *dm = pm;
            *dv = pv;
            *dp = p;
            if (A.img[0])
#pragma unroll
                for (int l = 0; l < 2; ++l) {
                    const int row = row_of_action(A.q[l], a3);
                    if (row < 0) continue;
                    if (tid < 64) put_bf16(A.img[l] + A.q[l].w3() + pol_offset(row, f3), p);
                    else reinterpret_cast<float*>(A.img[l] + A.q[l].b3())[row] = p;
                }
        }
    }
    QSTAMP(13);
#undef QT_ADAM
}

}  // namespace

struct se_qtrain {
    se_env* env = nullptr;
    int device = 0;
    QtDims d{};
    int64_t max_batch = 0, max_tiles = 0;
    void* d_ws = nullptr;
    QtWork W{};
    Mlp on{}, tg{}, m{}, v{};
    bool bound = false;
    uint64_t world_version = 0;
};

namespace {

Mlp mlp_of(const se_mlp* p) { return Mlp{p->w1, p->b1, p->w2, p->b2, p->w3, p->b3}; }

bool mlp_ok(const se_mlp* p) { return p && p->w1 && p->b1 && p->w2 && p->b2 && p->w3 && p->b3; }

int qtrain_pack(se_qtrain* q, int which, hipStream_t s) {
    se_env* env = q->env;
    QtPackArgs A{which ? q->tg : q->on, which, q->d, q->W, env->d_world, env->dims};
    qtrain_pack_kernel<<<256, kQABlock, 0, s>>>(A);
    HIP_TRY(hipGetLastError());
    return SE_OK;
}

}  // namespace

extern "C" {

int se_qtrain_create(se_qtrain** out, se_env* env, int64_t max_batch) {
    if (!out) return fail(SE_EINVAL, "null out");
    *out = nullptr;
    int rc = check_ready(env);
    if (rc) return rc;
    const int P = env->dims.P;
    if (P < 1 || P > 64) return fail(SE_EINVAL, "the fused update supports 1..64 ports");
    if (max_batch < 1 || max_batch > (int64_t(1) << 20)) return fail(SE_EINVAL, "max_batch must be in [1, 2^20]");
    DeviceGuard g(env->device);
    se_qtrain* q = new se_qtrain;
    q->env = env;
    q->device = env->device;
    q->d = QtDims{P, 6 + 4 * P, 4 + P + 250, (4 + P + 250 + 31) / 32};
    q->max_batch = max_batch;
    q->max_tiles = (max_batch + kQT - 1) / kQT;
    const size_t T = (size_t)q->max_tiles;
    const size_t mt3 = (size_t)q->d.mt3;
    constexpr size_t kW = 6;  // bytes per weight of fc2 / fc3's MFMA images
    const size_t sizes[] = {4 * 3 * 64, 4 * 3 * 64, 4 * 64 * 16 * kW, 4 * 64 * 16 * kW, 4 * 64 * 64,
                            mt3 * 16 * 64 * kW, 128, 128, (size_t)(4 * P),
                            T * 128 * 128, T * 128 * 6, T * 128, T * 128, T * 2, T * 32 * 128,
                            T * 32, T * 32, (mt3 * 32 * T + 3) / 4};
    size_t total = 0, off[18];
    for (int i = 0; i < 18; ++i) {
        off[i] = total;
        total += (sizes[i] * 4 + 255) & ~(size_t)255;
    }
    if (hipMalloc(&q->d_ws, total) != hipSuccess) {
        delete q;
        return fail(SE_EHIP, "hipMalloc of the update workspace failed");
    }
    float* b = static_cast<float*>(q->d_ws);
    auto at = [&](int i) { return b + off[i] / 4; };
    q->W = QtWork{{at(0), at(1)}, {at(2), at(3)}, at(4), at(5), {at(6), at(7)}, at(8),
                  at(9), at(10), at(11), at(12), at(13), at(14), at(15),
                  reinterpret_cast<int32_t*>(at(16)), reinterpret_cast<uint8_t*>(at(17)), (int64_t)T};
    *out = q;
    return SE_OK;
}

int se_qtrain_bind(se_qtrain* q, const se_mlp* online, const se_mlp* target, const se_mlp* adam_m,
                   const se_mlp* adam_v, void* stream) {
    if (!q) return fail(SE_EINVAL, "null qtrain");
    if (!mlp_ok(online) || !mlp_ok(target) || !mlp_ok(adam_m) || !mlp_ok(adam_v))
        return fail(SE_EINVAL, "null parameter pointer");
    DeviceGuard g(q->device);
    q->on = mlp_of(online);
    q->tg = mlp_of(target);
    q->m = mlp_of(adam_m);
    q->v = mlp_of(adam_v);
    int rc = qtrain_pack(q, 0, (hipStream_t)stream);
    if (rc) return rc;
    rc = qtrain_pack(q, 1, (hipStream_t)stream);
    if (rc) return rc;
    q->world_version = q->env->world_version;
    q->bound = true;
    return SE_OK;
}

int se_qtrain_pack(se_qtrain* q, int32_t which, void* stream) {
    if (!q) return fail(SE_EINVAL, "null qtrain");
    if (!q->bound) return fail(SE_ESTATE, "se_qtrain_bind has not been called");
    if (which != 0 && which != 1) return fail(SE_EINVAL, "which must be 0 (online) or 1 (target)");
    DeviceGuard g(q->device);
    return qtrain_pack(q, which, (hipStream_t)stream);
}

}  // extern "C"

namespace {
int qtrain_check_bound(se_qtrain* q) {
    if (!q) return fail(SE_EINVAL, "null qtrain");
    if (!q->bound) return fail(SE_ESTATE, "se_qtrain_bind has not been called");
    if (q->world_version != q->env->world_version)
        return fail(SE_ESTATE, "ports changed since se_qtrain_bind (the port block is folded into fc1)");
    return SE_OK;
}

// the policy must be packed from the very tensors the update changes (null: no policy)
int qtrain_check_qnet(se_qtrain* q, se_qnet* qn) {
    if (!qn) return SE_OK;
    if (!qn->packed) return fail(SE_ESTATE, "se_qnet_set_weights has not been called");
    if (qn->env != q->env) return fail(SE_EINVAL, "qnet and qtrain belong to different envs");
    if (qn->world_version != q->env->world_version)
        return fail(SE_ESTATE, "ports changed: call se_qnet_set_weights (the port block is folded into fc1)");
    const float* on[6] = {q->on.w1, q->on.b1, q->on.w2, q->on.b2, q->on.w3, q->on.b3};
    for (int k = 0; k < 6; ++k)
        if (qn->w[k] != on[k]) return fail(SE_EINVAL, "the qnet is not packed from the online parameters");
    return SE_OK;
}

QtAdamArgs adam_args(se_qtrain* q, se_qnet* qn, int64_t batch, const int64_t* act, float lr, float beta1,
                     float beta2, float eps, const int32_t* step_dev, float* loss_out, int32_t bumped,
                     int32_t mode, float* grad, int32_t* ctr_sync = nullptr) {
    const int64_t tiles = (batch + kQT - 1) / kQT;
    return QtAdamArgs{q->W, q->on, q->m, q->v, q->d, batch, tiles, act, lr, beta1, beta2, eps, step_dev, loss_out,
                      {qn ? qn->d_img : nullptr, qn ? qn->d_img + qn->c_off : nullptr},
                      {qn ? qn->q : QnetDims{}, qn ? qn->qc : QnetDims{}}, bumped, mode, grad, ctr_sync};
}

// T1, then T2 in mode 0 (grad null: sums + Adam) or mode 1 (the sums into grad)
// ring: T1 draws the minibatch itself (se_qtrain_step_replay; step_dev = ctr, two counters)
int qtrain_step(se_qtrain* q, se_qnet* qn, int64_t batch, const float* obs, const float* next_obs,
                const int64_t* act, const float* rew, const float* done, const float* weight, float gamma,
                float lr, float beta1, float beta2, float eps, int32_t* step_dev, float* loss_out,
                void* stream, float* grad = nullptr, const se_replay* ring = nullptr, int64_t t_host = -1) {
    if (int rc0 = qtrain_check_bound(q)) return rc0;
    if (batch < 1 || batch > q->max_batch) return fail(SE_EINVAL, "batch must be in [1, max_batch]");
    if (!ring && (!obs || !next_obs || !act || !rew || !done || !weight))
        return fail(SE_EINVAL, "null batch pointer");
    if (!grad && (!step_dev || !loss_out)) return fail(SE_EINVAL, "null counter / loss pointer");
    int rc = qtrain_check_qnet(q, qn);
    if (rc) return rc;
    DeviceGuard g(q->device);
    const hipStream_t s = (hipStream_t)stream;
    const int64_t tiles = (batch + kQT - 1) / kQT;
    const size_t lds = (size_t)(16 * kLS + 4 * 128 * kLS + 8 * 32 + 8 * 32) * 4 + (3 * 8 * 3 * 64 * 16 + 32 * 4 + 256);
    static std::atomic<uint64_t> lds_set{0};
    rc = allow_dynamic_lds(lds_set, reinterpret_cast<const void*>(qtrain_tile_kernel), (int)lds, q->device);
    if (rc) return rc;
    QtStepArgs A{q->W, q->on, q->tg, q->d, batch, obs, next_obs, act, rew, done, weight, gamma,
                 qn && !ring ? step_dev : nullptr, ring ? 1 : 0, ring ? ring->ring : Ring{},
                 ring ? ring->env->seed : 0, ring ? step_dev : nullptr, ring ? t_host : -1,
                 ring && t_host >= 0 ? ring->size : -1};
    qtrain_tile_kernel<<<(unsigned)tiles, kQTBlock, lds, s>>>(A);
    HIP_TRY(hipGetLastError());
    // T2 counts Adam steps from ctr[1] (set by T1) when T1 drew the batch, and syncs ctr[0]
    const QtAdamArgs B = adam_args(q, qn, batch, act, lr, beta1, beta2, eps, ring ? step_dev + 1 : step_dev,
                                   loss_out, qn || ring ? 1 : 0, grad ? 1 : 0, grad, ring ? step_dev : nullptr);
    qtrain_adam_kernel<<<384 + 64 * q->d.mt3, kQRBlock, 0, s>>>(B);
    HIP_TRY(hipGetLastError());
    return SE_OK;
}
}  // namespace

extern "C" {

int se_qtrain_step(se_qtrain* q, int64_t batch, const float* obs, const float* next_obs, const int64_t* act,
                   const float* rew, const float* done, const float* weight, float gamma, float lr, float beta1,
                   float beta2, float eps, const int32_t* step_dev, float* loss_out, void* stream) {
    return qtrain_step(q, nullptr, batch, obs, next_obs, act, rew, done, weight, gamma, lr, beta1, beta2, eps,
                       const_cast<int32_t*>(step_dev), loss_out, stream);
}

int se_qtrain_step_policy(se_qtrain* q, se_qnet* qn, int64_t batch, const float* obs, const float* next_obs,
                          const int64_t* act, const float* rew, const float* done, const float* weight,
                          float gamma, float lr, float beta1, float beta2, float eps, int32_t* step_dev,
                          float* loss_out, void* stream) {
    if (!qn) return fail(SE_EINVAL, "null qnet");
    return qtrain_step(q, qn, batch, obs, next_obs, act, rew, done, weight, gamma, lr, beta1, beta2, eps,
                       step_dev, loss_out, stream);
}

int se_qtrain_step_replay(se_qtrain* q, se_qnet* qn, se_replay* r, int64_t batch, float gamma, float lr,
                          float beta1, float beta2, float eps, int32_t* ctr, int64_t t, float* loss_out,
                          void* stream) {
    if (!r) return fail(SE_EINVAL, "null replay");
    if (!q || r->env != q->env) return fail(SE_EINVAL, "the replay and the qtrain belong to different envs");
    if (r->open) return fail(SE_ESTATE, "se_replay_begin without se_replay_end");
    if (t > 0xFFFFFFFFll) return fail(SE_EINVAL, "the sampler key t must be < 2^32 (or negative: read ctr[0])");
    return qtrain_step(q, qn, batch, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, gamma, lr, beta1, beta2,
                       eps, ctr, loss_out, stream, nullptr, r, t < 0 ? -1 : t);
}

int64_t se_qtrain_grad_size(const se_qtrain* q) { return q ? Grad::size(q->d) : 0; }

int se_qtrain_grad(se_qtrain* q, int64_t batch, const float* obs, const float* next_obs, const int64_t* act,
                   const float* rew, const float* done, const float* weight, float gamma, float* grad,
                   void* stream) {
    if (!grad) return fail(SE_EINVAL, "null grad");
    return qtrain_step(q, nullptr, batch, obs, next_obs, act, rew, done, weight, gamma, 0.0f, 0.0f, 0.0f, 0.0f,
                       nullptr, nullptr, stream, grad);
}

int se_qtrain_apply(se_qtrain* q, se_qnet* qn, const float* grad, float lr, float beta1, float beta2, float eps,
                    const int32_t* step_dev, float* loss_out, void* stream) {
    if (int rc = qtrain_check_bound(q)) return rc;
    if (!grad || !step_dev || !loss_out) return fail(SE_EINVAL, "null grad / counter / loss pointer");
    if (int rc = qtrain_check_qnet(q, qn)) return rc;
    DeviceGuard g(q->device);
    const QtAdamArgs B = adam_args(q, qn, 0, nullptr, lr, beta1, beta2, eps, step_dev, loss_out, 0, 2,
                                   const_cast<float*>(grad));
    qtrain_adam_kernel<<<384 + 64 * q->d.mt3, kQRBlock, 0, (hipStream_t)stream>>>(B);
    HIP_TRY(hipGetLastError());
    return SE_OK;
}

int se_qtrain_destroy(se_qtrain* q) {
    if (!q) return SE_OK;
    if (q->d_ws) {
        DeviceGuard g(q->device);
        (void)hipDeviceSynchronize();
        (void)hipFree(q->d_ws);
    }
    delete q;
    return SE_OK;
}

}  // extern "C"

#if SHIPENV_QTRACE
extern "C" int se_qtrace_read(void* host, size_t bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_qtrace), bytes) == hipSuccess ? 0 : -1;
}
#endif
