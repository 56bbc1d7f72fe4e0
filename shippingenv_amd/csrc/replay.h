// replay.h — the DQN experience replay ring on the device.
//
// Part of shipenv.hip's translation unit (included at its end, after qpolicy.h).
// Reference: agents/dqn.py DQNAgent.remember (:117-123, a deque(maxlen=memory_size)
// of (state, action, reward, next_state, done)) and the minibatch of update()
// (:213-224: random.sample(memory, batch_size), np.vstack of the preprocess_state
// rows, FloatTensor / LongTensor).
//
// A transition is kept in its compact form, 25 bytes, instead of two observation
// rows (2 x 104 B at P = 5, 2 x 1048 B at P = 64):
// * the ship's x, y, origin and dest bytes;
// * f32 fuel (the row's f32 value: FloatTensor rounds the f64 fuel once);
// * the agent-index action;
// * the f32 reward (the reference's f64 reward rounded once, as FloatTensor does);
// * a flags byte.
// for s and s'. The port block of a row is constant, so the sampler rebuilds it
// from the world image in LDS. The ring is SoA, written by one coalesced pass before
// and one after each vector step (se_replay_begin / _end: 13 + 17 bytes per env).
//
// Sampling without replacement, like random.sample: batch position j takes
// logical index perm(j) of a keyed 4-round Feistel permutation of [0, size)
// (cycle-walking over the next even power of two), so the B indices are distinct
// with no sort, no rejection table and no atomics, each thread on its own. A
// transition whose step raised (err != 0: the reference's loop breaks before
// remember, :281-309) is stored but flagged; its batch slot moves on to position
// j + B, j + 2B, ... (still distinct), and a slot that finds none in kReplayTries
// positions gets weight 0.

namespace {

constexpr int kReplayTries = 4;
constexpr int kSampleRows = 64;                   // transitions per sample workgroup
constexpr int64_t kReplayKeyId = -1;              // Philox key (seed, 2^64 - 1): no env has this id

struct Ring {
    uint32_t* s_pos;  // x | y << 8 | origin << 16 | dest << 24 of s
    float* s_fuel;
    int32_t* act;
    float* rew;
    uint8_t* flags;
    uint32_t* n_pos;  // s'
    float* n_fuel;
    int64_t* d_size;  // transitions stored (device copy, read by the sampler)
};

__device__ __forceinline__ uint32_t pack_pos(const se_state& st, int64_t i) {
    return (uint32_t)st.x[i] | (uint32_t)st.y[i] << 8 | (uint32_t)st.origin[i] << 16 | (uint32_t)st.dest[i] << 24;
}

struct RecordArgs {
    int64_t n, cap, head, new_size;
    se_state st;
    const int32_t* act;
    Ring ring;
    uint8_t* cut;
    int32_t max_steps;
    // se_replay_end_reset: reset() the cut envs in the same pass, exactly as se_reset(cut)
    // would (reset_kernel: Philox(seed, env) at (epoch, slot 5)); world null otherwise
    const uint32_t* world;
    WorldDims dims;
    uint64_t seed;
    int64_t env_base;
    uint32_t epoch;
    uint32_t t;  // the step counter after the recorded step (the next step's index): an
                 // episode's length is t - ep_start, and a restarted one starts at t
};

// s and a of every env, before se_step (remember's state, action)
__global__ __launch_bounds__(kBlock) void replay_begin_kernel(RecordArgs A) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < A.n; i += (int64_t)gridDim.x * kBlock) {
        int64_t slot = A.head + i;
        slot -= slot >= A.cap ? A.cap : 0;
        A.ring.s_pos[slot] = pack_pos(A.st, i);
        A.ring.s_fuel[slot] = (float)A.st.fuel[i];
        A.ring.act[slot] = A.act[i];
    }
}

// reward, done and s' after se_step; cut[i]: the episode must restart now (the
// step raised: the reference's loop breaks, :304-309; or it reached max_steps, :281)
__global__ __launch_bounds__(kBlock) void replay_end_kernel(RecordArgs A) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *A.ring.d_size = A.new_size;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < A.n; i += (int64_t)gridDim.x * kBlock) {
        int64_t slot = A.head + i;
        slot -= slot >= A.cap ? A.cap : 0;
        const bool raised = A.st.err[i] != SE_ERR_OK;
        A.ring.rew[slot] = A.st.reward[i];
        A.ring.flags[slot] = (uint8_t)((A.st.done[i] ? kRecDone : 0) | (raised ? kRecInvalid : 0));
        A.ring.n_pos[slot] = pack_pos(A.st, i);
        A.ring.n_fuel[slot] = (float)A.st.fuel[i];
        if (!A.cut) continue;
        const bool cut = raised | (A.max_steps > 0 && (int32_t)(A.t - (uint32_t)A.st.ep_start[i]) >= A.max_steps);
        A.cut[i] = (uint8_t)cut;
        if (A.world && cut) {  // reset_kernel's body for this env
            const LdsWorld w = world_view(A.dims, A.world);
            const U4 o = draw(env_key(A.seed, A.env_base + i), A.epoch, kSlotExplicitReset);
            Ship s;
            reset_ship(w, s, o.v[0], o.v[1]);
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
}

// replay_end_kernel for four consecutive envs per thread, when the ring slots of a group
// are consecutive too (head, cap and n multiples of 4): every field moves as one 4-byte
// (u8 fields) or 16-byte (f32 / i32 / f64 pair) lane access, as in the step kernel, where one
// env per thread issued a 1-byte access per u8 field. Same stores, same bits.
__device__ __forceinline__ uint32_t byte_at(uint32_t w, int j) { return (w >> (8 * j)) & 0xffu; }

__global__ __launch_bounds__(kBlock) void replay_end4_kernel(RecordArgs A) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *A.ring.d_size = A.new_size;
    const int64_t groups = A.n >> 2;
    for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < groups; g += (int64_t)gridDim.x * kBlock) {
        const int64_t i0 = g * 4;
        int64_t slot = A.head + i0;
        slot -= slot >= A.cap ? A.cap : 0;
        const uint32_t err4 = *reinterpret_cast<const uint32_t*>(A.st.err + i0);
        const uint32_t done4 = *reinterpret_cast<const uint32_t*>(A.st.done + i0);
        const uint32_t x4 = *reinterpret_cast<const uint32_t*>(A.st.x + i0);
        const uint32_t y4 = *reinterpret_cast<const uint32_t*>(A.st.y + i0);
        const uint32_t o4 = *reinterpret_cast<const uint32_t*>(A.st.origin + i0);
        const uint32_t d4 = *reinterpret_cast<const uint32_t*>(A.st.dest + i0);
        const float4 rew = *reinterpret_cast<const float4*>(A.st.reward + i0);
        const double2 f01 = *reinterpret_cast<const double2*>(A.st.fuel + i0);
        const double2 f23 = *reinterpret_cast<const double2*>(A.st.fuel + i0 + 2);
        uint32_t flags4 = 0, cut4 = 0;
        uint4 pos;
        uint32_t* pw = &pos.x;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool raised = byte_at(err4, j) != 0;
            flags4 |= ((byte_at(done4, j) ? kRecDone : 0u) | (raised ? kRecInvalid : 0u)) << (8 * j);
            pw[j] = byte_at(x4, j) | byte_at(y4, j) << 8 | byte_at(o4, j) << 16 | byte_at(d4, j) << 24;
            cut4 |= (uint32_t)raised << (8 * j);
        }
        *reinterpret_cast<float4*>(A.ring.rew + slot) = rew;
        *reinterpret_cast<uint32_t*>(A.ring.flags + slot) = flags4;
        *reinterpret_cast<uint4*>(A.ring.n_pos + slot) = pos;
        *reinterpret_cast<float4*>(A.ring.n_fuel + slot) =
            make_float4((float)f01.x, (float)f01.y, (float)f23.x, (float)f23.y);
        if (!A.cut) continue;
        if (A.max_steps > 0) {
            const uint4 st4 = *reinterpret_cast<const uint4*>(A.st.ep_start + i0);
            const int32_t lx = (int32_t)(A.t - st4.x), ly = (int32_t)(A.t - st4.y);
            const int32_t lz = (int32_t)(A.t - st4.z), lw = (int32_t)(A.t - st4.w);
            cut4 |= (uint32_t)(lx >= A.max_steps) | (uint32_t)(ly >= A.max_steps) << 8 |
                    (uint32_t)(lz >= A.max_steps) << 16 | (uint32_t)(lw >= A.max_steps) << 24;
        }
        *reinterpret_cast<uint32_t*>(A.cut + i0) = cut4;
        if (!A.world || !cut4) continue;
        const LdsWorld w = world_view(A.dims, A.world);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (!byte_at(cut4, j)) continue;
            const int64_t i = i0 + j;  // reset_kernel's body for this env
            const U4 o = draw(env_key(A.seed, A.env_base + i), A.epoch, kSlotExplicitReset);
            Ship sh;
            reset_ship(w, sh, o.v[0], o.v[1]);
            A.st.x[i] = (uint8_t)sh.x;
            A.st.y[i] = (uint8_t)sh.y;
            A.st.fuel[i] = sh.fuel;
            A.st.cargo[i] = sh.cargo;
            A.st.origin[i] = (uint8_t)sh.origin;
            A.st.dest[i] = (uint8_t)sh.dest;
            if (A.st.ep_return) A.st.ep_return[i] = 0.0f;
            if (A.st.ep_start) A.st.ep_start[i] = (int32_t)A.t;
            A.st.done[i] = 0;
            A.st.err[i] = 0;
            A.st.reward[i] = 0.0f;
        }
    }
}

__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {  // lowbias32 finaliser
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// Feistel half width for a domain of D elements: 2h >= ceil(log2 D), h >= 1
__host__ __device__ __forceinline__ uint32_t feistel_half(uint32_t D) {
    uint32_t bits = 2;
    while (bits < 32 && (1ull << bits) < (uint64_t)D) bits += 2;
    return bits / 2;
}

// A keyed permutation of [0, D), D <= 2^31: 4 Feistel rounds on 2h bits,
// cycle-walked back into the domain (p < D terminates: p lies on its own cycle).
__host__ __device__ __forceinline__ uint32_t feistel_perm(uint32_t p, uint32_t D, uint32_t h, const uint32_t* k) {
    const uint32_t m = (1u << h) - 1u;
    do {
        uint32_t L = p >> h, R = p & m;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t f = mix32(R ^ k[r]) & m;
            const uint32_t nl = R;
            R = L ^ f;
            L = nl;
        }
        p = (L << h) | R;
    } while (p >= D);
    return p;
}

struct SampleBatchArgs {
    const uint32_t* world;
    WorldDims dims;
    Ring ring;
    int64_t B;
    int32_t width;
    uint64_t seed;
    const uint32_t* t_dev;  // update counter in device memory (graph replay) or null
    uint32_t t;
    float* obs;
    float* next_obs;
    int64_t* act;
    float* rew;
    float* done;
    float* weight;
};

// one preprocess_state column of a stored ship (utils/preprocessing.py:25-62;
// column 3 is fuel again: _build_state's cargo = fuel, environment.py:206)
__device__ __forceinline__ float ship_col(uint32_t pos, float fuel, int c) {
    const uint32_t b = c < 2 ? (pos >> (8 * c)) & 0xffu : (pos >> (8 * (c - 2))) & 0xffu;
    const float v = b == SE_NONE ? -1.0f : (float)b;
    return c == 2 || c == 3 ? fuel : v;
}


// Minibatch slot j's transition (update()'s random.sample, agents/dqn.py:213-214): the
// keyed permutation's entry j, else j + B, j + 2B, ... while the one found is flagged
// (a raised step), up to kReplayTries; slot -1 when none is found. Shared by the sampler
// and the update kernel that draws its own rows (se_qtrain_step_replay), so both pick
// the same transitions bit for bit.
struct Pick {
    int64_t slot;
    uint32_t sp, np;
    float sf, nf, rw;
    int32_t ac;
    uint8_t fl;
};

__device__ __forceinline__ Pick pick_transition(const Ring& ring, int64_t size, const U4& key, uint32_t h,
                                                int64_t j, int64_t B, int k0 = 0) {
    Pick p{-1, 0u, 0u, 0.0f, 0.0f, 0.0f, 0, 0};
    for (int k = k0; k < kReplayTries; ++k) {
        const int64_t pos = j + (int64_t)k * B;
        if (pos >= size) break;
        const uint32_t l = feistel_perm((uint32_t)pos, (uint32_t)size, h, key.v);
        p.fl = ring.flags[l];
        p.sp = ring.s_pos[l];
        p.sf = ring.s_fuel[l];
        p.np = ring.n_pos[l];
        p.nf = ring.n_fuel[l];
        p.ac = ring.act[l];
        p.rw = ring.rew[l];
        if (!(p.fl & kRecInvalid)) {
            p.slot = l;
            break;
        }
    }
    return p;
}

// pick_transition split in two: the first try's loads issued (no wait, so that loads issued
// after them need not be waited for first), then the result, with the later tries only when
// the first candidate is flagged. Same picks, bit for bit.
struct PickFirst {
    Pick p;
    int64_t l;  // the first candidate's slot, -1 if row j has none (j >= size)
};
__device__ __forceinline__ PickFirst pick_issue(const Ring& ring, int64_t size, const U4& key, uint32_t h, int64_t j) {
    PickFirst f{{-1, 0u, 0u, 0.0f, 0.0f, 0.0f, 0, 0}, -1};
    if (j < size) {
        const uint32_t l = feistel_perm((uint32_t)j, (uint32_t)size, h, key.v);
        f.l = l;
        f.p.fl = ring.flags[l];
        f.p.sp = ring.s_pos[l];
        f.p.sf = ring.s_fuel[l];
        f.p.np = ring.n_pos[l];
        f.p.nf = ring.n_fuel[l];
        f.p.ac = ring.act[l];
        f.p.rw = ring.rew[l];
    }
    return f;
}
__device__ __forceinline__ Pick pick_resolve(const PickFirst& f, const Ring& ring, int64_t size, const U4& key,
                                             uint32_t h, int64_t j, int64_t B) {
    if (f.l < 0) return f.p;  // slot -1
    if (!(f.p.fl & kRecInvalid)) {
        Pick p = f.p;
        p.slot = f.l;
        return p;
    }
    return pick_transition(ring, size, key, h, j, B, 1);  // (a slot -1 pick's fields are not read)
}

// kSampleRows transitions per workgroup. The first wave picks the slots, loading each
// candidate's flags and its transition together (a flagged one is then dropped), and
// writes its row's six ship columns; all threads then write the constant port block from
// a small LDS copy of the port table, which the other threads load while the picks run.
// Three dependent memory steps (size, transition, stores) where staging the whole world
// image, a flags-only probe and a second gather behind a barrier made five.
__global__ __launch_bounds__(kBlock) void replay_sample_kernel(SampleBatchArgs A) {
    __shared__ int64_t slot_of[kSampleRows];
    __shared__ float port[4 * SE_MAX_PORTS];
    const int P = A.dims.P, width = A.width;
    const int64_t r0 = (int64_t)blockIdx.x * kSampleRows;
    {
        const LdsWorld wv = world_view(A.dims, A.world);  // the port table only, in place
        for (int c = (int)threadIdx.x - kSampleRows; c < 4 * P; c += kBlock - kSampleRows) {
            if (c < 0) continue;
            const int p = c >> 2, f = c & 3;
            port[c] = f == 0 ? (float)wv.px(p) : f == 1 ? (float)wv.py(p) : f == 2 ? (float)wv.pfuel(p) : (float)wv.pcargo(p);
        }
    }
    if (threadIdx.x < kSampleRows) {
        const int64_t size = *A.ring.d_size;
        const uint32_t t = A.t_dev ? *A.t_dev : A.t;
        const U4 key = draw(env_key(A.seed, kReplayKeyId), t, kSlotReplay);
        const uint32_t h = feistel_half((uint32_t)size);
        const int64_t j = r0 + threadIdx.x;
        int64_t slot = -1;
        if (j < A.B) {
            const Pick pk = pick_transition(A.ring, size, key, h, j, A.B);
            slot = pk.slot;
            const bool ok = slot >= 0;
            A.act[j] = ok ? (int64_t)pk.ac : 0;
            A.rew[j] = ok ? pk.rw : 0.0f;
            A.done[j] = ok && (pk.fl & kRecDone) ? 1.0f : 0.0f;
            A.weight[j] = ok ? 1.0f : 0.0f;
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                A.obs[j * width + c] = ok ? ship_col(pk.sp, pk.sf, c) : 0.0f;
                A.next_obs[j * width + c] = ok ? ship_col(pk.np, pk.nf, c) : 0.0f;
            }
        }
        slot_of[threadIdx.x] = slot;
    }
    __syncthreads();
    const int64_t rows = min((int64_t)kSampleRows, A.B - r0);
    const int pw = width - 6;
    for (int e = threadIdx.x; e < rows * pw; e += kBlock) {
        const int r = e / pw, c = e - r * pw;
        const float v = slot_of[r] >= 0 ? port[c] : 0.0f;
        A.obs[(r0 + r) * width + 6 + c] = v;
        A.next_obs[(r0 + r) * width + 6 + c] = v;
    }
}

}  // namespace

struct se_replay {
    se_env* env = nullptr;
    int device = 0;
    int64_t cap = 0, head = 0, size = 0;
    bool open = false;  // se_replay_begin called, se_replay_end pending
    void* d_block = nullptr;
    Ring ring{};
};

extern "C" {

int se_replay_create(se_replay** out, se_env* env, int64_t capacity) {
    if (!out) return fail(SE_EINVAL, "null out");
    *out = nullptr;
    int rc = check_ready(env);
    if (rc) return rc;
    if (capacity < env->n || capacity < 1 || capacity >= (int64_t(1) << 31))
        return fail(SE_EINVAL, "replay capacity must be in [max(n, 1), 2^31)");
    DeviceGuard g(env->device);
    const size_t C = (size_t)capacity;
    auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t o_sfuel = up(4 * C), o_act = o_sfuel + up(4 * C), o_rew = o_act + up(4 * C),
                 o_flags = o_rew + up(4 * C), o_npos = o_flags + up(C), o_nfuel = o_npos + up(4 * C),
                 o_size = o_nfuel + up(4 * C), total = o_size + 256;
    se_replay* r = new se_replay;
    r->env = env;
    r->device = env->device;
    r->cap = capacity;
    if (hipMalloc(&r->d_block, total) != hipSuccess) {
        delete r;
        return fail(SE_EHIP, "hipMalloc of the replay ring failed");
    }
    char* b = static_cast<char*>(r->d_block);
    r->ring = Ring{reinterpret_cast<uint32_t*>(b), reinterpret_cast<float*>(b + o_sfuel),
                   reinterpret_cast<int32_t*>(b + o_act), reinterpret_cast<float*>(b + o_rew),
                   reinterpret_cast<uint8_t*>(b + o_flags), reinterpret_cast<uint32_t*>(b + o_npos),
                   reinterpret_cast<float*>(b + o_nfuel), reinterpret_cast<int64_t*>(b + o_size)};
    if (hipMemset(r->d_block, 0, total) != hipSuccess) {
        (void)hipFree(r->d_block);
        delete r;
        return fail(SE_EHIP, "hipMemset of the replay ring failed");
    }
    *out = r;
    return SE_OK;
}

int se_replay_begin(se_replay* r, const int32_t* actions, void* stream) {
    if (!r) return fail(SE_EINVAL, "null replay");
    int rc = check_ready(r->env);
    if (rc) return rc;
    if (!actions) return fail(SE_EINVAL, "null actions");
    if (r->open) return fail(SE_ESTATE, "se_replay_begin twice without se_replay_end");
    se_env* env = r->env;
    DeviceGuard g(env->device);
    RecordArgs A{env->n, r->cap, r->head, 0, env->st, actions, r->ring, nullptr, 0, nullptr, {}, 0, 0, 0, 0};
    if (env->n > 0) {
        replay_begin_kernel<<<grid_for(env->n), kBlock, 0, (hipStream_t)stream>>>(A);
        HIP_TRY(hipGetLastError());
    }
    r->open = true;
    return SE_OK;
}

}  // extern "C"

namespace {
int replay_end(se_replay* r, uint8_t* cut, int32_t max_steps, bool reset_cut, void* stream) {
    if (!r) return fail(SE_EINVAL, "null replay");
    int rc = check_ready(r->env);
    if (rc) return rc;
    if (!r->open) return fail(SE_ESTATE, "se_replay_end without se_replay_begin");
    se_env* env = r->env;
    if (max_steps > 0 && (!cut || !(env->flags & SE_FLAG_AUTO_RESET) || !env->st.ep_start))
        return fail(SE_EINVAL, "max_steps needs a cut buffer and an auto-reset env (ep_start)");
    if (reset_cut && !cut) return fail(SE_EINVAL, "se_replay_end_reset needs a cut buffer");
    if (reset_cut && env->dims.P < 2) return fail(SE_EINVAL, "reset needs at least two ports");
    DeviceGuard g(env->device);
    const int64_t new_size = std::min(r->size + env->n, r->cap);
    RecordArgs A{env->n, r->cap, r->head, new_size, env->st, nullptr, r->ring, cut, max_steps,
                 reset_cut ? env->d_world : nullptr, env->dims, env->seed, env->env_base,
                 (uint32_t)env->epoch, (uint32_t)env->step_t};
    if (env->n % 4 == 0 && r->head % 4 == 0 && r->cap % 4 == 0 && ((uintptr_t)cut & 3u) == 0)
        replay_end4_kernel<<<grid_for(std::max<int64_t>(env->n / 4, 1)), kBlock, 0, (hipStream_t)stream>>>(A);
    else
        replay_end_kernel<<<grid_for(std::max<int64_t>(env->n, 1)), kBlock, 0, (hipStream_t)stream>>>(A);
    HIP_TRY(hipGetLastError());
    if (reset_cut) env->epoch += 1;  // as se_reset
    r->head = (r->head + env->n) % r->cap;
    r->size = new_size;
    r->open = false;
    return SE_OK;
}
}  // namespace

extern "C" {

int se_replay_end(se_replay* r, uint8_t* cut, int32_t max_steps, void* stream) {
    return replay_end(r, cut, max_steps, false, stream);
}

int se_replay_end_reset(se_replay* r, uint8_t* cut, int32_t max_steps, void* stream) {
    return replay_end(r, cut, max_steps, true, stream);
}

int se_step_record(se_replay* r, const int32_t* actions, uint8_t* cut, int32_t max_steps, void* stream) {
    if (!r) return fail(SE_EINVAL, "null replay");
    int rc = check_ready(r->env);
    if (rc) return rc;
    if (!r->open) return fail(SE_ESTATE, "se_step_record without se_replay_begin / se_policy_record");
    if (!cut) return fail(SE_EINVAL, "se_step_record needs a cut buffer");
    se_env* env = r->env;
    if (!(env->flags & SE_FLAG_AUTO_RESET) || !env->st.ep_start)
        return fail(SE_EINVAL, "se_step_record needs an auto-reset env");
    if (env->dims.P < 2) return fail(SE_EINVAL, "reset needs at least two ports");
    if (!actions || !aligned16(actions)) return fail(SE_EINVAL, "actions must be a 16-byte aligned buffer");
    // one launch where every group's ring slots are consecutive; otherwise the two
    // launches it replaces, with the same results
    if (env->n == 0 || env->n % 4 != 0 || r->head % 4 != 0 || r->cap % 4 != 0 || ((uintptr_t)cut & 3u) != 0 ||
        env->iters > kRecMaxIters) {
        rc = se_step(env, actions, stream);
        return rc ? rc : replay_end(r, cut, max_steps, true, stream);
    }
    const int64_t new_size = std::min(r->size + env->n, r->cap);
    const StepRecord rec{r->ring.rew, r->ring.flags, r->ring.n_pos, r->ring.n_fuel, r->ring.d_size,
                         r->head, r->cap, new_size, cut, max_steps, (uint32_t)env->epoch};
    rc = launch_step(env, false, false, actions, nullptr, nullptr, nullptr, stream, &rec);
    if (rc) return rc;
    env->epoch += 1;  // as se_reset
    r->head = (r->head + env->n) % r->cap;
    r->size = new_size;
    r->open = false;
    return SE_OK;
}

int se_policy_record(se_qnet* qn, se_replay* r, int32_t* actions, double epsilon, uint32_t t, void* stream) {
    if (!qn || !r) return fail(SE_EINVAL, "null qnet / replay");
    if (qn->env != r->env) return fail(SE_EINVAL, "the qnet and the replay belong to different envs");
    if (r->open) return fail(SE_ESTATE, "se_replay_begin twice without se_replay_end");
    const PolicyRecord rec{r->ring.s_pos, r->ring.s_fuel, r->ring.act, r->head, r->cap};
    const int rc = launch_policy(qn, actions, epsilon, t, nullptr, 0, &rec, stream);
    if (rc) return rc;
    r->open = true;
    return SE_OK;
}

int se_policy_record_f32(se_qnet* qn, se_replay* r, int32_t* actions, double epsilon, uint32_t t, void* stream) {
    if (!qn || !r) return fail(SE_EINVAL, "null qnet / replay");
    if (qn->env != r->env) return fail(SE_EINVAL, "the qnet and the replay belong to different envs");
    if (r->open) return fail(SE_ESTATE, "se_replay_begin twice without se_replay_end");
    const PolicyRecord rec{r->ring.s_pos, r->ring.s_fuel, r->ring.act, r->head, r->cap};
    const int rc = launch_policy_f32(qn, actions, epsilon, t, nullptr, 0, &rec, stream);
    if (rc) return rc;
    r->open = true;
    return SE_OK;
}

int se_replay_size(se_replay* r, int64_t* size, int64_t* capacity) {
    if (!r) return fail(SE_EINVAL, "null replay");
    if (size) *size = r->size;
    if (capacity) *capacity = r->cap;
    return SE_OK;
}

int se_replay_sample(se_replay* r, int64_t batch, const uint32_t* t_dev, uint32_t t, float* obs,
                     float* next_obs, int64_t* actions, float* rewards, float* dones, float* weights,
                     void* stream) {
    if (!r) return fail(SE_EINVAL, "null replay");
    int rc = check_ready(r->env);
    if (rc) return rc;
    if (batch < 1 || batch > (int64_t(1) << 24)) return fail(SE_EINVAL, "batch must be in [1, 2^24]");
    if (!obs || !next_obs || !actions || !rewards || !dones || !weights)
        return fail(SE_EINVAL, "null batch buffer");
    se_env* env = r->env;
    DeviceGuard g(env->device);
    SampleBatchArgs A{env->d_world, env->dims, r->ring, batch, 6 + 4 * env->dims.P, env->seed, t_dev, t,
                      obs, next_obs, actions, rewards, dones, weights};
    const int grid = (int)((batch + kSampleRows - 1) / kSampleRows);
    replay_sample_kernel<<<grid, kBlock, 0, (hipStream_t)stream>>>(A);
    HIP_TRY(hipGetLastError());
    return SE_OK;
}

int se_replay_destroy(se_replay* r) {
    if (!r) return SE_OK;
    if (r->d_block) {  // does not touch the env, which may be gone already
        DeviceGuard g(r->device);
        (void)hipDeviceSynchronize();
        (void)hipFree(r->d_block);
    }
    delete r;
    return SE_OK;
}

}  // extern "C"
