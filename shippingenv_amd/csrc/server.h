// server.h — the N = 1 drop-in's GPU stepper as one persistent wave (VERDICT r05
// item 8).
//
// Part of shipenv.hip's translation unit (included at its end). Reference callers: the agents
// step one env at a time, once per decision (agents/dqn.py:287) and ~500 times per MCTS
// decision (agents/mcts.py:228-236), each step() a few bytes in and out
// (environment.py:359-376). As a kernel launch plus a stream synchronise per step that is
// ~24 us, so the GPU stepper was 2.4x slower than the reference Python.
//
// Here one wave stays resident and steps on command: the host writes the step's inputs into a
// block of coherent pinned host memory (se_host_alloc), then the command word; the wave sees it
// with a system-scope load, copies the block into LDS (one coalesced load of the wave), runs
// replay_env, the per-env core of se_step_replay and se_host_step_replay (or se_reset_to's
// explicit reset), on that copy with the world image staged in LDS once per launch, copies the
// block back (one coalesced store) and answers with a system-scope store that the host spins on.
// No launch, no synchronise, no copy call.
//
// Mailbox (4 u32, 16-byte aligned, in the same pinned memory):
//   [0] command sequence   host: incremented per command (stored after [1] and the block)
//   [1] op                 host: SE_SERVER_STEP / SE_SERVER_RESET_TO / quit
//   [2] answered sequence  device: the command it finished (stored after the block)
//   [3] running            host: 1 at launch; device: 0 when the kernel ends
// The wave ends after kServerIdleTicks without a command (and on quit, se_server_destroy), so
// no kernel outlives an idle or crashed host by more than that; the next se_server_call
// launches it again, and a command that raced the exit is answered by the new kernel (it
// starts from [2] and runs any command past it). Every access to the mailbox and the block is
// a vector memory instruction (global loads / stores with sc0 sc1), which the ISA of
// server_kernel shows.

#include <chrono>

namespace {

constexpr uint64_t kServerIdleTicks = 2000000;  // s_memrealtime ticks (100 MHz): 20 ms
constexpr uint32_t kServerQuit = 0xffffffffu;

// byte offsets in the block of each buffer the step touches (-1: absent)
struct ServerLayout {
    int32_t x, y, fuel, cargo, origin, dest, reward, done, err, ep_return, ep_start, reward64, type, a, b, tape;
};

struct ServerArgs {
    const uint32_t* world;
    WorldDims dims;
    int32_t n;
    uint32_t step_t;  // se_reset_to's episode-start stamp (ep_start, if bound)
    ServerLayout at;
    uint32_t* mbox;
    uint32_t* block;  // the caller's pinned block (state, actions, tape)
    int32_t words;    // block size in u32 (<= 64 * kServerWordsPerLane)
};
constexpr int kServerWordsPerLane = 4;

template <typename T>
__device__ __forceinline__ T& lds_at(uint8_t* blk, int32_t off, int i) {
    return reinterpret_cast<T*>(blk + off)[i];
}

__global__ __launch_bounds__(64) void server_kernel(ServerArgs S) {
    // LDS: the world image (staged once per launch), then a copy of the block. The block
    // crosses the host link twice per command, as one coalesced load and one coalesced store
    // of the whole wave; lane 0 steps the envs in LDS with replay_env, the per-env core of
    // se_step_replay (and of se_host_step_replay), so no step access is a memory round trip.
    extern __shared__ uint32_t lds[];
    const LdsWorld w = stage_world(S.world, S.dims, lds);
    uint32_t* blk32 = lds + S.dims.padded();
    uint8_t* blk = reinterpret_cast<uint8_t*>(blk32);
    const ServerLayout& L = S.at;
    const int lane = threadIdx.x;
    uint32_t* mb = S.mbox;
    uint32_t last = __hip_atomic_load(mb + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    // No acquire / release fences: at system scope they invalidate and write back the L2
    // (buffer_inv / buffer_wbl2 sc0 sc1) on every poll. The host-side words are read and
    // written with system-scope relaxed accesses instead (sc0 sc1: to memory, past the
    // caches), issued after the poll that saw the command returned; the host stored the block
    // before the command word (x86 keeps its stores in order), and the answer is stored after
    // the block's stores have completed.
    for (;;) {
        const uint32_t c = __hip_atomic_load(mb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (c != last) {
            const uint32_t op = __hip_atomic_load(mb + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            uint32_t v[kServerWordsPerLane];
#pragma unroll
            for (int k = 0; k < kServerWordsPerLane; ++k) {
                const int i = k * 64 + lane;
                v[k] = i < S.words ? __hip_atomic_load(S.block + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
            }
#pragma unroll
            for (int k = 0; k < kServerWordsPerLane; ++k) {
                const int i = k * 64 + lane;
                if (i < S.words) blk32[i] = v[k];
            }
            __syncthreads();
            if (lane == 0) {
                for (int i = 0; i < S.n; ++i) {
                    if (op == SE_SERVER_STEP) {  // se_host_step_replay's loop body, on LDS
                        Ship sh{lds_at<uint8_t>(blk, L.x, i), lds_at<uint8_t>(blk, L.y, i), lds_at<double>(blk, L.fuel, i),
                                lds_at<int32_t>(blk, L.cargo, i), lds_at<uint8_t>(blk, L.origin, i),
                                lds_at<uint8_t>(blk, L.dest, i)};
                        Pending p;
                        se_tape& tp = lds_at<se_tape>(blk, L.tape, i);
                        tp.used = (int32_t)replay_env(w, sh, p, SE_ERR_OK, lds_at<int32_t>(blk, L.type, i),
                                                      lds_at<int32_t>(blk, L.a, i), lds_at<int32_t>(blk, L.b, i),
                                                      tp.u_fuel, tp.u_gate, &tp);
                        lds_at<uint8_t>(blk, L.x, i) = (uint8_t)sh.x;
                        lds_at<uint8_t>(blk, L.y, i) = (uint8_t)sh.y;
                        lds_at<double>(blk, L.fuel, i) = sh.fuel;
                        lds_at<int32_t>(blk, L.cargo, i) = sh.cargo;
                        lds_at<uint8_t>(blk, L.origin, i) = (uint8_t)sh.origin;
                        lds_at<uint8_t>(blk, L.dest, i) = (uint8_t)sh.dest;
                        lds_at<float>(blk, L.reward, i) = (float)p.r;  // one rounding of the f64 reward
                        lds_at<uint8_t>(blk, L.done, i) = (uint8_t)p.dead;
                        lds_at<int8_t>(blk, L.err, i) = (int8_t)p.e;
                        if (L.reward64 >= 0) lds_at<double>(blk, L.reward64, i) = p.r;
                    } else if (op == SE_SERVER_RESET_TO) {  // reset_kernel's explicit form
                        const int o = lds_at<int32_t>(blk, L.type, i), d = lds_at<int32_t>(blk, L.a, i);
                        if ((unsigned)o >= (unsigned)w.P || (unsigned)d >= (unsigned)w.P) continue;  // checked by the caller
                        lds_at<uint8_t>(blk, L.x, i) = (uint8_t)w.px(o);
                        lds_at<uint8_t>(blk, L.y, i) = (uint8_t)w.py(o);
                        lds_at<double>(blk, L.fuel, i) = kFuelInit;
                        lds_at<int32_t>(blk, L.cargo, i) = 0;
                        lds_at<uint8_t>(blk, L.origin, i) = (uint8_t)o;
                        lds_at<uint8_t>(blk, L.dest, i) = (uint8_t)d;
                        if (L.ep_return >= 0) lds_at<float>(blk, L.ep_return, i) = 0.0f;
                        if (L.ep_start >= 0) lds_at<int32_t>(blk, L.ep_start, i) = (int32_t)S.step_t;
                        lds_at<uint8_t>(blk, L.done, i) = 0;
                        lds_at<int8_t>(blk, L.err, i) = 0;
                        lds_at<float>(blk, L.reward, i) = 0.0f;
                    }
                }
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kServerWordsPerLane; ++k) {
                const int i = k * 64 + lane;
                if (i < S.words) __hip_atomic_store(S.block + i, blk32[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the block's stores have completed
            if (lane == 0) __hip_atomic_store(mb + 2, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            last = c;
            if (op == kServerQuit) break;
            t0 = __builtin_amdgcn_s_memrealtime();
        } else if (__builtin_amdgcn_s_memrealtime() - t0 > kServerIdleTicks) {
            break;
        } else {
            __builtin_amdgcn_s_sleep(1);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(mb + 3, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

struct se_server {
    se_env* env = nullptr;  // must outlive the server (destroy the server first)
    int device = 0;
    hipStream_t stream = nullptr;
    ServerArgs args{};
    uint32_t* mbox = nullptr;
    uint32_t seq = 0;
    bool launched = false;
    uint64_t launches = 0;
};

namespace {

uint32_t host_load(const uint32_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
void host_store(uint32_t* p, uint32_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }

// (re)launch the wave once the previous one has ended
int server_launch(se_server* s) {
    if (s->launched) HIP_TRY(hipStreamSynchronize(s->stream));  // returns once it has ended
    static std::atomic<uint64_t> lds_set{0};
    int rc = allow_dynamic_lds(lds_set, reinterpret_cast<const void*>(server_kernel), 160 * 1024, s->device);
    if (rc) return rc;
    host_store(s->mbox + 3, 1u);
    server_kernel<<<1, 64, lds_bytes(s->env) + (size_t)s->args.words * 4, s->stream>>>(s->args);
    HIP_TRY(hipGetLastError());
    s->launched = true;
    s->launches += 1;
    return SE_OK;
}

bool host_pinned(const void* p) {
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) return false;
    return at.type == hipMemoryTypeHost;
}

// post op and wait for its answer, relaunching the wave if it ended without answering
int server_post(se_server* s, uint32_t op, double timeout_s) {
    uint32_t* mb = s->mbox;
    if (!s->launched || host_load(mb + 3) == 0u) {
        int rc = server_launch(s);
        if (rc) return rc;
    }
    const uint32_t seq = ++s->seq;
    host_store(mb + 1, op);
    host_store(mb, seq);
    const auto t_start = std::chrono::steady_clock::now();
    for (uint64_t spin = 0;; ++spin) {
        if (host_load(mb + 2) == seq) return SE_OK;
        if (host_load(mb + 3) == 0u) {  // the wave ended (idle) as the command arrived
            if (op == kServerQuit) return SE_OK;
            HIP_TRY(hipStreamSynchronize(s->stream));
            if (host_load(mb + 2) == seq) return SE_OK;
            int rc = server_launch(s);  // the new wave answers the pending command
            if (rc) return rc;
        }
        if ((spin & 1023u) == 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count() > timeout_s)
            return fail(SE_ESTATE, "the stepper wave did not answer");
        __builtin_ia32_pause();
    }
}

}  // namespace

extern "C" {

int se_host_alloc(size_t bytes, void** out) {
    if (!out) return fail(SE_EINVAL, "null out");
    *out = nullptr;
    if (bytes == 0) return fail(SE_EINVAL, "zero bytes");
    void* p = nullptr;
    HIP_TRY(hipHostMalloc(&p, bytes, hipHostMallocCoherent | hipHostMallocMapped));
    memset(p, 0, bytes);
    *out = p;
    return SE_OK;
}

int se_host_free(void* p) {
    if (p) HIP_TRY(hipHostFree(p));
    return SE_OK;
}

int se_server_create(se_server** out, se_env* env, void* block, int64_t block_bytes, const int32_t* type,
                     const int32_t* a, const int32_t* b, se_tape* tape, uint32_t* mbox) {
    if (!out) return fail(SE_EINVAL, "null out");
    *out = nullptr;
    int rc = check_ready(env);
    if (rc) return rc;
    if (env->n < 1 || env->n > 3) return fail(SE_EINVAL, "the stepper wave steps 1 to 3 envs");
    if (env->flags & SE_FLAG_AUTO_RESET) return fail(SE_EINVAL, "the stepper wave replays tapes (no auto-reset)");
    if (!block || !type || !a || !b || !tape || !mbox) return fail(SE_EINVAL, "null block / action / tape / mailbox pointer");
    if (!aligned16(block) || !aligned16(type) || !aligned16(a) || !aligned16(b) || !aligned16(mbox))
        return fail(SE_EINVAL, "the block, the action buffers and the mailbox must be 16-byte aligned");
    if (block_bytes <= 0 || (block_bytes & 3) || block_bytes > 64 * kServerWordsPerLane * 4)
        return fail(SE_EINVAL, "block_bytes must be a multiple of 4 in (0, 1024]");
    if (!host_pinned(block) || !host_pinned(mbox))
        return fail(SE_EINVAL, "the block and the mailbox must be pinned host memory (se_host_alloc)");
    // every buffer the step touches lies in the block; the mailbox does not
    uint8_t* const lo = static_cast<uint8_t*>(block);
    uint8_t* const hi = lo + block_bytes;
    auto inside = [&](const void* p, int64_t bytes) {
        const uint8_t* q = static_cast<const uint8_t*>(p);
        return q >= lo && q + bytes <= hi;
    };
    const se_state& st = env->st;
    const int64_t n = env->n;
    if (!inside(st.x, n) || !inside(st.y, n) || !inside(st.fuel, 8 * n) || !inside(st.cargo, 4 * n) ||
        !inside(st.origin, n) || !inside(st.dest, n) || !inside(st.reward, 4 * n) || !inside(st.done, n) ||
        !inside(st.err, n) || (st.ep_return && !inside(st.ep_return, 4 * n)) ||
        (st.ep_start && !inside(st.ep_start, 4 * n)) || (st.reward64 && !inside(st.reward64, 8 * n)) ||
        !inside(type, 4 * n) || !inside(a, 4 * n) || !inside(b, 4 * n) || !inside(tape, (int64_t)sizeof(se_tape) * n))
        return fail(SE_EINVAL, "the bound state, the actions and the tape must lie in the block");
    if (static_cast<uint8_t*>(static_cast<void*>(mbox)) + 16 > lo && static_cast<uint8_t*>(static_cast<void*>(mbox)) < hi)
        return fail(SE_EINVAL, "the mailbox must lie outside the block");
    auto mis = [&](const void* p, int align) { return p && ((static_cast<const uint8_t*>(p) - lo) & (align - 1)); };
    if (mis(st.fuel, 8) || mis(st.reward64, 8) || mis(tape, 8) || mis(st.cargo, 4) || mis(st.reward, 4) ||
        mis(st.ep_return, 4) || mis(st.ep_start, 4))
        return fail(SE_EINVAL, "the block's f64 buffers and the tape must be 8-byte aligned, the 32-bit ones 4-byte aligned");
    if (lds_bytes(env) + (size_t)block_bytes > 160 * 1024) return fail(SE_EINVAL, "world image + block exceed the LDS");
    DeviceGuard g(env->device);
    se_server* s = new se_server;
    s->env = env;
    s->device = env->device;
    auto off = [&](const void* p) { return p ? (int32_t)(static_cast<const uint8_t*>(p) - lo) : (int32_t)-1; };
    ServerLayout& L = s->args.at;
    L.x = off(st.x);
    L.y = off(st.y);
    L.fuel = off(st.fuel);
    L.cargo = off(st.cargo);
    L.origin = off(st.origin);
    L.dest = off(st.dest);
    L.reward = off(st.reward);
    L.done = off(st.done);
    L.err = off(st.err);
    L.ep_return = off(st.ep_return);
    L.ep_start = off(st.ep_start);
    L.reward64 = off(st.reward64);
    L.type = off(type);
    L.a = off(a);
    L.b = off(b);
    L.tape = off(tape);
    s->args.world = env->d_world;
    s->args.dims = env->dims;
    s->args.n = (int32_t)env->n;
    s->args.step_t = (uint32_t)env->step_t;
    s->args.mbox = mbox;
    s->args.block = static_cast<uint32_t*>(block);
    s->args.words = (int32_t)(block_bytes / 4);
    s->mbox = mbox;
    for (int i = 0; i < 4; ++i) host_store(mbox + i, 0u);
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
        delete s;
        return fail(SE_EHIP, "hipStreamCreateWithFlags failed");
    }
    *out = s;
    return SE_OK;
}

int se_server_call(se_server* s, int32_t op) {
    if (!s) return fail(SE_EINVAL, "null server");
    if (op != SE_SERVER_STEP && op != SE_SERVER_RESET_TO) return fail(SE_EINVAL, "op must be SE_SERVER_STEP or SE_SERVER_RESET_TO");
    DeviceGuard g(s->device);
    return server_post(s, (uint32_t)op, 5.0);
}

int se_server_launches(se_server* s, uint64_t* out) {
    if (!s || !out) return fail(SE_EINVAL, "null server / out");
    *out = s->launches;
    return SE_OK;
}

int se_server_destroy(se_server* s) {
    if (!s) return SE_OK;
    int rc = SE_OK;
    {
        DeviceGuard g(s->device);
        if (s->launched) {
            if (host_load(s->mbox + 3) != 0u) rc = server_post(s, kServerQuit, 1.0);
            if (hipStreamSynchronize(s->stream) != hipSuccess && rc == SE_OK) rc = fail(SE_EHIP, "hipStreamSynchronize failed");
        }
        if (s->stream) (void)hipStreamDestroy(s->stream);
    }
    delete s;
    return rc;
}

}  // extern "C"
