// server.h — the N = 1 drop-in's GPU stepper as one persistent wave (VERDICT r05
// item 8).
//
// Part of shipenv.hip's translation unit (included at its end). Reference callers: the agents
// step one env at a time, once per decision (agents/dqn.py:287) and ~500 times per MCTS
// decision (agents/mcts.py:228-236), each step() a few bytes in and out
// (environment.py:359-376). As a kernel launch plus a stream synchronise per step that is
// ~22 us, so the GPU stepper was 2.4x slower than the reference Python.
//
// Here one wave stays resident and steps on command. The env's state, its typed action, its
// tape and the mailbox are one se_server_block (include/shipenv.h): two 64-byte lines of
// coherent pinned host memory. The host writes a call's inputs, then the call's sequence
// number into a word of each line (line 0's first, x86 keeps its stores in order). The wave
// polls the whole block with one coalesced load; a host-link read returns each 64-byte line
// as one snapshot, so when both lines carry the new sequence the inputs in them are complete,
// and the poll that sees the command has already brought them. Lane 0 runs replay_env, the
// per-env core of se_step_replay and se_host_step_replay (or se_reset_to's explicit reset), on
// a copy in LDS with the world image staged in LDS once per launch; the wave stores the
// state part back (one coalesced store), waits for the stores, and answers with the sequence.
// No launch, no synchronise, no copy call: two host-link transfers per step.
//
// The wave ends after kServerIdleTicks without a command (and on quit, se_server_destroy), so
// no kernel outlives an idle or crashed host by more than that; `running` then reads 0 and the
// next se_server_call launches it again (a command that raced the exit is answered by the new
// wave: it starts from `answer` and runs any command past it). Every access to the block is a
// vector memory instruction (global loads / stores with sc0 sc1: to memory, past the caches,
// no acquire / release fences, which at system scope would invalidate and write back the L2 on
// every poll); the ISA of server_kernel shows it.

#include <chrono>
#include <cstddef>

namespace {

constexpr uint64_t kServerIdleTicks = 2000000;  // s_memrealtime ticks (100 MHz): 20 ms
constexpr uint32_t kServerQuit = 0xffffffffu;

constexpr int kBlockWords = (int)(sizeof(se_server_block) / 4);  // 32: lanes 0-31 move one word each
constexpr int kStateWords = (int)(offsetof(se_server_block, seq1) / 4);  // 22: the words the wave writes back
constexpr int kSeq0 = (int)(offsetof(se_server_block, seq0) / 4), kSeq1 = (int)(offsetof(se_server_block, seq1) / 4);
constexpr int kOp = (int)(offsetof(se_server_block, op) / 4);
static_assert(sizeof(se_server_block) == 128 && offsetof(se_server_block, seq0) < 64 &&
                  offsetof(se_server_block, seq1) >= 64 && offsetof(se_server_block, tape) % 8 == 0,
              "se_server_block: two 64-byte lines, one sequence word in each");

struct ServerArgs {
    const uint32_t* world;
    WorldDims dims;
    uint32_t step_t;  // not read: the block has no episode-start stamp
    se_server_block* blk;
};

__global__ __launch_bounds__(64) void server_kernel(ServerArgs S) {
    extern __shared__ uint32_t lds[];
    const LdsWorld w = stage_world(S.world, S.dims, lds);  // once per launch
    uint32_t* l32 = lds + S.dims.padded();  // the block's copy
    se_server_block& B = *reinterpret_cast<se_server_block*>(l32);
    uint32_t* const h32 = reinterpret_cast<uint32_t*>(S.blk);
    const int lane = threadIdx.x;
    uint32_t last = __hip_atomic_load(&S.blk->answer, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const uint32_t v = lane < kBlockWords ? __hip_atomic_load(h32 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
        const uint32_t s0 = __builtin_amdgcn_readlane(v, kSeq0), s1 = __builtin_amdgcn_readlane(v, kSeq1);
        if (s0 == s1 && s1 != last) {  // both lines of the new command
            const uint32_t op = __builtin_amdgcn_readlane(v, kOp);
            if (lane < kBlockWords) l32[lane] = v;
            __syncthreads();
            if (lane == 0) {
                if (op == SE_SERVER_STEP) {  // se_host_step_replay's loop body, on LDS
                    Ship sh{B.x, B.y, B.fuel, B.cargo, B.origin, B.dest};
                    Pending p;
                    B.tape.used = (int32_t)replay_env(w, sh, p, SE_ERR_OK, B.type, B.a, B.b, B.tape.u_fuel,
                                                      B.tape.u_gate, &B.tape);
                    B.x = (uint8_t)sh.x;
                    B.y = (uint8_t)sh.y;
                    B.fuel = sh.fuel;
                    B.cargo = sh.cargo;
                    B.origin = (uint8_t)sh.origin;
                    B.dest = (uint8_t)sh.dest;
                    B.reward = (float)p.r;  // one rounding of the reference's f64 reward
                    B.reward64 = p.r;
                    B.done = (uint8_t)p.dead;
                    B.err = (int8_t)p.e;
                } else if (op == SE_SERVER_RESET_TO) {  // reset_kernel's explicit form
                    const int o = B.type, d = B.a;
                    if ((unsigned)o < (unsigned)w.P && (unsigned)d < (unsigned)w.P) {  // checked by the caller
                        B.x = (uint8_t)w.px(o);
                        B.y = (uint8_t)w.py(o);
                        B.fuel = kFuelInit;
                        B.cargo = 0;
                        B.origin = (uint8_t)o;
                        B.dest = (uint8_t)d;
                        B.done = 0;
                        B.err = 0;
                        B.reward = 0.0f;
                    }
                }
            }
            __syncthreads();
            if (lane < kStateWords) __hip_atomic_store(h32 + lane, l32[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the state's stores have completed
            if (lane == 0) __hip_atomic_store(&S.blk->answer, s1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            last = s1;
            if (op == kServerQuit) break;
            t0 = __builtin_amdgcn_s_memrealtime();
        } else if (__builtin_amdgcn_s_memrealtime() - t0 > kServerIdleTicks) {
            break;
        } else {
            __builtin_amdgcn_s_sleep(1);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(&S.blk->running, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

struct se_server {
    se_env* env = nullptr;  // must outlive the server (destroy the server first)
    int device = 0;
    hipStream_t stream = nullptr;
    ServerArgs args{};
    se_server_block* blk = nullptr;
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
    host_store(&s->blk->running, 1u);
    server_kernel<<<1, 64, lds_bytes(s->env) + sizeof(se_server_block), s->stream>>>(s->args);
    HIP_TRY(hipGetLastError());
    s->launched = true;
    s->launches += 1;
    return SE_OK;
}

bool host_pinned(const void* p) {
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory: clear the error, or the next launch check reports it
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

// post op and wait for its answer, relaunching the wave if it ended without answering
int server_post(se_server* s, uint32_t op, double timeout_s) {
    se_server_block* B = s->blk;
    if (!s->launched || host_load(&B->running) == 0u) {
        int rc = server_launch(s);
        if (rc) return rc;
    }
    const uint32_t seq = ++s->seq;
    host_store(&B->op, op);
    host_store(&B->seq0, seq);  // line 0 complete
    host_store(&B->seq1, seq);  // line 1 complete: the command
    const auto t_start = std::chrono::steady_clock::now();
    for (uint64_t spin = 0;; ++spin) {
        if (host_load(&B->answer) == seq) return SE_OK;
        if (host_load(&B->running) == 0u) {  // the wave ended (idle) as the command arrived
            if (op == kServerQuit) return SE_OK;
            HIP_TRY(hipStreamSynchronize(s->stream));
            if (host_load(&B->answer) == seq) return SE_OK;
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

int se_server_create(se_server** out, se_env* env, se_server_block* blk) {
    if (!out) return fail(SE_EINVAL, "null out");
    *out = nullptr;
    if (!env) return fail(SE_EINVAL, "null env");
    if (env->n != 1) return fail(SE_EINVAL, "the stepper wave steps a one-env handle");
    if (!blk) return fail(SE_EINVAL, "null block");
    if (reinterpret_cast<uintptr_t>(blk) & 63) return fail(SE_EINVAL, "the block must be 64-byte aligned");
    if (!host_pinned(blk)) return fail(SE_EINVAL, "the block must be pinned host memory (se_host_alloc)");
    if (lds_bytes(env) + sizeof(se_server_block) > 160 * 1024) return fail(SE_EINVAL, "the world image exceeds the LDS");
    DeviceGuard g(env->device);
    se_server* s = new se_server;
    s->env = env;
    s->device = env->device;
    s->blk = blk;
    s->args = ServerArgs{env->d_world, env->dims, (uint32_t)env->step_t, blk};
    host_store(&blk->seq0, 0u);
    host_store(&blk->seq1, 0u);
    host_store(&blk->answer, 0u);
    host_store(&blk->running, 0u);
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
            if (host_load(&s->blk->running) != 0u) rc = server_post(s, kServerQuit, 1.0);
            if (hipStreamSynchronize(s->stream) != hipSuccess && rc == SE_OK) rc = fail(SE_EHIP, "hipStreamSynchronize failed");
        }
        if (s->stream) (void)hipStreamDestroy(s->stream);
    }
    delete s;
    return rc;
}

}  // extern "C"
