// Host <-> GPU ping-pong latency through memory, for the N = 1 stepper wave (csrc/server.h).
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/linkprobe tools/linkprobe.hip && tools/linkprobe
//
// One wave polls a command word and answers through an answer word, as server_kernel does;
// the host posts N commands one at a time and spins on each answer. Forms (one JSON line each):
//   host:     both words in coherent pinned host memory (hipHostMalloc), the wave polls
//             across the host link (server_kernel's form)
//   devcmd:   the command word in fine-grained device memory written by the CPU through its
//             mapping (hipExtMallocWithFlags(hipDeviceMallocFinegrained)), the answer in host
//             memory: the wave polls its own memory; skipped if the CPU cannot map it
//   block:    host form plus a 256-byte block read and written back per command (the
//             server's copy in / copy out)
// Every kernel ends on a quit command or after 50 ms without one.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            return 1;                                                             \
        }                                                                         \
    } while (0)

constexpr uint32_t kQuit = 0xffffffffu;

__global__ void pong(uint32_t* cmd, uint32_t* ans, uint32_t* block, int words) {
    const int lane = threadIdx.x;
    uint32_t last = 0;
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const uint32_t c = __hip_atomic_load(cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (c != last) {
            if (words) {
                uint32_t v = lane < words ? __hip_atomic_load(block + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
                if (lane < words) __hip_atomic_store(block + lane, v + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            if (lane == 0) __hip_atomic_store(ans, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            last = c;
            if (c == kQuit) break;
            t0 = __builtin_amdgcn_s_memrealtime();
        } else if (__builtin_amdgcn_s_memrealtime() - t0 > 5000000) {
            break;
        }
    }
}

static int run(const char* name, uint32_t* cmd, uint32_t* cmd_dev, uint32_t* ans, uint32_t* block, int words,
               int iters) {
    __atomic_store_n(cmd, 0u, __ATOMIC_RELEASE);
    __atomic_store_n(ans, 0u, __ATOMIC_RELEASE);
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    pong<<<1, 64, 0, s>>>(cmd_dev, ans, block, words);
    CHECK(hipGetLastError());
    double best = 1e9, sum = 0.0;
    int done = 0;
    for (int i = 1; i <= iters; ++i) {
        const auto t = std::chrono::steady_clock::now();
        __atomic_store_n(cmd, (uint32_t)i, __ATOMIC_RELEASE);
        bool ok = false;
        for (long spin = 0; spin < 200000000L; ++spin) {
            if (__atomic_load_n(ans, __ATOMIC_ACQUIRE) == (uint32_t)i) {
                ok = true;
                break;
            }
            __builtin_ia32_pause();
        }
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count();
        if (!ok) {
            fprintf(stderr, "%s: no answer to command %d\n", name, i);
            break;
        }
        if (i > 10) {  // warm
            best = us < best ? us : best;
            sum += us;
            ++done;
        }
    }
    __atomic_store_n(cmd, kQuit, __ATOMIC_RELEASE);
    CHECK(hipStreamSynchronize(s));
    CHECK(hipStreamDestroy(s));
    printf("{\"form\": \"%s\", \"round_trips\": %d, \"us_mean\": %.3f, \"us_min\": %.3f}\n", name, done,
           done ? sum / done : -1.0, best);
    return 0;
}

int main() {
    CHECK(hipSetDevice(0));
    uint32_t* h = nullptr;
    CHECK(hipHostMalloc((void**)&h, 4096, hipHostMallocCoherent | hipHostMallocMapped));
    memset(h, 0, 4096);
    if (run("host", h, h, h + 16, nullptr, 0, 2000)) return 1;
    if (run("block", h, h, h + 16, h + 64, 64, 2000)) return 1;
    uint32_t* d = nullptr;
    if (hipExtMallocWithFlags((void**)&d, 4096, hipDeviceMallocFinegrained) == hipSuccess) {
        hipPointerAttribute_t at{};
        const bool mapped = hipPointerGetAttributes(&at, d) == hipSuccess && at.hostPointer != nullptr;
        printf("{\"form\": \"devcmd\", \"host_pointer\": %s, \"same_va\": %s}\n", mapped ? "true" : "false",
               at.hostPointer == d ? "true" : "false");
        fflush(stdout);
        if (mapped) {
            uint32_t* hc = static_cast<uint32_t*>(at.hostPointer);
            if (run("devcmd", hc, d, h + 16, nullptr, 0, 2000)) return 1;
        }
        CHECK(hipFree(d));
    } else {
        printf("{\"form\": \"devcmd\", \"alloc\": false}\n");
    }
    CHECK(hipHostFree(h));
    return 0;
}
