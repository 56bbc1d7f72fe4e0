// stepbench.cpp — K back-to-back se_step calls driven from C++ (tuning tool): the
// step rate without the Python host path, for one or more library builds.
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -o tools/stepbench tools/stepbench.cpp -ldl
//   tools/stepbench [--n N] [--config 3|4|5|6] [--steps K] [--rows R] [--floor R] lib.so [lib2.so ...]
// (--floor R: R alternating rounds of the product's K launches and K launches of streamfloor, a
// bare kernel on the same buffers and action rows with the step kernel's grid (one group of 4
// envs per thread, 256-thread workgroups) that moves exactly the step's bytes per env: 42 B, 50 B
// with auto-reset (ep_return read and written), plain loads, nontemporal stores; VERDICT r05
// item 6: how far config 4 sits from its streams alone)
// (config 5: 64 ports without auto-reset; 6: the 5 ports with auto-reset)
// (--rows R: step t reads action row t % R, so R small keeps the actions cache-resident)
// Config 3: the bundled map, the reference's 5 default ports; config 4: 64 ports on
// water cells (any fixed set: this tool times, it does not check), auto-reset.
// Prints one JSON line per library: us per step over K launches on a created
// stream, bracketed by hipEvents (no per-launch events).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../include/shipenv.h"

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

struct Api {
    decltype(&se_create) create;
    decltype(&se_bind) bind;
    decltype(&se_reset) reset;
    decltype(&se_gen_actions) gen;
    decltype(&se_step) step;
    decltype(&se_done_layout) layout;
    decltype(&se_destroy) destroy;
    decltype(&se_map_from_jpeg) map;
    decltype(&se_last_error) err;
};

template <typename F>
static void sym(void* h, const char* name, F& f) {
    f = (F)dlsym(h, name);
    if (!f) {
        fprintf(stderr, "missing %s\n", name);
        exit(1);
    }
}

static void* dev(size_t bytes) {
    void* p = nullptr;
    CK(hipMalloc(&p, bytes < 16 ? 16 : bytes));
    CK(hipMemset(p, 0, bytes < 16 ? 16 : bytes));
    return p;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <typename T>
__device__ __forceinline__ void nt_store(T* p, T v) {
    if constexpr (sizeof(T) == 16)
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, v), reinterpret_cast<u32x4*>(p));
    else
        __builtin_nontemporal_store(v, p);
}
// group g = 4 consecutive envs: x / y / origin / dest / done / err as one u32 each, cargo,
// action, reward and ep_return as one 16-byte lane access, fuel as two
template <bool kAuto>
__global__ __launch_bounds__(256) void streamfloor(se_state st, const int32_t* act, int64_t groups) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= groups) return;
    uint32_t* x = reinterpret_cast<uint32_t*>(st.x);
    uint32_t* y = reinterpret_cast<uint32_t*>(st.y);
    uint32_t* o = reinterpret_cast<uint32_t*>(st.origin);
    uint32_t* d = reinterpret_cast<uint32_t*>(st.dest);
    int4* c = reinterpret_cast<int4*>(st.cargo);
    double2* f = reinterpret_cast<double2*>(st.fuel);
    const int4 a = reinterpret_cast<const int4*>(act)[g];
    uint32_t vx = x[g], vy = y[g], vo = o[g], vd = d[g];
    int4 vc = c[g];
    double2 f0 = f[2 * g], f1 = f[2 * g + 1];
    float4 er = kAuto ? reinterpret_cast<float4*>(st.ep_return)[g] : make_float4(0.f, 0.f, 0.f, 0.f);
    vx ^= (uint32_t)a.x & 0x01010101u;
    vy ^= (uint32_t)a.y & 0x01010101u;
    vc.x += a.z;
    f0.x -= 1.0;
    f1.y -= 1.0;
    const float4 r = make_float4((float)a.x, (float)a.y, (float)a.z, (float)a.w);
    nt_store(&x[g], vx);
    nt_store(&y[g], vy);
    nt_store(&o[g], vo);
    nt_store(&d[g], vd);
    nt_store(&c[g], vc);
    nt_store(&f[2 * g], f0);
    nt_store(&f[2 * g + 1], f1);
    nt_store(&reinterpret_cast<float4*>(st.reward)[g], r);
    nt_store(&reinterpret_cast<uint32_t*>(st.done)[g], (uint32_t)a.w & 0x01010101u);
    nt_store(&reinterpret_cast<uint32_t*>(st.err)[g], 0u);
    if (kAuto) {
        er.x += r.x;
        er.y += r.y;
        er.z += r.z;
        er.w += r.w;
        nt_store(&reinterpret_cast<float4*>(st.ep_return)[g], er);
    }
}

int main(int argc, char** argv) {
    int64_t n = 1 << 20;
    int config = 3, steps = 1000, rows = 0, warm = 20;  // rows > 0: cycle through that many action rows
    int preroll = 0;  // untimed steps from reset before the warm-up (the bench's steady state), one row each
    bool gen_late = false;  // generate the timed rows after the warm-up steps (right before timing)
    bool per_launch = false;  // also print every timed launch's own event-pair duration
    int floor_rounds = 0;  // > 0: alternate the product's timed loop with streamfloor's
    std::vector<std::string> libs;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--n")) n = atoll(argv[++i]);
        else if (!strcmp(argv[i], "--config")) config = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--steps")) steps = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--rows")) rows = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--warm")) warm = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--gen-late")) gen_late = true;
        else if (!strcmp(argv[i], "--preroll")) preroll = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--per-launch")) per_launch = true;
        else if (!strcmp(argv[i], "--floor")) floor_rounds = atoi(argv[++i]);
        else libs.push_back(argv[i]);
    }
    FILE* f = fopen("shippingenv_amd/data/mapa_mundi_binario.jpg", "rb");
    if (!f) {
        fprintf(stderr, "run from the repository root\n");
        return 1;
    }
    std::vector<uint8_t> jpg;
    for (int c; (c = fgetc(f)) != EOF;) jpg.push_back((uint8_t)c);
    fclose(f);

    for (const std::string& path : libs) {
        void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            fprintf(stderr, "%s\n", dlerror());
            return 1;
        }
        Api a;
        sym(h, "se_create", a.create);
        sym(h, "se_bind", a.bind);
        sym(h, "se_reset", a.reset);
        sym(h, "se_gen_actions", a.gen);
        sym(h, "se_step", a.step);
        sym(h, "se_done_layout", a.layout);
        sym(h, "se_destroy", a.destroy);
        sym(h, "se_map_from_jpeg", a.map);
        sym(h, "se_last_error", a.err);
#define SE(x)                                                   \
        do {                                                    \
            if ((x) != 0) {                                     \
                fprintf(stderr, "%s: %s\n", #x, a.err());       \
                return 1;                                       \
            }                                                   \
        } while (0)

        std::vector<uint8_t> water(100 * 100);
        SE(a.map(jpg.data(), jpg.size(), 100, 100, water.data()));
        std::vector<int32_t> px, py, pf, pc;
        // config 4: 64 ports + auto-reset; 5: 64 ports, no auto-reset; 6: 5 ports + auto-reset
        const bool p64 = config == 4 || config == 5, aut = config == 4 || config == 6;
        if (p64) {
            for (int c = 0; c < 100 * 100 && (int)px.size() < 64; c += 37)
                if (water[c]) {
                    px.push_back(c / 100);
                    py.push_back(c % 100);
                    pf.push_back(5 + (int)px.size() % 16);
                    pc.push_back(20 - (int)px.size() % 16);
                }
        } else {
            const int d[5][2] = {{41, 40}, {60, 22}, {78, 29}, {49, 72}, {62, 72}};
            for (auto& p : d) {
                px.push_back(p[0]);
                py.push_back(p[1]);
                pf.push_back(12);
                pc.push_back(9);
            }
        }
        se_env* env = nullptr;
        SE(a.create(&env, 0, n, 0, 100, 100, water.data(), (int32_t)px.size(), px.data(), py.data(),
                    pf.data(), pc.data(), 2026, aut ? SE_FLAG_AUTO_RESET : 0));
        se_state st{};
        st.x = (uint8_t*)dev(n);
        st.y = (uint8_t*)dev(n);
        st.origin = (uint8_t*)dev(n);
        st.dest = (uint8_t*)dev(n);
        st.done = (uint8_t*)dev(n);
        st.err = (int8_t*)dev(n);
        st.fuel = (double*)dev(8 * n);
        st.cargo = (int32_t*)dev(4 * n);
        st.reward = (float*)dev(4 * n);
        if (aut) {
            int64_t stride = 0;
            int32_t segs = 0;
            SE(a.layout(env, &stride, &segs));
            st.ep_return = (float*)dev(4 * n);
            st.ep_start = (int32_t*)dev(4 * n);
            st.done_recs = (se_done_rec*)dev(2 * (size_t)segs * stride * sizeof(se_done_rec));
            st.done_count = (int32_t*)dev(2 * (size_t)segs * sizeof(int32_t));
        }
        SE(a.bind(env, &st));
        hipStream_t s;
        CK(hipStreamCreate(&s));
        // rows: warm-up rows first, then the timed ones (as bench.py: W warm-up steps,
        // then K steps on fresh rows)
        const int total = warm + steps;
        int32_t* acts = (int32_t*)dev((size_t)total * n * 4);
        for (int t = 0; t < (gen_late ? warm : total); ++t) SE(a.gen(env, acts + (size_t)t * n, (uint32_t)t, s));
        SE(a.reset(env, nullptr, s));
        if (preroll > 0) {
            int32_t* row = (int32_t*)dev((size_t)n * 4);
            for (int t = 0; t < preroll; ++t) {
                SE(a.gen(env, row, (uint32_t)(1000000 + t), s));
                SE(a.step(env, row, s));
            }
            CK(hipStreamSynchronize(s));
            CK(hipFree(row));
        }
        for (int t = 0; t < warm; ++t) SE(a.step(env, acts + (size_t)t * n, s));
        if (gen_late)
            for (int t = warm; t < total; ++t) SE(a.gen(env, acts + (size_t)t * n, (uint32_t)t, s));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipStreamSynchronize(s));
        std::vector<hipEvent_t> ev(per_launch ? steps + 1 : 0);
        for (auto& e : ev) CK(hipEventCreate(&e));
        CK(hipEventRecord(e0, s));
        const int r = rows > 0 && rows < steps ? rows : steps;
        for (int t = 0; t < steps; ++t) {
            if (per_launch) CK(hipEventRecord(ev[t], s));
            SE(a.step(env, acts + (size_t)(warm + t % r) * n, s));
        }
        if (per_launch) CK(hipEventRecord(ev[steps], s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        if (per_launch) {
            printf("{\"per_launch_us\": [");
            for (int t = 0; t < steps; ++t) {
                float m = 0.f;
                CK(hipEventElapsedTime(&m, ev[t], ev[t + 1]));
                printf("%s%.2f", t ? ", " : "", 1000.0 * m);
            }
            printf("]}\n");
            for (auto& e : ev) CK(hipEventDestroy(e));
        }
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const char* base = strrchr(path.c_str(), '/');
        for (int round = 0; round < floor_rounds; ++round) {  // product, then floor, alternating
            float mp = 0.f, mf = 0.f;
            CK(hipEventRecord(e0, s));
            for (int t = 0; t < steps; ++t) SE(a.step(env, acts + (size_t)(warm + t % r) * n, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&mp, e0, e1));
            const int64_t groups = n / 4;
            const unsigned grid = (unsigned)((groups + 255) / 256);
            CK(hipEventRecord(e0, s));
            for (int t = 0; t < steps; ++t) {
                if (aut) streamfloor<true><<<grid, 256, 0, s>>>(st, acts + (size_t)(warm + t % r) * n, groups);
                else streamfloor<false><<<grid, 256, 0, s>>>(st, acts + (size_t)(warm + t % r) * n, groups);
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&mf, e0, e1));
            printf("{\"lib\": \"%s\", \"n\": %lld, \"config\": %d, \"round\": %d, \"us_per_step\": %.3f, "
                   "\"floor_us_per_launch\": %.3f, \"floor_bytes_per_env\": %d}\n",
                   base ? base + 1 : path.c_str(), (long long)n, config, round, 1000.0 * mp / steps,
                   1000.0 * mf / steps, aut ? 50 : 42);
            fflush(stdout);
        }
        printf("{\"lib\": \"%s\", \"n\": %lld, \"config\": %d, \"steps\": %d, \"action_rows\": %d, "
               "\"warm\": %d, \"preroll\": %d, \"gen_late\": %d, \"step_blocks\": \"%s\", \"us_per_step\": %.3f}\n",
               base ? base + 1 : path.c_str(), (long long)n, config, steps, r, warm, preroll, (int)gen_late,
               getenv("SHIPENV_STEP_BLOCKS") ? getenv("SHIPENV_STEP_BLOCKS") : "default", 1000.0 * ms / steps);
        fflush(stdout);
        SE(a.destroy(env));
        for (void* p : {(void*)st.x, (void*)st.y, (void*)st.origin, (void*)st.dest, (void*)st.done,
                        (void*)st.err, (void*)st.fuel, (void*)st.cargo, (void*)st.reward,
                        (void*)st.ep_return, (void*)st.ep_start, (void*)st.done_recs,
                        (void*)st.done_count, (void*)acts})
            if (p) CK(hipFree(p));
        CK(hipStreamDestroy(s));
    }
    return 0;
}
