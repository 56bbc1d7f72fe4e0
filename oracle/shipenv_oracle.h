/* shipenv_oracle.h — CPU restatement of the reference step/reset (TEST INFRASTRUCTURE).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker. The product (shippingenv_amd/) never
 * links or calls it.
 *
 * Scalar, one env at a time, int32 fields, following the reference function by
 * function (citations are /root/reference/shipping/environment.py:LINE unless
 * stated). Two draw sources:
 *   - replay : variates recorded from the reference's own `random` calls
 *              (tests/golden/make_golden.py) -> pinned bit-exact to the reference;
 *   - philox : the production RNG contract shared with the HIP kernel
 *              (DESIGN.md "RNG contract").
 */
#ifndef SHIPENV_ORACLE_H
#define SHIPENV_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int32_t H, W, P;
    const uint8_t* nonground; /* H*W, row-major [x*W + y], 1 = not GROUND after ports stamped */
    const int32_t* port_x;
    const int32_t* port_y;
    const int32_t* port_fuel;
    const int32_t* port_cargo;
} orc_world;

/* One recorded MOVE's variates (Appendix A of SURVEY.md): u_fuel is the random()
 * behind uniform(-0.1, 0.1); NaN where a draw did not happen. */
typedef struct {
    double u_fuel, u_gate, u_type, beta;
    int32_t arrive_dest; /* accepted randint at arrival, -1 if none */
    int32_t pad;
} orc_tape;

/* Batched step over n independent envs (SoA, int32 positions / indices, -1 = None).
 * act_mode 0: agent-index encoding (utils/preprocessing.py:111-137) in act_a;
 * act_mode 1: typed [ActionType, value] with MOVE = (act_a, act_b).
 * tape != NULL -> replay draws; else Philox(seed, env_id_base + i, t).
 * reward is the reference's Python value (f64). Returns 0. */
int orc_step_batch(const orc_world* w, int64_t n, int act_mode, const int32_t* act_type,
                   const int32_t* act_a, const int32_t* act_b, const orc_tape* tape, uint64_t seed,
                   int64_t env_id_base, uint32_t t, int32_t* x, int32_t* y, double* fuel,
                   int32_t* cargo, int32_t* origin, int32_t* dest, double* reward, int32_t* done,
                   int32_t* err);

/* utils/preprocessing.py:111-137 for n agent indices: typed (type, a, b), err 9 where
 * the reference raises IndexError (index < -4). */
int orc_decode_agent(int32_t P, int64_t n, const int32_t* act, int32_t* type, int32_t* a, int32_t* b,
                     int32_t* err);

/* Auto-reset variant (config 4): after a step whose done==1 the env is reset with
 * Philox slot RESET of the same t; ep_return (f32 sum of f32 rewards) and ep_len
 * are accumulated, finished episodes are summed into stats[3] = {sum_return,
 * n_episodes, sum_len} in env order. */
int orc_step_batch_autoreset(const orc_world* w, int64_t n, const int32_t* actions, uint64_t seed,
                             int64_t env_id_base, uint32_t t, int32_t* x, int32_t* y, double* fuel,
                             int32_t* cargo, int32_t* origin, int32_t* dest, float* ep_return,
                             int32_t* ep_len, double* reward, int32_t* done, int32_t* err,
                             double* stats);

/* reset (environment.py:227-243) of env i where mask==NULL or mask[i]!=0.
 * origin_in/dest_in != NULL -> explicit values (replay); else Philox with
 * counter (env, epoch, SLOT_EXPLICIT_RESET). */
int orc_reset_batch(const orc_world* w, int64_t n, const uint8_t* mask, const int32_t* origin_in,
                    const int32_t* dest_in, uint64_t seed, int64_t env_id_base, uint32_t epoch,
                    int32_t* x, int32_t* y, double* fuel, int32_t* cargo, int32_t* origin,
                    int32_t* dest);

/* preprocess_state row (utils/preprocessing.py:25-62) as f32, ld = 6 + 4P. */
int orc_observe(const orc_world* w, int64_t n, const int32_t* x, const int32_t* y,
                const double* fuel, const int32_t* origin, const int32_t* dest, float* obs);

/* DQN is_valid_action (agents/dqn.py:125-175) for every agent index a < A=4+P+250;
 * bits row-major [i][a], packed MSB-first like numpy.packbits, row stride ceil(A/8). */
int orc_valid_mask(const orc_world* w, int64_t n, const int32_t* x, const int32_t* y,
                   const int32_t* origin, uint8_t* bits);

/* Philox4x32-10 block, for known-answer tests. */
/* sample_action (environment.py:245-263) per env from Philox(seed, env) at (t, slot
 * 11) word 0; type < 0 where the reference raises (-1) or never returns (-2). */
int orc_sample_actions(const orc_world* w, int64_t n, const int32_t* x, const int32_t* y,
                       const double* fuel, const int32_t* cargo, const int32_t* origin,
                       const int32_t* dest, uint64_t seed, int64_t env_id_base, uint32_t t,
                       int32_t* type, int32_t* a, int32_t* b);

/* MCTS random rollouts (agents/mcts.py:211-238) from copies of envs src[r]; draws
 * Philox(seed, rollout_base + r) at (attempt, slots 12 and 13). */
int orc_rollout(const orc_world* w, int64_t n, const int32_t* x, const int32_t* y,
                const double* fuel, const int32_t* cargo, const int32_t* origin,
                const int32_t* dest, int64_t m, const int32_t* src, int32_t max_steps,
                int32_t max_attempts, uint64_t seed, int64_t rollout_base, double* ret,
                int32_t* steps, int32_t* status);

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* synthetic action stream used by the bench (config 3/4 mix), oracle side. */
int orc_gen_actions(int64_t n, int32_t P, uint64_t seed, int64_t env_id_base, uint32_t t,
                    int32_t* actions);

/* update()'s minibatch indices (agents/dqn.py:213) under the build's sampler contract
 * (include/shipenv.h se_replay_sample): slot[j] in [0, size) or -1. */
uint32_t orc_feistel_perm(uint32_t p, uint32_t D, const uint32_t key[4]);
int orc_replay_pick(int64_t size, int64_t batch, const uint8_t* invalid, uint64_t seed, uint32_t t,
                    int64_t* slot);

#ifdef __cplusplus
}
#endif
#endif
