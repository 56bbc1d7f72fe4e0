/* shipenv.h — C-ABI of libshipenv_hip.so, the MI355X-native batched ShippingEnv step.
 *
 * The reference has no FFI: its "operator API" is the Python class
 * shipping.Environment (/root/reference/shipping/environment.py:28-376). Each
 * entry point below replaces one method of that class for N environments at
 * once; the Python mirror shippingenv_amd/shipping/environment.py binds them
 * through ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *  - Every function returns 0 on success or a negative SE_E* status; the text of
 *    the last failure on the calling thread is se_last_error().
 *  - All N-sized buffers are DEVICE pointers owned by the caller (e.g. torch
 *    tensors' data_ptr()); the library never frees them. They must be 16-byte
 *    aligned. The library owns only its staged map/ports copies and scratch.
 *  - Launching calls take a hipStream_t as void* (NULL = the null stream), are
 *    asynchronous on it and never synchronise the host.
 *  - Per-environment failures are not API errors: they are reported per env in
 *    err[i] (SE_ERR_*), exactly where the reference raises an exception; such an
 *    env's state is left untouched with reward 0 and done 0.
 *  - n = 0 (an empty batch) is valid: the env's calls then launch nothing and accept
 *    null N-sized buffers; a step still advances the step counter.
 */
#ifndef SHIPENV_H
#define SHIPENV_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SHIPENV_ABI_VERSION 2  /* 2: se_state.ep_start (episode-start stamps) replaces ep_len */

/* API status codes */
#define SE_OK 0
#define SE_EINVAL (-1)  /* bad argument */
#define SE_EHIP (-2)    /* HIP runtime error */
#define SE_ESTATE (-3)  /* call out of order (e.g. step before bind) */

/* Per-environment error classes; the Python mirror re-raises the reference's
 * exception type and message for each (shipping/environment.py line). */
#define SE_ERR_OK 0
#define SE_ERR_OOB 1            /* ValueError("Move is out of range")                       :284 */
#define SE_ERR_SAME_PORT 2      /* Exception("Destination port must be different ...")      :267 */
#define SE_ERR_PORT_RANGE 3     /* IndexError("Port index is out of range")                 :269 */
#define SE_ERR_NOT_AT_PORT 4    /* Exception("Not currently at port")                  :343, :352 */
#define SE_ERR_AMOUNT 5         /* ValueError("Invalid fuel amount")                   :346, :355 */
#define SE_ERR_NO_DEST 6        /* Exception("Cannot move without destination port")        :276 */
#define SE_ERR_BAD_CATEGORY 7   /* ValueError("Action category unknown")                    :374 */
#define SE_ERR_NO_PORTS 8       /* Exception("No ports available")                          :360 */
#define SE_ERR_BAD_INDEX 9      /* IndexError("list index out of range"), utils/preprocessing.py:127 */
#define SE_ERR_NEED_DRAW 10     /* replay only: the step needs a variate the tape lacks (no effect) */

/* se_tape.used bits written by se_step_replay: the reference draws the step consumed */
#define SE_USED_FUEL_GATE 1     /* uniform() for the fuel cost (:104) and the gate random() (:320) */
#define SE_USED_LOSS_TYPE 2     /* random() loss type (:177) */
#define SE_USED_BETA 4          /* betavariate(2, 2) (:195) */
#define SE_USED_ARRIVE 8        /* randint redraw of the destination (:333-335) */
#define SE_USED_MOVED 16        /* not a draw: the ship moved onto a non-ground cell (:296-300),
                                   so fuel became an np.float64 and the reward a float */

/* se_create flags */
#define SE_FLAG_AUTO_RESET 1u   /* reset an env inside se_step right after it reports done */

#define SE_NONE 255             /* origin/dest "None" in the u8 index fields */
#define SE_MAX_PORTS 254
#define SE_MAX_SIDE 256         /* H, W <= 256 (positions are u8) */

typedef struct se_env se_env;

/* Done-list entry written by the auto-reset path (wave-ballot compaction). */
typedef struct se_done_rec {
    int32_t env;         /* local env index */
    float ep_return;     /* return of the finished episode */
    int32_t ep_len;      /* its length in step calls */
    int32_t step;        /* the step counter value of the step that finished it */
} se_done_rec;

/* Per-env SoA state, one entry per environment, all device pointers (16-B aligned).
 * ep_return, ep_start, done_recs and done_count may be NULL unless SE_FLAG_AUTO_RESET.
 * All calls on one env must be ordered on one stream (or externally synchronised):
 * the step kernel updates each wave's statistics-slab entry and the done lists with
 * plain loads and stores, which assumes no other launch on the same env overlaps it. */
typedef struct se_state {
    uint8_t* x;         /* ship_position[0], row of np_game      (environment.py:37,:241,:297) */
    uint8_t* y;         /* ship_position[1], column of np_game */
    double* fuel;       /* self.fuel, f64 like the reference (int 200 - sum of np.float64)  :39 */
    int32_t* cargo;     /* self.cargo                                                      :38 */
    uint8_t* origin;    /* self.origin_port_index, SE_NONE = None                          :40 */
    uint8_t* dest;      /* self.destination_port_index, SE_NONE = None                     :41 */
    float* reward;      /* step() reward, the reference's f64 value rounded once to f32    :376 */
    uint8_t* done;      /* step() done                                                     :376 */
    int8_t* err;        /* SE_ERR_* per env */
    float* ep_return;   /* running episode return (auto-reset) */
    int32_t* ep_start;  /* auto-reset: the step-counter value (mod 2^32) at which the env's
                           current episode began; its running length in step calls is
                           (step counter - ep_start) mod 2^32. A step writes it only for
                           the envs it resets (about 1 in 240 per step), where a running
                           length was read and written for every env on every step.
                           se_reset / se_reset_to stamp the counter's current value; a
                           checkpoint restores it together with se_set_counters. */
    struct se_done_rec* done_recs; /* auto-reset done lists: 2 * segments * seg_stride records
                                      (se_done_layout), double-buffered by step parity */
    int32_t* done_count;           /* auto-reset per-segment counts: 2 * segments entries */
    double* reward64;              /* optional (NULL): the reference's f64 reward, unrounded */
} se_state;

/* One replayed MOVE's variates (the draws the reference made through `random`,
 * SURVEY.md Appendix A); used by se_step_replay only. 48 bytes. A variate the
 * step needs but the record lacks (NaN, or arrive_dest < 0) yields
 * SE_ERR_NEED_DRAW and no state change: a caller holding the reference's RNG
 * draws exactly that next variate and steps again (shipping.Environment does). */
typedef struct se_tape {
    double u_fuel;       /* random() behind uniform(-0.1, 0.1)                  :104 */
    double u_gate;       /* random() of the cargo-loss gate                       :320 */
    double u_type;       /* random() loss type (read only if the gate fires)      :177 */
    double beta;         /* betavariate(2, 2) (read only for a partial loss)      :195 */
    int32_t arrive_dest; /* accepted randint at arrival                          :333 */
    int32_t used;        /* out: SE_USED_* bits of the draws the step consumed */
} se_tape;

/* Environment.__init__ + _initialize_map + add_port (environment.py:29-65).
 * water: H*W bytes row-major [x*W + y], 0 = GROUND, nonzero = not ground (the
 * thresholded map of :45-55). Ports are stamped non-ground like add_port (:65).
 * port_fuel / port_cargo: the stocks add_port drew (:63-64). P may be 0.
 * env_id_base: global id of env 0 (rank * n for sharded runs): the Philox key
 * (seed, env_id_base + i) makes results shard-invariant. */
int se_create(se_env** out, int device, int64_t n, int64_t env_id_base, int32_t H, int32_t W,
              const uint8_t* water, int32_t P, const int32_t* port_x, const int32_t* port_y,
              const int32_t* port_fuel, const int32_t* port_cargo, uint64_t seed, uint32_t flags);

/* Replace the ports table (add_port / remove_port / attribute assignment); host arrays. */
int se_set_ports(se_env* env, int32_t P, const int32_t* port_x, const int32_t* port_y,
                 const int32_t* port_fuel, const int32_t* port_cargo);

/* Bind the caller-owned SoA buffers (n entries each, 16-byte aligned): device memory,
 * or pinned host memory, which ROCm maps into the GPU's address space (the N = 1
 * shipping.Environment binds one pinned 256-byte block and reads results in place). */
int se_bind(se_env* env, const se_state* state);

/* reset() (environment.py:227-243) for every env with mask[i] != 0 (mask NULL = all):
 * cargo 0, fuel 200, origin ~ U{0..P-1}, dest ~ U{others}, ship at the origin port.
 * Draws: Philox(seed, env) at counter (reset epoch, slot 5); the epoch advances per call. */
int se_reset(se_env* env, const uint8_t* mask, void* stream);

/* reset() with given origin/dest per env (device int32 arrays): replays a
 * recorded reset, or restores a state. */
int se_reset_to(se_env* env, const uint8_t* mask, const int32_t* origin, const int32_t* dest,
                void* stream);

/* step() for all envs with actions in the agent-index encoding of
 * utils/preprocessing.py:111-137 (a < 4 move N,E,S,W; < 4+P select; < 4+P+50
 * take cargo; else take fuel). Draws from Philox(seed, env) at counter
 * (step counter, slot); the step counter advances by one per call. */
int se_step(se_env* env, const int32_t* actions, void* stream);

/* `steps` consecutive se_step calls issued from native code: step k takes its actions
 * from actions + k * ld (ld >= n int32 entries, 16-byte aligned rows). The same
 * launches as a host loop over se_step, without the caller's per-step overhead, so a
 * fixed action schedule keeps the GPU queue full (a rollout of a pre-computed policy,
 * the bench's timed region). reward/done/err hold the last step's outputs. The kernel
 * is the same code as se_step's, under a name of its own in a kernel trace (without
 * auto-reset). An extension: the reference steps one call at a time
 * (environment.py:359-376). */
int se_step_seq(se_env* env, const int32_t* actions, int64_t ld, int32_t steps, void* stream);

/* se_step_seq that also records `event` (a hipEvent_t, may be NULL) on the stream right
 * after launch number `mark_after` (0..steps; 0 = before the first launch): a timer mark
 * in the same native call as the launches, with no host round trip between them
 * (tools/diag/wall_forms.py). */
int se_step_seq_mark(se_env* env, const int32_t* actions, int64_t ld, int32_t steps, void* stream,
                     void* event, int32_t mark_after);

/* step() with the reference's typed action [ActionType, value] (environment.py:359-376):
 * type 1..4 (shipping/type.py:1-5); MOVE value = (a, b) any integers; others value = a. */
int se_step_typed(se_env* env, const int32_t* type, const int32_t* a, const int32_t* b,
                  void* stream);

/* step() with typed actions whose variates come from tape[i] (replay of recorded
 * reference draws); writes tape[i].used. The step counter does not advance. */
int se_step_replay(se_env* env, const int32_t* type, const int32_t* a, const int32_t* b,
                   se_tape* tape, void* stream);

/* step() for agent-index actions (the se_step encoding) with the reference's draws from
 * tape[i] instead of Philox: the production step kernel's own code path (the agent path
 * se_step runs) in its replay-tape instantiation, for parity against the reference's
 * records. Writes tape[i].used; a step that needs a variate tape[i] lacks answers
 * SE_ERR_NEED_DRAW with no effect. The step counter does not advance. */
int se_step_agent_replay(se_env* env, const int32_t* actions, se_tape* tape, void* stream);

/* The N = 1 GPU stepper as one resident wave (csrc/server.h): se_step_replay / se_reset_to
 * on a one-env handle without a launch or a stream synchronise per call. The env's state,
 * typed action and tape and the mailbox are one se_server_block in coherent pinned host memory
 * (se_host_alloc, 64-byte aligned); the caller writes a call's inputs there, se_server_call
 * posts the op and returns when the wave has answered, the outputs then in the same block:
 *   SE_SERVER_STEP      se_step_replay (environment.py:359-376): x .. b and tape in, state,
 *                       reward, reward64, done, err and tape.used out
 *   SE_SERVER_RESET_TO  se_reset_to with origin = type, dest = a (:227-243); they must name
 *                       ports (not checked on the device)
 * The wave ends after 20 ms without a call and is launched again by the next one;
 * se_server_destroy ends it (destroy the server before its env). The handle may also be
 * bound (se_bind) to the block's fields for the launch path (se_step_replay). An extension:
 * the reference steps in Python (Environment.step). */
#define SE_SERVER_STEP 1
#define SE_SERVER_RESET_TO 2
typedef struct se_server_block {
    uint8_t x, y, origin, dest, done;  /* 0 (origin / dest SE_NONE = None) */
    int8_t err;
    uint8_t pad0[2];
    double fuel;                       /* 8 */
    int32_t cargo;                     /* 16 */
    float reward;                      /* 20 */
    double reward64;                   /* 24 */
    int32_t type, a, b;                /* 32 */
    uint32_t seq0;                     /* 44: se_server_call: the call's number, line 0's copy */
    se_tape tape;                      /* 48 */
    uint32_t seq1;                     /* 88: the call's number again, stored last */
    uint32_t op;                       /* 92 */
    uint32_t answer;                   /* 96: the wave: the number of the call it answered */
    uint32_t running;                  /* 100: the wave: 0 once it has ended */
    uint8_t pad1[24];
} se_server_block;                     /* 128 bytes: two 64-byte lines */
typedef struct se_server se_server;
int se_host_alloc(size_t bytes, void** out);  /* zeroed, coherent, device-mapped, 64-byte aligned */
int se_host_free(void* p);
int se_server_create(se_server** out, se_env* env, se_server_block* block);
int se_server_call(se_server* s, int32_t op);
int se_server_launches(se_server* s, uint64_t* out);  /* kernel launches so far (idle restarts + 1) */
int se_server_destroy(se_server* s);

/* Host-resident environments (no device, no HIP call): the N = 1 drop-in
 * shipping.Environment steps here by default (shippingenv_amd/shipping/_host.py), with the
 * step kernels' own per-env code compiled for the host (replay_env in shipenv.hip), so a
 * reference step() costs one C call instead of a kernel launch and a stream synchronise.
 * The state buffers are host memory; no alignment is required.
 *   se_host_create / se_host_set_ports   Environment.__init__ + add_port (:29-65)
 *   se_host_step_replay                  step() (:359-376) with the reference's draws from
 *                                        tape[i], exactly as se_step_replay
 *   se_host_reset_to                     reset() (:227-243) to given origin / dest
 */
typedef struct se_host se_host;
int se_host_create(se_host** out, int32_t H, int32_t W, const uint8_t* water, int32_t P,
                   const int32_t* port_x, const int32_t* port_y, const int32_t* port_fuel,
                   const int32_t* port_cargo);
int se_host_set_ports(se_host* h, int32_t P, const int32_t* port_x, const int32_t* port_y,
                      const int32_t* port_fuel, const int32_t* port_cargo);
int se_host_step_replay(se_host* h, int64_t n, const se_state* st, const int32_t* type,
                        const int32_t* a, const int32_t* b, se_tape* tape);
/* se_host_reset_to stamps ep_start = 0 (a host world keeps no step counter): lengths derived
 * from a host world's stamps (counter - ep_start) are meaningless; the host stepper reports
 * lengths through its own step records. */
int se_host_reset_to(se_host* h, int64_t n, const se_state* st, const uint8_t* mask,
                     const int32_t* origin, const int32_t* dest);
int se_host_destroy(se_host* h);

/* utils.preprocessing.preprocess_state rows (:25-62) as f32, row stride ld >= 6+4P:
 * [x, y, fuel, fuel ("cargo" is self.fuel, environment.py:206), origin, dest, (px,py,pfuel,pcargo)*P],
 * None -> -1. */
int se_observe(se_env* env, float* obs, int64_t ld, void* stream);

/* DQN is_valid_action (agents/dqn.py:125-175) for every agent index a < 4+P+250,
 * packed MSB-first per row (numpy.packbits order), row stride ceil((4+P+250)/8) bytes. */
int se_valid_mask(se_env* env, uint8_t* bits, void* stream);

/* Synthetic agent: fills actions[i] from Philox(seed, env) at (t, slot 6) with the
 * bench mix (90% move, 5% take cargo U{1..20}, 3% take fuel U{1..20}, 2% select). */
int se_gen_actions(se_env* env, int32_t* actions, uint32_t t, void* stream);

/* sample_action() (environment.py:245-263), the random policy of MCTS rollouts and
 * SARSA exploration, for every env from its current state, as typed actions (the
 * input of se_step_typed). One draw per env: Philox(seed, env) at (t, slot 11) word 0.
 *   at a port with no destination: SELECT_PORT uniform over the other ports   :247-253
 *   at a port with cargo 0:        TAKE_CARGO U{1..port_cargo} (randint :160)  :255-257
 *   at a port with fuel == 0:      the reference raises TypeError (self.fuel[idx], :163)
 *   otherwise:                     MOVE_SHIP N/E/S/W uniform (random.choice :165-167)
 * Where the reference raises (the fuel branch; randint(1, 0) on an empty port) the
 * type is SE_SAMPLE_RAISES; where it never returns (no other port, :253) it is
 * SE_SAMPLE_NO_OTHER_PORT. */
#define SE_SAMPLE_RAISES (-1)
#define SE_SAMPLE_NO_OTHER_PORT (-2)
int se_sample_actions(se_env* env, int32_t* type, int32_t* a, int32_t* b, uint32_t t, void* stream);

/* MCTS random rollouts (agents/mcts.py:211-238): rollout r starts from a copy of env
 * src[r]'s state (env state is not modified) and repeats sample_action + step until
 * the step reports done, max_steps steps have counted, or max_attempts attempts
 * have run. An attempt whose step raises is retried without counting (the
 * reference's `except Exception: continue`). Outputs (device, m entries):
 * ret[r] = the step rewards summed in f64 in order (total_reward, :226-230);
 * steps[r] = counted steps; status[r] = SE_ROLL_*.
 * Draws: Philox(seed, rollout_base + r) at (attempt, slot 12): sample word, u_fuel,
 * u_gate, u_type; and, for a partial loss or an arrival, (attempt, slot 13): three
 * beta uniforms, the new destination. */
#define SE_ROLL_DONE 0        /* the last counted step reported done */
#define SE_ROLL_MAX_STEPS 1   /* max_steps steps counted */
#define SE_ROLL_RAISED 2      /* sample_action raised; the exception leaves _rollout */
#define SE_ROLL_ATTEMPTS 3    /* max_attempts reached (the reference keeps retrying) */
#define SE_ROLL_BAD_SRC 4     /* src[r] outside [0, n) */
int se_rollout(se_env* env, const int32_t* src, int64_t m, int32_t max_steps, int32_t max_attempts,
               int64_t rollout_base, double* ret, int32_t* steps, int32_t* status, void* stream);

/* DQN policy step fused on the GPU (agents/dqn.py): DQNNetwork 6+4P -> 128 -> 128 -> A
 * (A = 4+P+250, :21-33) evaluated with bf16 MFMA and f32 accumulation on the
 * observation preprocess_state builds (utils/preprocessing.py:25-62; its constant port
 * block is folded into fc1's bias), fused with choose_action (:177-203): the first
 * maximum of Q over is_valid_action (:125-175), and epsilon-greedy exploration
 * (np.random.rand() <= epsilon, then random.choice over the valid actions). The
 * N x A Q matrix never reaches HBM (unless q_out asks for it). */
typedef struct se_qnet se_qnet;
int se_qnet_create(se_qnet** out, se_env* env);
/* Weights: DEVICE f32 arrays in torch nn.Linear layout (weight [out][in], bias [out]):
 * w1 [128][6+4P], b1 [128], w2 [128][128], b2 [128], w3 [A][128], b3 [A]. Packed on the
 * stream (bf16, MFMA fragment order). Call again after se_set_ports (the port block is
 * folded with the ports of that moment; se_policy refuses a stale packing). */
int se_qnet_set_weights(se_qnet* q, const float* w1, const float* b1, const float* w2,
                        const float* b2, const float* w3, const float* b3, void* stream);
/* actions[i]: the agent-index action (se_step input) for every env. Exploration draws
 * Philox(seed, env) at (t, slot 14): word 0 * 2^-32 <= epsilon explores, and word 1
 * picks the k-th valid action (ascending index) uniformly. q_out (optional, NULL):
 * the Q rows as computed, [n][ldq] f32, ldq >= A. */
int se_policy(se_qnet* q, int32_t* actions, double epsilon, uint32_t t, float* q_out, int64_t ldq,
              void* stream);
/* Repack from the device weights of the last se_qnet_set_weights (same tensors, new values:
 * after an optimizer step). bump (optional, device int32): incremented once on the stream
 * (a training loop's update counter, advanced where the new weights take effect). */
/* choose_action as se_policy, with DQNNetwork evaluated in fp32 as agents/dqn.py:198-200
 * runs it (fp32 weights and activations on v_mfma_f32_32x32x2_f32: exact f32 products,
 * f32 accumulation) instead of bf16: the fp32-faithful mode. Packs its image from the
 * weights of the last se_qnet_set_weights (their current values) on every call. */
int se_policy_f32(se_qnet* q, int32_t* actions, double epsilon, uint32_t t, float* q_out, int64_t ldq,
                  void* stream);
int se_qnet_repack(se_qnet* q, int32_t* bump, void* stream);
int se_qnet_destroy(se_qnet* q);  /* destroy a qnet before the env it was created on */

/* DQN experience replay on the device (agents/dqn.py): remember (:117-123) into a ring of
 * `capacity` transitions (deque(maxlen=memory_size)), and update()'s minibatch (:213-224:
 * random.sample, then the preprocess_state rows as f32). A transition is stored compactly
 * (ship bytes, f32 fuel, action, f32 reward, flags) for s and s'; the constant port block
 * of the rows is rebuilt from the world when sampling. capacity in [max(n, 1), 2^31). */
typedef struct se_replay se_replay;
int se_replay_create(se_replay** out, se_env* env, int64_t capacity);
/* Record s and the agent-index actions of every env: call right before se_step. */
int se_replay_begin(se_replay* r, const int32_t* actions, void* stream);
/* Record reward, done and s' after se_step: appends n transitions (FIFO eviction). A
 * step that raised (err != 0) is stored flagged and never sampled: the reference's loop
 * breaks before remember (:304-309). cut (optional, device u8[n]): 1 where the episode must
 * restart, i.e. the step raised or the episode length (step counter - ep_start) >= max_steps (max_steps > 0 needs an auto-reset
 * env, :281); pass it to se_reset. */
int se_replay_end(se_replay* r, uint8_t* cut, int32_t max_steps, void* stream);
/* The training loop's fused forms (one launch each instead of two):
 * se_policy_record = se_policy (q_out NULL) + se_replay_begin with the chosen actions
 * (remember's state and action, agents/dqn.py:117-123 and :285-291);
 * se_replay_end_reset = se_replay_end + se_reset(cut): the cut episodes restart in the
 * same pass, with the draws se_reset would make (the env's reset epoch advances). */
int se_policy_record(se_qnet* q, se_replay* r, int32_t* actions, double epsilon, uint32_t t, void* stream);
/* se_policy_record with the network in fp32 (se_policy_f32's kernel): the same record. */
int se_policy_record_f32(se_qnet* q, se_replay* r, int32_t* actions, double epsilon, uint32_t t, void* stream);
int se_replay_end_reset(se_replay* r, uint8_t* cut, int32_t max_steps, void* stream);
/* se_step_record = se_step + se_replay_end_reset in one launch: the step kernel writes the
 * ring's reward / done / s' record and restarts the cut envs from the state it holds
 * (env.step + remember + env.reset of the training loop, agents/dqn.py:281-309). Needs an
 * auto-reset env; when n, the ring head / capacity are not multiples of 4 or cut is not
 * 4-byte aligned it makes the two launches instead. Results are identical either way. */
int se_step_record(se_replay* r, const int32_t* actions, uint8_t* cut, int32_t max_steps, void* stream);
int se_replay_size(se_replay* r, int64_t* size, int64_t* capacity);
/* A minibatch of `batch` distinct transitions: batch position j takes logical index
 * perm(j) of a 4-round Feistel permutation of [0, size) keyed by Philox(seed, 2^64 - 1) at
 * (t, slot 15), skipping flagged ones through positions j + B, j + 2B, j + 3B (weight 0 if
 * all four are flagged or beyond size). t is read from t_dev (device u32) when non-NULL, so
 * the launch can be captured in a graph with a device-side update counter. Outputs
 * (device): obs and next_obs [batch][6+4P] f32 rows, actions int64, rewards, dones
 * (1.0 / 0.0) and weights (1.0 / 0.0) f32 [batch]. */
int se_replay_sample(se_replay* r, int64_t batch, const uint32_t* t_dev, uint32_t t, float* obs,
                     float* next_obs, int64_t* actions, float* rewards, float* dones, float* weights,
                     void* stream);
int se_replay_destroy(se_replay* r);  /* destroy a replay before the env it was created on */

/* The DQN update (agents/dqn.py:206-245) fused on f32 MFMA: two kernels per update.
 * Target y = r + gamma * max_a target(s')[a] * (1 - done), loss = sum w (q - y)^2 / sum w
 * (nn.MSELoss when every w is 1), backward, and one Adam step (torch.optim.Adam, no weight
 * decay) on the online parameters in place. Deterministic: no atomics, fixed summation
 * orders. Parameters: DEVICE f32 tensors of DQNNetwork (hidden 128, torch nn.Linear layout);
 * adam_m / adam_v: zero-initialised tensors of the same shapes (exp_avg, exp_avg_sq). */
typedef struct se_mlp {
    float* w1; float* b1;  /* fc1 [128][6+4P], [128] */
    float* w2; float* b2;  /* fc2 [128][128], [128] */
    float* w3; float* b3;  /* fc3 [A][128], [A]; A = 4+P+250 */
} se_mlp;
typedef struct se_qtrain se_qtrain;
int se_qtrain_create(se_qtrain** out, se_env* env, int64_t max_batch);  /* 1 <= P <= 64 */
/* Bind the parameter sets and build the kernel's images of both networks (fragment order,
 * fc1's port block folded with the env's ports of this moment). */
int se_qtrain_bind(se_qtrain* q, const se_mlp* online, const se_mlp* target, const se_mlp* adam_m,
                   const se_mlp* adam_v, void* stream);
/* Rebuild the images of one network (0 online, 1 target) after its parameters changed
 * outside se_qtrain_step (e.g. the target-network copy, update_target_model :109-111). */
int se_qtrain_pack(se_qtrain* q, int32_t which, void* stream);
/* One update on a minibatch (se_replay_sample's outputs, batch <= max_batch). step_dev:
 * device int32 holding the number of Adam steps already taken (bias correction uses it
 * + 1; the caller increments it). loss_out: device f32. Capturable in a graph. */
int se_qtrain_step(se_qtrain* q, int64_t batch, const float* obs, const float* next_obs, const int64_t* act,
                   const float* rew, const float* done, const float* weight, float gamma, float lr,
                   float beta1, float beta2, float eps, const int32_t* step_dev, float* loss_out,
                   void* stream);
/* se_qtrain_step, then what se_qnet_repack(qn, step_dev) would do, in the same two launches:
 * the first kernel advances step_dev (the second's bias correction then uses it as is),
 * and the second writes the policy's bf16 images (both layouts) from the parameters it
 * has just updated. qn must be packed (se_qnet_set_weights) from the very tensors bound
 * as `online` in se_qtrain_bind, on the same env. Same bits as the two calls. */
int se_qtrain_step_policy(se_qtrain* q, se_qnet* qn, int64_t batch, const float* obs,
                          const float* next_obs, const int64_t* act, const float* rew,
                          const float* done, const float* weight, float gamma, float lr, float beta1,
                          float beta2, float eps, int32_t* step_dev, float* loss_out, void* stream);
/* se_replay_sample then se_qtrain_step_policy (qn nullable: se_qtrain_step) in two launches
 * instead of three: the first kernel draws its own minibatch rows from r's ring, the very
 * transitions se_replay_sample(r, batch, t_dev = ctr) picks, without writing the batch
 * buffers. ctr: device int32[2], both entries = the updates taken so far; the sampler key is
 * ctr[0], the first kernel sets ctr[1] = ctr[0] + 1 (the bias-correction count) and the
 * second copies it back into ctr[0]. t >= 0: the caller's copy of ctr[0] (and the ring's size
 * as recorded on the host), so the first kernel does not wait on those device words; t < 0
 * reads them on the device (a graph capture, whose replays advance ctr). Same bits as the sampler plus the step with
 * step_dev = ctr (then advanced); r must record the same env as q and not be mid-record. */
int se_qtrain_step_replay(se_qtrain* q, se_qnet* qn, se_replay* r, int64_t batch, float gamma, float lr,
                          float beta1, float beta2, float eps, int32_t* ctr, int64_t t, float* loss_out,
                          void* stream);
/* Data-parallel update (one learner per GPU, the same parameters on every rank): se_qtrain_step
 * split at the exchange. se_qtrain_grad writes this rank's gradient sums (before the division
 * by sum w) and {sum w (q - y)^2, sum w} into grad, a device f32 vector of
 * se_qtrain_grad_size(q) floats, and changes no parameter. After an all-reduce(SUM) of grad
 * over the ranks, se_qtrain_apply takes one Adam step from it: the update on the union of
 * the ranks' minibatches (loss = global sum w d^2 / global sum w). Same bias-correction
 * counter as se_qtrain_step (step_dev + 1; the caller increments it). qn (nullable): also
 * write that policy's bf16 images, as se_qtrain_step_policy does. Both capturable. */
int64_t se_qtrain_grad_size(const se_qtrain* q);
int se_qtrain_grad(se_qtrain* q, int64_t batch, const float* obs, const float* next_obs, const int64_t* act,
                   const float* rew, const float* done, const float* weight, float gamma, float* grad,
                   void* stream);
int se_qtrain_apply(se_qtrain* q, se_qnet* qn, const float* grad, float lr, float beta1, float beta2,
                    float eps, const int32_t* step_dev, float* loss_out, void* stream);
int se_qtrain_destroy(se_qtrain* q);  /* destroy before the env it was created on */

/* Episode statistics accumulated by the auto-reset path since the last clear:
 * out[0] = sum of returns, out[1] = episodes, out[2] = sum of lengths (device
 * double[3]). Deterministic: per-wave partials are summed in a fixed order. */
int se_episode_stats(se_env* env, double* out, void* stream);
int se_clear_stats(se_env* env, void* stream);

/* Done lists (auto-reset). Every wave of the step kernel writes the envs it
 * finished, in env order, into its own segment; no global atomics, so the list is
 * deterministic. se_done_layout gives the segment stride and count the done_recs /
 * done_count buffers must be sized for (2 * segments * seg_stride records,
 * 2 * segments counts). se_done_list gives where the most recent step wrote
 * (record offset of its buffer, offset of its counts); that list stays intact
 * while the following step runs. Only the first done_count[s] records of segment s
 * are valid: records past the count may be stale, or filler records (env == -1,
 * step == the step counter) that pad a segment's records to whole 128-byte lines
 * (above 2^23 envs, or SHIPENV_DONE_PAD=1 at se_create). se_done_compact copies the
 * valid records contiguously (out: up to n records, out_count: 1 int) on the stream. */
int se_done_layout(se_env* env, int64_t* seg_stride, int32_t* segments);
int se_done_list(se_env* env, int64_t* rec_offset, int64_t* count_offset);
int se_done_compact(se_env* env, se_done_rec* out, int32_t* out_count, void* stream);

/* Step counter / reset epoch (checkpoint-resume; shard replay). */
int se_get_counters(se_env* env, uint64_t* step, uint64_t* epoch);
int se_set_counters(se_env* env, uint64_t step, uint64_t epoch);

int se_destroy(se_env* env);
/* ---- Map loader (host only, no GPU): Environment._initialize_map
 * (shipping/environment.py:45-55) without OpenCV. csrc/mapload.cpp. */

/* The luma (Y) plane of a JPEG as cv2.imread(IMREAD_GRAYSCALE) returns it:
 * baseline / extended / progressive Huffman, 8-bit, 1 or 3 components,
 * libjpeg's accurate integer IDCT. *height / *width are always set on success;
 * `out` (row-major, height*width bytes, may be NULL to query the size) is
 * written when cap is large enough. SE_EINVAL on a corrupt or unsupported file. */
int se_map_decode_luma(const uint8_t* data, size_t len, uint8_t* out, size_t cap,
                       int32_t* height, int32_t* width);
/* gray[row0:row1, col0:col1] -> cv2.resize((W, H), INTER_AREA) (generic,
 * downscaling) -> resized (H*W, may be NULL) and mask = resized > threshold (may be NULL). */
int se_map_area_threshold(const uint8_t* gray, int32_t height, int32_t width, int32_t row0,
                          int32_t row1, int32_t col0, int32_t col1, int32_t H, int32_t W,
                          uint8_t threshold, uint8_t* resized, uint8_t* mask);
/* The whole of _initialize_map: decode, crop rows 50:200 / cols 100:300, INTER_AREA
 * to W x H, > 128. water[x * W + y] = 1 for a non-GROUND cell (x = row, :65). */
int se_map_from_jpeg(const uint8_t* data, size_t len, int32_t H, int32_t W, uint8_t* water);

const char* se_last_error(void);
int se_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
