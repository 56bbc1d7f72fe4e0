/* shipenv_oracle.c — CPU restatement of the reference hot path (TEST INFRASTRUCTURE).
 *
 * Header: shipenv_oracle.h. Built by oracle/Makefile with -O2 -ffp-contract=off
 * (the reference's arithmetic is unfused IEEE f64: CPython floats and np.sqrt).
 *
 * Parity: pinned. The replay mode reproduces every record of
 * tests/golden/{tape,states}_seed*.npz (generated from the reference itself by
 * tests/golden/make_golden.py) bit for bit; tests/test_oracle_golden.py checks it.
 * The Philox mode is the production RNG contract, which the HIP
 * kernel must match bit for bit; its distributional equivalence to the
 * reference's MT19937 draws is argued in DESIGN.md.
 */
#include "shipenv_oracle.h"

#include <math.h>
#include <stddef.h>
#include <string.h>

/* ------------------------------------------------------------------ constants */
/* shipping/environment.py:8-26 */
#define INITIAL_FUEL 200
#define MAX_CARGO_CAPACITY 50
#define R_CARGO_DELIVER 2
#define R_REACH_DESTINATION 10
#define R_CLOSER 2
#define R_TAKE 0.05
#define P_OUT_OF_FUEL (-10)
#define P_GROUND (-5)
#define P_WATER (-1)
#define P_CARGO_LOSS (-3)
#define P_FARTHER (-2)
#define P_USE_FUEL (-0.0001)

/* shipping/type.py:1-5 */
enum { MOVE_SHIP = 1, SELECT_PORT = 2, TAKE_FUEL = 3, TAKE_CARGO = 4 };

/* error classes (include/shipenv.h SE_ERR_*) */
enum {
    E_OK = 0, E_OOB = 1, E_SAME_PORT = 2, E_PORT_RANGE = 3, E_NOT_AT_PORT = 4, E_AMOUNT = 5,
    E_NO_DEST = 6, E_BAD_CATEGORY = 7, E_NO_PORTS = 8, E_BAD_INDEX = 9, E_NEED_DRAW = 10
};
/* tape.used bits (include/shipenv.h SE_USED_*) */
enum { U_FUEL_GATE = 1, U_LOSS_TYPE = 2, U_BETA = 4, U_ARRIVE = 8 };

/* Philox counter slots (DESIGN.md "RNG contract", v5). Step draws are keyed by the
 * quad k = env / 4 at counter (k, t, slot): quad blocks give word j to env 4k+j
 * (FUEL, GATE, ARRIVE, RESET, RESET_DEST); a LOSS_r block (slots 1, 2, 8, 9 for
 * r = 0..3) belongs whole to the r-th env of the quad, in env order, whose gate
 * fired with cargo > 0: word 0 the loss type, words 1-3 the Beta(2, 2) uniforms.
 * The explicit reset and the synthetic agent draw one block per env. */
enum { SLOT_FUEL = 0, SLOT_LOSS0 = 1, SLOT_LOSS1 = 2, SLOT_ARRIVE = 3, SLOT_RESET0 = 4,
       SLOT_EXPLICIT_RESET = 5, SLOT_ACTION = 6, SLOT_GATE = 7, SLOT_LOSS2 = 8, SLOT_LOSS3 = 9,
       SLOT_RESET1 = 10, SLOT_SAMPLE = 11, SLOT_ROLLOUT = 12, SLOT_ROLLOUT_B = 13,
       SLOT_REPLAY = 15, SLOT_RESET2 = 16, SLOT_RESET3 = 17 };
static const uint32_t LOSS_SLOT[4] = {SLOT_LOSS0, SLOT_LOSS1, SLOT_LOSS2, SLOT_LOSS3};
/* RESET_r (slots 4, 10, 16, 17): the r-th env of the quad auto-reset in step t takes
 * the whole block: word 0 the origin, word 1 the destination */
static const uint32_t RESET_SLOT[4] = {SLOT_RESET0, SLOT_RESET1, SLOT_RESET2, SLOT_RESET3};

/* sample_action results where the reference raises / never returns (include/shipenv.h) */
enum { SAMPLE_RAISES = -1, SAMPLE_NO_OTHER_PORT = -2 };
enum { ROLL_DONE = 0, ROLL_MAX_STEPS = 1, ROLL_RAISED = 2, ROLL_ATTEMPTS = 3, ROLL_BAD_SRC = 4 };

/* ------------------------------------------------------------------ Philox4x32-10 */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static void draw4(uint64_t seed, int64_t env, uint32_t t, uint32_t slot, uint32_t out[4]) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {(uint32_t)(uint64_t)env, (uint32_t)((uint64_t)env >> 32), t, slot};
    orc_philox4x32_10(ctr, key, out);
}

static int32_t uniform_int(uint32_t r, int32_t m) { return (int32_t)(((uint64_t)r * (uint32_t)m) >> 32); }

/* a port index uniform over the P-1 ports other than `other` */
static int32_t pick_other(uint32_t r, int32_t P, int32_t other) {
    int32_t k = uniform_int(r, P - 1);
    return k + (k >= other);
}

static double med3(double a, double b, double c) {
    double lo = a < b ? a : b, hi = a < b ? b : a;
    return c < lo ? lo : (c > hi ? hi : c);
}

/* ------------------------------------------------------------------ draw source */
typedef struct {
    const orc_tape* tape; /* replay if non-NULL */
    uint64_t seed;
    int64_t env;
    uint32_t t;
    int32_t used;         /* U_* bits of the draws consumed */
    int need;             /* replay: a consumed draw is missing from the tape */
    const uint32_t* roll; /* rollout attempt t of rollout `env`: block A words (sample,
                             u_fuel, u_gate, u_type); block B (slot ROLLOUT_B) on demand */
    int32_t loss_rank;    /* Philox step: firing envs of this quad before this one */
    int32_t loss_drawn;   /* out: this env took a LOSS_r block */
} source;

/* rollout block B word k (three beta uniforms, the arrival redraw) */
static uint32_t roll_b(const source* s, int k) {
    uint32_t o[4];
    draw4(s->seed, s->env, s->t, SLOT_ROLLOUT_B, o);
    return o[k];
}

/* Philox: env e takes word e & 3 of the block at counter (e >> 2, t, slot) as a
 * 32-bit value; uniforms are u = w * 2^-32. */
static double u32(uint32_t w) { return (double)w * (1.0 / 4294967296.0); }

static uint32_t quad_word(uint64_t seed, int64_t env, uint32_t t, uint32_t slot) {
    uint32_t o[4];
    draw4(seed, (int64_t)((uint64_t)env >> 2), t, slot, o);
    return o[env & 3];
}

/* u_fuel and u_gate: environment.py:104 (uniform) and :320 (random), always both */
static void src_move(source* s, double* u_fuel, double* u_gate) {
    s->used |= U_FUEL_GATE;
    if (s->tape) {
        *u_fuel = s->tape->u_fuel;
        *u_gate = s->tape->u_gate;
        s->need |= isnan(*u_fuel) || isnan(*u_gate);
        return;
    }
    if (s->roll) {
        *u_fuel = u32(s->roll[1]);
        *u_gate = u32(s->roll[2]);
        return;
    }
    *u_fuel = u32(quad_word(s->seed, s->env, s->t, SLOT_FUEL));
    *u_gate = u32(quad_word(s->seed, s->env, s->t, SLOT_GATE));
}

/* Philox step: the env's LOSS_r block (r = its rank among the quad's firing envs) */
static void loss_block(source* s, uint32_t o[4]) {
    draw4(s->seed, (int64_t)((uint64_t)s->env >> 2), s->t, LOSS_SLOT[s->loss_rank & 3], o);
    s->loss_drawn = 1;
}

static double src_loss_type(source* s) { /* environment.py:177 */
    s->used |= U_LOSS_TYPE;
    if (s->tape) {
        s->need |= isnan(s->tape->u_type);
        return s->tape->u_type;
    }
    if (s->roll) return u32(s->roll[3]);
    uint32_t o[4];
    loss_block(s, o);
    return u32(o[0]);
}

/* environment.py:195, betavariate(2, 2): the median of three uniforms has the
 * Beta(2, 2) law exactly */
static double src_beta(source* s) {
    s->used |= U_BETA;
    if (s->tape) {
        s->need |= isnan(s->tape->beta);
        return s->tape->beta;
    }
    if (s->roll) return med3(u32(roll_b(s, 0)), u32(roll_b(s, 1)), u32(roll_b(s, 2)));
    uint32_t o[4]; /* the same LOSS_r block as the loss type */
    draw4(s->seed, (int64_t)((uint64_t)s->env >> 2), s->t, LOSS_SLOT[s->loss_rank & 3], o);
    return med3(u32(o[1]), u32(o[2]), u32(o[3]));
}

static int32_t src_arrive(source* s, int32_t P, int32_t origin) { /* :333-335 */
    s->used |= U_ARRIVE;
    if (s->tape) {
        s->need |= s->tape->arrive_dest < 0;
        return s->tape->arrive_dest;
    }
    if (s->roll) return pick_other(roll_b(s, 3), P, origin);
    return pick_other(quad_word(s->seed, s->env, s->t, SLOT_ARRIVE), P, origin);
}

/* ------------------------------------------------------------------ one env */
typedef struct {
    int32_t x, y;
    double fuel;
    int32_t cargo, origin, dest;
} ship;

static int ground_at(const orc_world* w, int32_t x, int32_t y) {
    return w->nonground[(size_t)x * w->W + y] == 0; /* np_game[x, y] == Entity.GROUND, :293 */
}

/* _is_within_map, :77-101 (x against size[0], y against size[1]) */
static int within(const orc_world* w, int64_t x, int64_t y) {
    return 0 <= x && x < w->H && 0 <= y && y < w->W;
}

/* _get_current_port_idx, :145-153: first port equal to the ship position */
static int32_t current_port(const orc_world* w, const ship* s) {
    for (int32_t i = 0; i < w->P; ++i)
        if (w->port_x[i] == s->x && w->port_y[i] == s->y) return i;
    return -1;
}

/* _move_ship, :273-339 */
static int move_ship(const orc_world* w, ship* s, int64_t mx, int64_t my, source* src,
                     double* reward, int32_t* done) {
    if (s->dest < 0) return E_NO_DEST; /* :276 */
    double r = 0.0;
    int32_t d = 0;
    int64_t nx = s->x + mx, ny = s->y + my; /* :280-282 */
    if (!within(w, nx, ny)) return E_OOB; /* :284, no draw consumed */

    double u_fuel, u_gate;
    src_move(src, &u_fuel, &u_gate);
    /* _calculate_fuel_cost :103-104 -> util.calculate_euclidean_distance (util.py:3-4):
     * np.sqrt of the integer sum of squares, times (1 + uniform(-0.1, 0.1)) */
    double dist = sqrt((double)(mx * mx + my * my));
    double uni = -0.1 + 0.2 * u_fuel; /* CPython uniform: a + (b - a) * random() */
    double cost = dist * (1.0 + uni);
    if (s->fuel < cost) { /* :288-290 */
        r += P_OUT_OF_FUEL;
        d = 1;
    }
    int32_t ox = s->x, oy = s->y;
    if (ground_at(w, (int32_t)nx, (int32_t)ny)) { /* :293-294 */
        r += P_GROUND;
    } else { /* :296-300, the ship moves even when it just ran out of fuel */
        src->used |= 16; /* SE_USED_MOVED: fuel becomes an np.float64, the reward a float */
        s->x = (int32_t)nx;
        s->y = (int32_t)ny;
        s->fuel -= cost;
        r += P_USE_FUEL;
        r += P_WATER;
    }
    /* :307-315: distance of the old and the ATTEMPTED cell to the destination */
    int32_t px = w->port_x[s->dest], py = w->port_y[s->dest];
    double prev = sqrt((double)((int64_t)(ox - px) * (ox - px) + (int64_t)(oy - py) * (oy - py)));
    double next = sqrt((double)((nx - px) * (nx - px) + (ny - py) * (ny - py)));
    if (prev - next > 0) r += R_CLOSER;
    else r += P_FARTHER;
    /* :318-323: loss gate normalize(cargo, 50, 0) = cargo / 50 (util.py:6-8) */
    double likelihood = (double)s->cargo / (double)MAX_CARGO_CAPACITY;
    const int production = !src->tape && !src->roll;
    if (u_gate <= likelihood && !(production && s->cargo == 0)) {
        /* _calculate_cargo_loss :169-200: the loss-type draw happens first, always
         * (production skips cargo 0, which loses nothing whatever the draw) */
        double lt = src_loss_type(src);
        int32_t loss;
        if (s->cargo == 0) loss = 0;
        else if (lt < 0.1) loss = 0;
        else if (lt > 0.9) loss = s->cargo;
        else loss = (int32_t)(src_beta(src) * (double)s->cargo); /* int() truncation */
        s->cargo -= loss;
        r += (double)(loss * P_CARGO_LOSS);
    }
    /* :325-337 arrival (also while blocked, if the ship already sits on dest) */
    if (s->x == w->port_x[s->dest] && s->y == w->port_y[s->dest]) {
        int32_t drop = s->cargo;
        s->cargo = 0;
        r += (double)(drop * R_CARGO_DELIVER);
        s->origin = s->dest;
        s->dest = src_arrive(src, w->P, s->origin);
        r += R_REACH_DESTINATION;
    }
    *reward = r;
    *done = d;
    return E_OK;
}

/* step, :359-376, with the typed action [category, value] */
static int step_typed(const orc_world* w, ship* s, int32_t type, int32_t a, int32_t b,
                      source* src, double* reward, int32_t* done) {
    *reward = 0.0;
    *done = 0;
    if (w->P == 0) return E_NO_PORTS; /* :360 */
    switch (type) {
    case SELECT_PORT: /* _select_port :265-271 */
        if (!(0 <= a && a < w->P)) return E_PORT_RANGE;
        if (s->origin == a) return E_SAME_PORT;
        s->dest = a;
        return E_OK;
    case TAKE_CARGO: { /* _take_cargo :341-348 */
        int32_t idx = current_port(w, s);
        if (idx < 0) return E_NOT_AT_PORT;
        if (!(0 < a && a <= w->port_cargo[idx])) return E_AMOUNT;
        s->cargo += a;
        *reward = R_TAKE;
        return E_OK;
    }
    case TAKE_FUEL: { /* _take_fuel :350-357 */
        int32_t idx = current_port(w, s);
        if (idx < 0) return E_NOT_AT_PORT;
        if (!(0 < a && a <= w->port_fuel[idx])) return E_AMOUNT;
        s->fuel += (double)a;
        *reward = R_TAKE;
        return E_OK;
    }
    case MOVE_SHIP: {
        int e = move_ship(w, s, a, b, src, reward, done);
        return (e == E_OK && src->need) ? E_NEED_DRAW : e;
    }
    default:
        return E_BAD_CATEGORY; /* :373-374 */
    }
}

/* utils/preprocessing.py:111-137 map_action_to_env_action (Python list indexing:
 * moves[-4..-1] wrap, anything below raises IndexError) */
static int decode_agent(int32_t P, int32_t act, int32_t* type, int32_t* a, int32_t* b) {
    static const int32_t mx[4] = {0, -1, 0, 1}; /* N, E, S, W (:126, shipping/type.py:8-16) */
    static const int32_t my[4] = {-1, 0, 1, 0};
    if (act < 4) {
        if (act < -4) return E_BAD_INDEX;
        int32_t k = act < 0 ? act + 4 : act;
        *type = MOVE_SHIP;
        *a = mx[k];
        *b = my[k];
    } else if (act < 4 + P) {
        *type = SELECT_PORT;
        *a = act - 4;
    } else if (act < 4 + P + MAX_CARGO_CAPACITY) {
        *type = TAKE_CARGO;
        *a = act - (4 + P);
    } else {
        *type = TAKE_FUEL;
        *a = act - (4 + P + MAX_CARGO_CAPACITY);
    }
    return E_OK;
}

/* decode_agent for n indices (tests pin it to the reference's own outputs,
 * tests/golden/decode_golden.json); err[i] = E_BAD_INDEX where the reference raises */
int orc_decode_agent(int32_t P, int64_t n, const int32_t* act, int32_t* type, int32_t* a, int32_t* b,
                     int32_t* err) {
    for (int64_t i = 0; i < n; ++i) {
        type[i] = a[i] = b[i] = 0;
        err[i] = decode_agent(P, act[i], &type[i], &a[i], &b[i]);
    }
    return 0;
}

static void load(ship* s, int64_t i, const int32_t* x, const int32_t* y, const double* fuel,
                 const int32_t* cargo, const int32_t* origin, const int32_t* dest) {
    s->x = x[i]; s->y = y[i]; s->fuel = fuel[i];
    s->cargo = cargo[i]; s->origin = origin[i]; s->dest = dest[i];
}

static void store(const ship* s, int64_t i, int32_t* x, int32_t* y, double* fuel, int32_t* cargo,
                  int32_t* origin, int32_t* dest) {
    x[i] = s->x; y[i] = s->y; fuel[i] = s->fuel;
    cargo[i] = s->cargo; origin[i] = s->origin; dest[i] = s->dest;
}

int orc_step_batch(const orc_world* w, int64_t n, int act_mode, const int32_t* act_type,
                   const int32_t* act_a, const int32_t* act_b, const orc_tape* tape, uint64_t seed,
                   int64_t env_id_base, uint32_t t, int32_t* x, int32_t* y, double* fuel,
                   int32_t* cargo, int32_t* origin, int32_t* dest, double* reward, int32_t* done,
                   int32_t* err) {
    int64_t quad = -1;
    int32_t fired = 0; /* envs of the current quad that took a LOSS_r block */
    for (int64_t i = 0; i < n; ++i) {
        ship s;
        load(&s, i, x, y, fuel, cargo, origin, dest);
        const int64_t e_id = env_id_base + i;
        if ((e_id >> 2) != quad) {
            quad = e_id >> 2;
            fired = 0;
        }
        source src = {tape ? tape + i : NULL, seed, e_id, t, 0, 0, NULL, fired, 0};
        int32_t ty = 0, a = 0, b = 0;
        int e;
        double r = 0.0;
        int32_t d = 0;
        if (act_mode == 0) {
            /* the decode runs before env.step (agents/dqn.py:286-287), so its
             * IndexError wins over "No ports available" */
            e = decode_agent(w->P, act_a[i], &ty, &a, &b);
        } else {
            ty = act_type[i]; a = act_a[i]; b = act_b[i];
            e = E_OK;
        }
        if (e == E_OK) {
            ship t2 = s;
            e = step_typed(w, &t2, ty, a, b, &src, &r, &d);
            if (e == E_OK) s = t2; /* an exception leaves the state as it was */
        }
        if (e != E_OK) {
            r = 0.0;
            d = 0;
        }
        fired += src.loss_drawn;
        if (tape) ((orc_tape*)tape)[i].pad = e == E_NEED_DRAW ? src.used : (e == E_OK ? src.used : 0);
        store(&s, i, x, y, fuel, cargo, origin, dest);
        reward[i] = r;
        done[i] = d;
        err[i] = e;
    }
    return 0;
}

/* reset :227-243 from an origin word and a destination word */
static void reset_words(const orc_world* w, ship* s, uint32_t r_origin, uint32_t r_dest) {
    s->origin = uniform_int(r_origin, w->P);
    s->dest = pick_other(r_dest, w->P, s->origin);
    s->cargo = 0;
    s->fuel = INITIAL_FUEL;
    s->x = w->port_x[s->origin];
    s->y = w->port_y[s->origin];
}

int orc_reset_batch(const orc_world* w, int64_t n, const uint8_t* mask, const int32_t* origin_in,
                    const int32_t* dest_in, uint64_t seed, int64_t env_id_base, uint32_t epoch,
                    int32_t* x, int32_t* y, double* fuel, int32_t* cargo, int32_t* origin,
                    int32_t* dest) {
    if (w->P < 2) return -1; /* the reference's dest != origin loop never ends for P < 2 */
    for (int64_t i = 0; i < n; ++i) {
        if (mask && !mask[i]) continue;
        ship s;
        if (origin_in) {
            s.origin = origin_in[i];
            s.dest = dest_in[i];
            s.cargo = 0;
            s.fuel = INITIAL_FUEL;
            s.x = w->port_x[s.origin];
            s.y = w->port_y[s.origin];
        } else {
            uint32_t o[4]; /* one block per env, epoch in the t word */
            draw4(seed, env_id_base + i, epoch, SLOT_EXPLICIT_RESET, o);
            reset_words(w, &s, o[0], o[1]);
        }
        store(&s, i, x, y, fuel, cargo, origin, dest);
    }
    return 0;
}

int orc_step_batch_autoreset(const orc_world* w, int64_t n, const int32_t* actions, uint64_t seed,
                             int64_t env_id_base, uint32_t t, int32_t* x, int32_t* y, double* fuel,
                             int32_t* cargo, int32_t* origin, int32_t* dest, float* ep_return,
                             int32_t* ep_len, double* reward, int32_t* done, int32_t* err,
                             double* stats) {
    if (w->P < 2) return -1;
    orc_step_batch(w, n, 0, NULL, actions, NULL, NULL, seed, env_id_base, t, x, y, fuel, cargo,
                   origin, dest, reward, done, err);
    int64_t quad = -1;
    int32_t resets = 0; /* envs of the current quad reset so far (RESET_r rank) */
    for (int64_t i = 0; i < n; ++i) {
        float rf = (float)reward[i];
        ep_return[i] += rf;
        ep_len[i] += 1;
        const int64_t e = env_id_base + i;
        if ((e >> 2) != quad) {
            quad = e >> 2;
            resets = 0;
        }
        if (done[i]) {
            stats[0] += (double)ep_return[i];
            stats[1] += 1.0;
            stats[2] += (double)ep_len[i];
            ship s;
            uint32_t o[4];
            draw4(seed, quad, t, RESET_SLOT[resets & 3], o);
            resets += 1;
            reset_words(w, &s, o[0], o[1]);
            store(&s, i, x, y, fuel, cargo, origin, dest);
            ep_return[i] = 0.0f;
            ep_len[i] = 0;
        }
    }
    return 0;
}

/* sample_action, environment.py:245-263, from one Philox word r. Returns the
 * action type, or SAMPLE_RAISES / SAMPLE_NO_OTHER_PORT where the reference raises
 * or never returns. */
static int32_t sample_action(const orc_world* w, const ship* s, uint32_t r, int32_t* a, int32_t* b) {
    static const int32_t mx[4] = {0, -1, 0, 1}; /* random.choice([NORTH, EAST, SOUTH, WEST]) :165-167 */
    static const int32_t my[4] = {-1, 0, 1, 0};
    const int32_t cur = current_port(w, s); /* _get_current_port_idx :145-153 */
    *a = 0;
    *b = 0;
    if (s->dest < 0 && cur >= 0) { /* :247-253: randint until != current port */
        if (w->P < 2) return SAMPLE_NO_OTHER_PORT;
        *a = pick_other(r, w->P, cur);
        return SELECT_PORT;
    }
    if (s->cargo == 0 && cur >= 0) { /* :255-257, randint(1, port_cargo[idx]) :160 */
        if (w->port_cargo[cur] < 1) return SAMPLE_RAISES; /* randint(1, 0): ValueError */
        *a = 1 + uniform_int(r, w->port_cargo[cur]);
        return TAKE_CARGO;
    }
    if (s->fuel == 0.0 && cur >= 0) return SAMPLE_RAISES; /* self.fuel[idx]: TypeError :163 */
    *a = mx[r & 3];
    *b = my[r & 3];
    return MOVE_SHIP;
}

int orc_sample_actions(const orc_world* w, int64_t n, const int32_t* x, const int32_t* y,
                       const double* fuel, const int32_t* cargo, const int32_t* origin,
                       const int32_t* dest, uint64_t seed, int64_t env_id_base, uint32_t t,
                       int32_t* type, int32_t* a, int32_t* b) {
    for (int64_t i = 0; i < n; ++i) {
        ship s;
        load(&s, i, x, y, fuel, cargo, origin, dest);
        uint32_t o[4];
        draw4(seed, env_id_base + i, t, SLOT_SAMPLE, o);
        type[i] = sample_action(w, &s, o[0], &a[i], &b[i]);
    }
    return 0;
}

/* MCTSAgent._rollout, agents/mcts.py:211-238: sample_action + step until done or
 * max_steps counted steps; a raising step is retried without counting (:231-233),
 * a raising sample_action leaves the loop (it sits outside the try, :227). The
 * reference retries without bound; max_attempts bounds it. */
int orc_rollout(const orc_world* w, int64_t n, const int32_t* x, const int32_t* y,
                const double* fuel, const int32_t* cargo, const int32_t* origin,
                const int32_t* dest, int64_t m, const int32_t* src, int32_t max_steps,
                int32_t max_attempts, uint64_t seed, int64_t rollout_base, double* ret,
                int32_t* steps, int32_t* status) {
    for (int64_t r = 0; r < m; ++r) {
        const int64_t i = src[r];
        if (i < 0 || i >= n) {
            ret[r] = 0.0;
            steps[r] = 0;
            status[r] = ROLL_BAD_SRC;
            continue;
        }
        ship s;
        load(&s, i, x, y, fuel, cargo, origin, dest);
        double total = 0.0;
        int32_t counted = 0, st = ROLL_ATTEMPTS;
        for (int32_t k = 0; k < max_attempts; ++k) {
            if (counted >= max_steps) { /* while not done and steps < max_rollout_steps (:225) */
                st = ROLL_MAX_STEPS;
                break;
            }
            uint32_t blk[4];
            draw4(seed, rollout_base + r, (uint32_t)k, SLOT_ROLLOUT, blk);
            int32_t a, b;
            const int32_t ty = sample_action(w, &s, blk[0], &a, &b);
            if (ty < 0) {
                st = ROLL_RAISED;
                break;
            }
            source src = {NULL, seed, rollout_base + r, (uint32_t)k, 0, 0, blk, 0, 0};
            double rw = 0.0;
            int32_t d = 0;
            if (step_typed(w, &s, ty, a, b, &src, &rw, &d) != E_OK) continue;
            total += rw; /* total_reward += reward (:229) */
            counted += 1;
            if (d) {
                st = ROLL_DONE;
                break;
            }
        }
        if (st == ROLL_ATTEMPTS && counted >= max_steps) st = ROLL_MAX_STEPS;
        ret[r] = total;
        steps[r] = counted;
        status[r] = st;
    }
    return 0;
}

int orc_observe(const orc_world* w, int64_t n, const int32_t* x, const int32_t* y,
                const double* fuel, const int32_t* origin, const int32_t* dest, float* obs) {
    const int64_t ld = 6 + 4 * (int64_t)w->P;
    for (int64_t i = 0; i < n; ++i) {
        float* row = obs + i * ld;
        row[0] = (float)x[i];
        row[1] = (float)y[i];
        row[2] = (float)fuel[i];
        row[3] = (float)fuel[i]; /* "cargo": self.fuel, shipping/environment.py:206 */
        row[4] = (float)origin[i]; /* None -> -1, utils/preprocessing.py:42-45 */
        row[5] = (float)dest[i];
        for (int32_t p = 0; p < w->P; ++p) {
            row[6 + 4 * p + 0] = (float)w->port_x[p];
            row[6 + 4 * p + 1] = (float)w->port_y[p];
            row[6 + 4 * p + 2] = (float)w->port_fuel[p];
            row[6 + 4 * p + 3] = (float)w->port_cargo[p];
        }
    }
    return 0;
}

int orc_valid_mask(const orc_world* w, int64_t n, const int32_t* x, const int32_t* y,
                   const int32_t* origin, uint8_t* bits) {
    const int32_t P = w->P, A = 4 + P + 50 + 200;
    const int64_t stride = (A + 7) / 8;
    memset(bits, 0, (size_t)(n * stride));
    for (int64_t i = 0; i < n; ++i) {
        ship s = {x[i], y[i], 0.0, 0, origin[i], 0};
        int32_t cur = current_port(w, &s);
        for (int32_t a = 0; a < A; ++a) {
            int v;
            if (a < 4) v = 1;
            else if (a < 4 + P) { /* must sit on that port and it must not be the origin */
                int32_t p = a - 4;
                v = !(origin[i] >= 0 && p == origin[i]) && w->port_x[p] == x[i] &&
                    w->port_y[p] == y[i];
            } else if (a < 4 + P + 50) {
                int32_t amt = a - (4 + P);
                v = cur >= 0 && 0 < amt && amt <= w->port_cargo[cur];
            } else {
                int32_t amt = a - (4 + P + 50);
                v = cur >= 0 && 0 < amt && amt <= w->port_fuel[cur];
            }
            if (v) bits[i * stride + a / 8] |= (uint8_t)(0x80u >> (a % 8));
        }
    }
    return 0;
}

/* Bench action mix: 90 % move (uniform direction),
 * 5 % TAKE_CARGO U{1..20}, 3 % TAKE_FUEL U{1..20}, 2 % SELECT U{0..P-1}. */
int orc_gen_actions(int64_t n, int32_t P, uint64_t seed, int64_t env_id_base, uint32_t t,
                    int32_t* actions) {
    for (int64_t i = 0; i < n; ++i) {
        uint32_t o[4];
        draw4(seed, env_id_base + i, t, SLOT_ACTION, o);
        int32_t c = uniform_int(o[0], 100);
        int32_t a;
        if (c < 90) a = (int32_t)(o[1] & 3u);
        else if (c < 95) a = 4 + P + 1 + uniform_int(o[1], 20);
        else if (c < 98) a = 4 + P + 50 + 1 + uniform_int(o[1], 20);
        else a = 4 + uniform_int(o[2], P);
        actions[i] = a;
    }
    return 0;
}

/* ------------------------------------------------------------------ DQN replay minibatch */
/* update()'s random.sample(memory, batch_size) (agents/dqn.py:213) under the build's
 * contract: a 4-round Feistel permutation of [0, size) on 2h bits (2h >= log2 size),
 * round function lowbias32(R ^ key[r]) masked to h bits, cycle-walked into the domain;
 * keys = Philox(seed, env id 2^64 - 1) at (t, SLOT_REPLAY). Batch position j takes the
 * first unflagged index among perm(j + k * B), k < 4, positions < size; else -1. */
static uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

uint32_t orc_feistel_perm(uint32_t p, uint32_t D, const uint32_t key[4]) {
    uint32_t bits = 2;
    while (bits < 32 && ((uint64_t)1 << bits) < (uint64_t)D) bits += 2;
    const uint32_t h = bits / 2, m = (1u << h) - 1u;
    do {
        uint32_t L = p >> h, R = p & m;
        for (int r = 0; r < 4; ++r) {
            const uint32_t nl = R;
            R = L ^ (lowbias32(R ^ key[r]) & m);
            L = nl;
        }
        p = (L << h) | R;
    } while (p >= D);
    return p;
}

int orc_replay_pick(int64_t size, int64_t batch, const uint8_t* invalid, uint64_t seed, uint32_t t,
                    int64_t* slot) {
    uint32_t key[4];
    draw4(seed, -1, t, SLOT_REPLAY, key);
    for (int64_t j = 0; j < batch; ++j) {
        slot[j] = -1;
        for (int k = 0; k < 4; ++k) {
            const int64_t pos = j + k * batch;
            if (pos >= size) break;
            const uint32_t l = orc_feistel_perm((uint32_t)pos, (uint32_t)size, key);
            if (!invalid[l]) {
                slot[j] = l;
                break;
            }
        }
    }
    return 0;
}
