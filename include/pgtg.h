/* include/pgtg.h -- C ABI of the MI355X-native batched PGTG environment (libpgtg_hip.so).
 *
 * The reference (Inuri04/pgtg) has no FFI: its hot path sits behind the Gymnasium Env API of
 * `PGTGEnv` (pgtg/environment.py:297-1281, registered as "pgtg-v4" in pgtg/__init__.py:7).  Each
 * entry point below replaces one piece of that surface for a BATCH of independent environments
 * resident in HBM; the Python facade in pgtg_amd/ (PGTGEnv, PGTGVecEnv) binds it with ctypes.
 *
 *   pgtg_create       <- PGTGEnv.__init__(map_path, **kwargs)          environment.py:302-515
 *   pgtg_reset        <- PGTGEnv.reset(seed=...)                        environment.py:581-656
 *   pgtg_step         <- PGTGEnv.step(action) + same-step auto-reset    environment.py:1092-1281
 *   pgtg_set_outputs  <- the obs/reward/terminated/truncated/info return values (device buffers)
 *   pgtg_get_cars / pgtg_get_env_state <- get_info() fields             environment.py:1538-1578
 *   pgtg_set_agent / pgtg_add_car      <- test-style state overrides (env.position = ..., env.cars.append)
 *   pgtg_get_map_plan <- EpisodeMap.map_plan / save_map                 pgtg/map.py:173-184
 *   pgtg_get_squares  <- EpisodeMap.squares feature sets (feature_at)   pgtg/map.py:49-69, parser.py:13-166
 *   pgtg_get_counters <- (new) device-side env-step / episode counters
 *
 * Conventions: all pointers named *_dev are device pointers (hipMalloc'd or torch data_ptr) on the
 * handle's device; everything else is host memory.  Calls on one handle are serialised by the
 * caller and enqueued on the handle's HIP stream (pgtg_set_stream); they do not synchronise unless
 * documented.  Every entry point returns PGTG_OK (0) or a negative PGTG_E_* code; the message is
 * available from pgtg_last_error(handle).
 */
#ifndef PGTG_H_
#define PGTG_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PGTG_ABI_VERSION 7

/* status codes (Python facade maps them to the reference's exception types) */
#define PGTG_OK 0
#define PGTG_E_INVALID -1      /* invalid configuration / argument  -> ValueError            */
#define PGTG_E_DONE -2         /* step on a finished env (no auto-reset) -> RuntimeError       */
#define PGTG_E_DEVICE -3       /* HIP runtime error                  -> RuntimeError           */
#define PGTG_E_UNSUPPORTED -4  /* outside this build's limits        -> ValueError             */
#define PGTG_E_MAP -5          /* map without route / no start square / empty route choice      */

/* limits of this build */
#define PGTG_MAX_TILES 256     /* width*height of the tile map (16 x 16; traffic: squares <= 255 per side) */
#define PGTG_MAX_CHANNELS 128  /* observation keys: distinct feature names (the vocabulary has 51; unknown names give zero channels) */
#define PGTG_MAX_RULES 8       /* traffic rules: the triggered-rule mask output is one byte per env */
#define PGTG_MAX_WINDOW 31     /* observation window side (9 fixed, 2*s+1 sliding, s <= 15) */

/* observation channel codes (one per key of the reference's obs["map"] dict) */
enum {
  PGTG_CH_ZERO = 0,        /* names that never occur on a square: all zeros */
  PGTG_CH_WALL = 1,        /* "walls" / "wall" */
  PGTG_CH_GOALS = 2,       /* "goals": subgoal or final goal */
  PGTG_CH_TRAFFIC = 3,     /* "traffic": a car on the square */
  PGTG_CH_TL_GREEN = 4,    /* "traffic_light" key -> traffic_light_{green,yellow,red} */
  PGTG_CH_TL_YELLOW = 5,
  PGTG_CH_TL_RED = 6,
  PGTG_CH_START = 7,
  PGTG_CH_SUBGOAL = 8,
  PGTG_CH_USED_SUBGOAL = 9,
  PGTG_CH_FINAL_GOAL = 10,
  PGTG_CH_ICE = 11,
  PGTG_CH_BROKEN = 12,
  PGTG_CH_SAND = 13,
  PGTG_CH_SPAWNER = 14,
  PGTG_CH_LANE0 = 32       /* + lane id 0..31, "car_lane <route> <type>" in sorted order */
};

typedef struct {
  int32_t tile_exits;       /* rule tile_type "NESW" bits as mask (bit0 north); -1 = never */
  int32_t speed_sq_min;     /* admissible vx^2+vy^2 interval for velocity_range (fp64 sqrt) */
  int32_t speed_sq_max;
  int32_t min_traffic;
  int32_t min_matching_traffic;
  /* weight[d][r]: maneuvers with agent direction d listing route r;
   * d: 0 south_to_north 1 west_to_east 2 north_to_south 3 east_to_west 4 stationary 5 near_goal */
  uint8_t weight[6][20];
} PgtgRule;

/* Raw constructor kwargs (pgtg/environment.py:302-359) plus the fixed map of map_path. */
typedef struct {
  int32_t abi_version;                 /* = PGTG_ABI_VERSION */
  int32_t width, height;               /* random_map_width / random_map_height */
  double pct_connections;              /* random_map_percentage_of_connections */
  int32_t start_mode, goal_mode;       /* 0 (x,y,dir)  1 (x,y)  2 "random" */
  int32_t start_x, start_y, start_dir; /* dir: 0 north 1 east 2 south 3 west; x/y may be -1 */
  int32_t goal_x, goal_y, goal_dir;
  int32_t min_distance;                /* random_map_minimum_distance_between_start_and_goal, -1 None */
  double obstacle_probability;
  double w_ice, w_broken, w_sand, w_tl;
  int32_t n_channels;
  int32_t channels[PGTG_MAX_CHANNELS];
  int32_t sliding, sliding_size, next_subgoal;
  double sum_subgoals_reward, final_goal_bonus, crash_penalty, tl_violation_penalty;
  double standing_still_penalty, visited_penalty;
  double ice_probability, street_damage_probability, sand_probability, traffic_density;
  int32_t phase_dur[3];
  int32_t ignore_traffic_collisions;
  double profile_pct[5];               /* conservative, normal, aggressive, elderly, reckless */
  int32_t separate_reward_cost;
  int32_t n_rules;
  PgtgRule rules[PGTG_MAX_RULES];
  /* fixed map (map_path): tiles row-major [y*w+x] */
  int32_t fixed_map, fm_w, fm_h;
  uint8_t fm_exits[PGTG_MAX_TILES];
  int8_t fm_obst_type[PGTG_MAX_TILES]; /* -1 none, 0 ice 1 broken road 2 sand 3 traffic_light */
  int8_t fm_obst_mask[PGTG_MAX_TILES]; /* -1 none, 0..13 (tools/gen_tables.py order) */
  int32_t fm_start[3], fm_goal[3];
  /* vector-env options (no reference equivalent; pgtg/train.py:21-41 wraps with TimeLimit) */
  int32_t autoreset;                   /* 1: same-step auto-reset (gymnasium/SB3 vector semantics) */
  int32_t max_episode_steps;           /* TimeLimit truncation, 0 = none */
  int32_t min_car_capacity;            /* car slots per env for pgtg_add_car (tests), 0 = from density */
  /* launch-shape overrides for tests and A/B runs (0 = automatic; the library reads no environment) */
  int32_t tune_envs_per_block;         /* 16, 32, 64, 128 or 256 env lanes per step workgroup */
  int32_t tune_obs_sub;                /* envs per observation sub-batch */
  int32_t tune_kt_grid, tune_kt_cap, tune_kt_wpc; /* k_traffic grid, envs per wave, workgroups per CU */
  int32_t tune_car_slots;              /* car slots per env (>= 3 x capacity + 4; tests of the bound) */
  int32_t tune_kt_serial;              /* 1: initial traffic's per-car draws on one lane per env (the
                                          rejection fallback of the lane-parallel path; tests) */
  int32_t tune_queue_mode;             /* map-queue step kernel: 0 automatic (k_envb for grids of <= 2 rounds
                                          of workgroups, else k_envq), 1 k_envq, 2 k_envb */
  int32_t tune_fault;                  /* tests of the error paths: bit 0 clears the path walk's north
                                          mask on maps whose tile 0 keeps its east exit (inconsistent masks ->
                                          PGTG_E_DEVICE for those envs, the launch finishes) */
} PgtgConfig;

/* Output buffers (device pointers, caller-owned, contiguous).  NULL = not produced. */
typedef struct {
  uint8_t* obs;            /* [N][n_channels][win][win] uint8 one-hot ([c][x][y] like the reference) */
  int32_t* position;       /* [N][2] */
  int32_t* velocity;       /* [N][2] */
  int32_t* next_subgoal;   /* [N] (use_next_subgoal_direction) */
  double* reward;          /* [N] */
  double* cost;            /* [N] (separate_reward_cost) */
  uint8_t* terminated;     /* [N] */
  uint8_t* truncated;      /* [N] */
  uint8_t* final_obs;      /* [N][n_channels][win][win]: terminal observation of envs reset this step */
  int32_t* final_position; /* [N][2] */
  int32_t* final_velocity; /* [N][2] */
  int32_t* final_next_subgoal; /* [N] */
  uint8_t* braking;        /* [N] triggered traffic rules, bit r = PgtgConfig.rules[r] (rule_triggers);
                              nonzero <=> info['traffic_rules']['braking_applied'] */
} PgtgOutputs;

typedef struct {
  int32_t x, y, vx, vy;
  int32_t terminated, flat_tire, phase, elapsed;
  int32_t n_cars, next_car_id, path_len, error;
  uint32_t spawn_counter;
  uint64_t seed;
  uint64_t used_subgoals[4];           /* bit t%64 of word t/64: tile t's subgoal used (all 256 tiles) */
  int32_t n_spawners, car_tail;        /* car slots in use (cars + empty slots before the last car) */
} PgtgEnvState;

typedef struct {
  int32_t id, x, y, route, profile, patience, delay;
} PgtgCar;

typedef struct pgtg_handle pgtg_handle;

int pgtg_create(const PgtgConfig* cfg, uint64_t n_envs, int32_t device, pgtg_handle** out);
int pgtg_destroy(pgtg_handle* h);
/* Queue work on this stream (hipStream_t); NULL = the null stream. */
int pgtg_set_stream(pgtg_handle* h, void* stream);
int pgtg_set_outputs(pgtg_handle* h, const PgtgOutputs* out);
/* Seeded reset of env i with seeds_host[i] (NULL: seed_base + global index), only where
 * mask_dev[i] != 0 (NULL: all).  Writes the reset observation to the bound outputs. */
int pgtg_reset(pgtg_handle* h, const uint64_t* seeds_host, uint64_t seed_base, const uint8_t* mask_dev);
/* Unseeded reset (next spawn block of each env's seed sequence) where mask_dev[i] != 0. */
int pgtg_reset_unseeded(pgtg_handle* h, const uint8_t* mask_dev);
/* One tick for every env.  actions_dev: [N] uint8 in [0, 9). */
int pgtg_step(pgtg_handle* h, const uint8_t* actions_dev);
/* `ticks` consecutive pgtg_step calls from a resident rollout action buffer: tick k reads the [N]
 * row at actions_dev + k * row_stride bytes (row_stride >= N).  Identical results to the loop of
 * pgtg_step calls (the outputs hold the last tick's); one host call, so the launches are queued
 * without per-tick host overhead.  Stops at the first launch error. */
int pgtg_step_many(pgtg_handle* h, const uint8_t* actions_dev, uint64_t row_stride, uint64_t ticks);
/* Fill [N] uint8 actions with a counter-based uniform hash of (seed, env_offset + env, t) --
 * synthetic rollouts; env_offset = global index of env 0 so that a sharded run draws the same
 * actions as one GPU running the whole batch. */
int pgtg_random_actions(pgtg_handle* h, uint8_t* actions_dev, uint64_t seed, uint64_t t, uint64_t env_offset);
/* Host-synchronising introspection (copies device state). */
int pgtg_get_env_state(pgtg_handle* h, uint64_t env, PgtgEnvState* st);
int pgtg_get_cars(pgtg_handle* h, uint64_t env, PgtgCar* cars, int32_t cap, int32_t* n);
int pgtg_get_map_plan(pgtg_handle* h, uint64_t env, int32_t* w, int32_t* h_, uint8_t* exits, int8_t* otype,
                      int8_t* omask, int32_t* start3, int32_t* goal3);
/* The episode map's squares as feature words, x-major (index x * height + y), height = 9 * tile rows:
 * bits 0-31 the car lanes (lane ids of the tables), then the PGTG_SQ_* flags below. */
#define PGTG_SQ_WALL (1ull << 32)
#define PGTG_SQ_SPAWNER (1ull << 37)
#define PGTG_SQ_START (1ull << 38)
#define PGTG_SQ_SUBGOAL (1ull << 39)
#define PGTG_SQ_USED_SUBGOAL (1ull << 40)
#define PGTG_SQ_FINAL_GOAL (1ull << 41)
#define PGTG_SQ_ICE (1ull << 42)
#define PGTG_SQ_BROKEN_ROAD (1ull << 43)
#define PGTG_SQ_SAND (1ull << 44)
#define PGTG_SQ_TRAFFIC_LIGHT (1ull << 45)
int pgtg_get_squares(pgtg_handle* h, uint64_t env, uint64_t* words, int32_t cap, int32_t* width, int32_t* height);
int pgtg_set_agent(pgtg_handle* h, uint64_t env, int32_t x, int32_t y, int32_t vx, int32_t vy);
/* Append a car (env.cars.append(Car(...)) in the reference tests); car_id < 0 takes the env's next id. */
int pgtg_add_car(pgtg_handle* h, uint64_t env, int32_t x, int32_t y, int32_t route, int32_t profile, int32_t car_id);
/* Whole-batch state for bit-exact replay: every device array that carries env state
 * between launches (agent records, seeds, tile plans, all RNG streams with their buffered halves,
 * visited bitsets, the car slots, traffic records with the persisted lane-square occupancy counters,
 * spawner lists, map queue, counters) as one host
 * blob.  pgtg_state_size gives the blob size; pgtg_load_state accepts only a blob dumped from a handle
 * of the same config (checked by a hash of every configuration field) and batch size.  Outputs are not state: call pgtg_observe after a load to
 * re-emit the observations.  Both synchronise.  (No reference equivalent: PGTGEnv deep-copies
 * itself in light_step, environment.py:1283-1299.) */
int pgtg_state_size(pgtg_handle* h, uint64_t* bytes);
int pgtg_dump_state(pgtg_handle* h, void* buf, uint64_t bytes);
int pgtg_load_state(pgtg_handle* h, const void* buf, uint64_t bytes);
/* PGTGEnv.set_to_state(state) (environment.py:1301-1342) for one env: position, velocity, flat tire
 * and the car list (patience/delay 0; next car id = last id + 1 if any cars).  Synchronises. */
int pgtg_set_to_state(pgtg_handle* h, uint64_t env, int32_t x, int32_t y, int32_t vx, int32_t vy, int32_t flat_tire,
                      const PgtgCar* cars, int32_t n_cars);
/* Replace the traffic rules of every env (add_traffic_rule / remove_traffic_rule,
 * environment.py:569-575); takes effect from the next step.  n_rules <= PGTG_MAX_RULES. */
int pgtg_set_rules(pgtg_handle* h, const PgtgRule* rules, int32_t n_rules);
/* FlattenObservation rows (pgtg/train.py:40; gymnasium's flatten of the Dict observation space of
 * environment.py:415-441, keys in name order), written by k_flatten after every launch that writes the
 * bound observation (step, reset, observe): per env, D = n_channels*win*win (+ 9) + 18 + 2 values
 *   map channels in `order` (order[k] = channel of the k-th name-sorted key), win*win each, [x][y] |
 *   next-subgoal one-hot at direction + 1 (9, only with use_next_subgoal_direction) |
 *   position one-hot of x (9), of y (9) | velocity (2)
 * as float32 (dtype 0) or int8 (dtype 1: exact, every value being 0/1 or a velocity) into flat_dev
 * [N][D]; final_flat_dev [N][D] receives the terminal observations of the envs that finished in a step
 * (their rows only; the other rows are left as they are).  Buffers 16-byte aligned; NULL, NULL = off.
 * Needs the corresponding PgtgOutputs bound first; a sliding window of size >= 9 is refused
 * (PGTG_E_UNSUPPORTED) as gymnasium's flatten raises for it.  No reference function: it replaces the
 * FlattenObservation wrapper the reference's caller puts around each env. */
int pgtg_set_flat_outputs(pgtg_handle* h, const int32_t* order, int32_t n_order, int32_t dtype, void* flat_dev,
                          void* final_flat_dev);
/* With flat rows bound, the observation pass of k_flatten also writes, per env, the reward as float32,
 * done = terminated | truncated and truncated-and-not-terminated (uint8 0/1) -- what an SB3-style
 * vector env returns -- into these [N] device buffers (all three or none; needs the reward, terminated
 * and truncated outputs bound).  No reference function: it replaces per-step tensor arithmetic. */
int pgtg_set_flat_scalars(pgtg_handle* h, float* reward_f32_dev, uint8_t* dones_dev, uint8_t* truncated_only_dev);
/* Re-emit the observation of every env into the bound outputs (after set_agent/add_car). */
int pgtg_observe(pgtg_handle* h);
/* Per-env uint64 digest of the car list into out_dev[N] (device; parity tests: the car term of
 * pgtg_amd/digest.py).  Traffic handles only.  Asynchronous on the handle's stream. */
int pgtg_car_digest(pgtg_handle* h, uint64_t* out_dev);
/* steps (env-steps executed) and episodes (resets) since create, summed over envs; synchronises. */
int pgtg_get_counters(pgtg_handle* h, uint64_t* env_steps, uint64_t* episodes);
/* Map-queue ring entries generated since create (k_qfill after resets + the step launches' helper
 * waves; 0 for handles without the queue): a window's delta beside its episode delta shows that the
 * maps the episodes consumed were generated in the window.  Synchronises. */
int pgtg_get_queue_maps(pgtg_handle* h, uint64_t* maps);
/* Map-queue refill requests served from the overflow lists since create (step launches of one round
 * of workgroups list at most 64 requests per workgroup; the rest go to lists shared by residue mod 8
 * and are served by other workgroups' helper waves in the next launch).  Synchronises. */
int pgtg_get_queue_overflow(pgtg_handle* h, uint64_t* served);
/* Number of envs whose last step reported an error (PGTG_E_DONE / PGTG_E_MAP); synchronises. */
int pgtg_error_count(pgtg_handle* h, uint64_t* n_errors, int32_t* first_code);
/* Measured HBM denominator of the roofline: a 16-B/lane stream copy of `bytes` between two device
 * buffers on `device`, `reps` timed passes; *copy_gbs = (read + write bytes) / s / 1e9.  Synchronises. */
int pgtg_measure_hbm(int32_t device, uint64_t bytes, int32_t reps, double* copy_gbs);
int pgtg_window(const pgtg_handle* h);
uint64_t pgtg_num_envs(const pgtg_handle* h);
/* Launch geometry of the step kernel: envs per 256-lane workgroup and dynamic LDS bytes. */
int pgtg_launch_info(const pgtg_handle* h, int32_t* envs_per_block, int32_t* lds_bytes);
/* Resident workgroups per CU of the step kernel this handle launches (HIP occupancy query). */
int pgtg_occupancy(const pgtg_handle* h, int32_t* step_blocks_per_cu);
/* Name of the kernel(s) one pgtg_step launches for this handle (measurement labels). */
const char* pgtg_step_kernel(const pgtg_handle* h);
const char* pgtg_last_error(const pgtg_handle* h);
/* Per-launch device timing of the step kernels with HIP events on the handle's stream.  every > 0:
 * every every-th pgtg_step brackets its kernels with an event pair (1: all; 0: off);
 * pgtg_timing_read synchronises and returns the summed milliseconds of the bracketed launches and
 * their number (reset=1 clears the tally). */
int pgtg_enable_timing(pgtg_handle* h, int32_t every);
int pgtg_timing_read(pgtg_handle* h, double* total_ms, uint64_t* launches, int32_t reset);

#ifdef __cplusplus
}
#endif
#endif /* PGTG_H_ */
