/* oracle/pgtg_oracle.c -- TEST INFRASTRUCTURE ONLY (see pgtg_oracle.h).
 *
 * A deliberately literal, scalar restatement of the reference: per-square feature SETS are
 * materialised (as 64-bit words) exactly like pgtg/parser.py builds them, the car list is a plain
 * array scanned linearly like pgtg/environment.py:944-948, the graph edge list is manipulated like
 * pgtg/map_generator.py:227-264.  It shares no code with the HIP product path.
 * Compile with -ffp-contract=off (fp64 decomposition and CDF arithmetic must not fuse).
 */
#include "pgtg_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle_tables.h"

typedef unsigned __int128 u128;

/* ----------------------------------------------------------------------------------------------
 * numpy RNG restatement.  numpy/random/bit_generator.pyx (SeedSequence), _pcg64.pyx /
 * src/pcg64/pcg64.h (PCG64 XSL-RR, next32 buffering), src/distributions/distributions.c
 * (buffered_bounded_lemire_uint32, random_interval), _generator.pyx (choice).
 * -------------------------------------------------------------------------------------------- */
#define SS_INIT_A 0x43b0d7e5u
#define SS_MULT_A 0x931e8875u
#define SS_INIT_B 0x8b51f9ddu
#define SS_MULT_B 0x58f38dedu
#define SS_MIX_L 0xca01f9ddu
#define SS_MIX_R 0x4973f715u

static uint32_t ss_hashmix(uint32_t v, uint32_t* hc) {
  v ^= *hc;
  *hc *= SS_MULT_A;
  v *= *hc;
  v ^= v >> 16;
  return v;
}
static uint32_t ss_mix(uint32_t x, uint32_t y) {
  uint32_t r = SS_MIX_L * x - SS_MIX_R * y;
  r ^= r >> 16;
  return r;
}

void orc_seed_seq_state(const uint32_t* entropy, int n, uint32_t out[8]) {
  uint32_t pool[4];
  uint32_t hc = SS_INIT_A;
  for (int i = 0; i < 4; i++) pool[i] = ss_hashmix(i < n ? entropy[i] : 0u, &hc);
  for (int s = 0; s < 4; s++)
    for (int d = 0; d < 4; d++)
      if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], &hc));
  for (int s = 4; s < n; s++)
    for (int d = 0; d < 4; d++) pool[d] = ss_mix(pool[d], ss_hashmix(entropy[s], &hc));
  uint32_t hb = SS_INIT_B;
  for (int i = 0; i < 8; i++) {
    uint32_t v = pool[i % 4];
    v ^= hb;
    hb *= SS_MULT_B;
    v *= hb;
    v ^= v >> 16;
    out[i] = v;
  }
}

static const u128 PCG_MULT = (((u128)0x2360ED051FC65DA4ull) << 64) | (u128)0x4385DF649FCCF645ull;

typedef struct { u128 state, inc; int has32; uint32_t buf32; } pcg_t;

static void pcg_step(pcg_t* g) { g->state = g->state * PCG_MULT + g->inc; }

static uint64_t pcg_next64(pcg_t* g) {
  pcg_step(g);
  uint64_t hi = (uint64_t)(g->state >> 64), lo = (uint64_t)g->state;
  unsigned rot = (unsigned)(g->state >> 122);
  uint64_t x = hi ^ lo;
  return (x >> rot) | (x << ((64 - rot) & 63));
}
static uint32_t pcg_next32(pcg_t* g) {
  if (g->has32) {
    g->has32 = 0;
    return g->buf32;
  }
  uint64_t n = pcg_next64(g);
  g->has32 = 1;
  g->buf32 = (uint32_t)(n >> 32);
  return (uint32_t)n;
}
static double pcg_double(pcg_t* g) { return (double)(pcg_next64(g) >> 11) * (1.0 / 9007199254740992.0); }

/* Generator(PCG64(SeedSequence(seed, spawn_key=(k,)))) as built by gymnasium seeding + spawn */
static void pcg_from_seed(pcg_t* g, uint64_t seed, int has_key, uint32_t key) {
  uint32_t ent[8];
  int n = 0;
  if (seed == 0) {
    ent[n++] = 0;
  } else {
    uint64_t s = seed;
    while (s) {
      ent[n++] = (uint32_t)(s & 0xffffffffu);
      s >>= 32;
    }
  }
  if (has_key) { /* get_assembled_entropy: pad run entropy to pool size when a spawn key exists */
    while (n < 4) ent[n++] = 0;
    ent[n++] = key;
  }
  uint32_t w[8];
  orc_seed_seq_state(ent, n, w);
  uint64_t v[4];
  for (int i = 0; i < 4; i++) v[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  u128 initstate = ((u128)v[0] << 64) | v[1];
  u128 initseq = ((u128)v[2] << 64) | v[3];
  g->state = 0;
  g->inc = (initseq << 1) | 1;
  pcg_step(g);
  g->state += initstate;
  pcg_step(g);
  g->has32 = 0;
  g->buf32 = 0;
}

static uint32_t lemire32(pcg_t* g, uint32_t rng) { /* result in [0, rng] */
  uint32_t excl = rng + 1;
  uint64_t m = (uint64_t)pcg_next32(g) * excl;
  uint32_t left = (uint32_t)m;
  if (left < excl) {
    uint32_t thr = (0xffffffffu - rng) % excl;
    while (left < thr) {
      m = (uint64_t)pcg_next32(g) * excl;
      left = (uint32_t)m;
    }
  }
  return (uint32_t)(m >> 32);
}

/* Generator.integers(lo, hi) (int64, endpoint False) == Generator.choice(n) index */
static int64_t gen_integers(pcg_t* g, int64_t lo, int64_t hi) {
  uint64_t rng = (uint64_t)(hi - lo - 1);
  if (rng == 0) return lo;
  if (rng == 0xffffffffull) return lo + pcg_next32(g);
  return lo + lemire32(g, (uint32_t)rng);
}

/* Generator.choice(a, p=p): cdf = cumsum(p); cdf /= cdf[-1]; searchsorted(random(), 'right') */
static int gen_choice_p(pcg_t* g, const double* p, int n) {
  double cdf[16];
  double acc = 0.0;
  for (int i = 0; i < n; i++) {
    acc += p[i];
    cdf[i] = acc;
  }
  double last = cdf[n - 1];
  for (int i = 0; i < n; i++) cdf[i] /= last;
  double u = pcg_double(g);
  int i = 0;
  while (i < n && !(u < cdf[i])) i++;
  return i;
}

/* Generator.choice(pop, size=k, replace=False) for pop <= 10000: Floyd, then _shuffle_int */
static void gen_choice_noreplace(pcg_t* g, int64_t pop, int64_t k, int64_t* out) {
  unsigned char* seen = (unsigned char*)calloc((size_t)pop + 1, 1);
  for (int64_t j = pop - k; j < pop; j++) {
    int64_t val = gen_integers(g, 0, j + 1);
    if (!seen[val]) {
      seen[val] = 1;
      out[j - pop + k] = val;
    } else {
      seen[j] = 1;
      out[j - pop + k] = j;
    }
  }
  free(seen);
  for (int64_t i = k - 1; i >= 1; i--) {
    int64_t j = gen_integers(g, 0, i + 1); /* _shuffle_int: random_bounded_uint64(0, i) (Lemire) */
    int64_t t = out[j];
    out[j] = out[i];
    out[i] = t;
  }
}

/* exported wrappers (known-answer tests against numpy) */
static void to_pub(const pcg_t* g, orc_pcg64* o) {
  o->st_hi = (uint64_t)(g->state >> 64);
  o->st_lo = (uint64_t)g->state;
  o->inc_hi = (uint64_t)(g->inc >> 64);
  o->inc_lo = (uint64_t)g->inc;
  o->has32 = g->has32;
  o->buf32 = g->buf32;
}
static void from_pub(const orc_pcg64* o, pcg_t* g) {
  g->state = ((u128)o->st_hi << 64) | o->st_lo;
  g->inc = ((u128)o->inc_hi << 64) | o->inc_lo;
  g->has32 = o->has32;
  g->buf32 = o->buf32;
}
void orc_pcg64_from_seed(uint64_t seed, uint32_t key, int has_key, orc_pcg64* o) {
  pcg_t g;
  pcg_from_seed(&g, seed, has_key, key);
  to_pub(&g, o);
}
#define WRAP(body) \
  pcg_t g;         \
  from_pub(o, &g); \
  body;            \
  to_pub(&g, o);
uint64_t orc_next64(orc_pcg64* o) { uint64_t r; WRAP(r = pcg_next64(&g)); return r; }
uint32_t orc_next32(orc_pcg64* o) { uint32_t r; WRAP(r = pcg_next32(&g)); return r; }
double orc_random(orc_pcg64* o) { double r; WRAP(r = pcg_double(&g)); return r; }
int64_t orc_integers(orc_pcg64* o, int64_t lo, int64_t hi) { int64_t r; WRAP(r = gen_integers(&g, lo, hi)); return r; }
int64_t orc_choice_p(orc_pcg64* o, const double* p, int n) { int64_t r; WRAP(r = gen_choice_p(&g, p, n)); return r; }
void orc_choice_noreplace(orc_pcg64* o, int64_t pop, int64_t k, int64_t* out) { WRAP(gen_choice_noreplace(&g, pop, k, out)); }

/* ----------------------------------------------------------------------------------------------
 * Environment state
 * -------------------------------------------------------------------------------------------- */
#define TILE 9
/* square feature word bits (oracle encoding, see tools/gen_tables.py) */
#define F_LANE_MASK 0xffffffffull
#define F_WALL (1ull << 32)
#define F_EXIT0 33 /* + dir */
#define F_SPAWNER (1ull << 37)
#define F_START (1ull << 38)
#define F_SUBGOAL (1ull << 39)
#define F_USED (1ull << 40)
#define F_FINAL (1ull << 41)
#define F_ICE (1ull << 42)
#define F_BROKEN (1ull << 43)
#define F_SAND (1ull << 44)
#define F_TLIGHT (1ull << 45)
#define F_EXITS (0xfull << 33)
#define LANE_ALL_UP 28 /* lane ids 28..31 = all up/down/left/right */

/* DRIVER_BEHAVIORS, pgtg/environment.py:64-109 (order of DriverProfile, :38-44) */
typedef struct {
  double yellow_stop, red_violation;
  int min_follow;
  double patience_level, speed_mult, reaction_delay;
} behavior_t;
static const behavior_t BEHAVIORS[5] = {
    {0.95, 0.01, 2, 0.9, 0.8, 0.1},   {0.75, 0.05, 1, 0.7, 1.0, 0.15}, {0.3, 0.15, 0, 0.3, 1.3, 0.05},
    {0.98, 0.001, 3, 0.95, 0.6, 0.3}, {0.1, 0.3, 0, 0.1, 1.5, 0.1},
};
/* ACTIONS_TO_ACCELERATION, pgtg/constants.py:6-16 */
static const int ACC[9][2] = {{-1, -1}, {-1, 0}, {-1, 1}, {0, -1}, {0, 0}, {0, 1}, {1, -1}, {1, 0}, {1, 1}};

typedef struct {
  int id, x, y, route, profile, patience, delay;
} car_t;

static void init_lanes(void);

struct orc_env {
  orc_config cfg;
  char err[256];
  /* np_random */
  int seeded;
  uint64_t seed;
  uint32_t spawn_counter;
  pcg_t map_rng, car_rng, ice_rng, broken_rng, sand_rng;
  /* map plan */
  int tw, th;
  uint8_t exits[1024];
  int8_t otype[1024], omask[1024];
  int start[3], goal[3];
  /* compiled map (EpisodeMap) */
  int W, H;
  uint64_t* sq; /* [x*H + y] */
  int path_len;
  int path[1024];      /* tile index y*tw+x */
  int tile_dir[1024];  /* subgoal_coordinates_to_direction incl. last (goal dir); -1 not on path */
  int num_subgoals;
  int *starters, n_starters;
  int *spawnable, n_spawnable;
  int *spawners, n_spawners;
  /* agent */
  int px, py, vx, vy;
  int terminated, flat_tire, phase, braking;
  double ind_reward;
  int* visited; /* positions_path as a bitset over [-2, W+1] x [-2, H+1] */
  /* traffic */
  car_t* cars;
  int ncars, capcars, next_car_id;
  double profile_p[5];
};

static int fail(orc_env* e, const char* m) {
  snprintf(e->err, sizeof e->err, "%s", m);
  return -1;
}
const char* orc_last_error(const orc_env* e) { return e->err; }

orc_env* orc_create(const orc_config* cfg) {
  orc_env* e = (orc_env*)calloc(1, sizeof(orc_env));
  init_lanes();
  e->cfg = *cfg;
  /* pgtg/environment.py:492-508 driver profile normalisation */
  double tot = 0.0;
  for (int i = 0; i < 5; i++) tot += cfg->profile_pct[i];
  if (tot > 0) {
    for (int i = 0; i < 5; i++) e->profile_p[i] = cfg->profile_pct[i] / tot;
  } else {
    for (int i = 0; i < 5; i++) e->profile_p[i] = 0.0;
    e->profile_p[1] = 1.0;
  }
  return e;
}

static void free_map(orc_env* e) {
  free(e->sq);
  free(e->starters);
  free(e->spawnable);
  free(e->spawners);
  free(e->visited);
  e->sq = NULL;
  e->starters = e->spawnable = e->spawners = e->visited = NULL;
}

void orc_destroy(orc_env* e) {
  if (!e) return;
  free_map(e);
  free(e->cars);
  free(e);
}

int orc_window(const orc_env* e) { return e->cfg.sliding ? 1 + 2 * e->cfg.sliding_size : TILE; }

static inline int inside(const orc_env* e, int x, int y) { return !(x < 0 || y < 0 || x >= e->W || y >= e->H); }
static inline uint64_t F(const orc_env* e, int x, int y) { return e->sq[x * e->H + y]; }

/* ----------------------------------------------------------------------------------------------
 * map generation (pgtg/map_generator.py)
 * -------------------------------------------------------------------------------------------- */
typedef struct { int a, b; } edge_t; /* node ids: tiles y*w+x (>=0), START=-1, END=-2 */

typedef struct {
  int n_keys;
  int keys[1100];             /* source nodes in first-use order (the nested dict's key order) */
  int dst[1100][5];           /* destinations in insertion order */
  int ndst[1100];
  int key_of[1100 + 2];       /* node -> key slot, -1 none */
  int count;                  /* number of directed edges */
} graph_t;

static int nid(int node) { return node + 2; } /* START=-1->1, END=-2->0 */

static void g_init(graph_t* g) {
  memset(g, 0, sizeof *g);
  for (int i = 0; i < 1102; i++) g->key_of[i] = -1;
}
static void g_add1(graph_t* g, int a, int b) { /* graph-theory add_edge(a, b), nested dict */
  int k = g->key_of[nid(a)];
  if (k < 0) {
    k = g->n_keys++;
    g->keys[k] = a;
    g->ndst[k] = 0;
    g->key_of[nid(a)] = k;
  }
  for (int i = 0; i < g->ndst[k]; i++)
    if (g->dst[k][i] == b) return; /* dict assignment keeps position */
  g->dst[k][g->ndst[k]++] = b;
  g->count++;
}
static void g_del1(graph_t* g, int a, int b) {
  int k = g->key_of[nid(a)];
  for (int i = 0; i < g->ndst[k]; i++)
    if (g->dst[k][i] == b) {
      memmove(&g->dst[k][i], &g->dst[k][i + 1], sizeof(int) * (size_t)(g->ndst[k] - i - 1));
      g->ndst[k]--;
      g->count--;
      return;
    }
}
static int g_has(const graph_t* g, int a, int b) {
  int k = g->key_of[nid(a)];
  if (k < 0) return 0;
  for (int i = 0; i < g->ndst[k]; i++)
    if (g->dst[k][i] == b) return 1;
  return 0;
}
/* BFS path start->end; returns length (0 if unreachable) */
static int g_bfs(const graph_t* g, int s, int t, int* path) {
  int par[1102], q[1102], seen[1102];
  memset(seen, 0, sizeof seen);
  int qh = 0, qt = 0;
  q[qt++] = s;
  seen[nid(s)] = 1;
  par[nid(s)] = -100;
  while (qh < qt) {
    int n = q[qh++];
    if (n == t) {
      int len = 0, c = t;
      int tmp[1102];
      while (c != -100) {
        tmp[len++] = c;
        c = par[nid(c)];
      }
      for (int i = 0; i < len; i++) path[i] = tmp[len - 1 - i];
      return len;
    }
    int k = g->key_of[nid(n)];
    if (k < 0) continue;
    for (int i = 0; i < g->ndst[k]; i++) {
      int m = g->dst[k][i];
      if (!seen[nid(m)]) {
        seen[nid(m)] = 1;
        par[nid(m)] = n;
        q[qt++] = m;
      }
    }
  }
  return 0;
}

/* pgtg/map_generator.py:602-626 */
static void rand_pos(orc_env* e, pcg_t* r, int* x, int* y) {
  int w = e->cfg.width, h = e->cfg.height;
  switch ((int)gen_integers(r, 0, 4)) {
    case 0: *x = (int)gen_integers(r, 0, w); *y = 0; break;
    case 1: *x = w - 1; *y = (int)gen_integers(r, 0, h); break;
    case 2: *x = (int)gen_integers(r, 0, w); *y = h - 1; break;
    default: *x = 0; *y = (int)gen_integers(r, 0, h); break;
  }
}
/* pgtg/map_generator.py:574-599 */
static int rand_dir(orc_env* e, pcg_t* r, int x, int y) {
  int w = e->cfg.width, h = e->cfg.height, opts[4], n = 0;
  if (y == 0) opts[n++] = 0;
  if (x == w - 1) opts[n++] = 1;
  if (y == h - 1) opts[n++] = 2;
  if (x == 0) opts[n++] = 3;
  return opts[gen_integers(r, 0, n)];
}

/* pgtg/map_generator.py:475-571 */
static void choose_start_goal(orc_env* e, pcg_t* r, int s[3], int* slen, int gl[3], int* glen) {
  const orc_config* c = &e->cfg;
  int w = c->width, h = c->height;
  if (c->start_mode == 2) {
    rand_pos(e, r, &s[0], &s[1]);
    *slen = 2;
  } else {
    s[0] = c->start_x != -1 ? c->start_x : w - 1;
    s[1] = c->start_y != -1 ? c->start_y : h - 1;
    *slen = c->start_mode == 1 ? 2 : 3;
    s[2] = c->start_dir;
  }
  if (c->goal_mode == 2) {
    rand_pos(e, r, &gl[0], &gl[1]);
    *glen = 2;
  } else {
    gl[0] = c->goal_x != -1 ? c->goal_x : w - 1;
    gl[1] = c->goal_y != -1 ? c->goal_y : h - 1;
    *glen = c->goal_mode == 1 ? 2 : 3;
    gl[2] = c->goal_dir;
  }
  if (c->min_distance >= 0) {
    while (abs(s[0] - gl[0]) + abs(s[1] - gl[1]) < c->min_distance) {
      rand_pos(e, r, &s[0], &s[1]);
      *slen = 2;
      rand_pos(e, r, &gl[0], &gl[1]);
      *glen = 2;
    }
  }
  if (*slen == 2) {
    s[2] = rand_dir(e, r, s[0], s[1]);
    *slen = 3;
  }
  if (*glen == 2) {
    gl[2] = rand_dir(e, r, gl[0], gl[1]);
    *glen = 3;
  }
  while (s[0] == gl[0] && s[1] == gl[1] && s[2] == gl[2]) {
    if (c->start_mode == 2) rand_pos(e, r, &s[0], &s[1]);
    if (c->start_mode == 2 || c->start_mode == 1) s[2] = rand_dir(e, r, s[0], s[1]);
    if (c->goal_mode == 2) rand_pos(e, r, &gl[0], &gl[1]);
    if (c->goal_mode == 2 || c->goal_mode == 1) gl[2] = rand_dir(e, r, gl[0], gl[1]);
    if (c->start_mode == 0 && c->goal_mode == 0) break; /* validated on host; avoid a hang */
  }
}

static double py_round(double x) { return nearbyint(x); } /* round-half-even (default FE mode) */

static int generate_map(orc_env* e) {
  const orc_config* c = &e->cfg;
  int w = c->width, h = c->height;
  pcg_t* r = &e->map_rng;
  int s[3], g3[3], sl, gl;
  choose_start_goal(e, r, s, &sl, g3, &gl);
  /* generate_map_graph, pgtg/map_generator.py:192-266 */
  graph_t* Gp = (graph_t*)malloc(sizeof(graph_t));
#define G (*Gp)
  g_init(&G);
  for (int x = 0; x < w; x++)
    for (int y = 0; y < h; y++) {
      if (x < w - 1) {
        g_add1(&G, y * w + x, y * w + x + 1);
        g_add1(&G, y * w + x + 1, y * w + x);
      }
      if (y < h - 1) {
        g_add1(&G, y * w + x, (y + 1) * w + x);
        g_add1(&G, (y + 1) * w + x, y * w + x);
      }
    }
  edge_t* rem = (edge_t*)malloc(sizeof(edge_t) * 2200);
  int nrem = 0;
  for (int k = 0; k < G.n_keys; k++)
    for (int i = 0; i < G.ndst[k]; i++) rem[nrem++] = (edge_t){G.keys[k], G.dst[k][i]};
  int st = s[1] * w + s[0], en = g3[1] * w + g3[0];
  g_add1(&G, -1, st);
  g_add1(&G, st, -1);
  g_add1(&G, -2, en);
  g_add1(&G, en, -2);
  int keep = (int)py_round((double)nrem * c->pct_connections);
  int path[1102];
  int plen = g_bfs(&G, -1, -2, path);
  while (G.count - 4 > keep && nrem > 0) {
    int idx = (int)gen_integers(r, 0, nrem);
    edge_t ch = rem[idx];
    /* removable_edges.remove(chosen); .remove(reverse) -- first occurrences */
    for (int pass = 0; pass < 2; pass++) {
      edge_t t = pass == 0 ? ch : (edge_t){ch.b, ch.a};
      for (int i = 0; i < nrem; i++)
        if (rem[i].a == t.a && rem[i].b == t.b) {
          memmove(&rem[i], &rem[i + 1], sizeof(edge_t) * (size_t)(nrem - i - 1));
          nrem--;
          break;
        }
    }
    g_del1(&G, ch.a, ch.b);
    g_del1(&G, ch.b, ch.a);
    int ina = 0, inb = 0;
    for (int i = 0; i < plen; i++) {
      if (path[i] == ch.a) ina = 1;
      if (path[i] == ch.b) inb = 1;
    }
    if (ina && inb) {
      int p2[1102];
      int l2 = g_bfs(&G, -1, -2, p2);
      if (l2) {
        memcpy(path, p2, sizeof(int) * (size_t)l2);
        plen = l2;
      } else {
        g_add1(&G, ch.a, ch.b);
        g_add1(&G, ch.b, ch.a);
      }
    }
  }
  /* map_graph_to_tile_map_object, pgtg/map_generator.py:269-334 */
  e->tw = w;
  e->th = h;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      int t = y * w + x, ex = 0;
      if (y > 0 && g_has(&G, t, t - w)) ex |= 1;
      if (x < w - 1 && g_has(&G, t, t + 1)) ex |= 2;
      if (y < h - 1 && g_has(&G, t, t + w)) ex |= 4;
      if (x > 0 && g_has(&G, t, t - 1)) ex |= 8;
      e->exits[t] = (uint8_t)ex;
      e->otype[t] = -1;
      e->omask[t] = -1;
    }
  free(rem);
#undef G
  free(Gp);
  e->exits[st] |= (uint8_t)(1 << s[2]);
  e->exits[en] |= (uint8_t)(1 << g3[2]);
  for (int i = 0; i < 3; i++) {
    e->start[i] = s[i];
    e->goal[i] = g3[i];
  }
  /* add_connections_to_borders, pgtg/map_generator.py:337-371 ; entries (tile_y, tile_x, dir) */
  int (*conn)[3] = (int (*)[3])malloc(sizeof(int) * 3 * 4096);
  int nc = 0;
  for (int x = 0; x < w; x++) { conn[nc][0] = 0; conn[nc][1] = x; conn[nc][2] = 0; nc++; }
  for (int y = 0; y < h; y++) { conn[nc][0] = y; conn[nc][1] = w - 1; conn[nc][2] = 1; nc++; }
  for (int x = 0; x < w; x++) { conn[nc][0] = h - 1; conn[nc][1] = x; conn[nc][2] = 2; nc++; }
  for (int y = 0; y < h; y++) { conn[nc][0] = y; conn[nc][1] = 0; conn[nc][2] = 3; nc++; }
  int rm[2][3] = {{h - 1, 0, 3}, {0, w - 1, 1}};
  for (int k = 0; k < 2; k++)
    for (int i = 0; i < nc; i++)
      if (conn[i][0] == rm[k][0] && conn[i][1] == rm[k][1] && conn[i][2] == rm[k][2]) {
        memmove(&conn[i], &conn[i + 1], sizeof(conn[0]) * (size_t)(nc - i - 1));
        nc--;
        break;
      }
  int nadd = (int)py_round((double)nc * c->pct_connections);
  for (int k = 0; k < nadd; k++) {
    int idx = (int)gen_integers(r, 0, nc);
    int ty = conn[idx][0], tx = conn[idx][1], d = conn[idx][2];
    memmove(&conn[idx], &conn[idx + 1], sizeof(conn[0]) * (size_t)(nc - idx - 1));
    nc--;
    e->exits[ty * w + tx] |= (uint8_t)(1 << d);
  }
  /* add_obstacles_to_map, pgtg/map_generator.py:374-472 */
  if (c->obstacle_probability > 0) {
    double ws = c->w_ice + c->w_broken + c->w_sand + c->w_tl;
    double p[4] = {c->w_ice / ws, c->w_broken / ws, c->w_sand / ws, c->w_tl / ws};
    for (int row = 0; row < h; row++)
      for (int col = 0; col < w; col++) {
        int t = row * w + col;
        if (pcg_double(r) < c->obstacle_probability && e->exits[t] != 0) {
          int ot = gen_choice_p(r, p, 4);
          e->otype[t] = (int8_t)ot;
          if (ot != 3) {
            e->omask[t] = (int8_t)gen_integers(r, 0, 8);
          } else {
            int opts[6], n = 0, ex = e->exits[t];
            int nex = __builtin_popcount((unsigned)ex);
            if (ex & 1) opts[n++] = 8;
            if (ex & 2) opts[n++] = 9;
            if (ex & 4) opts[n++] = 10;
            if (ex & 8) opts[n++] = 11;
            if ((ex & 1) && (ex & 4) && nex >= 3) opts[n++] = 12;
            if ((ex & 2) && (ex & 8) && nex >= 3) opts[n++] = 13;
            e->omask[t] = (int8_t)opts[gen_integers(r, 0, n)];
          }
        }
      }
  }
  free(conn);
  return 0;
}

/* ----------------------------------------------------------------------------------------------
 * parse_map_object (pgtg/parser.py:13-166) + EpisodeMap scans (pgtg/map.py:11-42)
 * -------------------------------------------------------------------------------------------- */
static int find_direction(int a, int b, int w) { /* pgtg/parser.py:279-306 */
  int ax = a % w, ay = a / w, bx = b % w, by = b / w;
  if (ay == by) {
    if (ax - bx < 0) return 1;
    if (ax - bx > 0) return 3;
  }
  if (ax == bx) {
    if (ay - by < 0) return 2;
    if (ay - by > 0) return 0;
  }
  return -1;
}

/* graph-theory shortest_path: heap Dijkstra, (cost, insertion counter) order (== FIFO BFS for unit
 * weights), neighbours in edge insertion order: N, E, S, W per tile (pgtg/parser.py:254-275). */
static int shortest_path(orc_env* e, int s, int t, int* out) {
  int w = e->tw, h = e->th, n = w * h;
  int* par = (int*)malloc(sizeof(int) * (size_t)n);
  int* state = (int*)calloc((size_t)n, sizeof(int)); /* 0 new 1 queued 2 visited */
  int* q = (int*)malloc(sizeof(int) * (size_t)n);
  int qh = 0, qt = 0, len = 0;
  q[qt++] = s;
  state[s] = 1;
  par[s] = -1;
  while (qh < qt) {
    int v = q[qh++];
    if (state[v] == 2) continue;
    state[v] = 2;
    if (v == t) {
      int c = t, tmp_len = 0;
      while (c != -1) {
        out[tmp_len++] = c;
        c = par[c];
      }
      for (int i = 0; i < tmp_len / 2; i++) {
        int z = out[i];
        out[i] = out[tmp_len - 1 - i];
        out[tmp_len - 1 - i] = z;
      }
      len = tmp_len;
      break;
    }
    int x = v % w, y = v / w, ex = e->exits[v];
    int nb[4], nn = 0;
    if ((ex & 1) && y > 0) nb[nn++] = v - w;
    if ((ex & 2) && x < w - 1) nb[nn++] = v + 1;
    if ((ex & 4) && y < h - 1) nb[nn++] = v + w;
    if ((ex & 8) && x > 0) nb[nn++] = v - 1;
    for (int i = 0; i < nn; i++) {
      int m = nb[i];
      if (state[m] != 0) continue; /* visited, or queued at <= cost */
      state[m] = 1;
      par[m] = v;
      q[qt++] = m;
    }
  }
  free(par);
  free(state);
  free(q);
  return len;
}

static int compile_map(orc_env* e) {
  int w = e->tw, h = e->th;
  free_map(e);
  e->W = w * TILE;
  e->H = h * TILE;
  e->sq = (uint64_t*)calloc((size_t)e->W * e->H, sizeof(uint64_t));
  int st = e->start[1] * w + e->start[0], en = e->goal[1] * w + e->goal[0];
  e->path_len = shortest_path(e, st, en, e->path);
  if (e->path_len == 0) return fail(e, "no path from start to goal");
  for (int i = 0; i < w * h; i++) e->tile_dir[i] = -1;
  for (int i = 0; i + 1 < e->path_len; i++) e->tile_dir[e->path[i]] = find_direction(e->path[i], e->path[i + 1], w);
  for (int tx = 0; tx < w; tx++)
    for (int ty = 0; ty < h; ty++) {
      int t = ty * w + tx, ex = e->exits[t];
      uint64_t tile[81];
      for (int i = 0; i < 81; i++) tile[i] = ORC_TILES[ex][i];
      int on_path_not_last = 0;
      for (int i = 0; i + 1 < e->path_len; i++)
        if (e->path[i] == t) on_path_not_last = 1;
      /* replace_features_in_tile(old, new): pgtg/parser.py:169-190 */
#define REPLACE(oldbit, newbit)                \
  for (int i = 0; i < 81; i++)                 \
    if (tile[i] & (oldbit)) {                  \
      tile[i] &= ~(oldbit);                    \
      tile[i] |= (newbit);                     \
    }
      if (on_path_not_last) { REPLACE(1ull << (F_EXIT0 + e->tile_dir[t]), F_SUBGOAL); }
      if (t == e->path[0]) { REPLACE(1ull << (F_EXIT0 + e->start[2]), F_START); }
      if (t == e->path[e->path_len - 1]) { REPLACE(1ull << (F_EXIT0 + e->goal[2]), F_FINAL); }
      for (int i = 0; i < 81; i++) tile[i] &= ~F_EXITS;
      if (e->otype[t] >= 0) { /* add_obstacles_to_tile, pgtg/parser.py:193-209 */
        static const uint64_t obit[4] = {F_ICE, F_BROKEN, F_SAND, F_TLIGHT};
        if (e->omask[t] < 0) return fail(e, "obstacle type without obstacle mask");
        for (int i = 0; i < 81; i++)
          if (ORC_OBST[e->omask[t]][i] && !(tile[i] & F_WALL)) tile[i] |= obit[(int)e->otype[t]];
      }
      if (ex != 0)
        for (int i = 0; i < 81; i++) tile[i] |= ORC_LANES[ex][i];
      /* border car spawners, pgtg/parser.py:120-148 (keep_old_features=True) */
      for (int i = 0; i < 81; i++) {
        if (tx == 0 && (tile[i] & (1ull << (LANE_ALL_UP + 3)))) tile[i] |= F_SPAWNER;
        if (tx == w - 1 && (tile[i] & (1ull << (LANE_ALL_UP + 2)))) tile[i] |= F_SPAWNER;
        if (ty == 0 && (tile[i] & (1ull << (LANE_ALL_UP + 1)))) tile[i] |= F_SPAWNER;
        if (ty == h - 1 && (tile[i] & (1ull << (LANE_ALL_UP + 0)))) tile[i] |= F_SPAWNER;
      }
      for (int lx = 0; lx < TILE; lx++)
        for (int ly = 0; ly < TILE; ly++) e->sq[(tx * TILE + lx) * e->H + ty * TILE + ly] = tile[lx * 9 + ly];
    }
  e->tile_dir[e->path[e->path_len - 1]] = e->goal[2];
  e->num_subgoals = e->path_len;
  /* EpisodeMap constructor scans, x-major (pgtg/map.py:31-42) */
  int n = e->W * e->H;
  e->starters = (int*)malloc(sizeof(int) * (size_t)n);
  e->spawnable = (int*)malloc(sizeof(int) * (size_t)n);
  e->spawners = (int*)malloc(sizeof(int) * (size_t)n);
  e->n_starters = e->n_spawnable = e->n_spawners = 0;
  for (int x = 0; x < e->W; x++)
    for (int y = 0; y < e->H; y++) {
      uint64_t f = F(e, x, y);
      int code = x * e->H + y;
      if (f & F_START) e->starters[e->n_starters++] = code;
      if (f & F_LANE_MASK) e->spawnable[e->n_spawnable++] = code;
      if (f & F_SPAWNER) e->spawners[e->n_spawners++] = code;
    }
  int vw = e->W + 4, vh = e->H + 4;
  e->visited = (int*)calloc((size_t)vw * vh, sizeof(int));
  return 0;
}

/* ----------------------------------------------------------------------------------------------
 * traffic (pgtg/environment.py:658-691, 830-1015)
 * -------------------------------------------------------------------------------------------- */
/* sorted non-"all" routes at a square (with duplicates), ascending lane id == sorted strings */
static int routes_at(const orc_env* e, int x, int y, int* out) {
  uint64_t f = F(e, x, y);
  int n = 0;
  for (int l = 0; l < 28; l++)
    if (f & (1ull << l)) out[n++] = l;
  return n;
}
static int lane_route_id_slow(int lane) {
  const char* s = ORC_LANE_NAMES[lane] + 9; /* skip "car_lane " */
  for (int r = 0; r < 20; r++) {
    size_t L = strlen(ORC_ROUTE_NAMES[r]);
    if (strncmp(s, ORC_ROUTE_NAMES[r], L) == 0 && s[L] == ' ') return r;
  }
  return -1;
}
static int lane_type_id_slow(int lane) {
  const char* s = strrchr(ORC_LANE_NAMES[lane], ' ') + 1;
  if (!strcmp(s, "up")) return 0;
  if (!strcmp(s, "down")) return 1;
  if (!strcmp(s, "left")) return 2;
  return 3;
}

static int LR[32], LT[32], lane_init;
static void init_lanes(void) {
  if (lane_init) return;
  for (int l = 0; l < 32; l++) {
    LR[l] = lane_route_id_slow(l);
    LT[l] = lane_type_id_slow(l);
  }
  lane_init = 1;
}
static int lane_route_id(int l) { return LR[l]; }
static int lane_type_id(int l) { return LT[l]; }

static void push_car(orc_env* e, car_t c) {
  if (e->ncars == e->capcars) {
    e->capcars = e->capcars ? e->capcars * 2 : 64;
    e->cars = (car_t*)realloc(e->cars, sizeof(car_t) * (size_t)e->capcars);
  }
  e->cars[e->ncars++] = c;
}

static int select_profile(orc_env* e) { return gen_choice_p(&e->car_rng, e->profile_p, 5); }

static int create_initial_traffic(orc_env* e) {
  int np = e->n_spawnable;
  int ncars = (int)((double)np * e->cfg.traffic_density);
  if (ncars > 0 && np > 0) {
    int k = ncars < np ? ncars : np;
    int64_t* idx = (int64_t*)malloc(sizeof(int64_t) * (size_t)k);
    gen_choice_noreplace(&e->car_rng, np, k, idx);
    for (int i = 0; i < k; i++) {
      int code = e->spawnable[idx[i]];
      int x = code / e->H, y = code % e->H, rl[8];
      int nr = routes_at(e, x, y, rl);
      if (nr == 0) {
        free(idx);
        return fail(e, "a car was spawned on a field where no car lane was found");
      }
      int prof = select_profile(e);
      int lane = rl[gen_integers(&e->car_rng, 0, nr)];
      push_car(e, (car_t){e->next_car_id++, x, y, lane_route_id(lane), prof, 0, 0});
    }
    free(idx);
  }
  return 0;
}

static int phase_of(const orc_env* e) { /* 0 green 1 yellow 2 red, pgtg/environment.py:1004-1015 */
  const int* d = e->cfg.phase_dur;
  if (e->phase < d[0]) return 0;
  if (e->phase < d[0] + d[1]) return 1;
  return 2;
}

static int should_car_move(orc_env* e, car_t* c) { /* :678-691 */
  const behavior_t* b = &BEHAVIORS[c->profile];
  if (c->delay > 0) {
    c->delay -= 1;
    return 0;
  }
  if (pcg_double(&e->car_rng) < b->reaction_delay) {
    c->delay = (int)gen_integers(&e->car_rng, 1, 4);
    return 0;
  }
  return pcg_double(&e->car_rng) < b->speed_mult;
}

/* returns 1 with new (x,y,route) or 0 for None; :881-968 */
static int next_car_position(orc_env* e, car_t* c, int* nx, int* ny, int* nroute) {
  if (!should_car_move(e, c)) {
    c->patience += 1;
    *nx = c->x; *ny = c->y; *nroute = c->route;
    return 1;
  }
  const behavior_t* b = &BEHAVIORS[c->profile];
  const int cand[4][2] = {{c->x, c->y - 1}, {c->x, c->y + 1}, {c->x - 1, c->y}, {c->x + 1, c->y}};
  for (int t = 0; t < 4; t++) {
    int px = cand[t][0], py = cand[t][1];
    if (!inside(e, px, py)) continue;
    uint64_t f = F(e, px, py);
    int all_lane = -1;
    for (int l = 28; l < 32; l++)
      if (f & (1ull << l)) all_lane = l;
    if (all_lane >= 0 && lane_type_id(all_lane) == t) {
      int rl[8], nr = routes_at(e, px, py, rl);
      c->patience = 0;
      if (nr == 0) return -2; /* numpy choice([]) -> ValueError */
      int lane = rl[gen_integers(&e->car_rng, 0, nr)];
      *nx = px; *ny = py; *nroute = lane_route_id(lane);
      return 1;
    }
    for (int l = 0; l < 28; l++) {
      if (!(f & (1ull << l))) continue;
      if (lane_route_id(l) != c->route || lane_type_id(l) != t) continue;
      if (f & F_TLIGHT) {
        int ph = phase_of(e), stop;
        if (ph == 0) stop = 0;
        else if (ph == 1) stop = pcg_double(&e->car_rng) < b->yellow_stop;
        else stop = pcg_double(&e->car_rng) >= b->red_violation;
        if (stop) { /* phase is red or yellow here */
          c->patience += 1;
          *nx = c->x; *ny = c->y; *nroute = c->route;
          return 1;
        }
      }
      int occupied = 0;
      for (int i = 0; i < e->ncars; i++)
        if (e->cars[i].x == px && e->cars[i].y == py) occupied = 1;
      if (occupied) {
        if (b->min_follow == 0 || (double)c->patience > b->patience_level * 10) {
          if (pcg_double(&e->car_rng) < (1.0 - b->patience_level)) {
            c->patience = 0;
            *nx = px; *ny = py; *nroute = c->route;
            return 1;
          }
        }
        c->patience += 1;
        *nx = c->x; *ny = c->y; *nroute = c->route;
        return 1;
      }
      c->patience = 0;
      *nx = px; *ny = py; *nroute = c->route;
      return 1;
    }
  }
  c->patience += 1;
  return 0;
}

static int spawn_new_car(orc_env* e, car_t* out) { /* :970-1002 */
  int x = 0, y = 0;
  if (e->n_spawners > 0) {
    int code = e->spawners[gen_integers(&e->car_rng, 0, e->n_spawners)];
    x = code / e->H;
    y = code % e->H;
  }
  int rl[8], nr = routes_at(e, x, y, rl);
  int prof = select_profile(e);
  if (nr == 0) return fail(e, "spawn square has no route (numpy choice of empty list)");
  int lane = rl[gen_integers(&e->car_rng, 0, nr)];
  *out = (car_t){e->next_car_id++, x, y, lane_route_id(lane), prof, 0, 0};
  return 0;
}

static int move_cars(orc_env* e) { /* :1121-1127 */
  int n0 = e->ncars;
  int* ids = (int*)malloc(sizeof(int) * (size_t)(n0 + 1));
  for (int i = 0; i < n0; i++) ids[i] = e->cars[i].id;
  for (int k = 0; k < n0; k++) {
    int i = 0;
    while (e->cars[i].id != ids[k]) i++; /* the snapshot's car object */
    int nx, ny, nr;
    int r = next_car_position(e, &e->cars[i], &nx, &ny, &nr);
    if (r == -2) {
      free(ids);
      return fail(e, "all-lane square without routes (numpy choice of empty list)");
    }
    if (r == 0) {
      memmove(&e->cars[i], &e->cars[i + 1], sizeof(car_t) * (size_t)(e->ncars - i - 1));
      e->ncars--;
      car_t nc;
      if (spawn_new_car(e, &nc)) {
        free(ids);
        return -1;
      }
      push_car(e, nc);
    } else {
      e->cars[i].x = nx;
      e->cars[i].y = ny;
      e->cars[i].route = nr;
    }
  }
  free(ids);
  return 0;
}

/* ----------------------------------------------------------------------------------------------
 * braking rules (pgtg/environment.py:162-294, 1037-1090)
 * -------------------------------------------------------------------------------------------- */
/* returns compass index 0..7 or -1 (all zeros) */
static int compass(const orc_env* e, int x, int y) {
  int best = -1, bx = 0, by = 0;
  long bd = 0;
  for (int tx = 0; tx < e->W; tx++)
    for (int ty = 0; ty < e->H; ty++)
      if (F(e, tx, ty) & (F_SUBGOAL | F_FINAL)) {
        long d = labs((long)tx - x) + labs((long)ty - y);
        if (best < 0 || d < bd) {
          best = 1;
          bd = d;
          bx = tx;
          by = ty;
        }
      }
  if (best < 0) return -1;
  int dx = bx - x, dy = by - y, s = e->cfg.sliding_size;
  if (abs(dx) <= s && abs(dy) <= s) return -1;
  double angle = atan2((double)dy, (double)dx);
  double P8 = M_PI / 8;
  if (-P8 <= angle && angle < P8) return 2;
  if (P8 <= angle && angle < 3 * P8) return 3;
  if (3 * P8 <= angle && angle < 5 * P8) return 4;
  if (5 * P8 <= angle && angle < 7 * P8) return 5;
  if (angle >= 7 * P8 || angle < -7 * P8) return 6;
  if (-7 * P8 <= angle && angle < -5 * P8) return 7;
  if (-5 * P8 <= angle && angle < -3 * P8) return 0;
  if (-3 * P8 <= angle && angle < -P8) return 1;
  return -1;
}

static int apply_braking(orc_env* e) {
  if (e->cfg.n_rules == 0) return 0;
  int tx = (int)floor((double)e->px / TILE), ty = (int)floor((double)e->py / TILE);
  if (tx < 0) tx = 0;
  if (tx > e->tw - 1) tx = e->tw - 1;
  if (ty < 0) ty = 0;
  if (ty > e->th - 1) ty = e->th - 1;
  int ex = e->exits[ty * e->tw + tx];
  double speed = sqrt((double)e->vx * e->vx + (double)e->vy * e->vy);
  int triggered = 0;
  for (int ri = 0; ri < e->cfg.n_rules; ri++) {
    const orc_rule* r = &e->cfg.rules[ri];
    if (r->tile_exits != ex) continue;
    if (!(r->vel_lo <= speed && speed <= r->vel_hi)) continue;
    int n_in = 0;
    for (int i = 0; i < e->ncars; i++)
      if (e->cars[i].x / TILE == tx && e->cars[i].y / TILE == ty) n_in++;
    if (n_in < r->min_traffic) continue;
    int cp = compass(e, e->px, e->py), dir;
    if (cp >= 0) dir = (cp <= 1) ? 0 : (cp <= 3) ? 1 : (cp <= 5) ? 2 : 3;
    else dir = speed < 0.1 ? 4 : 5;
    int match = 0;
    for (int i = 0; i < e->ncars; i++)
      if (e->cars[i].x / TILE == tx && e->cars[i].y / TILE == ty) match += r->weight[dir][e->cars[i].route];
    if (match < r->min_matching_traffic) continue;
    triggered |= 1 << ri; /* rule_triggers: every rule is evaluated */
  }
  return triggered;
}

/* ----------------------------------------------------------------------------------------------
 * observation (pgtg/environment.py:1344-1536) and used-subgoal flood fill (pgtg/map.py:143-171)
 * -------------------------------------------------------------------------------------------- */
static void set_subgoals_to_used(orc_env* e, int x, int y) {
  e->sq[x * e->H + y] &= ~F_SUBGOAL;
  e->sq[x * e->H + y] |= F_USED;
  /* (the reference's feature_at would raise outside the map; subgoal squares never touch it) */
  if (inside(e, x, y + 1) && (F(e, x, y + 1) & F_SUBGOAL)) set_subgoals_to_used(e, x, y + 1);
  if (inside(e, x, y - 1) && (F(e, x, y - 1) & F_SUBGOAL)) set_subgoals_to_used(e, x, y - 1);
  if (inside(e, x + 1, y) && (F(e, x + 1, y) & F_SUBGOAL)) set_subgoals_to_used(e, x + 1, y);
  if (inside(e, x - 1, y) && (F(e, x - 1, y) & F_SUBGOAL)) set_subgoals_to_used(e, x - 1, y);
}

static int ch_value(const orc_env* e, int code, uint64_t f, int ph) {
  switch (code) {
    case ORC_CH_WALL: return (f & F_WALL) != 0;
    case ORC_CH_GOALS: return (f & (F_SUBGOAL | F_FINAL)) != 0;
    case ORC_CH_TL_GREEN: return ph == 0 && (f & F_TLIGHT);
    case ORC_CH_TL_YELLOW: return ph == 1 && (f & F_TLIGHT);
    case ORC_CH_TL_RED: return ph == 2 && (f & F_TLIGHT);
    case ORC_CH_START: return (f & F_START) != 0;
    case ORC_CH_SUBGOAL: return (f & F_SUBGOAL) != 0;
    case ORC_CH_USED_SUBGOAL: return (f & F_USED) != 0;
    case ORC_CH_FINAL_GOAL: return (f & F_FINAL) != 0;
    case ORC_CH_ICE: return (f & F_ICE) != 0;
    case ORC_CH_BROKEN: return (f & F_BROKEN) != 0;
    case ORC_CH_SAND: return (f & F_SAND) != 0;
    case ORC_CH_SPAWNER: return (f & F_SPAWNER) != 0;
    default:
      if (code >= ORC_CH_LANE0 && code < ORC_CH_LANE0 + 32) return (f >> (code - ORC_CH_LANE0)) & 1;
      return 0;
  }
}

static void observe(orc_env* e, uint8_t* obs, orc_out* out) {
  const orc_config* c = &e->cfg;
  int pix = e->px < 0 ? 0 : e->px, piy = e->py < 0 ? 0 : e->py;
  if (pix > e->W - 1) pix = e->W - 1;
  if (piy > e->H - 1) piy = e->H - 1;
  int tx = pix / TILE, ty = piy / TILE;
  int x0, y0, win = orc_window(e);
  if (!c->sliding) {
    x0 = tx * TILE;
    y0 = ty * TILE;
  } else {
    x0 = e->px - c->sliding_size;
    y0 = e->py - c->sliding_size;
  }
  int ph = phase_of(e);
  for (int ci = 0; ci < c->n_channels; ci++) {
    int code = c->channels[ci];
    uint8_t* o = obs + (size_t)ci * win * win;
    for (int i = 0; i < win; i++)
      for (int j = 0; j < win; j++) {
        int x = x0 + i, y = y0 + j, v;
        if (code == ORC_CH_TRAFFIC) {
          v = 0;
        } else if (inside(e, x, y)) {
          v = ch_value(e, code, F(e, x, y), ph);
        } else {
          v = c->sliding ? ch_value(e, code, F_WALL, ph) : 0;
        }
        o[i * win + j] = (uint8_t)v;
      }
    if (code == ORC_CH_TRAFFIC)
      for (int k = 0; k < e->ncars; k++) {
        int x = e->cars[k].x, y = e->cars[k].y;
        if (x0 <= x && x <= x0 + win - 1 && y0 <= y && y <= y0 + win - 1) o[(x - x0) * win + (y - y0)] = 1;
      }
  }
  out->pos[0] = c->sliding ? c->sliding_size : pix - x0;
  out->pos[1] = c->sliding ? c->sliding_size : piy - y0;
  out->vel[0] = e->vx;
  out->vel[1] = e->vy;
  out->next_subgoal_direction = -1;
  if (c->next_subgoal) {
    int nsd = e->tile_dir[ty * e->tw + tx]; /* get_next_subgoal_direction, pgtg/map.py:120-141 */
    if (nsd == -1 || c->sliding) {
      int found = 0, bx = 0, by = 0;
      long bd = 0;
      for (int x = 0; x < e->W; x++)
        for (int y = 0; y < e->H; y++)
          if (F(e, x, y) & (F_SUBGOAL | F_FINAL)) {
            long d = labs((long)x - pix) + labs((long)y - piy);
            if (!found || d < bd) {
              found = 1;
              bd = d;
              bx = x;
              by = y;
            }
          }
      if (found) {
        int dx = bx - pix, dy = by - piy;
        double angle = atan2(-(double)dy, (double)dx);
        double q = (angle + M_PI) / (M_PI / 4);
        double m = fmod(q, 8.0);
        if (m < 0) m += 8.0;
        static const int remap[8] = {2, 1, 0, 7, 6, 5, 4, 3};
        nsd = remap[(int)m];
      }
    }
    out->next_subgoal_direction = nsd;
  }
}

/* ----------------------------------------------------------------------------------------------
 * reset / step
 * -------------------------------------------------------------------------------------------- */
static inline int* vis(orc_env* e, int x, int y) { return &e->visited[(x + 2) * (e->H + 4) + (y + 2)]; }

int orc_reset(orc_env* e, int64_t seed, uint8_t* obs, orc_out* out) {
  const orc_config* c = &e->cfg;
  if (seed >= 0) { /* gym.Env.reset(seed): np_random = Generator(PCG64(SeedSequence(seed))) */
    e->seeded = 1;
    e->seed = (uint64_t)seed;
    e->spawn_counter = 0;
  }
  if (!e->seeded) return fail(e, "first reset must be seeded");
  /* self.np_random.spawn(5), pgtg/environment.py:593-599 */
  uint32_t k = e->spawn_counter;
  pcg_from_seed(&e->map_rng, e->seed, 1, k + 0);
  pcg_from_seed(&e->car_rng, e->seed, 1, k + 1);
  pcg_from_seed(&e->ice_rng, e->seed, 1, k + 2);
  pcg_from_seed(&e->broken_rng, e->seed, 1, k + 3);
  pcg_from_seed(&e->sand_rng, e->seed, 1, k + 4);
  e->spawn_counter += 5;
  if (c->fixed_map) {
    e->tw = c->fm_w;
    e->th = c->fm_h;
    for (int i = 0; i < e->tw * e->th; i++) {
      e->exits[i] = c->fm_exits[i];
      e->otype[i] = c->fm_obst_type[i];
      e->omask[i] = c->fm_obst_mask[i];
    }
    for (int i = 0; i < 3; i++) {
      e->start[i] = c->fm_start[i];
      e->goal[i] = c->fm_goal[i];
    }
  } else {
    generate_map(e);
  }
  if (compile_map(e)) return -1;
  e->ind_reward = c->sum_subgoals_reward / (double)e->num_subgoals;
  if (e->n_starters == 0) return fail(e, "no start squares");
  int code = e->starters[gen_integers(&e->map_rng, 0, e->n_starters)];
  e->px = code / e->H;
  e->py = code % e->H;
  e->vx = e->vy = 0;
  e->terminated = 0;
  e->flat_tire = 0;
  e->braking = 0;
  *vis(e, e->px, e->py) = 1;
  e->ncars = 0;
  e->next_car_id = 0;
  e->phase = 0;
  if (c->traffic_density > 0)
    if (create_initial_traffic(e)) return -1;
  memset(out, 0, sizeof *out);
  observe(e, obs, out);
  return 0;
}

static int decompose(int dx, int dy, int parts[][2]) { /* pgtg/environment.py:693-748 */
  int res[256][2], n = 0;
  if (dx == 0 && dy == 0) return 0;
  if (dx == 0) {
    int m = dy > 0 ? 1 : -1;
    for (int i = 1; i <= abs(dy); i++) { res[n][0] = 0; res[n][1] = i * m; n++; }
  } else if (dy == 0) {
    int m = dx > 0 ? 1 : -1;
    for (int i = 1; i <= abs(dx); i++) { res[n][0] = i * m; res[n][1] = 0; n++; }
  } else if (abs(dx) >= abs(dy)) {
    double my = (double)dy / (double)abs(dx);
    int mx = dx > 0 ? 1 : -1;
    for (int i = 1; i <= abs(dx); i++) {
      double t = (double)i * my;
      t = t + 0.5;
      res[n][0] = i * mx;
      res[n][1] = (int)floor(t);
      n++;
    }
  } else {
    double mxv = (double)dx / (double)abs(dy);
    int my = dy > 0 ? 1 : -1;
    for (int i = 1; i <= abs(dy); i++) {
      double t = (double)i * mxv;
      t = t + 0.5;
      res[n][1] = i * my;
      res[n][0] = (int)floor(t);
      n++;
    }
  }
  int px = 0, py = 0;
  for (int i = 0; i < n; i++) {
    parts[i][0] = res[i][0] - px;
    parts[i][1] = res[i][1] - py;
    px = res[i][0];
    py = res[i][1];
  }
  return n;
}

int orc_step(orc_env* e, int32_t action, uint8_t* obs, orc_out* out) {
  const orc_config* c = &e->cfg;
  if (e->terminated) return fail(e, "Already done, step has no further effect");
  if (action < 0 || action > 8) return fail(e, "invalid action");
  e->phase = (e->phase + 1) % (c->phase_dur[0] + c->phase_dur[1] + c->phase_dur[2]);
  int ax = ACC[action][0], ay = ACC[action][1];
  if (move_cars(e)) return -1;
  double reward = 0.0, perf = 0.0, cost = 0.0;
  int cx = e->px, cy = e->py;
  e->vx += ax;
  e->vy += ay;
  e->braking = apply_braking(e);
  if (e->braking) e->vx = e->vy = 0;
  if (abs(e->vx) > 255 || abs(e->vy) > 255) return fail(e, "velocity out of supported range");
  int parts[257][2];
  int np = decompose(e->vx, e->vy, parts);
  for (int k = 0; k <= np; k++) { /* the trailing None is k == np */
    int crash = !inside(e, cx, cy) || (F(e, cx, cy) & F_WALL);
    if (!crash && !c->ignore_traffic_collisions)
      for (int i = 0; i < e->ncars; i++)
        if (e->cars[i].x == cx && e->cars[i].y == cy) crash = 1;
    if (crash) {
      if (c->separate_reward_cost) cost += c->crash_penalty;
      else reward -= c->crash_penalty;
      e->terminated = 1;
      break;
    }
    uint64_t f = F(e, cx, cy);
    if (f & F_FINAL) {
      double add = e->ind_reward + c->final_goal_bonus;
      if (c->separate_reward_cost) perf += add;
      else reward += add;
      e->terminated = 1;
      break;
    }
    if (f & F_SUBGOAL) {
      if (c->separate_reward_cost) perf += e->ind_reward;
      else reward += e->ind_reward;
      set_subgoals_to_used(e, cx, cy);
    }
    if (k == np) continue;
    int vx = parts[k][0], vy = parts[k][1];
    int nx = cx + vx, ny = cy + vy;
    if (inside(e, nx, ny) && (F(e, nx, ny) & F_TLIGHT) && phase_of(e) == 2) {
      if (c->separate_reward_cost) cost += c->tl_violation_penalty;
      else reward -= c->tl_violation_penalty;
    }
    f = F(e, cx, cy);
    if ((f & F_ICE) && pcg_double(&e->ice_rng) < c->ice_probability) {
      int a = (int)gen_integers(&e->ice_rng, 0, 9);
      vx = ACC[a][0];
      vy = ACC[a][1];
    }
    if ((f & F_BROKEN) && pcg_double(&e->broken_rng) < c->street_damage_probability) e->flat_tire = 1;
    if ((f & F_SAND) && pcg_double(&e->sand_rng) < c->sand_probability) {
      cx += vx;
      cy += vy;
      e->vx = e->vy = 0;
      break;
    }
    cx += vx;
    cy += vy;
  }
  if (e->flat_tire) e->vx = e->vy = 0;
  int moved_accel = !(ax == 0 && ay == 0);
  if (c->visited_penalty != 0 && moved_accel && *vis(e, cx, cy)) {
    if (c->separate_reward_cost) cost += c->visited_penalty;
    else reward -= c->visited_penalty;
  }
  int ox = e->px, oy = e->py;
  e->px = cx;
  e->py = cy;
  *vis(e, cx, cy) = 1;
  if (c->standing_still_penalty != 0 && !moved_accel && ox == cx && oy == cy) {
    if (c->separate_reward_cost) cost += c->standing_still_penalty;
    else reward -= c->standing_still_penalty;
  }
  memset(out, 0, sizeof *out);
  out->reward = c->separate_reward_cost ? perf : reward;
  out->cost = cost;
  out->terminated = e->terminated;
  out->truncated = 0;
  out->braking = e->braking;
  observe(e, obs, out);
  return 0;
}

/* ----------------------------------------------------------------------------------------------
 * introspection
 * -------------------------------------------------------------------------------------------- */
int orc_num_cars(const orc_env* e) { return e->ncars; }
int orc_get_cars(const orc_env* e, orc_car_out* cars, int cap) {
  int n = e->ncars < cap ? e->ncars : cap;
  for (int i = 0; i < n; i++) {
    const car_t* c = &e->cars[i];
    cars[i] = (orc_car_out){c->id, c->x, c->y, c->route, c->profile, c->patience, c->delay};
  }
  return e->ncars;
}
int orc_get_map_plan(const orc_env* e, int32_t* w, int32_t* h, uint8_t* exits, int8_t* otype,
                     int8_t* omask, int32_t* start3, int32_t* goal3) {
  *w = e->tw;
  *h = e->th;
  for (int i = 0; i < e->tw * e->th; i++) {
    exits[i] = e->exits[i];
    otype[i] = e->otype[i];
    omask[i] = e->omask[i];
  }
  for (int i = 0; i < 3; i++) {
    start3[i] = e->start[i];
    goal3[i] = e->goal[i];
  }
  return 0;
}
int orc_get_misc(const orc_env* e, int32_t* phase, int32_t* flat_tire, int32_t* next_car_id,
                 uint32_t* spawn_counter) {
  *phase = e->phase;
  *flat_tire = e->flat_tire;
  *next_car_id = e->next_car_id;
  *spawn_counter = e->spawn_counter;
  return 0;
}
int orc_set_agent(orc_env* e, int32_t x, int32_t y, int32_t vx, int32_t vy) {
  e->px = x;
  e->py = y;
  e->vx = vx;
  e->vy = vy;
  return 0;
}
/* env.cars.append(Car(id, Position(x, y), route, profile)) of the reference tests; id < 0 takes the
 * next id like _spawn_new_car (environment.py:970-1002), an explicit id leaves _next_car_id alone */
int orc_add_car(orc_env* e, int32_t x, int32_t y, int32_t route, int32_t profile, int32_t id) {
  push_car(e, (car_t){id < 0 ? e->next_car_id++ : id, x, y, route, profile, 0, 0});
  return 0;
}
/* PGTGEnv.set_to_state (environment.py:1301-1342): position, velocity, flat tire; the car list is
 * replaced by fresh Car objects (patience 0, delay 0) and _next_car_id = last id + 1 when the list is
 * non-empty; then get_observation. */
int orc_set_to_state(orc_env* e, int32_t x, int32_t y, int32_t vx, int32_t vy, int32_t flat_tire,
                     const orc_car_out* cars, int32_t n_cars, uint8_t* obs, orc_out* out) {
  e->px = x;
  e->py = y;
  e->vx = vx;
  e->vy = vy;
  e->flat_tire = flat_tire != 0;
  e->ncars = 0;
  for (int k = 0; k < n_cars; k++) push_car(e, (car_t){cars[k].id, cars[k].x, cars[k].y, cars[k].route, cars[k].profile, 0, 0});
  if (n_cars > 0) e->next_car_id = cars[n_cars - 1].id + 1;
  memset(out, 0, sizeof *out);
  observe(e, obs, out);
  return 0;
}
int orc_get_squares(const orc_env* e, uint64_t* out, int cap) {
  int n = e->W * e->H;
  for (int i = 0; i < n && i < cap; i++) out[i] = e->sq[i];
  return n;
}

/* CPU baseline leg of bench.py: n_envs envs, `steps` ticks each with uniform random actions from
 * the same splitmix hash as the GPU action kernel, same-step auto-reset, like the vector env.
 * Returns the number of env-steps executed (or -1). */
int64_t orc_bench(const orc_config* cfg, int n_envs, int steps, uint64_t seed_base, uint64_t act_seed) {
  int64_t done = 0;
  int win = cfg->sliding ? 1 + 2 * cfg->sliding_size : TILE;
  uint8_t* obs = (uint8_t*)malloc((size_t)cfg->n_channels * win * win + 1);
  orc_out out;
  for (int i = 0; i < n_envs; i++) {
    orc_env* e = orc_create(cfg);
    if (orc_reset(e, (int64_t)(seed_base + (uint64_t)i), obs, &out)) {
      orc_destroy(e);
      free(obs);
      return -1;
    }
    for (int t = 0; t < steps; t++) {
      uint64_t z = act_seed ^ ((uint64_t)t * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)i * 0xD1B54A32D192ED03ull);
      z += 0x9E3779B97F4A7C15ull;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      z ^= z >> 31;
      int a = (int)(((z >> 32) * 9ull) >> 32);
      if (orc_step(e, a, obs, &out)) {
        orc_destroy(e);
        free(obs);
        return -1;
      }
      done++;
      if (out.terminated && orc_reset(e, -1, obs, &out)) {
        orc_destroy(e);
        free(obs);
        return -1;
      }
    }
    orc_destroy(e);
  }
  free(obs);
  return done;
}

/* Per-env, per-step digests of a synthetic random-action rollout with same-step auto-reset, for the
 * exhaustive bench-size parity tests (tests/test_gpu_exhaustive.py).  Env i of the batch is global
 * env g = env_offset + i: seeded with g, actions from the splitmix hash of (act_seed, t, g) (the
 * GPU's k_random_actions).  digest[t * n_envs + i] = pgtg_amd/digest.py's formula over that step's
 * outputs: sum of W(j) over the observation's set bytes j, W(D + k) times the small outputs, and the
 * terminal observation's bytes at W(D + 16 + j) when the env finished, and with traffic the car list
 * after the step (dg_cars; all arithmetic mod 2^64). */
static uint64_t dg_w(uint64_t j) {
  uint64_t z = j + 1 + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static uint64_t dg_obs(const uint8_t* obs, int D, uint64_t base) {
  uint64_t d = 0;
  for (int j = 0; j < D; j++)
    if (obs[j]) d += (uint64_t)obs[j] * dg_w(base + (uint64_t)j);
  return d;
}
static uint64_t dg_small(const orc_out* o, int D, int nsd, int cost) {
  uint64_t d = 0, rb, cb;
  memcpy(&rb, &o->reward, 8);
  memcpy(&cb, &o->cost, 8);
  d += (uint64_t)(int64_t)o->pos[0] * dg_w(D + 0) + (uint64_t)(int64_t)o->pos[1] * dg_w(D + 1);
  d += (uint64_t)(int64_t)o->vel[0] * dg_w(D + 2) + (uint64_t)(int64_t)o->vel[1] * dg_w(D + 3);
  d += rb * dg_w(D + 4) + (uint64_t)(o->terminated != 0) * dg_w(D + 5) + (uint64_t)(o->truncated != 0) * dg_w(D + 6);
  if (nsd) d += (uint64_t)(int64_t)o->next_subgoal_direction * dg_w(D + 7);
  if (cost) d += cb * dg_w(D + 8);
  return d;
}
/* car-list term of the digest (traffic handles): W(CB) x n_cars + per car j in list order
 * W(CB + 1 + 2j) x (packed + 1) + W(CB + 2 + 2j) x patience, packed = id | x<<32 | y<<40 | route<<48 |
 * profile<<53 | delay<<56 (pgtg_amd/digest.py car_term, the device's k_car_digest) */
#define DG_CAR_BASE (1ull << 40)
static uint64_t dg_cars(const orc_env* e) {
  uint64_t d = (uint64_t)e->ncars * dg_w(DG_CAR_BASE);
  for (int j = 0; j < e->ncars; j++) {
    const car_t* c = &e->cars[j];
    const uint64_t pk = (uint64_t)(uint32_t)c->id | (uint64_t)c->x << 32 | (uint64_t)c->y << 40 |
                        (uint64_t)c->route << 48 | (uint64_t)c->profile << 53 | (uint64_t)c->delay << 56;
    d += (pk + 1) * dg_w(DG_CAR_BASE + 1 + 2 * (uint64_t)j) + (uint64_t)(int64_t)c->patience * dg_w(DG_CAR_BASE + 2 + 2 * (uint64_t)j);
  }
  return d;
}
int orc_rollout_digest(const orc_config* cfg, int64_t n_envs, uint64_t env_offset, int steps, uint64_t act_seed,
                       uint64_t* digest) {
  int win = cfg->sliding ? 1 + 2 * cfg->sliding_size : TILE;
  int D = cfg->n_channels * win * win;
  uint8_t* obs = (uint8_t*)malloc((size_t)D + 1);
  orc_out out;
  for (int64_t i = 0; i < n_envs; i++) {
    const uint64_t g = env_offset + (uint64_t)i;
    orc_env* e = orc_create(cfg);
    if (orc_reset(e, (int64_t)g, obs, &out)) {
      orc_destroy(e);
      free(obs);
      return -1;
    }
    for (int t = 0; t < steps; t++) {
      uint64_t z = act_seed ^ ((uint64_t)t * 0x9E3779B97F4A7C15ull) ^ (g * 0xD1B54A32D192ED03ull);
      z += 0x9E3779B97F4A7C15ull;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      z ^= z >> 31;
      int a = (int)(((z >> 32) * 9ull) >> 32);
      if (orc_step(e, a, obs, &out)) {
        orc_destroy(e);
        free(obs);
        return -1;
      }
      uint64_t d = 0;
      orc_out step_out = out;
      if (out.terminated) {
        d += dg_obs(obs, D, (uint64_t)D + 16);
        if (orc_reset(e, -1, obs, &out)) {
          orc_destroy(e);
          free(obs);
          return -1;
        }
        /* the vector env reports the step's reward/termination with the new episode's observation */
        step_out.pos[0] = out.pos[0];
        step_out.pos[1] = out.pos[1];
        step_out.vel[0] = out.vel[0];
        step_out.vel[1] = out.vel[1];
        step_out.next_subgoal_direction = out.next_subgoal_direction;
      }
      d += dg_obs(obs, D, 0) + dg_small(&step_out, D, cfg->next_subgoal, cfg->separate_reward_cost);
      if (cfg->traffic_density > 0) d += dg_cars(e);
      digest[(size_t)t * (size_t)n_envs + (size_t)i] = d;
    }
    orc_destroy(e);
  }
  free(obs);
  return 0;
}
