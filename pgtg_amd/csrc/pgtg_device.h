// pgtg_amd/csrc/pgtg_device.h -- device-side data layout and numpy-exact RNG for the batched
// PGTG kernels (gfx950).  One lane owns one environment; all per-env state is structure-of-arrays
// in HBM (coalesced 8/16/32-byte records, see DESIGN.md "Data layout in HBM").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pgtg.h"

namespace pgtg {

constexpr int kTile = 9;
constexpr int kMaxTiles = PGTG_MAX_TILES;
constexpr int kSmallTiles = 64;   // maps of <= 64 tiles: u64 tile masks, edge table and rewards in LDS
constexpr int kMaxEdges = 1024;   // directed interior edges of a <= 256-tile grid (<= 960)
constexpr int kSmallEdges = 256;  // directed interior edges of a <= 64-tile grid (<= 224): the LDS edge table
constexpr int kMaxBorder = 192;   // border-connection candidates (<= 2w+2h-2)
constexpr int kMaxWin = PGTG_MAX_WINDOW;
constexpr int kBlock = 256;       // lanes (= envs) per workgroup for the step kernels
constexpr int kSpCache = 24;      // spawner-list entries k_env keeps in LDS (the rest are read from HBM)

// agent flags (EnvRec.w2 bits 16..23)
constexpr uint32_t kFlagTerminated = 1u << 0;
constexpr uint32_t kFlagFlatTire = 1u << 1;
constexpr uint32_t kFlagBraking = 1u << 2;
constexpr uint32_t kFlagTruncated = 1u << 3;

// per-square feature flags (square_flags)
constexpr uint32_t SQ_WALL = 1u << 0, SQ_SUBGOAL = 1u << 1, SQ_USED = 1u << 2, SQ_FINAL = 1u << 3,
                   SQ_START = 1u << 4, SQ_ICE = 1u << 5, SQ_BROKEN = 1u << 6, SQ_SAND = 1u << 7,
                   SQ_TLIGHT = 1u << 8, SQ_SPAWNER = 1u << 9;

// Tile-plan entry (u16): bits 0-3 exits (N,E,S,W), 4-6 obstacle type (0 none, 1 ice, 2 broken
// road, 3 sand, 4 traffic light), 7-10 obstacle mask id, 11-13 subgoal exit direction + 1, 14 the
// tile's subgoal is used (maps of > 64 tiles; smaller maps keep the used tiles in EnvRec's u64).
constexpr uint32_t kPlanUsed = 1u << 14;
__host__ __device__ inline uint32_t plan_exits(uint32_t p) { return p & 15u; }
__host__ __device__ inline uint32_t plan_otype(uint32_t p) { return (p >> 4) & 7u; }
__host__ __device__ inline uint32_t plan_omask(uint32_t p) { return (p >> 7) & 15u; }
__host__ __device__ inline int plan_sgdir(uint32_t p) { return (int)((p >> 11) & 7u) - 1; }

// EnvRec (32 B, one uint4 pair per env):
//  w0 = px | py<<16 (int16)   w1 = vx | vy<<16 (int16)   w2 = phase | flags<<16 (4 bits) | path_len<<20
//  w3 = elapsed steps         w4 = start_tile | start_dir<<8 | goal_tile<<16 | goal_dir<<24
//  w5 = spawn counter (SeedSequence children spawned)   w6,w7 = used-subgoal tile mask (u64; maps of <= 64
//  tiles, larger maps mark the plan words, kPlanUsed)
struct EnvRec {
  uint4 a, b;
};

struct DevCfg {
  int32_t tw, th, nt, W, H;
  int32_t fixed_map;
  uint32_t fixed_sg;
  int32_t start_mode, goal_mode, sx, sy, sdir, gx, gy, gdir, min_distance;
  int32_t n_edges, keep;
  int32_t dual;       // the edge-removal test runs on the dual (wall) graph: >= 2 x 2, <= 64 tiles, w + h <= 31
  uint64_t h0[4][4];  // full-grid exit masks before removals: h0[64-tile word][N, E, S, W]
  int32_t n_border, n_border_add;
  uint8_t bt[kMaxBorder], bd[kMaxBorder];
  double obstacle_probability;
  uint64_t obst_cdf_t[4];  // obstacle-type CDF as 53-bit thresholds
  double ice_p, broken_p, sand_p;
  int32_t phase_total, phase_g, phase_gy;
  int32_t ignore_collisions, separate_cost, autoreset, max_steps;
  double crash_penalty, final_goal_bonus, tl_penalty, still_penalty, visited_penalty;
  int32_t n_channels, win, sliding, ss, next_subgoal, generic_channels;
  int32_t channels[PGTG_MAX_CHANNELS];
  int32_t need_car, need_ice, need_broken, need_sand;
  uint32_t zero_ch;  // channel codes (< 32) that are all-zero under this config (observation fast path)
  double density;
  uint64_t profile_t[5];  // profile CDF as 53-bit thresholds: random() < cdf[j]  <=>  (next64 >> 11) < t[j]
  int32_t car_cap;      // cars an env can hold (initial traffic <= this; pgtg_add_car / set_to_state limit)
  int32_t kt_serial;    // initial traffic's per-car draws on one lane per env (PgtgConfig.tune_kt_serial)
  int32_t kt_jump_bits; // bound of the jump lengths of the lane-parallel per-car draws (< 2^bits outputs)
  int32_t car_slots;    // car slots per env (>= 2 * car_cap: empty slots + a tick of respawns)
  int32_t max_spawners; // spawner list capacity per env (nt * 5)
  // DRIVER_BEHAVIORS (pgtg/environment.py:64-109) in DriverProfile order, thresholds precomputed
  // random() < p  <=>  (next64 >> 11) < ceil(p * 2^53): probabilities as integer thresholds
  uint64_t beh_t[5][5];  // [BEH_*][profile]
  int32_t beh_min_follow[5], beh_patience_thr[5];  // patience > level*10  <=>  patience > floor(level*10)
  int32_t traf_bytes;      // k_env per-lane LDS traffic region: occupancy counters, spawner cache
  int32_t sp_cache_off;    // byte offset of the spawner cache (kSpCache entries) in it
  int32_t rs_bytes;        // k_traffic per-lane reset scratch: Floyd output [0, 2*cap), seen set, column prefix
  int32_t rs_jj_off;       // the shuffle's draws (u16 x cap)
  int32_t rs_seen_off;
  int32_t rs_pre_off;
  int32_t rs_cm_off;        // per-column masks of spawnable rows (u32 pairs; maps of <= 7 tile rows, else 0)
  int32_t traffic_ch;      // index of the traffic channel in the observation, -1 if absent
  int32_t obs_fast;        // observation window == the agent's tile (k_traffic patches its traffic bits)
  int32_t manual_cars;     // cars may be added through pgtg_add_car
  int32_t n_rules;
  PgtgRule rules[PGTG_MAX_RULES];
  int32_t nsd_off, nsd_pitch;   // nsd table index (dx+off)*pitch + (dy+off)
  int32_t cmp_off, cmp_pitch;   // compass table index
  int32_t vis_pitch, vis_words; // visited bitset: ((x+2)*vis_pitch + (y+2))
  int32_t plan_stride;          // u16 per env in the global tile-plan array (a multiple of 8; of 64, whole
                                // lines, for the map queue's maps)
  int32_t plan_dq;              // 16-byte quads of it that hold tiles ((nt + 7) / 8)
  int32_t obs_bytes;            // n_channels * win * win
  int32_t qrec_dw;              // map-queue entry words (plan_dq * 4 + 4, in whole 128-byte lines)
  int32_t mask_words;           // ceil(win*win/32)
  // per-tile arrays of maps up to 256 tiles, kept behind the fields every launch reads
  uint16_t fixed_plan[kMaxTiles];
  double ind_reward[kMaxTiles + 1];
  int32_t tune_fault;  // PgtgConfig.tune_fault (tests of the kernels' error paths; 0 in every real config)
};

// Lane-indexed constant tables, copied once per workgroup into LDS (pgtg_env.hip): the head (sT:
// 81-bit tile masks, the graph-theory edge order, border candidates, per-path-length rewards) that
// every step kernel reads, and the tail (sTX: lane, traffic, rule and driver tables) that only the
// traffic and lane-channel paths read.  Two LDS objects, so that a kernel that never references the
// tail (k_envq without lane channels) is not allocated its 10 KB.
struct TablesHead {
  uint32_t wall[16][3];     // kTileWall
  uint32_t seg[4][3];       // kExitSeg
  uint32_t obst[14][3];     // kObstMask
  uint32_t spawner[16][3];  // kLaneSpawner
  double ind[kSmallTiles + 1];  // sum_subgoals_reward / num_subgoals (longer paths: DevCfg::ind_reward)
  // removable edges in graph-theory order, oriented: a | b<<8 | horizontal<<16 | reverse edge<<17 with
  // a the north/west tile (maps of <= 64 tiles; larger maps read DevState::epk)
  uint32_t epk[kSmallEdges];
  // per epk entry the removed edge's wall: corner codes p | q << 8 (interior corner (cy-1)(w-1) + cx-1,
  // or 64 + boundary position clockwise from the north-west corner), when DevCfg::dual
  uint16_t ewl[kSmallEdges];
  uint8_t bt[kMaxBorder], bd[kMaxBorder];
  // observation channel codes (DevCfg::channels as bytes): read per lane when the lanes of a group
  // build different channels of one env's image (a per-lane index into the DevCfg block would be a
  // dependent global load per channel)
  uint8_t chan[PGTG_MAX_CHANNELS];
};
struct TablesTail {
  uint32_t lanes[16][81];   // kLanes (copied only when traffic or lane/spawner channels need it)
  // traffic tables (copied with lanes): lane-square slot per square (255 = none), square per slot,
  // per-column masks (bit ly) of lane squares, lane-data spawners and the four "all" lanes
  uint8_t li[16][81];
  uint8_t slot_sq[16][32];
  uint16_t lanecol[16][9];
  uint16_t spcol[16][9];
  uint16_t allcol[16][4][9];
  uint8_t lane_route[32];
  alignas(4) uint8_t route_type_lane[20][4];  // read as one word per route
  uint8_t rule_w[PGTG_MAX_RULES][6][20];
  // DRIVER_BEHAVIORS per profile, read per car by profile index (kept in LDS, not in the DevCfg
  // constant block, so a per-lane index never becomes a dependent global load)
  uint64_t beh_t[5][5];    // [BEH_*][profile] 53-bit thresholds
  int32_t beh_mf[5], beh_pt[5];  // min_following_distance, floor(patience_level * 10)
};
// the global copy: head then tail, no padding between (asserted below)
struct Tables : TablesHead, TablesTail {};
constexpr size_t kTabHead = sizeof(TablesHead);  // byte offset of the tail in Tables
static_assert(sizeof(TablesHead) % 16 == 0 && sizeof(TablesHead) % alignof(TablesTail) == 0, "tail offset");
static_assert(sizeof(Tables) == sizeof(TablesHead) + sizeof(TablesTail), "Tables = head | tail");

// one PCG64 stream, SoA over envs
struct DevStream {
  uint64_t* shi;
  uint64_t* slo;
  uint64_t* ihi;
  uint64_t* ilo;
  uint64_t* buf;  // bit 32 = has_uint32, low 32 = buffered value
};

enum { BEH_DELAY = 0, BEH_SPEED = 1, BEH_YELLOW = 2, BEH_RED = 3, BEH_GO = 4 };

struct DevState {
  uint64_t n;
  EnvRec* rec;
  uint64_t* seed;
  uint16_t* plan;         // [n][plan_stride]
  DevStream car, ice, broken, sand;
  uint32_t* visited;      // [n][vis_words] or null
  // traffic: one bank of car slots per env in id order (= the reference's list order), slot-major /
  // env-minor ([slots][n]) so that the lanes of a wave read or write slot k of their envs with one
  // coalesced access.  w0 = x | y<<8 | route<<16 | profile<<21 | delay<<24 (bit 31: empty slot, a
  // despawned car), w1 = patience counter, id = car id.  Survivors are rewritten in place, respawns
  // appended behind the tail, the slots compacted when a tick's respawns could overrun them.
  // traf[n] = {n_cars | n_spawners<<16, next_id, tail (slots in use), flags}: flags bit 0 = the
  // occupancy counters are exact for the env's current cars (else k_env rebuilds them from the car
  // slots), bit 1 = fresh: the env's cars and counters are still in its staging block (below).
  // occ: the 4-bit lane-square occupancy counters (nt * 4 words per env, slot-major [word][n]) as the
  // last launch left them.
  // fresh: per env one contiguous staging block ([n][fresh_dw]) that k_traffic writes for an env it
  // gave initial traffic -- w0 of its cars at [0, k) (patience 0 and id = slot index implied), the
  // counters at [fresh_occ, fresh_occ + nt*4) -- as runs of consecutive words instead of one 4-byte
  // store per slot row of scattered envs; the env's next car pass reads its cars from there and
  // writes them (with their ids) to the slot rows beside every other env's.
  uint32_t* car_w0;
  uint32_t* car_w1;
  uint32_t* car_id;
  uint4* traf;
  uint32_t* occ;          // [nt * 4][n] or null
  uint32_t* fresh;        // [n][fresh_dw] or null
  uint16_t* spawners;     // [n][sp_pitch] square codes x | y<<8, x-major order (env-major: written once
                          // per episode by k_traffic as contiguous runs, read 24 at a time by k_env)
  uint32_t sp_pitch, fresh_dw, fresh_occ;
  uint32_t* tr_list;      // [n] envs k_env reset this launch (k_traffic's work list)
  uint32_t* tr_count;     // [2] list lengths, alternating launches
  // map queue (k_envq): per env a ring of kQueueDepth pre-generated episode maps, entry = plan
  // words then {px | py<<16, sg, path_len | error<<16, spawn tag}; qstate = head slot | kQueueStale
  uint32_t* qbuf;         // [n][kQueueDepth][qrec_dw] or null
  uint8_t* qstate;        // [n] or null
  uint2* qreq;            // [2][grid][cap] refill requests {env << 1 | slot, spawn counter} per k_envq
                          // workgroup, alternating launches
  uint2* qovf;            // [2][8][cap] one-round launches: the requests beyond a workgroup's first 64
  uint32_t* qctr;         // the lists' lengths, block counters, overflow lengths and heads (kQctr*)
  uint8_t* err;           // [n] last error code (negated PGTG_E_*)
  unsigned long long* counters;  // [2]: env steps, episodes
  unsigned long long* wg_ticks;  // [1]: wall-clock ticks of workgroup 0 in the last launch (start offsets)
  const int8_t* nsd_tab;
  const int8_t* cmp_tab;
  const uint32_t* epk;    // [n_edges] the Tables::epk edge table of maps of > 64 tiles (global memory)
};

// ------------------------------------------------------------------------------------------------
// numpy-exact RNG (Generator(PCG64(SeedSequence(seed, spawn_key=(k,))))): SeedSequence mixing
// (numpy/random/bit_generator.pyx), PCG64 XSL-RR 128-bit LCG with next_uint32 high-half buffering,
// Lemire bounded ints (distributions.c buffered_bounded_lemire_uint32), 53-bit doubles.
// ------------------------------------------------------------------------------------------------
struct Pcg {
  uint64_t shi, slo, ihi, ilo;
  uint32_t buf, has;
};

__device__ __forceinline__ void pcg_step(Pcg& g) {
  const uint64_t MH = 0x2360ED051FC65DA4ull, ML = 0x4385DF649FCCF645ull;
  uint64_t lo = g.slo * ML;
  uint64_t hi = __umul64hi(g.slo, ML) + g.slo * MH + g.shi * ML;
  uint64_t nlo = lo + g.ilo;
  hi += g.ihi + (nlo < lo ? 1ull : 0ull);
  g.slo = nlo;
  g.shi = hi;
}
__device__ __forceinline__ uint64_t pcg_next64(Pcg& g) {
  pcg_step(g);
  uint64_t x = g.shi ^ g.slo;
  unsigned rot = (unsigned)(g.shi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}
__device__ __forceinline__ uint32_t pcg_next32(Pcg& g) {
  if (g.has) {
    g.has = 0;
    return g.buf;
  }
  uint64_t v = pcg_next64(g);
  g.has = 1;
  g.buf = (uint32_t)(v >> 32);
  return (uint32_t)v;
}
__device__ __forceinline__ uint64_t pcg_u53(Pcg& g) { return pcg_next64(g) >> 11; }
__device__ __forceinline__ double pcg_double(Pcg& g) {
  return (double)(pcg_next64(g) >> 11) * (1.0 / 9007199254740992.0);
}
// integers(0, n) == choice(n): n == 1 draws nothing
__device__ __forceinline__ uint32_t pcg_int(Pcg& g, uint32_t n) {
  uint32_t rng = n - 1u;
  if (rng == 0u) return 0u;
  uint32_t excl = n;
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
// One draw of a per-lane sequence whose kind differs between lanes: random()'s 53-bit mantissa or
// integers(0, n) (Lemire on next_uint32 with the high-half buffer).  Callers skip the draw for
// integer draws with n <= 1 (numpy draws nothing there).  Keeping one PCG step site per draw slot
// instead of one per distribution keeps a divergent wave's instruction stream short.
__device__ __forceinline__ uint64_t pcg_draw(Pcg& g, bool is_int, uint32_t n) {
  const bool step = !is_int || !g.has;
  uint64_t v = 0;
  if (step) v = pcg_next64(g);
  if (!is_int) return v >> 11;
  uint32_t r32;
  if (step) {
    r32 = (uint32_t)v;
    g.has = 1;
    g.buf = (uint32_t)(v >> 32);
  } else {
    r32 = g.buf;
    g.has = 0;
  }
  uint64_t m = (uint64_t)r32 * n;
  uint32_t left = (uint32_t)m;
  if (left < n) {
    const uint32_t thr = (0xffffffffu - (n - 1u)) % n;
    while (left < thr) {
      m = (uint64_t)pcg_next32(g) * n;
      left = (uint32_t)m;
    }
  }
  return m >> 32;
}

// A PCG64 stream with its next 64-bit output computed one step ahead.  A draw takes the
// precomputed output at once and computes the following one, which does not depend on what the
// caller does with the draw, so the 128-bit multiply chain of a step overlaps the caller's work
// instead of sitting between consecutive dependent draws.  `g` is the consumed state (with the
// 32-bit buffer) -- what is stored back; identical outputs to Pcg's.
struct PcgAhead {
  Pcg g;
  uint64_t shi_a, slo_a;  // step(g)
  uint64_t out_a;         // its output: the next draw
};
__device__ __forceinline__ uint64_t pcg_output(uint64_t shi, uint64_t slo) {
  const uint64_t x = shi ^ slo;
  const unsigned rot = (unsigned)(shi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}
__device__ __forceinline__ PcgAhead ahead_init(const Pcg& g) {
  PcgAhead a;
  a.g = g;
  Pcg t = g;
  pcg_step(t);
  a.shi_a = t.shi;
  a.slo_a = t.slo;
  a.out_a = pcg_output(t.shi, t.slo);
  return a;
}
__device__ __forceinline__ uint64_t ahead_next64(PcgAhead& a) {
  const uint64_t r = a.out_a;
  a.g.shi = a.shi_a;
  a.g.slo = a.slo_a;
  Pcg t = a.g;
  pcg_step(t);
  a.shi_a = t.shi;
  a.slo_a = t.slo;
  a.out_a = pcg_output(t.shi, t.slo);
  return r;
}
__device__ __forceinline__ uint32_t ahead_next32(PcgAhead& a) {
  if (a.g.has) {
    a.g.has = 0;
    return a.g.buf;
  }
  const uint64_t v = ahead_next64(a);
  a.g.has = 1;
  a.g.buf = (uint32_t)(v >> 32);
  return (uint32_t)v;
}
// pcg_draw / pcg_int on a PcgAhead (same draws, same order)
__device__ __forceinline__ uint64_t ahead_draw(PcgAhead& a, bool is_int, uint32_t n) {
  const bool step = !is_int || !a.g.has;
  uint64_t v = 0;
  if (step) v = ahead_next64(a);
  if (!is_int) return v >> 11;
  uint32_t r32;
  if (step) {
    r32 = (uint32_t)v;
    a.g.has = 1;
    a.g.buf = (uint32_t)(v >> 32);
  } else {
    r32 = a.g.buf;
    a.g.has = 0;
  }
  uint64_t m = (uint64_t)r32 * n;
  uint32_t left = (uint32_t)m;
  if (left < n) {
    const uint32_t thr = (0xffffffffu - (n - 1u)) % n;
    while (left < thr) {
      m = (uint64_t)ahead_next32(a) * n;
      left = (uint32_t)m;
    }
  }
  return m >> 32;
}
__device__ __forceinline__ uint32_t ahead_int(PcgAhead& a, uint32_t n) {
  if (n <= 1u) return 0u;
  return (uint32_t)ahead_draw(a, true, n);
}

// ------------------------------------------------------------------------------------------------
// PCG64 jump-ahead.  s_{n+d} = M^d s_n + (1 + M + ... + M^(d-1)) inc, so a jump of d outputs
// composes the jumps of d's set bits: kPcgJump[b] = {M^(2^b), G(2^b)} (hi, lo words), G(2d) = G(d)
// (1 + M^d), M^(2d) = (M^d)^2.  Lanes that evaluate disjoint stretches of one stream start there.
// ------------------------------------------------------------------------------------------------
constexpr int kJumpBits = 16;  // jumps of < 65 536 outputs
struct JumpTab {
  uint64_t v[kJumpBits][4];  // M^(2^b) hi, lo, G(2^b) hi, lo
};
constexpr JumpTab make_jump_tab() {
  JumpTab t{};
  unsigned __int128 m = ((unsigned __int128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull, gsum = 1;
  for (int b = 0; b < kJumpBits; b++) {
    t.v[b][0] = (uint64_t)(m >> 64);
    t.v[b][1] = (uint64_t)m;
    t.v[b][2] = (uint64_t)(gsum >> 64);
    t.v[b][3] = (uint64_t)gsum;
    gsum = gsum * (m + 1);
    m = m * m;
  }
  return t;
}
__constant__ constexpr JumpTab kPcgJump = make_jump_tab();

// (ahi:alo) * (bhi:blo) mod 2^128
__device__ __forceinline__ void mul128(uint64_t ahi, uint64_t alo, uint64_t bhi, uint64_t blo, uint64_t& rhi, uint64_t& rlo) {
  rlo = alo * blo;
  rhi = __umul64hi(alo, blo) + alo * bhi + ahi * blo;
}
// advance g by d outputs (d < 2^nbits; nbits wave-uniform bounds the loop); the 32-bit buffer is
// left as it is
__device__ __forceinline__ void pcg_advance(Pcg& g, uint32_t d, int nbits) {
  for (int b = 0; b < nbits; b++) {
    if ((d >> b) & 1u) {
      const uint64_t mh = kPcgJump.v[b][0], ml = kPcgJump.v[b][1], gh = kPcgJump.v[b][2], gl = kPcgJump.v[b][3];
      uint64_t sh, sl, ch, cl;
      mul128(g.shi, g.slo, mh, ml, sh, sl);
      mul128(g.ihi, g.ilo, gh, gl, ch, cl);
      const uint64_t lo = sl + cl;
      g.shi = sh + ch + (lo < sl ? 1ull : 0ull);
      g.slo = lo;
    }
  }
}

// choice(k, p=p) with the host-normalised CDF (cumsum(p)/cumsum[-1]) as 53-bit thresholds:
// searchsorted(u, 'right') counts the entries <= u
template <int K>
__device__ __forceinline__ int pcg_choice_cdf(Pcg& g, const uint64_t* cdf_t) {
  const uint64_t m = pcg_u53(g);
  int i = 0;
#pragma unroll
  for (int j = 0; j < K - 1; j++) i += (m < cdf_t[j]) ? 0 : 1;
  return i;
}
// per-lane pick of a uniform 5-entry row (selects over scalar values instead of an indexed load)
template <typename T>
__device__ __forceinline__ T pick5(const T* a, int k) {
  T r = a[0];
  r = k == 1 ? a[1] : r;
  r = k == 2 ? a[2] : r;
  r = k == 3 ? a[3] : r;
  r = k == 4 ? a[4] : r;
  return r;
}

__device__ __forceinline__ uint32_t ss_hashmix(uint32_t v, uint32_t& hc) {
  v ^= hc;
  hc *= 0x931e8875u;
  v *= hc;
  v ^= v >> 16;
  return v;
}
__device__ __forceinline__ uint32_t ss_mix(uint32_t x, uint32_t y) {
  uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y;
  r ^= r >> 16;
  return r;
}
// SeedSequence pool after mixing the (zero-padded) run entropy of `seed`; hc continues from it.
struct SeedPool {
  uint32_t p[4];
  uint32_t hc;
};
__device__ __forceinline__ SeedPool ss_pool(uint64_t seed) {
  SeedPool s;
  uint32_t hc = 0x43b0d7e5u;
  uint32_t e[4] = {(uint32_t)seed, (uint32_t)(seed >> 32), 0u, 0u};
#pragma unroll
  for (int i = 0; i < 4; i++) s.p[i] = ss_hashmix(e[i], hc);
#pragma unroll
  for (int a = 0; a < 4; a++)
#pragma unroll
    for (int b = 0; b < 4; b++)
      if (a != b) s.p[b] = ss_mix(s.p[b], ss_hashmix(s.p[a], hc));
  s.hc = hc;
  return s;
}
// child stream with spawn key (key,): mix the key word, generate_state(4, uint64), seed PCG64
__device__ __forceinline__ Pcg ss_child(const SeedPool& sp, uint32_t key) {
  uint32_t p[4] = {sp.p[0], sp.p[1], sp.p[2], sp.p[3]};
  uint32_t hc = sp.hc;
#pragma unroll
  for (int d = 0; d < 4; d++) p[d] = ss_mix(p[d], ss_hashmix(key, hc));
  uint32_t w[8];
  uint32_t hb = 0x8b51f9ddu;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t v = p[i & 3];
    v ^= hb;
    hb *= 0x58f38dedu;
    v *= hb;
    v ^= v >> 16;
    w[i] = v;
  }
  uint64_t v0 = (uint64_t)w[0] | ((uint64_t)w[1] << 32), v1 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  uint64_t v2 = (uint64_t)w[4] | ((uint64_t)w[5] << 32), v3 = (uint64_t)w[6] | ((uint64_t)w[7] << 32);
  Pcg g;
  // inc = (initseq << 1) | 1 with initseq = v2:v3
  g.ihi = (v2 << 1) | (v3 >> 63);
  g.ilo = (v3 << 1) | 1ull;
  g.shi = 0;
  g.slo = 0;
  g.has = 0;
  g.buf = 0;
  pcg_step(g);
  uint64_t lo = g.slo + v1;
  g.shi = g.shi + v0 + (lo < g.slo ? 1ull : 0ull);
  g.slo = lo;
  pcg_step(g);
  return g;
}

__device__ __forceinline__ Pcg stream_load(const DevStream& s, uint64_t i) {
  Pcg g;
  g.shi = s.shi[i];
  g.slo = s.slo[i];
  g.ihi = s.ihi[i];
  g.ilo = s.ilo[i];
  uint64_t b = s.buf[i];
  g.buf = (uint32_t)b;
  g.has = (uint32_t)(b >> 32) & 1u;
  return g;
}
__device__ __forceinline__ void stream_store_state(const DevStream& s, uint64_t i, const Pcg& g) {
  s.shi[i] = g.shi;
  s.slo[i] = g.slo;
  s.buf[i] = (uint64_t)g.buf | ((uint64_t)g.has << 32);
}
__device__ __forceinline__ void stream_store_all(const DevStream& s, uint64_t i, const Pcg& g) {
  stream_store_state(s, i, g);
  s.ihi[i] = g.ihi;
  s.ilo[i] = g.ilo;
}

}  // namespace pgtg
