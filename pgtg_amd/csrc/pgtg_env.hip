// pgtg_amd/csrc/pgtg_env.hip -- MI355X (gfx950) kernels of the batched PGTG environment.
//
// One lane advances one independent environment (wave64, 256 lanes per workgroup).  Each lane
// reproduces, bit for bit, the reference's per-env control flow:
//   step   : pgtg/environment.py:1092-1281 (phase, cars, acceleration, braking, decomposition,
//            sub-step crash/goal/subgoal/red-light/ice/broken-road/sand handling, penalties)
//   reset  : pgtg/environment.py:581-656 with pgtg/map_generator.py:43-472 (procedural map) and
//            pgtg/parser.py:13-166 + pgtg/map.py:11-42 (map compilation) done in-kernel
//   obs    : pgtg/environment.py:1344-1536
// The map is never materialised per square: each env keeps a 2-byte-per-tile plan (staged in LDS
// for the kernel's lifetime) and square features are recomputed from constant 81-bit tile tables.
// Observations are staged as per-channel bitmasks in LDS and written to HBM cooperatively by the
// whole workgroup with 16-byte coalesced stores.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <cstddef>
#include <string>
#include <vector>

#include "pgtg_device.h"

namespace pgtg {
namespace dv {
#define PGTG_TBL_QUAL __constant__ static const
#include "pgtg_tables.h"
#undef PGTG_TBL_QUAL
}  // namespace dv
namespace hs {
#define PGTG_TBL_QUAL static const
#include "pgtg_tables.h"
#undef PGTG_TBL_QUAL
}  // namespace hs

__shared__ __attribute__((aligned(16))) TablesHead sT;  // per-workgroup LDS copy of the tables' head
__shared__ __attribute__((aligned(16))) TablesTail sTX;  // and of the tail (kernels that reference it)

// Copy `bytes` of a table into LDS: all of a thread's 16-byte loads are issued before the first
// LDS store (one memory latency instead of one per word).
__device__ __forceinline__ void stage_bytes(const void* __restrict__ gsrc, void* ldst, int bytes) {
  const int n4 = bytes >> 4, tid = (int)threadIdx.x;
  const uint4* src = reinterpret_cast<const uint4*>(gsrc);
  uint4* dst = reinterpret_cast<uint4*>(ldst);
  uint4 r[4];
#pragma unroll
  for (int j = 0; j < 4; j++) r[j] = src[tid + j * kBlock < n4 ? tid + j * kBlock : 0];  // unconditional: registers, not scratch
#pragma unroll
  for (int j = 0; j < 4; j++)
    if (tid + j * kBlock < n4) dst[tid + j * kBlock] = r[j];
  for (int k = tid + 4 * kBlock; k < n4; k += kBlock) dst[k] = src[k];
  for (int k = n4 * 4 + tid; k < bytes / 4; k += kBlock)
    reinterpret_cast<uint32_t*>(ldst)[k] = reinterpret_cast<const uint32_t*>(gsrc)[k];
}
// The head into sT; the tail into sTX when `tail` (a kernel whose code references sTX).
__device__ __forceinline__ void stage_tables(const Tables* __restrict__ gtab, bool tail) {
  stage_bytes(gtab, &sT, (int)sizeof(TablesHead));
  if (tail) stage_bytes(reinterpret_cast<const uint8_t*>(gtab) + kTabHead, &sTX, (int)sizeof(TablesTail));
}

// Workgroup barrier for LDS data only: unlike __syncthreads() it does not wait for the waves'
// outstanding global stores (outputs, state) to complete.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// One env's tile plan (its nq data quads of 8 u16 in HBM) into its LDS row of pdw words,
// in blocks of 8 x 16 bytes (BIG: maps of > 64 tiles; smaller maps are one block, straight-line code:
// a runtime block loop made the compiler wait for every load before the first LDS store), each
// block's loads first.
template <bool BIG>
__device__ __forceinline__ void stage_plan(const uint16_t* __restrict__ plan, int nq, uint32_t* dst, int pdw) {
  const uint4* src = reinterpret_cast<const uint4*>(plan);
  for (int k0 = 0; k0 < (BIG ? nq : 1); k0 += 8) {
    uint4 q[8];
#pragma unroll
    for (int k = 0; k < 8; k++) q[k] = src[k0 + k < nq ? k0 + k : k0];  // unconditional: registers, not scratch
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (k0 + k < nq) {
        const uint32_t wv[4] = {q[k].x, q[k].y, q[k].z, q[k].w};
#pragma unroll
        for (int j = 0; j < 4; j++)
          if ((k0 + k) * 4 + j < pdw) dst[(k0 + k) * 4 + j] = wv[j];
      }
    }
  }
}

// Diagnostic build only (-DPGTG_STAMPS): per-wave phase timestamps (s_memtime) into a debug buffer
// that nothing else reads.  The product build compiles these to nothing.
#ifdef PGTG_STAMPS
__device__ unsigned long long g_stamps[1 << 21];
#define STAMP(k)                                                                          \
  do {                                                                                    \
    if ((threadIdx.x & 63) == 0) {                                                        \
      unsigned long long t_ = __builtin_amdgcn_s_memtime();                               \
      g_stamps[((blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * 32 + (k)) & ((1 << 21) - 1)] = t_; \
    }                                                                                     \
  } while (0)
// wall-clock (s_memrealtime, 100 MHz, one clock for the chip) stamp k in {0, 1} of the wave
#define STAMPR(k)                                                                                     \
  do {                                                                                                \
    if ((threadIdx.x & 63) == 0)                                                                      \
      g_stamps[(1 << 20) | ((((blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * 8 + (k))) & ((1 << 20) - 1))] = \
          __builtin_amdgcn_s_memrealtime();                                                           \
  } while (0)
#else
#define STAMP(k) \
  do {           \
  } while (0)
#define STAMPR(k) \
  do {            \
  } while (0)
#endif

// ------------------------------------------------------------------------------------------------
// small device helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bit81(const uint32_t* m3, int sq) { return (m3[sq >> 5] >> (sq & 31)) & 1u; }

// exit segment a local square belongs to (north (3..5,0), east (8,3..5), south (3..5,8), west (0,3..5))
__device__ __forceinline__ int seg_dir(int lx, int ly) {
  bool mx = (unsigned)(lx - 3) <= 2u, my = (unsigned)(ly - 3) <= 2u;
  if (ly == 0 && mx) return 0;
  if (lx == 8 && my) return 1;
  if (ly == 8 && mx) return 2;
  if (lx == 0 && my) return 3;
  return -1;
}

struct EnvView {
  int px, py, vx, vy;
  uint32_t phase, flags, path_len, elapsed;
  uint32_t sg, spawn;
  uint64_t used;
};

__device__ __forceinline__ EnvView rec_view(const EnvRec& e) {
  EnvView v;
  v.px = (int)(int16_t)(e.a.x & 0xffffu);
  v.py = (int)(int16_t)(e.a.x >> 16);
  v.vx = (int)(int16_t)(e.a.y & 0xffffu);
  v.vy = (int)(int16_t)(e.a.y >> 16);
  v.phase = e.a.z & 0xffffu;
  v.flags = (e.a.z >> 16) & 0xfu;
  v.path_len = e.a.z >> 20;
  v.elapsed = e.a.w;
  v.sg = e.b.x;
  v.spawn = e.b.y;
  v.used = (uint64_t)e.b.z | ((uint64_t)e.b.w << 32);
  return v;
}
__device__ __forceinline__ EnvView rec_load(const EnvRec* r, uint64_t i) { return rec_view(r[i]); }
__device__ __forceinline__ void rec_store(EnvRec* r, uint64_t i, const EnvView& v) {
  EnvRec e;
  e.a.x = ((uint32_t)v.px & 0xffffu) | ((uint32_t)v.py << 16);
  e.a.y = ((uint32_t)v.vx & 0xffffu) | ((uint32_t)v.vy << 16);
  e.a.z = (v.phase & 0xffffu) | ((v.flags & 0xfu) << 16) | (v.path_len << 20);
  e.a.w = v.elapsed;
  e.b.x = v.sg;
  e.b.y = v.spawn;
  e.b.z = (uint32_t)v.used;
  e.b.w = (uint32_t)(v.used >> 32);
  r[i] = e;
}

// Tiles >= nt of a plan word (two u16 tiles per word) are padding, stored as 0 so that the device
// state is a function of the seeds alone (LDS plan rows may hold stale bytes there).
__device__ __forceinline__ uint32_t plan_word_mask(const DevCfg& c, int word) {
  const int t0 = 2 * word;
  return t0 + 1 < c.nt ? ~0u : (t0 < c.nt ? 0xffffu : 0u);
}
// The env's LDS plan row (pdw words) back to its HBM tile plan (plan_stride u16 words), padding as 0.
__device__ __forceinline__ void store_plan_row(const DevCfg& c, const DevState& S, uint64_t i, const uint32_t* pw, int pdw) {
  uint4* dstp = reinterpret_cast<uint4*>(S.plan + i * (uint64_t)c.plan_stride);
  for (int k = 0; k < c.plan_stride / 8; k++) {
    uint32_t wv[4];
#pragma unroll
    for (int j = 0; j < 4; j++) wv[j] = (k * 4 + j < pdw) ? pw[k * 4 + j] & plan_word_mask(c, k * 4 + j) : 0u;
    dstp[k] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
  }
}

// Per-lane LDS view of the env's tile plan.  Lane stride is an odd number of dwords so that 64
// lanes reading the same tile index hit distinct banks.
struct Plan {
  uint16_t* p;
  __device__ __forceinline__ uint32_t operator[](int t) const { return p[t]; }
};

// Has tile t's subgoal been used (EpisodeMap.set_subgoals_to_used, pgtg/map.py:143-171)?  p = the
// tile's plan word: maps of > 64 tiles (BIG) mark it there, smaller maps in the u64 of EnvRec.
template <bool BIG>
__device__ __forceinline__ bool used_bit(const EnvView& v, uint32_t p, int t) {
  return BIG ? (p & kPlanUsed) != 0u : ((v.used >> t) & 1ull) != 0ull;
}

// features of square (x, y) inside the map (pgtg/parser.py:47-155 semantics, see file header)
template <bool BIG>
__device__ __forceinline__ uint32_t square_flags(const DevCfg& c, const Plan& pl, const EnvView& v, int x, int y) {
  int tx = x / kTile, ty = y / kTile;
  int lx = x - tx * kTile, ly = y - ty * kTile;
  int t = ty * c.tw + tx;
  uint32_t p = pl[t];
  uint32_t ex = plan_exits(p);
  int sq = lx * 9 + ly;
  uint32_t f = 0;
  uint32_t wall = bit81(sT.wall[ex], sq);
  if (wall) f |= SQ_WALL;
  int d = seg_dir(lx, ly);
  if (d >= 0 && ((ex >> d) & 1u)) {
    if (plan_sgdir(p) == d) f |= used_bit<BIG>(v, p, t) ? SQ_USED : SQ_SUBGOAL;
    if ((int)(v.sg & 0xffu) == t && (int)((v.sg >> 8) & 0xffu) == d) f |= SQ_START;
    if ((int)((v.sg >> 16) & 0xffu) == t && (int)(v.sg >> 24) == d) f |= SQ_FINAL;
  }
  // (read unconditionally, at a valid row: a conditional LDS read is a branch waited on alone)
  const uint32_t ob = bit81(sT.obst[min(plan_omask(p), (uint32_t)PGTG_N_OBST_MASKS - 1u)], sq);
  uint32_t ot = plan_otype(p);
  if (ot && !wall && ob) f |= SQ_ICE << (ot - 1);
  return f;
}
__device__ __forceinline__ uint32_t square_lanes(const DevCfg& c, const Plan& pl, int x, int y) {
  int tx = x / kTile, ty = y / kTile;
  int lx = x - tx * kTile, ly = y - ty * kTile;
  uint32_t ex = plan_exits(pl[ty * c.tw + tx]);
  return ex ? sTX.lanes[ex][lx * 9 + ly] : 0u;
}
__device__ __forceinline__ bool square_spawner(const DevCfg& c, const Plan& pl, int x, int y) {
  int tx = x / kTile, ty = y / kTile;
  int lx = x - tx * kTile, ly = y - ty * kTile;
  uint32_t ex = plan_exits(pl[ty * c.tw + tx]);
  if (!ex) return false;
  int sq = lx * 9 + ly;
  if (bit81(sT.spawner[ex], sq)) return true;
  uint32_t l = sTX.lanes[ex][sq];
  return (tx == 0 && (l >> 31 & 1u)) || (tx == c.tw - 1 && (l >> 30 & 1u)) || (ty == 0 && (l >> 29 & 1u)) ||
         (ty == c.th - 1 && (l >> 28 & 1u));
}
__device__ __forceinline__ bool inside(const DevCfg& c, int x, int y) {
  return (unsigned)x < (unsigned)c.W && (unsigned)y < (unsigned)c.H;
}
__device__ __forceinline__ int phase_color(const DevCfg& c, uint32_t ph) {
  return (int)ph < c.phase_g ? 0 : ((int)ph < c.phase_gy ? 1 : 2);
}

// ------------------------------------------------------------------------------------------------
// traffic helpers: occupancy counters per lane square in LDS (tile t, lane slot li -> t*32 + li)
// ------------------------------------------------------------------------------------------------
// (both reads unconditional at valid indices, so that a batch of lookups goes out together)
__device__ __forceinline__ int lane_slot_tw(int tw, const Plan& pl, int x, int y) {
  int tx = x / kTile, ty = y / kTile;
  int lx = x - tx * kTile, ly = y - ty * kTile;
  int t = ty * tw + tx;
  uint32_t ex = plan_exits(pl[t]);
  const int li_raw = sTX.li[ex][lx * 9 + ly];
  const int li = ex ? li_raw : 255;
  return li == 255 ? -1 : t * 32 + li;
}
__device__ __forceinline__ int lane_slot(const DevCfg& c, const Plan& pl, int x, int y) {
  return lane_slot_tw(c.tw, pl, x, y);
}
// A DevCfg field as a value the compiler cannot re-load inside a loop (see ProfileCdf).
__device__ __forceinline__ int pinned(int x) {
  __asm__ volatile("" : "+s"(x));
  return x;
}
__device__ __forceinline__ bool square_tlight(const DevCfg& c, const Plan& pl, int x, int y) {
  int tx = x / kTile, ty = y / kTile;
  int lx = x - tx * kTile, ly = y - ty * kTile;
  uint32_t p = pl[ty * c.tw + tx];
  int sq = lx * 9 + ly;
  return plan_otype(p) == 4 && !bit81(sT.wall[plan_exits(p)], sq) && bit81(sT.obst[plan_omask(p)], sq);
}
// Occupancy counters are 4-bit (two lane slots per byte, 16 B per tile) so that 256 envs' counters
// fit a CU's LDS.  A counter saturates at kOccMax and raises the lane's `sat` flag; decrementing a
// saturated counter then recounts that square exactly from the car slots (rare: squares with 15
// cars), so every count the dynamics see is exact.  Test builds lower kOccMax to exercise it.
#ifndef PGTG_OCC_MAX
#define PGTG_OCC_MAX 15
#endif
constexpr int kOccMax = PGTG_OCC_MAX;
static_assert(kOccMax >= 1 && kOccMax <= 15, "4-bit occupancy counters");
__device__ __forceinline__ int occ_get(const uint8_t* o, int s) { return (o[s >> 1] >> ((s & 1) << 2)) & 15; }
__device__ __forceinline__ void occ_put(uint8_t* o, int s, int v) {
  const int sh = (s & 1) << 2;
  o[s >> 1] = (uint8_t)((o[s >> 1] & ~(15 << sh)) | (v << sh));
}
__device__ __forceinline__ void occ_inc(uint8_t* o, int s, bool& sat) {
  const int v = occ_get(o, s);
  if (v >= kOccMax) sat = true;
  else occ_put(o, s, v + 1);
}
__device__ __forceinline__ int occ_at(const DevCfg& c, const Plan& pl, const uint8_t* occ, int x, int y) {
  int s = lane_slot(c, pl, x, y);
  return s < 0 ? 0 : occ_get(occ, s);
}
// k-th (0-based) set bit of a 32-bit word, branch-free (popcount halving); -1 if there is none
__device__ __forceinline__ int select32(uint32_t x, int k) {
  int pos = 0;
#pragma unroll
  for (int sh = 16; sh >= 1; sh >>= 1) {
    const int c = __popc(x & ((1u << sh) - 1u));
    const bool up = k >= c;
    k -= up ? c : 0;
    x = up ? x >> sh : x;
    pos += up ? sh : 0;
  }
  return (x & 1u) && k == 0 ? pos : -1;
}
__device__ __forceinline__ int kth_bit(uint32_t m, int k) {
  for (int j = 0; j < k; j++) m &= m - 1u;
  return __ffs((int)m) - 1;
}

// The driver-profile CDF thresholds as values the compiler cannot re-load from the handle's
// DevCfg: under scalar-register pressure it rematerialises such loop-invariant loads inside the car
// loops, and every re-load is a scalar-cache round trip the loop then waits for.
struct ProfileCdf {
  uint64_t t[4];
};
__device__ __forceinline__ ProfileCdf pin_profile_cdf(const DevCfg& c) {
  ProfileCdf p;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    uint64_t x = c.profile_t[j];
    __asm__ volatile("" : "+s"(x));
    p.t[j] = x;
  }
  return p;
}
__device__ __forceinline__ int profile_of(const ProfileCdf& p, uint64_t u) {
  int prof = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) prof += (u < p.t[j]) ? 0 : 1;
  return prof;
}

constexpr uint32_t kCarEmpty = 1u << 31;  // w0 of a slot without a car
// One env's car slots (DevState::car_w0 layout: slot k of env i at k * n + i) through per-lane
// pointers at the env's slot 0: the three array bases stay in VGPRs instead of being re-read from
// spilled scalar registers at every access of the car loops.
// Global-address-space words: the slot pointers are pinned in VGPRs by the asm below, which hides
// where they came from, and a generic pointer compiles to flat loads and stores -- and a flat access
// counts on the LDS counter too, so every LDS wait of the car loop would also wait for the next
// slot's HBM prefetch.
typedef __attribute__((address_space(1))) uint32_t gu32;
struct CarSlots {
  gu32 *w0, *w1, *id;
  uint64_t n;  // stride between slots (= number of envs)
  __device__ __forceinline__ CarSlots(const DevState& S, uint64_t i)
      : w0((gu32*)(S.car_w0 + i)), w1((gu32*)(S.car_w1 + i)), id((gu32*)(S.car_id + i)), n(S.n) {
    __asm__ volatile("" : "+v"(w0), "+v"(w1), "+v"(id));
  }
  __device__ __forceinline__ uint64_t at(int k) const { return (uint64_t)k * n; }
};
// An env's staging block (DevState::fresh): w0 of its fresh cars at [0, k), counters at fresh_occ.
__device__ __forceinline__ gu32* fresh_block(const DevState& S, uint64_t i) {
  return (gu32*)(S.fresh + i * (uint64_t)S.fresh_dw);
}
constexpr uint32_t kTrafOccValid = 1u, kTrafFresh = 2u;  // traf.w flags

// ------------------------------------------------------------------------------------------------
// reset: seeding, procedural map, compilation, start square  (pgtg/environment.py:581-656)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void rand_pos(const DevCfg& c, Pcg& r, int& x, int& y) {  // map_generator.py:602-626
  switch (pcg_int(r, 4)) {
    case 0: x = (int)pcg_int(r, c.tw); y = 0; break;
    case 1: x = c.tw - 1; y = (int)pcg_int(r, c.th); break;
    case 2: x = (int)pcg_int(r, c.tw); y = c.th - 1; break;
    default: x = 0; y = (int)pcg_int(r, c.th); break;
  }
}
__device__ __forceinline__ int rand_dir(const DevCfg& c, Pcg& r, int x, int y) {  // map_generator.py:574-599
  // possible directions in the order north, east, south, west as a bitmask; pick the k-th set bit
  uint32_t m = (y == 0 ? 1u : 0u) | (x == c.tw - 1 ? 2u : 0u) | (y == c.th - 1 ? 4u : 0u) | (x == 0 ? 8u : 0u);
  int k = (int)pcg_int(r, (uint32_t)__popc(m));
  for (int j = 0; j < k; j++) m &= m - 1u;
  return __ffs((int)m) - 1;
}

// ------------------------------------------------------------------------------------------------
// tile masks: uint32_t (<= 32 tiles), uint64_t (<= 64) or Bits<4> (<= 256 tiles, 16 x 16 maps).  The
// generator and the path compiler are written once over these helpers; Bits keeps its words in named
// registers (every index is resolved with selects: no private-array indexing, no scratch).
// ------------------------------------------------------------------------------------------------
template <int NW>
struct Bits {
  uint64_t w[NW];
};
template <int NW>
__device__ __forceinline__ Bits<NW> operator|(Bits<NW> a, const Bits<NW>& b) {
#pragma unroll
  for (int q = 0; q < NW; q++) a.w[q] |= b.w[q];
  return a;
}
template <int NW>
__device__ __forceinline__ Bits<NW> operator&(Bits<NW> a, const Bits<NW>& b) {
#pragma unroll
  for (int q = 0; q < NW; q++) a.w[q] &= b.w[q];
  return a;
}
template <int NW>
__device__ __forceinline__ Bits<NW> operator~(Bits<NW> a) {
#pragma unroll
  for (int q = 0; q < NW; q++) a.w[q] = ~a.w[q];
  return a;
}
template <int NW>
__device__ __forceinline__ Bits<NW>& operator|=(Bits<NW>& a, const Bits<NW>& b) { return a = a | b; }
template <int NW>
__device__ __forceinline__ Bits<NW>& operator&=(Bits<NW>& a, const Bits<NW>& b) { return a = a & b; }
// shifts by 0 <= n < 64 (grid rows of <= 16 tiles, single columns)
template <int NW>
__device__ __forceinline__ Bits<NW> operator<<(const Bits<NW>& a, int n) {
  Bits<NW> r;
#pragma unroll
  for (int q = 0; q < NW; q++) r.w[q] = (a.w[q] << n) | (q > 0 && n ? a.w[q - 1] >> (64 - n) : 0ull);
  return r;
}
template <int NW>
__device__ __forceinline__ Bits<NW> operator>>(const Bits<NW>& a, int n) {
  Bits<NW> r;
#pragma unroll
  for (int q = 0; q < NW; q++) r.w[q] = (a.w[q] >> n) | (q + 1 < NW && n ? a.w[q + 1] << (64 - n) : 0ull);
  return r;
}
__device__ __forceinline__ bool mask_any(uint32_t m) { return m != 0u; }
__device__ __forceinline__ bool mask_any(uint64_t m) { return m != 0ull; }
template <int NW>
__device__ __forceinline__ bool mask_any(const Bits<NW>& m) {
  uint64_t o = 0;
#pragma unroll
  for (int q = 0; q < NW; q++) o |= m.w[q];
  return o != 0ull;
}
__device__ __forceinline__ bool mask_eq(uint32_t a, uint32_t b) { return a == b; }
__device__ __forceinline__ bool mask_eq(uint64_t a, uint64_t b) { return a == b; }
template <int NW>
__device__ __forceinline__ bool mask_eq(const Bits<NW>& a, const Bits<NW>& b) {
  uint64_t d = 0;
#pragma unroll
  for (int q = 0; q < NW; q++) d |= a.w[q] ^ b.w[q];
  return d == 0ull;
}
__device__ __forceinline__ bool mask_get(uint32_t m, int t) { return (m >> t) & 1u; }
__device__ __forceinline__ bool mask_get(uint64_t m, int t) { return (m >> t) & 1ull; }
template <int NW>
__device__ __forceinline__ bool mask_get(const Bits<NW>& m, int t) {
  uint64_t x = 0;
#pragma unroll
  for (int q = 0; q < NW; q++) x = (t >> 6) == q ? m.w[q] : x;
  return (x >> (t & 63)) & 1ull;
}
template <typename M>
__device__ __forceinline__ M mask_bit(int t) {
  return (M)1 << t;
}
template <>
__device__ __forceinline__ Bits<4> mask_bit<Bits<4>>(int t) {
  Bits<4> r;
#pragma unroll
  for (int q = 0; q < 4; q++) r.w[q] = (t >> 6) == q ? 1ull << (t & 63) : 0ull;
  return r;
}
template <typename M>
__device__ __forceinline__ M mask_zero() {
  return (M)0;
}
template <>
__device__ __forceinline__ Bits<4> mask_zero<Bits<4>>() {
  Bits<4> r;
#pragma unroll
  for (int q = 0; q < 4; q++) r.w[q] = 0ull;
  return r;
}
// index of the lowest set bit (m != 0)
__device__ __forceinline__ int mask_ctz(uint32_t m) { return __ffs((int)m) - 1; }
__device__ __forceinline__ int mask_ctz(uint64_t m) { return __ffsll((long long)m) - 1; }
template <int NW>
__device__ __forceinline__ int mask_ctz(const Bits<NW>& m) {
  int r = -1;
#pragma unroll
  for (int q = NW - 1; q >= 0; q--) r = m.w[q] ? q * 64 + __ffsll((long long)m.w[q]) - 1 : r;
  return r;
}
// the full-grid exit mask of direction d (DevCfg::h0) as an M
template <typename M>
__device__ __forceinline__ M mask_h0(const DevCfg& c, int d) {
  return (M)c.h0[0][d];
}
template <>
__device__ __forceinline__ Bits<4> mask_h0<Bits<4>>(const DevCfg& c, int d) {
  Bits<4> r;
#pragma unroll
  for (int q = 0; q < 4; q++) r.w[q] = c.h0[q][d];
  return r;
}

// k-th (0-based) set bit of a 64-bit word, branch-free (popcount halving)
__device__ __forceinline__ int select64(uint64_t x, int k) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  const int cl = __popc(lo);
  bool up = k >= cl;
  uint32_t y = up ? hi : lo;
  int base = up ? 32 : 0;
  k -= up ? cl : 0;
#pragma unroll
  for (int half = 16; half >= 1; half >>= 1) {
    const int cnt = __popc(y & ((1u << half) - 1u));
    up = k >= cnt;
    y = up ? y >> half : y;
    base += up ? half : 0;
    k -= up ? cnt : 0;
  }
  return base;
}

// NW x 64 edge bits (the reference's shrinking removable_edges list as a membership set)
template <int NW>
struct EdgeBits {
  uint64_t w[NW];
  __device__ __forceinline__ void init(int n) {
#pragma unroll
    for (int q = 0; q < NW; q++) {
      const int m = n - 64 * q;
      w[q] = m >= 64 ? ~0ull : (m <= 0 ? 0ull : ((1ull << m) - 1ull));
    }
  }
  __device__ __forceinline__ void clear(int i) {
#pragma unroll
    for (int q = 0; q < NW; q++) w[q] &= (i >> 6) == q ? ~(1ull << (i & 63)) : ~0ull;
  }
  __device__ __forceinline__ int select(int k) const {
    uint64_t x = w[0];
    int base = 0;
    bool go = true;
#pragma unroll
    for (int q = 0; q + 1 < NW; q++) {  // walk the words with uniform control flow
      const int cnt = __popcll(x);
      const bool next = go && k >= cnt;
      k -= next ? cnt : 0;
      base += next ? 64 : 0;
      x = next ? w[q + 1] : x;
      go = next;
    }
    return base + select64(x, k);
  }
};

// One BFS step on the tile graph given by the four exit masks (tile t reaches its neighbours in
// the directions of its exits).
template <typename M>
__device__ __forceinline__ M expand(M R, M hN, M hE, M hS, M hW, int w) {
  return R | ((R & hN) >> w) | ((R & hS) << w) | ((R & hE) << 1) | ((R & hW) >> 1);
}
// The same on a symmetric graph (t has a south exit iff t+w has a north exit, ...): "R's tiles with
// a south exit, moved one row down" equals "R moved one row down, restricted to tiles with a north
// exit" -- one shift and one and-or per direction, the four shifts independent of each other.
template <typename M>
__device__ __forceinline__ M expand_sym(M R, M hN, M hE, M hS, M hW, int w) {
  const M dn = R << w, up = R >> w, rt = R << 1, lf = R >> 1;
  return R | (dn & hN) | (up & hS) | (rt & hW) | (lf & hE);
}

// After deleting edge a-b from a graph in which start s and goal g were connected: are they still?
// Bidirectional flood from a and b: the fronts meet (a-b still connected -> yes), or one side's
// component is exhausted first, in which case s-g broke iff exactly one of s, g lies in it.
template <typename M>
__device__ __forceinline__ bool still_connected(M hN, M hE, M hS, M hW, int w, int a, int b, int s, int g) {
  // Two expansions per side between checks: the sets only grow, so meeting and exhaustion are
  // still detected (at most one expansion late) with half the loop control of a step-wise loop.
  // One exit condition keeps the loop's mask bookkeeping short.
  M Ra = mask_bit<M>(a), Rb = mask_bit<M>(b);
  bool done, res;
  do {
    const M Ma = expand_sym<M>(Ra, hN, hE, hS, hW, w), Mb = expand_sym<M>(Rb, hN, hE, hS, hW, w);
    const M Na = expand_sym<M>(Ma, hN, hE, hS, hW, w), Nb = expand_sym<M>(Mb, hN, hE, hS, hW, w);
    const bool meet = mask_any(Na & Nb), exa = mask_eq(Na, Ma), exb = mask_eq(Nb, Mb);
    const M X = exa ? Na : Nb;
    res = meet || mask_get(X, s) == mask_get(X, g);
    done = meet || exa || exb;
    Ra = Na;
    Rb = Nb;
  } while (!done);
  return res;
}

// generate_map_graph's edge-removal loop (map_generator.py:218-264) on exit masks of type M
// (uint32_t when the map has <= 32 tiles, Bits<4> beyond 64).  removable_edges keeps graph-theory's
// nested-dict order (edge table `epk`: the LDS copy for maps of <= 64 tiles, else global memory); an
// edge pair stays removed iff start->end stays connected, which is exactly the outcome of the
// reference's BFS-path test + re-add.  A removed edge whose two tiles still share an intact 4-cycle
// cannot disconnect anything; otherwise still_connected decides.
template <typename M, int NW>
__device__ __forceinline__ void remove_edges(const DevCfg& c, const uint32_t* __restrict__ epk, Pcg& r, int st_t,
                                             int gl_t, M& hN, M& hE, M& hS, M& hW) {
  // (pinned: re-loaded from the DevCfg in the loop under scalar-register pressure otherwise)
  const int w = pinned(c.tw), keep = pinned(c.keep), n_edges = pinned(c.n_edges);
  EdgeBits<NW> L;
  L.init(n_edges);
  int nrem = n_edges, count = n_edges;
  if (!(count > keep && nrem > 0)) return;
  // The candidate sequence (draw -> list index -> edge pair) does not depend on whether earlier
  // removals were undone, so the next candidate is drawn while the current one is tested (two
  // independent dependency chains per iteration); the speculative draw is rolled back on exit.
  // The next candidate's edge-table read overlaps the test; its reverse entry leaves the list at
  // the end of the iteration, before the following draw.
  auto draw_edge = [&](int n) {
    const int k = (int)pcg_draw(r, true, (uint32_t)n);  // n >= 2: always draws
    const int e = L.select(k);
    L.clear(e);
    return e;
  };
  uint32_t pk = epk[draw_edge(nrem)];
  L.clear((int)(pk >> 17));
  nrem -= 2;
#ifdef PGTG_STAMPS
  unsigned long long dbg_bfs = 0, dbg_iters = 0;
#endif
  for (;;) {
    Pcg r_before = r;
    const bool more = nrem > 0;  // uniform: every lane is in the same iteration
    int e_next = 0;
    if (more) e_next = draw_edge(nrem);
    const uint32_t pk_next = epk[e_next];
    // remove edge a-b (horizontal: a left of b; vertical: a above b), branch-free
    const int a = (int)(pk & 255u), b = (int)((pk >> 8) & 255u);
    const bool hz = (pk >> 16) & 1u;
    const M ma = mask_bit<M>(a), mb = mask_bit<M>(b), mab = ma | mb, z = mask_zero<M>();
    const M sN = hN, sE = hE, sS = hS, sW = hW;
    hE &= ~(hz ? ma : z);
    hW &= ~(hz ? mb : z);
    hS &= ~(hz ? z : ma);
    hN &= ~(hz ? z : mb);
    // an intact unit square through a and b on either side keeps everything connected
    const M P1 = hz ? hN : hW, P2 = hz ? hS : hE, F = hz ? hE : hS;
    const int off = hz ? w : 1;
    const bool cyc = (mask_eq(P1 & mab, mab) && mask_any(F & (ma >> off))) ||
                     (mask_eq(P2 & mab, mab) && mask_any(F & (ma << off)));
    count -= 2;
#ifdef PGTG_STAMPS
    const unsigned long long tb0 = __builtin_amdgcn_s_memtime();
#endif
    if (!cyc && !still_connected<M>(hN, hE, hS, hW, w, a, b, st_t, gl_t)) {
      hN = sN; hE = sE; hS = sS; hW = sW;
      count += 2;
    }
#ifdef PGTG_STAMPS
    dbg_bfs += __builtin_amdgcn_s_memtime() - tb0;
    dbg_iters++;
#endif
    if (!(count > keep && more)) {
      r = r_before;  // the reference stops drawing here
      break;
    }
    L.clear((int)(pk_next >> 17));
    pk = pk_next;
    nrem -= 2;
  }
#ifdef PGTG_STAMPS
  if ((threadIdx.x & 63) == 0) {  // lane 0's loop: cycles in the connectivity test, iterations
    g_stamps[((blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * 32 + 26) & ((1 << 21) - 1)] = dbg_bfs;
    g_stamps[((blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * 32 + 27) & ((1 << 21) - 1)] = dbg_iters;
  }
#endif
}

// The same loop decided on the dual graph (round 5; maps of <= 64 tiles, both sides >= 2, w + h <= 31).
// A removed edge is a wall segment between two corners of the tile grid.  Start s and goal g are border
// tiles, so their boundary segments split the outer boundary's corners into two arcs, A (clockwise
// from s to g) and B (from g back to s); s and g are disconnected iff walls join a corner of A to a
// corner of B (the planar separation of two boundary cells).  RA / RB hold the interior corners
// wall-connected to A / B, so a removal is undone iff its wall would join RA u A to RB u B: four bit
// tests instead of a flood of the tile graph.  A kept wall that attaches a corner to RA (RB) adds that
// corner's wall component, found by a flood over the interior walls that is usually one expansion
// (a fresh corner).  Checked against BFS connectivity on every border start/goal pair of 2x2 .. 8x8
// grids; the RNG draws, the removable list and the outcomes are the primal loop's.
struct DualArcs {
  uint64_t ba, bb;  // boundary corner positions (clockwise from the north-west corner) on arc A, arc B
};
// boundary segments of border tile t: the run [r0, r0 + len) of segment indices (segment i joins
// boundary positions i and i + 1; corner tiles own two consecutive segments)
__device__ __forceinline__ void border_run(int t, int w, int h, int& r0, int& len) {
  const int L = 2 * (w + h), x = t % w, y = t / w;
  if (y == 0) {
    r0 = x == 0 ? L - 1 : x;
    len = (x == 0 || x == w - 1) ? 2 : 1;
  } else if (x == w - 1) {
    r0 = w + y;
    len = y == h - 1 ? 2 : 1;
  } else if (y == h - 1) {
    r0 = w + h + (w - 1 - x);
    len = x == 0 ? 2 : 1;
  } else {
    r0 = 2 * w + h + (h - 1 - y);
    len = 1;
  }
}
// `cnt` consecutive positions from `from` on the cyclic boundary of L < 64 positions
__device__ __forceinline__ uint64_t arc_mask(int from, int cnt, int L) {
  const uint64_t m = cnt >= 64 ? ~0ull : (1ull << cnt) - 1ull, all = (1ull << L) - 1ull;
  return ((m << from) | (from ? m >> (L - from) : 0ull)) & all;
}
__device__ __forceinline__ DualArcs dual_arcs(int w, int h, int s, int g) {
  DualArcs d{0ull, 0ull};
  if (s == g) return d;  // one tile: never separated, no removal is undone
  const int L = 2 * (w + h);
  int s0, sl, g0, gl;
  border_run(s, w, h, s0, sl);
  border_run(g, w, h, g0, gl);
  const int a0 = (s0 + sl) % L, b0 = (g0 + gl) % L;  // first corner after s's run, after g's run
  d.ba = arc_mask(a0, (g0 - a0 + L) % L + 1, L);      // up to and including g's first corner
  d.bb = arc_mask(b0, (s0 - b0 + L) % L + 1, L);
  return d;
}
// corner code x (interior corner index < 64, or 64 + boundary position) in R (interior) / Bm (boundary)
template <typename CM>
__device__ __forceinline__ bool corner_in(int x, CM R, uint64_t Bm) {
  const bool rb = (R >> (x & (int)(sizeof(CM) * 8 - 1))) & 1u, bb = (Bm >> (x & 63)) & 1ull;
  return x >= 64 ? bb : rb;
}
template <typename M, int NW, typename CM>
__device__ __forceinline__ void remove_edges_dual(const DevCfg& c, const uint32_t* __restrict__ epk,
                                                  const uint16_t* __restrict__ ewl, Pcg& r, int st_t, int gl_t,
                                                  M& hN, M& hE, M& hS, M& hW) {
  const int w = pinned(c.tw), keep = pinned(c.keep), n_edges = pinned(c.n_edges), wi = w - 1;
  const DualArcs da = dual_arcs(w, c.th, st_t, gl_t);
  EdgeBits<NW> L;
  L.init(n_edges);
  int nrem = n_edges, count = n_edges;
  M RH = 0, RV = 0;          // removed tile edges: RH bit a = a|a+1 (horizontal), RV bit a = a|a+w
  CM RA = 0, RB = 0;         // interior corners wall-connected to arc A / arc B
  CM WE = 0, WS = 0;         // interior walls: WE bit k = corner k - k+1, WS bit k = corner k - k+wi
  while (count > keep && nrem > 0) {
    const int k = (int)pcg_draw(r, true, (uint32_t)nrem);  // nrem >= 2: always draws
    const int e = L.select(k);
    const uint32_t pk = epk[e], wl = ewl[e];
    L.clear(e);
    L.clear((int)(pk >> 17));
    nrem -= 2;
    const int p = (int)(wl & 255u), q = (int)(wl >> 8);
    const bool ap = corner_in<CM>(p, RA, da.ba), aq = corner_in<CM>(q, RA, da.ba);
    const bool bp = corner_in<CM>(p, RB, da.bb), bq = corner_in<CM>(q, RB, da.bb);
    if ((ap && bq) || (bp && aq)) continue;  // the wall would separate s from g: removal undone
    count -= 2;
    const bool hz = (pk >> 16) & 1u;
    const M ma = (M)1 << (pk & (sizeof(M) * 8 - 1));
    RH |= hz ? ma : (M)0;
    RV |= hz ? (M)0 : ma;
    if (ap != aq || bp != bq) {  // the wall attaches the other corner's component to an arc
      const bool toA = ap != aq;
      const int o = (toA ? ap : bp) ? q : p;  // interior (a boundary corner's side is fixed)
      CM C = (CM)1 << (o & (int)(sizeof(CM) * 8 - 1)), N;
      for (;;) {
        N = C | ((C & WE) << 1) | ((C >> 1) & WE) | ((C & WS) << wi) | ((C >> wi) & WS);
        if (N == C) break;
        C = N;
      }
      RA |= toA ? C : (CM)0;
      RB |= toA ? (CM)0 : C;
    }
    if ((p | q) < 64) {  // interior wall (the component floods above ran without it)
      const CM wb = (CM)1 << (min(p, q) & (int)(sizeof(CM) * 8 - 1));
      WS |= hz ? wb : (CM)0;
      WE |= hz ? (CM)0 : wb;
    }
  }
  hE &= ~RH;
  hW &= ~(RH << 1);
  hS &= ~RV;
  hN &= ~(RV << w);
}

template <int NW>
__device__ __forceinline__ void add_border_connections(const DevCfg& c, Pcg& r, uint16_t* plan) {
  EdgeBits<NW> B;
  B.init(c.n_border);
  int nb = c.n_border;
  for (int k = 0; k < c.n_border_add; k++) {
    const int j = B.select((int)pcg_int(r, (uint32_t)nb));
    B.clear(j);
    nb--;
    plan[sT.bt[j]] |= (uint16_t)(1u << sT.bd[j]);
  }
}

// generate_map (map_generator.py:43-189) -> tile plan (exits + obstacles) in LDS, start/goal
// (BIG: maps of > 64 tiles, 256-bit masks and the global edge table `epk`)
// `ix` (maps of <= 64 tiles, DevCfg::dual): the interior exit masks N, E, S, W of the generated graph,
// which compile_path_m takes instead of re-reading the plan.
template <bool BIG>
__device__ __forceinline__ void generate_map(const DevCfg& c, const uint32_t* __restrict__ epk, Pcg& r, uint16_t* plan,
                                             int& st_t, int& st_d, int& gl_t, int& gl_d, uint64_t* ix = nullptr) {
  const int w = c.tw;
  // chose_random_start_and_goal_position_and_direction (map_generator.py:475-571)
  int s0, s1, s2 = c.sdir, g0, g1, g2 = c.gdir;
  int slen, glen;
  if (c.start_mode == 2) {
    rand_pos(c, r, s0, s1);
    slen = 2;
  } else {
    s0 = c.sx != -1 ? c.sx : c.tw - 1;
    s1 = c.sy != -1 ? c.sy : c.th - 1;
    slen = c.start_mode == 1 ? 2 : 3;
  }
  if (c.goal_mode == 2) {
    rand_pos(c, r, g0, g1);
    glen = 2;
  } else {
    g0 = c.gx != -1 ? c.gx : c.tw - 1;
    g1 = c.gy != -1 ? c.gy : c.th - 1;
    glen = c.goal_mode == 1 ? 2 : 3;
  }
  int guard = 0;  // the reference loops forever on unsatisfiable settings; the kernel must not
  if (c.min_distance >= 0) {
    while (abs(s0 - g0) + abs(s1 - g1) < c.min_distance && ++guard < 100000) {
      rand_pos(c, r, s0, s1);
      slen = 2;
      rand_pos(c, r, g0, g1);
      glen = 2;
    }
  }
  if (slen == 2) s2 = rand_dir(c, r, s0, s1);
  if (glen == 2) g2 = rand_dir(c, r, g0, g1);
  while (s0 == g0 && s1 == g1 && s2 == g2 && ++guard < 100000) {
    if (c.start_mode == 2) rand_pos(c, r, s0, s1);
    if (c.start_mode != 0) s2 = rand_dir(c, r, s0, s1);
    if (c.goal_mode == 2) rand_pos(c, r, g0, g1);
    if (c.goal_mode != 0) g2 = rand_dir(c, r, g0, g1);
    if (c.start_mode == 0 && c.goal_mode == 0) break;  // rejected on the host
  }
  st_t = s1 * w + s0;
  st_d = s2;
  gl_t = g1 * w + g0;
  gl_d = g2;
  STAMP(13);

  // generate_map_graph (map_generator.py:192-266): full grid (host masks c.h0), then removals;
  // map_graph_to_tile_map_object (map_generator.py:269-334): exits straight into the LDS plan
  STAMP(14);
  if (BIG) {
    Bits<4> n = mask_h0<Bits<4>>(c, 0), e = mask_h0<Bits<4>>(c, 1), so = mask_h0<Bits<4>>(c, 2), we = mask_h0<Bits<4>>(c, 3);
    remove_edges<Bits<4>, 16>(c, epk, r, st_t, gl_t, n, e, so, we);
    for (int t = 0; t < c.nt; t++)
      plan[t] = (uint16_t)((uint32_t)mask_get(n, t) | (uint32_t)mask_get(e, t) << 1 | (uint32_t)mask_get(so, t) << 2 |
                           (uint32_t)mask_get(we, t) << 3);
  } else {
    uint64_t hN, hE, hS, hW;
    if (c.dual && c.nt <= 32) {
      uint32_t n = (uint32_t)c.h0[0][0], e = (uint32_t)c.h0[0][1], so = (uint32_t)c.h0[0][2], we = (uint32_t)c.h0[0][3];
      if (c.n_edges <= 64) remove_edges_dual<uint32_t, 1, uint32_t>(c, epk, sT.ewl, r, st_t, gl_t, n, e, so, we);
      else remove_edges_dual<uint32_t, 2, uint32_t>(c, epk, sT.ewl, r, st_t, gl_t, n, e, so, we);
      hN = n; hE = e; hS = so; hW = we;
    } else {
      hN = c.h0[0][0]; hE = c.h0[0][1]; hS = c.h0[0][2]; hW = c.h0[0][3];
      if (c.dual) remove_edges_dual<uint64_t, 4, uint64_t>(c, epk, sT.ewl, r, st_t, gl_t, hN, hE, hS, hW);
      else remove_edges<uint64_t, 4>(c, epk, r, st_t, gl_t, hN, hE, hS, hW);  // 1-wide maps, w + h > 31
    }
    if (c.dual) {
      // The exits stay in registers: add_connections_to_borders (map_generator.py:337-371) draws
      // candidate indices from the host's list (north row, east column from y = 1, south row, west
      // column up to y = h - 2 -- the two entries the reference removes), so the chosen set maps to
      // exit bits by arithmetic, and the plan is written once, two tiles per LDS word.
      ix[0] = hN; ix[1] = hE; ix[2] = hS; ix[3] = hW;
      const int h = c.th, nbd = pinned(c.n_border), nadd = pinned(c.n_border_add);
      const uint64_t all = (1ull << nbd) - 1ull;
      uint64_t B = all;
      for (int k = 0; k < nadd; k++) B &= ~(1ull << select64(B, (int)pcg_int(r, (uint32_t)(nbd - k))));
      const uint64_t ch = all & ~B, row = (1ull << w) - 1ull;
      uint64_t bE = 0, bW = 0;
      for (int y = 1; y < h; y++) {
        bE |= ((ch >> (w + y - 1)) & 1ull) << (y * w + w - 1);
        bW |= ((ch >> (2 * w + h - 2 + y)) & 1ull) << ((y - 1) * w);
      }
      const uint64_t sb = 1ull << st_t, gb = 1ull << gl_t;
      hN |= (ch & row) | (st_d == 0 ? sb : 0ull) | (gl_d == 0 ? gb : 0ull);
      hE |= bE | (st_d == 1 ? sb : 0ull) | (gl_d == 1 ? gb : 0ull);
      hS |= (((ch >> (w + h - 1)) & row) << ((h - 1) * w)) | (st_d == 2 ? sb : 0ull) | (gl_d == 2 ? gb : 0ull);
      hW |= bW | (st_d == 3 ? sb : 0ull) | (gl_d == 3 ? gb : 0ull);
      uint32_t* pw = reinterpret_cast<uint32_t*>(plan);
      for (int t = 0; t < c.nt; t += 2) {
        const uint64_t x0 = hN >> t, x1 = hE >> t, x2 = hS >> t, x3 = hW >> t;
        const uint32_t lo = (uint32_t)(x0 & 1ull) | (uint32_t)(x1 & 1ull) << 1 | (uint32_t)(x2 & 1ull) << 2 |
                            (uint32_t)(x3 & 1ull) << 3;
        const uint32_t hi = (uint32_t)(x0 & 2ull) >> 1 | (uint32_t)(x1 & 2ull) | (uint32_t)(x2 & 2ull) << 1 |
                            (uint32_t)(x3 & 2ull) << 2;
        pw[t >> 1] = lo | (t + 1 < c.nt ? hi << 16 : 0u);
      }
    } else {
      for (int t = 0; t < c.nt; t++)
        plan[t] = (uint16_t)((uint32_t)((hN >> t) & 1ull) | (uint32_t)((hE >> t) & 1ull) << 1 |
                             (uint32_t)((hS >> t) & 1ull) << 2 | (uint32_t)((hW >> t) & 1ull) << 3);
    }
  }
  STAMP(15);
  if (BIG || !c.dual) {
    plan[st_t] |= (uint16_t)(1u << st_d);
    plan[gl_t] |= (uint16_t)(1u << gl_d);
    // add_connections_to_borders (map_generator.py:337-371), candidate list from the host
    if (c.n_border <= 64) add_border_connections<1>(c, r, plan);
    else add_border_connections<3>(c, r, plan);
  }
  // add_obstacles_to_map (map_generator.py:374-472)
  if (c.obstacle_probability > 0.0) {
    for (int t = 0; t < c.nt; t++) {
      uint32_t e = plan[t];
      double u = pcg_double(r);
      if (u < c.obstacle_probability && e != 0u) {
        int ot = pcg_choice_cdf<4>(r, c.obst_cdf_t);
        uint32_t om;
        if (ot != 3) {
          om = pcg_int(r, 8);
        } else {
          // traffic-light masks in list order: north, east, south, west, north_and_south,
          // east_and_west (the last two only at >= 3 exits); option j <-> mask id 8 + j
          int n = __popc(e);
          uint32_t opt = (e & 15u) | (((e & 5u) == 5u && n >= 3) ? 16u : 0u) | (((e & 10u) == 10u && n >= 3) ? 32u : 0u);
          int k = (int)pcg_int(r, (uint32_t)__popc(opt));
          for (int j = 0; j < k; j++) opt &= opt - 1u;
          om = (uint32_t)(8 + __ffs((int)opt) - 1);
        }
        plan[t] = (uint16_t)(e | (uint32_t)(ot + 1) << 4 | om << 7);
      }
    }
  }
}

// parse_map_object's shortest path (graph-theory Dijkstra == FIFO BFS, neighbours N,E,S,W)
// -> subgoal directions in the plan; returns the path length (num_subgoals) or 0.
// parse_map_object's shortest_path (pgtg/parser.py:30-32, 244-306) on the tile exit graph, written as
// bit-parallel BFS layers from the goal (masks of type M) plus a greedy walk from the start that
// takes the first of north, east, south, west leading one layer closer.  That walk is the path a
// FIFO BFS with neighbour order N, E, S, W reconstructs (the assumed graph-theory tie-break,
// DESIGN.md section 2; checked against the queue BFS on random grids).  While the layers grow, the
// tiles whose N/E/S/W neighbour lies one layer closer are collected as masks, so the walk is
// register arithmetic.  Marks the direction to the next tile on every path tile but the goal's;
// returns the number of path tiles (0: unreachable).
// compile_path_m: the same from the interior exit masks (generate_map's `ix`), without the plan reads.
template <typename M>
__device__ __forceinline__ int compile_path_m(const DevCfg& c, uint16_t* plan, int s, int g, M hN, M hE, M hS, M hW,
                                              uint64_t* dirs = nullptr);
template <typename M>
__device__ __forceinline__ int compile_path(const DevCfg& c, uint16_t* plan, int s, int g) {
  M hN = mask_zero<M>(), hE = hN, hS = hN, hW = hN;
  for (int t = 0; t < c.nt; t++) {
    const uint32_t e = plan_exits(plan[t]);
    const M b = mask_bit<M>(t), z = mask_zero<M>();
    hN |= (e & 1u) ? b : z;
    hE |= (e & 2u) ? b : z;
    hS |= (e & 4u) ? b : z;
    hW |= (e & 8u) ? b : z;
  }
  hN &= mask_h0<M>(c, 0);  // interior exits only: border exits lead off the map
  hE &= mask_h0<M>(c, 1);
  hS &= mask_h0<M>(c, 2);
  hW &= mask_h0<M>(c, 3);
  return compile_path_m<M>(c, plan, s, g, hN, hE, hS, hW);
}
// dirs (<= 64 tiles): the path tiles per direction N, E, S, W are returned there instead of being
// marked in the plan (the map queue's entry write folds them into the words it stores)
template <typename M>
__device__ __forceinline__ int compile_path_m(const DevCfg& c, uint16_t* plan, int s, int g, M hN, M hE, M hS, M hW,
                                              uint64_t* dirs) {
  const int w = c.tw;
  STAMP(24);
  M vis = mask_bit<M>(g), front = vis;
  M cN = mask_zero<M>(), cE = cN, cS = cN, cW = cN;  // tiles with a neighbour one layer closer, per direction
  while (!mask_get(vis, s)) {
    const M nx = expand<M>(front, hN, hE, hS, hW, w) & ~vis;
    if (!mask_any(nx)) return 0;
    cN |= nx & hN & (front << w);
    cE |= nx & hE & (front >> 1);
    cS |= nx & hS & (front >> w);
    cW |= nx & hW & (front << 1);
    vis |= nx;
    front = nx;
  }
  STAMP(25);
  // (test knob: masks that disagree with the layers, on the maps whose tile 0 keeps its east exit)
  if ((c.tune_fault & 1) && mask_get(hE, 0)) cN = mask_zero<M>();
  // The walk is bounded: a shortest path moves at most nt - 1 times, and every tile it stands on must
  // have a tile one layer closer.  Masks that disagree with the BFS layers (the round-4 1-wide edge
  // directions did) end it with -1 (PGTG_E_DEVICE for the env) instead of a loop that never ends.
  int v = s, len = 1;
  if constexpr (sizeof(M) <= 8) {  // <= 64 tiles: the walk in registers, then the plan marks
    M pN = 0, pE = 0, pS = 0, pW = 0;
    while (v != g) {
      const M b = (M)1 << v;
      if (len >= c.nt || !((cN | cE | cS | cW) & b)) return -1;
      if (cN & b) { pN |= b; v -= w; }
      else if (cE & b) { pE |= b; v += 1; }
      else if (cS & b) { pS |= b; v += w; }
      else { pW |= b; v -= 1; }
      len++;
    }
    if (dirs) {
      dirs[0] = (uint64_t)pN;
      dirs[1] = (uint64_t)pE;
      dirs[2] = (uint64_t)pS;
      dirs[3] = (uint64_t)pW;
      return len;
    }
    for (M m = pN | pE | pS | pW; m; m &= m - 1) {
      const int t = __builtin_ctzll((uint64_t)m);
      const M b = (M)1 << t;
      const uint32_t d = (pN & b) ? 1u : (pE & b) ? 2u : (pS & b) ? 3u : 4u;
      plan[t] = (uint16_t)((plan[t] & ~(7u << 11)) | d << 11);
    }
  } else {  // larger maps: each path tile marked as the walk passes it
    while (v != g) {
      uint32_t d;
      int nv;
      if (len >= c.nt || !mask_get(cN | cE | cS | cW, v)) return -1;
      if (mask_get(cN, v)) { d = 1u; nv = v - w; }
      else if (mask_get(cE, v)) { d = 2u; nv = v + 1; }
      else if (mask_get(cS, v)) { d = 3u; nv = v + w; }
      else { d = 4u; nv = v - 1; }
      plan[v] = (uint16_t)((plan[v] & ~(7u << 11)) | d << 11);
      v = nv;
      len++;
    }
  }
  return len;
}

// The path of a map generate_map<BIG> just built: from its interior exit masks `ix` when it left them
// (small maps, DevCfg::dual), else from the plan.
// dirs: as compile_path_m's (maps of <= 64 tiles on the dual path; null otherwise, or the plan is marked)
template <bool BIG>
__device__ __forceinline__ int compile_generated(const DevCfg& c, uint16_t* plan, int s, int g, const uint64_t* ix,
                                                 uint64_t* dirs = nullptr) {
  if (BIG) return compile_path<Bits<4>>(c, plan, s, g);
  if (c.dual) {
    if (c.nt <= 32)
      return compile_path_m<uint32_t>(c, plan, s, g, (uint32_t)ix[0], (uint32_t)ix[1], (uint32_t)ix[2], (uint32_t)ix[3], dirs);
    return compile_path_m<uint64_t>(c, plan, s, g, ix[0], ix[1], ix[2], ix[3], dirs);
  }
  return c.nt <= 32 ? compile_path<uint32_t>(c, plan, s, g) : compile_path<uint64_t>(c, plan, s, g);
}

struct TrafState {
  uint32_t n_cars, n_spawners, next_id, tail;  // tail: car slots in use (cars and empty slots)
  uint32_t fresh;  // the cars are still in the env's staging block (traf.w kTrafFresh)
};

// spawner squares of local column lx of tile (tx, ty): lane-data spawners (dead ends) plus the
// border rule of pgtg/parser.py:120-148 ("car_lane all right" on the west border, ...)
__device__ __forceinline__ uint32_t spawner_colmask(const DevCfg& c, uint32_t ex, int tx, int ty, int lx) {
  if (!ex) return 0u;
  uint32_t m = sTX.spcol[ex][lx];
  if (tx == 0) m |= sTX.allcol[ex][3][lx];
  if (tx == c.tw - 1) m |= sTX.allcol[ex][2][lx];
  if (ty == 0) m |= sTX.allcol[ex][1][lx];
  if (ty == c.th - 1) m |= sTX.allcol[ex][0][lx];
  return m;
}

// Lanes of one wave exchanging LDS data: the wave's LDS accesses complete in program order, so a
// compiler fence at wavefront scope is all the ordering they need.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// One car of the initial traffic (pgtg/environment.py:840-879): square code -> lanes of the square
constexpr int kCarChunk = 4;  // cars whose lookups cars_group issues together
constexpr int kMaxGroup = 16;  // lanes of a wave that share one env in k_traffic
struct CarSquare {
  int x, y, tile, sq;
  uint32_t rl, nr;  // route lanes (kLanes bits 0..27) and their count
};
__device__ __forceinline__ CarSquare car_square(const DevCfg& c, const Plan& pl, uint32_t code) {
  CarSquare q;
  q.x = (int)(code & 255u);
  q.y = (int)(code >> 8);
  const int tx = (int)((uint32_t)q.x / (uint32_t)kTile), ty = (int)((uint32_t)q.y / (uint32_t)kTile);
  q.tile = ty * c.tw + tx;
  q.sq = (q.x - tx * kTile) * 9 + (q.y - ty * kTile);
  q.rl = sTX.lanes[plan_exits(pl[q.tile])][q.sq] & 0x0fffffffu;
  q.nr = __popc(q.rl);
  return q;
}
// the squares of cars m .. m+U-1 (indices clamped to mend-1, so every read is unconditional: a
// level's LDS reads go out together instead of one dependent chain per car)
template <int U>
__device__ __forceinline__ void car_squares(const DevCfg& c, const Plan& pl, const uint16_t* out, int m, int mend,
                                            CarSquare* q) {
  uint32_t code[U], p[U];
#pragma unroll
  for (int u = 0; u < U; u++) code[u] = out[min(m + u, mend - 1)];
#pragma unroll
  for (int u = 0; u < U; u++) {
    q[u].x = (int)(code[u] & 255u);
    q[u].y = (int)(code[u] >> 8);
    const int tx = (int)((uint32_t)q[u].x / (uint32_t)kTile), ty = (int)((uint32_t)q[u].y / (uint32_t)kTile);
    q[u].tile = ty * c.tw + tx;
    q[u].sq = (q[u].x - tx * kTile) * 9 + (q[u].y - ty * kTile);
    p[u] = pl[q[u].tile];
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    q[u].rl = sTX.lanes[plan_exits(p[u])][q[u].sq] & 0x0fffffffu;
    q[u].nr = __popc(q[u].rl);
  }
}
// A fresh car m of the env: w0 into the env's staging block (patience 0 and id m are implied by the
// fresh flag).  The lanes of a group write runs of consecutive words.
__device__ __forceinline__ void store_new_car(gu32* fw, const CarSquare& q, int route, int prof, int m) {
  fw[m] = (uint32_t)q.x | (uint32_t)q.y << 8 | (uint32_t)route << 16 | (uint32_t)prof << 21;
}

// The per-car draws on one lane, in id order: random() -> profile, then choice(routes) when the
// square has more than one route (numpy draws nothing for one).  `cr` enters as the stream after the
// shuffle and leaves after the last car.
__device__ __forceinline__ int cars_serial(const DevCfg& c, const CarSlots& cs, gu32* fw, const Plan& pl, const uint16_t* out,
                                        int k, int at, uint32_t* CR, Pcg& cr) {
  const ProfileCdf pcdf = pin_profile_cdf(c);
  PcgAhead ca = ahead_init(cr);
  CR[0] = CR[1] = CR[2] = 0u;
  for (int m = 0; m < k; m++) {
    const CarSquare q = car_square(c, pl, out[m]);
    if (q.tile == at) CR[q.sq >> 5] |= 1u << (q.sq & 31);
    if (q.nr == 0) return PGTG_E_MAP;  // "a car was spawned on a field where no car lane was found"
    const uint64_t u = ahead_draw(ca, false, 0u);
    const int prof = profile_of(pcdf, u);
    const uint32_t rk = q.nr > 1u ? (uint32_t)ahead_draw(ca, true, q.nr) : 0u;
    store_new_car(fw, q, sTX.lane_route[kth_bit(q.rl, (int)rk)], prof, m);
  }
  cr = ca.g;
  return 0;
}

// The same draws split over the g lanes of the env's group, lane `sub` taking cars [k sub/g,
// k (sub+1)/g).  Each car consumes one 64-bit output for its profile double and, when it has more
// than one route, one 32-bit half (numpy's next_uint32: the low half of a fresh output, whose high
// half is buffered for the next such draw; doubles do not touch the buffer).  So the stream position
// of every car follows from the counts of multi-route cars before it: the lanes count theirs, take
// prefix sums over the group, jump their copy of the stream there (pcg_advance) and draw their cars
// like the serial loop.  Lemire rejections (left < 2^32 mod n, probability < n / 2^32 per draw) would
// shift every later position: a group that meets one redoes the cars on one lane (cars_serial).
// Returns lane 0's result; on return every lane holds the stream after the last car in `cr` and
// lane 0 the group's agent-tile car squares in CR.
__device__ __forceinline__ int cars_group(const DevCfg& c, const CarSlots& cs, gu32* fw, const Plan& pl, const uint16_t* out,
                                          int k, int at, uint32_t* CR, Pcg& cr, int sub, int g) {
  const int q0 = (int)(threadIdx.x & 63u) - sub;  // the group's first lane
  // lane 0's post-shuffle stream to the group
  {
    const uint32_t a0 = __shfl((uint32_t)cr.shi, q0), a1 = __shfl((uint32_t)(cr.shi >> 32), q0);
    const uint32_t a2 = __shfl((uint32_t)cr.slo, q0), a3 = __shfl((uint32_t)(cr.slo >> 32), q0);
    const uint32_t a4 = __shfl(cr.buf, q0), a5 = __shfl(cr.has, q0);
    cr.shi = (uint64_t)a0 | (uint64_t)a1 << 32;
    cr.slo = (uint64_t)a2 | (uint64_t)a3 << 32;
    cr.buf = a4;
    cr.has = a5;
  }
  CR[0] = CR[1] = CR[2] = 0u;
  if (!c.kt_serial) {
    const int m0 = k * sub / g, m1 = k * (sub + 1) / g;
    // pass 1: the lane's multi-route cars (count, last one) and lane-less squares
    int cnt = 0, lastf = -1, bad = 0;
    for (int m = m0; m < m1; m += kCarChunk) {
      CarSquare q[kCarChunk];
      car_squares<kCarChunk>(c, pl, out, m, m1, q);
#pragma unroll
      for (int u = 0; u < kCarChunk; u++) {
        if (m + u < m1) {
          bad |= q[u].nr == 0u ? 1 : 0;
          cnt += q[u].nr > 1u ? 1 : 0;
          lastf = q[u].nr > 1u ? m + u : lastf;
        }
      }
    }
    int T = 0, prevf = -1;  // route draws before the lane's cars, the last multi-route car before them
    for (int j = 0; j < g; j++) {
      const int src = q0 + j;
      const int a = __shfl(cnt, src), lf = __shfl(lastf, src), bd = __shfl(bad, src);
      if (j < sub) {
        T += a;
        prevf = a > 0 ? lf : prevf;
      }
      bad |= bd;
    }
    if (bad) return PGTG_E_MAP;  // (the serial loop's error; cr stays the post-shuffle stream)
    // route draw t takes the buffered half when t < B0, else t' = t - B0 even: a fresh output, odd: the
    // buffered high half of draw t-1's output.  NC(t) = fresh outputs taken by draws 0 .. t-1.
    const int B0 = (int)cr.has;
    auto NC = [&](int t) { return t <= B0 ? 0 : (t - B0 + 1) >> 1; };
    const int nbits = c.kt_jump_bits;
    Pcg ls = cr;
    ls.has = 0u;
    if (T >= B0 && ((T - B0) & 1)) {  // the buffer holds the high half of the output of draw T-1
      Pcg q = cr;
      pcg_advance(q, (uint32_t)(prevf + 1 + NC(T - 1)), nbits);
      ls.buf = (uint32_t)(pcg_next64(q) >> 32);
      ls.has = 1u;
    } else if (T < B0) {
      ls.has = 1u;  // cr.buf
    }
    pcg_advance(ls, (uint32_t)(m0 + NC(T)), nbits);
    // pass 2: this lane's cars
    const ProfileCdf pcdf = pin_profile_cdf(c);
    PcgAhead ca = ahead_init(ls);
    int rej = 0;
    for (int m = m0; m < m1; m += kCarChunk) {
      CarSquare q[kCarChunk];
      car_squares<kCarChunk>(c, pl, out, m, m1, q);
      int prof[kCarChunk], lr[kCarChunk];
#pragma unroll
      for (int u = 0; u < kCarChunk; u++) {
        uint32_t rk = 0u;
        prof[u] = 0;
        if (m + u < m1) {
          if (q[u].tile == at) CR[q[u].sq >> 5] |= 1u << (q[u].sq & 31);
          prof[u] = profile_of(pcdf, ahead_next64(ca) >> 11);
          if (q[u].nr > 1u) {
            const uint64_t mm = (uint64_t)ahead_next32(ca) * q[u].nr;
            // a possible rejection (left < n; it is one iff left < 2^32 mod n): rare enough (n / 2^32)
            // to send the group to the serial loop without computing the modulo
            if ((uint32_t)mm < q[u].nr) rej = 1;
            rk = (uint32_t)(mm >> 32);
          }
        }
        lr[u] = max(select32(q[u].rl, (int)rk), 0);  // (a lane-less square of a clamped index reads row 0)
      }
      int route[kCarChunk];
#pragma unroll
      for (int u = 0; u < kCarChunk; u++) route[u] = sTX.lane_route[lr[u]];
#pragma unroll
      for (int u = 0; u < kCarChunk; u++)
        if (m + u < m1) store_new_car(fw, q[u], route[u], prof[u], m + u);
    }
    ls = ca.g;
    // the group's rejections; the stream after the last car is lane g-1's; CR merged on lane 0
    const int last = q0 + g - 1;
    uint32_t f0 = __shfl((uint32_t)ls.shi, last), f1 = __shfl((uint32_t)(ls.shi >> 32), last);
    uint32_t f2 = __shfl((uint32_t)ls.slo, last), f3 = __shfl((uint32_t)(ls.slo >> 32), last);
    uint32_t f4 = __shfl(ls.buf, last), f5 = __shfl(ls.has, last);
    uint32_t cr0 = 0u, cr1 = 0u, cr2 = 0u;
    for (int j = 0; j < g; j++) {
      const int src = q0 + j;
      cr0 |= __shfl(CR[0], src);
      cr1 |= __shfl(CR[1], src);
      cr2 |= __shfl(CR[2], src);
      rej |= __shfl(rej, src);
    }
    if (!rej) {
      CR[0] = cr0;
      CR[1] = cr1;
      CR[2] = cr2;
      cr.shi = (uint64_t)f0 | (uint64_t)f1 << 32;
      cr.slo = (uint64_t)f2 | (uint64_t)f3 << 32;
      cr.buf = f4;
      cr.has = f5;
      return 0;
    }
  }
  // one lane: the tune_kt_serial path, or a group whose draw positions a rejection shifted (redo)
  return sub == 0 ? cars_serial(c, cs, fw, pl, out, k, at, CR, cr) : 0;
}

// The draws of Generator.choice(np, k, replace=False) (numpy _generator.pyx: Floyd's loop over
// j = np-k .. np-1 drawing integers(0, j+1), then _shuffle_int drawing integers(0, m+1) for m = k-1
// .. 1), split over the g lanes of the env's group: draw d < k is Floyd's (n = np-k+d+1), d >= k the
// shuffle's (n = 2k-d).  Every draw with n > 1 takes one 32-bit half of the car stream (next_uint32:
// the low half of a fresh output, then its buffered high half), so draw d's half is known up front:
// lane `sub` jumps its copy of the stream to its first draw and evaluates its stretch [D sub/g,
// D (sub+1)/g) of the D = 2k-1 draws into out[d] / jj[d-k].  A Lemire rejection (left < 2^32 mod n)
// takes an extra half and shifts every later draw by one: the group finds its first rejected draw and
// re-evaluates from there with the shift, until none is left.  On return every lane holds the stream
// after the last draw in `cr`.
__device__ __forceinline__ void choice_draws_group(const DevCfg& c, uint16_t* out, uint16_t* jj, int np, int k, Pcg& cr,
                                                   int sub, int g) {
  const int q0 = (int)(threadIdx.x & 63u) - sub;
  const int D = 2 * k - 1, da = D * sub / g, db = D * (sub + 1) / g;
  const int z = np - k + 1 <= 1 ? 1 : 0;  // Floyd's first draw with n == 1 draws nothing
  const int B = (int)cr.has;
  const int nbits = c.kt_jump_bits + 1;
  int shift = 0, dstart = 0;
  Pcg ls = cr;
  for (;;) {
    const int d0 = max(da, dstart);
    // the stream at the first half this lane takes: half h -> buffered (h < B) or output (h-B)/2
    const int h0 = max(d0 - z, 0) + shift;
    ls = cr;
    if (h0 >= B) {
      const int hb = h0 - B;
      pcg_advance(ls, (uint32_t)(hb >> 1), nbits);
      ls.has = 0u;
      if (hb & 1) {  // the first draw takes the high half of output hb/2
        ls.buf = (uint32_t)(pcg_next64(ls) >> 32);
        ls.has = 1u;
      }
    }
    int rej = 0x7fffffff;
    for (int d = d0; d < db; d++) {
      const uint32_t n = d < k ? (uint32_t)(np - k + d + 1) : (uint32_t)(2 * k - d);
      uint32_t v = 0u;
      if (n > 1u) {
        const uint64_t mm = (uint64_t)pcg_next32(ls) * n;
        const uint32_t left = (uint32_t)mm;
        if (left < n && left < (0xffffffffu - (n - 1u)) % n && rej == 0x7fffffff) rej = d;
        v = (uint32_t)(mm >> 32);
      }
      if (d < k) out[d] = (uint16_t)v;
      else jj[d - k] = (uint16_t)v;
    }
    int first = rej;
    for (int j = 0; j < g; j++) first = min(first, __shfl(rej, q0 + j));
    if (first == 0x7fffffff) break;
    dstart = first;  // draws before it stand; it and the later ones take one half more
    shift++;
  }
  // the stream after the last draw: lane g-1's (its stretch ends at D; with an empty stretch, the
  // jump above landed exactly there)
  const int last = q0 + g - 1;
  const uint32_t f0 = __shfl((uint32_t)ls.shi, last), f1 = __shfl((uint32_t)(ls.shi >> 32), last);
  const uint32_t f2 = __shfl((uint32_t)ls.slo, last), f3 = __shfl((uint32_t)(ls.slo >> 32), last);
  const uint32_t f4 = __shfl(ls.buf, last), f5 = __shfl(ls.has, last);
  cr.shi = (uint64_t)f0 | (uint64_t)f1 << 32;
  cr.slo = (uint64_t)f2 | (uint64_t)f3 << 32;
  cr.buf = f4;
  cr.has = f5;
}

// Initial traffic of a fresh episode (EpisodeMap scans pgtg/map.py:31-42 and
// _create_initial_traffic pgtg/environment.py:830-879), run by k_traffic for the envs k_env reset.
// `g` (1..kMaxGroup) adjacent lanes of a wave share one env (`sub` 0..g-1): lane 0 runs the serial parts
// (Floyd's choice, the shuffle, the per-car draws in id order); the sweep and the square lookup of
// every chosen index, which have no RNG and no order, are split over the group.  `rs` is the env's
// LDS reset scratch: Floyd's output [0, 2*cap) (then the chosen square codes), its seen set, the
// per-column prefix of spawnable squares and (maps of <= 7 tile rows) each column's row mask.  CR
// collects the new cars on the agent's tile `at` (observation); lane 0's return value, state and CR
// are the result.
__device__ __forceinline__ int traffic_reset(const DevCfg& c, const DevState& S, uint64_t i, const Plan& pl,
                                             Pcg& cr, uint8_t* rs, TrafState& ts, int at, uint32_t* CR, int sub,
                                             int g) {
  STAMP(19);
  // x-major sweep, the group's lanes on g column ranges: count, exchange the counts, then car
  // spawners -> HBM list and spawnable squares (any car lane) -> per-column prefix counts
  uint16_t* colpre = reinterpret_cast<uint16_t*>(rs + c.rs_pre_off);
  const int xa = c.W * sub / g, xb = c.W * (sub + 1) / g;
  int cnp = 0, cnsp = 0;
  for (int x = xa; x < xb; x++) {
    const int tx = x / kTile, lx = x - tx * kTile;
    for (int ty = 0; ty < c.th; ty++) {
      const uint32_t ex = plan_exits(pl[ty * c.tw + tx]);
      cnp += __popc(sTX.lanecol[ex][lx]);  // row 0 (no exits) is empty
      cnsp += __popc(spawner_colmask(c, ex, tx, ty, lx));
    }
  }
  const int q0 = (int)(threadIdx.x & 63u) - sub;
  int np = 0, nsp = 0, tot_np = 0, tot_nsp = 0;
  for (int j = 0; j < g; j++) {  // (g is wave-uniform: every lane runs every shuffle)
    const int a = __shfl(cnp, q0 + j), b = __shfl(cnsp, q0 + j);
    np += j < sub ? a : 0;
    nsp += j < sub ? b : 0;
    tot_np += a;
    tot_nsp += b;
  }
  uint32_t* colm = c.rs_cm_off ? reinterpret_cast<uint32_t*>(rs + c.rs_cm_off) : nullptr;
  for (int x = xa; x < xb; x++) {
    const int tx = x / kTile, lx = x - tx * kTile;
    colpre[x] = (uint16_t)np;
    uint64_t cm = 0;
    for (int ty = 0; ty < c.th; ty++) {
      const uint32_t ex = plan_exits(pl[ty * c.tw + tx]);
      const uint32_t lc = sTX.lanecol[ex][lx];
      np += __popc(lc);
      cm |= (uint64_t)lc << (9 * (ty & 7));
      uint32_t m = spawner_colmask(c, ex, tx, ty, lx);
      while (m) {
        int ly = __ffs((int)m) - 1;
        m &= m - 1u;
        if (nsp < c.max_spawners) S.spawners[i * (uint64_t)S.sp_pitch + nsp] = (uint16_t)(x | (ty * kTile + ly) << 8);
        nsp++;
      }
    }
    if (colm) {
      colm[2 * x] = (uint32_t)cm;
      colm[2 * x + 1] = (uint32_t)(cm >> 32);
    }
  }
  np = tot_np;
  nsp = tot_nsp;
  if (sub == g - 1) colpre[c.W] = (uint16_t)np;
  wave_lds_sync();
  const int ncars = (int)((double)np * c.density);  // int(len(positions) * traffic_density)
  int k = 0;
  const CarSlots cs(S, i);
  if (ncars > 0 && np > 0) {
    k = min(ncars, np);
    if (k > c.car_cap) return PGTG_E_UNSUPPORTED;
    uint16_t* out = reinterpret_cast<uint16_t*>(rs);
    uint16_t* jj = reinterpret_cast<uint16_t*>(rs + c.rs_jj_off);
    uint32_t* seen = reinterpret_cast<uint32_t*>(rs + c.rs_seen_off);
    if (sub == 0)
      for (int w = 0; w < (np + 31) / 32; w++) seen[w] = 0u;
    STAMP(20);
    // Generator.choice(np, k, replace=False): Floyd's algorithm, then _shuffle_int.  Their draws
    // (values independent of the outcomes) are evaluated lane-parallel into out / jj
    // (choice_draws_group); the set and swap bookkeeping stays in order on lane 0.
    choice_draws_group(c, out, jj, np, k, cr, sub, g);
    wave_lds_sync();
    if (sub == 0) {
      for (int d = 0; d < k; d++) {
        const int j = np - k + d;
        int val = out[d];
        if ((seen[val >> 5] >> (val & 31)) & 1u) val = j;
        seen[val >> 5] |= 1u << (val & 31);
        out[d] = (uint16_t)val;
      }
      STAMP(21);
      for (int m = k - 1; m >= 1; m--) {
        const int q = jj[k - 1 - m];
        const uint16_t t = out[m], u = out[q];
        out[m] = u;
        out[q] = t;
      }
    }
    wave_lds_sync();
    STAMP(22);
    const int tw = c.tw, th = c.th;
    // the group looks up the squares: chosen index -> square code x | y << 8 in place, lane `sub` on
    // indices [k sub/g, k (sub+1)/g), kCarChunk at a time (each level's LDS reads issued together)
    const int la = k * sub / g, lb = k * (sub + 1) / g;
    for (int m = la; m < lb; m += kCarChunk) {
      int idx[kCarChunk], tx[kCarChunk];
#pragma unroll
      for (int u = 0; u < kCarChunk; u++) {
        idx[u] = out[min(m + u, lb - 1)];
        tx[u] = 0;
      }
      // column: the tile column from the prefixes at tile-column starts, then the column inside it
      for (int q = 1; q < tw; q++) {
        const int cv = colpre[q * kTile];
#pragma unroll
        for (int u = 0; u < kCarChunk; u++) tx[u] += cv <= idx[u] ? 1 : 0;
      }
      int cpv[kCarChunk][kTile];
#pragma unroll
      for (int u = 0; u < kCarChunk; u++)
#pragma unroll
        for (int j = 0; j < kTile; j++) cpv[u][j] = colpre[tx[u] * kTile + j];
      int x[kCarChunk], rr[kCarChunk];
#pragma unroll
      for (int u = 0; u < kCarChunk; u++) {
        int lx = 0, base = cpv[u][0];
#pragma unroll
        for (int j = 1; j < kTile; j++) {
          const bool le = cpv[u][j] <= idx[u];
          lx += le ? 1 : 0;
          base = le ? cpv[u][j] : base;
        }
        x[u] = tx[u] * kTile + lx;
        rr[u] = idx[u] - base;
      }
      int y[kCarChunk];
      if (colm) {  // row: the rr-th set bit of the column's row mask
        uint32_t wl[kCarChunk], wh[kCarChunk];
#pragma unroll
        for (int u = 0; u < kCarChunk; u++) {
          wl[u] = colm[2 * x[u]];
          wh[u] = colm[2 * x[u] + 1];
        }
#pragma unroll
        for (int u = 0; u < kCarChunk; u++) {
          uint32_t w = wl[u];
          int r = rr[u], base = 0;
          const int c32 = __popc(w);
          if (r >= c32) {
            r -= c32;
            w = wh[u];
            base = 32;
          }
#pragma unroll
          for (int sh = 16; sh >= 1; sh >>= 1) {
            const int cnt = __popc(w & ((1u << sh) - 1u));
            if (r >= cnt) {
              r -= cnt;
              w >>= sh;
              base += sh;
            }
          }
          y[u] = base;
        }
      } else {  // row: the tile of the column holding the rr-th spawnable square (no early exit)
#pragma unroll
        for (int u = 0; u < kCarChunk; u++) {
          const int txu = x[u] / kTile, lx = x[u] - txu * kTile;
          int ty_f = 0, rr_f = 0, r = rr[u];
          uint32_t msk_f = 0;
          for (int ty = 0; ty < th; ty++) {
            const uint32_t msk = sTX.lanecol[plan_exits(pl[ty * tw + txu])][lx];
            const int cnt = __popc(msk);
            if (r >= 0 && r < cnt) {
              ty_f = ty;
              msk_f = msk;
              rr_f = r;
            }
            r -= cnt;
          }
          y[u] = ty_f * kTile + kth_bit(msk_f, rr_f);
        }
      }
#pragma unroll
      for (int u = 0; u < kCarChunk; u++)
        if (m + u < lb) out[m + u] = (uint16_t)(x[u] | y[u] << 8);
    }
    wave_lds_sync();
    STAMP(26);  // (slot shared with k_env's removal-loop record: k_traffic runs later)
    // the cars in id order: profile and route draws -> slots 0 .. k-1 (lane-parallel, see cars_group)
    const int e = cars_group(c, cs, fresh_block(S, i), pl, out, k, at, CR, cr, sub, g);
    if (e) return sub == 0 ? e : 0;
    if (sub != 0) return 0;
  }
  STAMP(23);
  ts.n_cars = (uint32_t)k;
  ts.n_spawners = (uint32_t)min(nsp, c.max_spawners);
  ts.next_id = (uint32_t)k;
  ts.tail = (uint32_t)k;
  return 0;
}

// The occupancy counters of a fresh env's k cars (square codes x | y << 8 in out[0, k), one car per
// square: no counter overflows) for k_env, which loads them instead of rebuilding them from the car
// slots.  The g lanes of the env's group count into `cnt` (the reset scratch from rs_jj_off, free
// once the cars exist) with LDS adds and store the nt * 4 words to the env's staging block.
__device__ __forceinline__ void store_initial_counters(const DevCfg& c, const DevState& S, uint64_t i, const Plan& pl,
                                                       uint8_t* rs, int k, int sub, int g) {
  uint32_t* cnt = reinterpret_cast<uint32_t*>(rs + c.rs_jj_off);
  const uint16_t* out = reinterpret_cast<const uint16_t*>(rs);
  const int nw = c.nt * 4;
  for (int w = sub; w < nw; w += g) cnt[w] = 0u;
  wave_lds_sync();
  for (int m = k * sub / g; m < k * (sub + 1) / g; m++) {
    const uint32_t code = out[m];
    const int s = lane_slot(c, pl, (int)(code & 255u), (int)(code >> 8));
    if (s >= 0) __hip_atomic_fetch_add(cnt + (s >> 3), 1u << ((s & 7) << 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  }
  wave_lds_sync();
  gu32* fo = fresh_block(S, i) + S.fresh_occ;
  for (int w = sub; w < nw; w += g) fo[w] = cnt[w];
}

// The full per-env reset.  `key` = spawn counter (5 children per episode).  Returns 0 or -code.
template <bool TR, bool BIG>
__device__ __forceinline__ int env_reset(const DevCfg& c, const DevState& S, uint64_t i, EnvView& v, uint16_t* plan,
                                         TrafState& ts) {
  STAMP(8);
  uint64_t seed = S.seed[i];
  SeedPool sp = ss_pool(seed);
  uint32_t k = v.spawn;
  Pcg map_rng = ss_child(sp, k + 0u);
  Pcg car_rng;
  if ((TR && c.need_car)) car_rng = ss_child(sp, k + 1u);
  if (c.need_ice) stream_store_all(S.ice, i, ss_child(sp, k + 2u));
  if (c.need_broken) stream_store_all(S.broken, i, ss_child(sp, k + 3u));
  if (c.need_sand) stream_store_all(S.sand, i, ss_child(sp, k + 4u));
  v.spawn = k + 5u;
  STAMP(9);
  int st_t, st_d, gl_t, gl_d;
  int len;
  if (c.fixed_map) {
    for (int t = 0; t < c.nt; t++) plan[t] = c.fixed_plan[t];
    st_t = (int)(c.fixed_sg & 0xffu);
    st_d = (int)((c.fixed_sg >> 8) & 0xffu);
    gl_t = (int)((c.fixed_sg >> 16) & 0xffu);
    gl_d = (int)(c.fixed_sg >> 24);
    STAMP(10);
    len = BIG ? compile_path<Bits<4>>(c, plan, st_t, gl_t)
              : (c.nt <= 32 ? compile_path<uint32_t>(c, plan, st_t, gl_t) : compile_path<uint64_t>(c, plan, st_t, gl_t));
  } else {
    uint64_t ix[4];
    generate_map<BIG>(c, BIG ? S.epk : sT.epk, map_rng, plan, st_t, st_d, gl_t, gl_d, ix);
    STAMP(10);
    len = compile_generated<BIG>(c, plan, st_t, gl_t, ix);
  }
  v.sg = (uint32_t)st_t | (uint32_t)st_d << 8 | (uint32_t)gl_t << 16 | (uint32_t)gl_d << 24;
  STAMP(11);
  v.used = 0;
  v.path_len = (uint32_t)max(len, 0);
  v.flags = 0;
  v.phase = 0;
  v.elapsed = 0;
  v.vx = v.vy = 0;
  if (len <= 0 || !((plan_exits(plan[st_t]) >> st_d) & 1u)) {
    v.px = v.py = 0;
    return len < 0 ? PGTG_E_DEVICE : PGTG_E_MAP;  // (< 0: the path walk's masks were inconsistent)
  }
  // starters: the start tile's exit segment in the start direction, x-major (pgtg/map.py:31-34)
  int j = (int)pcg_int(map_rng, 3);
  int tx = st_t % c.tw, ty = st_t / c.tw, lx, ly;
  switch (st_d) {
    case 0: lx = 3 + j; ly = 0; break;
    case 1: lx = 8; ly = 3 + j; break;
    case 2: lx = 3 + j; ly = 8; break;
    default: lx = 0; ly = 3 + j; break;
  }
  v.px = tx * kTile + lx;
  v.py = ty * kTile + ly;
  STAMP(12);
  if (S.visited) {
    uint32_t* vis = S.visited + i * (uint64_t)c.vis_words;
    for (int q2 = 0; q2 < c.vis_words; q2++) vis[q2] = 0;
    int b = (v.px + 2) * c.vis_pitch + (v.py + 2);
    vis[b >> 5] |= 1u << (b & 31);
  }
  if ((TR && c.need_car)) {  // the cars are created by k_traffic from this stream
    stream_store_all(S.car, i, car_rng);
    ts = TrafState{0, 0, 0, 0};
  }
  return 0;
}

// ------------------------------------------------------------------------------------------------
// observation -> per-channel bitmasks in LDS (pgtg/environment.py:1344-1506)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t chan_bit(int code, uint32_t f, uint32_t lanes, bool spawner, int color) {
  switch (code) {
    case PGTG_CH_WALL: return f & SQ_WALL ? 1u : 0u;
    case PGTG_CH_GOALS: return f & (SQ_SUBGOAL | SQ_FINAL) ? 1u : 0u;
    case PGTG_CH_TL_GREEN: return (color == 0 && (f & SQ_TLIGHT)) ? 1u : 0u;
    case PGTG_CH_TL_YELLOW: return (color == 1 && (f & SQ_TLIGHT)) ? 1u : 0u;
    case PGTG_CH_TL_RED: return (color == 2 && (f & SQ_TLIGHT)) ? 1u : 0u;
    case PGTG_CH_START: return f & SQ_START ? 1u : 0u;
    case PGTG_CH_SUBGOAL: return f & SQ_SUBGOAL ? 1u : 0u;
    case PGTG_CH_USED_SUBGOAL: return f & SQ_USED ? 1u : 0u;
    case PGTG_CH_FINAL_GOAL: return f & SQ_FINAL ? 1u : 0u;
    case PGTG_CH_ICE: return f & SQ_ICE ? 1u : 0u;
    case PGTG_CH_BROKEN: return f & SQ_BROKEN ? 1u : 0u;
    case PGTG_CH_SAND: return f & SQ_SAND ? 1u : 0u;
    case PGTG_CH_SPAWNER: return spawner ? 1u : 0u;
    default:
      if (code >= PGTG_CH_LANE0 && code < PGTG_CH_LANE0 + 32) return (lanes >> (code - PGTG_CH_LANE0)) & 1u;
      return 0u;
  }
}

struct ObsInfo {
  int x0, y0;          // window origin
  int posx, posy;      // observation position
  int nsd;             // next_subgoal_direction
};

// nearest subgoal / final goal square from (x, y): min Manhattan, x-major first (environment.py:1471-1480)
template <bool BIG>
__device__ __forceinline__ bool nearest_goal_square(const DevCfg& c, const Plan& pl, const EnvView& v, int x, int y, int& bx, int& by) {
  int best = 0x7fffffff;
  bool found = false;
  int gl_t = (int)((v.sg >> 16) & 0xffu), gl_d = (int)(v.sg >> 24);
  for (int t = 0; t < c.nt; t++) {
    uint32_t p = pl[t];
    int d = -1;
    int sd = plan_sgdir(p);
    if (sd >= 0 && !used_bit<BIG>(v, p, t)) d = sd;
    for (int pass = 0; pass < 2; pass++) {
      int dd = pass == 0 ? d : (t == gl_t ? gl_d : -1);
      if (dd < 0) continue;
      int tx = (t % c.tw) * kTile, ty = (t / c.tw) * kTile;
      for (int j = 0; j < 3; j++) {
        int sx, sy;
        switch (dd) {
          case 0: sx = tx + 3 + j; sy = ty; break;
          case 1: sx = tx + 8; sy = ty + 3 + j; break;
          case 2: sx = tx + 3 + j; sy = ty + 8; break;
          default: sx = tx; sy = ty + 3 + j; break;
        }
        int dist = abs(sx - x) + abs(sy - y);
        if (!found || dist < best || (dist == best && (sx < bx || (sx == bx && sy < by)))) {
          found = true;
          best = dist;
          bx = sx;
          by = sy;
        }
      }
    }
  }
  return found;
}

// The observation image in LDS is a dense bit stream in output byte order: bit k = byte k of the
// image's slice of the uint8 output (env slot e, channel ci, window square b at bit
// e*C*WW + ci*WW + b).  A writer then turns any 16 consecutive bits into one 16-byte store with a
// funnel shift, whatever the window size.  An env's first and last words are shared with its
// neighbours in the stream and are merged with LDS and/or atomics (the neighbours' bits are
// disjoint, so concurrent merges commute); the words in between are plain stores.
struct BitSink {
  uint32_t* st;
  uint32_t w, fill, own;  // current word, bits held, bits of the current word this env owns
  uint64_t acc;
  __device__ __forceinline__ BitSink(uint32_t* s, uint32_t bit0)
      : st(s), w(bit0 >> 5), fill(bit0 & 31u), own(~0u << (bit0 & 31u)), acc(0) {}
  __device__ __forceinline__ void emit(uint32_t val, uint32_t mask) {
    if (mask == ~0u) {
      st[w] = val;
    } else {
      __hip_atomic_fetch_and(st + w, ~mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_or(st + w, val & mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  // append the n (1..32) low bits of val (higher bits zero)
  __device__ __forceinline__ void put(uint32_t val, uint32_t n) {
    acc |= (uint64_t)val << fill;
    fill += n;
    if (fill >= 32u) {
      emit((uint32_t)acc, own);
      own = ~0u;
      acc >>= 32;
      fill -= 32u;
      w++;
    }
  }
  // append n zero bits (a run of all-zero channels): whole words become plain zero stores
  __device__ __forceinline__ void skip(uint32_t n) {
    fill += n;
    if (fill >= 32u) {
      emit((uint32_t)acc, own);
      own = ~0u;
      acc = 0;
      fill -= 32u;
      w++;
      for (; fill >= 32u; fill -= 32u) st[w++] = 0u;
    }
  }
  __device__ __forceinline__ void finish() {
    if (fill) emit((uint32_t)acc, own & ((1u << fill) - 1u));
  }
};

template <typename T>
__device__ __forceinline__ T sel4(int k, T a0, T a1, T a2, T a3) {
  return k == 0 ? a0 : (k == 1 ? a1 : (k == 2 ? a2 : a3));
}

// One channel's 81 bits (3 words, square lx * 9 + ly) on tile t of the map: the tile tables' algebra of
// build_obs's one-tile fast path, for any channel code but the lane and spawner ones (square_flags and
// chan_bit semantics; occ: the tile counters of k_env<true>, null elsewhere).
template <bool TR, bool BIG>
__device__ __forceinline__ void tile_chan(const DevCfg& c, const EnvView& v, uint32_t p, int t, int code, int color,
                                          const uint8_t* occ, uint32_t (&m)[3]) {
  const uint32_t ex = plan_exits(p), ot = plan_otype(p);
  const int sd = plan_sgdir(p);
  const bool used = used_bit<BIG>(v, p, t);
  const int st_t = (int)(v.sg & 0xffu), st_d = (int)((v.sg >> 8) & 0xffu);
  const int gl_t = (int)((v.sg >> 16) & 0xffu), gl_d = (int)(v.sg >> 24);
  const bool sg_on = sd >= 0 && ((ex >> sd) & 1u), fi_on = t == gl_t && ((ex >> gl_d) & 1u);
  const bool st_on = t == st_t && ((ex >> st_d) & 1u);
  const uint32_t om = min(plan_omask(p), (uint32_t)PGTG_N_OBST_MASKS - 1u);
  // the obstacle kind this code shows (ice 1, broken road 2, sand 3, a light of the current colour 4)
  const uint32_t okind = code == PGTG_CH_ICE ? 1u : code == PGTG_CH_BROKEN ? 2u : code == PGTG_CH_SAND ? 3u
                       : (code == PGTG_CH_TL_GREEN && color == 0) || (code == PGTG_CH_TL_YELLOW && color == 1) ||
                         (code == PGTG_CH_TL_RED && color == 2) ? 4u : 0u;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint32_t W3 = sT.wall[ex][k];
    const uint32_t sgk = sT.seg[sd >= 0 ? sd : 0][k], fik = sT.seg[gl_d & 3][k], stk = sT.seg[st_d & 3][k];
    const uint32_t obk = sT.obst[om][k] & ~W3;
    const uint32_t SG = sg_on && !used ? sgk : 0u, US = sg_on && used ? sgk : 0u;
    const uint32_t FI = fi_on ? fik : 0u, ST = st_on ? stk : 0u;
    uint32_t val;
    switch (code) {
      case PGTG_CH_WALL: val = W3; break;
      case PGTG_CH_GOALS: val = SG | FI; break;
      case PGTG_CH_START: val = ST; break;
      case PGTG_CH_SUBGOAL: val = SG; break;
      case PGTG_CH_USED_SUBGOAL: val = US; break;
      case PGTG_CH_FINAL_GOAL: val = FI; break;
      default: val = (okind != 0u && ot == okind) ? obk : 0u; break;  // obstacles, lights; others zero
    }
    m[k] = val;
  }
  if (TR && code == PGTG_CH_TRAFFIC) {
    m[0] = m[1] = m[2] = 0u;
    if (c.need_car && occ && ex) {
      const uint32_t* ow = reinterpret_cast<const uint32_t*>(occ + t * 16);  // the tile's 32 nibbles
#pragma unroll
      for (int q = 0; q < 4; q++) {
        uint32_t nz = (ow[q] | (ow[q] >> 1) | (ow[q] >> 2) | (ow[q] >> 3)) & 0x11111111u;  // nonzero nibbles
        while (nz) {
          const int sq = sTX.slot_sq[ex][q * 8 + ((__ffs((int)nz) - 1) >> 2)];
          nz &= nz - 1u;
          const uint32_t b = 1u << (sq & 31);
          m[0] |= (sq >> 5) == 0 ? b : 0u;
          m[1] |= (sq >> 5) == 1 ? b : 0u;
          m[2] |= (sq >> 5) == 2 ? b : 0u;
        }
      }
    }
  }
}

// Observation of one env into the image at bit offset bit0 (see BitSink): channel by channel, each
// the window's squares row-major over x, then y.
// Channels [ch_lo, ch_hi) only (default all) when the lanes of a group share one env's image (the
// group's sinks merge at their shared words); `head`: also the next-subgoal direction.
template <bool TR, bool BIG, bool LC = true, bool ZS = true>  // LC: lane / spawner channels possible (they read sTX);
                                                               // ZS: all-zero channels appended as zero runs
__device__ __forceinline__ void build_obs(const DevCfg& c, const DevState& S, const Plan& pl, const EnvView& v,
                                          uint32_t* img, uint32_t bit0, ObsInfo& oi, const uint8_t* occ,
                                          int ch_lo = 0, int ch_hi = -1, bool head = true, bool lane_codes = false,
                                          bool occ_tile_only = false) {  // occ: the agent tile's 16 bytes only
#ifdef PGTG_STAMPS_OBS  // diagnostic: build_obs's setup (k_envq env waves only: slots 9-11 are free there)
  STAMP(9);
#endif
  const int WW = c.win * c.win;
  if (ch_hi < 0) ch_hi = c.n_channels;
  BitSink sink(img, bit0 + (uint32_t)(ch_lo * WW));
  int pix = min(max(0, v.px), c.W - 1), piy = min(max(0, v.py), c.H - 1);
  int tx = pix / kTile, ty = piy / kTile;
  int color = phase_color(c, v.phase);
  if (!c.sliding) {
    oi.x0 = tx * kTile;
    oi.y0 = ty * kTile;
    oi.posx = pix - oi.x0;
    oi.posy = piy - oi.y0;
  } else {
    oi.x0 = v.px - c.ss;
    oi.y0 = v.py - c.ss;
    oi.posx = oi.posy = c.ss;
  }
  if (!c.sliding && !c.generic_channels) {
    // fast path: the window is exactly one tile -> 81-bit table algebra
    int t = ty * c.tw + tx;
#ifdef PGTG_STAMPS_OBS
    STAMP(10);
#endif
    uint32_t p = pl[t];
    uint32_t ex = plan_exits(p);
#ifdef PGTG_STAMPS_OBS
    if (ex == 99u) ex = 0u;  // (forces the plan read before the stamp below)
    STAMP(11);
#endif
    uint32_t W3[3], SG[3] = {0, 0, 0}, US[3] = {0, 0, 0}, FI[3] = {0, 0, 0}, ST[3] = {0, 0, 0}, OB[3] = {0, 0, 0};
    int sd = plan_sgdir(p);
    bool used = used_bit<BIG>(v, p, t);
    int st_t = (int)(v.sg & 0xffu), st_d = (int)((v.sg >> 8) & 0xffu);
    int gl_t = (int)((v.sg >> 16) & 0xffu), gl_d = (int)(v.sg >> 24);
    uint32_t ot = plan_otype(p);
    uint32_t CR[3] = {0, 0, 0};  // squares of this tile holding a car
    if ((TR && c.need_car) && occ && ex) {
      const uint32_t* ow = reinterpret_cast<const uint32_t*>(occ + (occ_tile_only ? 0 : t * 16));  // the tile's 32 nibbles
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t wv = ow[q];
        uint32_t nz = (wv | (wv >> 1) | (wv >> 2) | (wv >> 3)) & 0x11111111u;  // nonzero nibbles
        while (nz) {
          const int sl = q * 8 + ((__ffs((int)nz) - 1) >> 2);
          nz &= nz - 1u;
          const int sq = sTX.slot_sq[ex][sl];
          CR[sq >> 5] |= 1u << (sq & 31);
        }
      }
    }
    // every table row read unconditionally at a valid index, then selected (conditional LDS reads
    // are branches whose reads are waited on one at a time)
    const bool sg_on = sd >= 0 && ((ex >> sd) & 1u), fi_on = t == gl_t && ((ex >> gl_d) & 1u);
    const bool st_on = t == st_t && ((ex >> st_d) & 1u);
    const uint32_t om = min(plan_omask(p), (uint32_t)PGTG_N_OBST_MASKS - 1u);
#pragma unroll
    for (int k = 0; k < 3; k++) {
      W3[k] = sT.wall[ex][k];
      const uint32_t sgk = sT.seg[sd >= 0 ? sd : 0][k], fik = sT.seg[gl_d & 3][k], stk = sT.seg[st_d & 3][k];
      const uint32_t obk = sT.obst[om][k];
      US[k] = sg_on && used ? sgk : 0u;
      SG[k] = sg_on && !used ? sgk : 0u;
      FI[k] = fi_on ? fik : 0u;
      ST[k] = st_on ? stk : 0u;
      OB[k] = ot ? (obk & ~W3[k]) : 0u;
    }
    STAMP(19);
    uint32_t gap = 0;  // bits of all-zero channels not yet appended
    for (int ci = ch_lo; ci < ch_hi; ci++) {
      const int code = lane_codes ? (int)sT.chan[ci] : c.channels[ci];
      if (ZS && code < 32 && ((c.zero_ch >> code) & 1u)) {
        gap += 81u;
        continue;
      }
      if (gap) {
        sink.skip(gap);
        gap = 0;
      }
      uint32_t out3[3];
#pragma unroll
      for (int k = 0; k < 3; k++) {
        uint32_t val;
        switch (code) {
          case PGTG_CH_WALL: val = W3[k]; break;
          case PGTG_CH_GOALS: val = SG[k] | FI[k]; break;
          case PGTG_CH_TL_GREEN: val = (color == 0 && ot == 4) ? OB[k] : 0u; break;
          case PGTG_CH_TL_YELLOW: val = (color == 1 && ot == 4) ? OB[k] : 0u; break;
          case PGTG_CH_TL_RED: val = (color == 2 && ot == 4) ? OB[k] : 0u; break;
          case PGTG_CH_START: val = ST[k]; break;
          case PGTG_CH_SUBGOAL: val = SG[k]; break;
          case PGTG_CH_USED_SUBGOAL: val = US[k]; break;
          case PGTG_CH_FINAL_GOAL: val = FI[k]; break;
          case PGTG_CH_ICE: val = ot == 1 ? OB[k] : 0u; break;
          case PGTG_CH_BROKEN: val = ot == 2 ? OB[k] : 0u; break;
          case PGTG_CH_SAND: val = ot == 3 ? OB[k] : 0u; break;
          case PGTG_CH_TRAFFIC: val = CR[k]; break;
          default: val = 0u; break;  // PGTG_CH_ZERO
        }
        out3[k] = val;
      }
      sink.put(out3[0], 32u);
      sink.put(out3[1], 32u);
      sink.put(out3[2] & 0x1ffffu, 17u);  // 81 = 32 + 32 + 17 bits
    }
    if (gap) sink.skip(gap);
  } else if (TR && c.sliding && !c.generic_channels && c.win <= 11) {
    // Sliding windows of <= 11 squares (size <= 5) without lane or spawner channels, traffic kernel:
    // the window touches <= 3 x 3 tiles.  Per channel and tile column, the 81-bit masks of its three
    // tiles (tile_chan, the fast path's table algebra), then the window rows of that column (one x, the
    // win y's each) cut from them: 9-bit tile columns placed at their offset, squares outside the map
    // walls (get_map_cutout's fill, environment.py:1384).  No per-square lookups: the caller workload's
    // 11 x 11 images were ~45 % of its k_env<true> waves.  The loops are uniform (a row outside this
    // lane's window is skipped by predication), so that the masks stay in 9 registers.
    const int win = c.win, x0 = oi.x0, y0 = oi.y0;
    const int tx0 = max(x0, 0) / kTile, ty0 = max(y0, 0) / kTile;
    const int txe = min(x0 + win - 1, c.W - 1) / kTile, tye = min(y0 + win - 1, c.H - 1) / kTile;
    const uint32_t wmask = (1u << win) - 1u;
    const int lo_out = min(win, max(0, -y0)), hi_in = min(win, max(0, c.H - y0));
    const uint32_t yfill = ((1u << lo_out) - 1u) | (wmask & ~((1u << hi_in) - 1u));  // y outside the map
    const int pre = min(win, max(0, -x0)), post = min(win, max(0, x0 + win - c.W));  // rows x < 0, x >= W
    uint32_t gap = 0;
    for (int ci = ch_lo; ci < ch_hi; ci++) {
      const int code = lane_codes ? (int)sT.chan[ci] : c.channels[ci];
      if (ZS && code < 32 && ((c.zero_ch >> code) & 1u)) {
        gap += (uint32_t)WW;
        continue;
      }
      if (gap) {
        sink.skip(gap);
        gap = 0;
      }
      const uint32_t fill = code == PGTG_CH_WALL ? wmask : 0u;
      for (int i = 0; i < pre; i++) sink.put(fill, (uint32_t)win);
      for (int a = 0; a < 3; a++) {
        if (tx0 + a > txe) continue;
        uint32_t M[3][3];
#pragma unroll
        for (int b = 0; b < 3; b++) {
          const bool ok = ty0 + b <= tye;
          const int t = ok ? (ty0 + b) * c.tw + tx0 + a : 0;
          tile_chan<TR, BIG>(c, v, pl[t], t, code, color, occ, M[b]);
          if (!ok) M[b][0] = M[b][1] = M[b][2] = 0u;
        }
        const int xa = (tx0 + a) * kTile;
        for (int lx = max(0, x0 - xa); lx < min(kTile, x0 + win - xa); lx++) {
          if (xa + lx >= c.W) break;
          const int off = lx * kTile, wd = off >> 5, sh = off & 31;
          uint64_t r64 = 0;
#pragma unroll
          for (int b = 0; b < 3; b++) {
            const uint32_t lo = wd == 0 ? M[b][0] : (wd == 1 ? M[b][1] : M[b][2]), hi = wd == 0 ? M[b][1] : M[b][2];
            const uint32_t c9 = ((lo >> sh) | (sh ? hi << (32 - sh) : 0u)) & 511u;
            const int s9 = (ty0 + b) * kTile - y0;
            r64 |= s9 >= 0 ? (uint64_t)c9 << s9 : (uint64_t)(c9 >> -s9);
          }
          sink.put(((uint32_t)r64 & wmask) | (fill & yfill), (uint32_t)win);
        }
      }
      for (int i = 0; i < post; i++) sink.put(fill, (uint32_t)win);
    }
    if (gap) sink.skip(gap);
  } else if (TR && WW <= 128) {
    // windows of <= 128 squares (sliding windows up to size 5) in the traffic kernel: each square is
    // looked up once per group of kGC channels, not once per channel -- the group's words of the whole
    // window are accumulated in registers, then appended channel by channel (the stream's order).
    // (Not compiled into the kernels without traffic: its 20 accumulators would raise their register
    // peak, set elsewhere in them.)
    constexpr int kGC = 5;
    const int win = c.win;
    for (int cg = ch_lo; cg < ch_hi; cg += kGC) {
      // each channel of the group as a branch-free test of the square's words (chan_bit's cases):
      // a flag mask, or the spawner / traffic bit, or a lane bit
      uint32_t fm[kGC];
      int lb[kGC];
      bool is_sp[kGC], is_tr[kGC];
      bool any_sp = false, any_ln = false, any_tr = false;
#pragma unroll
      for (int g = 0; g < kGC; g++) {
        const int code = cg + g < ch_hi ? (lane_codes ? (int)sT.chan[cg + g] : c.channels[cg + g]) : (int)PGTG_CH_ZERO;
        fm[g] = code == PGTG_CH_WALL ? SQ_WALL
              : code == PGTG_CH_GOALS ? (SQ_SUBGOAL | SQ_FINAL)
              : code == PGTG_CH_TL_GREEN ? (color == 0 ? SQ_TLIGHT : 0u)
              : code == PGTG_CH_TL_YELLOW ? (color == 1 ? SQ_TLIGHT : 0u)
              : code == PGTG_CH_TL_RED ? (color == 2 ? SQ_TLIGHT : 0u)
              : code == PGTG_CH_START ? SQ_START
              : code == PGTG_CH_SUBGOAL ? SQ_SUBGOAL
              : code == PGTG_CH_USED_SUBGOAL ? SQ_USED
              : code == PGTG_CH_FINAL_GOAL ? SQ_FINAL
              : code == PGTG_CH_ICE ? SQ_ICE
              : code == PGTG_CH_BROKEN ? SQ_BROKEN
              : code == PGTG_CH_SAND ? SQ_SAND : 0u;
        is_sp[g] = code == PGTG_CH_SPAWNER;
        is_tr[g] = code == PGTG_CH_TRAFFIC;
        lb[g] = (code >= PGTG_CH_LANE0 && code < PGTG_CH_LANE0 + 32) ? code - PGTG_CH_LANE0 : -1;
        any_sp = any_sp || is_sp[g];
        any_ln = any_ln || lb[g] >= 0;
        any_tr = any_tr || is_tr[g];
      }
      uint32_t acc[kGC][4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
#pragma unroll
        for (int g = 0; g < kGC; g++) acc[g][k] = 0u;
        const int nb = min(32, WW - 32 * k);
#pragma unroll 4
        for (int b = 0; b < nb; b++) {  // (unrolled: four squares' LDS lookups go out together)
          const int bb = 32 * k + b, i = bb / win, j = bb - i * win;
          const int x = oi.x0 + i, y = oi.y0 + j;
          // every lookup at clamped coordinates, then selected: no divergent branch per square
          const bool in = inside(c, x, y);
          const int xc = min(max(x, 0), c.W - 1), yc = min(max(y, 0), c.H - 1);
          uint32_t f = square_flags<BIG>(c, pl, v, xc, yc), lanes = 0;
          bool sp = false, car = false;
          if (LC && any_sp) sp = square_spawner(c, pl, xc, yc);
          if (LC && any_ln) lanes = square_lanes(c, pl, xc, yc);
          if ((TR && c.need_car) && occ && any_tr) car = occ_at(c, pl, occ, xc, yc) > 0;
          f = in ? f : (c.sliding ? SQ_WALL : 0u);  // get_map_cutout fill {"wall"} for sliding windows
          lanes = in ? lanes : 0u;
          sp = in && sp;
          car = in && car;
#pragma unroll
          for (int g = 0; g < kGC; g++) {
            const uint32_t bit = ((f & fm[g]) != 0u ? 1u : 0u) | (is_sp[g] && sp ? 1u : 0u) | (is_tr[g] && car ? 1u : 0u) |
                                 (lb[g] >= 0 ? (lanes >> (lb[g] & 31)) & 1u : 0u);
            acc[g][k] |= bit << b;
          }
        }
      }
#pragma unroll
      for (int g = 0; g < kGC; g++) {
        if (cg + g < ch_hi) {
#pragma unroll
          for (int k = 0; k < 4; k++)
            if (32 * k < WW) sink.put(acc[g][k], (uint32_t)min(32, WW - 32 * k));
        }
      }
    }
  } else {
    const int win = c.win;
    for (int ci = ch_lo; ci < ch_hi; ci++) {
      const int code = lane_codes ? (int)sT.chan[ci] : c.channels[ci];
      for (int w0 = 0; w0 < WW; w0 += 32) {
        uint32_t acc = 0;
        if (code == PGTG_CH_TRAFFIC) {
          if ((TR && c.need_car) && occ) {
            int nb = min(32, WW - w0);
            for (int b = 0; b < nb; b++) {
              int bb = w0 + b, ii = bb / win, j = bb - ii * win;
              int x = oi.x0 + ii, y = oi.y0 + j;
              if (inside(c, x, y) && occ_at(c, pl, occ, x, y) > 0) acc |= 1u << b;
            }
          }
        } else if (code != PGTG_CH_ZERO) {
          int nb = min(32, WW - w0);
          for (int b = 0; b < nb; b++) {
            int bb = w0 + b, i = bb / win, j = bb - i * win;
            int x = oi.x0 + i, y = oi.y0 + j;
            uint32_t f, lanes = 0;
            bool sp = false;
            if (inside(c, x, y)) {
              f = square_flags<BIG>(c, pl, v, x, y);
              if (LC && code == PGTG_CH_SPAWNER) sp = square_spawner(c, pl, x, y);
              if (LC && code >= PGTG_CH_LANE0) lanes = square_lanes(c, pl, x, y);
            } else {
              f = c.sliding ? SQ_WALL : 0u;  // get_map_cutout fill {"wall"} for sliding windows
            }
            acc |= chan_bit(code, f, lanes, sp, color) << b;
          }
        }
        sink.put(acc, (uint32_t)min(32, WW - w0));
      }
    }
  }
  STAMP(20);
  sink.finish();
  oi.nsd = -1;
  if (c.next_subgoal && head) {
    int t = ty * c.tw + tx;
    int sd = plan_sgdir(pl[t]);
    int gl_t = (int)((v.sg >> 16) & 0xffu);
    int nsd = sd >= 0 ? sd : (t == gl_t ? (int)(v.sg >> 24) : -1);
    if (nsd == -1 || c.sliding) {
      int bx = 0, by = 0;
      if (nearest_goal_square<BIG>(c, pl, v, pix, piy, bx, by))
        nsd = S.nsd_tab[(bx - pix + c.nsd_off) * c.nsd_pitch + (by - piy + c.nsd_off)];
    }
    oi.nsd = nsd;
  }
  STAMP(21);
}

// ------------------------------------------------------------------------------------------------
// step (pgtg/environment.py:1092-1281) for one lane; returns 0 or -code
// ------------------------------------------------------------------------------------------------
// ACTIONS_TO_ACCELERATION (pgtg/constants.py:6-16): action a -> (a/3 - 1, a%3 - 1)
constexpr int kPathChunk = 4;  // agent path squares looked up together (env_step)
__device__ __forceinline__ int acc_x(int a) { return a / 3 - 1; }
__device__ __forceinline__ int acc_y(int a) { return a % 3 - 1; }

struct BrakeQuery {
  uint32_t cand;  // rules whose tile/speed conditions hold
  int tile;       // agent tile (-1: nothing to count)
  int s2;         // squared speed after the acceleration
  int n_in;       // cars in the tile after the move
};
// Traffic tick: every car of the tick-start list, in list order (pgtg/environment.py:1121-1127,
// _get_next_car_position_and_route :881-968, _should_car_move :678-691, traffic lights :664-676,
// _spawn_new_car :970-1002).  Survivors keep their slots, respawned cars are appended behind the
// tail in creation order (slot order = list order); occupancy counters follow every move so later
// cars see earlier ones.

// The per-car work is organised for a divergent wave: every map lookup the car may need (its slot,
// the four neighbours, the first admissible one, light and occupancy there) is computed branch-free
// first; the random draws then go through five draw slots shared by all outcomes (a lane's draws
// keep numpy's order: delay?, delay length | speed, route | spawner | light, go | profile, route).
// Exact number of cars on lane slot s while the car in slot r leaves it: slots [0, w) hold the cars
// already moved this tick (w = r, or the packed count when the tick packs), (r, tail0) those still
// to move, [tail0, t_out) this tick's respawns.  Rare: only once a 4-bit occupancy counter saturated.
// A fresh env (fw0: its staging block) still holds the cars not yet moved, (r, tail0), there.
__device__ __noinline__ int recount_slot(const DevCfg& c, const Plan& pl, const CarSlots& cs, const gu32* fw0, int tail0,
                                         int r, int w, int t_out, int s) {
  int n = 0;
  for (int k = 0; k < t_out; k++) {
    if (k >= w && k <= r) continue;
    const uint32_t w0 = (fw0 && k > r && k < tail0) ? fw0[k] : cs.w0[cs.at(k)];
    if (w0 & kCarEmpty) continue;
    n += lane_slot(c, pl, (int)(w0 & 255u), (int)((w0 >> 8) & 255u)) == s ? 1 : 0;
  }
  return n;
}

// Empty slots an env may start a tick with before its wave packs the slots.  A wave iterates up to
// its longest list's tail, so empty slots cost every lane an iteration; a packing tick costs the
// wave an id read and write per car and scattered survivor writes for envs with empty slots.  A/B
// on configs[2] (k_env<true> + k_traffic per launch): slack 16 1464 us, 8 1456, 4 1402, 0 1450.
#ifndef PGTG_SLACK
#define PGTG_SLACK 4
#endif
constexpr int kCompactSlack = PGTG_SLACK;

// The car pass.  Slots are visited in order and all lanes of a wave are at the same slot, so the
// loads and the in-place stores of the survivors are coalesced rows (ids are neither read nor
// rewritten).  A despawned car leaves an empty slot; its replacement is appended behind the tail.
// A tick in which some env of the wave starts with more than kCompactSlack empty slots packs instead:
// survivors are written to the next packed slot w <= r (with their ids), the respawns moved down
// behind them at the end.
__device__ __forceinline__ int move_cars(const DevCfg& c, const DevState& S, uint64_t i, const EnvView& v,
                                         const Plan& pl, uint8_t* occ, bool& sat, const uint16_t* sp, TrafState& ts,
                                         Pcg& cr, int color, BrakeQuery& bq, uint8_t* hist) {
  const CarSlots cs(S, i);
  const int tw = c.tw, th = c.th;
  const uint32_t nsp = ts.n_spawners;
  const int tail0 = (int)ts.tail;
  // a fresh env (initial traffic from k_traffic) reads its cars from its staging block, patience 0;
  // every env writes the slot rows
  const bool fresh = ts.fresh != 0;
  gu32* const fb = fresh_block(S, i);
  const gu32* const rb = fresh ? fb : cs.w0;
  const uint64_t rstep = fresh ? 1ull : S.n;
  // (wave-uniform: packing is right for any list, and a uniform flag keeps the loop free of
  // exec-mask juggling around the packing writes)
  const bool pack = __any(tail0 > (int)ts.n_cars + kCompactSlack);
  const ProfileCdf pcdf = pin_profile_cdf(c);
  Pcg& ca = cr;
  int t_out = tail0, w = 0;
  const uint64_t nst = S.n;
  // software pipeline: the next slot's words are requested before the current car is processed, so
  // their HBM latency overlaps this car's work (slot indices advance by the env stride)
  uint64_t ar = cs.at(0), an = cs.at(tail0), ap = cs.at(0), rr = 0;
  uint32_t rn = 0;  // the prefetched slot (a fresh env's car ids are its slot indices)
  uint32_t na = rb[rr], npat = cs.w1[ar], nid = 0u;
  npat = fresh ? 0u : npat;
  if (pack) nid = cs.id[ar];
  nid = fresh ? rn : nid;
  for (int r = 0; r < tail0; r++) {
    const uint64_t aw = ar;
    const uint32_t a = na, id = nid;
    uint32_t pat = npat;
    if (r + 1 < tail0) {
      ar += nst;
      rr += rstep;
      rn++;
    }
    na = rb[rr];
    npat = cs.w1[ar];
    npat = fresh ? 0u : npat;
    if (pack) nid = cs.id[ar];
    nid = fresh ? rn : nid;
    if (!(a & kCarEmpty)) {
      const int x = (int)(a & 255u), y = (int)((a >> 8) & 255u), prof = (int)((a >> 21) & 7u);
      int route = (int)((a >> 16) & 31u), delay = (int)((a >> 24) & 3u);
      // ---- map lookups (no draws).  Every LDS read is unconditional at a valid index (a conditional
      // read is a branch the compiler cannot hoist the read out of, and each one waited alone); the
      // reads of one level go out together.
      const int tx = x / kTile, ty = y / kTile, lx = x - tx * kTile, ly = y - ty * kTile;
      const int t0 = ty * tw + tx, sq = lx * 9 + ly;
      // neighbours up, down, left, right (_get_next_car_position_and_route's order)
      const bool ok0 = !(ly == 0 && ty == 0), ok1 = !(ly == 8 && ty == th - 1);
      const bool ok2 = !(lx == 0 && tx == 0), ok3 = !(lx == 8 && tx == tw - 1);
      const int nt0 = ly == 0 ? t0 - tw : t0, nt1 = ly == 8 ? t0 + tw : t0;
      const int nt2 = lx == 0 ? t0 - 1 : t0, nt3 = lx == 8 ? t0 + 1 : t0;
      const int nq0 = ly == 0 ? sq + 8 : sq - 1, nq1 = ly == 8 ? sq - 8 : sq + 1;
      const int nq2 = lx == 0 ? sq + 72 : sq - 9, nq3 = lx == 8 ? sq - 72 : sq + 9;
      const uint32_t p0 = pl[t0];
      const uint32_t pn0 = pl[ok0 ? nt0 : t0], pn1 = pl[ok1 ? nt1 : t0];
      const uint32_t pn2 = pl[ok2 ? nt2 : t0], pn3 = pl[ok3 ? nt3 : t0];
      const uint32_t rtl = *reinterpret_cast<const uint32_t*>(sTX.route_type_lane[route]);
      // this car's behaviour thresholds (environment.py:64-109), read up front
      const uint64_t th_delay = sTX.beh_t[BEH_DELAY][prof], th_speed = sTX.beh_t[BEH_SPEED][prof];
      const uint64_t th_yellow = sTX.beh_t[BEH_YELLOW][prof], th_red = sTX.beh_t[BEH_RED][prof];
      const uint64_t th_go = sTX.beh_t[BEH_GO][prof];
      const int b_mf = sTX.beh_mf[prof], b_pt = sTX.beh_pt[prof];
      const uint32_t e0 = ok0 ? plan_exits(pn0) : 0u, e1 = ok1 ? plan_exits(pn1) : 0u;
      const uint32_t e2 = ok2 ? plan_exits(pn2) : 0u, e3 = ok3 ? plan_exits(pn3) : 0u;
      const int s_old = t0 * 32 + sTX.li[plan_exits(p0)][sq];
      const uint32_t l0 = sTX.lanes[e0][nq0], l1 = sTX.lanes[e1][nq1];  // row 0 (no exits) is empty
      const uint32_t l2 = sTX.lanes[e2][nq2], l3 = sTX.lanes[e3][nq3];
      int dec = -1;
      bool dec_all = false;
#pragma unroll
      for (int t = 3; t >= 0; t--) {  // the first direction with a lane "all <t>" or the route's lane
        const uint32_t ln = sel4(t, l0, l1, l2, l3);
        const bool all = (ln >> (28 + t)) & 1u;
        const uint32_t lane = (rtl >> (8 * t)) & 255u;
        const bool rt = lane != 255u && ((ln >> lane) & 1u);
        if (all || rt) {
          dec = t;
          dec_all = all;
        }
      }
      const int dk = dec < 0 ? 0 : dec;
      const int tg_t = sel4(dk, nt0, nt1, nt2, nt3), tg_q = sel4(dk, nq0, nq1, nq2, nq3);
      const uint32_t tg_ln = sel4(dk, l0, l1, l2, l3);
      const uint32_t p_tg = dec < 0 ? p0 : sel4(dk, pn0, pn1, pn2, pn3);  // pl[tg_t] (read above)
      const uint32_t ex_tg = plan_exits(p_tg);
      const uint32_t wall_tg = bit81(sT.wall[ex_tg], dec < 0 ? sq : tg_q);
      const uint32_t obst_tg = bit81(sT.obst[min(plan_omask(p_tg), (uint32_t)PGTG_N_OBST_MASKS - 1u)], dec < 0 ? sq : tg_q);
      const bool tl = plan_otype(p_tg) == 4u && !wall_tg && obst_tg;
      const int li_tg = sTX.li[ex_tg][tg_q];
      const int s_tg = dec < 0 ? s_old : tg_t * 32 + li_tg;
      const int occ_raw = occ_get(occ, s_tg);
      const int occ_tg = dec < 0 ? 0 : occ_raw;
      // ---- draws (_should_car_move, route choice / light / following, _spawn_new_car)
      const bool act = delay == 0;
      bool delayed = false, move = false;
      if (act) {
        delayed = pcg_draw(ca, false, 0u) < th_delay;
        const uint64_t r2 = pcg_draw(ca, delayed, 3u);
        if (delayed) delay = 1 + (int)r2;  // integers(1, 4)
        else move = r2 < th_speed;
      } else {
        delay -= 1;
      }
      const int kind = !move ? 0 : (dec < 0 ? 3 : (dec_all ? 1 : 2));  // stay, all-lane, route lane, respawn
      const uint32_t nr_all = __popc(tg_ln & 0x0fffffffu);
      if (kind == 1 && nr_all == 0) return PGTG_E_MAP;  // numpy choice([]) raises
      const bool lit = kind == 2 && tl && color != 0;
      const bool s3_int = kind != 2;
      const uint32_t s3_n = kind == 1 ? nr_all : nsp;
      uint64_t r3 = 0;
      if ((kind == 1 || kind == 3 || lit) && !(s3_int && s3_n <= 1u)) r3 = pcg_draw(ca, s3_int, s3_n);
      const bool stop = lit && (color == 1 ? r3 < th_yellow : !(r3 < th_red));
      const bool go_try = kind == 2 && !stop && occ_tg > 0 && (b_mf == 0 || (int)pat > b_pt);
      uint64_t r4 = 0;
      if (go_try || kind == 3) r4 = pcg_draw(ca, false, 0u);
      const bool leaves = kind == 3 || kind == 1 || (kind == 2 && !stop && (occ_tg == 0 || (go_try && r4 < th_go)));
      if (leaves) {  // the car's square loses it
        if (sat && occ_get(occ, s_old) >= kOccMax) {
          // exact recount from HBM (this car's slot still holds its old square)
          occ_put(occ, s_old, min(recount_slot(c, pl, cs, fresh ? fb : nullptr, tail0, r, pack ? w : r, t_out, s_old), kOccMax));
        } else {
          occ_put(occ, s_old, occ_get(occ, s_old) - 1);
        }
      }
      if (kind == 3) {
        // _spawn_new_car: choice(car_spawners) -> sorted routes -> profile -> route
        int sx = 0, sy = 0;
        if (nsp > 0) {
          // (two loads, not one through a selected pointer: that would be a flat load, whose wait
          // covers the LDS counter and the slot prefetch)
          uint32_t code = sp[r3 < (uint64_t)kSpCache ? r3 : 0];
          if (r3 >= (uint64_t)kSpCache) code = ((const __attribute__((address_space(1))) uint16_t*)S.spawners)[i * (uint64_t)S.sp_pitch + r3];
          sx = (int)(code & 255u);
          sy = (int)(code >> 8);
        }
        const uint32_t rl = square_lanes(c, pl, sx, sy) & 0x0fffffffu;
        const uint32_t nr = __popc(rl);
        const int nprof = profile_of(pcdf, r4);
        if (nr == 0) return PGTG_E_MAP;
        const uint32_t r5 = nr > 1u ? (uint32_t)pcg_draw(ca, true, nr) : 0u;
        const int nroute = sTX.lane_route[kth_bit(rl, (int)r5)];
        if (!pack) cs.w0[aw] = kCarEmpty;
        cs.w0[an] = (uint32_t)sx | (uint32_t)sy << 8 | (uint32_t)nroute << 16 | (uint32_t)nprof << 21;
        cs.w1[an] = 0u;
        cs.id[an] = ts.next_id++;
        an += nst;
        t_out++;
        const int s_new = lane_slot(c, pl, sx, sy);
        if (s_new < 0) return PGTG_E_UNSUPPORTED;
        occ_inc(occ, s_new, sat);
        if (bq.tile >= 0 && (s_new >> 5) == bq.tile) {
          bq.n_in++;
          hist[nroute]++;
        }
      } else {
        if (kind == 1) route = sTX.lane_route[kth_bit(tg_ln & 0x0fffffffu, (int)r3)];
        int nx = x, ny = y, s_cur = s_old;
        if (leaves) {
          nx = x + (dk == 2 ? -1 : (dk == 3 ? 1 : 0));
          ny = y + (dk == 0 ? -1 : (dk == 1 ? 1 : 0));
          s_cur = s_tg;
          occ_inc(occ, s_cur, sat);
          pat = 0;
        } else {
          pat += 1;
        }
        if (bq.tile >= 0 && (s_cur >> 5) == bq.tile) {
          bq.n_in++;
          hist[route]++;
        }
        const uint64_t ao = pack ? ap : aw;
        cs.w0[ao] = (uint32_t)nx | (uint32_t)ny << 8 | (uint32_t)route << 16 | (uint32_t)prof << 21 | (uint32_t)delay << 24;
        cs.w1[ao] = pat;
        if (pack) {
          cs.id[ao] = id;
          ap += nst;
          w++;
        } else if (fresh) {
          cs.id[ao] = id;  // (a slot row's ids are written only by the lanes of fresh envs)
        }
      }
    }
  }
  if (pack) {  // this tick's respawns, [tail0, t_out), moved down behind the packed survivors
    uint64_t as = cs.at(tail0);
    for (int k = tail0; k < t_out; k++) {
      const uint32_t x0 = cs.w0[as], x1 = cs.w1[as], x2 = cs.id[as];
      cs.w0[ap] = x0;
      cs.w1[ap] = x1;
      cs.id[ap] = x2;
      as += nst;
      ap += nst;
    }
    t_out = w + (t_out - tail0);
  }
  ts.tail = (uint32_t)t_out;
  ts.fresh = 0u;  // every car is in the slot rows now
  return 0;
}

// TrafficRuleEngine.apply_braking (pgtg/environment.py:226-294) on the agent's (clamped) tile after
// the cars moved.  Split in two: the rules that can fire for the tile and the new speed are found
// before the car pass, which then counts the cars ending in that tile into `hist` (per-lane LDS
// route histogram, 20 B), so the braking test needs no extra pass over the car list.
__device__ __forceinline__ BrakeQuery braking_query(const DevCfg& c, const EnvView& v, const Plan& pl, int vx, int vy) {
  BrakeQuery q{0u, -1, vx * vx + vy * vy, 0};
  const int tx = min(max((int)floorf((float)v.px / kTile), 0), c.tw - 1);
  const int ty = min(max((int)floorf((float)v.py / kTile), 0), c.th - 1);
  const uint32_t ex = plan_exits(pl[ty * c.tw + tx]);
  for (int r = 0; r < c.n_rules; r++)
    if (c.rules[r].tile_exits == (int)ex && q.s2 >= c.rules[r].speed_sq_min && q.s2 <= c.rules[r].speed_sq_max)
      q.cand |= 1u << r;
  if (q.cand) q.tile = ty * c.tw + tx;
  return q;
}
// returns the mask of triggered rules (TrafficRuleEngine.evaluate_all_rules, rule_triggers)
template <bool BIG>
__device__ __forceinline__ uint32_t braking_decide(const DevCfg& c, const DevState& S, const EnvView& v,
                                                   const Plan& pl, const BrakeQuery& q, const uint8_t* hist) {
  if (!q.cand) return 0u;
  // agent direction from the subgoal compass (environment.py:185-206, 1037-1090)
  int dir;
  int bx = 0, by = 0;
  int cp = -1;
  if (nearest_goal_square<BIG>(c, pl, v, v.px, v.py, bx, by))
    cp = S.cmp_tab[(bx - v.px + c.cmp_off) * c.cmp_pitch + (by - v.py + c.cmp_off)];
  if (cp >= 0) dir = cp >> 1;  // N,NE -> south_to_north; E,SE -> west_to_east; S,SW; W,NW
  else dir = q.s2 == 0 ? 4 : 5;  // "stationary" (speed < 0.1) / "near_goal"
  uint32_t trig = 0u;
  for (int r = 0; r < c.n_rules; r++) {
    if (!((q.cand >> r) & 1u)) continue;
    if (q.n_in < c.rules[r].min_traffic) continue;
    int match = 0;
    for (int k = 0; k < 20; k++) match += hist[k] * (int)sTX.rule_w[r][dir][k];
    if (match >= c.rules[r].min_matching_traffic) trig |= 1u << r;
  }
  return trig;
}

struct StepResult {
  double reward, cost;
  uint32_t triggered;  // traffic rules that triggered braking (bit r = rule r)
  bool plan_dirty;     // BIG maps: a subgoal was marked used in the LDS plan (write the row back)
};

template <bool TR, bool BIG>
__device__ __forceinline__ int env_step(const DevCfg& c, const DevState& S, uint64_t i, EnvView& v, const Plan& pl,
                                        int action, StepResult& res, uint8_t* occ, bool& occ_sat, const uint16_t* sp,
                                        TrafState& ts, uint8_t* hist) {
  res.reward = 0.0;
  res.cost = 0.0;
  res.plan_dirty = false;
  if (v.flags & (kFlagTerminated | kFlagTruncated)) return PGTG_E_DONE;
  if ((unsigned)action > 8u) return PGTG_E_INVALID;
  v.phase = (v.phase + 1u) % (uint32_t)c.phase_total;
  const int ax = acc_x(action), ay = acc_y(action);
  BrakeQuery bq{0u, -1, 0, 0};
  if (TR && c.n_rules > 0) {
    bq = braking_query(c, v, pl, v.vx + ax, v.vy + ay);
    if (bq.cand)
      for (int k = 0; k < 20; k++) hist[k] = 0;
  }
  // cars move first (environment.py:1120-1127), with this tick's light phase
  if ((TR && c.need_car) && ts.n_cars > 0) {
    Pcg cr = stream_load(S.car, i);
    STAMP(16);
    int e = move_cars(c, S, i, v, pl, occ, occ_sat, sp, ts, cr, phase_color(c, v.phase), bq, hist);
    STAMP(17);
    stream_store_state(S.car, i, cr);
    if (e) return e;
  }
  double reward = 0.0, perf = 0.0, cost = 0.0;
  int cx = v.px, cy = v.py;
  v.vx += ax;
  v.vy += ay;
  v.flags &= ~kFlagBraking;
  res.triggered = (TR && c.n_rules > 0) ? braking_decide<BIG>(c, S, v, pl, bq, hist) : 0u;
  if (res.triggered) {  // environment.py:1145
    v.vx = v.vy = 0;
    v.flags |= kFlagBraking;
  }
  STAMP(18);
  if (abs(v.vx) > 30000 || abs(v.vy) > 30000) return PGTG_E_UNSUPPORTED;
  Pcg ice, broken, sand;
  if (c.need_ice) ice = stream_load(S.ice, i);
  if (c.need_broken) broken = stream_load(S.broken, i);
  if (c.need_sand) sand = stream_load(S.sand, i);
  bool used_ice = false, used_broken = false, used_sand = false;
  // _decompose_velocity (environment.py:693-748) evaluated lazily: part k is cum(k+1) - cum(k)
  const int dx = v.vx, dy = v.vy;
  const int adx = abs(dx), ady = abs(dy);
  const int n = max(adx, ady);
  const bool xmajor = adx >= ady;
  const int smaj = xmajor ? (dx > 0 ? 1 : -1) : (dy > 0 ? 1 : -1);
  double m = 0.0;
  if (dx != 0 && dy != 0) m = xmajor ? (double)dy / (double)adx : (double)dx / (double)ady;
  int prev_minor = 0;
  const int gl_t = (int)((v.sg >> 16) & 0xffu), gl_d = (int)(v.sg >> 24);
  const int color = phase_color(c, v.phase);
  // the subgoal reward of this episode's path (one read for every subgoal the step may cross)
  const double ind_pl = BIG ? c.ind_reward[v.path_len] : sT.ind[v.path_len];
  // Without obstacle effects or cars a step's path depends on the velocity alone, so the squares
  // of kPathChunk parts are looked up together (one LDS latency per chunk instead of per part) and
  // then walked in order.  A subgoal tile marked used earlier in the same step is tested against
  // the updated mask (the lookups saw the step's initial one).
  const bool chunked = !c.need_ice && !c.need_broken && !c.need_sand && !(TR && c.need_car);
  for (int k0 = 0; chunked && k0 <= n; k0 += kPathChunk) {
    int X[kPathChunk + 1], Y[kPathChunk + 1];
    X[0] = cx;
    Y[0] = cy;
#pragma unroll
    for (int j = 0; j < kPathChunk; j++) {  // part k0 + j: position k0 + j -> k0 + j + 1
      int pxp = 0, pyp = 0;
      if (k0 + j < n) {
        int minor = 0;
        if (dx != 0 && dy != 0) {
          double t = (double)(k0 + j + 1) * m;
          t = t + 0.5;
          minor = (int)floor(t);
        }
        if (xmajor) {
          pxp = smaj;
          pyp = (dy == 0) ? 0 : minor - prev_minor;
        } else {
          pyp = smaj;
          pxp = (dx == 0) ? 0 : minor - prev_minor;
        }
        prev_minor = minor;
      }
      X[j + 1] = X[j] + pxp;
      Y[j + 1] = Y[j] + pyp;
    }
    uint32_t F[kPathChunk + 1];
#pragma unroll
    for (int j = 0; j <= kPathChunk; j++)
      F[j] = square_flags<BIG>(c, pl, v, min(max(X[j], 0), c.W - 1), min(max(Y[j], 0), c.H - 1));
    bool go = true;
#pragma unroll
    for (int j = 0; j < kPathChunk; j++) {
      if (go) {
        const int k = k0 + j, x = X[j], y = Y[j];
        const uint32_t f = F[j];
        cx = x;
        cy = y;
        if (!inside(c, x, y) || (f & SQ_WALL)) {  // crash: outside, wall
          if (c.separate_cost) cost += c.crash_penalty; else reward -= c.crash_penalty;
          v.flags |= kFlagTerminated;
          go = false;
        } else if (f & SQ_FINAL) {
          double add = ind_pl + c.final_goal_bonus;
          if (c.separate_cost) perf += add; else reward += add;
          v.flags |= kFlagTerminated;
          go = false;
        } else {
          const int t = (y / kTile) * c.tw + x / kTile;
          if ((f & SQ_SUBGOAL) && !used_bit<BIG>(v, pl[t], t)) {
            if (c.separate_cost) perf += ind_pl; else reward += ind_pl;
            if (BIG) {
              pl.p[t] |= (uint16_t)kPlanUsed;
              res.plan_dirty = true;
            } else {
              v.used |= 1ull << t;
            }
          }
          if (k == n) {
            go = false;
          } else if (color == 2 && inside(c, X[j + 1], Y[j + 1]) && (F[j + 1] & SQ_TLIGHT)) {
            if (c.separate_cost) cost += c.tl_penalty; else reward -= c.tl_penalty;
          }
        }
      }
    }
    if (!go) break;
    cx = X[kPathChunk];
    cy = Y[kPathChunk];
  }
  for (int k = 0; !chunked && k <= n; k++) {
    // part k (the move to the next square) first: it does not depend on this square, so both
    // squares' lookups go out together (unconditional reads at clamped coordinates)
    int pxp = 0, pyp = 0;
    if (k < n) {
      const int ii = k + 1;
      int minor = 0;
      if (dx != 0 && dy != 0) {
        double t = (double)ii * m;
        t = t + 0.5;
        minor = (int)floor(t);
      }
      if (xmajor) {
        pxp = smaj;
        pyp = (dy == 0) ? 0 : minor - prev_minor;
      } else {
        pyp = smaj;
        pxp = (dx == 0) ? 0 : minor - prev_minor;
      }
      prev_minor = minor;
    }
    const int nx = cx + pxp, ny = cy + pyp;
    const int ccx = min(max(cx, 0), c.W - 1), ccy = min(max(cy, 0), c.H - 1);
    const int cnx = min(max(nx, 0), c.W - 1), cny = min(max(ny, 0), c.H - 1);
    const uint32_t f_here = square_flags<BIG>(c, pl, v, ccx, ccy);
    const uint32_t f_next = square_flags<BIG>(c, pl, v, cnx, cny);
    int occ_here = 0;
    if (TR && c.need_car) occ_here = occ_at(c, pl, occ, ccx, ccy);
    // crash: outside, wall (cars: traffic pass)
    if (!inside(c, cx, cy)) {
      if (c.separate_cost) cost += c.crash_penalty; else reward -= c.crash_penalty;
      v.flags |= kFlagTerminated;
      break;
    }
    const uint32_t f = f_here;
    if ((f & SQ_WALL) || ((TR && c.need_car) && !c.ignore_collisions && occ_here > 0)) {
      if (c.separate_cost) cost += c.crash_penalty; else reward -= c.crash_penalty;
      v.flags |= kFlagTerminated;
      break;
    }
    if (f & SQ_FINAL) {
      double add = ind_pl + c.final_goal_bonus;
      if (c.separate_cost) perf += add; else reward += add;
      v.flags |= kFlagTerminated;
      break;
    }
    if (f & SQ_SUBGOAL) {
      if (c.separate_cost) perf += ind_pl; else reward += ind_pl;
      // set_subgoals_to_used: the flood fill covers exactly this tile's subgoal segment
      const int t = (cy / kTile) * c.tw + cx / kTile;
      if (BIG) {
        pl.p[t] |= (uint16_t)kPlanUsed;
        res.plan_dirty = true;
      } else {
        v.used |= 1ull << t;
      }
    }
    if (k == n) break;
    // red light at the next square (phase after this tick's increment)
    if (color == 2 && inside(c, nx, ny) && (f_next & SQ_TLIGHT)) {
      if (c.separate_cost) cost += c.tl_penalty; else reward -= c.tl_penalty;
    }
    if (f & SQ_ICE) {
      used_ice = true;
      if (pcg_double(ice) < c.ice_p) {
        int a = (int)pcg_int(ice, 9);
        pxp = acc_x(a);
        pyp = acc_y(a);
      }
    }
    if (f & SQ_BROKEN) {
      used_broken = true;
      if (pcg_double(broken) < c.broken_p) v.flags |= kFlagFlatTire;
    }
    if (f & SQ_SAND) {
      used_sand = true;
      if (pcg_double(sand) < c.sand_p) {
        cx += pxp;
        cy += pyp;
        v.vx = v.vy = 0;
        break;
      }
    }
    cx += pxp;
    cy += pyp;
  }
  (void)gl_t;
  (void)gl_d;
  if (used_ice) stream_store_state(S.ice, i, ice);
  if (used_broken) stream_store_state(S.broken, i, broken);
  if (used_sand) stream_store_state(S.sand, i, sand);
  if (v.flags & kFlagFlatTire) v.vx = v.vy = 0;
  const bool accel = !(ax == 0 && ay == 0);
  if (S.visited) {
    uint32_t* vis = S.visited + i * (uint64_t)c.vis_words;
    int b = (cx + 2) * c.vis_pitch + (cy + 2);
    if (c.visited_penalty != 0.0 && accel && ((vis[b >> 5] >> (b & 31)) & 1u)) {
      if (c.separate_cost) cost += c.visited_penalty; else reward -= c.visited_penalty;
    }
    vis[b >> 5] |= 1u << (b & 31);
  }
  const int ox = v.px, oy = v.py;
  v.px = cx;
  v.py = cy;
  if (c.still_penalty != 0.0 && !accel && ox == cx && oy == cy) {
    if (c.separate_cost) cost += c.still_penalty; else reward -= c.still_penalty;
  }
  v.elapsed += 1u;
  if (c.max_steps > 0 && (int)v.elapsed >= c.max_steps) v.flags |= kFlagTruncated;
  res.reward = c.separate_cost ? perf : reward;
  res.cost = cost;
  return 0;
}

// ------------------------------------------------------------------------------------------------
// cooperative observation writer: the output slice [cnt][obs_bytes] of `cnt` consecutive envs is
// the LDS segment image expanded bit -> byte, written with 16-byte stores.  Bytes outside the slice
// are never touched (neighbouring slices belong to other workgroups).  With sel != null a chunk is
// written only if one of its envs has sel == 1: final observations of the other envs are
// unspecified (gymnasium's info["final_observation"] is valid where "_final_observation" is set).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t expand4(uint32_t x) { return ((x & 15u) * 0x00204081u) & 0x01010101u; }
// floor(x / d) for x < 2^24 via an f32 reciprocal and one correction step each way
__device__ __forceinline__ uint32_t udiv_f(uint32_t x, uint32_t d, float inv) {
  uint32_t q = (uint32_t)((float)x * inv);
  if (q * d > x) q--;
  if ((q + 1) * d <= x) q++;
  return q;
}

// Write `cnt` envs' observations (OB bytes each) from the dense image to dst as 16-byte stores
// aligned to 16 B (the first and last chunks may be partial).  `nthr` threads share the chunks,
// this one with rank `rank` (default: the whole workgroup).  With `sel`, only 128-byte lines
// holding an env with sel == 1 are written (whole lines: the other envs' bytes in them get their
// own image, which the API leaves unspecified, and the memory system sees no partial lines); `lm`,
// when given, is the line mask of the selection (mark_lines) and replaces the per-env test.
// Line mask for the selection: the 128-byte lines (counted from the one holding dst) that env e's
// OB output bytes touch, or-ed into lm (cleared beforehand).
__device__ __forceinline__ void mark_lines(uint32_t* lm, const uint8_t* dst, uint32_t e, uint32_t OB) {
  const uintptr_t a0 = (uintptr_t)dst, base = a0 >> 7;
  uint32_t l = (uint32_t)(((a0 + (uintptr_t)e * OB) >> 7) - base);
  const uint32_t l1 = (uint32_t)(((a0 + (uintptr_t)(e + 1) * OB - 1) >> 7) - base);
  while (l <= l1) {
    const uint32_t hi = min(l1, l | 31u), n = hi - l + 1u;
    __hip_atomic_fetch_or(lm + (l >> 5), (n == 32u ? ~0u : ((1u << n) - 1u)) << (l & 31u), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
    l = hi + 1u;
  }
}

__device__ __forceinline__ void write_obs(uint8_t* __restrict__ dst, uint32_t cnt, uint32_t OB, const uint32_t* st,
                                          const uint8_t* sel, int rank = -1, int nthr = kBlock,
                                          const uint32_t* lm = nullptr) {
  if (rank < 0) rank = (int)threadIdx.x;
  const uint32_t total = cnt * OB;
  const uintptr_t a0 = (uintptr_t)dst;
  const uintptr_t c0 = a0 & ~(uintptr_t)15;
  const uint32_t nchunks = (uint32_t)((a0 + total - c0 + 15) >> 4);
  const float invOB = 1.0f / (float)OB;
  for (uint32_t ch = (uint32_t)rank; ch < nchunks; ch += (uint32_t)nthr) {
    const int r = (int)((intptr_t)(c0 + ((uintptr_t)ch << 4)) - (intptr_t)a0);  // > -16
    if (lm) {
      const uint32_t li = (uint32_t)(((c0 + ((uintptr_t)ch << 4)) >> 7) - (a0 >> 7));
      if (!((lm[li >> 5] >> (li & 31u)) & 1u)) continue;
    } else if (sel) {
      const intptr_t l0 = (intptr_t)((c0 + ((uintptr_t)ch << 4)) & ~(uintptr_t)127) - (intptr_t)a0;
      const uint32_t llo = l0 < 0 ? 0u : (uint32_t)l0;
      const uint32_t lhi = min((uint32_t)(l0 + 127), total - 1u);
      const uint32_t e0 = udiv_f(llo, OB, invOB), e1 = udiv_f(lhi, OB, invOB);
      bool any = false;
      for (uint32_t e = e0; e <= e1; e++) any = any || sel[e] == 1;
      if (!any) continue;
    }
    uint8_t* cp = dst + r;  // 16-byte aligned
    if (r >= 0 && (uint32_t)r + 16u <= total) {
      const uint32_t w = (uint32_t)r >> 5;
      const uint64_t two = (uint64_t)st[w] | ((uint64_t)st[w + 1] << 32);
      const uint32_t bits = (uint32_t)(two >> (r & 31));
#ifdef PGTG_NT_OBS  // A/B: streaming (nontemporal) observation stores
      typedef unsigned int v4u __attribute__((ext_vector_type(4)));
      v4u o = {expand4(bits), expand4(bits >> 4), expand4(bits >> 8), expand4(bits >> 12)};
      __builtin_nontemporal_store(o, reinterpret_cast<v4u*>(cp));
#else
      *reinterpret_cast<uint4*>(cp) = make_uint4(expand4(bits), expand4(bits >> 4), expand4(bits >> 8), expand4(bits >> 12));
#endif
    } else {
      for (int b = 0; b < 16; b++) {
        const int rb = r + b;
        if (rb >= 0 && (uint32_t)rb < total) cp[b] = (uint8_t)((st[rb >> 5] >> (rb & 31)) & 1u);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------------
struct Lds {
  int envs;            // envs per workgroup (<= kBlock); lanes >= envs only help with the writes
  int plan_stride_dw;  // per-lane plan words (odd)
  int scratch_dw;      // per-env reset hand-over words (odd): spawn in; position, sg, path length out
  int traf_dw;         // per-lane traffic region words (occupancy counters / reset scratch), odd or 0
  int hist_dw;         // per-lane route histogram words for the braking rules, odd or 0
  int seg_bits;        // per-env observation bits in the dense image (= output bytes per env)
  int sub_envs;        // envs per observation sub-batch (== envs when they all fit)
  int stream_words;    // observation image words (dense bit stream of sub_envs envs, +2 pad)
  int spread;          // env slots spread over the four waves (traffic: long per-lane chains)
  int compact;         // resets run on dense lanes (wave 0 first) instead of on their env's lane
  int queue;           // step launches use k_envq (maps generated one episode ahead by helper waves)
  int gen_off;         // k_envq: word offset of the helper lanes' plan scratch (kQueueLanes x plan_stride_dw)
  int lm_words;        // terminal-observation line mask words (0: test the selection bytes)
  int stagger;         // first-round start offsets (stagger_start) on
  int stagger_wgs;     // workgroups resident in the first round (blocks per CU x CUs)
  int ramp_pct;        // the ramp, in percent of the last launch's first workgroup duration
  int img_in_traf;     // k_env with traffic: the whole workgroup's image in the (after the car pass dead)
                       // traffic region; the agent tile's counters and the reset hand-over words in hist
  int prio;            // k_envb: issue priority of the env and writer waves over the helper (PGTG_TUNING
                       // builds only, PGTG_PRIO; 0 otherwise)
  int abl;             // diagnostic ablations (PGTG_TUNING builds only, PGTG_ABL; always 0 otherwise):
                       // k_envq bit 0 no ring refills (the stale entries taken as they are), bit 1 no
                       // terminal-observation writes, bit 2 no observation writes, bit 4 refills without
                       // the ring-entry stores, bit 5 no plan-row stores at resets, bit 7 k_envb writes the
                       // post-step image of every env as terminal rows (a valid A/B), bit 9 k_envb's ring
                       // entries without the folded path directions (marked in LDS; a valid A/B) (timing experiments:
                       // the results are wrong)
};
constexpr int kQueueLanes = 64;  // k_envq lanes that generate queued maps (one wave)
constexpr int kMaxQueueGrid = 4096;  // k_envq's persistent grid at most
// DevState::qctr: [2][kMaxQueueGrid] per-workgroup request counts (launch parity), [3] block
// counters, then per rotating set (3) and overflow list (8, one per workgroup residue mod 8) the
// overflow lists' lengths
constexpr int kQctrBlocks = 2 * kMaxQueueGrid;
constexpr int kQctrOvfLen = kQctrBlocks + 3;
constexpr int kQctrWords = kQctrOvfLen + 24;
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += (uint32_t)__shfl_xor((int)x, o);
  return x;
}
// refill requests one k_envq workgroup may make per launch (three times its share of the blocks: a
// workgroup stops taking blocks before it could exceed them)
__host__ __device__ inline uint64_t queue_req_cap(uint64_t nblk, uint64_t grid, int envs) {
  const uint64_t c = 3 * ((nblk + grid - 1) / grid) * (uint64_t)envs;
  return c < (uint64_t)kQueueLanes ? (uint64_t)kQueueLanes : c;  // (the helper reads its first kQueueLanes ahead)
}
constexpr uint64_t kStaggerMaxTicks = 20000;  // 200 us of 100 MHz wall clock: a bound, never reached
constexpr int kQueueDepth = 2;   // queued maps per env (a ring: the next two episodes') of k_envq
constexpr int kBlockDepth = 3;   // of k_envb (the rings refilled per block)
constexpr uint32_t kQueueStale = 0x80u;  // qstate flag: the ring's entries are not this env's (k_qfill)
constexpr int kViewDw = 8;       // k_envq with <= 32 envs: an env's view words for the image builders

// a ring entry's spawn tag (its last word): the spawn counter it was generated for, inverted so that
// zeroed memory matches none
__host__ __device__ inline uint32_t queue_tag(uint32_t spawn) { return ~spawn; }
__host__ __device__ inline int odd_up(int x) { return x | 1; }
// words of a dense observation image of `envs` envs (+2: the writers' funnel reads run one word
// ahead; a multiple of 4 so that what follows stays 16-byte aligned)
__host__ inline int img_words(int envs, int bits) { return ((int)(((int64_t)envs * bits + 31) / 32) + 2 + 3) & ~3; }

__host__ inline void lds_tail(Lds& l, const DevCfg& c);
__host__ inline Lds lds_layout(const DevCfg& c, int envs) {
  Lds l;
  l.envs = envs;
  l.plan_stride_dw = odd_up((c.nt + 1) / 2);
  l.scratch_dw = c.need_car ? 0 : 3;  // with traffic: inside the (by then dead) occupancy counters
  l.traf_dw = c.need_car ? odd_up(c.traf_bytes / 4) : 0;
  // route histogram of the braking rules: always with traffic (pgtg_set_rules may add rules later)
  l.hist_dw = (c.n_rules > 0 || c.need_car) ? 5 : 0;
  l.seg_bits = c.n_channels * c.win * c.win;
  const int budget_words = 12 * 1024;  // 48 KiB observation image
  int sub = l.seg_bits > 0 ? (int)(((int64_t)budget_words - 3) * 32 / l.seg_bits) : envs;
  l.sub_envs = sub > envs ? envs : (sub < 1 ? 1 : sub);
  l.stream_words = img_words(l.sub_envs, l.seg_bits);
  l.spread = c.need_car ? 1 : 0;
  l.compact = 1;
  // map queue: random maps without traffic, braking rules or lane channels (k_envq), a whole-workgroup
  // observation image and at least one wave without env slots
  l.queue = !c.need_car && c.n_rules == 0 && !c.fixed_map && !c.generic_channels && envs <= kBlock - 64 && l.sub_envs >= envs;
  l.stagger = 0;
  l.stagger_wgs = 0;
  // (1 048 576 envs, the persistent k_envq, one box: 25 % 402 us, 15 % 404, 35 % 406, 50 % 410; 100 %
  // 3.5 % slower than 50 % on another box)
  l.ramp_pct = 25;
  l.img_in_traf = 0;
  l.abl = 0;
  l.prio = 0;
#ifdef PGTG_TUNING  // A/B and diagnostic builds only: the product library reads no environment
  if (const char* e = getenv("PGTG_ABL")) l.abl = atoi(e);
  if (const char* e = getenv("PGTG_PRIO")) l.prio = atoi(e);
  if (const char* e = getenv("PGTG_RAMP")) l.ramp_pct = atoi(e);
  if (const char* e = getenv("PGTG_SPREAD")) l.spread = atoi(e);
  if (const char* e = getenv("PGTG_COMPACT")) l.compact = atoi(e);
  if (const char* e = getenv("PGTG_QUEUE")) l.queue = l.queue && atoi(e);
#endif
  lds_tail(l, c);
  return l;
}
// After the observation image: sel[kBlock] | 32 B (k_env: per-wave reset ballots) or 128 B (k_envq:
// barrier counter) | the terminal-observation line mask (lm_words) | k_envq: the
// refill lanes' plan scratch (gen_off).  Recomputed whenever the image size changes.
__host__ inline int tail_bytes(const Lds& l) {
  return kBlock + (l.queue ? 128 : 32) + 4 * l.lm_words + (l.queue && l.envs <= 32 ? 4 * kViewDw * l.envs : 0);
}
__host__ inline void lds_tail(Lds& l, const DevCfg& c) {
  // line mask: one bit per 128-byte output line of a whole-workgroup image (<= 64 words), else the
  // writers test the per-env selection bytes
  const int64_t total = (int64_t)l.envs * l.seg_bits;
  const int lines = (int)((127 + total) / 128) + 1;
  l.lm_words = (!c.need_car && l.sub_envs >= l.envs && lines <= 64 * 32) ? (lines + 31) / 32 : 0;
#ifdef PGTG_TUNING
  if (const char* e = getenv("PGTG_LINEMASK")) l.lm_words = atoi(e) ? l.lm_words : 0;
#endif
  l.gen_off = (int)(((size_t)l.envs * (l.plan_stride_dw + l.scratch_dw + l.traf_dw + l.hist_dw) + l.stream_words) +
                    tail_bytes(l) / 4);
}
__host__ inline size_t lds_bytes(const Lds& l) {
  return (size_t)4 * ((size_t)l.envs * (l.plan_stride_dw + l.scratch_dw + l.traf_dw + l.hist_dw) + l.stream_words) +
         tail_bytes(l) + (l.queue ? (size_t)4 * kQueueLanes * l.plan_stride_dw : 0);
}

// Traffic launches with one-tile windows: once the car pass is over, the traffic region (occupancy
// counters, spawner cache) is dead except for the 16 counter bytes of the agent's tile that the
// traffic channel reads, so the whole workgroup's observation image goes there (one pass instead of
// sub-batches) and hist (the braking histogram, dead after the step too) keeps those 16 bytes and the
// reset hand-over words: hist = 4 counter words + 3 hand-over words.
__host__ inline void lds_img_in_traf(Lds& l, const DevCfg& c) {
  if (!c.need_car || !c.obs_fast || l.envs < 1) return;
  if ((int64_t)img_words(l.envs, l.seg_bits) > (int64_t)l.envs * l.traf_dw) return;
  l.img_in_traf = 1;
  l.sub_envs = l.envs;
  l.stream_words = 0;
  l.hist_dw = 7;
  lds_tail(l, c);
}

enum { MODE_STEP = 0, MODE_RESET_SEEDED = 1, MODE_RESET_UNSEEDED = 2, MODE_OBSERVE = 3 };

__device__ __forceinline__ void write_small_outputs(const DevCfg& c, const PgtgOutputs& o, uint64_t i, const EnvView& v,
                                                    const ObsInfo& oi, bool final) {
  if (!final) {
    if (o.position) reinterpret_cast<int2*>(o.position)[i] = make_int2(oi.posx, oi.posy);
    if (o.velocity) reinterpret_cast<int2*>(o.velocity)[i] = make_int2(v.vx, v.vy);
    if (o.next_subgoal) o.next_subgoal[i] = oi.nsd;
  } else {
    if (o.final_position) reinterpret_cast<int2*>(o.final_position)[i] = make_int2(oi.posx, oi.posy);
    if (o.final_velocity) reinterpret_cast<int2*>(o.final_velocity)[i] = make_int2(v.vx, v.vy);
    if (o.final_next_subgoal) o.final_next_subgoal[i] = oi.nsd;
  }
}

// Observation pass over sub-batches: build the envs with want != 0 (small outputs as final or not)
// into the segment image, then write the image slice to dst (selection sel).
template <bool TR, bool BIG>
__device__ __forceinline__ void obs_pass(const DevCfg& c, const DevState& S, const Plan& pl, const EnvView& v,
                                         const PgtgOutputs& o, uint8_t* dst, uint64_t env0, int nb, bool want,
                                         bool final, const uint8_t* sel, uint32_t* st, const Lds& L,
                                         const uint8_t* occ, int slot) {
  for (int sb = 0; sb < nb; sb += L.sub_envs) {
    const int cnt = min(L.sub_envs, nb - sb);
    if (want && slot >= sb && slot < sb + cnt) {
      ObsInfo oi;
      build_obs<TR, BIG, true, !TR>(c, S, pl, v, st, (uint32_t)(slot - sb) * (uint32_t)c.obs_bytes, oi, occ);
      write_small_outputs(c, o, env0 + slot, v, oi, final);
    }
    lds_barrier();
    if (dst)
      write_obs(dst + (env0 + sb) * (uint64_t)c.obs_bytes, (uint32_t)cnt, (uint32_t)c.obs_bytes, st, sel ? sel + sb : nullptr);
    lds_barrier();
  }
}

// 4 waves per SIMD (<= 128 VGPRs) keeps 16 waves per CU resident to hide per-lane latency
// Workgroups of one launch run the same phases (staging, step, terminal writes, reset, image writes)
// and the first round starts them all at once, so the whole chip would write in the same windows
// and compute in the same windows.  Offsetting the first round's starts along a ramp keeps the
// offsets for every later round (a finishing workgroup's slot takes the next one at once), so the
// write phases of some workgroups overlap the compute phases of others.
// The ramp is a quarter of the workgroup duration the previous launch measured (workgroup 0's, in
// wall-clock ticks, S.wg_ticks), so it follows the phase length of whatever the kernel does on this
// device instead of a tuned constant; the first launch of a handle runs without offsets.
__device__ __forceinline__ uint64_t stagger_start(const Lds& L, const DevState& S) {
  if (!L.stagger) return 0;
  const uint64_t t0 = wall_clock64();
  if (blockIdx.x == 0 || blockIdx.x >= (unsigned)L.stagger_wgs) return t0;
  const uint64_t span = min(S.wg_ticks[0] * (uint64_t)L.ramp_pct / 100ull, (unsigned long long)kStaggerMaxTicks);
  const uint64_t wait = span * blockIdx.x / (unsigned)L.stagger_wgs;
  while (wall_clock64() - t0 < wait) __builtin_amdgcn_s_sleep(16);
  return t0;
}
// workgroup 0 records its duration for the next launch's ramp (timing only: not part of any result)
__device__ __forceinline__ void stagger_record(const Lds& L, const DevState& S, uint64_t t0) {
  if (L.stagger && blockIdx.x == 0 && threadIdx.x == 0) S.wg_ticks[0] = wall_clock64() - t0;
}

template <bool TR, bool BIG>
__global__ void __launch_bounds__(kBlock, TR ? 3 : 4) k_env(const DevCfg* __restrict__ cfg, const Tables* __restrict__ gtab,
                                                 DevState S, const uint8_t* __restrict__ actions,
                                                 const uint8_t* __restrict__ mask, PgtgOutputs out, int mode, Lds L,
                                                 uint32_t tr_slot) {
  extern __shared__ uint32_t lds[];
  const DevCfg& c = *cfg;
  const int tid = threadIdx.x;
  const uint64_t t_start = TR ? 0 : stagger_start(L, S);
  STAMP(0);
  // the traffic-reset list of the next launch starts empty (its previous consumer has finished)
  if ((TR && c.need_car) && mode != MODE_OBSERVE && blockIdx.x == 0 && tid == 0) S.tr_count[tr_slot ^ 1u] = 0u;
  // stage the lane-indexed tables (kLanes only when a pass needs it)
  stage_tables(gtab, c.generic_channels || (TR && c.need_car));
  const uint64_t env0 = (uint64_t)blockIdx.x * L.envs;
  const int nb = (int)min((uint64_t)L.envs, S.n - env0);
  // env slots: E/4 per wave when a workgroup holds fewer than 256 envs, so that all four SIMDs
  // work and a wave's divergence spans fewer envs; contiguous envs per wave (coalesced rows)
  const int per_wave = (!L.spread || L.envs >= kBlock) ? 64 : L.envs / 4;
  const bool has_slot = (tid & 63) < per_wave;
  const int slot = has_slot ? (tid >> 6) * per_wave + (tid & 63) : 0;
  const uint64_t i = env0 + slot;
  const bool live = has_slot && slot < nb;
  const int my_slot = slot;
  uint32_t* plan_w = lds + my_slot * L.plan_stride_dw;
  uint32_t* traf_w = lds + L.envs * (L.plan_stride_dw + L.scratch_dw) + my_slot * L.traf_dw;
  uint32_t* hist_w = lds + L.envs * (L.plan_stride_dw + L.scratch_dw + L.traf_dw) + my_slot * L.hist_dw;
  const int env_dw = L.plan_stride_dw + L.scratch_dw + L.traf_dw + L.hist_dw;
  uint32_t* st = (TR && L.img_in_traf) ? lds + L.envs * (L.plan_stride_dw + L.scratch_dw) : lds + L.envs * env_dw;
  uint8_t* sel = reinterpret_cast<uint8_t*>(lds + L.envs * env_dw + L.stream_words);  // [kBlock]
  uint64_t* wmask = reinterpret_cast<uint64_t*>(sel + kBlock);     // [4] reset ballot per wave
  uint32_t* lm = L.lm_words ? reinterpret_cast<uint32_t*>(sel + kBlock + 32) : nullptr;  // terminal lines
  const bool img_traf = TR && L.img_in_traf;
  const int xf_off = img_traf ? L.envs * (L.plan_stride_dw + L.scratch_dw + L.traf_dw) + 4
                   : L.envs * L.plan_stride_dw + ((TR && c.need_car) ? L.envs * L.scratch_dw : 0);
  const int xf_dw = img_traf ? L.hist_dw : (TR && c.need_car) ? L.traf_dw : L.scratch_dw;
  uint32_t* xf = lds + xf_off + my_slot * xf_dw;  // reset hand-over words
  uint8_t* occ = reinterpret_cast<uint8_t*>(traf_w);
  uint16_t* sp_l = reinterpret_cast<uint16_t*>(occ + c.sp_cache_off);  // first spawners of the list
  uint8_t* hist = reinterpret_cast<uint8_t*>(hist_w);
  Plan pl{reinterpret_cast<uint16_t*>(plan_w)};

  EnvView v{};
  TrafState ts{0, 0, 0, 0};
  bool occ_sat = false;  // a 4-bit occupancy counter saturated this launch (exact recounts from then on)
  bool occ_valid = false;  // the persisted counters of this env are exact (traf.w)
  int err = 0;
  int act = 0;
  if (live) {
    v = rec_load(S.rec, i);
    if (mode == MODE_STEP) act = actions[i];  // issued with the staging loads, not on the step's chain
    if ((TR && c.need_car)) {
      uint4 tr4 = S.traf[i];
      ts.n_cars = tr4.x & 0xffffu;
      ts.n_spawners = tr4.x >> 16;
      ts.next_id = tr4.y;
      ts.tail = tr4.z;
      ts.fresh = (tr4.w & kTrafFresh) ? 1u : 0u;
      occ_valid = (tr4.w & kTrafOccValid) != 0u;
    }
    stage_plan<BIG>(S.plan + i * (uint64_t)c.plan_stride, c.plan_dq, plan_w, L.plan_stride_dw);
  }
  for (int k = tid; k < L.lm_words; k += kBlock) lm[k] = 0u;
  lds_barrier();  // sT ready
  if (live && (TR && c.need_car) && occ_valid) {
    // the counters the last launch left (one coalesced row per counter word), or k_traffic in the
    // staging block of a fresh env
    const int nw = c.nt * 4;
    const gu32* ob = ts.fresh ? fresh_block(S, i) + S.fresh_occ : (const gu32*)(S.occ + i);
    const uint64_t ostep = ts.fresh ? 1ull : S.n;
    for (int w0 = 0; w0 < nw; w0 += 16) {
      uint32_t r[16];
#pragma unroll
      for (int u = 0; u < 16; u++) r[u] = ob[(uint64_t)min(w0 + u, nw - 1) * ostep];
#pragma unroll
      for (int u = 0; u < 16; u++)
        if (w0 + u < nw) traf_w[w0 + u] = r[u];
    }
  }
  if (live && (TR && c.need_car) && !occ_valid) {
    // occupancy counters from the current car positions (one coalesced slot row per slot index, 16
    // loads in flight per lane, the next 16 requested before the counters of the current ones are
    // updated so that their HBM latency overlaps the LDS work)
    for (int w = 0; w < c.nt * 4; w++) traf_w[w] = 0u;  // 16 B of 4-bit counters per tile
    const CarSlots cs(S, i);
    const gu32* rb = ts.fresh ? fresh_block(S, i) : cs.w0;  // (a fresh env's cars: its staging block)
    const uint64_t rstep = ts.fresh ? 1ull : S.n;
    const int tail = (int)ts.tail, tw = pinned(c.tw);
    uint32_t nx16[16];
#pragma unroll
    for (int g = 0; g < 16; g++) nx16[g] = rb[(uint64_t)(g < tail ? g : 0) * rstep];
    for (int k0 = 0; k0 < tail; k0 += 16) {
      uint32_t a16[16];
#pragma unroll
      for (int g = 0; g < 16; g++) a16[g] = nx16[g];
#pragma unroll
      for (int g = 0; g < 16; g++) nx16[g] = rb[(uint64_t)(k0 + 16 + g < tail ? k0 + 16 + g : 0) * rstep];
      // the 16 slot lookups first (every slot holds valid coordinates: empty slots read as (0, 0),
      // slots past the tail as slot 0), their reads batched; then the counter updates in order
      int sl[16];
#pragma unroll
      for (int g = 0; g < 16; g++) sl[g] = lane_slot_tw(tw, pl, (int)(a16[g] & 255u), (int)((a16[g] >> 8) & 255u));
#pragma unroll
      for (int g = 0; g < 16; g++) {
        if (k0 + g < tail && !(a16[g] & kCarEmpty)) {
          if (sl[g] < 0) err = PGTG_E_UNSUPPORTED;
          else occ_inc(occ, sl[g], occ_sat);
        }
      }
    }
  }
  if (live && (TR && c.need_car)) {
    // the head of the spawner list (respawn positions) into LDS
    // (the env's list is contiguous: 16-byte loads, all issued before the LDS stores)
    const int nsp = min((int)ts.n_spawners, kSpCache);
    const uint4* src = reinterpret_cast<const uint4*>(S.spawners + i * (uint64_t)S.sp_pitch);
    const int q_last = (int)(S.sp_pitch / 8u) - 1;
    uint4 q4[kSpCache / 8];
#pragma unroll
    for (int q = 0; q < kSpCache / 8; q++) q4[q] = src[min(q, q_last)];
    uint32_t* dl = reinterpret_cast<uint32_t*>(sp_l);
#pragma unroll
    for (int q = 0; q < kSpCache / 8; q++) {
      if (q * 8 < nsp) {
        dl[4 * q] = q4[q].x;
        dl[4 * q + 1] = q4[q].y;
        dl[4 * q + 2] = q4[q].z;
        dl[4 * q + 3] = q4[q].w;
      }
    }
  }
  STAMP(1);
  uint8_t my_sel = 0;
  if (live) {
    if (mode == MODE_STEP) {
      StepResult res{0.0, 0.0, 0u};
      if (!err) err = env_step<TR, BIG>(c, S, i, v, pl, act, res, occ, occ_sat, sp_l, ts, hist);
      if ((TR && c.need_car) && !occ_sat) {  // the counters after the car pass, for the next launch
        const int nw = c.nt * 4;
        for (int w = 0; w < nw; w++) S.occ[(uint64_t)w * S.n + i] = traf_w[w];
      }
      occ_valid = (TR && c.need_car) && !occ_sat && err == 0;
      const bool done = (v.flags & (kFlagTerminated | kFlagTruncated)) != 0;
      // BIG maps keep the used subgoals in the plan: the row goes back to HBM unless the env resets now
      if (BIG && res.plan_dirty && !(done && c.autoreset && err == 0)) store_plan_row(c, S, i, plan_w, L.plan_stride_dw);
      if (out.reward) out.reward[i] = res.reward;
      if (out.cost) out.cost[i] = res.cost;
      if (out.terminated) out.terminated[i] = (v.flags & kFlagTerminated) ? 1 : 0;
      if (out.truncated) out.truncated[i] = (v.flags & kFlagTruncated) ? 1 : 0;
      if (out.braking) out.braking[i] = (uint8_t)res.triggered;
      my_sel = (done && c.autoreset && err == 0) ? 1 : 0;
      if (lm && my_sel && out.final_obs) mark_lines(lm, out.final_obs + env0 * (uint64_t)c.obs_bytes, (uint32_t)slot, (uint32_t)c.obs_bytes);
    } else if (mode == MODE_RESET_SEEDED || mode == MODE_RESET_UNSEEDED) {
      const bool do_reset = mask == nullptr || mask[i] != 0;
      if (do_reset && mode == MODE_RESET_SEEDED) v.spawn = 0;
      my_sel = do_reset ? 2 : 0;
    }
  }
  if (has_slot) sel[slot] = my_sel;
  // the images read the counters of the agent's tile only: with the image in the traffic region, those
  // 16 bytes move to hist first (the barrier below orders this before any image store)
  const uint8_t* occ_img = occ;
  if (img_traf) {
    if (live) {
      const int pix = min(max(0, v.px), c.W - 1), piy = min(max(0, v.py), c.H - 1);
      const int t = (piy / kTile) * c.tw + pix / kTile;
#pragma unroll
      for (int q = 0; q < 4; q++) hist_w[q] = traf_w[t * 4 + q];
    }
    occ_img = hist;
  }
  STAMP(2);
  const bool single = L.sub_envs >= nb;  // the whole workgroup's image fits: build once, rebuild resets
  const bool reset_now = my_sel != 0;
  if (L.compact) {  // the workgroup's resets, in wave order, go to threads 0 .. n_resets-1
    const uint64_t m = __ballot(reset_now);
    if ((tid & 63) == 0) wmask[tid >> 6] = m;
  }
  int n_final = 0;
  if (L.compact) {  // step launches: every reset is a finished episode (my_sel == 1)
    lds_barrier();
    if (mode == MODE_STEP)
      for (int w = 0; w < kBlock / 64; w++) n_final += __popcll(wmask[w]);
  } else {
    n_final = __syncthreads_count(my_sel == 1);
  }
  const bool want_final = mode == MODE_STEP && n_final && (out.final_obs || out.final_position || out.final_velocity);
  int n_resets = 0, wslot = -1;
  if (L.compact) {
#pragma unroll
    for (int w = 0; w < kBlock / 64; w++) {
      const uint64_t m = wmask[w];
      const int cw = __popcll(m);
      if (tid >= n_resets && tid < n_resets + cw) wslot = w * per_wave + select64(m, tid - n_resets);
      n_resets += cw;
    }
  }
  // threads without a reset (compacted), or waves without env slots (workgroups of fewer than 256
  // unspread envs), write the terminal observations while the resets run
  const int t_help = L.compact ? ((n_resets + 63) / 64) * 64
                               : ((L.spread || L.envs >= kBlock) ? kBlock : ((L.envs + 63) / 64) * 64);
  const bool helpers = single && t_help < kBlock;
  if (single) {
    if (live && (my_sel != 2)) {
      ObsInfo oi;
      build_obs<TR, BIG, true, !TR>(c, S, pl, v, st, (uint32_t)slot * (uint32_t)c.obs_bytes, oi, occ_img, 0, -1, true, false, img_traf);
      write_small_outputs(c, out, i, v, oi, my_sel == 1);
    }
    if (L.compact && reset_now) xf[0] = v.spawn;  // after the terminal image read the counters
    STAMP(28);
    lds_barrier();
    STAMP(29);
    if (want_final && out.final_obs && !helpers)
      write_obs(out.final_obs + env0 * (uint64_t)c.obs_bytes, (uint32_t)nb, (uint32_t)c.obs_bytes, st, sel, -1, kBlock, lm);
  } else {
    if (want_final) obs_pass<TR, BIG>(c, S, pl, v, out, out.final_obs, env0, nb, my_sel == 1, true, sel, st, L, occ, slot);
    if (L.compact) {
      if (reset_now) xf[0] = v.spawn;
      lds_barrier();
    }
  }
  STAMP(3);
  bool tr_push = false;
  if (!L.compact) n_resets = __syncthreads_count(reset_now);
  if (tid == 0 && n_resets) atomicAdd(&S.counters[1], (unsigned long long)n_resets);
  if (helpers && want_final && out.final_obs && tid >= t_help)
    write_obs(out.final_obs + env0 * (uint64_t)c.obs_bytes, (uint32_t)nb, (uint32_t)c.obs_bytes, st, sel, tid - t_help,
              kBlock - t_help, lm);
  if (L.compact) {
    if (wslot >= 0) {
      uint32_t* xw = lds + xf_off + wslot * xf_dw;
      uint32_t* pw = lds + wslot * L.plan_stride_dw;
      const uint64_t iw = env0 + wslot;
      EnvView vv{};
      vv.spawn = xw[0];
      TrafState tw{0, 0, 0, 0};
      const int e2 = env_reset<TR, BIG>(c, S, iw, vv, reinterpret_cast<uint16_t*>(pw), tw);
      store_plan_row(c, S, iw, pw, L.plan_stride_dw);
      xw[0] = ((uint32_t)vv.px & 0xffffu) | ((uint32_t)vv.py << 16);
      xw[1] = vv.sg;
      xw[2] = vv.path_len | (uint32_t)(-e2) << 16;
    }
    lds_barrier();  // hand-over words ready (and the terminal observations read from the image)
    if (reset_now) {  // env_reset's state on the env's own lane
      const uint32_t x0 = xf[0], x2 = xf[2];
      v.px = (int)(int16_t)(x0 & 0xffffu);
      v.py = (int)(int16_t)(x0 >> 16);
      v.sg = xf[1];
      v.path_len = x2 & 0xffffu;
      v.spawn += 5u;
      v.used = 0;
      v.flags = 0;
      v.phase = 0;
      v.elapsed = 0;
      v.vx = v.vy = 0;
      const int e2 = -(int)(x2 >> 16);
      if (e2) err = e2;
      tr_push = (TR && c.need_car) && e2 == 0;
      if ((TR && c.need_car) && e2 == 0) ts = TrafState{0, 0, 0, 0};
    }
  } else if (reset_now) {
    int e2 = env_reset<TR, BIG>(c, S, i, v, pl.p, ts);
    if (e2) err = e2;
    tr_push = (TR && c.need_car) && e2 == 0;
    store_plan_row(c, S, i, plan_w, L.plan_stride_dw);
  }
  STAMP(4);
  if (live) {
    if (mode != MODE_OBSERVE) {
      rec_store(S.rec, i, v);
      // (a reset env's counters come from k_traffic with its fresh cars; until then invalid)
      if ((TR && c.need_car))
        S.traf[i] = make_uint4(ts.n_cars | ts.n_spawners << 16, ts.next_id, ts.tail,
                               (occ_valid && !reset_now ? kTrafOccValid : 0u) | (ts.fresh ? kTrafFresh : 0u));
    }
    if (mode != MODE_OBSERVE || err) S.err[i] = (uint8_t)(-err);
    if (S.qstate && reset_now) S.qstate[i] = (uint8_t)kQueueStale;  // maps generated here: the queued ones are stale
  }
  if (TR && c.need_car) {
    // k_traffic's work list: one wave-aggregated atomic per wave
    const uint64_t m = __ballot(tr_push);
    if (m) {
      const int lane = tid & 63, leader = __ffsll((long long)m) - 1;
      uint32_t base = 0;
      if (lane == leader) base = atomicAdd(&S.tr_count[tr_slot], (uint32_t)__popcll(m));
      base = __shfl(base, leader);
      if (tr_push) S.tr_list[base + __popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)i;
    }
  }
  STAMP(5);
  if (single) {
    if (helpers && !L.compact) lds_barrier();  // the terminal observations are written before slots are rebuilt
    if (reset_now) {
      ObsInfo oi;
      build_obs<TR, BIG, true, !TR>(c, S, pl, v, st, (uint32_t)slot * (uint32_t)c.obs_bytes, oi, nullptr);  // cars come from k_traffic
      write_small_outputs(c, out, i, v, oi, false);
    }
    STAMP(30);
    lds_barrier();
    STAMP(31);
    if (out.obs)
      write_obs(out.obs + env0 * (uint64_t)c.obs_bytes, (uint32_t)nb, (uint32_t)c.obs_bytes, st, nullptr);
  } else {
    obs_pass<TR, BIG>(c, S, pl, v, out, out.obs, env0, nb, live, false, nullptr, st, L, reset_now ? nullptr : occ,
                 slot);
  }
  if (mode == MODE_STEP && tid == 0) atomicAdd(&S.counters[0], (unsigned long long)nb);
  if (!TR) stagger_record(L, S, t_start);
  STAMP(6);
  if (TR) STAMPR(0);
}

// ------------------------------------------------------------------------------------------------
// Map queue.  Everything env_reset derives from the map stream -- the map, its compiled path, the
// start square -- depends only on (seed, spawn counter), not on the episode before it, so the next
// two episodes' maps of every env are generated ahead and a reset takes the head of the env's ring.
// ------------------------------------------------------------------------------------------------
// One ring entry: generate_map + compile_path + the start draw of env_reset for spawn counter `k`,
// built in the lane's LDS plan scratch and written to HBM.
template <bool BIG>
__device__ __forceinline__ void gen_queue_entry(const DevCfg& c, const DevState& S, uint64_t i, uint32_t k,
                                                uint16_t* plan, int pdw, uint32_t* __restrict__ dst,
                                                bool no_store = false, bool fold_ok = true) {
  SeedPool sp = ss_pool(S.seed[i]);
  Pcg map_rng = ss_child(sp, k);
  int st_t, st_d, gl_t, gl_d;
  uint64_t ix[4];
  generate_map<BIG>(c, BIG ? S.epk : sT.epk, map_rng, plan, st_t, st_d, gl_t, gl_d, ix);
  // the path's subgoal directions: kept as four tile masks and folded into the words stored below
  // (maps of <= 64 tiles on the dual path) instead of a read-modify-write of every path tile's LDS word.
  // k_envb folds (one-round launches, where the helper's chain counts: 131 072 envs 70.4 vs 71.2 us),
  // k_envq does not (eight rounds, where the helpers' instructions count against the env waves' issue:
  // 1 048 576 envs 400 vs 406.7 us; profiles/r06/s8); k_qfill's entries are the same either way
  uint64_t dirs[4] = {0ull, 0ull, 0ull, 0ull};
  const bool fold = !BIG && c.dual && fold_ok;
  int len = compile_generated<BIG>(c, plan, st_t, gl_t, ix, fold ? dirs : nullptr);
  int px = 0, py = 0, err = 0;
  if (len <= 0 || !((plan_exits(plan[st_t]) >> st_d) & 1u)) {
    err = len < 0 ? PGTG_E_DEVICE : PGTG_E_MAP;  // (< 0: the path walk's masks were inconsistent)
    len = 0;
  } else {  // env_reset's starter square (pgtg/map.py:31-34)
    const int j = (int)pcg_int(map_rng, 3);
    const int tx = st_t % c.tw, ty = st_t / c.tw;
    int lx, ly;
    switch (st_d) {
      case 0: lx = 3 + j; ly = 0; break;
      case 1: lx = 8; ly = 3 + j; break;
      case 2: lx = 3 + j; ly = 8; break;
      default: lx = 0; ly = 3 + j; break;
    }
    px = tx * kTile + lx;
    py = ty * kTile + ly;
  }
  const uint32_t* pw = reinterpret_cast<const uint32_t*>(plan);
  uint4* d4 = reinterpret_cast<uint4*>(dst);
  const int pwords = c.plan_dq * 4;
#ifdef PGTG_TUNING
  if (no_store) {  // (timing experiment: the entry is built but not written)
    if (len == 12345 && px == 7) d4[0] = make_uint4(0, 0, 0, 0);
    return;
  }
#endif
  for (int q = 0; q < pwords / 4; q++) {
    uint32_t wv[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      // tiles >= nt are padding: written as 0 (the scratch holds stale LDS there), so that the queue
      // and the plans taken from it are a function of the seeds alone (byte-identical state dumps)
      wv[j] = (q * 4 + j < pdw) ? (pw[q * 4 + j] & plan_word_mask(c, q * 4 + j)) : 0u;
      if (fold) {  // direction + 1 into bits 11-13 of both tiles of the word
        const int t0 = 2 * (q * 4 + j);
        const uint32_t d0 = (uint32_t)((dirs[0] >> t0) & 1ull) + 2u * (uint32_t)((dirs[1] >> t0) & 1ull) +
                            3u * (uint32_t)((dirs[2] >> t0) & 1ull) + 4u * (uint32_t)((dirs[3] >> t0) & 1ull);
        const uint32_t d1 = t0 + 1 < 64 ? (uint32_t)((dirs[0] >> (t0 + 1)) & 1ull) + 2u * (uint32_t)((dirs[1] >> (t0 + 1)) & 1ull) +
                                          3u * (uint32_t)((dirs[2] >> (t0 + 1)) & 1ull) + 4u * (uint32_t)((dirs[3] >> (t0 + 1)) & 1ull)
                                        : 0u;
        wv[j] |= (d0 << 11 | d1 << 27) & plan_word_mask(c, q * 4 + j);
      }
    }
    d4[q] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
  }
  d4[pwords / 4] = make_uint4(((uint32_t)px & 0xffffu) | ((uint32_t)py << 16),
                              (uint32_t)st_t | (uint32_t)st_d << 8 | (uint32_t)gl_t << 16 | (uint32_t)gl_d << 24,
                              (uint32_t)len | (uint32_t)(-err) << 16, queue_tag(k));
  for (int q = pwords / 4 + 1; q < c.qrec_dw / 4; q++) d4[q] = make_uint4(0u, 0u, 0u, 0u);  // the line's rest
}

// k_envq ablations (tools/ab_multi.sh, PGTG_ABL): compiled in only in the tuning build; the product kernel tests
// no runtime flag for them
#ifdef PGTG_TUNING
#define ABLATE(L, bit) (((L).abl & (bit)) != 0)
#else
#define ABLATE(L, bit) false
#endif

// Barrier among the waves of a workgroup that take part (lane 0 of each arrives at an LDS counter
// that only grows; `target` = uses so far x participating waves), for phases that must not wait
// for a wave busy elsewhere.
// LDS-only fences: the waves exchange LDS data only, so their global stores stay in flight across
// the barrier (a plain workgroup fence waits for every outstanding global access first).
__device__ __forceinline__ void sub_barrier(uint32_t* ctr, uint32_t target) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Step launch with the map queue (no traffic; workgroups of <= 192 envs), persistent: the grid is the
// workgroups resident at once; each takes env block blockIdx.x, then the next free one from a counter
// (fetched one block ahead), until none is left.  Its env and writer waves step a block, write the
// terminal observations, take the ring heads of the envs that finished -- requesting the
// next-but-one episode's map for the slot taken, in the workgroup's own list -- and write the new
// observations, synchronising among themselves only.  Its helper wave (wave `env_waves`, the first
// without env slots) meanwhile generates the maps its workgroup requested in the previous launch,
// kQueueLanes at a time, so that neither role waits for the other at a block's end.  A request made
// in launch t is served in launch t + 1 and its entry taken in t + 2 at the earliest: two entries
// per env suffice, and no entry is written while it can be read.
// (One shared request list instead: 497 vs 456 us per 1 048 576-env launch, its counter a hot spot on
// every env wave's path; static blocks blockIdx.x + k * gridDim.x: 455 us against the counter's 424.)
// The map-queue step's observation images.  With <= 32 envs per workgroup they all sit in wave 0
// and most of its lanes are idle, so each env's image is built by a group of G = 192 / E lanes of
// the three non-helper waves (the env wave publishes its envs' views in LDS): lane e of wave 0 (the
// env's own) and the lanes of rank e + E, e + 2E, ... take 1/G of the channels each (their bit sinks
// merge at the shared words), the env's lane also the next-subgoal direction.  `want`: this lane's
// env needs an image.  Otherwise every env lane builds its own.  Called by every non-helper wave;
// with <= 32 envs it synchronises them once (the running sub_barrier target `bar`).
template <bool BIG>
__device__ __forceinline__ void group_obs(const DevCfg& c, const DevState& S, const EnvView& v, bool want,
                                          uint32_t* st, ObsInfo& oi, const Lds& L, int wave, int lane,
                                          uint32_t* ctr, uint32_t& bar, int np, int rank, uint32_t* vw,
                                          bool post = true) {
  const int vtid = wave * 64 + lane;
  const int E = L.envs;
  if (E <= 32) {
    if (wave == 0 && lane < E) {
      uint32_t* q = vw + lane * kViewDw;
      q[0] = (uint32_t)v.px;
      q[1] = (uint32_t)v.py;
      q[2] = v.sg;
      q[3] = v.phase;
      q[4] = (uint32_t)v.used;
      q[5] = (uint32_t)(v.used >> 32);
      q[6] = want ? 1u : 0u;
    }
    sub_barrier(ctr, bar += (uint32_t)np);
    STAMP(post ? 9 : 16);
    const int G = np * 64 / E, e = rank % E, sub = rank / E;
    if (sub >= G) return;
    const uint32_t* q = vw + e * kViewDw;
    if (!q[6]) return;
    const int C = c.n_channels, lo = sub * C / G, hi = (sub + 1) * C / G;
    if (lo == hi && sub != 0) return;
    EnvView ve{};
    ve.px = (int)q[0];
    ve.py = (int)q[1];
    ve.sg = q[2];
    ve.phase = q[3];
    ve.used = (uint64_t)q[4] | (uint64_t)q[5] << 32;
    STAMP(post ? 10 : 17);
    extern __shared__ uint32_t lds[];
    const Plan pl{reinterpret_cast<uint16_t*>(lds + e * L.plan_stride_dw)};
    build_obs<false, BIG, false, false>(c, S, pl, ve, st, (uint32_t)e * (uint32_t)c.obs_bytes, oi, nullptr, lo, hi, sub == 0,
                                 true);
    STAMP(post ? 11 : 18);
    return;
  }
  if (want) {
    extern __shared__ uint32_t lds[];
    const int slot = vtid;
    const Plan pl{reinterpret_cast<uint16_t*>(lds + slot * L.plan_stride_dw)};
    build_obs<false, BIG, false, false>(c, S, pl, v, st, (uint32_t)slot * (uint32_t)c.obs_bytes, oi, nullptr);
  }
}

// A reset's ring take: the head entry of env i's ring (slot qh, made for spawn counter k0) becomes its
// episode -- the tile plan into its HBM row and its LDS row, the obstacle streams of the episode, and
// {px | py << 16, start/goal word, path length | error << 16} returned (env_reset without the generation).
template <bool BIG>
__device__ __forceinline__ uint3 ring_take(const DevCfg& c, const DevState& S, const Lds& L, uint64_t i, uint32_t qh,
                                           uint32_t k0, uint32_t* plan_w, int pdw, int depth = kQueueDepth) {
  const uint4* q4 = reinterpret_cast<const uint4*>(S.qbuf + (i * (uint64_t)depth + qh) * (uint64_t)c.qrec_dw);
  uint4* dstp = reinterpret_cast<uint4*>(S.plan + i * (uint64_t)c.plan_stride);
  // all loads of the entry first: a load after a store to S.plan (which the compiler cannot
  // tell apart from the queue) would wait for the one before it, one HBM latency per 16 bytes
  const int nq = c.plan_dq;  // 16-byte words of the tile plan (<= 8 unless BIG)
  const uint4 meta = q4[nq];
  for (int k0q = 0; k0q < (BIG ? nq : 1); k0q += 8) {
    uint4 qw[8];
#pragma unroll
    for (int k = 0; k < 8; k++) qw[k] = q4[k0q + k < nq ? k0q + k : k0q];  // unconditional: registers, not scratch
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (k0q + k < nq) {
        if (!ABLATE(L, 32)) dstp[k0q + k] = qw[k];
        const uint32_t wv[4] = {qw[k].x, qw[k].y, qw[k].z, qw[k].w};
#pragma unroll
        for (int j = 0; j < 4; j++)
          if ((k0q + k) * 4 + j < pdw) plan_w[(k0q + k) * 4 + j] = wv[j];
      }
    }
  }
  if (!ABLATE(L, 32))
    for (int k = nq; k < c.plan_stride / 8; k++) dstp[k] = make_uint4(0u, 0u, 0u, 0u);  // the row's whole lines
  if (c.need_ice || c.need_broken || c.need_sand) {
    SeedPool sp = ss_pool(S.seed[i]);
    if (c.need_ice) stream_store_all(S.ice, i, ss_child(sp, k0 + 2u));
    if (c.need_broken) stream_store_all(S.broken, i, ss_child(sp, k0 + 3u));
    if (c.need_sand) stream_store_all(S.sand, i, ss_child(sp, k0 + 4u));
  }
  // the entry was generated for this episode (spawn counter k0): k_envq serves every request of a
  // launch in the next one and its ring holds two entries, k_envb refills every empty head before the
  // take, so it always is -- a mismatch is reported as a device error, never used
  const int e2 = (meta.w != queue_tag(k0) && !ABLATE(L, 1 | 16)) ? PGTG_E_DEVICE : -(int)(meta.z >> 16);
  return make_uint3(meta.x, meta.y, (meta.z & 0xffffu) | (uint32_t)(-e2) << 16);
}

template <bool BIG>
__global__ void __launch_bounds__(kBlock, 4) k_envq(const DevCfg* __restrict__ cfg, const Tables* __restrict__ gtab,
                                                    DevState S, const uint8_t* __restrict__ actions, PgtgOutputs out,
                                                    Lds L, uint32_t qsel) {
  extern __shared__ uint32_t lds[];
  const DevCfg& c = *cfg;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const uint64_t t_start = stagger_start(L, S);
  STAMP(0);  // (the env waves' is each block's start)
  STAMPR(2);  // (wall clock: every wave's start and end, slots 2 and 3 -- the launch's ramp and tail)
  const int env_waves = (L.envs + 63) / 64, gen_wave = env_waves;
  const bool env_wave = wave < env_waves;
  // refill requests: this launch's into list qsel & 3 (buffer qsel >> 2), the previous launch's from
  // list (qsel + 2) % 3 (the other buffer); the third list's counters are cleared for the next launch
  const uint32_t par = qsel >> 2;
  const uint64_t nblk = (S.n + (uint64_t)L.envs - 1) / (uint64_t)L.envs;
  const uint64_t cap = queue_req_cap(nblk, gridDim.x, L.envs);  // requests per workgroup and launch
  uint2* req_new = S.qreq + ((uint64_t)par * gridDim.x + blockIdx.x) * cap;
  const uint2* req_old = S.qreq + ((uint64_t)(par ^ 1u) * gridDim.x + blockIdx.x) * cap;
  // One round of blocks (every workgroup one block): a helper's time is on the launch's path, so a
  // workgroup lists at most kQueueLanes requests (one batch) and appends the rest to an overflow
  // list shared by the workgroups of its residue mod 8, whose helpers fill their spare lanes from it.
  const bool one_round = nblk <= gridDim.x;
  const uint32_t ox = blockIdx.x & 7u, set_new = qsel & 3u, set_old = (set_new + 2u) % 3u;
  const uint64_t ocap = ((gridDim.x + 7u) / 8u) * (uint64_t)L.envs;  // an overflow list's capacity
  // the helper's list length and first requests, issued before the tables are staged
  uint32_t cnt = 0;
  uint2 r0 = make_uint2(0u, 0u);
  if (wave == gen_wave) {
    cnt = S.qctr[(par ^ 1u) * gridDim.x + blockIdx.x];
    r0 = req_old[lane];  // (cap >= kQueueLanes: inside the list, used only below cnt)
  }
  if (blockIdx.x == 0 && tid < 8) S.qctr[kQctrOvfLen + ((set_new + 1u) % 3u) * 8u + tid] = 0u;  // (the launch after next's)
  const int pdw = L.plan_stride_dw;
  stage_tables(gtab, false);  // (the map queue runs without lane channels: no sTX reference here)
  uint32_t* st = lds + L.envs * (pdw + L.scratch_dw + L.traf_dw + L.hist_dw);
  uint8_t* sel = reinterpret_cast<uint8_t*>(st + L.stream_words);  // [kBlock]
  uint32_t* ctr = reinterpret_cast<uint32_t*>(sel + kBlock);  // sub_barrier counter
  uint32_t* lm = L.lm_words ? reinterpret_cast<uint32_t*>(sel + kBlock + 128) : nullptr;  // terminal lines
  uint32_t* vw = reinterpret_cast<uint32_t*>(sel + kBlock + 128) + L.lm_words;  // env views (<= 32 envs)
  uint32_t* qn = ctr + 1;  // this launch's requests so far
  uint32_t* nxt = ctr + 2;  // the next block
  // blocks after the first: taken from a counter (three, rotating: this launch's, the next one's
  // cleared here), one block ahead
  uint32_t* bctr = S.qctr + kQctrBlocks;
  if (blockIdx.x == 0 && tid == 0) bctr[((qsel & 3u) + 1u) % 3u] = 0u;
  if (tid == 0) {
    *ctr = 0u;
    *qn = 0u;
  }
  lds_barrier();  // tables, counters

  if (wave == gen_wave) {
    STAMP(1);
    // the helper: the previous launch's requests, kQueueLanes at a time, until none is left
    uint16_t* gplan = reinterpret_cast<uint16_t*>(lds + L.gen_off + lane * pdw);
    uint32_t made = 0, ovs = 0;  // maps generated, of them overflow requests
    if (!ABLATE(L, 1)) {
      // one round: this helper's share of its residue's overflow list -- as many as its spare lanes,
      // after those of the workgroups before it (a prefix sum over their list lengths, no atomics:
      // 128 helpers claiming from one counter waited 7 us for it); what outgrows every spare lane
      // follows in whole batches by workgroup order
      const uint2* ovf = S.qovf + ((uint64_t)(par ^ 1u) * 8u + ox) * ocap;
      uint32_t ob = 0, on = 0, olen = 0, tot = 0;
      const uint32_t nj = (gridDim.x - ox + 7u) / 8u, jme = blockIdx.x / 8u;
      if (one_round) {
        olen = S.qctr[kQctrOvfLen + set_old * 8u + ox];
        if (olen > 0) {
          uint32_t pre = 0;
          for (uint32_t j0 = 0; j0 < nj; j0 += kQueueLanes) {
            const uint32_t j = j0 + (uint32_t)lane;
            const uint32_t sp = j < nj ? kQueueLanes - min(S.qctr[(par ^ 1u) * gridDim.x + ox + 8u * j], (uint32_t)kQueueLanes) : 0u;
            pre += wave_sum(j < jme ? sp : 0u);
            tot += wave_sum(sp);
          }
          on = olen > pre ? min(olen - pre, kQueueLanes - min(cnt, (uint32_t)kQueueLanes)) : 0u;
          ob = pre;
        }
      }
      for (uint32_t base = 0;; base += kQueueLanes) {  // the workgroup's own requests (and the spare lanes')
        const uint32_t own = base < cnt ? min((uint32_t)kQueueLanes, cnt - base) : 0u;
        const uint32_t oth = base == 0 ? on : 0u;
        if (own + oth == 0) break;
        made += own + oth;
        ovs += oth;
        if ((uint32_t)lane < own + oth) {
          const uint2 r = (uint32_t)lane >= own ? ovf[ob + (lane - own)] : base == 0 ? r0 : req_old[base + lane];
          const uint64_t ie = r.x >> 1;
          gen_queue_entry<BIG>(c, S, ie, r.y, gplan, pdw, S.qbuf + (ie * kQueueDepth + (r.x & 1u)) * (uint64_t)c.qrec_dw,
                               ABLATE(L, 16), false);
        }
        if (base + kQueueLanes >= cnt) break;
      }
      for (uint64_t st0 = tot + (uint64_t)jme * kQueueLanes; st0 < olen; st0 += (uint64_t)nj * kQueueLanes) {
        const uint32_t m = (uint32_t)min((uint64_t)kQueueLanes, olen - st0);
        made += m;
        ovs += m;
        if ((uint32_t)lane < m) {
          const uint2 r = ovf[st0 + lane];
          const uint64_t ie = r.x >> 1;
          gen_queue_entry<BIG>(c, S, ie, r.y, gplan, pdw, S.qbuf + (ie * kQueueDepth + (r.x & 1u)) * (uint64_t)c.qrec_dw,
                               ABLATE(L, 16), false);
        }
      }
    }
    if (lane == 0 && made) atomicAdd(&S.counters[2], (unsigned long long)made);  // maps generated
    if (lane == 0 && ovs) atomicAdd(&S.counters[3], (unsigned long long)ovs);  // overflow requests served
    STAMP(7);
    STAMPR(3);
    return;
  }

  // ---- env and writer waves (all but the helper), block after block ----
  const int np = kBlock / 64 - 1;  // participating waves
  const int nthr = np * 64;
  uint32_t bar = 0;  // running sub_barrier target
  for (uint64_t blk = blockIdx.x; blk < nblk;) {
    STAMP(0);
    uint32_t got = 0xffffffffu;
    if (tid == 0 && nblk > gridDim.x && *qn + 2u * (uint32_t)L.envs <= cap) got = atomicAdd(&bctr[qsel & 3u], 1u);
    // the per-lane values derive from an opaque copy of the lane id, block by block: hoisted out of
    // the loop, they and what the compiler derives from them would hold registers through every
    // block (the env waves spilled at 128 VGPRs)
    int tid_o = tid;
    asm volatile("" : "+v"(tid_o));
    const int lane = tid_o & 63;
    const int rank = (wave < gen_wave ? wave : wave - 1) * 64 + lane;
    const int slot = tid_o;
    uint32_t* plan_w = lds + (env_wave ? slot : 0) * pdw;
    Plan pl{reinterpret_cast<uint16_t*>(plan_w)};
    const uint64_t env0 = blk * (uint64_t)L.envs;
    const int nb = (int)min((uint64_t)L.envs, S.n - env0);
    const uint64_t i = env0 + slot;
    const bool live = env_wave && slot < nb;
    EnvView v{};
    uint32_t qh = 0;
    int act = 0;
    if (live) {
      v = rec_load(S.rec, i);
      qh = S.qstate[i] & 1u;
      act = actions[i];  // issued with the staging loads, not on the step's chain
      stage_plan<BIG>(S.plan + i * (uint64_t)c.plan_stride, c.plan_dq, plan_w, pdw);
    }
    for (int k = rank; k < L.lm_words; k += nthr) lm[k] = 0u;
    sub_barrier(ctr, bar += (uint32_t)np);  // plans, line mask (and the last block's images written)
    STAMP(1);
    uint8_t my_sel = 0;
    int err = 0;
    if (live) {
      StepResult res{0.0, 0.0, 0u};
      bool occ_sat = false;
      TrafState ts{0, 0, 0, 0};
      err = env_step<false, BIG>(c, S, i, v, pl, act, res, nullptr, occ_sat, nullptr, ts, nullptr);
      STAMP(22);
      const bool done = (v.flags & (kFlagTerminated | kFlagTruncated)) != 0;
      if (out.reward) out.reward[i] = res.reward;
      if (out.cost) out.cost[i] = res.cost;
      if (out.terminated) out.terminated[i] = (v.flags & kFlagTerminated) ? 1 : 0;
      if (out.truncated) out.truncated[i] = (v.flags & kFlagTruncated) ? 1 : 0;
      if (out.braking) out.braking[i] = 0;
      my_sel = (done && c.autoreset && err == 0) ? 1 : 0;
      if (BIG && res.plan_dirty && !my_sel) store_plan_row(c, S, i, plan_w, pdw);  // used subgoals (kPlanUsed)
      if (lm && my_sel && out.final_obs) mark_lines(lm, out.final_obs + env0 * (uint64_t)c.obs_bytes, (uint32_t)slot, (uint32_t)c.obs_bytes);
      STAMP(23);
    }
    // the post-step image of every env (terminal for the finished ones)
    {
      ObsInfo oi;
      group_obs<BIG>(c, S, v, live, st, oi, L, wave, lane, ctr, bar, np, rank, vw);
      if (live) write_small_outputs(c, out, i, v, oi, my_sel == 1);
    }
    if (env_wave) sel[slot] = my_sel;
    const uint64_t rm = __ballot(my_sel == 1);
    if (env_wave && lane == 0 && rm) atomicAdd(&S.counters[1], (unsigned long long)__popcll(rm));
    STAMP(2);
    STAMP(28);
    sub_barrier(ctr, bar += (uint32_t)np);
    STAMP(29);
    if (out.final_obs && !ABLATE(L, 2))
      write_obs(out.final_obs + env0 * (uint64_t)c.obs_bytes, (uint32_t)nb, (uint32_t)c.obs_bytes, st, sel, rank, nthr, lm);
    STAMP(3);
    sub_barrier(ctr, bar += (uint32_t)np);  // terminal images written before they are rebuilt
    const bool reset_now = my_sel != 0;
    const uint32_t k0 = v.spawn;
    if (reset_now) {  // the ring's head becomes the episode (env_reset without the generation)
      const uint4* q4 = reinterpret_cast<const uint4*>(S.qbuf + (i * kQueueDepth + qh) * (uint64_t)c.qrec_dw);
      uint4* dstp = reinterpret_cast<uint4*>(S.plan + i * (uint64_t)c.plan_stride);
      // all loads of the entry first: a load after a store to S.plan (which the compiler cannot
      // tell apart from the queue) would wait for the one before it, one HBM latency per 16 bytes
      const int nq = c.plan_dq;  // 16-byte words of the tile plan (<= 8 unless BIG)
      const uint4 meta = q4[nq];
      for (int k0q = 0; k0q < (BIG ? nq : 1); k0q += 8) {
        uint4 qw[8];
#pragma unroll
        for (int k = 0; k < 8; k++) qw[k] = q4[k0q + k < nq ? k0q + k : k0q];  // unconditional: registers, not scratch
#pragma unroll
        for (int k = 0; k < 8; k++) {
          if (k0q + k < nq) {
            if (!ABLATE(L, 32)) dstp[k0q + k] = qw[k];
            const uint32_t wv[4] = {qw[k].x, qw[k].y, qw[k].z, qw[k].w};
#pragma unroll
            for (int j = 0; j < 4; j++)
              if ((k0q + k) * 4 + j < pdw) plan_w[(k0q + k) * 4 + j] = wv[j];
          }
        }
      }
      if (!ABLATE(L, 32))
        for (int k = nq; k < c.plan_stride / 8; k++) dstp[k] = make_uint4(0u, 0u, 0u, 0u);  // the row's whole lines
      if (c.need_ice || c.need_broken || c.need_sand) {
        SeedPool sp = ss_pool(S.seed[i]);
        if (c.need_ice) stream_store_all(S.ice, i, ss_child(sp, k0 + 2u));
        if (c.need_broken) stream_store_all(S.broken, i, ss_child(sp, k0 + 3u));
        if (c.need_sand) stream_store_all(S.sand, i, ss_child(sp, k0 + 4u));
      }
      v.spawn = k0 + 5u;
      v.sg = meta.y;
      v.used = 0;
      v.path_len = meta.z & 0xffffu;
      v.flags = 0;
      v.phase = 0;
      v.elapsed = 0;
      v.vx = v.vy = 0;
      v.px = (int)(int16_t)(meta.x & 0xffffu);
      v.py = (int)(int16_t)(meta.x >> 16);
      // the entry was generated for this episode (spawn counter k0): every launch serves all of the
      // previous launch's requests and the ring holds two entries, so it always is -- a mismatch is
      // reported as a device error, never used
      const int e2 = (meta.w != queue_tag(k0) && !ABLATE(L, 1 | 16)) ? PGTG_E_DEVICE : -(int)(meta.z >> 16);
      if (e2) err = e2;
      if (S.visited && e2 == 0) {
        uint32_t* vis = S.visited + i * (uint64_t)c.vis_words;
        for (int q2 = 0; q2 < c.vis_words; q2++) vis[q2] = 0;
        int b = (v.px + 2) * c.vis_pitch + (v.py + 2);
        vis[b >> 5] |= 1u << (b & 31);
      }
    }
    STAMP(4);
    // refill request: the next-but-one episode's map (spawn counter k0 + 10) into the slot just taken
    const uint64_t rb = __ballot(reset_now);
    if (rb) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(qn, (uint32_t)__popcll(rb));
      base = __builtin_amdgcn_readfirstlane(base);
      const uint32_t k = (uint32_t)__popcll(rb);
      // one round: list positions >= kQueueLanes go to the overflow list
      const uint32_t ovn = (one_round && base + k > (uint32_t)kQueueLanes) ? base + k - max(base, (uint32_t)kQueueLanes) : 0u;
      uint32_t obase = 0;
      if (ovn) {
        if (lane == 0) obase = atomicAdd(&S.qctr[kQctrOvfLen + set_new * 8u + ox], ovn);
        obase = __builtin_amdgcn_readfirstlane(obase);
      }
      if (reset_now) {
        const uint32_t p = base + (uint32_t)__popcll(rb & ((1ull << lane) - 1ull));
        const uint2 r = make_uint2((uint32_t)i << 1 | qh, k0 + 10u);
        if (one_round && p >= (uint32_t)kQueueLanes)
          S.qovf[((uint64_t)par * 8u + ox) * ocap + obase + (p - max(base, (uint32_t)kQueueLanes))] = r;
        else
          req_new[p] = r;
        S.qstate[i] = (uint8_t)(qh ^ 1u);  // (every env's byte instead: 403.3 vs 401.4 us)
      }
    }
    if (live) {
      rec_store(S.rec, i, v);
      S.err[i] = (uint8_t)(-err);
    }
    STAMP(5);
    {
      ObsInfo oi;
      group_obs<BIG>(c, S, v, reset_now, st, oi, L, wave, lane, ctr, bar, np, rank, vw, false);
      if (reset_now) write_small_outputs(c, out, i, v, oi, false);
    }
    if (tid == 0) *nxt = got;
    STAMP(30);
    sub_barrier(ctr, bar += (uint32_t)np);
    STAMP(31);
    if (tid == 0)  // (every request of the block is in)
      S.qctr[par * gridDim.x + blockIdx.x] = one_round ? min(*qn, (uint32_t)kQueueLanes) : *qn;
    const uint32_t g = *nxt;  // (written before the last barrier, rewritten after the next block's first)
    if (out.obs && !ABLATE(L, 4))
      write_obs(out.obs + env0 * (uint64_t)c.obs_bytes, (uint32_t)nb, (uint32_t)c.obs_bytes, st, nullptr, rank, nthr);
    if (tid == 0) atomicAdd(&S.counters[0], (unsigned long long)nb);
    if (blk == blockIdx.x) stagger_record(L, S, t_start);
    STAMP(6);
    blk = g == 0xffffffffu ? nblk : (uint64_t)gridDim.x + g;
  }  STAMPR(3);
}

// Step launch with the map queue for grids of at most two rounds of workgroups (k_envb: the map
// queue per block).  Each workgroup steps its own block once; its helper wave refills the block's
// rings from the ring states the env waves staged in LDS -- the heads of empty rings first (the env
// waves wait for those at one barrier), then the second and third entries of the rings that need
// them, at most kQueueLanes per launch (the rest wait for a later launch: a ring of three entries
// has the slack).  No request lists, no block counter, no overflow lists: at one or two rounds each
// helper's fill is on the launch's path, and these measured faster than k_envq's there (131 072 5x5
// envs: 71.7-73.4 against 78.6-80.8 us per launch, 262 144: 131.5-132.1 against 142.2-143.2 us,
// configs[1]'s 4 096 3x3 envs: 20.1 against 22.2 us; profiles/r06/s2/), while k_envq's persistent grid
// wins from four rounds on.  qstate = entries held | head slot << 2.
template <bool BIG>
__global__ void __launch_bounds__(kBlock, 4) k_envb(const DevCfg* __restrict__ cfg, const Tables* __restrict__ gtab,
                                                    DevState S, const uint8_t* __restrict__ actions, PgtgOutputs out,
                                                    Lds L) {
  extern __shared__ uint32_t lds[];
  const DevCfg& c = *cfg;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const uint64_t t_start = stagger_start(L, S);
  STAMP(0);
  STAMPR(2);  // (wall clock: every wave's start and end, slots 2 and 3)
  stage_tables(gtab, false);  // (the map queue runs without lane channels: no sTX reference here)
  const uint64_t env0 = (uint64_t)blockIdx.x * L.envs;
  const int nb = (int)min((uint64_t)L.envs, S.n - env0);
  const int env_waves = (L.envs + 63) / 64, gen_wave = env_waves;
#ifdef PGTG_TUNING
  if (wave != gen_wave) {  // (A/B) the env and writer waves ahead of the helper in issue arbitration
    if (L.prio == 1) __builtin_amdgcn_s_setprio(1);
    else if (L.prio == 2) __builtin_amdgcn_s_setprio(2);
    else if (L.prio == 3) __builtin_amdgcn_s_setprio(3);
  }
#endif
  // ring entries of levels 1.. regenerated per launch: one per helper lane, two with three env waves
  // (192 envs reset ~80 times per launch at configs[4]'s rate)
  const int qcap = env_waves > 2 ? 2 * kQueueLanes : kQueueLanes;
  const bool env_wave = wave < env_waves;
  const int slot = tid;
  const uint64_t i = env0 + slot;
  const bool live = env_wave && slot < nb;
  const int pdw = L.plan_stride_dw;
  uint32_t* plan_w = lds + (env_wave ? slot : 0) * pdw;
  uint32_t* xf = lds + L.envs * pdw;  // per env slot: spawn counter, ring state at launch start
  uint32_t* st = lds + L.envs * (pdw + L.scratch_dw + L.traf_dw + L.hist_dw);
  uint8_t* sel = reinterpret_cast<uint8_t*>(st + L.stream_words);  // [kBlock]
  uint64_t* fm = reinterpret_cast<uint64_t*>(sel + kBlock);  // [level][env wave]: envs refilled at ring level
  uint32_t* ctr = reinterpret_cast<uint32_t*>(fm + 3 * kBlockDepth);  // sub_barrier counter
  uint32_t* lm = L.lm_words ? reinterpret_cast<uint32_t*>(sel + kBlock + 128) : nullptr;  // terminal lines
  uint32_t* vw = reinterpret_cast<uint32_t*>(sel + kBlock + 128) + L.lm_words;  // env views (<= 32 envs)
  Plan pl{reinterpret_cast<uint16_t*>(plan_w)};

  EnvView v{};
  uint32_t qs = 0;
  int act = 0;
  if (live) {
    v = rec_load(S.rec, i);
    qs = S.qstate[i];
    act = actions[i];  // issued with the staging loads, not on the step's chain
    stage_plan<BIG>(S.plan + i * (uint64_t)c.plan_stride, c.plan_dq, plan_w, pdw);
    xf[slot * L.scratch_dw] = v.spawn;
    xf[slot * L.scratch_dw + 1] = qs;
  }
  const uint32_t qn = qs & 3u, qh = (qs >> 2) & 3u;
  if (env_wave) {  // refills: ring level l (0 = head) for the envs holding <= l maps
#pragma unroll
    for (int l = 0; l < kBlockDepth; l++) {
      const uint64_t m = __ballot(live && qn <= (uint32_t)l);
      if (lane == 0) fm[l * 3 + wave] = m;
    }
  }
  if (tid == 0) *ctr = 0u;
  for (int k = tid; k < L.lm_words; k += kBlock) lm[k] = 0u;
  lds_barrier();  // tables, plans, refill masks, counter, line mask
  STAMP(1);
  // refills: the heads of empty rings (level 0, all of them), then levels 1.. in order (the first
  // kQueueLanes this launch; the rest wait for a later launch)
  int F[kBlockDepth];
#pragma unroll
  for (int l = 0; l < kBlockDepth; l++) {
    F[l] = 0;
    for (int w = 0; w < env_waves; w++) F[l] += __popcll(fm[l * 3 + w]);
  }
  const bool any_empty = F[0] != 0;
#ifdef PGTG_STAMPS
  if ((threadIdx.x & 63) == 0)  // diagnostic: empty rings and level-1/2 refills wanted in this workgroup
    g_stamps[((blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * 32 + 12) & ((1 << 21) - 1)] =
        (unsigned long long)F[0] | (unsigned long long)F[1] << 16 | (unsigned long long)F[2] << 32;
#endif

  if (wave == gen_wave) {
    uint16_t* gplan = reinterpret_cast<uint16_t*>(lds + L.gen_off + lane * pdw);
    auto refill = [&](int k, int l) {
      int e = 0, pre = 0;
      for (int w = 0; w < env_waves; w++) {
        const uint64_t m = fm[l * 3 + w];
        const int cw = __popcll(m);
        if (k >= pre && k < pre + cw) e = w * 64 + select64(m, k - pre);
        pre += cw;
      }
      const uint64_t ie = env0 + e;
      const uint32_t qe = xf[e * L.scratch_dw + 1];
      const uint32_t rslot = (((qe >> 2) & 3u) + (uint32_t)l) % (uint32_t)kBlockDepth;
      gen_queue_entry<BIG>(c, S, ie, xf[e * L.scratch_dw] + 5u * (uint32_t)l, gplan, pdw,
                      S.qbuf + (ie * kBlockDepth + rslot) * (uint64_t)c.qrec_dw, ABLATE(L, 16), !ABLATE(L, 512));
    };
    if (ABLATE(L, 1)) {
      if (any_empty) __syncthreads();
      return;
    }
    for (int k = lane; k < F[0]; k += kQueueLanes) refill(k, 0);  // every empty ring's head
    if (any_empty) __syncthreads();  // head refills visible to the other waves
    for (int k0 = lane; k0 < qcap; k0 += kQueueLanes) {  // levels 1.. in list order, up to qcap entries
      int k = k0, l = 1;
      while (l < kBlockDepth && k >= F[l]) {
        k -= F[l];
        l++;
      }
      if (l < kBlockDepth) refill(k, l);
    }
    if (lane == 0) {  // maps generated (S.counters[2]): the heads, then up to qcap for levels 1..
      int rest = 0;
      for (int l = 1; l < kBlockDepth; l++) rest += F[l];
      atomicAdd(&S.counters[2], (unsigned long long)(F[0] + min(rest, qcap)));
    }
    STAMP(7);
    STAMPR(3);
    return;
  }

  // ---- env and writer waves (all but the refill wave) ----
  const int np = kBlock / 64 - 1;                            // participating waves
  const int rank = (wave < gen_wave ? wave : wave - 1) * 64 + lane, nthr = np * 64;
  uint32_t bar = 0;  // running sub_barrier target
  uint8_t my_sel = 0;
  int err = 0;
  if (live) {
    StepResult res{0.0, 0.0, 0u};
    bool occ_sat = false;
    TrafState ts{0, 0, 0, 0};
    err = env_step<false, BIG>(c, S, i, v, pl, act, res, nullptr, occ_sat, nullptr, ts, nullptr);
    STAMP(22);
    const bool done = (v.flags & (kFlagTerminated | kFlagTruncated)) != 0;
    if (out.reward) out.reward[i] = res.reward;
    if (out.cost) out.cost[i] = res.cost;
    if (out.terminated) out.terminated[i] = (v.flags & kFlagTerminated) ? 1 : 0;
    if (out.truncated) out.truncated[i] = (v.flags & kFlagTruncated) ? 1 : 0;
    if (out.braking) out.braking[i] = 0;
    my_sel = (done && c.autoreset && err == 0) ? 1 : 0;
    if (BIG && res.plan_dirty && !my_sel) store_plan_row(c, S, i, plan_w, pdw);  // used subgoals (kPlanUsed)
    if (lm && my_sel && out.final_obs) mark_lines(lm, out.final_obs + env0 * (uint64_t)c.obs_bytes, (uint32_t)slot, (uint32_t)c.obs_bytes);
    STAMP(23);
  }
  // the post-step image of every env (terminal for the finished ones)
  {
    ObsInfo oi;
    group_obs<BIG>(c, S, v, live, st, oi, L, wave, lane, ctr, bar, np, rank, vw);
    if (live) write_small_outputs(c, out, i, v, oi, my_sel == 1);
  }
  if (env_wave) sel[slot] = my_sel;
  const uint64_t rm = __ballot(my_sel == 1);
  if (env_wave && lane == 0 && rm) atomicAdd(&S.counters[1], (unsigned long long)__popcll(rm));
  STAMP(2);
  STAMP(28);
  sub_barrier(ctr, bar += (uint32_t)np);
  STAMP(29);
  if (out.final_obs && !ABLATE(L, 2))
    write_obs(out.final_obs + env0 * (uint64_t)c.obs_bytes, (uint32_t)nb, (uint32_t)c.obs_bytes, st,
              ABLATE(L, 128) ? nullptr : sel, rank, nthr, ABLATE(L, 128) ? nullptr : lm);  // (A/B: every line)
  STAMP(3);
  sub_barrier(ctr, bar += (uint32_t)np);  // terminal images written before they are rebuilt
  if (any_empty) __syncthreads();  // the head refills
  const bool reset_now = my_sel != 0;
  if (reset_now) {  // the ring's head becomes the episode (env_reset without the generation)
    const uint32_t k0 = v.spawn;
    const uint3 tk = ring_take<BIG>(c, S, L, i, qh, k0, plan_w, pdw, kBlockDepth);
    v.spawn = k0 + 5u;
    v.sg = tk.y;
    v.used = 0;
    v.path_len = tk.z & 0xffffu;
    v.flags = 0;
    v.phase = 0;
    v.elapsed = 0;
    v.vx = v.vy = 0;
    v.px = (int)(int16_t)(tk.x & 0xffffu);
    v.py = (int)(int16_t)(tk.x >> 16);
    const int e2 = -(int)(tk.z >> 16);
    if (e2) err = e2;
    if (S.visited && e2 == 0) {
      uint32_t* vis = S.visited + i * (uint64_t)c.vis_words;
      for (int q2 = 0; q2 < c.vis_words; q2++) vis[q2] = 0;
      int b = (v.px + 2) * c.vis_pitch + (v.py + 2);
      vis[b >> 5] |= 1u << (b & 31);
    }
  }
  STAMP(4);
  if (live) {
    rec_store(S.rec, i, v);
    S.err[i] = (uint8_t)(-err);
    // ring entries after this launch: the refills served (same list order as the refill wave)
    // minus the head a reset took
    uint32_t have = qn == 0u ? 1u : qn;
    int base = 0;  // list index of the first item of the level
#pragma unroll
    for (int l = 1; l < kBlockDepth; l++) {
      int pre = 0;
      for (int w = 0; w < wave; w++) pre += __popcll(fm[l * 3 + w]);
      if (qn <= (uint32_t)l && base + pre + __popcll(fm[l * 3 + wave] & ((1ull << lane) - 1ull)) < qcap) have++;
      base += F[l];
    }
    const uint32_t nq = reset_now ? have - 1u : have;  // have >= 1: every head is refilled
    const uint32_t nh = reset_now ? (qh + 1u) % (uint32_t)kBlockDepth : qh;
    S.qstate[i] = (uint8_t)(nq | nh << 2);
  }
  STAMP(5);
  {
    ObsInfo oi;
    group_obs<BIG>(c, S, v, reset_now, st, oi, L, wave, lane, ctr, bar, np, rank, vw, false);
    if (reset_now) write_small_outputs(c, out, i, v, oi, false);
  }
  STAMP(30);
  sub_barrier(ctr, bar += (uint32_t)np);
  STAMP(31);
  if (out.obs && !ABLATE(L, 4))
    write_obs(out.obs + env0 * (uint64_t)c.obs_bytes, (uint32_t)nb, (uint32_t)c.obs_bytes, st, nullptr, rank, nthr);
  if (tid == 0) atomicAdd(&S.counters[0], (unsigned long long)nb);
  stagger_record(L, S, t_start);
  STAMP(6);
  STAMPR(3);
}


// Fill every env's map ring: after a reset launch (whose k_env generated the current episodes' maps
// and marked the reset envs' rings stale), a state dump (the requests still pending) or a change of
// step kernel.  One lane per env checks both entries' spawn tags against the env's next two episodes
// (spawn counters s and s + 5, the head first) and generates the ones that do not match -- the maps
// k_envq's helpers would generate -- so that the step launches start with full rings.  The entries
// are a function of (seed, spawn counter) alone: results are unchanged.
template <bool BIG>
__global__ void __launch_bounds__(kBlock) k_qfill(const DevCfg* __restrict__ cfg, const Tables* __restrict__ gtab,
                                                  DevState S, int pdw) {
  extern __shared__ uint32_t lds[];
  const DevCfg& c = *cfg;
  stage_tables(gtab, false);
  lds_barrier();
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  uint32_t made = 0;
  if (i < S.n) {
    const uint32_t qs = S.qstate[i];
    const bool stale = (qs & kQueueStale) != 0;
    const uint32_t qh = stale ? 0u : (qs & 1u);
    const uint32_t spawn = S.rec[i].b.y;  // EnvRec w5
    const int tag_w = c.plan_dq * 4 + 3;
    uint16_t* plan = reinterpret_cast<uint16_t*>(lds + threadIdx.x * pdw);
    for (uint32_t l = 0; l < (uint32_t)kQueueDepth; l++) {
      uint32_t* dst = S.qbuf + (i * kQueueDepth + (qh ^ l)) * (uint64_t)c.qrec_dw;
      if (stale || dst[tag_w] != queue_tag(spawn + 5u * l)) {
        gen_queue_entry<BIG>(c, S, i, spawn + 5u * l, plan, pdw, dst);
        made++;
      }
    }
    if (stale) S.qstate[i] = 0;
  }
  // maps generated (S.counters[2]): one atomic per wave
  const uint32_t wsum = (uint32_t)__popcll(__ballot(made & 1u)) + 2u * (uint32_t)__popcll(__ballot(made & 2u));
  if ((threadIdx.x & 63) == 0 && wsum) atomicAdd(&S.counters[2], (unsigned long long)wsum);
}

// k_qfill for k_envb's rings (three entries; qstate = held | head << 2, kQueueStale: none held): the
// missing entries of every ring, levels held .. 2, the maps k_envb's helpers would generate.
template <bool BIG>
__global__ void __launch_bounds__(kBlock) k_qfill_b(const DevCfg* __restrict__ cfg, const Tables* __restrict__ gtab,
                                                    DevState S, int pdw) {
  extern __shared__ uint32_t lds[];
  const DevCfg& c = *cfg;
  stage_tables(gtab, false);
  lds_barrier();
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  uint32_t made = 0;
  if (i < S.n) {
    const uint32_t qs = S.qstate[i];
    const uint32_t qn = (qs & kQueueStale) ? 0u : (qs & 3u), qh = (qs & kQueueStale) ? 0u : ((qs >> 2) & 3u);
    if (qn < (uint32_t)kBlockDepth) {
      const uint32_t spawn = S.rec[i].b.y;  // EnvRec w5
      uint16_t* plan = reinterpret_cast<uint16_t*>(lds + threadIdx.x * pdw);
      for (uint32_t l = qn; l < (uint32_t)kBlockDepth; l++)
        gen_queue_entry<BIG>(c, S, i, spawn + 5u * l, plan, pdw,
                             S.qbuf + (i * kBlockDepth + (qh + l) % (uint32_t)kBlockDepth) * (uint64_t)c.qrec_dw);
      S.qstate[i] = (uint8_t)((uint32_t)kBlockDepth | qh << 2);
      made = (uint32_t)kBlockDepth - qn;
    }
  }
  // maps generated (S.counters[2]): one atomic per wave
  const uint32_t wsum = (uint32_t)__popcll(__ballot(made & 1u)) + 2u * (uint32_t)__popcll(__ballot(made & 2u));
  if ((threadIdx.x & 63) == 0 && wsum) atomicAdd(&S.counters[2], (unsigned long long)wsum);
}

#ifdef PGTG_STAMPS
__global__ void __launch_bounds__(kBlock) k_gen_bench(const DevCfg* __restrict__ cfg, const Tables* __restrict__ gtab,
                                                      DevState S, int reps, int active, int pdw) {
  extern __shared__ uint32_t lds[];
  const DevCfg& c = *cfg;
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(gtab);
    uint32_t* dstt = reinterpret_cast<uint32_t*>(&sT);
    for (int k = threadIdx.x; k < (int)(sizeof(TablesHead) / 4); k += blockDim.x) dstt[k] = src[k];
  }
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  uint16_t* plan = reinterpret_cast<uint16_t*>(lds + threadIdx.x * pdw);
  unsigned long long tg = 0, tc = 0;
  uint32_t chk = 0;
  if ((threadIdx.x & 63) < active && i < S.n) {
    SeedPool sp = ss_pool(S.seed[i]);
    for (int r = 0; r < reps; r++) {
      Pcg g = ss_child(sp, 5u * (uint32_t)r);
      int st_t, st_d, gl_t, gl_d;
      const unsigned long long t0 = __builtin_amdgcn_s_memtime();
      uint64_t ix[4];
      generate_map<false>(c, sT.epk, g, plan, st_t, st_d, gl_t, gl_d, ix);
      const unsigned long long t1 = __builtin_amdgcn_s_memtime();
      const int len = compile_generated<false>(c, plan, st_t, gl_t, ix);
      const unsigned long long t2 = __builtin_amdgcn_s_memtime();
      tg += t1 - t0;
      tc += t2 - t1;
      chk += (uint32_t)len + plan[st_t];
    }
  }
  const uint64_t wv = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0) {
    g_stamps[(wv * 32 + 0) & ((1 << 21) - 1)] = tg;
    g_stamps[(wv * 32 + 1) & ((1 << 21) - 1)] = tc;
  }
  if (chk == 0xdeadbeefu) S.err[i] = 1;  // keeps the work alive
}
#endif

// Initial traffic of the envs k_env reset in this launch (its work list) with the reset scratch in
// LDS; the observation k_env wrote for them gets the new cars' squares (traffic channel only: the
// agent's tile window from the group's CR, other windows from the square list).  One workgroup per CU, and
// the list is spread evenly over all of their waves: a wave's time is its envs' serial chain whatever
// the number of active lanes, so the envs per wave are levelled first (`e`, at most `cap_w` in LDS
// at once, in rounds beyond that), then the wave's 64 lanes are shared out: 4 per env up to 16
// envs, 3 up to 21, 2 up to 32 (traffic_reset splits the sweep and the square lookup over them).
__global__ void __launch_bounds__(kBlock) k_traffic(const DevCfg* __restrict__ cfg, const Tables* __restrict__ gtab,
                                                    DevState S, PgtgOutputs out, uint32_t tr_slot, int plan_dw,
                                                    int rs_dw, int cap_w) {
  extern __shared__ uint32_t lds[];
  STAMP(27);  // (k_traffic's wave start and end: slots 27 and 24, after k_env's last use of them)
  STAMPR(1);
  const DevCfg& c = *cfg;
  const uint32_t n = S.tr_count[tr_slot];
  const uint32_t W = gridDim.x * (kBlock / 64);  // waves of the grid
  const uint32_t rounds = (n + W * (uint32_t)cap_w - 1) / (W * (uint32_t)cap_w);
  if (rounds == 0) return;
  const uint32_t e = (n + W * rounds - 1) / (W * rounds);  // envs per wave and round, <= cap_w
  if ((uint64_t)blockIdx.x * (kBlock / 64) * e >= n) return;  // whole workgroup idle
  // lanes per env: all a wave has for its e envs (<= kMaxGroup: the per-lane stretches of the sweep,
  // the draws and the lookups stop paying once they are a few items long)
  const int g = min(kMaxGroup, 64 / (int)e);
  const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63u);
  const int slot = lane / g, sub = lane - slot * g;
  stage_tables(gtab, true);
  __syncthreads();
  STAMP(25);
#ifdef PGTG_STAMPS
  if ((threadIdx.x & 63) == 0)  // the launch's shape (last launch): list length, rounds, envs per wave, capacity
    g_stamps[((blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * 32 + 15) & ((1 << 21) - 1)] =
        (unsigned long long)n | (unsigned long long)rounds << 32 | (unsigned long long)e << 40 | (unsigned long long)cap_w << 48;
#endif
  if ((uint32_t)slot >= e) return;
  const int ls = wave * cap_w + slot;  // LDS slot of the env
  uint32_t* plan_w = lds + ls * plan_dw;
  uint8_t* rs = reinterpret_cast<uint8_t*>(lds + (kBlock / 64) * cap_w * plan_dw + ls * rs_dw);
  for (uint32_t r = 0; r < rounds; r++) {
    const uint32_t j = (r * W + blockIdx.x * (kBlock / 64) + (uint32_t)wave) * e + (uint32_t)slot;
    if (j >= n) break;
    const uint64_t i = S.tr_list[j];
    if (c.nt > kSmallTiles) stage_plan<true>(S.plan + i * (uint64_t)c.plan_stride, c.plan_dq, plan_w, plan_dw);
    else stage_plan<false>(S.plan + i * (uint64_t)c.plan_stride, c.plan_dq, plan_w, plan_dw);
    Plan pl{reinterpret_cast<uint16_t*>(plan_w)};
    const EnvView v = rec_load(S.rec, i);
    const int pix = min(max(0, v.px), c.W - 1), piy = min(max(0, v.py), c.H - 1);
    const int at = (piy / kTile) * c.tw + pix / kTile;
    Pcg cr = stream_load(S.car, i);
    TrafState ts{0, 0, 0, 0};
    uint32_t CR[3] = {0u, 0u, 0u};
    const int err = traffic_reset(c, S, i, pl, cr, rs, ts, at, CR, sub, g);
    const int q0 = lane - sub;  // (traffic_reset's result is lane 0's)
    const int err0 = __shfl(err, q0), k0 = __shfl((int)ts.n_cars, q0);
    if (err0 == 0) {
      store_initial_counters(c, S, i, pl, rs, k0, sub, g);
      if (!c.obs_fast && c.traffic_ch >= 0 && out.obs && k0 > 0) {
        // generic windows (sliding, lane channels): k_env built this observation without cars; the
        // traffic channel -- the only one cars change -- gets the new cars' squares inside the window
        // (the group's lanes take every g-th car of the square list traffic_reset left in rs)
        const int win = c.win;
        const int x0 = c.sliding ? v.px - c.ss : (pix / kTile) * kTile;
        const int y0 = c.sliding ? v.py - c.ss : (piy / kTile) * kTile;
        const uint16_t* sqs = reinterpret_cast<const uint16_t*>(rs);
        uint8_t* o = out.obs + i * (uint64_t)c.obs_bytes + (uint64_t)c.traffic_ch * (uint64_t)(win * win);
        for (int m = sub; m < k0; m += g) {
          const uint32_t code = sqs[m];
          const int a = (int)(code & 255u) - x0, b = (int)(code >> 8) - y0;
          if (a >= 0 && a < win && b >= 0 && b < win) o[a * win + b] = 1;
        }
      }
    }
    if (sub == 0) {
      stream_store_state(S.car, i, cr);
      S.traf[i] = make_uint4(ts.n_cars | ts.n_spawners << 16, ts.next_id, ts.tail, err == 0 ? kTrafOccValid | kTrafFresh : 0u);
      if (err) S.err[i] = (uint8_t)(-err);
      if (c.obs_fast && c.traffic_ch >= 0 && out.obs) {
        // the tile window's traffic channel: k_env wrote it with no cars; set the car squares
        uint8_t* o = out.obs + i * (uint64_t)c.obs_bytes + (uint64_t)c.traffic_ch * 81u;
#pragma unroll
        for (int k = 0; k < 3; k++) {
          uint32_t m = CR[k];
          while (m) {
            const int b = __ffs((int)m) - 1;
            m &= m - 1u;
            o[k * 32 + b] = 1;
          }
        }
      }
    }
    wave_lds_sync();  // the group's scratch is reused by the next round
  }
  STAMP(24);
}

// Feature words of every square of env i's map (introspection: get_info, tests); one workgroup.
__global__ void __launch_bounds__(kBlock) k_squares(const DevCfg* __restrict__ cfg, const Tables* __restrict__ gtab,
                                                    DevState S, uint64_t i, uint64_t* __restrict__ words) {
  __shared__ uint16_t plan_s[kMaxTiles];
  const DevCfg& c = *cfg;
  const int tid = threadIdx.x;
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(gtab);
    uint32_t* dstt = reinterpret_cast<uint32_t*>(&sT);
    for (int k = tid; k < (int)(sizeof(TablesHead) / 4); k += blockDim.x) dstt[k] = src[k];
    uint32_t* dstx = reinterpret_cast<uint32_t*>(&sTX);
    for (int k = tid; k < (int)(sizeof(TablesTail) / 4); k += blockDim.x) dstx[k] = src[kTabHead / 4 + k];
    for (int t = tid; t < c.nt; t += blockDim.x) plan_s[t] = S.plan[i * (uint64_t)c.plan_stride + t];
  }
  __syncthreads();
  const EnvView v = rec_load(S.rec, i);
  const Plan pl{plan_s};
  for (int q = tid; q < c.W * c.H; q += blockDim.x) {
    const int x = q / c.H, y = q - x * c.H;
    const uint32_t f = c.nt > kSmallTiles ? square_flags<true>(c, pl, v, x, y) : square_flags<false>(c, pl, v, x, y);
    uint64_t w = square_lanes(c, pl, x, y);
    if (f & SQ_WALL) w |= 1ull << 32;
    if (square_spawner(c, pl, x, y)) w |= 1ull << 37;
    if (f & SQ_START) w |= 1ull << 38;
    if (f & SQ_SUBGOAL) w |= 1ull << 39;
    if (f & SQ_USED) w |= 1ull << 40;
    if (f & SQ_FINAL) w |= 1ull << 41;
    if (f & SQ_ICE) w |= 1ull << 42;
    if (f & SQ_BROKEN) w |= 1ull << 43;
    if (f & SQ_SAND) w |= 1ull << 44;
    if (f & SQ_TLIGHT) w |= 1ull << 45;
    words[q] = w;
  }
}

__global__ void k_random_actions(uint8_t* a, uint64_t n, uint64_t seed, uint64_t t, uint64_t offset) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // splitmix64 of (seed, t, global env index) -> Lemire multiply-shift to [0, 9)
  const uint64_t g = i + offset;
  uint64_t z = seed ^ (t * 0x9E3779B97F4A7C15ull) ^ (g * 0xD1B54A32D192ED03ull);
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  a[i] = (uint8_t)(((z >> 32) * 9ull) >> 32);
}

// Stream copy: the measured HBM denominator of the roofline (pgtg_measure_hbm).  16 B per lane,
// U independent loads in flight per lane, grid-stride (a grid covering the buffer copies it in one
// pass); NT: nontemporal loads and stores (streamed data bypasses the caches' retention).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <int U, bool NT>
__global__ void __launch_bounds__(256) k_hbm_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; b < n16; b += stride) {
    u32x4 r[U];
#pragma unroll
    for (int j = 0; j < U; j++) {
      const uint64_t k = b + j * 256 < n16 ? b + j * 256 : b;
      r[j] = NT ? __builtin_nontemporal_load(src + k) : src[k];
    }
#pragma unroll
    for (int j = 0; j < U; j++)
      if (b + j * 256 < n16) {
        if (NT) __builtin_nontemporal_store(r[j], dst + b + j * 256);
        else dst[b + j * 256] = r[j];
      }
  }
}

// Per-env digest term of the car list (pgtg_amd/digest.py car_term, oracle dg_cars): the cars in
// list order (slot order, empty slots skipped), coalesced slot rows.  Test/parity infrastructure.
__device__ __forceinline__ uint64_t dg_w(uint64_t j) {
  uint64_t z = j + 1 + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ void __launch_bounds__(256) k_car_digest(DevState S, uint64_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S.n) return;
  constexpr uint64_t CB = 1ull << 40;
  const uint4 t = S.traf[i];
  const CarSlots cs(S, i);
  const bool fresh = (t.w & kTrafFresh) != 0u;
  const gu32* fb = fresh_block(S, i);
  uint64_t d = (uint64_t)(t.x & 0xffffu) * dg_w(CB), j = 0;
  for (int k = 0; k < (int)t.z; k++) {
    const uint32_t w0 = fresh ? fb[k] : cs.w0[cs.at(k)];
    if (w0 & kCarEmpty) continue;
    const uint32_t id = fresh ? (uint32_t)k : cs.id[cs.at(k)];
    const uint64_t pk = (uint64_t)id | (uint64_t)(w0 & 255u) << 32 | (uint64_t)((w0 >> 8) & 255u) << 40 |
                        (uint64_t)((w0 >> 16) & 31u) << 48 | (uint64_t)((w0 >> 21) & 7u) << 53 |
                        (uint64_t)((w0 >> 24) & 3u) << 56;
    const uint32_t w1 = fresh ? 0u : cs.w1[cs.at(k)];
    d += (pk + 1) * dg_w(CB + 1 + 2 * j) + (uint64_t)w1 * dg_w(CB + 2 + 2 * j);
    j++;
  }
  out[i] = d;
}

// FlattenObservation rows (pgtg/train.py:40 wraps the env in gymnasium's FlattenObservation, whose
// flatten of the Dict space of environment.py:415-441 orders the keys by name): per env
//   map channels in name order (win*win each, [x][y]) | next-subgoal one-hot at d + 1 (9, with
//   use_next_subgoal_direction) | position one-hot of x (9) and of y (9) | velocity (2)
// as float32 or int8 (every value is a 0/1 entry or a velocity), from the observation the step kernels
// just wrote.  The N x D values are one flat array: a thread writes 16 consecutive bytes of it (4
// float32 or 16 int8 values; rows need not be aligned), reading the obs bytes they come from.  `final`:
// the terminal observations, written only on the rows of envs that finished this step.
struct FlatArgs {
  const uint8_t* obs;
  const int32_t* pos;
  const int32_t* vel;
  const int32_t* nsd;
  const uint8_t* term;
  const uint8_t* trunc;
  void* dst;
  // the SB3 path's per-env scalars, written by the observation pass when bound (pgtg_set_flat_scalars):
  // the reward as float32, done = terminated | truncated, and truncated-but-not-terminated
  const double* rew;
  float* rew32;
  uint8_t* dones;
  uint8_t* tonly;
  // the terminal observation's set (final == 2: both passes in one launch)
  const uint8_t* fobs;
  const int32_t* fpos;
  const int32_t* fvel;
  const int32_t* fnsd;
  void* fdst;
  uint64_t n;
  int32_t D, OB, w2, cw2, nsd_on, final;  // final: 0 the observation rows, 1 the terminal rows, 2 both
  uint8_t order[PGTG_MAX_CHANNELS];  // channel (in the observation) of the k-th name-sorted key
};
// One workgroup takes K consecutive rows (K = ceil(N / G) <= 256 for the grid's G workgroups): it lists
// the rows to write (every row, or the finished envs' for the terminal rows) and its waves write them,
// a row per wave.  A thread per 16 output bytes of the whole array,
// the first version, spent its time in a 64-bit division and in launching 18 M threads, most of which
// had nothing to do on the terminal pass (166 us per pass at 65 536 envs, profiles/r06/s8).
template <typename T>
__device__ __forceinline__ T flat_tail(const FlatArgs& a, int k, int nsdv, int px, int py, int vx, int vy) {
  if (a.nsd_on) {
    if (k < 9) return (T)(k == nsdv ? 1 : 0);
    k -= 9;
  }
  if (k < 9) return (T)(k == px ? 1 : 0);
  if (k < 18) return (T)(k - 9 == py ? 1 : 0);
  return (T)(k == 18 ? vx : vy);
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kFlatU = 18;  // values per lane in one pass of a row: rows of up to 18 x 64 = 1 152 in one pass
// a wave-uniform pointer the compiler can see is uniform (its halves through readfirstlane), so that a
// buffer descriptor built from it sits in scalar registers without a per-access waterfall loop
__device__ __forceinline__ void* uniform_ptr(const void* p) {
  const uint64_t u = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return (void*)(uintptr_t)((uint64_t)hi << 32 | lo);
}
__device__ __forceinline__ void flat_store(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, 0);
}
__device__ __forceinline__ void flat_store(__amdgpu_buffer_rsrc_t r, uint32_t off, int8_t v) {
  __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, r, off, 0, 0);
}
template <typename T, int V>
__device__ __forceinline__ void flat_store_v(__amdgpu_buffer_rsrc_t r, uint32_t off, const T (&f)[V]) {
  if constexpr (V == 1) {
    flat_store(r, off, f[0]);
  } else {
    static_assert(V == 2 && sizeof(T) == 4, "pairs of float32 only");
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 x = {__builtin_bit_cast(uint32_t, f[0]), __builtin_bit_cast(uint32_t, f[1])};
    __builtin_amdgcn_raw_buffer_store_b64(x, r, off, 0, 0);
  }
}
// ONE: rows of at most kFlatU x 64 values (one pass per row, software-pipelined); otherwise rows in
// passes of kFlatU x 64 values
template <typename T, bool ONE, int V>
__global__ void __launch_bounds__(256, 6) k_flatten(FlatArgs a) {
  // obs byte offset of the row's first kFlatU x 64 values (channels in name order), built once
  __shared__ uint32_t offs[kFlatU * 64];
  __shared__ uint32_t rows[512];  // t (observation row) or 256 + t (terminal row)
  __shared__ uint32_t nrows;
  const int t = threadIdx.x;
  const uint32_t D = (uint32_t)a.D, w2 = (uint32_t)a.w2, cw2 = (uint32_t)a.cw2;
  for (uint32_t j = t; j < (uint32_t)(kFlatU * 64); j += 256) {
    const uint32_t slot = j < cw2 ? j / w2 : 0u;
    offs[j] = j < cw2 ? (uint32_t)a.order[slot] * w2 + (j - slot * w2) : 0u;
  }
  if (t == 0) nrows = 0u;
  __syncthreads();
  // this workgroup's rows: K consecutive envs (coalesced flag reads and scalar writes, contiguous rows)
  const uint64_t K = (a.n + gridDim.x - 1) / gridDim.x;  // <= 256 (launch_flatten)
  const uint64_t e = (uint64_t)blockIdx.x * K + (uint64_t)t;
  const bool valid = (uint64_t)t < K && e < a.n;
  const bool done = valid && a.final != 0 && (a.term[e] | a.trunc[e]) != 0;
  if (valid && a.final != 1 && a.dones) {
    const uint8_t te = a.term[e], tr = a.trunc[e];
    a.dones[e] = (uint8_t)((te | tr) != 0);
    a.tonly[e] = (uint8_t)(tr != 0 && te == 0);
    a.rew32[e] = (float)a.rew[e];
  }
#pragma unroll
  for (int f = 0; f < 2; f++) {  // the observation rows, then the terminal rows
    const bool keep = f == 0 ? (valid && a.final != 1) : done;
    const uint64_t m = __ballot(keep);
    if (m) {
      uint32_t base = 0;
      if ((t & 63) == 0) base = atomicAdd(&nrows, (uint32_t)__popcll(m));
      base = __shfl(base, 0);
      if (keep) rows[base + __popcll(m & ((1ull << (t & 63)) - 1ull))] = (uint32_t)t + 256u * (uint32_t)f;
    }
  }
  __syncthreads();
  // one row per wave at a time (the workgroup's four waves on four rows), and every load of a row --
  // the observation bytes and the tail's scalars -- issued before its first store
  const int ln = t & 63;
  // (the row loop's bounds made visibly uniform: its branches and the descriptors stay scalar)
  const uint32_t nr = __builtin_amdgcn_readfirstlane(nrows);
  const uint32_t wv = __builtin_amdgcn_readfirstlane((uint32_t)(t >> 6));
  if constexpr (ONE) {
    // Software-pipelined: the next row's loads are issued before this row's stores.  (gfx9 counts
    // loads and stores on one in-order counter, so a wave that loads after storing waits for its
    // stores to drain; here the wait for row r + 4's bytes lets row r's stores stay in flight.)
    // A row's observation bytes arrive with two 16-byte loads per lane into registers, go through the
    // wave's LDS window, and come back in name order with byte reads: per row 2 + 1 loads instead of
    // one byte load per value, the memory pipeline's instructions being what bounds this kernel.
    // Buffer loads and stores through per-row descriptors built from wave-uniform values; the range
    // check drops the lanes past a row's end (per dword, so the row's last bytes when OB % 4 != 0 come
    // with a byte load of their own).
    __shared__ u32x4 win[4][128];  // per wave: a row's observation bytes (<= 2 048)
    uint8_t* wb = reinterpret_cast<uint8_t*>(&win[wv][0]);
    struct Row {
      u32x4 q0, q1;  // observation bytes 16 ln .. and 1 024 + 16 ln ..
      uint32_t tb;   // byte OB & ~3 + ln (lanes below OB % 4)
      int mv[3];     // summed: lanes 0..4 the row's x, y, vx, vy, next subgoal (read back with readlane)
      __amdgpu_buffer_rsrc_t dst;
      __amdgpu_buffer_rsrc_t dsto;  // the row's chunks below pb
    };
    // V consecutive values per lane and store (V = 2: float pairs, rows of an even D), chunks of 64 V
    constexpr int NC = kFlatU / V;
    constexpr uint32_t CH = 64u * (uint32_t)V;
    const uint32_t lo = (uint32_t)ln * (uint32_t)(V * sizeof(T));
    const uint32_t pb = cw2 / CH;  // the chunk where the tail starts
    const uint32_t OB = (uint32_t)a.OB, obt = OB & ~3u;
    // the scalars' lane offsets: lane 0-1 in the 8 position bytes, 2-3 in the velocity's, 4 in the next
    // subgoal's; every other lane past its descriptor's end (without 32-bit wrap-around)
    const uint32_t lo4 = (uint32_t)ln * 4u, ovel = ln >= 2 ? lo4 - 8u : 1u << 20, onsd = ln >= 4 ? lo4 - 16u : 1u << 20;
    uint32_t offv[NC + 1][V];  // this lane's source offsets: chunks 0 .. NC - 1, then chunk pb
#pragma unroll
    for (int u = 0; u <= NC; u++)
#pragma unroll
      for (int h = 0; h < V; h++) {
        const uint32_t j = (uint32_t)(V * ln + h) + (u == NC ? pb : (uint32_t)u) * CH;
        offv[u][h] = j < cw2 ? offs[j] : 0u;
      }
    auto load_row = [&](uint32_t r, Row& m) {
      const uint32_t ent = __builtin_amdgcn_readfirstlane(rows[r]);
      const bool fr = ent >= 256u;
      const uint64_t er = (uint64_t)blockIdx.x * K + (ent & 255u);
      const uint8_t* orow = (fr ? a.fobs : a.obs) + er * (uint64_t)OB;
      T* row = reinterpret_cast<T*>(fr ? a.fdst : a.dst) + er * (uint64_t)D;
      const auto src = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(orow), 0, (int)OB, 0x00020000);
      m.dst = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(row), 0,
                                                __builtin_amdgcn_readfirstlane((int)(D * sizeof(T))), 0x00020000);
      m.dsto = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(row), 0,
                                                 __builtin_amdgcn_readfirstlane((int)(pb * CH * sizeof(T))), 0x00020000);
      // (three dword loads through descriptors of 8, 8 and 4 bytes: the range check gives the other
      // lanes 0, so the sum has x, y in lanes 0-1, vx, vy in 2-3 and the next subgoal in lane 4)
      const auto dpos = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr((fr ? a.fpos : a.pos) + 2 * er), 0, 8, 0x00020000);
      const auto dvel = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr((fr ? a.fvel : a.vel) + 2 * er), 0, 8, 0x00020000);
      const auto dnsd = __builtin_amdgcn_make_buffer_rsrc(
          uniform_ptr(a.nsd_on ? (fr ? a.fnsd : a.nsd) + er : (fr ? a.fpos : a.pos)), 0, a.nsd_on ? 4 : 0, 0x00020000);
      // (summed where the row is stored: an add here would wait for the loads just issued)
      m.mv[0] = (int)__builtin_amdgcn_raw_buffer_load_b32(dpos, lo4, 0, 0);
      m.mv[1] = (int)__builtin_amdgcn_raw_buffer_load_b32(dvel, ovel, 0, 0);
      m.mv[2] = (int)__builtin_amdgcn_raw_buffer_load_b32(dnsd, onsd, 0, 0);
      m.q0 = __builtin_amdgcn_raw_buffer_load_b128(src, lo4 * 4u, 0, 0);
      m.q1 = __builtin_amdgcn_raw_buffer_load_b128(src, 1024u + lo4 * 4u, 0, 0);
      m.tb = __builtin_amdgcn_raw_buffer_load_b8(src, obt + (uint32_t)ln, 0, 0);
    };
    auto store_row = [&](const Row& m) {
      win[wv][ln] = m.q0;
      win[wv][64 + ln] = m.q1;
      if ((uint32_t)ln < OB - obt) wb[obt + (uint32_t)ln] = (uint8_t)m.tb;  // (after the 16-byte writes)
      const int mv = m.mv[0] + m.mv[1] + m.mv[2];
      const int px = __builtin_amdgcn_readlane(mv, 0), py = __builtin_amdgcn_readlane(mv, 1);
      const int vx = __builtin_amdgcn_readlane(mv, 2), vy = __builtin_amdgcn_readlane(mv, 3);
      const int nsdv = __builtin_amdgcn_readlane(mv, 4) + 1;
      // the chunks below the tail's chunk pb hold observation bytes only; chunk pb holds the last
      // ones and the tail's start, chunk pb + 1 the tail's rest (<= 29 values)
      // (the first through a descriptor ending at chunk pb: the range check drops the rest, no branches)
#pragma unroll
      for (int p = 0; p < NC; p++) {
        T f[V];
#pragma unroll
        for (int h = 0; h < V; h++) f[h] = (T)wb[offv[p][h]];
        flat_store_v<T, V>(m.dsto, lo + (uint32_t)p * CH * (uint32_t)sizeof(T), f);
      }
      uint32_t obb[V];  // chunk pb's observation bytes
#pragma unroll
      for (int h = 0; h < V; h++) obb[h] = wb[offv[NC][h]];
#pragma unroll
      for (int s = 0; s < 2; s++) {
        const uint32_t pc = pb + (uint32_t)s;
        T f[V];
#pragma unroll
        for (int h = 0; h < V; h++) {
          const int k = V * ln + h + (int)(pc * CH) - (int)cw2;  // tail index of the value (< 0: observation)
          const int k2 = a.nsd_on ? k - 9 : k;
          int tv = (int)(k2 == px);
          tv = k2 < 9 ? tv : (int)(k2 - 9 == py);
          tv = k2 < 18 ? tv : (k2 == 18 ? vx : vy);
          tv = (a.nsd_on && k < 9) ? (int)(k == nsdv) : tv;
          f[h] = k < 0 ? (T)obb[h] : (T)tv;
        }
        if (pc * CH < D) flat_store_v<T, V>(m.dst, lo + pc * CH * (uint32_t)sizeof(T), f);  // (lanes past D dropped)
      }
    };
    // Two rows per iteration: the registers alternate without copies.  The next row's loads are
    // unconditional (the last row re-read at the end), and the first row is peeled off, so that every
    // path into a row's stores has the same loads and stores outstanding: the compiler's counter
    // waits then leave the previous row's stores in flight (a path without them, the first row's,
    // merged into the loop made it wait for every earlier store).
    Row mA{}, mB{};
    uint32_t r = wv;
    if (r < nr) {
      load_row(r, mA);
      load_row(min(r + 4u, nr - 1u), mB);
      store_row(mA);
      r += 4u;
      while (r < nr) {  // (mB holds row r)
        load_row(min(r + 4u, nr - 1u), mA);
        store_row(mB);
        r += 4u;
        if (r >= nr) break;
        load_row(min(r + 4u, nr - 1u), mB);
        store_row(mA);
        r += 4u;
      }
    }
  } else {
    for (uint32_t r = wv; r < nr; r += 4u) {
      const uint32_t ent = rows[r];
      const bool fr = ent >= 256u;  // (uniform: one row per wave)
      const uint64_t er = (uint64_t)blockIdx.x * K + (ent & 255u);
      const uint8_t* __restrict__ orow = (fr ? a.fobs : a.obs) + er * (uint64_t)a.OB;
      T* __restrict__ row = reinterpret_cast<T*>(fr ? a.fdst : a.dst) + er * (uint64_t)D;
      const int32_t* pos = fr ? a.fpos : a.pos;
      const int32_t* vel = fr ? a.fvel : a.vel;
      const int nsdv = a.nsd_on ? (fr ? a.fnsd : a.nsd)[er] + 1 : -1;
      const int px = pos[2 * er], py = pos[2 * er + 1], vx = vel[2 * er], vy = vel[2 * er + 1];
      for (uint32_t j0 = 0; j0 < D; j0 += kFlatU * 64u) {  // a pass: kFlatU loads per lane, then the stores
        uint32_t ob[kFlatU];
#pragma unroll
        for (int u = 0; u < kFlatU; u++) {
          const uint32_t j = j0 + (uint32_t)ln + (uint32_t)u * 64u;
          const uint32_t off = j0 == 0 ? offs[j - j0] : (j < cw2 ? (uint32_t)a.order[j / w2] * w2 + j % w2 : 0u);
          ob[u] = orow[j < cw2 ? off : 0u];  // (unconditional: one batch of loads)
        }
#pragma unroll
        for (int p = 0; p < kFlatU; p++) {
          const uint32_t j = j0 + (uint32_t)ln + (uint32_t)p * 64u;
          const T f = j < cw2 ? (T)ob[p] : flat_tail<T>(a, (int)(j - cw2), nsdv, px, py, vx, vy);
          if (j < D) row[j] = f;
        }
      }
    }
  }
}

__global__ void k_fill_seeds(uint64_t* seed, uint64_t n, uint64_t base, uint64_t offset) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) seed[i] = base + offset + i;
}

}  // namespace pgtg

// ==================================================================================================
// host side: config derivation + C ABI
// ==================================================================================================
using namespace pgtg;

struct pgtg_handle {
  int device = 0;
  uint64_t n = 0;
  hipStream_t stream = nullptr;
  DevCfg hcfg{};
  DevCfg* dcfg = nullptr;
  Tables* dtab = nullptr;
  DevState S{};
  PgtgOutputs out{};
  Lds L{};
  size_t lds = 0;
  std::vector<void*> allocs;
  std::string err;
  uint64_t seed_offset = 0;  // global index of env 0 (for sharded runs)
  int tune_epb = 0, tune_obs_sub = 0, tune_kt_grid = 0, tune_kt_cap = 0, tune_kt_wpc = 0;  // PgtgConfig.tune_*
  int timing = 0;             // bracket every `timing`-th step launch with an event pair (0: off)
  uint64_t step_launches = 0;
  std::vector<hipEvent_t> evpool;  // pairs (start, stop) per timed launch
  size_t ev_used = 0;
  double acc_ms = 0.0;
  uint64_t acc_n = 0;
  // k_traffic: work-list parity, grid (one workgroup per CU), envs per wave in LDS, dynamic LDS
  std::vector<uint32_t> epk;  // the map's edge table (derive_cfg): LDS copy (<= 64 tiles) or S.epk
  std::vector<uint16_t> ewl;  // and its walls (Tables::ewl) for the dual removal test
  uint32_t tr_slot = 0;
  int kt_grid = 0, kt_cap = 16;
  int kt_plan_dw = 0, kt_rs_dw = 0;
  size_t kt_lds = 0;
  // k_envq: step launches so far (its request lists rotate per launch) and its persistent grid
  uint64_t q_launch = 0;
  uint64_t q_grid = 0;
  // map-queue step kernel, fixed at create: 1 k_envb (<= 2 rounds of workgroups), 0 k_envq, -1 not yet
  int q_block = -1;
  int tune_queue_mode = 0;  // PgtgConfig.tune_queue_mode
  // FlattenObservation rows after every launch (pgtg_set_flat_outputs): k_flatten's arguments
  FlatArgs flat{};
  const void* flat_fn = nullptr;  // k_flatten variant of the last launch, and its resident workgroups
  uint64_t flat_wgs = 1536;
  void* flat_dst = nullptr;
  void* final_flat_dst = nullptr;
  float* flat_rew32 = nullptr;  // pgtg_set_flat_scalars
  uint8_t* flat_dones = nullptr;
  uint8_t* flat_tonly = nullptr;
  int flat_dtype = 0;  // 0 float32, 1 int8
};


// The step kernel instance a launch of `mode` runs (traffic/rules: k_env<true>; random maps without
// them: k_envq for steps when the map queue is on, else k_env<false>; BIG: maps of > 64 tiles).
static const void* step_fn(const pgtg_handle* h, int mode) {
  const bool big = h->hcfg.nt > kSmallTiles;
  if (h->hcfg.need_car || h->hcfg.n_rules > 0) return big ? (const void*)k_env<true, true> : (const void*)k_env<true, false>;
  if (mode == MODE_STEP && h->L.queue) {
    if (h->q_block == 1) return big ? (const void*)k_envb<true> : (const void*)k_envb<false>;
    return big ? (const void*)k_envq<true> : (const void*)k_envq<false>;
  }
  return big ? (const void*)k_env<false, true> : (const void*)k_env<false, false>;
}

// entries per env ring of this handle's map queue (k_envb 3, k_envq 2)
static int queue_depth(const pgtg_handle* h) { return h->q_block == 1 ? kBlockDepth : kQueueDepth; }

static thread_local std::string g_create_err;

#define HIPCHK(h, x)                                                                 \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      (h)->err = std::string(#x) + ": " + hipGetErrorString(e_);                     \
      return PGTG_E_DEVICE;                                                          \
    }                                                                                \
  } while (0)

static int timing_flush(pgtg_handle* h) {
  for (size_t k = 0; k + 1 < h->ev_used; k += 2) {
    float ms = 0.f;
    HIPCHK(h, hipEventSynchronize(h->evpool[k + 1]));
    HIPCHK(h, hipEventElapsedTime(&ms, h->evpool[k], h->evpool[k + 1]));
    h->acc_ms += ms;
    h->acc_n++;
  }
  h->ev_used = 0;
  return 0;
}

template <typename T>
static int dalloc(pgtg_handle* h, T** p, size_t count) {
  void* q = nullptr;
  if (count == 0) count = 1;
  HIPCHK(h, hipMalloc(&q, count * sizeof(T)));
  HIPCHK(h, hipMemset(q, 0, count * sizeof(T)));
  h->allocs.push_back(q);
  *p = reinterpret_cast<T*>(q);
  return 0;
}

static int fail(pgtg_handle* h, int code, const std::string& m) {
  h->err = m;
  return code;
}

// atan2 octant tables (host libm == CPython math.atan2) ---------------------------------------
static int8_t nsd_dir(int dx, int dy) {  // environment.py:1483-1502
  double angle = atan2(-(double)dy, (double)dx);
  double q = (angle + M_PI) / (M_PI / 4);
  double mq = fmod(q, 8.0);
  if (mq < 0) mq += 8.0;
  static const int remap[8] = {2, 1, 0, 7, 6, 5, 4, 3};
  return (int8_t)remap[(int)mq];
}
static int8_t compass_dir(int dx, int dy, int s) {  // environment.py:1058-1090
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

// random() < p  <=>  m < p * 2^53 for the 53-bit integer m  <=>  m < ceil(p * 2^53) (exact: scaling by
// a power of two is exact in binary64)
static uint64_t u53_threshold(double p) {
  if (!(p > 0.0)) return 0;
  if (p >= 1.0) return 1ull << 53;
  return (uint64_t)ceil(ldexp(p, 53));
}

static int derive_cfg(pgtg_handle* h, const PgtgConfig& in, DevCfg& c) {
  memset(&c, 0, sizeof c);
  if (in.abi_version != PGTG_ABI_VERSION) return fail(h, PGTG_E_INVALID, "ABI version mismatch");
  int tw = in.fixed_map ? in.fm_w : in.width, th = in.fixed_map ? in.fm_h : in.height;
  if (tw < 1 || th < 1) return fail(h, PGTG_E_INVALID, "map width and height must be >= 1");
  if (tw * th > PGTG_MAX_TILES) return fail(h, PGTG_E_UNSUPPORTED, "this build supports width*height <= 256 tiles");
  c.tw = tw;
  c.th = th;
  c.nt = tw * th;
  c.W = tw * kTile;
  c.H = th * kTile;
  c.fixed_map = in.fixed_map;
  c.tune_fault = in.tune_fault;
  if (in.fixed_map) {
    for (int t = 0; t < c.nt; t++) {
      uint32_t p = in.fm_exits[t] & 15u;
      if (in.fm_obst_type[t] >= 0) p |= (uint32_t)(in.fm_obst_type[t] + 1) << 4 | (uint32_t)in.fm_obst_mask[t] << 7;
      c.fixed_plan[t] = (uint16_t)p;
    }
    int st = in.fm_start[1] * tw + in.fm_start[0], gl = in.fm_goal[1] * tw + in.fm_goal[0];
    if (in.fm_start[0] < 0 || in.fm_start[0] >= tw || in.fm_start[1] < 0 || in.fm_start[1] >= th || in.fm_goal[0] < 0 ||
        in.fm_goal[0] >= tw || in.fm_goal[1] < 0 || in.fm_goal[1] >= th)
      return fail(h, PGTG_E_INVALID, "fixed map start/goal outside the map");
    c.fixed_sg = (uint32_t)st | (uint32_t)in.fm_start[2] << 8 | (uint32_t)gl << 16 | (uint32_t)in.fm_goal[2] << 24;
  }
  c.start_mode = in.start_mode;
  c.goal_mode = in.goal_mode;
  c.sx = in.start_x;
  c.sy = in.start_y;
  c.sdir = in.start_dir;
  c.gx = in.goal_x;
  c.gy = in.goal_y;
  c.gdir = in.goal_dir;
  c.min_distance = in.min_distance;
  // removable_edges in graph-theory nested-dict order (map_generator.py:218-227): sources keyed in
  // first-use order while adding (x,y)-(x+1,y) and (x,y)-(x,y+1) bidirectionally, x outer, y inner.
  {
    std::vector<int> keys;
    std::vector<std::vector<std::array<int, 2>>> dst(c.nt);  // (target, direction N/E/S/W)
    std::vector<int> seen(c.nt, 0);
    auto add1 = [&](int a, int b, int d) {
      if (!seen[a]) {
        seen[a] = 1;
        keys.push_back(a);
      }
      dst[a].push_back({b, d});
    };
    for (int x = 0; x < tw; x++)
      for (int y = 0; y < th; y++) {
        int t = y * tw + x;
        if (x < tw - 1) {
          add1(t, t + 1, 1);
          add1(t + 1, t, 3);
        }
        if (y < th - 1) {
          add1(t, t + tw, 2);
          add1(t + tw, t, 0);
        }
      }
    // (the direction is recorded, not inferred from the index difference: on a 1-wide map the
    // southern neighbour t + tw is also t + 1)
    std::vector<int> ea, eb, ed;
    for (int a : keys)
      for (const auto& bd : dst[a]) {
        ea.push_back(a);
        eb.push_back(bd[0]);
        ed.push_back(bd[1]);
      }
    const int n = (int)ea.size();
    if (n > kMaxEdges) return fail(h, PGTG_E_UNSUPPORTED, "too many map edges");
    c.n_edges = n;
    memset(c.h0, 0, sizeof c.h0);
    for (int e = 0; e < n; e++) c.h0[ea[e] >> 6][ed[e]] |= 1ull << (ea[e] & 63);
    // the edge table (Tables::epk / DevState::epk): a = north/west tile, horizontal flag, reverse edge
    std::vector<int> pos(c.nt * 4, -1);  // (tile, direction) -> list index
    for (int e = 0; e < n; e++) pos[ea[e] * 4 + ed[e]] = e;
    h->epk.assign(n, 0u);
    for (int e = 0; e < n; e++) {
      int a = ea[e], b = eb[e], d = ed[e];
      const int rev = pos[b * 4 + (d + 2) % 4];
      if (d == 0 || d == 3) {  // orient: a = north/west tile, d in {E (1), S (2)}
        std::swap(a, b);
        d = d == 0 ? 2 : 1;
      }
      h->epk[e] = (uint32_t)a | (uint32_t)b << 8 | (uint32_t)(d == 1 ? 1 : 0) << 16 | (uint32_t)rev << 17;
    }
    // the dual test (remove_edges_dual): the wall of each removable edge as two corner codes
    c.dual = (tw >= 2 && th >= 2 && c.nt <= kSmallTiles && tw + th <= 31) ? 1 : 0;
    h->ewl.assign(n, 0);
    if (c.dual) {
      auto ccode = [&](int cx, int cy) -> int {
        if (cx >= 1 && cx <= tw - 1 && cy >= 1 && cy <= th - 1) return (cy - 1) * (tw - 1) + (cx - 1);
        if (cy == 0 && cx < tw) return 64 + cx;                      // north side, clockwise
        if (cx == tw) return 64 + tw + cy;                          // east side
        if (cy == th) return 64 + tw + th + (tw - cx);              // south side
        return 64 + 2 * tw + th + (th - cy);                        // west side
      };
      for (int e = 0; e < n; e++) {
        const uint32_t pk = h->epk[e];
        const int a = (int)(pk & 255u), ax = a % tw, ay = a / tw;
        const bool hz = (pk >> 16) & 1u;
        const int p = hz ? ccode(ax + 1, ay) : ccode(ax, ay + 1), q = ccode(ax + 1, ay + 1);
        h->ewl[e] = (uint16_t)(p | q << 8);
      }
    }
    c.keep = (int)nearbyint((double)n * in.pct_connections);  // Python round (half to even)
  }
  // border candidates (map_generator.py:352-364)
  {
    std::vector<std::array<int, 3>> L;
    for (int x = 0; x < tw; x++) L.push_back({0, x, 0});
    for (int y = 0; y < th; y++) L.push_back({y, tw - 1, 1});
    for (int x = 0; x < tw; x++) L.push_back({th - 1, x, 2});
    for (int y = 0; y < th; y++) L.push_back({y, 0, 3});
    std::array<int, 3> rm[2] = {{th - 1, 0, 3}, {0, tw - 1, 1}};
    for (auto& r : rm)
      for (size_t i = 0; i < L.size(); i++)
        if (L[i] == r) {
          L.erase(L.begin() + i);
          break;
        }
    if ((int)L.size() > kMaxBorder) return fail(h, PGTG_E_UNSUPPORTED, "too many border connections");
    c.n_border = (int)L.size();
    for (size_t i = 0; i < L.size(); i++) {
      c.bt[i] = (uint8_t)(L[i][0] * tw + L[i][1]);
      c.bd[i] = (uint8_t)L[i][2];
    }
    c.n_border_add = (int)nearbyint((double)L.size() * in.pct_connections);
    if (c.dual) {  // generate_map's dual path maps a candidate index to (tile, direction) by arithmetic
      bool ok = c.n_border == 2 * tw + 2 * th - 2 && c.n_border < 64;
      for (int j = 0; ok && j < c.n_border; j++) {
        int t, d;
        if (j < tw) { t = j; d = 0; }
        else if (j < tw + th - 1) { t = (j - tw + 1) * tw + tw - 1; d = 1; }
        else if (j < 2 * tw + th - 1) { t = (th - 1) * tw + (j - tw - th + 1); d = 2; }
        else { t = (j - 2 * tw - th + 1) * tw; d = 3; }
        ok = c.bt[j] == t && c.bd[j] == d;
      }
      if (!ok) c.dual = 0;
    }
  }
  c.obstacle_probability = in.obstacle_probability;
  {
    double ws = in.w_ice + in.w_broken + in.w_sand + in.w_tl;
    double p[4] = {in.w_ice / ws, in.w_broken / ws, in.w_sand / ws, in.w_tl / ws};
    double acc = 0.0, cdf[4];
    for (int k = 0; k < 4; k++) {
      acc += p[k];
      cdf[k] = acc;
    }
    for (int k = 0; k < 4; k++) c.obst_cdf_t[k] = u53_threshold(cdf[k] / cdf[3]);
  }
  c.ice_p = in.ice_probability;
  c.broken_p = in.street_damage_probability;
  c.sand_p = in.sand_probability;
  c.phase_total = in.phase_dur[0] + in.phase_dur[1] + in.phase_dur[2];
  if (c.phase_total <= 0 || c.phase_total > 65535) return fail(h, PGTG_E_INVALID, "invalid traffic light phases");
  c.phase_g = in.phase_dur[0];
  c.phase_gy = in.phase_dur[0] + in.phase_dur[1];
  c.ignore_collisions = in.ignore_traffic_collisions;
  c.separate_cost = in.separate_reward_cost;
  c.autoreset = in.autoreset;
  c.max_steps = in.max_episode_steps;
  c.crash_penalty = in.crash_penalty;
  c.final_goal_bonus = in.final_goal_bonus;
  c.tl_penalty = in.tl_violation_penalty;
  c.still_penalty = in.standing_still_penalty;
  c.visited_penalty = in.visited_penalty;
  for (int k = 1; k <= kMaxTiles; k++) c.ind_reward[k] = in.sum_subgoals_reward / (double)k;  // fp64 like Python
  c.n_channels = in.n_channels;
  if (c.n_channels < 0 || c.n_channels > PGTG_MAX_CHANNELS) return fail(h, PGTG_E_INVALID, "bad channel count");
  c.sliding = in.sliding;
  c.ss = in.sliding_size;
  c.win = in.sliding ? 1 + 2 * in.sliding_size : kTile;
  if (c.win < 1 || c.win > kMaxWin) return fail(h, PGTG_E_UNSUPPORTED, "observation window larger than 31 (sliding_observation_window_size > 15)");
  c.next_subgoal = in.next_subgoal;
  c.generic_channels = 0;
  for (int k = 0; k < c.n_channels; k++) {
    c.channels[k] = in.channels[k];
    if (in.channels[k] == PGTG_CH_SPAWNER || in.channels[k] >= PGTG_CH_LANE0) c.generic_channels = 1;
  }
  c.mask_words = (c.win * c.win + 31) / 32;
  c.obs_bytes = c.n_channels * c.win * c.win;
  c.traffic_ch = -1;
  for (int k = 0; k < c.n_channels; k++)
    if (c.channels[k] == PGTG_CH_TRAFFIC) c.traffic_ch = k;
  c.obs_fast = !c.sliding && !c.generic_channels;
  // streams that can ever be drawn from (unobservable streams are never materialised)
  bool obst_possible = in.fixed_map ? false : in.obstacle_probability > 0;
  bool kinds[4] = {false, false, false, false};
  if (in.fixed_map) {
    for (int t = 0; t < c.nt; t++)
      if (in.fm_obst_type[t] >= 0) kinds[in.fm_obst_type[t]] = true;
  } else if (obst_possible) {
    double w[4] = {in.w_ice, in.w_broken, in.w_sand, in.w_tl};
    for (int k = 0; k < 4; k++) kinds[k] = w[k] > 0;
  }
  c.need_ice = kinds[0];
  c.need_broken = kinds[1];
  c.need_sand = kinds[2];
  // observation channels no square can set: no obstacle of the kind can exist, no car
  c.zero_ch = 1u << PGTG_CH_ZERO;
  if (!kinds[0]) c.zero_ch |= 1u << PGTG_CH_ICE;
  if (!kinds[1]) c.zero_ch |= 1u << PGTG_CH_BROKEN;
  if (!kinds[2]) c.zero_ch |= 1u << PGTG_CH_SAND;
  if (!kinds[3]) c.zero_ch |= 1u << PGTG_CH_TL_GREEN | 1u << PGTG_CH_TL_YELLOW | 1u << PGTG_CH_TL_RED;
  c.density = in.traffic_density;
  c.manual_cars = in.min_car_capacity > 0;
  c.need_car = in.traffic_density > 0 || c.manual_cars;
  if (!c.need_car) c.zero_ch |= 1u << PGTG_CH_TRAFFIC;
  if (c.need_car) {
    if (c.W > 255 || c.H > 255) return fail(h, PGTG_E_UNSUPPORTED, "traffic needs maps of at most 28x28 tiles");
    int cap = (int)((double)(c.nt * 32) * in.traffic_density);
    if (cap < in.min_car_capacity) cap = in.min_car_capacity;
    if (cap < 1) cap = 1;
    c.car_cap = cap;
    // initial traffic consumes <= 1 + 2 cap outputs of the car stream after the shuffle (a profile
    // double and a route draw per car)
    c.kt_jump_bits = 1;
    while ((2 * cap + 2) >> c.kt_jump_bits) c.kt_jump_bits++;
    if (c.kt_jump_bits > kJumpBits) return fail(h, PGTG_E_UNSUPPORTED, "car capacity above the jump-ahead table");
    c.kt_serial = in.tune_kt_serial != 0;
    // one bank: a tick starts with at most 2 x cap + kCompactSlack slots in use (a tick that does not
    // pack starts with <= cap + kCompactSlack and appends <= cap respawns) and appends <= cap more
    c.car_slots = 3 * cap + kCompactSlack;  // configs[2]: 1 204 slots x 12 B x 65 536 envs = 947 MB
    if (in.tune_car_slots > 0) {
      if (in.tune_car_slots < c.car_slots) return fail(h, PGTG_E_INVALID, "tune_car_slots < 3 x car capacity + 4");
      c.car_slots = in.tune_car_slots;
    }
    c.max_spawners = c.nt * 5;
    // k_env: occupancy counters (nt * 32 lane slots, 4 bit) then the spawner cache
    c.sp_cache_off = c.nt * 16;
    c.traf_bytes = c.sp_cache_off + 2 * kSpCache;
    // k_traffic: Floyd output (u16 x cap), the shuffle's draws (u16 x cap), seen bits of the spawnable
    // squares (<= nt * 32), column prefix
    c.rs_jj_off = ((2 * cap + 3) / 4) * 4;  // the shuffle's draws (u16 x cap)
    c.rs_seen_off = c.rs_jj_off + ((2 * cap + 3) / 4) * 4;
    c.rs_pre_off = c.rs_seen_off + 4 * c.nt;
    c.rs_bytes = (c.rs_pre_off + 2 * (c.W + 1) + 3) / 4 * 4;
    c.rs_bytes = std::max(c.rs_bytes, c.rs_jj_off + 16 * c.nt);  // store_initial_counters' words
    c.rs_cm_off = 0;
    if (c.th <= 7) {  // a column's spawnable squares as one 63-bit mask: the lookup's row search is one read
      c.rs_cm_off = c.rs_bytes;
      c.rs_bytes += 8 * c.W;
    }
  }
  {  // DRIVER_BEHAVIORS (pgtg/environment.py:64-109)
    const double ys[5] = {0.95, 0.75, 0.3, 0.98, 0.1}, rv[5] = {0.01, 0.05, 0.15, 0.001, 0.3};
    const int mf[5] = {2, 1, 0, 3, 0};
    const double pl[5] = {0.9, 0.7, 0.3, 0.95, 0.1}, sm[5] = {0.8, 1.0, 1.3, 0.6, 1.5}, rd[5] = {0.1, 0.15, 0.05, 0.3, 0.1};
    for (int k = 0; k < 5; k++) {
      c.beh_t[BEH_YELLOW][k] = u53_threshold(ys[k]);
      c.beh_t[BEH_RED][k] = u53_threshold(rv[k]);
      c.beh_min_follow[k] = mf[k];
      c.beh_patience_thr[k] = (int)floor(pl[k] * 10);
      c.beh_t[BEH_GO][k] = u53_threshold(1.0 - pl[k]);
      c.beh_t[BEH_SPEED][k] = u53_threshold(sm[k]);
      c.beh_t[BEH_DELAY][k] = u53_threshold(rd[k]);
    }
  }
  {
    double tot = 0.0, p[5];
    for (int k = 0; k < 5; k++) tot += in.profile_pct[k];
    for (int k = 0; k < 5; k++) p[k] = tot > 0 ? in.profile_pct[k] / tot : (k == 1 ? 1.0 : 0.0);
    double acc = 0.0, cdf[5];
    for (int k = 0; k < 5; k++) {
      acc += p[k];
      cdf[k] = acc;
    }
    for (int k = 0; k < 5; k++) c.profile_t[k] = u53_threshold(cdf[k] / cdf[4]);
  }
  c.n_rules = in.n_rules;
  if (in.n_rules < 0 || in.n_rules > PGTG_MAX_RULES) return fail(h, PGTG_E_INVALID, "bad rule count");
  for (int k = 0; k < in.n_rules; k++) c.rules[k] = in.rules[k];
  {  // rules that need cars can never fire without traffic: skip the braking pass entirely then
    bool possible = c.need_car;
    for (int k = 0; k < in.n_rules; k++) possible = possible || in.rules[k].min_traffic <= 0;
    if (!possible) c.n_rules = 0;
  }
  c.nsd_off = c.W > c.H ? c.W : c.H;
  c.nsd_pitch = 2 * c.nsd_off + 1;
  c.cmp_off = c.nsd_off + 2;
  c.cmp_pitch = 2 * c.cmp_off + 1;
  c.vis_pitch = c.H + 4;
  c.vis_words = ((c.W + 4) * (c.H + 4) + 31) / 32;
  // plan rows, read as the quads that hold tiles.  Random maps of >= 16 tiles without traffic (the
  // map queue's, whose resets copy rows): whole 128-byte lines, written whole (1 048 576 5x5 envs
  // 401 -> 397 us per launch); smaller ones in 16-byte quads (262 144 3x3 envs: 128-byte rows 97
  // against 92 us, the in-place resets writing four times the bytes)
  c.plan_dq = (c.nt + 7) / 8;
  c.plan_stride = (!c.need_car && !c.fixed_map && c.nt >= 16) ? ((c.nt + 63) / 64) * 64 : c.plan_dq * 8;
  // map-queue entries in whole 128-byte lines, written whole: partly written lines cost the step
  // launch 37 us of its 425 (1 048 576 5x5 envs, 80-byte entries)
  c.qrec_dw = (c.plan_dq * 4 + 4 + 31) & ~31;
#ifdef PGTG_TUNING
  if (const char* e = getenv("PGTG_QPAD"))
    if (!atoi(e)) c.qrec_dw = c.plan_dq * 4 + 4;
  if (const char* e = getenv("PGTG_PPAD"))
    if (!atoi(e)) c.plan_stride = c.plan_dq * 8;
#endif
  return 0;
}

extern "C" {

// Launch shapes of a handle from its config and batch size: envs per workgroup, the LDS layout of
// the step kernels (observation sub-batch, map queue), k_traffic's grid and envs per wave.  Called at
// create and again when pgtg_set_rules changes which step kernel runs.  `allow_queue`: the map
// queue's buffers exist (or may still be allocated).  The tune_* fields of the handle (PgtgConfig,
// 0 = automatic) force shapes for tests and A/B runs.
static int choose_launch(pgtg_handle* h, bool allow_queue) {
  const DevCfg& c = h->hcfg;
  const uint64_t n_envs = h->n;
  // envs per 256-lane workgroup.  A workgroup's time is the slowest of its lanes' serial chains, so
  // small batches use fewer envs per workgroup to reach every CU; large batches of maps of >= 16
  // tiles without traffic or rules keep 128 env lanes and a helper wave that generates the next
  // episodes' maps (k_envq, the map queue: 1 048 576 5x5 envs 2.27 G vs 1.77 G env-steps/s), smaller
  // maps, fixed maps and rules a full workgroup of env lanes (262 144 3x3 envs: 2.50 G vs 2.07 G);
  // traffic 128 (LDS).
  const bool queue_able = allow_queue && !c.need_car && c.n_rules == 0 && !c.fixed_map && !c.generic_channels && c.nt >= 16;
  int envs = c.need_car ? 128
           : n_envs <= (uint64_t)8 * 1024 ? 16
           : n_envs <= (uint64_t)16 * 1024 ? 32
           : n_envs <= (uint64_t)64 * 1024 ? 64
           : (n_envs <= (uint64_t)128 * 1024 || queue_able) ? 128 : kBlock;
  if (h->tune_epb) envs = h->tune_epb;
  if (envs != 16 && envs != 32 && envs != 64 && envs != 128 && envs != 192 && envs != kBlock) envs = kBlock;
  if (envs == 192 && !queue_able) envs = kBlock;  // (three env waves and a map-generating one: k_envq only)
  while (envs > 16 && lds_bytes(lds_layout(c, envs)) + sizeof(Tables) > 150 * 1024) envs /= 2;
  h->L = lds_layout(c, envs);
  if (c.need_car) {
    // traffic: the most envs per workgroup (<= 128) for which two workgroups share a CU's LDS
    // after shrinking the observation sub-batch; else the largest that fits at all
    auto shrink = [&](Lds l) {
      while (l.sub_envs > 8 && lds_bytes(l) + sizeof(Tables) > 80 * 1024) {
        l.sub_envs /= 2;
        l.stream_words = img_words(l.sub_envs, l.seg_bits);
      }
      return l;
    };
    Lds best = shrink(lds_layout(c, envs));
    while (best.envs > 16 && lds_bytes(best) + sizeof(Tables) > 80 * 1024) best = shrink(lds_layout(c, best.envs / 2));
    if (lds_bytes(best) + sizeof(Tables) > 80 * 1024) best = shrink(lds_layout(c, envs));
    // Batches that fill every CU with 256 envs: one workgroup per CU with 64 env lanes in each of
    // its four waves (one wave per SIMD, the observation image sub-batched to fit) instead of two
    // workgroups of 128 envs (two half-filled waves per SIMD): the car pass issues half as many
    // instructions per env.  configs[2] (65 536 envs): k_env<true> + k_traffic 1 405 -> 1 283 us.
    // (Two workgroups of two waves each land on three SIMDs, tools/micro/hwid2.hip.)
    if ((h->tune_epb == 0 && n_envs >= (uint64_t)256 * kBlock) || h->tune_epb == kBlock) {
      Lds l = lds_layout(c, kBlock);
      while (l.sub_envs > 8 && lds_bytes(l) + sizeof(Tables) > 160 * 1024) {
        l.sub_envs /= 2;
        l.stream_words = img_words(l.sub_envs, l.seg_bits);
      }
      if (lds_bytes(l) + sizeof(Tables) <= 160 * 1024) best = l;
    }
    h->L = best;
  }
  if (!c.need_car && h->L.envs == kBlock) {
    // Large batches: when the grid needs more workgroups per CU than fit the LDS (up to the 4 that
    // the registers allow), observe in sub-batches so that the whole grid runs in one round.
    const uint64_t blocks = (n_envs + kBlock - 1) / kBlock;
    const int want = (int)std::min<uint64_t>(4, (blocks + 255) / 256);
    auto fit = [&](const Lds& l) { return (int)((160 * 1024) / (lds_bytes(l) + sizeof(Tables))); };
    while (fit(h->L) < want && h->L.sub_envs > 64) {
      h->L.sub_envs /= 2;
      h->L.stream_words = img_words(h->L.sub_envs, h->L.seg_bits);
    }
  }
  if (h->tune_obs_sub >= 1 && h->tune_obs_sub < h->L.sub_envs) {  // forced observation sub-batch
    h->L.sub_envs = h->tune_obs_sub;
    h->L.stream_words = img_words(h->tune_obs_sub, h->L.seg_bits);
  } else {
    lds_img_in_traf(h->L, c);
  }
  if (c.need_car) {
    // k_traffic: per-lane plan + reset scratch
    h->kt_plan_dw = odd_up((c.nt + 1) / 2);
    h->kt_rs_dw = odd_up(c.rs_bytes / 4);
    // workgroups per CU (two: a second wave per SIMD hides part of the per-lane LDS latency --
    // round 4, configs[2] 910 -> 877 us and the caller workload 733 -> 695 us per step against one,
    // profiles/r04/x17; an earlier tree had measured one faster), then the envs per wave that fit the
    // LDS of that many workgroups
    const size_t per_env = (size_t)4 * (h->kt_plan_dw + h->kt_rs_dw);
    int wpc = h->tune_kt_wpc ? std::max(1, std::min(4, h->tune_kt_wpc)) : 2;
    for (;; wpc--) {
      h->kt_cap = 32;  // envs per wave held in LDS at once
      while (h->kt_cap > 1 && wpc * (4 * h->kt_cap * per_env + sizeof(Tables) + 256) > 160 * 1024) h->kt_cap--;
      if (wpc == 1 || wpc * (4 * h->kt_cap * per_env + sizeof(Tables) + 256) <= 160 * 1024) break;
    }
    if (h->tune_kt_cap >= 1 && h->tune_kt_cap <= h->kt_cap) h->kt_cap = h->tune_kt_cap;
    h->kt_lds = 4 * h->kt_cap * per_env;
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || ncu < 1) ncu = 256;
    h->kt_grid = (int)std::min<uint64_t>((uint64_t)ncu * wpc, (h->n + 3) / 4);
    if (h->tune_kt_grid > 0) h->kt_grid = h->tune_kt_grid;  // forced grid: rounds, lane groups
    if (h->kt_lds + sizeof(Tables) > 160 * 1024) return fail(h, PGTG_E_UNSUPPORTED, "LDS budget exceeded (traffic reset scratch)");
    if (h->kt_lds > 64 * 1024)
      (void)hipFuncSetAttribute((const void*)k_traffic, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->kt_lds);
  }
  // map queue (k_envq): recheck after the adjustments above, place the helper scratch
  h->L.queue = h->L.queue && allow_queue && h->L.sub_envs >= h->L.envs && h->L.envs <= kBlock - 64;
  lds_tail(h->L, c);
  if (h->L.queue && lds_bytes(h->L) + kTabHead > 40 * 1024) {  // keep 4 workgroups per CU
    h->L.queue = 0;
    lds_tail(h->L, c);
  }
  h->lds = lds_bytes(h->L);
  if (h->lds + sizeof(Tables) > 160 * 1024) return fail(h, PGTG_E_UNSUPPORTED, "LDS budget exceeded");
  if (h->lds > 64 * 1024) {
    const void* fns[] = {(const void*)k_env<true, false>, (const void*)k_env<false, false>, (const void*)k_envq<false>,
                         (const void*)k_env<true, true>, (const void*)k_env<false, true>, (const void*)k_envq<true>,
                         (const void*)k_envb<false>, (const void*)k_envb<true>};
    for (const void* f : fns) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds);
  }
  // first-round start offsets (stagger_start) for the launches without traffic
  if (!c.need_car && c.n_rules == 0) {
    int ncu = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || ncu < 1) ncu = 256;
    const void* fn = step_fn(h, MODE_STEP);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kBlock, h->lds) != hipSuccess || per_cu < 1) per_cu = 1;
    h->L.stagger_wgs = ncu * per_cu;
    // only launches of two rounds or more: one round has no later workgroups to keep the offsets
    // (1 048 576 5x5 envs, 8 rounds: k_envq 476 -> 460 us; 262 144 envs, 2 rounds: 140 -> 133 us;
    // one round: 66 -> 78 us, profiles/r03/abrec/stagger_by_shard.txt)
    const uint64_t blocks = (h->n + h->L.envs - 1) / h->L.envs;
    h->L.stagger = blocks >= (uint64_t)2 * h->L.stagger_wgs ? 1 : 0;
    // k_envq: the workgroups resident at once
    // (more, with the later ones waiting for a slot: 125 % of them 429 vs 424 us per 1 048 576-env
    // launch, 150 % 450 us)
    h->q_grid = std::max<uint64_t>(1, std::min(std::min(blocks, (uint64_t)h->L.stagger_wgs), (uint64_t)kMaxQueueGrid));
    // the map queue's step kernel, once per handle (its ring layout follows): k_envb for grids of at
    // most two rounds of workgroups, k_envq's persistent grid beyond
    if (h->q_block < 0 && h->L.queue)
      h->q_block = h->tune_queue_mode ? (h->tune_queue_mode == 2 ? 1 : 0)
                                      : (blocks <= (uint64_t)2 * h->L.stagger_wgs ? 1 : 0);
#ifdef PGTG_TUNING
    if (const char* e = getenv("PGTG_STAGGER")) h->L.stagger = atoi(e);
#endif
  }
  return PGTG_OK;
}

int pgtg_create(const PgtgConfig* cfg, uint64_t n_envs, int32_t device, pgtg_handle** out) {
  if (!cfg || !out) return PGTG_E_INVALID;
  pgtg_handle* h = new pgtg_handle();
  *out = nullptr;
  h->device = device;
  h->n = n_envs;
  h->tune_epb = cfg->tune_envs_per_block;
  h->tune_obs_sub = cfg->tune_obs_sub;
  h->tune_kt_grid = cfg->tune_kt_grid;
  h->tune_kt_cap = cfg->tune_kt_cap;
  h->tune_kt_wpc = cfg->tune_kt_wpc;
  h->tune_queue_mode = cfg->tune_queue_mode;
  int rc = 0;
  if (n_envs == 0) rc = fail(h, PGTG_E_INVALID, "n_envs must be > 0");
  if (!rc) rc = derive_cfg(h, *cfg, h->hcfg);
  if (rc) {
    g_create_err = h->err;
    delete h;
    return rc;
  }
  if (hipSetDevice(device) != hipSuccess) {
    g_create_err = "hipSetDevice failed";
    delete h;
    return PGTG_E_DEVICE;
  }
  const DevCfg& c = h->hcfg;
  DevState& S = h->S;
  S.n = n_envs;
  uint64_t n = n_envs;
#define ALLOC(p, cnt)                 \
  if ((rc = dalloc(h, &(p), (cnt)))) { \
    g_create_err = h->err;            \
    pgtg_destroy(h);                  \
    return rc;                        \
  }
  ALLOC(h->dcfg, 1);
  ALLOC(S.rec, n);
  ALLOC(S.seed, n);
  ALLOC(S.plan, n * (uint64_t)c.plan_stride);
  ALLOC(S.err, n);
  ALLOC(S.counters, 4);  // env steps, episodes, map-queue entries generated, overflow requests served
                         // (state blob: the first two)
  ALLOC(S.wg_ticks, 1);
  DevStream* streams[4] = {&S.car, &S.ice, &S.broken, &S.sand};
  int needs[4] = {c.need_car, c.need_ice, c.need_broken, c.need_sand};
  for (int k = 0; k < 4; k++)
    if (needs[k]) {
      ALLOC(streams[k]->shi, n);
      ALLOC(streams[k]->slo, n);
      ALLOC(streams[k]->ihi, n);
      ALLOC(streams[k]->ilo, n);
      ALLOC(streams[k]->buf, n);
    }
  if (c.visited_penalty != 0.0) ALLOC(S.visited, n * (uint64_t)c.vis_words);
  if (c.nt > kSmallTiles) {  // maps of > 64 tiles read their edge table from global memory
    uint32_t* e = nullptr;
    ALLOC(e, h->epk.size());
    if (hipMemcpy(e, h->epk.data(), h->epk.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
      g_create_err = "edge table upload failed";
      pgtg_destroy(h);
      return PGTG_E_DEVICE;
    }
    S.epk = e;
  }
  if (c.need_car) {
    ALLOC(S.car_w0, (uint64_t)c.car_slots * n);
    ALLOC(S.car_w1, (uint64_t)c.car_slots * n);
    S.sp_pitch = (uint32_t)((c.max_spawners + 7) & ~7);
    S.fresh_occ = (uint32_t)((c.car_cap + 3) & ~3);
    S.fresh_dw = S.fresh_occ + (uint32_t)c.nt * 4u;
    ALLOC(S.car_id, (uint64_t)c.car_slots * n);
    ALLOC(S.traf, n);
    ALLOC(S.occ, (uint64_t)c.nt * 4 * n);
    ALLOC(S.fresh, (uint64_t)S.fresh_dw * n);
    ALLOC(S.spawners, (uint64_t)S.sp_pitch * n);
    ALLOC(S.tr_list, n);
    ALLOC(S.tr_count, 2);
  }
  // atan2 tables
  {
    std::vector<int8_t> nsd((size_t)c.nsd_pitch * c.nsd_pitch), cmp((size_t)c.cmp_pitch * c.cmp_pitch);
    for (int a = 0; a < c.nsd_pitch; a++)
      for (int b = 0; b < c.nsd_pitch; b++) nsd[(size_t)a * c.nsd_pitch + b] = nsd_dir(a - c.nsd_off, b - c.nsd_off);
    for (int a = 0; a < c.cmp_pitch; a++)
      for (int b = 0; b < c.cmp_pitch; b++)
        cmp[(size_t)a * c.cmp_pitch + b] = compass_dir(a - c.cmp_off, b - c.cmp_off, cfg->sliding_size);
    int8_t *dn = nullptr, *dc = nullptr;
    ALLOC(dn, nsd.size());
    ALLOC(dc, cmp.size());
    if (hipMemcpy(dn, nsd.data(), nsd.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dc, cmp.data(), cmp.size(), hipMemcpyHostToDevice) != hipSuccess) {
      g_create_err = "table upload failed";
      pgtg_destroy(h);
      return PGTG_E_DEVICE;
    }
    S.nsd_tab = dn;
    S.cmp_tab = dc;
  }
#undef ALLOC
  {
    Tables t;
    memset(&t, 0, sizeof t);
    memcpy(t.wall, hs::kTileWall, sizeof t.wall);
    memcpy(t.seg, hs::kExitSeg, sizeof t.seg);
    memcpy(t.obst, hs::kObstMask, sizeof t.obst);
    memcpy(t.spawner, hs::kLaneSpawner, sizeof t.spawner);
    memcpy(t.lanes, hs::kLanes, sizeof t.lanes);
    memcpy(t.ind, c.ind_reward, sizeof t.ind);
    if (c.n_edges <= kSmallEdges) memcpy(t.epk, h->epk.data(), h->epk.size() * sizeof(uint32_t));
    if (c.n_edges <= kSmallEdges) memcpy(t.ewl, h->ewl.data(), h->ewl.size() * sizeof(uint16_t));
    memcpy(t.bt, c.bt, sizeof t.bt);
    memcpy(t.bd, c.bd, sizeof t.bd);
    for (int k = 0; k < PGTG_MAX_CHANNELS; k++) t.chan[k] = (uint8_t)c.channels[k];
    memset(t.li, 255, sizeof t.li);
    memset(t.slot_sq, 255, sizeof t.slot_sq);
    for (int ex = 0; ex < 16; ex++) {
      int n = 0;
      for (int lx = 0; lx < 9; lx++)
        for (int ly = 0; ly < 9; ly++) {
          int sq = lx * 9 + ly;
          uint32_t ln = hs::kLanes[ex][sq];
          if (ln) {
            t.li[ex][sq] = (uint8_t)n;
            t.slot_sq[ex][n] = (uint8_t)sq;
            n++;
            t.lanecol[ex][lx] |= (uint16_t)(1u << ly);
          }
          if ((hs::kLaneSpawner[ex][sq >> 5] >> (sq & 31)) & 1u) t.spcol[ex][lx] |= (uint16_t)(1u << ly);
          for (int ty = 0; ty < 4; ty++)
            if ((ln >> (28 + ty)) & 1u) t.allcol[ex][ty][lx] |= (uint16_t)(1u << ly);
        }
    }
    memcpy(t.lane_route, hs::kLaneRoute, sizeof t.lane_route);
    memcpy(t.route_type_lane, hs::kRouteTypeLane, sizeof t.route_type_lane);
    for (int r = 0; r < cfg->n_rules && r < PGTG_MAX_RULES; r++) memcpy(t.rule_w[r], cfg->rules[r].weight, sizeof t.rule_w[r]);
    memcpy(t.beh_t, h->hcfg.beh_t, sizeof t.beh_t);
    memcpy(t.beh_mf, h->hcfg.beh_min_follow, sizeof t.beh_mf);
    memcpy(t.beh_pt, h->hcfg.beh_patience_thr, sizeof t.beh_pt);
    if ((rc = dalloc(h, &h->dtab, 1)) || hipMemcpy(h->dtab, &t, sizeof t, hipMemcpyHostToDevice) != hipSuccess) {
      g_create_err = "table upload failed";
      pgtg_destroy(h);
      return PGTG_E_DEVICE;
    }
  }
  if (hipMemcpy(h->dcfg, &h->hcfg, sizeof(DevCfg), hipMemcpyHostToDevice) != hipSuccess) {
    g_create_err = "config upload failed";
    pgtg_destroy(h);
    return PGTG_E_DEVICE;
  }
  if ((rc = choose_launch(h, true))) {
    g_create_err = h->err;
    pgtg_destroy(h);
    return rc;
  }
  if (h->L.queue) {
    if ((rc = dalloc(h, &h->S.qbuf, n * (uint64_t)queue_depth(h) * (uint64_t)c.qrec_dw)) || (rc = dalloc(h, &h->S.qstate, n)) ||
        (!h->q_block &&
         ((rc = dalloc(h, &h->S.qreq, 2 * h->q_grid * queue_req_cap((n + h->L.envs - 1) / h->L.envs, h->q_grid, h->L.envs))) ||
          (rc = dalloc(h, &h->S.qovf, 2 * 8 * ((h->q_grid + 7) / 8) * (uint64_t)h->L.envs)) ||
          (rc = dalloc(h, &h->S.qctr, kQctrWords))))) {
      g_create_err = h->err;
      pgtg_destroy(h);
      return rc;
    }
  }
  *out = h;
  return PGTG_OK;
}

int pgtg_destroy(pgtg_handle* h) {
  if (!h) return PGTG_OK;
  for (void* p : h->allocs) (void)hipFree(p);
  for (auto e : h->evpool) (void)hipEventDestroy(e);
  delete h;
  return PGTG_OK;
}

int pgtg_set_stream(pgtg_handle* h, void* stream) {
  if (!h) return PGTG_E_INVALID;
  h->stream = reinterpret_cast<hipStream_t>(stream);
  return PGTG_OK;
}

int pgtg_set_outputs(pgtg_handle* h, const PgtgOutputs* o) {
  if (!h || !o) return PGTG_E_INVALID;
  h->out = *o;
  return PGTG_OK;
}

// k_flatten over the bound observation (final: the terminal observations, finished envs' rows only)
// mode: 0 the observation rows, 1 the terminal rows, 2 both (one launch after a step)
static int launch_flatten(pgtg_handle* h, int mode) {
  FlatArgs a = h->flat;
  const PgtgOutputs& o = h->out;
  const bool final = mode == 1;
  a.obs = final ? o.final_obs : o.obs;
  a.pos = final ? o.final_position : o.position;
  a.vel = final ? o.final_velocity : o.velocity;
  a.nsd = final ? o.final_next_subgoal : o.next_subgoal;
  a.term = o.terminated;
  a.trunc = o.truncated;
  a.dst = final ? h->final_flat_dst : h->flat_dst;
  a.fobs = o.final_obs;
  a.fpos = o.final_position;
  a.fvel = o.final_velocity;
  a.fnsd = o.final_next_subgoal;
  a.fdst = h->final_flat_dst;
  a.final = mode;
  a.rew = o.reward;
  a.rew32 = final ? nullptr : h->flat_rew32;
  a.dones = final ? nullptr : h->flat_dones;
  a.tonly = final ? nullptr : h->flat_tonly;
  // (float pairs per store: 128 vs 137.7 us per step at 65 536 envs in the pipelined kernel, profiles/r06/s27;
  // in the first row-per-wave kernel they had been slower, 94.7 vs 81.1 us per pass)
  const bool one = a.D <= kFlatU * 64 && a.OB <= 2048;  // (rows of one pass; the bytes fit the LDS window)
  const bool pair = one && !h->flat_dtype && a.D % 2 == 0;  // float pairs: rows 8-byte aligned, none straddles D
  const void* fn = h->flat_dtype ? (one ? (const void*)k_flatten<int8_t, true, 1> : (const void*)k_flatten<int8_t, false, 1>)
                                 : (pair ? (const void*)k_flatten<float, true, 2>
                                         : (one ? (const void*)k_flatten<float, true, 1> : (const void*)k_flatten<float, false, 1>));
  if (h->flat_fn != fn) {  // the workgroups resident at once (kernel registers), fixed per variant
    int ncu = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || ncu < 1) ncu = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, 0) != hipSuccess || per_cu < 1) per_cu = 1;
    h->flat_fn = fn;
    h->flat_wgs = (uint64_t)ncu * (uint64_t)per_cu;
  }
  // rows per workgroup <= 256; one round of resident workgroups where the batch allows.  (The grid
  // hardly matters: 256 / 512 / 1 536 / 3 072 workgroups 150 / 138 / 139 / 134 us per step at 65 536
  // envs, profiles/r06/flat_grid_sweep.txt -- the kernel is bound chip-wide, not by waves in flight)
  const uint64_t G = std::max<uint64_t>(std::min<uint64_t>(h->n, h->flat_wgs), (h->n + 255) / 256);
  if (h->flat_dtype) {
    if (one) hipLaunchKernelGGL((k_flatten<int8_t, true, 1>), dim3((unsigned)G), dim3(256), 0, h->stream, a);
    else hipLaunchKernelGGL((k_flatten<int8_t, false, 1>), dim3((unsigned)G), dim3(256), 0, h->stream, a);
  } else if (pair) {
    hipLaunchKernelGGL((k_flatten<float, true, 2>), dim3((unsigned)G), dim3(256), 0, h->stream, a);
  } else {
    if (one) hipLaunchKernelGGL((k_flatten<float, true, 1>), dim3((unsigned)G), dim3(256), 0, h->stream, a);
    else hipLaunchKernelGGL((k_flatten<float, false, 1>), dim3((unsigned)G), dim3(256), 0, h->stream, a);
  }
  HIPCHK(h, hipGetLastError());
  return PGTG_OK;
}

static int launch(pgtg_handle* h, const uint8_t* actions, const uint8_t* mask, int mode) {
  HIPCHK(h, hipSetDevice(h->device));
  uint64_t blocks = (h->n + h->L.envs - 1) / h->L.envs;
  const bool timed = h->timing > 0 && mode == MODE_STEP && (h->step_launches++ % (uint64_t)h->timing) == 0;
  if (timed) {
    if (h->evpool.empty()) {
      h->evpool.resize(2048);
      for (auto& e : h->evpool) HIPCHK(h, hipEventCreate(&e));
    }
    if (h->ev_used + 2 > h->evpool.size()) {
      int rc = timing_flush(h);
      if (rc) return rc;
    }
    HIPCHK(h, hipEventRecord(h->evpool[h->ev_used], h->stream));
  }
  const void* fn = step_fn(h, mode);
  void* args[] = {&h->dcfg, &h->dtab, &h->S, &actions, &mask, &h->out, &mode, &h->L, &h->tr_slot};
  if (fn == (const void*)k_envb<false> || fn == (const void*)k_envb<true>) {
    void* bargs[] = {&h->dcfg, &h->dtab, &h->S, &actions, &h->out, &h->L};
    HIPCHK(h, hipLaunchKernel(fn, dim3((unsigned)blocks), dim3(kBlock), bargs, h->lds, h->stream));
  } else if (fn == (const void*)k_envq<false> || fn == (const void*)k_envq<true>) {
    uint32_t qsel = (uint32_t)(h->q_launch % 3) | (uint32_t)(h->q_launch & 1) << 2;
    h->q_launch++;
    void* qargs[] = {&h->dcfg, &h->dtab, &h->S, &actions, &h->out, &h->L, &qsel};
    HIPCHK(h, hipLaunchKernel(fn, dim3((unsigned)std::min(blocks, h->q_grid)), dim3(kBlock), qargs, h->lds, h->stream));
  } else {
    HIPCHK(h, hipLaunchKernel(fn, dim3((unsigned)blocks), dim3(kBlock), args, h->lds, h->stream));
  }
  HIPCHK(h, hipGetLastError());
  if (h->hcfg.need_car && mode != MODE_OBSERVE) {
    // initial traffic of the envs reset by this launch; it also sets their new cars' squares in the
    // observation's traffic channel
    hipLaunchKernelGGL(k_traffic, dim3((unsigned)h->kt_grid), dim3(kBlock), h->kt_lds, h->stream, h->dcfg, h->dtab,
                       h->S, h->out, h->tr_slot, h->kt_plan_dw, h->kt_rs_dw, h->kt_cap);
    HIPCHK(h, hipGetLastError());
    h->tr_slot ^= 1u;
  }
  {
    const bool fl = h->flat_dst != nullptr, ff = h->final_flat_dst != nullptr && mode == MODE_STEP;
    if (fl || ff)  // (both row sets in one launch after a step)
      if (int rc = launch_flatten(h, fl && ff ? 2 : (ff ? 1 : 0))) return rc;
  }
  if (timed) {
    HIPCHK(h, hipEventRecord(h->evpool[h->ev_used + 1], h->stream));
    h->ev_used += 2;
  }
  return PGTG_OK;
}

// After a reset launch of a map-queue handle, before a state dump and when the step kernel changes:
// drop the pending refill requests and fill every ring (k_qfill) -- the entries the requests asked for
// and the rings of the envs a reset gave new maps.
static int queue_fill(pgtg_handle* h) {
  if (!h->L.queue || !h->S.qbuf) return PGTG_OK;
  if (h->S.qctr) HIPCHK(h, hipMemsetAsync(h->S.qctr, 0, kQctrWords * sizeof(uint32_t), h->stream));
#ifdef PGTG_TUNING
  if (const char* e = getenv("PGTG_QFILL"))
    if (!atoi(e)) return PGTG_OK;
#endif
  const int pdw = h->L.plan_stride_dw;
  const size_t lds = (size_t)4 * kBlock * pdw;
  const bool big = h->hcfg.nt > kSmallTiles;
  const void* fn = h->q_block == 1 ? (big ? (const void*)k_qfill_b<true> : (const void*)k_qfill_b<false>)
                                   : (big ? (const void*)k_qfill<true> : (const void*)k_qfill<false>);
  if (lds > 64 * 1024) HIPCHK(h, hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const uint64_t blocks = (h->n + kBlock - 1) / kBlock;
  void* args[] = {&h->dcfg, &h->dtab, &h->S, (void*)&pdw};
  HIPCHK(h, hipLaunchKernel(fn, dim3((unsigned)blocks), dim3(kBlock), args, lds, h->stream));
  HIPCHK(h, hipGetLastError());
  return PGTG_OK;
}

int pgtg_reset(pgtg_handle* h, const uint64_t* seeds_host, uint64_t seed_base, const uint8_t* mask_dev) {
  if (!h) return PGTG_E_INVALID;
  HIPCHK(h, hipSetDevice(h->device));
  if (seeds_host) {
    HIPCHK(h, hipMemcpyAsync(h->S.seed, seeds_host, h->n * sizeof(uint64_t), hipMemcpyHostToDevice, h->stream));
  } else {
    hipLaunchKernelGGL(k_fill_seeds, dim3((unsigned)((h->n + 255) / 256)), dim3(256), 0, h->stream, h->S.seed, h->n,
                       seed_base, (uint64_t)0);
    HIPCHK(h, hipGetLastError());
  }
  if (int rc = launch(h, nullptr, mask_dev, MODE_RESET_SEEDED)) return rc;
  return queue_fill(h);
}

int pgtg_reset_unseeded(pgtg_handle* h, const uint8_t* mask_dev) {
  if (!h) return PGTG_E_INVALID;
  if (int rc = launch(h, nullptr, mask_dev, MODE_RESET_UNSEEDED)) return rc;
  return queue_fill(h);
}

int pgtg_step(pgtg_handle* h, const uint8_t* actions_dev) {
  if (!h || !actions_dev) return PGTG_E_INVALID;
  return launch(h, actions_dev, nullptr, MODE_STEP);
}

int pgtg_step_many(pgtg_handle* h, const uint8_t* actions_dev, uint64_t row_stride, uint64_t ticks) {
  if (!h || !actions_dev || row_stride < h->n) return PGTG_E_INVALID;
  for (uint64_t k = 0; k < ticks; k++)
    if (int rc = launch(h, actions_dev + k * row_stride, nullptr, MODE_STEP)) return rc;
  return PGTG_OK;
}

int pgtg_observe(pgtg_handle* h) {
  if (!h) return PGTG_E_INVALID;
  return launch(h, nullptr, nullptr, MODE_OBSERVE);
}

int pgtg_random_actions(pgtg_handle* h, uint8_t* actions_dev, uint64_t seed, uint64_t t, uint64_t env_offset) {
  if (!h || !actions_dev) return PGTG_E_INVALID;
  HIPCHK(h, hipSetDevice(h->device));
  hipLaunchKernelGGL(k_random_actions, dim3((unsigned)((h->n + 255) / 256)), dim3(256), 0, h->stream, actions_dev, h->n,
                     seed, t, env_offset);
  HIPCHK(h, hipGetLastError());
  return PGTG_OK;
}

static int read_traf(pgtg_handle* h, uint64_t env, uint4* t) {
  HIPCHK(h, hipMemcpy(t, h->S.traf + env, sizeof *t, hipMemcpyDeviceToHost));
  return 0;
}

int pgtg_get_env_state(pgtg_handle* h, uint64_t env, PgtgEnvState* st) {
  if (!h || !st || env >= h->n) return PGTG_E_INVALID;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  EnvRec r;
  uint64_t seed;
  uint8_t e;
  HIPCHK(h, hipMemcpy(&r, h->S.rec + env, sizeof r, hipMemcpyDeviceToHost));
  HIPCHK(h, hipMemcpy(&seed, h->S.seed + env, sizeof seed, hipMemcpyDeviceToHost));
  HIPCHK(h, hipMemcpy(&e, h->S.err + env, 1, hipMemcpyDeviceToHost));
  memset(st, 0, sizeof *st);
  st->x = (int16_t)(r.a.x & 0xffffu);
  st->y = (int16_t)(r.a.x >> 16);
  st->vx = (int16_t)(r.a.y & 0xffffu);
  st->vy = (int16_t)(r.a.y >> 16);
  st->phase = (int)(r.a.z & 0xffffu);
  uint32_t fl = (r.a.z >> 16) & 0xfu;
  st->terminated = (fl & kFlagTerminated) ? 1 : 0;
  st->flat_tire = (fl & kFlagFlatTire) ? 1 : 0;
  st->path_len = (int)(r.a.z >> 20);
  st->elapsed = (int)r.a.w;
  st->spawn_counter = r.b.y;
  st->used_subgoals[0] = (uint64_t)r.b.z | ((uint64_t)r.b.w << 32);
  if (h->hcfg.nt > kSmallTiles) {  // maps of > 64 tiles mark the plan words (kPlanUsed)
    std::vector<uint16_t> p(h->hcfg.plan_stride);
    HIPCHK(h, hipMemcpy(p.data(), h->S.plan + env * (uint64_t)h->hcfg.plan_stride, p.size() * 2, hipMemcpyDeviceToHost));
    st->used_subgoals[0] = 0;
    for (int t = 0; t < h->hcfg.nt; t++) st->used_subgoals[t >> 6] |= (uint64_t)((p[t] & kPlanUsed) != 0) << (t & 63);
  }
  st->seed = seed;
  st->error = -(int)e;
  if (h->hcfg.need_car) {
    uint4 t;
    if (int rc = read_traf(h, env, &t)) return rc;
    st->n_cars = (int)(t.x & 0xffffu);
    st->n_spawners = (int)(t.x >> 16);
    st->next_car_id = (int)t.y;
    st->car_tail = (int)t.z;
  }
  return PGTG_OK;
}


// One env's cars in list order (empty slots skipped): a strided copy of its slots.
static int host_read_cars(pgtg_handle* h, uint64_t env, const uint4& t, std::vector<PgtgCar>& cars) {
  cars.clear();
  const int tail = (int)t.z;
  if (tail == 0) return 0;
  const uint64_t N = h->n;
  std::vector<uint32_t> w0(tail), w1(tail, 0u), id(tail);
  if (t.w & kTrafFresh) {  // initial traffic still in the env's staging block (patience 0, id = slot)
    HIPCHK(h, hipMemcpy(w0.data(), h->S.fresh + env * (uint64_t)h->S.fresh_dw, 4 * (size_t)tail, hipMemcpyDeviceToHost));
    for (int k = 0; k < tail; k++) id[k] = (uint32_t)k;
  } else {
    HIPCHK(h, hipMemcpy2D(w0.data(), 4, h->S.car_w0 + env, N * 4, 4, tail, hipMemcpyDeviceToHost));
    HIPCHK(h, hipMemcpy2D(w1.data(), 4, h->S.car_w1 + env, N * 4, 4, tail, hipMemcpyDeviceToHost));
    HIPCHK(h, hipMemcpy2D(id.data(), 4, h->S.car_id + env, N * 4, 4, tail, hipMemcpyDeviceToHost));
  }
  for (int k = 0; k < tail; k++) {
    if (w0[k] & kCarEmpty) continue;
    cars.push_back(PgtgCar{(int32_t)id[k], (int32_t)(w0[k] & 255u), (int32_t)((w0[k] >> 8) & 255u),
                           (int32_t)((w0[k] >> 16) & 31u), (int32_t)((w0[k] >> 21) & 7u), (int32_t)w1[k],
                           (int32_t)((w0[k] >> 24) & 3u)});
  }
  if ((int)cars.size() != (int)(t.x & 0xffffu)) return fail(h, PGTG_E_DEVICE, "car slots disagree with the car count");
  return 0;
}

// One env's car list written packed into slots [0, n); the traffic record gets n cars, tail n and
// next id `next_id`.
static int host_write_cars(pgtg_handle* h, uint64_t env, uint4 t, const std::vector<PgtgCar>& cars, uint32_t next_id) {
  const int n = (int)cars.size();
  if (n > h->hcfg.car_cap) return fail(h, PGTG_E_UNSUPPORTED, "more cars than the handle's car capacity");
  const uint64_t N = h->n;
  std::vector<uint32_t> w0(n), w1(n), id(n);
  for (int k = 0; k < n; k++) {
    const PgtgCar& q = cars[k];
    w0[k] = (uint32_t)q.x | (uint32_t)q.y << 8 | (uint32_t)q.route << 16 | (uint32_t)q.profile << 21 |
            (uint32_t)q.delay << 24;
    w1[k] = (uint32_t)q.patience;
    id[k] = (uint32_t)q.id;
  }
  if (n > 0) {
    HIPCHK(h, hipMemcpy2D(h->S.car_w0 + env, N * 4, w0.data(), 4, 4, n, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy2D(h->S.car_w1 + env, N * 4, w1.data(), 4, 4, n, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemcpy2D(h->S.car_id + env, N * 4, id.data(), 4, 4, n, hipMemcpyHostToDevice));
  }
  t.x = (t.x & 0xffff0000u) | (uint32_t)n;
  t.y = next_id;
  t.z = (uint32_t)n;
  t.w = 0u;  // the slot rows hold the list (not fresh); the counters no longer match: rebuilt next launch
  HIPCHK(h, hipMemcpy(h->S.traf + env, &t, sizeof t, hipMemcpyHostToDevice));
  return 0;
}

int pgtg_get_cars(pgtg_handle* h, uint64_t env, PgtgCar* cars, int32_t cap, int32_t* n) {
  if (!h || env >= h->n || !n) return PGTG_E_INVALID;
  *n = 0;
  if (!h->hcfg.need_car) return PGTG_OK;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  uint4 t;
  if (int rc = read_traf(h, env, &t)) return rc;
  *n = (int)(t.x & 0xffffu);
  if (cars && cap > 0 && *n > 0) {
    std::vector<PgtgCar> v;
    if (int rc = host_read_cars(h, env, t, v)) return rc;
    for (int k = 0; k < (int)v.size() && k < cap; k++) cars[k] = v[k];
  }
  return PGTG_OK;
}

int pgtg_get_map_plan(pgtg_handle* h, uint64_t env, int32_t* w, int32_t* h_, uint8_t* exits, int8_t* otype,
                      int8_t* omask, int32_t* start3, int32_t* goal3) {
  if (!h || env >= h->n) return PGTG_E_INVALID;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  const DevCfg& c = h->hcfg;
  std::vector<uint16_t> p(c.plan_stride);
  EnvRec r;
  HIPCHK(h, hipMemcpy(p.data(), h->S.plan + env * (uint64_t)c.plan_stride, c.plan_stride * 2, hipMemcpyDeviceToHost));
  HIPCHK(h, hipMemcpy(&r, h->S.rec + env, sizeof r, hipMemcpyDeviceToHost));
  *w = c.tw;
  *h_ = c.th;
  for (int t = 0; t < c.nt; t++) {
    exits[t] = (uint8_t)plan_exits(p[t]);
    int ot = (int)plan_otype(p[t]);
    otype[t] = (int8_t)(ot - 1);
    omask[t] = (int8_t)(ot ? (int)plan_omask(p[t]) : -1);
  }
  uint32_t sg = r.b.x;
  start3[0] = (int)(sg & 0xffu) % c.tw;
  start3[1] = (int)(sg & 0xffu) / c.tw;
  start3[2] = (int)((sg >> 8) & 0xffu);
  goal3[0] = (int)((sg >> 16) & 0xffu) % c.tw;
  goal3[1] = (int)((sg >> 16) & 0xffu) / c.tw;
  goal3[2] = (int)(sg >> 24);
  return PGTG_OK;
}

int pgtg_get_squares(pgtg_handle* h, uint64_t env, uint64_t* words, int32_t cap, int32_t* width, int32_t* height) {
  if (!h || env >= h->n) return PGTG_E_INVALID;
  const DevCfg& c = h->hcfg;
  if (width) *width = c.W;
  if (height) *height = c.H;
  if (!words) return PGTG_OK;
  if (cap < c.W * c.H) return fail(h, PGTG_E_INVALID, "squares buffer too small");
  HIPCHK(h, hipSetDevice(h->device));
  uint64_t* d = nullptr;
  HIPCHK(h, hipMalloc(&d, (size_t)c.W * c.H * 8));
  hipLaunchKernelGGL(k_squares, dim3(1), dim3(kBlock), 0, h->stream, h->dcfg, h->dtab, h->S, env, d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
  if (e == hipSuccess) e = hipMemcpy(words, d, (size_t)c.W * c.H * 8, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(h, PGTG_E_DEVICE, std::string("pgtg_get_squares: ") + hipGetErrorString(e));
  return PGTG_OK;
}

int pgtg_set_rules(pgtg_handle* h, const PgtgRule* rules, int32_t n_rules) {
  if (!h || n_rules < 0 || n_rules > PGTG_MAX_RULES || (n_rules > 0 && !rules))
    return h ? fail(h, PGTG_E_INVALID, "bad rule count") : PGTG_E_INVALID;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  DevCfg& c = h->hcfg;
  const DevCfg old_cfg = c;
  const Lds old_L = h->L;
  const size_t old_lds = h->lds;
  bool possible = c.need_car;
  for (int k = 0; k < n_rules; k++) {
    c.rules[k] = rules[k];
    possible = possible || rules[k].min_traffic <= 0;
  }
  c.n_rules = possible ? n_rules : 0;
  if ((old_cfg.n_rules > 0) != (c.n_rules > 0)) {
    // the step kernel changes (k_env<true> with the rules' route histogram vs k_envq / k_env<false>):
    // lay the launch out again; the map queue only if its buffers exist
    if (int rc = choose_launch(h, h->S.qbuf != nullptr)) {
      c = old_cfg;
      h->L = old_L;
      h->lds = old_lds;
      return rc;
    }
  }
  const bool refill = h->L.queue && !old_L.queue;  // back to k_envq: rings k_env's resets left stale
  uint8_t w[PGTG_MAX_RULES][6][20] = {};
  for (int k = 0; k < n_rules; k++) memcpy(w[k], rules[k].weight, sizeof w[k]);
  HIPCHK(h, hipMemcpy(h->dcfg, &c, sizeof(DevCfg), hipMemcpyHostToDevice));
  HIPCHK(h, hipMemcpy(reinterpret_cast<uint8_t*>(h->dtab) + kTabHead + offsetof(TablesTail, rule_w), w, sizeof w, hipMemcpyHostToDevice));
  if (refill) return queue_fill(h);
  return PGTG_OK;
}

int pgtg_set_agent(pgtg_handle* h, uint64_t env, int32_t x, int32_t y, int32_t vx, int32_t vy) {
  if (!h || env >= h->n) return PGTG_E_INVALID;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  EnvRec r;
  HIPCHK(h, hipMemcpy(&r, h->S.rec + env, sizeof r, hipMemcpyDeviceToHost));
  r.a.x = ((uint32_t)x & 0xffffu) | ((uint32_t)y << 16);
  r.a.y = ((uint32_t)vx & 0xffffu) | ((uint32_t)vy << 16);
  HIPCHK(h, hipMemcpy(h->S.rec + env, &r, sizeof r, hipMemcpyHostToDevice));
  return PGTG_OK;
}

int pgtg_add_car(pgtg_handle* h, uint64_t env, int32_t x, int32_t y, int32_t route, int32_t profile, int32_t car_id) {
  if (!h || env >= h->n) return PGTG_E_INVALID;
  if (!h->hcfg.need_car) return fail(h, PGTG_E_UNSUPPORTED, "create the handle with min_car_capacity > 0 or traffic");
  if (x < 0 || y < 0 || x >= h->hcfg.W || y >= h->hcfg.H || route < 0 || route >= 20 || profile < 0 || profile >= 5)
    return fail(h, PGTG_E_INVALID, "car outside the map or bad route/profile");
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  uint4 t;
  if (int rc = read_traf(h, env, &t)) return rc;
  std::vector<PgtgCar> v;
  if (int rc = host_read_cars(h, env, t, v)) return rc;
  if ((int)v.size() >= h->hcfg.car_cap) return fail(h, PGTG_E_UNSUPPORTED, "car capacity exhausted");
  const uint32_t id = car_id < 0 ? t.y : (uint32_t)car_id;
  v.push_back(PgtgCar{(int32_t)id, x, y, route, profile, 0, 0});
  return host_write_cars(h, env, t, v, car_id < 0 ? t.y + 1u : t.y);
}

// ---- whole-batch state dump / load (bit-exact replay) ----------------------------------------
// Every device array that carries an env's state from one launch to the next: agent records, seeds,
// tile plans, error codes, counters, the four RNG streams, the visited bitsets, the car slots, the
// traffic records, the spawner lists and the map queue.  The k_traffic work list is per-launch
// scratch (its counters are zeroed on load).  Blob: PgtgStateHeader, n_sections x {id, pad, bytes},
// then each section's bytes at a 16-byte aligned offset.
namespace {
struct StateSection {
  uint32_t id;
  void* ptr;
  uint64_t bytes;
};
struct PgtgStateHeader {
  char magic[4];  // "PGTS"
  uint32_t version;
  uint64_t n;
  uint32_t n_sections, nt, car_cap, plan_stride;
  uint32_t max_spawners, vis_words, qrec_dw, car_slots;
  uint64_t cfg_hash;  // FNV-1a of the handle's DevCfg: every semantic field (probabilities, rewards, map, rules)
};
struct PgtgSectionEntry {
  uint32_t id, pad;
  uint64_t bytes;
};
constexpr uint32_t kStateVersion = 5;
uint64_t cfg_hash(const DevCfg& c) {  // DevCfg is zero-initialised (derive_cfg), so padding hashes as 0
  const uint8_t* p = reinterpret_cast<const uint8_t*>(&c);
  uint64_t h = 0xcbf29ce484222325ull;
  for (size_t k = 0; k < sizeof c; k++) h = (h ^ p[k]) * 0x100000001b3ull;
  return h;
}
}  // namespace

static std::vector<StateSection> state_sections(pgtg_handle* h) {
  const DevCfg& c = h->hcfg;
  const DevState& S = h->S;
  const uint64_t n = h->n;
  std::vector<StateSection> v;
  auto add = [&](uint32_t id, void* p, uint64_t b) {
    if (p) v.push_back({id, p, b});
  };
  add(1, S.rec, n * sizeof(EnvRec));
  add(2, S.seed, n * 8);
  add(3, S.plan, n * (uint64_t)c.plan_stride * 2);
  add(4, S.err, n);
  add(5, S.counters, 16);
  const DevStream* st[4] = {&S.car, &S.ice, &S.broken, &S.sand};
  for (uint32_t k = 0; k < 4; k++) {
    add(10 + 5 * k, st[k]->shi, n * 8);
    add(11 + 5 * k, st[k]->slo, n * 8);
    add(12 + 5 * k, st[k]->ihi, n * 8);
    add(13 + 5 * k, st[k]->ilo, n * 8);
    add(14 + 5 * k, st[k]->buf, n * 8);
  }
  add(30, S.visited, n * (uint64_t)c.vis_words * 4);
  add(31, S.car_w0, (uint64_t)c.car_slots * n * 4);
  add(32, S.car_w1, (uint64_t)c.car_slots * n * 4);
  add(33, S.car_id, (uint64_t)c.car_slots * n * 4);
  add(34, S.traf, n * sizeof(uint4));
  add(36, S.occ, (uint64_t)c.nt * 4 * n * 4);
  add(35, S.spawners, (uint64_t)S.sp_pitch * n * 2);
  add(37, S.fresh, (uint64_t)S.fresh_dw * n * 4);
  add(40, S.qbuf, n * (uint64_t)queue_depth(h) * (uint64_t)c.qrec_dw * 4);
  add(41, S.qstate, n);
  return v;
}

static uint64_t state_blob_bytes(const std::vector<StateSection>& v) {
  uint64_t b = sizeof(PgtgStateHeader) + v.size() * sizeof(PgtgSectionEntry);
  for (const auto& s : v) b = ((b + 15) & ~15ull) + s.bytes;
  return b;
}

int pgtg_state_size(pgtg_handle* h, uint64_t* bytes) {
  if (!h || !bytes) return PGTG_E_INVALID;
  *bytes = state_blob_bytes(state_sections(h));
  return PGTG_OK;
}

int pgtg_dump_state(pgtg_handle* h, void* buf, uint64_t bytes) {
  if (!h || !buf) return PGTG_E_INVALID;
  const auto v = state_sections(h);
  if (bytes < state_blob_bytes(v)) return fail(h, PGTG_E_INVALID, "pgtg_dump_state: buffer smaller than pgtg_state_size");
  HIPCHK(h, hipSetDevice(h->device));
  // the map rings complete (the pending refill requests served now rather than by the next step
  // launch): the blob holds no request list, whose order depends on timing
  if (int rc = queue_fill(h)) return rc;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  uint8_t* p = static_cast<uint8_t*>(buf);
  PgtgStateHeader hd{};
  memcpy(hd.magic, "PGTS", 4);
  hd.version = kStateVersion;
  hd.n = h->n;
  hd.n_sections = (uint32_t)v.size();
  hd.nt = (uint32_t)h->hcfg.nt;
  hd.car_cap = (uint32_t)h->hcfg.car_cap;
  hd.plan_stride = (uint32_t)h->hcfg.plan_stride;
  hd.max_spawners = (uint32_t)h->hcfg.max_spawners;
  hd.vis_words = (uint32_t)h->hcfg.vis_words;
  hd.qrec_dw = (uint32_t)h->hcfg.qrec_dw;
  hd.car_slots = (uint32_t)h->hcfg.car_slots;
  hd.cfg_hash = cfg_hash(h->hcfg);
  memcpy(p, &hd, sizeof hd);
  uint64_t off = sizeof hd;
  for (const auto& s : v) {
    PgtgSectionEntry e{s.id, 0, s.bytes};
    memcpy(p + off, &e, sizeof e);
    off += sizeof e;
  }
  for (const auto& s : v) {
    off = (off + 15) & ~15ull;
    HIPCHK(h, hipMemcpy(p + off, s.ptr, s.bytes, hipMemcpyDeviceToHost));
    off += s.bytes;
  }
  return PGTG_OK;
}

int pgtg_load_state(pgtg_handle* h, const void* buf, uint64_t bytes) {
  if (!h || !buf) return PGTG_E_INVALID;
  const auto v = state_sections(h);
  const uint8_t* p = static_cast<const uint8_t*>(buf);
  PgtgStateHeader hd;
  if (bytes < sizeof hd) return fail(h, PGTG_E_INVALID, "pgtg_load_state: truncated state");
  memcpy(&hd, p, sizeof hd);
  if (memcmp(hd.magic, "PGTS", 4) != 0 || hd.version != kStateVersion)
    return fail(h, PGTG_E_INVALID, "pgtg_load_state: not a state blob of this version");
  if (hd.n != h->n || hd.n_sections != v.size() || hd.nt != (uint32_t)h->hcfg.nt ||
      hd.car_cap != (uint32_t)h->hcfg.car_cap || hd.plan_stride != (uint32_t)h->hcfg.plan_stride ||
      hd.max_spawners != (uint32_t)h->hcfg.max_spawners || hd.vis_words != (uint32_t)h->hcfg.vis_words ||
      hd.qrec_dw != (uint32_t)h->hcfg.qrec_dw || hd.car_slots != (uint32_t)h->hcfg.car_slots ||
      bytes < state_blob_bytes(v))
    return fail(h, PGTG_E_INVALID, "pgtg_load_state: the state was dumped from a handle of another shape");
  if (hd.cfg_hash != cfg_hash(h->hcfg))
    return fail(h, PGTG_E_INVALID, "pgtg_load_state: the state was dumped from a handle of another configuration");
  uint64_t off = sizeof hd;
  for (const auto& s : v) {
    PgtgSectionEntry e;
    memcpy(&e, p + off, sizeof e);
    off += sizeof e;
    if (e.id != s.id || e.bytes != s.bytes) return fail(h, PGTG_E_INVALID, "pgtg_load_state: section table mismatch");
  }
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  for (const auto& s : v) {
    off = (off + 15) & ~15ull;
    HIPCHK(h, hipMemcpy(s.ptr, p + off, s.bytes, hipMemcpyHostToDevice));
    off += s.bytes;
  }
  if (h->S.tr_count) HIPCHK(h, hipMemset(h->S.tr_count, 0, 2 * sizeof(uint32_t)));
  if (h->S.qctr) HIPCHK(h, hipMemset(h->S.qctr, 0, kQctrWords * sizeof(uint32_t)));  // (dumped with full rings)
  return PGTG_OK;
}

// PGTGEnv.set_to_state (environment.py:1301-1342) for env `env`: position, velocity and flat tire,
// then the car list replaced by `cars` (patience and delay 0, like the reference's fresh Car
// objects); the next car id becomes the last car's id + 1 when the list is non-empty.  Map, RNG
// streams, termination and subgoals are untouched.  n_cars <= 0: no cars.
int pgtg_set_to_state(pgtg_handle* h, uint64_t env, int32_t x, int32_t y, int32_t vx, int32_t vy, int32_t flat_tire,
                      const PgtgCar* cars, int32_t n_cars) {
  if (!h || env >= h->n || (n_cars > 0 && !cars)) return PGTG_E_INVALID;
  if (abs(vx) > 30000 || abs(vy) > 30000 || abs(x) > 30000 || abs(y) > 30000)
    return fail(h, PGTG_E_UNSUPPORTED, "position/velocity outside the 16-bit state range");
  const DevCfg& c = h->hcfg;
  if (n_cars > 0 && !c.need_car) return fail(h, PGTG_E_UNSUPPORTED, "create the handle with min_car_capacity > 0 or traffic");
  if (n_cars > c.car_cap) return fail(h, PGTG_E_UNSUPPORTED, "more cars than the handle's car capacity");
  for (int k = 0; k < n_cars; k++) {
    const PgtgCar& q = cars[k];
    if (q.x < 0 || q.y < 0 || q.x >= c.W || q.y >= c.H || q.route < 0 || q.route >= 20 || q.profile < 0 || q.profile >= 5)
      return fail(h, PGTG_E_INVALID, "car outside the map or bad route/profile");
  }
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  EnvRec r;
  HIPCHK(h, hipMemcpy(&r, h->S.rec + env, sizeof r, hipMemcpyDeviceToHost));
  r.a.x = ((uint32_t)x & 0xffffu) | ((uint32_t)y << 16);
  r.a.y = ((uint32_t)vx & 0xffffu) | ((uint32_t)vy << 16);
  uint32_t flags = (r.a.z >> 16) & 0xfu;
  flags = flat_tire ? (flags | kFlagFlatTire) : (flags & ~kFlagFlatTire);
  r.a.z = (r.a.z & 0xfff0ffffu) | (flags << 16);
  HIPCHK(h, hipMemcpy(h->S.rec + env, &r, sizeof r, hipMemcpyHostToDevice));
  if (c.need_car) {
    uint4 t;
    if (int rc = read_traf(h, env, &t)) return rc;
    std::vector<PgtgCar> v;
    for (int k = 0; k < n_cars; k++) v.push_back(PgtgCar{cars[k].id, cars[k].x, cars[k].y, cars[k].route, cars[k].profile, 0, 0});
    if (int rc = host_write_cars(h, env, t, v, n_cars > 0 ? (uint32_t)cars[n_cars - 1].id + 1u : t.y)) return rc;
  }
  return PGTG_OK;
}

int pgtg_car_digest(pgtg_handle* h, uint64_t* out_dev) {
  if (!h || !out_dev) return PGTG_E_INVALID;
  if (!h->hcfg.need_car) return fail(h, PGTG_E_UNSUPPORTED, "pgtg_car_digest: the handle has no traffic");
  HIPCHK(h, hipSetDevice(h->device));
  hipLaunchKernelGGL(k_car_digest, dim3((unsigned)((h->n + 255) / 256)), dim3(256), 0, h->stream, h->S, out_dev);
  HIPCHK(h, hipGetLastError());
  return PGTG_OK;
}

int pgtg_get_counters(pgtg_handle* h, uint64_t* env_steps, uint64_t* episodes) {
  if (!h) return PGTG_E_INVALID;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  unsigned long long c[2];
  HIPCHK(h, hipMemcpy(c, h->S.counters, sizeof c, hipMemcpyDeviceToHost));
  if (env_steps) *env_steps = c[0];
  if (episodes) *episodes = c[1];
  return PGTG_OK;
}

int pgtg_get_queue_maps(pgtg_handle* h, uint64_t* maps) {
  if (!h || !maps) return PGTG_E_INVALID;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  unsigned long long c[3];
  HIPCHK(h, hipMemcpy(c, h->S.counters, sizeof c, hipMemcpyDeviceToHost));
  *maps = c[2];
  return PGTG_OK;
}

int pgtg_set_flat_outputs(pgtg_handle* h, const int32_t* order, int32_t n_order, int32_t dtype, void* flat_dev,
                          void* final_flat_dev) {
  if (!h) return PGTG_E_INVALID;
  h->flat_dst = h->final_flat_dst = nullptr;
  if (!flat_dev && !final_flat_dev) return PGTG_OK;
  const DevCfg& c = h->hcfg;
  const PgtgOutputs& o = h->out;
  if (dtype != 0 && dtype != 1) return fail(h, PGTG_E_INVALID, "flat dtype: 0 float32, 1 int8");
  if (!order || n_order != c.n_channels) return fail(h, PGTG_E_INVALID, "flat order: one entry per channel");
  uint64_t seen[2] = {0, 0};
  for (int k = 0; k < n_order; k++) {
    if (order[k] < 0 || order[k] >= n_order || ((seen[order[k] >> 6] >> (order[k] & 63)) & 1u))
      return fail(h, PGTG_E_INVALID, "flat order: not a permutation of the channels");
    seen[order[k] >> 6] |= 1ull << (order[k] & 63);
  }
  if (c.sliding && c.ss >= 9)  // gymnasium's flatten of MultiDiscrete([9, 9]) indexes past its 18 entries
    return fail(h, PGTG_E_UNSUPPORTED, "position (s, s) of a sliding window of size >= 9 is outside MultiDiscrete([9, 9])");
  if (flat_dev && (!o.obs || !o.position || !o.velocity || (c.next_subgoal && !o.next_subgoal)))
    return fail(h, PGTG_E_INVALID, "flat rows need the obs, position, velocity (and next_subgoal) outputs");
  if (final_flat_dev && (!o.final_obs || !o.final_position || !o.final_velocity || !o.terminated || !o.truncated ||
                         (c.next_subgoal && !o.final_next_subgoal)))
    return fail(h, PGTG_E_INVALID, "terminal flat rows need the final_* and terminated/truncated outputs");
  if (((uintptr_t)flat_dev | (uintptr_t)final_flat_dev) & 15u) return fail(h, PGTG_E_INVALID, "flat rows: 16-byte aligned buffers");
  FlatArgs& a = h->flat;
  a.n = h->n;
  a.w2 = c.win * c.win;
  a.OB = c.obs_bytes;
  a.cw2 = c.n_channels * a.w2;
  a.nsd_on = c.next_subgoal ? 1 : 0;
  a.D = a.cw2 + (a.nsd_on ? 9 : 0) + 20;
  for (int k = 0; k < n_order; k++) a.order[k] = (uint8_t)order[k];
  h->flat_dtype = dtype;
  h->flat_dst = flat_dev;
  h->final_flat_dst = final_flat_dev;
  return PGTG_OK;
}

int pgtg_set_flat_scalars(pgtg_handle* h, float* reward_f32_dev, uint8_t* dones_dev, uint8_t* truncated_only_dev) {
  if (!h) return PGTG_E_INVALID;
  h->flat_rew32 = nullptr;
  h->flat_dones = h->flat_tonly = nullptr;
  if (!reward_f32_dev && !dones_dev && !truncated_only_dev) return PGTG_OK;
  if (!reward_f32_dev || !dones_dev || !truncated_only_dev)
    return fail(h, PGTG_E_INVALID, "flat scalars: all three buffers or none");
  if (!h->out.reward || !h->out.terminated || !h->out.truncated)
    return fail(h, PGTG_E_INVALID, "flat scalars need the reward, terminated and truncated outputs");
  h->flat_rew32 = reward_f32_dev;
  h->flat_dones = dones_dev;
  h->flat_tonly = truncated_only_dev;
  return PGTG_OK;
}

int pgtg_get_queue_overflow(pgtg_handle* h, uint64_t* served) {
  if (!h || !served) return PGTG_E_INVALID;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  unsigned long long c[4];
  HIPCHK(h, hipMemcpy(c, h->S.counters, sizeof c, hipMemcpyDeviceToHost));
  *served = c[3];
  return PGTG_OK;
}

int pgtg_error_count(pgtg_handle* h, uint64_t* n_errors, int32_t* first_code) {
  if (!h) return PGTG_E_INVALID;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  std::vector<uint8_t> e(h->n);
  HIPCHK(h, hipMemcpy(e.data(), h->S.err, h->n, hipMemcpyDeviceToHost));
  uint64_t cnt = 0;
  int first = 0;
  for (uint64_t i = 0; i < h->n; i++)
    if (e[i]) {
      if (!cnt) first = -(int)e[i];
      cnt++;
    }
  if (n_errors) *n_errors = cnt;
  if (first_code) *first_code = first;
  return PGTG_OK;
}

#ifdef PGTG_STAMPS
// Map generation alone: `active` lanes of every wave run `reps` generate_map + compile_path from
// their env's seed; per-wave cycle sums (generate, compile) land in g_stamps slots 0 and 1.
int pgtg_gen_bench(pgtg_handle* h, int32_t reps, int32_t active, float* ms) {
  if (!h || reps < 1 || active < 1 || active > 64) return PGTG_E_INVALID;
  HIPCHK(h, hipSetDevice(h->device));
  const int pdw = h->L.plan_stride_dw;
  const size_t lds = (size_t)kBlock * pdw * 4;
  const unsigned blocks = (unsigned)((h->n + kBlock - 1) / kBlock);
  hipEvent_t e0, e1;
  HIPCHK(h, hipEventCreate(&e0));
  HIPCHK(h, hipEventCreate(&e1));
  HIPCHK(h, hipEventRecord(e0, h->stream));
  hipLaunchKernelGGL(k_gen_bench, dim3(blocks), dim3(kBlock), lds, h->stream, h->dcfg, h->dtab, h->S, reps, active, pdw);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipEventRecord(e1, h->stream));
  HIPCHK(h, hipEventSynchronize(e1));
  float t = 0.f;
  HIPCHK(h, hipEventElapsedTime(&t, e0, e1));
  if (ms) *ms = t;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return PGTG_OK;
}
int pgtg_read_stamps(uint64_t* out, uint64_t n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
}
#endif

// The best of a few copy shapes (loads in flight per lane x workgroups per CU): the denominator is
// what a plain stream copy reaches on this device, not the spec sheet.
int pgtg_measure_hbm(int32_t device, uint64_t bytes, int32_t reps, double* copy_gbs) {
  if (bytes < 16 * 1024 || reps < 1 || !copy_gbs) return PGTG_E_INVALID;
  if (hipSetDevice(device) != hipSuccess) return PGTG_E_DEVICE;
  const uint64_t n16 = bytes / 16;
  void *a = nullptr, *b = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = PGTG_E_DEVICE;
  int ncu = 256;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
  double best = 0.0;
  if (hipMalloc(&a, n16 * 16) == hipSuccess && hipMalloc(&b, n16 * 16) == hipSuccess &&
      hipMemset(a, 1, n16 * 16) == hipSuccess && hipMemset(b, 2, n16 * 16) == hipSuccess &&
      hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess) {
    rc = PGTG_OK;
    // shapes: loads in flight per lane (1, 4), plain or nontemporal, workgroups per CU (4, 8, 16)
    // or one pass over the buffer (wpc 0: a workgroup per 256 x U chunks)
    for (int shape = 0; shape < 16 && rc == PGTG_OK; shape++) {
      const int U = (shape & 1) ? 4 : 1;
      const bool nt = (shape >> 1) & 1;
      const int wpc = (shape >> 2) == 0 ? 0 : (4 << ((shape >> 2) - 1));
      const uint64_t full = (n16 + 256 * U - 1) / (256 * U);
      const unsigned grid = (unsigned)(wpc ? std::min<uint64_t>((uint64_t)ncu * wpc, full) : std::min<uint64_t>(full, 1u << 30));
      auto pass = [&](int r) {
        const u32x4* src = (const u32x4*)((r & 1) ? b : a);
        u32x4* dst = (u32x4*)((r & 1) ? a : b);
        if (U == 4 && nt) hipLaunchKernelGGL((k_hbm_copy<4, true>), dim3(grid), dim3(256), 0, 0, src, dst, n16);
        else if (U == 4) hipLaunchKernelGGL((k_hbm_copy<4, false>), dim3(grid), dim3(256), 0, 0, src, dst, n16);
        else if (nt) hipLaunchKernelGGL((k_hbm_copy<1, true>), dim3(grid), dim3(256), 0, 0, src, dst, n16);
        else hipLaunchKernelGGL((k_hbm_copy<1, false>), dim3(grid), dim3(256), 0, 0, src, dst, n16);
      };
      pass(0);  // untimed: page-in, clocks
      (void)hipEventRecord(e0, 0);
      for (int r = 0; r < reps; r++) pass(r);
      (void)hipEventRecord(e1, 0);
      float ms = 0.f;
      if (hipGetLastError() != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
          hipEventElapsedTime(&ms, e0, e1) != hipSuccess || !(ms > 0.f)) {
        rc = PGTG_E_DEVICE;
        break;
      }
      best = std::max(best, 2.0 * (double)(n16 * 16) * reps / (ms * 1e-3) / 1e9);  // read + write bytes
    }
  }
  if (rc == PGTG_OK) *copy_gbs = best;
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (a) (void)hipFree(a);
  if (b) (void)hipFree(b);
  return rc;
}

int pgtg_window(const pgtg_handle* h) { return h ? h->hcfg.win : 0; }
uint64_t pgtg_num_envs(const pgtg_handle* h) { return h ? h->n : 0; }
const char* pgtg_step_kernel(const pgtg_handle* h) {
  if (!h) return "";
  const bool big = h->hcfg.nt > kSmallTiles;
  if (h->hcfg.need_car) return big ? "pgtg::k_env<true, true> + pgtg::k_traffic" : "pgtg::k_env<true, false> + pgtg::k_traffic";
  if (h->hcfg.n_rules > 0) return big ? "pgtg::k_env<true, true>" : "pgtg::k_env<true, false>";
  if (h->L.queue && h->q_block == 1) return big ? "pgtg::k_envb<true>" : "pgtg::k_envb<false>";
  if (h->L.queue) return big ? "pgtg::k_envq<true>" : "pgtg::k_envq<false>";
  return big ? "pgtg::k_env<false, true>" : "pgtg::k_env<false, false>";
}

int pgtg_occupancy(const pgtg_handle* h, int32_t* step_blocks_per_cu) {
  if (!h) return PGTG_E_INVALID;
  int nb = 0;
  const void* fn = step_fn(h, MODE_STEP);  // the kernel launch() picks
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kBlock, h->lds) != hipSuccess) return PGTG_E_DEVICE;
  if (step_blocks_per_cu) *step_blocks_per_cu = nb;
  return PGTG_OK;
}

int pgtg_launch_info(const pgtg_handle* h, int32_t* envs_per_block, int32_t* lds_bytes) {
  if (!h) return PGTG_E_INVALID;
  if (envs_per_block) *envs_per_block = h->L.envs;
  if (lds_bytes) *lds_bytes = (int32_t)(h->lds + (h->L.queue ? kTabHead : sizeof(Tables)));  // + the static table copy
  return PGTG_OK;
}
const char* pgtg_last_error(const pgtg_handle* h) { return h ? h->err.c_str() : g_create_err.c_str(); }

int pgtg_enable_timing(pgtg_handle* h, int32_t on) {
  if (!h) return PGTG_E_INVALID;
  h->timing = on < 0 ? 0 : on;
  h->step_launches = 0;
  return PGTG_OK;
}

int pgtg_timing_read(pgtg_handle* h, double* total_ms, uint64_t* launches, int32_t reset) {
  if (!h) return PGTG_E_INVALID;
  HIPCHK(h, hipSetDevice(h->device));
  int rc = timing_flush(h);
  if (rc) return rc;
  if (total_ms) *total_ms = h->acc_ms;
  if (launches) *launches = h->acc_n;
  if (reset) {
    h->acc_ms = 0.0;
    h->acc_n = 0;
  }
  return PGTG_OK;
}

}  // extern "C"
