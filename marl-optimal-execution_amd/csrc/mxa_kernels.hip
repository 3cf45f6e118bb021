// mxa_kernels.hip — MI355X (gfx950) kernels of the vectorised ABIDES market step.
//
// Execution model: ONE wavefront (64 lanes) simulates ONE independent market (env)
// end to end — the reference's Kernel.runner loop (Kernel.py:190-292) with its
// agents.  Control flow is wave-uniform (every branch of every agent handler is taken
// by the whole wave, so there is no divergence between envs); the 64 lanes are used as
// a SIMD engine for the data-parallel parts of each event:
//   * event queue (heapq of Kernel.messages): QCAP slots in LDS; every lane owns
//     SQ slots and caches their minimum (t, recipient, type, seq) key in VGPRs, so a
//     pop is one 64-lane lexicographic min-reduction + one rescan by the winning lane;
//   * limit order book (util/OrderBook.py): a pool of OCAP resting orders held in VGPRs
//     (SO slots per lane); best price, level volume and FIFO head (price-time priority)
//     are wave min/max/sum reductions, so insert/cancel/match never walk a list;
//   * MT19937 twist (numpy legacy RandomState): cooperative over the 64 lanes;
//   * agent state: the recipient's 512-byte record is loaded with ONE coalesced
//     64-lane load per event and its fields read with v_readlane.
// Everything that is not in LDS/VGPRs is one contiguous per-env HBM block (mxa_layout.h).
//
// Arithmetic follows the reference bit for bit: numpy-legacy MT19937 and distributions,
// glibc log/exp/pow (glibc_math.h), Python round-half-even / truncation, pandas ns
// truncation.  Compiled with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>
// single-configuration variant builds (-DMXA_ONLY_RMSC03 [-DMXA_ONLY_CFG=<id>]) carry the
// GymKernel step kernel only for the GymKernel configurations
#if defined(MXA_ONLY_RMSC03) && !(defined(MXA_ONLY_CFG) && (MXA_ONLY_CFG == 3 || MXA_ONLY_CFG == 4))
#define MXA_NO_GYM
#endif

#include "../../include/mxa.h"
#include "glibc_math.h"
#include "mxa_layout.h"
#include "mxa_config.h"


typedef uint64_t u64;
typedef int64_t i64;
typedef uint32_t u32;
typedef int32_t i32;

#ifdef MXA_DEV_NOINLINE  // diagnostics build: every engine helper a real call
#define DEV __device__ __attribute__((noinline))
#else
#define DEV __device__ __forceinline__
#endif
#define FNV_OFF 0xCBF29CE484222325ull
#define FNV_PRIME 0x100000001B3ull
#define KEY_EMPTY 0xFFFFFFFFFFFFFFFFull
#define NS_SEC 1000000000LL

namespace mxa {

DEV int laneid() { return (int)__lane_id(); }
DEV u32 rdl(u32 v, int l) { return (u32)__builtin_amdgcn_readlane((int)v, l); }
DEV i32 rdli(i32 v, int l) { return __builtin_amdgcn_readlane(v, l); }
// one memory round trip for a wave of independent words: each lane's address is selected with
// VALU ops and ONE load is issued (lanes with ok false load nothing).  A chain of per-lane
// `if (lane == k) v = A[..]; else if ...` arms instead became one load and one wait per arm
DEV i32 gather1(const i32* a, bool ok) {
  i32 v = 0;
  if (ok) v = *a;
  return v;
}
// the i64 whose lo / hi words a gather put in lanes l / l + 1
DEV i64 rdl64g(i32 g, int l) { return (i64)(((u64)(u32)__builtin_amdgcn_readlane(g, l + 1) << 32) | (u32)__builtin_amdgcn_readlane(g, l)); }
DEV u64 rdl64(u64 v, int l) {
  return ((u64)rdl((u32)(v >> 32), l) << 32) | rdl((u32)v, l);
}
DEV double rdl_d(double v, int l) { return __builtin_bit_cast(double, rdl64(__builtin_bit_cast(u64, v), l)); }
DEV u64 bal(bool p) { return __ballot(p); }
DEV int ffs64(u64 b) { return __ffsll((unsigned long long)b) - 1; }
// the lowest set bit of a mask known to be non-zero: one s_ff1, without ffs64's zero test
DEV int ctz64(u64 b) { return __builtin_ctzll(b); }
DEV int ffs32(u32 b) { return __ffs(b) - 1; }
DEV u32 sxor(u32 v, int m) { return (u32)__shfl_xor((int)v, m, 64); }
// ---- wave reductions on DPP (row_shr 1/2/4/8 inside 16-lane rows, then row_bcast15/31
// across rows): lane 63 ends with the result, read back with v_readlane.  Every step is a
// VALU op with a DPP source operand — no LDS round trip (ds_swizzle/bpermute).
template <int CTRL, int ROWMASK>
DEV u32 dpp(u32 identity, u32 v) {
  return (u32)__builtin_amdgcn_update_dpp((int)identity, (int)v, CTRL, ROWMASK, 0xf, false);
}
#define MXA_DPP_STEPS(OP, ID, V)                        \
  V = OP(V, dpp<0x111, 0xf>(ID, V));                    \
  V = OP(V, dpp<0x112, 0xf>(ID, V));                    \
  V = OP(V, dpp<0x114, 0xf>(ID, V));                    \
  V = OP(V, dpp<0x118, 0xf>(ID, V));                    \
  V = OP(V, dpp<0x142, 0xa>(ID, V));                    \
  V = OP(V, dpp<0x143, 0xc>(ID, V));
DEV u32 op_minu(u32 a, u32 b) { return a < b ? a : b; }
DEV u32 op_add(u32 a, u32 b) { return a + b; }
DEV u32 op_maxi(u32 a, u32 b) { return (i32)a > (i32)b ? a : b; }
DEV u32 op_mini(u32 a, u32 b) { return (i32)a < (i32)b ? a : b; }
DEV i32 wmax_i32(i32 x) {
  u32 v = (u32)x;
  MXA_DPP_STEPS(op_maxi, 0x80000000u, v)
  return (i32)rdl(v, 63);
}
DEV i32 wmin_i32(i32 x) {
  u32 v = (u32)x;
  MXA_DPP_STEPS(op_mini, 0x7fffffffu, v)
  return (i32)rdl(v, 63);
}
DEV u32 wmin_u32(u32 v) {
  MXA_DPP_STEPS(op_minu, 0xffffffffu, v)
  return rdl(v, 63);
}
DEV u64 wmin_u64(u64 v) {  // two 32-bit wave-mins (high word, then the low word among its ties)
  const u32 hi = wmin_u32((u32)(v >> 32));
  const u32 lo = wmin_u32((u32)(v >> 32) == hi ? (u32)v : 0xFFFFFFFFu);
  return ((u64)hi << 32) | lo;
}
// 64-bit sum: reduce the two 32-bit halves separately (each fits: |parts| < 2^32 * 64)
DEV i64 wsum_i64(i64 x) {
  // values summed here are non-negative quantities < 2^31; sum the low and high 32 bits as
  // 64-bit-safe u32 pairs would need carries, so use two 32-bit sums of 16-bit splits
  u32 lo = (u32)((u64)x & 0xFFFFu), hi = (u32)((u64)x >> 16);
  MXA_DPP_STEPS(op_add, 0u, lo)
  MXA_DPP_STEPS(op_add, 0u, hi)
  return (i64)(((u64)rdl(hi, 63) << 16) + rdl(lo, 63));
}
DEV u32 wsum_u32(u32 v) {
  MXA_DPP_STEPS(op_add, 0u, v)
  return rdl(v, 63);
}
// inclusive prefix sum over the lanes (lane l gets v_0 + ... + v_l)
DEV u32 wscan_u32(u32 v) {
  const int l = laneid();
  for (int d = 1; d < 64; d <<= 1) {
    const u32 o = (u32)__shfl_up((int)v, d, 64);
    v += l >= d ? o : 0u;
  }
  return v;
}
// lexicographic (key64, seq32) min over the wave; returns in k/s (uniform)
DEV void wmin_key(u64& k, u32& s) {
  u32 kh = (u32)(k >> 32), kl = (u32)k;
#define MXA_KSTEP(CTRL, RM)                                                   \
  {                                                                           \
    u32 th = dpp<CTRL, RM>(0xffffffffu, kh), tl = dpp<CTRL, RM>(0xffffffffu, kl); \
    u32 ts = dpp<CTRL, RM>(0xffffffffu, s);                                    \
    bool lt = th < kh || (th == kh && (tl < kl || (tl == kl && ts < s)));      \
    kh = lt ? th : kh;                                                        \
    kl = lt ? tl : kl;                                                        \
    s = lt ? ts : s;                                                          \
  }
  MXA_KSTEP(0x111, 0xf)
  MXA_KSTEP(0x112, 0xf)
  MXA_KSTEP(0x114, 0xf)
  MXA_KSTEP(0x118, 0xf)
  MXA_KSTEP(0x142, 0xa)
  MXA_KSTEP(0x143, 0xc)
#undef MXA_KSTEP
  k = ((u64)rdl(kh, 63) << 32) | rdl(kl, 63);
  s = rdl(s, 63);
}
DEV void wfence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }
DEV i64 py_round(double x) { return (i64)__builtin_rint(x); }
DEV double as_d(u64 x) { return __builtin_bit_cast(double, x); }
DEV u64 as_u(double x) { return __builtin_bit_cast(u64, x); }

// ------------------------------------------------------------------------------------
// numpy legacy RandomState (numpy/random/src/mt19937, distributions/legacy)
// ------------------------------------------------------------------------------------
// Stream storage: TWO 624-word MT blocks (double buffer, 1280 words per stream).  Output
// index p lives in block p/624 at word (p/624 & 1)*624 + p%624; block b is generated from
// block b-1 (mt19937_gen) into the other half.  The run kernel keeps one block of look-ahead
// materialized at every event boundary (rs_maint, one code instance in the event loop), so
// the draw sites inside the agent handlers never contain the twist; the build kernel
// (BUILD = true) materializes blocks on demand instead.
#define LDSP __attribute__((address_space(3)))
#define GLBP __attribute__((address_space(1)))
template <bool BUILD>
struct RSt {
  u32* key;
  i32 p;      // absolute output index since seeding (first output: p = 624)
  i32 m;      // highest materialized block
  i32 hasg;   // bit0: cached second gauss (legacy_gauss); bit1: look-ahead overrun
  double gauss;
  // run kernel, global streams G/O/K/L: a 64-word window of the stream's outputs in LDS (words
  // lw0 .. lw0 + lwn - 1, untempered), so a draw is an LDS read instead of an HBM round trip;
  // lw == nullptr: draws read the MT block in HBM (agent streams, the build kernel)
  LDSP u32* lw;
  i32 lw0, lwn;
};

// materialize block b (>= 1) from block b-1, cooperatively over the wave in the four
// dependency phases of mt19937_gen: [0,227) reads A only; [227,454) reads B[i-227] of
// phase 1; [454,623) reads B[227..396); 623 reads B[0], B[396].
DEV void mt_gen_block(u32* key, int b) {
  const int lane = laneid();
  const u32* A = key + ((b - 1) & 1) * MXA_MT_N;
  u32* B = key + (b & 1) * MXA_MT_N;
  for (int i = lane; i < 227; i += 64) {
    u32 y = (A[i] & 0x80000000u) | (A[i + 1] & 0x7fffffffu);
    B[i] = A[i + 397] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
  }
  wfence();
  for (int i = 227 + lane; i < 454; i += 64) {
    u32 y = (A[i] & 0x80000000u) | (A[i + 1] & 0x7fffffffu);
    B[i] = B[i - 227] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
  }
  wfence();
  for (int i = 454 + lane; i < 623; i += 64) {
    u32 y = (A[i] & 0x80000000u) | (A[i + 1] & 0x7fffffffu);
    B[i] = B[i - 227] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
  }
  wfence();
  if (lane == 0) {
    u32 y = (A[623] & 0x80000000u) | (B[0] & 0x7fffffffu);
    B[623] = B[396] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
  }
  wfence();
}

// the same block in ONE memory round trip (build kernel): lane L computes the words L + 64k of
// each dependency phase, and a phase's recurrence term B[i - 227] is the word the same lane and
// k computed in the phase before, so it stays in a register; every A word is loaded up front and
// B[623] takes B[396] and B[0] by readlane.  One store pass, one fence.
DEV u32 mt_mix(u32 a0, u32 a1) {
  const u32 y = (a0 & 0x80000000u) | (a1 & 0x7fffffffu);
  return (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
}
// two streams' blocks in the same round trip (both streams' A words loaded before either is
// stored: one in-order vmcnt covers loads and stores); `two` false: the first only
DEV void mt_gen_pair(u32* k1, int b1, u32* k2, int b2, bool two) {
  const int lane = laneid();
  u32* key[2] = {k1, k2};
  const int bb[2] = {b1, b2};
  u32 a0[2][11], a1[2][11], a3[2][4], a623[2];
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const u32* A = key[q] + ((bb[q] - 1) & 1) * MXA_MT_N;
    const bool on = q == 0 || two;
#pragma unroll
    for (int k = 0; k < 11; k++) {  // k 0-3: phase 1, 4-7: phase 2, 8-10: phase 3
      const int ph = k < 4 ? 0 : k < 8 ? 1 : 2, kk = k - 4 * ph;
      const int i = 227 * ph + lane + 64 * kk;
      const bool ok = on && kk * 64 + lane < (ph < 2 ? 227 : 169);
      a0[q][k] = ok ? A[i] : 0u;
      a1[q][k] = ok ? A[i + 1] : 0u;
      if (ph == 0) a3[q][k] = ok ? A[i + 397] : 0u;
    }
    a623[q] = on ? A[623] : 0u;
  }
#pragma unroll
  for (int q = 0; q < 2; q++) {
    if (q == 1 && !two) break;
    u32* B = key[q] + (bb[q] & 1) * MXA_MT_N;
    u32 y[11];
#pragma unroll
    for (int k = 0; k < 4; k++) y[k] = a3[q][k] ^ mt_mix(a0[q][k], a1[q][k]);
#pragma unroll
    for (int k = 4; k < 11; k++) y[k] = y[k - 4] ^ mt_mix(a0[q][k], a1[q][k]);
    const u32 b396 = rdl(y[6], 41), b0 = rdl(y[0], 0);  // 396 = 227 + 41 + 64 * 2; 0 = lane 0, k 0
#pragma unroll
    for (int k = 0; k < 11; k++) {
      const int ph = k < 4 ? 0 : k < 8 ? 1 : 2, kk = k - 4 * ph;
      if (kk * 64 + lane < (ph < 2 ? 227 : 169)) B[227 * ph + lane + 64 * kk] = y[k];
    }
    if (lane == 0) B[623] = b396 ^ mt_mix(a623[q], b0);
  }
  wfence();
}
DEV void mt_gen_block_batched(u32* key, int b) { mt_gen_pair(key, b, key, b, false); }

// the build kernel's block generation (the run kernel keeps mt_gen_block: a register-staged
// form inlined into the event loop cost every configuration 1-3 %)
#ifndef MXA_BUILD_BATCHED_GEN
#define MXA_BUILD_BATCHED_GEN 1
#endif
DEV void mt_gen_build(u32* key, int b) {
  if constexpr (MXA_BUILD_BATCHED_GEN) mt_gen_block_batched(key, b);
  else mt_gen_block(key, b);
}

// init_genrand (numpy _legacy_seeding with an int) into block 0: every lane runs the
// recurrence, lane (i % 64) stores word i.
DEV void mt_seed(u32* key, u32 s) {
  const int lane = laneid();
  for (int i = 0; i < MXA_MT_N; i++) {
    if ((i & 63) == lane) key[i] = s;
    s = 1812433253u * (s ^ (s >> 30)) + (u32)i + 1u;
  }
  wfence();
}

// the build kernel's draws through LDS windows too (one coalesced 64-word fill instead of a
// dependent load per word): G/O/K/L their run-kernel windows, an agent stream the L window (the
// build never draws from L)
#ifndef MXA_BUILD_WINDOWS
#define MXA_BUILD_WINDOWS 1
#endif
// refill a stream window from position p: lane i loads output word p + i if its block is in
// the double buffer (materialized and not yet overwritten); the window ends at the first word
// that is not, and an empty window is the look-ahead overrun
template <bool B>
DEV void rs_fill(RSt<B>& r) {
  const int lane = laneid();
  const int q = r.p + lane, b = q / MXA_MT_N;
  const bool ok = b <= r.m && b >= r.m - 1;
  u32 v = 0;
  if (ok) v = r.key[(b & 1) * MXA_MT_N + (q - b * MXA_MT_N)];
  r.lw[lane] = v;
  const u64 okb = __ballot(ok);
  r.lwn = ~okb == 0 ? 64 : __ffsll((unsigned long long)~okb) - 1;
  r.lw0 = r.p;
  if (r.lwn == 0) r.hasg |= 2;
  __threadfence_block();
}
template <bool B>
DEV u32 rs_u32(RSt<B>& r) {
  if constexpr (!B || MXA_BUILD_WINDOWS) {
    if (r.lw) {
      u32 off = (u32)(r.p - r.lw0);
      if (off >= (u32)r.lwn) {
        if constexpr (B) {  // the build materializes blocks as it draws
          const int blk = r.p / MXA_MT_N;
          while (r.m < blk) {
            mt_gen_build(r.key, r.m + 1);
            r.m++;
          }
        }
        rs_fill(r);
        off = 0;
      }
      u32 y = r.lw[off];
      r.p++;
      y ^= (y >> 11);
      y ^= (y << 7) & 0x9d2c5680u;
      y ^= (y << 15) & 0xefc60000u;
      y ^= (y >> 18);
      return y;
    }
  }
  int blk = r.p / MXA_MT_N;
  if (B) {
    while (r.m < blk) {
      mt_gen_build(r.key, r.m + 1);
      r.m++;
    }
  } else if (blk > r.m) {
    r.hasg |= 2;  // more than one block of draws inside one event: flagged, never silent
  }
  u32 y = r.key[(blk & 1) * MXA_MT_N + (r.p - blk * MXA_MT_N)];
  r.p++;
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}
template <bool B>
DEV double rs_double(RSt<B>& r) {
  i32 a = (i32)(rs_u32(r) >> 5);
  i32 b = (i32)(rs_u32(r) >> 6);
  return ((double)a * 67108864.0 + (double)b) / 9007199254740992.0;
}
template <bool B>
DEV i64 rs_randint(RSt<B>& r, i64 lo, i64 hi) {
  u64 rng = (u64)(hi - lo - 1);
  if (rng == 0) return lo;
  if (rng == 0xFFFFFFFFull) return lo + (i64)rs_u32(r);
  u32 mask = (u32)rng;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
  u32 v;
  do {
    v = rs_u32(r) & mask;
  } while (v > (u32)rng);
  return lo + (i64)v;
}
// the run kernel's normal draws (numpy legacy_gauss).  A wave-parallel form (16 polar
// candidates across the wave in one load round trip) was built, checked bit-exact and measured in
// round 4: neutral on sparse_zi_1000 (721.9 vs 722 ms) and rmsc02's run kernel grew (62.1 k vs
// 54.4 k instructions); removed in round 5
template <bool B>
DEV double rs_gauss(RSt<B>& r) {
  return rs_gauss_serial(r);
}
template <bool B>
DEV double rs_gauss_serial(RSt<B>& r) {
  if (r.hasg & 1) {
    double t = r.gauss;
    r.hasg &= ~1;
    r.gauss = 0.0;
    return t;
  }
  double f, x1, x2, r2;
  do {
    x1 = 2.0 * rs_double(r) - 1.0;
    x2 = 2.0 * rs_double(r) - 1.0;
    r2 = x1 * x1 + x2 * x2;
  } while (r2 >= 1.0 || r2 == 0.0);
  f = __builtin_sqrt(-2.0 * gm_log(r2) / r2);
  r.gauss = f * x1;
  r.hasg |= 1;
  return f * x2;
}
template <bool B>
DEV double rs_normal(RSt<B>& r, double loc, double scale) { return loc + scale * rs_gauss(r); }
template <bool B>
DEV double rs_exponential(RSt<B>& r, double scale) { return scale * -gm_log(1.0 - rs_double(r)); }
template <bool B>
DEV double rs_uniform(RSt<B>& r, double lo, double hi) { return lo + (hi - lo) * rs_double(r); }
// advance by k outputs without tempering them (build kernel only)
DEV void rs_skip_words(RSt<true>& r, i64 k) {
  i64 target = (i64)r.p + k;
  while ((i64)r.m < target / MXA_MT_N) {
    mt_gen_build(r.key, r.m + 1);
    r.m++;
  }
  r.p = (i32)target;
}
// keep one block of look-ahead materialized (called at event boundaries)
// agent streams keep MXA_AGENT_LA words of look-ahead materialized instead of a whole block:
// an agent event draws a few dozen words at most (the MarketMakerAgent's ladder sizes), and most
// agents of the wide configurations draw a few words per session, so their second block is never
// built.  A draw past the look-ahead is still ERR_RNG_OVERRUN, never a silent value.
#ifndef MXA_MAINT_LANES
#define MXA_MAINT_LANES 1
#endif
#ifndef MXA_WAKE_LANES
#define MXA_WAKE_LANES 1
#endif
#ifndef MXA_ZI_THETA_LANES
#define MXA_ZI_THETA_LANES 1
#endif
#ifndef MXA_SEED_TILE
#define MXA_SEED_TILE 1
#endif
#ifndef MXA_AGENT_LA
#define MXA_AGENT_LA 256
#endif
template <bool B>
DEV void rs_maint(RSt<B>& r, int la = MXA_MT_N) {
  while (r.m < (r.p + la) / MXA_MT_N) {
    if constexpr (B) mt_gen_build(r.key, r.m + 1);
    else mt_gen_block(r.key, r.m + 1);
    r.m++;
  }
}

// ------------------------------------------------------------------------------------
// message payload: w0 = kind | buy<<6 | closed<<7 | dfloat<<8 | nb<<9 | na<<10 | hasdata<<11
// | agent<<16, w1..w5 fields; w6/w7 only in the marketreplay config (24 B / 32 B queued)
// ------------------------------------------------------------------------------------
struct Msg {
  u32 w[8];
};
DEV u32 m_kind(const Msg& m) { return m.w[0] & 63u; }
DEV int m_buy(const Msg& m) { return (m.w[0] >> 6) & 1; }
DEV int m_closed(const Msg& m) { return (m.w[0] >> 7) & 1; }
DEV int m_dfloat(const Msg& m) { return (m.w[0] >> 8) & 1; }
DEV int m_nb(const Msg& m) { return (m.w[0] >> 9) & 1; }
DEV int m_na(const Msg& m) { return (m.w[0] >> 10) & 1; }
DEV int m_hasdata(const Msg& m) { return (m.w[0] >> 11) & 1; }
DEV i32 m_agent(const Msg& m) { return (i32)(m.w[0] >> 16); }
DEV i64 m_i64(const Msg& m, int i) { return (i64)(((u64)m.w[i + 1] << 32) | m.w[i]); }
DEV u32 msel(const Msg& m, int i) {
  u32 v = m.w[0];
  v = i == 1 ? m.w[1] : v;
  v = i == 2 ? m.w[2] : v;
  v = i == 3 ? m.w[3] : v;
  v = i == 4 ? m.w[4] : v;
  v = i == 5 ? m.w[5] : v;
  v = i == 6 ? m.w[6] : v;
  v = i == 7 ? m.w[7] : v;
  return v;
}
DEV Msg msg_make(u32 kind, i32 agent) {
  Msg m;
  m.w[0] = kind | ((u32)agent << 16);
  m.w[1] = m.w[2] = m.w[3] = m.w[4] = m.w[5] = m.w[6] = m.w[7] = 0;
  return m;
}
#define MF_NOT_SAME (1u << 12)  // MODIFY_ORDER whose new order carries another id
// queue-internal (never part of a message's content): another member of the same batched push
// (q_push_lanes) follows this one with the same key and the next seq, so the pop of this event
// starts an event run (Eng::run_event)
#define MF_RUN (1u << 13)
DEV Msg msg_order(u32 kind, i32 oid, i32 agent, int is_buy, i32 qty, i32 price, i32 fill) {
  Msg m = msg_make(kind, agent);
  m.w[0] |= (u32)is_buy << 6;
  m.w[1] = (u32)oid;
  m.w[2] = (u32)qty;
  m.w[3] = (u32)price;
  m.w[4] = (u32)fill;
  return m;
}

// the 10-word parity record (tests/golden/gen_fixtures.py encode()).  WIDE: spread replies
// carry level counts (w6/w7 >> 20) instead of the 0/1 flags (depth-500 queries)
struct Rec {  // named scalars, not an array: a private i64[10] is promoted to a VGPR vector
  i64 t, rcp, type, kind, f0, f1, f2, f3, f4, f5;
  DEV i64 at(int i) const {
    switch (i) {
    case 0: return t; case 1: return rcp; case 2: return type; case 3: return kind;
    case 4: return f0; case 5: return f1; case 6: return f2; case 7: return f3;
    case 8: return f4; default: return f5;
    }
  }
};
template <bool WIDE, bool MDK, int KSH>
DEV Rec encode(u64 key, const Msg& m) {
  Rec r;
  r.t = (i64)(key >> KSH);
  r.rcp = (i64)((key >> 2) & MXA_KEY_RCP);
  i32 type = (i32)(key & 3);
  r.type = type;
  r.f0 = r.f1 = r.f2 = r.f3 = r.f4 = r.f5 = 0;
  u32 k = m_kind(m);
  if (type != MT_MESSAGE) {
    r.kind = type == MT_WAKEUP ? MK_WAKEUP : MK_KCANCEL;
    return r;
  }
  r.kind = k;
  switch (k) {
  case MK_WHEN_OPEN_REQ: case MK_WHEN_CLOSE_REQ: case MK_LAST_REQ:
    r.f0 = m_agent(m);
    break;
  case MK_WHEN_OPEN: case MK_WHEN_CLOSE:
    r.f0 = m_i64(m, 1);
    break;
  case MK_SPREAD_REQ:
    r.f0 = m_agent(m);
    r.f1 = (i32)m.w[1];
    break;
  case MK_SPREAD: {
    int nb = WIDE ? (int)(m.w[6] >> 20) : m_nb(m), na = WIDE ? (int)(m.w[7] >> 20) : m_na(m);
    i64 d = (i32)m.w[5];
    r.f0 = nb ? (i64)(i32)m.w[1] : -1;
    r.f1 = nb ? (i64)(i32)m.w[2] : 0;
    r.f2 = na ? (i64)(i32)m.w[3] : -1;
    r.f3 = na ? (i64)(i32)m.w[4] : 0;
    r.f4 = !m_hasdata(m) ? -1 : (m_dfloat(m) ? d * 10000 : d);
    r.f5 = (i64)m_closed(m) + 2 * (i64)nb + ((i64)1 << 20) * na;
    break;
  }
  case MK_LAST: {
    i64 d = (i32)m.w[5];
    r.f0 = !m_hasdata(m) ? -1 : (m_dfloat(m) ? d * 10000 : d);
    r.f5 = m_closed(m);
    break;
  }
  case MK_TV_REQ:
    r.f0 = m_agent(m);
    r.f1 = m_i64(m, 1);
    break;
  case MK_TV:
    r.f0 = m_i64(m, 1);
    r.f5 = m_closed(m);
    break;
  case MK_STREAM_REQ:
    r.f0 = m_agent(m);
    r.f1 = (i32)m.w[1];
    break;
  case MK_STREAM:
    r.f0 = (i32)m.w[1];
    r.f5 = m_closed(m);
    break;
  case MK_LIMIT: case MK_ACCEPTED: case MK_CANCELLED: case MK_MODIFY: case MK_MODIFIED:
  case MK_CANCEL: case MK_EXECUTED:
    r.f0 = (i32)m.w[1];
    r.f1 = m_agent(m);
    r.f2 = m_buy(m);
    r.f3 = (k == MK_CANCEL || k == MK_MODIFIED) ? 0 : (i64)(i32)m.w[2];  // (see gen_fixtures)
    r.f4 = (i32)m.w[3];
    if (k == MK_EXECUTED) r.f5 = (i32)m.w[4];
    break;
  default:
    break;
  }
  // market-data kinds only where they exist: extra cases cost the other configurations' event
  // loop registers (the hash path is compiled in even with the hash off)
  if constexpr (MDK) {
    if (k == MK_MARKET_DATA) {  // best levels, last transaction, level counts (w6 = nb | na << 8)
      const int nb = (int)(m.w[6] & 0xFF), na = (int)((m.w[6] >> 8) & 0xFF);
      const i64 d = (i32)m.w[5];
      r.f0 = nb ? (i64)(i32)m.w[1] : -1;
      r.f1 = nb ? (i64)(i32)m.w[2] : 0;
      r.f2 = na ? (i64)(i32)m.w[3] : -1;
      r.f3 = na ? (i64)(i32)m.w[4] : 0;
      r.f4 = m_dfloat(m) ? d * 10000 : d;
      r.f5 = (i64)nb + ((i64)na << 8);
    } else if (k == MK_MD_SUB_REQ) {
      r.f0 = m_agent(m);
      r.f1 = (i32)m.w[1];
      r.f2 = m_i64(m, 2);
    } else if (k == MK_MD_SUB_CANCEL) {
      r.f0 = m_agent(m);
    }
  }
  return r;
}
DEV u64 fnv(u64 h, i64 v) { return (h ^ (u64)v) * FNV_PRIME; }
DEV u64 rec_hash(u64 h, const Rec& r) {
  h = fnv(h, r.t); h = fnv(h, r.rcp); h = fnv(h, r.type); h = fnv(h, r.kind);
  h = fnv(h, r.f0); h = fnv(h, r.f1); h = fnv(h, r.f2); h = fnv(h, r.f3); h = fnv(h, r.f4);
  return fnv(h, r.f5);
}

// ------------------------------------------------------------------------------------
// the engine: one instance per wave (= per env), lives in registers / LDS
// ------------------------------------------------------------------------------------
// uniform view of a value the compiler cannot prove wave-uniform (loads of a wave-uniform
// address): moves it to SGPRs so the arithmetic on it is scalar
DEV i32 U(i32 v) { return __builtin_amdgcn_readfirstlane(v); }
DEV u32 U(u32 v) { return (u32)__builtin_amdgcn_readfirstlane((i32)v); }
DEV i64 U(i64 v) {
  u32 lo = (u32)__builtin_amdgcn_readfirstlane((i32)(u32)(u64)v);
  u32 hi = (u32)__builtin_amdgcn_readfirstlane((i32)(u32)((u64)v >> 32));
  return (i64)(((u64)hi << 32) | lo);
}
#ifdef MXA_PROF
// diagnostics build only: per-phase shader-cycle totals over all envs (tools/prof_phases.py)
__device__ unsigned long long g_mxa_prof[128];
DEV u64 stamp() {
  u64 t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define PROF_T(v) u64 v = stamp()
#define PROF_ADD(b, v) do { u64 _t = stamp(); if (lane == 0) prof[b] += _t - (v); v = _t; } while (0)
#define PROF_CNT(b) do { if (lane == 0) prof[b] += 1; } while (0)
// inclusive function timers (slots 64..95, call counts at +32): nested inside the phases above
#define PROF_IN(v) u64 v = stamp()
#define PROF_OUT(b, v) do { u64 _t = stamp(); if (lane == 0) { prof[b] += _t - (v); prof[(b) + 32] += 1; } } while (0)
struct ProfScope {
  LDSP unsigned long long* p;
  int b, lane;
  unsigned long long t0;
  DEV ProfScope(LDSP unsigned long long* p_, int b_, int l) : p(p_), b(b_), lane(l), t0(stamp()) {}
  DEV ~ProfScope() {
    const unsigned long long t = stamp();
    if (lane == 0) {
      p[b] += t - t0;
      p[b + 32] += 1;
    }
  }
};
#define PROF_SCOPE(b) ProfScope _pscope((LDSP unsigned long long*)prof, b, lane)
#else
#define PROF_SCOPE(b)
#define PROF_IN(v)
#define PROF_OUT(b, v)
#define PROF_T(v)
#define PROF_ADD(b, v)
#define PROF_CNT(b)
#endif
// diagnostics build (-DMXA_RP_CHECK): the replay book's computed indices are range-checked before
// the global access they address; a bad one prints and ends the env with ERR_BAD_CONFIG
// instead of faulting the device
#ifdef MXA_RP_CHECK
#define RPCHK(c, what, v)                                                                     \
  do {                                                                                        \
    if (!(c)) {                                                                               \
      if (lane == 0) printf("RPCHK %s = %lld at pop %lld\n", what, (long long)(v), (long long)pops); \
      fail(ERR_BAD_CONFIG);                                                                   \
      return;                                                                                 \
    }                                                                                         \
  } while (0)
#else
#define RPCHK(c, what, v)
#endif
template <int CFG, bool BUILD = false, bool LOG = false, bool INSTR = true>
struct Eng {
  // every configuration constant is an immediate (mxa_config.h)
  static constexpr MxaParams PC = mxa_cfg::params(CFG);
  static constexpr int SQ = mxa_cfg::shape(CFG).sq;
  static constexpr int SO = mxa_cfg::shape(CFG).so;
  static constexpr bool PL_LDS = mxa_cfg::shape(CFG).pl;
  static constexpr int PW = mxa_cfg::shape(CFG).pw;           // payload words queued
  // (event loop: record beside the HBM payload).  Not on the two-tier queue configurations:
  // there it measured neutral (393.1 vs 393.7 ms) and loads the records of the acknowledgements
  // that take a fast path, +46 B/event of HBM traffic
  static constexpr bool EARLY_REC = !BUILD && !PL_LDS && !(mxa_cfg::sq_lds(CFG) < mxa_cfg::shape(CFG).sq);
  // grouped lane-min cache for deep queues (sparse_zi_1000: 48 slots per lane): a lane's slots
  // in groups of QG, each group's min (key, seq, slot) kept in VGPRs, so a remove or requeue
  // rescans one group of QG slots instead of all SQ
#ifndef MXA_TIER_NEAR_NS
#define MXA_TIER_NEAR_NS 1000000000LL  // two-tier queue: events due within this many ns take LDS slots
#endif
#ifndef MXA_QG
#define MXA_QG 12  // group size at SQ >= 16 (measured, sparse_zi_1000: 4 -> 1194 ms, 6/8 -> 973, 12 -> 958)
#endif
#ifndef MXA_QHIER_MIN
// grouped minima from 9 slots per lane; 8 slots and fewer take the flat select tree (same per-env
// results: r03 s29 value_noise 20.7 -> 18.9 ms, rmsc02 1087 -> 1003 ms against two groups of 3;
// s31 sparse_zi_100 120.1 -> 116.8 ms against two groups of 4)
#define MXA_QHIER_MIN 9
#endif
  static constexpr int QG = SQ >= 16 ? MXA_QG : SQ / 2;
  static constexpr bool TIER_CFG = mxa_cfg::sq_lds(CFG) < SQ;  // (TIER below)
  static constexpr bool QHIER = SQ >= MXA_QHIER_MIN && SQ > QG;
  // a group size that does not tile the deep queues is a build error, never a silent fall-back
  // to the flat scan (a -DMXA_QG sweep must measure what it names)
  static_assert(!QHIER || SQ % QG == 0, "queue groups must tile the lane's slots (MXA_QG)");
  // the two-tier queue keeps the LDS tier's groups and ONE entry for the lane's whole HBM tier
  // (its SQH far slots): a push there is a select on that entry, and only a pop or rekey of an
  // HBM-tier slot rescans it, in the owner lane alone (a twelfth of the pops in
  // random_fund_value).  One VGPR entry instead of six per-group entries, which the run kernel
  // spilled on every push (880 scratch instructions at q_gupd, r04 isa_lines)
  static constexpr int NG = QHIER ? (TIER_CFG ? mxa_cfg::sq_lds(CFG) / QG + 1 : SQ / QG) : 1;
  // group rescans as one batch of loads and a select tree (q_scan): groups of 4 and more slots.
  // r03 s20, same per-env results: sparse_zi_1000 916 -> 826 ms, random_fund_value 778 -> 575,
  // sparse_zi_100 132.5 -> 125.7, value_noise 22.0 -> 21.2; rmsc02 (groups of 3) 1053 -> 1086, so
  // it keeps the serial scan
  static constexpr bool QTREE = QHIER && QG >= 4;
  static constexpr int HOT = BUILD ? 0 : mxa_cfg::shape(CFG).hot;  // LDS-resident agent records
  // the replay book + tape (ABIDESEnv's composition, or config/marketreplay.py under Kernel.runner)
  static constexpr bool RP = CFG == MXA_CFG_MARKETREPLAY || CFG == MXA_CFG_MARKETREPLAY_RUNNER ||
                             CFG == MXA_CFG_MARKETREPLAY_TWAP;
  static constexpr bool GYM = CFG == MXA_CFG_MARKETREPLAY || CFG == MXA_CFG_RMSC03_RL;  // a GymKernel with a DummyRL agent
  // ORDER_ACCEPTED to a background TradingAgent is a no-op (TradingAgent.orderAccepted only
  // logs, TradingAgent.py:409-420; no ZI/Noise/Value/POV-MM/Momentum branch reacts to it, and the
  // POV-MM's both-replies-in test cannot fire on it). With every computation delay 0 the busy
  // check cannot requeue it, so its whole effect is Kernel.agentCurrentTimes[a] = t: one 8-byte
  // store, no record round trip (rmsc03: a quarter of all pops).
  static constexpr bool ACK_FAST = !BUILD && !RP && PC.default_comp_delay == 0 && PC.ex_comp == 0 &&
                                   PC.n_obi == 0;  // OrderBookImbalanceAgent sets a 1 ns delay at runtime
  // ABIDESEnv replay: the exchange and ORDER_ACCEPTED shortcuts hold as well (MarketReplayAgent
  // ignores ORDER_ACCEPTED too, every delay is 0); ORDER_CANCELLED updates its orders table, so
  // the CANCELLED shortcut (open-order list) stays off
  static constexpr bool RP_FAST = !BUILD && RP && PC.default_comp_delay == 0 && PC.ex_comp == 0;
  static constexpr int ACK_LIMIT = GYM ? PC.first_rl : PC.n_agents;  // background agents 1..ACK_LIMIT-1
  typedef RSt<BUILD> RS;
  typedef typename std::conditional<PL_LDS, LDSP u32*, u32*>::type PlPtr;
  static constexpr int QCAP = SQ * 64;
  // event key t << KSH | recipient << 2 | type (13 recipient bits: random_fund_value's 5,101 agents)
  static constexpr int KSH = MXA_KEY_SHIFT;
  static constexpr u64 KRCP = MXA_KEY_RCP;
  static_assert(PC.n_agents <= (int)KRCP, "recipient field of the event key");
  // two-tier queue (random_fund_value): slots j < SQL of every lane in LDS, the rest in HBM; an
  // event is placed by its due time (far wakeups in the HBM tier), which the pop never sees
  static constexpr int SQL = mxa_cfg::sq_lds(CFG);
  static constexpr bool TIER = SQL < SQ;
  static constexpr int QCL = SQL * 64;
  static_assert(!TIER || (!PL_LDS && SQL % 12 == 0 && SQ >= 16), "HBM queue tier: payloads in HBM, whole groups per tier");
  // the env block.  The two-tier queue configuration spells out the global address space (its
  // generic env-derived pointers otherwise became flat accesses); the others keep the generic
  // pointer their measured code generation was tuned with (rmsc01 1116 -> 1250 ms with it)
  typedef typename std::conditional<TIER, GLBP char*, char*>::type EnvPtr;
  EnvPtr env;
  int lane;
  LDSP EnvHdr& h;  // cold header fields live in LDS for the duration of a launch
  // hot header fields in SGPRs
  i64 cur, pops, ocnt;
  i64 stop_t;  // Kernel.runner's stopTime: the config's unless the header overrides it (EnvHdr::t_stop)
  u64 hash;
  u32 seq;
  i32 status, err, qcount;
  // event queue: keys in LDS, payload in LDS (PL_LDS) or HBM; per-lane min cache
  LDSP u64* qk;
  LDSP u32* qs;
  // HBM tier (TIER): keys and sequence numbers of slots QCL .. QCAP - 1.  Global address space
  // spelled out: a generic pointer next to the LDS arrays let the optimizer merge the two tiers
  // into flat accesses (273 flat loads, 1,949 scratch reloads, 2x slower)
  // Lane-major: a lane's SQH tier slots are contiguous, so the owner lane's group rescan reads
  // 96 + 48 contiguous bytes instead of the 64-lane block of the group (r03: 29.5x the counted
  // bytes were these rescans)
  static constexpr size_t OFF_HQ = PC.L.off_q + sizeof(SavedEvent) * QCAP + (PL_LDS ? 0 : (size_t)QCAP * 4 * PW);
  static constexpr int SQH = SQ - SQL;
  static DEV int hidx(int slot) { return (slot & 63) * SQH + ((slot >> 6) - SQL); }
  DEV GLBP u64* hqk() { return (GLBP u64*)(env + OFF_HQ); }
  DEV GLBP u32* hqs() { return (GLBP u32*)(env + OFF_HQ + (size_t)(QCAP - QCL) * 8); }
  DEV u64 qk_get(int slot) {
    if constexpr (TIER) {
      if (slot >= QCL) return hqk()[hidx(slot)];
    }
    return qk[slot];
  }
  DEV u32 qs_get(int slot) {
    if constexpr (TIER) {
      if (slot >= QCL) return hqs()[hidx(slot)];
    }
    return qs[slot];
  }
  DEV void qk_put(int slot, u64 v) {
    if constexpr (TIER) {
      if (slot >= QCL) {
        hqk()[hidx(slot)] = v;
        return;
      }
    }
    qk[slot] = v;
  }
  DEV void qs_put(int slot, u32 v) {
    if constexpr (TIER) {
      if (slot >= QCL) {
        hqs()[hidx(slot)] = v;
        return;
      }
    }
    qs[slot] = v;
  }
  // this lane's slot j (every use of the key/seq arrays is the owning lane's own slot)
  DEV u64 qkey(int j) {
    if constexpr (TIER) return qk_get(j * 64 + lane);
    else return qk[j * 64 + lane];
  }
  DEV u32 qseq(int j) {
    if constexpr (TIER) return qs_get(j * 64 + lane);
    else return qs[j * 64 + lane];
  }
  DEV void qset(int j, u64 k, u32 s, bool me) {
    if (me) {
      if constexpr (TIER) {
        qk_put(j * 64 + lane, k);
        qs_put(j * 64 + lane, s);
      } else {
        qk[j * 64 + lane] = k;
        qs[j * 64 + lane] = s;
      }
    }
  }
  DEV void qsetk(int j, u64 k, bool me) {
    if (me) {
      if constexpr (TIER) qk_put(j * 64 + lane, k);
      else qk[j * 64 + lane] = k;
    }
  }
  PlPtr qpl;
  u64 mk;
  u32 ms;
  i32 mj;
  u64 gk[NG];  // QHIER: per-group min of this lane's slots
  u32 gs[NG];
  i32 gj[NG];
  // free-slot mask of this lane, bit j = slot j (128 bits above 64 slots per lane: the wide
  // random_fund_value queue)
  static_assert(SQ <= 128, "at most 128 queue slots per lane");
  typedef typename std::conditional<(SQ > 64), unsigned __int128, u64>::type QM;
  static DEV QM qm_bit(int j) { return (QM)1 << j; }
  static DEV int qm_ffs(QM m) {
    if constexpr (SQ > 64) {
      const u64 lo = (u64)m;
      return lo ? ffs64(lo) : 64 + ffs64((u64)(m >> 64));
    } else {
      return ffs64(m);
    }
  }
  static DEV int qm_ctz(QM m) {  // m != 0
    if constexpr (SQ > 64) {
      const u64 lo = (u64)m;
      return lo ? ctz64(lo) : 64 + ctz64((u64)(m >> 64));
    } else {
      return ctz64(m);
    }
  }
  static DEV int qm_pop(QM m) {
    if constexpr (SQ > 64) return __popcll((u64)m) + __popcll((u64)(m >> 64));
    else return __popcll(m);
  }
  static DEV QM qm_rdl(QM m, int L) {
    if constexpr (SQ > 64) return (QM)rdl64((u64)m, L) | ((QM)rdl64((u64)(m >> 64), L) << 64);
    else return rdl64(m, L);
  }
  QM qfree;
  // order book pool in VGPRs: slot (j, lane).  An array whose bit is set in BKL lives in LDS for
  // a launch instead (mxa_cfg::book_lds; the builder keeps VGPR arrays and writes the env block),
  // at [j][64], read and written through BkL with the same bp[j] syntax
  template <class T>
  struct BkL {
    LDSP T* p;  // this lane's element of slot row 0
    DEV LDSP T& operator[](int j) const { return p[j * 64]; }
  };
  static constexpr int BKL = BUILD ? 0 : mxa_cfg::book_lds(CFG);
  template <int BIT, class T>
  using BkT = typename std::conditional<((BKL >> BIT) & 1) != 0, BkL<T>, T[SO]>::type;
  BkT<0, i32> bp;
  BkT<1, i32> bq;
  BkT<2, i32> bo;
  BkT<3, i32> bm;
  BkT<4, u32> ba;
  BkT<5, i32> bh;
  template <int BIT, class A>
  DEV void bk_bind(A& a, LDSP char* base) {
    if constexpr (((BKL >> BIT) & 1) != 0)
      a.p = (decltype(a.p))(base + (size_t)__builtin_popcount(BKL & ((1 << BIT) - 1)) * SO * 256) + lane;
  }
  // HBL configurations: OrderBook.history restated as an order-history ring in HBM (one OhRec
  // per handled limit order); a resting order keeps its record index to flag its transactions
  static constexpr bool OH = PC.n_hbl > 0;
  static constexpr bool TW = PC.n_twap > 0;  // a TWAPExecutionAgent (execution_marketreplay.py)
  // market-data subscription configs (rmsc02): the exchange publishes after book changes
  static constexpr bool MD = PC.md_sub != 0;
  static_assert(!MD || PW == 8, "MARKET_DATA carries its level counts and slot tag in w6 / w7");
  i32 bx[OH ? SO : 1];
  // current agent record (lane l holds dwords 2l, 2l+1)
  u32 rlo, rhi;
  u32 rdirty;  // record quarters changed since rec_load (bit q: dwords 32q .. 32q + 31)
  i32 cur_agent;
  i64 add_delay;
  u32 dirty;  // RNG streams touched by this event: bits 0-3 G/O/K/L, bit 4 the agent's own
  i64* trace;
  i32 trace_cap;
  bool hash_on;  // per-pop parity hash (kernel argument trace_cap < 0: off, and no trace ring)
  // marketreplay / hist_fund: tape + runtime layout (nullptr otherwise).  Read through the
  // constant address space: the context never changes during a launch, so its fields (the
  // layout offsets every replay handler starts from) come from scalar loads, not from a vector
  // load round trip at the head of each handler's chain
  const __attribute__((address_space(4))) RpCtx* rx;
  i32 end_step;     // GymKernel: the RL agent's spread reply ends a step
  u32 run_skip;     // event runs: members below this seq are popped one by one (a LIMIT run that crosses)
  // book-update log of this env: a kernel variant of its own (LOG), so the event loop of the
  // plain kernels carries none of it
  static constexpr bool BLOG = LOG;
  BlRec* blog;
  i32 blog_cap;
#ifdef MXA_PROF
  LDSP u64* prof;
#endif
  LDSP u64* hotrec;  // [HOT][64]: the exchange's (and the market maker's or replay agent's) agent record
  // the exchange's latency row in LDS for the launch (MXA_LAT_LDS_MASK): every send reads one
  // entry, which from HBM is a dependent memory round trip on the event chain
  static constexpr int LATL = BUILD ? 0 : mxa_cfg::lat_lds(CFG);
  LDSP double* latl;
  // the replay / gym header (RpHdr) for a launch of the run / step kernel (RPH): every replay
  // handler reads and updates it on its dependent chain.  load() copies it in and save() out;
  // the builder (BUILD) writes the env block's copy directly and never touches this one
  static constexpr bool RPH = !BUILD && mxa_cfg::rp_hdr_lds(CFG);
  LDSP RpHdr* rhl;
  LDSP i32* scr;     // [64] rank -> queue slot, then [64] u64 staged keys (MXA_QREG)
  LDSP u32* rwin;    // [4][64] output windows of the global RNG streams (RSt::lw)

  static constexpr size_t LDS_Q = (size_t)QCL * (12 + (PL_LDS ? 4 * PW : 0));
  DEV Eng(char* e, char* lds, i32 tcap, const RpCtx* ctx = nullptr, BlRec* bl = nullptr, i32 bl_cap = 0)
      : env((EnvPtr)e), h(*(LDSP EnvHdr*)(lds + LDS_Q)) {
    rx = (const __attribute__((address_space(4))) RpCtx*)ctx;
    blog = bl;
    blog_cap = bl_cap;
    end_step = 0;
    add_delay = 0;
    run_skip = 0;
    rdirty = 0;
    lane = laneid();
    qk = (LDSP u64*)lds;
    qs = (LDSP u32*)(lds + 8 * QCL);
    if constexpr (PL_LDS) qpl = (LDSP u32*)(lds + 12 * QCL);
    else qpl = (u32*)(env + PC.L.off_q + sizeof(SavedEvent) * QCAP);  // [QCAP][PW] after the saved queue
    dirty = 0;
    hash_on = tcap >= 0;
    trace_cap = tcap > 0 ? tcap : 0;
#ifdef MXA_PROF
    prof = (LDSP u64*)(lds + LDS_Q + sizeof(EnvHdr));
    prof[lane] = 0;
    prof[64 + lane] = 0;
#endif
    trace = tcap > 0 ? (i64*)(env + PC.L.off_trace) : nullptr;
    scr = (LDSP i32*)(lds + mxa_cfg::lds_bytes(CFG) - 256);
    rwin = (LDSP u32*)((LDSP char*)scr - 1024);
#ifdef MXA_PROF
    hotrec = (LDSP u64*)(lds + LDS_Q + 512 + 1024);
#else
    hotrec = (LDSP u64*)(lds + LDS_Q + 512);
#endif
    latl = (LDSP double*)(hotrec + mxa_cfg::shape(CFG).hot * 64);
    rhl = (LDSP RpHdr*)(latl + mxa_cfg::lat_lds(CFG));
    if constexpr (BKL != 0) {
      LDSP char* bk = (LDSP char*)rhl + (mxa_cfg::rp_hdr_lds(CFG) ? 256 : 0);
      bk_bind<0>(bp, bk);
      bk_bind<1>(bq, bk);
      bk_bind<2>(bo, bk);
      bk_bind<3>(bm, bk);
      bk_bind<4>(ba, bk);
      bk_bind<5>(bh, bk);
    }
  }

  // ---------------- env block accessors
  DEV EnvHdr* hdr() { return (EnvHdr*)env; }
  DEV u64* agent_ptr(int a) { return (u64*)(env + PC.L.off_ag + (size_t)a * 512); }
  DEV OpenOrder* open_ptr(int a) { return (OpenOrder*)(env + PC.L.off_open + (size_t)a * PC.L.open_cap * sizeof(OpenOrder)); }
  DEV u32* rng_key(int s) { return (u32*)(env + PC.L.off_rng + (size_t)s * MXA_RNG_WORDS * 4); }
  DEV double* lat() { return (double*)(env + PC.L.off_lat); }
  DEV SubRec* subs() { return (SubRec*)(env + PC.L.off_sub); }
  DEV u32* md_slot(int agent) { return (u32*)(env + PC.L.off_md) + (size_t)agent * MD_WORDS; }
  DEV LDSP i32* ep_entries() { return h.ep_n; }  // header field: LDS for the launch
  DEV TxRec* txr() { return (TxRec*)(env + PC.L.off_tx + 64); }

  DEV void fail(int code) {
    if (status != ST_ERROR) {
      status = ST_ERROR;
      err = code;
    }
  }

  // ---------------- agent record
  // the exchange and the market maker take ~95 % of rmsc03's events: their records live in
  // LDS for the launch (load()/save() move them), every other agent's comes from HBM
  // second hot record: the market maker (rmsc03) or the MarketReplayAgent (the replay configs,
  // whose every other event is its wakeup or an execution report)
  static constexpr int HOT1 = PC.n_mm > 0 ? PC.first_mm : PC.n_replay > 0 ? PC.first_replay : -1;
  DEV int hot_slot(int a) {
    if (HOT > 0 && a == 0) return 0;
    if (HOT > 1 && HOT1 >= 0 && a == HOT1) return 1;
    return -1;
  }
  DEV u64 rec_fetch(int a) {
    const int hs = hot_slot(a);
    if (hs >= 0) return hotrec[hs * 64 + lane];
    return agent_ptr(a)[lane];
  }
  DEV void rec_load(int a) { rec_set(a, rec_fetch(a)); }
  DEV void rec_set(int a, u64 v) {
    PROF_SCOPE(77);
    rlo = (u32)v;
    rhi = (u32)(v >> 32);
    cur_agent = a;
    rdirty = 0;
    if constexpr (INSTR && !BUILD) {
      if ((hash_on || trace) && lane == 0) h.kc[MXA_KC_REC]++;  // class counters (mxa_read_counters)
    }
  }
  // write-back of the record: with DIRTY_WB only its 128-byte quarters (whole L2 lines, 16
  // lanes each) that an rs* call changed since rec_load (the builder writes whole records)
  static constexpr bool DIRTY_WB = ((MXA_DIRTY_WB_MASK) >> CFG) & 1;
  DEV void rec_store() {
    const u64 v = ((u64)rhi << 32) | rlo;
    const int hs = hot_slot(cur_agent);
    if (hs >= 0) hotrec[hs * 64 + lane] = v;
    else if (BUILD || !DIRTY_WB || ((rdirty >> (lane >> 4)) & 1)) agent_ptr(cur_agent)[lane] = v;
  }
  // Kernel.agentCurrentTimes[a] = t without loading the record (AF_ATIME: lane AF_ATIME/2's u64)
  DEV void atime_store(int a, i64 t) {
    const int hs = hot_slot(a);
    if (lane == AF_ATIME / 2) {
      if (hs >= 0) hotrec[hs * 64 + lane] = (u64)t;
      else agent_ptr(a)[lane] = (u64)t;
    }
  }
  DEV int hot_agent(int hs) { return hs == 0 ? 0 : HOT1; }
  DEV u32 rg(int f) { return (f & 1) ? rdl(rhi, f >> 1) : rdl(rlo, f >> 1); }
  DEV i32 rgi(int f) { return (i32)rg(f); }
  DEV i64 rg64(int f) { return (i64)(((u64)rdl(rhi, f >> 1) << 32) | rdl(rlo, f >> 1)); }
  DEV double rgd(int f) { return as_d((u64)rg64(f)); }
  // record writes are lane selects (v_cndmask), not divergent branches
  DEV void rs(int f, u32 v) {
    rdirty |= 1u << (f >> 5);  // the record quarter (dwords 32q .. 32q + 31) of field f
    bool me = lane == (f >> 1);
    if (f & 1) rhi = me ? v : rhi;
    else rlo = me ? v : rlo;
  }
  DEV void rs64(int f, i64 v) {
    rdirty |= 1u << (f >> 5);
    bool me = lane == (f >> 1);
    rlo = me ? (u32)(u64)v : rlo;
    rhi = me ? (u32)((u64)v >> 32) : rhi;
  }
  DEV void rsd(int f, double v) { rs64(f, (i64)as_u(v)); }
  DEV u32 flags() { return rg(AF_FLAGS); }
  DEV bool fl(u32 bit) { return (flags() & bit) != 0; }
  DEV void fl_set(u32 bit, bool on) {
    u32 f = flags();
    rs(AF_FLAGS, on ? (f | bit) : (f & ~bit));
  }

  // agent RNG stream (Agent.random_state): key words in HBM, pos/gauss cache in the record
  DEV RS agent_rs() {
    RS r;
    r.lw = BUILD && MXA_BUILD_WINDOWS ? rwin + 3 * 64 : nullptr;
    r.lw0 = r.lwn = 0;
    r.key = rng_key(4 + cur_agent);
    r.p = rgi(AF_RS_POS);
    r.m = rgi(AF_RS_M);
    r.hasg = rgi(AF_RS_HASG);
    r.gauss = rgd(AF_RS_GAUSS);
    return r;
  }
  DEV void agent_rs_put(const RS& r) {
    rs(AF_RS_POS, (u32)r.p);
    rs(AF_RS_M, (u32)r.m);
    rs(AF_RS_HASG, (u32)r.hasg);
    rsd(AF_RS_GAUSS, r.gauss);
    dirty |= rs_needs_maint(r, MXA_AGENT_LA) ? 16u : 0u;
  }
  // whether rng_maint has work for a stream in this state: a look-ahead overrun to report, or
  // no materialized block after the one holding position p.  Decided where the state is put
  // (registers) instead of re-read from the header and the record at the event's end
  DEV bool rs_needs_maint(const RS& r, int la = MXA_MT_N) {
    if constexpr (BUILD) return true;
    return (r.hasg & 2) || r.m < (r.p + la) / MXA_MT_N;
  }
  // global streams: 0 = G (np.random), 1 = O (oracle symbol), 2 = K (kernel), 3 = L (latency)
  DEV RS grs(int s) {
    RS r;
    r.key = rng_key(s);
    r.p = h.rs_pos[s];
    r.m = h.rs_m[s];
    r.hasg = h.rs_has_gauss[s];
    r.gauss = h.rs_gauss[s];
    if constexpr (BUILD) {  // an empty window: the first draw fills it
      r.lw = MXA_BUILD_WINDOWS ? rwin + s * 64 : nullptr;
      r.lw0 = r.lwn = 0;
    } else {
      r.lw = rwin + s * 64;
      r.lw0 = h.rs_w0[s];
      r.lwn = h.rs_wn[s];
    }
    return r;
  }
  // the kernel stream K (Kernel.random_state: latency noise, one draw per send) in registers for
  // the launch instead of the LDS header (MXA_KREG_MASK): loaded and saved with the header, the
  // window itself stays in LDS
#ifndef MXA_KREG_MASK
// same per-env results: r03 s38 rmsc02 1002 -> 927 ms, obi_rmsc02 356 -> 346, value_noise 19.2 -> 18.5,
// sparse_zi_1000 736 -> 731; s40 (the L stream of the cubic latency model) sparse_zi_100 116.8 -> 114.6
#define MXA_KREG_MASK ((1 << MXA_CFG_SPARSE_ZI_1000) | (1 << MXA_CFG_VALUE_NOISE) | (1 << MXA_CFG_RMSC02) | \
                       (1 << MXA_CFG_OBI_RMSC02) | (1 << MXA_CFG_SPARSE_ZI_100))
#endif
  // the stream a send draws from: L (latency model, lat_mode 2) or K (the noise of lat_mode 0/1)
  static constexpr int KS = PC.lat_mode == 2 ? 3 : 2;
  static constexpr bool KREG = !BUILD && (((MXA_KREG_MASK) >> CFG) & 1) && (PC.lat_mode == 2 || PC.noise_len > 1);
  i32 kp, km, khg, kw0, kwn;
  DEV RS grs_k() {
    RS r;
    r.key = rng_key(KS);
    r.p = kp;
    r.m = km;
    r.hasg = khg;
    r.gauss = 0.0;  // randint / uniform never read or write it; the header keeps the cached gauss
    r.lw = rwin + KS * 64;
    r.lw0 = kw0;
    r.lwn = kwn;
    return r;
  }
  DEV void grs_put_k(const RS& r) {
    kp = r.p;
    km = r.m;
    khg = r.hasg;
    kw0 = r.lw0;
    kwn = r.lwn;
    dirty |= rs_needs_maint(r) ? 1u << KS : 0u;
  }
  DEV void grs_put(int s, const RS& r) {
    h.rs_pos[s] = r.p;
    h.rs_m[s] = r.m;
    h.rs_has_gauss[s] = r.hasg;
    h.rs_gauss[s] = r.gauss;
    if constexpr (!BUILD) {
      h.rs_w0[s] = r.lw0;
      h.rs_wn[s] = r.lwn;
    }
    dirty |= rs_needs_maint(r) ? 1u << s : 0u;
  }
  // event boundary: keep one MT block of look-ahead for every stream this event drew from
  DEV void rng_maint() {
    PROF_SCOPE(78);
#pragma unroll 1
    for (int k = 0; k < 5; k++) {
      if (!((dirty >> k) & 1)) continue;
      const bool kr = KREG && k == KS;
      const i32 p = kr ? kp : k < 4 ? h.rs_pos[k] : rgi(AF_RS_POS), m = kr ? km : k < 4 ? h.rs_m[k] : rgi(AF_RS_M);
      const i32 hg = kr ? khg : k < 4 ? h.rs_has_gauss[k] : rgi(AF_RS_HASG);
      if (hg & 2) fail(ERR_RNG_OVERRUN);
      const int la = k < 4 ? MXA_MT_N : MXA_AGENT_LA;
      if (m >= (p + la) / MXA_MT_N) continue;  // the look-ahead is there (almost always)
      RS r = kr ? grs_k() : k < 4 ? grs(k) : agent_rs();
      rs_maint(r, la);
      if (kr) {
        km = r.m;
      } else if (k < 4) {
        h.rs_m[k] = r.m;
      } else {
        rs(AF_RS_M, (u32)r.m);
      }
    }
    dirty = 0;
  }

  // ---------------- event queue
  // (k, s, j) = lexicographic min of itself and (k2, s2, j2): lane selects, no branch
  static DEV void q_min2(u64& k, u32& s, i32& j, u64 k2, u32 s2, i32 j2) {
    const bool lt = (k2 < k) | ((k2 == k) & (s2 < s));
    k = lt ? k2 : k;
    s = lt ? s2 : s;
    j = lt ? j2 : j;
  }
  // min (key, seq, slot) over this lane's slots [j0, j0 + n)
  DEV void q_scan(int j0, int n, u64& bk, u32& bs, i32& bj) {
    if constexpr (QTREE) {
      // every load of the group first, then a pairwise tree of selects: one memory latency per
      // rescan instead of QG dependent load -> compare -> branch steps (the serial scan was
      // 21 % of sparse_zi_1000's cycles, r03 s8).  Ties (only empty slots) keep the lower slot,
      // as the serial scan does; an all-empty group still reports j = -1.
      u64 k[QG];
      u32 s[QG];
      i32 j[QG];
      if (TIER && j0 >= SQL) {
        constexpr int ST = 1;  // word stride between a lane's consecutive slots (lane-major)
        const int b0 = lane * SQH + (j0 - SQL);
        const GLBP u64* K = hqk() + b0;
        const GLBP u32* S = hqs() + b0;
#pragma unroll
        for (int i = 0; i < QG; i++) {
          k[i] = K[i * ST];
          s[i] = S[i * ST];
        }
      } else {
#pragma unroll
        for (int i = 0; i < QG; i++) {
          k[i] = qk[(j0 + i) * 64 + lane];
          s[i] = qs[(j0 + i) * 64 + lane];
        }
      }
#pragma unroll
      for (int i = 0; i < QG; i++) j[i] = j0 + i;
#pragma unroll
      for (int w = 1; w < QG; w *= 2) {
#pragma unroll
        for (int i = 0; i + w < QG; i += 2 * w) q_min2(k[i], s[i], j[i], k[i + w], s[i + w], j[i + w]);
      }
      bk = k[0];
      bs = s[0];
      bj = (k[0] == KEY_EMPTY && s[0] == 0xFFFFFFFFu) ? -1 : j[0];
      return;
    }
    bk = KEY_EMPTY;
    bs = 0xFFFFFFFFu;
    bj = -1;
    if constexpr (TIER) {
      if (j0 >= SQL) {  // a whole group of the HBM tier (groups never straddle the tiers)
        constexpr int ST = 1;
        const int b0 = lane * SQH + (j0 - SQL);
        const GLBP u64* K = hqk() + b0;
        const GLBP u32* S = hqs() + b0;
        for (int j = 0; j < n; j++) {
          const u64 k = K[j * ST];
          const u32 s = S[j * ST];
          if (k < bk || (k == bk && s < bs)) {
            bk = k;
            bs = s;
            bj = j0 + j;
          }
        }
        return;
      }
    }
    for (int j = j0; j < j0 + n; j++) {
      int slot = j * 64 + lane;
      u64 k = qk[slot];
      u32 s = qs[slot];
      if (k < bk || (k == bk && s < bs)) {
        bk = k;
        bs = s;
        bj = j;
      }
    }
  }
  DEV void q_lanemin() {  // QHIER: lane min from the group mins
    u64 bk = gk[0];
    u32 bs = gs[0];
    i32 bj = gj[0];
    if constexpr (QTREE) {
#pragma unroll
      for (int g = 1; g < NG; g++) q_min2(bk, bs, bj, gk[g], gs[g], gj[g]);
    } else {
      for (int g = 1; g < NG; g++) {
        if (gk[g] < bk || (gk[g] == bk && gs[g] < bs)) {
          bk = gk[g];
          bs = gs[g];
          bj = gj[g];
        }
      }
    }
    mk = bk;
    ms = bs;
    mj = bj;
  }
  // min (key, seq, slot) over this lane's HBM-tier slots, QG at a time
  DEV void q_scan_hbm(u64& bk, u32& bs, i32& bj) {
    q_scan(SQL, QG, bk, bs, bj);
#pragma unroll 1
    for (int j0 = SQL + QG; j0 < SQ; j0 += QG) {
      u64 k;
      u32 s;
      i32 j;
      q_scan(j0, QG, k, s, j);
      q_min2(bk, bs, bj, k, s, j);
    }
    if (bk == KEY_EMPTY && bs == 0xFFFFFFFFu) bj = -1;
  }
  // a pop or rekey in the HBM tier: the owner lane's SQH far slots in ONE round trip,
  // spread over the wave (lane i holds slots SQL + i and SQL + 64 + i), then a wave-wide
  // lexicographic min (as q_peek).  Results are wave-uniform.  The owner-lane scan took SQH / QG
  // dependent round trips (34 % of random_fund_value's cycles in q_remove, r04 s12)
  DEV void q_scan_hbm_wave(int owner, u64& bk, u32& bs, i32& bj) {
    static_assert(SQH <= 128, "two far slots per lane");
    u64 k0 = KEY_EMPTY, k1 = KEY_EMPTY;
    u32 s0 = 0xFFFFFFFFu, s1 = 0xFFFFFFFFu;
    i32 j0 = SQL + lane, j1 = SQL + 64 + lane;
    if (lane < SQH) {
      const int h = hidx(j0 * 64 + owner);
      k0 = hqk()[h];
      s0 = hqs()[h];
    }
    if (64 + lane < SQH) {
      const int h = hidx(j1 * 64 + owner);
      k1 = hqk()[h];
      s1 = hqs()[h];
    }
    q_min2(k0, s0, j0, k1, s1, j1);
    const u32 kh = (u32)(k0 >> 32), kl = (u32)k0;
    const u32 m1 = wmin_u32(kh);
    u64 b = bal(kh == m1);
    if (__popcll(b) > 1) {
      const u32 m2 = wmin_u32(kh == m1 ? kl : 0xFFFFFFFFu);
      b = bal(kh == m1 && kl == m2);
      if (__popcll(b) > 1) {
        const u32 m3 = wmin_u32((kh == m1 && kl == m2) ? s0 : 0xFFFFFFFFu);
        b = bal(kh == m1 && kl == m2 && s0 == m3);
      }
    }
    const int L = ffs64(b);
    bk = ((u64)m1 << 32) | rdl(kl, L);
    bs = rdl(s0, L);
    bj = (bk == KEY_EMPTY && bs == 0xFFFFFFFFu) ? -1 : rdli(j0, L);
  }
  // QHIER: the slot's group changed.  An LDS-tier group is rescanned in every lane (the group
  // index is wave-uniform; lanes whose group did not change recompute the same values), then the
  // lane mins.  An HBM-tier slot: its owner lane alone rescans the whole tier (one aggregate
  // entry), the other lanes' entries are unchanged and their rescans were HBM traffic
  DEV void q_regroup(int slot) {
    const int g = (slot >> 6) / QG, owner = slot & 63;
    if constexpr (TIER) {
      if ((slot >> 6) >= SQL) {
        u64 k;
        u32 s;
        i32 j;
        q_scan_hbm_wave(owner, k, s, j);
        if (lane == owner) {
          gk[NG - 1] = k;
          gs[NG - 1] = s;
          gj[NG - 1] = j;
          q_lanemin();
        }
        return;
      }
    }
    u64 k;
    u32 s;
    i32 j;
    q_scan(g * QG, QG, k, s, j);
#pragma unroll
    for (int gg = 0; gg < NG; gg++) {
      if (gg == g) {
        gk[gg] = k;
        gs[gg] = s;
        gj[gg] = j;
      }
    }
    q_lanemin();
  }
  DEV void q_gupd(int j, u64 k, u32 s, bool me = true) {  // QHIER: slot j of this lane (me) now holds (k, s)
    const int g = (TIER && j >= SQL) ? NG - 1 : j / QG;
    if constexpr (QTREE) {
#pragma unroll
      for (int gg = 0; gg < NG; gg++) {  // selects: g differs between lanes
        const bool w = me & (gg == g) & ((k < gk[gg]) | ((k == gk[gg]) & (s < gs[gg])));
        gk[gg] = w ? k : gk[gg];
        gs[gg] = w ? s : gs[gg];
        gj[gg] = w ? j : gj[gg];
      }
    } else {
      for (int gg = 0; gg < NG; gg++) {
        if (me && gg == g && (k < gk[gg] || (k == gk[gg] && s < gs[gg]))) {
          gk[gg] = k;
          gs[gg] = s;
          gj[gg] = j;
        }
      }
    }
  }
  DEV void q_rescan() {  // recompute this lane's min over its own slots
    if constexpr (QHIER) {
      if constexpr (TIER) {  // unrolled: a rolled loop indexes gk/gs/gj dynamically (scratch)
#pragma unroll
        for (int g = 0; g < NG - 1; g++) q_scan(g * QG, QG, gk[g], gs[g], gj[g]);
        q_scan_hbm(gk[NG - 1], gs[NG - 1], gj[NG - 1]);
      } else {  // (unrolled here too: the same time for sparse_zi_1000, +0.5-2 % for sparse_zi_100 and value_noise, r03 s9)
        for (int g = 0; g < NG; g++) q_scan(g * QG, QG, gk[g], gs[g], gj[g]);
      }
      q_lanemin();
      return;
    }
    // every slot's load first, then a select tree (as q_scan).  r03 s24, same per-env results:
    // rmsc03 43.8 -> 41.4 ms, rmsc01 1073 -> 963, obi_rmsc02 386 -> 373
    if constexpr (!TIER) {
      u64 k[SQ];
      u32 s[SQ];
      i32 j[SQ];
#pragma unroll
      for (int i = 0; i < SQ; i++) {
        k[i] = qk[i * 64 + lane];
        s[i] = qs[i * 64 + lane];
        j[i] = i;
      }
#pragma unroll
      for (int w = 1; w < SQ; w *= 2) {
#pragma unroll
        for (int i = 0; i + w < SQ; i += 2 * w) q_min2(k[i], s[i], j[i], k[i + w], s[i + w], j[i + w]);
      }
      mk = k[0];
      ms = s[0];
      mj = (k[0] == KEY_EMPTY && s[0] == 0xFFFFFFFFu) ? -1 : j[0];
      return;
    }
    u64 bk = KEY_EMPTY;
    u32 bs = 0xFFFFFFFFu;
    i32 bj = -1;
    for (int j = 0; j < SQ; j++) {
      int slot = j * 64 + lane;
      u64 k = qk[slot];
      u32 s = qs[slot];
      if (k < bk || (k == bk && s < bs)) {
        bk = k;
        bs = s;
        bj = j;
      }
    }
    mk = bk;
    ms = bs;
    mj = bj;
  }
  DEV void pl_write(int slot, const Msg& m) {
    for (int i = 0; i < PW; i++) qpl[slot * PW + i] = m.w[i];
  }
  DEV Msg pl_read(int slot) {
    Msg m;
    // (readfirstlane'd SGPR copies of the words measured 3 % slower on rmsc03, r01 s3b, and
    // neutral on rmsc02 / random_fund_value / random_fund_diverse, r05 ab_rmsc02_writes.txt)
    for (int i = 0; i < PW; i++) m.w[i] = qpl[slot * PW + i];
    for (int i = PW; i < 8; i++) m.w[i] = 0;
    return m;
  }
  // the queue's high-water mark (EnvHdr::max_q, a diagnostic): a register for the launch (loaded
  // and saved with the header) instead of an LDS read-modify-write on every push
// get_transacted_volume's duplicate test from a ballot of equal-t block starts and one shuffle per
// distance (rmsc03 x4096 37.9 -> 37.8 ms, profiles/r06/ab/ab10_tv_blocks.txt); rmsc01 keeps four
// shuffles and a ballot per distance: the new form's registers cost it 4 % though it never runs
// there (773 vs 802 ms, r06/ab/ab16_rmsc01.txt), and value_noise and rmsc02 measured the other way
// (16.4 vs 17.0 ms, 777 vs 789 ms: r06/ab/ab16_vn.txt, r06/s10/run_kernels.txt)
#ifndef MXA_TV_BLOCKS_MASK
#define MXA_TV_BLOCKS_MASK (~(1 << MXA_CFG_RMSC01))
#endif
#ifndef MXA_MAXQ_REG_MASK
  // same results: r03 s28 sparse_zi_1000 762 -> 736 ms, rmsc02 1096 -> 1084; s31 random_fund_value
  // 553 -> 541; not set where it cost: rmsc03 40.7 -> 42.8 (s28), rmsc01 1013 -> 1051 (s31).  r06
  // (profiles/r06/ab/ab2_ibm.txt, same digests): the replay step kernel, IBM x512 0.3164 -> 0.3099 ms,
  // GOOG 0.4559 -> 0.4478; its Kernel.runner twins take it too
#define MXA_MAXQ_REG_MASK ((1 << MXA_CFG_SPARSE_ZI_1000) | (1 << MXA_CFG_RMSC02) | (1 << MXA_CFG_RANDOM_FUND_VALUE) | \
                           (1 << MXA_CFG_RANDOM_FUND_DIVERSE) | (1 << MXA_CFG_HIST_FUND_VALUE) | (1 << MXA_CFG_HIST_FUND_DIVERSE) | \
                           (1 << MXA_CFG_MARKETREPLAY) | (1 << MXA_CFG_MARKETREPLAY_RUNNER) | (1 << MXA_CFG_MARKETREPLAY_TWAP))
#endif
  static constexpr bool MAXQ_REG = !BUILD && (((MXA_MAXQ_REG_MASK) >> CFG) & 1);
  static constexpr bool TVB = ((MXA_TV_BLOCKS_MASK) >> CFG) & 1;
  i32 maxq;
  DEV void note_max_q() {
    if constexpr (MAXQ_REG) maxq = qcount > maxq ? qcount : maxq;
    else if (qcount > h.max_q) h.max_q = qcount;
  }
  DEV void q_push(u64 key, u32 seq, const Msg& m) {
    PROF_SCOPE(65);
    QM use = qfree;
    if constexpr (TIER) {  // due within a second: an LDS slot; later: an HBM slot (either if full)
      const QM lm = ((QM)1 << SQL) - 1;
      const bool far = (i64)(key >> KSH) - cur > MXA_TIER_NEAR_NS;
      use = far ? (qfree & ~lm) : (qfree & lm);
      if (bal(use != 0) == 0) use = qfree;
    }
    u64 b = bal(use != 0);
    if (b == 0) {
      fail(ERR_QUEUE_FULL);
      return;
    }
    // the lowest lane with a free slot (r05: a lane chosen round-robin by seq cost a 64-bit rotate
    // on the chain; placement is invisible to the pop: replay step 0.361 -> 0.356 ms, rmsc03 41.5
    // -> 40.8, sparse_zi_1000 725 -> 721, same per-env digests), then its first free slot
    const int L = ctz64(b);
    const int jl = qm_ctz(qm_rdl(use, L));  // lane L has a free slot
    const bool me = lane == L;
    qset(jl, key, seq, me);
    // lane L's minimum and free mask by selects, not a branch: the short-circuit test inside a
    // lane-divergent region compiled to ~10 exec-mask instructions on the scalar unit per push
    const bool lt = me & ((key < mk) | ((key == mk) & (seq < ms)));
    mk = lt ? key : mk;
    ms = lt ? seq : ms;
    mj = lt ? jl : mj;
    qfree = me ? (qfree & ~qm_bit(jl)) : qfree;
    if constexpr (QHIER) q_gupd(jl, key, seq, me);
    if (PL_LDS && me) pl_write(jl * 64 + lane, m);
    if (!PL_LDS) {
      const int slot = jl * 64 + L;
      if (lane < PW) qpl[slot * PW + lane] = msel(m, lane);
    }
    qcount++;
    note_max_q();
  }
  // One q_push per active lane, in lane order (ranks 0..n-1, seqs seq..seq+n-1): the same
  // (key, seq, message) set as n q_push calls, so the pop order is unchanged; only the slot
  // placement differs, which the pop never sees. Free slots are ranked across lanes, the rank ->
  // slot table goes through LDS, each message lane writes its own slot, and every lane rescans
  // its slots once for the whole batch instead of a wave-serial push per message.
  DEV void q_push_lanes(bool act, u64 key, const Msg& m) {
    if constexpr (BLOG && PC.ex_log_orders) {  // a batch of new orders: their time_placed (send_ex)
      if (h.exlog && m_kind(m) == MK_LIMIT) bl_put_lanes(act, cur, BL_EV_PLACE, (i32)m.w[1]);
    }
    const u64 ab = bal(act);
    const int n = __popcll(ab);
    if (n == 0) return;
    const int r = (int)__builtin_amdgcn_mbcnt_hi((u32)(ab >> 32), __builtin_amdgcn_mbcnt_lo((u32)ab, 0u));
    const int c = qm_pop(qfree);
    int base = 0, total = 0;
    for (int k = 0; k < SQ; k++) {
      const u64 b = bal(c > k);
      base += (int)__builtin_amdgcn_mbcnt_hi((u32)(b >> 32), __builtin_amdgcn_mbcnt_lo((u32)b, 0u));
      total += __popcll(b);
    }
    if (total < n) {
      fail(ERR_QUEUE_FULL);
      return;
    }
    QM f = qfree;
    int tj[SQ];
    for (int t = 0; t < SQ; t++) {
      tj[t] = -1;
      if (f && base + t < n) {
        const int j = qm_ffs(f);
        f &= f - 1;
        scr[base + t] = j * 64 + lane;
        qfree &= ~qm_bit(j);
        tj[t] = j;
      }
    }
    __threadfence_block();
    if (act) {
      const int slot = scr[r];
      if constexpr (TIER) {
        qk_put(slot, key);
        qs_put(slot, seq + (u32)r);
      } else {
        qk[slot] = key;
        qs[slot] = seq + (u32)r;
      }
      Msg mw = m;
      if (r < n - 1) mw.w[0] |= MF_RUN;
      if constexpr (PL_LDS) pl_write(slot, mw);
      else
        for (int i = 0; i < PW; i++) qpl[slot * PW + i] = mw.w[i];
    }
    __threadfence_block();
    if constexpr (QHIER) {  // only the new slots changed: fold them into the group mins
      for (int t = 0; t < SQ; t++) {
        if (tj[t] < 0) break;
        const int slot = tj[t] * 64 + lane;
        if constexpr (TIER) q_gupd(tj[t], qk_get(slot), qs_get(slot));
        else q_gupd(tj[t], qk[slot], qs[slot]);
      }
      q_lanemin();
    } else {
      q_rescan();
    }
    seq += (u32)n;
    qcount += n;
    note_max_q();
  }
  // lexicographic wave-min of the per-lane cached (key, seq); returns winning slot or -1
  // three 32-bit wave-mins (key high word, key low word, seq), each only while the previous
  // word still ties across lanes: (key, seq) pairs are unique, so a single candidate lane
  // after any phase is the winner
  DEV int q_peek(u64& key, u32& seq) {
    const u32 kh = (u32)(mk >> 32), kl = (u32)mk;
    const u32 m1 = wmin_u32(kh);
    if (m1 == (u32)(KEY_EMPTY >> 32)) return -1;
    u64 b = bal(kh == m1);
    if (__popcll(b) > 1) {
      const u32 m2 = wmin_u32(kh == m1 ? kl : 0xFFFFFFFFu);
      b = bal(kh == m1 && kl == m2);
      if (__popcll(b) > 1) {
        const u32 m3 = wmin_u32((kh == m1 && kl == m2) ? ms : 0xFFFFFFFFu);
        b = bal(kh == m1 && kl == m2 && ms == m3);
      }
    }
    const int L = ctz64(b);
    key = ((u64)m1 << 32) | rdl(kl, L);
    seq = rdl(ms, L);
    return rdli(mj, L) * 64 + L;
  }
  DEV void q_remove(int slot) {
    qset(slot >> 6, KEY_EMPTY, 0xFFFFFFFFu, lane == (slot & 63));
    qfree |= (lane == (slot & 63)) ? qm_bit(slot >> 6) : (QM)0;
    if constexpr (QHIER) {
      q_regroup(slot);
      qcount--;
      return;
    }
    u64 k0 = mk;
    u32 s0 = ms;
    i32 j0 = mj;
    q_rescan();  // every lane rescans (no divergence); only the owner lane keeps the result
    bool me = lane == (slot & 63);
    mk = me ? mk : k0;
    ms = me ? ms : s0;
    mj = me ? mj : j0;
    qcount--;
  }
  DEV void q_rekey(int slot, u64 key) {
    qsetk(slot >> 6, key, lane == (slot & 63));
    if constexpr (QHIER) {
      q_regroup(slot);
      return;
    }
    u64 k0 = mk;
    u32 s0 = ms;
    i32 j0 = mj;
    q_rescan();
    bool me = lane == (slot & 63);
    mk = me ? mk : k0;
    ms = me ? ms : s0;
    mj = me ? mj : j0;
  }

  // ---------------- kernel services
  // Kernel.sendMessage (Kernel.py:347-425)
  DEV void send(int recipient, const Msg& m, i64 delay) {
    PROF_SCOPE(64);
    i64 sent = cur + rg64(AF_COMP) + add_delay + delay;
    i64 deliver;
    if (PC.lat_mode == 2) {
      double x;
      if constexpr (KREG) {
        RS L = grs_k();
        x = rs_uniform(L, PC.clip, 1.0);
        grs_put_k(L);
      } else {
        RS L = grs(3);
        x = rs_uniform(L, PC.clip, 1.0);
        grs_put(3, L);
      }
      double mn = cur_agent == 0 ? lat()[recipient] : lat()[PC.n_agents + cur_agent];
      double l = mn + ((PC.jitter / gm_pow(x, 3.0)) * (mn / PC.unit));
      deliver = sent + (i64)l;
    } else {
      double l = 0.0;
      if (PC.lat_mode == 1) {
        const int li = cur_agent == 0 ? recipient : (PC.lat_asym ? PC.n_agents : 0) + cur_agent;
        if constexpr (LATL > 0) l = latl[li];
        else l = lat()[li];
      }
      i64 noise = 0;
      if (PC.noise_len > 1) {
        if constexpr (KREG) {
          RS K = grs_k();
          noise = rs_randint(K, 0, PC.noise_len);
          grs_put_k(K);
        } else {
          RS K = grs(2);
          noise = rs_randint(K, 0, PC.noise_len);
          grs_put(2, K);
        }
      }
      deliver = sent + (i64)(l + (double)noise);
    }
    u64 key = ((u64)deliver << KSH) | ((u64)recipient << 2) | MT_MESSAGE;
    q_push(key, seq++, m);
  }
  // Kernel.setWakeup (Kernel.py:435-462)
  DEV void wakeup_at(int agent, i64 t) {
    if (t < cur) {
      fail(ERR_WAKEUP_PAST);
      return;
    }
    Msg m = msg_make(MK_WAKEUP, 0);
    u64 key = ((u64)t << KSH) | ((u64)agent << 2) | MT_WAKEUP;
    q_push(key, seq++, m);
  }
  // Order.generateOrderId (Order.py:35-42): the smallest id >= the counter that no Order of this
  // process holds; ocnt is the next candidate.  Only the replay's explicit tape ids can be met
  // (every auto id is below ocnt), and only from the second episode of a process on
  DEV i64 next_order_id() {
    if constexpr (RP) {
      i64 c = ocnt;
      if (c >= (i64)U(rx->umin)) c = rp_skip_used(c);
      ocnt = c + 1;
      return c;
    }
    return ocnt++;
  }

  // ---------------- ExternalFileOracle (util/oracle/ExternalFileOracle.py:52-159)
  static constexpr bool EXT = PC.oracle_ext != 0;
  // pandas Timedelta.total_seconds(): days * 86400 + seconds (an int) + microseconds / 1e6 of
  // the duration floored to whole microseconds (nanoseconds dropped; measured, pandas 2.3.3)
  static DEV double td_seconds(i64 ns) {
    const i64 us = ns >= 0 ? ns / 1000 : -((-ns + 999) / 1000);
    const i64 s = us >= 0 ? us / 1000000 : -((-us + 999999) / 1000000);
    return (double)s + (double)(us - s * 1000000) / 1000000.0;
  }
  // getPriceAtTime (:52-97): the first / last value outside the series, else bisect_left and
  // getInterpolatedPrice (:131-159) between the entries either side; a query at the first
  // timestamp reads lower index -1 (Python's series[-1], the last entry), as the reference does
  DEV double efo_price(i64 t) {
    const i32 n = U(rx->fs_n);
    const i64* T = rx->fs_t;
    const double* V = rx->fs_v;
    if (t < U(T[0])) return V[0];
    if (t > U(T[n - 1])) return V[n - 1];
    i32 lo = 0, hi = n;
    while (lo < hi) {  // bisect_left
      const i32 mid = (lo + hi) >> 1;
      if (U(T[mid]) < t) lo = mid + 1;
      else hi = mid;
    }
    i32 li = lo - 1;
    const i32 ui = li < n - 1 ? li + 1 : li;
    if (li < 0) li += n;
    const double pl = V[li], ph = V[ui];
    const i64 tl = U(T[li]), th = U(T[ui]);
    const double slope = pl != ph ? (ph - pl) / td_seconds(th - tl) : 0.0;
    const double v = pl + td_seconds(t - tl) * slope;
    if constexpr (BLOG) efo_log(t, v);  // f_log[symbol].append (:97): the interpolating branch only
    return v;
  }
  // ExternalFileOracle.f_log entry (FundamentalTime, FundamentalValue): two book-log records
  DEV void efo_log(i64 t, double v) {
    const u64 b = as_u(v);
    bl_put(t, BL_FUND_LO, (i32)(u32)b);
    bl_put(t, BL_FUND_HI, (i32)(u32)(b >> 32));
  }
  // the value agents' r_bar = oracle.fundamentals[symbol].values[0] and sigma_n = r_bar / 10
  // (config/hist_fund_value.py:80-82), else the config's constants
  DEV double v_rbar() {
    if constexpr (EXT) return rx->fs_v[0];
    else return PC.v_rbar;
  }
  DEV double v_sigma_n() {
    if constexpr (EXT) return rx->fs_v[0] / 10;
    else return PC.v_sigma_n;
  }

  // ---------------- SparseMeanRevertingOracle (SMRO:88-227)
  DEV double o_compute(i64 ts, double v_adj, i64 pt, double pv) {
    i64 d = ts - pt;
    double mu = PC.o_rbar, gamma = PC.o_kappa, theta = PC.o_fundvol;
    // the two exponentials are independent: lane 0 and lane 1 of ONE gm_exp evaluation.
    // theta ** 2 (a constant of the config) was evaluated with the same glibc pow at build time
    const double ex = gm_exp(lane == 0 ? -gamma * (double)d : -2 * gamma * (double)d);
    double loc = mu + (pv - mu) * rdl_d(ex, 0);
    double scale = (h.o_th2 / (2 * gamma)) * (1 - rdl_d(ex, 1));
    (void)theta;
    RS O = grs(1);
    double v = rs_normal(O, loc, scale);
    grs_put(1, O);
    v += v_adj;
    if (!(v > 0)) v = 0;
    i64 vi = py_round(v);
    h.o_pt = ts;
    h.o_pv = (double)vi;
    if constexpr (BLOG) bl_put(ts, BL_FUNDAMENTAL, (i32)vi);  // f_log (SMRO:122)
    return (double)vi;
  }
  DEV double o_advance(i64 t) {
    i64 pt = h.o_pt;
    double pv = h.o_pv;
    if (t <= pt) return pv;
    while (h.o_mst < t) {
      double v = o_compute(h.o_mst, h.o_msv, pt, pv);
      pt = h.o_mst;
      pv = v;
      RS G = grs(0);
      h.o_mst = pt + (i64)rs_exponential(G, 1.0 / PC.o_lambda);
      grs_put(0, G);
      RS O = grs(1);
      double msv = rs_normal(O, PC.o_msmean, __builtin_sqrt(PC.o_msvar));
      h.o_msv = rs_randint(O, 0, 2) == 0 ? msv : -msv;
      grs_put(1, O);
    }
    return o_compute(t, 0, pt, pv);
  }
  DEV i64 o_observe(i64 t, double sigma_n) {
    PROF_SCOPE(69);
    if constexpr (EXT) {  // ExternalFileOracle.observePrice (ExternalFileOracle.py:110-129): no clamp, no draws
      const double tp = efo_price(t);
      if (sigma_n == 0) return py_round(tp);
      RS A = agent_rs();
      const i64 obs = py_round(rs_normal(A, tp, __builtin_sqrt(sigma_n)));
      agent_rs_put(A);
      return obs;
    }
    double r_t = t >= PC.mkt_close ? o_advance(PC.mkt_close - 1) : o_advance(t);
    if (sigma_n == 0) return (i64)r_t;
    RS A = agent_rs();
    i64 obs = py_round(rs_normal(A, r_t, __builtin_sqrt(sigma_n)));
    agent_rs_put(A);
    return obs;
  }

  // ---------------- order book pool (VGPR resident)
  // (a best-price cache, invalidated when an order at the cached price leaves, measured slower in
  // round 3: rmsc03 40.6 -> 44.8 ms, sparse_zi_1000 unchanged)
  DEV i32 b_best(int buy_side) {  // best bid (max) or best ask (min); INT_MIN/INT_MAX if empty
    PROF_SCOPE(68);
    i32 v = buy_side ? INT32_MIN : INT32_MAX;
    for (int j = 0; j < SO; j++) {
      bool m = bm[j] >= 0 && (bm[j] & 1) == buy_side;
      if (m) v = buy_side ? (bp[j] > v ? bp[j] : v) : (bp[j] < v ? bp[j] : v);
    }
    v = buy_side ? wmax_i32(v) : wmin_i32(v);
    return v;
  }
  DEV i64 b_level_qty(int buy_side, i32 price) {
    i64 s = 0;
    for (int j = 0; j < SO; j++)
      if (bm[j] >= 0 && (bm[j] & 1) == buy_side && bp[j] == price) s += bq[j];
    return wsum_i64(s);
  }
  // the SPREAD reply's inside of both sides in two fused passes (OrderBook.getInsideBids/Asks(1)):
  // best bid / ask (INT_MIN / INT_MAX if a side is empty) and the quantity at each.  The level
  // sums take one packed 32-bit wave sum when every lane's partials are below 2^10 (the totals
  // then fit 16 bits each), else two 64-bit ones.  b_best x2 + b_level_qty x2 before: four passes
  // over the pool and six DPP reductions
  DEV void b_inside(i32& bb, i32& aa, i64& bqs, i64& aqs) {
    i32 vb = INT32_MIN, va = INT32_MAX;
    for (int j = 0; j < SO; j++) {
      const bool live = bm[j] >= 0, buy = (bm[j] & 1) != 0;
      vb = live && buy && bp[j] > vb ? bp[j] : vb;
      va = live && !buy && bp[j] < va ? bp[j] : va;
    }
    bb = wmax_i32(vb);
    aa = wmin_i32(va);
    i64 sb = 0, sa = 0;
    for (int j = 0; j < SO; j++) {
      const bool live = bm[j] >= 0, buy = (bm[j] & 1) != 0;
      sb += live && buy && bp[j] == bb ? (i64)bq[j] : 0;
      sa += live && !buy && bp[j] == aa ? (i64)bq[j] : 0;
    }
    if (!bal(sb >= 1024 || sa >= 1024)) {
      const u32 t = wsum_u32((u32)sb | ((u32)sa << 16));
      bqs = t & 0xFFFF;
      aqs = t >> 16;
    } else {
      bqs = wsum_i64(sb);
      aqs = wsum_i64(sa);
    }
  }
  // FIFO head of a price level: min arrival; returns slot j*64+L
  DEV int b_head(int buy_side, i32 price) {
    u32 a = 0xFFFFFFFFu;
    for (int j = 0; j < SO; j++)
      if (bm[j] >= 0 && (bm[j] & 1) == buy_side && bp[j] == price && ba[j] < a) a = ba[j];
    u32 amin = wmin_u32(a);
    for (int j = 0; j < SO; j++) {
      u64 b = bal(bm[j] >= 0 && (bm[j] & 1) == buy_side && bp[j] == price && ba[j] == amin);
      if (b) return j * 64 + ctz64(b);
    }
    return -1;
  }
  DEV int b_find(int buy_side, i32 price, i32 oid) {
    for (int j = 0; j < SO; j++) {
      u64 b = bal(bm[j] >= 0 && (bm[j] & 1) == buy_side && bp[j] == price && bo[j] == oid);
      if (b) return j * 64 + ctz64(b);
    }
    return -1;
  }
  template <class A>
  DEV i32 b_get(const A& arr, int slot) {
    if constexpr (!std::is_array<A>::value) {  // LDS: one broadcast read
      return __builtin_amdgcn_readfirstlane((i32)arr.p[slot - lane]);
    } else {
      i32 v = 0;
      for (int j = 0; j < SO; j++)
        if (j == (slot >> 6)) v = rdli(arr[j], slot & 63);
      return v;
    }
  }
  template <class A>
  DEV void b_set(A& arr, int slot, i32 v) {
    if constexpr (!std::is_array<A>::value) {
      if (lane == (slot & 63)) arr.p[slot - lane] = v;
    } else {
      for (int j = 0; j < SO; j++)
        if (j == (slot >> 6) && lane == (slot & 63)) arr[j] = v;
    }
  }
  DEV int b_free_slot() {
    for (int j = 0; j < SO; j++) {
      u64 b = bal(bm[j] < 0);
      if (b) return j * 64 + ctz64(b);
    }
    return -1;
  }
  // OrderBook.getInsideBids/Asks(depth) level count (distinct prices, at most `cap`) from the best
  // price `best` toward worse prices; the level-2 price in `second` (0 without one)
  DEV i32 b_levels(int buy_side, i32 best, i32 cap, i32& second) {
    i32 n = 1, p = best;
    second = 0;
    while (n < cap) {
      i32 v = buy_side ? INT32_MIN : INT32_MAX;
      for (int j = 0; j < SO; j++) {
        bool m = bm[j] >= 0 && (bm[j] & 1) == buy_side && (buy_side ? bp[j] < p : bp[j] > p);
        if (m) v = buy_side ? (bp[j] > v ? bp[j] : v) : (bp[j] < v ? bp[j] : v);
      }
      v = buy_side ? wmax_i32(v) : wmin_i32(v);
      if (v == (buy_side ? INT32_MIN : INT32_MAX)) break;
      if (n == 1) second = v;
      n++;
      p = v;
    }
    return n;
  }
  DEV void b_enter(i32 oid, i32 agent, int is_buy, i32 qty, i32 price, i32 hep, i32 ridx = 0) {
    int s = b_free_slot();
    if (s < 0) {
      fail(ERR_BOOK_FULL);
      return;
    }
    u32 arr = h.arrival++;
    for (int j = 0; j < SO; j++)
      if (j == (s >> 6) && lane == (s & 63)) {
        bp[j] = price;
        bq[j] = qty;
        bo[j] = oid;
        bm[j] = (agent << 1) | is_buy;
        ba[j] = arr;
        bh[j] = hep;
        if constexpr (OH) bx[j] = ridx;
      }
    h.b_count++;
    if (h.b_count > h.max_book) h.max_book = h.b_count;
  }
  DEV void b_free(int s) {
    b_set(bm, s, -1);
    h.b_count--;
  }

  // ---------------- OrderBook.history transaction ring (OrderBook.py:146-149, 227-237, 400-436)
  DEV void tx_add(i64 t, i32 q, i32 ep) {
    TxRec* R = txr();
    int cap = PC.L.tx_cap;
    int pos = h.tx_head % cap;
    if (h.tx_head >= cap) {  // overwriting the oldest record: it must be dead
      TxRec old = R[pos];
      if (old.epoch >= h.epoch - PC.stream_history) {
        fail(ERR_TX_FULL);
        return;
      }
    }
    if (lane == 0) {
      TxRec r;
      r.t = t;
      r.q = q;
      r.epoch = ep;
      R[pos] = r;
    }
    h.tx_head++;
  }
  DEV i64 transacted_volume(i64 lookback, int* perr) {
    int lo_ep = h.epoch - PC.stream_history;
    i32 entries = 0;
    LDSP i32* EP = ep_entries();
    for (int e = lo_ep < 0 ? 0 : lo_ep; e <= h.epoch; e++) entries += EP[e & 15];
    if (entries == 0) return 0;
    TxRec* R = txr();
    int cap = PC.L.tx_cap;
    int n = h.tx_head < cap ? h.tx_head : cap;
    int first = h.tx_head - n;
    i64 start = cur - lookback;
    i64 vol = 0;
    // Newest records first, 64 per chunk (lane L = record lo + L, chronological).  Records are
    // appended in time order, so once a chunk's oldest record is before `start` every older
    // record is too, and the window is usually inside the newest chunk.  Whether ANY live
    // record exists (pandas raising otherwise) is decided by the newest chunk: a maker logs its
    // own entry epoch, which is never above the epoch its taker logs in the same match, and
    // epochs never decrease, so the newest taker record (one of the two newest records) holds
    // the largest epoch of the ring.  Duplicate (t, q) pairs sit in one contiguous equal-t
    // block: lanes compare with their predecessors by shuffles, and only a block that crosses
    // into the older chunk walks back through memory.
    bool any = false;
    for (int hi = n; hi > 0; hi -= 64) {
      const int lo = hi > 64 ? hi - 64 : 0;
      const int k = lo + lane;
      const bool valid = k < hi;
      TxRec r;
      r.t = 0;
      r.q = 0;
      r.epoch = -1;
      if (valid) r = R[(first + k) % cap];
      const bool live = valid && r.epoch >= lo_ep;
      const bool inwin = valid && r.t >= start;
      if (hi == n) any = bal(live) != 0;
      bool dup = false;
      if constexpr (!TVB) {  // per distance: four shuffles and a ballot
        for (int d = 1; d < 64; d++) {
          const int src = lane - d < 0 ? 0 : lane - d;
          const i64 pt = (i64)(((u64)(u32)__shfl((i32)((u64)r.t >> 32), src, 64) << 32) |
                               (u32)__shfl((i32)(u32)(u64)r.t, src, 64));
          const i32 pq = __shfl(r.q, src, 64), pe = __shfl(r.epoch, src, 64);
          const bool same = lane - d >= 0 && pt == r.t;
          dup = dup || (same && pe >= lo_ep && pq == r.q);
          if (!bal(same && live && inwin && !dup)) break;
        }
      } else {  // equal-t blocks from one ballot of block starts, then one shuffle per distance
        const int src1 = lane == 0 ? 0 : lane - 1;
        const i64 pt = (i64)(((u64)(u32)__shfl((i32)((u64)r.t >> 32), src1, 64) << 32) |
                             (u32)__shfl((i32)(u32)(u64)r.t, src1, 64));
        const u64 S = bal(lane == 0 || pt != r.t);
        const u64 below = lane == 63 ? S : S & ((2ull << lane) - 1);
        const int bs = 63 - __clzll((long long)below);  // bit 0 is always set
        const int dmax = wmax_i32(live && inwin ? lane - bs : 0);
        const i32 qk = live ? r.q : INT32_MIN;
        for (int d = 1; d <= dmax; d++) {
          const i32 pq = __shfl(qk, lane - d < 0 ? 0 : lane - d, 64);
          dup = dup || (lane - d >= bs && pq == r.q);
        }
      }
      if (lo > 0) {  // an equal-t block that started in the older chunk
        const TxRec o = R[(first + lo - 1) % cap];
        const i64 t0 = (i64)rdl64((u64)r.t, 0);
        if (U(o.t) == t0) {
          for (int j = lo - 1; live && inwin && !dup && r.t == o.t && j >= 0; j--) {
            const TxRec p = R[(first + j) % cap];
            if (p.t != r.t) break;
            if (p.epoch >= lo_ep && p.q == r.q) dup = true;
          }
        }
      }
      vol += wsum_i64((live && !dup && inwin) ? (i64)r.q : 0);
      if (!(bal(inwin) & 1ull)) break;  // the chunk's oldest record is before the window
    }
    if (!any) *perr = 1;  // pandas raises when no transaction records exist
    return vol;
  }

  // ---------------- OrderBook.handleLimitOrder / executeOrder / cancelOrder
  DEV void ex_notify(int recipient, const Msg& m) {
    // ExchangeAgent.sendMessage: ORDER_* notifications carry the pipeline delay
    u32 k = m_kind(m);
    i64 d = (k == MK_ACCEPTED || k == MK_CANCELLED || k == MK_EXECUTED) ? PC.ex_pipeline : 0;
    // ... and, with log_orders, are logged with their order (ExchangeAgent.py:477-482)
    if constexpr (BLOG && PC.ex_log_orders)
      if (h.exlog && (k == MK_ACCEPTED || k == MK_CANCELLED || k == MK_EXECUTED)) {
        bl_put(cur, BL_EV_NT + (i32)k, recipient);
        exl_order(m, k == MK_EXECUTED ? (i32)m.w[4] : (i32)BL_FILL_NONE);
      }
    send(recipient, m, d);
  }
  // ---------------- OrderBook.history as a ring of per-order records (HBL configurations)
  DEV OhRec* ohr() { return (OhRec*)(env + PC.L.off_oh); }
  // history[0][order_id] = {...} (OrderBook.py:52-60): one record per handled limit order
  DEV i32 oh_append(i32 oid, i32 price, int is_buy) {
    const i32 r = h.oh_head;
    if (lane == 0) {
      OhRec x;
      x.oid = oid;
      x.price = price;
      x.meta = is_buy;
      x.epoch = h.epoch;
      ohr()[r % PC.L.oh_cap] = x;
    }
    h.oh_head = r + 1;
    return r;
  }
  // an order's "transactions" list becomes non-empty (its record still in the ring)
  DEV void oh_mark_tx(i32 r) {
    if (h.oh_head - r <= PC.L.oh_cap && lane == 0) ohr()[r % PC.L.oh_cap].meta |= 2;
  }
  // ---------------- book-update log (OrderBook.book_log rows, ExchangeAgent BEST_BID/ASK/LAST_TRADE)
  // one record per handled limit order and per cancellation; the host replays the level
  // volumes (matching at level granularity is exact: a level gives min(remaining, volume))
  // (past the capacity the count still advances, so the kernelStopping pass, which cannot
  // fail an env, leaves an overflow the host sees)
  DEV void bl_put(i64 t, i32 price, i32 qty) {
    const i32 n = h.blog_n;
    if (n < blog_cap && lane == 0) {
      BlRec r;
      r.t = t;
      r.price = price;
      r.qty = qty;
      blog[n] = r;
    }
    h.blog_n = n + 1;
    if (n >= blog_cap) fail(ERR_BOOK_LOG_FULL);
  }
  // one record per active lane, in lane order (a batched push of orders)
  DEV void bl_put_lanes(bool act, i64 t, i32 price, i32 qty) {
    const u64 ab = bal(act);
    const i32 n = h.blog_n, c = __popcll(ab);
    if (c == 0) return;
    const i32 r = (i32)__builtin_amdgcn_mbcnt_hi((u32)(ab >> 32), __builtin_amdgcn_mbcnt_lo((u32)ab, 0u));
    if (act && n + r < blog_cap) {
      BlRec x;
      x.t = t;
      x.price = price;
      x.qty = qty;
      blog[n + r] = x;
    }
    h.blog_n = n + c;
    if (n + c > blog_cap) fail(ERR_BOOK_LOG_FULL);
  }
  // the exchange's own log (ExchangeAgent.log, EXCHANGE_AGENT.bz2; mxa_set_exchange_log): the order
  // record that follows a LIMIT_ORDER / CANCEL_ORDER or an ORDER_* notification row (mxa_layout.h)
  DEV void exl_order(const Msg& m, i32 fill) {
    const i32 q = (i32)m.w[2];
    bl_put((i64)(((u64)(u32)fill << 32) | (u64)m.w[1]), (i32)m.w[3], m_buy(m) ? q : -q);
  }
  DEV void handle_limit(i32 oid, i32 agent, int is_buy, i32 qty, i32 price) {
    PROF_SCOPE(66);
    if (qty <= 0) return;
    if constexpr (BLOG) bl_put(cur, price, is_buy ? qty : -qty);
    i32 hep = h.epoch;
    LDSP i32* EP = ep_entries();
    i32 ne = EP[h.epoch & 15] + 1;
    if (lane == 0) EP[h.epoch & 15] = ne;
    i32 ridx = 0;
    if constexpr (OH) ridx = oh_append(oid, price, is_buy);
    i64 ex_q = 0, ex_pq = 0;
    bool executed = false;
    for (;;) {
      int opp = is_buy ? 0 : 1;  // resting side: asks for a buy (is_buy == 0)
      i32 best = b_best(opp);
      bool any = opp ? best != INT32_MIN : best != INT32_MAX;
      bool match = any && (is_buy ? price >= best : price <= best);
      if (match) {
        int s = b_head(opp, best);
        i32 hq = b_get(bq, s), ho = b_get(bo, s), hm = b_get(bm, s), hh = b_get(bh, s);
        i32 mq;
        if (qty >= hq) {
          mq = hq;
          b_free(s);
        } else {
          mq = qty;
          b_set(bq, s, hq - qty);
        }
        // history: taker logs its pre-match remaining qty; maker its matched qty if retained
        tx_add(cur, qty, h.epoch);
        if (hh >= h.epoch - PC.stream_history) tx_add(cur, mq, hh);
        if constexpr (OH) {
          const i32 mx = b_get(bx, s);
          oh_mark_tx(ridx);
          if (hh >= h.epoch - PC.stream_history) oh_mark_tx(mx);
        }
        qty -= mq;
        Msg mt = msg_order(MK_EXECUTED, oid, agent, is_buy, mq, price, best);
        ex_notify(agent, mt);
        Msg mm = msg_order(MK_EXECUTED, ho, hm >> 1, hm & 1, mq, best, best);
        ex_notify(hm >> 1, mm);
        ex_q += mq;
        ex_pq += (i64)best * mq;
        executed = true;
        if (qty <= 0) break;
      } else {
        b_enter(oid, agent, is_buy, qty, price, hep, ridx);
        Msg ma = msg_order(MK_ACCEPTED, oid, agent, is_buy, qty, price, 0);
        ex_notify(agent, ma);
        break;
      }
      if (status == ST_ERROR) return;
    }
    if (executed) {
      h.last_trade = py_round((double)ex_pq / (double)ex_q);
      h.last_trade_float = 0;
      h.epoch++;
      if (lane == 0) EP[h.epoch & 15] = 0;
    }
    if constexpr (MD) {  // OrderBook.py:169
      h.ob_last_update = cur;
      h.has_last_update = 1;
    }
  }
  DEV void cancel_order(const Msg& m) {
    PROF_SCOPE(67);
    int buy = m_buy(m);
    int s = b_find(buy, (i32)m.w[3], (i32)m.w[1]);
    if (s < 0) return;
    i32 q = b_get(bq, s), o = b_get(bo, s), mm = b_get(bm, s), p = b_get(bp, s);
    b_free(s);
    if constexpr (BLOG) bl_put(cur, -p, buy ? q : -q);
    Msg r = msg_order(MK_CANCELLED, o, mm >> 1, mm & 1, q, p, 0);
    ex_notify(m_agent(m), r);
    if constexpr (MD) {  // OrderBook.py:338
      h.ob_last_update = cur;
      h.has_last_update = 1;
    }
  }

  // ---------------- market-data subscriptions (ExchangeAgent.py:342-387)
  // updateSubscriptionDict: a request (re)sets the sender's entry in place, a cancellation
  // deletes its symbol (the entry stays, empty)
  DEV void md_subscribe(const Msg& m) {
    h.md_next_due = 0;  // the due-time cache is rebuilt by the next publish
    const i32 sender = m_agent(m);
    SubRec* S = subs();
    const i32 ns = h.nsub;
    const bool mine = lane < ns && S[lane < MD_MAX_SUBS ? lane : 0].agent == sender;
    const u64 hit = bal(mine);
    const int i = hit ? ffs64(hit) : ns;
    if (m_kind(m) == MK_MD_SUB_CANCEL) {
      if (!hit || !U(S[i].live)) {
        fail(ERR_MD_KEYERROR);
        return;
      }
      if (lane == 0) S[i].live = 0;
      return;
    }
    if (i >= MD_MAX_SUBS) {
      fail(ERR_MD_SUBS);
      return;
    }
    if (lane == 0) {
      SubRec r;
      r.agent = sender;
      r.levels = (i32)m.w[1];
      r.live = 1;
      r.pad = 0;
      r.freq = m_i64(m, 2);
      r.last = cur;
      S[i] = r;
    }
    if (!hit) h.nsub = ns + 1;
  }
  // publishOrderBookData: every subscription, in insertion order, whose freq is 0 or whose last
  // update is at least freq ns before the book's gets the top `levels` of both sides and the last
  // trade.  The best levels travel in the message; the deeper prices wait in the subscriber's slot
  // (freq >= the latency keeps one MARKET_DATA in flight per subscriber; a second one fails)
  DEV void md_publish() {
    // nothing comes due before h.md_next_due (kept by the previous publish): no table read
    if (!h.md_any0 && h.has_last_update && h.ob_last_update < h.md_next_due) return;
    const i32 ns = h.nsub;
    SubRec* S = subs();
    SubRec r;
    r.agent = r.levels = r.live = 0;
    r.freq = r.last = 0;
    if (lane < ns) r = S[lane];
    const bool live = lane < ns && r.live;
    const bool due = live && (r.freq == 0 || (h.has_last_update && h.ob_last_update > r.last &&
                                              (double)(h.ob_last_update - r.last) >= (double)r.freq));
    if (bal(live && r.freq != 0 && !h.has_last_update)) {
      fail(ERR_MD_NO_UPDATE);
      return;
    }
    {  // the earliest update time at which a freq > 0 subscription comes due, after this publish
      const i64 nl = due ? h.ob_last_update : r.last;
      h.md_next_due = (i64)wmin_u64(live && r.freq > 0 ? (u64)(nl + r.freq) : ~0ull);
      h.md_any0 = bal(live && r.freq <= 0) != 0;
    }
    u64 b = bal(due);
    if (!b) return;
    if (bal(due && (r.levels < 0 || r.levels > MD_LEVELS))) {
      fail(ERR_MD_SUBS);
      return;
    }
    // the book's top levels once (as deep as the deepest due subscription), lane-distributed in
    // the slot layout: lane MD_BIDS + k the k-th bid price, MD_BIDQ + k its volume, asks alike
    const i32 maxlv = wmax_i32(due ? r.levels : 0);
    u32 snap = 0;
    i32 nb = 0, na = 0;
    for (int side = 1; side >= 0; side--) {
      i32 p = side ? INT32_MAX : INT32_MIN;
      i32 c = 0;
      for (int k = 0; k < maxlv; k++) {
        i32 v = side ? INT32_MIN : INT32_MAX;
        for (int j = 0; j < SO; j++) {
          const bool in = bm[j] >= 0 && (bm[j] & 1) == side && (side ? bp[j] < p : bp[j] > p);
          if (in) v = side ? (bp[j] > v ? bp[j] : v) : (bp[j] < v ? bp[j] : v);
        }
        v = side ? wmax_i32(v) : wmin_i32(v);
        if (v == (side ? INT32_MIN : INT32_MAX)) break;
        const i64 q = b_level_qty(side, v);
        snap = lane == (side ? MD_BIDS : MD_ASKS) + k ? (u32)v : snap;
        snap = lane == (side ? MD_BIDQ : MD_ASKQ) + k ? (u32)q : snap;
        p = v;
        c++;
      }
      if (side) nb = c;
      else na = c;
    }
    while (b) {
      const int L = ctz64(b);
      b &= b - 1;
      const i32 ag = rdli(r.agent, L), lv = rdli(r.levels, L);
      const i32 nbs = nb < lv ? nb : lv, nas = na < lv ? na : lv;
      const u32 tag = ++h.md_seq;
      u32* slot = md_slot(ag);
      const int j = lane;
      const bool keep = (j >= MD_BIDS && j < MD_BIDS + nbs) || (j >= MD_ASKS && j < MD_ASKS + nas) ||
                        (j >= MD_BIDQ && j < MD_BIDQ + nbs) || (j >= MD_ASKQ && j < MD_ASKQ + nas);
      const u32 w = j == MD_TAG ? tag : j == MD_COUNTS ? ((u32)nbs | ((u32)nas << 8)) : keep ? snap : 0u;
      if (lane < MD_WORDS) slot[lane] = w;
      Msg md = msg_make(MK_MARKET_DATA, 0);
      md.w[0] |= (1u << 11) | ((u32)h.last_trade_float << 8);
      md.w[1] = nbs ? rdl(snap, MD_BIDS) : 0;
      md.w[2] = nbs ? rdl(snap, MD_BIDQ) : 0;
      md.w[3] = nas ? rdl(snap, MD_ASKS) : 0;
      md.w[4] = nas ? rdl(snap, MD_ASKQ) : 0;
      md.w[5] = (u32)h.last_trade;
      md.w[6] = (u32)nbs | ((u32)nas << 8);
      md.w[7] = tag;
      ex_notify(ag, md);
      if (lane == L) S[L].last = h.ob_last_update;
    }
  }

  // ExchangeAgent.receiveMessage (ExchangeAgent.py:129-340)
  DEV void ex_receive(const Msg& m) {
    PROF_SCOPE(73);
    rs64(AF_COMP, PC.ex_comp);
    u32 k = m_kind(m);
    i32 sender = m_agent(m);
    bool closed = cur > PC.mkt_close;
    if (closed) {
      if (k == MK_LIMIT || k == MK_CANCEL || k == MK_MODIFY) {
        ex_notify(sender, msg_make(MK_MKT_CLOSED, 0));
        return;
      } else if (k == MK_SPREAD_REQ || k == MK_LAST_REQ || k == MK_TV_REQ || k == MK_STREAM_REQ) {
      } else {
        ex_notify(sender, msg_make(MK_MKT_CLOSED, 0));
        return;
      }
    }
    // the exchange's log (ExchangeAgent.py:162-167): order messages with their order, and only
    // with log_orders; every other message with its sender
    if constexpr (BLOG) {
      if (h.exlog) {
        const bool ord = k == MK_LIMIT || k == MK_CANCEL;
        if (!ord || PC.ex_log_orders) {
          bl_put(cur, BL_EV_RX + (i32)k, sender);
          if (ord) exl_order(m, (i32)BL_FILL_NONE);
        }
      }
    }
    if constexpr (RP) {
      if (k == MK_LIMIT) return rp_handle_limit(m);
      if (k == MK_CANCEL) return rp_cancel(m);
      if (k == MK_MODIFY) return rp_modify(m);
      if (k == MK_SPREAD_REQ) return rp_spread(m, closed);
    }
    switch (k) {
    case MK_WHEN_OPEN_REQ:
    case MK_WHEN_CLOSE_REQ: {
      rs64(AF_COMP, 0);
      Msg r = msg_make(k == MK_WHEN_OPEN_REQ ? MK_WHEN_OPEN : MK_WHEN_CLOSE, 0);
      i64 d = k == MK_WHEN_OPEN_REQ ? PC.mkt_open : PC.mkt_close;
      r.w[0] |= 1u << 11;
      r.w[1] = (u32)(u64)d;
      r.w[2] = (u32)((u64)d >> 32);
      ex_notify(sender, r);
      break;
    }
    case MK_LAST_REQ: {
      Msg r = msg_make(MK_LAST, 0);
      u32 hasd = 1;
      if constexpr (RP) hasd = (u32)U(rh()->ex_has_last);
      r.w[0] |= (hasd << 11) | ((u32)h.last_trade_float << 8) | ((u32)closed << 7);
      r.w[5] = (u32)h.last_trade;
      ex_notify(sender, r);
      break;
    }
    case MK_SPREAD_REQ: {
      i32 depth = (i32)m.w[1];
      Msg r = msg_make(MK_SPREAD, 0);
      i32 bb, aa;
      i64 bqs, aqs;
      b_inside(bb, aa, bqs, aqs);
      bool hb = bb != INT32_MIN && depth > 0, ha = aa != INT32_MAX && depth > 0;
      if (hb) {
        r.w[1] = (u32)bb;
        r.w[2] = (u32)bqs;
      }
      if (ha) {
        r.w[3] = (u32)aa;
        r.w[4] = (u32)aqs;
      }
      r.w[5] = (u32)h.last_trade;
      r.w[0] |= ((u32)hb << 9) | ((u32)ha << 10) | (1u << 11) | ((u32)h.last_trade_float << 8) | ((u32)closed << 7);
      if constexpr (PW == 8) {  // level counts and level-2 prices (w6/w7 = price2 | count << 20)
        i32 b2 = 0, a2 = 0;
        i32 nb = hb ? b_levels(1, bb, depth, b2) : 0, na = ha ? b_levels(0, aa, depth, a2) : 0;
        if ((u32)b2 >= (1u << 20) || (u32)a2 >= (1u << 20)) fail(ERR_RP_PRICE);
        r.w[6] = (u32)b2 | ((u32)nb << 20);
        r.w[7] = (u32)a2 | ((u32)na << 20);
      }
      ex_notify(sender, r);
      break;
    }
    case MK_TV_REQ: {
      int perr = 0;
      i64 vol = transacted_volume(m_i64(m, 1), &perr);
      if (perr) {
        fail(ERR_PANDAS_NO_TX);
        return;
      }
      Msg r = msg_make(MK_TV, 0);
      r.w[0] |= (1u << 11) | ((u32)closed << 7);
      r.w[1] = (u32)(u64)vol;
      r.w[2] = (u32)((u64)vol >> 32);
      ex_notify(sender, r);
      break;
    }
    case MK_STREAM_REQ: {  // QUERY_ORDER_STREAM (ExchangeAgent.py:251-279): history[1 : length + 1]
      if constexpr (OH) {
        const i32 avail = h.epoch < PC.stream_history ? h.epoch : PC.stream_history;  // len(history) - 1
        const i32 len = (i32)m.w[1] < avail ? (i32)m.w[1] : avail;
        const i64 hi = (i64)h.epoch - 1;  // absolute epoch of history[1]
        Msg r = msg_make(MK_STREAM, 0);
        r.w[0] |= (1u << 11) | ((u32)closed << 7);
        r.w[1] = (u32)(len < 0 ? 0 : len);
        r.w[2] = (u32)(u64)hi;
        r.w[3] = (u32)((u64)hi >> 32);
        ex_notify(sender, r);
      }
      break;
    }
    case MK_LIMIT:
      handle_limit((i32)m.w[1], sender, m_buy(m), (i32)m.w[2], (i32)m.w[3]);
      if constexpr (MD) {
        if (h.nsub && status != ST_ERROR) md_publish();
      }
      break;
    case MK_CANCEL:
      cancel_order(m);
      if constexpr (MD) {
        if (h.nsub && status != ST_ERROR) md_publish();
      }
      break;
    case MK_MD_SUB_REQ:
    case MK_MD_SUB_CANCEL:
      if constexpr (MD) md_subscribe(m);
      break;
    default:
      break;
    }
  }

  // ---------------- TradingAgent (TradingAgent.py)
  DEV void send_ex(Msg m) {
    m.w[0] = (m.w[0] & 0xFFFFu) | ((u32)cur_agent << 16);
    if constexpr (BLOG && PC.ex_log_orders) {  // an order created now: its time_placed (LimitOrder(...))
      const u32 k = m_kind(m);
      if (h.exlog && (k == MK_LIMIT || k == MK_MODIFY)) bl_put(cur, BL_EV_PLACE, (i32)m.w[1]);
    }
    send(0, m, 0);
  }
  DEV void get_spread(int depth) {
    Msg m = msg_make(MK_SPREAD_REQ, cur_agent);
    m.w[1] = (u32)depth;
    send_ex(m);
  }
  DEV void get_tv(i64 lookback) {
    Msg m = msg_make(MK_TV_REQ, cur_agent);
    m.w[1] = (u32)(u64)lookback;
    m.w[2] = (u32)((u64)lookback >> 32);
    send_ex(m);
  }
  // placeLimitOrder (TradingAgent.py:309-349)
  DEV void place_limit(i64 qty, int is_buy, i64 price) {
    PROF_SCOPE(72);
    place_limit_oid(qty, is_buy, price, next_order_id());
  }
  // placeLimitOrder with the order's id: an auto id (LimitOrder() consumed it even for a zero
  // quantity) or the caller's order_id (SpreadBasedMarketMakerAgent)
  DEV void place_limit_oid(i64 qty, int is_buy, i64 price, i64 oid) {
    if (qty > 0) {
      i32 n = rgi(AF_NORD);
      if (n >= PC.L.open_cap) {
        fail(ERR_OPEN_FULL);
        return;
      }
      OpenOrder* oo = open_ptr(cur_agent);
      i32 u = rgi(AF_NUSED);
      if (u >= PC.L.open_cap) u = open_compact();
      if (lane == 0) {
        OpenOrder o;
        o.oid = (i32)oid;
        o.is_buy = is_buy;
        o.qty = (i32)qty;
        o.price = (i32)price;
        oo[u] = o;
      }
      rs(AF_NUSED, (u32)(u + 1));
      rs(AF_NORD, (u32)(n + 1));
      Msg lm = msg_order(MK_LIMIT, (i32)oid, cur_agent, is_buy, (i32)qty, (i32)price, 0);
      if constexpr (RP) lm.w[5] = (u32)agent_dense(oid);
      send_ex(lm);
    }
  }
  // cancelOrder for every open order in dict (= ascending order id) order
  // TradingAgent.orders (dict, insertion order) as an append-only list in HBM: deletions leave
  // a tombstone (oid -1), the list is compacted when its slots run out
  static constexpr int OC = (PC.L.open_cap + 63) / 64;
  // zero latency, no noise draw, no replay dense ids: a message to the exchange is delivered at
  // currentTime + computation delay, so a run of sends can be pushed as one batch
  static constexpr bool BATCH = !RP && PC.lat_mode == 0 && PC.noise_len <= 1;
  DEV u64 ex_key() { return ((u64)(cur + rg64(AF_COMP) + add_delay) << KSH) | MT_MESSAGE; }
  // cancelOrder for every open order in dict (= list) order
  DEV void cancel_all() {
    PROF_SCOPE(71);
    if constexpr (BATCH) {
      const i32 u = rgi(AF_NUSED);
      const OpenOrder* oo = open_ptr(cur_agent);
      const u64 key = ex_key();
      for (int j = 0; j < OC; j++) {
        if (j * 64 >= u) break;
        OpenOrder o;
        o.oid = -1;
        o.is_buy = o.qty = o.price = 0;
        if (j * 64 + lane < u) o = oo[j * 64 + lane];
        Msg cm = msg_order(MK_CANCEL, o.oid, cur_agent, o.is_buy, o.qty, o.price, 0);
        q_push_lanes(o.oid != -1, key, cm);
      }
      return;
    }
    const i32 u = rgi(AF_NUSED);
    OpenOrder* oo = open_ptr(cur_agent);
    OpenOrder my[OC];
    for (int j = 0; j < OC; j++) {
      my[j].oid = -1;
      if (j * 64 + lane < u) my[j] = oo[j * 64 + lane];
    }
    for (int j = 0; j < OC; j++) {
      u64 b = bal(my[j].oid != -1);
      while (b) {
        int L = ctz64(b);
        b &= b - 1;
        i32 oid = rdli(my[j].oid, L), ib = rdli(my[j].is_buy, L), q = rdli(my[j].qty, L), p = rdli(my[j].price, L);
        Msg cm = msg_order(MK_CANCEL, oid, cur_agent, ib, q, p, 0);
        if constexpr (RP) cm.w[5] = (u32)agent_dense(oid);
        send_ex(cm);
      }
    }
  }
  DEV int find_open(i32 oid, OpenOrder& out) {
    const i32 u = rgi(AF_NUSED);
    OpenOrder* oo = open_ptr(cur_agent);
    OpenOrder my[OC];
    for (int j = 0; j < OC; j++) {  // all chunks in flight at once
      my[j].oid = -1;
      if (j * 64 + lane < u) my[j] = oo[j * 64 + lane];
    }
    for (int j = 0; j < OC; j++) {
      u64 hit = bal(my[j].oid == oid);
      if (hit) {
        int L = ctz64(hit);
        out.oid = oid;
        out.is_buy = rdli(my[j].is_buy, L);
        out.qty = rdli(my[j].qty, L);
        out.price = rdli(my[j].price, L);
        return j * 64 + L;
      }
    }
    return -1;
  }
  DEV void del_open(int idx) {
    OpenOrder* oo = open_ptr(cur_agent);
    if (lane == 0) oo[idx].oid = -1;
    i32 n = rgi(AF_NORD) - 1;
    rs(AF_NORD, (u32)n);
    if (n == 0) rs(AF_NUSED, 0u);
  }
  DEV i32 open_compact() {  // keep live entries in order; returns the new used count
    OpenOrder* oo = open_ptr(cur_agent);
    const i32 u = rgi(AF_NUSED);
    OpenOrder my[OC];
    for (int j = 0; j < OC; j++) {
      my[j].oid = -1;
      if (j * 64 + lane < u) my[j] = oo[j * 64 + lane];
    }
    __threadfence_block();
    i32 base = 0;
    for (int j = 0; j < OC; j++) {
      bool live = my[j].oid != -1;
      u64 b = bal(live);
      i32 r = base + (i32)__builtin_amdgcn_mbcnt_hi((u32)(b >> 32), __builtin_amdgcn_mbcnt_lo((u32)b, 0u));
      if (live) oo[r] = my[j];
      base += __popcll(b);
    }
    __threadfence_block();
    rs(AF_NUSED, (u32)base);
    return base;
  }

  // TradingAgent.wakeup (TradingAgent.py:142-158)
  DEV bool ta_wakeup() {
    PROF_SCOPE(75);
    u32 f = flags();
    if (f & FL_FIRST_WAKE) rs(AF_FLAGS, f & ~FL_FIRST_WAKE);
    if (!(f & FL_HAS_OPEN)) {
      send_ex(msg_make(MK_WHEN_OPEN_REQ, cur_agent));
      send_ex(msg_make(MK_WHEN_CLOSE_REQ, cur_agent));
    }
    f = flags();
    return (f & FL_HAS_OPEN) && (f & FL_HAS_CLOSE) && !(f & FL_MKT_CLOSED);
  }
  DEV i64 wake_frequency(int type) {
    if (type == AG_POVMM) return mm_wake();
    if (type == AG_MOMENTUM) return PC.mom_wake;
    if (type == AG_MKTMAKER) return PC.mk_wake;  // pd.Timedelta(wake_up_freq) (MarketMakerAgent.py:148-149)
    if (type == AG_OBI) return PC.obi_wake;      // pd.Timedelta("1s") (OrderBookImbalanceAgent.py:187-188)
    if (type == AG_SBMM) return PC.sb_wake;      // pd.Timedelta(wake_up_freq) (SpreadBasedMarketMakerAgent.py:290-292)
    if constexpr (RP) {
      if (type == AG_REPLAY) return U(rx->tm[0]) - PC.mkt_open;  // MarketReplayAgent.py:94-96
      if constexpr (TW) {
        if (type == AG_TWAP) return PC.rl_h0 - PC.mkt_open;  // ExecutionAgent.getWakeFrequency
      }
    }
    if constexpr (GYM) {
      if (type == AG_DUMMYRL) return PC.rl_h0 - PC.mkt_open;     // execution_agent.py:129-130
    }
    RS A = agent_rs();
    i64 v = rs_randint(A, 0, 100);
    agent_rs_put(A);
    return v;
  }
  DEV void query_last_trade(const Msg& m) {
    u32 f = flags() | FL_HAS_LAST;
    f = m_dfloat(m) ? (f | FL_LAST_FLOAT) : (f & ~FL_LAST_FLOAT);
    if (f & FL_MKT_CLOSED) f |= FL_DAILY_CLOSE;
    rs(AF_FLAGS, f);
    rs64(AF_LAST_TRADE, (i64)(i32)m.w[5]);
  }
  // TradingAgent.receiveMessage (TradingAgent.py:181-268)
  DEV void ta_receive(const Msg& m, int type) {
    PROF_SCOPE(74);
    u32 f0 = flags();
    bool had = (f0 & FL_HAS_OPEN) && (f0 & FL_HAS_CLOSE);
    switch (m_kind(m)) {
    case MK_WHEN_OPEN:
      rs64(AF_MKT_OPEN, m_i64(m, 1));
      fl_set(FL_HAS_OPEN, true);
      break;
    case MK_WHEN_CLOSE:
      rs64(AF_MKT_CLOSE, m_i64(m, 1));
      fl_set(FL_HAS_CLOSE, true);
      break;
    case MK_EXECUTED: {  // orderExecuted (TradingAgent.py:422-462)
      i64 q = m_buy(m) ? (i64)(i32)m.w[2] : -(i64)(i32)m.w[2];
      rs64(AF_SHARES, rg64(AF_SHARES) + q);
      rs64(AF_CASH, rg64(AF_CASH) - q * (i64)(i32)m.w[4]);
      if constexpr (RP) {
        if (type == AG_REPLAY) {  // MarketReplayAgent.orders: dense-indexed table
          RPCHK((i32)m.w[5] >= 0 && (i32)m.w[5] < U(rx->L.D), "ta_receive EXECUTED dense", (i32)m.w[5]);
          RpOrder* o = mro() + (i32)m.w[5];
          const RpOrder ov = *o;  // one 16-byte load: present and qty in the same round trip
          if (U(ov.present)) {  // all lanes store the same value
            if ((i32)m.w[2] >= U(ov.qty)) o->present = 0;
            else o->qty = U(ov.qty) - (i32)m.w[2];
          }
          break;
        }
      }
      OpenOrder o;
      int idx = find_open((i32)m.w[1], o);
      if (idx >= 0) {
        if ((i32)m.w[2] >= o.qty) del_open(idx);
        else if (lane == 0) open_ptr(cur_agent)[idx].qty = o.qty - (i32)m.w[2];
      }
      break;
    }
    case MK_CANCELLED: {
      if constexpr (RP) {
        if (type == AG_REPLAY) {
          RPCHK((i32)m.w[5] >= 0 && (i32)m.w[5] < U(rx->L.D), "ta_receive CANCELLED dense", (i32)m.w[5]);
          mro()[(i32)m.w[5]].present = 0;
          break;
        }
      }
      OpenOrder o;
      int idx = find_open((i32)m.w[1], o);
      if (idx >= 0) del_open(idx);
      break;
    }
    case MK_MKT_CLOSED:
      fl_set(FL_MKT_CLOSED, true);
      break;
    case MK_LAST:
      if (m_closed(m)) fl_set(FL_MKT_CLOSED, true);
      query_last_trade(m);
      break;
    case MK_SPREAD: {
      if (m_closed(m)) fl_set(FL_MKT_CLOSED, true);
      query_last_trade(m);
      u32 f = flags() | FL_HAS_KNOWN;
      f = m_nb(m) ? (f | FL_NB) : (f & ~FL_NB);
      f = m_na(m) ? (f | FL_NA) : (f & ~FL_NA);
      rs(AF_FLAGS, f);
      rs(AF_BID, m.w[1]);
      rs(AF_BIDQ, m.w[2]);
      rs(AF_ASK, m.w[3]);
      rs(AF_ASKQ, m.w[4]);
      break;
    }
    case MK_TV:
      if (m_closed(m)) fl_set(FL_MKT_CLOSED, true);
      rs64(AF_TV, m_i64(m, 1));
      break;
    case MK_MARKET_DATA:  // handleMarketData (TradingAgent.py:539-546): known levels, last trade
      if constexpr (MD) {
        u32 f = flags() | FL_HAS_KNOWN | FL_HAS_LAST;
        f = (m.w[6] & 0xFF) ? (f | FL_NB) : (f & ~FL_NB);
        f = (m.w[6] & 0xFF00) ? (f | FL_NA) : (f & ~FL_NA);
        f = m_dfloat(m) ? (f | FL_LAST_FLOAT) : (f & ~FL_LAST_FLOAT);
        rs(AF_FLAGS, f);
        rs(AF_BID, m.w[1]);
        rs(AF_BIDQ, m.w[2]);
        rs(AF_ASK, m.w[3]);
        rs(AF_ASKQ, m.w[4]);
        rs64(AF_LAST_TRADE, (i64)(i32)m.w[5]);
      }
      break;
    case MK_STREAM:  // queryOrderStream (TradingAgent.py:240-246, 549-554)
      if constexpr (OH) {
        if (m_closed(m)) fl_set(FL_MKT_CLOSED, true);
        fl_set(FL_HAS_STREAM, true);
        rs(AF_STREAM_N, m.w[1]);
        rs64(AF_STREAM_HI, m_i64(m, 2));
      }
      break;
    default:
      break;
    }
    u32 f1 = flags();
    bool have = (f1 & FL_HAS_OPEN) && (f1 & FL_HAS_CLOSE);
    if (have && !had) {
      i64 off = wake_frequency(type);
      wakeup_at(cur_agent, rg64(AF_MKT_OPEN) + off);
    }
  }
  DEV bool known_bid(i32& bid) {
    bid = rgi(AF_BID);
    return fl(FL_NB) && bid != 0;
  }
  DEV bool known_ask(i32& ask) {
    ask = rgi(AF_ASK);
    return fl(FL_NA) && ask != 0;
  }

  // Bayesian estimate shared by ZI (ZI.py:215-263) and Value (ValueAgent.py:153-201)
  DEV i64 bayes_r_T(i64 obs, double kappa, double r_bar, double sigma_n, double sigma_s) {
    PROF_SCOPE(70);
    if (!fl(FL_PREV_WAKE)) {
      fl_set(FL_PREV_WAKE, true);
      rs64(AF_PREV_WAKE, rg64(AF_MKT_OPEN));
    }
    double delta = (double)(cur - rg64(AF_PREV_WAKE));
    double c = 1 - kappa;
    double d2 = (double)(rg64(AF_MKT_CLOSE) - cur);
    if (!(d2 > 0)) d2 = 0;
    // the four powers of c are independent: lanes 0-3 of ONE gm_pow evaluation
    const double pw = gm_pow(c, lane == 0 ? delta : lane == 1 ? 2 * delta : lane == 2 ? 2.0 : d2);
    const double p_d = rdl_d(pw, 0), p_2d = rdl_d(pw, 1), p_2 = rdl_d(pw, 2), p_d2 = rdl_d(pw, 3);
    double r_t = rgd(AF_R_T), sigma_t = rgd(AF_SIGMA_T);
    double r_tprime = (1 - p_d) * r_bar;
    r_tprime += p_d * r_t;
    double sigma_tprime = p_2d * sigma_t;
    sigma_tprime += ((1 - p_2d) / (1 - p_2)) * sigma_s;
    r_t = (sigma_n / (sigma_n + sigma_tprime)) * r_tprime;
    r_t += (sigma_tprime / (sigma_n + sigma_tprime)) * (double)obs;
    sigma_t = (sigma_n * sigma_t) / (sigma_n + sigma_t);
    double r_T = (1 - p_d2) * r_bar;
    r_T += p_d2 * r_t;
    rsd(AF_R_T, r_t);
    rsd(AF_SIGMA_T, sigma_t);
    rs64(AF_PREV_WAKE, cur);
    return py_round(r_T);
  }

  // ---------------- ZeroIntelligenceAgent (ZI.py:125-309)
  // ZeroIntelligenceAgent.wakeup; a subclass (HBL) does not query the spread but becomes ACTIVE
  // (ZI.py:183-187)
  DEV void zi_wakeup_as(bool is_zi) {
    ta_wakeup();
    rs(AF_STATE, AS_INACTIVE);
    if (!fl(FL_HAS_OPEN) || !fl(FL_HAS_CLOSE)) return;
    fl_set(FL_TRADING, true);
    if (fl(FL_MKT_CLOSED) && fl(FL_DAILY_CLOSE)) return;
    RS A = agent_rs();
    double dt = rs_exponential(A, 1.0 / PC.zi_lambda);
    agent_rs_put(A);
    wakeup_at(cur_agent, cur + py_round(dt));
    if (fl(FL_MKT_CLOSED) && !fl(FL_DAILY_CLOSE)) {
      get_spread(1);
      rs(AF_STATE, AS_AWAITING_SPREAD);
      return;
    }
    cancel_all();
    if (is_zi) {
      get_spread(1);
      rs(AF_STATE, AS_AWAITING_SPREAD);
    } else {
      rs(AF_STATE, AS_ACTIVE);
    }
  }
  DEV void zi_wakeup() { zi_wakeup_as(true); }
  // updateEstimates (ZI.py:189-275): the total unit valuation v and the side; false where the
  // reference raises (theta IndexError)
  DEV bool zi_update_estimates(i64& v, int& buy) {
    i64 obs = o_observe(cur, PC.zi_sigma_n);
    i64 q = (i64)((double)rg64(AF_SHARES) / 100);
    if (q >= PC.zi_qmax) buy = 0;
    else if (q <= -PC.zi_qmax) buy = 1;
    else {
      RS A = agent_rs();
      buy = (int)rs_randint(A, 0, 2);
      agent_rs_put(A);
    }
    i64 r_T = bayes_r_T(obs, PC.zi_kappa, PC.zi_rbar, PC.zi_sigma_n, PC.zi_sigma_s);
    q += PC.zi_qmax - 1;
    i64 idx = buy ? q + 1 : q;
    if (idx < 0) idx += 2 * PC.zi_qmax;
    if (idx < 0 || idx >= 2 * PC.zi_qmax) {
      fail(ERR_THETA_INDEX);
      return false;
    }
    v = r_T + (i64)rgi(AF_THETA + (int)idx);
    return true;
  }
  DEV void zi_place() {
    i64 v;
    int buy;
    if (!zi_update_estimates(v, buy)) return;
    int g = rgi(AF_GROUP);
    RS A = agent_rs();
    i64 R = rs_randint(A, PC.zi_rmin[g], (i64)PC.zi_rmax[g] + 1);
    agent_rs_put(A);
    i64 p = buy ? v - R : v + R;
    i32 bid = 0, ask = 0;
    i64 bid_vol = fl(FL_NB) ? (i64)rgi(AF_BIDQ) : 0, ask_vol = fl(FL_NA) ? (i64)rgi(AF_ASKQ) : 0;
    bid = rgi(AF_BID);
    ask = rgi(AF_ASK);
    if (buy && ask_vol > 0) {
      i64 R_ask = v - ask;
      if ((double)R_ask >= PC.zi_eta[g] * (double)R) p = ask;
    } else if (!buy && bid_vol > 0) {
      i64 R_bid = bid - v;
      if ((double)R_bid >= PC.zi_eta[g] * (double)R) p = bid;
    }
    place_limit(100, buy, p);
  }
  DEV void zi_receive(const Msg& m) {
    ta_receive(m, AG_ZI);
    if (rgi(AF_STATE) == AS_AWAITING_SPREAD && m_kind(m) == MK_SPREAD) {
      if (fl(FL_MKT_CLOSED)) return;
      zi_place();
      rs(AF_STATE, AS_AWAITING_WAKEUP);
    }
  }

  // ---------------- ValueAgent (ValueAgent.py:100-268)
  DEV void value_wakeup() {
    ta_wakeup();
    rs(AF_STATE, AS_INACTIVE);
    if (!fl(FL_HAS_OPEN) || !fl(FL_HAS_CLOSE)) return;
    fl_set(FL_TRADING, true);
    if (fl(FL_MKT_CLOSED) && fl(FL_DAILY_CLOSE)) return;
    RS A = agent_rs();
    double dt = rs_exponential(A, 1.0 / PC.v_lambda);
    agent_rs_put(A);
    wakeup_at(cur_agent, cur + py_round(dt));
    if (fl(FL_MKT_CLOSED) && !fl(FL_DAILY_CLOSE)) {
      get_spread(1);
      rs(AF_STATE, AS_AWAITING_SPREAD);
      return;
    }
    cancel_all();
    get_spread(1);
    rs(AF_STATE, AS_AWAITING_SPREAD);
  }
  DEV void value_place() {
    i64 obs = o_observe(cur, v_sigma_n());
    i64 r_T = bayes_r_T(obs, PC.v_kappa, v_rbar(), v_sigma_n(), PC.v_sigma_s);
    i32 bid, ask;
    bool hb = known_bid(bid), ha = known_ask(ask);
    int buy;
    i64 p;
    RS G = grs(0);
    if (hb && ha) {
      i64 mid = (i64)((double)((i64)ask + bid) / 2);
      i64 spread = (i64)ask - bid;
      if (spread < 0) spread = -spread;
      i64 adj;
      if (rs_double(G) < PC.v_percent_aggr) adj = 0;
      else adj = rs_randint(G, 0, PC.v_depth_spread * spread);
      if (r_T < mid) {
        buy = 0;
        p = bid + adj;
      } else {
        buy = 1;
        p = ask - adj;
      }
    } else {
      buy = (int)rs_randint(G, 0, 2);
      p = r_T;
    }
    grs_put(0, G);
    place_limit(rgi(AF_SIZE), buy, p);
  }
  DEV void value_receive(const Msg& m) {
    ta_receive(m, AG_VALUE);
    if (rgi(AF_STATE) == AS_AWAITING_SPREAD && m_kind(m) == MK_SPREAD) {
      if (fl(FL_MKT_CLOSED)) return;
      value_place();
      rs(AF_STATE, AS_AWAITING_WAKEUP);
    }
  }

  // ---------------- NoiseAgent (NoiseAgent.py:82-154)
  DEV void noise_wakeup() {
    ta_wakeup();
    rs(AF_STATE, AS_INACTIVE);
    if (!fl(FL_HAS_OPEN) || !fl(FL_HAS_CLOSE)) return;
    fl_set(FL_TRADING, true);
    if (fl(FL_MKT_CLOSED) && fl(FL_DAILY_CLOSE)) return;
    i64 wt = rg64(AF_WAKEUP_TIME);
    if (wt > cur) wakeup_at(cur_agent, wt);
    get_spread(1);
    rs(AF_STATE, AS_AWAITING_SPREAD);
  }
  DEV void noise_receive(const Msg& m) {
    ta_receive(m, AG_NOISE);
    if (rgi(AF_STATE) == AS_AWAITING_SPREAD && m_kind(m) == MK_SPREAD) {
      if (fl(FL_MKT_CLOSED)) return;
      RS G = grs(0);
      int buy = (int)rs_randint(G, 0, 2);
      grs_put(0, G);
      i32 bid, ask;
      bool hb = known_bid(bid), ha = known_ask(ask);
      if (buy && ha) place_limit(rgi(AF_SIZE), 1, ask);
      else if (!buy && hb) place_limit(rgi(AF_SIZE), 0, bid);
      rs(AF_STATE, AS_AWAITING_WAKEUP);
    }
  }

  // ---------------- POVMarketMakerAgent (POVMarketMakerAgent.py:83-206)
  // its options: the config script's constants, or (MXA_CFG_RMSC03_MM) this env's, from its record
  DEV double mm_pov() { if constexpr (PC.mm_rt) return rgd(AF_MM_POV); else return PC.mm_pov; }
  DEV i64 mm_min() { if constexpr (PC.mm_rt) return rgi(AF_MM_MIN); else return PC.mm_min_size; }
  DEV i64 mm_window() { if constexpr (PC.mm_rt) return rgi(AF_MM_WIN); else return PC.mm_window; }
  DEV i64 mm_ticks() { if constexpr (PC.mm_rt) return rgi(AF_MM_TICKS); else return PC.mm_ticks; }
  DEV i64 mm_wake() { if constexpr (PC.mm_rt) return rg64(AF_MM_WAKE); else return PC.mm_wake; }
  DEV void mm_wakeup() {
    if (ta_wakeup()) {
      get_spread(1);
      get_tv(mm_wake());  // lookback_period = wake_up_freq
    }
  }
  DEV void mm_receive(const Msg& m) {
    ta_receive(m, AG_POVMM);
    i64 mid = rg64(AF_LAST_MID);
    u32 k = m_kind(m);
    if (k == MK_TV && fl(FL_AW_TV)) {
      i64 qty = py_round(mm_pov() * (double)rg64(AF_TV));
      const i64 mn = mm_min();
      if (qty > INT32_MAX) {  // the order words are 32-bit: stop loudly, never wrap
        fail(ERR_ORDER_SIZE);
        return;
      }
      rs(AF_ORDER_SIZE, (u32)(qty >= mn ? qty : mn));
      fl_set(FL_AW_TV, false);
    }
    if (k == MK_SPREAD && fl(FL_AW_SPREAD)) {
      i32 bid, ask;
      bool hb = known_bid(bid), ha = known_ask(ask);
      if (hb && ha) {
        mid = (i64)((double)((i64)ask + bid) / 2);
        rs64(AF_LAST_MID, mid);
        fl_set(FL_LAST_MID, true);
        fl_set(FL_AW_SPREAD, false);
      }
    }
    if (!fl(FL_AW_SPREAD) && !fl(FL_AW_TV)) {
      cancel_all();
      const i64 ticks = mm_ticks();
      i64 hb = mid - 1, la = mid + mm_window();
      i64 lb = hb - ticks, ha = la + ticks;
      i64 sz = rgi(AF_ORDER_SIZE);
      const int NL = 2 * (int)(ticks + 1);
      if (BATCH && NL <= MM_LADDER_MAX && sz > 0 && rgi(AF_NORD) + NL <= PC.L.open_cap) {
        mm_place_ladder(sz, lb, la, (int)ticks + 1);
      } else {
        for (i64 p = lb; p <= hb; p++) place_limit(sz, 1, p);
        for (i64 p = la; p <= ha; p++) place_limit(sz, 0, p);
      }
      fl_set(FL_AW_SPREAD, true);
      fl_set(FL_AW_TV, true);
      wakeup_at(cur_agent, cur + mm_wake());
    }
  }

  // the ladder's placeLimitOrder calls in batched passes of 64: member i places bid lb+i (i < NB)
  // or ask la+i-NB; ids, open-order list entries and queue seqs in the same order as the loop.
  // Each pass is one batched push (one exchange-side LIMIT run); two passes cover 63 ticks
  static constexpr int MM_LADDER_MAX = PC.mm_rt ? 128 : 64;
  DEV void mm_place_ladder(i64 sz, i64 lb, i64 la, int NB) {
    if constexpr (!PC.mm_rt) {  // the script's constant ladder: one pass (the measured rmsc03 code)
      constexpr int CNB = PC.mm_ticks + 1, CNL = 2 * CNB;
      i32 u = rgi(AF_NUSED);
      if (u + CNL > PC.L.open_cap) u = open_compact();
      const bool act = lane < CNL;
      const int buy = lane < CNB;
      const i32 price = (i32)(buy ? lb + lane : la + (lane - CNB));
      const i32 oid = (i32)(ocnt + lane);
      ocnt += CNL;
      if (act) {
        OpenOrder o;
        o.oid = oid;
        o.is_buy = buy;
        o.qty = (i32)sz;
        o.price = price;
        open_ptr(cur_agent)[u + lane] = o;
      }
      rs(AF_NUSED, (u32)(u + CNL));
      rs(AF_NORD, (u32)(rgi(AF_NORD) + CNL));
      Msg lm = msg_order(MK_LIMIT, oid, cur_agent, buy, (i32)sz, price, 0);
      lm.w[0] = (lm.w[0] & 0xFFFFu) | ((u32)cur_agent << 16);
      q_push_lanes(act, ex_key(), lm);
      return;
    }
    const int NL = 2 * NB;
    i32 u = rgi(AF_NUSED);
    if (u + NL > PC.L.open_cap) u = open_compact();
    const i64 o0 = ocnt;
    ocnt += NL;
    rs(AF_NUSED, (u32)(u + NL));
    rs(AF_NORD, (u32)(rgi(AF_NORD) + NL));
    const u64 key = ex_key();
    for (int c = 0; c < MM_LADDER_MAX / 64; c++) {
      if (c * 64 >= NL) break;
      const int i = c * 64 + lane;
      const bool act = i < NL;
      const int buy = i < NB;
      const i32 price = (i32)(buy ? lb + i : la + (i - NB));
      const i32 oid = (i32)(o0 + i);
      if (act) {
        OpenOrder o;
        o.oid = oid;
        o.is_buy = buy;
        o.qty = (i32)sz;
        o.price = price;
        open_ptr(cur_agent)[u + i] = o;
      }
      Msg lm = msg_order(MK_LIMIT, oid, cur_agent, buy, (i32)sz, price, 0);
      lm.w[0] = (lm.w[0] & 0xFFFFu) | ((u32)cur_agent << 16);
      q_push_lanes(act, key, lm);
    }
  }

  // ---------------- SpreadBasedMarketMakerAgent (agent/market_makers/SpreadBasedMarketMakerAgent.py)
  // The Chakraborty-Kearns ladder: num_ticks + 1 one-cent levels per side around the mid, shifted
  // by whole ticks as the mid moves.  current_bids / current_asks are rings of order ids in the
  // record (AF_SB_IDS: bids, then asks) with one head and one length; their prices run from
  // AF_SB_BLO / AF_SB_ALO up by one cent per entry
  static constexpr int SBC = PC.n_sb > 0 ? PC.sb_ticks + 1 : 1;
  static_assert(PC.n_sb == 0 || AF_SB_IDS + 2 * SBC <= AF_RS_M, "SpreadBased ladder ids inside the agent record");
  static DEV int sb_wrap(int r) { return r >= SBC ? r - SBC : r; }
  // cancelOrders (:166-179): self.orders[id] -> cancelOrder; an id no longer open (KeyError) is skipped
  DEV void cancel_oid(i32 oid) {
    OpenOrder o;
    if (find_open(oid, o) < 0) return;
    send_ex(msg_order(MK_CANCEL, oid, cur_agent, o.is_buy, o.qty, o.price, 0));
  }
  // computeOrdersToCancel + cancelOrders + computeOrdersToPlace + placeOrders (:111-113, :128-130)
  // at `mid`; AF_LAST_MID still holds the previous mid
  DEV void sb_update(i64 mid) {
    i32 n = rgi(AF_SB_N);
    if (fl(FL_SB_INIT)) {  // computeOrdersToCancel (:134-164)
      const i64 k = mid - rg64(AF_LAST_MID);
      const i64 ak = k > 0 ? k : -k;
      for (i64 i = 0; i < ak && n > 0; i++) {  // popleft on a rise, pop on a fall; empty deques ignored
        const i32 hd = rgi(AF_SB_HEAD);
        const int r = k > 0 ? hd : sb_wrap(hd + n - 1);
        const i32 bo = rgi(AF_SB_IDS + r), ao = rgi(AF_SB_IDS + SBC + r);
        if (k > 0) {
          rs(AF_SB_HEAD, (u32)sb_wrap(hd + 1));
          rs(AF_SB_BLO, (u32)(rgi(AF_SB_BLO) + 1));
          rs(AF_SB_ALO, (u32)(rgi(AF_SB_ALO) + 1));
        }
        n--;
        rs(AF_SB_N, (u32)n);
        cancel_oid(bo);  // the list order: bid, ask, bid, ask, ...
        cancel_oid(ao);
      }
    }
    if (!fl(FL_SB_INIT) || n == 0) {  // `not self.current_asks or not self.current_bids`
      cancel_all();                    // cancelAllOrders (:294-297)
      // initialiseBidsAsksDeques (:257-277), anchor "bottom": ids for the bids, then the asks
      const i64 lb = mid - 1 - PC.sb_ticks, la = mid + PC.sb_window;
      const i32 c0 = rgi(AF_SB_CNT);
      for (int i = 0; i < SBC; i++) {
        rs(AF_SB_IDS + i, (u32)(MXA_SB_ID_BASE + c0 + 1 + i));
        rs(AF_SB_IDS + SBC + i, (u32)(MXA_SB_ID_BASE + c0 + 1 + SBC + i));
      }
      rs(AF_SB_CNT, (u32)(c0 + 2 * SBC));
      rs(AF_SB_HEAD, 0u);
      rs(AF_SB_N, (u32)SBC);
      rs(AF_SB_BLO, (u32)lb);
      rs(AF_SB_ALO, (u32)la);
      fl_set(FL_SB_INIT, true);
      for (int i = 0; i < SBC; i++) place_limit_oid(PC.sb_size, 1, lb + i, MXA_SB_ID_BASE + c0 + 1 + i);
      for (int i = 0; i < SBC; i++) place_limit_oid(PC.sb_size, 0, la + i, MXA_SB_ID_BASE + c0 + 1 + SBC + i);
      return;
    }
    const i64 k = fl(FL_LAST_MID) ? mid - rg64(AF_LAST_MID) : 0;
    if (k == 0) return;
    // new levels beyond the moving end, one id each, bid before ask (generateNewOrderId order);
    // |k| < the deque length here (a longer move emptied the deques above)
    const i32 c0 = rgi(AF_SB_CNT);
    const i64 ak = k > 0 ? k : -k;
    const i64 b0 = k > 0 ? rgi(AF_SB_BLO) + n - 1 : rgi(AF_SB_BLO);
    const i64 a0 = k > 0 ? rgi(AF_SB_ALO) + n - 1 : rgi(AF_SB_ALO);
    for (i64 inc = 1; inc <= ak; inc++) {
      const i32 bo = MXA_SB_ID_BASE + c0 + (i32)(2 * inc - 1), ao = bo + 1;
      i32 hd = rgi(AF_SB_HEAD);
      int r;
      if (k > 0) {  // append
        r = sb_wrap(hd + n);
      } else {      // appendleft
        hd = sb_wrap(hd + SBC - 1);
        r = hd;
        rs(AF_SB_HEAD, (u32)hd);
        rs(AF_SB_BLO, (u32)(rgi(AF_SB_BLO) - 1));
        rs(AF_SB_ALO, (u32)(rgi(AF_SB_ALO) - 1));
      }
      rs(AF_SB_IDS + r, (u32)bo);
      rs(AF_SB_IDS + SBC + r, (u32)ao);
      n++;
    }
    rs(AF_SB_N, (u32)n);
    rs(AF_SB_CNT, (u32)(c0 + 2 * ak));
    const i64 dir = k > 0 ? 1 : -1;
    for (i64 inc = 1; inc <= ak; inc++) place_limit_oid(PC.sb_size, 1, b0 + dir * inc, MXA_SB_ID_BASE + c0 + 2 * inc - 1);
    for (i64 inc = 1; inc <= ak; inc++) place_limit_oid(PC.sb_size, 0, a0 + dir * inc, MXA_SB_ID_BASE + c0 + 2 * inc);
  }
  DEV void sb_wakeup() {  // wakeup (:75-84)
    const bool can = ta_wakeup();
    if constexpr (PC.sb_sub) {
      if (!fl(FL_SUB_REQ)) request_subscription(1);  // level 1 every subscribe_freq (10e9 ns)
      return;
    }
    if (can) {
      get_spread(1);
      rs(AF_STATE, AS_AWAITING_SPREAD);
    }
  }
  DEV void sb_receive(const Msg& m) {  // receiveMessage (:86-132)
    ta_receive(m, AG_SBMM);
    const u32 k = m_kind(m);
    i32 bid, ask;
    if constexpr (!PC.sb_sub) {
      if (!(rgi(AF_STATE) == AS_AWAITING_SPREAD && k == MK_SPREAD)) return;
      const bool hb = known_bid(bid), ha = known_ask(ask);  // getKnownBidAsk; `if bid and ask`
      i64 mid = rg64(AF_LAST_MID);
      if (hb && ha) mid = (i64)((double)((i64)ask + bid) / 2);
      else if (!fl(FL_LAST_MID)) {  // `mid` never bound
        fail(ERR_SB_MID);
        return;
      }
      sb_update(mid);
      wakeup_at(cur_agent, cur + PC.sb_wake);
      rs(AF_STATE, AS_AWAITING_WAKEUP);
      rs64(AF_LAST_MID, mid);
      fl_set(FL_LAST_MID, true);
    } else {
      if (!(rgi(AF_STATE) == AS_AWAITING_MD && k == MK_MARKET_DATA)) return;
      const bool hb = known_bid(bid), ha = known_ask(ask);  // known_bids[symbol][0][0] if known_bids[symbol] else None
      if (!(hb && ha)) return;
      const i64 mid = (i64)((double)((i64)ask + bid) / 2);
      sb_update(mid);
      rs64(AF_LAST_MID, mid);
      fl_set(FL_LAST_MID, true);
    }
  }

  // ---------------- MarketMakerAgent (agent/market_makers/MarketMakerAgent.py, polling mode)
  // TradingAgent.requestDataSubscription (TradingAgent.py:160-172)
  DEV void request_subscription(i32 levels) {
    Msg m = msg_make(MK_MD_SUB_REQ, cur_agent);
    m.w[1] = (u32)levels;
    m.w[2] = (u32)(u64)PC.md_freq;
    m.w[3] = (u32)((u64)PC.md_freq >> 32);
    send_ex(m);
    fl_set(FL_SUB_REQ, true);
    rs(AF_STATE, AS_AWAITING_MD);
  }
  DEV void mk_wakeup() {
    const bool can = ta_wakeup();  // MarketMakerAgent.py:69-79
    if constexpr (MD) {            // subscribe=True: one request, later wakeups do nothing
      if (!fl(FL_SUB_REQ)) request_subscription(PC.md_mk_levels);
      return;
    }
    if (can) {
      cancel_all();
      get_spread(PC.mk_depth);
      rs(AF_STATE, AS_AWAITING_SPREAD);
    }
  }
  // MarketMakerAgent.receiveMessage subscribe branch + placeOrders (MarketMakerAgent.py:109-141):
  // cancel every open order; num_levels = randint(1, 5) (1-4); with both sides known one size
  // draw, then per side a dict price -> round(split[i] * size) in first-insertion order, where a
  // missing level i quotes one cent beyond the last known level (repeated misses overwrite that
  // entry); bids placed first
  DEV void mk_market_data(const Msg& m) {
    cancel_all();
    RS A = agent_rs();
    const i32 nl = (i32)rs_randint(A, 1, 5);
    const i32 nb = (i32)(m.w[6] & 0xFF), na = (i32)((m.w[6] >> 8) & 0xFF);
    if (!(nb && na)) {
      agent_rs_put(A);
      return;
    }
    const i64 size = (i64)__builtin_rint((double)rs_randint(A, PC.mk_min, PC.mk_max) / 2);
    agent_rs_put(A);
    rs(AF_SIZE, (u32)size);
    const u32* slot = md_slot(cur_agent);
    if (U(slot[MD_TAG]) != m.w[7]) {
      fail(ERR_MD_SLOT);
      return;
    }
    for (int side = 1; side >= 0; side--) {
      const i32 n = side ? nb : na;
      const int base = side ? MD_BIDS : MD_ASKS;
      i32 px[MD_LEVELS], vol[MD_LEVELS];
      int k = 0;
      for (int i = 0; i < nl; i++) {
        const double split = nl == 1 ? 1.0 : nl == 2 ? 0.5 : nl == 3 ? (i == 0 ? 0.34 : 0.33) : 0.25;
        const i32 v = (i32)__builtin_rint(split * (double)size);
        const i32 p = i < n ? (i32)U(slot[base + i]) : (i32)U(slot[base + n - 1]) + (side ? -1 : 1);
        int j = 0;
        while (j < k && px[j] != p) j++;
        if (j == k) px[k++] = p;
        vol[j] = v;
      }
      for (int j = 0; j < k; j++) place_limit(vol[j], side, px[j]);
    }
  }
  DEV void mk_receive(const Msg& m) {
    ta_receive(m, AG_MKTMAKER);  // MarketMakerAgent.py:81-107
    if constexpr (MD) {
      if (rgi(AF_STATE) == AS_AWAITING_MD && m_kind(m) == MK_MARKET_DATA) mk_market_data(m);
      return;
    }
    if (!(rgi(AF_STATE) == AS_AWAITING_SPREAD && m_kind(m) == MK_SPREAD)) return;
    cancel_all();
    i64 mid = rg64(AF_LAST_TRADE), spread;
    i32 bid, ask;
    const bool hb = known_bid(bid), ha = known_ask(ask);  // getKnownBidAsk; `if bid and ask`
    if (hb && ha) {
      mid = (i64)((double)((i64)ask + bid) / 2);
      spread = (i64)((double)(ask > bid ? (i64)ask - bid : (i64)bid - ask) / 2);
    } else {
      // mid = last_trade: while it is the exchange's opening price (a python float) the ladder's
      // prices would travel as floats; not restated, so a loud error instead of a divergence
      if (fl(FL_LAST_FLOAT)) {
        fail(ERR_FLOAT_PRICE);
        return;
      }
      spread = PC.mk_last_spread;
    }
    mk_place_ladder(mid, spread);
    wakeup_at(cur_agent, cur + PC.mk_wake);
    rs(AF_STATE, AS_AWAITING_WAKEUP);
  }
  // for i < num_levels (2 x depth): size = round(A.randint(min, max) / 2); a bid at mid - spread - i
  // and an ask at mid + spread + i.  The sizes are drawn first (placeLimitOrder draws nothing), then
  // the 4 x depth orders are placed in one pass: lane 2i the bid, lane 2i + 1 the ask, ids, list
  // entries and queue seqs in the loop's order
  DEV void mk_place_ladder(i64 mid, i64 spread) {
    constexpr int NL = 4 * PC.mk_depth;
    RS A = agent_rs();
    i32 sz = 0;
    i64 last = 0;
    for (int i = 0; i < 2 * PC.mk_depth; i++) {
      last = (i64)__builtin_rint((double)rs_randint(A, PC.mk_min, PC.mk_max) / 2);
      sz = (lane >> 1) == i ? (i32)last : sz;
    }
    agent_rs_put(A);
    rs(AF_SIZE, (u32)last);
    if (BATCH && NL <= 64 && PC.mk_min >= 2 && rgi(AF_NORD) + NL <= PC.L.open_cap) {  // every size >= 1
      i32 u = rgi(AF_NUSED);
      if (u + NL > PC.L.open_cap) u = open_compact();
      const bool act = lane < NL;
      const int buy = !(lane & 1);
      const i64 lvl = lane >> 1;
      const i32 price = (i32)(buy ? mid - spread - lvl : mid + spread + lvl);
      const i32 oid = (i32)(ocnt + lane);
      ocnt += NL;
      if (act) {
        OpenOrder o;
        o.oid = oid;
        o.is_buy = buy;
        o.qty = sz;
        o.price = price;
        open_ptr(cur_agent)[u + lane] = o;
      }
      rs(AF_NUSED, (u32)(u + NL));
      rs(AF_NORD, (u32)(rgi(AF_NORD) + NL));
      Msg lm = msg_order(MK_LIMIT, oid, cur_agent, buy, sz, price, 0);
      q_push_lanes(act, ex_key(), lm);
    } else {
      for (int i = 0; i < 2 * PC.mk_depth; i++) {
        const i64 q = rdli(sz, 2 * i);
        place_limit(q, 1, mid - spread - i);
        place_limit(q, 0, mid + spread + i);
      }
    }
  }

  // ---------------- OrderBookImbalanceAgent (agent/OrderBookImbalanceAgent.py)
  // wakeup (:67-71): TradingAgent.wakeup, a (re)subscription to 10 levels every hour, then a
  // computation delay of 1 ns for every later event of the agent
  DEV void obi_wakeup() {
    ta_wakeup();
    Msg m = msg_make(MK_MD_SUB_REQ, cur_agent);
    m.w[1] = (u32)PC.obi_levels;
    m.w[2] = (u32)(u64)PC.obi_freq;
    m.w[3] = (u32)((u64)PC.obi_freq >> 32);
    send_ex(m);
    rs64(AF_COMP, 1);
  }
  // receiveMessage (:73-186): on MARKET_DATA cancel every open order; with liquidity on both sides
  // trade the bid share of the received levels against the entry threshold and the trailing stop;
  // computeRequiredPrice (:190-206) always ends on the deepest received level's price
  DEV void obi_receive(const Msg& m) {
    ta_receive(m, AG_OBI);
    if (m_kind(m) != MK_MARKET_DATA) return;
    cancel_all();
    const u32* slot = md_slot(cur_agent);
    const u32 x = lane < MD_WORDS ? slot[lane] : 0u;
    if (rdl(x, MD_TAG) != m.w[7]) {
      fail(ERR_MD_SLOT);
      return;
    }
    const i32 nb = (i32)(m.w[6] & 0xFF), na = (i32)((m.w[6] >> 8) & 0xFF);
    const i64 bl = wsum_i64(lane >= MD_BIDQ && lane < MD_BIDQ + nb ? (i64)x : 0);
    const i64 al = wsum_i64(lane >= MD_ASKQ && lane < MD_ASKQ + na ? (i64)x : 0);
    if (bl == 0 || al == 0) return;  // "zero bid or ask liquidity"
    const double bid_pct = (double)bl / (double)(bl + al);
    const double trail = PC.obi_trail;
    double stop = rgd(AF_OBI_STOP);
    i64 target;
    if (fl(FL_OBI_SHORT)) {
      if (bid_pct - trail > stop) stop = bid_pct - trail;
      if (bid_pct < stop) {
        target = 0;
        fl_set(FL_OBI_SHORT, false);
      } else {
        target = -100;
      }
    } else if (fl(FL_OBI_LONG)) {
      if (bid_pct + trail < stop) stop = bid_pct + trail;
      if (bid_pct > stop) {
        target = 0;
        fl_set(FL_OBI_LONG, false);
      } else {
        target = 100;
      }
    } else if (bid_pct < (0.5 - PC.obi_entry)) {
      target = 100;
      fl_set(FL_OBI_LONG, true);
      stop = bid_pct + trail;
    } else if (bid_pct > (0.5 + PC.obi_entry)) {
      target = -100;
      fl_set(FL_OBI_SHORT, true);
      stop = bid_pct - trail;
    } else {
      target = 0;
    }
    rsd(AF_OBI_STOP, stop);
    const i64 delta = target - rg64(AF_SHARES);
    const int dir = delta > 0;
    const i32 price = (i32)rdl(x, dir ? MD_ASKS + na - 1 : MD_BIDS + nb - 1);
    if (delta != 0) place_limit(delta > 0 ? delta : -delta, dir, price);
  }

  // ---------------- HeuristicBeliefLearningAgent (agent/HeuristicBeliefLearningAgent.py)
  DEV void hbl_wakeup() {
    zi_wakeup_as(false);  // HBL.py:61-73
    if (rgi(AF_STATE) != AS_ACTIVE) return;
    Msg m = msg_make(MK_STREAM_REQ, cur_agent);  // getOrderStream(symbol, length=L)
    m.w[1] = (u32)PC.hbl_L;
    send_ex(m);
    rs(AF_STATE, AS_AWAITING_STREAM);
  }
  DEV void hbl_receive(const Msg& m) {
    ta_receive(m, AG_HBL);
    // ZeroIntelligenceAgent.receiveMessage (ZI.py:311-334) with HBL's placeOrder
    if (rgi(AF_STATE) == AS_AWAITING_SPREAD && m_kind(m) == MK_SPREAD && !fl(FL_MKT_CLOSED)) {
      hbl_place();
      rs(AF_STATE, AS_AWAITING_WAKEUP);
    }
    // HBL.receiveMessage (HBL.py:197-217)
    if (rgi(AF_STATE) == AS_AWAITING_STREAM && m_kind(m) == MK_STREAM && !fl(FL_MKT_CLOSED)) {
      get_spread(1);
      rs(AF_STATE, AS_AWAITING_SPREAD);
    }
  }
  // HBL.placeOrder (HBL.py:75-195).  The streamed epochs are the exchange's live history dicts
  // (the reply carried references), so their orders and "transactions" flags are read from the
  // order-history ring as they are now.  The reference's dense arrays over [low_p, high_p] become a
  // price histogram (4 categories in 16-bit fields of one u64 per price, in an HBM scratch that is
  // zeroed again as it is scanned) and one 64-price-per-step scan: the cumulative sums, Pr = num /
  // denom (0 for 0/0, np.nan_to_num) and the expected surplus in double, and numpy's first-maximum
  // argmax.  Every count is an exact integer, so the doubles equal numpy's.
  DEV void hbl_place() {
    if (!fl(FL_HAS_STREAM) || rgi(AF_STREAM_N) < PC.hbl_L) {  // insufficient history: ZI.placeOrder
      zi_place();
      return;
    }
    i64 v;
    int buy;
    if (!zi_update_estimates(v, buy)) return;
    const i32 n = rgi(AF_STREAM_N);
    const i64 hi = rg64(AF_STREAM_HI), lo_e = hi - n + 1;
    if (lo_e < 0) {
      fail(ERR_HBL_WINDOW);
      return;
    }
    // ring records of epochs lo_e..hi: [s0, s1).  Epochs that left the exchange's 11-epoch window
    // since the reply (with latency, trades keep coming) are the dicts the reply still holds:
    // frozen, their records unchanged in the ring
    i32 s0, s1;
    if ((i64)h.epoch - lo_e <= 15) {  // within the 16-epoch entry-count ring: walk back from the current epoch
      LDSP i32* EP = ep_entries();
      s1 = h.oh_head - EP[h.epoch & 15];
      for (i64 e = (i64)h.epoch - 1; e > hi; e--) s1 -= EP[e & 15];
      s0 = s1;
      for (i64 e = hi; e >= lo_e; e--) s0 -= EP[e & 15];
    } else {  // older: count the ring's records by their epoch tags, newest chunk first
      const OhRec* R0 = ohr();
      i32 c0 = 0, c1 = 0;
      for (i32 top = h.oh_head; top > 0; top -= 64) {
        const i32 lo = top > 64 ? top - 64 : 0;
        if (h.oh_head - lo > PC.L.oh_cap) {
          fail(ERR_HBL_WINDOW);
          return;
        }
        const i32 k = lo + lane;
        const i64 ep = k < top ? (i64)R0[k % PC.L.oh_cap].epoch : (i64)INT32_MAX;
        c1 += __popcll(bal(k < top && ep > hi));
        c0 += __popcll(bal(k < top && ep >= lo_e));
        if (bal(k < top && ep < lo_e)) break;
      }
      s1 = h.oh_head - c1;
      s0 = h.oh_head - c0;
    }
    if (h.oh_head - s0 > PC.L.oh_cap) {
      fail(ERR_HBL_WINDOW);  // overwritten in the device ring (MXA_OH_CAP)
      return;
    }
    const OhRec* R = ohr();
    constexpr i32 CAP = PC.L.oh_cap;
    i32 lowp = INT32_MAX, highp = 0;  // low_p = sys.maxsize, high_p = 0 (HBL.py:100-110)
    u32 t01 = 0, t23 = 0;             // category totals (sell-tx | buy-tx << 16, sell-none | buy-none << 16)
    for (i32 b = s0; b < s1; b += 64) {
      const i32 k = b + lane;
      if (k < s1) {
        const OhRec x = R[k % CAP];
        lowp = x.price < lowp ? x.price : lowp;
        highp = x.price > highp ? x.price : highp;
      }
    }
    lowp = wmin_i32(lowp);
    highp = wmax_i32(highp);
    const i64 NB = (i64)highp - lowp + 1;
    if (s1 <= s0 || NB <= 0 || NB > PC.L.hbl_range) {
      fail(ERR_HBL_RANGE);
      return;
    }
    u64* hist = (u64*)(env + PC.L.off_hh);
    for (i32 b = s0; b < s1; b += 64) {
      const i32 k = b + lane;
      if (k < s1) {
        const OhRec x = R[k % CAP];
        const int tx = (x.meta >> 1) & 1, ib = x.meta & 1;
        const int cat = ib ? (tx ? 1 : 3) : (tx ? 0 : 2);  // nd columns sa, sb, ua, ub
        atomicAdd((unsigned long long*)&hist[x.price - lowp], 1ull << (16 * cat));
        t01 += cat == 0 ? 1u : cat == 1 ? 0x10000u : 0u;
        t23 += cat == 2 ? 1u : cat == 3 ? 0x10000u : 0u;
      }
    }
    // every lane's atomics performed at L2 before any lane reads a bucket back, and the reads
    // bypass the CU's L1 (agent-scope loads below), which may hold a stale line of the buckets.  A
    // device-scope __threadfence here also wrote back this XCD's whole L2 on every call: ~900 B of
    // HBM writes per rmsc02 event (r05 PMC, tools/ab_traffic.sh).
    // Two assumptions pin this: (1) an env's buckets are touched by ONE wave, the
    // env's own (every engine kernel is __launch_bounds__(64), one wave per env block), so no
    // other wave's atomics need to be ordered with these; (2) gfx950 (gfx9 family) counts
    // non-returning global atomics in vmcnt, so s_waitcnt(0) waits for them to be performed at
    // L2 (gfx10+ counts them in vscnt, where this sequence would not be enough)
#if !defined(__gfx950__) && defined(__HIP_DEVICE_COMPILE__)
#error "the HBL histogram readback relies on gfx9-family vmcnt accounting of global atomics"
#endif
    wfence();
    __builtin_amdgcn_s_waitcnt(0);
    wfence();
    t01 = wsum_u32(t01);
    t23 = wsum_u32(t23);
    const i64 T0 = t01 & 0xFFFF, T1 = t01 >> 16, T2 = t23 & 0xFFFF, T3 = t23 >> 16;
    i64 run0 = 0, run1 = 0, run2 = 0, run3 = 0;  // cumulative counts below this step's prices
    u64 best = 0;
    i64 bestp = lowp;
    for (i64 b = 0; b < NB; b += 64) {
      const i64 i = b + lane;
      u64 x = 0;
      if (i < NB) {
        x = __hip_atomic_load(&hist[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the reset at agent scope as well: ordered at L2 with the next call's atomics
        __hip_atomic_store(&hist[i], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const u32 c01 = (u32)(x & 0xFFFF) | ((u32)((x >> 16) & 0xFFFF) << 16);
      const u32 c23 = (u32)((x >> 32) & 0xFFFF) | ((u32)(x >> 48) << 16);
      const u32 s01 = wscan_u32(c01), s23 = wscan_u32(c23);  // inclusive, per 16-bit field
      const i64 le0 = run0 + (s01 & 0xFFFF), le1 = run1 + (s01 >> 16);
      const i64 le2 = run2 + (s23 & 0xFFFF), le3 = run3 + (s23 >> 16);
      const i64 ge0 = T0 - (le0 - (c01 & 0xFFFF)), ge1 = T1 - (le1 - (c01 >> 16));
      const i64 ge3 = T3 - (le3 - (c23 >> 16));
      const i64 num = buy ? le0 + le1 + le2 : ge0 + ge1 + ge3;
      const i64 den = buy ? num + ge3 : num + le2;
      const double pr = den > 0 ? (double)num / (double)den : 0.0;
      const i64 p = (i64)lowp + i;
      double es = pr * (double)(buy ? v - p : p - v);
      if (es == 0.0) es = 0.0;  // -0.0 ties +0.0 in numpy's argmax
      const u64 bits = as_u(es);
      const u64 key = i < NB ? ((bits >> 63) ? ~bits : (bits | (1ull << 63))) : 0ull;
      const u32 kh = ~wmin_u32(~(u32)(key >> 32));
      const u32 kl = ~wmin_u32((u32)(key >> 32) == kh ? ~(u32)key : 0xFFFFFFFFu);
      const u64 kmax = ((u64)kh << 32) | kl;
      if (b == 0 || kmax > best) {  // first maximum: a later step must be strictly greater
        best = kmax;
        bestp = (i64)lowp + b + ffs64(bal(key == kmax));
      }
      run0 += rdl(s01, 63) & 0xFFFF;
      run1 += rdl(s01, 63) >> 16;
      run2 += rdl(s23, 63) & 0xFFFF;
      run3 += rdl(s23, 63) >> 16;
    }
    const double best_es = as_d((best >> 63) ? (best & ~(1ull << 63)) : ~best);
    if (best_es > 0) place_limit(100, buy, bestp);
  }

  // ---------------- MomentumAgent (MomentumAgent.py:53-99)
  // the mean of the last n mids (n <= 50 < AF_NMID): the ring entries (nm - n .. nm - 1) % 50
  // summed across the record's lanes at once (an exact integer sum, any order)
  DEV double mom_avg(int n) {
    static_assert(AF_MIDS % 2 == 0, "the mid ring starts on a lane's low dword");
    const i32 nm = rgi(AF_NMID);
    const i32 newest = (nm - 1) % 50;
    i64 part = 0;
    for (int hw = 0; hw < 2; hw++) {
      const int k = 2 * lane + hw - AF_MIDS;  // this dword's ring index
      i32 back = newest - k;                   // how many entries older than the newest
      if (back < 0) back += 50;
      if (k >= 0 && k < 50 && back < n) part += (i64)(i32)(hw ? rhi : rlo);
    }
    const i64 s2 = wsum_i64(part);
    double x = ((double)s2 / 2.0) / (double)n;
    return __builtin_rint(x * 100.0) / 100.0;
  }
  // MomentumAgent subscribe=True (rmsc02 / obi_rmsc02): md_mom_levels > 0; rmsc03's poll
  static constexpr bool MOM_SUB = MD && PC.md_mom_levels > 0;
  DEV void mom_wakeup() {
    const bool can = ta_wakeup();
    if constexpr (MOM_SUB) {  // subscribe=True (MomentumAgent.py:54-62): level-1 data every 10 s
      if (!fl(FL_SUB_REQ)) request_subscription(PC.md_mom_levels);
      return;
    }
    if (can) {
      get_spread(1);
      rs(AF_STATE, AS_AWAITING_SPREAD);
    }
  }
  DEV void mom_receive(const Msg& m) {
    ta_receive(m, AG_MOMENTUM);
    if constexpr (MOM_SUB) {  // MomentumAgent.py:71-75: `if bids and asks`, then placeOrders(best bid, best ask)
      if (rgi(AF_STATE) == AS_AWAITING_MD && m_kind(m) == MK_MARKET_DATA) {
        i32 bid, ask;
        const bool hb = known_bid(bid), ha = known_ask(ask);
        if (hb && ha) mom_place(bid, ask);
      }
      return;
    }
    if (rgi(AF_STATE) == AS_AWAITING_SPREAD && m_kind(m) == MK_SPREAD) {
      i32 bid, ask;
      bool hb = known_bid(bid), ha = known_ask(ask);
      if (hb && ha) mom_place(bid, ask);
      wakeup_at(cur_agent, cur + PC.mom_wake);
      rs(AF_STATE, AS_AWAITING_WAKEUP);
    }
  }
  // MomentumAgent.placeOrders (MomentumAgent.py:82-93) with both prices known
  DEV void mom_place(i32 bid, i32 ask) {
    i32 nm = rgi(AF_NMID);
    rs(AF_MIDS + (nm % 50), (u32)(bid + ask));
    nm++;
    rs(AF_NMID, (u32)nm);
    if (nm > 20) {
      rsd(AF_AVG20, mom_avg(20));
      rs(AF_N20, rg(AF_N20) + 1);
    }
    if (nm > 50) {
      rsd(AF_AVG50, mom_avg(50));
      rs(AF_N50, rg(AF_N50) + 1);
    }
    if (rgi(AF_N20) > 0 && rgi(AF_N50) > 0) {
      if (rgd(AF_AVG20) >= rgd(AF_AVG50)) place_limit(rgi(AF_SIZE), 1, ask);
      else place_limit(rgi(AF_SIZE), 0, bid);
    }
  }

  // ---------------- dispatch
  // =====================================================================================
  // marketreplay / ABIDESEnv.  Compiled only into the
  // marketreplay instantiation (member templates are instantiated on use).
  // The book is a price ladder in HBM: per side and price level a FIFO list of entries
  // (count, head, tail, total qty); entries come from a per-env pool; the live entries of one
  // order id are chained so cancel/modify find them without walking a level.
  // =====================================================================================
  // the replay / gym header (best levels, free-stack top, replay cursor, RL state): the env
  // block's copy (rh_g) is the one between launches and the builder's; a run / step launch works
  // on the LDS copy (rhl, RPH).  Round 4's first LDS version faulted because the builder's save()
  // copied the LDS header -- never loaded in a build launch, so whatever an earlier kernel left
  // there -- over the header it had just written to the env block
  DEV RpHdr* rh_g() { return (RpHdr*)(env + rx->L.off_rh); }
  DEV auto rh() {
    if constexpr (RPH) return rhl;
    else return rh_g();
  }
  DEV i32* lv_cnt(int s) { return (i32*)(env + rx->L.off_lvc) + (size_t)s * U(rx->L.P); }
  DEV i32* lv_head(int s) { return (i32*)(env + rx->L.off_lvh) + (size_t)s * U(rx->L.P); }
  DEV i32* lv_tail(int s) { return (i32*)(env + rx->L.off_lvt) + (size_t)s * U(rx->L.P); }
  DEV i64* lv_qty(int s) { return (i64*)(env + rx->L.off_lvq) + (size_t)s * U(rx->L.P); }
  DEV RpEntry* pool() { return (RpEntry*)(env + rx->L.off_pool); }
  DEV i32* freel() { return (i32*)(env + rx->L.off_free); }
  DEV i32* idh() { return (i32*)(env + rx->L.off_idh); }
  DEV i32* idep() { return (i32*)(env + rx->L.off_idep); }
  DEV RpOrder* mro() { return (RpOrder*)(env + rx->L.off_mro); }
  DEV RpLob* ring() { return (RpLob*)(env + rx->L.off_ring); }
  // auto ids (DummyRL's orders, the tape's ORDER_ID 0 records) map after the tape's dense ids,
  // from this episode's first auto id on; the last dense id is never an order (orders.get(0) in
  // a later episode of the process, when no auto id 0 exists)
  DEV i32 agent_dense(i64 oid) {
    const i64 k = oid - (i64)U(rh()->id_base);
    i32 d = U(rx->L.n_ids) + (i32)k;
    if (k < 0 || d >= U(rx->L.D) - 1) {
      fail(ERR_RP_IDS);
      return 0;
    }
    return d;
  }
  DEV i32 zero_dense() { return U(rh()->id_base) == 0 ? U(rx->L.n_ids) : U(rx->L.D) - 1; }
  // generateOrderId's skip over Order._order_ids: an explicit tape id is taken once its first
  // SIZE > 0 record has been handled, in an earlier episode of the process or this one
  DEV i64 rp_skip_used(i64 c) {
    const i32 n = U(rx->nuid);
    auto R = rh();
    const i32 hi = max(U(R->tape_hi), U(R->mr_done));
    for (;;) {
      i32 lo = 0, h2 = n - 1, f = -1;
      while (lo <= h2) {  // uniform binary search over the sorted ids
        const i32 mid = (lo + h2) >> 1;
        const i64 v = (i64)U(rx->uid[mid]);
        if (v == c) {
          f = U(rx->ufirst[mid]);
          break;
        }
        if (v < c) lo = mid + 1;
        else h2 = mid - 1;
      }
      if (f < 0 || f >= hi) return c;
      c++;
    }
  }
  DEV i32 lvl_index(i32 price) {
    i32 x = price - U(rx->L.pmin);
    if (x < 0 || x >= U(rx->L.P)) {
      fail(ERR_RP_PRICE);
      return -1;
    }
    return x;
  }
  // first non-empty level from `from` toward worse prices (bids down, asks up); wave-parallel
  DEV i32 lvl_next(int side, i32 from) {
    const i32* c = lv_cnt(side);
    const i32 P = U(rx->L.P);
    for (i32 b = from; side == 0 ? b >= 0 : b < P; b += side == 0 ? -64 : 64) {
      i32 x = side == 0 ? b - lane : b + lane;
      bool ok = x >= 0 && x < P && c[x] > 0;
      u64 m = bal(ok);
      if (m) return side == 0 ? b - ctz64(m) : b + ctz64(m);
    }
    return -1;
  }
  DEV void id_link(i32 d, i32 e) {
    RpEntry* E = pool();
    i32 hd = U(idh()[d]);
    {  // every lane stores the same (uniform) value
      E[e].idprev = -1;
      E[e].idnext = hd;
      if (hd >= 0) E[hd].idprev = e;
      idh()[d] = e;
    }
  }
  DEV void id_unlink(i32 d, i32 e) {
    RpEntry* E = pool();
    i32 p = U(E[e].idprev), n = U(E[e].idnext);
    {  // every lane stores the same (uniform) value
      if (p >= 0) E[p].idnext = n;
      else idh()[d] = n;
      if (n >= 0) E[n].idprev = p;
    }
  }
  // enterOrder (OrderBook.py:256-282): append to the level FIFO
  DEV void rp_enter(i32 oid, i32 d, i32 agent, int buy, i32 qty, i32 price) {
    auto R = rh();
    const int side = buy ? 0 : 1;
    const i32 x = price - U(rx->L.pmin);
    const bool xin = x >= 0 && x < U(rx->L.P);
    rp_enter_pf(oid, d, agent, buy, qty, price, x, U(R->free_top), xin ? U(lv_tail(side)[x]) : -1,
                xin ? U(lv_cnt(side)[x]) : 0, U(R->nlev[side]), U(R->best[side]), U(idh()[d]),
                xin ? U(lv_qty(side)[x]) : (i64)0);
  }
  // rp_enter with the words it reads already loaded (rp_handle_limit gathers them in one round
  // trip): the free-stack top, the level's tail, count and quantity, the side's level count and
  // best, and the id's live-entry chain head.  No load follows its stores (a load issued after a
  // store waits for the store as well)
  DEV void rp_enter_pf(i32 oid, i32 d, i32 agent, int buy, i32 qty, i32 price, i32 x, i32 top, i32 tl, i32 cnt,
                       i32 nl, i32 bs, i32 hd, i64 lq) {
    auto R = rh();
    const int side = buy ? 0 : 1;
    if (x < 0 || x >= U(rx->L.P)) {
      fail(ERR_RP_PRICE);
      return;
    }
    if (top <= 0) {
      fail(ERR_RP_POOL);
      return;
    }
    RPCHK(top <= U(rx->L.C), "rp_enter free_top", top);
    i32 e = U(freel()[top - 1]);
    RPCHK(e >= 0 && e < U(rx->L.C), "rp_enter entry", e);
    RPCHK(d >= 0 && d < U(rx->L.D), "rp_enter dense", d);
    u32 arr = h.arrival++;
    RPCHK(tl >= -1 && tl < U(rx->L.C), "rp_enter tail", tl);
    RpEntry* E = pool();
    {  // every lane stores the same (uniform) value
      R->free_top = top - 1;
      RpEntry n;
      n.price = price;
      n.qty = qty;
      n.oid = oid;
      n.dense = d;
      n.meta = (agent << 1) | buy;
      n.arrival = arr;
      n.prev = tl;
      n.next = -1;
      n.idprev = -1;
      n.idnext = hd;  // id_link: the entry heads the id's live-entry chain
      n.pad[0] = n.pad[1] = 0;
      E[e] = n;
      if (tl >= 0) E[tl].next = e;
      else lv_head(side)[x] = e;
      lv_tail(side)[x] = e;
      lv_cnt(side)[x] = cnt + 1;
      lv_qty(side)[x] = lq + qty;
      if (hd >= 0) E[hd].idprev = e;
      idh()[d] = e;
    }
    if (cnt == 0) {
      {  // every lane stores the same (uniform) value
        R->nlev[side] = nl + 1;
        if (bs < 0 || (side == 0 ? x > bs : x < bs)) R->best[side] = x;
      }
    }
    h.b_count++;
    if (h.b_count > h.max_book) h.max_book = h.b_count;
  }
  // every word rp_unlink reads, in one round trip: lanes 0-9 the entry's words (RpEntry order:
  // price qty oid dense meta arrival prev next idprev idnext), 10/11 the level's quantity (lo,
  // hi), 12 the level's count, 13 free_top, 14/15 the side's level count and best
  DEV i32 rp_gather(int side, i32 x, i32 e) {
    RPCHK(e >= 0 && e < U(rx->L.C) && x >= 0 && x < U(rx->L.P), "rp_unlink entry/level", (i64)e * 100000 + x);
    const u64 sx = (u64)side * (u32)rx->L.P + (u32)x;
    const u64 o_w = rx->L.off_pool + (u64)e * sizeof(RpEntry), o_c = rx->L.off_lvc + 4 * sx, o_q = rx->L.off_lvq + 8 * sx,
              o_rh = rx->L.off_rh;
    asm volatile("" ::"s"(o_w), "s"(o_c), "s"(o_q), "s"(o_rh));
    const u64 ob = lane < 10 ? o_w + 4 * lane : lane < 12 ? o_q + 4 * (lane - 10) : lane == 12 ? o_c
                   : lane == 13 ? o_rh + offsetof(RpHdr, free_top) : lane == 14 ? o_rh + offsetof(RpHdr, nlev) + 4 * side
                                : o_rh + 4 * side;
    if constexpr (RPH) {  // the header words from its LDS copy, beside the gathered load
      i32 v = gather1((const i32*)(env + ob), lane < 13);
      const int hw = lane == 13 ? (int)(offsetof(RpHdr, free_top) / 4) : lane == 14 ? 2 + side : side;
      const i32 hv = ((const LDSP i32*)rhl)[hw];
      return lane >= 13 && lane < 16 ? hv : v;
    } else {
      return gather1((const i32*)(env + ob), lane < 16);
    }
  }
  // remove entry e (level x of `side`, its words gathered in g) from the book; returns the
  // side's best level after the removal
  DEV i32 rp_unlink(int side, i32 x, i32 e, i32 g) {
    auto R = rh();
    RpEntry* E = pool();
    const i32 q = rdli(g, 1), d = rdli(g, 3), p = rdli(g, 6), n = rdli(g, 7), ip = rdli(g, 8), in = rdli(g, 9);
    const i32 cnt = rdli(g, 12), top = rdli(g, 13), nl = rdli(g, 14), b = rdli(g, 15);
    RPCHK(p >= -1 && p < U(rx->L.C) && n >= -1 && n < U(rx->L.C) && d >= 0 && d < U(rx->L.D) && top >= 0 && top < U(rx->L.C),
          "rp_unlink links", (i64)p * 1000000 + n);
    {  // every lane stores the same (uniform) value
      if (p >= 0) E[p].next = n;
      else lv_head(side)[x] = n;
      if (n >= 0) E[n].prev = p;
      else lv_tail(side)[x] = p;
      lv_cnt(side)[x] = cnt - 1;
      lv_qty(side)[x] = rdl64g(g, 10) - q;
      freel()[top] = e;
      R->free_top = top + 1;
      // the id's live-entry chain
      if (ip >= 0) E[ip].idnext = in;
      else idh()[d] = in;
      if (in >= 0) E[in].idprev = ip;
    }
    h.b_count--;
    if (cnt != 1) return b;
    i32 nb = b;
    if (b == x) {
      __threadfence_block();
      nb = lvl_next(side, side == 0 ? x - 1 : x + 1);
    }
    {  // every lane stores the same (uniform) value
      R->nlev[side] = nl - 1;
      R->best[side] = nb;
    }
    return nb;
  }
  // handleLimitOrder / executeOrder (OrderBook.py:38-254) on the ladder
  DEV void rp_handle_limit(const Msg& m) {
    PROF_SCOPE(84);
    i32 oid = (i32)m.w[1], qty = (i32)m.w[2], price = (i32)m.w[3], d = (i32)m.w[5];
    i32 agent = m_agent(m);
    int buy = m_buy(m);
    if (qty <= 0) return;
    RPCHK(d >= 0 && d < U(rx->L.D), "rp_handle_limit dense", d);
    if constexpr (BLOG) bl_put(cur, price, buy ? qty : -qty);
    const i32 hep = h.epoch;
    auto R = rh();
    RpEntry* E = pool();
    const i32 pmin = U(rx->L.pmin);
    const int side = buy ? 0 : 1;
    const i32 x = price - pmin;
    const bool xin = x >= 0 && x < U(rx->L.P);
    // every word the first pass reads whose address is known now, in one round trip: lanes
    // 0-11 the id's entry epochs, 16/17 best[bids/asks], 18/19 nlev, 20 free_top, 21 the id's
    // live-entry head, 22/23 the own level's count and tail, 24/25 its quantity (lo, hi)
    PROF_IN(pt_g);
    i32 pf;
    {
      static_assert(offsetof(RpHdr, nlev) == 8 && offsetof(RpHdr, free_top) == 16, "RpHdr: best, nlev, free_top");
      // the layout words first, in one batch of scalar loads (selected per lane below: loads in
      // the arms of the select became one scalar-cache wait per arm)
      const u64 o_ep = rx->L.off_idep, o_idh = rx->L.off_idh, o_c = rx->L.off_lvc, o_t = rx->L.off_lvt, o_rh = rx->L.off_rh,
                o_q = rx->L.off_lvq;
      const u64 px = 4 * ((u64)side * (u32)rx->L.P + (u32)x);
      asm volatile("" ::"s"(o_ep), "s"(o_idh), "s"(o_c), "s"(o_t), "s"(o_rh), "s"(o_q), "s"(px));
      const u64 ob = lane < MXA_ID_EPOCHS ? o_ep + 4 * ((u64)MXA_ID_EPOCHS * d + lane)
                     : lane < 21          ? o_rh + 4 * (lane - 16)
                     : lane == 21         ? o_idh + 4 * (u64)d
                     : lane == 22         ? o_c + px
                     : lane == 23         ? o_t + px
                                          : o_q + 2 * px + 4 * (lane - 24);
      if constexpr (RPH) {  // lanes 16-20 from the header's LDS copy (best, nlev, free_top)
        pf = gather1((const i32*)(env + ob), lane < MXA_ID_EPOCHS || lane == 21 || (xin && lane >= 22 && lane < 26));
        const i32 hv = ((const LDSP i32*)rhl)[lane >= 16 && lane < 21 ? lane - 16 : 0];
        if (lane >= 16 && lane < 21) pf = hv;
      } else {
        pf = gather1((const i32*)(env + ob),
                     lane < MXA_ID_EPOCHS || (lane >= 16 && lane < 22) || (xin && lane >= 22 && lane < 26));
      }
    }
    // history[0][order_id] = ... (OrderBook.py:51-60): the id's distinct entry epochs, newest
    // first, one per lane (lanes < MXA_ID_EPOCHS).  Stored after the handler's loads (below):
    // a load issued after a store waits for that store too (one in-order vmcnt on gfx9-class
    // parts), and nothing in the handler reads these words
    static_assert(MXA_ID_EPOCHS > PC.stream_history, "the id's entry epochs must cover the history window");
    const bool ep_new = rdli(pf, 0) != hep;
    PROF_OUT(76, pt_g);  // (the gather's wait lands here: rdli uses it)
    const i32 ep_up = __shfl_up(pf, 1, 64);
    i64 ex_q = 0, ex_pq = 0;
    bool executed = false;
    i32 nb_opp = -1;
    for (;;) {
      const int opp = buy ? 1 : 0;
      __threadfence_block();
      // the opposite side's best: gathered, then tracked through the fills
      i32 b = executed ? nb_opp : rdli(pf, 16 + opp);
      bool match = b >= 0 && (buy ? price >= pmin + b : price <= pmin + b);
      if (!match) {
        PROF_IN(pt_e);
        if (!executed)  // no fill changed the gathered words
          rp_enter_pf(oid, d, agent, buy, qty, price, x, rdli(pf, 20), xin ? rdli(pf, 23) : -1,
                      xin ? rdli(pf, 22) : 0, rdli(pf, 18 + side), rdli(pf, 16 + side), rdli(pf, 21), rdl64g(pf, 24));
        else
          rp_enter(oid, d, agent, buy, qty, price);
        PROF_OUT(79, pt_e);
        PROF_IN(pt_n);
        Msg ma = msg_order(MK_ACCEPTED, oid, agent, buy, qty, price, 0);
        ma.w[5] = (u32)d;
        ex_notify(agent, ma);
        PROF_OUT(80, pt_n);
        break;
      }
      RPCHK(b < U(rx->L.P), "rp_handle_limit best", b);
      i32 e = U(lv_head(opp)[b]);
      RPCHK(e >= 0 && e < U(rx->L.C), "rp_handle_limit head", e);
      const i32 g = rp_gather(opp, b, e);
      i32 hq = rdli(g, 1), ho = rdli(g, 2), hd = rdli(g, 3), hm = rdli(g, 4), hp = rdli(g, 0);
      i32 mq;
      if (qty >= hq) {
        mq = hq;
        nb_opp = rp_unlink(opp, b, e, g);
      } else {
        mq = qty;
        {  // every lane stores the same (uniform) value
          E[e].qty = hq - qty;
          lv_qty(opp)[b] = rdl64g(g, 10) - qty;
        }
      }
      qty -= mq;
      Msg mt = msg_order(MK_EXECUTED, oid, agent, buy, mq, price, hp);
      mt.w[5] = (u32)d;
      ex_notify(agent, mt);
      Msg mm = msg_order(MK_EXECUTED, ho, hm >> 1, hm & 1, mq, hp, hp);
      mm.w[5] = (u32)hd;
      ex_notify(hm >> 1, mm);
      ex_q += mq;
      ex_pq += (i64)hp * mq;
      executed = true;
      if (qty <= 0 || status == ST_ERROR) break;
    }
    if (executed) {
      h.last_trade = py_round((double)ex_pq / (double)ex_q);
      h.last_trade_float = 0;
      h.epoch = hep + 1;
      R->ex_has_last = 1;
    }
    if (ep_new && lane < MXA_ID_EPOCHS) idep()[MXA_ID_EPOCHS * (size_t)d + lane] = lane == 0 ? hep : ep_up;
  }
  // cancelOrder (OrderBook.py:284-339): first live entry of the id at the request's level
  DEV void rp_cancel(const Msg& m) {
    PROF_SCOPE(86);
    i32 oid = (i32)m.w[1], price = (i32)m.w[3], d = (i32)m.w[5];
    const int side = m_buy(m) ? 0 : 1;
    i32 x = price - U(rx->L.pmin);
    if (x < 0 || x >= U(rx->L.P)) return;
    RPCHK(d >= 0 && d < U(rx->L.D), "rp_cancel dense", d);
    RpEntry* E = pool();
    i32 best = -1;
    u32 ba = 0xFFFFFFFFu;
    i32 guard = 0;
    for (i32 e = U(idh()[d]); e >= 0 && guard < (1 << 16); e = U(E[e].idnext), guard++) {
      bool at = U(E[e].price) == price && (U(E[e].meta) & 1) == (side == 0) && U(E[e].oid) == oid;
      u32 a = U(E[e].arrival);
      if (at && a < ba) {
        ba = a;
        best = e;
      }
    }
    if (best < 0) return;
    i32 q = U(E[best].qty), mt = U(E[best].meta);
    if constexpr (BLOG) bl_put(cur, -price, side == 0 ? q : -q);
    rp_unlink(side, x, best, rp_gather(side, x, best));
    Msg r = msg_order(MK_CANCELLED, oid, mt >> 1, mt & 1, q, price, 0);
    r.w[5] = (u32)d;
    ex_notify(m_agent(m), r);
  }
  // modifyOrder (OrderBook.py:341-372): each entry of the id at the level replaces the level
  // HEAD with the new order; one ORDER_MODIFIED per match per history epoch holding the id
  DEV void rp_modify(const Msg& m) {
    PROF_SCOPE(85);
    if (m.w[0] & MF_NOT_SAME) return;  // isSameOrder(order, new_order) is False
    i32 oid = (i32)m.w[1], qty = (i32)m.w[2], price = (i32)m.w[3], oprice = (i32)m.w[4], d = (i32)m.w[5];
    const int buy = m_buy(m), side = buy ? 0 : 1;
    i32 agent = m_agent(m);
    i32 x = oprice - U(rx->L.pmin);
    if (x < 0 || x >= U(rx->L.P)) return;
    RPCHK(d >= 0 && d < U(rx->L.D), "rp_modify dense", d);
    // the words known now, in one round trip: lanes 0-11 the id's entry epochs, 12/13 the
    // level's count and head, 14 the id's live-entry head
    const i32* EP = idep() + MXA_ID_EPOCHS * (size_t)d;
    i32 g;
    {
      const u64 px = 4 * ((u64)side * (u32)rx->L.P + (u32)x);
      const u64 o_ep = rx->L.off_idep + 4 * (u64)MXA_ID_EPOCHS * d, o_c = rx->L.off_lvc + px, o_h = rx->L.off_lvh + px,
                o_idh = rx->L.off_idh + 4 * (u64)d, o_q = rx->L.off_lvq + 2 * px;
      asm volatile("" ::"s"(o_ep), "s"(o_c), "s"(o_h), "s"(o_idh), "s"(o_q));
      // lanes 0-11 the id's epochs, 12/13 the level's count and head, 14 the id's chain head,
      // 15/16 the level's quantity (lo, hi)
      const u64 ob = lane < MXA_ID_EPOCHS ? o_ep + 4 * lane : lane == 12 ? o_c : lane == 13 ? o_h : lane == 14 ? o_idh
                                                                                     : o_q + 4 * (lane - 15);
      g = gather1((const i32*)(env + ob), lane < 17);
    }
    if (rdli(g, 12) == 0) return;
    if (price != oprice) {
      fail(ERR_RP_MODIFY);
      return;
    }
    RpEntry* E = pool();
    const i32 hd = rdli(g, 13);
    RPCHK(hd >= 0 && hd < U(rx->L.C), "rp_modify head", hd);
    // one round trip: lanes 0-9 the id chain's first entry, 16-25 the level head's entry
    const i32 e0 = rdli(g, 14);
    const i32 g2 = gather1(lane < 10 ? (const i32*)(E + (e0 >= 0 ? e0 : 0)) + lane : (const i32*)(E + hd) + (lane - 16),
                           (lane < 10 && e0 >= 0) || (lane >= 16 && lane < 26));
    int matches = 0;
    i32 guard = 0, e = e0;
    if (e >= 0) {
      if (rdli(g2, 0) == oprice && (rdli(g2, 4) & 1) == buy && rdli(g2, 2) == oid) matches++;
      e = rdli(g2, 9);
      guard = 1;
    }
    for (; e >= 0 && guard < (1 << 16); e = U(E[e].idnext), guard++)
      if (U(E[e].price) == oprice && (U(E[e].meta) & 1) == buy && U(E[e].oid) == oid) matches++;
    if (matches == 0) return;
    i32 hq = rdli(g2, 17), hdense = rdli(g2, 19);
    if (hdense != d) {  // the head moves from its id's live-entry chain to the new id's
      const i32 p = rdli(g2, 24), n = rdli(g2, 25);
      {  // every lane stores the same (uniform) value
        if (p >= 0) E[p].idnext = n;
        else idh()[hdense] = n;
        if (n >= 0) E[n].idprev = p;
        // (the chain of d is untouched by that: its head is still e0)
        E[hd].idprev = -1;
        E[hd].idnext = e0;
        if (e0 >= 0) E[e0].idprev = hd;
        idh()[d] = hd;
      }
    }
    {  // every lane stores the same (uniform) value
      E[hd].oid = oid;
      E[hd].dense = d;
      E[hd].qty = qty;
      E[hd].meta = (agent << 1) | buy;
      lv_qty(side)[x] = rdl64g(g, 15) + (i64)(qty - hq);
    }
    if constexpr (BLOG) bl_put(cur, -(oprice | BL_MODIFY | (side << 29)), qty - hq);
    // one ORDER_MODIFIED per retained history epoch holding the id (OrderBook.py:352-355)
    const i32 lo = h.epoch - PC.stream_history;
    const int neps = __popcll(bal(lane < MXA_ID_EPOCHS && g >= lo));
    for (int k = 0; k < matches * neps; k++) {
      Msg r = msg_order(MK_MODIFIED, oid, agent, buy, qty, price, 0);
      r.w[5] = (u32)d;
      ex_notify(agent, r);
    }
  }
  // QUERY_SPREAD reply with `depth` levels (ExchangeAgent.py:215-245): level-1 price/qty,
  // level-2 prices and the level counts (w6/w7 = price2 | count << 20)
  DEV void rp_spread(const Msg& m, bool closed) {
    auto R = rh();
    const i32 pmin = U(rx->L.pmin);
    i32 depth = (i32)m.w[1];
    i32 nb = U(R->nlev[0]), na = U(R->nlev[1]);
    nb = nb < depth ? nb : depth;
    na = na < depth ? na : depth;
    Msg r = msg_make(MK_SPREAD, 0);
    i32 bb = U(R->best[0]), ab = U(R->best[1]);
    if (nb > 0) {
      r.w[1] = (u32)(pmin + bb);
      r.w[2] = (u32)U(lv_qty(0)[bb]);
    }
    if (na > 0) {
      r.w[3] = (u32)(pmin + ab);
      r.w[4] = (u32)U(lv_qty(1)[ab]);
    }
    i32 b2 = 0, a2 = 0;
    if (nb > 1) b2 = pmin + lvl_next(0, bb - 1);
    if (na > 1) a2 = pmin + lvl_next(1, ab + 1);
    r.w[6] = (u32)b2 | ((u32)nb << 20);
    r.w[7] = (u32)a2 | ((u32)na << 20);
    r.w[5] = (u32)h.last_trade;
    u32 hasd = (u32)U(R->ex_has_last);
    r.w[0] |= ((u32)(nb > 0) << 9) | ((u32)(na > 0) << 10) | (hasd << 11) | ((u32)closed << 7);
    ex_notify(m_agent(m), r);
  }

  // ---------------- MarketReplayAgent (MarketReplayAgent.py:50-96)
  // ORDER_ID 0 records: `orders.get(0)` finds the order whose auto id is 0 (dense index n_ids in
  // the first episode of a process; never later: zero_dense);
  // placing or modifying builds LimitOrder(order_id=0), which takes the next auto id
  // (Order.py:26), so a modify then fails isSameOrder at the exchange (OrderBook.py:343-344)
  DEV void mr_place_record(i32 r) {
    PROF_SCOPE(91);
    mr_place_record_v(r, U(rx->oid[r]), U(rx->price[r]), U(rx->size[r]), U(rx->dense[r]), (i32)rx->buy[r]);
  }
  // record r with its tape words already loaded (mr_wakeup gathers the next record's with the
  // group times)
  DEV void mr_place_record_v(i32 r, i32 oid, i32 price, i32 size, i32 dense, i32 buy) {
    RPCHK(r >= 0 && r < U(rx->L.nrec), "mr_place_record record", r);
    const i32 d = oid == 0 ? zero_dense() : dense;
    RPCHK(d >= 0 && d < U(rx->L.D), "mr_place_record dense", d);
    mr_place_record_as(r, oid, d, price, size, U(buy));
    rh()->mr_done = r + 1;  // record r's explicit id (if SIZE > 0) is in Order._order_ids now
    rs(AF_MR_DONE, (u32)(r + 1));
  }
  DEV void mr_place_record_as(i32 r, i32 oid, i32 d, i32 price, i32 size, int buy) {
    const RpOrder O = mro()[d];  // one 16-byte load: every field the three branches read
    const i32 present = U(O.present);
    if (!present && size > 0) {  // placeLimitOrder(..., order_id=ORDER_ID)
      i32 id = oid, dd = d;
      if (oid == 0) {
        id = (i32)next_order_id();
        dd = agent_dense(id);
      }
      {  // every lane stores the same (uniform) value
        RpOrder o;
        o.qty = size;
        o.price = price;
        o.is_buy = buy;
        o.present = 1;
        mro()[dd] = o;
      }
      Msg lm = msg_order(MK_LIMIT, id, cur_agent, buy, size, price, 0);
      lm.w[5] = (u32)dd;
      send_ex(lm);
    } else if (present && size == 0) {  // cancelOrder(existing_order)
      Msg cm = msg_order(MK_CANCEL, oid, cur_agent, U(O.is_buy), U(O.qty), U(O.price), 0);
      cm.w[5] = (u32)d;
      send_ex(cm);
    } else if (present) {  // modifyOrder(existing_order, LimitOrder(..., order_id))
      i32 id = oid;
      if (oid == 0) id = (i32)next_order_id();
      else if (buy != U(O.is_buy)) {
        fail(ERR_RP_MODIFY);
        return;
      }
      Msg mm = msg_order(MK_MODIFY, id, cur_agent, buy, size, price, U(O.price));
      mm.w[5] = (u32)d;
      if (id != oid) mm.w[0] |= MF_NOT_SAME;
      send_ex(mm);
    }
  }
  DEV void mr_wakeup() {
    PROF_SCOPE(87);
    ta_wakeup();
    u32 f = flags();
    if (!((f & FL_HAS_OPEN) && (f & FL_HAS_CLOSE))) return;
    const i32 wi = rgi(AF_MR_WI);
    const i32 ntm = U(rx->L.ntm);
    if (wi >= ntm) return;  // IndexError: every order submitted (the last group never is)
    // one round trip for the tape words this wakeup reads in the common case: lane 0 tm[wi],
    // lane 1 tm[wi - 1], lanes 2-4 tm0[wi - 1 .. wi + 1] (tm0 has ntm + 1 entries), and lanes
    // 8-12 the words of record rn, the next one in tape order (a group's first on time)
    PROF_IN(pt_w);
    const i32 rn = rgi(AF_MR_DONE);
    const bool rn_ok = rn < U(rx->L.nrec);
    // 32-bit words: lanes 0/1 tm[wi] (lo, hi), 2/3 tm[wi - 1], 4-6 tm0[wi - 1 .. wi + 1], 8-11 the
    // record's oid / price / size / dense, 12 the aligned word holding its int8 side
    i32 tw;
    {
      // the tape's array addresses first, in one batch of scalar loads, then one select per lane
      const u64 a_tm = (u64)rx->tm, a_tm0 = (u64)rx->tm0, a_oid = (u64)rx->oid, a_pr = (u64)rx->price,
                a_sz = (u64)rx->size, a_dn = (u64)rx->dense, a_buy = (u64)rx->buy;
      asm volatile("" ::"s"(a_tm), "s"(a_tm0), "s"(a_oid), "s"(a_pr), "s"(a_sz), "s"(a_dn), "s"(a_buy));
      const u64 a = lane < 2    ? a_tm + 8 * (i64)wi + 4 * lane
                    : lane < 4  ? a_tm + 8 * (i64)(wi - 1) + 4 * (lane - 2)
                    : lane < 8  ? a_tm0 + 4 * (i64)(wi - 5 + lane)
                    : lane == 8 ? a_oid + 4 * (i64)rn
                    : lane == 9 ? a_pr + 4 * (i64)rn
                    : lane == 10 ? a_sz + 4 * (i64)rn
                    : lane == 11 ? a_dn + 4 * (i64)rn
                                 : ((a_buy + (u64)rn) & ~(u64)3);
      const bool ok = lane < 2 || ((lane == 2 || lane == 3 || lane == 4) && wi > 0) || lane == 5 || lane == 6 ||
                      (lane >= 8 && lane < 13 && rn_ok);
      tw = gather1((const i32*)a, ok);
    }
    const i64 tn = (i64)(((u64)(u32)rdli(tw, 1) << 32) | (u32)rdli(tw, 0));
    const i64 tprev = (i64)(((u64)(u32)rdli(tw, 3) << 32) | (u32)rdli(tw, 2));
    const i32 rbuy = (i32)(int8_t)(rdli(tw, 12) >> (8 * (rn & 3)));
    PROF_OUT(81, pt_w);
    PROF_IN(pt_k);
    wakeup_at(cur_agent, tn);
    rs(AF_MR_WI, (u32)(wi + 1));
    PROF_OUT(82, pt_k);
    // orders[currentTime]: tm is strictly increasing (sorted tape), so the match is unique. A
    // wakeup on time is at the group just scheduled before (wi - 1) or at wi itself (the first
    // one); anything else (a delayed wakeup) takes the binary search
    i32 lo = 0, hi = ntm - 1, g = -1;
    if (tn == cur) g = wi, lo = hi + 1;
    else if (wi > 0 && tprev == cur) g = wi - 1, lo = hi + 1;
    if (g >= 0) {  // the group's record range from the batch
      const i32 r0 = rdli(tw, g == wi ? 5 : 4), r1 = rdli(tw, g == wi ? 6 : 5);
      RPCHK(r0 >= 0 && r0 <= r1 && r1 <= U(rx->L.nrec), "mr_wakeup group", (i64)r0 * 1000000 + r1);
      for (i32 r = r0; r < r1; r++) {
        if (r == rn && rn_ok) {
          PROF_IN(pt_p);
          mr_place_record_v(r, rdli(tw, 8), rdli(tw, 9), rdli(tw, 10), rdli(tw, 11), rbuy);
          PROF_OUT(83, pt_p);
        }
        else
          mr_place_record(r);
      }
      return;
    }
    while (lo <= hi) {
      i32 mid = (lo + hi) >> 1;
      i64 tv = U(rx->tm[mid]);
      if (tv == cur) {
        g = mid;
        break;
      }
      if (tv < cur) lo = mid + 1;
      else hi = mid - 1;
    }
    if (g < 0) {
      fail(ERR_RP_KEYERROR);
      return;
    }
    const i32 r1 = U(rx->tm0[g + 1]);
    for (i32 r = U(rx->tm0[g]); r < r1; r++) mr_place_record(r);
  }
  DEV void mr_receive(const Msg& m) {
    PROF_SCOPE(88);
    ta_receive(m, AG_REPLAY);
  }

  // ---------------- DummyRLExecutionAgent (dummy_rl_execution_agent.py) + GymKernel hooks
  DEV void kcancel_at(i64 t) {  // GymKernel.setCancelOrder(sender, t - Timedelta(0.5) = t)
    if (t < cur) {
      fail(ERR_WAKEUP_PAST);
      return;
    }
    Msg m = msg_make(MK_KCANCEL, 0);
    u64 key = ((u64)t << KSH) | ((u64)cur_agent << 2) | MT_CANCEL_ORDER;
    q_push(key, seq++, m);
  }
  DEV void rl_wakeup() {
    if (!ta_wakeup()) return;
    auto R = rh();
    // first horizon time strictly after now
    i32 k = cur < PC.rl_h0 ? 0 : (i32)((cur - PC.rl_h0) / PC.rl_hstep) + 1;
    i32 trade = U(R->rl_trade);
    if (trade) {
      if (k < PC.rl_nh) kcancel_at(PC.rl_h0 + (i64)k * PC.rl_hstep);
      else trade = 0;
    }
    if (trade) {  // effective_time_horizon = execution_time_horizon[:-1]
      if (k < PC.rl_nh - 1) wakeup_at(cur_agent, PC.rl_h0 + (i64)k * PC.rl_hstep);
      else trade = 0;
    }
    R->rl_trade = trade;
    get_spread(PC.rl_depth);
    rs(AF_STATE, AS_AWAITING_SPREAD);
  }
  // ABIDESEnvMetrics.addLOB: deque(maxlen=100), newest first
  DEV void rl_add_lob(const Msg& m) {
    auto R = rh();
    const i32 nb = (i32)(m.w[6] >> 20), na = (i32)(m.w[7] >> 20);
    const int dnone = !m_hasdata(m);
    i32 ph = U(R->ph_n), cnt = U(R->m_cnt), hd = U(R->m_head);
    RPCHK(cnt >= 0 && cnt <= 100 && hd >= 0 && hd < 100, "rl_add_lob ring", (i64)cnt * 1000 + hd);
    hd = (hd + 99) % 100;
    {  // every lane stores the same (uniform) value
      if (ph == 0) {
        R->p0 = (i32)m.w[5];
        R->p0_none = dnone;
      }
      RpLob l;
      l.bid = (i32)m.w[1];
      l.ask = (i32)m.w[3];
      l.data = (i32)m.w[5];
      l.flags = (nb > 0 ? 1 : 0) | (na > 0 ? 2 : 0) | (dnone ? 4 : 0);
      ring()[hd] = l;
      R->m_head = hd;
      R->m_cnt = cnt < 100 ? cnt + 1 : 100;
      R->m_nb = nb;
      R->m_na = na;
      R->m_bq = (i32)m.w[2];
      R->m_aq = (i32)m.w[4];
      R->m_b2 = (i32)(m.w[6] & 0xFFFFFu);
      R->m_a2 = (i32)(m.w[7] & 0xFFFFFu);
      R->ph_n = ph + 1;
      if (dnone) R->ph_none = 1;
    }
  }
  DEV void rl_receive(const Msg& m) {
    PROF_SCOPE(89);
    ta_receive(m, AG_DUMMYRL);
    auto R = rh();
    const u32 k = m_kind(m);
    if (k == MK_EXECUTED) {  // ExecutionAgent.handleOrderExecution (the DummyRL override is misspelt)
      i64 ex = U(R->rl_exec) + (i32)m.w[2];
      {  // every lane stores the same (uniform) value
        R->rl_exec = ex;
        R->rl_rem = PC.rl_quantity - ex;
      }
    }
    __threadfence_block();
    if (U(R->rl_rem) > 0 && rgi(AF_STATE) == AS_AWAITING_SPREAD && k == MK_SPREAD) {
      rs(AF_STATE, AS_AWAITING_WAKEUP);
      rl_add_lob(m);
    }
    if (k == MK_SPREAD) {  // GymKernel.stepRunner: observation, end of step
      __threadfence_block();
      rl_observe();
      end_step = 1;
    }
  }
  // numpy pairwise summation (n <= 128) and np.std
  // numpy's pairwise sum (pairwise_sum, numpy/core/src/umath/loops_utils.h: 8 accumulators below
  // 128 elements) over a[i] = lane i % 64 of v0 (i < 64) / v1 (i >= 64), in numpy's order
  DEV double np_pairwise_lanes(double v0, double v1, int n) {
    auto at = [&](int i) -> double { return i < 64 ? rdl_d(v0, i) : rdl_d(v1, i - 64); };
    if (n < 8) {
      double r = 0.;
      for (int i = 0; i < n; i++) r += at(i);
      return r;
    }
    double r0 = at(0), r1 = at(1), r2 = at(2), r3 = at(3), r4 = at(4), r5 = at(5), r6 = at(6), r7 = at(7);
    int i;
    for (i = 8; i < n - (n % 8); i += 8) {
      r0 += at(i);
      r1 += at(i + 1);
      r2 += at(i + 2);
      r3 += at(i + 3);
      r4 += at(i + 4);
      r5 += at(i + 5);
      r6 += at(i + 6);
      r7 += at(i + 7);
    }
    double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < n; i++) res += at(i);
    return res;
  }
  // DummyRL.get_observation (dummy_rl:291-312): float64[9] into the replay header
  DEV void rl_observe() {
    auto R = rh();
    const i64 fl = (cur / PC.rl_hstep) * PC.rl_hstep;  // currentTime.floor("30S")
    i32 rem = PC.rl_nh;
    if (fl >= PC.rl_h0 && (fl - PC.rl_h0) / PC.rl_hstep < PC.rl_nh) rem = PC.rl_nh - 1 - (i32)((fl - PC.rl_h0) / PC.rl_hstep);
    const i32 cnt = U(R->m_cnt), hd = U(R->m_head);
    RPCHK(cnt >= 0 && cnt <= 100 && hd >= 0 && hd < 100, "rl_observe ring", (i64)cnt * 1000 + hd);
    double o[9];
    o[0] = (double)rem;
    o[1] = (double)U(R->rl_rem);
    if (cnt == 0) {
      fail(ERR_RP_OBS);
      return;
    }
    const RpLob* L = ring();
    const i32 f0 = U(L[hd].flags);
    if ((f0 & 4) || U(R->p0_none)) {
      fail(ERR_RP_OBS);
      return;
    }
    const i64 p0 = U(R->p0), pt = U(L[hd].data);
    const i64 bid = U(L[hd].bid), ask = U(L[hd].ask), bv = U(R->m_bq), av = U(R->m_aq);
    // the deque's log mid returns, lane-parallel: entry i in lane i % 64, register i / 64 (at
    // most 100 entries); one coalesced load and one log evaluation per register
    double lv[2];
    bool bad = false;
    for (int c = 0; c < 2; c++) {
      const int i = c * 64 + lane;
      double x = 1.0;
      if (i < cnt) {
        const RpLob li = L[(hd + i) % 100];
        bad |= (li.flags & 3) != 3;
        x = (double)((i64)li.bid + li.ask) / 2 / (double)p0;
      }
      lv[c] = gm_log(x);
    }
    if (bal(bad)) {  // the reference raises at the first LOB with a missing side
      fail(ERR_RP_OBS);
      return;
    }
    o[2] = gm_log((double)pt / (double)p0);
    o[3] = (double)(ask - bid);
    o[4] = (double)(bv - av) / (double)(bv + av);
    o[5] = tanh((double)ask / (double)av - (double)bid / (double)bv);
    const double mean = np_pairwise_lanes(lv[0], lv[1], cnt) / cnt;
    for (int c = 0; c < 2; c++) {
      const double dd = lv[c] - mean;
      lv[c] = dd * dd;
    }
    o[6] = __builtin_sqrt(np_pairwise_lanes(lv[0], lv[1], cnt) / cnt);
    const double mt = (double)(bid + ask) / 2;
    int dir;
    if ((double)pt > mt) dir = 1;
    else if ((double)pt < mt) dir = -1;
    else {  // idx - 1 == -1: the oldest stored LOB
      const RpLob ll = L[(hd + cnt - 1) % 100];
      double ml = (double)((i64)U(ll.bid) + U(ll.ask)) / 2;
      dir = mt > ml ? 1 : -1;
    }
    o[7] = (double)dir;
    o[8] = (double)(2 * dir) * ((double)pt - mt) / mt;
    {  // every lane stores the same (uniform) value
      for (int i = 0; i < 9; i++) R->obs[i] = o[i];
      R->has_obs = 1;
    }
  }
  // DummyRL.process_action + place_orders (dummy_rl:138-179), called by the step kernel
  DEV void rl_place_orders(const double* act) {
    PROF_SCOPE(90);
    auto R = rh();
    rec_load(PC.first_rl);
    const double q0 = (double)PC.rl_quantity, q = q0;  // metrics.rem_quantity is never updated
    const double x = act[0], sum = 0.0 + act[1] + act[2];
    double oh0 = 0.5, oh1 = 0.5;
    if (sum != 0.0) {
      oh0 = act[1] / sum;
      oh1 = act[2] / sum;
    }
    const double qh = q / q0;
    const double total = __builtin_rint(q0 * qh * gm_pow(x, gm_pow(qh, 0.5)));
    const double o0 = __builtin_rint(total * oh0);
    const double o1 = total - (0.0 + o0);
    const i32 cnt = U(R->m_cnt), hd = U(R->m_head), nb = U(R->m_nb), na = U(R->m_na);
    for (int l = 0; l < 2; l++) {
      if (cnt == 0 || nb == 0 || na == 0 || l >= nb || l >= na) continue;  // raises: skipped
      i32 price = l == 0 ? U(ring()[hd].bid) : U(R->m_b2);                  // BUY at bid level l+1
      place_limit((i64)(l == 0 ? o0 : o1), 1, price);
    }
    rec_store();
  }
  // GymKernel CANCEL_ORDER branch (GymKernel.py:244-249): get_reward (None), cancelAllOrders
  DEV void rl_kernel_cancel() {
    auto R = rh();
    if (U(R->m_cnt) == 0 || U(R->ph_none)) {
      fail(ERR_RP_OBS);
      return;
    }
    rec_load(PC.first_rl);
    cancel_all();
    rec_store();
  }
  // GymKernel.terminateRunner -> ExecutionAgent.kernelStopping (execution_agent.py:45-58)
  DEV void rp_terminate() {
    auto R = rh();
    if (U(R->finished)) return;
    R->finished = 1;
    if (U(R->rl_trade)) fail(ERR_RP_STOPPING);
  }

  // ---------------- TWAPExecutionAgent (agent/execution/baselines/twap_agent.py:9-63) on the
  // replay: ExecutionAgent.wakeup / receiveMessage / placeOrders (execution_agent.py:65-123).
  // The horizon is pd.date_range(rl_h0, ..., rl_hstep) (rl_nh times); RpHdr::rl_trade = -e.
  DEV void tw_wakeup() {
    if (!ta_wakeup()) return;
    if (!U(rh()->rl_trade)) return;
    // [time for time in execution_time_horizon if time > currentTime][0] (IndexError: none)
    const i32 k = cur < PC.rl_h0 ? 0 : (i32)((cur - PC.rl_h0) / PC.rl_hstep) + 1;
    if (k < PC.rl_nh) wakeup_at(cur_agent, PC.rl_h0 + (i64)k * PC.rl_hstep);
    get_spread(PC.rl_depth);
    rs(AF_STATE, AS_AWAITING_SPREAD);
  }
  // The schedule is keyed by the 60 s bins of pd.interval_range(start, end, freq) (twap_agent.py:
  // 50-55) and read with a 30 s Interval (execution_agent.py:118): the first limit order raises
  // KeyError, so no TWAP order reaches the exchange (nothing executes, rem_quantity stays > 0)
  DEV void tw_receive(const Msg& m) {
    ta_receive(m, AG_TWAP);
    if (rgi(AF_STATE) != AS_AWAITING_SPREAD || m_kind(m) != MK_SPREAD) return;
    // cancelOrders(): self.orders is empty.  placeOrders(currentTime):
    const i64 d = cur - PC.rl_h0;
    if (d < 0 || d % PC.rl_hstep != 0 || d / PC.rl_hstep >= PC.rl_nh) return;  // not a horizon time
    const i64 k = d / PC.rl_hstep;
    if (k == PC.rl_nh - 2) {
      fail(ERR_TWAP_MARKET);
      return;
    }
    if (k < PC.rl_nh - 2) {
      const u32 f = flags();
      fail((f & FL_NB) && (f & FL_NA) ? ERR_TWAP_SCHEDULE : ERR_TWAP_QUOTE);
    }
  }

  // agent classes absent from the configuration are compiled out
  DEV void dispatch(int type, bool wake, const Msg& m) {
    if (wake) {
      if constexpr (PC.n_zi > 0)
        if (type == AG_ZI) return zi_wakeup();
      if constexpr (PC.n_noise > 0)
        if (type == AG_NOISE) return noise_wakeup();
      if constexpr (PC.n_value > 0)
        if (type == AG_VALUE) return value_wakeup();
      if constexpr (PC.n_mm > 0)
        if (type == AG_POVMM) return mm_wakeup();
      if constexpr (PC.n_mom > 0)
        if (type == AG_MOMENTUM) return mom_wakeup();
      if constexpr (PC.n_mk > 0)
        if (type == AG_MKTMAKER) return mk_wakeup();
      if constexpr (PC.n_hbl > 0)
        if (type == AG_HBL) return hbl_wakeup();
      if constexpr (PC.n_obi > 0)
        if (type == AG_OBI) return obi_wakeup();
      if constexpr (PC.n_sb > 0)
        if (type == AG_SBMM) return sb_wakeup();
      if constexpr (RP) {
        if (type == AG_REPLAY) return mr_wakeup();
        if constexpr (TW) {
          if (type == AG_TWAP) return tw_wakeup();
        }
      }
      if constexpr (GYM) {
        if (type == AG_DUMMYRL) return rl_wakeup();
      }
      // ExchangeAgent: Agent.wakeup does nothing
    } else {
      if (type == AG_EXCHANGE) return ex_receive(m);
      if constexpr (PC.n_zi > 0)
        if (type == AG_ZI) return zi_receive(m);
      if constexpr (PC.n_noise > 0)
        if (type == AG_NOISE) return noise_receive(m);
      if constexpr (PC.n_value > 0)
        if (type == AG_VALUE) return value_receive(m);
      if constexpr (PC.n_mm > 0)
        if (type == AG_POVMM) return mm_receive(m);
      if constexpr (PC.n_mom > 0)
        if (type == AG_MOMENTUM) return mom_receive(m);
      if constexpr (PC.n_mk > 0)
        if (type == AG_MKTMAKER) return mk_receive(m);
      if constexpr (PC.n_hbl > 0)
        if (type == AG_HBL) return hbl_receive(m);
      if constexpr (PC.n_obi > 0)
        if (type == AG_OBI) return obi_receive(m);
      if constexpr (PC.n_sb > 0)
        if (type == AG_SBMM) return sb_receive(m);
      if constexpr (RP) {
        if (type == AG_REPLAY) return mr_receive(m);
        if constexpr (TW) {
          if (type == AG_TWAP) return tw_receive(m);
        }
      }
      if constexpr (GYM) {
        if (type == AG_DUMMYRL) return rl_receive(m);
      }
    }
  }

  // ---------------- Kernel.runner after the loop: kernelStopping per agent in id order
  // (Kernel.py:305-312).  FINAL_VALUATION of ZI (ZeroIntelligenceAgent.py:80-112), Noise
  // (NoiseAgent.py:44-68) and Value (ValueAgent.py:66-86) agents; ZI and Value observe the
  // oracle at their own currentTime (the last event they handled = agentCurrentTimes minus
  // their computation delay) with sigma_n = 0, advancing it in agent order.
  DEV static i64 round_hundreds(i64 x) {  // int(round(x, -2) / 100), Python half-to-even
    i64 q = x / 100, r = x % 100;
    if (r < 0) {
      r += 100;
      q -= 1;
    }
    if (r > 50 || (r == 50 && (q & 1))) q += 1;
    return q;
  }
  DEV void stop(mxa_agent_final* out) {
    for (int a = 1; a < PC.n_agents; a++) {
      rec_load(a);
      const int ty = rgi(AF_TYPE);
      mxa_agent_final f;
      f.final_fundamental = 0;
      f.valuation_int = 0;
      f.valuation = 0.0;
      f.kind = 0;
      f.err = 0;
      const i64 cash = rg64(AF_CASH), start = rg64(AF_START_CASH);
      const i64 H = round_hundreds(rg64(AF_SHARES));
      const u32 fl = flags();
      if (ty == AG_NOISE) {
        f.kind = 2;
        if (!(fl & FL_HAS_KNOWN)) {
          f.err = 1;
        } else if ((fl & FL_NB) && (fl & FL_NA) && rgi(AF_BID) != 0 && rgi(AF_ASK) != 0) {
          const double rT = (double)((i64)rgi(AF_BID) + rgi(AF_ASK)) / 2.0;  // int(bid + ask) / 2
          f.valuation = (rT * (double)H + (double)(cash - start)) / (double)start;
        } else if (!(fl & FL_HAS_LAST)) {
          f.err = 1;
        } else if (fl & FL_LAST_FLOAT) {  // rT = last_trade[symbol], a python float
          f.valuation = ((double)rg64(AF_LAST_TRADE) * (double)H + (double)(cash - start)) / (double)start;
        } else {
          f.valuation = (double)(rg64(AF_LAST_TRADE) * H + cash - start) / (double)start;
        }
      } else if (ty == AG_VALUE || ty == AG_ZI || ty == AG_HBL) {  // HBL inherits ZI.kernelStopping
        const i64 rT = o_observe(rg64(AF_ATIME) - rg64(AF_COMP), 0.0);
        if (dirty) rng_maint();
        f.final_fundamental = rT;
        if (ty == AG_VALUE) {
          f.kind = 2;
          f.valuation = (double)(rT * H + cash - start) / (double)start;
        } else {
          f.kind = 1;
          const int nq = 2 * PC.zi_qmax;
          i64 s = 0;
          if (H > nq - PC.zi_qmax || H < -nq - PC.zi_qmax) {
            f.err = 2;  // theta[x + q_max - 1] outside [-2 q_max, 2 q_max) (IndexError)
          } else if (H > 0) {
            for (i64 x = 1; x <= H; x++) s += rgi(AF_THETA + (int)(x + PC.zi_qmax - 1));
          } else if (H < 0) {
            for (i64 x = H + 1; x <= 0; x++) {
              i64 i = x + PC.zi_qmax - 1;
              s -= rgi(AF_THETA + (int)(i < 0 ? i + nq : i));  // Python negative indices wrap
            }
          }
          f.valuation_int = s + rT * H + cash - start;
        }
      }
      if (lane == 0) out[a] = f;
    }
    if (lane == 0) out[0] = mxa_agent_final{0, 0, 0.0, 0, 0};
  }

  // ---------------- state save/restore around a launch
  DEV void hdr_from_global() {
    const u64* src = (const u64*)hdr();
    u64* dst = (u64*)&h;
    if (lane < (int)(sizeof(EnvHdr) / 8)) dst[lane] = src[lane];
    wfence();
    cur = h.cur;
    stop_t = h.t_stop > 0 ? h.t_stop : PC.stop;
    pops = h.pops;
    ocnt = h.order_counter;
    hash = h.hash;
    seq = h.seq;
    status = h.status;
    err = h.err;
    qcount = h.q_count;
    maxq = h.max_q;
    if (lane < 4) h.rs_wn[lane] = 0;  // the LDS stream windows did not survive the last launch
    wfence();
    if constexpr (KREG) {
      kp = h.rs_pos[KS];
      km = h.rs_m[KS];
      khg = h.rs_has_gauss[KS];
      kw0 = h.rs_w0[KS];
      kwn = 0;
    }
  }
  DEV void hdr_to_global() {
    if (lane == 0) {
      h.cur = cur;
      h.pops = pops;
      h.order_counter = ocnt;
      h.hash = hash;
      h.seq = seq;
      h.status = status;
      h.err = err;
      h.q_count = qcount;
      if constexpr (MAXQ_REG) h.max_q = maxq;
      if constexpr (KREG) {
        h.rs_pos[KS] = kp;
        h.rs_m[KS] = km;
        h.rs_has_gauss[KS] = khg;
        h.rs_w0[KS] = kw0;
        h.rs_wn[KS] = kwn;
      }
    }
    wfence();
    const u64* src = (const u64*)&h;
    u64* dst = (u64*)hdr();
    if (lane < (int)(sizeof(EnvHdr) / 8)) dst[lane] = src[lane];
  }
  static constexpr int RPW = (int)(sizeof(RpHdr) / 8);
  static_assert(sizeof(RpHdr) % 8 == 0 && RPW <= 32, "RpHdr: one u64 per lane, 256 LDS bytes");
  static_assert(!RPH || RP || GYM, "an LDS replay header needs the replay / gym context");
  DEV void load() {
    hdr_from_global();
    if constexpr (RPH)
      if (lane < RPW) ((LDSP u64*)rhl)[lane] = ((const u64*)rh_g())[lane];
    for (int hs = 0; hs < HOT; hs++) hotrec[hs * 64 + lane] = agent_ptr(hot_agent(hs))[lane];
    for (int i = lane; i < LATL; i += 64) latl[i] = lat()[i];
    SavedEvent* sq = (SavedEvent*)(env + PC.L.off_q);
    qfree = 0;
    for (int j = 0; j < SQ; j++) {
      int slot = j * 64 + lane;
      SavedEvent e = sq[slot];
      qset(j, e.key, e.seq, true);
      if (PL_LDS)
        for (int i = 0; i < PW; i++) qpl[slot * PW + i] = e.pl[i];
      if (e.key == KEY_EMPTY) qfree |= qm_bit(j);
    }
    q_rescan();
    SavedOrder* so = (SavedOrder*)(env + PC.L.off_book);
    for (int j = 0; j < SO; j++) {
      SavedOrder o = so[j * 64 + lane];
      bp[j] = o.price;
      bq[j] = o.qty;
      bo[j] = o.oid;
      bm[j] = o.meta;
      ba[j] = o.arrival;
      bh[j] = o.hepoch;
      if constexpr (OH) bx[j] = o.pad[0];
    }
  }
  DEV void save() {
    SavedEvent* sq = (SavedEvent*)(env + PC.L.off_q);
    for (int j = 0; j < SQ; j++) {
      int slot = j * 64 + lane;
      SavedEvent e;
      e.key = qkey(j);
      e.seq = qseq(j);
      e.pad = 0;
      // an empty slot saves no payload: its LDS words are whatever the slot last held (or, in a
      // slot never used since the build, LDS contents of an earlier kernel)
      const bool live = e.key != KEY_EMPTY;
      for (int i = 0; i < 8; i++) e.pl[i] = (live && PL_LDS && i < PW) ? qpl[slot * PW + i] : 0u;
      sq[slot] = e;
    }
    SavedOrder* so = (SavedOrder*)(env + PC.L.off_book);
    for (int j = 0; j < SO; j++) {
      SavedOrder o;
      o.price = bp[j];
      o.qty = bq[j];
      o.oid = bo[j];
      o.meta = bm[j];
      o.arrival = ba[j];
      o.hepoch = bh[j];
      o.pad[0] = OH ? bx[OH ? j : 0] : 0;
      o.pad[1] = 0;
      so[j * 64 + lane] = o;
    }
    for (int hs = 0; hs < HOT; hs++) agent_ptr(hot_agent(hs))[lane] = hotrec[hs * 64 + lane];
    if constexpr (RPH) {
      wfence();
      if (lane < RPW) ((u64*)rh_g())[lane] = ((const LDSP u64*)rhl)[lane];
    }
    hdr_to_global();
  }

  // ---------------- Kernel.runner event loop (Kernel.py:190-292)
  // the per-pop bookkeeping of the fast paths: currentTime, parity trace + hash, ttl_messages
  // event class of a pop for the instrumented runs' counters (EnvHdr::kc)
  static DEV int pop_class(u64 key, const Msg& m) {
    const int type = (int)(key & 3);
    return type == MT_MESSAGE ? (int)m_kind(m) : type == MT_WAKEUP ? MK_WAKEUP : MK_KCANCEL;
  }
  DEV void account_pop(i64 t, u64 key, const Msg& m) {
    cur = t;
    if (INSTR && (hash_on || trace)) {  // parity instrumentation (trace ring, per-pop hash, class counters)
      if (lane == 0) h.kc[pop_class(key, m)]++;
      const Rec rec = encode<PW == 8, MD, KSH>(key, m);
      if (hash_on) hash = rec_hash(hash, rec);
      if (trace && h.trace_len < trace_cap) {
        if (lane < 10) trace[h.trace_len * 10 + lane] = rec.at(lane);
        h.trace_len++;
      }
    }
    pops++;
  }

  // ---------------- event runs (zero-latency configurations: rmsc03, rmsc03 + DummyRL)
  // A batched push (TradingAgent.cancelOrders, the POV market maker's 42-order ladder) and the
  // exchange's replies to it leave n events with ONE key (t, recipient, MESSAGE) and
  // consecutive seqs in the queue.  Once the first of them is the queue minimum, the other n-1
  // are the next n-1 pops of Kernel.runner: every event pushed while they are handled takes a
  // later seq, and none takes a smaller key (the exchange replies to recipients > 0 at
  // t + pipeline delay; the acknowledgement handlers push nothing).  Such a run is handled in
  // one pass, member i in lane i, with the per-pop effects of the reference applied in member
  // order; ttl_messages (pops) and the parity hash count every member as its own pop.
  // Handled: CANCEL_ORDER and non-crossing LIMIT_ORDER runs at the exchange, ORDER_ACCEPTED and
  // ORDER_CANCELLED runs at a background TradingAgent.  About 95 % of rmsc03's pops are such
  // members (the market maker's cancel / re-quote cycle every second).
  static constexpr bool RUNS = ACK_FAST && BATCH && PL_LDS;
  // members of the run that starts at (key, s0): lane i gets member i's queue slot (-1 past
  // the run); returns the run length (consecutive seqs from s0 that carry `key`)
  DEV int run_collect(u64 key, u32 s0, int& mslot) {
    scr[lane] = -1;
    __threadfence_block();
    for (int j = 0; j < SQ; j++) {
      const int slot = j * 64 + lane;
      const u32 d = qs_get(slot) - s0;
      if (qk_get(slot) == key && d < 64u) scr[d] = slot;
    }
    __threadfence_block();
    mslot = scr[lane];
    const u64 b = bal(mslot >= 0);
    return ~b == 0 ? 64 : ctz64(~b);
  }
  // the run's n slots leave the queue together (each lane rebuilds its free mask and minimum)
  DEV void q_remove_run(int n, int mslot) {
    if (lane < n) {
      qk_put(mslot, KEY_EMPTY);
      qs_put(mslot, 0xFFFFFFFFu);
    }
    __threadfence_block();
    QM fr = 0;
    for (int j = 0; j < SQ; j++)
      if (qk_get(j * 64 + lane) == KEY_EMPTY) fr |= qm_bit(j);
    qfree = fr;
    q_rescan();
    qcount -= n;
  }
  // per-pop accounting of the members, in member order
  DEV void run_account(u64 key, i64 t, const Msg& mm, int n) {
    if (INSTR && (hash_on || trace)) {
      if (lane == 0) h.kc[MXA_KC_RUN] += n;
      for (int i = 0; i < n; i++) {
        Msg m;
        for (int w = 0; w < 8; w++) m.w[w] = w < PW ? rdl(mm.w[w], i) : 0u;
        account_pop(t, key, m);
      }
    } else {
      cur = t;
      pops += n;
    }
  }
  // OrderBook.cancelOrder for each member in order (OrderBook.py:284-339): the order is found
  // by (side, price, id) and removed; ORDER_CANCELLED with the book's remaining quantity goes
  // to the requester.  Members whose order is gone are silent no-ops.
  // Matching is one LDS bucket per member (order id mod 64): every book slot looks up its id's
  // bucket and checks (id, price, side) against that member, so the cost does not grow with
  // the run.  Ids are unique among live orders, so at most one live slot matches a member;
  // members that share a bucket (ids 64 apart, or one id cancelled twice) take the serial path,
  // which finds the orders member by member exactly as the reference's sequence does.
  DEV void run_ex_cancel(i64 t, const Msg& mm, int n) {
    i32 nq = 0, nm = 0;
    bool found = false;
    const bool mem = lane < n;
    const i32 moid = (i32)mm.w[1], mprice = (i32)mm.w[3];
    const i32 mside = m_buy(mm);
    scr[lane] = -1;
    __threadfence_block();
    if (mem) scr[moid & 63] = lane;
    __threadfence_block();
    const bool coll = mem && scr[moid & 63] != lane;
    if (!bal(coll)) {
      int hit[SO];
      int nfreed = 0;
      for (int j = 0; j < SO; j++) {
        const int c = scr[bo[j] & 63];
        const int cs = c < 0 ? 0 : c;
        const i32 co = __shfl(moid, cs, 64), cp = __shfl(mprice, cs, 64), csd = __shfl(mside, cs, 64);
        hit[j] = (bm[j] >= 0 && c >= 0 && bo[j] == co && bp[j] == cp && (bm[j] & 1) == csd) ? c : -1;
      }
      __threadfence_block();
      scr[lane] = -1;
      __threadfence_block();
      for (int j = 0; j < SO; j++) {
        if (hit[j] >= 0) scr[hit[j]] = j * 64 + lane;  // member -> its book slot
        nfreed += __popcll(bal(hit[j] >= 0));
      }
      __threadfence_block();
      const int s = scr[lane];
      const int sl = s < 0 ? 0 : (s & 63), sj = s < 0 ? 0 : (s >> 6);
      for (int j = 0; j < SO; j++) {
        const i32 q = __shfl(bq[j], sl, 64), mt = __shfl(bm[j], sl, 64);
        nq = sj == j ? q : nq;
        nm = sj == j ? mt : nm;
      }
      found = s >= 0;
      for (int j = 0; j < SO; j++) bm[j] = hit[j] >= 0 ? -1 : bm[j];  // b_free
      h.b_count -= nfreed;
    } else {
      for (int i = 0; i < n; i++) {
        const u32 w0 = rdl(mm.w[0], i);
        const int s = b_find((int)((w0 >> 6) & 1), (i32)rdl(mm.w[3], i), (i32)rdl(mm.w[1], i));
        if (s >= 0) {
          const i32 q = b_get(bq, s), mt = b_get(bm, s);
          b_free(s);
          const bool me = lane == i;
          found = me || found;
          nq = me ? q : nq;
          nm = me ? mt : nm;
        }
      }
    }
    const Msg r = msg_order(MK_CANCELLED, (i32)mm.w[1], nm >> 1, nm & 1, nq, (i32)mm.w[3], 0);
    const u64 rkey = ((u64)(t + PC.ex_pipeline) << KSH) | ((u64)(u32)m_agent(mm) << 2) | MT_MESSAGE;
    q_push_lanes(found, rkey, r);
  }
  // OrderBook.handleLimitOrder for a run of limit orders none of which can match: every buy is
  // below the best ask and every sell above the best bid, counting the run's own earlier
  // orders.  Each valid order (qty > 0) enters the book in member order (the same free slots,
  // arrival stamps and history epoch as one-by-one entry) and gets ORDER_ACCEPTED.
  // run_ex_limit_ok: no member can match and the book has room (else the run is popped one by
  // one, and an overflow fails exactly where the reference's sequence would).
  DEV bool run_ex_limit_ok(const Msg& mm, int n) {
    const bool v = lane < n && (i32)mm.w[2] > 0;
    const int buy = m_buy(mm);
    const i32 price = (i32)mm.w[3];
    const i32 bb = b_best(1), ba = b_best(0);
    const i32 maxb = wmax_i32(v && buy ? price : INT32_MIN);
    const i32 mins = wmin_i32(v && !buy ? price : INT32_MAX);
    const int m = __popcll(bal(v));
    int nfree = 0;
    for (int j = 0; j < SO; j++) nfree += __popcll(bal(bm[j] < 0));
    return maxb < ba && mins > bb && maxb < mins && nfree >= m;
  }
  DEV void run_ex_limit(i64 t, const Msg& mm, int n) {
    const bool v = lane < n && (i32)mm.w[2] > 0;
    const int buy = m_buy(mm);
    const i32 price = (i32)mm.w[3];
    const u64 vb = bal(v);
    const int m = __popcll(vb);
    if (m > 0) {
      const int r = (int)__builtin_amdgcn_mbcnt_hi((u32)(vb >> 32), __builtin_amdgcn_mbcnt_lo((u32)vb, 0u));
      if (v) scr[r] = lane;  // rank -> member lane
      __threadfence_block();
      const i32 agent = m_agent(mm), qty = (i32)mm.w[2], oid = (i32)mm.w[1];
      const i32 meta = (agent << 1) | buy;
      const i32 hep = h.epoch;
      const u32 arr0 = h.arrival;
      i32 oh0 = 0;
      if constexpr (OH) {  // history[0][id] for each member in order (records oh0 + rank)
        oh0 = h.oh_head;
        if (v) {
          OhRec x;
          x.oid = oid;
          x.price = price;
          x.meta = buy;
          x.epoch = hep;
          ohr()[(oh0 + r) % PC.L.oh_cap] = x;
        }
        h.oh_head = oh0 + m;
      }
      int base = 0;
      for (int j = 0; j < SO; j++) {  // the k-th free slot in (j, lane) order takes rank k
        const u64 fb = bal(bm[j] < 0);
        const int fr = base + (int)__builtin_amdgcn_mbcnt_hi((u32)(fb >> 32), __builtin_amdgcn_mbcnt_lo((u32)fb, 0u));
        const bool take = bm[j] < 0 && fr < m;
        const int src = scr[take ? fr : 0];
        const i32 sp = __shfl(price, src, 64), sq = __shfl(qty, src, 64), so = __shfl(oid, src, 64),
                  sm = __shfl(meta, src, 64);
        if (take) {
          bp[j] = sp;
          bq[j] = sq;
          bo[j] = so;
          bm[j] = sm;
          ba[j] = arr0 + (u32)fr;
          bh[j] = hep;
          if constexpr (OH) bx[j] = oh0 + fr;
        }
        base += __popcll(fb);
      }
      h.arrival = arr0 + (u32)m;
      h.b_count += m;
      if (h.b_count > h.max_book) h.max_book = h.b_count;
      LDSP i32* EP = ep_entries();
      const i32 ne = EP[h.epoch & 15] + m;
      if (lane == 0) EP[h.epoch & 15] = ne;
      const Msg a = msg_order(MK_ACCEPTED, oid, agent, buy, qty, price, 0);
      const u64 akey = ((u64)(t + PC.ex_pipeline) << KSH) | ((u64)(u32)agent << 2) | MT_MESSAGE;
      q_push_lanes(v, akey, a);
    }
  }
  // TradingAgent.orderCancelled for each member (TradingAgent.py:464-480): del orders[id]
  // (the same id buckets as run_ex_cancel: each live list entry looks up its id; a shared
  // bucket takes the serial path)
  DEV void run_ta_cancelled(int rcp, i64 t, const Msg& mm, int n, OpenOrder* my) {
    i32 u = rgi(AF_NUSED), nord = rgi(AF_NORD);
    u32 dead = 0;
    const i32 moid = (i32)mm.w[1];
    scr[lane] = -1;
    __threadfence_block();
    if (lane < n) scr[moid & 63] = lane;
    __threadfence_block();
    const bool coll = lane < n && scr[moid & 63] != lane;
    if (!bal(coll)) {
      int nhit = 0;
      for (int j = 0; j < OC; j++) {
        const bool live = j * 64 + lane < u && my[j].oid != -1;
        const int c = scr[my[j].oid & 63];
        const i32 co = __shfl(moid, c < 0 ? 0 : c, 64);
        const bool hit = live && c >= 0 && co == my[j].oid;
        dead |= hit ? (1u << j) : 0u;
        nhit += __popcll(bal(hit));
      }
      nord -= nhit;
      if (nhit > 0 && nord == 0) u = 0;
      n = 0;  // done
    }
    for (int i = 0; i < n; i++) {
      const i32 oid = (i32)rdl(mm.w[1], i);
      for (int j = 0; j < OC; j++) {
        const u64 hit = bal(j * 64 + lane < u && my[j].oid == oid);
        if (hit) {
          const bool me = lane == ctz64(hit);
          my[j].oid = me ? -1 : my[j].oid;
          dead |= me ? (1u << j) : 0u;
          nord--;
          if (nord == 0) u = 0;
          break;
        }
      }
    }
    OpenOrder* oo = open_ptr(rcp);
    for (int j = 0; j < OC; j++)
      if ((dead >> j) & 1) oo[j * 64 + lane].oid = -1;
    rs(AF_NORD, (u32)nord);
    rs(AF_NUSED, (u32)u);
    rs64(AF_ATIME, t);
    rec_store();
  }
  // one run starting at the popped event; returns the pops handled (0: pop it one by one)
  DEV int run_event(u64 key, u32 s0, i64 t, int rcp, u32 kind, i64 budget) {
    int mslot;
    int n = run_collect(key, s0, mslot);
    if (n < 2) return 0;
    const Msg mm = pl_read(mslot >= 0 ? mslot : 0);
    const u64 kb = bal(lane < n && m_kind(mm) == kind);  // same-kind prefix
    n = ~kb == 0 ? 64 : ctz64(~kb);
    if ((i64)n > budget) n = (int)budget;
    if (n < 2) return 0;
    if (rcp == 0) {
      cur_agent = 0;
      rlo = rhi = 0;
      if (kind == MK_LIMIT) {
        if (!run_ex_limit_ok(mm, n)) {
          run_skip = s0 + (u32)n;
          return 0;
        }
      }
      run_account(key, t, mm, n);
      q_remove_run(n, mslot);
      if (kind == MK_CANCEL) run_ex_cancel(t, mm, n);
      else run_ex_limit(t, mm, n);
      atime_store(0, t);
      return n;
    }
    if (kind == MK_CANCELLED) {
      rec_load(rcp);
      OpenOrder my[OC];
      const OpenOrder* oo = open_ptr(rcp);
      for (int j = 0; j < OC; j++) {
        my[j].oid = -1;
        if (j * 64 + lane < PC.L.open_cap) my[j] = oo[j * 64 + lane];
      }
      run_account(key, t, mm, n);
      q_remove_run(n, mslot);
      run_ta_cancelled(rcp, t, mm, n, my);
      return n;
    }
    run_account(key, t, mm, n);  // ORDER_ACCEPTED: agentCurrentTimes only (see ACK_FAST)
    q_remove_run(n, mslot);
    atime_store(rcp, t);
    return n;
  }
  DEV void run(i64 max_pops) {
    if constexpr (BLOG && EXT) {  // f_log's opening entry (kept by the build in o_pt / o_pv)
      if (pops == 0 && h.blog_n == 0 && h.o_pt >= 0) efo_log(h.o_pt, h.o_pv);
    }
    for (i64 n = 0; n < max_pops && status == ST_RUNNING; n++) {
      if constexpr (GYM) {
        if (end_step) break;  // GymKernel.stepRunner: `while not end_step and ...`
      }
      {  // opaque per event: env-derived addresses are recomputed, not pinned in SGPRs by LICM
         // (without this the event loop hoists ~1000 SGPRs of addresses and spills them)
        u64 pv = (u64)env;
        u32 plo = (u32)__builtin_amdgcn_readfirstlane((int)(u32)pv);
        u32 phi = (u32)__builtin_amdgcn_readfirstlane((int)(u32)(pv >> 32));
        asm volatile("" : "+s"(plo), "+s"(phi));
        env = (EnvPtr)(GLBP char*)(((u64)phi << 32) | plo);
        // lane-derived masks (lane == field/2 ...) are rebuilt per use, not hoisted
        asm volatile("" : "+v"(lane));
      }
      PROF_T(t0);
      u64 key;
      u32 eseq;
      int slot = q_peek(key, eseq);
      if (slot < 0 || !(cur <= stop_t)) {
        status = ST_DONE;
        break;
      }
      i64 t = (i64)(key >> KSH);
      int rcp = (int)((key >> 2) & KRCP);
      int type = (int)(key & 3);
      // payload in HBM: the recipient's record is loaded beside it, one round trip for both
      // instead of payload -> fast-path test -> record (the record of an acknowledgement that
      // takes a fast path is loaded for nothing: 512 B, no latency)
      u64 rv_early = 0;
      if constexpr (EARLY_REC) {
        if (rcp != 0) rv_early = rec_fetch(rcp);
      }
      Msg m = pl_read(slot);
      if constexpr (EARLY_REC) asm volatile("" ::"v"(rv_early));
      if constexpr (RUNS) {
        // a run past stopTime is not batched: the loop stops after its first member
        if (type == MT_MESSAGE && (m.w[0] & MF_RUN) && t <= stop_t && eseq >= run_skip) {
          const u32 k = m_kind(m);
          const bool exr = rcp == 0 && (k == MK_CANCEL || k == MK_LIMIT) && !(t > PC.mkt_close) && !BLOG && !MD;
          const bool ackr = rcp > 0 && rcp < ACK_LIMIT && (k == MK_ACCEPTED || k == MK_CANCELLED);
          if (exr || ackr) {
            PROF_ADD(0, t0);
            const int nr = run_event(key, eseq, t, rcp, k, max_pops - n);
            if (nr > 0) {
#ifdef MXA_PROF
              const int kx = rcp == 0 ? (k == MK_CANCEL ? 0 : 1) : (k == MK_ACCEPTED ? 2 : 3);
              PROF_ADD(34 + kx, t0);
              PROF_CNT(38 + kx);
              if (lane == 0) prof[42 + kx] += nr;
#endif
              n += nr - 1;
              continue;
            }
            PROF_ADD(46, t0);  // run detection that fell back to single pops
          }
        }
      }
      if constexpr (ACK_FAST || RP_FAST) {
        if (type == MT_MESSAGE && rcp == 0) {
          // ExchangeAgent.receiveMessage reads nothing from its agent record but the
          // computation delay, which is 0 here: no record round trip (half of all pops)
          cur_agent = 0;
          rlo = rhi = 0;
          PROF_ADD(0, t0);
          account_pop(t, key, m);
          PROF_ADD(32, t0);
          q_remove(slot);
          PROF_ADD(33, t0);
          ex_receive(m);
#ifdef MXA_PROF
          {  // by request kind: 48 SPREAD_REQ, 49 TV_REQ, 50 LIMIT, 51 CANCEL, 52 other (counts +8)
            const u32 kk = m_kind(m);
            const int eb = kk == MK_SPREAD_REQ ? 48 : kk == MK_TV_REQ ? 49 : kk == MK_LIMIT ? 50 : kk == MK_CANCEL ? 51 : 52;
            PROF_ADD(eb, t0);
            PROF_CNT(eb + 8);
          }
#endif
          if (dirty) rng_maint();
          PROF_ADD(30, t0);
          atime_store(0, t);
          PROF_ADD(31, t0);
          continue;
        }
        // ORDER_ACCEPTED, and ORDER_MODIFIED, which no agent of the reference handles (only
        // util/OrderBook.py sends it; TradingAgent.receiveMessage has no branch for it): the
        // whole effect is agentCurrentTimes[a] = t
        if (type == MT_MESSAGE && (m_kind(m) == MK_ACCEPTED || m_kind(m) == MK_MODIFIED) && rcp > 0 && rcp < ACK_LIMIT) {
          PROF_ADD(0, t0);
          account_pop(t, key, m);
          PROF_ADD(32, t0);
          q_remove(slot);
          PROF_ADD(33, t0);
          atime_store(rcp, t);
          PROF_ADD(14, t0);
          PROF_CNT(28);
          continue;
        }
        if (ACK_FAST && type == MT_MESSAGE && m_kind(m) == MK_CANCELLED && rcp > 0 && rcp < ACK_LIMIT) {
          // TradingAgent.orderCancelled (TradingAgent.py:464-480): del self.orders[id]. The
          // open-order chunks are loaded with the record, not after it (one latency, not two)
          if constexpr (EARLY_REC) rec_set(rcp, rv_early);
          else rec_load(rcp);
          OpenOrder my[OC];
          {
            const OpenOrder* oo = open_ptr(rcp);
            for (int j = 0; j < OC; j++) {
              my[j].oid = -1;
              if (j * 64 + lane < PC.L.open_cap) my[j] = oo[j * 64 + lane];
            }
          }
          PROF_ADD(0, t0);
          account_pop(t, key, m);
          PROF_ADD(32, t0);
          q_remove(slot);
          PROF_ADD(33, t0);
          const i32 u = rgi(AF_NUSED), oid = (i32)m.w[1];
          for (int j = 0; j < OC; j++) {
            const u64 hit = bal(j * 64 + lane < u && my[j].oid == oid);
            if (hit) {
              del_open(j * 64 + ctz64(hit));
              break;
            }
          }
          rs64(AF_ATIME, t);
          rec_store();
          PROF_ADD(15, t0);
          PROF_CNT(29);
          continue;
        }
      }
      PROF_ADD(0, t0);
      // (the exchange's record is not fetched early: its messages take the fast path)
      if constexpr (EARLY_REC) {
        if (rcp != 0) rec_set(rcp, rv_early);
        else rec_load(rcp);
      } else {
        rec_load(rcp);  // issued before the trace encode/hash so its latency overlaps them
      }
      cur = t;
      if (INSTR && (hash_on || trace)) {
        if (lane == 0) h.kc[pop_class(key, m)]++;
        const Rec rec = encode<PW == 8, MD, KSH>(key, m);
        if (hash_on) hash = rec_hash(hash, rec);
        if (trace && h.trace_len < trace_cap) {
          if (lane < 10) trace[h.trace_len * 10 + lane] = rec.at(lane);
          h.trace_len++;
        }
      }
      pops++;
      PROF_ADD(32, t0);
      add_delay = 0;
      if constexpr (GYM) {
        if (type == MT_CANCEL_ORDER) {  // GymKernel CANCEL_ORDER: no busy check, no delay
          q_remove(slot);
          rl_kernel_cancel();
          if (dirty) rng_maint();
          continue;
        }
      }
      i64 at = rg64(AF_ATIME);
      PROF_ADD(0, t0);
      if (at > t) {  // agent in the future: requeue unchanged (same uniq)
        q_rekey(slot, ((u64)at << KSH) | (key & ((1ull << KSH) - 1)));
        if (INSTR && (hash_on || trace) && lane == 0) h.kc[MXA_KC_REQUEUE]++;
        PROF_ADD(1, t0);
        continue;
      }
      PROF_ADD(0, t0);
      q_remove(slot);
      PROF_ADD(33, t0);
      rs64(AF_ATIME, t);
#ifdef MXA_PROF
      int pb = 2 + 2 * (rgi(AF_TYPE) & 7) + (type == MT_WAKEUP), pc = pb + 14;
      if (type == MT_MESSAGE && m_kind(m) == MK_SPREAD && rgi(AF_TYPE) == AG_VALUE) pb = 53, pc = 61;
      if (type == MT_MESSAGE && m_kind(m) == MK_SPREAD && rgi(AF_TYPE) == AG_POVMM) pb = 54, pc = 62;
      if (type == MT_MESSAGE && m_kind(m) == MK_TV) pb = 55, pc = 63;
      if (type == MT_MESSAGE && rcp == 0) {  // the exchange by request kind (as the fast path)
        const u32 kk = m_kind(m);
        pb = kk == MK_SPREAD_REQ ? 48 : kk == MK_TV_REQ ? 49 : kk == MK_LIMIT ? 50 : kk == MK_CANCEL ? 51 : 52;
        pc = pb + 8;
      }
      if constexpr (RP) {  // replay: 92 / 93 MarketReplayAgent message / wakeup, 94 / 95 the RL agent's (counts +32)
        const int at = rgi(AF_TYPE);
        if (at == AG_REPLAY || at == AG_DUMMYRL) {
          pb = 92 + 2 * (at == AG_DUMMYRL) + (type == MT_WAKEUP);
          pc = pb + 32;
        }
      }
      if (type == MT_MESSAGE && rgi(AF_TYPE) == AG_ZI) {  // ZI messages: 80 SPREAD, 81 ACCEPTED, 82 EXECUTED, 83 other
        const u32 kk = m_kind(m);
        pb = kk == MK_SPREAD ? 80 : kk == MK_ACCEPTED ? 81 : kk == MK_EXECUTED ? 82 : 83;
        pc = pb + 32;
      }
#endif
      dispatch(rgi(AF_TYPE), type == MT_WAKEUP, m);
      PROF_ADD(pb, t0);
      PROF_CNT(pc);
      if (dirty) rng_maint();
      PROF_ADD(30, t0);
      rs64(AF_ATIME, t + rg64(AF_COMP) + add_delay);
      rec_store();
      PROF_ADD(31, t0);
    }
  }
};

// ------------------------------------------------------------------------------------
// env construction (config scripts' global-RNG draw order)
// ------------------------------------------------------------------------------------
template <int CFG>
struct Builder : Eng<CFG, true> {
  typedef Eng<CFG, true> E;
  typedef typename E::RS RS;
  DEV Builder(char* e, char* lds, const RpCtx* ctx = nullptr) : E(e, lds, 0, ctx) {}
  const MmParams* mmp = nullptr;  // MXA_CFG_RMSC03_MM: this env's market-maker options

  DEV u32 g_seed(RS& G) { return (u32)rs_randint(G, 0, 4294967296LL); }
  DEV void set_seed(int stream, u32 s) {
    if (this->lane == 0) this->rng_key(stream)[0] = s;
  }
  DEV void rec_init(int a, int type) {
    this->rlo = this->rhi = 0;
    this->cur_agent = a;
    this->rs(AF_TYPE, (u32)type);
    this->rs(AF_FLAGS, FL_FIRST_WAKE | FL_AW_SPREAD | FL_AW_TV);
    this->rs(AF_RS_POS, MXA_MT_N);
    this->rs(AF_RS_M, 0);
    const i64 cash = type == AG_VALUE ? E::PC.v_starting_cash : E::PC.starting_cash;
    this->rs64(AF_START_CASH, cash);
    this->rs64(AF_CASH, cash);
    this->rs64(AF_ATIME, E::PC.start);
    this->rs64(AF_COMP, E::PC.default_comp_delay);
  }
  DEV i64 get_wake_time(RS& G, i64 open, i64 close) { return wake_time_of(rs_double(G), open, close); }
  // the noise agents' wakeup times from their uniforms (kept in AF_WAKEUP_TIME by the draw loop),
  // lane = agent: the same glibc pow restatement per lane
  DEV void wake_times_lanes() {
    const MxaParams& P = E::PC;
    wfence();
    for (int a0 = P.first_noise; a0 < P.first_noise + P.n_noise; a0 += 64) {
      const int a = a0 + this->lane;
      if (a < P.first_noise + P.n_noise) {
        u32* rw = (u32*)this->agent_ptr(a);
        const double u = as_d(((u64)rw[AF_WAKEUP_TIME + 1] << 32) | rw[AF_WAKEUP_TIME]);
        const u64 wt = (u64)wake_time_of(u, P.noise_open, P.noise_close);
        rw[AF_WAKEUP_TIME] = (u32)wt;
        rw[AF_WAKEUP_TIME + 1] = (u32)(wt >> 32);
      }
    }
    wfence();
  }
  DEV i64 wake_time_of(double u, i64 open, i64 close) {  // util/util.py:35-58
    double alpha = 12.0, beta = 0.5;
    double n = (3 / alpha) * u - gm_pow(beta - 0, 3.0);
    double c = n < 0 ? -gm_pow(-n, 1.0 / 3.0) : gm_pow(n, 1.0 / 3.0);
    double mult = c + beta;
    return open + (i64)(mult * (double)(close - open));
  }
  // expand every stream's init_genrand in parallel (lane = stream).  With room in the LDS queue
  // area (empty until the kernelStarting wakeups) each lane's 16-word runs go through an LDS tile
  // and leave as 64-byte runs of 4 streams per store instead of 64 scattered dwords.
  static constexpr bool SEED_TILE = MXA_SEED_TILE && E::LDS_Q >= 64 * 17 * 4;
  DEV void seed_streams(int first) {
    const MxaParams& P = E::PC;
    wfence();
    const int lane = this->lane;
    for (int b = first; b < P.n_streams; b += 64) {
      int s = b + lane;
      if constexpr (SEED_TILE) {
        LDSP u32* tile = (LDSP u32*)this->qk;  // [64 streams][17] (16 words + a bank-conflict pad)
        u32 x = s < P.n_streams ? this->rng_key(s)[0] : 0u;
        for (int i0 = 1; i0 < MXA_MT_N; i0 += 16) {
#pragma unroll
          for (int j = 0; j < 16; j++) {
            x = 1812433253u * (x ^ (x >> 30)) + (u32)(i0 + j);
            tile[lane * 17 + j] = x;
          }
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int t = 0; t < 16; t++) {  // 4 streams x 16 words per store
            const int st = 4 * t + (lane >> 4), w = lane & 15;
            if (b + st < P.n_streams && i0 + w < MXA_MT_N) this->rng_key(b + st)[i0 + w] = tile[st * 17 + w];
          }
          __builtin_amdgcn_wave_barrier();
        }
      } else if (s < P.n_streams) {
        u32* key = this->rng_key(s);
        u32 x = key[0];
        for (int i = 1; i < MXA_MT_N; i++) {
          x = 1812433253u * (x ^ (x >> 30)) + (u32)i;
          key[i] = x;
        }
      }
    }
    wfence();
    if constexpr (SEED_TILE) {  // the queue area again: every slot empty
      for (int j = 0; j < E::SQ; j++) this->qset(j, KEY_EMPTY, 0xFFFFFFFFu, true);
      if constexpr (E::QHIER) this->q_rescan();
    }
  }

  // rs_maint(agent stream, MXA_AGENT_LA) for every agent without a record round trip each: 64
  // records' stream position and block per load, the blocks two streams per round trip, the
  // block numbers written back per lane (the builder's records are all in HBM: HOT is 0)
  DEV void maint_agents() {
    const int n = E::PC.n_agents, lane = this->lane;
    wfence();  // the records' stores above
    for (int a0 = 0; a0 < n; a0 += 64) {
      const int a = a0 + lane;
      const bool act = a < n;
      u32* rw = (u32*)this->agent_ptr(act ? a : a0);
      const i32 p = act ? (i32)rw[AF_RS_POS] : 0;
      i32 m = act ? (i32)rw[AF_RS_M] : 0;
      const i32 need = (p + MXA_AGENT_LA) / MXA_MT_N;
      for (;;) {
        u64 t = bal(act && m < need);
        if (!t) break;
        const int l1 = ctz64(t);
        t &= t - 1;
        const int l2 = t ? ctz64(t) : l1;
        const int m1 = rdl((u32)m, l1), m2 = rdl((u32)m, l2);
        mt_gen_pair(this->rng_key(4 + a0 + l1), m1 + 1, this->rng_key(4 + a0 + l2), m2 + 1, l2 != l1);
        m += (lane == l1 || lane == l2) ? 1 : 0;
      }
      if (act) rw[AF_RS_M] = (u32)m;
    }
    wfence();
  }

  // The ZI / HBL agents' theta (ZeroIntelligenceAgent.py:65-71: sorted(np.round(random_state.normal(
  // 0, sqrt(sigma_pv), 2 q_max)), reverse=True)), 64 agents at once: lane L runs agent a0 + L's
  // polar normals on its own stream (numpy legacy_gauss: pairs of doubles from 4 words, the second
  // normal cached), sorts them and writes the agent's record fields.  Every stream is fresh here
  // (p = 624, block 1 materialized just before); a lane whose draws would leave block 1 leaves its
  // agent untouched and flags it for the one-agent-at-a-time path below (never in practice: 2 q_max
  // normals take ~6 q_max words of the 624).
  u64 zi_fb[(E::PC.n_zi + E::PC.n_hbl + 63) / 64 + 1];
  DEV bool zi_fallback(int a) {
    const int i = a - E::PC.first_zi;
    return (zi_fb[i >> 6] >> (i & 63)) & 1;
  }
  DEV void zi_theta_lanes() {
    const MxaParams& P = E::PC;
    constexpr int NQ = 2 * E::PC.zi_qmax;
    static_assert(NQ <= 20, "theta fits the agent record");
    const int lo = P.first_zi, hi = P.first_zi + P.n_zi + P.n_hbl;
    const double sd = __builtin_sqrt(P.zi_sigma_pv);
    const int lane = this->lane;
    for (int a0 = lo; a0 < hi; a0 += 64) {
      for (int j = 0; j < 64 && a0 + j < hi; j += 2)
        mt_gen_pair(this->rng_key(4 + a0 + j), 1, this->rng_key(4 + a0 + j + 1), 1, a0 + j + 1 < hi);
      const int a = a0 + lane;
      const bool act = a < hi;
      const u32* key = this->rng_key(4 + (act ? a : a0));
      i32 p = MXA_MT_N;
      bool cached = false, fb = false;
      double cache = 0.0;
      double th[NQ];
#pragma unroll
      for (int i = 0; i < NQ; i++) th[i] = 0.0;
      int k = 0;
      while (bal(act && !fb && k < NQ)) {
        if (act && !fb && k < NQ) {
          double z = 0.0;
          bool out = false;
          if (cached) {
            z = cache;
            cached = false;
            cache = 0.0;
            out = true;
          } else if (p + 4 > 2 * MXA_MT_N) {
            fb = true;
          } else {
            u32 w[4];
#pragma unroll
            for (int t = 0; t < 4; t++) {
              u32 y = key[p + t];  // block 1 holds words 624..1247 at key[624..1247]
              y ^= (y >> 11);
              y ^= (y << 7) & 0x9d2c5680u;
              y ^= (y << 15) & 0xefc60000u;
              y ^= (y >> 18);
              w[t] = y;
            }
            p += 4;
            const double d1 = ((double)(i32)(w[0] >> 5) * 67108864.0 + (double)(i32)(w[1] >> 6)) / 9007199254740992.0;
            const double d2 = ((double)(i32)(w[2] >> 5) * 67108864.0 + (double)(i32)(w[3] >> 6)) / 9007199254740992.0;
            const double x1 = 2.0 * d1 - 1.0, x2 = 2.0 * d2 - 1.0;
            const double r2 = x1 * x1 + x2 * x2;
            if (!(r2 >= 1.0 || r2 == 0.0)) {
              const double f = __builtin_sqrt(-2.0 * gm_log(r2) / r2);
              cache = f * x1;
              cached = true;
              z = f * x2;
              out = true;
            }
          }
          if (out) {
            const double v = __builtin_rint(0 + sd * z);
#pragma unroll
            for (int i = 0; i < NQ; i++) th[i] = i == k ? v : th[i];
            k++;
          }
        }
      }
      // descending (sorted(..., reverse=True)); equal values are equal doubles, so order among
      // them is invisible
#pragma unroll
      for (int i = 0; i < NQ; i++)
#pragma unroll
        for (int j = 0; j + 1 < NQ - i; j++) {
          const double x = th[j], y = th[j + 1];
          th[j] = x < y ? y : x;
          th[j + 1] = x < y ? x : y;
        }
      if (act && !fb) {
        u32* rw = (u32*)this->agent_ptr(a);
#pragma unroll
        for (int i = 0; i < NQ; i++) rw[AF_THETA + i] = (u32)(i32)th[i];
        rw[AF_RS_POS] = (u32)p;
        rw[AF_RS_M] = 1u;
        rw[AF_RS_HASG] = cached ? 1u : 0u;
        const u64 gb = as_u(cached ? cache : 0.0);
        rw[AF_RS_GAUSS] = (u32)gb;
        rw[AF_RS_GAUSS + 1] = (u32)(gb >> 32);
      }
      zi_fb[(a0 - lo) >> 6] = bal(act && fb);
    }
    wfence();
  }

  // GymKernel-side state of the DummyRL agent: ABIDESEnvMetrics deque, trade flag, quantities
  DEV void init_gym() {
    RpLob* rg = this->ring();
    for (int i = this->lane; i < 100; i += 64) {
      RpLob z;
      z.bid = z.ask = z.data = z.flags = 0;
      rg[i] = z;
    }
    u32* rw = (u32*)this->rh();
    for (int i = this->lane; i < (int)(sizeof(RpHdr) / 4); i += 64) rw[i] = 0;
    __threadfence_block();
    RpHdr* R = this->rh();
    R->rl_trade = 1;
    R->rl_rem = E::PC.rl_quantity;
    R->ex_has_last = 1;
    __threadfence_block();
  }

  // ABIDESEnv.reset (ABIDESEnv.py:51-103): agents, empty ladder book, kernelStarting wakeups.
  // No RNG stream is ever drawn in this composition.
  DEV void build_replay(i32 id_base, i32 tape_hi) {
    const MxaParams& P = E::PC;
    const __attribute__((address_space(4))) RpLayout& L = this->rx->L;
    const i32 Pn = U(L.P), C = U(L.C), D = U(L.D);
    for (int s = 0; s < 2; s++) {
      i32 *c = this->lv_cnt(s), *hd = this->lv_head(s), *tl = this->lv_tail(s);
      i64* q = this->lv_qty(s);
      for (i32 i = this->lane; i < Pn; i += 64) {
        c[i] = 0;
        hd[i] = -1;
        tl[i] = -1;
        q[i] = 0;
      }
    }
    i32* fr = this->freel();
    for (i32 i = this->lane; i < C; i += 64) fr[i] = C - 1 - i;
    i32 *ih = this->idh(), *ie = this->idep();
    RpOrder* mo = this->mro();
    for (i32 i = this->lane; i < D; i += 64) {
      ih[i] = -1;
      for (int k = 0; k < MXA_ID_EPOCHS; k++) ie[MXA_ID_EPOCHS * i + k] = INT32_MIN;
      RpOrder z;
      z.qty = z.price = z.is_buy = z.present = 0;
      mo[i] = z;
    }
    init_gym();
    RpHdr* R = this->rh();
    R->id_base = id_base;
    R->tape_hi = tape_hi;
    R->mr_done = 0;
    R->best[0] = R->best[1] = -1;
    R->free_top = C;
    R->ex_has_last = 0;  // no oracle: getDailyOpenPrice raises, last_trade stays None
    rec_init(0, AG_EXCHANGE);
    this->rs64(AF_COMP, P.default_comp_delay);
    this->rec_store();
    rec_init(P.first_replay, AG_REPLAY);
    this->rec_store();
    if constexpr (E::PC.n_rl > 0) {
      rec_init(P.first_rl, AG_DUMMYRL);
      this->rec_store();
    }
    if constexpr (E::PC.n_twap > 0) {  // TWAP_EXECUTION_AGENT: trades only with -e
      rec_init(P.first_twap, AG_TWAP);
      this->rec_store();
      R->rl_trade = U(this->rx->twap_trade);
    }
    this->h.last_trade = 0;
    this->h.last_trade_float = 0;
    this->cur = P.start;
    for (int a = 0; a < P.n_agents; a++) this->wakeup_at(a, P.start);
    count_base();
    this->save();
    __threadfence_block();
  }
  // counter baselines (EnvHdr::q0, rng0): what the build itself pushed and drew
  DEV void count_base() {
    const MxaParams& P = E::PC;
    wfence();
    u64 w = 0;
    for (int a = this->lane; a < P.n_agents; a += 64)
      w += (u64)(((const u32*)(this->env + P.L.off_ag + (size_t)a * 512))[AF_RS_POS] - MXA_MT_N);
    w = (u64)wsum_i64((i64)w);
    for (int k = 0; k < 4; k++) w += (u64)(this->h.rs_pos[k] - MXA_MT_N);
    this->h.q0 = this->qcount;
    this->h.rng0 = w;
  }

  // keep_ids: ABIDESEnv.reset in the same process (Order.order_id / _order_ids carry over)
  DEV void build(u32 seed, bool keep_ids = false) {
    const MxaParams& P = E::PC;
    LDSP EnvHdr& h = this->h;
    i64 ocnt0 = 0;
    i32 tape_hi0 = 0;
    if (keep_ids) {  // the previous episode's counters, before anything is rebuilt
      ocnt0 = U(((const EnvHdr*)this->env)->order_counter);
      if constexpr (E::RP) {
        const RpHdr* R = this->rh();
        tape_hi0 = max(U(R->tape_hi), U(R->mr_done));
      }
    }
    {
      LDSP u32* hw = (LDSP u32*)&h;
      for (int i = this->lane; i < (int)(sizeof(EnvHdr) / 4); i += 64) hw[i] = 0;
      wfence();
    }
    this->hash = FNV_OFF;
    this->status = ST_RUNNING;
    this->err = 0;
    this->pops = 0;
    this->ocnt = ocnt0;
    this->seq = 0;
    this->qcount = 0;
    this->cur = P.start;
    for (int s = 0; s < 4; s++) {
      h.rs_pos[s] = MXA_MT_N;
      h.rs_m[s] = 0;
    }
    this->mk = KEY_EMPTY;
    this->ms = 0xFFFFFFFFu;
    this->mj = -1;
    typedef typename E::QM QM;
    this->qfree = E::SQ >= (int)(8 * sizeof(QM)) ? ~(QM)0 : (((QM)1 << E::SQ) - 1);
    for (int j = 0; j < E::SQ; j++) {
      this->qset(j, KEY_EMPTY, 0xFFFFFFFFu, true);
    }
    if constexpr (E::QHIER) this->q_rescan();  // empty group mins
    for (int j = 0; j < E::SO; j++) {  // every field: a slot never used is saved as the build left it
      this->bm[j] = -1;
      this->bp[j] = 0;
      this->bq[j] = 0;
      this->bo[j] = 0;
      this->ba[j] = 0;
      this->bh[j] = 0;
      if constexpr (E::OH) this->bx[j] = 0;
    }
    if constexpr (E::RP) {
      build_replay((i32)ocnt0, tape_hi0);
      return;
    }
    mt_seed(this->rng_key(0), seed);
    RS G = this->grs(0);
    int n = P.n_agents;
    u32 tmp;
    if (P.config == MXA_CFG_RMSC03 || P.config == MXA_CFG_RMSC03_MM || P.config == MXA_CFG_RMSC03_RL ||
        P.config == MXA_CFG_RANDOM_FUND_VALUE ||
        P.config == MXA_CFG_RMSC03_SBMM || P.config == MXA_CFG_RMSC03_SBMM_POLL ||
        P.config == MXA_CFG_RANDOM_FUND_DIVERSE || P.config == MXA_CFG_HIST_FUND_VALUE ||
        P.config == MXA_CFG_HIST_FUND_DIVERSE) {
      // config/rmsc03.py, config/random_fund_value.py and config/random_fund_diverse.py: the same
      // global-draw order (random_fund_diverse's MarketMakerAgent seed after the value agents);
      // config/hist_fund_*.py draw the oracle's RandomState seed too, but ExternalFileOracle
      // draws nothing at construction
      set_seed(1, g_seed(G));  // O
      if constexpr (!E::EXT) {
        h.o_pt = P.mkt_open;
        h.o_pv = P.o_rbar;
        h.o_th2 = gm_pow(P.o_fundvol, 2.0);  // SMRO: theta ** 2 (SparseMeanRevertingOracle.py:105)
        h.o_mst = P.mkt_open + (i64)rs_exponential(G, 1.0 / P.o_lambda);
      }
      tmp = g_seed(G);  // exchange
      set_seed(4 + 0, tmp);
      for (int a = P.first_noise; a < P.first_noise + P.n_noise; a++) {
        // get_wake_time's uniform now; its math for 64 agents at once below (wake_times_lanes)
        const double u = rs_double(G);
        set_seed(4 + a, g_seed(G));
        i64 size = rs_randint(G, 20, 50);
        rec_init(a, AG_NOISE);
        if constexpr (MXA_WAKE_LANES) this->rsd(AF_WAKEUP_TIME, u);
        else this->rs64(AF_WAKEUP_TIME, wake_time_of(u, P.noise_open, P.noise_close));
        this->rs(AF_SIZE, (u32)size);
        this->rec_store();
      }
      if constexpr (MXA_WAKE_LANES) wake_times_lanes();
      for (int a = P.first_value; a < P.first_value + P.n_value; a++) {
        set_seed(4 + a, g_seed(G));
        i64 size = rs_randint(G, 20, 50);
        rec_init(a, AG_VALUE);
        this->rs(AF_SIZE, (u32)size);
        this->rsd(AF_R_T, this->v_rbar());
        this->rec_store();
      }
      for (int a = P.first_mm; a < P.first_mm + P.n_mm; a++) {
        set_seed(4 + a, g_seed(G));
        rec_init(a, AG_POVMM);
        if constexpr (P.mm_rt) {  // this env's --mm-* options (POVMarketMakerAgent.py:19-60)
          const MmParams mp = *mmp;
          this->rsd(AF_MM_POV, mp.pov);
          this->rs(AF_MM_MIN, (u32)mp.min_order_size);
          this->rs(AF_MM_WIN, (u32)mp.window_size);
          this->rs(AF_MM_TICKS, (u32)mp.num_ticks);
          this->rs64(AF_MM_WAKE, mp.wake_up_freq);
          this->rs(AF_ORDER_SIZE, (u32)mp.min_order_size);  // order_size = min_order_size
        } else {
          this->rs(AF_ORDER_SIZE, (u32)P.mm_min_size);
        }
        this->rec_store();
      }
      for (int a = P.first_sb; a < P.first_sb + P.n_sb; a++) {  // rmsc03_sbmm*: the market maker's slot and draw
        set_seed(4 + a, g_seed(G));
        rec_init(a, AG_SBMM);
        this->rec_store();
      }
      for (int a = P.first_mk; a < P.first_mk + P.n_mk; a++) {  // random_fund_diverse
        set_seed(4 + a, g_seed(G));
        rec_init(a, AG_MKTMAKER);
        this->rec_store();
      }
      for (int a = P.first_mom; a < P.first_mom + P.n_mom; a++) {
        set_seed(4 + a, g_seed(G));
        rec_init(a, AG_MOMENTUM);
        this->rec_store();
      }
      if constexpr (E::GYM) {  // DummyRLExecutionAgent 64: constructed after the config, draws nothing
        rec_init(P.first_rl, AG_DUMMYRL);
        this->rs64(AF_START_CASH, 0);  // starting_cash=0 (agent_config.py:115-137)
        this->rs64(AF_CASH, 0);
        this->rec_store();
        init_gym();
      }
      set_seed(2, g_seed(G));  // K
    } else if (P.config == MXA_CFG_RMSC01 || P.config == MXA_CFG_RMSC02 || P.config == MXA_CFG_OBI_RMSC02) {
      // config/rmsc01.py: the exchange's seed, the market maker's, the oracle symbol's, the
      // oracle's first megashock time, per ZI and HBL agent its seed, per momentum agent its
      // seed, the kernel's (each agent's own __init__ draws come after seed_streams);
      // config/rmsc02.py then draws the 101 x 101 latency matrix
      set_seed(4 + 0, g_seed(G));  // exchange
      for (int a = P.first_mk; a < P.first_mk + P.n_mk; a++) {
        set_seed(4 + a, g_seed(G));
        rec_init(a, AG_MKTMAKER);
        this->rec_store();
      }
      set_seed(1, g_seed(G));  // O
      h.o_pt = P.mkt_open;
      h.o_pv = P.o_rbar;
      h.o_th2 = gm_pow(P.o_fundvol, 2.0);  // SMRO: theta ** 2 (SparseMeanRevertingOracle.py:105)
      h.o_mst = P.mkt_open + (i64)rs_exponential(G, 1.0 / P.o_lambda);
      for (int a = P.first_zi; a < P.first_zi + P.n_zi + P.n_hbl; a++) {  // ZI, then HBL (ids follow)
        set_seed(4 + a, g_seed(G));
        rec_init(a, a < P.first_zi + P.n_zi ? AG_ZI : AG_HBL);
        this->rs(AF_GROUP, 0u);
        this->rsd(AF_R_T, P.zi_rbar);
        this->rec_store();
      }
      for (int a = P.first_obi; a < P.first_obi + P.n_obi; a++) {  // obi_rmsc02: after the ZI agents
        set_seed(4 + a, g_seed(G));
        rec_init(a, AG_OBI);
        this->rsd(AF_OBI_STOP, 0.0);
        this->rec_store();
      }
      for (int a = P.first_mom; a < P.first_mom + P.n_mom; a++) {
        set_seed(4 + a, g_seed(G));
        rec_init(a, AG_MOMENTUM);
        this->rec_store();
      }
      set_seed(2, g_seed(G));  // K
      if (P.config == MXA_CFG_RMSC02 || P.config == MXA_CFG_OBI_RMSC02) {  // G.uniform(lo, hi, (n, n)), C order: row 0, then column 0
        double* lat = this->lat();
        const i64 total = (i64)n * n;
        i64 prev = -1;
        for (i64 k = 0; k < 2 * (i64)n - 1; k++) {
          const i64 d = k < n ? k : (k - n + 1) * (i64)n;
          rs_skip_words(G, 2 * (d - prev - 1));
          const double v = rs_uniform(G, P.lat_lo, P.lat_hi);
          if (this->lane == 0) {
            if (d < n) lat[d] = v;        // latency[0][d]: exchange -> agent d
            if (d % n == 0) lat[n + d / n] = v;  // latency[d / n][0]: agent -> exchange
          }
          prev = d;
        }
        rs_skip_words(G, 2 * (total - prev - 1));
        wfence();
      }
      if constexpr (E::OH) {  // the HBL price histogram starts (and stays) zeroed
        u64* hist = (u64*)(this->env + P.L.off_hh);
        for (int i = this->lane; i < P.L.hbl_range; i += 64) hist[i] = 0;
      }
    } else if (P.config == MXA_CFG_VALUE_NOISE) {
      // config/value_noise.py: O and K seeds (the kernel is built before the oracle), the
      // oracle's first megashock time, the exchange; per noise agent its seed, its wakeup_time
      // open + rand() * (close - open) (pandas float * Timedelta truncates), NoiseAgent's size;
      // per value agent its seed and size; then the 151 x 151 latency matrix
      set_seed(1, g_seed(G));  // O
      set_seed(2, g_seed(G));  // K
      h.o_pt = P.mkt_open;
      h.o_pv = P.o_rbar;
      h.o_th2 = gm_pow(P.o_fundvol, 2.0);  // SMRO: theta ** 2 (SparseMeanRevertingOracle.py:105)
      h.o_mst = P.mkt_open + (i64)rs_exponential(G, 1.0 / P.o_lambda);
      set_seed(4 + 0, g_seed(G));  // exchange
      for (int a = P.first_noise; a < P.first_noise + P.n_noise; a++) {
        set_seed(4 + a, g_seed(G));
        const i64 wt = P.mkt_open + (i64)(rs_double(G) * (double)(P.mkt_close - P.mkt_open));
        const i64 size = rs_randint(G, 20, 50);
        rec_init(a, AG_NOISE);
        this->rs64(AF_WAKEUP_TIME, wt);
        this->rs(AF_SIZE, (u32)size);
        this->rec_store();
      }
      for (int a = P.first_value; a < P.first_value + P.n_value; a++) {
        set_seed(4 + a, g_seed(G));
        const i64 size = rs_randint(G, 20, 50);
        rec_init(a, AG_VALUE);
        this->rs(AF_SIZE, (u32)size);
        this->rsd(AF_R_T, P.v_rbar);
        this->rec_store();
      }
      // symmetrised matrix: latency[a][0] = latency[0][a], so row 0 is all that is read
      double* lat = this->lat();
      const i64 total = (i64)n * n;
      for (i64 d = 0; d < n; d++) {
        double v = rs_uniform(G, P.lat_lo, P.lat_hi);
        if (this->lane == 0) lat[d] = d == 0 ? 20000.0 : v;
      }
      rs_skip_words(G, 2 * (total - n));
      wfence();
    } else {
      set_seed(1, g_seed(G));  // O
      set_seed(2, g_seed(G));  // K
      if (P.config == MXA_CFG_SPARSE_ZI_100) set_seed(3, g_seed(G));  // L
      h.o_pt = P.mkt_open;
      h.o_pv = P.o_rbar;
      h.o_th2 = gm_pow(P.o_fundvol, 2.0);  // SMRO: theta ** 2 (SparseMeanRevertingOracle.py:105)
      h.o_mst = P.mkt_open + (i64)rs_exponential(G, 1.0 / P.o_lambda);
      set_seed(4 + 0, g_seed(G));  // exchange
      int a = P.first_zi;
      for (int g = 0; g < P.zi_ngroups; g++)
        for (int k = 0; k < P.zi_group_count[g]; k++, a++) {
          set_seed(4 + a, g_seed(G));
          rec_init(a, AG_ZI);
          this->rs(AF_GROUP, (u32)g);
          this->rsd(AF_R_T, P.zi_rbar);
          this->rec_store();
        }
      // latency matrix G.uniform(lo, hi, (n, n)) in C order: only min_latency[0][*] and
      // (sparse_zi_100) min_latency[*][0] are ever read; the other draws only advance G.
      double* lat = this->lat();
      i64 total = (i64)n * n, prev = -1;
      bool col = P.config == MXA_CFG_SPARSE_ZI_100;
      i64 nneed = col ? 2 * (i64)n - 1 : (i64)n;
      for (i64 k = 0; k < nneed; k++) {
        i64 d = k < n ? k : (k - n + 1) * (i64)n;  // row 0, then column 0 (d = r*n)
        rs_skip_words(G, 2 * (d - prev - 1));
        double v = rs_uniform(G, P.lat_lo, P.lat_hi);
        if (this->lane == 0) {
          if (d < n) lat[d] = v;
          if (col && d % n == 0) lat[n + d / n] = v;
        }
        prev = d;
      }
      rs_skip_words(G, 2 * (total - prev - 1));
      if (P.config == MXA_CFG_SPARSE_ZI_1000) {
        if (this->lane == 0) lat[0] = 20000.0;  // diagonal (never used)
      }
      wfence();
    }
    this->grs_put(0, G);
    // expand all other streams, then the per-stream config-time draws
    seed_streams(1);
    h.rs_pos[1] = h.rs_pos[2] = h.rs_pos[3] = MXA_MT_N;
    h.rs_m[1] = h.rs_m[2] = h.rs_m[3] = 0;
    if constexpr (!E::EXT) {  // oracle first megashock (SMRO:71-72)
      RS O = this->grs(1);
      double msv = rs_normal(O, P.o_msmean, __builtin_sqrt(P.o_msvar));
      h.o_msv = rs_randint(O, 0, 2) == 0 ? msv : -msv;
      this->grs_put(1, O);
    }
    // exchange record
    rec_init(0, AG_EXCHANGE);
    this->rs64(AF_COMP, P.default_comp_delay);
    this->rec_store();
    // momentum size = A.randint(min, max); ZI theta = sorted(round(A.normal(0, sqrt(sigma_pv), 2 qmax)))
    for (int a = P.first_mom; a < P.first_mom + P.n_mom; a++) {
      this->rec_load(a);
      RS A = this->agent_rs();
      this->rs(AF_SIZE, (u32)rs_randint(A, P.mom_min, P.mom_max));
      this->agent_rs_put(A);
      this->rec_store();
    }
    for (int a = P.first_mk; a < P.first_mk + P.n_mk; a++) {  // MarketMakerAgent.py:51
      this->rec_load(a);
      RS A = this->agent_rs();
      this->rs(AF_SIZE, (u32)(i64)__builtin_rint((double)rs_randint(A, P.mk_min, P.mk_max) / 2));
      this->agent_rs_put(A);
      this->rec_store();
    }
    constexpr bool ZI_LANES = MXA_ZI_THETA_LANES && E::PC.n_zi + E::PC.n_hbl > 0;
    if constexpr (ZI_LANES) zi_theta_lanes();
    for (int a = P.first_zi; a < P.first_zi + P.n_zi + P.n_hbl; a++) {  // HBL agents are ZI subclasses
      if (ZI_LANES && !zi_fallback(a)) continue;  // done by zi_theta_lanes
      this->rec_load(a);
      RS A = this->agent_rs();
      double th[20];
      int nq = 2 * P.zi_qmax;
      for (int i = 0; i < 20; i++) th[i] = 0;
      for (int i = 0; i < nq; i++) th[i] = __builtin_rint(rs_normal(A, 0, __builtin_sqrt(P.zi_sigma_pv)));
      // stable descending insertion sort (wave-uniform, 20 elements)
      for (int i = 1; i < nq; i++) {
        double x = th[i];
        int j = i - 1;
        while (j >= 0 && th[j] < x) {
          th[j + 1] = th[j];
          j--;
        }
        th[j + 1] = x;
      }
      for (int i = 0; i < nq; i++) this->rs(AF_THETA + i, (u32)(i32)th[i]);
      this->agent_rs_put(A);
      this->rec_store();
    }
    // run-kernel invariant: every stream has the block after its current one materialized
    for (int k = 0; k < 4; k++) {
      RS r = this->grs(k);
      rs_maint(r);
      this->grs_put(k, r);
    }
    if constexpr (MXA_MAINT_LANES) {
      maint_agents();
    } else {
      for (int a = 0; a < n; a++) {
        this->rec_load(a);
        RS A = this->agent_rs();
        rs_maint(A, MXA_AGENT_LA);
        this->agent_rs_put(A);
        this->rec_store();
      }
    }
    // Kernel.runner: kernelInitializing (exchange opening price = r_bar, a python float; with the
    // ExternalFileOracle int(round(price at the open)), ExternalFileOracle.py:37-50),
    // kernelStarting (every agent wakes at startTime, in id order)
    if constexpr (E::EXT) {
      const double op = this->efo_price(P.mkt_open);
      h.last_trade = py_round(op);
      h.last_trade_float = 0;
      // getDailyOpenPrice's getPriceAtTime logs f_log's first entry when the open lies inside the
      // series; the build has no book-update log, so the first logged launch writes it (efo_open)
      const i64 t0 = U(this->rx->fs_t[0]), t1 = U(this->rx->fs_t[U(this->rx->fs_n) - 1]);
      h.o_pt = (P.mkt_open >= t0 && P.mkt_open <= t1) ? P.mkt_open : -1;
      h.o_pv = op;
    } else {
      h.last_trade = (i64)P.o_rbar;
      h.last_trade_float = 1;
    }
    this->cur = P.start;
    for (int a = 0; a < n; a++) this->wakeup_at(a, P.start);
    count_base();
    this->save();
    // the transaction ring (the history-epoch entry counts are header fields, zeroed above)
    TxRec* R = this->txr();
    for (int i = this->lane; i < P.L.tx_cap; i += 64) {
      TxRec z;
      z.t = 0;
      z.q = 0;
      z.epoch = -1000000;
      R[i] = z;
    }
  }
};

}  // namespace mxa

// ------------------------------------------------------------------------------------
// kernels (one wavefront per env; grid = n_envs)
// ------------------------------------------------------------------------------------
template <int CFG>
__global__ __launch_bounds__(64) void mxa_build_kernel(char* base, uint64_t stride, int n_envs, const uint32_t* seeds, const uint8_t* mask,
                                                       const RpCtx* ctx) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  int env = blockIdx.x;
  if (env >= n_envs) return;
  if (mask && !mask[env]) return;
  mxa::Builder<CFG> b(base + (size_t)env * stride, lds, ctx);
  if constexpr (mxa::Eng<CFG>::PC.mm_rt) b.mmp = ctx->mmp + env;
  b.build(seeds[env], mask && mask[env] == 2);  // 2: a later episode of the same process
}

// INSTR: the parity instrumentation (per-pop hash, trace ring) compiled in; the variant without
// it is what a run with the hash off and no trace ring launches (same results, fewer registers)
template <int CFG, bool LOG, bool INSTR>
__global__ __launch_bounds__(64, mxa_cfg::shape(CFG).waves) void mxa_run_kernel(char* base, uint64_t stride, int n_envs, int trace_cap, int64_t max_pops,
                                                                              const RpCtx* ctx, BlRec* blog, int blog_cap,
                                                                              const int32_t* list) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  // list (nullable): the envs still running after the previous launch, compacted by
  // mxa_compact_kernel (mxa_api.hip); the grid is then one wave per listed env, so the dispatcher
  // spreads only live envs over the CUs instead of leaving the slots of finished ones idle
  int env = list ? list[blockIdx.x] : (int)blockIdx.x;
  if (env >= n_envs) return;
  char* e = base + (size_t)env * stride;
  if (((EnvHdr*)e)->status != ST_RUNNING) return;
  mxa::Eng<CFG, false, LOG, INSTR> g(e, lds, trace_cap, ctx, LOG ? blog + (size_t)env * blog_cap : nullptr, blog_cap);
  g.load();
  g.run(max_pops);
  g.save();
#ifdef MXA_PROF
  atomicAdd(&mxa::g_mxa_prof[g.lane], (unsigned long long)g.prof[g.lane]);
  atomicAdd(&mxa::g_mxa_prof[64 + g.lane], (unsigned long long)g.prof[64 + g.lane]);
#endif
}

template <int CFG, bool LOG>
__global__ __launch_bounds__(64) void mxa_stop_kernel(char* base, uint64_t stride, int n_envs, mxa_agent_final* out,
                                                      BlRec* blog, int blog_cap, const RpCtx* ctx) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  int env = blockIdx.x;
  if (env >= n_envs) return;
  char* e = base + (size_t)env * stride;
  mxa::Eng<CFG, false, LOG> g(e, lds, 0, ctx, LOG ? blog + (size_t)env * blog_cap : nullptr, blog_cap);
  g.load();
  g.stop(out + (size_t)env * mxa::Eng<CFG>::PC.n_agents);  // no save(): the pass is idempotent
  // the oracle observations of the pass append to the log after the run's records; only
  // their end is kept (a second pass rewrites the same records)
  if (LOG && g.lane == 0) ((EnvHdr*)e)->blog_fin = g.h.blog_n;
}

#ifndef MXA_NO_GYM
// ABIDESEnv.step for every env: DummyRL.place_orders(action), then the GymKernel loop until
// the RL agent's spread reply (end of step) or the end of the episode.  obs [n][9] float64;
// flags [n]: bit0 done, bit1 observation valid, bit2 env error.  INSTR as for the run kernel.
// MANY: k_steps consecutive steps in one launch with actions given up front ([k][n][3];
// obs [k][n][9], flags [k][n]): each env runs its own steps without waiting for the slowest env
// of every step, and its state stays in LDS and registers between them.  Every step is the same
// code as a one-step launch, so results, observations and flags are the same step by step.
template <int CFG, bool INSTR, bool MANY>
__global__ __launch_bounds__(64, mxa_cfg::shape(CFG).waves) void mxa_step_kernel(
    char* base, uint64_t stride, int n_envs, int trace_cap, int64_t max_pops, const RpCtx* ctx, const double* actions,
    double* obs, int32_t* flags, int k_steps) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  int env = blockIdx.x;
  if (env >= n_envs) return;
  char* e = base + (size_t)env * stride;
  mxa::Eng<CFG, false, false, INSTR> g(e, lds, trace_cap, ctx);
  g.load();
  const int ks = MANY ? k_steps : 1;
  for (int i = 0; i < ks; i++) {
    if (g.status == ST_RUNNING) {
      double a[3];
      for (int j = 0; j < 3; j++) a[j] = actions[3 * ((size_t)i * n_envs + env) + j];
      g.rl_place_orders(a);
      g.end_step = 0;
      g.run(max_pops);
      if (g.status == ST_RUNNING) {  // after the loop: terminateRunner if the queue ran dry / past stop
        u64 key;
        u32 s;
        if (g.q_peek(key, s) < 0 || g.cur > mxa::Eng<CFG>::PC.stop) g.status = ST_DONE;
      }
      if (g.status == ST_DONE) g.rp_terminate();
    }
    if (!MANY) g.save();
    auto R = g.rh();
    const size_t row = (size_t)i * n_envs + env;
    if (g.lane < 9) obs[9 * row + g.lane] = R->obs[g.lane];
    u64 key;
    u32 sq;
    const bool pending = g.q_peek(key, sq) >= 0;  // all lanes: DPP reduction
    // ABIDESEnv.step: done = not (queue non-empty and currentTime <= stopTime)
    const int done = !(pending && g.cur <= mxa::Eng<CFG>::PC.stop) || g.status != ST_RUNNING;
    const int hobs = mxa::U(R->has_obs);
    if (g.lane == 0) flags[row] = done | (hobs ? 2 : 0) | (g.status == ST_ERROR ? 4 : 0);
  }
  if (MANY) g.save();
#ifdef MXA_PROF
  atomicAdd(&mxa::g_mxa_prof[g.lane], (unsigned long long)g.prof[g.lane]);
  atomicAdd(&mxa::g_mxa_prof[64 + g.lane], (unsigned long long)g.prof[64 + g.lane]);
#endif
}
#endif

#ifdef MXA_API_TU  // (compiled once, in the C-ABI translation unit)
// parity helpers: numpy-legacy RNG draws and glibc math on the device (tests only call
// these through the C-ABI; they exercise exactly the device functions the engine uses)
__global__ __launch_bounds__(64) void mxa_rng_probe_kernel(uint32_t seed, int mode, double a, double b, int n, double* out, uint32_t* scratch) {
  mxa::mt_seed(scratch, seed);
  mxa::RSt<true> r;
  r.lw = nullptr;  // draws read the MT block in HBM
  r.lw0 = r.lwn = 0;
  r.key = scratch;
  r.p = MXA_MT_N;
  r.m = 0;
  r.hasg = 0;
  r.gauss = 0;
  for (int i = 0; i < n; i++) {
    double v;
    switch (mode) {
    case 0: v = (double)mxa::rs_u32(r); break;
    case 1: v = mxa::rs_double(r); break;
    case 2: v = (double)mxa::rs_randint(r, (int64_t)a, (int64_t)b); break;
    case 3: v = mxa::rs_normal(r, a, b); break;
    case 4: v = mxa::rs_exponential(r, a); break;
    default: v = mxa::rs_uniform(r, a, b); break;
    }
    if (__lane_id() == 0) out[i] = v;
  }
}
__global__ void mxa_math_probe_kernel(int mode, const double* x, const double* y, double* out, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = mode == 0 ? gm_log(x[i]) : mode == 1 ? gm_exp(x[i]) : gm_pow(x[i], y[i]);
}
#endif
