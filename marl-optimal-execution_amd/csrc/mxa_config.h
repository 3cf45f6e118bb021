// mxa_config.h — the reference configurations as compile-time constants.
//
// Each reference config script (config/rmsc03.py, config/sparse_zi_100.py,
// config/sparse_zi_1000.py) is a fixed set of constants once its argparse defaults are
// taken.  They are restated here as constexpr MxaParams so the device engine is
// instantiated per configuration with every parameter folded into immediates: no
// parameter loads and no registers pinned for them in the event loop.  The host side
// (mxa_api.hip) uses the same functions for the layout and the readers, then adds the
// per-handle runtime values (n_envs, trace capacity, env stride).
#pragma once
#include <stddef.h>
#include "mxa_layout.h"
#include "../../include/mxa.h"

namespace mxa_cfg {

constexpr int64_t NS = 1000000000LL;
constexpr int64_t MIN = 60 * NS;
constexpr int64_t HOUR = 60 * MIN;

// engine shape per configuration: queue slots per lane (SQ), book slots per lane (SO),
// payload in LDS (PL), run-kernel waves per SIMD the register budget targets (W)
struct Shape {
  int sq, so;
  bool pl;
  int waves;
  int pw;  // message payload words kept in the queue
  int hot;  // agent records kept in LDS for a launch: the exchange, then the market maker
  int sql = 0;  // queue slots per lane in LDS (0: all sq); the rest are an HBM tier (far events)
};
constexpr int sq_lds(int cfg);
constexpr int lat_lds(int cfg);
constexpr Shape shape(int cfg);
#ifndef MXA_RMSC03_WAVES
#define MXA_RMSC03_WAVES 4
#endif
#ifndef MXA_RMSC01_WAVES
#define MXA_RMSC01_WAVES 4
#endif
// run-kernel waves per SIMD the register budget targets (-D overrides for A/B builds)
#ifndef MXA_W_RMSC02
#define MXA_W_RMSC02 2
#endif
// rmsc02's book arrays held in LDS for a launch instead of VGPRs (bit: 0 price, 1 qty, 2 order id,
// 3 agent/side, 4 arrival, 5 history epoch).  The 576-slot book in VGPRs left the run kernel at 256
// VGPRs and 352 B/lane of scratch, ~900 B/event of spill writes in the PMC record (r05).  The
// order id, arrival and epoch arrays (read only when an order is matched or cancelled) move to LDS,
// price / side / quantity (every best-price and level scan) stay in VGPRs; 88 B/lane of scratch
// remain.  To keep 8 waves per CU with the payloads in LDS the queue has 4 slots per lane (256;
// the oracle's maximum over the 131,072 bench seeds is 225 pending events, a full queue is env
// error 1).  r05 A/B, rmsc02 x4096 run kernel, same digest (profiles/r05/ab_mr/ab_book.txt): 871.5
// -> 816.9 ms; the whole book in LDS with HBM payloads 936.5, HBM payloads alone 1052.4.  (The
// exchange record in LDS as well, which fills the 160 KB exactly: 815.1 -> 817.5 ms, r05)
#ifndef MXA_BOOK_LDS_RMSC02
#define MXA_BOOK_LDS_RMSC02 0x34
#endif
#ifndef MXA_PL_RMSC02
#define MXA_PL_RMSC02 1
#endif
#ifndef MXA_SQ_RMSC02
#define MXA_SQ_RMSC02 4
#endif
#ifndef MXA_SO_RMSC02
// 576 book slots: the oracle's maximum over every seed of bench.py --gpus <= 8 is 537 (512
// overflowed).  The book lives in VGPRs: 640 slots measured 1319 ms against 1054 ms for 576
// (rmsc02 x4096 run kernel, same digest; 848 vs 535 static scratch instructions)
#define MXA_SO_RMSC02 9
#endif
#ifndef MXA_SQ_Z1K
#define MXA_SQ_Z1K 36  // sparse_zi_1000 queue slots per lane (2,304; the oracle's maximum over the 32,768 seeds of
                       // bench.py --gpus 1-8 is 2,007 pending events, profiles/r04/capacity_sparse_zi_1000.json);
                       // r03 s22 run kernel: 48 slots 821 ms, 36 slots 796
#endif
// configurations whose exchange latency row (the only row Kernel.sendMessage reads with a
// symmetric matrix) is copied to LDS for each launch (bit = config id)
#ifndef MXA_LAT_LDS_MASK
#define MXA_LAT_LDS_MASK (1 << MXA_CFG_SPARSE_ZI_1000)  // r03 s22: 796 -> 784 ms (8 KB row, room from the 36-slot queue)
#endif
#ifndef MXA_SO_Z1K
#define MXA_SO_Z1K 13  // sparse_zi_1000 book slots per lane (832; oracle max 738 resting orders over the 32,768 seeds of bench.py --gpus 1-8); r03 s9 run kernel: 16 slots 1004 ms, 14 952, 13 925
#endif
#ifndef MXA_SO_RFD
#define MXA_SO_RFD 9
#endif
// random_fund_diverse with 576 book slots and 128 open orders per agent (r03 s4, x2048, same
// results): 2 waves/SIMD 2421 ms, 1 wave 1861 ms, 1 wave + 48 LDS queue slots per lane 1810 ms
#ifndef MXA_RFD_WAVES
#define MXA_RFD_WAVES 1
#endif
#ifndef MXA_RFD_SQL
#define MXA_RFD_SQL 24  // r06: 48 -> 24 with the LDS book arrays, 1315.2 -> 1180.7 ms (ab6_rfd_book_lds.txt)
#endif
// configurations whose agent-record write-back stores only the changed 128-byte quarters
// (bit = config id; measured per configuration)
#ifndef MXA_DIRTY_WB_MASK
// r03 s5: random_fund_value 840 -> 795 ms; rmsc03 +2 % (s38 on the final build: +5 %); rmsc01 +4 % in s5, but
// -4.6 % on the final build (s48: 1023 -> 976 ms); rmsc02 unchanged (s48).  r05, after the HBL fence
// fix: rmsc02 PMC writes 300 -> 240 B/event (reads 297) for 780 -> 790 ms (ab_dwb_rmsc02.txt), on;
// obi_rmsc02 307 vs 305 ms, rmsc03 39.4 vs 38.2 ms (ab_dwb_levels.txt), off
#define MXA_DIRTY_WB_MASK ((1 << 9) | (1 << 10) | (1 << 11) | (1 << 12) | (1 << MXA_CFG_RMSC01) | (1 << MXA_CFG_RMSC02))
#endif
#ifndef MXA_OPEN_RFD
#define MXA_OPEN_RFD 128
#endif
#ifndef MXA_AUTO_SKIP
#define MXA_AUTO_SKIP 1024  // replay: explicit tape ids one episode's auto ids may skip (Order.generateOrderId)
#endif
#ifndef MXA_W_OBI
#define MXA_W_OBI 2
#endif
#ifndef MXA_W_Z1
#define MXA_W_Z1 2
#endif
#ifndef MXA_W_VN
#define MXA_W_VN 2
#endif
#ifndef MXA_RFV_WAVES
#define MXA_RFV_WAVES 2  // random_fund_value / _diverse waves per SIMD (rfv run kernel x2048: 1 wave 1412 ms, 2 waves 1230; x4096: 2 waves 2446, 3 4014, 4 4378)
#endif
#ifndef MXA_RFV_SQL
#define MXA_RFV_SQL 12  // LDS-resident queue slots per lane (96 = no HBM tier); rfv x2048 run kernel (r02, before the
                        // lane-major HBM tier): 12 -> 1220 ms, 24 -> 840, 36 -> 1237 (fewer waves fit); r06: 24 -> 338.1,
                        // 12 with the LDS book arrays 330.2 (MXA_BOOK_LDS_RFV)
#endif
#ifndef MXA_RP_HOT
#define MXA_RP_HOT 2  // replay configurations: the exchange's and the MarketReplayAgent's records in LDS
#endif
constexpr Shape shape_builtin(int cfg) {
  // rmsc03: 192 queue slots (the oracle's maximum over the 4096 bench seeds is 146, over 1024
  // rmsc03_rl episodes 146), so 16 waves per CU fit the queue, the header and the exchange and
  // market-maker records in LDS
  return cfg == MXA_CFG_RMSC03 ? Shape{3, 2, true, MXA_RMSC03_WAVES, 6, 0}
       // rmsc03 + SpreadBasedMarketMakerAgent: MARKET_DATA carries level counts (8 payload words)
       : cfg == MXA_CFG_RMSC03_SBMM ? Shape{3, 2, true, 4, 8, 0}
       : cfg == MXA_CFG_RMSC03_SBMM_POLL ? Shape{3, 2, true, 4, 6, 0}
       : cfg == MXA_CFG_RMSC03_RL ? Shape{3, 2, true, 4, 8, 0}  // wide spread replies (depth 500)
       // rmsc03 with per-env market-maker options: scripts/rmsc03.sh's 50 ticks (a 102-order ladder)
       // peak at 266 pending events and 122 resting orders (oracle, 4,096 seeds of the script's
       // options and of a mixed grid: pov 0.01-0.2, sizes 10-50, windows 1-10, 5-50 ticks, 1-60 s);
       // 320 queue slots, 192 book slots; the LDS queue holds the wave count to 3 per SIMD
       : cfg == MXA_CFG_RMSC03_MM ? Shape{5, 3, true, 3, 6, 0}
       // rmsc01: oracle maxima over seeds 123456789 / 7: 140 pending events, 75 resting orders;
       // wide replies for the market maker's depth-5 spread queries
       : cfg == MXA_CFG_RMSC01 ? Shape{3, 2, true, MXA_RMSC01_WAVES, 8, 0}
       // rmsc02: oracle maxima over the 131,072 seeds bench.py draws at --gpus 1-8 (batches 0-3 of
       // ranks 0-7, tools/capacity_sweep.py, profiles/r04/capacity_rmsc02.json): 225 pending
       // events (256 queue slots), 537 resting orders, 59 open orders of one agent (576 book slots)
       : cfg == MXA_CFG_RMSC02 ? Shape{MXA_SQ_RMSC02, MXA_SO_RMSC02, MXA_PL_RMSC02 != 0, MXA_W_RMSC02, 8, 0}
       // obi_rmsc02: oracle maxima over the 131,072 seeds of bench.py --gpus 1-8: 211 pending
       // events, 149 resting orders (192 book slots; 128 overflowed)
       : cfg == MXA_CFG_OBI_RMSC02 ? Shape{4, 3, true, MXA_W_OBI, 8, 0}
       : cfg == MXA_CFG_SPARSE_ZI_100 ? Shape{8, 2, true, MXA_W_Z1, 6, 0}
       : cfg == MXA_CFG_VALUE_NOISE ? Shape{6, 2, true, MXA_W_VN, 6, 0}  // 384 slots: oracle max 301 (2048 seeds)
       : cfg == MXA_CFG_SPARSE_ZI_1000 ? Shape{MXA_SQ_Z1K, MXA_SO_Z1K, false, 1, 6, 0}
       // random_fund_value: 6,144 queue slots (every agent keeps a wakeup pending: the oracle's
       // maximum over the 8,192 bench seeds is 5,125 events), payload in HBM; 320 book slots (max 279)
       // the first MXA_RFV_SQL slots per lane (12: 768) in LDS for events due within a second,
       // the other 72 per lane an HBM tier for the far wakeups (the two-tier queue, q_push)
       : (cfg == MXA_CFG_RANDOM_FUND_VALUE || cfg == MXA_CFG_HIST_FUND_VALUE) ? Shape{96, 5, false, MXA_RFV_WAVES, 6, 0, MXA_RFV_SQL}
       // random_fund_diverse: the same queue; 576 book slots (oracle max 503 resting orders and 5,153
       // pending events over the 65,536 seeds of bench.py --gpus 1-8: 448 slots overflowed) and wide
       // replies for the market maker's depth-5 spread queries
       : (cfg == MXA_CFG_RANDOM_FUND_DIVERSE || cfg == MXA_CFG_HIST_FUND_DIVERSE)
           ? Shape{96, MXA_SO_RFD, false, MXA_RFD_WAVES, 8, 0, MXA_RFD_SQL}
                                       : Shape{4, 1, true, 2, 8, MXA_RP_HOT};  // marketreplay (both): book in HBM; 256 queue slots (GOOG 2012-06-21 peaks at 113)
}
constexpr int sq_lds(int cfg) { return shape(cfg).sql ? shape(cfg).sql : shape(cfg).sq; }
// configurations whose replay / gym header (RpHdr: best levels, free-stack top, replay cursor, RL
// state) is LDS-resident for a launch of the run / step kernel: the replay ladder's handlers read
// and update it on every event (IBM x512 step 0.369 -> 0.363 ms).  Not rmsc03_rl, whose header
// only DummyRL's events touch: there it cost the step kernel 1.88 -> 2.05 ms (r05 s1)
constexpr bool rp_hdr_lds(int cfg) {
  return cfg == MXA_CFG_MARKETREPLAY || cfg == MXA_CFG_MARKETREPLAY_RUNNER || cfg == MXA_CFG_MARKETREPLAY_TWAP;
}
// random_fund_* / hist_fund_*: the book's order-id, arrival and epoch arrays in LDS for a launch
// (as rmsc02's), with a 12-slot-per-lane LDS queue tier (random_fund_value) or 24 (the _diverse
// pair) so the arrays fit.  r06 A/B, same digests (profiles/r06/ab/ab5_rfv_book_lds.txt, ab6_rf?_book_*.txt):
// random_fund_value x2048 360.3 -> 330.2 ms (the smaller tier alone 338.1; the arrays at 24 slots
// overflow the LDS budget: 639.3); random_fund_diverse x2048 1315.2 -> 1180.7 ms
#ifndef MXA_BOOK_LDS_RFV
#define MXA_BOOK_LDS_RFV 0x34
#endif
constexpr int book_lds(int cfg) {
  return cfg == MXA_CFG_RMSC02 ? MXA_BOOK_LDS_RMSC02
         : (cfg >= MXA_CFG_RANDOM_FUND_VALUE && cfg <= MXA_CFG_HIST_FUND_DIVERSE) ? MXA_BOOK_LDS_RFV
                                                                                 : 0;
}
constexpr size_t lds_bytes(int cfg) {
  return (size_t)sq_lds(cfg) * 64 * (12 + (shape(cfg).pl ? 4 * shape(cfg).pw : 0)) + 512  // queue + EnvHdr
         + (size_t)shape(cfg).hot * 512                                                       // hot agent records
         + 1024                                                                               // RNG stream windows
         + (size_t)lat_lds(cfg) * 8                                                           // exchange latency row
         + (rp_hdr_lds(cfg) ? 256 : 0)                                                        // RpHdr (replay / gym)
         + (size_t)__builtin_popcount(book_lds(cfg)) * shape(cfg).so * 256                    // LDS book arrays
         + 256  // batched-push scratch: slot table
#ifdef MXA_PROF
         + 1024  // phase counters and inclusive function timers (128 x u64)
#endif
      ;
}

constexpr void base_params(MxaParams& P) {
  P.o_rbar = 1e5;
  P.o_kappa = 1.67e-12;
  P.o_fundvol = 1e-4;
  P.o_lambda = 2.77778e-13;
  P.o_msmean = 1e3;
  P.o_msvar = 5e4;
  P.starting_cash = 10000000;
  P.ex_pipeline = 0;
  P.ex_comp = 0;
  P.stream_history = 10;
  P.mkt_open = 9 * HOUR + 30 * MIN;
}

// config/rmsc03.py:55-235 (defaults of its argparse options)
constexpr void params_rmsc03(MxaParams& P) {
  base_params(P);
  P.config = MXA_CFG_RMSC03;
  P.ex_log_orders = 1;  // config/rmsc03.py:102
  P.mkt_close = 9 * HOUR + 45 * MIN;
  P.start = P.mkt_open;
  P.stop = P.mkt_close + MIN;
  P.default_comp_delay = 0;
  P.lat_mode = 0;
  P.noise_len = 1;
  P.first_noise = 1;
  P.n_noise = 50;
  P.first_value = 51;
  P.n_value = 10;
  P.first_mm = 61;
  P.n_mm = 1;
  P.first_mom = 62;
  P.n_mom = 2;
  P.n_agents = 64;
  P.v_sigma_n = 1e5 / 10;
  P.v_rbar = 1e5;
  P.v_kappa = 1.67e-15;
  P.v_sigma_s = 100000;
  P.v_lambda = 7e-11;
  P.v_percent_aggr = 0.1;
  P.v_depth_spread = 2;
  P.v_starting_cash = 10000000;
  P.noise_open = 9 * HOUR;
  P.noise_close = 16 * HOUR;
  P.mm_pov = 0.05;
  P.mm_min_size = 20;
  P.mm_window = 5;
  P.mm_ticks = 20;
  P.mm_wake = NS;
  P.mom_min = 1;
  P.mom_max = 10;
  P.mom_wake = 20 * NS;
  P.L.open_cap = 128;
  P.L.tx_cap = 256;
  P.L.lat_len = 0;
}

// config/rmsc03.py with its market-maker options per env (--mm-pov, --mm-min-order-size,
// --mm-window-size, --mm-num-ticks, --mm-wake-up-freq; config/rmsc03.py:39-43, 158-177): the
// values here are the defaults, the build kernel writes each env's into the market maker's
// record.  The market maker's open orders peak at twice its ladder (the cancelled ladder stays
// in TradingAgent.orders until ORDER_CANCELLED): 204 at 50 ticks, so 256 per agent
constexpr void params_rmsc03_mm(MxaParams& P) {
  params_rmsc03(P);
  P.config = MXA_CFG_RMSC03_MM;
  P.mm_rt = 1;
  P.L.open_cap = 256;
}

// rmsc03 with a SpreadBasedMarketMakerAgent in its market maker's slot (agent 61), built from the
// same script arguments (window 5, 20 ticks, wake-up 1 s, order_size = --mm-min-order-size);
// tests/golden/gen_fixtures.py rmsc03_sbmm / rmsc03_sbmm_poll.  subscribe=True requests level-1
// MARKET_DATA every 10e9 ns (SpreadBasedMarketMakerAgent.py:28-30, 78-80)
constexpr void params_rmsc03_sbmm(MxaParams& P, bool subscribe) {
  params_rmsc03(P);
  P.config = subscribe ? MXA_CFG_RMSC03_SBMM : MXA_CFG_RMSC03_SBMM_POLL;
  P.first_mm = 0;
  P.n_mm = 0;
  P.first_sb = 61;
  P.n_sb = 1;
  P.sb_sub = subscribe ? 1 : 0;
  P.sb_size = 20;
  P.sb_window = 5;
  P.sb_ticks = 20;
  P.sb_wake = NS;
  P.md_sub = subscribe ? 1 : 0;
  P.md_mk_levels = 1;
  P.md_mom_levels = 0;  // rmsc03's momentum agents poll (subscribe=False, config/rmsc03.py:180-197)
  P.md_freq = 10 * NS;
}

// config/random_fund_value.py:59-180: rmsc03's agent classes at 5,100 agents over a whole day:
// 5000 noise agents (wakeup_time in 09:30-16:00), 100 value agents (sigma_n 1e4, lambda_a 1e-12),
// no market maker or momentum agents; market 09:30-16:00, kernel 09:30-16:01, zero latency
constexpr void params_random_fund_value(MxaParams& P) {
  params_rmsc03(P);
  P.config = MXA_CFG_RANDOM_FUND_VALUE;
  P.mkt_close = 16 * HOUR;
  P.start = P.mkt_open;
  P.stop = P.mkt_close + MIN;
  P.n_noise = 5000;
  P.first_value = 5001;
  P.n_value = 100;
  P.first_mm = 0;
  P.n_mm = 0;
  P.first_mom = 0;
  P.n_mom = 0;
  P.n_agents = 5101;
  P.v_lambda = 1e-12;
  P.noise_open = P.mkt_open;
  P.noise_close = 16 * HOUR;
  P.L.open_cap = 8;
  P.L.tx_cap = 64;
}

// config/random_fund_diverse.py:157-198: random_fund_value plus a MarketMakerAgent (polling,
// 100-101 shares, depth-5 spread queries, "1min") and 25 momentum agents (1-10 shares, 60 s)
constexpr void params_random_fund_diverse(MxaParams& P) {
  params_random_fund_value(P);
  P.config = MXA_CFG_RANDOM_FUND_DIVERSE;
  P.first_mk = 5101;
  P.n_mk = 1;
  P.mk_min = 100;
  P.mk_max = 101;
  P.mk_depth = 5;
  P.mk_wake = MIN;
  P.mk_last_spread = 10;
  P.first_mom = 5102;
  P.n_mom = 25;
  P.mom_min = 1;
  P.mom_max = 10;
  P.mom_wake = MIN;
  P.n_agents = 5127;
  P.L.open_cap = MXA_OPEN_RFD;  // the market maker's ladder: oracle max 78 open orders over the 8,192 bench seeds (64 overflowed)
}

// config/hist_fund_value.py / config/hist_fund_diverse.py: random_fund_value / _diverse with the
// ExternalFileOracle (util/oracle/ExternalFileOracle.py) on a fundamental series given at create
// time; the value agents' r_bar is the series' first value and sigma_n = r_bar / 10 (runtime)
constexpr void params_hist_fund(MxaParams& P, bool diverse) {
  if (diverse) params_random_fund_diverse(P);
  else params_random_fund_value(P);
  P.config = diverse ? MXA_CFG_HIST_FUND_DIVERSE : MXA_CFG_HIST_FUND_VALUE;
  P.oracle_ext = 1;
}

// config/sparse_zi_100.py:73-334 and config/sparse_zi_1000.py
constexpr void params_sparse_zi(MxaParams& P, bool big) {
  base_params(P);
  P.config = big ? MXA_CFG_SPARSE_ZI_1000 : MXA_CFG_SPARSE_ZI_100;
  P.ex_log_orders = big ? 0 : 1;  // sparse_zi_100.py:187 log_orders=True; sparse_zi_1000.py:183 the -o option (off)
  P.mkt_close = 16 * HOUR;
  P.start = 0;
  P.stop = 17 * HOUR;
  P.default_comp_delay = 1000000000;
  constexpr int n100[7] = {15, 15, 14, 14, 14, 14, 14};
  constexpr int n1000[7] = {143, 143, 143, 143, 143, 143, 142};
  constexpr int rmin[7] = {0, 0, 0, 0, 0, 250, 250};
  constexpr int rmax[7] = {250, 500, 1000, 1000, 2000, 500, 500};
  constexpr double eta[7] = {1, 1, 0.8, 1, 0.8, 0.8, 1};
  P.zi_ngroups = 7;
  int n = 0;
  for (int g = 0; g < 7; g++) {
    P.zi_group_count[g] = big ? n1000[g] : n100[g];
    P.zi_rmin[g] = rmin[g];
    P.zi_rmax[g] = rmax[g];
    P.zi_eta[g] = eta[g];
    n += P.zi_group_count[g];
  }
  P.first_zi = 1;
  P.n_zi = n;
  P.n_agents = 1 + n;
  P.zi_sigma_n = 1000000.0;
  P.zi_rbar = 1e5;
  P.zi_kappa = 1.67e-15;
  P.zi_sigma_s = 1e-4;
  P.zi_lambda = 1e-12;
  P.zi_sigma_pv = 5e6;
  P.zi_qmax = 10;
  if (!big) {
    P.lat_mode = 2;
    P.jitter = 0.3;
    P.clip = 0.05;
    P.unit = 5;
    P.lat_lo = 21000;
    P.lat_hi = 100000;
    P.L.lat_len = 2 * P.n_agents;
  } else {
    P.lat_mode = 1;
    P.noise_len = 6;
    P.lat_lo = 21000;
    P.lat_hi = 13000000;
    P.L.lat_len = P.n_agents;
  }
  P.L.open_cap = 8;
  P.L.tx_cap = 256;
}

// ABIDESEnv composition (ABIDESEnv.py:59-103, agent_config.py): Exchange, MarketReplayAgent,
// DummyRLExecutionAgent; GymKernel start midnight, stop 16:10, compute delays 0, latency 0,
// noise [1.0] (no draw).  Nothing draws from an RNG.
constexpr void params_marketreplay(MxaParams& P) {
  base_params(P);
  P.config = MXA_CFG_MARKETREPLAY;
  P.ex_log_orders = 1;  // config/marketreplay.py:77, agent_config.py:54
  P.mkt_close = 16 * HOUR;
  P.start = 0;
  P.stop = 16 * HOUR + 10 * MIN;
  P.default_comp_delay = 0;
  P.lat_mode = 0;
  P.noise_len = 1;
  P.starting_cash = 0;
  P.first_replay = 1;
  P.n_replay = 1;
  P.first_rl = 2;
  P.n_rl = 1;
  P.n_agents = 3;
  P.rl_quantity = 100000;
  P.rl_h0 = 9 * HOUR + 40 * MIN;
  P.rl_hstep = 30 * NS;
  P.rl_nh = 761;      // pd.date_range(09:40, 16:00, freq="30S")
  P.rl_depth = 500;   // getCurrentSpread(depth=500)
  P.rl_ids = 4096;    // DummyRL order ids (2 per step at most)
  P.L.open_cap = 64;
  P.L.tx_cap = 64;
  P.L.lat_len = 0;
}

// config/marketreplay.py:60-140: the exchange and the MarketReplayAgent alone under
// Kernel.runner (midnight to 16:01, compute delay 0, latency 0, noise [0.0]); nothing draws
constexpr void params_marketreplay_runner(MxaParams& P) {
  params_marketreplay(P);
  P.config = MXA_CFG_MARKETREPLAY_RUNNER;
  P.stop = 16 * HOUR + MIN;
  P.first_rl = 0;
  P.n_rl = 0;
  P.n_agents = 2;
}

// config/execution/marketreplay/execution_marketreplay.py:55-160: config/marketreplay.py's exchange
// and MarketReplayAgent plus TWAP_EXECUTION_AGENT 2 (TWAPExecutionAgent: BUY 12e3 over
// execution_time_horizon = pd.date_range(10:00, 12:00, "60S"), spread depth 500); whether it
// trades (the script's -e flag) is a runtime choice (RpCtx::twap_trade)
constexpr void params_marketreplay_twap(MxaParams& P) {
  params_marketreplay_runner(P);
  P.config = MXA_CFG_MARKETREPLAY_TWAP;
  P.n_agents = 3;
  P.first_twap = 2;
  P.n_twap = 1;
  P.rl_quantity = 12000;
  P.rl_h0 = 10 * HOUR;
  P.rl_hstep = 60 * NS;
  P.rl_nh = 121;
  P.rl_depth = 500;
}

// rmsc03 + DummyRL (BASELINE.json configs[3]; tests/golden/gen_rl_fixtures.py): rmsc03's 64
// agents under a GymKernel with DummyRLExecutionAgent 64 (agent_config.py:115-137 parameters:
// BUY 1e5, 30 s, order_level 2, spread depth 500), horizon pd.date_range(09:31, 09:44, "30S").
// The DummyRL draws nothing, so rmsc03's global draw order is unchanged.
constexpr void params_rmsc03_rl(MxaParams& P) {
  params_rmsc03(P);
  P.config = MXA_CFG_RMSC03_RL;
  P.first_rl = 64;
  P.n_rl = 1;
  P.n_agents = 65;
  P.rl_quantity = 100000;
  P.rl_h0 = 9 * HOUR + 31 * MIN;
  P.rl_hstep = 30 * NS;
  P.rl_nh = 27;
  P.rl_depth = 500;
}

// config/rmsc01.py:49-263 (RMSC-1): 1 exchange, 1 MarketMakerAgent (500-1000 shares, 1 s, depth 5),
// 50 ZI and 25 HBL agents (sigma_n 1e4, sigma_s = fund_vol 1e-4, kappa 1.67e-15, sigma_pv 5e4,
// R 0-100, eta 1, lambda_a 1e-12, q_max 10; HBL L = 2), 24 momentum agents (1-10 shares, 60 s);
// market 09:30-16:00, kernel 09:30-16:01, compute delay 0, zero latency
#ifndef MXA_OH_CAP
#define MXA_OH_CAP 16384  // order-history ring records (HBL streams reached 3,895 orders on seed 123456789)
#endif
#ifndef MXA_HBL_RANGE
#define MXA_HBL_RANGE 16384  // HBL price-histogram bins (largest streamed range on seed 123456789: 4,399)
#endif
constexpr void params_rmsc01(MxaParams& P) {
  base_params(P);
  P.config = MXA_CFG_RMSC01;
  P.ex_log_orders = 0;  // config/rmsc01.py:84
  P.mkt_close = 16 * HOUR;
  P.start = P.mkt_open;
  P.stop = 16 * HOUR + MIN;
  P.default_comp_delay = 0;
  P.lat_mode = 0;
  P.noise_len = 1;
  P.first_mk = 1;
  P.n_mk = 1;
  P.mk_min = 500;
  P.mk_max = 1000;
  P.mk_depth = 5;
  P.mk_wake = NS;
  P.mk_last_spread = 10;
  P.zi_ngroups = 1;
  P.zi_group_count[0] = 50;
  P.zi_rmin[0] = 0;
  P.zi_rmax[0] = 100;
  P.zi_eta[0] = 1;
  P.first_zi = 2;
  P.n_zi = 50;
  P.first_hbl = 52;
  P.n_hbl = 25;
  P.hbl_L = 2;
  P.zi_sigma_n = 10000;
  P.zi_rbar = 1e5;
  P.zi_kappa = 1.67e-15;
  P.zi_sigma_s = 1e-4;
  P.zi_lambda = 1e-12;
  P.zi_sigma_pv = 5e4;
  P.zi_qmax = 10;
  P.first_mom = 77;
  P.n_mom = 24;
  P.mom_min = 1;
  P.mom_max = 10;
  P.mom_wake = 60 * NS;
  P.n_agents = 101;
  P.L.open_cap = 64;
  P.L.tx_cap = 256;
  P.L.lat_len = 0;
  P.L.oh_cap = MXA_OH_CAP;
  P.L.hbl_range = MXA_HBL_RANGE;
}

// config/rmsc02.py (RMSC-2): rmsc01's agents with subscribe=True for the market maker
// (5 levels) and the momentum agents (1 level), both every 10e9 ns; kernel midnight-17:00;
// latency G.uniform(21000, 13e6, (101, 101)) drawn after the kernel seed (not symmetrised:
// row 0 and column 0 are read) with 6-way noise
constexpr void params_rmsc02(MxaParams& P) {
  params_rmsc01(P);
  P.config = MXA_CFG_RMSC02;
  P.ex_log_orders = 1;  // config/rmsc02.py:84
  P.start = 0;
  P.stop = 17 * HOUR;
  P.lat_mode = 1;
  P.noise_len = 6;
  P.lat_lo = 21000;
  P.lat_hi = 13000000;
  P.lat_asym = 1;
  P.md_sub = 1;
  P.md_mk_levels = 5;
  P.md_mom_levels = 1;
  P.md_freq = 10 * NS;
  P.L.lat_len = 2 * P.n_agents;
}

// config/obi_rmsc02.py: rmsc02's market (subscribing market maker, latency matrix, midnight-17:00)
// with 89 ZI agents, 5 OrderBookImbalanceAgent (10 levels every hour, entry 0.17, trail 0.085,
// 1 s wake frequency, starting cash 1e7) and 5 subscribing momentum agents; no HBL
constexpr void params_obi_rmsc02(MxaParams& P) {
  params_rmsc02(P);
  P.config = MXA_CFG_OBI_RMSC02;
  P.ex_log_orders = 0;  // config/obi_rmsc02.py:86
  P.zi_group_count[0] = 89;
  P.n_zi = 89;
  P.first_hbl = 0;
  P.n_hbl = 0;
  P.first_obi = 91;
  P.n_obi = 5;
  P.obi_levels = 10;
  P.obi_freq = 3600 * NS;
  P.obi_wake = NS;
  P.obi_entry = 0.17;
  P.obi_trail = 0.085;
  P.first_mom = 96;
  P.n_mom = 5;
  P.L.oh_cap = 0;
  P.L.hbl_range = 0;
}

constexpr uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

// per-env HBM block: header, agent records, open orders, RNG streams, latency row/col,
// saved queue, saved book, transaction ring, then the optional trace (runtime-sized, last)
constexpr void layout(MxaParams& P, int cfg) {
  const Shape S = shape(cfg);
  Layout& L = P.L;
  P.n_streams = 4 + P.n_agents;
  L.n_agents = P.n_agents;
  L.n_streams = P.n_streams;
  L.qcap = S.sq * 64;
  L.ocap = S.so * 64;
  L.trace_cap = 0;
  uint64_t off = align_up(sizeof(EnvHdr), 256);
  L.off_ag = (uint32_t)off;
  off = align_up(off + (uint64_t)P.n_agents * 512, 256);
  L.off_open = (uint32_t)off;
  off = align_up(off + (uint64_t)P.n_agents * L.open_cap * sizeof(OpenOrder), 256);
  L.off_rng = (uint32_t)off;
  off = align_up(off + (uint64_t)P.n_streams * MXA_RNG_WORDS * 4, 256);
  L.off_lat = (uint32_t)off;
  off = align_up(off + (uint64_t)L.lat_len * 8, 256);
  L.off_q = (uint32_t)off;
  off = align_up(off + (uint64_t)L.qcap * sizeof(SavedEvent) + (S.pl ? 0 : (uint64_t)L.qcap * 4 * S.pw) +
                     (uint64_t)(S.sq - sq_lds(cfg)) * 64 * 12,  // HBM queue tier: keys, then sequence numbers
                 256);
  L.off_book = (uint32_t)off;
  off = align_up(off + (uint64_t)L.ocap * sizeof(SavedOrder), 256);
  L.off_tx = (uint32_t)off;
  off = align_up(off + 64 + (uint64_t)L.tx_cap * sizeof(TxRec), 256);
  L.off_oh = off;  // order-history ring (HBL configs; oh_cap = 0 otherwise)
  off = align_up(off + (uint64_t)L.oh_cap * sizeof(OhRec), 256);
  L.off_hh = off;  // HBL price histogram (zeroed between uses)
  off = align_up(off + (uint64_t)L.hbl_range * 8, 256);
  L.off_sub = off;  // market-data subscriptions (md_sub configs)
  off = align_up(off + (P.md_sub ? (uint64_t)MD_MAX_SUBS * sizeof(SubRec) : 0), 256);
  L.off_md = off;
  off = align_up(off + (P.md_sub ? (uint64_t)P.n_agents * MD_WORDS * 4 : 0), 256);
  L.off_trace = (uint32_t)off;
  L.env_stride = off;  // without trace; the handle adds trace_cap records
}

// config/value_noise.py:45-200 (argparse defaults; obs_noise 1e6): 1 exchange, 100 noise and 50
// value agents on JPM, market 09:30-10:30, kernel midnight-17:00, compute delay 1 s, latency
// matrix U(21000, 13e6) symmetrised (only the exchange row is read), 6-way uniform noise.
// ValueAgents take their default starting_cash (ValueAgent.py:17).
constexpr void params_value_noise(MxaParams& P) {
  base_params(P);
  P.config = MXA_CFG_VALUE_NOISE;
  P.ex_log_orders = 0;  // config/value_noise.py:177 the -o option (off)
  P.mkt_close = 10 * HOUR + 30 * MIN;
  P.start = 0;
  P.stop = 17 * HOUR;
  P.default_comp_delay = 1000000000;
  P.lat_mode = 1;
  P.noise_len = 6;
  P.lat_lo = 21000;
  P.lat_hi = 13000000;
  P.first_noise = 1;
  P.n_noise = 100;
  P.first_value = 101;
  P.n_value = 50;
  P.n_agents = 151;
  P.v_sigma_n = 1000000.0;
  P.v_rbar = 1e5;
  P.v_kappa = 1.67e-15;
  P.v_sigma_s = 1e-4;
  P.v_lambda = 1e-12;
  P.v_percent_aggr = 0.1;
  P.v_depth_spread = 2;
  P.v_starting_cash = 100000;
  P.L.open_cap = 8;
  P.L.tx_cap = 256;
  P.L.lat_len = P.n_agents;
}

constexpr MxaParams params_builtin(int cfg) {
  MxaParams P{};
  if (cfg == MXA_CFG_RMSC03) params_rmsc03(P);
  else if (cfg == MXA_CFG_RMSC03_MM) params_rmsc03_mm(P);
  else if (cfg == MXA_CFG_RMSC03_SBMM || cfg == MXA_CFG_RMSC03_SBMM_POLL) params_rmsc03_sbmm(P, cfg == MXA_CFG_RMSC03_SBMM);
  else if (cfg == MXA_CFG_RMSC03_RL) params_rmsc03_rl(P);
  else if (cfg == MXA_CFG_MARKETREPLAY) params_marketreplay(P);
  else if (cfg == MXA_CFG_MARKETREPLAY_RUNNER) params_marketreplay_runner(P);
  else if (cfg == MXA_CFG_MARKETREPLAY_TWAP) params_marketreplay_twap(P);
  else if (cfg == MXA_CFG_VALUE_NOISE) params_value_noise(P);
  else if (cfg == MXA_CFG_RMSC01) params_rmsc01(P);
  else if (cfg == MXA_CFG_RMSC02) params_rmsc02(P);
  else if (cfg == MXA_CFG_OBI_RMSC02) params_obi_rmsc02(P);
  else if (cfg == MXA_CFG_RANDOM_FUND_VALUE) params_random_fund_value(P);
  else if (cfg == MXA_CFG_RANDOM_FUND_DIVERSE) params_random_fund_diverse(P);
  else if (cfg == MXA_CFG_HIST_FUND_VALUE) params_hist_fund(P, false);
  else if (cfg == MXA_CFG_HIST_FUND_DIVERSE) params_hist_fund(P, true);
  else params_sparse_zi(P, cfg == MXA_CFG_SPARSE_ZI_1000);
  return P;
}

// ---- runtime compositions (include/mxa.h mxa_config): a base script's construction with the
// caller's counts and parameters.  The engine is specialised per composition (mxa_config_compile:
// the translation unit of the base configuration, compiled with MXA_CUSTOM_HDR naming the
// composition), so these functions run both on the host and as constant expressions.
constexpr bool custom_base_ok(int b) {
  return b == MXA_CFG_RMSC03 || b == MXA_CFG_VALUE_NOISE || b == MXA_CFG_SPARSE_ZI_100 || b == MXA_CFG_SPARSE_ZI_1000;
}
constexpr bool custom_zi(int b) { return b == MXA_CFG_SPARSE_ZI_100 || b == MXA_CFG_SPARSE_ZI_1000; }

// the base script's values as a composition (mxa_config_defaults)
constexpr void config_defaults(int base, mxa_config& c) {
  const MxaParams P = params_builtin(base);
  c = mxa_config{};
  c.base = base;
  c.log_orders = P.ex_log_orders;
  c.n_noise = P.n_noise;
  c.n_value = P.n_value;
  c.n_mm = P.n_mm;
  c.n_momentum = P.n_mom;
  c.n_zi_groups = custom_zi(base) ? P.zi_ngroups : 0;
  c.zi_q_max = P.zi_qmax ? P.zi_qmax : 10;
  for (int g = 0; g < MXA_CONFIG_ZI_GROUPS; g++) {
    c.zi_count[g] = g < c.n_zi_groups ? P.zi_group_count[g] : 0;
    c.zi_r_min[g] = g < c.n_zi_groups ? P.zi_rmin[g] : 0;
    c.zi_r_max[g] = g < c.n_zi_groups ? P.zi_rmax[g] : 0;
    c.zi_eta[g] = g < c.n_zi_groups ? P.zi_eta[g] : 0.0;
  }
  c.zi_sigma_n = P.zi_sigma_n;
  c.zi_r_bar = P.zi_rbar;
  c.zi_kappa = P.zi_kappa;
  c.zi_sigma_s = P.zi_sigma_s;
  c.zi_sigma_pv = P.zi_sigma_pv;
  c.zi_lambda_a = P.zi_lambda;
  c.mkt_open_ns = P.mkt_open;
  c.mkt_close_ns = P.mkt_close;
  c.kernel_start_ns = P.start;
  c.kernel_stop_ns = P.stop;
  c.noise_wake_open_ns = P.noise_open;
  c.noise_wake_close_ns = P.noise_close;
  c.date_ns = 1561680000LL * NS;  // 2019-06-28, the date of the scripts' runs (-d 20190628)
  c.starting_cash = P.starting_cash;
  c.default_computation_delay_ns = P.default_comp_delay;
  c.r_bar = P.o_rbar;
  c.kappa = P.o_kappa;
  c.fund_vol = P.o_fundvol;
  c.megashock_lambda_a = P.o_lambda;
  c.megashock_mean = P.o_msmean;
  c.megashock_var = P.o_msvar;
  c.value_sigma_n = P.v_sigma_n;
  c.value_r_bar = P.v_rbar;
  c.value_kappa = P.v_kappa;
  c.value_sigma_s = P.v_sigma_s;
  c.value_lambda_a = P.v_lambda;
  c.value_starting_cash = P.v_starting_cash;
  c.mm.mm_pov = P.mm_pov;
  c.mm.mm_min_order_size = P.mm_min_size;
  c.mm.mm_window_size = P.mm_window;
  c.mm.mm_num_ticks = P.mm_ticks;
  c.mm.mm_wake_up_freq_ns = P.mm_wake;
  c.mom_min_size = P.mom_min;
  c.mom_max_size = P.mom_max;
  c.mom_wake_up_freq_ns = P.mom_wake;
  c.lat_low = P.lat_lo;
  c.lat_high = P.lat_hi;
  c.queue_capacity = 0;
  c.book_capacity = 0;
}

constexpr int custom_n_agents(const mxa_config& c) {
  int n = 1 + c.n_noise + c.n_value + c.n_mm + c.n_momentum;
  for (int g = 0; g < c.n_zi_groups && g < MXA_CONFIG_ZI_GROUPS; g++) n += c.zi_count[g];
  return n;
}

// the engine shape: the base script's, with the queue and the book sized for the counts (or the
// caller's capacities).  A full queue or book is an env error, never a silent drop (§4)
constexpr Shape custom_shape(const mxa_config& c) {
  Shape S = shape_builtin(c.base);
  const int n = custom_n_agents(c);
  int zi = 0;
  for (int g = 0; g < c.n_zi_groups && g < MXA_CONFIG_ZI_GROUPS; g++) zi += c.zi_count[g];
  const int ladder = c.n_mm * 2 * (c.mm.mm_num_ticks + 1);  // the POV market maker's cancel + place cycle
  // pending events: one wakeup per agent plus what is in flight; the base scripts' measured peaks
  // (§4: rmsc03 146 of 192 at 64 agents, value_noise 301 of 384 at 151, sparse_zi_1000 2,007 of
  // 2,304 at 1,001) sit under these
  int q = c.queue_capacity > 0 ? c.queue_capacity
        : custom_zi(c.base) || c.base == MXA_CFG_VALUE_NOISE ? 2 * n + 128
                                                              : n + 2 * ladder + 32;
  int sq = (q + 63) / 64;
  if (sq < 2) sq = 2;
  if (sq >= 9 && sq < 16) sq += sq & 1;       // grouped minima: groups of sq / 2 (Eng::QG)
  if (sq >= 16) sq = (sq + 11) / 12 * 12;     // groups of 12
  // resting orders: the market maker's ladder, the value agents' quotes, a few noise orders; ZI
  // books hold ~0.8 orders per agent.  Oracle peaks over 2,048 seeds (r06): rmsc03 with 100 noise /
  // 20 value agents 74 (128 here), rmsc03_alt 58 (128), 60 ZI 52 (128), 199 ZI 160 (256),
  // value_noise_alt 37 (128); the base scripts' own peaks are in DESIGN.md §4
  int b = c.book_capacity > 0 ? c.book_capacity
        : custom_zi(c.base) ? (3 * zi) / 4 + 64
                            : ladder + 2 * c.n_value + c.n_noise / 8 + 32;
  int so = (b + 63) / 64;
  if (so < 1) so = 1;
  S.sq = sq;
  S.so = so;
  S.sql = 0;
  // queue payloads in LDS up to 12 slots per lane (sparse_zi_1000's 36 keep them in HBM)
  S.pl = sq <= 12;
  // the register budget: the base's waves per SIMD while the book fits its VGPRs
  if (so > 2 && S.waves > 2) S.waves = 2;
  if ((so > 6 || sq > 12) && S.waves > 1) S.waves = 1;
  return S;
}

// 0, or why the composition cannot be built (mxa_config_compile / mxa_create_config: MXA_EINVAL)
constexpr const char* custom_check(const mxa_config& c) {
  if (!custom_base_ok(c.base)) return "base must be MXA_RMSC03, MXA_VALUE_NOISE, MXA_SPARSE_ZI_100 or MXA_SPARSE_ZI_1000";
  if (c.n_noise < 0 || c.n_value < 0 || c.n_mm < 0 || c.n_momentum < 0 || c.n_zi_groups < 0) return "negative count";
  if (c.n_zi_groups > MXA_CONFIG_ZI_GROUPS) return "more than MXA_CONFIG_ZI_GROUPS ZI groups";
  for (int g = 0; g < c.n_zi_groups; g++)
    if (c.zi_count[g] < 0 || c.zi_r_min[g] < 0 || c.zi_r_max[g] < c.zi_r_min[g] || !(c.zi_eta[g] >= 0))
      return "ZI group: count >= 0, 0 <= R_min <= R_max, eta >= 0";
  if (custom_zi(c.base)) {
    if (c.n_noise || c.n_value || c.n_mm || c.n_momentum) return "sparse_zi bases hold ZI agents only";
    if (c.n_zi_groups < 1) return "sparse_zi bases need a ZI strategy table";
    if (c.zi_q_max < 1 || c.zi_q_max > 10) return "zi_q_max in 1..10";
    if (!(c.zi_sigma_pv >= 0) || !(c.zi_lambda_a > 0) || !(c.zi_sigma_n >= 0)) return "ZI parameters";
  } else {
    if (c.n_zi_groups) return "ZI groups belong to the sparse_zi bases";
    if (c.base == MXA_CFG_VALUE_NOISE && (c.n_mm || c.n_momentum)) return "value_noise holds noise and value agents";
    if (c.n_mm > 1) return "at most one POVMarketMakerAgent";
    if (c.n_mm && (c.mm.mm_window_size < 0 || c.mm.mm_num_ticks < 0 || c.mm.mm_num_ticks > 60 ||
                   c.mm.mm_wake_up_freq_ns <= 0 || !(c.mm.mm_pov >= 0) || c.mm.mm_min_order_size < 0))
      return "market maker options (num_ticks <= 60)";
    if (c.n_momentum && (c.mom_min_size < 0 || c.mom_max_size <= c.mom_min_size || c.mom_wake_up_freq_ns <= 0))
      return "momentum options: 0 <= min_size < max_size, wake_up_freq > 0";
    if (!(c.value_lambda_a > 0) || !(c.value_sigma_n >= 0)) return "value agent parameters";
  }
  const int n = custom_n_agents(c);
  if (n < 2 || n > MXA_MAX_AGENTS) return "2 to 8191 agents";
  if (c.mkt_open_ns < 0 || c.mkt_close_ns <= c.mkt_open_ns || c.kernel_start_ns < 0 || c.kernel_stop_ns < c.kernel_start_ns ||
      c.kernel_stop_ns >= (1LL << 47))
    return "session: 0 <= mkt_open < mkt_close, 0 <= kernel_start <= kernel_stop < 2^47 ns";
  if (c.base == MXA_CFG_RMSC03 && c.noise_wake_close_ns < c.noise_wake_open_ns) return "noise wake window";
  if (!(c.megashock_lambda_a > 0) || !(c.megashock_var >= 0) || !(c.fund_vol >= 0)) return "oracle parameters";
  if (c.default_computation_delay_ns < 0 || c.starting_cash < 0) return "delay / cash";
  if (!custom_zi(c.base) && c.base != MXA_CFG_VALUE_NOISE && (c.lat_low != 0 || c.lat_high != 0)) {
    // rmsc03's latency is zeros (no draw); the field is not used there
  }
  if ((c.base != MXA_CFG_RMSC03) && !(c.lat_high >= c.lat_low && c.lat_low >= 0)) return "latency bounds";
  const Shape S = custom_shape(c);
  if (S.sq > 128) return "more than 128 queue slots per lane (8,192 pending events)";
  if (S.so > 16) return "more than 16 book slots per lane (1,024 resting orders)";
  return nullptr;
}

// the parameter block of a composition (before the layout)
constexpr MxaParams custom_params_raw(const mxa_config& c) {
  MxaParams P = params_builtin(c.base);
  P.ex_log_orders = c.log_orders ? 1 : 0;
  P.mkt_open = c.mkt_open_ns;
  P.mkt_close = c.mkt_close_ns;
  P.start = c.kernel_start_ns;
  P.stop = c.kernel_stop_ns;
  P.starting_cash = c.starting_cash;
  P.default_comp_delay = c.default_computation_delay_ns;
  P.o_rbar = c.r_bar;
  P.o_kappa = c.kappa;
  P.o_fundvol = c.fund_vol;
  P.o_lambda = c.megashock_lambda_a;
  P.o_msmean = c.megashock_mean;
  P.o_msvar = c.megashock_var;
  P.lat_lo = c.lat_low;
  P.lat_hi = c.lat_high;
  P.first_noise = P.n_noise = P.first_value = P.n_value = P.first_mm = P.n_mm = P.first_mom = P.n_mom = 0;
  P.first_zi = P.n_zi = 0;
  int a = 1;
  if (custom_zi(c.base)) {
    P.zi_ngroups = c.n_zi_groups;
    int nz = 0;
    for (int g = 0; g < 8; g++) {
      const bool on = g < c.n_zi_groups;
      P.zi_group_count[g] = on ? c.zi_count[g] : 0;
      P.zi_rmin[g] = on ? c.zi_r_min[g] : 0;
      P.zi_rmax[g] = on ? c.zi_r_max[g] : 0;
      P.zi_eta[g] = on ? c.zi_eta[g] : 0.0;
      nz += P.zi_group_count[g];
    }
    P.first_zi = 1;
    P.n_zi = nz;
    a += nz;
    P.zi_qmax = c.zi_q_max;
    P.zi_sigma_n = c.zi_sigma_n;
    P.zi_rbar = c.zi_r_bar;
    P.zi_kappa = c.zi_kappa;
    P.zi_sigma_s = c.zi_sigma_s;
    P.zi_sigma_pv = c.zi_sigma_pv;
    P.zi_lambda = c.zi_lambda_a;
  } else {
    P.n_noise = c.n_noise;
    P.first_noise = c.n_noise ? a : 0;
    a += c.n_noise;
    P.n_value = c.n_value;
    P.first_value = c.n_value ? a : 0;
    a += c.n_value;
    P.n_mm = c.n_mm;
    P.first_mm = c.n_mm ? a : 0;
    a += c.n_mm;
    P.n_mom = c.n_momentum;
    P.first_mom = c.n_momentum ? a : 0;
    a += c.n_momentum;
    P.noise_open = c.noise_wake_open_ns;
    P.noise_close = c.noise_wake_close_ns;
    P.v_sigma_n = c.value_sigma_n;
    P.v_rbar = c.value_r_bar;
    P.v_kappa = c.value_kappa;
    P.v_sigma_s = c.value_sigma_s;
    P.v_lambda = c.value_lambda_a;
    P.v_starting_cash = c.value_starting_cash;
    P.mm_pov = c.mm.mm_pov;
    P.mm_min_size = c.mm.mm_min_order_size;
    P.mm_window = c.mm.mm_window_size;
    P.mm_ticks = c.mm.mm_num_ticks;
    P.mm_wake = c.mm.mm_wake_up_freq_ns;
    P.mom_min = c.mom_min_size;
    P.mom_max = c.mom_max_size;
    P.mom_wake = c.mom_wake_up_freq_ns;
  }
  P.n_agents = a;
  // the latency rows the engine reads: exchange row and column (cubic model), the exchange row
  // of the symmetric matrix, none for zero latency
  P.L.lat_len = c.base == MXA_CFG_SPARSE_ZI_100 ? 2 * a : (c.base == MXA_CFG_RMSC03 ? 0 : a);
  // open orders per agent: the market maker's cancelled ladder stays in TradingAgent.orders until
  // ORDER_CANCELLED (twice its ladder), the base's otherwise
  if (c.n_mm) {
    const int need = 4 * (c.mm.mm_num_ticks + 1) + 16;
    int cap = 64;
    while (cap < need) cap *= 2;
    if (cap > P.L.open_cap) P.L.open_cap = cap;
  }
  // the transaction ring: the base's, and more for a crowded book
  if (a > 256 && P.L.tx_cap < 512) P.L.tx_cap = 512;
  return P;
}

#ifdef MXA_CUSTOM_HDR
// the composition of this specialisation (mxa_config_compile): its bytes, and the base it follows
#include MXA_CUSTOM_HDR
struct CustomBytes {
  unsigned char b[sizeof(mxa_config)];
};
constexpr mxa_config custom_cfg() { return __builtin_bit_cast(mxa_config, CustomBytes{MXA_CUSTOM_BYTES}); }
static_assert(custom_cfg().base == MXA_INST_CFG, "the specialisation is compiled in its base's translation unit");
static_assert(custom_check(custom_cfg()) == nullptr, "a composition mxa_config_compile accepted");
constexpr bool is_custom(int cfg) { return cfg == MXA_INST_CFG; }
#else
constexpr bool is_custom(int) { return false; }
constexpr mxa_config custom_cfg() { return mxa_config{}; }
#endif
constexpr Shape shape(int cfg) { return is_custom(cfg) ? custom_shape(custom_cfg()) : shape_builtin(cfg); }
constexpr MxaParams params(int cfg) {
  MxaParams P = is_custom(cfg) ? custom_params_raw(custom_cfg()) : params_builtin(cfg);
  layout(P, cfg);
  return P;
}
// doubles of the latency row held in LDS (MXA_LAT_LDS_MASK): the exchange's row of a symmetric
// matrix (lat_mode 1 without lat_asym), else none
constexpr int lat_lds(int cfg) {
  return (((MXA_LAT_LDS_MASK) >> cfg) & 1) && params(cfg).lat_mode == 1 && !params(cfg).lat_asym ? (int)params(cfg).L.lat_len : 0;
}

// runtime stride of one env block with `trace_cap` trace records
constexpr uint64_t env_stride(int cfg, int trace_cap) {
  return align_up(params(cfg).L.off_trace + (uint64_t)trace_cap * MXA_TRACE_WORDS * 8, 256);
}

// replay sections appended after the trace: header, ladder (count/head/tail/qty per side),
// entry pool + free stack, per-dense-id live-entry chain heads and entry epochs, the replay
// agent's orders, the RL metrics deque
inline RpLayout replay_layout(uint64_t base, int pmin, int P, int C, int n_ids, int agent_ids, int ntm, int nrec) {
  RpLayout L{};
  L.pmin = pmin;
  L.P = P;
  L.C = C;
  L.n_ids = n_ids;
  L.D = n_ids + agent_ids;
  L.ntm = ntm;
  L.nrec = nrec;
  uint64_t off = align_up(base, 256);
  L.off_rh = off;
  off = align_up(off + sizeof(RpHdr), 256);
  L.off_lvc = off;
  off = align_up(off + 2ull * P * 4, 256);
  L.off_lvh = off;
  off = align_up(off + 2ull * P * 4, 256);
  L.off_lvt = off;
  off = align_up(off + 2ull * P * 4, 256);
  L.off_lvq = off;
  off = align_up(off + 2ull * P * 8, 256);
  L.off_pool = off;
  off = align_up(off + (uint64_t)C * sizeof(RpEntry), 256);
  L.off_free = off;
  off = align_up(off + (uint64_t)C * 4, 256);
  L.off_idh = off;
  off = align_up(off + (uint64_t)L.D * 4, 256);
  L.off_idep = off;
  off = align_up(off + (uint64_t)L.D * MXA_ID_EPOCHS * 4, 256);
  L.off_mro = off;
  off = align_up(off + (uint64_t)L.D * sizeof(RpOrder), 256);
  L.off_ring = off;
  off = align_up(off + 100 * sizeof(RpLob), 256);
  L.end = off;
  return L;
}

}  // namespace mxa_cfg
