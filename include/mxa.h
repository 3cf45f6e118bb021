/* mxa.h — C-ABI of libmxa, the MI355X-native vectorised ABIDES market step.
 *
 * One handle = n_envs independent markets (envs) of one configuration on one GPU,
 * simulated by HIP kernels (one wavefront per env).  Plain pointers and sizes only; the
 * caller owns every host array.  Every entry point returns 0 on success or a negative
 * MXA_E* code; mxa_last_error() gives the message.  A handle is bound to one device and
 * one HIP stream and is not thread-safe; multi-GPU runs use one process per GPU.
 *
 * Reference interfaces replaced (file:line in yutiansut/marl-optimal-execution):
 *   mxa_create ......... config/{rmsc01,rmsc02,obi_rmsc02,rmsc03,sparse_zi_100,sparse_zi_1000,value_noise}.py module body
 *   mxa_create_params .. config/rmsc03.py with its --mm-* options (config/rmsc03.py:39-43), per env
 *                        (and rmsc03 with SpreadBasedMarketMakerAgent.py:17-297, MXA_RMSC03_SBMM*)
 *                        (agent/oracle/kernel construction, global-RNG draw order) and
 *                        Kernel.__init__ (Kernel.py:13-46)
 *   mxa_create_config .. a config script's agent list given at run time: Kernel.runner(agents, ...)
 *                        (Kernel.py:50-64) built as config/rmsc03.py:95-197, config/value_noise.py,
 *                        config/sparse_zi_100.py:177-334 build theirs (counts, parameters, session)
 *   mxa_reset .......... Kernel.runner kernelInitializing/kernelStarting (Kernel.py:143-177),
 *                        ABIDESEnv.reset (ABIDESEnv.py:51-57)
 *   mxa_run / mxa_launch Kernel.runner event loop (Kernel.py:190-292)
 *   mxa_read_summary ... Kernel.runner's ttl_messages / currentTime (Kernel.py:211, 321-326)
 *   mxa_read_agents .... TradingAgent.holdings / orders (TradingAgent.py:45-46, 112-138)
 *   mxa_read_book ...... OrderBook.bids / asks (util/OrderBook.py:24-25, 377-398)
 *   mxa_read_trace ..... (parity tooling; no reference equivalent)
 *   mxa_finalize ....... Kernel.runner's kernelStopping loop (Kernel.py:305-312): agents'
 *                        FINAL_VALUATION, the summary log of Kernel.writeSummaryLog (Kernel.py:549-565)
 *   mxa_create_replay .. ABIDESEnv.__init__/reset (ABIDESEnv.py:8-57, 59-103), agent_config.py
 *                        Agents (Exchange, MarketReplayAgent on a LOBSTER tape, DummyRL),
 *                        LOBSTEROrdersProcessor output (MarketReplayAgent.py:162-220)
 *   mxa_create(MXA_RMSC03_RL) config/rmsc03.py agents + DummyRLExecutionAgent
 *                        (dummy_rl_execution_agent.py:77-137) + GymKernel.initRunner (GymKernel.py:24-156)
 *   mxa_step ........... ABIDESEnv.step (ABIDESEnv.py:30-49) = GymKernel.stepRunner
 *                        (GymKernel.py:158-306) with DummyRL.place_orders/get_observation
 *                        (dummy_rl_execution_agent.py:138-179, 291-312)
 *   mxa_step_many ...... k ABIDESEnv.step calls in a row with the actions given up front, one launch
 */
#ifndef MXA_H
#define MXA_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct mxa_handle mxa_handle;

/* MXA_RMSC03_RL: rmsc03's 64 agents + DummyRLExecutionAgent 64 under a GymKernel (BASELINE.json
 * configs[3]; composition of tests/golden/gen_rl_fixtures.py).  Created by mxa_create like
 * the plain configs (per-env seeds), advanced by mxa_step / mxa_step_device like a replay handle. */
enum { MXA_RMSC03 = 0, MXA_SPARSE_ZI_100 = 1, MXA_SPARSE_ZI_1000 = 2, MXA_MARKETREPLAY = 3, MXA_RMSC03_RL = 4,
       MXA_VALUE_NOISE = 5 /* config/value_noise.py: 100 noise + 50 value agents, latency matrix */,
       MXA_RMSC01 = 6 /* config/rmsc01.py: market maker, 50 ZI, 25 HBL, 24 momentum agents */,
       MXA_RMSC02 = 7 /* config/rmsc02.py: rmsc01 with market-data subscriptions and a latency matrix */,
       MXA_OBI_RMSC02 = 8 /* config/obi_rmsc02.py: rmsc02's market with 89 ZI, 5 order-book-imbalance agents */,
       MXA_RANDOM_FUND_VALUE = 9 /* config/random_fund_value.py: 5000 noise + 100 value agents, 09:30-16:00 */,
       MXA_RANDOM_FUND_DIVERSE = 10 /* config/random_fund_diverse.py: random_fund_value + market maker + 25 momentum */,
       MXA_HIST_FUND_VALUE = 11 /* config/hist_fund_value.py: random_fund_value on an ExternalFileOracle (mxa_create_hist) */,
       MXA_HIST_FUND_DIVERSE = 12 /* config/hist_fund_diverse.py: random_fund_diverse on an ExternalFileOracle */,
       MXA_MARKETREPLAY_RUNNER = 13 /* config/marketreplay.py: exchange + MarketReplayAgent under Kernel.runner */,
       MXA_MARKETREPLAY_TWAP = 14 /* config/execution/marketreplay/execution_marketreplay.py: + TWAPExecutionAgent */,
       /* config/rmsc03.py with agent/market_makers/SpreadBasedMarketMakerAgent.py in the market maker's
        * slot (no reference config uses that agent; composition of tests/golden/gen_fixtures.py):
        * subscribe=True (level-1 MARKET_DATA every 10 s) and the polling mode (QUERY_SPREAD every second) */
       MXA_RMSC03_SBMM = 15, MXA_RMSC03_SBMM_POLL = 16,
       /* config/rmsc03.py with per-env market-maker options: the handles of mxa_create_params.
        * mxa_create(MXA_RMSC03_MM, ...) gives every env the script's defaults (mxa_mm_defaults) */
       MXA_RMSC03_MM = 17 };
enum {
  MXA_OK = 0, MXA_EINVAL = -1, MXA_EHIP = -2, MXA_ENOMEM = -3, MXA_ERANGE = -4
};
/* per-env status */
enum { MXA_ENV_RUNNING = 0, MXA_ENV_DONE = 1, MXA_ENV_ERROR = 2 };

typedef struct {
  int32_t status;        /* MXA_ENV_* */
  int32_t err;           /* capacity overflow / reference-crash code when status == ERROR */
  int64_t events;        /* Kernel pops so far (ttl_messages, incl. busy requeues) */
  uint64_t hash;         /* rolling FNV-1a-64 over the 10-word trace records */
  int64_t current_time;  /* Kernel.currentTime, ns since midnight of the simulated date */
  int64_t order_counter; /* next order id (Order.order_id + 1) */
  int64_t last_trade;    /* OrderBook.last_trade (cents) */
  int32_t max_queue, max_book; /* high-water marks of pending events / resting orders */
} mxa_env_summary;

typedef struct {
  int64_t cash, shares, n_open;
  int64_t last_trade;    /* the agent's last known trade price (TradingAgent.last_trade) */
  int32_t type, flags;   /* agent class, TradingAgent state flags (mxa_layout.h FL_*) */
  int64_t starting_cash; /* TradingAgent.starting_cash (the base of Kernel's mean ending value) */
} mxa_agent_state;

/* one agent's kernelStopping valuation (Kernel.runner's after-loop pass, Kernel.py:305-312) */
typedef struct {
  int64_t final_fundamental; /* oracle.observePrice(sym, currentTime, sigma_n=0) (ZI, Value), else 0 */
  int64_t valuation_int;     /* FINAL_VALUATION when the reference logs an int (ZeroIntelligenceAgent) */
  double valuation;          /* FINAL_VALUATION when it logs a float (NoiseAgent, ValueAgent) */
  int32_t kind;              /* 0 no FINAL_VALUATION, 1 int, 2 float */
  int32_t err;               /* nonzero where the reference raises: 1 KeyError (no known quote), 2 IndexError */
} mxa_agent_final;

/* configuration id + per-env seeds (the reference config's -s/--seed) */
int mxa_create(int32_t config, int32_t n_envs, const uint32_t* seeds, int32_t device,
               int32_t trace_cap, mxa_handle** out);
/* MXA_HIST_FUND_VALUE / MXA_HIST_FUND_DIVERSE: the configuration with its ExternalFileOracle series
 * (util/oracle/ExternalFileOracle.py:15-35 reads it from a pickled pandas Series of mid prices,
 * util/formatting/mid_price_from_orderbook.py): n_fund time-sorted entries, fund_t ns since
 * midnight of the simulated date, fund_v the values (cents, float).  Prices between entries are
 * interpolated exactly as getPriceAtTime / getInterpolatedPrice do (ExternalFileOracle.py:52-159). */
int mxa_create_hist(int32_t config, int32_t n_envs, const uint32_t* seeds, int32_t device, int32_t trace_cap,
                    const int64_t* fund_t, const double* fund_v, int32_t n_fund, mxa_handle** out);
/* config/rmsc03.py's market-maker options (config/rmsc03.py:39-43, 158-177), the parameters its
 * only driver script sweeps (scripts/rmsc03.sh:5-13, 29-39).  They reach POVMarketMakerAgent.__init__
 * only (POVMarketMakerAgent.py:19-60) and change no draw. */
typedef struct {
  double mm_pov;               /* --mm-pov (default 0.05) */
  int32_t mm_min_order_size;   /* --mm-min-order-size (20) */
  int32_t mm_window_size;      /* --mm-window-size (5) */
  int32_t mm_num_ticks;        /* --mm-num-ticks (20): a ladder of 2 * (num_ticks + 1) orders */
  int32_t pad;
  int64_t mm_wake_up_freq_ns;  /* --mm-wake-up-freq as pd.Timedelta(freq).value ("1S": 1e9) */
} mxa_mm_params;
mxa_mm_params mxa_mm_defaults(void);
/* config/rmsc03.py -s seeds[i] --mm-* per_env[i] for every env i: a parameter sweep is one batch.
 * config must be MXA_RMSC03; the handle's instantiation (MXA_RMSC03_MM) reads the options from the
 * market maker's record and holds 320 pending events, 192 resting orders and 256 open orders per
 * agent (scripts/rmsc03.sh's 50 ticks peak at 266 / 122 / 204); beyond that an env stops with a
 * capacity error, never silently.  MXA_EINVAL for options the script cannot run (negative
 * window or ticks, wake-up period <= 0). */
int mxa_create_params(int32_t config, int32_t n_envs, const uint32_t* seeds, const mxa_mm_params* per_env,
                      int32_t device, int32_t trace_cap, mxa_handle** out);
/* A Kernel.runner composition given at run time (SURVEY.md §8(b) "mxa_config"): the agent list a
 * config script builds (Kernel.runner(agents, startTime, stopTime, ...), Kernel.py:50-64) from the
 * existing agent classes, with its counts, per-class parameters, session times and date.  `base`
 * names the script whose construction (global-RNG draw order, latency model) it follows:
 *   MXA_RMSC03        config/rmsc03.py:95-197 (config/random_fund_value.py is the same
 *                     construction): exchange, n_noise NoiseAgent (util.get_wake_time in the noise
 *                     window), n_value ValueAgent, n_mm POVMarketMakerAgent (0 or 1), n_momentum
 *                     MomentumAgent; zero latency, compute delay 0
 *   MXA_VALUE_NOISE   config/value_noise.py:45-200: exchange, n_noise, n_value; latency matrix
 *                     G.uniform(lat_low, lat_high) with 6-way noise, compute delay
 *   MXA_SPARSE_ZI_100 config/sparse_zi_100.py:177-334: exchange and the ZI strategy table (count,
 *                     R_min, R_max, eta per group); cubic LatencyModel (min_latency U(lat_low, lat_high))
 *   MXA_SPARSE_ZI_1000 config/sparse_zi_1000.py: the same agents on the symmetric matrix latency
 * Agent ids follow the scripts' order.  mxa_config_defaults fills the base script's values; a
 * caller edits what its script changes.  Times are ns since midnight of the simulated date. */
#define MXA_CONFIG_ZI_GROUPS 8
typedef struct {
  int32_t base;               /* MXA_RMSC03, MXA_VALUE_NOISE, MXA_SPARSE_ZI_100, MXA_SPARSE_ZI_1000 */
  int32_t log_orders;         /* ExchangeAgent(log_orders=...) (what the exchange log records) */
  int32_t n_noise, n_value;   /* NoiseAgent / ValueAgent counts (rmsc03, value_noise) */
  int32_t n_mm, n_momentum;   /* POVMarketMakerAgent (0 or 1) / MomentumAgent counts (rmsc03) */
  int32_t n_zi_groups;        /* ZI strategy table rows (sparse_zi_*), at most MXA_CONFIG_ZI_GROUPS */
  int32_t zi_q_max;           /* ZeroIntelligenceAgent q_max (1..10) */
  int32_t zi_count[MXA_CONFIG_ZI_GROUPS], zi_r_min[MXA_CONFIG_ZI_GROUPS], zi_r_max[MXA_CONFIG_ZI_GROUPS];
  double zi_eta[MXA_CONFIG_ZI_GROUPS];
  double zi_sigma_n, zi_r_bar, zi_kappa, zi_sigma_s, zi_sigma_pv, zi_lambda_a;
  int64_t mkt_open_ns, mkt_close_ns;          /* the exchange's (and the oracle's) session */
  int64_t kernel_start_ns, kernel_stop_ns;    /* Kernel.runner(startTime, stopTime) */
  int64_t noise_wake_open_ns, noise_wake_close_ns; /* rmsc03: get_wake_time(noise_mkt_open, noise_mkt_close) */
  int64_t date_ns;            /* the -d historical date (its midnight, ns since the Unix epoch): output timestamps only */
  int64_t starting_cash;      /* TradingAgent starting_cash (cents) */
  int64_t default_computation_delay_ns;
  /* SparseMeanRevertingOracle symbols dict: r_bar, kappa, fund_vol, megashock_lambda_a, _mean, _var */
  double r_bar, kappa, fund_vol, megashock_lambda_a, megashock_mean, megashock_var;
  double value_sigma_n, value_r_bar, value_kappa, value_sigma_s, value_lambda_a;
  int64_t value_starting_cash;
  mxa_mm_params mm;           /* POVMarketMakerAgent (config/rmsc03.py's --mm-* options) */
  int32_t mom_min_size, mom_max_size;
  int64_t mom_wake_up_freq_ns;
  double lat_low, lat_high;   /* G.uniform bounds of the latency matrix / the cubic model's min_latency */
  int32_t queue_capacity, book_capacity; /* pending events / resting orders per env; 0: derived from the counts */
} mxa_config;
/* the base script's own values (MXA_EINVAL for any other config id) */
int mxa_config_defaults(int32_t base, mxa_config* out);
/* The engine is specialised per composition: every count and parameter becomes an immediate of
 * the kernels, as for the built-in configurations.  mxa_config_compile builds the
 * specialisation (hipcc, gfx950; ~40 s) into `cache_dir` (NULL: the lib/custom directory beside
 * libmxa.so) unless it is there already, and writes the library's path to path_out.  It uses no
 * GPU.  MXA_EINVAL for a composition outside the bounds above or the device capacities (8191
 * agents, 128 queue slots and 16 book slots per lane). */
int mxa_config_compile(const mxa_config* cfg, const char* cache_dir, char* path_out, int32_t path_cap);
/* the specialisation's cache key (16 hex digits + NUL: the composition and this library's build id) */
int mxa_config_key(const mxa_config* cfg, char* out17);
/* a plain Kernel.runner handle (mxa_run, mxa_finalize, the readers) of the composition, one env
 * per seed.  Its specialisation must have been compiled (mxa_config_compile, same cache_dir):
 * MXA_ERANGE otherwise, and nothing is compiled here. */
int mxa_create_config(const mxa_config* cfg, int32_t n_envs, const uint32_t* seeds, int32_t device, int32_t trace_cap,
                      const char* cache_dir, mxa_handle** out);
/* per-configuration facts of a built-in configuration id: out8 = (n_agents, ExchangeAgent
 * log_orders, queue capacity, book capacity, mkt_open, mkt_close, kernel start, kernel stop) */
int mxa_config_info(int32_t config, int64_t* out8);
/* replace the options the next mxa_reset builds with (handles of mxa_create_params) */
int mxa_set_mm_params(mxa_handle* h, const mxa_mm_params* per_env);
/* envs of the handle resident on the device at once (run / step kernel occupancy x CUs, at most
 * n_envs): the resident waves of the latency bound */
int mxa_resident_envs(const mxa_handle* h);
/* rebuild envs from their seeds (env_mask: NULL = all) — runs the config construction.  On a
 * GymKernel handle (mxa_create_replay, MXA_RMSC03_RL) a reset is ABIDESEnv.reset in the same
 * process: Order.order_id / Order._order_ids carry over from the env's previous episode
 * (util/order/Order.py:8-9, 27-42), so auto ids continue and skip
 * every id used before; mxa_set_id_persistence(h, 0) makes every reset a fresh process. */
int mxa_reset(mxa_handle* h, const uint8_t* env_mask);
/* GymKernel handles only (MXA_EINVAL otherwise): 1 (the default) = consecutive episodes of one
 * process per env, 0 = every mxa_reset starts a fresh process (order ids from 0) */
int mxa_set_id_persistence(mxa_handle* h, int32_t on);
/* one asynchronous launch: every running env performs up to max_pops kernel pops */
int mxa_launch(mxa_handle* h, int64_t max_pops);
int mxa_sync(mxa_handle* h);
/* launches of `chunk` pops until every env is done/errored (or max_launches reached).  After each
 * launch the envs still running are compacted into a list and the next launch is one wave per
 * listed env, so the CUs share the live envs evenly (envs that end early, e.g. rmsc03's stalled
 * market maker, no longer leave their CU's slots idle while the others run on).  Results do not
 * depend on the launch sizes (the engine saves and reloads its state between launches). */
int mxa_run(mxa_handle* h, int64_t chunk, int32_t max_launches, int32_t* launches_out);
/* mxa_run's launch sizes: first_chunk > 0 makes its first launch first_chunk pops and the later
 * ones `chunk`, so envs that finish early (e.g. rmsc03's stalled market maker) leave the grid
 * after one short launch; 0 (the default) = every launch `chunk` pops.  Kept across resets. */
int mxa_set_launch_schedule(mxa_handle* h, int64_t first_chunk);
/* Kernel.runner(startTime, stopTime) with a caller's stopTime (Kernel.py:50-64, 190-196): every env
 * of a Kernel.runner handle stops at its first pop with currentTime past t_stop_ns (ns since the
 * simulated midnight; that event is handled, as the reference's loop test comes before its get)
 * instead of the config script's kernelStopTime.  Kept across mxa_reset; t_stop_ns <= 0 restores
 * the config's.  Set it before the run: an env already stopped stays stopped.  GymKernel handles:
 * MXA_EINVAL. */
int mxa_set_stop_time(mxa_handle* h, int64_t t_stop_ns);
/* mxa_set_stop_time + mxa_run to the end of every env (chunks of 2^20 pops); events_out
 * (nullable, [n_envs]): each env's ttl_messages.  The §8(b) mxa_run_until entry point. */
int mxa_run_until(mxa_handle* h, int64_t t_stop_ns, int64_t* events_out);
/* Kernel.runner's kernelStopping pass for every env once the run is over: the agents'
 * FINAL_VALUATION entries of the summary log (ZeroIntelligenceAgent.py:80-112, NoiseAgent.py:44-68,
 * ValueAgent.py:66-86), observing the oracle in agent order.  Idempotent (state is not saved);
 * plain Kernel.runner configs only (MXA_EINVAL for GymKernel handles). */
int mxa_finalize(mxa_handle* h);
/* env's rows of the last mxa_finalize, one per agent (row 0, the exchange, is empty) */
int mxa_read_final(mxa_handle* h, int32_t env, mxa_agent_final* out, int32_t cap);
int mxa_read_summary(mxa_handle* h, mxa_env_summary* out /* [n_envs] */);
int mxa_read_agents(mxa_handle* h, int32_t env, mxa_agent_state* out, int32_t cap);
/* book side 0 bids / 1 asks: levels best-first, FIFO within level; each order is
 * (order_id, agent_id, quantity, price).  Returns the total number of orders on the side;
 * min(total, cap) are written (cap 0 / out4 NULL: count only). */
int mxa_read_book(mxa_handle* h, int32_t env, int32_t side, int64_t* out4, int32_t cap);
int mxa_read_trace(mxa_handle* h, int32_t env, int64_t* out /* [cap][10] */, int64_t cap, int64_t* n);
/* replace the per-env seeds used by the next mxa_reset (n_envs values) */
int mxa_set_seeds(mxa_handle* h, const uint32_t* seeds);
/* write the per-env episode record [n_envs][4] int64 = (events, hash, status, current_time)
 * into DEVICE memory on the handle's stream (e.g. a torch tensor to all-gather over RCCL) */
int mxa_write_results(mxa_handle* h, void* device_out);
/* the episode record each rank contributes to the multi-GPU all-gather (replaces
 * config/parallel.py:15-25's one-process-per-simulation result collection): DEVICE array
 * [n_envs][MXA_RECORD_WORDS] int64 = (events, hash, status, current_time, err, seed, last_trade,
 * order_counter, cash, holdings, gain, 0).  cash / holdings / gain: sums over the trading agents
 * 1.. of TradingAgent.holdings['CASH'], the share position and markToMarket - starting_cash
 * (TradingAgent.py:609-633; Kernel.py:330-341 averages the gain per agent type) for Kernel.runner
 * handles, the execution agent's own for GymKernel handles; word 11 is the caller's (a learner's
 * episode return).  Asynchronous on the handle's stream. */
#define MXA_RECORD_WORDS 12
int mxa_write_records(mxa_handle* h, void* device_out);
/* event-class counters since the envs' last reset, kept by instrumented runs only (parity hash on
 * or a trace ring; the measured kernels carry none of it): HOST array [n_envs][MXA_COUNTER_WORDS]
 * int64 = pops per message kind MK_0..MK_24 (WAKEUP pops at 0, GymKernel CANCEL_ORDER at 19),
 * busy requeues (25), events pushed (26), RNG words drawn (27), pops (28), max pending events
 * (29), max resting orders (30), agent-record round trips (31), pops handled inside batched event
 * runs (32), 0.  The inputs of the SURVEY.md §8(d) algorithmic-byte count (mxabides.counters).
 * Synchronous. */
#define MXA_COUNTER_WORDS 34
int mxa_read_counters(mxa_handle* h, int64_t* out);
/* diagnostics: copy `bytes` raw bytes of env `env`'s HBM block starting at `offset`; and
 * the block's section offsets (Layout: ag, open, rng, lat, q, book, tx, trace) */
int mxa_read_raw(mxa_handle* h, int32_t env, int64_t offset, int64_t bytes, void* out);
int mxa_layout(const mxa_handle* h, int64_t* offsets8);
int32_t mxa_n_agents(const mxa_handle* h);
int32_t mxa_n_envs(const mxa_handle* h);
/* device memory bytes per env block */
int64_t mxa_env_bytes(const mxa_handle* h);
/* replace the handle's HIP stream (hipStream_t as void*); NULL restores the own stream */
int mxa_set_stream(mxa_handle* h, void* stream);
/* HIP event timing of the last mxa_run / mxa_launch sequence, milliseconds */
double mxa_last_kernel_ms(const mxa_handle* h);
const char* mxa_last_error(const mxa_handle* h); /* NULL: the last mxa_config_* / mxa_create_config error */
void mxa_destroy(mxa_handle* h);

/* ABIDESEnv on a replay tape: n_rec time-sorted records (ns since midnight, order id > 0,
 * price in cents < 2^20, size, side 1 = buy), as LOBSTEROrdersProcessor produces them.  One
 * env per handle slot; envs differ only by the actions they are stepped with. */
int mxa_create_replay(const int64_t* t, const int64_t* oid, const int64_t* price, const int64_t* size,
                      const int8_t* buy, int32_t n_rec, int32_t n_envs, int32_t device, int32_t trace_cap,
                      mxa_handle** out);
/* config/marketreplay.py (config/marketreplay.py:60-140): the exchange and the MarketReplayAgent on
 * the same tape under Kernel.runner, midnight to 16:01 — a plain Kernel.runner handle (mxa_run,
 * mxa_finalize, the readers); the tape format of mxa_create_replay */
int mxa_create_replay_runner(const int64_t* t, const int64_t* oid, const int64_t* price, const int64_t* size,
                             const int8_t* buy, int32_t n_rec, int32_t n_envs, int32_t device, int32_t trace_cap,
                             mxa_handle** out);
/* config/execution/marketreplay/execution_marketreplay.py (:55-160): the handle of
 * mxa_create_replay_runner plus TWAP_EXECUTION_AGENT 2 (TWAPExecutionAgent, twap_agent.py:9-63:
 * BUY 12e3 over pd.date_range(10:00, 12:00, "60S"), QUERY_SPREAD depth 500).  trade = the script's
 * -e flag; with it the agent's first placeOrders raises the reference's KeyError (a 30 s Interval
 * looked up in its 60 s schedule, execution_agent.py:118) and every env ends in error
 * 25 (ERR_TWAP_SCHEDULE) at 10:00, as the reference run does. */
int mxa_create_replay_twap(const int64_t* t, const int64_t* oid, const int64_t* price, const int64_t* size,
                           const int8_t* buy, int32_t n_rec, int32_t trade, int32_t n_envs, int32_t device,
                           int32_t trace_cap, mxa_handle** out);
/* (replay and MXA_RMSC03_RL handles) one ABIDESEnv.step per env: actions [n][3] (float64) -> obs [n][9] (float64) and flags [n]
 * (bit0 done, bit1 observation valid, bit2 env error).  Host arrays; synchronous. */
int mxa_step(mxa_handle* h, const double* actions, double* obs, int32_t* flags);
/* the same on device arrays, asynchronous on the handle's stream */
int mxa_step_device(mxa_handle* h, const double* d_actions, double* d_obs, int32_t* d_flags);
/* k consecutive ABIDESEnv.step calls in ONE launch, with every action given up front (an
 * open-loop schedule: an impact study's order sizes, or actions drawn ahead as bench.py does):
 * device arrays actions [k][n_envs][3] -> obs [k][n_envs][9], flags [k][n_envs].  Step i of every
 * env equals the i-th of k mxa_step_device calls, observation and flags included; each env runs
 * its steps without waiting for the slowest env of each step.  Asynchronous on the handle's
 * stream; GymKernel handles only (MXA_EINVAL otherwise). */
int mxa_step_many(mxa_handle* h, int32_t k, const double* d_actions, double* d_obs, int32_t* d_flags);
/* the per-pop parity hash (mxa_env_summary.hash: a rolling FNV-1a over every pop's trace
 * record, the test harness's checksum; the reference computes nothing like it) is on by
 * default.  Turning it off leaves every market result identical and the hash field frozen at
 * its initial value; a handle with a trace ring keeps it on. */
int mxa_set_parity_hash(mxa_handle* h, int32_t enabled);
/* the execution agent's state after the last step, for a learner on the device (the reward
 * inputs of DDQLearningExecutionAgent.compute_reward, ddqlearning_execution_agent.py:409-446):
 * DEVICE array [n_envs][MXA_RL_STATE_WORDS] float64 = (CASH, holdings, executed quantity,
 * best bid, best ask, best-bid size, best-ask size, lob flags: 1 bids, 2 asks) of
 * DummyRLExecutionAgent, the LOB being the newest ABIDESEnvMetrics entry (dummy_rl:294-315).
 * Asynchronous on the handle's stream; GymKernel handles only. */
#define MXA_RL_STATE_WORDS 8
int mxa_write_rl_state(mxa_handle* h, double* device_out);
/* identity of the kernel sources this library was built from (a hash of csrc/ and this header
 * plus the compile flags): profile records (profiles/hbm_traffic_*.json) carry it, so a bench
 * attaches measured HBM traffic only to the build it was measured on */
const char* mxa_build_id(void);

/* book-update log, the input of the reference's order-book outputs: OrderBook.book_log rows
 * (OrderBook.py:151-168, archived by ExchangeAgent.logOrderBookSnapshots, ExchangeAgent.py:389-469,
 * as ORDERBOOK_<sym>_FULL) and the exchange's BEST_BID / BEST_ASK / LAST_TRADE events
 * (OrderBook.py:112-141).  One record per handled limit order (price, qty > 0 for a buy, < 0
 * for a sell) and per cancellation (-price, the cancelled quantity, > 0 on the bid side).  The
 * host replays the price-level volumes (mxabides.booklog): matching at level granularity is
 * exact, as a level gives min(remaining quantity, its volume) at its price. */
typedef struct {
  int64_t t;      /* Kernel.currentTime, ns since midnight (FundamentalTime for f_log records) */
  int32_t price;  /* cents (limit orders), -cents (cancellations), MXA_BL_FUNDAMENTAL */
  int32_t qty;
} mxa_book_rec;
/* the stream also carries SparseMeanRevertingOracle.f_log (SMRO:122): one record per computed
 * fundamental value (price MXA_BL_FUNDAMENTAL, qty the value), including the oracle
 * observations of the last mxa_finalize, the series written as fundamental_<sym>.bz2 */
#define MXA_BL_FUNDAMENTAL (-2147483647 - 1)
/* Kernel.runner configs (the replay of mxa_create_replay_runner / _twap included: its records add
 * modifyOrder's head-replace as a level-volume change, price -(p | 1 << 30 | side << 29); the
 * ExternalFileOracle's f_log travels as (low, high) word pairs of the double, prices -2^31 + 1 and
 * -2^31 + 2): `cap` records per env (0 = off); resets every env's record
 * count, so enable it after mxa_create / mxa_reset and before the first launch.  An env that
 * fills its log stops with error ERR_BOOK_LOG_FULL (20).  The exchange's event runs (batched
 * LIMIT/CANCEL handling) are off while logging. */
int mxa_set_book_log(mxa_handle* h, int32_t cap);
/* the exchange's own log, ExchangeAgent.log (agent/ExchangeAgent.py:39 log_events=True), which
 * Agent.kernelTerminating writes as EXCHANGE_AGENT.bz2 (agent/Agent.py:86-95), rides in the same
 * stream when on != 0 (kept across mxa_reset; needs mxa_set_book_log first).  Codes, price = code +
 * message kind (MK_* = the trace kinds):
 *   MXA_BL_EV_RX    a message the exchange logs on receipt (ExchangeAgent.py:162-167): qty = sender;
 *                   LIMIT_ORDER / CANCEL_ORDER only when the config's exchange has log_orders
 *   MXA_BL_EV_NT    ORDER_ACCEPTED / ORDER_CANCELLED / ORDER_EXECUTED sent, with log_orders
 *                   (ExchangeAgent.py:477-482): qty = recipient
 *   MXA_BL_EV_PLACE an order created (LimitOrder.time_placed), with log_orders: t, qty = order id
 * An RX record of LIMIT_ORDER / CANCEL_ORDER and every NT record is followed by its order:
 * t = fill_price << 32 | (uint32)order_id (fill_price INT32_MIN: None), price = limit price,
 * qty = quantity (> 0 buy, < 0 sell).  The BEST_BID / BEST_ASK / LAST_TRADE rows follow from the
 * limit-order records (mxabides.booklog.exchange_log rebuilds the frame).  Replaces the
 * reference's in-process log list (Agent.logEvent, Agent.py:97-110).  Set it before the first
 * launch (or after a whole-handle mxa_reset): switching it once envs have popped events is
 * MXA_EINVAL, since rows would name orders placed before the log started. */
#define MXA_BL_EV_RX (-2147483647 - 1 + 256)
#define MXA_BL_EV_NT (MXA_BL_EV_RX + 256)
#define MXA_BL_EV_PLACE (MXA_BL_EV_RX + 512)
#define MXA_BL_EV_END (MXA_BL_EV_RX + 768)
int mxa_set_exchange_log(mxa_handle* h, int32_t on);
/* env's records: min(total, cap, log capacity) are written to out, the total to *n (above the
 * log capacity: the log overflowed) */
int mxa_read_book_log(mxa_handle* h, int32_t env, mxa_book_rec* out, int64_t cap, int64_t* n);

/* parity probes: device numpy-legacy RNG (mode 0 u32, 1 double, 2 randint(a,b),
 * 3 normal(a,b), 4 exponential(a), 5 uniform(a,b)) and device glibc math (mode 0 log, 1 exp,
 * 2 pow) */
int mxa_rng_probe(int32_t device, uint32_t seed, int32_t mode, double a, double b, int32_t n, double* out);
int mxa_math_probe(int32_t device, int32_t mode, const double* x, const double* y, double* out, int64_t n);

#ifdef __cplusplus
}
#endif
#endif
