/* abides_oracle.h — CPU restatement of the reference ABIDES hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only
 * as the checker / reported CPU baseline.  The product path (libmxa, HIP) never
 * links or calls it.
 *
 * Restates (file:line of /root/reference):
 *   Kernel.runner loop ........................ Kernel.py:190-292
 *   Kernel.sendMessage / setWakeup ............ Kernel.py:347-462
 *   OrderBook (match/enter/cancel/history) .... util/OrderBook.py:38-436
 *   ExchangeAgent.receiveMessage .............. agent/ExchangeAgent.py:129-340,471-485
 *   TradingAgent protocol ..................... agent/TradingAgent.py:99-268,309-462,514-535,609-680
 *   ZeroIntelligenceAgent ..................... agent/ZeroIntelligenceAgent.py:65-350
 *   NoiseAgent / ValueAgent ................... agent/NoiseAgent.py, agent/ValueAgent.py
 *   POVMarketMakerAgent / MomentumAgent ....... agent/market_makers/POVMarketMakerAgent.py,
 *                                               agent/examples/MomentumAgent.py
 *   SparseMeanRevertingOracle ................. util/oracle/SparseMeanRevertingOracle.py:36-227
 *   LatencyModel (cubic) ...................... model/LatencyModel.py:109-140
 *   configs sparse_zi_100 / sparse_zi_1000 / rmsc03 (global-RNG draw order)
 *   ABIDESEnv / GymKernel step loop ........... ABIDESEnv.py:8-103, GymKernel.py:158-389
 *   MarketReplayAgent + OrderBook.modifyOrder .. agent/examples/MarketReplayAgent.py:50-96,
 *                                               util/OrderBook.py:341-372
 *   DummyRLExecutionAgent + ABIDESEnvMetrics ... agent/execution/rl/dummy_rl_execution_agent.py,
 *                                               ABIDESEnvMetrics.py, execution_agent.py
 *   numpy legacy RandomState (MT19937 + legacy_gauss/exponential/bounded ints), numpy 2.2.6
 *   transcendental math: the host glibc libm (the same libm the reference ran on).
 *
 * Parity is pinned by the fixtures in tests/golden/ (traces produced by the reference itself) and by
 * the reference's own known-answer file tests/sparse_zi_1000.txt.
 */
#ifndef ABIDES_ORACLE_H
#define ABIDES_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct ora_env ora_env;

/* config: sparse_zi_100, sparse_zi_1000 or rmsc03 */
int ora_create(const char* config, uint32_t seed, ora_env** out);
/* the ExternalFileOracle series of hist_fund_value / hist_fund_diverse (process-wide): n
 * time-sorted entries, ns since midnight and values */
void ora_set_fundamental(const int64_t* t, const double* v, int n);
void ora_destroy(ora_env* e);
/* run up to max_pops kernel pops (<0: unlimited); returns pops performed by this call */
int64_t ora_run(ora_env* e, int64_t max_pops);
/* run the after-loop lifecycle (kernelStopping): fills the "Final holdings" lines */
int ora_finish(ora_env* e);
int ora_done(const ora_env* e);
int ora_error(const ora_env* e);
const char* ora_error_str(const ora_env* e);
uint64_t ora_hash(const ora_env* e);
int64_t ora_events(const ora_env* e);
int64_t ora_current_time(const ora_env* e);
/* optional trace capture: records of 10 int64 (see DESIGN.md "trace record") */
void ora_set_trace(ora_env* e, int64_t* buf, int64_t cap_records);
int64_t ora_trace_len(const ora_env* e);
/* OrderBook.book_log (OrderBook.py:151-168) as flat rows: t, n, executed qty, average trade price
 * (0 without an execution), n x (price, volume; bids negative).  Returns the word count. */
void ora_set_book_log(ora_env* e, int on);
int64_t ora_book_log(const ora_env* e, int64_t* buf, int64_t cap);
/* the same run as device book-update records (include/mxa.h mxa_book_rec) as int64 triples
 * (t, price, qty); returns the record count */
int64_t ora_book_records(const ora_env* e, int64_t* buf, int64_t cap);
/* the exchange's own log (ExchangeAgent.log) in those records (include/mxa.h MXA_BL_EV_*) */
void ora_set_exchange_log(ora_env* e, int on);
int ora_n_agents(const ora_env* e);
/* per agent: cash, shares, number of open orders */
int ora_agent_state(const ora_env* e, int id, int64_t* cash, int64_t* shares, int64_t* n_open);
/* book side (0 bids, 1 asks) flattened: [n_levels, (n_orders, (id, agent, qty, price)*n)*] */
int64_t ora_book(const ora_env* e, int side, int64_t* buf, int64_t cap);
int64_t ora_order_counter(const ora_env* e);
int64_t ora_last_trade(const ora_env* e);
void ora_stats(const ora_env* e, int64_t* out);
/* Kernel.summaryLog after ora_finish: (agent, type 0 STARTING_CASH / 1 FINAL_CASH_POSITION /
 * 2 ENDING_CASH / 3 FINAL_VALUATION, is-float, int value, float value); returns the row count */
const char* ora_agent_type_name(const ora_env* e, int id); /* Agent.type (the summary's AgentStrategy) */
int ora_summary(const ora_env* e, int* agent, int* type, int* isf, int64_t* vi, double* vf, int cap);
/* stdout restatement after ora_finish: "Final holdings ..." lines then "Mean..." lines */
int64_t ora_report(const ora_env* e, char* buf, int64_t cap);

/* marketreplay / ABIDESEnv: a LOBSTER tape as parsed by
 * LOBSTEROrdersProcessor (MarketReplayAgent.py:162-220): per record the time (ns since
 * midnight), order id, price (cents), size, side; time-sorted, file order within a time. */
int ora_create_mr(const int64_t* t, const int64_t* oid, const int64_t* price, const int64_t* size,
                  const int8_t* buy, int n, ora_env** out);
/* config/marketreplay.py: the exchange and the MarketReplayAgent under Kernel.runner (ora_run) */
void ora_set_symbol(ora_env* e, const char* sym);
void ora_set_stop(ora_env* e, int64_t t_stop);
/* config/execution/marketreplay/execution_marketreplay.py: the replay of ora_create_mr_runner plus
 * TWAPExecutionAgent 2; trade = the script's -e flag */
int ora_create_mr_twap(const int64_t* t, const int64_t* oid, const int64_t* price, const int64_t* size,
                       const int8_t* buy, int n, int trade, ora_env** out);
int ora_create_mr_runner(const int64_t* t, const int64_t* oid, const int64_t* price, const int64_t* size,
                         const int8_t* buy, int n, ora_env** out);
/* ABIDESEnv.step(action[3]): obs_out[9] (valid when *has_obs), *done; returns 0 or an error */
int ora_gym_step(ora_env* e, const double* action, double* obs_out, int* has_obs, int* done_out);
/* DummyRL: remaining quantity, executed quantity, trade flag; replay agent's open orders */
int ora_rl_state(const ora_env* e, int64_t* out4);

/* CPU baseline: n independent envs (seeds[i]) over `threads` OS threads, one env per task.
 * Each env runs at most max_pops pops (<0: to completion). Returns 0 on success. */
int ora_run_batch(const char* config, const uint32_t* seeds, int n, int threads, int64_t max_pops,
                  int64_t* events_out, uint64_t* hash_out, double* seconds_out);
/* ora_run_batch plus each env's error code (0 ok; negative = the fail() code) */
int ora_run_batch_err(const char* config, const uint32_t* seeds, int n, int threads, int64_t max_pops,
                      int64_t* events_out, uint64_t* hash_out, int32_t* err_out, double* seconds_out);
/* capacity statistics of n envs run to completion: stats_out[n][4] = ora_stats */
int ora_run_batch_stats(const char* config, const uint32_t* seeds, int n, int threads, int64_t* stats_out);
/* config/rmsc03.py with its market-maker options (config/rmsc03.py:39-43, swept by
 * scripts/rmsc03.sh): --mm-pov, --mm-min-order-size, --mm-window-size, --mm-num-ticks and
 * --mm-wake-up-freq (as pd.Timedelta(...).value ns).  Same layout as include/mxa.h mxa_mm_params. */
typedef struct {
    double mm_pov;
    int32_t mm_min_order_size, mm_window_size, mm_num_ticks, pad;
    int64_t mm_wake_up_freq_ns;
} ora_mm_params;
int ora_create_mm(uint32_t seed, const ora_mm_params* p, ora_env** out);
/* ora_run_batch_err / _stats of rmsc03 envs with per-env market-maker options params[n] */
int ora_run_batch_mm(const uint32_t* seeds, const ora_mm_params* params, int n, int threads, int64_t max_pops,
                     int64_t* events_out, uint64_t* hash_out, int32_t* err_out, int64_t* stats_out, double* seconds_out);
/* runtime compositions (include/mxa.h mxa_config, the same layout): a base script's construction
 * ("rmsc03", "value_noise", "sparse_zi_100", "sparse_zi_1000") with the caller's agent counts,
 * per-class parameters and session.  rmsc03, random_fund_value, value_noise and sparse_zi_* are
 * built through the same parameterised builders, so their fixtures pin them. */
#define ORA_CONFIG_ZI_GROUPS 8
typedef struct {
    int32_t base; /* 0 rmsc03, 5 value_noise, 1 sparse_zi_100, 2 sparse_zi_1000 (include/mxa.h ids) */
    int32_t log_orders, n_noise, n_value, n_mm, n_momentum, n_zi_groups, zi_q_max;
    int32_t zi_count[ORA_CONFIG_ZI_GROUPS], zi_r_min[ORA_CONFIG_ZI_GROUPS], zi_r_max[ORA_CONFIG_ZI_GROUPS];
    double zi_eta[ORA_CONFIG_ZI_GROUPS];
    double zi_sigma_n, zi_r_bar, zi_kappa, zi_sigma_s, zi_sigma_pv, zi_lambda_a;
    int64_t mkt_open_ns, mkt_close_ns, kernel_start_ns, kernel_stop_ns, noise_wake_open_ns, noise_wake_close_ns;
    int64_t date_ns, starting_cash, default_computation_delay_ns;
    double r_bar, kappa, fund_vol, megashock_lambda_a, megashock_mean, megashock_var;
    double value_sigma_n, value_r_bar, value_kappa, value_sigma_s, value_lambda_a;
    int64_t value_starting_cash;
    ora_mm_params mm;
    int32_t mom_min_size, mom_max_size;
    int64_t mom_wake_up_freq_ns;
    double lat_low, lat_high;
    int32_t queue_capacity, book_capacity; /* the device's capacities (unused here) */
} ora_config;
int ora_config_defaults(const char* base, ora_config* out);
int ora_create_config(const ora_config* c, uint32_t seed, ora_env** out);
/* ora_run_batch_err / _stats of one composition over n seeds */
int ora_run_batch_config(const ora_config* c, const uint32_t* seeds, int n, int threads, int64_t max_pops,
                         int64_t* events_out, uint64_t* hash_out, int32_t* err_out, int64_t* stats_out,
                         double* seconds_out);
/* the ExchangeAgent's log_orders of a configuration (the exchange-log switch) */
int ora_config_log_orders(const char* config);
/* n GymKernel episodes, each stepped with actions[k][i][0..2] until done or error (config
 * "rmsc03_rl" with seeds, or NULL: the replay composition on the tape t/oid/price/size/buy).
 * Per env: pops, hash, error code, steps taken and the last valid observation [n][9]. */
/* ABIDESEnv.reset in the same process: rebuild the composition (rmsc03_rl from `seed`, or the
 * replay on the same tape), carrying Order.order_id / Order._order_ids; *pe is replaced */
int ora_gym_reset(ora_env** pe, uint32_t seed);
int ora_gym_batch(const char* config, const uint32_t* seeds, const int64_t* t, const int64_t* oid,
                  const int64_t* price, const int64_t* size, const int8_t* buy, int n_rec, int n, int n_steps,
                  const double* actions, int threads, int64_t* ev_out, uint64_t* hash_out, int32_t* err_out,
                  int32_t* steps_out, double* obs_out, double* seconds_out);

/* numpy-legacy RNG known-answer helpers (tests) */
typedef struct ora_rs ora_rs;
ora_rs* ora_rs_new(uint32_t seed);
void ora_rs_free(ora_rs* r);
uint32_t ora_rs_u32(ora_rs* r);
double ora_rs_double(ora_rs* r);
int64_t ora_rs_randint(ora_rs* r, int64_t lo, int64_t hi);
double ora_rs_normal(ora_rs* r, double loc, double scale);
double ora_rs_exponential(ora_rs* r, double scale);
double ora_rs_uniform(ora_rs* r, double lo, double hi);

#ifdef __cplusplus
}
#endif
#endif
