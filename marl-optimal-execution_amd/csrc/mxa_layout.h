// mxa_layout.h — plain-old-data shared by the host C-ABI (mxa_api.cpp) and the HIP
// kernels (mxa_kernels.hip): configuration parameters, the per-environment HBM block
// layout, the 24-byte message payload and the 10-word trace record.
//
// One environment (= one independent market = one reference Kernel run) is simulated by
// ONE wavefront.  Its state lives in one contiguous HBM block ("env block", stride
// Layout::env_stride) so that every per-env array is read/written by the wave as
// coalesced 64-lane accesses; while a kernel runs, the event queue lives in LDS and the
// limit order book in VGPRs (see DESIGN.md §Data layout).
#pragma once
#include <stdint.h>

#define MXA_MAX_AGENTS 8191  // 13-bit recipient field in the event key
#define MXA_KEY_SHIFT 15     // key = t << 15 | recipient << 2 | type (t < 2^48 ns: 78 h after midnight)
#define MXA_KEY_RCP 0x1FFF
#define MXA_MT_N 624
#define MXA_MT_M 397
#define MXA_RNG_WORDS 1280    // two 624-word MT blocks (double buffer) + pad (5120 B per stream)

enum mxa_config_id { MXA_CFG_RMSC03 = 0, MXA_CFG_SPARSE_ZI_100 = 1, MXA_CFG_SPARSE_ZI_1000 = 2, MXA_CFG_MARKETREPLAY = 3,
                     MXA_CFG_RMSC03_RL = 4, MXA_CFG_VALUE_NOISE = 5, MXA_CFG_RMSC01 = 6,
                     MXA_CFG_RMSC02 = 7, MXA_CFG_OBI_RMSC02 = 8, MXA_CFG_RANDOM_FUND_VALUE = 9,
                     MXA_CFG_RANDOM_FUND_DIVERSE = 10, MXA_CFG_HIST_FUND_VALUE = 11,
                     MXA_CFG_HIST_FUND_DIVERSE = 12, MXA_CFG_MARKETREPLAY_RUNNER = 13,
                     MXA_CFG_MARKETREPLAY_TWAP = 14,
                     // rmsc03 with a SpreadBasedMarketMakerAgent in the market maker's slot: subscribe=True
                     // (the agent's default) and the polling mode
                     MXA_CFG_RMSC03_SBMM = 15, MXA_CFG_RMSC03_SBMM_POLL = 16,
                     // config/rmsc03.py with per-env market-maker options (--mm-pov ... --mm-wake-up-freq,
                     // config/rmsc03.py:39-43; the sweep of scripts/rmsc03.sh) and the capacities they need
                     MXA_CFG_RMSC03_MM = 17 };

// config/rmsc03.py's market-maker options of one env (include/mxa.h mxa_mm_params): read by the
// build kernel into the POVMarketMakerAgent's record (AF_MM_*)
typedef struct {
  double pov;                  // --mm-pov
  int32_t min_order_size;      // --mm-min-order-size
  int32_t window_size;         // --mm-window-size
  int32_t num_ticks;           // --mm-num-ticks
  int32_t pad;
  int64_t wake_up_freq;        // --mm-wake-up-freq as pd.Timedelta(...).value (ns)
} MmParams;

// message kinds (tests/golden/gen_fixtures.py KIND; oracle/abides_oracle.c)
enum {
  MK_WAKEUP = 0, MK_WHEN_OPEN_REQ = 1, MK_WHEN_CLOSE_REQ = 2, MK_WHEN_OPEN = 3, MK_WHEN_CLOSE = 4,
  MK_SPREAD_REQ = 5, MK_SPREAD = 6, MK_LAST_REQ = 7, MK_LAST = 8, MK_TV_REQ = 9, MK_TV = 10,
  MK_LIMIT = 11, MK_CANCEL = 12, MK_MODIFY = 13, MK_ACCEPTED = 14, MK_EXECUTED = 15, MK_CANCELLED = 16,
  MK_MKT_CLOSED = 17, MK_MODIFIED = 18, MK_KCANCEL = 19, MK_MARKET_DATA = 20,
  MK_STREAM_REQ = 21, MK_STREAM = 22,  // QUERY_ORDER_STREAM request / reply
  MK_MD_SUB_REQ = 23, MK_MD_SUB_CANCEL = 24  // MARKET_DATA_SUBSCRIPTION_REQUEST / _CANCELLATION
};
// kernel message types (message/Message.py:5-8)
enum { MT_MESSAGE = 1, MT_WAKEUP = 2, MT_CANCEL_ORDER = 3 };

// agent classes
enum { AG_EXCHANGE = 0, AG_ZI = 1, AG_NOISE = 2, AG_VALUE = 3, AG_POVMM = 4, AG_MOMENTUM = 5, AG_REPLAY = 6, AG_DUMMYRL = 7,
       AG_MKTMAKER = 8, AG_HBL = 9, AG_OBI = 10, AG_TWAP = 11, AG_SBMM = 12 };
// SpreadBasedMarketMakerAgent's string order ids "<name>_<id>_<n>" (generateNewOrderId,
// SpreadBasedMarketMakerAgent.py:279-288) are carried as MXA_SB_ID_BASE + n: compared for
// identity only, never equal to an auto id
#define MXA_SB_ID_BASE 0x40000000

// env status flags (EnvHdr::status)
enum { ST_RUNNING = 0, ST_DONE = 1, ST_ERROR = 2 };
enum {
  ERR_NONE = 0, ERR_QUEUE_FULL = 1, ERR_BOOK_FULL = 2, ERR_OPEN_FULL = 3, ERR_TX_FULL = 4,
  ERR_PANDAS_NO_TX = 5, ERR_WAKEUP_PAST = 6, ERR_THETA_INDEX = 7, ERR_BAD_CONFIG = 8,
  ERR_RNG_OVERRUN = 9,
  // marketreplay / ABIDESEnv: reference crash paths and capacity limits
  ERR_RP_PRICE = 10,      // tape/agent price outside the ladder
  ERR_RP_POOL = 11,       // book entry pool exhausted
  ERR_RP_IDS = 12,        // agent order ids beyond the dense-id capacity
  ERR_RP_KEYERROR = 13,   // MarketReplayAgent: no tape group at the wake time
  ERR_RP_OBS = 14,        // get_observation / get_reward on missing or None data
  ERR_RP_STOPPING = 15,   // ExecutionAgent.kernelStopping with trade still on (arrival_price None)
  ERR_RP_MODIFY = 16,     // modify changing price or side (head-replace would re-key the level)
  // HeuristicBeliefLearningAgent
  ERR_HBL_WINDOW = 17,    // a streamed history epoch left the exchange's window / the device ring
  ERR_HBL_RANGE = 18,     // streamed price range beyond the device scratch (MXA_HBL_RANGE)
  ERR_FLOAT_PRICE = 19,   // a limit price that the reference would carry as a python float (not restated)
  ERR_BOOK_LOG_FULL = 20, // the book-update log of mxa_set_book_log ran out of records
  // market-data subscriptions (ExchangeAgent.publishOrderBookData)
  ERR_MD_NO_UPDATE = 21,  // a publish before the book's first change: None > Timestamp (TypeError)
  ERR_MD_SUBS = 22,       // more subscriptions than the device table (64)
  ERR_MD_KEYERROR = 23,   // cancelling a subscription that does not exist (KeyError)
  ERR_MD_SLOT = 24,       // a second MARKET_DATA in flight to one agent (freq below the latency)
  // TWAPExecutionAgent (ExecutionAgent.placeOrders, execution_agent.py:108-123)
  ERR_TWAP_SCHEDULE = 25, // schedule[Interval(t, t + 30 s)] of a 60 s schedule (KeyError)
  ERR_TWAP_QUOTE = 26,    // (bid + ask) / 2 with a None side (TypeError)
  ERR_TWAP_MARKET = 27,   // placeMarketOrder at horizon[-2] (not restated; unreachable in the script)
  // SpreadBasedMarketMakerAgent.receiveMessage: a QUERY_SPREAD with a missing side before any mid
  // was known leaves `mid` unbound (UnboundLocalError)
  ERR_SB_MID = 28,
  // an order quantity beyond the device's 32-bit order words (POVMarketMakerAgent: pov x transacted
  // volume with a large --mm-pov); the reference's Python int has no bound, so the env stops
  ERR_ORDER_SIZE = 29
};

// per-env scalar header (first bytes of the env block)
typedef struct {
  int64_t cur;          // Kernel.currentTime (ns since midnight of the simulated date)
  int64_t pops;         // ttl_messages
  uint64_t hash;        // rolling FNV over trace records
  int64_t order_counter;
  int32_t status, err;
  uint32_t seq;         // Message.uniq analogue (per env)
  uint32_t arrival;     // book FIFO arrival counter
  int32_t epoch;        // OrderBook.history shift counter
  int32_t tx_head;      // transaction ring write position (monotonic)
  int64_t last_trade;
  int32_t last_trade_float, pad0;
  int32_t ep_n[16];     // OrderBook.history: order entries per epoch (ring of 16 epochs)
  // oracle (SparseMeanRevertingOracle)
  int64_t o_pt, o_mst;
  double o_pv, o_msv;
  // global RNG streams G, O, K, L: output index / materialized block / gauss cache
  int32_t rs_pos[4], rs_has_gauss[4];
  double rs_gauss[4];
  int32_t rs_m[4];
  int32_t rs_w0[4], rs_wn[4];    // run kernel: LDS output window of each stream (start, length)
  int32_t oh_head;               // order-history ring: records written so far (HBL configs)
  int32_t blog_n;                // book-update log: records written (mxa_set_book_log)
  int32_t q_count, b_count;      // saved queue / book occupancy
  int64_t trace_len;
  int64_t ex_comp_delay;         // exchange's current computation delay
  int32_t max_q, max_book;       // capacity high-water marks (diagnostics)
  double o_th2;                  // oracle fund_vol ** 2 (glibc pow, evaluated at build)
  int32_t blog_fin;              // book-update log: records after the last kernelStopping pass
  int32_t exlog;                 // the exchange's own log rides in the book-update log (mxa_set_exchange_log)
  int64_t ob_last_update;        // OrderBook.last_update_ts (market-data configs)
  int32_t nsub, has_last_update; // ExchangeAgent.subscription_dict entries; last_update_ts not None
  uint32_t md_seq;               // MARKET_DATA messages sent (their snapshot-slot tags)
  int32_t md_any0;               // a live subscription with freq <= 0 (due at every update)
  int64_t md_next_due;           // no freq > 0 subscription is due before this update time (0: unknown)
  // event-class counters of instrumented runs (parity hash on / trace ring): pops per message
  // kind (MK_*; WAKEUP pops at MK_WAKEUP, GymKernel CANCEL_ORDER pops at MK_KCANCEL), then busy
  // requeues at MXA_KC_REQUEUE, agent-record round trips (MXA_KC_REC) and pops handled as members
  // of a batched event run (MXA_KC_RUN); the algorithmic-byte count of bench.py (mxa_read_counters)
  uint32_t kc[28];
  int32_t q0;                    // queue occupancy when the build ended (the kernelStarting wakeups)
  int32_t pad4;
  uint64_t rng0;                 // RNG words the build drew (sum over streams of position - 624)
  int64_t t_stop;                // Kernel.runner's stopTime if > 0 (mxa_set_stop_time), else the config's
} EnvHdr;
#define MXA_KC_REQUEUE 25
#define MXA_KC_REC 26
#define MXA_KC_RUN 27

#ifdef __cplusplus
static_assert(sizeof(EnvHdr) % 8 == 0 && sizeof(EnvHdr) <= 512, "EnvHdr: copied by 64 lanes x 8 B, 512 B of LDS");
#endif

// book-update log, the input of OrderBook.book_log and the exchange's BEST_BID / BEST_ASK /
// LAST_TRADE events (OrderBook.py:112-168): one record per handled limit order (price, qty
// positive for a buy, negative for a sell) and per cancellation (-price, the cancelled
// quantity, positive on the bid side).  The host replays the level volumes.  The same stream
// carries SparseMeanRevertingOracle.f_log (SMRO:122): price BL_FUNDAMENTAL, qty = the value,
// t = FundamentalTime.
typedef struct {
  int64_t t;       // Kernel.currentTime (ns since midnight)
  int32_t price;
  int32_t qty;
} BlRec;
enum { BL_FUNDAMENTAL = -2147483647 - 1 };
// ExternalFileOracle.f_log entries (ExternalFileOracle.py:97): the interpolated value is a double,
// so it travels as two records at the query time: the low word (price BL_FUND_LO), then the high
// word (price BL_FUND_HI)
enum { BL_FUND_LO = -2147483647, BL_FUND_HI = -2147483646 };
// OrderBook.modifyOrder on the replay ladder (OrderBook.py:341-372): the level HEAD becomes the new
// order, so the level's volume changes by qty = new quantity - the old head's; price =
// -(level price | BL_MODIFY | side << 29), side 0 bids (prices < 2^20 on the replay tape)
#define BL_MODIFY (1 << 30)
// the exchange's own log (ExchangeAgent.log, written as EXCHANGE_AGENT.bz2 by Agent.kernelTerminating,
// agent/Agent.py:86-95) in the same stream, with mxa_set_exchange_log; price = code + message kind:
//  BL_EV_RX    a message the exchange logs as it receives it (ExchangeAgent.py:162-167): qty = sender
//  BL_EV_NT    an ORDER_ACCEPTED / _CANCELLED / _EXECUTED it sends with log_orders (:477-482): qty = recipient
//  BL_EV_PLACE an order created (LimitOrder(...), its time_placed): t = currentTime, qty = order id
// An RX record of LIMIT_ORDER / CANCEL_ORDER (written only with log_orders) and every NT record is
// followed by its order: t = fill_price << 32 | (u32)order_id (fill_price INT32_MIN: None), price =
// limit price, qty = quantity (> 0 buy, < 0 sell).  Codes lie below every modifyOrder record while
// prices stay below 2^29 - 768
enum { BL_EV_RX = -2147483647 - 1 + 256, BL_EV_NT = BL_EV_RX + 256, BL_EV_PLACE = BL_EV_RX + 512, BL_EV_END = BL_EV_RX + 768 };
#define BL_FILL_NONE (-2147483647 - 1)

// one event slot as saved between launches (and payload as pushed)
typedef struct {
  uint64_t key;   // t << MXA_KEY_SHIFT | recipient << 2 | type
  uint32_t seq;
  uint32_t pad;
  uint32_t pl[8]; // payload (6 words used except by the marketreplay config)
} SavedEvent;   // 48 B

// book slot as saved between launches
typedef struct {
  int32_t price, qty, oid, meta;  // meta = agent << 1 | is_buy, -1 = free
  uint32_t arrival;
  int32_t hepoch;
  int32_t pad[2];
} SavedOrder;   // 32 B

typedef struct {  // transaction record of OrderBook.history (util/OrderBook.py:227,235)
  int64_t t;
  int32_t q, epoch;
} TxRec;

typedef struct {  // OrderBook.history entry of one limit order (util/OrderBook.py:52-60), HBL configs
  int32_t oid, price;
  int32_t meta;   // bit0 is_buy_order, bit1 "transactions" non-empty
  int32_t epoch;  // absolute history epoch it was entered in
} OhRec;

typedef struct {  // ExchangeAgent.subscription_dict entry (agent -> [levels, freq, last update])
  int32_t agent, levels;
  int32_t live, pad;
  int64_t freq, last;
} SubRec;         // 32 B
// MARKET_DATA snapshot slot of one subscriber (64 words): the message carries the best levels
// and the last trade (and the slot tag); the level prices and volumes wait here for the receipt
enum { MD_LEVELS = 10, MD_TAG = 0, MD_COUNTS = 1, MD_BIDS = 2, MD_ASKS = 12, MD_BIDQ = 22, MD_ASKQ = 32, MD_WORDS = 64,
       MD_MAX_SUBS = 64 };

typedef struct {  // TradingAgent.orders entry (agent's copy of an open order)
  int32_t oid, is_buy, qty, price;
} OpenOrder;

// ---- marketreplay / ABIDESEnv (runtime-sized sections after the fixed layout) ----
// entry epochs kept per order id (replay book): the OrderBook.history window is
// stream_history + 1 = 11 epochs, and an id re-entered after a cancel can sit in several
#define MXA_ID_EPOCHS 12
typedef struct {  // one resting order of the price-ladder book (OrderBook level entries)
  int32_t price, qty, oid, dense;  // dense = order-id index (tape ids, then agent ids)
  int32_t meta;                    // agent << 1 | is_buy
  uint32_t arrival;                // FIFO position stamp
  int32_t prev, next;              // level list
  int32_t idprev, idnext;          // live entries of the same order id
  int32_t pad[2];
} RpEntry;        // 48 B
typedef struct {  // MarketReplayAgent.orders (agent copy) per dense id
  int32_t qty, price, is_buy, present;
} RpOrder;
typedef struct {  // ABIDESEnvMetrics deque entry (level-1 book + last trade of one LOB)
  int32_t bid, ask, data, flags;   // flags: 1 has bids, 2 has asks, 4 data is None
} RpLob;
typedef struct {  // per-env replay / gym state
  int32_t best[2];      // best level index per side (bids max, asks min), -1 = empty
  int32_t nlev[2];      // non-empty levels per side
  int32_t free_top, mr_wi, ex_has_last, rl_trade;
  int64_t rl_exec, rl_rem;
  int32_t m_cnt, m_head, m_nb, m_na;
  int64_t m_bq, m_aq;
  int32_t m_b2, m_a2, p0, p0_none;
  int32_t ph_n, ph_none, end_step, has_obs;
  double obs[9];
  int32_t finished;
  // Order.order_id across ABIDESEnv.reset in one process (Order.py:8-9):
  // the episode's first auto-id candidate (auto ids map to dense ids from it), and how far into
  // the tape earlier episodes got (their explicit ids stay in Order._order_ids)
  int32_t id_base, tape_hi;
  int32_t mr_done;  // tape records handled this episode (their explicit ids are taken)
  int32_t pad[2];
} RpHdr;          // 208 B
typedef struct {  // runtime layout of the replay sections (offsets from the env block)
  int32_t pmin, P;      // price ladder [pmin, pmin + P)
  int32_t C, D;         // entry capacity, dense-id capacity
  int32_t n_ids;        // dense ids used by the tape (agent ids start here)
  int32_t ntm, nrec, pad;
  uint64_t off_rh, off_lvc, off_lvh, off_lvt, off_lvq, off_pool, off_free, off_idh, off_idep, off_mro, off_ring,
      end;
} RpLayout;
typedef struct {  // device-resident tape (shared by all envs of a handle)
  const int64_t* t;     // [nrec] ns since midnight, time-sorted
  const int32_t* oid;   // [nrec]
  const int32_t* dense; // [nrec]
  const int32_t* price; // [nrec] cents
  const int32_t* size;  // [nrec]
  const int8_t* buy;    // [nrec]
  const int64_t* tm;    // [ntm] distinct times
  const int32_t* tm0;   // [ntm + 1] first record of each time group
  // Order._order_ids of the tape: the distinct explicit ids that some record with SIZE > 0 turns
  // into a LimitOrder (placing and modifying both do, MarketReplayAgent.py:69-91), sorted, and the
  // first such record of each; generateOrderId skips an id once that record has been handled
  const int32_t* uid;   // [nuid] sorted
  const int32_t* ufirst;  // [nuid]
  int32_t nuid, umin;   // umin: smallest such id (auto ids below it need no lookup)
  // ExternalFileOracle fundamental series (hist_fund_* configs): time-sorted ns since midnight
  // and values (the mid prices of util/formatting/mid_price_from_orderbook.py)
  const int64_t* fs_t;
  const double* fs_v;
  int32_t fs_n;
  int32_t twap_trade;   // execution_marketreplay.py -e: the TWAP agent trades
  RpLayout L;
  const MmParams* mmp;  // MXA_CFG_RMSC03_MM: [n_envs] market-maker options (read by the build kernel)
} RpCtx;

typedef struct {
  uint64_t env_stride;
  uint32_t off_ag, off_open, off_rng, off_lat, off_q, off_book, off_tx, off_trace;
  int32_t n_agents, n_streams, qcap, ocap, open_cap, tx_cap, trace_cap, lat_len;
  int32_t oh_cap, hbl_range;    // order-history ring records; HBL price-histogram bins (0: none)
  uint64_t off_oh, off_hh;      // order-history ring; HBL histogram scratch (u64 bins)
  uint64_t off_sub, off_md;     // subscription table [MD_MAX_SUBS]; per-agent MARKET_DATA slots
} Layout;

// agent record: 128 dwords (512 B); lane i of the owning wave holds dwords 2i, 2i+1
enum {
  AF_TYPE = 0, AF_FLAGS = 1, AF_STATE = 2, AF_NORD = 3,
  AF_MKT_OPEN = 4, AF_MKT_CLOSE = 6, AF_CASH = 8, AF_SHARES = 10, AF_LAST_TRADE = 12,
  AF_BID = 14, AF_BIDQ = 15, AF_ASK = 16, AF_ASKQ = 17, AF_TV = 18, AF_PREV_WAKE = 20,
  AF_R_T = 22, AF_SIGMA_T = 24, AF_START_CASH = 26, AF_SIZE = 28, AF_GROUP = 29,
  AF_WAKEUP_TIME = 30, AF_RS_POS = 32, AF_RS_HASG = 33, AF_RS_GAUSS = 34, AF_LAST_MID = 36,
  AF_ORDER_SIZE = 38, AF_NMID = 39, AF_N20 = 40, AF_N50 = 41, AF_AVG20 = 42, AF_AVG50 = 44,
  AF_THETA = 46,      // 20 x int32
  // SpreadBasedMarketMakerAgent (its own fields in the ZI / momentum areas): the two ladder deques
  // current_bids / current_asks as rings of order ids with one head and one length (they always
  // have equal lengths), prices contiguous from the left end's
  AF_SB_N = 39, AF_SB_HEAD = 40, AF_SB_BLO = 41, AF_SB_ALO = 42, AF_SB_CNT = 43, AF_SB_IDS = 46,
  // POVMarketMakerAgent with per-env options (MXA_CFG_RMSC03_MM): pov, min_order_size, window_size,
  // num_ticks, wake_up_freq in the ZI / momentum areas it never uses
  AF_MM_POV = AF_R_T, AF_MM_MIN = 46, AF_MM_WIN = 47, AF_MM_TICKS = 48, AF_MM_WAKE = 50,
  // MarketReplayAgent: the next wakeup group (the reference's wakeup index) and the tape records
  // handled, in its LDS-resident record (RpHdr::mr_done stays the copy other agents read)
  AF_MR_WI = 46, AF_MR_DONE = 47,
  AF_MIDS = 66,       // 50 x int32 (2*mid ring), momentum
  AF_STREAM_N = 66,   // HBL: epochs of the last QUERY_ORDER_STREAM reply (momentum's AF_MIDS area)
  AF_STREAM_HI = 68,  // HBL: absolute history epoch of its first entry (history[1]), int64
  AF_RS_M = 116,      // highest materialized MT block of the agent's stream
  AF_NUSED = 117,     // open-order list slots used (live + tombstones); AF_NORD = live
  AF_ATIME = 120,     // Kernel.agentCurrentTimes[a]
  AF_COMP = 122,      // Kernel.agentComputationDelays[a]
  AF_END = 128
};
// AF_FLAGS bits
enum {
  FL_HAS_OPEN = 1, FL_HAS_CLOSE = 2, FL_MKT_CLOSED = 4, FL_FIRST_WAKE = 8, FL_DAILY_CLOSE = 16,
  FL_TRADING = 32, FL_HAS_KNOWN = 64, FL_NB = 128, FL_NA = 256, FL_HAS_LAST = 512,
  FL_LAST_FLOAT = 1024, FL_PREV_WAKE = 2048, FL_AW_SPREAD = 4096, FL_AW_TV = 8192, FL_LAST_MID = 16384,
  FL_HAS_STREAM = 32768, FL_SUB_REQ = 65536,
  FL_OBI_LONG = 131072, FL_OBI_SHORT = 262144,  // OrderBookImbalanceAgent.is_long / is_short
  FL_SB_INIT = 524288  // SpreadBasedMarketMakerAgent: current_bids / current_asks are not None
};
enum { AF_OBI_STOP = AF_R_T };  // OrderBookImbalanceAgent.trailing_stop (double; OBI has no r_t)
enum { AS_AWAITING_WAKEUP = 0, AS_INACTIVE = 1, AS_AWAITING_SPREAD = 2, AS_ACTIVE = 3, AS_AWAITING_STREAM = 4,
       AS_AWAITING_MD = 5 };

typedef struct {
  int32_t config, n_envs, n_agents, n_streams;
  int64_t start, stop, mkt_open, mkt_close, default_comp_delay;
  int32_t lat_mode, noise_len;   // 0 zero, 1 matrix (+uniform noise index), 2 cubic model
  double jitter, clip, unit;
  int64_t ex_pipeline, ex_comp;
  int32_t stream_history;
  int32_t ex_log_orders;  // ExchangeAgent(log_orders=...) of the config script (ExchangeAgent.py:163-165, 481-482)
  double o_rbar, o_kappa, o_fundvol, o_lambda, o_msmean, o_msvar;
  int64_t starting_cash;
  int32_t first_zi, n_zi, first_noise, n_noise, first_value, n_value, first_mm, n_mm, first_mom, n_mom;
  // ZeroIntelligenceAgent
  double zi_sigma_n, zi_rbar, zi_kappa, zi_sigma_s, zi_lambda, zi_sigma_pv;
  int32_t zi_qmax, zi_ngroups;
  int32_t zi_group_count[8], zi_rmin[8], zi_rmax[8];
  double zi_eta[8];
  // ValueAgent
  double v_sigma_n, v_rbar, v_kappa, v_sigma_s, v_lambda, v_percent_aggr;
  int32_t v_depth_spread, pad1;
  int64_t v_starting_cash;
  // NoiseAgent wake window
  int64_t noise_open, noise_close;
  // POVMarketMakerAgent
  double mm_pov;
  int32_t mm_min_size, mm_window, mm_ticks;
  int32_t mm_rt;           // 1: the options above are per env, in the market maker's record (AF_MM_*)
  int64_t mm_wake;
  // MomentumAgent
  int32_t mom_min, mom_max;
  int64_t mom_wake;
  double lat_lo, lat_hi;   // G.uniform bounds of the latency matrix
  // marketreplay / ABIDESEnv composition (agent_config.py:30-160)
  int32_t first_replay, n_replay, first_rl, n_rl;
  int64_t rl_quantity, rl_h0, rl_hstep;   // DummyRL: BUY 1e5 over date_range(h0, ..., hstep)
  int32_t rl_nh, rl_depth, rl_ids, n_twap;  // horizon length, spread depth, agent-id capacity; TWAP agents (the horizon is rl_*)
  // MarketMakerAgent (agent/market_makers/MarketMakerAgent.py, polling mode)
  int32_t first_mk, n_mk, mk_min, mk_max;
  int32_t mk_depth, pad4;
  int64_t mk_wake, mk_last_spread;
  // HeuristicBeliefLearningAgent (ZI parameters of group 0, plus L)
  int32_t first_hbl, n_hbl, hbl_L, first_twap;
  // market-data subscriptions (rmsc02: MarketMakerAgent / MomentumAgent subscribe=True)
  int32_t md_sub, md_mk_levels, md_mom_levels, lat_asym;  // lat_asym: latency row 0 + column 0
  int64_t md_freq;
  // OrderBookImbalanceAgent (agent/OrderBookImbalanceAgent.py defaults)
  int32_t first_obi, n_obi, obi_levels;
  int32_t oracle_ext;      // 1: util/oracle/ExternalFileOracle.py on a runtime series (RpCtx::fs_*)
  int64_t obi_freq, obi_wake;
  double obi_entry, obi_trail;
  // SpreadBasedMarketMakerAgent (agent/market_makers/SpreadBasedMarketMakerAgent.py)
  int32_t first_sb, n_sb, sb_sub, sb_size, sb_window, sb_ticks;
  int64_t sb_wake;
  Layout L;
} MxaParams;

#define MXA_TRACE_WORDS 10
