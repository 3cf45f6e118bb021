/* abides_oracle.c — CPU restatement (parity oracle) of the reference ABIDES hot path.
 * TEST INFRASTRUCTURE ONLY — see abides_oracle.h for scope and the reference map.
 *
 * Structure intentionally mirrors the reference's Python objects (heap of events,
 * per-side lists of price levels each holding a FIFO list of orders, per-agent
 * ordered dict of open orders, history epochs) so that each function can be read
 * side by side with the cited reference lines.  Transcendentals call the host libm
 * (glibc), which is the libm the reference's numpy/math calls resolve to.
 */
#define _GNU_SOURCE
#include "abides_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------- */
/* numpy legacy RandomState (numpy/random/src/mt19937, distributions/legacy)  */
/* ------------------------------------------------------------------------- */
#define MT_N 624
#define MT_M 397
struct ora_rs {
    uint32_t key[MT_N];
    int pos;
    int has_gauss;
    double gauss;
};

/* mt19937_seed == init_genrand (numpy _legacy_seeding with an int seed) */
static void rs_seed(ora_rs* r, uint32_t s) {
    for (int i = 0; i < MT_N; i++) {
        r->key[i] = s;
        s = (uint32_t)(1812433253u * (s ^ (s >> 30)) + (uint32_t)i + 1u);
    }
    r->pos = MT_N;
    r->has_gauss = 0;
    r->gauss = 0.0;
}

static void mt_gen(ora_rs* r) {
    uint32_t y;
    int i;
    for (i = 0; i < MT_N - MT_M; i++) {
        y = (r->key[i] & 0x80000000u) | (r->key[i + 1] & 0x7fffffffu);
        r->key[i] = r->key[i + MT_M] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
    }
    for (; i < MT_N - 1; i++) {
        y = (r->key[i] & 0x80000000u) | (r->key[i + 1] & 0x7fffffffu);
        r->key[i] = r->key[i + (MT_M - MT_N)] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
    }
    y = (r->key[MT_N - 1] & 0x80000000u) | (r->key[0] & 0x7fffffffu);
    r->key[MT_N - 1] = r->key[MT_M - 1] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
    r->pos = 0;
}

static uint32_t rs_u32(ora_rs* r) {
    if (r->pos == MT_N) mt_gen(r);
    uint32_t y = r->key[r->pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

/* mt19937_next_double: 53-bit (a>>5, b>>6) */
static double rs_double(ora_rs* r) {
    int32_t a = (int32_t)(rs_u32(r) >> 5), b = (int32_t)(rs_u32(r) >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

/* RandomState.randint(lo, hi) (legacy, masked rejection on 32-bit draws);
 * rng == 0 consumes nothing (random_bounded_uint64_fill) */
static int64_t rs_randint(ora_rs* r, int64_t lo, int64_t hi) {
    uint64_t rng = (uint64_t)(hi - lo - 1);
    if (rng == 0) return lo;
    if (rng == 0xFFFFFFFFull) return lo + (int64_t)rs_u32(r);
    uint32_t mask = (uint32_t)rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (rs_u32(r) & mask)) > (uint32_t)rng) {
    }
    return lo + (int64_t)v;
}

/* legacy_gauss: polar method with cached second value */
static double rs_gauss(ora_rs* r) {
    if (r->has_gauss) {
        double t = r->gauss;
        r->has_gauss = 0;
        r->gauss = 0.0;
        return t;
    }
    double f, x1, x2, r2;
    do {
        x1 = 2.0 * rs_double(r) - 1.0;
        x2 = 2.0 * rs_double(r) - 1.0;
        r2 = x1 * x1 + x2 * x2;
    } while (r2 >= 1.0 || r2 == 0.0);
    f = sqrt(-2.0 * log(r2) / r2);
    r->gauss = f * x1;
    r->has_gauss = 1;
    return f * x2;
}
static double rs_normal(ora_rs* r, double loc, double scale) { return loc + scale * rs_gauss(r); }
static double rs_exponential(ora_rs* r, double scale) { return scale * -log(1.0 - rs_double(r)); }
static double rs_uniform(ora_rs* r, double lo, double hi) { return lo + (hi - lo) * rs_double(r); }

ora_rs* ora_rs_new(uint32_t seed) {
    ora_rs* r = (ora_rs*)malloc(sizeof(ora_rs));
    rs_seed(r, seed);
    return r;
}
void ora_rs_free(ora_rs* r) { free(r); }
uint32_t ora_rs_u32(ora_rs* r) { return rs_u32(r); }
double ora_rs_double(ora_rs* r) { return rs_double(r); }
int64_t ora_rs_randint(ora_rs* r, int64_t lo, int64_t hi) { return rs_randint(r, lo, hi); }
double ora_rs_normal(ora_rs* r, double loc, double scale) { return rs_normal(r, loc, scale); }
double ora_rs_exponential(ora_rs* r, double scale) { return rs_exponential(r, scale); }
double ora_rs_uniform(ora_rs* r, double lo, double hi) { return rs_uniform(r, lo, hi); }

/* Python round(float) -> int : half-to-even (default FE_TONEAREST rint) */
static int64_t py_round(double x) { return (int64_t)rint(x); }

/* ------------------------------------------------------------------------- */
/* message kinds / trace record (tests/golden/gen_fixtures.py KIND)           */
/* ------------------------------------------------------------------------- */
enum {
    K_WAKEUP = 0, K_WHEN_OPEN_REQ = 1, K_WHEN_CLOSE_REQ = 2, K_WHEN_OPEN = 3, K_WHEN_CLOSE = 4,
    K_SPREAD_REQ = 5, K_SPREAD = 6, K_LAST_REQ = 7, K_LAST = 8, K_TV_REQ = 9, K_TV = 10,
    K_LIMIT = 11, K_CANCEL = 12, K_MODIFY = 13, K_ACCEPTED = 14, K_EXECUTED = 15, K_CANCELLED = 16,
    K_MKT_CLOSED = 17, K_MODIFIED = 18, K_KCANCEL = 19, K_MARKET_DATA = 20,
    K_STREAM_REQ = 21, K_STREAM = 22, /* QUERY_ORDER_STREAM request / reply */
    K_MD_SUB_REQ = 23, K_MD_SUB_CANCEL = 24 /* MARKET_DATA_SUBSCRIPTION_REQUEST / _CANCELLATION */
};
#define MD_LEVELS 10 /* deepest market-data subscription restated (OrderBookImbalanceAgent's 10 levels) */
enum { T_MESSAGE = 1, T_WAKEUP = 2, T_CANCEL_ORDER = 3 };

typedef struct {
    int kind;
    int32_t sender;
    /* order payload */
    int64_t oid;
    int32_t oagent;
    int is_buy;
    int64_t qty, price, fill;
    /* query payload */
    int64_t data;
    int data_float; /* reference returned a python float (daily open price) */
    int has_data;
    int depth, mkt_closed;
    int nb, na;
    int64_t bpx, bq, apx, aq;
    int64_t b2px, a2px; /* second level prices (depth >= 2 replies; DummyRL metrics) */
    int64_t lookback;
    /* MODIFY_ORDER: the agent's current copy of the order (the new order is oid/qty/price) */
    int64_t ooid, oqty, oprice;
    int obuy, oagent2;
    /* MARKET_DATA: level prices and volumes, best first (nb / na levels; bq / aq the best volumes) */
    int64_t lvb[MD_LEVELS], lva[MD_LEVELS], lvbq[MD_LEVELS], lvaq[MD_LEVELS];
    /* MARKET_DATA_SUBSCRIPTION_REQUEST: levels in depth, freq in lookback */
} msg_t;

typedef struct {
    int64_t t;
    int32_t rcp, type;
    uint64_t seq;
    int32_t mi;
} ev_t;

/* ------------------------------------------------------------------------- */
/* order book (util/OrderBook.py)                                             */
/* ------------------------------------------------------------------------- */
typedef struct {
    int64_t id;
    int32_t agent;
    int is_buy;
    int64_t qty, price;
} bord_t;
typedef struct {
    bord_t* o;
    int n, cap;
} level_t;
typedef struct {
    level_t* lv;
    int n, cap;
} side_t;
typedef struct {
    int64_t t, q;
} txn_t;
typedef struct {
    int64_t oid;
    int64_t price; /* "limit_price" and "is_buy_order" of the history entry (HBL reads them) */
    int is_buy;
    txn_t* tx;
    int ntx, captx;
} hent_t;
typedef struct {
    hent_t* e;
    int n, cap;
} epoch_t;

/* ------------------------------------------------------------------------- */
/* agents                                                                     */
/* ------------------------------------------------------------------------- */
enum { AG_EXCHANGE = 0, AG_ZI, AG_NOISE, AG_VALUE, AG_POVMM, AG_MOMENTUM, AG_REPLAY, AG_DUMMYRL, AG_MKTMAKER, AG_HBL, AG_OBI,
       AG_TWAP, AG_SBMM };
/* SpreadBasedMarketMakerAgent's string order ids "<name>_<id>_<n>" (generateNewOrderId,
 * SpreadBasedMarketMakerAgent.py:279-288) as SB_ID_BASE + n: only ever compared for identity, and
 * never equal to an auto id (Order.generateOrderId tests ints against a list of mixed ids) */
#define SB_ID_BASE 0x40000000LL
#define SB_MAX 32 /* ladder deque capacity (2 x num_ticks + 1 = 21 per side at most) */
enum { ST_AWAITING_WAKEUP = 0, ST_INACTIVE, ST_AWAITING_SPREAD, ST_ACTIVE, ST_AWAITING_STREAM, ST_AWAITING_MARKET_DATA };

typedef struct {
    int64_t id;
    int is_buy;
    int64_t qty, price;
} aord_t;

typedef struct {
    int id, type;
    char name[96], tname[96];
    ora_rs rs;
    int64_t cur_time;
    /* TradingAgent */
    int has_open, has_close, mkt_closed, first_wake, has_daily_close, trading;
    int64_t mkt_open, mkt_close;
    int64_t starting_cash, cash, shares;
    aord_t* ord;
    int nord, capord;
    int has_last_trade, last_trade_float;
    int64_t last_trade;
    int has_known, nb, na;
    int64_t bid, bidq, ask, askq;
    int64_t tv;
    int state;
    /* ZI / Value */
    double sigma_n, r_bar, kappa, sigma_s, lambda_a, eta;
    int q_max;
    int64_t R_min, R_max;
    int64_t theta[20];
    double r_t, sigma_t;
    int has_prev_wake;
    int64_t prev_wake;
    int64_t size;
    /* Noise */
    int64_t wakeup_time;
    /* POV market maker */
    double pov;
    int64_t min_size, window, num_ticks, wake_freq, order_size;
    int aw_spread, aw_tv, has_last_mid;
    int64_t last_mid;
    /* Momentum */
    int64_t* mids2;
    int nmid, capmid, n20, n50;
    double avg20, avg50;
    /* MarketMakerAgent (agent/market_makers/MarketMakerAgent.py) */
    int64_t mk_min, mk_max, last_spread;
    int spread_depth;
    /* HeuristicBeliefLearningAgent: L, and the last order stream as absolute history epochs
     * [stream_hi - stream_n + 1, stream_hi] (the reply holds live references to those dicts) */
    int L, stream_n, has_stream;
    int64_t stream_hi;
    /* market-data subscription (MarketMakerAgent / MomentumAgent subscribe=True) and the known
     * level prices of the last MARKET_DATA (TradingAgent.known_bids / known_asks) */
    int subscribe, sub_requested;
    int64_t kb[MD_LEVELS], ka[MD_LEVELS];
    /* OrderBookImbalanceAgent: position state and trailing stop */
    int obi_long, obi_short;
    double obi_stop;
    /* SpreadBasedMarketMakerAgent: current_bids / current_asks (deques of (price, id), index 0 =
     * the left end; both always hold the same number of entries), None until the first ladder */
    int64_t sb_bpx[SB_MAX], sb_bid[SB_MAX], sb_apx[SB_MAX], sb_aid[SB_MAX];
    int sb_n, sb_init;
    int64_t sb_cnt; /* order_id_counter */
} agent_t;

#define HIST_RETIRED 48
struct ora_env {
    char config[32];
    int has_cfg, cfg_log_orders; /* a runtime composition (ora_create_config) and its exchange's log_orders */
    int n;
    agent_t* ag;
    /* exchange (agent 0) */
    int64_t ex_open, ex_close, ex_pipeline, ex_comp;
    int stream_history;
    side_t book[2]; /* 0 bids, 1 asks */
    int64_t last_trade;
    int last_trade_float;
    /* OrderBook.history: hist[0, nhist) the window (history[0] newest), then nret epochs that
     * left it, kept unchanged for QUERY_ORDER_STREAM replies still holding them */
    epoch_t hist[16 + HIST_RETIRED];
    int nhist, nret;
    int64_t epoch_abs; /* absolute number of hist[0]: history shifts so far */
    /* SparseMeanRevertingOracle (one symbol) */
    ora_rs O;
    double o_rbar, o_kappa, o_fundvol, o_lambda, o_msmean, o_msvar;
    int efo; /* ExternalFileOracle (hist_fund_* configs) instead of the SparseMeanRevertingOracle */
    int64_t o_open, o_close, o_pt, o_mst;
    double o_pv, o_msv;
    /* global / kernel / latency RNGs */
    ora_rs G, K, L;
    /* kernel */
    int64_t start, stop, cur;
    int have_cur;
    int64_t* agent_time;
    int64_t* comp_delay;
    int64_t add_delay;
    int lat_mode; /* 0 zero, 1 matrix + noise, 2 cubic model */
    double* lat;  /* n*n */
    int noise_len;
    double jitter, clip, unit;
    ev_t* heap;
    int nheap, capheap;
    msg_t* msgs;
    int* freem;
    int nfree, capmsg, nmsg;
    uint64_t seq;
    int64_t pops;
    uint64_t hash;
    int64_t* trace;
    int64_t trace_cap, trace_len;
    /* ExchangeAgent.subscription_dict (ExchangeAgent.py:342-357) in insertion order, and
     * OrderBook.last_update_ts (None until the first book change) */
    int nsub;
    int32_t sub_agent[128], sub_levels[128], sub_live[128];
    double sub_freq[128];
    int64_t sub_last[128];
    int has_last_update;
    int64_t last_update;
    /* OrderBook.book_log rows (ora_set_book_log): t, n levels, executed qty, average trade
     * price, then n (price, volume) pairs, bids (negative volume) best-first, then asks */
    int book_log;
    int64_t *blg, nblg, capblg;
    /* the device's record stream for the same run (mxa_book_rec: t, price, qty) */
    int64_t *blr, nblr, capblr;
    /* the exchange's own log (ExchangeAgent.log, EXCHANGE_AGENT.bz2) in that stream
     * (ora_set_exchange_log; include/mxa.h MXA_BL_EV_*), and the config's log_orders */
    int exlog, ex_log_orders;
    int done, err;
    char errstr[160];
    int64_t order_counter;
    /* Order._order_ids restricted to what generateOrderId can still meet: the explicit (tape)
     * ids appended in this "process" (auto ids are all below order_counter).  Open addressing,
     * carried across ora_gym_reset like the reference's class attributes (Order.py:8-9) */
    int64_t* used_ids;
    int used_cap, used_n;
    char sym[16]; /* the report's symbol when set (ora_set_symbol): -t/--ticker of replay configs */
    int64_t st_max_heap, st_max_resting, st_max_open, st_resting, st_max_hist_tx;
    char* report;
    int64_t report_len;
    /* Kernel.summaryLog: (agent, event type, int or float value) rows */
    int nsum;
    int* sum_agent;
    int* sum_type;  /* 0 STARTING_CASH, 1 FINAL_CASH_POSITION, 2 ENDING_CASH, 3 FINAL_VALUATION */
    int* sum_isf;
    int64_t* sum_i;
    double* sum_f;
    int ex_has_last; /* OrderBook.last_trade is not None */
    /* ---- marketreplay / ABIDESEnv (GymKernel) ---- */
    int gym;
    int end_step, has_obs, finished;
    double obs[9];
    /* LOBSTER tape (LOBSTEROrdersProcessor output), grouped by timestamp */
    int64_t *tp_t, *tp_oid, *tp_price, *tp_size;
    int8_t* tp_buy;
    int tp_n;
    int64_t* tm;  /* distinct timestamps */
    int* tm_start; /* first record of each group (ntm + 1 entries) */
    int ntm, mr_wi;
    /* replay agent's open orders: open-addressing map oid -> slot */
    int64_t* mr_key;
    int32_t* mr_val;
    int mr_cap, mr_used;
    aord_t* mr_ord;
    int mr_nord, mr_capord;
    /* DummyRLExecutionAgent + ABIDESEnvMetrics */
    int64_t rl_quantity, rl_exec_sum, rl_rem;
    int rl_trade, rl_id; /* DummyRL agent id (2 in ABIDESEnv, 64 in rmsc03_rl) */
    int64_t* hz;
    int nhz;
    int m_cnt, m_head;               /* deque(maxlen=100), index 0 = most recent */
    int64_t m_bid[100], m_ask[100], m_data[100];
    int m_nb[100], m_na[100], m_dnone[100];
    int64_t m_bq, m_aq, m_b2, m_a2;  /* most recent LOB: level-1 qtys, level-2 prices */
    int64_t p0;
    int p0_none, ph_none, ph_n;
};

#define NS_SEC 1000000000LL
#define NS_MIN (60LL * NS_SEC)
#define NS_HOUR (3600LL * NS_SEC)
#define FNV_OFF 0xCBF29CE484222325ull
#define FNV_PRIME 0x100000001B3ull

static void fail(ora_env* e, int code, const char* s) {
    if (!e->err) {
        e->err = code;
        snprintf(e->errstr, sizeof e->errstr, "%s", s);
    }
    e->done = 1;
}

/* ---------------------------- event heap ---------------------------------- */
static int ev_less(const ev_t* a, const ev_t* b) {
    if (a->t != b->t) return a->t < b->t;
    if (a->rcp != b->rcp) return a->rcp < b->rcp;
    if (a->type != b->type) return a->type < b->type;
    return a->seq < b->seq;
}
static void heap_push(ora_env* e, ev_t v) {
    if (e->nheap == e->capheap) {
        e->capheap = e->capheap ? 2 * e->capheap : 256;
        e->heap = (ev_t*)realloc(e->heap, sizeof(ev_t) * e->capheap);
    }
    int i = e->nheap++;
    while (i > 0) {
        int p = (i - 1) >> 1;
        if (!ev_less(&v, &e->heap[p])) break;
        e->heap[i] = e->heap[p];
        i = p;
    }
    e->heap[i] = v;
    if (e->nheap > e->st_max_heap) e->st_max_heap = e->nheap;
}
static ev_t heap_pop(ora_env* e) {
    ev_t top = e->heap[0];
    ev_t last = e->heap[--e->nheap];
    int i = 0, n = e->nheap;
    for (;;) {
        int l = 2 * i + 1, r = l + 1, m = i;
        const ev_t* best = &last;
        if (l < n && ev_less(&e->heap[l], best)) { m = l; best = &e->heap[l]; }
        if (r < n && ev_less(&e->heap[r], best)) { m = r; best = &e->heap[r]; }
        if (m == i) break;
        e->heap[i] = e->heap[m];
        i = m;
    }
    if (n > 0) e->heap[i] = last;
    return top;
}
static int msg_alloc(ora_env* e) {
    if (e->nfree) return e->freem[--e->nfree];
    if (e->nmsg == e->capmsg) {
        e->capmsg = e->capmsg ? 2 * e->capmsg : 256;
        e->msgs = (msg_t*)realloc(e->msgs, sizeof(msg_t) * e->capmsg);
        e->freem = (int*)realloc(e->freem, sizeof(int) * e->capmsg);
    }
    return e->nmsg++;
}
static void msg_free(ora_env* e, int mi) { e->freem[e->nfree++] = mi; }

/* ---------------------------- kernel services ----------------------------- */
/* LatencyModel.get_latency, cubic (model/LatencyModel.py:119-140) */
static double get_latency(ora_env* e, int s, int r) {
    double x = rs_uniform(&e->L, e->clip, 1.0);
    double m = e->lat[(size_t)s * e->n + r];
    return m + ((e->jitter / pow(x, 3.0)) * (m / e->unit));
}

/* Kernel.sendMessage (Kernel.py:347-425) */
static void k_send(ora_env* e, int sender, int recipient, const msg_t* m, int64_t delay) {
    int64_t sent = e->cur + e->comp_delay[sender] + e->add_delay + delay;
    int64_t deliver;
    if (e->lat_mode == 2) {
        double lat = get_latency(e, sender, recipient);
        deliver = sent + (int64_t)lat; /* pd.Timedelta(float) truncates */
    } else {
        double lat = e->lat_mode == 1 ? e->lat[(size_t)sender * e->n + recipient] : 0.0;
        int64_t noise = e->noise_len > 1 ? rs_randint(&e->K, 0, e->noise_len) : 0; /* choice(len,1,list) */
        deliver = sent + (int64_t)(lat + (double)noise);
    }
    int mi = msg_alloc(e);
    e->msgs[mi] = *m;
    ev_t v = {deliver, recipient, T_MESSAGE, e->seq++, mi};
    heap_push(e, v);
}

/* Kernel.setWakeup (Kernel.py:435-462) */
static void k_wakeup(ora_env* e, int sender, int64_t t) {
    if (e->have_cur && t < e->cur) {
        fail(e, -3, "setWakeup() called with requested time not in future");
        return;
    }
    ev_t v = {t, sender, T_WAKEUP, e->seq++, -1};
    heap_push(e, v);
}

/* Order._order_ids for explicit ids (Order.py:27-28: every Order appends its id) */
static int used_has(const ora_env* e, int64_t id) {
    if (!e->used_n) return 0;
    for (uint64_t i = (uint64_t)id * 0x9E3779B97F4A7C15ull >> 40;; i++) {
        int64_t k = e->used_ids[i & (uint64_t)(e->used_cap - 1)];
        if (k == id) return 1;
        if (k == -1) return 0;
    }
}
static void used_add(ora_env* e, int64_t id) {
    if (used_has(e, id)) return;
    if (2 * (e->used_n + 1) > e->used_cap) {
        int64_t* old = e->used_ids;
        int oc = e->used_cap;
        e->used_cap = oc ? 2 * oc : 1024;
        e->used_ids = (int64_t*)malloc(sizeof(int64_t) * e->used_cap);
        for (int i = 0; i < e->used_cap; i++) e->used_ids[i] = -1;
        e->used_n = 0;
        for (int i = 0; i < oc; i++)
            if (old[i] != -1) used_add(e, old[i]);
        free(old);
    }
    for (uint64_t i = (uint64_t)id * 0x9E3779B97F4A7C15ull >> 40;; i++) {
        int64_t* k = &e->used_ids[i & (uint64_t)(e->used_cap - 1)];
        if (*k == -1) {
            *k = id;
            e->used_n++;
            return;
        }
    }
}
/* Order.generateOrderId (util/order/Order.py:35-42): the smallest id >= the class counter that
 * no Order of this process has taken yet; order_counter holds the next candidate */
static int64_t next_order_id(ora_env* e) {
    int64_t c = e->order_counter;
    while (used_has(e, c)) c++;
    e->order_counter = c + 1;
    return c;
}

/* --------------------------- oracle (SMRO) -------------------------------- */
static void blr_push(ora_env* e, int64_t t, int64_t price, int64_t qty);
#define BL_FUNDAMENTAL (-2147483647 - 1) /* f_log records in the book-record stream */
#define BL_FUND_LO (-2147483647)           /* ExternalFileOracle f_log: the value's low word */
#define BL_FUND_HI (-2147483646)           /* ... and its high word */
#define BL_MODIFY (1 << 30)                /* modifyOrder: -(price | BL_MODIFY | side << 29), volume delta */
#define BL_EV_RX (-2147483647 - 1 + 256)    /* the exchange's log: a message it logs on receipt, qty = sender */
#define BL_EV_NT (BL_EV_RX + 256)           /* ... an ORDER_* notification it sends (log_orders), qty = recipient */
#define BL_EV_PLACE (BL_EV_RX + 512)        /* ... an order created (time_placed), qty = order id */
#define BL_FILL_NONE (-2147483647 - 1)      /* an order record's fill_price None */
/* compute_fundamental_at_timestamp (SMRO:88-125); f_log append at SMRO:122 */
static double o_compute(ora_env* e, int64_t ts, double v_adj, int64_t pt, double pv) {
    int64_t d = ts - pt;
    double mu = e->o_rbar, gamma = e->o_kappa, theta = e->o_fundvol;
    double loc = mu + (pv - mu) * exp(-gamma * (double)d);
    double scale = (pow(theta, 2.0) / (2 * gamma)) * (1 - exp(-2 * gamma * (double)d));
    double v = rs_normal(&e->O, loc, scale);
    v += v_adj;
    if (!(v > 0)) v = 0; /* max(0, v) */
    int64_t vi = py_round(v);
    e->o_pt = ts;
    e->o_pv = (double)vi;
    if (e->book_log) blr_push(e, ts, BL_FUNDAMENTAL, vi);
    return (double)vi;
}
/* advance_fundamental_value_series (SMRO:131-181) */
static double o_advance(ora_env* e, int64_t t) {
    int64_t pt = e->o_pt;
    double pv = e->o_pv;
    if (t <= pt) return pv;
    while (e->o_mst < t) {
        double v = o_compute(e, e->o_mst, e->o_msv, pt, pv);
        pt = e->o_mst;
        pv = v;
        e->o_mst = pt + (int64_t)rs_exponential(&e->G, 1.0 / e->o_lambda);
        double msv = rs_normal(&e->O, e->o_msmean, sqrt(e->o_msvar));
        e->o_msv = rs_randint(&e->O, 0, 2) == 0 ? msv : -msv;
    }
    return o_compute(e, t, 0, pt, pv);
}
/* ExternalFileOracle (util/oracle/ExternalFileOracle.py) on a series set once per process
 * (ora_set_fundamental; test infrastructure like the rest of this file) */
static int64_t* g_fs_t;
static double* g_fs_v;
static int g_fs_n;
void ora_set_fundamental(const int64_t* t, const double* v, int n) {
    free(g_fs_t);
    free(g_fs_v);
    g_fs_t = (int64_t*)malloc(sizeof(int64_t) * n);
    g_fs_v = (double*)malloc(sizeof(double) * n);
    memcpy(g_fs_t, t, sizeof(int64_t) * n);
    memcpy(g_fs_v, v, sizeof(double) * n);
    g_fs_n = n;
}
/* pandas Timedelta.total_seconds(): days * 86400 + seconds + microseconds / 1e6 of the duration
 * floored to whole microseconds */
static int64_t floor_div(int64_t a, int64_t b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
static double td_seconds(int64_t ns) {
    int64_t us = floor_div(ns, 1000), s = floor_div(us, 1000000);
    return (double)s + (double)(us - s * 1000000) / 1000000.0;
}
/* getPriceAtTime (ExternalFileOracle.py:52-97) + getInterpolatedPrice (:131-159) */
static void blr_push(ora_env* e, int64_t t, int64_t price, int64_t qty);
/* ExternalFileOracle.f_log entry (ExternalFileOracle.py:97) as two book-log records (the value's
 * low and high words; include/mxa.h, mxa_layout.h BL_FUND_LO / BL_FUND_HI) */
static void efo_log(ora_env* e, int64_t t, double v) {
    uint64_t b;
    memcpy(&b, &v, 8);
    blr_push(e, t, BL_FUND_LO, (int32_t)(uint32_t)b);
    blr_push(e, t, BL_FUND_HI, (int32_t)(uint32_t)(b >> 32));
}
/* getPriceAtTime (ExternalFileOracle.py:52-97); e (nullable) logs the interpolating branch's value */
static double efo_price_e(ora_env* e, int64_t t) {
    int n = g_fs_n;
    if (t < g_fs_t[0]) return g_fs_v[0];
    if (t > g_fs_t[n - 1]) return g_fs_v[n - 1];
    int lo = 0, hi = n;
    while (lo < hi) { /* bisect_left */
        int mid = (lo + hi) / 2;
        if (g_fs_t[mid] < t) lo = mid + 1;
        else hi = mid;
    }
    int li = lo - 1, ui = li < n - 1 ? li + 1 : li;
    if (li < 0) li += n; /* fundamental_series[-1] */
    double pl = g_fs_v[li], ph = g_fs_v[ui];
    double slope = pl != ph ? (ph - pl) / td_seconds(g_fs_t[ui] - g_fs_t[li]) : 0.0;
    double v = pl + td_seconds(t - g_fs_t[li]) * slope;
    if (e && e->book_log) efo_log(e, t, v);
    return v;
}
static double efo_price(int64_t t) { return efo_price_e(NULL, t); }

/* observePrice (SMRO:210-227; ExternalFileOracle.py:110-129) */
static int64_t o_observe(ora_env* e, int64_t t, double sigma_n, ora_rs* rs) {
    if (e->efo) {
        double tp = efo_price_e(e, t);
        if (sigma_n == 0) return py_round(tp);
        return py_round(rs_normal(rs, tp, sqrt(sigma_n)));
    }
    double r_t = t >= e->o_close ? o_advance(e, e->o_close - 1) : o_advance(e, t);
    if (sigma_n == 0) return (int64_t)r_t;
    return py_round(rs_normal(rs, r_t, sqrt(sigma_n)));
}

/* ------------------------------ trace -------------------------------------- */
static void encode(const ora_env* e, const ev_t* v, int64_t rec[10]) {
    memset(rec, 0, sizeof(int64_t) * 10);
    rec[0] = v->t;
    rec[1] = v->rcp;
    rec[2] = v->type;
    if (v->mi < 0) {
        rec[3] = v->type == T_WAKEUP ? K_WAKEUP : K_KCANCEL;
        return;
    }
    const msg_t* m = &e->msgs[v->mi];
    int64_t* f = rec + 4;
    rec[3] = m->kind;
    switch (m->kind) {
    case K_WHEN_OPEN_REQ: case K_WHEN_CLOSE_REQ: case K_LAST_REQ:
        f[0] = m->sender;
        break;
    case K_WHEN_OPEN: case K_WHEN_CLOSE:
        f[0] = m->data;
        break;
    case K_SPREAD_REQ:
        f[0] = m->sender;
        f[1] = m->depth;
        break;
    case K_SPREAD:
        f[0] = m->nb ? m->bpx : -1;
        f[1] = m->nb ? m->bq : 0;
        f[2] = m->na ? m->apx : -1;
        f[3] = m->na ? m->aq : 0;
        f[4] = !m->has_data ? -1 : (m->data_float ? m->data * 10000 : m->data);
        f[5] = (m->mkt_closed ? 1 : 0) + 2 * (int64_t)m->nb + ((int64_t)1 << 20) * m->na;
        break;
    case K_LAST:
        f[0] = !m->has_data ? -1 : (m->data_float ? m->data * 10000 : m->data);
        f[5] = m->mkt_closed ? 1 : 0;
        break;
    case K_TV_REQ:
        f[0] = m->sender;
        f[1] = m->lookback;
        break;
    case K_TV:
        f[0] = m->data;
        f[5] = m->mkt_closed ? 1 : 0;
        break;
    case K_LIMIT: case K_ACCEPTED: case K_CANCELLED: case K_MODIFY:
        f[0] = m->oid; f[1] = m->oagent; f[2] = m->is_buy; f[3] = m->qty; f[4] = m->price;
        break;
    case K_MODIFIED: /* quantity left out: the reference message aliases the live book order */
    case K_CANCEL:
        f[0] = m->oid; f[1] = m->oagent; f[2] = m->is_buy; f[3] = 0; f[4] = m->price;
        break;
    case K_EXECUTED:
        f[0] = m->oid; f[1] = m->oagent; f[2] = m->is_buy; f[3] = m->qty; f[4] = m->price; f[5] = m->fill;
        break;
    case K_STREAM_REQ:
        f[0] = m->sender;
        f[1] = m->depth;
        break;
    case K_STREAM:
        f[0] = m->data;
        f[5] = m->mkt_closed ? 1 : 0;
        break;
    case K_MARKET_DATA:
        f[0] = m->nb ? m->bpx : -1;
        f[1] = m->nb ? m->bq : 0;
        f[2] = m->na ? m->apx : -1;
        f[3] = m->na ? m->aq : 0;
        f[4] = m->data_float ? m->data * 10000 : m->data;
        f[5] = (int64_t)m->nb + ((int64_t)m->na << 8);
        break;
    case K_MD_SUB_REQ:
        f[0] = m->sender;
        f[1] = m->depth;
        f[2] = m->lookback;
        break;
    case K_MD_SUB_CANCEL:
        f[0] = m->sender;
        break;
    default:
        break;
    }
}

/* ------------------------------ order book --------------------------------- */
static void level_remove(level_t* L, int i) {
    memmove(L->o + i, L->o + i + 1, sizeof(bord_t) * (L->n - i - 1));
    L->n--;
}
static void level_append(level_t* L, bord_t o) {
    if (L->n == L->cap) {
        L->cap = L->cap ? 2 * L->cap : 4;
        L->o = (bord_t*)realloc(L->o, sizeof(bord_t) * L->cap);
    }
    L->o[L->n++] = o;
}
static void side_delete_level(side_t* S, int i) {
    free(S->lv[i].o);
    memmove(S->lv + i, S->lv + i + 1, sizeof(level_t) * (S->n - i - 1));
    S->n--;
}
static void side_insert_level(side_t* S, int i, bord_t o) {
    if (S->n == S->cap) {
        S->cap = S->cap ? 2 * S->cap : 16;
        S->lv = (level_t*)realloc(S->lv, sizeof(level_t) * S->cap);
    }
    memmove(S->lv + i + 1, S->lv + i, sizeof(level_t) * (S->n - i));
    S->n++;
    level_t L = {0, 0, 0};
    level_append(&L, o);
    S->lv[i] = L;
}
static int is_better(const bord_t* a, const bord_t* b) {
    return a->is_buy ? (a->price > b->price) : (a->price < b->price);
}

/* history: epochs of {order_id -> transactions} (OrderBook.py:33, 51-60, 146-149) */
static hent_t* hist_find(epoch_t* ep, int64_t oid) {
    for (int i = 0; i < ep->n; i++)
        if (ep->e[i].oid == oid) return &ep->e[i];
    return NULL;
}
static void hist_add_order(ora_env* e, int64_t oid, int64_t price, int is_buy) {
    epoch_t* ep = &e->hist[0];
    hent_t* h = hist_find(ep, oid);
    if (h) { /* dict re-assignment keeps position, resets value */
        h->ntx = 0;
        h->price = price;
        h->is_buy = is_buy;
        return;
    }
    if (ep->n == ep->cap) {
        ep->cap = ep->cap ? 2 * ep->cap : 16;
        ep->e = (hent_t*)realloc(ep->e, sizeof(hent_t) * ep->cap);
    }
    hent_t n0 = {oid, price, is_buy, NULL, 0, 0};
    ep->e[ep->n++] = n0;
}
static void hent_add_tx(hent_t* h, int64_t t, int64_t q) {
    if (h->ntx == h->captx) {
        h->captx = h->captx ? 2 * h->captx : 2;
        h->tx = (txn_t*)realloc(h->tx, sizeof(txn_t) * h->captx);
    }
    txn_t x = {t, q};
    h->tx[h->ntx++] = x;
}
static void epoch_free(epoch_t* ep) {
    for (int i = 0; i < ep->n; i++) free(ep->e[i].tx);
    free(ep->e);
    ep->e = NULL;
    ep->n = ep->cap = 0;
}
static void hist_shift(ora_env* e) {
    /* history.insert(0, {}); history = history[:stream_history + 1] */
    int keep = e->stream_history + 1;
    if (e->nhist >= keep) { /* the oldest window epochs retire (a stream reply may still read them) */
        e->nret += e->nhist - (keep - 1);
        e->nhist = keep - 1;
    }
    while (e->nhist + e->nret + 1 > 16 + HIST_RETIRED) {
        epoch_free(&e->hist[e->nhist + e->nret - 1]);
        e->nret--;
    }
    memmove(e->hist + 1, e->hist, sizeof(epoch_t) * (e->nhist + e->nret));
    memset(&e->hist[0], 0, sizeof(epoch_t));
    e->nhist++;
    e->epoch_abs++;
}

/* the order a LIMIT_ORDER / CANCEL_ORDER row or an ORDER_* notification row of the exchange's log
 * carries (js.dump(order, strip_privates=True)): t = fill_price << 32 | order id, price = limit
 * price, qty = quantity signed by side (include/mxa.h MXA_BL_EV_*) */
static void exl_order(ora_env* e, const msg_t* m, int64_t fill) {
    blr_push(e, (int64_t)(((uint64_t)(uint32_t)(int32_t)fill << 32) | (uint32_t)(int32_t)m->oid), m->price,
             m->is_buy ? m->qty : -m->qty);
}
static void ex_send(ora_env* e, int recipient, msg_t* m) {
    /* ExchangeAgent.sendMessage: order-book notifications carry the pipeline delay, and with
     * log_orders are logged with their order (ExchangeAgent.py:477-482) */
    int note = m->kind == K_ACCEPTED || m->kind == K_CANCELLED || m->kind == K_EXECUTED;
    int64_t d = note ? e->ex_pipeline : 0;
    if (note && e->exlog && e->ex_log_orders) {
        blr_push(e, e->cur, BL_EV_NT + m->kind, recipient);
        exl_order(e, m, m->kind == K_EXECUTED ? m->fill : BL_FILL_NONE);
    }
    k_send(e, 0, recipient, m, d);
}

static void order_msg(msg_t* m, int kind, const bord_t* o) {
    memset(m, 0, sizeof *m);
    m->kind = kind;
    m->oid = o->id;
    m->oagent = o->agent;
    m->is_buy = o->is_buy;
    m->qty = o->qty;
    m->price = o->price;
    m->fill = -1;
}

/* executeOrder (OrderBook.py:172-240); returns 1 and fills *matched if a match happened */
static int execute_order(ora_env* e, bord_t* order, bord_t* matched) {
    side_t* book = &e->book[order->is_buy ? 1 : 0];
    if (book->n == 0) return 0;
    bord_t* head = &book->lv[0].o[0];
    int match = order->is_buy ? (order->price >= head->price) : (order->price <= head->price);
    if (!match) return 0;
    if (order->qty >= head->qty) {
        *matched = *head;
        e->st_resting--;
        level_remove(&book->lv[0], 0);
        if (book->lv[0].n == 0) side_delete_level(book, 0);
    } else {
        *matched = *head;
        matched->qty = order->qty;
        head->qty -= matched->qty;
    }
    /* history[0][order.order_id]['transactions'].append((t, order.quantity)) */
    hent_t* h = hist_find(&e->hist[0], order->id);
    if (h) hent_add_tx(h, e->cur, order->qty);
    for (int i = 0; i < e->nhist; i++) {
        hent_t* hm = hist_find(&e->hist[i], matched->id);
        if (hm) hent_add_tx(hm, e->cur, matched->qty);
    }
    return 1;
}

/* enterOrder (OrderBook.py:256-282) */
static void enter_order(ora_env* e, bord_t o) {
    if (++e->st_resting > e->st_max_resting) e->st_max_resting = e->st_resting;
    side_t* book = &e->book[o.is_buy ? 0 : 1];
    if (book->n == 0) {
        side_insert_level(book, 0, o);
        return;
    }
    bord_t* last = &book->lv[book->n - 1].o[0];
    if (!is_better(&o, last) && o.price != last->price) {
        side_insert_level(book, book->n, o);
        return;
    }
    for (int i = 0; i < book->n; i++) {
        bord_t* h = &book->lv[i].o[0];
        if (is_better(&o, h)) {
            side_insert_level(book, i, o);
            return;
        }
        if (o.price == h->price) {
            level_append(&book->lv[i], o);
            return;
        }
    }
}

static void blr_push(ora_env* e, int64_t t, int64_t price, int64_t qty) {
    if (e->nblr + 3 > e->capblr) {
        e->capblr = e->capblr ? 2 * e->capblr : 4096;
        e->blr = (int64_t*)realloc(e->blr, sizeof(int64_t) * e->capblr);
    }
    e->blr[e->nblr++] = t;
    e->blr[e->nblr++] = price;
    e->blr[e->nblr++] = qty;
}
static void blg_push(ora_env* e, int64_t w) {
    if (e->nblg == e->capblg) {
        e->capblg = e->capblg ? 2 * e->capblg : 4096;
        e->blg = (int64_t*)realloc(e->blg, sizeof(int64_t) * e->capblg);
    }
    e->blg[e->nblg++] = w;
}
/* the tail of handleLimitOrder (OrderBook.py:112-168): BEST_BID / BEST_ASK / LAST_TRADE come
 * from the first levels and the executed list; the book_log row holds every level
 * (getInsideBids/getInsideAsks with the default depth), bids as negative volumes */
static void book_log_row(ora_env* e, int64_t ex_q, int64_t avg) {
    blg_push(e, e->cur);
    blg_push(e, e->book[0].n + e->book[1].n);
    blg_push(e, ex_q);
    blg_push(e, avg);
    for (int s = 0; s < 2; s++)
        for (int i = 0; i < e->book[s].n; i++) {
            const level_t* L = &e->book[s].lv[i];
            int64_t v = 0;
            for (int j = 0; j < L->n; j++) v += L->o[j].qty;
            blg_push(e, L->o[0].price);
            blg_push(e, s == 0 ? -v : v);
        }
}

/* handleLimitOrder (OrderBook.py:38-170) */
static void handle_limit_order(ora_env* e, bord_t order) {
    if (order.qty <= 0) return;
    if (e->book_log) blr_push(e, e->cur, order.price, order.is_buy ? order.qty : -order.qty);
    hist_add_order(e, order.id, order.price, order.is_buy);
    int64_t ex_q = 0, ex_pq = 0;
    int executed = 0;
    for (;;) {
        bord_t matched;
        if (execute_order(e, &order, &matched)) {
            bord_t filled = order;
            filled.qty = matched.qty;
            order.qty -= filled.qty;
            msg_t m;
            order_msg(&m, K_EXECUTED, &filled);
            m.fill = matched.price;
            ex_send(e, order.agent, &m);
            order_msg(&m, K_EXECUTED, &matched);
            m.fill = matched.price;
            ex_send(e, matched.agent, &m);
            ex_q += filled.qty;
            ex_pq += matched.price * filled.qty;
            executed = 1;
            if (order.qty <= 0) break;
        } else {
            enter_order(e, order);
            msg_t m;
            order_msg(&m, K_ACCEPTED, &order);
            ex_send(e, order.agent, &m);
            break;
        }
    }
    if (executed) {
        e->last_trade = py_round((double)ex_pq / (double)ex_q);
        e->last_trade_float = 0;
        e->ex_has_last = 1;
        hist_shift(e);
    }
    if (e->book_log) book_log_row(e, ex_q, executed ? e->last_trade : 0);
    e->last_update = e->cur; /* OrderBook.py:169 */
    e->has_last_update = 1;
}

/* cancelOrder (OrderBook.py:284-339) */
static void cancel_order(ora_env* e, const msg_t* req) {
    side_t* book = &e->book[req->is_buy ? 0 : 1];
    for (int i = 0; i < book->n; i++) {
        level_t* L = &book->lv[i];
        if (L->o[0].price != req->price) continue;
        for (int j = 0; j < L->n; j++) {
            if (L->o[j].id == req->oid) {
                bord_t c = L->o[j];
                if (e->book_log) blr_push(e, e->cur, -c.price, req->is_buy ? c.qty : -c.qty);
                e->st_resting--;
                level_remove(L, j);
                if (L->n == 0) side_delete_level(book, i);
                msg_t m;
                order_msg(&m, K_CANCELLED, &c);
                ex_send(e, req->oagent, &m);
                e->last_update = e->cur; /* OrderBook.py:338 */
                e->has_last_update = 1;
                return;
            }
        }
    }
}

/* modifyOrder (OrderBook.py:341-372).  Reference quirk kept: every order at the level
 * whose id matches replaces the level HEAD (book[i][0] = new_order), not itself, and one
 * ORDER_MODIFIED goes to the requester per history epoch that holds the id. */
static void modify_order(ora_env* e, const msg_t* req) {
    if (req->ooid != req->oid) return; /* isSameOrder(order, new_order) (OrderBook.py:343-344) */
    side_t* book = &e->book[req->obuy ? 0 : 1];
    if (book->n == 0) return;
    e->last_update = e->cur; /* OrderBook.py:372 (nothing below returns early) */
    e->has_last_update = 1;
    bord_t nw = {req->oid, req->oagent, req->is_buy, req->qty, req->price};
    for (int i = 0; i < book->n; i++) {
        level_t* L = &book->lv[i];
        if (L->o[0].price != req->oprice) continue;
        const int64_t head_q = L->o[0].qty;
        int hit = 0;
        for (int j = 0; j < L->n; j++) {
            if (L->o[j].id != req->ooid) continue;
            if (!hit++ && e->book_log) /* the level's volume changes by new - old head (BL_MODIFY) */
                blr_push(e, e->cur, -(req->oprice | BL_MODIFY | ((req->obuy ? 0 : 1) << 29)), nw.qty - head_q);
            L->o[0] = nw;
            for (int h = 0; h < e->nhist; h++) {
                if (!hist_find(&e->hist[h], nw.id)) continue;
                msg_t m;
                order_msg(&m, K_MODIFIED, &nw);
                k_send(e, 0, req->oagent2, &m, 0);
            }
        }
    }
}

/* get_transacted_volume (OrderBook.py:400-436), restated: distinct (t, qty) pairs of
 * all transaction records in the retained history with t >= now - lookback. */
static int cmp_txn(const void* a, const void* b) {
    const txn_t *x = (const txn_t*)a, *y = (const txn_t*)b;
    if (x->t != y->t) return x->t < y->t ? -1 : 1;
    if (x->q != y->q) return x->q < y->q ? -1 : 1;
    return 0;
}
static int64_t transacted_volume(ora_env* e, int64_t lookback, int* err) {
    int entries = 0, ntx = 0;
    for (int i = 0; i < e->nhist; i++) {
        entries += e->hist[i].n;
        for (int j = 0; j < e->hist[i].n; j++) ntx += e->hist[i].e[j].ntx;
    }
    if (entries == 0) return 0;
    if (ntx == 0) { /* pandas raises AttributeError here (no transaction records) */
        *err = 1;
        return 0;
    }
    txn_t* all = (txn_t*)malloc(sizeof(txn_t) * ntx);
    int k = 0;
    for (int i = 0; i < e->nhist; i++)
        for (int j = 0; j < e->hist[i].n; j++)
            for (int t = 0; t < e->hist[i].e[j].ntx; t++) all[k++] = e->hist[i].e[j].tx[t];
    qsort(all, ntx, sizeof(txn_t), cmp_txn);
    if (ntx > e->st_max_hist_tx) e->st_max_hist_tx = ntx;
    int64_t start = e->cur - lookback, vol = 0;
    for (int i = 0; i < ntx; i++) {
        if (i > 0 && cmp_txn(&all[i], &all[i - 1]) == 0) continue;
        if (all[i].t >= start) vol += all[i].q;
    }
    free(all);
    return vol;
}

/* ExchangeAgent.publishOrderBookData (ExchangeAgent.py:359-387): after every LIMIT / CANCEL /
 * MODIFY, each subscription in insertion order gets the top `levels` of both sides and the last
 * trade when freq == 0 or the book changed at least freq ns after its last update */
static void publish(ora_env* e) {
    for (int i = 0; i < e->nsub; i++) {
        if (!e->sub_live[i]) continue;
        if (e->sub_freq[i] != 0) {
            if (!e->has_last_update) { /* None > Timestamp */
                fail(e, -14, "publishOrderBookData: book never updated (TypeError comparing None)");
                return;
            }
            if (!(e->last_update > e->sub_last[i] && (double)(e->last_update - e->sub_last[i]) >= e->sub_freq[i]))
                continue;
        }
        msg_t r;
        memset(&r, 0, sizeof r);
        r.kind = K_MARKET_DATA;
        int lv = e->sub_levels[i];
        const side_t* b = &e->book[0];
        const side_t* a = &e->book[1];
        r.nb = b->n < lv ? b->n : lv;
        r.na = a->n < lv ? a->n : lv;
        if (r.nb > MD_LEVELS || r.na > MD_LEVELS) {
            fail(e, -15, "market-data subscription deeper than the restated levels");
            return;
        }
        for (int k = 0; k < r.nb; k++) {
            r.lvb[k] = b->lv[k].o[0].price;
            for (int j = 0; j < b->lv[k].n; j++) r.lvbq[k] += b->lv[k].o[j].qty;
        }
        for (int k = 0; k < r.na; k++) {
            r.lva[k] = a->lv[k].o[0].price;
            for (int j = 0; j < a->lv[k].n; j++) r.lvaq[k] += a->lv[k].o[j].qty;
        }
        if (r.nb) {
            r.bpx = r.lvb[0];
            r.bq = r.lvbq[0];
        }
        if (r.na) {
            r.apx = r.lva[0];
            r.aq = r.lvaq[0];
        }
        r.data = e->last_trade;
        r.data_float = e->last_trade_float;
        r.has_data = 1;
        ex_send(e, e->sub_agent[i], &r);
        e->sub_last[i] = e->last_update;
    }
}

/* ExchangeAgent.updateSubscriptionDict (ExchangeAgent.py:342-357): a request (re)sets the
 * agent's entry, keeping its place in the dict; a cancellation empties it */
static void update_subscription(ora_env* e, const msg_t* m) {
    int i = 0;
    while (i < e->nsub && e->sub_agent[i] != m->sender) i++;
    if (m->kind == K_MD_SUB_CANCEL) {
        if (i == e->nsub || !e->sub_live[i]) { /* del of a missing key */
            fail(e, -16, "MARKET_DATA_SUBSCRIPTION_CANCELLATION without a subscription (KeyError)");
            return;
        }
        e->sub_live[i] = 0;
        return;
    }
    if (i == e->nsub) {
        if (e->nsub == 128) {
            fail(e, -15, "too many market-data subscriptions");
            return;
        }
        e->nsub++;
    }
    e->sub_agent[i] = m->sender;
    e->sub_levels[i] = m->depth;
    e->sub_freq[i] = (double)m->lookback;
    e->sub_last[i] = e->cur;
    e->sub_live[i] = 1;
}

/* ExchangeAgent.receiveMessage (ExchangeAgent.py:129-340) */
static void ex_receive(ora_env* e, const msg_t* m) {
    e->comp_delay[0] = e->ex_comp;
    int closed = e->cur > e->ex_close;
    msg_t r;
    memset(&r, 0, sizeof r);
    if (closed) {
        if (m->kind == K_LIMIT || m->kind == K_CANCEL || m->kind == K_MODIFY) {
            r.kind = K_MKT_CLOSED;
            ex_send(e, m->sender, &r);
            return;
        } else if (m->kind == K_SPREAD_REQ || m->kind == K_LAST_REQ || m->kind == K_TV_REQ || m->kind == K_STREAM_REQ) {
        } else {
            r.kind = K_MKT_CLOSED;
            ex_send(e, m->sender, &r);
            return;
        }
    }
    /* Log order messages only with log_orders, every other message with its sender
     * (ExchangeAgent.py:162-167) */
    if (e->exlog) {
        int ord = m->kind == K_LIMIT || m->kind == K_CANCEL;
        if (!ord || e->ex_log_orders) {
            blr_push(e, e->cur, BL_EV_RX + m->kind, m->sender);
            if (ord) exl_order(e, m, BL_FILL_NONE);
        }
    }
    if (m->kind == K_MD_SUB_REQ || m->kind == K_MD_SUB_CANCEL) update_subscription(e, m);
    switch (m->kind) {
    case K_WHEN_OPEN_REQ:
    case K_WHEN_CLOSE_REQ:
        e->comp_delay[0] = 0;
        r.kind = m->kind == K_WHEN_OPEN_REQ ? K_WHEN_OPEN : K_WHEN_CLOSE;
        r.data = m->kind == K_WHEN_OPEN_REQ ? e->ex_open : e->ex_close;
        r.has_data = 1;
        ex_send(e, m->sender, &r);
        break;
    case K_LAST_REQ:
        r.kind = K_LAST;
        r.data = e->last_trade;
        r.data_float = e->last_trade_float;
        r.has_data = e->ex_has_last;
        r.mkt_closed = closed;
        ex_send(e, m->sender, &r);
        break;
    case K_SPREAD_REQ: {
        r.kind = K_SPREAD;
        r.depth = m->depth;
        side_t* b = &e->book[0];
        side_t* a = &e->book[1];
        r.nb = b->n < m->depth ? b->n : m->depth;
        r.na = a->n < m->depth ? a->n : m->depth;
        if (r.nb) {
            r.bpx = b->lv[0].o[0].price;
            for (int j = 0; j < b->lv[0].n; j++) r.bq += b->lv[0].o[j].qty;
        }
        if (r.na) {
            r.apx = a->lv[0].o[0].price;
            for (int j = 0; j < a->lv[0].n; j++) r.aq += a->lv[0].o[j].qty;
        }
        if (r.nb > 1) r.b2px = b->lv[1].o[0].price;
        if (r.na > 1) r.a2px = a->lv[1].o[0].price;
        r.data = e->last_trade;
        r.data_float = e->last_trade_float;
        r.has_data = e->ex_has_last;
        r.mkt_closed = closed;
        ex_send(e, m->sender, &r);
        break;
    }
    case K_TV_REQ: {
        int perr = 0;
        int64_t vol = transacted_volume(e, m->lookback, &perr);
        if (perr) {
            fail(e, -5, "get_transacted_volume: no transaction records (pandas AttributeError)");
            return;
        }
        r.kind = K_TV;
        r.data = vol;
        r.has_data = 1;
        r.mkt_closed = closed;
        ex_send(e, m->sender, &r);
        break;
    }
    case K_STREAM_REQ: {
        /* QUERY_ORDER_STREAM (ExchangeAgent.py:251-279): history[1 : length + 1], live references */
        int avail = e->nhist - 1;
        r.kind = K_STREAM;
        r.data = m->depth < avail ? m->depth : avail; /* number of epochs returned */
        if (r.data < 0) r.data = 0;
        r.lookback = e->epoch_abs - 1; /* absolute number of history[1] */
        r.mkt_closed = closed;
        ex_send(e, m->sender, &r);
        break;
    }
    case K_LIMIT: {
        bord_t o = {m->oid, m->oagent, m->is_buy, m->qty, m->price};
        handle_limit_order(e, o);
        if (e->nsub) publish(e);
        break;
    }
    case K_CANCEL:
        cancel_order(e, m);
        if (e->nsub) publish(e);
        break;
    case K_MODIFY:
        modify_order(e, m);
        if (e->nsub) publish(e);
        break;
    default:
        break;
    }
}

/* --------------------------- TradingAgent --------------------------------- */
static void ta_send_ex(ora_env* e, agent_t* a, msg_t* m) {
    m->sender = a->id;
    /* an order created now (LimitOrder(agent, currentTime, ...)): its time_placed, for the
     * exchange's log rows that carry it */
    if (e->exlog && e->ex_log_orders && (m->kind == K_LIMIT || m->kind == K_MODIFY))
        blr_push(e, e->cur, BL_EV_PLACE, m->oid);
    k_send(e, a->id, 0, m, 0);
}
static void get_spread(ora_env* e, agent_t* a, int depth) {
    msg_t m;
    memset(&m, 0, sizeof m);
    m.kind = K_SPREAD_REQ;
    m.depth = depth;
    ta_send_ex(e, a, &m);
}
static void get_tv(ora_env* e, agent_t* a, int64_t lookback) {
    msg_t m;
    memset(&m, 0, sizeof m);
    m.kind = K_TV_REQ;
    m.lookback = lookback;
    ta_send_ex(e, a, &m);
}
/* placeLimitOrder (TradingAgent.py:309-349) */
static void place_limit(ora_env* e, agent_t* a, int64_t qty, int is_buy, int64_t price) {
    int64_t oid = next_order_id(e);
    if (qty > 0) {
        if (a->nord == a->capord) {
            a->capord = a->capord ? 2 * a->capord : 8;
            a->ord = (aord_t*)realloc(a->ord, sizeof(aord_t) * a->capord);
        }
        aord_t o = {oid, is_buy, qty, price};
        a->ord[a->nord++] = o;
        if (a->nord > e->st_max_open) e->st_max_open = a->nord;
        msg_t m;
        memset(&m, 0, sizeof m);
        m.kind = K_LIMIT;
        m.oid = oid;
        m.oagent = a->id;
        m.is_buy = is_buy;
        m.qty = qty;
        m.price = price;
        m.fill = -1;
        ta_send_ex(e, a, &m);
    }
}
/* cancelOrder for every open order, dict insertion order */
static void cancel_all(ora_env* e, agent_t* a) {
    for (int i = 0; i < a->nord; i++) {
        msg_t m;
        memset(&m, 0, sizeof m);
        m.kind = K_CANCEL;
        m.oid = a->ord[i].id;
        m.oagent = a->id;
        m.is_buy = a->ord[i].is_buy;
        m.qty = a->ord[i].qty;
        m.price = a->ord[i].price;
        m.fill = -1;
        ta_send_ex(e, a, &m);
    }
}
static int find_ord(agent_t* a, int64_t oid) {
    for (int i = 0; i < a->nord; i++)
        if (a->ord[i].id == oid) return i;
    return -1;
}
static void del_ord(agent_t* a, int i) {
    memmove(a->ord + i, a->ord + i + 1, sizeof(aord_t) * (a->nord - i - 1));
    a->nord--;
}

/* open-order lookups: the replay agent keeps thousands of orders (hash map), everybody
 * else a short insertion-ordered list */
static int mr_slot(const ora_env* e, int64_t oid, int insert) {
    uint64_t h = (uint64_t)oid * 0x9E3779B97F4A7C15ull;
    int mask = e->mr_cap - 1, tomb = -1;
    for (int i = (int)(h >> 40) & mask;; i = (i + 1) & mask) {
        if (e->mr_key[i] == oid) return i;
        if (e->mr_key[i] == -2 && tomb < 0) tomb = i;
        if (e->mr_key[i] == -1) return insert ? (tomb >= 0 ? tomb : i) : -1;
    }
}
static aord_t* ord_get(ora_env* e, agent_t* a, int64_t oid) {
    if (a->type == AG_REPLAY) {
        int i = mr_slot(e, oid, 0);
        return i >= 0 ? &e->mr_ord[i] : NULL;
    }
    int i = find_ord(a, oid);
    return i >= 0 ? &a->ord[i] : NULL;
}
static void ord_del(ora_env* e, agent_t* a, int64_t oid) {
    if (a->type == AG_REPLAY) {
        int i = mr_slot(e, oid, 0);
        if (i >= 0) {
            e->mr_key[i] = -2;
            e->mr_nord--;
        }
        return;
    }
    int i = find_ord(a, oid);
    if (i >= 0) del_ord(a, i);
}

/* TradingAgent.wakeup (TradingAgent.py:142-158); returns "ready to trade" */
static int ta_wakeup(ora_env* e, agent_t* a) {
    a->cur_time = e->cur;
    if (a->first_wake) a->first_wake = 0;
    if (!a->has_open) {
        msg_t m;
        memset(&m, 0, sizeof m);
        m.kind = K_WHEN_OPEN_REQ;
        ta_send_ex(e, a, &m);
        m.kind = K_WHEN_CLOSE_REQ;
        ta_send_ex(e, a, &m);
    }
    return (a->has_open && a->has_close) && !a->mkt_closed;
}

static int64_t wake_frequency(agent_t* a) {
    switch (a->type) {
    case AG_POVMM: return a->wake_freq;
    case AG_MOMENTUM: return a->wake_freq;
    case AG_MKTMAKER: return a->wake_freq; /* pd.Timedelta(wake_up_freq) (MarketMakerAgent.py:148-149) */
    case AG_OBI: return NS_SEC;           /* pd.Timedelta("1s") (OrderBookImbalanceAgent.py:187-188) */
    case AG_REPLAY: return a->wake_freq;  /* first tape time - mkt_open (MarketReplayAgent.py:94-96) */
    case AG_DUMMYRL: return a->wake_freq; /* horizon[0] - mkt_open (execution_agent.py:129-130) */
    case AG_TWAP: return a->wake_freq;    /* the same ExecutionAgent.getWakeFrequency */
    case AG_SBMM: return a->wake_freq;    /* pd.Timedelta(wake_up_freq) (SpreadBasedMarketMakerAgent.py:290-292) */
    default: return rs_randint(&a->rs, 0, 100);
    }
}

static void query_last_trade(agent_t* a, const msg_t* m) {
    a->has_last_trade = 1;
    a->last_trade = m->data;
    a->last_trade_float = m->data_float;
    if (a->mkt_closed) a->has_daily_close = 1;
}

/* TradingAgent.receiveMessage (TradingAgent.py:181-268) */
static void ta_receive(ora_env* e, agent_t* a, const msg_t* m) {
    a->cur_time = e->cur;
    int had = a->has_open && a->has_close;
    switch (m->kind) {
    case K_WHEN_OPEN: a->mkt_open = m->data; a->has_open = 1; break;
    case K_WHEN_CLOSE: a->mkt_close = m->data; a->has_close = 1; break;
    case K_EXECUTED: { /* orderExecuted (TradingAgent.py:422-462) */
        int64_t q = m->is_buy ? m->qty : -m->qty;
        a->shares += q;
        a->cash -= q * m->fill;
        aord_t* o = ord_get(e, a, m->oid);
        if (o) {
            if (m->qty >= o->qty) ord_del(e, a, m->oid);
            else o->qty -= m->qty;
        }
        break;
    }
    case K_ACCEPTED: break;
    case K_CANCELLED:
        ord_del(e, a, m->oid);
        break;
    case K_MKT_CLOSED: a->mkt_closed = 1; break;
    case K_LAST:
        if (m->mkt_closed) a->mkt_closed = 1;
        query_last_trade(a, m);
        break;
    case K_SPREAD:
        if (m->mkt_closed) a->mkt_closed = 1;
        query_last_trade(a, m);
        a->has_last_trade = m->has_data;
        a->has_known = 1;
        a->nb = m->nb;
        a->na = m->na;
        a->bid = m->bpx;
        a->bidq = m->bq;
        a->ask = m->apx;
        a->askq = m->aq;
        break;
    case K_TV:
        if (m->mkt_closed) a->mkt_closed = 1;
        a->tv = m->data;
        break;
    case K_MARKET_DATA: /* handleMarketData (TradingAgent.py:539-546) */
        a->has_known = 1;
        a->nb = m->nb;
        a->na = m->na;
        a->bid = m->bpx;
        a->bidq = m->bq;
        a->ask = m->apx;
        a->askq = m->aq;
        memcpy(a->kb, m->lvb, sizeof a->kb);
        memcpy(a->ka, m->lva, sizeof a->ka);
        a->has_last_trade = 1;
        a->last_trade = m->data;
        a->last_trade_float = m->data_float;
        break;
    case K_STREAM: /* queryOrderStream (TradingAgent.py:240-246, 549-554) */
        if (m->mkt_closed) a->mkt_closed = 1;
        a->has_stream = 1;
        a->stream_n = (int)m->data;
        a->stream_hi = m->lookback;
        break;
    default: break;
    }
    int have = a->has_open && a->has_close;
    if (have && !had) {
        int64_t off = wake_frequency(a);
        k_wakeup(e, a->id, a->mkt_open + off);
    }
}

/* Bayesian fundamental estimate shared by ZI (ZI.py:215-263) and Value (ValueAgent.py:153-201) */
static int64_t bayes_r_T(ora_env* e, agent_t* a, int64_t obs_t) {
    if (!a->has_prev_wake) {
        a->has_prev_wake = 1;
        a->prev_wake = a->mkt_open;
    }
    double delta = (double)(e->cur - a->prev_wake);
    double c = 1 - a->kappa;
    double r_tprime = (1 - pow(c, delta)) * a->r_bar;
    r_tprime += pow(c, delta) * a->r_t;
    double sigma_tprime = pow(c, 2 * delta) * a->sigma_t;
    sigma_tprime += ((1 - pow(c, 2 * delta)) / (1 - pow(c, 2.0))) * a->sigma_s;
    a->r_t = (a->sigma_n / (a->sigma_n + sigma_tprime)) * r_tprime;
    a->r_t += (sigma_tprime / (a->sigma_n + sigma_tprime)) * (double)obs_t;
    a->sigma_t = (a->sigma_n * a->sigma_t) / (a->sigma_n + a->sigma_t);
    double d2 = (double)(a->mkt_close - e->cur);
    if (!(d2 > 0)) d2 = 0;
    double r_T = (1 - pow(c, d2)) * a->r_bar;
    r_T += pow(c, d2) * a->r_t;
    a->prev_wake = e->cur;
    return py_round(r_T);
}

/* --------------------------- ZeroIntelligenceAgent -------------------------- */
/* ZeroIntelligenceAgent.wakeup (ZI.py:125-187).  A subclass (HBL) does not query the spread
 * here: its state becomes ACTIVE (ZI.py:183-187). */
static void zi_wakeup_as(ora_env* e, agent_t* a, int is_zi) {
    ta_wakeup(e, a);
    a->state = ST_INACTIVE;
    if (!a->has_open || !a->has_close) return;
    a->trading = 1;
    if (a->mkt_closed && a->has_daily_close) return;
    double dt = rs_exponential(&a->rs, 1.0 / a->lambda_a);
    k_wakeup(e, a->id, e->cur + py_round(dt));
    if (a->mkt_closed && !a->has_daily_close) {
        get_spread(e, a, 1);
        a->state = ST_AWAITING_SPREAD;
        return;
    }
    cancel_all(e, a);
    if (is_zi) {
        get_spread(e, a, 1);
        a->state = ST_AWAITING_SPREAD;
    } else {
        a->state = ST_ACTIVE;
    }
}
static void zi_wakeup(ora_env* e, agent_t* a) { zi_wakeup_as(e, a, 1); }
/* updateEstimates (ZI.py:189-275): total unit valuation v and side; 0 on the reference's IndexError */
static int zi_update_estimates(ora_env* e, agent_t* a, int64_t* v_out, int* buy_out) {
    int64_t obs = o_observe(e, e->cur, a->sigma_n, &a->rs);
    int64_t q = (int64_t)((double)a->shares / 100); /* int(h / 100): truncation */
    int buy;
    if (q >= a->q_max) buy = 0;
    else if (q <= -a->q_max) buy = 1;
    else buy = (int)rs_randint(&a->rs, 0, 2);
    int64_t r_T = bayes_r_T(e, a, obs);
    q += a->q_max - 1;
    int64_t idx = buy ? q + 1 : q;
    if (idx < 0) idx += 20; /* python negative index */
    if (idx < 0 || idx >= 20) {
        fail(e, -6, "ZeroIntelligenceAgent theta index out of range (IndexError)");
        return 0;
    }
    *v_out = r_T + a->theta[idx];
    *buy_out = buy;
    return 1;
}
static void zi_place(ora_env* e, agent_t* a) {
    int64_t v;
    int buy;
    if (!zi_update_estimates(e, a, &v, &buy)) return;
    /* placeOrder (ZI.py:277-309) */
    int64_t R = rs_randint(&a->rs, a->R_min, a->R_max + 1);
    int64_t p = buy ? v - R : v + R;
    int64_t bid = a->nb ? a->bid : 0, bid_vol = a->nb ? a->bidq : 0;
    int64_t ask = a->na ? a->ask : 0, ask_vol = a->na ? a->askq : 0;
    if (buy && ask_vol > 0) {
        int64_t R_ask = v - ask;
        if ((double)R_ask >= a->eta * (double)R) p = ask;
    } else if (!buy && bid_vol > 0) {
        int64_t R_bid = bid - v;
        if ((double)R_bid >= a->eta * (double)R) p = bid;
    }
    place_limit(e, a, 100, buy, p);
}
static void zi_receive(ora_env* e, agent_t* a, const msg_t* m) {
    ta_receive(e, a, m);
    if (a->state == ST_AWAITING_SPREAD && m->kind == K_SPREAD) {
        if (a->mkt_closed) return;
        zi_place(e, a);
        a->state = ST_AWAITING_WAKEUP;
    }
}

/* ------------------------------- ValueAgent -------------------------------- */
static void value_wakeup(ora_env* e, agent_t* a) {
    ta_wakeup(e, a);
    a->state = ST_INACTIVE;
    if (!a->has_open || !a->has_close) return;
    a->trading = 1;
    if (a->mkt_closed && a->has_daily_close) return;
    double dt = rs_exponential(&a->rs, 1.0 / a->lambda_a);
    k_wakeup(e, a->id, e->cur + py_round(dt));
    if (a->mkt_closed && !a->has_daily_close) {
        get_spread(e, a, 1);
        a->state = ST_AWAITING_SPREAD;
        return;
    }
    cancel_all(e, a);
    get_spread(e, a, 1);
    a->state = ST_AWAITING_SPREAD;
}
static void value_place(ora_env* e, agent_t* a) {
    int64_t obs = o_observe(e, e->cur, a->sigma_n, &a->rs);
    int64_t r_T = bayes_r_T(e, a, obs);
    int have_bid = a->nb && a->bid != 0, have_ask = a->na && a->ask != 0;
    int buy;
    int64_t p;
    if (have_bid && have_ask) {
        int64_t mid = (int64_t)((double)(a->ask + a->bid) / 2);
        int64_t spread = llabs(a->ask - a->bid);
        int64_t adj;
        if (rs_double(&e->G) < 0.1) adj = 0;
        else adj = rs_randint(&e->G, 0, 2 * spread);
        if (r_T < mid) {
            buy = 0;
            p = a->bid + adj;
        } else {
            buy = 1;
            p = a->ask - adj;
        }
    } else {
        buy = (int)rs_randint(&e->G, 0, 2);
        p = r_T;
    }
    place_limit(e, a, a->size, buy, p);
}
static void value_receive(ora_env* e, agent_t* a, const msg_t* m) {
    ta_receive(e, a, m);
    if (a->state == ST_AWAITING_SPREAD && m->kind == K_SPREAD) {
        if (a->mkt_closed) return;
        value_place(e, a);
        a->state = ST_AWAITING_WAKEUP;
    }
}

/* ------------------------------- NoiseAgent -------------------------------- */
static void noise_wakeup(ora_env* e, agent_t* a) {
    ta_wakeup(e, a);
    a->state = ST_INACTIVE;
    if (!a->has_open || !a->has_close) return;
    a->trading = 1;
    if (a->mkt_closed && a->has_daily_close) return;
    if (a->wakeup_time > e->cur) k_wakeup(e, a->id, a->wakeup_time);
    if (a->mkt_closed && !a->has_daily_close) {
        get_spread(e, a, 1);
        a->state = ST_AWAITING_SPREAD;
        return;
    }
    get_spread(e, a, 1);
    a->state = ST_AWAITING_SPREAD;
}
static void noise_receive(ora_env* e, agent_t* a, const msg_t* m) {
    ta_receive(e, a, m);
    if (a->state == ST_AWAITING_SPREAD && m->kind == K_SPREAD) {
        if (a->mkt_closed) return;
        int buy = (int)rs_randint(&e->G, 0, 2);
        int have_bid = a->nb && a->bid != 0, have_ask = a->na && a->ask != 0;
        if (buy && have_ask) place_limit(e, a, a->size, 1, a->ask);
        else if (!buy && have_bid) place_limit(e, a, a->size, 0, a->bid);
        a->state = ST_AWAITING_WAKEUP;
    }
}

/* --------------------------- POVMarketMakerAgent ---------------------------- */
static void mm_wakeup(ora_env* e, agent_t* a) {
    int can_trade = ta_wakeup(e, a);
    if (can_trade) {
        get_spread(e, a, 1);
        get_tv(e, a, a->wake_freq);
    }
}
static void mm_receive(ora_env* e, agent_t* a, const msg_t* m) {
    ta_receive(e, a, m);
    int64_t mid = a->last_mid;
    if (m->kind == K_TV && a->aw_tv) {
        int64_t qty = py_round(a->pov * (double)a->tv);
        a->order_size = qty >= a->min_size ? qty : a->min_size;
        a->aw_tv = 0;
    }
    if (m->kind == K_SPREAD && a->aw_spread) {
        int have_bid = a->nb && a->bid != 0, have_ask = a->na && a->ask != 0;
        if (have_bid && have_ask) {
            mid = (int64_t)((double)(a->ask + a->bid) / 2);
            a->last_mid = mid;
            a->has_last_mid = 1;
            a->aw_spread = 0;
        }
    }
    if (!a->aw_spread && !a->aw_tv) {
        cancel_all(e, a);
        int64_t hb = mid - 1, la = mid + a->window;
        int64_t lb = hb - a->num_ticks, ha = la + a->num_ticks;
        for (int64_t p = lb; p <= hb; p++) place_limit(e, a, a->order_size, 1, p);
        for (int64_t p = la; p <= ha; p++) place_limit(e, a, a->order_size, 0, p);
        a->aw_spread = a->aw_tv = 1;
        k_wakeup(e, a->id, e->cur + a->wake_freq);
    }
}

/* ------------------------------- MomentumAgent ------------------------------ */
static double mom_avg(agent_t* a, int n) {
    /* MomentumAgent.ma(mid_list, n)[-1].round(2): exact half-integer sums */
    int64_t s2 = 0;
    for (int i = a->nmid - n; i < a->nmid; i++) s2 += a->mids2[i];
    double x = ((double)s2 / 2.0) / (double)n;
    return rint(x * 100.0) / 100.0;
}
/* TradingAgent.requestDataSubscription (TradingAgent.py:160-172) */
static void request_subscription(ora_env* e, agent_t* a, int levels, int64_t freq) {
    msg_t m;
    memset(&m, 0, sizeof m);
    m.kind = K_MD_SUB_REQ;
    m.depth = levels;
    m.lookback = freq;
    ta_send_ex(e, a, &m);
    a->sub_requested = 1;
}
/* MomentumAgent.placeOrders (MomentumAgent.py:82-93) */
static void mom_place(ora_env* e, agent_t* a, int64_t bid, int64_t ask) {
    if (!(bid && ask)) return;
    if (a->nmid == a->capmid) {
        a->capmid = a->capmid ? 2 * a->capmid : 64;
        a->mids2 = (int64_t*)realloc(a->mids2, sizeof(int64_t) * a->capmid);
    }
    a->mids2[a->nmid++] = bid + ask;
    if (a->nmid > 20) { a->avg20 = mom_avg(a, 20); a->n20++; }
    if (a->nmid > 50) { a->avg50 = mom_avg(a, 50); a->n50++; }
    if (a->n20 > 0 && a->n50 > 0) {
        if (a->avg20 >= a->avg50) place_limit(e, a, a->size, 1, ask);
        else place_limit(e, a, a->size, 0, bid);
    }
}
/* MomentumAgent.wakeup / receiveMessage (MomentumAgent.py:54-80); subscribe=True requests
 * level-1 data every 10 s on the first wakeup and trades on each MARKET_DATA */
static void mom_wakeup(ora_env* e, agent_t* a) {
    int can_trade = ta_wakeup(e, a);
    if (a->subscribe && !a->sub_requested) {
        request_subscription(e, a, 1, 10000000000LL);
        a->state = ST_AWAITING_MARKET_DATA;
    } else if (can_trade && !a->subscribe) {
        get_spread(e, a, 1);
        a->state = ST_AWAITING_SPREAD;
    }
}
static void mom_receive(ora_env* e, agent_t* a, const msg_t* m) {
    ta_receive(e, a, m);
    if (!a->subscribe && a->state == ST_AWAITING_SPREAD && m->kind == K_SPREAD) {
        /* getKnownBidAsk: the best levels or None */
        mom_place(e, a, a->nb ? a->bid : 0, a->na ? a->ask : 0);
        k_wakeup(e, a->id, e->cur + a->wake_freq);
        a->state = ST_AWAITING_WAKEUP;
    } else if (a->subscribe && a->state == ST_AWAITING_MARKET_DATA && m->kind == K_MARKET_DATA) {
        if (a->nb && a->na) mom_place(e, a, a->kb[0], a->ka[0]); /* `if bids and asks` (lists) */
    }
}


/* --------------------------- MarketMakerAgent ------------------------------ */
/* agent/market_makers/MarketMakerAgent.py, polling mode (subscribe=False) */
static void mk_wakeup(ora_env* e, agent_t* a) {
    int can_trade = ta_wakeup(e, a); /* MarketMakerAgent.py:69-79 */
    if (a->subscribe && !a->sub_requested) {
        request_subscription(e, a, a->spread_depth, 10000000000LL); /* subscribe_freq 10e9 */
        a->state = ST_AWAITING_MARKET_DATA;
    } else if (can_trade && !a->subscribe) {
        cancel_all(e, a);
        get_spread(e, a, a->spread_depth);
        a->state = ST_AWAITING_SPREAD;
    }
}
/* DEFAULT_LEVELS_QUOTE_DICT (MarketMakerAgent.py:6-12) */
static const double MK_SPLIT[6][5] = {{0}, {1, 0, 0, 0, 0}, {0.5, 0.5, 0, 0, 0}, {0.34, 0.33, 0.33, 0, 0},
                                      {0.25, 0.25, 0.25, 0.25, 0}, {0.20, 0.20, 0.20, 0.20, 0.20}};
/* MarketMakerAgent.receiveMessage subscribe branch + placeOrders (MarketMakerAgent.py:109-141):
 * cancel every open order, 1-4 levels (randint(1, 5)), one size draw, then per side a dict
 * price -> volume in first-insertion order, a missing level i quoting one cent beyond the last
 * known level (repeated misses overwrite that one entry) */
static void mk_market_data(ora_env* e, agent_t* a) {
    cancel_all(e, a);
    int nl = (int)rs_randint(&a->rs, 1, 5);
    if (!(a->nb && a->na)) return;
    a->size = (int64_t)rint((double)rs_randint(&a->rs, a->mk_min, a->mk_max) / 2);
    for (int side = 1; side >= 0; side--) { /* buy quotes first, then sell */
        const int64_t* lv = side ? a->kb : a->ka;
        int n = side ? a->nb : a->na;
        int64_t px[5], vol[5];
        int k = 0;
        for (int i = 0; i < nl; i++) {
            int64_t v = (int64_t)rint(MK_SPLIT[nl][i] * (double)a->size);
            int64_t p = i < n ? lv[i] : (side ? lv[n - 1] - 1 : lv[n - 1] + 1);
            int j = 0;
            while (j < k && px[j] != p) j++;
            if (j == k) px[k++] = p;
            vol[j] = v;
        }
        for (int j = 0; j < k; j++) place_limit(e, a, vol[j], side, px[j]);
    }
}
static void mk_receive(ora_env* e, agent_t* a, const msg_t* m) {
    ta_receive(e, a, m); /* MarketMakerAgent.py:81-107 */
    if (a->subscribe) {
        if (a->state == ST_AWAITING_MARKET_DATA && m->kind == K_MARKET_DATA) mk_market_data(e, a);
        return;
    }
    if (!(a->state == ST_AWAITING_SPREAD && m->kind == K_SPREAD)) return;
    cancel_all(e, a);
    int64_t mid = a->last_trade, spread;
    /* getKnownBidAsk: best levels or None; `if bid and ask` (0 is falsy too) */
    if (a->nb && a->na && a->bid && a->ask) {
        mid = (int64_t)((double)(a->ask + a->bid) / 2);
        spread = (int64_t)((double)llabs(a->ask - a->bid) / 2);
    } else {
        if (a->last_trade_float) { /* mid = the opening price, a python float: float prices (not restated) */
            fail(e, -13, "MarketMakerAgent: ladder priced from a float last trade (not restated)");
            return;
        }
        spread = a->last_spread;
    }
    for (int i = 0; i < 2 * a->spread_depth; i++) {
        a->size = (int64_t)rint((double)rs_randint(&a->rs, a->mk_min, a->mk_max) / 2); /* round(x / 2) */
        place_limit(e, a, a->size, 1, mid - spread - i);
        place_limit(e, a, a->size, 0, mid + spread + i);
    }
    k_wakeup(e, a->id, e->cur + a->wake_freq);
    a->state = ST_AWAITING_WAKEUP;
}

/* ------------------------ SpreadBasedMarketMakerAgent ------------------------ */
/* agent/market_makers/SpreadBasedMarketMakerAgent.py: the Chakraborty-Kearns ladder of num_ticks + 1
 * one-cent levels per side around the mid, shifted by whole ticks as the mid moves */
/* placeLimitOrder(..., order_id=<the ladder's id>) (TradingAgent.py:309-349) */
static void place_limit_id(ora_env* e, agent_t* a, int64_t qty, int is_buy, int64_t price, int64_t oid) {
    if (qty <= 0) return;
    if (a->nord == a->capord) {
        a->capord = a->capord ? 2 * a->capord : 8;
        a->ord = (aord_t*)realloc(a->ord, sizeof(aord_t) * a->capord);
    }
    aord_t o = {oid, is_buy, qty, price};
    a->ord[a->nord++] = o;
    if (a->nord > e->st_max_open) e->st_max_open = a->nord;
    msg_t m;
    memset(&m, 0, sizeof m);
    m.kind = K_LIMIT;
    m.oid = oid;
    m.oagent = a->id;
    m.is_buy = is_buy;
    m.qty = qty;
    m.price = price;
    m.fill = -1;
    ta_send_ex(e, a, &m);
}
/* cancelOrders (:166-179): self.orders[id] -> cancelOrder; an id no longer open is a KeyError, skipped */
static void cancel_oid(ora_env* e, agent_t* a, int64_t oid) {
    int i = find_ord(a, oid);
    if (i < 0) return;
    msg_t m;
    memset(&m, 0, sizeof m);
    m.kind = K_CANCEL;
    m.oid = oid;
    m.oagent = a->id;
    m.is_buy = a->ord[i].is_buy;
    m.qty = a->ord[i].qty;
    m.price = a->ord[i].price;
    m.fill = -1;
    ta_send_ex(e, a, &m);
}
static int64_t sb_new_id(agent_t* a) { return SB_ID_BASE + ++a->sb_cnt; } /* generateNewOrderId */
static void sb_pop(int64_t* px, int64_t* id, int n, int left, int64_t* out_id) {
    if (left) {
        *out_id = id[0];
        memmove(px, px + 1, sizeof(int64_t) * (n - 1));
        memmove(id, id + 1, sizeof(int64_t) * (n - 1));
    } else {
        *out_id = id[n - 1];
    }
}
static void sb_push(int64_t* px, int64_t* id, int n, int left, int64_t p, int64_t oid) {
    if (left) {
        memmove(px + 1, px, sizeof(int64_t) * n);
        memmove(id + 1, id, sizeof(int64_t) * n);
        px[0] = p;
        id[0] = oid;
    } else {
        px[n] = p;
        id[n] = oid;
    }
}
/* computeOrdersToCancel + cancelOrders + placeOrders (receiveMessage :111-113 / :128-130) at `mid`;
 * self.last_mid is still the previous mid here */
static void sb_update(ora_env* e, agent_t* a, int64_t mid) {
    /* computeOrdersToCancel (:134-164): per tick of the move one order from each deque, the lowest
     * levels on a rise (popleft), the highest on a fall (pop); an empty deque is ignored */
    int64_t cancel[2 * SB_MAX];
    int nc = 0;
    if (a->sb_init) {
        const int64_t k = mid - a->last_mid;
        for (int64_t i = 0; i < (k > 0 ? k : -k) && a->sb_n > 0; i++) {
            sb_pop(a->sb_bpx, a->sb_bid, a->sb_n, k > 0, &cancel[nc++]);
            sb_pop(a->sb_apx, a->sb_aid, a->sb_n, k > 0, &cancel[nc++]);
            a->sb_n--;
        }
    }
    for (int i = 0; i < nc; i++) cancel_oid(e, a, cancel[i]);
    /* computeOrdersToPlace (:181-238), placeOrders (:240-255): bids first, then asks */
    int64_t bp[SB_MAX], bi[SB_MAX], ap[SB_MAX], ai[SB_MAX];
    int np = 0;
    if (!a->sb_init || a->sb_n == 0) {
        cancel_all(e, a); /* cancelAllOrders (:294-297): every order of self.orders */
        /* initialiseBidsAsksDeques (:257-277), anchor "bottom" */
        const int64_t hb = mid - 1, la = mid + a->window, lb = hb - a->num_ticks, ha = la + a->num_ticks;
        const int nl = (int)(hb - lb + 1);
        if (nl > SB_MAX || nl <= 0) {
            fail(e, -19, "SpreadBasedMarketMakerAgent: ladder width beyond the restated deque");
            return;
        }
        for (int i = 0; i < nl; i++) {
            a->sb_bpx[i] = lb + i;
            a->sb_bid[i] = sb_new_id(a);
        }
        for (int i = 0; i < nl; i++) {
            a->sb_apx[i] = la + i;
            a->sb_aid[i] = sb_new_id(a);
        }
        (void)ha;
        a->sb_n = nl;
        a->sb_init = 1;
        for (int i = 0; i < nl; i++) place_limit_id(e, a, a->order_size, 1, a->sb_bpx[i], a->sb_bid[i]);
        for (int i = 0; i < nl; i++) place_limit_id(e, a, a->order_size, 0, a->sb_apx[i], a->sb_aid[i]);
        return;
    }
    const int64_t k = a->has_last_mid ? mid - a->last_mid : 0;
    if (k > 0) {
        const int64_t b0 = a->sb_bpx[a->sb_n - 1], a0 = a->sb_apx[a->sb_n - 1];
        for (int64_t inc = 1; inc <= k; inc++) {
            bp[np] = b0 + inc;
            bi[np] = sb_new_id(a);
            ap[np] = a0 + inc;
            ai[np] = sb_new_id(a);
            sb_push(a->sb_bpx, a->sb_bid, a->sb_n, 0, bp[np], bi[np]);
            sb_push(a->sb_apx, a->sb_aid, a->sb_n, 0, ap[np], ai[np]);
            a->sb_n++;
            np++;
        }
    } else if (k < 0) {
        const int64_t b0 = a->sb_bpx[0], a0 = a->sb_apx[0];
        for (int64_t inc = 1; inc <= -k; inc++) {
            bp[np] = b0 - inc;
            bi[np] = sb_new_id(a);
            ap[np] = a0 - inc;
            ai[np] = sb_new_id(a);
            sb_push(a->sb_bpx, a->sb_bid, a->sb_n, 1, bp[np], bi[np]);
            sb_push(a->sb_apx, a->sb_aid, a->sb_n, 1, ap[np], ai[np]);
            a->sb_n++;
            np++;
        }
    }
    for (int i = 0; i < np; i++) place_limit_id(e, a, a->order_size, 1, bp[i], bi[i]);
    for (int i = 0; i < np; i++) place_limit_id(e, a, a->order_size, 0, ap[i], ai[i]);
}
/* wakeup (:75-84) */
static void sb_wakeup(ora_env* e, agent_t* a) {
    int can_trade = ta_wakeup(e, a);
    if (a->subscribe && !a->sub_requested) {
        request_subscription(e, a, 1, 10000000000LL); /* subscribe_num_levels 1, subscribe_freq 10e9 */
        a->state = ST_AWAITING_MARKET_DATA;
    } else if (can_trade && !a->subscribe) {
        get_spread(e, a, 1);
        a->state = ST_AWAITING_SPREAD;
    }
}
/* receiveMessage (:86-132) */
static void sb_receive(ora_env* e, agent_t* a, const msg_t* m) {
    ta_receive(e, a, m);
    if (!a->subscribe && a->state == ST_AWAITING_SPREAD && m->kind == K_SPREAD) {
        int64_t mid = a->last_mid;
        /* getKnownBidAsk: the best levels or None; `if bid and ask` */
        if (a->nb && a->na && a->bid && a->ask) {
            mid = (int64_t)((double)(a->ask + a->bid) / 2);
        } else if (!a->has_last_mid) { /* `mid` never bound: UnboundLocalError */
            fail(e, -18, "SpreadBasedMarketMakerAgent: no spread and no last mid (UnboundLocalError)");
            return;
        }
        sb_update(e, a, mid);
        k_wakeup(e, a->id, e->cur + a->wake_freq);
        a->state = ST_AWAITING_WAKEUP;
        a->last_mid = mid;
        a->has_last_mid = 1;
    } else if (a->subscribe && a->state == ST_AWAITING_MARKET_DATA && m->kind == K_MARKET_DATA) {
        /* known_bids[symbol][0][0] if known_bids[symbol] else None */
        if (!(a->nb && a->na && a->kb[0] && a->ka[0])) return;
        const int64_t mid = (int64_t)((double)(a->ka[0] + a->kb[0]) / 2);
        sb_update(e, a, mid);
        a->last_mid = mid;
        a->has_last_mid = 1;
    }
}

/* ------------------------- OrderBookImbalanceAgent ---------------------------- */
/* agent/OrderBookImbalanceAgent.py: every wakeup (re)subscribes to 10 levels every hour and sets
 * its computation delay to 1 ns (wakeup, :67-71); each MARKET_DATA cancels its orders and trades
 * the bid share of the top-10 liquidity against entry / trailing-stop thresholds (:73-186) */
static void obi_wakeup(ora_env* e, agent_t* a) {
    ta_wakeup(e, a);
    msg_t m;
    memset(&m, 0, sizeof m);
    m.kind = K_MD_SUB_REQ;
    m.depth = 10;
    m.lookback = 3600000000000LL;
    ta_send_ex(e, a, &m);
    e->comp_delay[a->id] = 1; /* setComputationDelay(1) */
}
static void obi_receive(ora_env* e, agent_t* a, const msg_t* m) {
    ta_receive(e, a, m);
    if (m->kind != K_MARKET_DATA) return;
    cancel_all(e, a);
    int64_t bl = 0, al = 0;
    for (int k = 0; k < m->nb; k++) bl += m->lvbq[k];
    for (int k = 0; k < m->na; k++) al += m->lvaq[k];
    if (bl == 0 || al == 0) return; /* "zero bid or ask liquidity" */
    const double entry = 0.17, trail = 0.085;
    double bid_pct = (double)bl / (double)(bl + al);
    int64_t target;
    if (a->obi_short) {
        if (bid_pct - trail > a->obi_stop) a->obi_stop = bid_pct - trail;
        if (bid_pct < a->obi_stop) {
            target = 0;
            a->obi_short = 0;
        } else {
            target = -100;
        }
    } else if (a->obi_long) {
        if (bid_pct + trail < a->obi_stop) a->obi_stop = bid_pct + trail;
        if (bid_pct > a->obi_stop) {
            target = 0;
            a->obi_long = 0;
        } else {
            target = 100;
        }
    } else if (bid_pct < (0.5 - entry)) {
        target = 100;
        a->obi_long = 1;
        a->obi_stop = bid_pct + trail;
    } else if (bid_pct > (0.5 + entry)) {
        target = -100;
        a->obi_short = 1;
        a->obi_stop = bid_pct - trail;
    } else {
        target = 0;
    }
    int64_t delta = target - a->shares;
    int dir = delta > 0;
    /* computeRequiredPrice (:190-206): the loop leaves p at the deepest level either way */
    int n = dir ? m->na : m->nb;
    int64_t price = dir ? m->lva[n - 1] : m->lvb[n - 1];
    if (delta != 0) place_limit(e, a, delta > 0 ? delta : -delta, dir, price);
}

/* ------------------------- HeuristicBeliefLearningAgent ----------------------- */
/* agent/HeuristicBeliefLearningAgent.py */
static void hbl_wakeup(ora_env* e, agent_t* a) {
    zi_wakeup_as(e, a, 0); /* HBL.py:61-73 */
    if (a->state != ST_ACTIVE) return;
    msg_t m;
    memset(&m, 0, sizeof m);
    m.kind = K_STREAM_REQ; /* getOrderStream(symbol, length=L) (TradingAgent.py:285-289) */
    m.depth = a->L;
    ta_send_ex(e, a, &m);
    a->state = ST_AWAITING_STREAM;
}
/* HBL.placeOrder (HBL.py:75-195): the orders of the streamed history epochs as they are NOW (the
 * reply held references to the exchange's live dicts), dense over [low_p, high_p] as written */
static void hbl_place(ora_env* e, agent_t* a) {
    if (!a->has_stream || a->stream_n < a->L) { /* insufficient history: exactly ZI.placeOrder */
        zi_place(e, a);
        return;
    }
    int64_t v;
    int buy;
    if (!zi_update_estimates(e, a, &v, &buy)) return;
    int64_t low_p = INT64_MAX, high_p = 0;
    int nent = 0;
    for (int k = 0; k < a->stream_n; k++) {
        int64_t idx = e->epoch_abs - (a->stream_hi - k);
        if (idx < 1 || idx >= e->nhist + e->nret) {
            fail(e, -11, "HBL: streamed history epoch beyond the retained history");
            return;
        }
        const epoch_t* ep = &e->hist[idx];
        for (int j = 0; j < ep->n; j++) {
            int64_t p = ep->e[j].price;
            if (p < low_p) low_p = p;
            if (p > high_p) high_p = p;
            nent++;
        }
    }
    if (nent == 0 || high_p - low_p + 1 <= 0) {
        fail(e, -12, "HBL: empty order stream (numpy ValueError)");
        return;
    }
    int64_t np_ = high_p - low_p + 1;
    double* nd = (double*)calloc((size_t)np_ * 8, sizeof(double)); /* sa, sb, ua, ub, num, denom, Pr, Es */
#define ND(i, c) nd[(size_t)(i) * 8 + (c)]
    for (int k = 0; k < a->stream_n; k++) {
        const epoch_t* ep = &e->hist[e->epoch_abs - (a->stream_hi - k)];
        for (int j = 0; j < ep->n; j++) {
            int64_t i = ep->e[j].price - low_p;
            int tx = ep->e[j].ntx > 0;
            if (ep->e[j].is_buy) ND(i, tx ? 1 : 3) += 1;
            else ND(i, tx ? 0 : 2) += 1;
        }
    }
    if (buy) {
        for (int64_t i = 1; i < np_; i++)
            for (int c = 0; c < 3; c++) ND(i, c) += ND(i - 1, c);
        for (int64_t i = np_ - 2; i >= 0; i--) ND(i, 3) += ND(i + 1, 3);
        for (int64_t i = 0; i < np_; i++) ND(i, 4) = ND(i, 0) + ND(i, 1) + ND(i, 2);
    } else {
        for (int64_t i = np_ - 2; i >= 0; i--) {
            ND(i, 0) += ND(i + 1, 0);
            ND(i, 1) += ND(i + 1, 1);
            ND(i, 3) += ND(i + 1, 3);
        }
        for (int64_t i = 1; i < np_; i++) ND(i, 2) += ND(i - 1, 2);
        for (int64_t i = 0; i < np_; i++) ND(i, 4) = ND(i, 0) + ND(i, 1) + ND(i, 3);
    }
    int64_t best = 0;
    for (int64_t i = 0; i < np_; i++) {
        ND(i, 5) = ND(i, 0) + ND(i, 1) + ND(i, 2) + ND(i, 3);
        double pr = ND(i, 4) / ND(i, 5);
        if (isnan(pr)) pr = 0.0; /* np.nan_to_num (inf cannot occur: num <= denom) */
        ND(i, 6) = pr;
        ND(i, 7) = pr * (double)(buy ? v - (low_p + i) : (low_p + i) - v);
        if (ND(i, 7) > ND(best, 7)) best = i; /* np.argmax: first maximum */
    }
    double best_es = ND(best, 7);
    free(nd);
#undef ND
    if (best_es > 0) place_limit(e, a, 100, buy, low_p + best);
}
static void hbl_receive(ora_env* e, agent_t* a, const msg_t* m) {
    ta_receive(e, a, m);
    /* ZeroIntelligenceAgent.receiveMessage (ZI.py:311-334), placeOrder dispatching to HBL's */
    if (a->state == ST_AWAITING_SPREAD && m->kind == K_SPREAD) {
        if (a->mkt_closed) return;
        hbl_place(e, a);
        a->state = ST_AWAITING_WAKEUP;
    }
    /* HBL.receiveMessage (HBL.py:197-217) */
    if (a->state == ST_AWAITING_STREAM && m->kind == K_STREAM) {
        if (a->mkt_closed) return;
        get_spread(e, a, 1);
        a->state = ST_AWAITING_SPREAD;
    }
}

/* ------------------------ marketreplay / ABIDESEnv -------------------------- */
/* MarketReplayAgent.placeOrder (MarketReplayAgent.py:69-91) for one tape record.
 * ORDER_ID 0: `self.orders.get(0)` finds only an order whose auto id is 0, and
 * LimitOrder(..., order_id=0) takes the next auto id (Order.py:26, generateOrderId), both when
 * placing and when building the modify's new order (whose id then differs: isSameOrder fails
 * at the exchange, OrderBook.py:343-344).  In a later episode of the same process
 * (ora_gym_reset) no order of this agent holds auto id 0, and auto ids skip every explicit id
 * the process has used (next_order_id). */
static void mr_place(ora_env* e, agent_t* a, int r) {
    int64_t oid = e->tp_oid[r], size = e->tp_size[r], price = e->tp_price[r];
    int buy = e->tp_buy[r];
    int slot = mr_slot(e, oid, 0);
    /* placing and modifying both build LimitOrder(..., order_id=ORDER_ID): an explicit id joins
     * Order._order_ids (a cancel or a size-0 record of an unknown id builds nothing) */
    if (oid && size > 0) used_add(e, oid);
    msg_t m;
    memset(&m, 0, sizeof m);
    m.fill = -1;
    if (slot < 0 && size > 0) { /* placeLimitOrder(..., order_id=ORDER_ID) */
        int64_t id = oid ? oid : next_order_id(e);
        int i = mr_slot(e, id, 1);
        e->mr_key[i] = id;
        aord_t o = {id, buy, size, price};
        e->mr_ord[i] = o;
        if (++e->mr_nord > e->st_max_open) e->st_max_open = e->mr_nord;
        m.kind = K_LIMIT;
        m.oid = id;
        m.oagent = a->id;
        m.is_buy = buy;
        m.qty = size;
        m.price = price;
        ta_send_ex(e, a, &m);
    } else if (slot >= 0 && size == 0) { /* cancelOrder(existing_order) */
        aord_t* o = &e->mr_ord[slot];
        m.kind = K_CANCEL;
        m.oid = o->id;
        m.oagent = a->id;
        m.is_buy = o->is_buy;
        m.qty = o->qty;
        m.price = o->price;
        ta_send_ex(e, a, &m);
    } else if (slot >= 0) { /* modifyOrder(existing_order, LimitOrder(..., order_id)) */
        aord_t* o = &e->mr_ord[slot];
        m.kind = K_MODIFY;
        m.oid = oid ? oid : next_order_id(e);
        m.oagent = a->id;
        m.is_buy = buy;
        m.qty = size;
        m.price = price;
        m.ooid = o->id;
        m.oqty = o->qty;
        m.oprice = o->price;
        m.obuy = o->is_buy;
        m.oagent2 = a->id;
        ta_send_ex(e, a, &m);
    }
}
/* MarketReplayAgent.wakeup (MarketReplayAgent.py:50-61).  The wakeup list starts with the
 * first tape time, which is also the first wake time: that group is submitted twice and the
 * last group never (both reference behaviour). */
static void mr_wakeup(ora_env* e, agent_t* a) {
    ta_wakeup(e, a);
    if (!(a->has_open && a->has_close)) return;
    if (e->mr_wi >= e->ntm) return; /* IndexError: all orders submitted */
    k_wakeup(e, a->id, e->tm[e->mr_wi]);
    e->mr_wi++;
    int lo = 0, hi = e->ntm - 1, g = -1;
    while (lo <= hi) {
        int mid = (lo + hi) / 2;
        if (e->tm[mid] == e->cur) { g = mid; break; }
        if (e->tm[mid] < e->cur) lo = mid + 1;
        else hi = mid - 1;
    }
    if (g < 0) {
        fail(e, -7, "MarketReplayAgent: no tape orders at wake time (KeyError)");
        return;
    }
    for (int r = e->tm_start[g]; r < e->tm_start[g + 1]; r++) mr_place(e, a, r);
}
static void mr_receive(ora_env* e, agent_t* a, const msg_t* m) { ta_receive(e, a, m); }

/* GymKernel.setCancelOrder (GymKernel.py:364-389) via DummyRL.setCancelOrder: the requested
 * time minus pd.Timedelta(0.5), which truncates to 0 ns */
static void k_cancel_order(ora_env* e, int sender, int64_t t) {
    if (t < e->cur) {
        fail(e, -3, "setCancelOrder() called with requested time not in future");
        return;
    }
    ev_t v = {t, sender, T_CANCEL_ORDER, e->seq++, -1};
    heap_push(e, v);
}
/* DummyRLExecutionAgent.wakeup (dummy_rl_execution_agent.py:181-213) */
static void rl_wakeup(ora_env* e, agent_t* a) {
    if (!ta_wakeup(e, a)) return;
    if (e->rl_trade) {
        int k = -1;
        for (int i = 0; i < e->nhz; i++)
            if (e->hz[i] > e->cur) { k = i; break; }
        if (k >= 0) k_cancel_order(e, a->id, e->hz[k]);
        else e->rl_trade = 0;
    }
    if (e->rl_trade) { /* effective_time_horizon = execution_time_horizon[:-1] */
        int k = -1;
        for (int i = 0; i < e->nhz - 1; i++)
            if (e->hz[i] > e->cur) { k = i; break; }
        if (k >= 0) k_wakeup(e, a->id, e->hz[k]);
        else e->rl_trade = 0;
    }
    get_spread(e, a, 500);
    a->state = ST_AWAITING_SPREAD;
}
/* TWAPExecutionAgent (agent/execution/baselines/twap_agent.py:9-63) runs ExecutionAgent.wakeup
 * (execution_agent.py:65-76): the next horizon time strictly after now (IndexError: no wakeup),
 * then QUERY_SPREAD at depth 500 */
static void tw_wakeup(ora_env* e, agent_t* a) {
    if (!ta_wakeup(e, a)) return;
    if (!e->rl_trade) return;
    for (int i = 0; i < e->nhz; i++)
        if (e->hz[i] > e->cur) {
            k_wakeup(e, a->id, e->hz[i]);
            break;
        }
    get_spread(e, a, 500);
    a->state = ST_AWAITING_SPREAD;
}
/* ExecutionAgent.receiveMessage / placeOrders (execution_agent.py:78-123).  The schedule is keyed
 * by the 60 s intervals of pd.interval_range(start, end, freq) (twap_agent.py:50-55) and looked up
 * with a 30 s interval (execution_agent.py:118): the first limit order raises KeyError, so no
 * TWAP order ever reaches the exchange and ORDER_EXECUTED / ORDER_ACCEPTED never arrive. */
static void tw_receive(ora_env* e, agent_t* a, const msg_t* m) {
    ta_receive(e, a, m);
    if (e->rl_rem > 0 && a->state == ST_AWAITING_SPREAD && m->kind == K_SPREAD) {
        /* cancelOrders(): self.orders is empty; placeOrders(currentTime) */
        int k = -1;
        for (int i = 0; i < e->nhz; i++)
            if (e->hz[i] == e->cur) { k = i; break; }
        if (k >= 0 && k == e->nhz - 2) {
            fail(e, -19, "ExecutionAgent.placeOrders: placeMarketOrder at horizon[-2] (not restated)");
            return;
        }
        if (k >= 0 && k < e->nhz - 2) {
            if (!a->nb || !a->na) {
                fail(e, -18, "ExecutionAgent.placeOrders: (bid + ask) / 2 with a None side (TypeError)");
                return;
            }
            fail(e, -17, "ExecutionAgent.placeOrders: schedule[Interval(t, t + 30 s)] (KeyError)");
        }
    }
}
/* ABIDESEnvMetrics.addLOB (ABIDESEnvMetrics.py:68-94): deque(maxlen=100), newest first */
static void metrics_add(ora_env* e, const msg_t* m) {
    if (e->ph_n == 0) {
        e->p0 = m->data;
        e->p0_none = !m->has_data;
    }
    e->m_head = (e->m_head + 99) % 100;
    int s = e->m_head;
    e->m_bid[s] = m->bpx;
    e->m_ask[s] = m->apx;
    e->m_nb[s] = m->nb;
    e->m_na[s] = m->na;
    e->m_data[s] = m->data;
    e->m_dnone[s] = !m->has_data;
    if (e->m_cnt < 100) e->m_cnt++;
    e->m_bq = m->bq;
    e->m_aq = m->aq;
    e->m_b2 = m->b2px;
    e->m_a2 = m->a2px;
    e->ph_n++;
    if (!m->has_data) e->ph_none = 1;
}
/* DummyRL.receiveMessage (dummy_rl_execution_agent.py:222-240); the execution handler is
 * ExecutionAgent's because of the reference's `hanldeOrderExecution` typo (dummy_rl:273) */
static void rl_receive(ora_env* e, agent_t* a, const msg_t* m) {
    ta_receive(e, a, m);
    if (m->kind == K_EXECUTED) {
        e->rl_exec_sum += m->qty;
        e->rl_rem = e->rl_quantity - e->rl_exec_sum;
    }
    if (e->rl_rem > 0 && a->state == ST_AWAITING_SPREAD && m->kind == K_SPREAD) {
        a->state = ST_AWAITING_WAKEUP;
        metrics_add(e, m);
    }
}
/* numpy pairwise summation (loops_utils.h pairwise_sum) for n <= 128 */
static double np_pairwise(const double* a, int n) {
    if (n < 8) {
        double r = 0.;
        for (int i = 0; i < n; i++) r += a[i];
        return r;
    }
    double r[8];
    for (int j = 0; j < 8; j++) r[j] = a[j];
    int i;
    for (i = 8; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; j++) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; i++) res += a[i];
    return res;
}
static double np_std(const double* x, int n) {
    double mean = np_pairwise(x, n) / n, sq[100];
    for (int i = 0; i < n; i++) {
        double d = x[i] - mean;
        sq[i] = d * d;
    }
    return sqrt(np_pairwise(sq, n) / n);
}
static int m_slot(const ora_env* e, int idx) { /* python index into the deque (negative ok) */
    if (idx < 0) idx += e->m_cnt;
    return (e->m_head + idx) % 100;
}
/* DummyRL.get_observation (dummy_rl_execution_agent.py:291-312) with ABIDESEnvMetrics */
static void rl_observe(ora_env* e) {
    int64_t fl = (e->cur / (30 * NS_SEC)) * (30 * NS_SEC); /* currentTime.floor("30S") */
    int rem = e->nhz;
    for (int i = 0; i < e->nhz; i++)
        if (e->hz[i] == fl) { rem = e->nhz - 1 - i; break; }
    double* o = e->obs;
    o[0] = rem;
    o[1] = (double)e->rl_rem;
    if (e->m_cnt == 0) { fail(e, -8, "get_observation: no LOB stored (IndexError)"); return; }
    int s0 = m_slot(e, 0);
    if (e->m_dnone[s0] || e->p0_none) { fail(e, -8, "get_observation: last trade is None (TypeError)"); return; }
    o[2] = log((double)e->m_data[s0] / (double)e->p0);
    for (int i = 0; i < e->m_cnt; i++) {
        int si = m_slot(e, i);
        if (!e->m_nb[si] || !e->m_na[si]) { fail(e, -8, "get_observation: empty book side (ValueError)"); return; }
    }
    int64_t bid = e->m_bid[s0], ask = e->m_ask[s0], bv = e->m_bq, av = e->m_aq;
    o[3] = (double)(ask - bid);
    o[4] = (double)(bv - av) / (double)(bv + av);
    o[5] = tanh((double)ask / (double)av - (double)bid / (double)bv);
    double lm[100];
    for (int i = 0; i < e->m_cnt; i++) {
        int si = m_slot(e, i);
        double mid = (double)(e->m_bid[si] + e->m_ask[si]) / 2;
        lm[i] = log(mid / (double)e->p0);
    }
    o[6] = np_std(lm, e->m_cnt);
    double mt = (double)(bid + ask) / 2;
    int64_t pt = e->m_data[s0];
    int d;
    if ((double)pt > mt) d = 1;
    else if ((double)pt < mt) d = -1;
    else { /* idx - 1 = -1: the oldest stored LOB */
        int sl = m_slot(e, -1);
        double ml = (double)(e->m_bid[sl] + e->m_ask[sl]) / 2;
        d = mt > ml ? 1 : -1;
    }
    o[7] = d;
    o[8] = (double)(2 * d) * ((double)pt - mt) / mt;
    e->has_obs = 1;
}
/* DummyRL.process_action + place_orders (dummy_rl_execution_agent.py:138-179) */
static void rl_place_orders(ora_env* e, const double* act) {
    agent_t* a = &e->ag[e->rl_id];
    double q0 = (double)e->rl_quantity, q = q0; /* metrics.rem_quantity is never updated */
    double x = act[0], sum = 0.0 + act[1] + act[2], oh0, oh1;
    if (sum == 0.0) oh0 = oh1 = 0.5;
    else { oh0 = act[1] / sum; oh1 = act[2] / sum; }
    double qh = q / q0;
    double total = rint(q0 * qh * pow(x, pow(qh, 0.5)));
    double o0 = rint(total * oh0);
    double o1 = total - (0.0 + o0);
    double ol[2] = {o0, o1};
    for (int l = 0; l < 2; l++) {
        if (e->m_cnt == 0) continue; /* getBookCount on empty metrics raises */
        int s0 = m_slot(e, 0);
        int nb = e->m_nb[s0], na = e->m_na[s0];
        if (nb == 0 || na == 0) continue;       /* ValueError */
        if (l >= nb || l >= na) continue;       /* IndexError */
        int64_t price = l == 0 ? e->m_bid[s0] : e->m_b2; /* BUY: bid of level l+1 */
        place_limit(e, a, (int64_t)ol[l], 1, price);
    }
}
/* GymKernel CANCEL_ORDER branch (GymKernel.py:244-249): get_reward, then cancelAllOrders */
static void rl_kernel_cancel(ora_env* e) {
    agent_t* a = &e->ag[e->rl_id];
    if (e->m_cnt == 0) { fail(e, -8, "get_reward: no LOB stored (IndexError)"); return; }
    if (e->ph_none) { fail(e, -8, "get_reward: None in price history (TypeError)"); return; }
    cancel_all(e, a);
}

/* ------------------------------- dispatch ---------------------------------- */
static void dispatch_wakeup(ora_env* e, int id) {
    agent_t* a = &e->ag[id];
    switch (a->type) {
    case AG_EXCHANGE: a->cur_time = e->cur; break; /* Agent.wakeup: no action */
    case AG_ZI: zi_wakeup(e, a); break;
    case AG_NOISE: noise_wakeup(e, a); break;
    case AG_VALUE: value_wakeup(e, a); break;
    case AG_POVMM: mm_wakeup(e, a); break;
    case AG_MOMENTUM: mom_wakeup(e, a); break;
    case AG_REPLAY: mr_wakeup(e, a); break;
    case AG_DUMMYRL: rl_wakeup(e, a); break;
    case AG_TWAP: tw_wakeup(e, a); break;
    case AG_MKTMAKER: mk_wakeup(e, a); break;
    case AG_HBL: hbl_wakeup(e, a); break;
    case AG_OBI: obi_wakeup(e, a); break;
    case AG_SBMM: sb_wakeup(e, a); break;
    }
}
static void dispatch_message(ora_env* e, int id, const msg_t* m) {
    agent_t* a = &e->ag[id];
    switch (a->type) {
    case AG_EXCHANGE: ex_receive(e, m); break;
    case AG_ZI: zi_receive(e, a, m); break;
    case AG_HBL: hbl_receive(e, a, m); break;
    case AG_MKTMAKER: mk_receive(e, a, m); break;
    case AG_OBI: obi_receive(e, a, m); break;
    case AG_SBMM: sb_receive(e, a, m); break;
    case AG_NOISE: noise_receive(e, a, m); break;
    case AG_VALUE: value_receive(e, a, m); break;
    case AG_POVMM: mm_receive(e, a, m); break;
    case AG_MOMENTUM: mom_receive(e, a, m); break;
    case AG_REPLAY: mr_receive(e, a, m); break;
    case AG_TWAP: tw_receive(e, a, m); break;
    case AG_DUMMYRL:
        rl_receive(e, a, m);
        if (m->kind == K_SPREAD) { /* GymKernel: the step ends at the RL agent's spread reply */
            rl_observe(e);
            e->end_step = 1;
        }
        break;
    }
}

/* one pop of Kernel.runner (Kernel.py:190-292) / GymKernel.stepRunner (GymKernel.py:158-306) */
static void pop_one(ora_env* e) {
        ev_t v = heap_pop(e);
        e->cur = v.t;
        e->have_cur = 1;
        int64_t rec[10];
        encode(e, &v, rec);
        for (int i = 0; i < 10; i++) e->hash = (e->hash ^ (uint64_t)rec[i]) * FNV_PRIME;
        if (e->trace && e->trace_len < e->trace_cap) memcpy(e->trace + 10 * e->trace_len++, rec, sizeof rec);
        e->pops++;
        e->add_delay = 0;
        int a = v.rcp;
        if (v.type == T_CANCEL_ORDER) { /* no busy check, no delay accounting */
            rl_kernel_cancel(e);
            return;
        }
        if (e->agent_time[a] > e->cur) { /* agent in the future: requeue unchanged */
            v.t = e->agent_time[a];
            heap_push(e, v);
            return;
        }
        e->agent_time[a] = e->cur;
        if (v.type == T_WAKEUP) {
            dispatch_wakeup(e, a);
        } else {
            msg_t m = e->msgs[v.mi];
            msg_free(e, v.mi);
            dispatch_message(e, a, &m);
        }
        e->agent_time[a] += e->comp_delay[a] + e->add_delay;
}

/* Kernel.runner event loop (Kernel.py:190-292) */
int64_t ora_run(ora_env* e, int64_t max_pops) {
    int64_t done = 0;
    while (!e->done) {
        if (max_pops >= 0 && done >= max_pops) break;
        if (e->nheap == 0 || !(e->cur <= e->stop)) {
            e->done = 1;
            break;
        }
        pop_one(e);
        done++;
    }
    return done;
}

/* ABIDESEnv.step (ABIDESEnv.py:30-49) = GymKernel.stepRunner: place the action's orders,
 * run until the RL agent's spread reply (or the end), return obs and done. */
int ora_gym_step(ora_env* e, const double* action, double* obs_out, int* has_obs, int* done_out) {
    if (!e->gym) return -1;
    rl_place_orders(e, action);
    e->end_step = 0;
    while (!e->end_step && !e->err && e->nheap > 0 && e->cur <= e->stop) pop_one(e);
    if (!e->err && (e->nheap == 0 || e->cur > e->stop) && !e->finished) {
        e->finished = 1; /* terminateRunner -> ExecutionAgent.kernelStopping */
        e->done = 1;
        if (e->rl_trade) fail(e, -8, "ExecutionAgent.kernelStopping: arrival_price is None (TypeError)");
    }
    *done_out = !(e->nheap > 0 && e->cur <= e->stop);
    memcpy(obs_out, e->obs, sizeof e->obs);
    *has_obs = e->has_obs;
    return e->err ? e->err : 0;
}

/* ------------------------------- reporting --------------------------------- */
static void rep_append(ora_env* e, const char* s) {
    size_t l = strlen(s);
    e->report = (char*)realloc(e->report, e->report_len + l + 2);
    memcpy(e->report + e->report_len, s, l);
    e->report_len += l;
    e->report[e->report_len++] = '\n';
    e->report[e->report_len] = 0;
}

/* Kernel.appendSummaryLog (Kernel.py:549-554) */
static void sum_add(ora_env* e, int agent, int type, int isf, int64_t vi, double vf) {
    int k = e->nsum++;
    e->sum_agent = (int*)realloc(e->sum_agent, sizeof(int) * e->nsum);
    e->sum_type = (int*)realloc(e->sum_type, sizeof(int) * e->nsum);
    e->sum_isf = (int*)realloc(e->sum_isf, sizeof(int) * e->nsum);
    e->sum_i = (int64_t*)realloc(e->sum_i, sizeof(int64_t) * e->nsum);
    e->sum_f = (double*)realloc(e->sum_f, sizeof(double) * e->nsum);
    e->sum_agent[k] = agent;
    e->sum_type[k] = type;
    e->sum_isf[k] = isf;
    e->sum_i[k] = vi;
    e->sum_f[k] = vf;
}
/* int(round(shares, -2) / 100): Python int rounding to hundreds, half to even */
static int64_t round_hundreds(int64_t x) {
    int64_t q = x / 100, r = x % 100;
    if (r < 0) { r += 100; q -= 1; } /* floor divmod */
    if (r > 50 || (r == 50 && (q & 1))) q += 1;
    return q;
}
/* the FINAL_VALUATION of ZeroIntelligenceAgent.kernelStopping (ZeroIntelligenceAgent.py:80-112),
 * NoiseAgent.kernelStopping (NoiseAgent.py:44-68) and ValueAgent.kernelStopping
 * (ValueAgent.py:66-86), in Kernel.runner's agent order (the oracle advances as it goes) */
static void final_valuation(ora_env* e, agent_t* a) {
    int64_t H = round_hundreds(a->shares);
    if (a->type == AG_NOISE) {
        int64_t si;
        double sf;
        int isf;
        if (!a->has_known) { fail(e, -9, "NoiseAgent.kernelStopping: no known quote (KeyError)"); return; }
        if (a->nb && a->na && a->bid && a->ask) { /* rT = int(bid + ask) / 2 (a float) */
            sf = (double)(a->bid + a->ask) / 2.0 * (double)H;
            isf = 1;
            si = 0;
        } else { /* rT = last_trade[symbol] */
            if (!a->has_last_trade) { fail(e, -9, "NoiseAgent.kernelStopping: no last trade (KeyError)"); return; }
            isf = a->last_trade_float;
            si = a->last_trade * H;
            sf = (double)a->last_trade * (double)H;
        }
        double v = isf ? (sf + (double)(a->cash - a->starting_cash)) / (double)a->starting_cash
                       : (double)(si + a->cash - a->starting_cash) / (double)a->starting_cash;
        sum_add(e, a->id, 3, 1, 0, v);
    } else if (a->type == AG_VALUE) {
        int64_t rT = o_observe(e, a->cur_time, 0, NULL);
        sum_add(e, a->id, 3, 1, 0, (double)(rT * H + a->cash - a->starting_cash) / (double)a->starting_cash);
    } else if (a->type == AG_ZI || a->type == AG_HBL) { /* HBL inherits ZI.kernelStopping */
        int64_t rT = o_observe(e, a->cur_time, 0, NULL);
        int64_t s = 0;
        int nq = 2 * a->q_max;
        if (H > 0) {
            for (int64_t x = 1; x <= H; x++) {
                int64_t i = x + a->q_max - 1;
                if (i >= nq) { fail(e, -10, "ZeroIntelligenceAgent.kernelStopping: theta index (IndexError)"); return; }
                s += a->theta[i];
            }
        } else if (H < 0) {
            for (int64_t x = H + 1; x <= 0; x++) {
                int64_t i = x + a->q_max - 1;
                if (i < -nq) { fail(e, -10, "ZeroIntelligenceAgent.kernelStopping: theta index (IndexError)"); return; }
                s -= a->theta[i < 0 ? i + nq : i]; /* Python negative indices wrap */
            }
        }
        s += rT * H;
        s += a->cash - a->starting_cash;
        sum_add(e, a->id, 3, 0, s, 0);
    }
}

/* TradingAgent.kernelStopping (TradingAgent.py:112-138) + Kernel mean print (Kernel.py:337-341) */
int ora_finish(ora_env* e) {
    char line[512];
    const char* sym = e->sym[0] ? e->sym
                      : strncmp(e->config, "rmsc03", 6) == 0 || strncmp(e->config, "random_fund_", 12) == 0 ? "ABM" : "JPM";
    /* one entry per distinct agent type string (value_noise names every ValueAgent's type apart) */
    char (*tnames)[96] = (char (*)[96])malloc(sizeof(char[96]) * (size_t)e->n);
    long long* gains = (long long*)malloc(sizeof(long long) * (size_t)e->n);
    int* counts = (int*)malloc(sizeof(int) * (size_t)e->n);
    int nt = 0;
    /* TradingAgent.kernelStarting logged STARTING_CASH for every trading agent (TradingAgent.py:101) */
    e->nsum = 0;
    for (int i = 1; i < e->n; i++) sum_add(e, i, 0, 0, e->ag[i].starting_cash, 0);
    for (int i = 1; i < e->n; i++) {
        agent_t* a = &e->ag[i];
        char hold[128];
        if (a->shares != 0) snprintf(hold, sizeof hold, "{ %s: %lld, CASH: %lld }", sym, (long long)a->shares, (long long)a->cash);
        else snprintf(hold, sizeof hold, "{ CASH: %lld }", (long long)a->cash);
        long long mtm = a->cash;
        int mtm_float = 0;
        if (a->shares != 0) {
            mtm += (long long)a->last_trade * a->shares;
            mtm_float = a->last_trade_float;
        }
        sum_add(e, i, 1, 0, a->cash, 0);
        sum_add(e, i, 2, mtm_float, mtm, (double)mtm);
        final_valuation(e, a);
        if (mtm_float) snprintf(line, sizeof line, "Final holdings for %s: %s.  Marked to market: %lld.0", a->name, hold, mtm);
        else snprintf(line, sizeof line, "Final holdings for %s: %s.  Marked to market: %lld", a->name, hold, mtm);
        rep_append(e, line);
        int k;
        for (k = 0; k < nt; k++)
            if (strcmp(tnames[k], a->tname) == 0) break;
        if (k == nt) {
            snprintf(tnames[nt], 96, "%s", a->tname);
            gains[nt] = 0;
            counts[nt] = 0;
            nt++;
        }
        gains[k] += mtm - a->starting_cash;
        counts[k]++;
    }
    for (int k = 0; k < nt; k++) {
        snprintf(line, sizeof line, "%s: %lld", tnames[k], (long long)rint((double)gains[k] / (double)counts[k]));
        rep_append(e, line);
    }
    free(tnames);
    free(gains);
    free(counts);
    return 0;
}

/* ------------------------------- configs ----------------------------------- */
static agent_t* add_agent(ora_env* e, int type) {
    e->ag = (agent_t*)realloc(e->ag, sizeof(agent_t) * (e->n + 1));
    agent_t* a = &e->ag[e->n];
    memset(a, 0, sizeof *a);
    a->id = e->n++;
    a->type = type;
    a->first_wake = 1;
    a->state = ST_AWAITING_WAKEUP;
    return a;
}
static uint32_t seed_u32(ora_rs* G) { return (uint32_t)rs_randint(G, 0, 4294967296LL); }

static void oracle_init(ora_env* e, int64_t open, int64_t close, double r_bar, double kappa, double fund_vol,
                        double lam, double ms_mean, double ms_var) {
    e->o_open = open;
    e->o_close = close;
    e->o_rbar = r_bar;
    e->o_kappa = kappa;
    e->o_fundvol = fund_vol;
    e->o_lambda = lam;
    e->o_msmean = ms_mean;
    e->o_msvar = ms_var;
    e->o_pt = open;
    e->o_pv = r_bar;
    e->o_mst = open + (int64_t)rs_exponential(&e->G, 1.0 / lam);
    double msv = rs_normal(&e->O, ms_mean, sqrt(ms_var));
    e->o_msv = rs_randint(&e->O, 0, 2) == 0 ? msv : -msv;
}

static void trading_init(agent_t* a, int64_t cash) {
    a->starting_cash = cash;
    a->cash = cash;
}

static int cmp_desc(const void* x, const void* y) {
    double a = *(const double*)x, b = *(const double*)y;
    return a < b ? 1 : (a > b ? -1 : 0);
}

/* get_wake_time (util/util.py:35-58) with the global RNG */
static int64_t get_wake_time(ora_env* e, int64_t open, int64_t close) {
    double u = rs_double(&e->G);
    double alpha = 12.0, beta = 0.5;
    double n = (3 / alpha) * u - pow(beta - 0, 3.0);
    double c = n < 0 ? -pow(-n, 1.0 / 3.0) : pow(n, 1.0 / 3.0);
    double mult = c + beta;
    return open + (int64_t)(mult * (double)(close - open));
}

/* the base scripts' compositions (include/mxa.h mxa_config_defaults: mxa_config.h config_defaults
 * restates the same values for the device; tests/test_composition.py checks they agree) */
int ora_config_defaults(const char* base, ora_config* c) {
    memset(c, 0, sizeof *c);
    const int64_t open = 9 * NS_HOUR + 30 * NS_MIN;
    c->date_ns = 1561680000LL * NS_SEC; /* 2019-06-28 */
    c->r_bar = 1e5;
    c->kappa = 1.67e-12;
    c->fund_vol = 1e-4;
    c->megashock_lambda_a = 2.77778e-13;
    c->megashock_mean = 1e3;
    c->megashock_var = 5e4;
    c->starting_cash = 10000000;
    c->mkt_open_ns = open;
    c->zi_q_max = 10;
    /* the fields the base leaves at params_base / MxaParams defaults (device config_defaults) */
    c->mm.mm_pov = 0;
    if (!strcmp(base, "rmsc03")) { /* config/rmsc03.py:55-235 */
        c->base = 0;
        c->log_orders = 1;
        c->n_noise = 50;
        c->n_value = 10;
        c->n_mm = 1;
        c->n_momentum = 2;
        c->mkt_close_ns = 9 * NS_HOUR + 45 * NS_MIN;
        c->kernel_start_ns = open;
        c->kernel_stop_ns = c->mkt_close_ns + NS_MIN;
        c->noise_wake_open_ns = 9 * NS_HOUR;
        c->noise_wake_close_ns = 16 * NS_HOUR;
        c->value_sigma_n = 1e5 / 10;
        c->value_r_bar = 1e5;
        c->value_kappa = 1.67e-15;
        c->value_sigma_s = 100000;
        c->value_lambda_a = 7e-11;
        c->value_starting_cash = 10000000;
        c->mm.mm_pov = 0.05;
        c->mm.mm_min_order_size = 20;
        c->mm.mm_window_size = 5;
        c->mm.mm_num_ticks = 20;
        c->mm.mm_wake_up_freq_ns = NS_SEC;
        c->mom_min_size = 1;
        c->mom_max_size = 10;
        c->mom_wake_up_freq_ns = 20 * NS_SEC;
        return 0;
    }
    if (!strcmp(base, "value_noise")) { /* config/value_noise.py:45-200 */
        c->base = 5;
        c->log_orders = 0;
        c->n_noise = 100;
        c->n_value = 50;
        c->mkt_close_ns = 10 * NS_HOUR + 30 * NS_MIN;
        c->kernel_start_ns = 0;
        c->kernel_stop_ns = 17 * NS_HOUR;
        c->default_computation_delay_ns = 1000000000;
        c->value_sigma_n = 1000000.0;
        c->value_r_bar = 1e5;
        c->value_kappa = 1.67e-15;
        c->value_sigma_s = 1e-4;
        c->value_lambda_a = 1e-12;
        c->value_starting_cash = 100000;
        c->lat_low = 21000;
        c->lat_high = 13000000;
        return 0;
    }
    if (!strcmp(base, "sparse_zi_100") || !strcmp(base, "sparse_zi_1000")) { /* config/sparse_zi_100.py:73-334 */
        const int big = !strcmp(base, "sparse_zi_1000");
        static const int n100[7] = {15, 15, 14, 14, 14, 14, 14};
        static const int n1000[7] = {143, 143, 143, 143, 143, 143, 142};
        static const int rmin[7] = {0, 0, 0, 0, 0, 250, 250};
        static const int rmax[7] = {250, 500, 1000, 1000, 2000, 500, 500};
        static const double eta[7] = {1, 1, 0.8, 1, 0.8, 0.8, 1};
        c->base = big ? 2 : 1;
        c->log_orders = big ? 0 : 1;
        c->n_zi_groups = 7;
        for (int g = 0; g < 7; g++) {
            c->zi_count[g] = big ? n1000[g] : n100[g];
            c->zi_r_min[g] = rmin[g];
            c->zi_r_max[g] = rmax[g];
            c->zi_eta[g] = eta[g];
        }
        c->zi_sigma_n = 1000000.0;
        c->zi_r_bar = 1e5;
        c->zi_kappa = 1.67e-15;
        c->zi_sigma_s = 1e-4;
        c->zi_sigma_pv = 5e6;
        c->zi_lambda_a = 1e-12;
        c->mkt_close_ns = 16 * NS_HOUR;
        c->kernel_start_ns = 0;
        c->kernel_stop_ns = 17 * NS_HOUR;
        c->default_computation_delay_ns = 1000000000;
        c->lat_low = 21000;
        c->lat_high = big ? 13000000 : 100000;
        return 0;
    }
    return -1;
}

/* %g of a strategy table's eta as the script's "{}" prints it (1 for the int 1, 0.8) */
static void eta_str(char* b, size_t n, double eta) { snprintf(b, n, "%g", eta); }

static int build_sparse_zi(ora_env* e, uint32_t seed, const ora_config* c) {
    /* config/sparse_zi_100.py:73-334 (sparse_zi_1000.py: big, the symmetric latency matrix) */
    const int big = c->base == 2;
    rs_seed(&e->G, seed);
    rs_seed(&e->O, seed_u32(&e->G));
    rs_seed(&e->K, seed_u32(&e->G));
    if (!big) rs_seed(&e->L, seed_u32(&e->G));
    e->start = c->kernel_start_ns;
    e->stop = c->kernel_stop_ns;
    int64_t open = c->mkt_open_ns, close = c->mkt_close_ns;
    oracle_init(e, open, close, c->r_bar, c->kappa, c->fund_vol, c->megashock_lambda_a, c->megashock_mean,
                c->megashock_var);
    agent_t* ex = add_agent(e, AG_EXCHANGE);
    rs_seed(&ex->rs, seed_u32(&e->G));
    snprintf(ex->name, 96, "Exchange Agent 0");
    snprintf(ex->tname, 96, "ExchangeAgent");
    e->ex_open = open;
    e->ex_close = close;
    e->ex_pipeline = 0;
    e->ex_comp = 0;
    e->stream_history = 10;
    const int nq = 2 * c->zi_q_max;
    for (int g = 0; g < c->n_zi_groups; g++) {
        char etas[32];
        eta_str(etas, sizeof etas, c->zi_eta[g]);
        for (int k = 0; k < c->zi_count[g]; k++) {
            agent_t* a = add_agent(e, AG_ZI);
            rs_seed(&a->rs, seed_u32(&e->G));
            snprintf(a->name, 96, "ZI Agent %d Type %d [%d <= R <= %d, eta=%s]", a->id, g + 1, c->zi_r_min[g],
                     c->zi_r_max[g], etas);
            snprintf(a->tname, 96, "ZeroIntelligenceAgent Type %d [%d <= R <= %d, eta=%s]", g + 1, c->zi_r_min[g],
                     c->zi_r_max[g], etas);
            trading_init(a, c->starting_cash);
            a->sigma_n = c->zi_sigma_n;
            a->r_bar = c->zi_r_bar;
            a->kappa = c->zi_kappa;
            a->sigma_s = c->zi_sigma_s;
            a->q_max = c->zi_q_max;
            a->R_min = c->zi_r_min[g];
            a->R_max = c->zi_r_max[g];
            a->eta = c->zi_eta[g];
            a->lambda_a = c->zi_lambda_a;
            a->r_t = c->zi_r_bar;
            a->sigma_t = 0;
            double th[20];
            for (int i = 0; i < nq; i++) th[i] = rint(rs_normal(&a->rs, 0, sqrt(c->zi_sigma_pv)));
            qsort(th, nq, sizeof(double), cmp_desc);
            for (int i = 0; i < nq; i++) a->theta[i] = (int64_t)th[i];
        }
    }
    int n = e->n;
    e->lat = (double*)malloc(sizeof(double) * (size_t)n * n);
    for (size_t i = 0; i < (size_t)n * n; i++) e->lat[i] = rs_uniform(&e->G, c->lat_low, c->lat_high);
    if (!big) {
        e->lat_mode = 2;
        e->jitter = 0.3;
        e->clip = 0.05;
        e->unit = 5;
        e->noise_len = 0;
    } else {
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) {
                if (i > j) e->lat[(size_t)i * n + j] = e->lat[(size_t)j * n + i];
                else if (i == j) e->lat[(size_t)i * n + j] = 20000;
            }
        e->lat_mode = 1;
        e->noise_len = 6;
    }
    e->agent_time = (int64_t*)calloc(n, sizeof(int64_t));
    e->comp_delay = (int64_t*)calloc(n, sizeof(int64_t));
    for (int i = 0; i < n; i++) {
        e->agent_time[i] = e->start;
        e->comp_delay[i] = c->default_computation_delay_ns;
    }
    return 0;
}

/* config/rmsc03.py:55-235 (rfv = 0) and config/random_fund_value.py:59-180 (rfv = 1): the same
 * global-draw order (oracle symbol seed, first megashock, exchange seed, per noise agent its
 * wakeup_time then seed then size, per value agent seed then size, [market maker, momentum],
 * kernel seed); random_fund_value has 5000 noise agents waking in 09:30-16:00, 100 value agents
 * (lambda_a 1e-12), no market maker or momentum agents, market 09:30-16:00, kernel 09:30-16:01 */
/* rfv: 0 rmsc03, 1 random_fund_value, 2 random_fund_diverse, 3 / 4 hist_fund_value / _diverse
 * (config/hist_fund_*.py: the same agents on an ExternalFileOracle, which draws nothing at
 * construction; the value agents' r_bar is the series' first value, sigma_n = r_bar / 10) */
static int build_rmsc03_like(ora_env* e, uint32_t seed, int rfv, const ora_config* c) {
    const int hist = rfv >= 3;
    if (hist) {
        if (!g_fs_n) return -2; /* ora_set_fundamental first */
        rfv -= 2;
    }
    rs_seed(&e->G, seed);
    int64_t open = c->mkt_open_ns, close = c->mkt_close_ns;
    rs_seed(&e->O, seed_u32(&e->G));
    if (hist) {
        e->efo = 1;
        e->o_open = open;
        e->o_close = close;
    } else {
        oracle_init(e, open, close, c->r_bar, c->kappa, c->fund_vol, c->megashock_lambda_a, c->megashock_mean,
                    c->megashock_var);
    }
    const double vr_bar = hist ? g_fs_v[0] : c->value_r_bar;
    agent_t* ex = add_agent(e, AG_EXCHANGE);
    rs_seed(&ex->rs, seed_u32(&e->G));
    snprintf(ex->name, 96, "EXCHANGE_AGENT");
    snprintf(ex->tname, 96, "ExchangeAgent");
    e->ex_open = open;
    e->ex_close = close;
    e->ex_pipeline = 0;
    e->ex_comp = 0;
    e->stream_history = 10;
    int64_t nopen = c->noise_wake_open_ns, nclose = c->noise_wake_close_ns;
    for (int j = 0; j < c->n_noise; j++) {
        int64_t wt = get_wake_time(e, nopen, nclose);
        agent_t* a = add_agent(e, AG_NOISE);
        a->wakeup_time = wt;
        rs_seed(&a->rs, seed_u32(&e->G));
        a->size = rs_randint(&e->G, 20, 50);
        snprintf(a->name, 96, "NoiseAgent %d", a->id);
        snprintf(a->tname, 96, "NoiseAgent");
        trading_init(a, c->starting_cash);
    }
    for (int j = 0; j < c->n_value; j++) {
        agent_t* a = add_agent(e, AG_VALUE);
        rs_seed(&a->rs, seed_u32(&e->G));
        a->size = rs_randint(&e->G, 20, 50);
        snprintf(a->name, 96, "Value Agent %d", a->id);
        snprintf(a->tname, 96, "ValueAgent");
        trading_init(a, c->value_starting_cash);
        a->sigma_n = hist ? vr_bar / 10 : c->value_sigma_n; /* hist_fund_*: r_bar / 10 of the series' r_bar */
        a->r_bar = vr_bar;
        a->kappa = c->value_kappa;
        a->sigma_s = c->value_sigma_s;
        a->lambda_a = c->value_lambda_a;
        a->r_t = vr_bar;
        a->sigma_t = 0;
    }
    for (int j = 0; j < c->n_mm; j++) {
        agent_t* a = add_agent(e, AG_POVMM);
        rs_seed(&a->rs, seed_u32(&e->G));
        snprintf(a->name, 96, "POV_MARKET_MAKER_AGENT_%d", a->id);
        snprintf(a->tname, 96, "POVMarketMakerAgent");
        trading_init(a, c->starting_cash);
        a->pov = c->mm.mm_pov;
        a->min_size = c->mm.mm_min_order_size;
        a->window = c->mm.mm_window_size;
        a->num_ticks = c->mm.mm_num_ticks;
        a->wake_freq = c->mm.mm_wake_up_freq_ns;
        a->order_size = c->mm.mm_min_order_size; /* order_size = min_order_size */
        a->aw_spread = a->aw_tv = 1;
    }
    for (int j = 0; j < c->n_momentum; j++) {
        agent_t* a = add_agent(e, AG_MOMENTUM);
        rs_seed(&a->rs, seed_u32(&e->G));
        a->size = rs_randint(&a->rs, c->mom_min_size, c->mom_max_size);
        snprintf(a->name, 96, "MOMENTUM_AGENT_%d", a->id);
        snprintf(a->tname, 96, "MomentumAgent");
        trading_init(a, c->starting_cash);
        a->wake_freq = c->mom_wake_up_freq_ns;
    }
    if (rfv == 2) { /* config/random_fund_diverse.py:157-198: a MarketMakerAgent (100-101 shares, 1 min,
                       polling) and 25 momentum agents (1-10 shares, the default 60 s) */
        agent_t* a = add_agent(e, AG_MKTMAKER);
        rs_seed(&a->rs, seed_u32(&e->G));
        snprintf(a->name, 96, "MARKET_MAKER_AGENT_%d", a->id);
        snprintf(a->tname, 96, "MarketMakerAgent");
        trading_init(a, 10000000);
        a->mk_min = 100;
        a->mk_max = 101;
        a->size = (int64_t)rint((double)rs_randint(&a->rs, a->mk_min, a->mk_max) / 2);
        a->wake_freq = 60 * NS_SEC;
        a->spread_depth = 5;
        a->last_spread = 10;
        a->subscribe = 0;
        for (int j = 0; j < 25; j++) {
            agent_t* m = add_agent(e, AG_MOMENTUM);
            rs_seed(&m->rs, seed_u32(&e->G));
            m->size = rs_randint(&m->rs, 1, 10);
            snprintf(m->name, 96, "MOMENTUM_AGENT_%d", m->id);
            snprintf(m->tname, 96, "MomentumAgent");
            trading_init(m, 10000000);
            m->wake_freq = 60 * NS_SEC;
            m->subscribe = 0;
        }
    }
    rs_seed(&e->K, seed_u32(&e->G));
    e->start = c->kernel_start_ns;
    e->stop = c->kernel_stop_ns;
    e->lat_mode = 0;
    e->noise_len = 1;
    int n = e->n;
    e->agent_time = (int64_t*)calloc(n, sizeof(int64_t));
    e->comp_delay = (int64_t*)calloc(n, sizeof(int64_t));
    for (int i = 0; i < n; i++) {
        e->agent_time[i] = e->start;
        e->comp_delay[i] = c->default_computation_delay_ns;
    }
    return 0;
}

/* config/rmsc01.py:49-263: 1 exchange, 1 MarketMakerAgent, 50 ZI, 25 HBL, 24 Momentum on JPM
 * 2019-06-28, market 09:30-16:00, kernel 09:30-16:01, compute delay 0, latency zeros, noise [0.0].
 * Global draw order: exchange seed, market maker seed (its __init__ draws its size from its
 * own stream), the oracle symbol's seed, the oracle's megashock init, per ZI / HBL agent its
 * seed (theta from its own stream), per momentum agent its seed (size from its own stream),
 * the kernel's seed.  book_freq="M" only archives snapshots at the end (logging). */
static void zi_params(agent_t* a, int64_t rmin, int64_t rmax, double sigma_n, double sigma_s, double sigma_pv) {
    trading_init(a, 10000000);
    a->sigma_n = sigma_n;
    a->r_bar = 1e5;
    a->kappa = 1.67e-15;
    a->sigma_s = sigma_s;
    a->q_max = 10;
    a->R_min = rmin;
    a->R_max = rmax;
    a->eta = 1;
    a->lambda_a = 1e-12;
    a->r_t = 1e5;
    a->sigma_t = 0;
    double th[20];
    for (int i = 0; i < 20; i++) th[i] = rint(rs_normal(&a->rs, 0, sqrt(sigma_pv)));
    qsort(th, 20, sizeof(double), cmp_desc);
    for (int i = 0; i < 20; i++) a->theta[i] = (int64_t)th[i];
}
/* config/rmsc02.py: rmsc01's agents with subscribe=True for the market maker (5 levels) and the
 * momentum agents (1 level), both every 10 s; kernel midnight-17:00; latency
 * U(21000, 13e6)[n][n] drawn after the kernel seed (not symmetrised) with 6-way noise */
/* config/obi_rmsc02.py: rmsc02's market with 89 ZI agents, 5 OrderBookImbalanceAgent (built
 * after the ZI agents, each drawing only its seed) and 5 momentum agents; no HBL */
/* rmsc03 with its market-maker slot (config/rmsc03.py:158-177) a SpreadBasedMarketMakerAgent built
 * from the same arguments (tests/golden/gen_fixtures.py rmsc03_sbmm*): window 5, 20 ticks, wake-up
 * 1 s, order_size = --mm-min-order-size (20); the random_state draw is the POV maker's */
static int build_rmsc03_sbmm(ora_env* e, uint32_t seed, int subscribe) {
    ora_config c;
    ora_config_defaults("rmsc03", &c);
    int rc = build_rmsc03_like(e, seed, 0, &c);
    if (rc) return rc;
    agent_t* a = &e->ag[61];
    a->type = AG_SBMM;
    snprintf(a->name, 96, "SPREAD_BASED_MARKET_MAKER_AGENT_%d", a->id);
    snprintf(a->tname, 96, "SpreadBasedMarketMakerAgent");
    a->order_size = 20;
    a->window = 5;
    a->num_ticks = 20;
    a->wake_freq = NS_SEC;
    a->subscribe = subscribe;
    a->sub_requested = 0;
    a->state = ST_AWAITING_WAKEUP;
    a->has_last_mid = 0;
    a->sb_n = 0;
    a->sb_init = 0;
    a->sb_cnt = 0;
    return 0;
}
static int build_rmsc0x(ora_env* e, uint32_t seed, int v2, int obi) {
    rs_seed(&e->G, seed);
    int64_t open = 9 * NS_HOUR + 30 * NS_MIN, close = 16 * NS_HOUR;
    agent_t* ex = add_agent(e, AG_EXCHANGE);
    rs_seed(&ex->rs, seed_u32(&e->G));
    snprintf(ex->name, 96, "EXCHANGE_AGENT");
    snprintf(ex->tname, 96, "ExchangeAgent");
    e->ex_open = open;
    e->ex_close = close;
    e->ex_pipeline = 0;
    e->ex_comp = 0;
    e->stream_history = 10;
    {
        agent_t* a = add_agent(e, AG_MKTMAKER);
        rs_seed(&a->rs, seed_u32(&e->G));
        snprintf(a->name, 96, "MARKET_MAKER_AGENT_%d", a->id);
        snprintf(a->tname, 96, "MarketMakerAgent");
        trading_init(a, 10000000);
        a->mk_min = 500;
        a->mk_max = 1000;
        a->size = (int64_t)rint((double)rs_randint(&a->rs, a->mk_min, a->mk_max) / 2);
        a->wake_freq = NS_SEC;
        a->spread_depth = 5;
        a->last_spread = 10;
        a->subscribe = v2;
    }
    rs_seed(&e->O, seed_u32(&e->G));
    oracle_init(e, open, close, 1e5, 1.67e-12, 1e-4, 2.77778e-13, 1e3, 5e4);
    for (int j = 0; j < (obi ? 89 : 50); j++) {
        agent_t* a = add_agent(e, AG_ZI);
        rs_seed(&a->rs, seed_u32(&e->G));
        snprintf(a->name, 96, "ZI_AGENT_%d", a->id);
        snprintf(a->tname, 96, "ZeroIntelligenceAgent");
        zi_params(a, 0, 100, 10000, 1e-4, 5e4);
    }
    for (int j = 0; j < (obi ? 5 : 0); j++) {
        agent_t* a = add_agent(e, AG_OBI);
        rs_seed(&a->rs, seed_u32(&e->G));
        snprintf(a->name, 96, "OBI_AGENT_%d", a->id);
        snprintf(a->tname, 96, "OrderBookImbalanceAgent");
        trading_init(a, 10000000);
    }
    for (int j = 0; j < (obi ? 0 : 25); j++) {
        agent_t* a = add_agent(e, AG_HBL);
        rs_seed(&a->rs, seed_u32(&e->G));
        snprintf(a->name, 96, "HBL_AGENT_%d", a->id);
        snprintf(a->tname, 96, "HeuristicBeliefLearningAgent");
        zi_params(a, 0, 100, 10000, 1e-4, 5e4);
        a->L = 2;
    }
    for (int j = 0; j < (obi ? 5 : 24); j++) {
        agent_t* a = add_agent(e, AG_MOMENTUM);
        rs_seed(&a->rs, seed_u32(&e->G));
        a->size = rs_randint(&a->rs, 1, 10);
        snprintf(a->name, 96, "MOMENTUM_AGENT_%d", a->id);
        snprintf(a->tname, 96, "MomentumAgent");
        trading_init(a, 10000000);
        a->wake_freq = 60 * NS_SEC;
        a->subscribe = v2;
    }
    rs_seed(&e->K, seed_u32(&e->G));
    int n = e->n;
    if (v2) {
        e->start = 0;
        e->stop = 17 * NS_HOUR;
        e->lat = (double*)malloc(sizeof(double) * (size_t)n * n);
        for (size_t i = 0; i < (size_t)n * n; i++) e->lat[i] = rs_uniform(&e->G, 21000, 13000000);
        e->lat_mode = 1;
        e->noise_len = 6;
    } else {
        e->start = open;
        e->stop = 16 * NS_HOUR + NS_MIN;
        e->lat_mode = 0;
        e->noise_len = 1;
    }
    e->agent_time = (int64_t*)calloc(n, sizeof(int64_t));
    e->comp_delay = (int64_t*)calloc(n, sizeof(int64_t));
    for (int i = 0; i < n; i++) e->agent_time[i] = e->start;
    return 0;
}

/* config/value_noise.py:45-200 (argparse defaults: obs_noise 1e6): 1 exchange, 100 noise and
 * 50 value agents on JPM 2019-06-28, market 09:30-10:30, kernel midnight-17:00, compute delay
 * 1 s, latency matrix U(21000, 13e6) symmetrised (diagonal 20000), 6-way uniform noise.
 * Global draw order: O seed, K seed (kernel built before the oracle), oracle megashock
 * exponential, exchange seed; per noise agent its seed, then wakeup_time = open + rand() *
 * (close - open) (pandas float * Timedelta truncates to ns), then NoiseAgent.__init__'s
 * size; per value agent its seed, then its size; then the 151 x 151 latency draws. */
static int build_value_noise(ora_env* e, uint32_t seed, const ora_config* c) {
    rs_seed(&e->G, seed);
    int64_t open = c->mkt_open_ns, close = c->mkt_close_ns;
    rs_seed(&e->O, seed_u32(&e->G));
    rs_seed(&e->K, seed_u32(&e->G));
    oracle_init(e, open, close, c->r_bar, c->kappa, c->fund_vol, c->megashock_lambda_a, c->megashock_mean,
                c->megashock_var);
    agent_t* ex = add_agent(e, AG_EXCHANGE);
    rs_seed(&ex->rs, seed_u32(&e->G));
    snprintf(ex->name, 96, "Exchange Agent 0");
    snprintf(ex->tname, 96, "ExchangeAgent");
    e->ex_open = open;
    e->ex_close = close;
    e->ex_pipeline = 0;
    e->ex_comp = 0;
    e->stream_history = 10;
    for (int j = 0; j < c->n_noise; j++) {
        agent_t* a = add_agent(e, AG_NOISE);
        rs_seed(&a->rs, seed_u32(&e->G));
        a->wakeup_time = open + (int64_t)(rs_double(&e->G) * (double)(close - open));
        a->size = rs_randint(&e->G, 20, 50);
        snprintf(a->name, 96, "NoiseAgent %d", a->id);
        snprintf(a->tname, 96, "NoiseAgent");
        trading_init(a, c->starting_cash);
    }
    for (int j = 0; j < c->n_value; j++) {
        agent_t* a = add_agent(e, AG_VALUE);
        rs_seed(&a->rs, seed_u32(&e->G));
        a->size = rs_randint(&e->G, 20, 50);
        snprintf(a->name, 96, "Value Agent %d", a->id);
        snprintf(a->tname, 96, "ValueAgent %d", a->id);
        trading_init(a, c->value_starting_cash); /* ValueAgent's default starting_cash in the script */
        a->sigma_n = c->value_sigma_n;
        a->r_bar = c->value_r_bar;
        a->kappa = c->value_kappa;
        a->sigma_s = c->value_sigma_s;
        a->lambda_a = c->value_lambda_a;
        a->r_t = c->value_r_bar;
        a->sigma_t = 0;
    }
    int n = e->n;
    e->lat = (double*)malloc(sizeof(double) * (size_t)n * n);
    for (size_t i = 0; i < (size_t)n * n; i++) e->lat[i] = rs_uniform(&e->G, c->lat_low, c->lat_high);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            if (i > j) e->lat[(size_t)i * n + j] = e->lat[(size_t)j * n + i];
            else if (i == j) e->lat[(size_t)i * n + j] = 20000;
        }
    e->lat_mode = 1;
    e->noise_len = 6;
    e->start = c->kernel_start_ns;
    e->stop = c->kernel_stop_ns;
    e->agent_time = (int64_t*)calloc(n, sizeof(int64_t));
    e->comp_delay = (int64_t*)calloc(n, sizeof(int64_t));
    for (int i = 0; i < n; i++) {
        e->agent_time[i] = e->start;
        e->comp_delay[i] = c->default_computation_delay_ns;
    }
    return 0;
}

/* rmsc03 + DummyRL (BASELINE.json configs[3]; tests/golden/gen_rl_fixtures.py): config/rmsc03.py's
 * 64 agents, oracle and kernel RandomState, plus DummyRLExecutionAgent 64 (agent_config.py:115-137
 * parameters: BUY 1e5, freq 30 s, order_level 2) with execution_time_horizon =
 * pd.date_range(09:31, 09:44, "30S"), run by a GymKernel with rmsc03's start/stop, latency
 * zeros(65, 65), noise [0.0] and compute delay 0.  The DummyRL draws nothing. */
static int build_rmsc03_rl(ora_env* e, uint32_t seed) {
    ora_config c;
    ora_config_defaults("rmsc03", &c);
    int rc = build_rmsc03_like(e, seed, 0, &c);
    if (rc) return rc;
    agent_t* r = add_agent(e, AG_DUMMYRL);
    trading_init(r, 0);
    snprintf(r->name, sizeof r->name, "%d_DUMMY_RL_EXECUTION_AGENT", r->id);
    snprintf(r->tname, sizeof r->tname, "DummyRLExecutionAgent");
    e->rl_id = r->id;
    e->nhz = 27;
    e->hz = (int64_t*)malloc(sizeof(int64_t) * e->nhz);
    for (int i = 0; i < e->nhz; i++) e->hz[i] = 9 * NS_HOUR + 31 * NS_MIN + (int64_t)i * 30 * NS_SEC;
    r->wake_freq = e->hz[0] - e->ex_open;
    e->rl_quantity = 100000;
    e->rl_rem = 100000;
    e->rl_trade = 1;
    e->gym = 1;
    int n = e->n;
    e->agent_time = (int64_t*)realloc(e->agent_time, sizeof(int64_t) * n);
    e->comp_delay = (int64_t*)realloc(e->comp_delay, sizeof(int64_t) * n);
    e->agent_time[n - 1] = e->start;
    e->comp_delay[n - 1] = 0;
    return 0;
}

/* ABIDESEnv.initAgents / initKernel (ABIDESEnv.py:59-103; agent_config.py:30-160):
 * Exchange (id 0), MarketReplayAgent (1) on a LOBSTER tape, DummyRLExecutionAgent (2);
 * GymKernel start = midnight, stop = 16:10, compute delays 0, latencies 0, noise [1.0].
 * Nothing in this composition draws from an RNG. */
/* runner 0: ABIDESEnv's composition (agent_config.py: Exchange, MarketReplayAgent, DummyRL under
 * a GymKernel); runner 1: config/marketreplay.py (Exchange and MarketReplayAgent under
 * Kernel.runner, midnight to 16:01, agents named as that script names them); runner 2 / 3:
 * config/execution/marketreplay/execution_marketreplay.py, the same plus TWAP_EXECUTION_AGENT 2
 * (BUY 12e3 over pd.date_range(10:00, 12:00, "60S"); 3: -e, the agent trades) */
static int create_mr(const int64_t* t, const int64_t* oid, const int64_t* price, const int64_t* size,
                     const int8_t* buy, int n, int runner, ora_env** out) {
    if (n <= 0) return -1;
    ora_env* e = (ora_env*)calloc(1, sizeof(ora_env));
    snprintf(e->config, sizeof e->config, runner >= 2 ? "marketreplay_twap" : runner ? "marketreplay_runner" : "marketreplay");
    int64_t open = 9 * NS_HOUR + 30 * NS_MIN, close = 16 * NS_HOUR;
    agent_t* x = add_agent(e, AG_EXCHANGE);
    snprintf(x->name, sizeof x->name, runner ? "EXCHANGE_AGENT" : "0_EXCHANGE_AGENT");
    snprintf(x->tname, sizeof x->tname, "ExchangeAgent");
    e->ex_open = open;
    e->ex_close = close;
    e->ex_pipeline = 0;
    e->ex_comp = 0;
    e->stream_history = 10;
    agent_t* a = add_agent(e, AG_REPLAY);
    trading_init(a, 0);
    snprintf(a->name, sizeof a->name, runner ? "MARKET_REPLAY_AGENT" : "1_MARKET_REPLAY_AGENT");
    snprintf(a->tname, sizeof a->tname, "MarketReplayAgent");
    agent_t* r = NULL;
    if (!runner) {
        r = add_agent(e, AG_DUMMYRL);
        trading_init(r, 0);
        snprintf(r->name, sizeof r->name, "2_DUMMY_RL_EXECUTION_AGENT");
    } else if (runner >= 2) {
        r = add_agent(e, AG_TWAP);
        trading_init(r, 0);
        snprintf(r->name, sizeof r->name, "TWAP_EXECUTION_AGENT");
        snprintf(r->tname, sizeof r->tname, "ExecutionAgent");
    }
    e->tp_n = n;
    e->tp_t = (int64_t*)malloc(sizeof(int64_t) * n);
    e->tp_oid = (int64_t*)malloc(sizeof(int64_t) * n);
    e->tp_price = (int64_t*)malloc(sizeof(int64_t) * n);
    e->tp_size = (int64_t*)malloc(sizeof(int64_t) * n);
    e->tp_buy = (int8_t*)malloc(n);
    memcpy(e->tp_t, t, sizeof(int64_t) * n);
    memcpy(e->tp_oid, oid, sizeof(int64_t) * n);
    memcpy(e->tp_price, price, sizeof(int64_t) * n);
    memcpy(e->tp_size, size, sizeof(int64_t) * n);
    memcpy(e->tp_buy, buy, n);
    e->tm = (int64_t*)malloc(sizeof(int64_t) * n);
    e->tm_start = (int*)malloc(sizeof(int) * (n + 1));
    for (int i = 0; i < n; i++) {
        if (i > 0 && t[i] < t[i - 1]) { free(e); return -2; } /* tape must be time-sorted */
        if (i == 0 || t[i] != t[i - 1]) {
            e->tm[e->ntm] = t[i];
            e->tm_start[e->ntm++] = i;
        }
    }
    e->tm_start[e->ntm] = n;
    e->mr_cap = 1;
    while (e->mr_cap < 2 * n + 64) e->mr_cap <<= 1;
    e->mr_key = (int64_t*)malloc(sizeof(int64_t) * e->mr_cap);
    for (int i = 0; i < e->mr_cap; i++) e->mr_key[i] = -1;
    e->mr_ord = (aord_t*)calloc(e->mr_cap, sizeof(aord_t));
    a = &e->ag[1]; /* add_agent reallocs: re-fetch */
    a->wake_freq = e->tm[0] - open;
    if (!runner) {
        r = &e->ag[2];
        /* execution_time_horizon = pd.date_range(09:40, 16:00, freq="30S") */
        e->nhz = 761;
        e->hz = (int64_t*)malloc(sizeof(int64_t) * e->nhz);
        for (int i = 0; i < e->nhz; i++) e->hz[i] = 9 * NS_HOUR + 40 * NS_MIN + (int64_t)i * 30 * NS_SEC;
        r->wake_freq = e->hz[0] - open;
        e->rl_quantity = 100000;
        e->rl_rem = 100000;
        e->rl_trade = 1;
        e->rl_id = 2;
        e->gym = 1;
    } else if (runner >= 2) {
        r = &e->ag[2];
        e->nhz = 121; /* pd.date_range(10:00, 12:00, freq="60S") */
        e->hz = (int64_t*)malloc(sizeof(int64_t) * e->nhz);
        for (int i = 0; i < e->nhz; i++) e->hz[i] = 10 * NS_HOUR + (int64_t)i * 60 * NS_SEC;
        r->wake_freq = e->hz[0] - open;
        e->rl_quantity = 12000;
        e->rl_rem = 12000;
        e->rl_trade = runner == 3;
    }
    e->start = 0;
    e->stop = runner ? 16 * NS_HOUR + NS_MIN : 16 * NS_HOUR + 10 * NS_MIN;
    e->lat_mode = 0;
    e->noise_len = 1;
    e->agent_time = (int64_t*)calloc(e->n, sizeof(int64_t));
    e->comp_delay = (int64_t*)calloc(e->n, sizeof(int64_t));
    e->nhist = 1;
    e->hash = FNV_OFF;
    e->ex_has_last = 0; /* no oracle: getDailyOpenPrice raises AttributeError, last_trade None */
    for (int i = 0; i < e->n; i++) k_wakeup(e, i, e->start);
    e->cur = e->start;
    *out = e;
    return 0;
}
int ora_create_mr(const int64_t* t, const int64_t* oid, const int64_t* price, const int64_t* size,
                  const int8_t* buy, int n, ora_env** out) {
    return create_mr(t, oid, price, size, buy, n, 0, out);
}
void ora_set_symbol(ora_env* e, const char* sym) { snprintf(e->sym, sizeof e->sym, "%s", sym); }
/* Kernel.runner(startTime, stopTime=...) with another stopTime than the config script's
 * (Kernel.py:50-64; the loop test `currentTime <= stopTime`, Kernel.py:190-196) */
void ora_set_stop(ora_env* e, int64_t t_stop) { e->stop = t_stop; }
int ora_create_mr_runner(const int64_t* t, const int64_t* oid, const int64_t* price, const int64_t* size,
                         const int8_t* buy, int n, ora_env** out) {
    return create_mr(t, oid, price, size, buy, n, 1, out);
}
int ora_create_mr_twap(const int64_t* t, const int64_t* oid, const int64_t* price, const int64_t* size,
                       const int8_t* buy, int n, int trade, ora_env** out) {
    return create_mr(t, oid, price, size, buy, n, trade ? 3 : 2, out);
}
int ora_rl_state(const ora_env* e, int64_t* out4) {
    out4[0] = e->rl_rem;
    out4[1] = e->rl_exec_sum;
    out4[2] = e->rl_trade;
    out4[3] = e->mr_nord;
    return 0;
}

/* config/random_fund_value.py:59-180 as a composition of rmsc03's construction: 5000 noise agents
 * waking in 09:30-16:00, 100 value agents (lambda_a 1e-12), no market maker or momentum agents,
 * market 09:30-16:00, kernel 09:30-16:01 (random_fund_diverse / hist_fund_* add their extras) */
static void cfg_random_fund(ora_config* c) {
    ora_config_defaults("rmsc03", c);
    c->mkt_close_ns = 16 * NS_HOUR;
    c->kernel_start_ns = c->mkt_open_ns;
    c->kernel_stop_ns = c->mkt_close_ns + NS_MIN;
    c->noise_wake_open_ns = c->mkt_open_ns;
    c->noise_wake_close_ns = 16 * NS_HOUR;
    c->n_noise = 5000;
    c->n_value = 100;
    c->n_mm = 0;
    c->n_momentum = 0;
    c->value_lambda_a = 1e-12;
}

/* a composition's construction by its base script */
static int build_config(ora_env* e, uint32_t seed, const ora_config* c) {
    switch (c->base) {
    case 0: return build_rmsc03_like(e, seed, 0, c);
    case 5: return build_value_noise(e, seed, c);
    case 1:
    case 2: return build_sparse_zi(e, seed, c);
    default: return -1;
    }
}

/* kernelInitializing / kernelStarting of a built env (every creation path) */
static int create_finish(ora_env* e, int rc, ora_env** out);

int ora_create_config(const ora_config* c, uint32_t seed, ora_env** out) {
    static const char* names[6] = {"rmsc03", "sparse_zi_100", "sparse_zi_1000", NULL, NULL, "value_noise"};
    if (!c || c->base < 0 || c->base > 5 || !names[c->base]) return -1;
    if (c->n_zi_groups < 0 || c->n_zi_groups > ORA_CONFIG_ZI_GROUPS || c->zi_q_max < 0 || c->zi_q_max > 10) return -1;
    ora_env* e = (ora_env*)calloc(1, sizeof(ora_env));
    snprintf(e->config, sizeof e->config, "%s", names[c->base]);
    e->cfg_log_orders = c->log_orders ? 1 : 0;
    e->has_cfg = 1;
    return create_finish(e, build_config(e, seed, c), out);
}

int ora_create(const char* config, uint32_t seed, ora_env** out) {
    ora_env* e = (ora_env*)calloc(1, sizeof(ora_env));
    snprintf(e->config, sizeof e->config, "%s", config);
    int rc;
    ora_config c;
    if (!strcmp(config, "sparse_zi_100") || !strcmp(config, "sparse_zi_1000") || !strcmp(config, "value_noise") ||
        !strcmp(config, "rmsc03")) {
        ora_config_defaults(config, &c);
        rc = build_config(e, seed, &c);
    } else if (!strncmp(config, "random_fund_", 12) || !strncmp(config, "hist_fund_", 10)) {
        cfg_random_fund(&c);
        const int rfv = !strcmp(config, "random_fund_value") ? 1 : !strcmp(config, "random_fund_diverse") ? 2
                        : !strcmp(config, "hist_fund_value") ? 3 : !strcmp(config, "hist_fund_diverse") ? 4 : -1;
        rc = rfv < 0 ? -1 : build_rmsc03_like(e, seed, rfv, &c);
    }
    else if (!strcmp(config, "rmsc03_sbmm")) rc = build_rmsc03_sbmm(e, seed, 1);
    else if (!strcmp(config, "rmsc03_sbmm_poll")) rc = build_rmsc03_sbmm(e, seed, 0);
    else if (!strcmp(config, "rmsc03_rl")) rc = build_rmsc03_rl(e, seed);
    else if (!strcmp(config, "rmsc01")) rc = build_rmsc0x(e, seed, 0, 0);
    else if (!strcmp(config, "rmsc02")) rc = build_rmsc0x(e, seed, 1, 0);
    else if (!strcmp(config, "obi_rmsc02")) rc = build_rmsc0x(e, seed, 1, 1);
    else rc = -1;
    return create_finish(e, rc, out);
}

static int create_finish(ora_env* e, int rc, ora_env** out) {
    if (rc) {
        free(e);
        return rc;
    }
    e->nhist = 1; /* history = [{}] */
    e->hash = FNV_OFF;
    /* kernelInitializing: exchange opening price = oracle.getDailyOpenPrice = r_bar (a float); the
     * ExternalFileOracle's is int(round(price at the open)) (ExternalFileOracle.py:37-50) */
    if (e->efo) {
        e->last_trade = py_round(efo_price(e->ex_open));
        e->last_trade_float = 0;
    } else {
        e->last_trade = (int64_t)e->o_rbar;
        e->last_trade_float = 1;
    }
    e->ex_has_last = 1;
    /* kernelStarting: every agent requests a wakeup at startTime, in id order */
    for (int i = 0; i < e->n; i++) k_wakeup(e, i, e->start);
    e->cur = e->start; /* Kernel.runner: currentTime = startTime before the loop */
    *out = e;
    return 0;
}

/* config/rmsc03.py -s SEED --mm-pov ... (config/rmsc03.py:39-43, 158-177): the options only reach
 * POVMarketMakerAgent.__init__ (pov, min_order_size, window_size, num_ticks, wake_up_freq;
 * POVMarketMakerAgent.py:19-60, order_size = min_order_size), never a draw, so the build is
 * rmsc03's with the market maker's fields replaced */
int ora_create_mm(uint32_t seed, const ora_mm_params* p, ora_env** out) {
    if (!p || p->mm_window_size < 0 || p->mm_num_ticks < 0 || p->mm_wake_up_freq_ns <= 0) return -1;
    int rc = ora_create("rmsc03", seed, out);
    if (rc) return rc;
    ora_env* e = *out;
    for (int i = 0; i < e->n; i++) {
        agent_t* a = &e->ag[i];
        if (a->type != AG_POVMM) continue;
        a->pov = p->mm_pov;
        a->min_size = p->mm_min_order_size;
        a->window = p->mm_window_size;
        a->num_ticks = p->mm_num_ticks;
        a->wake_freq = p->mm_wake_up_freq_ns;
        a->order_size = p->mm_min_order_size;
    }
    return 0;
}

void ora_destroy(ora_env* e) {
    if (!e) return;
    for (int i = 0; i < e->n; i++) {
        free(e->ag[i].ord);
        free(e->ag[i].mids2);
    }
    free(e->ag);
    for (int s = 0; s < 2; s++) {
        for (int i = 0; i < e->book[s].n; i++) free(e->book[s].lv[i].o);
        free(e->book[s].lv);
    }
    for (int i = 0; i < e->nhist + e->nret; i++) epoch_free(&e->hist[i]);
    free(e->blg);
    free(e->blr);
    free(e->lat);
    free(e->agent_time);
    free(e->comp_delay);
    free(e->heap);
    free(e->msgs);
    free(e->freem);
    free(e->report);
    free(e->tp_t);
    free(e->tp_oid);
    free(e->tp_price);
    free(e->tp_size);
    free(e->tp_buy);
    free(e->tm);
    free(e->tm_start);
    free(e->mr_key);
    free(e->mr_ord);
    free(e->used_ids);
    free(e->hz);
    free(e);
}

int ora_done(const ora_env* e) { return e->done; }
int ora_error(const ora_env* e) { return e->err; }
const char* ora_error_str(const ora_env* e) { return e->errstr; }
uint64_t ora_hash(const ora_env* e) { return e->hash; }
int64_t ora_events(const ora_env* e) { return e->pops; }
int64_t ora_current_time(const ora_env* e) { return e->cur; }
void ora_set_trace(ora_env* e, int64_t* buf, int64_t cap) {
    e->trace = buf;
    e->trace_cap = cap;
    e->trace_len = 0;
}
int64_t ora_trace_len(const ora_env* e) { return e->trace_len; }
int ora_n_agents(const ora_env* e) { return e->n; }
int ora_agent_state(const ora_env* e, int id, int64_t* cash, int64_t* shares, int64_t* n_open) {
    if (id < 0 || id >= e->n) return -1;
    *cash = e->ag[id].cash;
    *shares = e->ag[id].shares;
    *n_open = e->ag[id].type == AG_REPLAY ? e->mr_nord : e->ag[id].nord;
    return 0;
}
int64_t ora_book(const ora_env* e, int side, int64_t* buf, int64_t cap) {
    const side_t* S = &e->book[side ? 1 : 0];
    int64_t k = 0;
#define PUT(x) do { if (k < cap) buf[k] = (x); k++; } while (0)
    PUT(S->n);
    for (int i = 0; i < S->n; i++) {
        PUT(S->lv[i].n);
        for (int j = 0; j < S->lv[i].n; j++) {
            PUT(S->lv[i].o[j].id);
            PUT(S->lv[i].o[j].agent);
            PUT(S->lv[i].o[j].qty);
            PUT(S->lv[i].o[j].price);
        }
    }
#undef PUT
    return k;
}
int64_t ora_order_counter(const ora_env* e) { return e->order_counter; }
const char* ora_agent_type_name(const ora_env* e, int id) { return id >= 0 && id < e->n ? e->ag[id].tname : ""; }
/* Kernel.summaryLog rows after ora_finish; returns the row count (copies at most cap rows) */
int ora_summary(const ora_env* e, int* agent, int* type, int* isf, int64_t* vi, double* vf, int cap) {
    for (int k = 0; k < e->nsum && k < cap; k++) {
        agent[k] = e->sum_agent[k];
        type[k] = e->sum_type[k];
        isf[k] = e->sum_isf[k];
        vi[k] = e->sum_i[k];
        vf[k] = e->sum_f[k];
    }
    return e->nsum;
}
/* capacity statistics: max pending events, max resting orders, max open orders of one agent,
 * max live transaction records */
void ora_stats(const ora_env* e, int64_t* out) {
    out[0] = e->st_max_heap;
    out[1] = e->st_max_resting;
    out[2] = e->st_max_open;
    out[3] = e->st_max_hist_tx;
}
int64_t ora_last_trade(const ora_env* e) { return e->last_trade; }
int64_t ora_report(const ora_env* e, char* buf, int64_t cap) {
    if (!e->report) return 0;
    if (buf && cap > 0) {
        int64_t n = e->report_len < cap - 1 ? e->report_len : cap - 1;
        memcpy(buf, e->report, n);
        buf[n] = 0;
    }
    return e->report_len;
}

/* ------------------------------- batch runner ------------------------------- */
typedef struct {
    const char* config;
    const uint32_t* seeds;
    int n, next;
    int64_t max_pops;
    int64_t* ev;
    uint64_t* h;
    int32_t* err; /* optional: the env's oracle error code (0 ok, negative: fail() codes) */
    int64_t* stats; /* optional: [n][4] ora_stats of each env */
    const ora_mm_params* mm; /* optional: rmsc03 with per-env market-maker options */
    const ora_config* cfg;   /* optional: a runtime composition */
    pthread_mutex_t mu;
    int rc;
} batch_t;

static void* batch_worker(void* p) {
    batch_t* b = (batch_t*)p;
    for (;;) {
        pthread_mutex_lock(&b->mu);
        int i = b->next++;
        pthread_mutex_unlock(&b->mu);
        if (i >= b->n) break;
        ora_env* e = NULL;
        if (b->cfg ? ora_create_config(b->cfg, b->seeds[i], &e)
            : b->mm ? ora_create_mm(b->seeds[i], &b->mm[i], &e) : ora_create(b->config, b->seeds[i], &e)) {
            b->rc = -1;
            continue;
        }
        ora_run(e, b->max_pops);
        b->ev[i] = e->pops;
        b->h[i] = e->hash;
        if (b->err) b->err[i] = e->err;
        if (b->stats) ora_stats(e, b->stats + 4 * (size_t)i);
        ora_destroy(e);
    }
    return NULL;
}

static int run_batch_impl(const char* config, const uint32_t* seeds, int n, int threads, int64_t max_pops,
                          int64_t* events_out, uint64_t* hash_out, int32_t* err_out, int64_t* stats_out,
                          double* seconds_out, const ora_mm_params* mm, const ora_config* cfg) {
    batch_t b;
    memset(&b, 0, sizeof b);
    b.mm = mm;
    b.cfg = cfg;
    b.err = err_out;
    b.stats = stats_out;
    b.config = config;
    b.seeds = seeds;
    b.n = n;
    b.max_pops = max_pops;
    b.ev = events_out;
    b.h = hash_out;
    pthread_mutex_init(&b.mu, NULL);
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, batch_worker, &b);
    for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (seconds_out) *seconds_out = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
    free(th);
    pthread_mutex_destroy(&b.mu);
    return b.rc;
}

int ora_run_batch(const char* config, const uint32_t* seeds, int n, int threads, int64_t max_pops,
                  int64_t* events_out, uint64_t* hash_out, double* seconds_out) {
    return run_batch_impl(config, seeds, n, threads, max_pops, events_out, hash_out, NULL, NULL, seconds_out, NULL, NULL);
}

/* the same, with each env's error code (ora_error) in err_out[n] */
int ora_run_batch_err(const char* config, const uint32_t* seeds, int n, int threads, int64_t max_pops,
                      int64_t* events_out, uint64_t* hash_out, int32_t* err_out, double* seconds_out) {
    return run_batch_impl(config, seeds, n, threads, max_pops, events_out, hash_out, err_out, NULL, seconds_out, NULL, NULL);
}

/* capacity statistics (ora_stats) of n envs: stats_out[n][4] */
int ora_run_batch_stats(const char* config, const uint32_t* seeds, int n, int threads, int64_t* stats_out) {
    int64_t* ev = (int64_t*)calloc(n, sizeof(int64_t));
    uint64_t* h = (uint64_t*)calloc(n, sizeof(uint64_t));
    int rc = run_batch_impl(config, seeds, n, threads, -1, ev, h, NULL, stats_out, NULL, NULL, NULL);
    free(ev);
    free(h);
    return rc;
}

int ora_run_batch_config(const ora_config* c, const uint32_t* seeds, int n, int threads, int64_t max_pops,
                         int64_t* events_out, uint64_t* hash_out, int32_t* err_out, int64_t* stats_out,
                         double* seconds_out) {
    return run_batch_impl("composition", seeds, n, threads, max_pops, events_out, hash_out, err_out, stats_out,
                          seconds_out, NULL, c);
}
int ora_run_batch_mm(const uint32_t* seeds, const ora_mm_params* params, int n, int threads, int64_t max_pops,
                     int64_t* events_out, uint64_t* hash_out, int32_t* err_out, int64_t* stats_out, double* seconds_out) {
    if (!params) return -1;
    return run_batch_impl("rmsc03", seeds, n, threads, max_pops, events_out, hash_out, err_out, stats_out, seconds_out,
                          params, NULL);
}

void ora_set_book_log(ora_env* e, int on) {
    e->book_log = on;
    e->nblg = 0;
    e->nblr = 0;
    /* ExternalFileOracle: getDailyOpenPrice at kernelInitializing logged f_log's first entry when
     * the open lies inside the series (the device writes it at its first logged launch) */
    if (on && e->efo && e->pops == 0 && e->ex_open >= g_fs_t[0] && e->ex_open <= g_fs_t[g_fs_n - 1])
        efo_log(e, e->ex_open, efo_price(e->ex_open));
}
/* the exchange's own log in the record stream (include/mxa.h mxa_set_exchange_log); log_orders is
 * the config script's ExchangeAgent(log_orders=...) */
void ora_set_exchange_log(ora_env* e, int on) {
    e->exlog = on;
    e->ex_log_orders = e->has_cfg ? e->cfg_log_orders : ora_config_log_orders(e->config);
}
int ora_config_log_orders(const char* config) {
    /* each script's ExchangeAgent(log_orders=...): config/rmsc03.py:102 (its compositions: the
     * market-maker sweep, the SpreadBasedMarketMakerAgent and DummyRL ones), sparse_zi_100.py:187,
     * rmsc02.py:84, random_fund_*.py, hist_fund_*.py, marketreplay.py:77 / agent_config.py:54 */
    static const char* lo[] = {"rmsc03", "rmsc03_rl", "sparse_zi_100", "rmsc02", "random_fund_value",
                               "random_fund_diverse", "hist_fund_value", "hist_fund_diverse", "marketreplay",
                               "marketreplay_runner", "marketreplay_twap", "rmsc03_sbmm", "rmsc03_sbmm_poll", NULL};
    for (int i = 0; lo[i]; i++)
        if (strcmp(config, lo[i]) == 0) return 1;
    return 0;
}
int64_t ora_book_records(const ora_env* e, int64_t* buf, int64_t cap) {
    if (buf) memcpy(buf, e->blr, sizeof(int64_t) * (size_t)(cap < e->nblr ? cap : e->nblr));
    return e->nblr / 3;
}
int64_t ora_book_log(const ora_env* e, int64_t* buf, int64_t cap) {
    if (buf) memcpy(buf, e->blg, sizeof(int64_t) * (size_t)(cap < e->nblg ? cap : e->nblg));
    return e->nblg;
}

/* ABIDESEnv.reset (ABIDESEnv.py:51-57) in the same process: new agents and kernel (the
 * rmsc03 + DummyRL composition from `seed`, or the replay composition on the same tape), while
 * Order.order_id / Order._order_ids carry over (Order.py:8-9).
 * *pe is replaced; a trace buffer must be set again. */
int ora_gym_reset(ora_env** pe, uint32_t seed) {
    ora_env* old = *pe;
    ora_env* e = NULL;
    int rc = old->tp_n ? create_mr(old->tp_t, old->tp_oid, old->tp_price, old->tp_size, old->tp_buy, old->tp_n,
                                   !old->gym, &e)
                       : ora_create(old->config, seed, &e);
    if (rc) return rc;
    e->order_counter = old->order_counter;
    free(e->used_ids);
    e->used_ids = old->used_ids;
    e->used_cap = old->used_cap;
    e->used_n = old->used_n;
    old->used_ids = NULL;
    ora_destroy(old);
    *pe = e;
    return 0;
}

/* ------------------------------ gym batch runner ------------------------------ */
/* n independent GymKernel episodes (ABIDESEnv.step loop, ABIDESEnv.py:30-49), each stepped with
 * its own action rows until done or an error: the rmsc03 + DummyRL composition from per-env seeds
 * (config "rmsc03_rl") or the replay composition on one tape (config NULL).  Test
 * infrastructure: bench-size parity of mxa_step against this restatement. */
typedef struct {
    const char* config;
    const uint32_t* seeds;
    const int64_t *t, *oid, *price, *size;
    const int8_t* buy;
    int n_rec, n, n_steps, next;
    const double* act; /* [n_steps][n][3] */
    int64_t* ev;
    uint64_t* h;
    int32_t* err;
    int32_t* steps;
    double* obs; /* [n][9]: the last valid observation */
    pthread_mutex_t mu;
    int rc;
} gym_batch_t;

static void* gym_batch_worker(void* p) {
    gym_batch_t* b = (gym_batch_t*)p;
    for (;;) {
        pthread_mutex_lock(&b->mu);
        int i = b->next++;
        pthread_mutex_unlock(&b->mu);
        if (i >= b->n) break;
        ora_env* e = NULL;
        int rc = b->config ? ora_create(b->config, b->seeds[i], &e)
                           : ora_create_mr(b->t, b->oid, b->price, b->size, b->buy, b->n_rec, &e);
        if (rc) {
            b->rc = -1;
            continue;
        }
        double obs[9];
        int has = 0, done = 0, k = 0;
        memset(b->obs + 9 * (size_t)i, 0, sizeof obs);
        for (k = 0; k < b->n_steps; k++) {
            int r = ora_gym_step(e, b->act + 3 * ((size_t)k * b->n + i), obs, &has, &done);
            if (has && !r) memcpy(b->obs + 9 * (size_t)i, obs, sizeof obs);
            if (r || done) {
                k++;
                break;
            }
        }
        b->ev[i] = e->pops;
        b->h[i] = e->hash;
        b->err[i] = e->err;
        b->steps[i] = k;
        ora_destroy(e);
    }
    return NULL;
}

int ora_gym_batch(const char* config, const uint32_t* seeds, const int64_t* t, const int64_t* oid,
                  const int64_t* price, const int64_t* size, const int8_t* buy, int n_rec, int n, int n_steps,
                  const double* actions, int threads, int64_t* ev_out, uint64_t* hash_out, int32_t* err_out,
                  int32_t* steps_out, double* obs_out, double* seconds_out) {
    gym_batch_t b;
    memset(&b, 0, sizeof b);
    b.config = config;
    b.seeds = seeds;
    b.t = t;
    b.oid = oid;
    b.price = price;
    b.size = size;
    b.buy = buy;
    b.n_rec = n_rec;
    b.n = n;
    b.n_steps = n_steps;
    b.act = actions;
    b.ev = ev_out;
    b.h = hash_out;
    b.err = err_out;
    b.steps = steps_out;
    b.obs = obs_out;
    pthread_mutex_init(&b.mu, NULL);
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, gym_batch_worker, &b);
    for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (seconds_out) *seconds_out = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
    free(th);
    pthread_mutex_destroy(&b.mu);
    return b.rc;
}
