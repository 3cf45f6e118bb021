// mxa_api.hip — host side of libmxa: the C-ABI declared in include/mxa.h.
//
// Builds the per-configuration parameter block (the constants of the reference config
// scripts), lays out one HBM block per env, and launches the kernels of mxa_kernels.hip.
// Each configuration's engine is its own translation unit (mxa_inst.hip, mxa_entry.h); an
// rmsc03-only variant build (-DMXA_ONLY_RMSC03) compiles everything in this one.
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <spawn.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

extern char** environ;

#include "../../include/mxa.h"
#define MXA_API_TU
#include "mxa_kernels.hip"
#include "mxa_entry.h"
#ifdef MXA_ONLY_RMSC03
#ifndef MXA_ONLY_CFG  // single-configuration variant builds (profiling): that one configuration
#define MXA_ONLY_CFG 0
#endif
#define MXA_INST_CFG MXA_ONLY_CFG
#include "mxa_inst.hip"
#endif

namespace {

// the envs still running, in env order, and their count: one workgroup of 16 waves walks the env
// headers 1024 at a time (a ballot per wave, the waves' counts through LDS).  The next launch of
// mxa_run is one wave per listed env
__global__ __launch_bounds__(1024) void mxa_compact_kernel(const char* base, uint64_t stride, int n, int32_t* list,
                                                           int* count) {
  __shared__ int wn[16];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  int done = 0;
  for (int i0 = 0; i0 < n; i0 += 1024) {
    const int i = i0 + (int)threadIdx.x;
    const bool run = i < n && ((const EnvHdr*)(base + (size_t)i * stride))->status == ST_RUNNING;
    const uint64_t m = __ballot(run);
    if (l == 0) wn[w] = __popcll(m);
    __syncthreads();
    int off = done, tot = 0;
    for (int k = 0; k < 16; k++) {
      off += k < w ? wn[k] : 0;
      tot += wn[k];
    }
    if (run) list[off + __popcll(m & ((1ull << l) - 1))] = i;
    done += tot;
    __syncthreads();  // wn is rewritten by the next block of envs
  }
  if (threadIdx.x == 0) *count = done;
}

// Kernel.runner's stopTime of every env (EnvHdr::t_stop; 0 = the config's own)
// the exchange-log switch of every env (EnvHdr::exlog)
__global__ void mxa_set_exlog_kernel(char* base, uint64_t stride, int n, int32_t on) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ((EnvHdr*)(base + (size_t)i * stride))->exlog = on;
}
__global__ void mxa_set_stop_kernel(char* base, uint64_t stride, int n, int64_t t_stop) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ((EnvHdr*)(base + (size_t)i * stride))->t_stop = t_stop;
}

__global__ void mxa_results_kernel(const char* base, uint64_t stride, int n, int64_t* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const EnvHdr* h = (const EnvHdr*)(base + (size_t)i * stride);
  out[4 * i + 0] = h->pops;
  out[4 * i + 1] = (int64_t)h->hash;
  out[4 * i + 2] = h->status;
  out[4 * i + 3] = h->cur;
}

// per-env episode record of the multi-GPU all-gather (events, status, final cash,
// holdings, return; one wave per env): [n][MXA_RECORD_WORDS] int64, see include/mxa.h.  The cash /
// holdings / gain words sum TradingAgent.holdings over agents 1.. (Kernel.runner configs; the gain
// is markToMarket - starting_cash, TradingAgent.py:609-633, summed over the agents whose mean
// Kernel.runner prints, Kernel.py:330-341) or are the execution agent's own (GymKernel handles)
__global__ __launch_bounds__(64) void mxa_records_kernel(const char* base, uint64_t stride, int n, const uint32_t* seeds,
                                                         uint32_t off_ag, int a0, int a1, int64_t* out) {
  const int i = blockIdx.x, lane = threadIdx.x;
  if (i >= n) return;
  const char* e = base + (size_t)i * stride;
  long long cash = 0, shares = 0, gain = 0;
  for (int a = a0 + lane; a < a1; a += 64) {
    const uint32_t* r = (const uint32_t*)(e + off_ag + (size_t)a * 512);
    auto g64 = [&](int f) { return (long long)(((uint64_t)r[f + 1] << 32) | r[f]); };
    const long long c = g64(AF_CASH), s = g64(AF_SHARES);
    cash += c;
    shares += s;
    gain += c + (s ? s * g64(AF_LAST_TRADE) : 0) - g64(AF_START_CASH);
  }
  for (int d = 32; d >= 1; d >>= 1) {
    cash += __shfl_xor(cash, d, 64);
    shares += __shfl_xor(shares, d, 64);
    gain += __shfl_xor(gain, d, 64);
  }
  if (lane == 0) {
    const EnvHdr* h = (const EnvHdr*)e;
    int64_t* o = out + (size_t)MXA_RECORD_WORDS * i;
    o[0] = h->pops;
    o[1] = (int64_t)h->hash;
    o[2] = h->status;
    o[3] = h->cur;
    o[4] = h->status == ST_ERROR ? h->err : 0;
    o[5] = seeds[i];
    o[6] = h->last_trade;
    o[7] = h->order_counter;
    o[8] = cash;
    o[9] = shares;
    o[10] = gain;
    o[11] = 0;
  }
}

// event-class counters of an instrumented run (include/mxa.h mxa_read_counters), one wave per env
__global__ __launch_bounds__(64) void mxa_counters_kernel(const char* base, uint64_t stride, int n, uint32_t off_ag,
                                                          int n_agents, int64_t* out) {
  const int i = blockIdx.x, lane = threadIdx.x;
  if (i >= n) return;
  const char* e = base + (size_t)i * stride;
  const EnvHdr* h = (const EnvHdr*)e;
  long long w = 0;
  for (int a = lane; a < n_agents; a += 64)
    w += (long long)(((const uint32_t*)(e + off_ag + (size_t)a * 512))[AF_RS_POS] - MXA_MT_N);
  for (int d = 32; d >= 1; d >>= 1) w += __shfl_xor(w, d, 64);
  int64_t* o = out + (size_t)MXA_COUNTER_WORDS * i;
  if (lane < 26) o[lane] = h->kc[lane];
  if (lane == 0) {
    for (int k = 0; k < 4; k++) w += h->rs_pos[k] - MXA_MT_N;
    const int64_t req = h->kc[MXA_KC_REQUEUE];
    o[26] = (int64_t)h->q_count - h->q0 + h->pops - req;  // every pop but a requeue removed one event
    o[27] = w - (int64_t)h->rng0;
    o[28] = h->pops;
    o[29] = h->max_q;
    o[30] = h->max_book;
    o[31] = h->kc[MXA_KC_REC];
    o[32] = h->kc[MXA_KC_RUN];
    o[33] = 0;
  }
}

// execution-agent state after a step, for a learner on the device: [n][MXA_RL_STATE_WORDS]
// doubles = (CASH, holdings, executed qty, best bid, best ask, bid size, ask size, lob flags)
// of DummyRLExecutionAgent (TradingAgent.holdings, ExecutionAgent.executed quantity,
// ABIDESEnvMetrics' newest LOB: dummy_rl:294-315, execution_agent.py:88-100)
__global__ void mxa_rl_state_kernel(const char* base, uint64_t stride, int n, uint32_t off_rec, uint64_t off_rh,
                                    uint64_t off_ring, double* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const char* e = base + (size_t)i * stride;
  const uint32_t* r = (const uint32_t*)(e + off_rec);
  const RpHdr* R = (const RpHdr*)(e + off_rh);
  const RpLob* L = (const RpLob*)(e + off_ring);
  auto g64 = [&](int f) { return (int64_t)(((uint64_t)r[f + 1] << 32) | r[f]); };
  double* o = out + (size_t)MXA_RL_STATE_WORDS * i;
  o[0] = (double)g64(AF_CASH);
  o[1] = (double)g64(AF_SHARES);
  o[2] = (double)R->rl_exec;
  if (R->m_cnt > 0) {
    const RpLob l = L[R->m_head];
    o[3] = (double)l.bid;
    o[4] = (double)l.ask;
    o[5] = (double)R->m_bq;
    o[6] = (double)R->m_aq;
    o[7] = (double)(l.flags & 3);
  } else {
    o[3] = o[4] = o[5] = o[6] = o[7] = 0.0;
  }
}

}  // namespace

struct mxa_handle {
  MxaParams P;
  int device = 0;
  hipStream_t own = nullptr, stream = nullptr;
  char* d_env = nullptr;
  uint32_t* d_seeds = nullptr;
  uint8_t* d_mask = nullptr;
  int* d_count = nullptr;
  int32_t* d_list = nullptr;  // [n_envs] the running envs after a launch (mxa_compact_kernel)
  int64_t first_chunk = 0;    // mxa_set_launch_schedule: mxa_run's first launch (0: every launch `chunk`)
  size_t lds = 0;
  mxa_build_fn build = nullptr;
  mxa_run_fn run = nullptr, run_log = nullptr;     // run_log: with the book-update log
  mxa_run_fn run_fast = nullptr;                   // hash off, no trace ring: instrumentation compiled out
  mxa_step_fn step = nullptr, step_fast = nullptr;  // GymKernel handles (replay, rmsc03_rl)
  mxa_step_many_fn step_many = nullptr, step_many_fast = nullptr;  // k steps per launch
  mxa_stop_fn stop = nullptr, stop_log = nullptr;  // kernelStopping pass (plain Kernel.runner configs)
  mxa_agent_final* d_final = nullptr;
  BlRec* d_blog = nullptr;  // book-update log [n_envs][blog_cap] (mxa_set_book_log)
  int32_t blog_cap = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  double last_ms = 0;
  std::string err;
  // GymKernel handles (ABIDESEnv replay, rmsc03 + DummyRL): stepped with actions
  bool gym = false;
  bool replay = false;  // the replay ladder book + tape
  RpCtx ctx{};             // host copy (pointers are device pointers)
  RpCtx* d_ctx = nullptr;
  char* d_tape = nullptr;
  double *d_act = nullptr, *d_obs = nullptr;
  int32_t* d_flags = nullptr;
  bool parity_hash = true;  // per-pop trace hash (test instrumentation); off: kernel tcap -1
  // GymKernel handles: mxa_reset continues Order.order_id / Order._order_ids of the previous
  // episode (one process running consecutive ABIDESEnv episodes)
  bool persist_ids = false;
  int32_t exlog = 0;   // mxa_set_exchange_log: the exchange's own log rides in the book-update log
  bool started = false;  // a launch ran since the last whole-handle mxa_reset (the exchange log is fixed then)
  int64_t t_stop = 0;  // mxa_set_stop_time: Kernel.runner's stopTime override (0: the config's)
  int32_t tcap_arg() const { return (parity_hash || P.L.trace_cap > 0) ? P.L.trace_cap : -1; }
  // the run kernel of the current settings: the log variant, the instrumented one, or (hash off,
  // no trace ring) the one without the parity instrumentation
  mxa_run_fn run_kernel() const {
    if (d_blog) return run_log;
    return (tcap_arg() < 0 && run_fast) ? run_fast : run;
  }
  std::vector<char> tape_blob;  // host staging of the tape (uploaded by create_common)
  size_t tb_t, tb_oid, tb_dense, tb_price, tb_size, tb_buy, tb_tm, tb_tm0, tb_uid, tb_ufirst;
  bool ext = false;  // ExternalFileOracle configurations: the fundamental series in d_tape
  size_t tb_fs_t = 0, tb_fs_v = 0;
  // MXA_RMSC03_MM: per-env market-maker options (config/rmsc03.py --mm-*), read by every build
  std::vector<MmParams> mm;
  MmParams* d_mmp = nullptr;
  mxa_occ_fn occ = nullptr;  // resident waves per CU of the handle's measured kernel
};

static int hip_fail(mxa_handle* h, hipError_t e, const char* what) {
  if (h) h->err = std::string(what) + ": " + hipGetErrorString(e);
  return MXA_EHIP;
}
#define HIPCHK(h, x)                                 \
  do {                                               \
    hipError_t _e = (x);                             \
    if (_e != hipSuccess) return hip_fail(h, _e, #x); \
  } while (0)

static int create_common(mxa_handle* h, int32_t n_envs, const uint32_t* seeds, int32_t device, mxa_handle** out);

// the configuration's launchers (mxa_entry.h); false: not built into this library
static bool bind(mxa_handle* h, int cfg) {
  MxaEntry e{};
  switch (cfg) {
#ifdef MXA_ONLY_RMSC03
  case MXA_ONLY_CFG: e = MXA_ENTRY_CAT(mxa_entry_, MXA_ONLY_CFG)(); break;
#else
  case 0: e = mxa_entry_0(); break;
  case 1: e = mxa_entry_1(); break;
  case 2: e = mxa_entry_2(); break;
  case 3: e = mxa_entry_3(); break;
  case 4: e = mxa_entry_4(); break;
  case 5: e = mxa_entry_5(); break;
  case 6: e = mxa_entry_6(); break;
  case 7: e = mxa_entry_7(); break;
  case 8: e = mxa_entry_8(); break;
  case 9: e = mxa_entry_9(); break;
  case 10: e = mxa_entry_10(); break;
  case 11: e = mxa_entry_11(); break;
  case 12: e = mxa_entry_12(); break;
  case 13: e = mxa_entry_13(); break;
  case 14: e = mxa_entry_14(); break;
  case 15: e = mxa_entry_15(); break;
  case 16: e = mxa_entry_16(); break;
  case 17: e = mxa_entry_17(); break;
#endif
  default: return false;
  }
  h->build = e.build;
  h->run = e.run;
  h->run_log = e.run_log;
  h->run_fast = e.run_fast;
  h->stop = e.stop;
  h->stop_log = e.stop_log;
  h->step = e.step;
  h->step_fast = e.step_fast;
  h->step_many = e.step_many;
  h->step_many_fast = e.step_many_fast;
  h->gym = e.step != nullptr;
  h->occ = e.occ;
  h->lds = mxa_cfg::lds_bytes(cfg);
  return true;
}

extern "C" {

#ifdef MXA_PROF
// diagnostics build only (not in include/mxa.h): phase cycle totals, then cleared
int mxa_prof_read(uint64_t* out64) {
  if (hipMemcpyFromSymbol(out64, HIP_SYMBOL(mxa::g_mxa_prof), 128 * 8) != hipSuccess) return MXA_EHIP;
  static const uint64_t z[128] = {0};
  if (hipMemcpyToSymbol(HIP_SYMBOL(mxa::g_mxa_prof), z, 128 * 8) != hipSuccess) return MXA_EHIP;
  return MXA_OK;
}
#endif

int mxa_create(int32_t config, int32_t n_envs, const uint32_t* seeds, int32_t device, int32_t trace_cap,
               mxa_handle** out) {
  if (!out || n_envs <= 0 || !seeds || trace_cap < 0) return MXA_EINVAL;
  mxa_handle* h = new mxa_handle();
  static_assert((int)MXA_RMSC03 == (int)MXA_CFG_RMSC03 && (int)MXA_SPARSE_ZI_100 == (int)MXA_CFG_SPARSE_ZI_100 &&
                    (int)MXA_SPARSE_ZI_1000 == (int)MXA_CFG_SPARSE_ZI_1000 &&
                    (int)MXA_MARKETREPLAY == (int)MXA_CFG_MARKETREPLAY && (int)MXA_RMSC03_RL == (int)MXA_CFG_RMSC03_RL &&
                    (int)MXA_VALUE_NOISE == (int)MXA_CFG_VALUE_NOISE && (int)MXA_RMSC01 == (int)MXA_CFG_RMSC01 &&
                    (int)MXA_RMSC02 == (int)MXA_CFG_RMSC02 && (int)MXA_OBI_RMSC02 == (int)MXA_CFG_OBI_RMSC02 &&
                    (int)MXA_RANDOM_FUND_VALUE == (int)MXA_CFG_RANDOM_FUND_VALUE &&
                    (int)MXA_RANDOM_FUND_DIVERSE == (int)MXA_CFG_RANDOM_FUND_DIVERSE &&
                    (int)MXA_HIST_FUND_VALUE == (int)MXA_CFG_HIST_FUND_VALUE &&
                    (int)MXA_HIST_FUND_DIVERSE == (int)MXA_CFG_HIST_FUND_DIVERSE &&
                    (int)MXA_MARKETREPLAY_RUNNER == (int)MXA_CFG_MARKETREPLAY_RUNNER &&
                    (int)MXA_MARKETREPLAY_TWAP == (int)MXA_CFG_MARKETREPLAY_TWAP &&
                    (int)MXA_RMSC03_SBMM == (int)MXA_CFG_RMSC03_SBMM &&
                    (int)MXA_RMSC03_SBMM_POLL == (int)MXA_CFG_RMSC03_SBMM_POLL &&
                    (int)MXA_RMSC03_MM == (int)MXA_CFG_RMSC03_MM,
                "config ids");
  static_assert(MXA_N_CONFIGS == (int)MXA_CFG_RMSC03_MM + 1, "one entry per configuration");
  static_assert(sizeof(mxa_mm_params) == sizeof(MmParams) && offsetof(mxa_mm_params, mm_wake_up_freq_ns) ==
                    offsetof(MmParams, wake_up_freq) && offsetof(mxa_mm_params, mm_num_ticks) == offsetof(MmParams, num_ticks),
                "mxa_mm_params is MmParams");
  if (config == MXA_RMSC03_MM) {  // the config script's defaults in every env
    std::vector<mxa_mm_params> d(n_envs > 0 ? n_envs : 0);
    for (auto& x : d) x = mxa_mm_defaults();
    delete h;
    return mxa_create_params(MXA_RMSC03, n_envs, seeds, d.data(), device, trace_cap, out);
  }
  // replay handles: mxa_create_replay(_runner); ExternalFileOracle configurations: mxa_create_hist
  if (config == MXA_MARKETREPLAY || config == MXA_MARKETREPLAY_RUNNER || config == MXA_MARKETREPLAY_TWAP ||
      config == MXA_HIST_FUND_VALUE ||
      config == MXA_HIST_FUND_DIVERSE || !bind(h, config)) {
    delete h;
    return MXA_EINVAL;
  }
  h->P = mxa_cfg::params(config);
  h->P.n_envs = n_envs;
  h->P.L.trace_cap = trace_cap;
  h->P.L.env_stride = mxa_cfg::env_stride(config, trace_cap);
  if (h->gym) {  // the DummyRL metrics header + deque after the trace (no ladder, no tape)
    h->ctx.L = mxa_cfg::replay_layout(h->P.L.env_stride, 0, 0, 0, 0, 0, 0, 0);
    h->P.L.env_stride = h->ctx.L.end;
  }
  return create_common(h, n_envs, seeds, device, out);
}

static int check_mm(const mxa_mm_params* p, int n) {
  for (int i = 0; i < n; i++) {
    const mxa_mm_params& x = p[i];
    // the reference raises nowhere on these, but a negative window / tick count, a
    // non-positive wake-up period or a NaN / negative pov is no option the script can run.  A pov
    // whose order size outgrows the 32-bit order words stops that env with MXA_ERR_ORDER_SIZE
    // at the order (the cap here only keeps pov x volume exact in a double)
    if (!(x.mm_pov == x.mm_pov) || x.mm_pov < 0 || x.mm_pov > 1e12 || x.mm_min_order_size < 0 || x.mm_window_size < 0 ||
        x.mm_num_ticks < 0 || x.mm_num_ticks > 100000 || x.mm_wake_up_freq_ns <= 0)
      return MXA_EINVAL;
  }
  return MXA_OK;
}

mxa_mm_params mxa_mm_defaults(void) {
  mxa_mm_params p{};
  const MxaParams P = mxa_cfg::params(MXA_CFG_RMSC03);
  p.mm_pov = P.mm_pov;
  p.mm_min_order_size = P.mm_min_size;
  p.mm_window_size = P.mm_window;
  p.mm_num_ticks = P.mm_ticks;
  p.mm_wake_up_freq_ns = P.mm_wake;
  return p;
}

// config/rmsc03.py with each env's market-maker options; see include/mxa.h
int mxa_create_params(int32_t config, int32_t n_envs, const uint32_t* seeds, const mxa_mm_params* per_env,
                      int32_t device, int32_t trace_cap, mxa_handle** out) {
  if (!out || n_envs <= 0 || !seeds || !per_env || trace_cap < 0 || config != MXA_RMSC03) return MXA_EINVAL;
  if (check_mm(per_env, n_envs)) return MXA_EINVAL;
  mxa_handle* h = new mxa_handle();
  if (!bind(h, MXA_CFG_RMSC03_MM)) {
    delete h;
    return MXA_EINVAL;
  }
  h->P = mxa_cfg::params(MXA_CFG_RMSC03_MM);
  h->P.n_envs = n_envs;
  h->P.L.trace_cap = trace_cap;
  h->P.L.env_stride = mxa_cfg::env_stride(MXA_CFG_RMSC03_MM, trace_cap);
  h->mm.assign((const MmParams*)per_env, (const MmParams*)per_env + n_envs);
  return create_common(h, n_envs, seeds, device, out);
}

int mxa_set_mm_params(mxa_handle* h, const mxa_mm_params* per_env) {
  if (!h || !per_env || !h->d_mmp) return MXA_EINVAL;
  if (check_mm(per_env, h->P.n_envs)) return MXA_EINVAL;
  HIPCHK(h, hipSetDevice(h->device));
  memcpy(h->mm.data(), per_env, sizeof(MmParams) * h->P.n_envs);
  HIPCHK(h, hipMemcpyAsync(h->d_mmp, h->mm.data(), sizeof(MmParams) * h->P.n_envs, hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return MXA_OK;
}

int mxa_resident_envs(const mxa_handle* h) {
  if (!h || !h->occ) return MXA_EINVAL;
  int dev = 0, cus = 0;
  if (hipSetDevice(h->device) != hipSuccess || hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return MXA_EHIP;
  const int per_cu = h->occ(h->lds);
  if (per_cu < 0) return MXA_EHIP;
  return per_cu * cus < h->P.n_envs ? per_cu * cus : h->P.n_envs;
}

// config/hist_fund_value.py / hist_fund_diverse.py: the ExternalFileOracle's series is the
// handle's (shared by its envs, device-resident); see include/mxa.h
int mxa_create_hist(int32_t config, int32_t n_envs, const uint32_t* seeds, int32_t device, int32_t trace_cap,
                    const int64_t* fund_t, const double* fund_v, int32_t n_fund, mxa_handle** out) {
  if (!out || n_envs <= 0 || !seeds || trace_cap < 0 || !fund_t || !fund_v || n_fund <= 0) return MXA_EINVAL;
  if (config != MXA_HIST_FUND_VALUE && config != MXA_HIST_FUND_DIVERSE) return MXA_EINVAL;
  for (int i = 0; i < n_fund; i++)
    if ((i && fund_t[i] < fund_t[i - 1]) || !(fund_v[i] == fund_v[i]) || fund_v[i] > 1e15 || fund_v[i] < -1e15)
      return MXA_EINVAL;  // unsorted times or a value int(round()) cannot take (NaN raises in the reference)
  mxa_handle* h = new mxa_handle();
  if (!bind(h, config)) {
    delete h;
    return MXA_EINVAL;
  }
  h->P = mxa_cfg::params(config);
  h->P.n_envs = n_envs;
  h->P.L.trace_cap = trace_cap;
  h->P.L.env_stride = mxa_cfg::env_stride(config, trace_cap);
  auto al = [](size_t x) { return (x + 255) / 256 * 256; };
  h->tb_fs_t = 0;
  h->tb_fs_v = al(8ull * n_fund);
  h->tape_blob.assign(al(h->tb_fs_v + 8ull * n_fund), 0);
  memcpy(h->tape_blob.data() + h->tb_fs_t, fund_t, 8ull * n_fund);
  memcpy(h->tape_blob.data() + h->tb_fs_v, fund_v, 8ull * n_fund);
  h->ctx.fs_n = n_fund;
  h->ext = true;
  return create_common(h, n_envs, seeds, device, out);
}

// ---- runtime compositions (include/mxa.h mxa_config): one specialised library per composition
#ifndef MXA_BUILD_ID
#define MXA_BUILD_ID "unknown"
#endif
// the compile line of a specialisation: build_lib.py's flags (passed in when this file is
// compiled), per base configuration its extra flags ("<cfg>:<flags>;...")
#ifndef MXA_JIT_FLAGS
#define MXA_JIT_FLAGS "--offload-arch=gfx950 -O3 -std=c++20"
#endif
#ifndef MXA_JIT_CFG_FLAGS
#define MXA_JIT_CFG_FLAGS ""
#endif
static std::string g_cfg_err;  // mxa_last_error(NULL): the last composition error

static int cfg_fail(const std::string& what) {
  g_cfg_err = what;
  return MXA_EINVAL;
}

// the directory holding this library (lib/), from which csrc/ and include/ are found
static std::string lib_dir() {
  Dl_info di{};
  if (!dladdr((void*)&mxa_config_defaults, &di) || !di.dli_fname) return ".";
  std::string p = di.dli_fname;
  const size_t k = p.rfind('/');
  return k == std::string::npos ? "." : p.substr(0, k);
}

static std::vector<std::string> split_ws(const std::string& s) {
  std::vector<std::string> v;
  size_t i = 0;
  while (i < s.size()) {
    while (i < s.size() && s[i] == ' ') i++;
    size_t j = i;
    while (j < s.size() && s[j] != ' ') j++;
    if (j > i) v.push_back(s.substr(i, j - i));
    i = j;
  }
  return v;
}

static std::string cfg_key(const mxa_config& c) {
  mxa_config k = c;
  k.date_ns = 0;  // output timestamps only: one specialisation serves every date
  uint64_t h = 0xCBF29CE484222325ull;
  const unsigned char* b = (const unsigned char*)&k;
  for (size_t i = 0; i < sizeof k; i++) h = (h ^ b[i]) * 0x100000001B3ull;
  for (const char* p = MXA_BUILD_ID; *p; p++) h = (h ^ (unsigned char)*p) * 0x100000001B3ull;
  char buf[17];
  snprintf(buf, sizeof buf, "%016llx", (unsigned long long)h);
  return buf;
}

static std::string cfg_dir(const char* cache_dir) { return cache_dir && *cache_dir ? cache_dir : lib_dir() + "/custom"; }
static std::string cfg_lib(const char* cache_dir, const std::string& key) {
  return cfg_dir(cache_dir) + "/libmxa_cfg_" + key + ".so";
}

int mxa_config_defaults(int32_t base, mxa_config* out) {
  if (!out || !mxa_cfg::custom_base_ok(base)) return cfg_fail("mxa_config_defaults: no such base script");
  static_assert(sizeof(mxa_config) % 8 == 0, "mxa_config: no tail padding (its bytes are the cache key)");
  mxa_cfg::config_defaults(base, *out);
  return MXA_OK;
}

int mxa_config_key(const mxa_config* cfg, char* out17) {
  if (!cfg || !out17) return MXA_EINVAL;
  snprintf(out17, 17, "%s", cfg_key(*cfg).c_str());
  return MXA_OK;
}

int mxa_config_compile(const mxa_config* cfg, const char* cache_dir, char* path_out, int32_t path_cap) {
  if (!cfg) return cfg_fail("mxa_config_compile: null composition");
  if (const char* why = mxa_cfg::custom_check(*cfg)) return cfg_fail(std::string("mxa_config_compile: ") + why);
  const std::string key = cfg_key(*cfg), dir = cfg_dir(cache_dir), so = cfg_lib(cache_dir, key);
  if (path_out && path_cap > 0) snprintf(path_out, path_cap, "%s", so.c_str());
  struct stat st{};
  if (stat(so.c_str(), &st) == 0) return MXA_OK;  // compiled before
  mkdir(dir.c_str(), 0755);
  const std::string hdr = dir + "/mxa_cfg_" + key + ".h";
  {
    FILE* f = fopen(hdr.c_str(), "w");
    if (!f) return cfg_fail("mxa_config_compile: cannot write " + hdr);
    fprintf(f, "// a runtime composition (include/mxa.h mxa_config), written by mxa_config_compile\n");
    fprintf(f, "#define MXA_CUSTOM_BYTES {");
    const unsigned char* b = (const unsigned char*)cfg;
    for (size_t i = 0; i < sizeof(mxa_config); i++) fprintf(f, "%s%u", i ? "," : "", b[i]);
    fprintf(f, "}\n");
    fclose(f);
  }
  const std::string ld = lib_dir(), src = ld + "/../csrc", inc = ld + "/../../include";
  const char* hipcc = getenv("HIPCC");
  std::vector<std::string> argv = {hipcc && *hipcc ? hipcc : "/opt/rocm/bin/hipcc"};
  for (auto& x : split_ws(MXA_JIT_FLAGS)) argv.push_back(x);
  {  // the base's own backend flags
    const std::string all = MXA_JIT_CFG_FLAGS, pre = std::to_string(cfg->base) + ":";
    size_t i = 0;
    while (i < all.size()) {
      size_t j = all.find(';', i);
      if (j == std::string::npos) j = all.size();
      const std::string item = all.substr(i, j - i);
      if (item.compare(0, pre.size(), pre) == 0)
        for (auto& x : split_ws(item.substr(pre.size()))) argv.push_back(x);
      i = j + 1;
    }
  }
  const std::string tmp = so + ".tmp." + std::to_string((long)getpid());
  for (const std::string& x : {std::string("-fvisibility=hidden"), std::string("-fvisibility-inlines-hidden"),
                               std::string("-Wl,-Bsymbolic"), std::string("-shared"),
                               "-DMXA_INST_CFG=" + std::to_string(cfg->base), "-DMXA_CUSTOM_HDR=\"" + hdr + "\"",
                               std::string("-DMXA_BUILD_ID=\"") + MXA_BUILD_ID + "\"", "-I" + src, "-I" + inc,
                               src + "/mxa_inst.hip", std::string("-o"), tmp})
    argv.push_back(x);
  std::vector<char*> av;
  for (auto& x : argv) av.push_back((char*)x.c_str());
  av.push_back(nullptr);
  pid_t pid = 0;
  // a child process (posix_spawn), never an exec of this one
  if (posix_spawn(&pid, av[0], nullptr, nullptr, av.data(), environ) != 0)
    return cfg_fail("mxa_config_compile: cannot start " + argv[0]);
  int status = 0;
  if (waitpid(pid, &status, 0) < 0 || !WIFEXITED(status) || WEXITSTATUS(status) != 0) {
    unlink(tmp.c_str());
    std::string cmd;
    for (auto& x : argv) cmd += x + " ";
    return cfg_fail("mxa_config_compile: the compile failed: " + cmd);
  }
  if (rename(tmp.c_str(), so.c_str()) != 0) return cfg_fail("mxa_config_compile: cannot place " + so);
  return MXA_OK;
}

typedef int (*mxa_custom_entry_fn)(MxaEntry*, MxaParams*, size_t*, mxa_config*, const char**);

int mxa_create_config(const mxa_config* cfg, int32_t n_envs, const uint32_t* seeds, int32_t device, int32_t trace_cap,
                      const char* cache_dir, mxa_handle** out) {
  if (!out || n_envs <= 0 || !seeds || trace_cap < 0 || !cfg) return cfg_fail("mxa_create_config: bad arguments");
  if (const char* why = mxa_cfg::custom_check(*cfg)) return cfg_fail(std::string("mxa_create_config: ") + why);
  const std::string key = cfg_key(*cfg), so = cfg_lib(cache_dir, key);
  static std::mutex mu;
  static std::map<std::string, void*> loaded;  // specialisations stay loaded: their kernels are registered
  void* dl = nullptr;
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = loaded.find(so);
    if (it != loaded.end()) {
      dl = it->second;
    } else {
      struct stat st{};
      if (stat(so.c_str(), &st) != 0) {
        g_cfg_err = "mxa_create_config: not compiled (mxa_config_compile first): " + so;
        return MXA_ERANGE;
      }
      dl = dlopen(so.c_str(), RTLD_NOW | RTLD_LOCAL);
      if (!dl) return cfg_fail(std::string("mxa_create_config: dlopen: ") + dlerror());
      loaded[so] = dl;
    }
  }
  auto fn = (mxa_custom_entry_fn)dlsym(dl, "mxa_custom_entry");
  if (!fn) return cfg_fail("mxa_create_config: " + so + " is not a specialisation");
  MxaEntry e{};
  MxaParams P{};
  size_t lds = 0;
  mxa_config c{};
  const char* bid = nullptr;
  if (fn(&e, &P, &lds, &c, &bid) != (int)sizeof(MxaParams) || !bid || strcmp(bid, MXA_BUILD_ID) != 0)
    return cfg_fail("mxa_create_config: " + so + " was built by another libmxa");
  c.date_ns = cfg->date_ns;
  if (memcmp(&c, cfg, sizeof c) != 0) return cfg_fail("mxa_create_config: " + so + " holds another composition");
  mxa_handle* h = new mxa_handle();
  h->build = e.build;
  h->run = e.run;
  h->run_log = e.run_log;
  h->run_fast = e.run_fast;
  h->stop = e.stop;
  h->stop_log = e.stop_log;
  h->step = e.step;
  h->step_fast = e.step_fast;
  h->gym = false;
  h->occ = e.occ;
  h->lds = lds;
  h->P = P;
  h->P.n_envs = n_envs;
  h->P.L.trace_cap = trace_cap;
  h->P.L.env_stride = mxa_cfg::align_up(P.L.off_trace + (uint64_t)trace_cap * MXA_TRACE_WORDS * 8, 256);
  return create_common(h, n_envs, seeds, device, out);
}

int mxa_config_info(int32_t config, int64_t* out8) {
  if (!out8 || config < 0 || config >= MXA_N_CONFIGS) return MXA_EINVAL;
  const MxaParams P = mxa_cfg::params(config);
  const mxa_cfg::Shape S = mxa_cfg::shape(config);
  out8[0] = P.n_agents;
  out8[1] = P.ex_log_orders;
  out8[2] = (int64_t)S.sq * 64;
  out8[3] = (int64_t)S.so * 64;
  out8[4] = P.mkt_open;
  out8[5] = P.mkt_close;
  out8[6] = P.start;
  out8[7] = P.stop;
  return MXA_OK;
}

static int create_common(mxa_handle* h, int32_t n_envs, const uint32_t* seeds, int32_t device, mxa_handle** out) {
  h->device = device;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    *out = h;
    return hip_fail(h, e, "hipSetDevice");
  }
  *out = h;
  HIPCHK(h, hipStreamCreateWithFlags(&h->own, hipStreamNonBlocking));
  h->stream = h->own;
  HIPCHK(h, hipEventCreate(&h->ev0));
  HIPCHK(h, hipEventCreate(&h->ev1));
  size_t bytes = (size_t)h->P.L.env_stride * n_envs;
  HIPCHK(h, hipMalloc(&h->d_env, bytes));
  HIPCHK(h, hipMalloc(&h->d_seeds, sizeof(uint32_t) * n_envs));
  HIPCHK(h, hipMalloc(&h->d_mask, n_envs));
  HIPCHK(h, hipMalloc(&h->d_count, sizeof(int)));
  HIPCHK(h, hipMalloc(&h->d_list, sizeof(int32_t) * (size_t)std::max(1, h->P.n_envs)));
  HIPCHK(h, hipMemsetAsync(h->d_env, 0, bytes, h->stream));
  HIPCHK(h, hipMemcpyAsync(h->d_seeds, seeds, sizeof(uint32_t) * n_envs, hipMemcpyHostToDevice, h->stream));
  if (h->replay) {
    HIPCHK(h, hipMalloc(&h->d_tape, h->tape_blob.size()));
    HIPCHK(h, hipMemcpyAsync(h->d_tape, h->tape_blob.data(), h->tape_blob.size(), hipMemcpyHostToDevice, h->stream));
    h->ctx.t = (const int64_t*)(h->d_tape + h->tb_t);
    h->ctx.oid = (const int32_t*)(h->d_tape + h->tb_oid);
    h->ctx.dense = (const int32_t*)(h->d_tape + h->tb_dense);
    h->ctx.price = (const int32_t*)(h->d_tape + h->tb_price);
    h->ctx.size = (const int32_t*)(h->d_tape + h->tb_size);
    h->ctx.buy = (const int8_t*)(h->d_tape + h->tb_buy);
    h->ctx.tm = (const int64_t*)(h->d_tape + h->tb_tm);
    h->ctx.tm0 = (const int32_t*)(h->d_tape + h->tb_tm0);
    h->ctx.uid = (const int32_t*)(h->d_tape + h->tb_uid);
    h->ctx.ufirst = (const int32_t*)(h->d_tape + h->tb_ufirst);
  }
  if (h->ext) {
    HIPCHK(h, hipMalloc(&h->d_tape, h->tape_blob.size()));
    HIPCHK(h, hipMemcpyAsync(h->d_tape, h->tape_blob.data(), h->tape_blob.size(), hipMemcpyHostToDevice, h->stream));
    h->ctx.fs_t = (const int64_t*)(h->d_tape + h->tb_fs_t);
    h->ctx.fs_v = (const double*)(h->d_tape + h->tb_fs_v);
  }
  if (!h->mm.empty()) {
    HIPCHK(h, hipMalloc(&h->d_mmp, sizeof(MmParams) * n_envs));
    HIPCHK(h, hipMemcpyAsync(h->d_mmp, h->mm.data(), sizeof(MmParams) * n_envs, hipMemcpyHostToDevice, h->stream));
    h->ctx.mmp = h->d_mmp;
  }
  if (h->gym || h->ext || h->replay || !h->mm.empty()) {
    HIPCHK(h, hipMalloc(&h->d_ctx, sizeof(RpCtx)));
    HIPCHK(h, hipMemcpyAsync(h->d_ctx, &h->ctx, sizeof(RpCtx), hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipMalloc(&h->d_act, sizeof(double) * 3 * n_envs));
    HIPCHK(h, hipMalloc(&h->d_obs, sizeof(double) * 9 * n_envs));
    HIPCHK(h, hipMalloc(&h->d_flags, sizeof(int32_t) * n_envs));
  }
  if (h->gym || h->ext || h->replay || !h->mm.empty()) HIPCHK(h, hipStreamSynchronize(h->stream));
  const int rc = mxa_reset(h, nullptr);  // a fresh process: ids from 0
  h->persist_ids = h->gym;               // later resets continue the process (Order.py:8-9)
  return rc;
}

// ABIDESEnv on a LOBSTER tape (agent_config.py / ABIDESEnv.py), or config/marketreplay.py under
// Kernel.runner (cfg MXA_CFG_MARKETREPLAY_RUNNER); see include/mxa.h
static int create_replay(int cfg, const int64_t* t, const int64_t* oid, const int64_t* price, const int64_t* size,
                         const int8_t* buy, int32_t n_rec, int32_t n_envs, int32_t device, int32_t trace_cap,
                         mxa_handle** out, int32_t twap_trade = 0);
int mxa_create_replay(const int64_t* t, const int64_t* oid, const int64_t* price, const int64_t* size,
                      const int8_t* buy, int32_t n_rec, int32_t n_envs, int32_t device, int32_t trace_cap,
                      mxa_handle** out) {
  return create_replay(MXA_CFG_MARKETREPLAY, t, oid, price, size, buy, n_rec, n_envs, device, trace_cap, out);
}
int mxa_create_replay_runner(const int64_t* t, const int64_t* oid, const int64_t* price, const int64_t* size,
                             const int8_t* buy, int32_t n_rec, int32_t n_envs, int32_t device, int32_t trace_cap,
                             mxa_handle** out) {
  return create_replay(MXA_CFG_MARKETREPLAY_RUNNER, t, oid, price, size, buy, n_rec, n_envs, device, trace_cap, out);
}
int mxa_create_replay_twap(const int64_t* t, const int64_t* oid, const int64_t* price, const int64_t* size,
                           const int8_t* buy, int32_t n_rec, int32_t trade, int32_t n_envs, int32_t device,
                           int32_t trace_cap, mxa_handle** out) {
  return create_replay(MXA_CFG_MARKETREPLAY_TWAP, t, oid, price, size, buy, n_rec, n_envs, device, trace_cap, out,
                       trade != 0);
}
static int create_replay(int cfg, const int64_t* t, const int64_t* oid, const int64_t* price, const int64_t* size,
                         const int8_t* buy, int32_t n_rec, int32_t n_envs, int32_t device, int32_t trace_cap,
                         mxa_handle** out, int32_t twap_trade) {
  if (!out || !t || !oid || !price || !size || !buy || n_rec <= 0 || n_envs <= 0 || trace_cap < 0) return MXA_EINVAL;
#ifdef MXA_NO_GYM
  return MXA_EINVAL;
#else
  int64_t pmin = INT64_MAX, pmax = INT64_MIN, min_id = INT64_MAX;
  int n_zero = 0;  // ORDER_ID 0 records: LimitOrder(order_id=0) takes an auto id (Order.py:26)
  for (int i = 0; i < n_rec; i++) {
    if ((i && t[i] < t[i - 1]) || oid[i] < 0 || oid[i] >= INT32_MAX || size[i] < 0 || size[i] >= INT32_MAX ||
        price[i] < 0 || price[i] >= (1 << 20))
      return MXA_EINVAL;  // unsorted tape or out-of-range fields
    pmin = std::min(pmin, price[i]);
    pmax = std::max(pmax, price[i]);
    if (oid[i] == 0) n_zero++;
    else min_id = std::min(min_id, oid[i]);
  }
  const MxaParams P0 = mxa_cfg::params(cfg);
  // auto ids (DummyRL's orders and the tape's ORDER_ID 0 records) count up from 0 in one
  // global sequence; Order.generateOrderId would skip explicit tape ids it met, which cannot
  // happen while every auto id stays below the smallest tape id
  const int64_t auto_cap = (int64_t)P0.rl_ids + n_zero;
  if (min_id <= auto_cap) return MXA_EINVAL;
  // Order._order_ids of the tape (for later episodes of a process): each explicit id with its
  // first SIZE > 0 record, sorted by id
  std::vector<std::pair<int32_t, int32_t>> uf;
  for (int i = 0; i < n_rec; i++)
    if (oid[i] != 0 && size[i] > 0) uf.push_back({(int32_t)oid[i], i});
  std::sort(uf.begin(), uf.end());
  uf.erase(std::unique(uf.begin(), uf.end(), [](const std::pair<int32_t, int32_t>& a, const std::pair<int32_t, int32_t>& b) {
             return a.first == b.first;
           }),
           uf.end());  // sorted by (id, record): the first of each id is kept
  mxa_handle* h = new mxa_handle();
  if (!bind(h, cfg)) {
    delete h;
    return MXA_EINVAL;
  }
  h->replay = true;
  h->P = P0;
  h->P.n_envs = n_envs;
  h->P.L.trace_cap = trace_cap;
  // dense order-id index in first-appearance order; distinct times and their first records
  std::vector<int32_t> dense(n_rec), tm0;
  std::vector<int64_t> tm;
  std::vector<std::pair<int64_t, int32_t>> ids;
  ids.reserve(n_rec);
  for (int i = 0; i < n_rec; i++)
    if (oid[i] != 0) ids.push_back({oid[i], i});
  std::sort(ids.begin(), ids.end());
  int n_ids = 0;
  for (size_t i = 0; i < ids.size(); i++) {
    if (i == 0 || ids[i].first != ids[i - 1].first) n_ids++;
    dense[ids[i].second] = n_ids - 1;
  }
  // ORDER_ID 0 records look up `orders.get(0)`: the order whose auto id is 0, which sits at
  // the first auto-id dense index
  for (int i = 0; i < n_rec; i++)
    if (oid[i] == 0) dense[i] = n_ids;
  for (int i = 0; i < n_rec; i++)
    if (i == 0 || t[i] != t[i - 1]) {
      tm.push_back(t[i]);
      tm0.push_back(i);
    }
  tm0.push_back(n_rec);
  const int ntm = (int)tm.size();
  const int C = n_rec + h->P.rl_ids;  // every placement could rest at once
  // auto-id dense range: the episode's auto ids, the explicit ids they may skip over in a later
  // episode (MXA_AUTO_SKIP), and one never-present index (orders.get(0) without an auto id 0)
  h->ctx.L = mxa_cfg::replay_layout(mxa_cfg::env_stride(cfg, trace_cap), (int)pmin, (int)(pmax - pmin + 1), C,
                                    n_ids, (int)auto_cap + MXA_AUTO_SKIP + 1, ntm, n_rec);
  h->ctx.nuid = (int32_t)uf.size();
  h->ctx.twap_trade = twap_trade;
  h->ctx.umin = uf.empty() ? INT32_MAX : uf[0].first;
  h->P.L.env_stride = h->ctx.L.end;
  // tape blob: t, oid, dense, price, size, buy, tm, tm0 (256-B aligned pieces)
  auto al = [](size_t x) { return (x + 255) / 256 * 256; };
  size_t off = 0;
  h->tb_t = off;
  off = al(off + 8ull * n_rec);
  h->tb_oid = off;
  off = al(off + 4ull * n_rec);
  h->tb_dense = off;
  off = al(off + 4ull * n_rec);
  h->tb_price = off;
  off = al(off + 4ull * n_rec);
  h->tb_size = off;
  off = al(off + 4ull * n_rec);
  h->tb_buy = off;
  off = al(off + n_rec);
  h->tb_tm = off;
  off = al(off + 8ull * ntm);
  h->tb_tm0 = off;
  off = al(off + 4ull * (ntm + 1));
  h->tb_uid = off;
  off = al(off + 4ull * uf.size() + 4);
  h->tb_ufirst = off;
  off = al(off + 4ull * uf.size() + 4);
  h->tape_blob.assign(off, 0);
  char* b = h->tape_blob.data();
  for (int i = 0; i < n_rec; i++) {
    ((int64_t*)(b + h->tb_t))[i] = t[i];
    ((int32_t*)(b + h->tb_oid))[i] = (int32_t)oid[i];
    ((int32_t*)(b + h->tb_dense))[i] = dense[i];
    ((int32_t*)(b + h->tb_price))[i] = (int32_t)price[i];
    ((int32_t*)(b + h->tb_size))[i] = (int32_t)size[i];
    ((int8_t*)(b + h->tb_buy))[i] = buy[i] ? 1 : 0;
  }
  memcpy(b + h->tb_tm, tm.data(), 8ull * ntm);
  memcpy(b + h->tb_tm0, tm0.data(), 4ull * (ntm + 1));
  for (size_t i = 0; i < uf.size(); i++) {
    ((int32_t*)(b + h->tb_uid))[i] = uf[i].first;
    ((int32_t*)(b + h->tb_ufirst))[i] = uf[i].second;
  }
  std::vector<uint32_t> seeds(n_envs, 0u);  // nothing in this composition draws
  return create_common(h, n_envs, seeds.data(), device, out);
#endif
}

// ABIDESEnv.step for every env: actions [n][3] -> obs [n][9], flags [n] (all host arrays)
int mxa_step(mxa_handle* h, const double* actions, double* obs, int32_t* flags) {
  if (!h || !h->gym || !actions || !obs || !flags) return MXA_EINVAL;
#ifdef MXA_NO_GYM
  return MXA_EINVAL;
#else
  HIPCHK(h, hipSetDevice(h->device));
  int n = h->P.n_envs;
  HIPCHK(h, hipMemcpyAsync(h->d_act, actions, sizeof(double) * 3 * n, hipMemcpyHostToDevice, h->stream));
  int rc = mxa_step_device(h, h->d_act, h->d_obs, h->d_flags);
  if (rc) return rc;
  HIPCHK(h, hipMemcpyAsync(obs, h->d_obs, sizeof(double) * 9 * n, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipMemcpyAsync(flags, h->d_flags, sizeof(int32_t) * n, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  float ms = 0;
  HIPCHK(h, hipEventElapsedTime(&ms, h->ev0, h->ev1));
  h->last_ms = ms;
  return MXA_OK;
#endif
}

// k consecutive steps in one launch, device arrays: actions [k][n][3] -> obs [k][n][9], flags [k][n]
int mxa_step_many(mxa_handle* h, int32_t k, const double* d_actions, double* d_obs, int32_t* d_flags) {
  if (!h || !h->gym || k <= 0 || !d_actions || !d_obs || !d_flags) return MXA_EINVAL;
#ifdef MXA_NO_GYM
  return MXA_EINVAL;
#else
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipEventRecord(h->ev0, h->stream));
  (h->tcap_arg() < 0 && h->step_many_fast ? h->step_many_fast : h->step_many)(
      dim3(h->P.n_envs), dim3(64), h->lds, h->stream, h->d_env, h->P.L.env_stride, h->P.n_envs, h->tcap_arg(),
      (int64_t)1 << 40, (const RpCtx*)h->d_ctx, d_actions, d_obs, d_flags, k);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipEventRecord(h->ev1, h->stream));
  return MXA_OK;
#endif
}

// the same with device arrays (e.g. torch tensors), asynchronous on the handle's stream
int mxa_step_device(mxa_handle* h, const double* d_actions, double* d_obs, int32_t* d_flags) {
  if (!h || !h->gym) return MXA_EINVAL;
#ifdef MXA_NO_GYM
  return MXA_EINVAL;
#else
  HIPCHK(h, hipEventRecord(h->ev0, h->stream));
  (h->tcap_arg() < 0 && h->step_fast ? h->step_fast : h->step)(dim3(h->P.n_envs), dim3(64), h->lds, h->stream, h->d_env,
                                                                 h->P.L.env_stride, h->P.n_envs, h->tcap_arg(),
          (int64_t)1 << 40, (const RpCtx*)h->d_ctx, d_actions, d_obs, d_flags);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipEventRecord(h->ev1, h->stream));
  return MXA_OK;
#endif
}

int mxa_reset(mxa_handle* h, const uint8_t* mask) {
  if (!h) return MXA_EINVAL;
  HIPCHK(h, hipSetDevice(h->device));
  const uint8_t* dm = nullptr;
  if (h->persist_ids) {  // mask value 2: rebuild the env, keep its order-id counters
    std::vector<uint8_t> m2(h->P.n_envs);
    for (int i = 0; i < h->P.n_envs; i++) m2[i] = (!mask || mask[i]) ? 2 : 0;
    HIPCHK(h, hipMemcpyAsync(h->d_mask, m2.data(), h->P.n_envs, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));  // m2 is a host temporary
    dm = h->d_mask;
  } else if (mask) {
    std::vector<uint8_t> m1(h->P.n_envs);
    for (int i = 0; i < h->P.n_envs; i++) m1[i] = mask[i] ? 1 : 0;
    HIPCHK(h, hipMemcpyAsync(h->d_mask, m1.data(), h->P.n_envs, hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    dm = h->d_mask;
  }
  h->build(dim3(h->P.n_envs), dim3(64), h->lds, h->stream, h->d_env, h->P.L.env_stride, h->P.n_envs, h->d_seeds, dm,
           h->d_ctx);
  HIPCHK(h, hipGetLastError());
  if (!mask) h->started = false;
  if (h->exlog) {  // the build cleared the header: the switch outlives resets
    const int n = h->P.n_envs;
    hipLaunchKernelGGL(mxa_set_exlog_kernel, dim3((n + 255) / 256), dim3(256), 0, h->stream, h->d_env,
                       h->P.L.env_stride, n, h->exlog);
    HIPCHK(h, hipGetLastError());
  }
  if (h->t_stop > 0) {  // the build cleared the header: the override outlives resets
    const int n = h->P.n_envs;
    hipLaunchKernelGGL(mxa_set_stop_kernel, dim3((n + 255) / 256), dim3(256), 0, h->stream, h->d_env,
                       h->P.L.env_stride, n, h->t_stop);
    HIPCHK(h, hipGetLastError());
  }
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return MXA_OK;
}

int mxa_set_stop_time(mxa_handle* h, int64_t t_stop_ns) {
  if (!h || h->gym) return MXA_EINVAL;  // GymKernel handles: ABIDESEnv's own stop (ABIDESEnv.py:42-46)
  HIPCHK(h, hipSetDevice(h->device));
  h->t_stop = t_stop_ns > 0 ? t_stop_ns : 0;
  const int n = h->P.n_envs;
  hipLaunchKernelGGL(mxa_set_stop_kernel, dim3((n + 255) / 256), dim3(256), 0, h->stream, h->d_env, h->P.L.env_stride,
                     n, h->t_stop);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return MXA_OK;
}

int mxa_run_until(mxa_handle* h, int64_t t_stop_ns, int64_t* events_out) {
  if (!h || h->gym) return MXA_EINVAL;
  int rc = mxa_set_stop_time(h, t_stop_ns);
  if (rc != MXA_OK) return rc;
  if ((rc = mxa_run(h, (int64_t)1 << 20, 0, nullptr)) != MXA_OK) return rc;
  if (events_out) {
    const int n = h->P.n_envs;
    std::vector<mxa_env_summary> s(n);
    if ((rc = mxa_read_summary(h, s.data())) != MXA_OK) return rc;
    for (int i = 0; i < n; i++) events_out[i] = s[i].events;
  }
  return MXA_OK;
}

int mxa_set_id_persistence(mxa_handle* h, int32_t on) {
  if (!h || (on && !h->gym)) return MXA_EINVAL;
  h->persist_ids = on != 0;
  return MXA_OK;
}

int mxa_launch(mxa_handle* h, int64_t max_pops) {
  if (!h || h->gym) return MXA_EINVAL;  // GymKernel handles advance by mxa_step
  HIPCHK(h, hipSetDevice(h->device));  // the caller's current device may differ
  h->started = true;
  h->run_kernel()(dim3(h->P.n_envs), dim3(64), h->lds, h->stream, h->d_env, h->P.L.env_stride, h->P.n_envs, h->tcap_arg(), max_pops,
         h->d_ctx, h->d_blog, h->blog_cap, nullptr);
  HIPCHK(h, hipGetLastError());
  return MXA_OK;
}

int mxa_sync(mxa_handle* h) {
  if (!h) return MXA_EINVAL;
  HIPCHK(h, hipSetDevice(h->device));  // the caller's current device may differ
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return MXA_OK;
}

int mxa_run(mxa_handle* h, int64_t chunk, int32_t max_launches, int32_t* launches_out) {
  if (!h || chunk <= 0 || h->gym) return MXA_EINVAL;
  HIPCHK(h, hipSetDevice(h->device));
  int launches = 0;
  float total = 0;
  h->started = true;
  const int n = h->P.n_envs;
  // the envs still running (an earlier mxa_run / mxa_launch may have finished some)
  auto compact = [&](int& running) -> int {
    hipLaunchKernelGGL(mxa_compact_kernel, dim3(1), dim3(1024), 0, h->stream, h->d_env, h->P.L.env_stride, n,
                       h->d_list, h->d_count);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipMemcpyAsync(&running, h->d_count, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (running < 0 || running > n) {
      h->err = "mxa_run: running-env count out of range";
      return MXA_EHIP;
    }
    return MXA_OK;
  };
  int running = 0, rc;
  if ((rc = compact(running)) != MXA_OK) return rc;
  int64_t pops = h->first_chunk > 0 ? std::min(chunk, h->first_chunk) : chunk;
  while (running > 0) {
    if (max_launches > 0 && launches >= max_launches) break;
    // one wave per running env: every env (no list) while none has finished
    HIPCHK(h, hipEventRecord(h->ev0, h->stream));
    h->run_kernel()(dim3(running), dim3(64), h->lds, h->stream, h->d_env, h->P.L.env_stride, n, h->tcap_arg(), pops,
                    h->d_ctx, h->d_blog, h->blog_cap, running == n ? nullptr : h->d_list);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipEventRecord(h->ev1, h->stream));
    launches++;
    if ((rc = compact(running)) != MXA_OK) return rc;
    float ms = 0;
    HIPCHK(h, hipEventElapsedTime(&ms, h->ev0, h->ev1));
    total += ms;
    pops = chunk;  // mxa_set_launch_schedule: the first launch only is first_chunk
  }
  h->last_ms = total;
  if (launches_out) *launches_out = launches;
  return MXA_OK;
}

int mxa_set_launch_schedule(mxa_handle* h, int64_t first_chunk) {
  if (!h || first_chunk < 0) return MXA_EINVAL;
  h->first_chunk = first_chunk;
  return MXA_OK;
}

// book-update log (OrderBook.book_log / the exchange's BEST_BID, BEST_ASK, LAST_TRADE events):
// `cap` records per env in one device buffer; every env's record count restarts at 0
int mxa_set_book_log(mxa_handle* h, int32_t cap) {
  // Kernel.runner handles, the replay's (config/marketreplay.py) included; not GymKernel handles
  if (!h || h->gym || !h->run_log || cap < 0) return MXA_EINVAL;
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (h->d_blog) HIPCHK(h, hipFree(h->d_blog));
  h->d_blog = nullptr;
  h->blog_cap = 0;
  if (cap > 0) {
    HIPCHK(h, hipMalloc(&h->d_blog, sizeof(BlRec) * (size_t)cap * h->P.n_envs));
    h->blog_cap = cap;
  }
  HIPCHK(h, hipMemset2DAsync(h->d_env + offsetof(EnvHdr, blog_n), h->P.L.env_stride, 0, sizeof(int32_t), h->P.n_envs,
                             h->stream));
  HIPCHK(h, hipMemset2DAsync(h->d_env + offsetof(EnvHdr, blog_fin), h->P.L.env_stride, 0, sizeof(int32_t),
                             h->P.n_envs, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return MXA_OK;
}

// the exchange's own log (ExchangeAgent.log -> EXCHANGE_AGENT.bz2) in the book-update log: the
// log-variant kernels write its records (mxa_layout.h BL_EV_*) while EnvHdr::exlog is set
int mxa_set_exchange_log(mxa_handle* h, int32_t on) {
  if (!h || h->gym || !h->run_log || on < 0 || on > 1) return MXA_EINVAL;
  if (on && !h->d_blog) return MXA_EINVAL;  // it rides in the book-update log: mxa_set_book_log first
  if (h->started && on != h->exlog) {
    // placements logged before the switch would be missing from the log (its order rows name
    // them), and a log switched off mid-run ends without its tail: set it before the run
    h->err = "mxa_set_exchange_log: set it before the first launch (or after a whole-handle mxa_reset)";
    return MXA_EINVAL;
  }
  HIPCHK(h, hipSetDevice(h->device));
  h->exlog = on;
  const int n = h->P.n_envs;
  hipLaunchKernelGGL(mxa_set_exlog_kernel, dim3((n + 255) / 256), dim3(256), 0, h->stream, h->d_env, h->P.L.env_stride,
                     n, on);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return MXA_OK;
}

int mxa_read_book_log(mxa_handle* h, int32_t env, mxa_book_rec* out, int64_t cap, int64_t* n) {
  if (!h || env < 0 || env >= h->P.n_envs || !n || cap < 0 || (cap > 0 && !out)) return MXA_EINVAL;
  static_assert(sizeof(mxa_book_rec) == sizeof(BlRec) && offsetof(mxa_book_rec, qty) == offsetof(BlRec, qty),
                "mxa_book_rec mirrors BlRec");
  static_assert((int)MXA_BL_FUNDAMENTAL == (int)BL_FUNDAMENTAL, "f_log record tag");
  static_assert((int)MXA_BL_EV_RX == (int)BL_EV_RX && (int)MXA_BL_EV_NT == (int)BL_EV_NT &&
                    (int)MXA_BL_EV_PLACE == (int)BL_EV_PLACE && (int)MXA_BL_EV_END == (int)BL_EV_END,
                "exchange-log record codes");
  HIPCHK(h, hipSetDevice(h->device));
  EnvHdr hd;
  HIPCHK(h, hipMemcpyAsync(&hd, h->d_env + (size_t)env * h->P.L.env_stride, sizeof(hd), hipMemcpyDeviceToHost,
                           h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  // after a kernelStopping pass: its oracle observations follow the run's records
  int64_t cnt = h->d_blog ? (hd.blog_fin > hd.blog_n ? hd.blog_fin : hd.blog_n) : 0;
  *n = cnt;  // beyond the capacity: the log overflowed (the first `blog_cap` records are kept)
  if (cnt > h->blog_cap) cnt = h->blog_cap;
  const int64_t m = cnt < cap ? cnt : cap;
  if (m > 0)
    HIPCHK(h, hipMemcpyAsync(out, h->d_blog + (size_t)env * h->blog_cap, sizeof(BlRec) * m, hipMemcpyDeviceToHost,
                             h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return MXA_OK;
}

int mxa_finalize(mxa_handle* h) {
  if (!h || h->gym || !h->stop) return MXA_EINVAL;
  HIPCHK(h, hipSetDevice(h->device));
  const size_t rows = (size_t)h->P.n_envs * h->P.n_agents;
  if (!h->d_final) HIPCHK(h, hipMalloc(&h->d_final, rows * sizeof(mxa_agent_final)));
  (h->d_blog ? h->stop_log : h->stop)(dim3(h->P.n_envs), dim3(64), h->lds, h->stream, h->d_env, h->P.L.env_stride, h->P.n_envs, h->d_final,
          h->d_blog, h->blog_cap, h->d_ctx);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return MXA_OK;
}

int mxa_read_final(mxa_handle* h, int32_t env, mxa_agent_final* out, int32_t cap) {
  if (!h || !h->d_final || env < 0 || env >= h->P.n_envs || !out || cap < h->P.n_agents) return MXA_EINVAL;
  HIPCHK(h, hipSetDevice(h->device));  // the caller's current device may differ
  HIPCHK(h, hipMemcpyAsync(out, h->d_final + (size_t)env * h->P.n_agents, sizeof(mxa_agent_final) * h->P.n_agents,
                           hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return h->P.n_agents;
}

int mxa_read_summary(mxa_handle* h, mxa_env_summary* out) {
  if (!h || !out) return MXA_EINVAL;
  HIPCHK(h, hipSetDevice(h->device));  // the caller's current device may differ
  int n = h->P.n_envs;
  std::vector<EnvHdr> hd(n);
  HIPCHK(h, hipMemcpy2DAsync(hd.data(), sizeof(EnvHdr), h->d_env, h->P.L.env_stride, sizeof(EnvHdr), n,
                             hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  for (int i = 0; i < n; i++) {
    out[i].status = hd[i].status;
    out[i].err = hd[i].err;
    out[i].events = hd[i].pops;
    out[i].hash = hd[i].hash;
    out[i].current_time = hd[i].cur;
    out[i].order_counter = hd[i].order_counter;
    out[i].last_trade = hd[i].last_trade;
    out[i].max_queue = hd[i].max_q;
    out[i].max_book = hd[i].max_book;
  }
  return MXA_OK;
}

int mxa_read_agents(mxa_handle* h, int32_t env, mxa_agent_state* out, int32_t cap) {
  if (!h || env < 0 || env >= h->P.n_envs) return MXA_ERANGE;
  HIPCHK(h, hipSetDevice(h->device));  // the caller's current device may differ
  int n = std::min(cap, h->P.n_agents);
  std::vector<uint32_t> rec((size_t)h->P.n_agents * 128);
  HIPCHK(h, hipMemcpy(rec.data(), h->d_env + (size_t)env * h->P.L.env_stride + h->P.L.off_ag, rec.size() * 4,
                      hipMemcpyDeviceToHost));
  for (int a = 0; a < n; a++) {
    const uint32_t* r = &rec[(size_t)a * 128];
    auto g64 = [&](int f) { return (int64_t)(((uint64_t)r[f + 1] << 32) | r[f]); };
    out[a].cash = g64(AF_CASH);
    out[a].shares = g64(AF_SHARES);
    out[a].n_open = (int32_t)r[AF_NORD];
    out[a].last_trade = g64(AF_LAST_TRADE);
    out[a].type = (int32_t)r[AF_TYPE];
    out[a].flags = (int32_t)r[AF_FLAGS];
    out[a].starting_cash = g64(AF_START_CASH);
    if (h->replay && out[a].type == AG_REPLAY) {  // MarketReplayAgent.orders lives in the dense table
      std::vector<RpOrder> mo(h->ctx.L.D);
      HIPCHK(h, hipMemcpy(mo.data(), h->d_env + (size_t)env * h->P.L.env_stride + h->ctx.L.off_mro,
                          sizeof(RpOrder) * mo.size(), hipMemcpyDeviceToHost));
      int64_t c = 0;
      for (auto& o : mo) c += o.present ? 1 : 0;
      out[a].n_open = c;
    }
  }
  return n;
}

int mxa_read_book(mxa_handle* h, int32_t env, int32_t side, int64_t* out4, int32_t cap) {
  if (!h || env < 0 || env >= h->P.n_envs) return MXA_ERANGE;
  HIPCHK(h, hipSetDevice(h->device));  // the caller's current device may differ
  if (h->replay) {  // price ladder: levels best-first, FIFO lists
    const RpLayout& L = h->ctx.L;
    char* e = h->d_env + (size_t)env * h->P.L.env_stride;
    std::vector<int32_t> cnt(L.P), head(L.P);
    std::vector<RpEntry> pool(L.C);
    HIPCHK(h, hipMemcpy(cnt.data(), e + L.off_lvc + 4ull * side * L.P, 4ull * L.P, hipMemcpyDeviceToHost));
    HIPCHK(h, hipMemcpy(head.data(), e + L.off_lvh + 4ull * side * L.P, 4ull * L.P, hipMemcpyDeviceToHost));
    HIPCHK(h, hipMemcpy(pool.data(), e + L.off_pool, sizeof(RpEntry) * L.C, hipMemcpyDeviceToHost));
    int n = 0;
    for (int k = 0; k < L.P; k++) {
      int x = side == 0 ? L.P - 1 - k : k;
      if (!cnt[x]) continue;
      for (int q = head[x]; q >= 0; q = pool[q].next) {
        if (n < cap) {
          out4[4 * n + 0] = pool[q].oid;
          out4[4 * n + 1] = pool[q].meta >> 1;
          out4[4 * n + 2] = pool[q].qty;
          out4[4 * n + 3] = pool[q].price;
        }
        n++;
      }
    }
    return n;
  }
  int oc = h->P.L.ocap;
  std::vector<SavedOrder> so(oc);
  HIPCHK(h, hipMemcpy(so.data(), h->d_env + (size_t)env * h->P.L.env_stride + h->P.L.off_book,
                      sizeof(SavedOrder) * oc, hipMemcpyDeviceToHost));
  std::vector<SavedOrder> v;
  int buy = side == 0 ? 1 : 0;
  for (auto& o : so)
    if (o.meta >= 0 && (o.meta & 1) == buy) v.push_back(o);
  std::sort(v.begin(), v.end(), [&](const SavedOrder& a, const SavedOrder& b) {
    if (a.price != b.price) return buy ? a.price > b.price : a.price < b.price;
    return a.arrival < b.arrival;
  });
  for (int n = 0; n < (int)v.size() && n < cap; n++) {
    out4[4 * n + 0] = v[n].oid;
    out4[4 * n + 1] = v[n].meta >> 1;
    out4[4 * n + 2] = v[n].qty;
    out4[4 * n + 3] = v[n].price;
  }
  return (int)v.size();  // total on the side; min(total, cap) written
}

int mxa_read_trace(mxa_handle* h, int32_t env, int64_t* out, int64_t cap, int64_t* nout) {
  if (!h || env < 0 || env >= h->P.n_envs) return MXA_ERANGE;
  HIPCHK(h, hipSetDevice(h->device));  // the caller's current device may differ
  EnvHdr hd;
  char* e = h->d_env + (size_t)env * h->P.L.env_stride;
  HIPCHK(h, hipMemcpy(&hd, e, sizeof hd, hipMemcpyDeviceToHost));
  int64_t n = std::min<int64_t>(std::min<int64_t>(hd.trace_len, h->P.L.trace_cap), cap);
  if (n > 0) HIPCHK(h, hipMemcpy(out, e + h->P.L.off_trace, (size_t)n * 80, hipMemcpyDeviceToHost));
  if (nout) *nout = n;
  return MXA_OK;
}

int mxa_set_seeds(mxa_handle* h, const uint32_t* seeds) {
  if (!h || !seeds) return MXA_EINVAL;
  HIPCHK(h, hipSetDevice(h->device));  // the caller's current device may differ
  HIPCHK(h, hipMemcpyAsync(h->d_seeds, seeds, sizeof(uint32_t) * h->P.n_envs, hipMemcpyHostToDevice, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return MXA_OK;
}

int mxa_write_results(mxa_handle* h, void* device_out) {
  if (!h || !device_out) return MXA_EINVAL;
  HIPCHK(h, hipSetDevice(h->device));  // the caller's current device may differ
  int n = h->P.n_envs;
  hipLaunchKernelGGL(mxa_results_kernel, dim3((n + 255) / 256), dim3(256), 0, h->stream, h->d_env, h->P.L.env_stride,
                     n, (int64_t*)device_out);
  HIPCHK(h, hipGetLastError());
  return MXA_OK;
}

int mxa_write_records(mxa_handle* h, void* device_out) {
  if (!h || !device_out) return MXA_EINVAL;
  HIPCHK(h, hipSetDevice(h->device));
  int n = h->P.n_envs;
  // GymKernel handles: the execution agent; Kernel.runner handles: every trading agent
  const int a0 = h->gym ? h->P.first_rl : 1, a1 = h->gym ? h->P.first_rl + 1 : h->P.n_agents;
  hipLaunchKernelGGL(mxa_records_kernel, dim3(n), dim3(64), 0, h->stream, h->d_env, h->P.L.env_stride, n, h->d_seeds,
                     h->P.L.off_ag, a0, a1, (int64_t*)device_out);
  HIPCHK(h, hipGetLastError());
  return MXA_OK;
}

int mxa_read_counters(mxa_handle* h, int64_t* out) {
  if (!h || !out) return MXA_EINVAL;
  HIPCHK(h, hipSetDevice(h->device));
  const int n = h->P.n_envs;
  int64_t* d = nullptr;
  HIPCHK(h, hipMallocAsync((void**)&d, sizeof(int64_t) * MXA_COUNTER_WORDS * n, h->stream));
  hipLaunchKernelGGL(mxa_counters_kernel, dim3(n), dim3(64), 0, h->stream, h->d_env, h->P.L.env_stride, n, h->P.L.off_ag,
                     h->P.n_agents, d);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipMemcpyAsync(out, d, sizeof(int64_t) * MXA_COUNTER_WORDS * n, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipFreeAsync(d, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return MXA_OK;
}

int mxa_set_parity_hash(mxa_handle* h, int32_t enabled) {
  if (!h) return MXA_EINVAL;
  h->parity_hash = enabled != 0;
  return MXA_OK;
}

int mxa_write_rl_state(mxa_handle* h, double* device_out) {
  if (!h || !device_out || !h->gym || h->P.n_rl != 1) return MXA_EINVAL;
  int n = h->P.n_envs;
  hipLaunchKernelGGL(mxa_rl_state_kernel, dim3((n + 255) / 256), dim3(256), 0, h->stream, h->d_env, h->P.L.env_stride,
                     n, (uint32_t)(h->P.L.off_ag + 512u * (uint32_t)h->P.first_rl), h->ctx.L.off_rh, h->ctx.L.off_ring,
                     device_out);
  HIPCHK(h, hipGetLastError());
  return MXA_OK;
}

int mxa_read_raw(mxa_handle* h, int32_t env, int64_t offset, int64_t bytes, void* out) {
  if (!h || env < 0 || env >= h->P.n_envs || offset < 0 || bytes < 0 || offset + bytes > (int64_t)h->P.L.env_stride)
    return MXA_ERANGE;
  HIPCHK(h, hipSetDevice(h->device));  // the caller's current device may differ
  HIPCHK(h, hipStreamSynchronize(h->stream));
  HIPCHK(h, hipMemcpy(out, h->d_env + (size_t)env * h->P.L.env_stride + offset, bytes, hipMemcpyDeviceToHost));
  return MXA_OK;
}

int mxa_layout(const mxa_handle* h, int64_t* o) {
  if (!h || !o) return MXA_EINVAL;
  const Layout& L = h->P.L;
  o[0] = L.off_ag; o[1] = L.off_open; o[2] = L.off_rng; o[3] = L.off_lat;
  o[4] = L.off_q; o[5] = L.off_book; o[6] = L.off_tx; o[7] = L.off_trace;
  return MXA_OK;
}

int32_t mxa_n_agents(const mxa_handle* h) { return h ? h->P.n_agents : 0; }
int32_t mxa_n_envs(const mxa_handle* h) { return h ? h->P.n_envs : 0; }
int64_t mxa_env_bytes(const mxa_handle* h) { return h ? (int64_t)h->P.L.env_stride : 0; }
int mxa_set_stream(mxa_handle* h, void* s) {
  if (!h) return MXA_EINVAL;
  h->stream = s ? (hipStream_t)s : h->own;
  return MXA_OK;
}
double mxa_last_kernel_ms(const mxa_handle* h) { return h ? h->last_ms : 0; }
const char* mxa_last_error(const mxa_handle* h) { return h ? h->err.c_str() : g_cfg_err.c_str(); }

const char* mxa_build_id(void) { return MXA_BUILD_ID; }

void mxa_destroy(mxa_handle* h) {
  if (!h) return;
  hipSetDevice(h->device);
  if (h->d_env) hipFree(h->d_env);
  if (h->d_seeds) hipFree(h->d_seeds);
  if (h->d_mask) hipFree(h->d_mask);
  if (h->d_count) hipFree(h->d_count);
  if (h->d_list) hipFree(h->d_list);
  if (h->d_tape) hipFree(h->d_tape);
  if (h->d_ctx) hipFree(h->d_ctx);
  if (h->d_mmp) hipFree(h->d_mmp);
  if (h->d_act) hipFree(h->d_act);
  if (h->d_obs) hipFree(h->d_obs);
  if (h->d_flags) hipFree(h->d_flags);
  if (h->d_final) hipFree(h->d_final);
  if (h->d_blog) hipFree(h->d_blog);
  if (h->ev0) hipEventDestroy(h->ev0);
  if (h->ev1) hipEventDestroy(h->ev1);
  if (h->own) hipStreamDestroy(h->own);
  delete h;
}

int mxa_rng_probe(int32_t device, uint32_t seed, int32_t mode, double a, double b, int32_t n, double* out) {
  if (n <= 0 || !out) return MXA_EINVAL;
  if (hipSetDevice(device) != hipSuccess) return MXA_EHIP;
  double* d_out = nullptr;
  uint32_t* d_s = nullptr;
  if (mode < 0 || mode > 5) return MXA_EINVAL;
  if (hipMalloc(&d_out, sizeof(double) * n) != hipSuccess) return MXA_ENOMEM;
  if (hipMalloc(&d_s, MXA_RNG_WORDS * 4) != hipSuccess) return MXA_ENOMEM;
  hipLaunchKernelGGL(mxa_rng_probe_kernel, dim3(1), dim3(64), 0, 0, seed, mode, a, b, n, d_out, d_s);
  hipError_t e = hipMemcpy(out, d_out, sizeof(double) * n, hipMemcpyDeviceToHost);
  hipFree(d_out);
  hipFree(d_s);
  return e == hipSuccess ? MXA_OK : MXA_EHIP;
}

int mxa_math_probe(int32_t device, int32_t mode, const double* x, const double* y, double* out, int64_t n) {
  if (n <= 0 || !x || !out) return MXA_EINVAL;
  if (hipSetDevice(device) != hipSuccess) return MXA_EHIP;
  double *dx = nullptr, *dy = nullptr, *dout = nullptr;
  size_t bytes = sizeof(double) * n;
  if (hipMalloc(&dx, bytes) != hipSuccess || hipMalloc(&dy, bytes) != hipSuccess || hipMalloc(&dout, bytes) != hipSuccess)
    return MXA_ENOMEM;
  hipMemcpy(dx, x, bytes, hipMemcpyHostToDevice);
  hipMemcpy(dy, y ? y : x, bytes, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(mxa_math_probe_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, mode, dx, dy, dout, n);
  hipError_t e = hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost);
  hipFree(dx);
  hipFree(dy);
  hipFree(dout);
  return e == hipSuccess ? MXA_OK : MXA_EHIP;
}

}  // extern "C"
