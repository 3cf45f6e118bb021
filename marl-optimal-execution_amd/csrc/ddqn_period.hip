// ddqn_period.hip — the DDQN execution learner's per-period bookkeeping in one launch
// (libmxa_ddqn.so; mxabides/ddqn.py run_episode, fused path).
//
// After each ABIDESEnv.step of every env the learner loop (ddqlearning_execution_agent.py:275-299,
// 409-446) needs: the transition mask, the reward of the step's fills (compute_reward, BUY), the
// next discretised state, the per-env step count, the replay append in env order, the masked
// reward row and the next alive mask.  In PyTorch that is ~45 small elementwise kernels per period,
// each a few microseconds on a 4096-env batch; here it is one workgroup of 1024 lanes walking the
// envs in blocks of 1024 with one block-wide prefix count for the replay positions.  Every float
// operation is the PyTorch path's, in the same order (built with -ffp-contract=off), so the outputs
// are bitwise the same (tests/test_gpu_ddqn.py compares the two paths).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

// torch.bucketize(x, bd, right=True): searchsorted's upper bound, NaN sorting last
__device__ int64_t upper_bound(double x, const double* bd, int n) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    if (!(bd[mid] > x)) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// PyTorch divides a tensor by a Python scalar as a multiplication by the scalar's reciprocal
// (the true-division kernel's CPU-scalar case), which rounds differently from x / b
__device__ double div_scalar(double x, double b) { return x * (1.0 / b); }

// ExecutionTask.state: discretize([2 * rem_t / nh - 1, 2 * rem_q / q0 - 1])
__device__ void state_of(const double* o, const double* g0, int n0, const double* g1, int n1, double nh, double q0,
                         float* out) {
  const double tr = 2.0 * div_scalar(o[0], nh) - 1.0;
  const double qr = 2.0 * div_scalar(o[1], q0) - 1.0;
  out[0] = (float)upper_bound(tr, g0, n0);
  out[1] = (float)upper_bound(qr, g1, n1);
}

struct PeriodArgs {
  int n, obs_w, st_w, train;
  const double *obs, *st, *prev, *arrival;
  const int32_t* flags;
  const uint8_t* alive;   // before the step
  uint8_t* alive_next;    // ok & not done
  uint8_t* live;          // [1] any(alive): the learner's update mask for this period
  const float* s;         // [n][2] the state the action was chosen on
  const int64_t* a;       // [n]
  float* s2;              // [n][2] the state after the step (the next period's s)
  double* r_row;          // [n] where(ok, r, 0)
  int64_t* env_steps;     // [n] += alive
  const double *g0, *g1;
  int n0, n1;
  double nh, q0, rscale;  // rscale = 1e4 / q0, the Python float of task.reward
  float *ring_s, *ring_s2, *ring_r;
  int64_t* ring_a;
  int64_t cap;
  int64_t* n_dev;   // rows written so far (ReplayRing.n_dev)
  int64_t* stored;  // run_episode's stored count
};

__global__ __launch_bounds__(1024) void ddqn_period_kernel(PeriodArgs p) {
  __shared__ int wn[16];
  __shared__ int any_alive;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (threadIdx.x == 0) any_alive = 0;
  __syncthreads();
  const int64_t n_dev0 = *p.n_dev;
  int64_t done = 0;
  for (int i0 = 0; i0 < p.n; i0 += 1024) {
    const int i = i0 + (int)threadIdx.x;
    bool ok = false;
    double rr = 0.0;
    float s2v[2] = {0.f, 0.f};
    if (i < p.n) {
      const int32_t f = p.flags[i];
      const bool al = p.alive[i] != 0;
      if (al) any_alive = 1;  // any writer stores the same value
      ok = al && (f & 2) != 0 && (f & 4) == 0;
      const double* cur = p.st + (size_t)i * p.st_w;
      const double* pre = p.prev + (size_t)i * p.st_w;
      const double dq = cur[2] - pre[2];
      const double dcash = cur[0] - pre[0];
      rr = dq > 0 ? p.rscale * (2.0 * dq + dcash / p.arrival[i]) : 0.0;
      state_of(p.obs + (size_t)i * p.obs_w, p.g0, p.n0, p.g1, p.n1, p.nh, p.q0, s2v);
      p.s2[2 * i] = s2v[0];
      p.s2[2 * i + 1] = s2v[1];
      p.env_steps[i] += al ? 1 : 0;
      p.r_row[i] = ok ? rr : 0.0;
      p.alive_next[i] = ok && (f & 1) == 0;
    }
    // replay positions in env order: (n_dev + inclusive count - 1) % cap, as ReplayRing.add_device
    const uint64_t m = __ballot(p.train && ok);
    if (l == 0) wn[w] = __popcll(m);
    __syncthreads();
    int off = 0, tot = 0;
    for (int k = 0; k < 16; k++) {
      off += k < w ? wn[k] : 0;
      tot += wn[k];
    }
    if (p.train && ok) {
      const int64_t c = done + off + __popcll(m & ((1ull << l) - 1)) + 1;
      const int64_t pos = (n_dev0 + c - 1) % p.cap;
      p.ring_s[2 * pos] = p.s[2 * i];
      p.ring_s[2 * pos + 1] = p.s[2 * i + 1];
      p.ring_s2[2 * pos] = s2v[0];
      p.ring_s2[2 * pos + 1] = s2v[1];
      p.ring_a[pos] = p.a[i];
      p.ring_r[pos] = (float)rr;
    }
    done += tot;
    __syncthreads();  // wn is rewritten by the next block
  }
  if (threadIdx.x == 0) {
    *p.live = any_alive ? 1 : 0;
    if (p.train) {
      *p.n_dev = n_dev0 + done;
      *p.stored += done;
    }
  }
}

__global__ __launch_bounds__(256) void ddqn_state_kernel(int n, int obs_w, const double* obs, const double* g0, int n0,
                                                         const double* g1, int n1, double nh, double q0, float* s) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) state_of(obs + (size_t)i * obs_w, g0, n0, g1, n1, nh, q0, s + 2 * i);
}

// ExecutionTask.actions: the action table's row of a, or on the horizon's last step
// (remaining time 1) the whole remaining quantity at allocation (1, 0)
__global__ __launch_bounds__(256) void ddqn_actions_kernel(int n, int obs_w, const double* obs, const int64_t* a,
                                                           const double* table, double q0, double* act) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* t = table + 3 * a[i];
  const double* o = obs + (size_t)i * obs_w;
  const bool last = o[0] == 1.0;
  act[3 * i] = last ? div_scalar(o[1], q0) : t[0];
  act[3 * i + 1] = last ? 1.0 : t[1];
  act[3 * i + 2] = last ? 0.0 : t[2];
}

}  // namespace

extern "C" {

// ExecutionTask.actions for every env in one launch: act [n][3] f64 from a [n] and table [k][3]
int mxa_ddqn_actions(hipStream_t stream, int n, int obs_w, const double* obs, const int64_t* a, const double* table,
                     double q0, double* act) {
  if (n < 0 || obs_w < 2) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  hipLaunchKernelGGL(ddqn_actions_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, n, obs_w, obs, a, table, q0,
                     act);
  return (int)hipGetLastError();
}

// one period's bookkeeping (see PeriodArgs); 0 on success, else the hipError_t of the launch
int mxa_ddqn_period(hipStream_t stream, int n, int obs_w, int st_w, int train, const double* obs, const double* st,
                    const double* prev, const double* arrival, const int32_t* flags, const uint8_t* alive,
                    uint8_t* alive_next, uint8_t* live, const float* s, const int64_t* a, float* s2, double* r_row,
                    int64_t* env_steps, const double* g0, int n0, const double* g1, int n1, double nh, double q0,
                    double rscale, float* ring_s, float* ring_s2, int64_t* ring_a, float* ring_r, int64_t cap,
                    int64_t* n_dev, int64_t* stored) {
  if (n < 0 || cap <= 0 || obs_w < 2 || st_w < 3) return (int)hipErrorInvalidValue;
  PeriodArgs p{n, obs_w, st_w, train, obs, st, prev, arrival, flags, alive, alive_next, live, s, a, s2, r_row,
               env_steps, g0, g1, n0, n1, nh, q0, rscale, ring_s, ring_s2, ring_r, ring_a, cap, n_dev, stored};
  hipLaunchKernelGGL(ddqn_period_kernel, dim3(1), dim3(1024), 0, stream, p);
  return (int)hipGetLastError();
}

// ExecutionTask.state for every env in one launch
int mxa_ddqn_state(hipStream_t stream, int n, int obs_w, const double* obs, const double* g0, int n0, const double* g1,
                   int n1, double nh, double q0, float* s) {
  if (n < 0 || obs_w < 2) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  hipLaunchKernelGGL(ddqn_state_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, n, obs_w, obs, g0, n0, g1, n1, nh,
                     q0, s);
  return (int)hipGetLastError();
}

}  // extern "C"
