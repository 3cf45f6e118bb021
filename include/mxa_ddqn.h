/* mxa_ddqn.h — libmxa_ddqn.so: the DDQN execution learner's per-period bookkeeping on the device
 * (mxabides/ddqn.py run_episode; marl-optimal-execution_amd/csrc/ddqn_period.hip).
 *
 * Replaces, per ABIDESEnv.step of a VecABIDESEnv batch, the PyTorch ops that follow the step in
 * the learner loop of agent/execution/ddqlearning_execution_agent.py:275-299 (place_order: the
 * transition, compute_reward :409-446, the next state :301-331, memory.store_transition :115-116)
 * with one launch; bitwise the same results (tests/test_gpu_ddqn.py). Pointers are device
 * pointers; `stream` is a hipStream_t. Returns 0 or a hipError_t. */
#ifndef MXA_DDQN_H
#define MXA_DDQN_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* one period: ok = alive & obs valid & no env error; r = compute_reward(prev, st) (BUY); s2 =
 * discretize(obs); env_steps += alive; if train: replay rows (s, a, s2, r) of the ok envs appended
 * in env order at n_dev (mod cap), n_dev and stored += their count; r_row = ok ? r : 0;
 * alive_next = ok & !done; live = any(alive). obs [n][obs_w] f64, st / prev [n][st_w] f64
 * (mxa_write_rl_state rows), arrival [n] f64, flags [n] i32 (mxa_step), alive / alive_next [n]
 * bool, live [1] bool, s / s2 [n][2] f32, a [n] i64, r_row [n] f64, env_steps [n] i64, g0 / g1 the
 * state grid's split points (f64), rscale = 1e4 / q0; ring_s / ring_s2 [cap + 1][2] f32, ring_a
 * [cap + 1] i64, ring_r [cap + 1] f32, n_dev / stored i64 scalars. */
int mxa_ddqn_period(void* stream, int n, int obs_w, int st_w, int train, const double* obs, const double* st,
                    const double* prev, const double* arrival, const int32_t* flags, const uint8_t* alive,
                    uint8_t* alive_next, uint8_t* live, const float* s, const int64_t* a, float* s2, double* r_row,
                    int64_t* env_steps, const double* g0, int n0, const double* g1, int n1, double nh, double q0,
                    double rscale, float* ring_s, float* ring_s2, int64_t* ring_a, float* ring_r, int64_t cap,
                    int64_t* n_dev, int64_t* stored);
/* ExecutionTask.state of every env: s [n][2] f32 = discretize(obs) */
int mxa_ddqn_state(void* stream, int n, int obs_w, const double* obs, const double* g0, int n0, const double* g1,
                   int n1, double nh, double q0, float* s);
/* ExecutionTask.actions of every env: act [n][3] f64 = table[a] (table [k][3] f64), or on the last
 * horizon step (obs[0] == 1) (obs[1] / q0, 1, 0) */
int mxa_ddqn_actions(void* stream, int n, int obs_w, const double* obs, const int64_t* a, const double* table,
                     double q0, double* act);
#ifdef __cplusplus
}
#endif
#endif
