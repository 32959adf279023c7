/* reacher_ppo.h -- C ABI of the teacher's PPO training on batched Reacher-v2 (libreacher.so).
 *
 * The reference trains its teacher with baselines ppo1 (reference teacher.py:23-37):
 *   pposgd_simple.learn(env, MlpPolicy(hid_size=64, num_hid_layers=2),
 *       timesteps_per_actorbatch=2048, clip_param=0.2, entcoeff=0.0, optim_epochs=10,
 *       optim_stepsize=3e-4, optim_batchsize=64, gamma=0.99, lam=0.95, schedule='linear')
 * Here one iteration collects n_envs x horizon env steps (the actor batch) with the
 * stochastic policy (mean + exp(logstd) N(0,1)), computes GAE(lambda) advantages and
 * returns, standardizes the advantages, updates the observation filter (RunningMeanStd),
 * freezes the old policy, and runs optim_epochs epochs of shuffled minibatch TF1/MpiAdam
 * steps on pol_surr + vf_loss (entcoeff 0), with the linear lr/clip schedule.
 *
 * Parameters: policy [RDP_POLICY_PARAMS = 5060] in the MlpPolicy layout of
 * reacher_distill.h (W1 b1 W2 b2 W3 b3 logstd; it plugs into rdd_set_teacher with the
 * filter from rdp_get_obfilter); value net [RDP_VALUE_PARAMS = 4993] = V1[11][64] c1
 * V2[64][64] c2 V3[64][1] c3.
 * Randomness: action noise of env g at iteration k, step t = Box-Muller of words 0, 1 of
 * Philox4x32-10(ctr = {g lo, g hi, k, t}, key = {seed lo, seed hi ^ 0xA5A5A5A5}); resets as
 * reacher.h (Philox(seed, g, episode)), each env keeps its own 50-step episode clock.
 * Conventions as in reacher.h.  Single GPU (baselines' MPI all-reduce per minibatch is not
 * reproduced).
 */
#ifndef REACHER_PPO_H
#define REACHER_PPO_H
#include <stdint.h>

#include "reacher.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RDP_POLICY_PARAMS 5060
#define RDP_VALUE_PARAMS 4993
#define RDP_METRICS 8   /* ep_ret_mean, episodes, pol_surr, vf_loss, entropy, clipfrac, lrmult, timesteps */

typedef struct {
    int64_t n_envs;           /* parallel envs                                          */
    int32_t horizon;          /* steps per env per iteration (actor batch = n_envs x horizon) */
    uint64_t seed;
    int64_t env_base;         /* global id of env 0                                      */
    float clip_param;         /* 0.2    */
    float entcoeff;           /* 0.0 (only 0 is supported: the reference's value)       */
    int32_t optim_epochs;     /* 10     */
    float optim_stepsize;     /* 3e-4   */
    int32_t optim_batchsize;  /* 64 in the reference; 0 = the whole actor batch         */
    float gamma, lam;         /* 0.99, 0.95 */
    int32_t schedule_linear;  /* 1: lrmult = max(1 - timesteps / max_timesteps, 0); 0: 1 */
    int64_t max_timesteps;
    int32_t metrics_len;      /* per-iteration metrics ring; 0 = 1024                   */
} rdp_config;

typedef struct rdp_trainer rdp_trainer;

int rdp_param_counts(int32_t* policy, int32_t* value);
int rdp_create(rdp_trainer** out, const rdp_config* cfg, int device, void* hip_stream);
int rdp_destroy(rdp_trainer* t);
int rdp_set_stream(rdp_trainer* t, void* hip_stream);
/* parameters (device pointers) */
int rdp_set_policy(rdp_trainer* t, const float* policy);
int rdp_get_policy(rdp_trainer* t, float* policy);
int rdp_set_value(rdp_trainer* t, const float* value);
int rdp_get_value(rdp_trainer* t, float* value);
/* observation filter as float32 (mean[11], std[11]) the policy normalises with */
int rdp_get_obfilter(rdp_trainer* t, float* mean, float* std);
/* envs, episode clocks, filter (count 1e-2), Adam, counters to their initial state */
int rdp_reset(rdp_trainer* t);
/* one PPO iteration (pposgd_simple.learn loop body) == rdp_rollout + rdp_optimize */
int rdp_iterate(rdp_trainer* t);
/* traj_segment_generator + add_vtarg_and_adv + the filter update + oldpi <- pi */
int rdp_rollout(rdp_trainer* t);
/* the optim_epochs of minibatch Adam steps and the schedule update */
int rdp_optimize(rdp_trainer* t);
/* the last actor batch (device pointers, any may be null), rows t-major (t n_envs + n):
 * ob [S][11], ac [S][2], vpred [S], rew [S], new [S] (1 = first step of an episode),
 * nextvpred [n_envs], adv [S], ret [S] (tdlamret) */
int rdp_get_batch(rdp_trainer* t, float* ob, float* ac, float* vpred, float* rew, float* newf, float* nextvpred,
                  float* adv, float* ret);
float* rdp_grad_buffer(rdp_trainer* t);   /* gradient of the last minibatch [5060 + 4993] */
int rdp_bind_grad_buffer(rdp_trainer* t, float* grad);   /* use the caller's buffer (null: own) */
int rdp_get_counter(rdp_trainer* t, int64_t* iterations);
int rdp_read_metrics(rdp_trainer* t, int64_t count, double* out);   /* [count][RDP_METRICS] */

#ifdef __cplusplus
}
#endif
#endif
