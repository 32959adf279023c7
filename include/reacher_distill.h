/* reacher_distill.h -- C ABI of the fused rollout + distillation step (libreacher.so).
 *
 * One rdd_step() is one iteration of the reference's hot loop, batched over N envs in
 * lockstep on one GPU (reference mlp_train.py:143-204, phase 2; the batched on-policy
 * form of backup/student_rollout.py:618-740 train_student):
 *   teacher query      sess.run(teacher.pi.pd.flat | ob)        mlp_train.py:165-167
 *   student forward    student graph on the observation          mlp_train.py:38-66,173-186
 *   distillation loss  kl_loss(s_pdflat, t_pdflat) (loss.py:3-13) or action-MSE
 *   optimiser          AdamOptimizer(lr,.9,.999,1e-8).minimize    mlp_train.py:73-80,148-161
 *   env.step           with the teacher mean (teacher-driven) or the student mean
 *                      (DAgger, mlp_train.py:196)                  + auto-reset at 50 steps
 * The policy is baselines' MlpPolicy(hid_size=64, num_hid_layers=2) for both teacher
 * (reference teacher.py:14-16) and student; flat parameter layout (P = 5060 floats):
 *   W1[11][64] | b1[64] | W2[64][64] | b2[64] | W3[64][2] | b3[2] | logstd[2]
 * plus a fixed observation filter (mean[11], std[11]) per network:
 *   obz = clip((ob - mean) / std, -5, 5).
 *
 * Conventions as in reacher.h: device pointers, asynchronous on the handle's stream, no
 * host sync except rdd_read_metrics / rdd_get_counter; 0 = OK, RD_EINVAL, -(hipError_t).
 *
 * Multi-GPU (one process per GPU, envs sharded contiguously): bind an RCCL communicator
 * (rdd_bind_comm, reacher_comm.h) and rdd_step() issues rollout, reduce, the all-reduce
 * (SUM) of the gradient and Adam on the trainer's stream from one call; or per step call
 * rdd_rollout(), all-reduce rdd_grad_buffer() across ranks yourself, then rdd_apply().
 * Single GPU: rdd_step() == rdd_rollout() + rdd_apply() fused into two kernels.
 */
#ifndef REACHER_DISTILL_H
#define REACHER_DISTILL_H
#include <stdint.h>

#include "reacher.h"
#include "reacher_comm.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RDD_LOSS_MSE 0      /* mean((mu_s - mu_t)^2) over [N_global, 2] (BASELINE configs 2, 5) */
#define RDD_LOSS_KL 1       /* sum over envs of KL(s||t), reference loss.py:3-13 (config 3)    */
#define RDD_ACT_TEACHER 0   /* env stepped with the teacher mean (configs 2-4)               */
#define RDD_ACT_STUDENT 1   /* env stepped with the student mean: DAgger (config 5)          */

typedef struct {
    int64_t n_envs;          /* envs on this rank                                   */
    int64_t n_envs_global;   /* envs over all ranks (MSE normalisation)             */
    int64_t env_base;        /* global id of this rank's env 0 (Philox stream key)   */
    uint64_t seed;           /* Philox reset seed                                   */
    int32_t loss;            /* RDD_LOSS_*                                          */
    int32_t act_with;        /* RDD_ACT_*                                           */
    float lr, beta1, beta2, eps;   /* Adam (reference: 1e-4, .9, .999, 1e-8)         */
    int32_t grid;            /* rollout workgroups; 0 = auto (<= one per CU)          */
    int32_t metrics_len;     /* ring length of the per-step metrics history; 0 = 4096 */
    int32_t stagger;         /* 0: lockstep TimeLimit (all envs share the episode phase);
                                1: env g runs at phase C + (g / RDD_STAGGER_GROUP) % 50, so a
                                   batch mixes all 50 episode phases (see below)          */
    int32_t student_dtype;   /* RDD_DTYPE_F32, or RDD_DTYPE_BF16 (BASELINE config 5: bf16
                                student MLP; see below)                                  */
    int32_t accum_steps;     /* K env steps (rollouts) per optimiser step; 0 or 1 = the
                                reference's one Adam step per env step.  Scales the MSE
                                normalisation to 1 / (K n_envs_global)                  */
    int32_t f32_split;       /* 0: every f32 product on v_mfma_f32_16x16x4_f32 (exact f32);
                                1: the K = 64 hidden-layer products of the f32 nets (both
                                layer 2s; the f32 student's dH1) as f32 emulated on bf16
                                MFMAs with three-piece operand splits (see below)        */
    int32_t group_envs;      /* envs per producer/consumer group of the rollout: 0 = auto
                                (64, or 32/16 when the batch cannot give every wave pair a
                                64-env group); 16, 32 or 64 fixes it.  Changes only the
                                order of the gradient's summation.  Auto also picks the
                                helper-pair layout for a batch of at most two 16-env groups
                                per CU (pairs 2, 3 of a workgroup run the teacher forwards
                                of pairs 0, 1); a fixed size never does      */
} rdd_config;

/* Student precision.  RDD_DTYPE_F32: every product exact f32 (v_mfma_f32_16x16x4_f32).
 * RDD_DTYPE_BF16 (mixed precision, f32 master weights + f32 Adam): the student's weight
 * matrices W1, W2, W3 are used as bf16 roundings of the master, and the MFMA operands
 * built from activations / back-propagated errors (z, h1, dZ2, dZ1) are rounded to bf16;
 * biases, log-std, tanh, the loss and every accumulation stay f32.  The teacher is f32
 * either way.  oracle/policy_np.py forward_bf16/backward_bf16 define the arithmetic. */
#define RDD_DTYPE_F32 0
#define RDD_DTYPE_BF16 1

/* f32_split = 1 keeps f32 accuracy on gfx950's 16x faster bf16 matrix path: each f32
 * operand is split EXACTLY into three bf16 pieces (x = x0 + x1 + x2: x truncated to bf16,
 * the remainder truncated, the rest, which has at most 8 significant bits), and a product
 * sums the six partial products x2y0 + x1y1 + x0y2 + x1y0 + x0y1 + x0y0 (each exact in the
 * MFMA) into the f32 accumulator; the three dropped terms are below 2^-24 |x||y|.  Layer 1
 * (K = 12), the weight gradients, biases, tanh, the loss and Adam are unchanged f32. */

/* Staggered episodes.  The reference steps ONE env and trains on random windows drawn
 * from past episodes (dataset.py:179-194), so a training batch mixes episode phases.  N
 * envs in lockstep would instead hand the optimiser a batch in which every env is at the
 * same step of its episode, and the student would chase the phase.
 * With stagger = 1, env g's episode clock is offset by (g / 32) % 50 steps: its first
 * episode is truncated to 50 - offset steps, every later one runs the full 50 steps, and
 * the reset after an episode that ends at phase u draws Philox(seed, g, u / 50 + 1).
 * Groups of 32 consecutive envs share an offset so that a wave's resets stay uniform. */
#define RDD_STAGGER_GROUP 32

typedef struct rdd_trainer rdd_trainer;

int rdd_create(rdd_trainer** out, const rdd_config* cfg, int device, void* hip_stream);
int rdd_destroy(rdd_trainer* tr);
int rdd_param_count(void);
/* Subsequent launches go to `hip_stream` (e.g. a graph-capture stream). */
int rdd_set_stream(rdd_trainer* tr, void* hip_stream);

/* Copy network parameters in (device pointers; params [P], ob_mean/ob_std [11]). */
int rdd_set_teacher(rdd_trainer* tr, const float* params, const float* ob_mean, const float* ob_std);
int rdd_set_student(rdd_trainer* tr, const float* params, const float* ob_mean, const float* ob_std);
int rdd_get_student(rdd_trainer* tr, float* params);

/* Envs <- Philox episode-0 resets, step counter <- 0, Adam moments/powers <- initial. */
int rdd_reset(rdd_trainer* tr);

/* The step: rollout (env + teacher + student fwd/bwd + loss, per-workgroup gradient
 * partials) and reduction into rdd_grad_buffer(), env-step counter++; rdd_apply(): TF1
 * Adam, optimiser-step counter++. */
int rdd_rollout(rdd_trainer* tr);
int rdd_apply(rdd_trainer* tr);
int rdd_step(rdd_trainer* tr);
/* One optimiser step of K = accum_steps env steps in ONE rollout launch (SURVEY.md §8d's
 * K = 50 reading, the reference's MpiAdam step per batch of backup/student_rollout.py:658-709):
 * the weight images stay in LDS and the per-workgroup gradient partials in registers over
 * the K env steps (the student is frozen between optimiser steps, and each env's next step
 * depends only on its own state), so the image prologue, the partial row, the reduction and
 * the launch gaps are paid once per K env steps.  The same gradient as K x (rdd_launch_stage
 * ROLLOUT, REDUCE(_ACCUM)) up to f32 reordering of the sums, the same env states (bitwise)
 * and metrics slot.  rdd_rollout_accum: the launch + reduction into rdd_grad_buffer() and
 * env clock += K; rdd_step_accum: + the bound all-reduce + Adam.  accum_steps <= 1: K = 1. */
int rdd_rollout_accum(rdd_trainer* tr);
int rdd_step_accum(rdd_trainer* tr);
/* Observation-batch mode: the same fused teacher relabel + student forward/backward +
 * loss, on caller-given observation rows obs [n][11] (device) instead of the envs' state,
 * and no env step -- the reference's training on windows drawn from its dataset buffer
 * (mlp_train.py:146-161 over dataset.py:179-194 training_batches).  The MSE is normalised
 * by n_global (all ranks' rows).  rdd_rollout_obs fills rdd_grad_buffer() (all-reduce it,
 * then rdd_apply); rdd_step_obs is the single-rank rollout_obs + apply.  These advance the
 * optimiser-step counter only; the envs' episode clocks advance with env rollouts. */
int rdd_rollout_obs(rdd_trainer* tr, const float* obs, int64_t n, int64_t n_global);
int rdd_step_obs(rdd_trainer* tr, const float* obs, int64_t n);
/* Rows mode: the same student forward/backward + loss + Adam on caller-given rows whose
 * teacher output is already recorded -- obs [n][11] and t_pdflat [n][4] = the teacher's
 * mean[2] | logstd[2] per row (device, t_pdflat 16-byte aligned); no teacher network runs.
 * The reference's training step on its dataset: sess.run([loss, minimize_adam],
 * {..., t_pdflat_batch_ph: t_pdflat_batch_array}) (mlp_train.py:146-161, the t_pdflat of
 * dataset.py:179-194 training_batches).  rdd_rollout_rows fills rdd_grad_buffer() (MSE
 * normalised by n_global); rdd_step_rows = rollout_rows + apply on one rank. */
int rdd_rollout_rows(rdd_trainer* tr, const float* obs, const float* t_pdflat, int64_t n, int64_t n_global);
int rdd_step_rows(rdd_trainer* tr, const float* obs, const float* t_pdflat, int64_t n);

/* The same work as individual launches (for per-kernel timing with events in between, and
 * for accumulating several rollouts into one optimiser step):
 * RDD_STAGE_ROLLOUT = the fused rollout kernel only; RDD_STAGE_REDUCE = partials -> grad
 * (+ the env clock advances); RDD_STAGE_APPLY = Adam + optimiser step counter;
 * RDD_STAGE_REDUCE_APPLY = both in one launch; RDD_STAGE_REDUCE_ACCUM(_APPLY) = as REDUCE
 * (_APPLY) but grad and the step's metrics slot ADD this rollout's sums.
 * rdd_step == ROLLOUT then REDUCE_APPLY.  One optimiser step per K env steps
 * (rdd_config.accum_steps = K): ROLLOUT, REDUCE, then K-1 x (ROLLOUT, REDUCE_ACCUM), then
 * APPLY (after the all-reduce when multi-GPU). */
#define RDD_STAGE_ROLLOUT 1
#define RDD_STAGE_REDUCE 2
#define RDD_STAGE_APPLY 3
#define RDD_STAGE_REDUCE_APPLY 4
#define RDD_STAGE_REDUCE_ACCUM 5
#define RDD_STAGE_REDUCE_ACCUM_APPLY 6
int rdd_launch_stage(rdd_trainer* tr, int stage);
float* rdd_grad_buffer(rdd_trainer* tr);   /* device [P], valid after rdd_rollout */
/* Use a caller-owned device buffer [P] as the gradient buffer (e.g. a torch tensor that
 * the host all-reduces in place with RCCL); NULL restores the trainer's own buffer. */
int rdd_bind_grad_buffer(rdd_trainer* tr, float* grad);
/* Bind (NULL: unbind) the communicator of this rank.  While bound, rdd_step() =
 * rollout, reduce, rd_comm_allreduce_f32(grad) on the trainer's stream, Adam; and
 * rdd_allreduce_grad() all-reduces the gradient buffer (between the REDUCE and APPLY
 * stages, or rdd_rollout_obs and rdd_apply).  The trainer does not own the communicator. */
int rdd_bind_comm(rdd_trainer* tr, rd_comm* comm);
int rdd_allreduce_grad(rdd_trainer* tr);

/* Policy query without stepping (teacher.pi.pd.flat / student pdflat):
 * obs [n][11] -> t_pdflat, s_pdflat [n][4] (either output may be NULL). */
int rdd_forward(rdd_trainer* tr, const float* obs, int64_t n, float* t_pdflat, float* s_pdflat);

/* Env state hooks (state [8][n_envs] SoA, see reacher.h). */
int rdd_get_env_state(rdd_trainer* tr, float* state);
/* rdd_set_env_state checks the caller's joint angles first (host-synchronising): the fused
 * rollout's trig is exact for |q0| < 8192 and |q1| <= 4 rad (an episode's own states never
 * leave that range); outside it, or not finite -> RD_EINVAL and the trainer's state is unchanged.
 * The gym-API env (reacher.h rd_set_state) takes any state. */
int rdd_set_env_state(rdd_trainer* tr, const float* state);

/* Host-synchronising readers (they also report a timed-out producer/consumer hand-off
 * inside a rollout as an error).  Metrics per optimiser step s (ring of metrics_len):
 * {sum reward, loss, sum (mu_s - mu_t)^2, envs}; out [count][4] for the last `count` steps. */
int rdd_get_counter(rdd_trainer* tr, int64_t* steps);              /* env steps */
int rdd_get_counters(rdd_trainer* tr, int64_t* env_steps, int64_t* opt_steps);
int rdd_read_metrics(rdd_trainer* tr, int64_t count, double* out);

#ifdef __cplusplus
}
#endif
#endif
