/* reacher_student_lstm.h -- C ABI of the reference's LSTM student: forward over unrolled
 * windows and one truncated-BPTT distillation training step (libreacher.so).
 *
 * Graph: student_lstm_graph (reference src/distilation/student_nn.py:21-49), T unrolled steps
 * (STEPS_UNROLLED = 10, config.py:25) over B windows (LSTM_BATCH_SIZE = 20, config.py:26):
 *     p_t = dense(prev_pdflat_t, 32)                         linear
 *     x_t = [dropout(ob_t)[11], p_t[32]]
 *     (c_t, h_t) = LSTMCell(200)(x_t, (c_{t-1}, h_{t-1}))     TF1: gates i, j, f, o of
 *                                                             [x_t, h_{t-1}] . Wl + bl,
 *                                                             forget_bias 1, tanh
 *     pdflat_t = dense(tanh dense 32(tanh dense 64(tanh dense 128(tanh dense 64(h_t))))), 4)
 * with ONE HEAD PER UNROLLED STEP: the reference calls tf.layers.dense inside its Python loop
 * over the T steps without reuse (student_nn.py:40-47), so step t's five layers are their own
 * variables (dense_{5t+1} .. dense_{5t+5}); the LSTMCell and the prev-pdflat dense are shared.
 * Flat parameters (RDL_PARAMS_T(T) floats; RDL_PARAMS at the reference's T = 10) in
 * variable-creation order, each kernel W[in][out] row-major then its bias:
 *     Wp[4][32] bp | Wl[243][800] bl | head_0 | ... | head_{T-1},
 *     head_t = W1[200][64] b1 | W2[64][128] b2 | W3[128][64] b3 | W4[64][32] b4 | W5[32][4] b5
 * Tensors: ob [T][B][11], prev_pdflat [T][B][4], t_pdflat / pdflat [T][B][4], LSTM state
 * [2][B][200] = (c, m) as the reference's initial_state_batch_ph (lstm_train.py:51).
 * Loss: kl_loss summed over T and B (loss.py:3-13), or action-MSE over T x rows_global.
 * Optimiser: TF1 Adam (reference lr 1e-3, lstm_train.py:73-79).
 *
 * Conventions as in reacher.h: device pointers, asynchronous on the handle's stream,
 * 0 = OK, RD_EINVAL, -(hipError_t).  Multi-GPU: windows sharded by the caller (row_base =
 * this rank's first global window); rdl_rollout, all-reduce(SUM) rdl_grad_buffer(), rdl_apply.
 */
#ifndef REACHER_STUDENT_LSTM_H
#define REACHER_STUDENT_LSTM_H
#include <stdint.h>

#include "reacher.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RDL_CELL_PARAMS 195360                                   /* Wp bp Wl bl          */
#define RDL_HEAD_PARAMS 31652                                    /* one step's head      */
#define RDL_PARAMS_T(T) (RDL_CELL_PARAMS + (T) * RDL_HEAD_PARAMS)
#define RDL_PARAMS RDL_PARAMS_T(10)                              /* 511,880              */
#define RDL_UNITS 200
#define RDL_LOSS_MSE 0
#define RDL_LOSS_KL 1

typedef struct {
    int32_t loss;                  /* RDL_LOSS_*                                             */
    float lr, beta1, beta2, eps;   /* Adam (reference: 1e-3, .9, .999, 1e-8)                 */
    int32_t steps;                 /* T, unrolled steps per window (reference 10)            */
    int32_t max_windows;           /* capacity: largest B passed to any call                 */
    int32_t metrics_len;           /* per-step metrics ring length; 0 = 4096                 */
    float keep_prob;               /* dropout on ob while training (reference KEEP_PROB 0.5);
                                      mask of ob[t][b][k] at optimiser step S: keep iff
                                      u < keep_prob, u = word k%4 of Philox4x32-10(ctr =
                                      {w lo, w hi, S, 4t + k/4}, key = seed), w = row_base + b */
    uint64_t seed;
    int64_t row_base;              /* global index of this rank's window 0                  */
    int32_t kernels;               /* 0 = automatic kernel selection; RDL_KERNELS_* bits force
                                      the general path (same results, tests compare them)    */
} rdl_config;

/* rdl_config.kernels: by default at most 32 windows run the whole recurrence / BPTT as one
 * persistent launch each and at most 16,384 rows run the heads as one launch each way (when
 * their backward's partial rows fit 512 MB at max_windows: rdl_head_path reports it); these
 * bits keep the per-step recurrence launches / the per-layer head GEMMs at any size. */
#define RDL_KERNELS_STEP_RECURRENCE 1
#define RDL_KERNELS_LAYER_HEAD 2

typedef struct rdl_trainer rdl_trainer;

/* flat parameters of a trainer with `steps` unrolled steps (RDL_PARAMS_T(steps)), -1 if steps <= 0 */
int64_t rdl_param_count(int32_t steps);
/* the 'LSTM' scope: graph, kl_loss and Adam (lstm_train.py:35-79) */
int rdl_create(rdl_trainer** out, const rdl_config* cfg, int device, void* hip_stream);
int rdl_destroy(rdl_trainer* t);
int rdl_set_stream(rdl_trainer* t, void* hip_stream);
/* initialisation / saver.restore (lstm_train.py:82-107): params [RDL_PARAMS_T(steps)] */
int rdl_set_params(rdl_trainer* t, const float* params);
int rdl_get_params(rdl_trainer* t, float* params);
/* Adam slots, beta powers, step counter to zero (lstm_train.py:99) */
int rdl_reset(rdl_trainer* t);
/* the Adam slots m, v [RDL_PARAMS_T(steps)] (device pointers): with the params, what the reference's
 * tf.train.Saver over the 'LSTM' scope checkpoints every episode and restores with -r
 * (lstm_train.py:86-87,102-107,199); the beta powers are not in that scope, so a restore
 * starts them afresh (rdl_reset, then rdl_set_params + rdl_set_slots) */
int rdl_get_slots(rdl_trainer* t, float* m, float* v);
int rdl_set_slots(rdl_trainer* t, const float* m, const float* v);
/* sess.run((s_action, s_pdflat_slice, final_state)) (lstm_train.py:171-183), all T x B outputs:
 * state0 may be null (zero state); state_out may be null */
int rdl_forward(rdl_trainer* t, const float* ob, const float* prev_pdflat, const float* state0, int64_t windows,
                float* pdflat, float* state_out);
/* forward + loss + BPTT of B windows (of windows_global over all ranks) from state0 (null =
 * zeros, as lstm_train.py:159): gradient into rdl_grad_buffer() */
int rdl_rollout(rdl_trainer* t, const float* ob, const float* prev_pdflat, const float* t_pdflat,
                const float* state0, int64_t windows, int64_t windows_global);
int rdl_apply(rdl_trainer* t);
/* final_state_batch of the last forward pass (rdl_forward / rdl_rollout / rdl_step) of
 * `windows` windows, as [2][windows][200] = (c, h): the truncated-BPTT driver feeds it back as
 * the next window's initial state (backup/lstm_bbpt.py:141-155 fetches it in the training
 * sess.run); RD_EINVAL if the last pass had another window count */
int rdl_final_state(rdl_trainer* t, int64_t windows, float* state_out);
/* sess.run([loss, minimize_adam]) (lstm_train.py:145-160) == rollout + apply */
int rdl_step(rdl_trainer* t, const float* ob, const float* prev_pdflat, const float* t_pdflat,
             const float* state0, int64_t windows);
float* rdl_grad_buffer(rdl_trainer* t);
int rdl_bind_grad_buffer(rdl_trainer* t, float* grad);
/* optimiser steps taken; RD_EINVAL if a persistent recurrence launch (<= 32 windows) gave up
 * at its grid barrier since the trainer was created (its steps are invalid) */
int rdl_get_counter(rdl_trainer* t, int64_t* opt_steps);
/* 1: batches of at most 16,384 rows run the fused head kernels (their backward's partial rows,
 * T x workgroups x 31,652 floats at max_windows, were allocated: at most 512 MB); 0: the
 * per-layer head GEMMs at every size (RDL_KERNELS_LAYER_HEAD, or the rows would not fit). */
int rdl_head_path(const rdl_trainer* t);
/* [count][4] = loss, sum |mu_s - mu_t|^2, rows (T x B), 0 */
int rdl_read_metrics(rdl_trainer* t, int64_t count, double* out);

#ifdef __cplusplus
}
#endif
#endif
