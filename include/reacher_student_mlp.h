/* reacher_student_mlp.h -- C ABI of the reference's own MLP student: forward and one
 * distillation training step on a batch of rows (libreacher.so).
 *
 * Graph: student_mlp_graph (reference src/distilation/student_nn.py:51-57)
 *     x[16] -> dense 24, tanh -> dense 128, tanh -> dense 128 -> dense 32, tanh -> dense 4
 * x row = dropout(ob)[11] | prev_pdflat[4] | prev_rew[1]   (mlp_train.py:38-52; the caller
 * assembles rows, keep_prob = 1), output = s_pdflat = mean[2] | logstd[2] (a state-dependent
 * log-std, unlike MlpPolicy's free logstd).
 * Flat parameters (RDM_PARAMS = 24,380 floats), tf.layers.dense order per layer:
 *     kernel W[in][out] row-major, then bias[out];  layers 16x24, 24x128, 128x128, 128x32, 32x4.
 * Loss: kl_loss(s_pdflat, t_pdflat) (reference loss.py:3-13: sum over rows of KL(s||t)),
 * or action-MSE: sum over rows of |mu_s - mu_t|^2 / (2 n_global).
 * Optimiser: TF1 Adam (mlp_train.py:73-80), f32 master weights and slots.
 *
 * Conventions as in reacher.h: device pointers (x 16-byte aligned), asynchronous on the
 * handle's stream, 0 = OK, RD_EINVAL, -(hipError_t).  Multi-GPU: rows sharded by the
 * caller; per step rdm_rollout(), all-reduce(SUM) rdm_grad_buffer(), rdm_apply().
 */
#ifndef REACHER_STUDENT_MLP_H
#define REACHER_STUDENT_MLP_H
#include <stdint.h>

#include "reacher.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RDM_PARAMS 24380
#define RDM_IN 16
#define RDM_OUT 4
#define RDM_LOSS_MSE 0
#define RDM_LOSS_KL 1

typedef struct {
    int32_t loss;                  /* RDM_LOSS_*                                         */
    float lr, beta1, beta2, eps;   /* Adam (reference: 1e-4, .9, .999, 1e-8)             */
    int32_t grid;                  /* workgroups (64 rows each per pass); 0 = one per CU */
    int32_t metrics_len;           /* per-step metrics ring length; 0 = 4096             */
    float keep_prob;               /* dropout on the 11 ob inputs while training
                                      (tf.nn.dropout, mlp_train.py:50; reference KEEP_PROB =
                                      0.5); 1 = off.  Mask of input k of global row r at
                                      optimiser step S: keep iff u < keep_prob, u = word k%4
                                      of Philox4x32-10(ctr = {r lo, r hi, S, k/4}, key = seed),
                                      u = (word >> 8) * 2^-24; kept inputs are x / keep_prob */
    uint64_t seed;                 /* dropout key                                        */
    int64_t row_base;              /* global index of this rank's row 0 (sharded batches) */
} rdm_config;

typedef struct rdm_trainer rdm_trainer;

int rdm_param_count(void);
/* the 'MLP' scope: student graph, loss and Adam (mlp_train.py:35-80) */
int rdm_create(rdm_trainer** out, const rdm_config* cfg, int device, void* hip_stream);
int rdm_destroy(rdm_trainer* t);
int rdm_set_stream(rdm_trainer* t, void* hip_stream);
/* variable initialisation / restore (mlp_train.py:82-99): params [RDM_PARAMS] */
int rdm_set_params(rdm_trainer* t, const float* params);
int rdm_get_params(rdm_trainer* t, float* params);
/* Adam slots, beta powers and step counter to zero (mlp_train.py:93) */
int rdm_reset(rdm_trainer* t);
/* sess.run(s_pdflat_slice) (mlp_train.py:170-183), all rows: x [n][16] -> pdflat [n][4] */
int rdm_forward(rdm_trainer* t, const float* x, int64_t n, float* pdflat);
/* forward + loss + backward of n rows (of n_global over all ranks): gradient into
 * rdm_grad_buffer(); metrics (loss, sum |mu_s - mu_t|^2, rows) into the ring at apply */
int rdm_rollout(rdm_trainer* t, const float* x, const float* t_pdflat, int64_t n, int64_t n_global);
/* Adam on rdm_grad_buffer() (after an optional all-reduce), step counter + 1 */
int rdm_apply(rdm_trainer* t);
/* sess.run([loss, minimize_adam]) (mlp_train.py:145-160) == rollout + apply */
int rdm_step(rdm_trainer* t, const float* x, const float* t_pdflat, int64_t n);
float* rdm_grad_buffer(rdm_trainer* t);
int rdm_bind_grad_buffer(rdm_trainer* t, float* grad);
int rdm_get_counter(rdm_trainer* t, int64_t* opt_steps);
/* last `count` optimiser steps, oldest first: [count][4] = loss, sq err, rows, 0 */
int rdm_read_metrics(rdm_trainer* t, int64_t count, double* out);

#ifdef __cplusplus
}
#endif
#endif
