/* ORACLE -- test infrastructure only.  CPU restatement of the reference's hot path:
 *
 *   env.step/env.reset  : gym 0.10.5 ReacherEnv on MuJoCo 1.50 (RK4, frame_skip 2),
 *                         called at reference mlp_train.py:112,135,138,196,200.
 *                         Formulas: SURVEY.md App. A; same restatement as reacher_np.py.
 *   teacher query       : baselines MlpPolicy pol branch (reference teacher.py:14-16,
 *                         queried at mlp_train.py:123-125,165-167): obfilter clip +-5,
 *                         2x64 tanh, linear mean, state-independent logstd.
 *   distillation loss   : kl_loss (reference loss.py:3-13, KL(s||t) summed) or the
 *                         BASELINE action-MSE (mean over [N,2]).
 *   optimiser           : tf.train.AdamOptimizer (reference mlp_train.py:73-80), TF1 form
 *                         lr_t = lr*sqrt(1-b2^t)/(1-b1^t); theta -= lr_t*m/(sqrt(v)+eps).
 *
 * Parity: the env part is pinned by the reference's fixture through reacher_np.py
 * (tests/test_oracle_fixture.py checks this C code against the same golden file).
 * The policy/loss/Adam part restates third-party TF/baselines math that has no
 * reference test: it is checked against reacher_np/policy_np (f64) only -- parity
 * of that part is "unpinned" beyond the formulas.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this
 * library (oracle/_build/libreacher_oracle.so).  It is never part of the product.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <string.h>

/* model constants as constant expressions */
#define RDO_PI 3.14159265358979323846
#define RDO_ML (1000.0 * RDO_PI * 0.01 * 0.01 * 0.11)
#define RDO_IC (RDO_ML * (3 * 0.01 * 0.01 + 0.11 * 0.11) / 12.0)
#define RDO_MF (1000.0 * 4.0 / 3.0 * RDO_PI * 0.01 * 0.01 * 0.01)
#define RDO_IF (0.4 * RDO_MF * 0.01 * 0.01)
#define RDO_A0 (RDO_IC + RDO_ML * 0.05 * 0.05 + (RDO_ML + RDO_MF) * 0.1 * 0.1)
#define RDO_I2 (RDO_IC + RDO_ML * 0.05 * 0.05 + RDO_IF + RDO_MF * 0.11 * 0.11)
#define RDO_HC (0.1 * (RDO_ML * 0.05 + RDO_MF * 0.11))
#define RDO_M11_0 (RDO_A0 + RDO_I2 + 2 * RDO_HC + 1.0)
#define RDO_M12_0 (RDO_I2 + RDO_HC)
#define RDO_M22_0 (RDO_I2 + 1.0)
#define RDO_INVW0 (RDO_M11_0 / (RDO_M11_0 * RDO_M22_0 - RDO_M12_0 * RDO_M12_0))
#define RDO_BREF (2.0 / (0.95 * 0.02))
#define RDO_KREF (1.0 / (0.95 * 0.95 * 0.02 * 0.02))

/* ---- f64 instance */
#define REAL double
#define SFX f64
#define COS cos
#define SIN sin
#define SQRT sqrt
#define FABS fabs
#include "reacher_ref_impl.h"
#undef REAL
#undef SFX
#undef COS
#undef SIN
#undef SQRT
#undef FABS
/* ---- f32 instance */
#define REAL float
#define SFX f32
#define COS cosf
#define SIN sinf
#define SQRT sqrtf
#define FABS fabsf
#include "reacher_ref_impl.h"

void rdo_constants(double* out) {
    out[0] = RDO_A0; out[1] = RDO_I2; out[2] = RDO_HC; out[3] = RDO_INVW0;
    out[4] = RDO_BREF; out[5] = RDO_KREF;
}

/* ------------------------------------------------------------------ Philox4x32-10
 * Synthetic reset stream: key = seed, counter = (env_id lo/hi,
 * episode, block).  Integer-exact, so the HIP reset kernel must match bit for bit. */
static void philox4x32_10(uint32_t ctr[4], uint32_t k0, uint32_t k1, uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static inline float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

/* draws[6] f32 for (seed, env_id, episode): qpos U(-.1,.1)x2, qvel U(-.005,.005)x2,
 * goal U(-.2,.2)x2 (ReacherEnv.reset_model ranges); value = fmaf(hi-lo, u, lo). */
void rdo_philox_draw(uint64_t seed, uint64_t env_id, uint32_t episode, float* draws) {
    uint32_t ctr[4] = {(uint32_t)env_id, (uint32_t)(env_id >> 32), episode, 0u};
    uint32_t o[4], p[4];
    philox4x32_10(ctr, (uint32_t)seed, (uint32_t)(seed >> 32), o);
    ctr[3] = 1u;
    philox4x32_10(ctr, (uint32_t)seed, (uint32_t)(seed >> 32), p);
    draws[0] = fmaf(0.2f, u01(o[0]), -0.1f);
    draws[1] = fmaf(0.2f, u01(o[1]), -0.1f);
    draws[2] = fmaf(0.01f, u01(o[2]), -0.005f);
    draws[3] = fmaf(0.01f, u01(o[3]), -0.005f);
    draws[4] = fmaf(0.4f, u01(p[0]), -0.2f);
    draws[5] = fmaf(0.4f, u01(p[1]), -0.2f);
}

/* ------------------------------------------------------------------ MlpPolicy (f32)
 * flat params (P = 5060): W1[11][64], b1[64], W2[64][64], b2[64], W3[64][2], b3[2],
 * logstd[2]; obfilter mu[11], sd[11] separate (not trained). */
#define OBD 11
#define HID 64
#define ACD 2
#define P_W1 0
#define P_B1 (P_W1 + OBD * HID)
#define P_W2 (P_B1 + HID)
#define P_B2 (P_W2 + HID * HID)
#define P_W3 (P_B2 + HID)
#define P_B3 (P_W3 + HID * ACD)
#define P_LS (P_B3 + ACD)
#define P_TOT (P_LS + ACD)

int rdo_param_count(void) { return P_TOT; }

typedef struct {
    float z[OBD], h1[HID], h2[HID], mean[ACD];
} fwd_t;

static void mlp_fwd(const float* p, const float* mu, const float* sd, const float* ob, fwd_t* f) {
    for (int k = 0; k < OBD; ++k) {
        float z = (ob[k] - mu[k]) / sd[k];
        f->z[k] = z < -5.f ? -5.f : (z > 5.f ? 5.f : z);
    }
    for (int j = 0; j < HID; ++j) {
        float a = p[P_B1 + j];
        for (int k = 0; k < OBD; ++k) a += f->z[k] * p[P_W1 + k * HID + j];
        f->h1[j] = tanhf(a);
    }
    for (int j = 0; j < HID; ++j) {
        float a = p[P_B2 + j];
        for (int k = 0; k < HID; ++k) a += f->h1[k] * p[P_W2 + k * HID + j];
        f->h2[j] = tanhf(a);
    }
    for (int d = 0; d < ACD; ++d) {
        float a = p[P_B3 + d];
        for (int k = 0; k < HID; ++k) a += f->h2[k] * p[P_W3 + k * ACD + d];
        f->mean[d] = a;
    }
}

/* accumulate dL/dparams for one env given dL/dmean[2] and dL/dlogstd[2] */
static void mlp_bwd(const float* p, const fwd_t* f, const float* dmean, const float* dls, float* g) {
    float dz2[HID], dz1[HID];
    for (int d = 0; d < ACD; ++d) { g[P_B3 + d] += dmean[d]; g[P_LS + d] += dls[d]; }
    for (int k = 0; k < HID; ++k) {
        float dh = 0.f;
        for (int d = 0; d < ACD; ++d) {
            g[P_W3 + k * ACD + d] += f->h2[k] * dmean[d];
            dh += p[P_W3 + k * ACD + d] * dmean[d];
        }
        dz2[k] = dh * (1.f - f->h2[k] * f->h2[k]);
    }
    for (int j = 0; j < HID; ++j) g[P_B2 + j] += dz2[j];
    for (int k = 0; k < HID; ++k) {
        float dh = 0.f;
        for (int j = 0; j < HID; ++j) {
            g[P_W2 + k * HID + j] += f->h1[k] * dz2[j];
            dh += p[P_W2 + k * HID + j] * dz2[j];
        }
        dz1[k] = dh * (1.f - f->h1[k] * f->h1[k]);
    }
    for (int j = 0; j < HID; ++j) g[P_B1 + j] += dz1[j];
    for (int k = 0; k < OBD; ++k)
        for (int j = 0; j < HID; ++j) g[P_W1 + k * HID + j] += f->z[k] * dz1[j];
}

/* TF1 ApplyAdam functor (tensorflow/core/kernels/training_ops.cc) over a flat buffer:
 *   alpha = lr*sqrt(1-b2p)/(1-b1p); m += (g-m)(1-b1); v += (g^2-v)(1-b2);
 *   var -= m*alpha/(sqrt(v)+eps).  b1p/b2p are the float32 beta powers for this step. */
void rdo_adam_tf1(int64_t n, float* theta, float* m, float* v, const float* g, float b1p, float b2p,
                  float lr, float b1, float b2, float eps) {
    const float alpha = lr * sqrtf(1.f - b2p) / (1.f - b1p);
    for (int64_t i = 0; i < n; ++i) {
        m[i] += (g[i] - m[i]) * (1.f - b1);
        v[i] += (g[i] * g[i] - v[i]) * (1.f - b2);
        theta[i] -= (m[i] * alpha) / (sqrtf(v[i]) + eps);
    }
}

/* One rollout+distill step over n envs (lockstep), f32, the CPU baseline / f32 checker.
 *   state [8][n] SoA (q0,q1,v0,v1,tx,ty,dx,dy); step = global completed-step counter C.
 *   Env g = env_base+i runs at phase u = C + off(g), off(g) = stagger ? (g / 32) % 50 : 0
 *   (episode = u/50, t = u%50; done when t == 49 -> reset from Philox(seed, g, episode+1)).
 *   stagger = 0 is the lockstep TimeLimit; stagger = 1 spreads the envs' episode phases
 *   teacher/student: flat params + obfilter (mu, sd)
 *   loss: 0 = MSE(mean over n_global*2), 1 = KL(s||t) summed
 *   act_student: 0 = step env with teacher mean, 1 = with student mean (DAgger)
 *   grad [P] (zeroed here, filled with the rank-local gradient, unscaled by other ranks)
 *   metrics[4] += {sum reward, loss, sum (mu_s-mu_t)^2, n}
 * Returns nothing; Adam is a separate call (so the multi-rank path can all-reduce). */
void rdo_distill_step(int64_t n, int64_t n_global, int64_t env_base, uint64_t seed, int64_t step,
                      float* state, const float* tp, const float* tmu, const float* tsd,
                      const float* sp, const float* smu, const float* ssd, int loss, int act_student,
                      int stagger, float* grad, double* metrics, int nthreads) {
    memset(grad, 0, sizeof(float) * P_TOT);
    const float tls0 = tp[P_LS], tls1 = tp[P_LS + 1];
    const float sls0 = sp[P_LS], sls1 = sp[P_LS + 1];
    if (nthreads < 1) nthreads = 1;
    /* per-thread partials, summed in thread order afterwards: the result does not depend on
       which thread finishes first (deterministic for a given nthreads) */
    float* gpart = (float*)calloc((size_t)nthreads * P_TOT, sizeof(float));
    double* mpart = (double*)calloc((size_t)nthreads * 3, sizeof(double));
#pragma omp parallel num_threads(nthreads)
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        float* g = gpart + (size_t)tid * P_TOT;
        double rsum = 0, lsum = 0, msum = 0;
#pragma omp for schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            float s[8], ob[OBD];
            for (int k = 0; k < 8; ++k) s[k] = state[k * n + i];
            ob[0] = cosf(s[0]); ob[1] = cosf(s[1]); ob[2] = sinf(s[0]); ob[3] = sinf(s[1]);
            ob[4] = s[4]; ob[5] = s[5]; ob[6] = s[2]; ob[7] = s[3]; ob[8] = s[6]; ob[9] = s[7];
            ob[10] = 0.f;
            fwd_t ft, fs;
            mlp_fwd(tp, tmu, tsd, ob, &ft);
            mlp_fwd(sp, smu, ssd, ob, &fs);
            float dmean[2], dls[2];
            for (int d = 0; d < 2; ++d) {
                float diff = fs.mean[d] - ft.mean[d];
                msum += (double)diff * diff;
                if (loss == 0) {
                    dmean[d] = diff / (float)n_global;
                    dls[d] = 0.f;
                    lsum += (double)diff * diff / (2.0 * (double)n_global);
                } else {
                    float tl = d ? tls1 : tls0, sl = d ? sls1 : sls0;
                    float tvar = expf(2.f * tl), svar = expf(2.f * sl);
                    dmean[d] = diff / tvar;
                    dls[d] = svar / tvar - 1.f;
                    lsum += (double)(tl - sl + (svar + diff * diff) / (2.f * tvar) - 0.5f);
                }
            }
            mlp_bwd(sp, &fs, dmean, dls, g);
            float a0 = act_student ? fs.mean[0] : ft.mean[0];
            float a1 = act_student ? fs.mean[1] : ft.mean[1];
            float obn[OBD];
            rsum += env_step_f32(s, a0, a1, obn);
            const int64_t u = step + (stagger ? ((env_base + i) / 32) % 50 : 0);  /* RDD_STAGGER_GROUP */
            if (u % 50 == 49) {
                float dr[6];
                rdo_philox_draw(seed, (uint64_t)(env_base + i), (uint32_t)(u / 50 + 1), dr);
                env_reset_f32(s, dr, obn);
            }
            for (int k = 0; k < 8; ++k) state[k * n + i] = s[k];
        }
        mpart[3 * tid] = rsum;
        mpart[3 * tid + 1] = lsum;
        mpart[3 * tid + 2] = msum;
    }
    double rsum = 0, lsum = 0, msum = 0;
    for (int t = 0; t < nthreads; ++t) {
        for (int k = 0; k < P_TOT; ++k) grad[k] += gpart[(size_t)t * P_TOT + k];
        rsum += mpart[3 * t];
        lsum += mpart[3 * t + 1];
        msum += mpart[3 * t + 2];
    }
    free(gpart);
    free(mpart);
    metrics[0] += rsum;
    metrics[1] += lsum;
    metrics[2] += msum;
    metrics[3] += (double)n;
}

/* Fresh episode-0 states from the Philox stream. */
void rdo_philox_reset(int64_t n, int64_t env_base, uint64_t seed, uint32_t episode, float* state) {
    for (int64_t i = 0; i < n; ++i) {
        float dr[6], s[8], ob[OBD];
        rdo_philox_draw(seed, (uint64_t)(env_base + i), episode, dr);
        env_reset_f32(s, dr, ob);
        for (int k = 0; k < 8; ++k) state[k * n + i] = s[k];
    }
}
