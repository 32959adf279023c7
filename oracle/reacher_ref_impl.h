/* ORACLE (test infrastructure only) -- textually included by reacher_ref.c once per
 * precision with REAL / SFX defined.  Same restatement as oracle/reacher_np.py
 * (MuJoCo 1.50 RK4 Reacher-v2), plain C, one env per loop iteration.
 * Never linked into the product library.
 */
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)
#define FN(name) CAT(name, SFX)

static inline void FN(qacc_)(REAL q1, REAL v0, REAL v1, REAL c0, REAL c1, REAL* a0o, REAL* a1o) {
    const REAL A0 = (REAL)RDO_A0, I2 = (REAL)RDO_I2, HC = (REAL)RDO_HC;
    REAL c = COS(q1), s = SIN(q1);
    REAL m11 = A0 + I2 + (REAL)2 * HC * c + (REAL)1;
    REAL m12 = I2 + HC * c;
    REAL m22 = I2 + (REAL)1;
    REAL b0 = -HC * s * ((REAL)2 * v0 * v1 + v1 * v1);
    REAL b1 = HC * s * v0 * v0;
    REAL cc0 = c0 < (REAL)-1 ? (REAL)-1 : (c0 > (REAL)1 ? (REAL)1 : c0);
    REAL cc1 = c1 < (REAL)-1 ? (REAL)-1 : (c1 > (REAL)1 ? (REAL)1 : c1);
    REAL t0 = (REAL)200 * cc0 - v0 - b0;
    REAL t1 = (REAL)200 * cc1 - v1 - b1;
    REAL det = m11 * m22 - m12 * m12;
    REAL i11 = m22 / det, i12 = -m12 / det, i22 = m11 / det;
    REAL a0 = i11 * t0 + i12 * t1;
    REAL a1 = i12 * t0 + i22 * t1;
    REAL lower = q1 + (REAL)3, upper = (REAL)3 - q1;
    if (lower < 0 || upper < 0) {
        REAL dist = lower < 0 ? lower : upper;
        REAL J = lower < 0 ? (REAL)1 : (REAL)-1;
        REAL x = FABS(dist) / (REAL)0.001;
        if (x > 1) x = 1;
        REAL y = x <= (REAL)0.5 ? (REAL)2 * x * x : (REAL)1 - (REAL)2 * (1 - x) * (1 - x);
        REAL d = (REAL)0.9 + y * (REAL)0.05;
        REAL aref = -(REAL)RDO_BREF * (J * v1) - (REAL)RDO_KREF * d * dist;
        REAL R = (1 - d) / d * (REAL)RDO_INVW0;
        REAL f = (aref - J * a1) / (i22 + R);
        if (f < 0) f = 0;
        a0 += i12 * J * f;
        a1 += i22 * J * f;
    }
    *a0o = a0;
    *a1o = a1;
}

/* One env.step (2 x mj_step RK4).  s[0..7] = q0,q1,v0,v1,tx,ty,dx,dy where (dx,dy) is
 * fingertip-target at the kinematics MuJoCo holds (stale stage-4 position).
 * Writes obs[11], returns reward.  Reward uses the incoming (dx,dy) and float32 ctrl cost. */
static inline REAL FN(env_step_)(REAL* s, float a0f, float a1f, REAL* obs) {
    const REAL h = (REAL)0.01;
    REAL q0 = s[0], q1 = s[1], v0 = s[2], v1 = s[3], tx = s[4], ty = s[5];
    float ctrl = a0f * a0f + a1f * a1f;                       /* float32 like gym */
    REAL r = -SQRT(s[6] * s[6] + s[7] * s[7]) - (REAL)ctrl;
    REAL c0 = (REAL)a0f, c1 = (REAL)a1f;
    REAL kq0 = q0, kq1 = q1;
    for (int sub = 0; sub < 2; ++sub) {
        REAL k1a, k1b, k2a, k2b, k3a, k3b, k4a, k4b;
        FN(qacc_)(q1, v0, v1, c0, c1, &k1a, &k1b);
        REAL v0b = v0 + h * ((REAL)0.5 * k1a), v1b = v1 + h * ((REAL)0.5 * k1b);
        REAL q1b = q1 + h * ((REAL)0.5 * v1);
        FN(qacc_)(q1b, v0b, v1b, c0, c1, &k2a, &k2b);
        REAL v0c = v0 + h * ((REAL)0.5 * k2a), v1c = v1 + h * ((REAL)0.5 * k2b);
        REAL q1c = q1 + h * ((REAL)0.5 * v1b);
        FN(qacc_)(q1c, v0c, v1c, c0, c1, &k3a, &k3b);
        REAL v0d = v0 + h * k3a, v1d = v1 + h * k3b;
        kq0 = q0 + h * v0c;
        kq1 = q1 + h * v1c;
        FN(qacc_)(kq1, v0d, v1d, c0, c1, &k4a, &k4b);
        const REAL b1 = (REAL)1 / (REAL)6, b2 = (REAL)1 / (REAL)3;
        REAL dq0 = v0 * b1 + v0b * b2 + v0c * b2 + v0d * b1;
        REAL dq1 = v1 * b1 + v1b * b2 + v1c * b2 + v1d * b1;
        REAL dv0 = k1a * b1 + k2a * b2 + k3a * b2 + k4a * b1;
        REAL dv1 = k1b * b1 + k2b * b2 + k3b * b2 + k4b * b1;
        q0 += h * dq0;
        q1 += h * dq1;
        v0 += h * dv0;
        v1 += h * dv1;
    }
    REAL fx = (REAL)0.1 * COS(kq0) + (REAL)0.11 * COS(kq0 + kq1);
    REAL fy = (REAL)0.1 * SIN(kq0) + (REAL)0.11 * SIN(kq0 + kq1);
    s[0] = q0; s[1] = q1; s[2] = v0; s[3] = v1;
    s[6] = fx - tx; s[7] = fy - ty;
    obs[0] = COS(q0); obs[1] = COS(q1); obs[2] = SIN(q0); obs[3] = SIN(q1);
    obs[4] = tx; obs[5] = ty; obs[6] = v0; obs[7] = v1;
    obs[8] = s[6]; obs[9] = s[7]; obs[10] = 0;
    return r;
}

/* reset_model + set_state + sim.forward(): fresh kinematics */
static inline void FN(env_reset_)(REAL* s, const REAL* draw, REAL* obs) {
    REAL q0 = draw[0], q1 = draw[1];
    s[0] = q0; s[1] = q1; s[2] = draw[2]; s[3] = draw[3]; s[4] = draw[4]; s[5] = draw[5];
    REAL fx = (REAL)0.1 * COS(q0) + (REAL)0.11 * COS(q0 + q1);
    REAL fy = (REAL)0.1 * SIN(q0) + (REAL)0.11 * SIN(q0 + q1);
    s[6] = fx - s[4]; s[7] = fy - s[5];
    obs[0] = COS(q0); obs[1] = COS(q1); obs[2] = SIN(q0); obs[3] = SIN(q1);
    obs[4] = s[4]; obs[5] = s[5]; obs[6] = s[2]; obs[7] = s[3];
    obs[8] = s[6]; obs[9] = s[7]; obs[10] = 0;
}

/* Batched, SoA state [8][n]; act [n][2] float32; obs [n][11]; rew [n]. */
void FN(rdo_step_)(int64_t n, REAL* state, const float* act, REAL* obs, REAL* rew) {
#pragma omp parallel for schedule(static) if (n >= 1024)
    for (int64_t i = 0; i < n; ++i) {
        REAL s[8];
        for (int k = 0; k < 8; ++k) s[k] = state[k * n + i];
        rew[i] = FN(env_step_)(s, act[2 * i], act[2 * i + 1], obs + 11 * i);
        for (int k = 0; k < 8; ++k) state[k * n + i] = s[k];
    }
}

/* draws [n][6] = (q0,q1,v0,v1,tx,ty) */
void FN(rdo_reset_)(int64_t n, REAL* state, const REAL* draws, REAL* obs) {
#pragma omp parallel for schedule(static) if (n >= 1024)
    for (int64_t i = 0; i < n; ++i) {
        REAL s[8];
        FN(env_reset_)(s, draws + 6 * i, obs + 11 * i);
        for (int k = 0; k < 8; ++k) state[k * n + i] = s[k];
    }
}

#undef FN
#undef CAT
#undef CAT2
