// Reacher-v2 (gym 0.10.5 on MuJoCo 1.50) dynamics for gfx950: device-side, f32,
// one environment per lane.  Restates what the reference's env.step()/env.reset()
// execute inside mujoco-py (reference mlp_train.py:112,135,138,196,200 ->
// gym ReacherEnv.step -> do_simulation(a, frame_skip=2) -> 2 x mj_step(RK4)).
//
// Model (pinned against src/distilation/tests/data/dataset.json):
//   M(q1)   = [[A0+I2+2HC cos q1 + 1, I2 + HC cos q1], [., I2 + 1]]   (armature 1)
//   bias    = HC sin q1 * [-(2 v0 v1 + v1^2), v0^2]                    (RNE)
//   tau     = 200 clip(a,-1,1) - v - bias                               (gear, damping 1)
//   joint-1 limit +-3: one soft constraint, solref (.02,1), solimp (.9,.95,.001),
//   R = (1-d)/d * invweight0 -- solved exactly (scalar).
//   RK4 (h = .01), kinematics left at the last stage (stale fingertip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rd {

// Rounding fixed by the source, not by the inlining context: within these functions a * b + c
// fuses into one FMA only inside one expression (clang fp contract "on"), never across
// statements by the backend (-ffp-contract=fast-honor-pragmas, HIP's default).  So every kernel
// that inlines the env step -- the fused rollout's K = 1 and K-step instances, the helper pairs,
// the gym-API env kernel, PPO's rollout -- rounds it identically (bitwise the same states).
#define FP_SOURCE_ROUNDING() _Pragma("clang fp contract(on)")

// ------------------------------------------------------------------ constants
constexpr double kPi = 3.14159265358979323846;
constexpr double kMl = 1000.0 * kPi * 0.01 * 0.01 * 0.11;
constexpr double kIc = kMl * (3 * 0.01 * 0.01 + 0.11 * 0.11) / 12.0;
constexpr double kMf = 1000.0 * 4.0 / 3.0 * kPi * 0.01 * 0.01 * 0.01;
constexpr double kIf = 0.4 * kMf * 0.01 * 0.01;
constexpr double kA0 = kIc + kMl * 0.05 * 0.05 + (kMl + kMf) * 0.1 * 0.1;
constexpr double kI2 = kIc + kMl * 0.05 * 0.05 + kIf + kMf * 0.11 * 0.11;
constexpr double kHC = 0.1 * (kMl * 0.05 + kMf * 0.11);
constexpr double kM110 = kA0 + kI2 + 2 * kHC + 1.0;
constexpr double kM120 = kI2 + kHC;
constexpr double kM220 = kI2 + 1.0;
constexpr double kInvW0 = kM110 / (kM110 * kM220 - kM120 * kM120);
constexpr double kBref = 2.0 / (0.95 * 0.02);
constexpr double kKref = 1.0 / (0.95 * 0.95 * 0.02 * 0.02);

constexpr int kEpisodeSteps = 50;   // gym TimeLimit (reference config.py:17 EPISODE_STEPS)
constexpr int kObsDim = 11;         // reference config.py:19 OBSPACE_SHAPE
constexpr int kActDim = 2;          // reference config.py:20 ACSPACE_SHAPE
constexpr int kStateDim = 8;        // q0 q1 v0 v1 tx ty dx dy (SoA rows)

struct State {
    float q0, q1, v0, v1, tx, ty, dx, dy;   // (dx,dy) = fingertip - target at the held kinematics
};

// sin and cos together for the joint angles.  Cody-Waite reduction by pi/2 with a 3-part
// constant (fma, exact k*C1 for |x| < 8192 rad) and Cephes' minimax polynomials on
// [-pi/4, pi/4]: <= 2 ulp, ~20 VALU instead of the ~45 of the libm path.  With kWideRange
// larger arguments take the libm path; the fused rollout (kWideRange = false) only sees
// angles of episodes at most 50 steps old (|q| < ~200 rad).
template <bool kWideRange = true>
__device__ __forceinline__ void sincos_acc(float x, float* s, float* c) {
    FP_SOURCE_ROUNDING();
    if (kWideRange && __builtin_expect(fabsf(x) > 8192.0f, 0)) {
        sincosf(x, s, c);
        return;
    }
    const float k = rintf(x * 0.636619772367581343f);          // 2/pi
    float r = __fmaf_rn(k, -1.5703125f, x);                     // exact: k*1.5703125 fits
    r = __fmaf_rn(k, -4.837512969970703125e-4f, r);
    r = __fmaf_rn(k, -7.54978995489188216e-8f, r);
    const float z = r * r;
    float ps = __fmaf_rn(-1.9515295891e-4f, z, 8.3321608736e-3f);
    ps = __fmaf_rn(ps, z, -1.6666654611e-1f);
    const float sr = __fmaf_rn(ps * z, r, r);
    float pc = __fmaf_rn(2.443315711809948e-5f, z, -1.388731625493765e-3f);
    pc = __fmaf_rn(pc, z, 4.166664568298827e-2f);
    const float cr = __fmaf_rn(pc * z, z, __fmaf_rn(-0.5f, z, 1.0f));
    const int q = (int)k & 3;
    const float sv = (q & 1) ? cr : sr;
    const float cv = (q & 1) ? sr : cr;
    *s = (q & 2) ? -sv : sv;
    *c = ((q + 1) & 2) ? -cv : cv;
}


// sin and cos of a JOINT-1 angle (q1, the RK4 stage angles, the held kinematics' kq1): the
// hardware v_sin_f32 / v_cos_f32 (argument in revolutions).  Joint 1 is limited to +-3 rad (a soft
// constraint: |q1| stays below ~3.2), where |error| <= 3.5e-7 (scripts/micro/trig_acc.hip; 9e-8
// for sincos_acc): in the dynamics sin/cos(q1) enter M(q1) and the bias only through HC = 2.2e-4
// beside the armature-dominated diagonal (a < 1e-10 relative change), in the fingertip and the
// observation 0.11 sin / cos(q0 + q1) and sin / cos(q1) directly (< 4e-8 and 3.5e-7 absolute) --
// 3 VALU instead of ~23.  Joint 0 is unlimited (|q0| reaches tens of rad within an episode, where
// the hardware's f32 argument scaling alone costs ~|q0| 2^-24 rev): sincos_q0 reduces it first.
// kWideRange (the gym-API env, whose states a caller may set): beyond |q1| = 4 rad -- past the
// joint's limit, where that scaling error would grow to ~|q1| 2^-24 2 pi (3e-5 at 512 rad) --
// sincos_q0's 2-pi reduction (and its libm path beyond 8192 rad).
template <bool kWideRange = true>
__device__ __forceinline__ void sincos_q0(float x, float* s, float* c);
template <bool kWideRange = true>
__device__ __forceinline__ void sincos_q1(float x, float* s, float* c) {
    FP_SOURCE_ROUNDING();
    if (kWideRange && __builtin_expect(fabsf(x) > 4.0f, 0)) {
        sincos_q0<true>(x, s, c);
        return;
    }
    const float r = x * 0.159154943091895336f;   // 1 / (2 pi)
    *s = __builtin_amdgcn_sinf(r);
    *c = __builtin_amdgcn_cosf(r);
}

// sin and cos of a JOINT-0 angle (the observation's q0, the held kinematics' kq0): joint 0 is
// unlimited, so the angle is first reduced by 2 pi (Cody-Waite, two constants: k 6.28125 is exact
// for |k| < 2^16, the second constant's rounding costs |k| 1e-10) to |r| <= pi, then the hardware
// v_sin_f32 / v_cos_f32 of r in revolutions: |error| <= 3.5e-7 at any |q0| below 8192 rad (the
// measured bound of sincos_q1's range), 9 VALU instead of ~23 for sincos_acc.  kWideRange: beyond
// 8192 rad the libm path, as sincos_acc.  (env_reset keeps sincos_acc: once per episode.)
template <bool kWideRange>
__device__ __forceinline__ void sincos_q0(float x, float* s, float* c) {
    FP_SOURCE_ROUNDING();
    if (kWideRange && __builtin_expect(fabsf(x) > 8192.0f, 0)) {
        sincosf(x, s, c);
        return;
    }
    const float k = rintf(x * 0.159154943091895336f);     // 1 / (2 pi)
    float r = __fmaf_rn(k, -6.28125f, x);                  // exact product
    r = __fmaf_rn(k, -1.9353071795864769e-3f, r);          // 2 pi - 6.28125
    const float u = r * 0.159154943091895336f;             // |u| <= 0.5 revolutions
    *s = __builtin_amdgcn_sinf(u);
    *c = __builtin_amdgcn_cosf(u);
}

// The joint angles the kWideRange = false paths (the fused rollout) are exact for: joint 1 on the
// hardware within its limit (+-3, soft: an episode stays within ~3.3), joint 0 reduced by 2 pi
// below 8192 rad (an episode's 50 steps stay within ~200 rad).  rdd_set_env_state rejects a
// caller's state outside them.
constexpr float kRolloutMaxQ0 = 8192.0f;
constexpr float kRolloutMaxQ1 = 4.0f;

// One MuJoCo forward pass -> constrained qacc of the two arm dofs; (s, c) = sin, cos q1.
__device__ __forceinline__ void qacc_sc(float q1, float s, float c, float v0, float v1, float c0, float c1,
                                        float& a0, float& a1) {
    FP_SOURCE_ROUNDING();
    const float A0 = (float)kA0, I2 = (float)kI2, HC = (float)kHC;
    const float m11 = A0 + I2 + 2.0f * HC * c + 1.0f;
    const float m12 = I2 + HC * c;
    const float m22 = I2 + 1.0f;
    const float b0 = -HC * s * (2.0f * v0 * v1 + v1 * v1);
    const float b1 = HC * s * v0 * v0;
    const float t0 = 200.0f * c0 - v0 - b0;
    const float t1 = 200.0f * c1 - v1 - b1;
    const float rdet = __builtin_amdgcn_rcpf(m11 * m22 - m12 * m12);   // 1 ulp
    const float i11 = m22 * rdet, i12 = -m12 * rdet, i22 = m11 * rdet;
    a0 = i11 * t0 + i12 * t1;
    a1 = i12 * t0 + i22 * t1;
    const float lower = q1 + 3.0f, upper = 3.0f - q1;
    if (lower < 0.0f || upper < 0.0f) {               // rare: joint-1 limit active
        const bool lo = lower < 0.0f;
        const float dist = lo ? lower : upper;
        const float J = lo ? 1.0f : -1.0f;
        const float x = fminf(fabsf(dist) * 1000.0f, 1.0f);
        const float y = x <= 0.5f ? 2.0f * x * x : 1.0f - 2.0f * (1.0f - x) * (1.0f - x);
        const float d = 0.9f + y * 0.05f;
        const float aref = -(float)kBref * (J * v1) - (float)kKref * d * dist;
        const float R = (1.0f - d) * __builtin_amdgcn_rcpf(d) * (float)kInvW0;
        const float f = fmaxf(0.0f, (aref - J * a1) * __builtin_amdgcn_rcpf(i22 + R));
        a0 += i12 * J * f;
        a1 += i22 * J * f;
    }
}

template <bool kWideRange = true>
__device__ __forceinline__ void qacc(float q1, float v0, float v1, float c0, float c1, float& a0, float& a1) {
    FP_SOURCE_ROUNDING();
    float s, c;
    sincos_q1<kWideRange>(q1, &s, &c);
    qacc_sc(q1, s, c, v0, v1, c0, c1, a0, a1);
}

// env.step on one env: returns the reward (computed from the held stale fingertip,
// float32 ctrl cost of the UNCLIPPED action), advances the state by 2 RK4 substeps.
template <bool kWideRange = true>
__device__ __forceinline__ float env_step(State& st, float a0, float a1) {
    FP_SOURCE_ROUNDING();
    const float h = 0.01f;
    const float r = -__builtin_amdgcn_sqrtf(st.dx * st.dx + st.dy * st.dy) - (a0 * a0 + a1 * a1);   // 1 ulp
    const float c0 = fminf(fmaxf(a0, -1.0f), 1.0f);   // ctrlrange +-1 (ctrllimited)
    const float c1 = fminf(fmaxf(a1, -1.0f), 1.0f);
    float q0 = st.q0, q1 = st.q1, v0 = st.v0, v1 = st.v1;
    float kq0 = q0, kq1 = q1, s4 = 0.0f, c4 = 1.0f;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
        float k1a, k1b, k2a, k2b, k3a, k3b, k4a, k4b;
        qacc<kWideRange>(q1, v0, v1, c0, c1, k1a, k1b);
        const float v0b = v0 + h * (0.5f * k1a), v1b = v1 + h * (0.5f * k1b);
        qacc<kWideRange>(q1 + h * (0.5f * v1), v0b, v1b, c0, c1, k2a, k2b);
        const float v0c = v0 + h * (0.5f * k2a), v1c = v1 + h * (0.5f * k2b);
        qacc<kWideRange>(q1 + h * (0.5f * v1b), v0c, v1c, c0, c1, k3a, k3b);
        const float v0d = v0 + h * k3a, v1d = v1 + h * k3b;
        kq0 = q0 + h * v0c;
        kq1 = q1 + h * v1c;
        sincos_q1<kWideRange>(kq1, &s4, &c4);   // also the held kinematics' q1 after the 2nd substep
        qacc_sc(kq1, s4, c4, v0d, v1d, c0, c1, k4a, k4b);
        const float b1 = 1.0f / 6.0f, b2 = 1.0f / 3.0f;
        q0 += h * (v0 * b1 + v0b * b2 + v0c * b2 + v0d * b1);
        q1 += h * (v1 * b1 + v1b * b2 + v1c * b2 + v1d * b1);
        v0 += h * (k1a * b1 + k2a * b2 + k3a * b2 + k4a * b1);
        v1 += h * (k1b * b1 + k2b * b2 + k3b * b2 + k4b * b1);
    }
    float s0, c0k;
    sincos_q0<kWideRange>(kq0, &s0, &c0k);
    const float s01 = __fmaf_rn(s0, c4, c0k * s4);    // sin(kq0 + kq1)
    const float c01 = __fmaf_rn(c0k, c4, -s0 * s4);   // cos(kq0 + kq1)
    st.q0 = q0; st.q1 = q1; st.v0 = v0; st.v1 = v1;
    st.dx = 0.1f * c0k + 0.11f * c01 - st.tx;
    st.dy = 0.1f * s0 + 0.11f * s01 - st.ty;
    return r;
}

// reset_model + set_state + sim.forward(): kinematics fresh at the reset position.
__device__ __forceinline__ void env_reset(State& st, const float* d /*q0 q1 v0 v1 tx ty*/) {
    FP_SOURCE_ROUNDING();
    st.q0 = d[0]; st.q1 = d[1]; st.v0 = d[2]; st.v1 = d[3]; st.tx = d[4]; st.ty = d[5];
    float s0, c0, s01, c01;
    sincos_acc(st.q0, &s0, &c0);
    sincos_acc(st.q0 + st.q1, &s01, &c01);
    st.dx = 0.1f * c0 + 0.11f * c01 - st.tx;
    st.dy = 0.1f * s0 + 0.11f * s01 - st.ty;
}

// gym ReacherEnv._get_obs: [cos q, sin q, target, qvel, fingertip - target (x,y,0)]
template <bool kWideRange = true>
__device__ __forceinline__ void observe(const State& st, float* ob) {
    FP_SOURCE_ROUNDING();
    float s0, c0, s1, c1;
    sincos_q0<kWideRange>(st.q0, &s0, &c0);
    sincos_q1<kWideRange>(st.q1, &s1, &c1);
    ob[0] = c0; ob[1] = c1; ob[2] = s0; ob[3] = s1;
    ob[4] = st.tx; ob[5] = st.ty; ob[6] = st.v0; ob[7] = st.v1;
    ob[8] = st.dx; ob[9] = st.dy; ob[10] = 0.0f;
}

// ------------------------------------------------------------------ Philox4x32-10
// Synthetic reset stream: key = seed, counter = (env_id lo, env_id hi, episode, block).
__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                       uint32_t k0, uint32_t k1, uint32_t out[4]) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// draws (q0,q1,v0,v1,tx,ty) with ReacherEnv.reset_model's ranges
__device__ __forceinline__ void philox_draw(uint64_t seed, uint64_t env_id, uint32_t episode, float d[6]) {
    FP_SOURCE_ROUNDING();
    uint32_t o[4], p[4];
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    philox((uint32_t)env_id, (uint32_t)(env_id >> 32), episode, 0u, k0, k1, o);
    philox((uint32_t)env_id, (uint32_t)(env_id >> 32), episode, 1u, k0, k1, p);
    d[0] = __fmaf_rn(0.2f, u01(o[0]), -0.1f);
    d[1] = __fmaf_rn(0.2f, u01(o[1]), -0.1f);
    d[2] = __fmaf_rn(0.01f, u01(o[2]), -0.005f);
    d[3] = __fmaf_rn(0.01f, u01(o[3]), -0.005f);
    d[4] = __fmaf_rn(0.4f, u01(p[0]), -0.2f);
    d[5] = __fmaf_rn(0.4f, u01(p[1]), -0.2f);
}

}  // namespace rd
