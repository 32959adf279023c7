// Fused rollout + distillation step for gfx950 (include/reacher_distill.h).
//
// One launch of rollout_kernel runs, for every env, one iteration of the reference's hot
// loop (mlp_train.py:143-204): observation -> teacher MlpPolicy (teacher.py:14-16) ->
// student MlpPolicy -> loss (loss.py:3-13 KL, or action-MSE) -> student backward ->
// env.step(action) with auto-reset; per-workgroup gradient partials go to a workspace.
// reduce_adam_kernel then sums the partials and applies TF1 Adam (mlp_train.py:73-80).
//
// MI355X mapping:
//  * 512-thread workgroups (8 waves = 2 per SIMD, <= 256 VGPR+AGPR each) so that one
//    wave's VALU work (physics, tanh, staging) issues while its SIMD partner's MFMAs run.
//  * a wave owns a GROUP of 64 envs: the physics runs once per env (one env per lane);
//    the networks run on 16-env TILES (4 per group) with v_mfma_f32_16x16x4_f32 in the
//    transposed orientation Z^T[feature x env] = W^T[feature x in] . X^T[in x env]:
//    lane l = (env j = l&15, k-group g = l>>4); a layer's accumulator (features 4g+r in
//    registers, env on the lane) IS the B operand of the next layer (k-step r uses the
//    features {4g + r}), so activations never leave registers in the forward/backward
//    chain.  Layer-1 bias rides in the K padding (input 11 = 1).
//  * weights of both nets live in LDS for the whole launch as [k][j][fb] images (one
//    conflict-free ds_read_b128 feeds the 4 MFMAs of a k-step, prefetched a step ahead);
//    the student also keeps W2^T for dH1 = W2 . dZ2.
//  * weight gradients (sums over envs) are MFMAs with the env as K: H1, dZ2 and dZ1 are
//    transposed through a per-wave LDS scratch (private to the wave: ordered by a
//    wave-level barrier, never s_barrier); accumulators persist across the wave's tiles
//    and are reduced once per workgroup, in a fixed order (deterministic).
//  * exact f32 arithmetic throughout (f32-input MFMA = k-ordered fmaf chain).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <new>

#include "../../include/reacher_distill.h"
#include "rd_comm_impl.h"
#include "rd_common.h"
#include "rd_physics.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int OBD = 11, HID = 64, ACD = 2;
constexpr int P_W1 = 0;
constexpr int P_B1 = P_W1 + OBD * HID;   // 704
constexpr int P_W2 = P_B1 + HID;         // 768
constexpr int P_B2 = P_W2 + HID * HID;   // 4864
constexpr int P_W3 = P_B2 + HID;         // 4928
constexpr int P_B3 = P_W3 + HID * ACD;   // 5056
constexpr int P_LS = P_B3 + ACD;         // 5058
constexpr int P_TOT = P_LS + ACD;        // 5060
constexpr int P_PAD = P_TOT + 4;         // + metrics: reward, loss, sq err, envs
constexpr int N_MET = 4;

constexpr int WAVES = 8, BLOCK = 64 * WAVES;   // rollout: 2 waves per SIMD
constexpr int FWAVES = 4, FBLOCK = 64 * FWAVES; // forward_kernel
constexpr int GROUP = 64;                      // envs per wave pass (one per lane)
constexpr int TILE = 16;                       // envs per MFMA tile

// ---------------------------------------------------------------- LDS image of a net
// Weight images are [k][j][fb] = W[k][16 fb + j]: the four A operands a lane needs for one
// k-step (output blocks fb = 0..3, row j) are one 16-B ds_read_b128, and a 16-lane group
// reads one contiguous 256-B row: conflict-free, no padding.
constexpr int N_W1 = 0;                  // [12][16][4]: rows 0..10 = W1, row 11 = b1
constexpr int N_W2 = N_W1 + 12 * HID;    // [64][16][4]
constexpr int N_B2 = N_W2 + HID * HID;   // [64]
constexpr int N_W3 = N_B2 + HID;         // [64][2]
constexpr int N_B3 = N_W3 + HID * ACD;   // [2]
constexpr int N_LS = N_B3 + ACD;         // [2]
constexpr int N_MU = N_LS + ACD;         // [12] filter mean (0 for the bias input 11)
constexpr int N_RS = N_MU + 12;          // [12] 1/std     (1 for the bias input 11)
constexpr int NET = (N_RS + 12 + 3) & ~3;
constexpr int N_W2T = NET;               // student only: [j][i&15][i>>4] = W2[i][j]
constexpr int NET_S = NET + HID * HID;
static_assert(N_B2 % 4 == 0 && N_W3 % 4 == 0 && NET % 4 == 0, "16-B aligned LDS vectors");

// ---------------------------------------------------------------- per-pair scratch
// Waves w and w + 4 of a workgroup share a SIMD.  They form a PAIR with fixed roles:
// the producer (w < 4) computes observations, teacher and student forwards, the loss and
// dZ2; the consumer (w + 4) computes the weight gradients and dH1/dZ1 and steps the envs.
// They hand over one 16-env tile at a time through an LDS slot guarded by two counters.
constexpr int PAIRS = WAVES / 2;
constexpr int SOS = 12;                         // raw obs rows (11 + the bias input = 1)
constexpr int SAS = 68;                         // transposed activation rows [env][64 + pad]
constexpr int P_SO = 0;                         // [64][12] raw obs of the producer's group (its own)
constexpr int P_ACT = P_SO + GROUP * SOS;       // [64][2] actions (the producer's env step)
constexpr int P_H1T = P_ACT + GROUP * 2;        // slot: H1^T [16][SAS]
constexpr int P_DZT = P_H1T + TILE * SAS;       // slot: dZ2^T [16][SAS]
constexpr int P_SA = P_DZT + TILE * SAS;        // consumer-private: dZ1^T [16][SAS]
constexpr int P_SOB = P_SA + TILE * SAS;        // slot: the tile's raw obs rows [16][12] (the consumer's dW1 inputs)
constexpr int P_SACT = P_SOB + TILE * SOS;      // slot: the tile's actions [16][2] (CP: for the consumer's env step)
constexpr int P_FLAGS = P_SACT + TILE * 2;      // u32 [0] tiles published [1] tiles consumed
constexpr int PSCR = P_FLAGS + 4;
constexpr int LDS_FLOATS = NET + NET_S + PAIRS * PSCR;
static_assert(LDS_FLOATS * 4 <= 160 * 1024, "LDS budget");
static_assert(PSCR % 4 == 0 && P_H1T % 4 == 0 && P_DZT % 4 == 0 && P_SA % 4 == 0 && P_SOB % 4 == 0,
              "16-B aligned scratch");
// Final per-workgroup reduction: pair p fills LDS region p.  The 76 rows of 64 that hold
// W1 (with b1 as row 11) and W2 are stored with a row stride of 68 floats, so that the
// consumer's register-layout writes (lane (g, j) -> row 4g + r, column j) hit 64 distinct
// banks; everything after W2 follows at +304 (region of RPAD floats).
constexpr int RROW = 68;
constexpr int RSHIFT = (P_B2 / HID) * (RROW - HID);   // 304
constexpr int RPAD = P_PAD + RSHIFT;
static_assert(P_B1 == P_W1 + OBD * HID && P_W2 == P_B1 + HID && P_B2 % HID == 0, "W1|b1|W2 rows");
static_assert(PAIRS * RPAD <= LDS_FLOATS && RPAD % 4 == 0 && P_PAD % 4 == 0, "final reduction must fit in the LDS");
__device__ __forceinline__ int ridx(int p) { return p < P_B2 ? (p >> 6) * RROW + (p & 63) : p + RSHIFT; }
[[maybe_unused]] constexpr int NSTAMP = 24;                      // RD_STAMPS debug slots per wave (scripts/stamps.py)
constexpr uint32_t SPIN_LIMIT = 1u << 22;       // ~0.1 s of s_sleep: a broken hand-off ends the launch

// ctl words: [0] env steps C (the episode clocks), [1] optimiser steps S (metrics ring),
// [2] beta1^S, [3] beta2^S (f32 bits); [4..7] the rollout's snapshot of [0..3], which this
// kernel reads so that block 0 may rewrite [0..3] without racing the other blocks (no
// atomics, no fences: stream order suffices); [8] hand-off timeout; [12] 1 if the last
// rollout stepped the envs.
struct ReduceArgs {
    const float* ws;
    int nblk;
    float* grad;       // [P]
    float* params;     // student params [P] (in the student net buffer)
    float* m;
    float* v;
    uint32_t* ctl;
    float* hist;       // [hist_len][4]
    int hist_len;
    int reduce, adam, accum;   // accum: grad (and the metrics slot) += this rollout's sums
    int bump_env, bump_opt;    // advance the env clock (after a reduce) / the optimiser step
    float lr, b1, b2, eps;
    float* simg;       // student LDS image, refreshed with every updated parameter
    int img_kind;      // IMG_F32 / IMG_SPLIT / IMG_BF16
    const uint32_t* xerr;   // bound exchange's failure word (xGMI) or null: nonzero = skip Adam
};

// The partials workspace is column-chunked: chunk c (params 32c .. 32c+31) holds the rows of
// every workgroup of the launch contiguously, [chunk][row][RED_COLS], one 128-B line per row,
// so one reduce block per chunk reads one contiguous run and the reduce spreads over 159
// blocks (with [row][P_PAD] rows a block needed 64 columns for 256-B segments: 80 blocks
// pulled c4's 5.2 MB of partials).  Bitwise the same sums (the row order per column depends
// on RED_ROWS only).  16-column chunks (317 blocks) make the rollout's stores half lines and
// cost it 5 us at c4 (profiles/r02_ws_chunked.txt).
constexpr int RED_COLS = 32;                        // params per reduce block = chunk width
constexpr int RED_ROWS = 16;                        // partial rows summed in parallel
constexpr int RED_BLOCK = RED_COLS * RED_ROWS;
constexpr int RED_GRID = (P_PAD + RED_COLS - 1) / RED_COLS;
constexpr int P_WS = RED_GRID * RED_COLS;           // workspace floats per partial row
__device__ __forceinline__ int64_t ws_index(int p, int row, int rows) {
    return ((int64_t)(p / RED_COLS) * rows + row) * RED_COLS + (p % RED_COLS);
}

struct RolloutArgs {
    int64_t n, env_base;
    uint64_t seed;
    float* state;                          // [8][n]
    const float* tnet;                     // teacher: params[P], mu[11], sd[11] (contiguous); in
                                           // distill_rows_kernel the rows' recorded teacher pdflat [n][4]
    const float* snet;                     // student
    uint32_t* ctl;                         // [0] completed steps, [4..7] snapshot
    float* ws;                             // [RED_GRID][gridDim.x][RED_COLS] (ws_index)
    int loss, act_student, stagger;
    float inv_n_global;
    int gs;                                // envs per group (16, 32 or 64)
    int ksteps;                            // env steps of this launch (rdd_step_accum: accum_steps)
    unsigned long long* dbg;               // RD_STAMPS builds: [grid*WAVES][NSTAMP] stamp sums
    const float* obs_in;                   // observation-batch mode: [n][11] rows, no env step
    const float* timg;                     // prepacked LDS images (pack_net_kernel)
    const float* simg;
};

// f32 MFMA.  FENCE: an empty asm that reads the result and clobbers memory follows it, so the
// MFMA has completed (the compiler waits for its result) before any later LDS / global load
// issues.  Needed wherever the compiler would otherwise issue a load into a register that an
// in-flight 8-pass v_mfma_f32_16x16x4_f32 still reads as SrcC: ROCm 7.2 protects that WAR
// for the XDL (bf16) MFMAs but emits such loads 0-1 wait states after the f32 form, and a
// load returning there is lost for the lanes of the MFMA's last row group (rows 12-15 =
// lanes 48-63) when the MFMA is still reading (found statically with
// scripts/isa/hazards.py, confirmed with profiles/r03_srcc_probe_*.txt; the consumer-side env
// step of the bf16-student kernel fences its teacher's f32 layer 1).  -DRD_MFMA_SRCC_FENCE
// fences every f32 MFMA (diagnostic builds).
__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// SrcC fence around a group of four f32 MFMAs (FENCE): the group's accumulators pass through
// an empty asm before and after it (so its MFMAs stay between them, and no load -- the asm
// clobbers memory -- moves into the group), and each result is read by a VALU before the
// closing asm, so the compiler waits for every MFMA of the group to complete first.
// Needed wherever the compiler would otherwise issue a load into a register that an in-flight
// 8-pass v_mfma_f32_16x16x4_f32 still reads as SrcC: ROCm 7.2 protects that WAR for the XDL
// (bf16) MFMAs but emits such loads 0-1 wait states after the f32 form, and a load returning
// there is lost for the lanes of the MFMA's last row group (rows 12-15 = lanes 48-63) while
// the MFMA still reads (found statically with scripts/isa/hazards.py, confirmed
// by profiles/r03_srcc_probe_*.txt).  The consumer-side-env-step kernels (bf16 student) fence
// their teacher's f32 MFMAs; -DRD_MFMA_SRCC_FENCE fences every group (diagnostic builds).
#ifdef RD_MFMA_SRCC_FENCE
constexpr bool kFenceAll = true;
#else
constexpr bool kFenceAll = false;
#endif
template <bool FENCE>
__device__ __forceinline__ void fence_begin(f32x4 (&acc)[4]) {   // the group's MFMAs read acc: they follow
    if constexpr (FENCE || kFenceAll)
        asm volatile("" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])::"memory");
}
template <bool FENCE>
__device__ __forceinline__ void fence_end(f32x4 (&acc)[4]) {   // every MFMA of the group precedes it
    if constexpr (FENCE || kFenceAll) {
#pragma unroll
        for (int fb = 0; fb < 4; ++fb) acc[fb][3] = __builtin_amdgcn_fmed3f(acc[fb][3], acc[fb][3], acc[fb][3]);
        asm volatile("" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])::"memory");
    }
}

// Forward weight images are pre-scaled by 2 log2(e), so a layer's accumulator is already
// y = 2 log2(e) z and tanh(z) = 1 - 2/(2^y + 1): v_exp_f32 + v_add + v_rcp_f32 + v_fma.
// (The backward only needs tanh's output; W2^T for dH1 keeps the unscaled weights.)
constexpr float kTanhScale = 2.8853900817779268f;
__device__ __forceinline__ float tanh_pre(float y) {
    return fmaf(-2.0f, __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(y) + 1.0f), 1.0f);
}
// tanh_pre on the four rows of an accumulator, as scalar VALU.  No packed-f32 forms: a
// v_pk_add/fma_f32 whose sources a later load overwrites before anything reads its result can
// lose lanes 48-63 (PKWAR), and in an MFMA gap a packed op costs more issue than
// the two scalar ones (MI355X_MICROARCH.md: +22 cycles for v_pk_fma_f32).  The rollout kernels
// contain no v_pk_*_f32 at all (tests/test_product_hygiene.py).
__device__ __forceinline__ f32x4 tanh4(f32x4 y) {
    return f32x4{tanh_pre(y[0]), tanh_pre(y[1]), tanh_pre(y[2]), tanh_pre(y[3])};
}

// The per-wave scratch is private to its wave: LDS instructions of one wave execute in
// issue order, so staging needs only a compiler-level barrier, not s_barrier.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// x + x from the partner row (lane ^ 16) / half (lane ^ 32): v_permlane16/32_swap (VALU,
// no LDS round trip).  Every lane gets the bitwise-identical sum.
__device__ __forceinline__ float xsum16(float x) {
    const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}
__device__ __forceinline__ float xsum32(float x) {
    const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// state row k of env i: (state + k n)[i] -- uniform 64-bit row base, 32-bit lane offset
__device__ __forceinline__ float ldst(const float* p) { return *p; }
__device__ __forceinline__ void load_state(const float* s, int64_t n, uint32_t i, rd::State& st) {
    st.q0 = ldst(s + 0 * n + i); st.q1 = ldst(s + 1 * n + i); st.v0 = ldst(s + 2 * n + i); st.v1 = ldst(s + 3 * n + i);
    st.tx = ldst(s + 4 * n + i); st.ty = ldst(s + 5 * n + i); st.dx = ldst(s + 6 * n + i); st.dy = ldst(s + 7 * n + i);
}

// Diagnostic build only (-DRD_STAMPS, libreacher_stamps.so): per-wave s_memtime stamps
// of the kernel's phases into a debug buffer nothing else reads.
#ifdef RD_STAMPS
#define STAMP(idx)                                                                      \
    do {                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                              \
        unsigned long long t_;                                                          \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");     \
        __builtin_amdgcn_sched_barrier(0);                                              \
        if (lane == 0 && a.dbg) a.dbg[(blockIdx.x * WAVES + wave) * NSTAMP + (idx)] += t_;   \
    } while (0)
// s_memrealtime (100 MHz) at kernel start/end: with the s_memtime stamps, the shader clock
#define RTSTAMP(idx)                                                                    \
    do {                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                              \
        const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                 \
        __builtin_amdgcn_sched_barrier(0);                                              \
        if (lane == 0 && a.dbg) a.dbg[(blockIdx.x * WAVES + wave) * NSTAMP + (idx)] += t_;   \
    } while (0)
#else
#define STAMP(idx) do {} while (0)
#define RTSTAMP(idx) do {} while (0)
#endif

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
// (a + b) + (c + d) per component as scalar adds (a vector add would be v_pk_add_f32)
__device__ __forceinline__ f32x4 sum4(f32x4 a, f32x4 b, f32x4 c, f32x4 d) {
    f32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (a[i] + b[i]) + (c[i] + d[i]);
    return r;
}
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

// Global stores, plain or non-temporal (NT).  The bf16-student kernels (c5) write the rollout's
// partial row NT (__builtin_nontemporal_store): the rows no longer wait dirty in the writer's L2
// for the end-of-kernel writeback, c5 -0.5 us per step; the f32-student kernels keep plain stores
// (neutral at c4, -0.25 us at c3, +0.25 at c2's 64 workgroups; DESIGN.md §3,
// profiles/r03k_nt_stores.txt, profiles/r03y_sched_nt.txt).  An inline-asm NT store that chose per
// launch made the first rollout of a process differ in one gradient entry and is gone
// (profiles/r03x_nt_asm_rejected.txt; no wait-state pair explains it, profiles/r04_r03x_isa.txt).
// NT state, reduce+Adam and all-kernel row stores measured no gain
// (profiles/r04_removed_diagnostic_variants.diff).
template <bool NT, class T>
__device__ __forceinline__ void gst(T* p, T v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
template <class T>
__device__ __forceinline__ void put(T* p, T v) { *p = v; }

// global net = params[P] | mu[11] | sd[11]  ->  LDS image (+ W2^T if `transposed`); the
// forward images of W1, b1, W2, b2 carry the tanh scale (kTanhScale)
__device__ void load_net(float* L, const float* g, bool transposed, int nthreads) {
    const float* mu = g + P_TOT;
    const float* sd = g + P_TOT + OBD;
    for (int i = threadIdx.x; i < 12 * HID; i += nthreads) {
        const int k = i >> 6, f = i & 63;
        L[N_W1 + k * HID + (f & 15) * 4 + (f >> 4)] = kTanhScale * (k < OBD ? g[P_W1 + i] : g[P_B1 + f]);
    }
    for (int i = threadIdx.x; i < HID * HID; i += nthreads) {
        const int k = i >> 6, f = i & 63;
        L[N_W2 + k * HID + (f & 15) * 4 + (f >> 4)] = kTanhScale * g[P_W2 + i];
    }
    if (transposed)   // k fastest across lanes: the LDS writes spread over the banks
        for (int i = threadIdx.x; i < HID * HID; i += nthreads) {
            const int f = i >> 6, k = i & 63;
            L[N_W2T + f * HID + (k & 15) * 4 + (k >> 4)] = g[P_W2 + k * HID + f];
        }
    for (int i = threadIdx.x; i < HID; i += nthreads) L[N_B2 + i] = kTanhScale * g[P_B2 + i];
    for (int i = threadIdx.x; i < HID * ACD; i += nthreads) L[N_W3 + i] = g[P_W3 + i];
    if (threadIdx.x < ACD) {
        L[N_B3 + threadIdx.x] = g[P_B3 + threadIdx.x];
        L[N_LS + threadIdx.x] = g[P_LS + threadIdx.x];
    }
    if (threadIdx.x < 12) {
        const int k = threadIdx.x;
        L[N_MU + k] = k < OBD ? mu[k] : 0.0f;
        L[N_RS + k] = k < OBD ? 1.0f / sd[k] : 1.0f;
    }
}

// MlpPolicy forward of the 16-env tile whose raw observations are rows ob[0..15] of the
// wave's obs scratch (row stride SOS, component 11 = 1).  Lane (j, g):
// H1, H2 = hidden activations, features 16 fb + 4 g + r of env j; (m0, m1) = action mean
// of env j (identical in the four k-groups).
template <bool FENCE = false>
__device__ __forceinline__ void mlp_forward(const float* L, const float* ob, int j, int g, f32x4 (&H1)[4],
                                            f32x4 (&H2)[4], float& m0, float& m1) {
    f32x4 acc[4];
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) acc[fb] = f32x4{0.f, 0.f, 0.f, 0.f};
    // layer 1: K = 12 (11 filtered inputs + the bias input), k-step s covers inputs 4s+g
#pragma unroll
    for (int s = 0; s < 3; ++s) {
        const int k = 4 * s + g;
        const float z = fminf(fmaxf((ob[j * SOS + k] - L[N_MU + k]) * L[N_RS + k], -5.0f), 5.0f);
        const f32x4 w = ld4(L + N_W1 + k * HID + 4 * j);
        fence_begin<FENCE>(acc);
#pragma unroll
        for (int fb = 0; fb < 4; ++fb) acc[fb] = mfma(w[fb], z, acc[fb]);
        fence_end<FENCE>(acc);
    }
#pragma unroll
    for (int fb = 0; fb < 4; ++fb)
        H1[fb] = tanh4(acc[fb]);
    // layer 2: K = 64; k-step (kb, r) uses features 16 kb + 4 g + r = this lane's H1[kb][r]
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) acc[fb] = ld4(L + N_B2 + 16 * fb + 4 * g);
    // A operands prefetched one k-step ahead (LDS latency vs 4 MFMAs of 32 cycles)
    f32x4 wn = ld4(L + N_W2 + (4 * g) * HID + 4 * j);
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const f32x4 w = wn;
            if (kb * 4 + r < 15) {
                const int kn = (r == 3) ? 16 * (kb + 1) + 4 * g : 16 * kb + 4 * g + r + 1;
                wn = ld4(L + N_W2 + kn * HID + 4 * j);
            }
            fence_begin<FENCE>(acc);
#pragma unroll
            for (int fb = 0; fb < 4; ++fb) acc[fb] = mfma(w[fb], H1[kb][r], acc[fb]);
            fence_end<FENCE>(acc);
        }
    float p0 = 0.0f, p1 = 0.0f;
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) {
        const f32x4 wa = ld4(L + N_W3 + (16 * fb + 4 * g) * 2);       // W3[f][0..1], f = 16fb+4g+0,1
        const f32x4 wb = ld4(L + N_W3 + (16 * fb + 4 * g) * 2 + 4);   // f = 16fb+4g+2,3
        H2[fb] = tanh4(acc[fb]);
        p0 = fmaf(H2[fb][0], wa[0], p0); p1 = fmaf(H2[fb][0], wa[1], p1);
        p0 = fmaf(H2[fb][1], wa[2], p0); p1 = fmaf(H2[fb][1], wa[3], p1);
        p0 = fmaf(H2[fb][2], wb[0], p0); p1 = fmaf(H2[fb][2], wb[1], p1);
        p0 = fmaf(H2[fb][3], wb[2], p0); p1 = fmaf(H2[fb][3], wb[3], p1);
    }
    p0 = xsum32(xsum16(p0));
    p1 = xsum32(xsum16(p1));
    m0 = p0 + L[N_B3];
    m1 = p1 + L[N_B3 + 1];
}

// Teacher and student forwards of one tile, interleaved layer by layer: 8 independent
// accumulator chains per layer, and one net's tanh can issue behind the other's MFMAs.
// Returns the student's hidden activations (needed by the backward) and both means.
// FENCE: every MFMA group SrcC-fenced; LAST: only layer 2's last k-step, whose results the
// tanh / W3 epilogue follows (hipcc hoists the W3 loads into that step's in-flight SrcC
// registers, hazards.py scan_ldsrc; layer 1's end is interlocked by its own tanh reads)
constexpr unsigned kPairFence = 0x8a00u;   // layer-2 k-steps 9, 11, 15 (below)
template <bool FENCE = false, unsigned FM = FENCE ? 0xffffu : 0u>
__device__ __forceinline__ void mlp_forward_pair(const float* LT, const float* LS, const float* ob, int j, int g,
                                                 f32x4 (&H1)[4], f32x4 (&H2)[4], float& mt0, float& mt1,
                                                 float& ms0, float& ms1) {
    f32x4 at[4], as[4];
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) at[fb] = as[fb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 3; ++s) {
        const int k = 4 * s + g;
        const float x = ob[j * SOS + k];
        const float zt = fminf(fmaxf((x - LT[N_MU + k]) * LT[N_RS + k], -5.0f), 5.0f);
        const float zs = fminf(fmaxf((x - LS[N_MU + k]) * LS[N_RS + k], -5.0f), 5.0f);
        const f32x4 wt = ld4(LT + N_W1 + k * HID + 4 * j);
        const f32x4 ws = ld4(LS + N_W1 + k * HID + 4 * j);
        fence_begin<FENCE>(at);
        fence_begin<FENCE>(as);
#pragma unroll
        for (int fb = 0; fb < 4; ++fb) {
            at[fb] = mfma(wt[fb], zt, at[fb]);
            as[fb] = mfma(ws[fb], zs, as[fb]);
        }
        fence_end<FENCE>(at);
        fence_end<FENCE>(as);
    }
    f32x4 T1[4];
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) {
        T1[fb] = tanh4(at[fb]);
        H1[fb] = tanh4(as[fb]);
    }
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) {
        at[fb] = ld4(LT + N_B2 + 16 * fb + 4 * g);
        as[fb] = ld4(LS + N_B2 + 16 * fb + 4 * g);
    }
    f32x4 wtn = ld4(LT + N_W2 + (4 * g) * HID + 4 * j);
    f32x4 wsn = ld4(LS + N_W2 + (4 * g) * HID + 4 * j);
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const f32x4 wt = wtn, ws = wsn;
            if (kb * 4 + r < 15) {
                const int kn = (r == 3) ? 16 * (kb + 1) + 4 * g : 16 * kb + 4 * g + r + 1;
                wtn = ld4(LT + N_W2 + kn * HID + 4 * j);
                wsn = ld4(LS + N_W2 + kn * HID + 4 * j);
            }
            if (FENCE || ((FM >> (kb * 4 + r)) & 1u)) {
                fence_begin<true>(at);
                fence_begin<true>(as);
            }
#pragma unroll
            for (int fb = 0; fb < 4; ++fb) {
                at[fb] = mfma(wt[fb], T1[kb][r], at[fb]);
                as[fb] = mfma(ws[fb], H1[kb][r], as[fb]);
            }
            if (FENCE || ((FM >> (kb * 4 + r)) & 1u)) {
                fence_end<true>(at);
                fence_end<true>(as);
            }
        }
    float pt0 = 0.0f, pt1 = 0.0f, ps0 = 0.0f, ps1 = 0.0f;
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) {
        const f32x4 ta = ld4(LT + N_W3 + (16 * fb + 4 * g) * 2), tb = ld4(LT + N_W3 + (16 * fb + 4 * g) * 2 + 4);
        const f32x4 sa = ld4(LS + N_W3 + (16 * fb + 4 * g) * 2), sb = ld4(LS + N_W3 + (16 * fb + 4 * g) * 2 + 4);
        f32x4 t2;
        t2 = tanh4(at[fb]);
        H2[fb] = tanh4(as[fb]);
        pt0 = fmaf(t2[0], ta[0], pt0); pt1 = fmaf(t2[0], ta[1], pt1);
        pt0 = fmaf(t2[1], ta[2], pt0); pt1 = fmaf(t2[1], ta[3], pt1);
        pt0 = fmaf(t2[2], tb[0], pt0); pt1 = fmaf(t2[2], tb[1], pt1);
        pt0 = fmaf(t2[3], tb[2], pt0); pt1 = fmaf(t2[3], tb[3], pt1);
        ps0 = fmaf(H2[fb][0], sa[0], ps0); ps1 = fmaf(H2[fb][0], sa[1], ps1);
        ps0 = fmaf(H2[fb][1], sa[2], ps0); ps1 = fmaf(H2[fb][1], sa[3], ps1);
        ps0 = fmaf(H2[fb][2], sb[0], ps0); ps1 = fmaf(H2[fb][2], sb[1], ps1);
        ps0 = fmaf(H2[fb][3], sb[2], ps0); ps1 = fmaf(H2[fb][3], sb[3], ps1);
    }
    mt0 = xsum32(xsum16(pt0)) + LT[N_B3];
    mt1 = xsum32(xsum16(pt1)) + LT[N_B3 + 1];
    ms0 = xsum32(xsum16(ps0)) + LS[N_B3];
    ms1 = xsum32(xsum16(ps1)) + LS[N_B3 + 1];
}

// ---------------------------------------------------------------- bf16 student (RDD_DTYPE_BF16)
// v_mfma_f32_16x16x32_bf16 (lane l: A[row l&15][k 8(l>>4)+jj], B[k 8(l>>4)+jj][col l&15],
// jj = 0..7) for the layers and dH1, v_mfma_f32_16x16x16_bf16 (k = 4(l>>4)+jj, jj = 0..3)
// where K is the tile's 16 envs (dW2, dW1).  C/D layout as the f32 forms.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma_k32(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_k16(s16x4 a, s16x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ unsigned short bf16_bits(float x) { return __builtin_bit_cast(unsigned short, (__bf16)x); }
__device__ __forceinline__ float bf16_round(float x) { return (float)(__bf16)x; }
__device__ __forceinline__ s16x4 pack4(float a, float b, float c, float d) {
    return s16x4{(short)bf16_bits(a), (short)bf16_bits(b), (short)bf16_bits(c), (short)bf16_bits(d)};
}
__device__ __forceinline__ bf16x8 pack8(f32x4 lo, f32x4 hi) {
    return bf16x8{(__bf16)lo[0], (__bf16)lo[1], (__bf16)lo[2], (__bf16)lo[3],
                  (__bf16)hi[0], (__bf16)hi[1], (__bf16)hi[2], (__bf16)hi[3]};
}
__device__ __forceinline__ bf16x8 ldbf8(const float* base, int half) {
    return *reinterpret_cast<const bf16x8*>(reinterpret_cast<const unsigned short*>(base) + half);
}

// Student image in the bf16 mode (offsets in floats; bf16 arrays hold 2 per float):
//   W1 A operands [g 4][fb 4][i 16][jj 8] = W1[8g+jj][16fb+i] (0 beyond input 10)
//   W2 forward    [s 2][g 4][fb 4][i 16][jj 8] = W2[kp(s,g,jj)][16fb+i]
//   W2 for dH1    [s 2][g 4][mb 4][i 16][jj 8] = W2[16mb+i][kp(s,g,jj)]
//   kp(s,g,jj) = 32s + 4g + (jj&3) + 16(jj>>2): the k order in which a layer's accumulator
//   (lane g holds features 16fb+4g+r) feeds the next 16x16x32 step with no lane movement.
//   f32: b1, b2, W3 (bf16-rounded values), b3, logstd, filter mean, 1/std.
constexpr int NB_W1 = 0;
constexpr int NB_W2F = NB_W1 + 4 * 4 * 16 * 8 / 2;
constexpr int NB_W2B = NB_W2F + 2 * 4 * 4 * 16 * 8 / 2;
constexpr int NB_B1 = NB_W2B + 2 * 4 * 4 * 16 * 8 / 2;
constexpr int NB_B2 = NB_B1 + HID;
constexpr int NB_W3 = NB_B2 + HID;
constexpr int NB_B3 = NB_W3 + HID * ACD;
constexpr int NB_LS = NB_B3 + ACD;
constexpr int NB_MU = NB_LS + ACD;
constexpr int NB_RS = NB_MU + 12;
constexpr int NETB_S = (NB_RS + 12 + 3) & ~3;   // bf16 student image (floats)
static_assert(NETB_S <= NET_S && NB_B1 % 4 == 0 && NB_W3 % 4 == 0, "bf16 student image");

__device__ __forceinline__ int kperm(int s, int g, int jj) { return 32 * s + 4 * g + (jj & 3) + 16 * (jj >> 2); }

__device__ void load_net_bf16(float* L, const float* g, int nthreads) {
    unsigned short* w1 = reinterpret_cast<unsigned short*>(L + NB_W1);
    unsigned short* w2f = reinterpret_cast<unsigned short*>(L + NB_W2F);
    unsigned short* w2b = reinterpret_cast<unsigned short*>(L + NB_W2B);
    for (int x = threadIdx.x; x < 4 * 4 * 16 * 8; x += nthreads) {
        const int jj = x & 7, i = (x >> 3) & 15, fb = (x >> 7) & 3, gg = x >> 9;
        const int k = 8 * gg + jj;
        w1[x] = bf16_bits(k < OBD ? g[P_W1 + k * HID + 16 * fb + i] : 0.0f);
    }
    for (int x = threadIdx.x; x < 2 * 4 * 4 * 16 * 8; x += nthreads) {
        const int jj = x & 7, i = (x >> 3) & 15, b = (x >> 7) & 3, gg = (x >> 9) & 3, s = x >> 11;
        const int kp = kperm(s, gg, jj);
        w2f[x] = bf16_bits(g[P_W2 + kp * HID + 16 * b + i]);
        w2b[x] = bf16_bits(g[P_W2 + (16 * b + i) * HID + kp]);
    }
    for (int x = threadIdx.x; x < HID; x += nthreads) {
        L[NB_B1 + x] = g[P_B1 + x];
        L[NB_B2 + x] = g[P_B2 + x];
    }
    for (int x = threadIdx.x; x < HID * ACD; x += nthreads) L[NB_W3 + x] = bf16_round(g[P_W3 + x]);
    if (threadIdx.x < ACD) {
        L[NB_B3 + threadIdx.x] = g[P_B3 + threadIdx.x];
        L[NB_LS + threadIdx.x] = g[P_LS + threadIdx.x];
    }
    if (threadIdx.x < 12) {
        const int k = threadIdx.x;
        L[NB_MU + k] = k < OBD ? g[P_TOT + k] : 0.0f;
        L[NB_RS + k] = k < OBD ? 1.0f / g[P_TOT + OBD + k] : 1.0f;
    }
}

// ---------------------------------------------------------------- f32 on bf16 MFMAs (split images)
// gfx950 runs f32 MFMAs at 1/16 of the bf16 rate, and beside them VALU work serialises on
// the SIMD's issue.  With rdd_config.f32_split the hidden-layer products
// (K = 64: both nets' layer 2 and the student's dH1 = W2 dZ2) run as f32 EMULATED on
// v_mfma_f32_16x16x32_bf16: each operand is split exactly into three bf16 pieces
//   x = x0 + x1 + x2,  x0 = x truncated to bf16, x1 = (x - x0) truncated, x2 = the rest,
// (x2 has at most 8 significant bits, so the split loses nothing) and a K = 32 step sums
// the six partial products of order >= 2^-16 (x2y0, x1y1, x0y2, x1y0, x0y1, x0y0, smallest
// first), each exact in the MFMA, into the f32 accumulator.  The dropped terms are below
// 2^-24 of |x||y|: f32 accuracy (scripts/micro/split_layer.hip: max error 1.5e-7 of
// sum|terms| vs 1.3e-7 for the exact f32 MFMA form; 1.54x its throughput).  Weight pieces
// are prepacked (pack_param); activation pieces are made per tile (split8).
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split1(float x, unsigned short (&h)[3]) {
    const uint32_t u = __float_as_uint(x);
    const float r = x - __uint_as_float(u & 0xffff0000u);
    const uint32_t ur = __float_as_uint(r);
    const float l = r - __uint_as_float(ur & 0xffff0000u);
    h[0] = (unsigned short)(u >> 16);
    h[1] = (unsigned short)(ur >> 16);
    h[2] = (unsigned short)(__float_as_uint(l) >> 16);
}

// split1's arithmetic as bit patterns whose high halves are the three pieces
__device__ __forceinline__ void split_bits(float x, uint32_t& u0, uint32_t& u1, uint32_t& u2) {
    u0 = __float_as_uint(x);
    const float r = x - __uint_as_float(u0 & 0xffff0000u);
    u1 = __float_as_uint(r);
    u2 = __float_as_uint(r - __uint_as_float(u1 & 0xffff0000u));
}

// lo = features k-slots jj 0..3, hi = jj 4..7 (the B operand order of the permuted images)
__device__ __forceinline__ void split8(f32x4 lo, f32x4 hi, bf16x8 (&p)[3]) {
    const float x[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    uint32_t u0[8], u1[8], u2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) split_bits(x[i], u0[i], u1[i], u2[i]);   // scalar: no packed-f32 ops
    u32x4 q0, q1, q2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // high halves of two words -> one packed pair
        q0[i] = __builtin_amdgcn_perm(u0[2 * i + 1], u0[2 * i], 0x07060302u);
        q1[i] = __builtin_amdgcn_perm(u1[2 * i + 1], u1[2 * i], 0x07060302u);
        q2[i] = __builtin_amdgcn_perm(u2[2 * i + 1], u2[2 * i], 0x07060302u);
    }
    p[0] = __builtin_bit_cast(bf16x8, q0);
    p[1] = __builtin_bit_cast(bf16x8, q1);
    p[2] = __builtin_bit_cast(bf16x8, q2);
}

// one bf16 pair (lo = high half of a, hi = high half of b)
__device__ __forceinline__ uint32_t pair_hi(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); }

// acc += W . X over one K = 32 step from split pieces w[3] (A) and x[3] (B)
__device__ __forceinline__ f32x4 mfma_split(const bf16x8 (&w)[3], const bf16x8 (&x)[3], f32x4 c) {
    c = mfma_k32(w[2], x[0], c);
    c = mfma_k32(w[1], x[1], c);
    c = mfma_k32(w[0], x[2], c);
    c = mfma_k32(w[1], x[0], c);
    c = mfma_k32(w[0], x[1], c);
    return mfma_k32(w[0], x[0], c);
}

// dW2 += H1^T dZ2 over a tile's 16 envs as f32 emulated on v_mfma_f32_32x32x16_bf16 (f32_split, f32
// student): K = the tile's 16 envs (lane half h = lane >> 5 carries envs 8h .. 8h + 7), the 64 x 64
// gradient as 2 x 2 blocks of 32 x 32 (C/D: column lane & 31, row (reg & 3) + 8 (reg >> 2) + 4 h).
// x[mb][e] = H1[32 mb + (lane & 31)][env 8h + e], y[nb][e] = dZ2[32 nb + (lane & 31)][env 8h + e],
// each split into its three bf16 pieces (split8); per block the six products of order >= 2^-16,
// smallest first (mfma_split): 24 MFMAs of 32 cycles that hold the SIMD's VALU issue for 8 each,
// where the round-5 16x16x32 form took 48 of 16 holding it for 8 (c4 75.2 -> 74.3 us per step,
// c3 28.1 -> 27.8, profiles/r06p_dw2_32x32_ab.jsonl) --
// half the held issue for the same MFMA time, and 17 % fewer VALU (no piece re-pairing).
typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ f32x16 mfma_32k16(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void dw2_split32(const float (&x)[2][8], const float (&y)[2][8], f32x16 (&g)[2][2]) {
    bf16x8 xp[2][3], yp[2][3];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        split8(f32x4{x[b][0], x[b][1], x[b][2], x[b][3]}, f32x4{x[b][4], x[b][5], x[b][6], x[b][7]}, xp[b]);
        split8(f32x4{y[b][0], y[b][1], y[b][2], y[b][3]}, f32x4{y[b][4], y[b][5], y[b][6], y[b][7]}, yp[b]);
    }
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
            f32x16 c = g[mb][nb];
            c = mfma_32k16(xp[mb][2], yp[nb][0], c);
            c = mfma_32k16(xp[mb][1], yp[nb][1], c);
            c = mfma_32k16(xp[mb][0], yp[nb][2], c);
            c = mfma_32k16(xp[mb][1], yp[nb][0], c);
            c = mfma_32k16(xp[mb][0], yp[nb][1], c);
            g[mb][nb] = mfma_32k16(xp[mb][0], yp[nb][0], c);
        }
}

// Split-mode image of a net (offsets in floats): the small vectors first, then the three
// pieces of the scaled W2 in the bf16 student's permuted forward order
// [q][s 2][g 4][fb 4][i 16][jj 8] = piece q of kTanhScale W2[kperm(s,g,jj)][16fb+i], then layer 1:
// the A operands of layer1_split's two piece pairings [v 2][g 4][fb 4][i 16][jj 8]: slot
// jj = 2s + c (s < 3) holds piece (v ? (0,1) : (0,2))[c] of kTanhScale W1[4s + g][16fb + i]
// (row 11 = b1), slots 6, 7 zero.  The student adds the pieces of the unscaled W2 for dH1 in
// the NB_W2B order.
constexpr int SP_PIECE = 2 * 4 * 4 * 16 * 8;      // bf16 elements per piece
constexpr int NX_B2 = 0;
constexpr int NX_W3 = NX_B2 + HID;                // 64
constexpr int NX_B3 = NX_W3 + HID * ACD;          // 192
constexpr int NX_LS = NX_B3 + ACD;
constexpr int NX_MU = NX_LS + ACD;
constexpr int NX_RS = NX_MU + 12;
constexpr int NX_W2F = NX_RS + 12;                // 220
constexpr int NX_W1S = NX_W2F + 3 * SP_PIECE / 2; // 6364
constexpr int NETX = NX_W1S + 2 * 4 * 4 * 16 * 8 / 2;   // 8412
constexpr int NX_W2B = NETX;                      // student only
constexpr int NETX_S = NX_W2B + 3 * SP_PIECE / 2; // 14556
static_assert(NX_W3 % 4 == 0 && NX_B2 % 4 == 0 && NX_W2F % 4 == 0 && NX_W1S % 4 == 0 && NETX % 4 == 0 &&
              NETX_S % 4 == 0, "16-B aligned split images");

// the student image's W3 / filter offsets by kind: exact f32 (N_*), split (NX_*), bf16 (NB_*)
template <int K> struct Off;
template <> struct Off<0> { static constexpr int W3 = N_W3, MU = N_MU, RS = N_RS; };
template <> struct Off<1> { static constexpr int W3 = NX_W3, MU = NX_MU, RS = NX_RS; };
template <> struct Off<2> { static constexpr int W3 = NB_W3, MU = NB_MU, RS = NB_RS; };

__device__ __forceinline__ void ld_pieces(const float* L, int base, int o, bf16x8 (&w)[3]) {
    const unsigned short* h = reinterpret_cast<const unsigned short*>(L + base);
#pragma unroll
    for (int q = 0; q < 3; ++q) w[q] = *reinterpret_cast<const bf16x8*>(h + q * SP_PIECE + o);
}

// Layer 1 of a split image's net on v_mfma_f32_16x16x32_bf16 (f32 emulated by three-piece splits):
// lane group g's inputs 4s + g (s < 3; input 11 is the bias input 1) as three pieces each, a
// K = 32 step carrying two pieces of each input (slots 2s, 2s + 1), the six products of order
// >= 2^-16 in three MFMAs per output block: w0z2 + w2z0, w0z1 + w1z1, w0z0 + w1z0.  12 bf16
// MFMAs instead of 12 f32 ones, which hold the SIMD's VALU issue for 32 cycles each and read
// their SrcC for 8 passes (the hazard the consumer-side-step kernels had to fence).
__device__ __forceinline__ void layer1_split(const float* L, const float* ob, int j, int g, f32x4 (&acc)[4]) {
    u32x4 b[3];
#pragma unroll
    for (int s = 0; s < 3; ++s) {
        const int k = 4 * s + g;
        const float z = fminf(fmaxf((ob[j * SOS + k] - L[NX_MU + k]) * L[NX_RS + k], -5.0f), 5.0f);
        uint32_t z0, z1, z2;
        split_bits(z, z0, z1, z2);
        b[0][s] = pair_hi(z2, z0);
        b[1][s] = pair_hi(z1, z1);
        b[2][s] = pair_hi(z0, z0);
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        b[q][3] = 0u;
        const bf16x8 bq = __builtin_bit_cast(bf16x8, b[q]);
#pragma unroll
        for (int fb = 0; fb < 4; ++fb)
            acc[fb] = mfma_k32(ldbf8(L + NX_W1S, ((((q ? 1 : 0) * 4 + g) * 4 + fb) * 16 + j) * 8), bq, acc[fb]);
    }
}

// Teacher and student forwards of one tile with split images (both nets, interleaved):
// layer 1 (layer1_split) and layer 2 on split bf16 MFMAs.  Layer 2 runs in three scheduling
// regions: the first K step's splits | its MFMAs with the second step's splits in their gaps
// (per output block its six piece loads, then 12 x (one MFMA, three VALU)) | the second
// step's MFMAs (c4 80.9 -> 79.7 us per step, profiles/r03y_sched_nt.txt; 3 VALU per MFMA
// -0.25 us vs 2, profiles/r03ze_ps_per.txt).
__device__ __forceinline__ void mlp_forward_pair_split(const float* LT, const float* LS, const float* ob, int j, int g,
                                                       f32x4 (&H1)[4], f32x4 (&H2)[4], float& mt0, float& mt1,
                                                       float& ms0, float& ms1) {
    f32x4 at[4], as[4];
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) at[fb] = as[fb] = f32x4{0.f, 0.f, 0.f, 0.f};
    layer1_split(LT, ob, j, g, at);
    layer1_split(LS, ob, j, g, as);
    f32x4 T1[4];
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) {
        T1[fb] = tanh4(at[fb]);
        H1[fb] = tanh4(as[fb]);
    }
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) {
        at[fb] = ld4(LT + NX_B2 + 16 * fb + 4 * g);
        as[fb] = ld4(LS + NX_B2 + 16 * fb + 4 * g);
    }
    {   // three regions: split s0 | s0 MFMAs + split s1 | s1 MFMAs
        bf16x8 tp[2][3], sp[2][3];
        __builtin_amdgcn_sched_barrier(0);
        split8(T1[0], T1[1], tp[0]);
        split8(H1[0], H1[1], sp[0]);
        __builtin_amdgcn_sched_barrier(0);
        split8(T1[2], T1[3], tp[1]);
        split8(H1[2], H1[3], sp[1]);
#pragma unroll
        for (int fb = 0; fb < 4; ++fb) {
            const int o = (((0 * 4 + g) * 4 + fb) * 16 + j) * 8;
            bf16x8 wt[3], ws[3];
            ld_pieces(LT, NX_W2F, o, wt);
            ld_pieces(LS, NX_W2F, o, ws);
            at[fb] = mfma_split(wt, tp[0], at[fb]);
            as[fb] = mfma_split(ws, sp[0], as[fb]);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 6, 2);
#pragma unroll
        for (int fb = 0; fb < 4; ++fb) {
            if (fb < 3) __builtin_amdgcn_sched_group_barrier(0x100, 6, 2);
#pragma unroll
            for (int m = 0; m < 12; ++m) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 2);
                __builtin_amdgcn_sched_group_barrier(0x002, 3, 2);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int fb = 0; fb < 4; ++fb) {
            const int o = (((1 * 4 + g) * 4 + fb) * 16 + j) * 8;
            bf16x8 wt[3], ws[3];
            ld_pieces(LT, NX_W2F, o, wt);
            ld_pieces(LS, NX_W2F, o, ws);
            at[fb] = mfma_split(wt, tp[1], at[fb]);
            as[fb] = mfma_split(ws, sp[1], as[fb]);
        }
    }
    float pt0 = 0.0f, pt1 = 0.0f, ps0 = 0.0f, ps1 = 0.0f;
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) {
        const f32x4 ta = ld4(LT + NX_W3 + (16 * fb + 4 * g) * 2), tb = ld4(LT + NX_W3 + (16 * fb + 4 * g) * 2 + 4);
        const f32x4 sa = ld4(LS + NX_W3 + (16 * fb + 4 * g) * 2), sb = ld4(LS + NX_W3 + (16 * fb + 4 * g) * 2 + 4);
        f32x4 t2;
        t2 = tanh4(at[fb]);
        H2[fb] = tanh4(as[fb]);
        pt0 = fmaf(t2[0], ta[0], pt0); pt1 = fmaf(t2[0], ta[1], pt1);
        pt0 = fmaf(t2[1], ta[2], pt0); pt1 = fmaf(t2[1], ta[3], pt1);
        pt0 = fmaf(t2[2], tb[0], pt0); pt1 = fmaf(t2[2], tb[1], pt1);
        pt0 = fmaf(t2[3], tb[2], pt0); pt1 = fmaf(t2[3], tb[3], pt1);
        ps0 = fmaf(H2[fb][0], sa[0], ps0); ps1 = fmaf(H2[fb][0], sa[1], ps1);
        ps0 = fmaf(H2[fb][1], sa[2], ps0); ps1 = fmaf(H2[fb][1], sa[3], ps1);
        ps0 = fmaf(H2[fb][2], sb[0], ps0); ps1 = fmaf(H2[fb][2], sb[1], ps1);
        ps0 = fmaf(H2[fb][3], sb[2], ps0); ps1 = fmaf(H2[fb][3], sb[3], ps1);
    }
    mt0 = xsum32(xsum16(pt0)) + LT[NX_B3];
    mt1 = xsum32(xsum16(pt1)) + LT[NX_B3 + 1];
    ms0 = xsum32(xsum16(ps0)) + LS[NX_B3];
    ms1 = xsum32(xsum16(ps1)) + LS[NX_B3 + 1];
}

// One net's forward with a split image (the teacher beside the bf16 student; HO: also
// return the hidden activations).
template <bool HO>
__device__ __forceinline__ void mlp_forward_split_t(const float* L, const float* ob, int j, int g, f32x4 (&H1)[4],
                                                    f32x4 (&H2)[4], float& m0, float& m1) {
    f32x4 acc[4];
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) acc[fb] = f32x4{0.f, 0.f, 0.f, 0.f};
    layer1_split(L, ob, j, g, acc);
#pragma unroll
    for (int fb = 0; fb < 4; ++fb)
        H1[fb] = tanh4(acc[fb]);
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) acc[fb] = ld4(L + NX_B2 + 16 * fb + 4 * g);
    {   // three regions, as the pair's layer 2 (c5 37.2-37.6 -> 36.6 us per step, profiles/r03za_tsched.txt)
        bf16x8 hp[2][3];
        __builtin_amdgcn_sched_barrier(0);
        split8(H1[0], H1[1], hp[0]);
        __builtin_amdgcn_sched_barrier(0);
        split8(H1[2], H1[3], hp[1]);
#pragma unroll
        for (int fb = 0; fb < 4; ++fb) {
            bf16x8 w[3];
            ld_pieces(L, NX_W2F, (((0 * 4 + g) * 4 + fb) * 16 + j) * 8, w);
            acc[fb] = mfma_split(w, hp[0], acc[fb]);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, 3, 3);
#pragma unroll
        for (int fb = 0; fb < 4; ++fb) {
            if (fb < 3) __builtin_amdgcn_sched_group_barrier(0x100, 3, 3);
#pragma unroll
            for (int m = 0; m < 6; ++m) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 3);
                __builtin_amdgcn_sched_group_barrier(0x002, 2, 3);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int fb = 0; fb < 4; ++fb) {
            bf16x8 w[3];
            ld_pieces(L, NX_W2F, (((1 * 4 + g) * 4 + fb) * 16 + j) * 8, w);
            acc[fb] = mfma_split(w, hp[1], acc[fb]);
        }
    }
    float p0 = 0.0f, p1 = 0.0f;
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) {
        const f32x4 wa = ld4(L + NX_W3 + (16 * fb + 4 * g) * 2);
        const f32x4 wb = ld4(L + NX_W3 + (16 * fb + 4 * g) * 2 + 4);
        f32x4 h2;
        h2 = tanh4(acc[fb]);
        if constexpr (HO) H2[fb] = h2;
        p0 = fmaf(h2[0], wa[0], p0); p1 = fmaf(h2[0], wa[1], p1);
        p0 = fmaf(h2[1], wa[2], p0); p1 = fmaf(h2[1], wa[3], p1);
        p0 = fmaf(h2[2], wb[0], p0); p1 = fmaf(h2[2], wb[1], p1);
        p0 = fmaf(h2[3], wb[2], p0); p1 = fmaf(h2[3], wb[3], p1);
    }
    m0 = xsum32(xsum16(p0)) + L[NX_B3];
    m1 = xsum32(xsum16(p1)) + L[NX_B3 + 1];
}
__device__ __forceinline__ void mlp_forward_split(const float* L, const float* ob, int j, int g, float& m0, float& m1) {
    f32x4 h1[4], h2[4];
    mlp_forward_split_t<false>(L, ob, j, g, h1, h2, m0, m1);
}


// ---------------------------------------------------------------- prepacked LDS images
// The rollout's LDS images (teacher NET floats, student NET_S floats) are kept ready in
// HBM: pack_param() writes one parameter's value into every image slot it occupies.  The
// images are built once by pack_net_kernel (rdd_set_teacher / rdd_set_student) and the
// student's is refreshed by reduce_adam_kernel as it updates each parameter, so a rollout's
// prologue is a plain 16-B copy instead of a gather with index arithmetic.
// image kinds: IMG_F32 (N_* layout), IMG_SPLIT (NX_*), IMG_BF16 (NB_*, student only)
constexpr int IMG_F32 = 0, IMG_SPLIT = 1, IMG_BF16 = 2;

__device__ __forceinline__ void pack_param(float* img, int p, float v, bool student, int kind) {
    if (kind == IMG_SPLIT) {
        unsigned short* h = reinterpret_cast<unsigned short*>(img);
        unsigned short q[3];
        if (p < P_W2) {   // W1 rows 0..10, b1 as row 11
            const int k = p < P_B1 ? p >> 6 : OBD, f = p < P_B1 ? p & 63 : p - P_B1;
            // layer1_split's A operands: slots 2s, 2s + 1 of lane group k & 3
            split1(kTanhScale * v, q);
            const int o = 2 * NX_W1S + (((k & 3) * 4 + (f >> 4)) * 16 + (f & 15)) * 8 + 2 * (k >> 2);
            constexpr int V1 = 4 * 4 * 16 * 8;   // the (0,1) pairing follows the (0,2) one
            put(h + (o), q[0]); put(h + (o + 1), q[2]);
            put(h + (o + V1), q[0]); put(h + (o + V1 + 1), q[1]);
        } else if (p < P_B2) {
            const int k = (p - P_W2) >> 6, f = (p - P_W2) & 63;
            {   // forward: k is the permuted K index (as NB_W2F), pieces of the scaled weight
                const int s = k >> 5, r = k & 31, gg = (r & 15) >> 2, jj = (r & 3) + 4 * (r >> 4);
                const int o = 2 * NX_W2F + (((s * 4 + gg) * 4 + (f >> 4)) * 16 + (f & 15)) * 8 + jj;
                split1(kTanhScale * v, q);
                put(h + (o), q[0]); put(h + (o + SP_PIECE), q[1]); put(h + (o + 2 * SP_PIECE), q[2]);
            }
            if (student) {   // dH1: f is the permuted K index (as NB_W2B), unscaled
                const int s = f >> 5, r = f & 31, gg = (r & 15) >> 2, jj = (r & 3) + 4 * (r >> 4);
                const int o = 2 * NX_W2B + (((s * 4 + gg) * 4 + (k >> 4)) * 16 + (k & 15)) * 8 + jj;
                split1(v, q);
                put(h + (o), q[0]); put(h + (o + SP_PIECE), q[1]); put(h + (o + 2 * SP_PIECE), q[2]);
            }
        } else if (p < P_W3) {
            put(img + (NX_B2 + (p - P_B2)), kTanhScale * v);
        } else if (p < P_B3) {
            put(img + (NX_W3 + (p - P_W3)), v);
        } else if (p < P_LS) {
            put(img + (NX_B3 + (p - P_B3)), v);
        } else if (p < P_TOT) {
            put(img + (NX_LS + (p - P_LS)), v);
        }
        return;
    }
    if (kind == IMG_F32) {
        if (p < P_B1) {
            const int k = p >> 6, f = p & 63;
            put(img + (N_W1 + k * HID + (f & 15) * 4 + (f >> 4)), kTanhScale * v);
        } else if (p < P_W2) {
            const int f = p - P_B1;
            put(img + (N_W1 + OBD * HID + (f & 15) * 4 + (f >> 4)), kTanhScale * v);
        } else if (p < P_B2) {
            const int k = (p - P_W2) >> 6, f = (p - P_W2) & 63;
            put(img + (N_W2 + k * HID + (f & 15) * 4 + (f >> 4)), kTanhScale * v);
            if (student) put(img + (N_W2T + f * HID + (k & 15) * 4 + (k >> 4)), v);
        } else if (p < P_W3) {
            put(img + (N_B2 + (p - P_B2)), kTanhScale * v);
        } else if (p < P_B3) {
            put(img + (N_W3 + (p - P_W3)), v);
        } else if (p < P_LS) {
            put(img + (N_B3 + (p - P_B3)), v);
        } else if (p < P_TOT) {
            put(img + (N_LS + (p - P_LS)), v);
        }
        return;
    }
    unsigned short* h = reinterpret_cast<unsigned short*>(img);
    if (p < P_B1) {
        const int k = p >> 6, f = p & 63;   // k = 8gg + jj
        put(h + (2 * NB_W1 + (((k >> 3) * 4 + (f >> 4)) * 16 + (f & 15)) * 8 + (k & 7)), bf16_bits(v));
    } else if (p < P_W2) {
        put(img + (NB_B1 + (p - P_B1)), v);
    } else if (p < P_B2) {
        const int k = (p - P_W2) >> 6, f = (p - P_W2) & 63;
        // forward image: k (H1 feature) is the permuted K index, f the output row
        {
            const int s = k >> 5, r = k & 31, gg = (r & 15) >> 2, jj = (r & 3) + 4 * (r >> 4);
            put(h + (2 * NB_W2F + (((s * 4 + gg) * 4 + (f >> 4)) * 16 + (f & 15)) * 8 + jj), bf16_bits(v));
        }
        // dH1 image: f (dZ2 feature) is the permuted K index, k the output row
        {
            const int s = f >> 5, r = f & 31, gg = (r & 15) >> 2, jj = (r & 3) + 4 * (r >> 4);
            put(h + (2 * NB_W2B + (((s * 4 + gg) * 4 + (k >> 4)) * 16 + (k & 15)) * 8 + jj), bf16_bits(v));
        }
    } else if (p < P_W3) {
        put(img + (NB_B2 + (p - P_B2)), v);
    } else if (p < P_B3) {
        put(img + (NB_W3 + (p - P_W3)), bf16_round(v));
    } else if (p < P_LS) {
        put(img + (NB_B3 + (p - P_B3)), v);
    } else if (p < P_TOT) {
        put(img + (NB_LS + (p - P_LS)), v);
    }
}

// net = params[P] | mu[11] | sd[11] -> image (every slot, including zero padding and filter)
__global__ __launch_bounds__(256) void pack_net_kernel(const float* net, float* img, int img_floats, int student,
                                                       int kind) {
    const int x = blockIdx.x * 256 + threadIdx.x;
    // phase 1 (one launch): zero the image, then the filter words, then every parameter
    for (int i = x; i < img_floats; i += gridDim.x * 256) img[i] = 0.0f;
    __syncthreads();   // (single-block launch: see rdd host code)
    if (x < 12) {
        const int mu = kind == IMG_BF16 ? NB_MU : kind == IMG_SPLIT ? NX_MU : N_MU;
        const int rs = kind == IMG_BF16 ? NB_RS : kind == IMG_SPLIT ? NX_RS : N_RS;
        img[mu + x] = x < OBD ? net[P_TOT + x] : 0.0f;
        img[rs + x] = x < OBD ? 1.0f / net[P_TOT + OBD + x] : 1.0f;
    }
    for (int p = x; p < P_TOT; p += gridDim.x * 256) pack_param(img, p, net[p], student != 0, kind);
}

// Both rollout images (contiguous in LDS: teacher then student) by LDS-DMA: every 16-B piece is
// one global_load_lds_dwordx4 (wave-uniform LDS base + lane x 16 B, per-lane global address), so
// the copy needs no staging VGPRs and no ds_write pass.  `between` runs while they are in flight
// (the producers' first observations); every wave then drains its DMA (vmcnt(0)) before the
// caller's __syncthreads publishes the image.  Round 4 measured it 0.2-0.3 us per step faster
// than the register-staged copy (profiles/r04c_imgdma_ab.txt) but reverted it: its first rollout
// in a process differed in lanes-48-63 dW3 entries.  Round 5 found that signature's cause on the
// compute side -- the SLP-packed dW3 accumulators at the tile loop's latch (PKWAR, DESIGN.md §3;
// distill.hip is now built without SLP) -- and re-landed the fill; the register-staged form is
// in profiles/r04_removed_diagnostic_variants.diff.
template <int V4A, int V4B, int NT, class F>
__device__ __forceinline__ void copy_images(float* L, const float* ta, const float* sb, F&& between) {
    constexpr int TOT = V4A + V4B, PER = (TOT + NT - 1) / NT;
    const int wbase = threadIdx.x & ~63;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int x = threadIdx.x + u * NT;
        if (x < TOT)
            __builtin_amdgcn_global_load_lds(x < V4A ? ta + 4 * x : sb + 4 * (x - V4A), L + 4 * (wbase + u * NT), 16, 0, 0);
    }
    between();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's image pieces have landed in LDS
}

// kTanhScale * x as four scalar multiplies: a vector multiply would be a v_pk_mul_f32, and packed-f32
// ops are kept out of the rollout's hot loops (PKWAR)
__device__ __forceinline__ f32x4 scale4(f32x4 x) {
    return f32x4{kTanhScale * x[0], kTanhScale * x[1], kTanhScale * x[2], kTanhScale * x[3]};
}

// bf16-student forward of a 16-env tile (same outputs/layouts as mlp_forward).
__device__ __forceinline__ void mlp_forward_bf16(const float* L, const float* ob, int j, int g, f32x4 (&H1)[4],
                                                 f32x4 (&H2)[4], float& m0, float& m1) {
    f32x4 acc[4];
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) acc[fb] = ld4(L + NB_B1 + 16 * fb + 4 * g);
    // layer 1: one K = 32 step, lane group g supplies inputs 8g .. 8g+7 (zero past input 10)
    bf16x8 zb;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
        const int k = 8 * g + jj;
        const int kc = k < OBD ? k : 0;
        const float z = fminf(fmaxf((ob[j * SOS + kc] - L[NB_MU + kc]) * L[NB_RS + kc], -5.0f), 5.0f);
        zb[jj] = (__bf16)(k < OBD ? z : 0.0f);
    }
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) acc[fb] = mfma_k32(ldbf8(L + NB_W1, ((g * 4 + fb) * 16 + j) * 8), zb, acc[fb]);
#pragma unroll
    for (int fb = 0; fb < 4; ++fb)
        H1[fb] = tanh4(scale4(acc[fb]));
    // layer 2: two K = 32 steps over the permuted feature order kperm
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) acc[fb] = ld4(L + NB_B2 + 16 * fb + 4 * g);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const bf16x8 hb = pack8(H1[2 * s], H1[2 * s + 1]);
#pragma unroll
        for (int fb = 0; fb < 4; ++fb)
            acc[fb] = mfma_k32(ldbf8(L + NB_W2F, (((s * 4 + g) * 4 + fb) * 16 + j) * 8), hb, acc[fb]);
    }
    float p0 = 0.0f, p1 = 0.0f;
#pragma unroll
    for (int fb = 0; fb < 4; ++fb) {
        const f32x4 wa = ld4(L + NB_W3 + (16 * fb + 4 * g) * 2);
        const f32x4 wb = ld4(L + NB_W3 + (16 * fb + 4 * g) * 2 + 4);
        H2[fb] = tanh4(scale4(acc[fb]));
        p0 = fmaf(H2[fb][0], wa[0], p0); p1 = fmaf(H2[fb][0], wa[1], p1);
        p0 = fmaf(H2[fb][1], wa[2], p0); p1 = fmaf(H2[fb][1], wa[3], p1);
        p0 = fmaf(H2[fb][2], wb[0], p0); p1 = fmaf(H2[fb][2], wb[1], p1);
        p0 = fmaf(H2[fb][3], wb[2], p0); p1 = fmaf(H2[fb][3], wb[3], p1);
    }
    m0 = xsum32(xsum16(p0)) + L[NB_B3];
    m1 = xsum32(xsum16(p1)) + L[NB_B3 + 1];
}

// Hand-off counters live in LDS; each is written by one wave only.  Acquire/release at
// workgroup scope order the slot data (LDS) around them.  A spin that exceeds SPIN_LIMIT
// raises ctl[8] and returns false: the caller leaves its loop, so the launch always ends.
__device__ __forceinline__ bool wait_ge(const uint32_t* f, uint32_t target, uint32_t* err) {
    for (uint32_t spins = 0;; ++spins) {
        if (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) return true;
        if (spins > SPIN_LIMIT) {
            if ((threadIdx.x & 63) == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

__device__ __forceinline__ void publish(uint32_t* f, uint32_t v) {
    __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// env.step of this lane's env with the policy's action, the episode clock (lockstep or
// staggered) and the auto-reset; writes the state back and returns the reward (0 for a lane
// without an env).  met_n counts the stepped envs.
__device__ __forceinline__ float env_step_group(const RolloutArgs& a, uint32_t C, int64_t i, bool valid, float act0,
                                                float act1, rd::State& st, float& met_n) {
    const uint32_t iu = (uint32_t)i;
    const float rew = rd::env_step<false>(st, act0, act1);
    // episode clock of this env (RDD_STAGGER_GROUP envs share an offset)
    const int64_t gid = a.env_base + i;
    const uint32_t u = C + (a.stagger ? (uint32_t)((gid / RDD_STAGGER_GROUP) % rd::kEpisodeSteps) : 0u);
    const bool done_step = (u % rd::kEpisodeSteps) == rd::kEpisodeSteps - 1;
    if (done_step) {
        float dr[6];
        rd::philox_draw(a.seed, (uint64_t)gid, u / rd::kEpisodeSteps + 1, dr);
        rd::env_reset(st, dr);
    }
    if (!valid) return 0.0f;
    float* s = a.state;
    const int64_t n = a.n;
    put(s + 0 * n + iu, st.q0); put(s + 1 * n + iu, st.q1);
    put(s + 2 * n + iu, st.v0); put(s + 3 * n + iu, st.v1);
    if (done_step) { put(s + 4 * n + iu, st.tx); put(s + 5 * n + iu, st.ty); }
    put(s + 6 * n + iu, st.dx); put(s + 7 * n + iu, st.dy);
    met_n += 1.0f;
    return rew;
}

// The per-column arithmetic of the reduction: RED_ROWS row-threads per parameter, each
// summing rows row, row + RED_ROWS, ... in four interleaved partial sums; the row-threads'
// sums are then added in a fixed order (deterministic).
__device__ __forceinline__ float col_rows(const float* ws, int nblk, int p, int row) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    const float* w = ws + ws_index(p, 0, nblk);   // row b of column p at w[b * RED_COLS]
    int b = row;
#pragma unroll 4
    for (; b + 3 * RED_ROWS < nblk; b += 4 * RED_ROWS) {
        s0 += w[b * RED_COLS];
        s1 += w[(b + RED_ROWS) * RED_COLS];
        s2 += w[(b + 2 * RED_ROWS) * RED_COLS];
        s3 += w[(b + 3 * RED_ROWS) * RED_COLS];
    }
    for (; b < nblk; b += RED_ROWS) s0 += w[b * RED_COLS];
    return (s0 + s1) + (s2 + s3);
}

// parameter p: total of its row-threads' sums (part[r * stride], r < RED_ROWS), the gradient /
// metrics slot, then the TF1 ApplyAdam functor (training_ops.cc) and the image refresh
__device__ __forceinline__ void col_finish(const ReduceArgs& a, int p, const float* part, int stride, float m_p,
                                           float v_p, float w_p, uint32_t S, float b1p, float b2p) {
    float g;
    if (a.reduce) {
        float q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < RED_ROWS; ++r) q[r & 3] += part[r * stride];
        g = (q[0] + q[1]) + (q[2] + q[3]);
        if (p < P_TOT) {
            if (a.accum) g += a.grad[p];
            put(a.grad + p, g);
        } else {
            float* h = a.hist + (int64_t)(S % (uint32_t)a.hist_len) * N_MET + (p - P_TOT);
            put(h, a.accum ? *h + g : g);
        }
    } else {
        g = p < P_TOT ? a.grad[p] : 0.f;
    }
    if (a.adam && p < P_TOT) {
        const float alpha = a.lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
        float m = m_p, v = v_p;
        m += (g - m) * (1.0f - a.b1);
        v += (g * g - v) * (1.0f - a.b2);
        put(a.m + p, m);
        put(a.v + p, v);
        const float w = w_p - (m * alpha) / (sqrtf(v) + a.eps);
        put(a.params + p, w);
        pack_param(a.simg, p, w, true, a.img_kind);
    }
}

__device__ __forceinline__ void bump_ctl(const ReduceArgs& a, uint32_t C, uint32_t S, float b1p, float b2p,
                                         uint32_t stepped) {
    if (a.bump_env) a.ctl[0] = C + stepped;   // env steps: only after a launch that stepped the envs
    if (a.bump_opt) {
        a.ctl[1] = S + 1u;                     // optimiser steps
        a.ctl[2] = __float_as_uint(b1p * a.b1);
        a.ctl[3] = __float_as_uint(b2p * a.b2);
    }
}

// LDS floats of the teacher / student images of a rollout instance
constexpr int img_t(bool SPL) { return SPL ? NETX : NET; }
constexpr int img_s(bool BS, bool SPL) { return BS ? NETB_S : (SPL ? NETX_S : NET_S); }
static_assert((NETX + NETX_S + PAIRS * PSCR) * 4 <= 160 * 1024 && (NETX + NETB_S + PAIRS * PSCR) * 4 <= 160 * 1024,
              "LDS budget (split images)");

// BS: bf16 student (RDD_DTYPE_BF16); SPL: split-bf16 f32 hidden layers; CP: the consumer wave
// steps the envs (else the producer does, from the state it loaded for the observations);
// MD: MD_TEACHER the teacher network is queried; MD_ROWS observation rows with their recorded
// teacher pdflat (a.tnet), no teacher network (no teacher image in LDS); MD_HELPER (f32
// student, one 16-env tile per pair's group, launch_rollout): pairs 0, 1 own the groups and
// pairs 2, 3 run their tiles' teacher forwards on the other two SIMDs
constexpr int MD_TEACHER = 0, MD_ROWS = 1, MD_HELPER = 2;
// KS: a.ksteps env steps in one launch (rdd_step_accum); the K = 1 instances are compiled without
// the step loop.
// TC (bf16 student with the split teacher, config 5): the consumer wave runs the teacher forward
// of each group's odd tiles from the producer's observation rows and hands the means back
// (P_TM, flag [3]); the producer publishes each group's observations (flag [2]) and runs the
// teacher of the even tiles beside the student forwards (c5 -0.5 us per step).
template <bool BS, bool SPL, bool CP, int MD, bool KS = false, bool TC = false>
__global__ __launch_bounds__(BLOCK, 2) void rollout_kernel(RolloutArgs a) {
    constexpr bool TGT = MD == MD_ROWS, HLP = MD == MD_HELPER;
    static_assert(!TC || (BS && MD == MD_TEACHER && !KS), "teacher on the consumer: bf16 student, K = 1");
    constexpr int P_TM = CP ? P_ACT : P_SACT;   // TC: the consumer's teacher means of one tile [16][2]
    static_assert(!HLP || !BS, "helper pairs: f32 student kernels only");
    constexpr int TN = TGT ? 0 : img_t(SPL), SN = img_s(BS, SPL);
    __shared__ __attribute__((aligned(16))) float lds[TN + SN + PAIRS * PSCR];
    float* LT = lds;
    float* LS = lds + TN;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int j = lane & 15, g = lane >> 4;
    const int pair = wave & (PAIRS - 1);
    const bool producer = wave < PAIRS;
    uint32_t* flags = reinterpret_cast<uint32_t*>(lds + TN + SN + pair * PSCR + P_FLAGS);
    uint32_t* err = a.ctl + 8;

    RTSTAMP(16);
    STAMP(0);
    const int gs = a.gs;   // envs per group: 64, or 32 / 16 to spread a small batch over more pairs
    // 32-bit group / env indices (n <= 2^31, rdd_create): fewer SGPRs live across the loops
    const uint32_t n32 = (uint32_t)a.n;
    const uint32_t ngroups = (n32 + (uint32_t)gs - 1) / (uint32_t)gs;
    // HLP: the owner pairs 0, 1 take the groups (one each), pairs 2, 3 none (they help).  The
    // layout holds at most one group per owner (launch_rollout): a launch that breaks this ends
    // at once with the hand-off error raised (rdd_counter reports it)
    // KS (K env steps in one launch): the producer re-reads the state its own lanes wrote, so
    // the consumer-side env step (CP), the helper layout and the observation modes stay K = 1
    static_assert(!KS || (!CP && MD == MD_TEACHER), "K-step launches: teacher mode, producer-side env step");
    if constexpr (KS) {
        if (a.obs_in) {
            if (threadIdx.x == 0) __hip_atomic_store(a.ctl + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    }
    if constexpr (HLP) {
        if (ngroups > 2u * gridDim.x) {
            if (threadIdx.x == 0) __hip_atomic_store(a.ctl + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    }
    const bool helper = HLP && pair >= 2;
    const uint32_t gstride = gridDim.x * (HLP ? 2 : PAIRS);
    const uint32_t gfirst = helper ? ngroups : blockIdx.x * (HLP ? 2 : PAIRS) + pair;
    // a producer's first group of envs: its state loads are issued before the image copy so
    // that their HBM latency overlaps the prologue
    rd::State st0{};
    if (producer && !a.obs_in && gfirst < ngroups && lane < gs && gfirst * gs + lane < a.n)
        load_state(a.state, a.n, (uint32_t)(gfirst * gs + lane), st0);
    // HLP with the teacher acting: the helper producer steps its owner's envs (below), so it loads
    // their state here instead of the owner
    const uint32_t og = blockIdx.x * 2 + (pair & 1);   // HLP: the owner group a helper serves
    const bool hstep = helper && producer && !a.obs_in && !a.act_student;
    if constexpr (HLP) {
        if (hstep && og < ngroups && lane < gs && og * gs + lane < a.n)
            load_state(a.state, a.n, (uint32_t)(og * gs + lane), st0);
    }
    static_assert(NET % 4 == 0 && NET_S % 4 == 0, "16-B images");
    // ... and its observations are formed (into obs buffer 0) while the image loads are in flight
    float* PS = lds + TN + SN + pair * PSCR;
    const bool first_obs = producer && gfirst < ngroups;
    auto group_obs = [&](uint32_t k, uint32_t i, bool lvalid, rd::State& st) {
        float ob[OBD];
        if (a.obs_in) {   // observation-batch mode: rows given by the caller
#pragma unroll
            for (int q = 0; q < OBD; ++q) ob[q] = lvalid ? a.obs_in[(size_t)i * OBD + q] : 0.0f;
        } else {
            rd::observe<false>(st, ob);
        }
        float* o = PS + P_SO + lane * SOS;
        st4(o, f32x4{ob[0], ob[1], ob[2], ob[3]});
        st4(o + 4, f32x4{ob[4], ob[5], ob[6], ob[7]});
        st4(o + 8, f32x4{ob[8], ob[9], ob[10], 1.0f});
    };
    copy_images<TN / 4, SN / 4, BLOCK>(LT, a.timg, a.simg, [&] {   // LS = LT + TN
        if (first_obs) {
            const uint32_t i = gfirst * (uint32_t)gs + (uint32_t)lane;
            group_obs(0, i, lane < gs && i < n32, st0);
        }
    });
    using SO = Off<BS ? IMG_BF16 : (SPL ? IMG_SPLIT : IMG_F32)>;
    constexpr int SW3 = SO::W3, SMU = SO::MU, SRS = SO::RS;
    if (threadIdx.x < PAIRS * 4)
        reinterpret_cast<uint32_t*>(lds + TN + SN + (threadIdx.x >> 2) * PSCR + P_FLAGS)[threadIdx.x & 3] = 0u;

    const uint32_t C = a.ctl[0];
    // snapshot of the step words for reduce_adam_kernel, which rewrites ctl[0..3]; ctl[12]
    // tells it whether this launch stepped the envs (the env clock advances only then)
    if (blockIdx.x == 0 && threadIdx.x < 4) a.ctl[4 + threadIdx.x] = a.ctl[threadIdx.x];
    if (blockIdx.x == 0 && threadIdx.x == 4) a.ctl[12] = a.obs_in ? 0u : (KS ? (uint32_t)a.ksteps : 1u);
    __syncthreads();
    STAMP(1);

    if (producer) {
        // ============================================================ producer wave
        // partial sums: dW3 (env j of this lane, features 16x+4g+r), db3, dlogstd, metrics
        f32x4 gw3a[4], gw3b[4];
#pragma unroll
        for (int x = 0; x < 4; ++x) gw3a[x] = gw3b[x] = f32x4{0.f, 0.f, 0.f, 0.f};
        float gb3a = 0, gb3b = 0, gls0 = 0, gls1 = 0, met_l = 0, met_m = 0, met_r = 0, met_n = 0;
        // teacher log-std (TGT: per row, from the recorded pdflat, below)
        const float tl0 = TGT ? 0.0f : a.tnet[P_LS], tl1 = TGT ? 0.0f : a.tnet[P_LS + 1];
        const float sl0 = a.snet[P_LS], sl1 = a.snet[P_LS + 1];
        const float sv0 = __expf(2.0f * sl0), sv1 = __expf(2.0f * sl1);
        const float rtv0 = 1.0f / __expf(2.0f * tl0), rtv1 = 1.0f / __expf(2.0f * tl1);
        uint32_t tiles = 0;
        uint32_t k = 0;
        uint32_t tct = 0;   // TC: teacher tiles taken from the consumer
        bool ok = true;
        // HLP helper (pair 2 + o): the teacher forward of owner o's first tile (its observations
        // were formed in the prologue, before the barrier), means into this pair's P_ACT, flag [0]
        if constexpr (HLP) {
            if (helper && og < ngroups) {
                STAMP(18);
                const float* oobs = lds + TN + SN + (pair & 1) * PSCR + P_SO;
                float m0, m1;
                if constexpr (SPL) {
                    mlp_forward_split(LT, oobs, j, g, m0, m1);
                } else {
                    f32x4 h1[4], h2[4];
                    mlp_forward<true>(LT, oobs, j, g, h1, h2, m0, m1);
                }
                if (g == 0) {
                    PS[P_ACT + 2 * j] = m0;
                    PS[P_ACT + 2 * j + 1] = m1;
                }
                publish(flags, 1u);
                STAMP(19);
                // ... and, with the teacher acting, steps the owner's envs with these means (lane
                // j < 16 holds env j's): the owner's producer skips its env step
                if (hstep && lane < gs) {
                    const uint32_t i = og * (uint32_t)gs + (uint32_t)lane;
                    met_r += env_step_group(a, C, i, i < n32, m0, m1, st0, met_n);
                }
                STAMP(23);
            }
        }
        // K env steps per launch (rdd_step_accum): the images stay in LDS and the gradient
        // partials in registers over all K; a pair that owns one group keeps its envs' state in
        // registers from one step to the next (the rest re-read the state they wrote)
        // (KS: st0 carries it over)
        const uint32_t K = KS ? (uint32_t)a.ksteps : 1u;
        const bool resident = KS && gfirst + gstride >= ngroups;
        for (uint32_t kk = 0;; ++kk) {   // (K = 1: no loop; the K = 1 instances' ISA is that of round 4)
        for (uint32_t grp = gfirst; ok && grp < ngroups; grp += gstride, ++k) {
            STAMP(8);
            const uint32_t Ck = C + kk;   // the episode clock of this env step
            const uint32_t base = grp * (uint32_t)gs;
            const uint32_t i = base + (uint32_t)lane;   // n <= 2^31 (rdd_create)
            const bool lvalid = lane < gs && i < n32;   // this lane has an env
            float* obs = PS + P_SO;
            float* act = PS + P_ACT;
            rd::State st{};   // this lane's env, kept in registers for the env.step after the tiles
            if (k == 0) {
                st = st0;   // observations formed in the prologue
            } else if (resident) {
                if (lvalid) st = st0;   // the state this lane stepped at the previous env step
                group_obs(k, i, lvalid, st);
            } else {
                if (!a.obs_in && lvalid) load_state(a.state, a.n, i, st);
                group_obs(k, i, lvalid, st);
            }
            STAMP(11);
            wave_sync();
            if constexpr (TC) publish(flags + 2, k + 1);   // this group's observation rows are in P_SO
            const int ntile = (int)min((uint32_t)(gs / TILE), (n32 - base + TILE - 1) / TILE);
            for (int t = 0; t < ntile; ++t) {
                const bool tvalid = base + TILE * t + j < a.n;
                const float* obt = obs + TILE * t * SOS;
                f32x4 H1[4], H2[4];
                float mt0, mt1, ms0, ms1;
                float rl0 = tl0, rl1 = tl1, rr0 = rtv0, rr1 = rtv1;   // this row's teacher log-std, 1/var
                STAMP(10);
                if constexpr (TGT) {
                    // the reference's t_pdflat feed (mlp_train.py:146-161): this env's recorded
                    // teacher mean and log-std instead of a teacher query; the student alone runs
                    const uint32_t row = base + TILE * t + j;
                    const f32x4 tq = tvalid ? ld4(a.tnet + (size_t)row * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
                    if constexpr (BS) mlp_forward_bf16(LS, obt, j, g, H1, H2, ms0, ms1);
                    else if constexpr (SPL) mlp_forward_split_t<true>(LS, obt, j, g, H1, H2, ms0, ms1);
                    else mlp_forward(LS, obt, j, g, H1, H2, ms0, ms1);
                    mt0 = tq[0];
                    mt1 = tq[1];
                    rl0 = tq[2];
                    rl1 = tq[3];
                    rr0 = 1.0f / __expf(2.0f * rl0);
                    rr1 = 1.0f / __expf(2.0f * rl1);
                } else if constexpr (HLP) {
                    if (k == 0) {
                        // owner: the student's forward of its tile; the teacher's comes from the
                        // helper pair on another SIMD (gs = 16: one tile, t = 0)
                        if constexpr (SPL) mlp_forward_split_t<true>(LS, obt, j, g, H1, H2, ms0, ms1);
                        else mlp_forward<true>(LS, obt, j, g, H1, H2, ms0, ms1);
                        const float* hp = lds + TN + SN + (pair + 2) * PSCR;
                        if (!(ok = wait_ge(reinterpret_cast<const uint32_t*>(hp + P_FLAGS), 1u, err))) break;
                        mt0 = hp[P_ACT + 2 * j];
                        mt1 = hp[P_ACT + 2 * j + 1];
                    } else {   // later groups (not launched in this layout): both forwards here
                        if constexpr (SPL) mlp_forward_pair_split(LT, LS, obt, j, g, H1, H2, mt0, mt1, ms0, ms1);
                        else mlp_forward_pair<true>(LT, LS, obt, j, g, H1, H2, mt0, mt1, ms0, ms1);
                    }
                } else if constexpr (BS) {
                    if (TC && (t & 1)) {   // the consumer ran this tile's teacher forward
                        mlp_forward_bf16(LS, obt, j, g, H1, H2, ms0, ms1);
                        if (!(ok = wait_ge(flags + 3, ++tct, err))) break;
                        mt0 = PS[P_TM + 2 * j];
                        mt1 = PS[P_TM + 2 * j + 1];
                    } else {
                    // CP, KS: in these kernels' schedules the compiler issues loads into the SrcC
                    // registers of the exact teacher's f32 MFMAs: fenced (see mfma())
                    if constexpr (SPL) mlp_forward_split(LT, obt, j, g, mt0, mt1);
                    else mlp_forward<CP || KS || TC>(LT, obt, j, g, H1, H2, mt0, mt1);
                    mlp_forward_bf16(LS, obt, j, g, H1, H2, ms0, ms1);
                    }
                } else {
                    // exact f32: unfenced, hipcc issues a W3 load / an A-operand prefetch into the SrcC
                    // registers of an in-flight f32 MFMA of layer 2 (hazards.py scan_ldsrc).  Fencing
                    // k-steps 9, 11 and 15 (kPairFence) leaves no such load in any instance -- the
                    // hygiene test re-checks the built ISA -- at 3 % of the kernel, where fencing all
                    // 16 cost 16 % (c4 exact 110.1 / 113.8 / 128.0 us per step unfenced / kPairFence /
                    // every step, profiles/r06a_*, r06b_*)
                    if constexpr (SPL) mlp_forward_pair_split(LT, LS, obt, j, g, H1, H2, mt0, mt1, ms0, ms1);
                    else mlp_forward_pair<false, kPairFence>(LT, LS, obt, j, g, H1, H2, mt0, mt1, ms0, ms1);
                }
                STAMP(12);
                // loss
                const float d0 = ms0 - mt0, d1 = ms1 - mt1;
                float dm0, dm1, dl0 = 0.0f, dl1 = 0.0f, lossv;
                if (a.loss == RDD_LOSS_MSE) {
                    dm0 = d0 * a.inv_n_global;
                    dm1 = d1 * a.inv_n_global;
                    lossv = (d0 * d0 + d1 * d1) * (0.5f * a.inv_n_global);
                } else {
                    dm0 = d0 * rr0;
                    dm1 = d1 * rr1;
                    dl0 = sv0 * rr0 - 1.0f;
                    dl1 = sv1 * rr1 - 1.0f;
                    lossv = (rl0 - sl0 + (sv0 + d0 * d0) * (0.5f * rr0) - 0.5f) +
                            (rl1 - sl1 + (sv1 + d1 * d1) * (0.5f * rr1) - 0.5f);
                }
                if (!tvalid) { dm0 = dm1 = dl0 = dl1 = 0.0f; }
                if (g == 0 && tvalid) {
                    met_l += lossv;
                    met_m += d0 * d0 + d1 * d1;
                    gb3a += dm0; gb3b += dm1; gls0 += dl0; gls1 += dl1;
                    if (!CP) {   // the producer steps the envs itself, after the group's tiles
                        act[(TILE * t + j) * 2] = a.act_student ? ms0 : mt0;
                        act[(TILE * t + j) * 2 + 1] = a.act_student ? ms1 : mt1;
                    }
                }
                // dW3 partials (env j of this lane) and dZ2 = (W3 . dmean) * (1 - H2^2)
                f32x4 dZ[4];
#pragma unroll
                for (int fb = 0; fb < 4; ++fb) {
                    const f32x4 wa = ld4(LS + SW3 + (16 * fb + 4 * g) * 2);
                    const f32x4 wb = ld4(LS + SW3 + (16 * fb + 4 * g) * 2 + 4);
                    const float w0[4] = {wa[0], wa[2], wb[0], wb[2]}, w1[4] = {wa[1], wa[3], wb[1], wb[3]};
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float h = H2[fb][r];
                        gw3a[fb][r] = fmaf(h, dm0, gw3a[fb][r]);
                        gw3b[fb][r] = fmaf(h, dm1, gw3b[fb][r]);
                        dZ[fb][r] = fmaf(w0[r], dm0, w1[r] * dm1) * fmaf(-h, h, 1.0f);
                    }
                }
                // hand the tile over: H1^T, dZ2^T (env-major rows) into the slot
                STAMP(2);
                if (!(ok = wait_ge(flags + 1, tiles, err))) break;
                STAMP(3);
                float* h1t = PS + P_H1T;
                float* dzt = PS + P_DZT;
#pragma unroll
                for (int fb = 0; fb < 4; ++fb) {
                    st4(h1t + j * SAS + 16 * fb + 4 * g, H1[fb]);
                    st4(dzt + j * SAS + 16 * fb + 4 * g, dZ[fb]);
                }
                if (lane < TILE * SOS / 4) st4(PS + P_SOB + 4 * lane, ld4(obt + 4 * lane));
                if (CP && g == 0) {   // the consumer steps these envs: their actions travel with the slot
                    PS[P_SACT + 2 * j] = a.act_student ? ms0 : mt0;
                    PS[P_SACT + 2 * j + 1] = a.act_student ? ms1 : mt1;
                }
                publish(flags, ++tiles);
            }
            if (!ok) break;
            // ---------------------------------------------------------- env.step (one env per lane)
            // !CP: the producer computed this group's actions itself, so it steps the envs at
            // once from the state it holds (the consumer's share is then the gradient tiles
            // only).  CP: the consumer steps them after its last tile of the group, which
            // balances the roles when the producer's forward is the longer one (split / bf16).
            STAMP(4);
            if constexpr (!CP) {
                if (a.obs_in) {   // observation-batch mode: no env to step
                    if (lvalid) met_n += 1.0f;
                } else if (HLP && k == 0 && !a.act_student) {
                    // the helper pair steps these envs (above)
                } else {
                    wave_sync();   // act[] rows were written by the g = 0 lanes of each tile
                    if (lane < gs) met_r += env_step_group(a, Ck, i, lvalid, act[lane * 2], act[lane * 2 + 1], st, met_n);
                }
            }
            if constexpr (KS) st0 = st;
            STAMP(5);
        }
        if (!KS || !ok || kk + 1 >= K) break;
        }
        // ------------------------------------------------------------ this wave's share
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int r = 0; r < 4; ++r)   // sum over the env axis (the 16 lanes of a row)
#pragma unroll
                for (int o = 8; o >= 1; o >>= 1) {
                    gw3a[x][r] += __shfl_xor(gw3a[x][r], o, 16);
                    gw3b[x][r] += __shfl_xor(gw3b[x][r], o, 16);
                }
        gb3a = wave_sum(gb3a); gb3b = wave_sum(gb3b);
        gls0 = wave_sum(gls0); gls1 = wave_sum(gls1);
        met_l = wave_sum(met_l); met_m = wave_sum(met_m);
        met_r = wave_sum(met_r); met_n = wave_sum(met_n);
        STAMP(6);
        __syncthreads();   // (one of the two barriers every wave meets) weights/scratch are free
        STAMP(9);
        float* R = lds + pair * RPAD + RSHIFT;   // pair p fills region p (entries past W2: ridx = p + RSHIFT)
        if (j == 0) {
#pragma unroll
            for (int fb = 0; fb < 4; ++fb)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int f = 16 * fb + 4 * g + r;
                    R[P_W3 + 2 * f] = gw3a[fb][r];
                    R[P_W3 + 2 * f + 1] = gw3b[fb][r];
                }
        }
        if (lane == 0) {
            R[P_B3] = gb3a; R[P_B3 + 1] = gb3b; R[P_LS] = gls0; R[P_LS + 1] = gls1;
            R[P_TOT + 1] = met_l; R[P_TOT + 2] = met_m;
            if constexpr (!CP) { R[P_TOT] = met_r; R[P_TOT + 3] = met_n; }
        }
    } else {
        // ============================================================ consumer wave
        // partial sums: dW2, dW1 (+db1 in row 11), db2 (envs 4s+g of feature 16x+j), rewards
        f32x4 gW2[4][4], gW1[4];
        float gb2[4];
        // split mode and the bf16 student: dW2 in 32 x 32 blocks (v_mfma_f32_32x32x16_bf16) and db2 of
        // features 32 nb + (lane & 31) over the envs of this lane half
        constexpr bool D32 = SPL || BS;
        f32x16 gW2s[2][2];
        float gb2s[2] = {0.f, 0.f};
#pragma unroll
        for (int x = 0; x < 4; ++x) {
#pragma unroll
            for (int y = 0; y < 4; ++y) gW2[x][y] = f32x4{0.f, 0.f, 0.f, 0.f};
            gW1[x] = f32x4{0.f, 0.f, 0.f, 0.f};
            gb2[x] = 0.0f;
        }
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y)
#pragma unroll
                for (int r = 0; r < 16; ++r) gW2s[x][y][r] = 0.0f;
        const int c32 = lane & 31, h32 = lane >> 5;   // D32: the 32 x 32 operand / accumulator lane map
        // student filter of input j for the dW1 A operand (lane-constant)
        const float smu = j < 12 ? LS[SMU + j] : 0.0f, srs = j < 12 ? LS[SRS + j] : 0.0f;
        float met_r = 0.0f, met_n = 0.0f;   // CP: reward and env count of the envs this wave steps
        uint32_t tiles = 0;   // tiles taken from the slot (the pair's global tile count)
        bool ok = true;
        // backward of the pair's next tile (tile t of its group): its slot is taken (tiles + 1
        // published), read, freed, and its gradients accumulated
        float act0 = 0.0f, act1 = 0.0f;   // CP: the action of this lane's env (taken from its tile's slot)
        auto bwd_tile = [&](int t) -> bool {
            STAMP(2);
            if (!wait_ge(flags, tiles + 1, err)) return false;
            STAMP(3);
            // read the whole slot, then free it for the producer's next tile
            const float* h1t = PS + P_H1T;
            const float* dzt = PS + P_DZT;
            // dW1 inputs: raw input j of the tile's envs 4g + e (BS) / 4e + g, e < 4
            float xin[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) xin[e] = PS[P_SOB + (BS ? 4 * g + e : 4 * e + g) * SOS + (j < 12 ? j : 0)];
            f32x4 H1[4], dZ[4], acc[4];
            if constexpr (BS) {
                // dW2 operands over the tile's envs 4g..4g+3 (K = 16 envs), rounded to bf16
                // dW2 on v_mfma_f32_32x32x16_bf16 (as dw2_split32's layout, one product per block): K =
                // the tile's 16 envs, lane half h32 carries envs 8h..8h+7, operands rounded to bf16
                bf16x8 xa8[2], yb8[2];
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    float xv[8], yv[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        xv[e] = h1t[(8 * h32 + e) * SAS + 32 * b + c32];   // H1[32b + c][env 8h+e]
                        yv[e] = dzt[(8 * h32 + e) * SAS + 32 * b + c32];   // dZ2[32b + c][env 8h+e]
                    }
                    gb2s[b] += ((yv[0] + yv[1]) + (yv[2] + yv[3])) + ((yv[4] + yv[5]) + (yv[6] + yv[7]));   // db2 (f32)
                    xa8[b] = pack8(f32x4{xv[0], xv[1], xv[2], xv[3]}, f32x4{xv[4], xv[5], xv[6], xv[7]});
                    yb8[b] = pack8(f32x4{yv[0], yv[1], yv[2], yv[3]}, f32x4{yv[4], yv[5], yv[6], yv[7]});
                }
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    H1[b] = ld4(h1t + j * SAS + 16 * b + 4 * g);   // accumulator layout
                    dZ[b] = ld4(dzt + j * SAS + 16 * b + 4 * g);
                }
                if (CP && (lane >> 4) == t) {
                    act0 = PS[P_SACT + 2 * (lane & 15)];
                    act1 = PS[P_SACT + 2 * (lane & 15) + 1];
                }
                publish(flags + 1, ++tiles);
                STAMP(13);
#pragma unroll
                for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                    for (int nb = 0; nb < 2; ++nb) gW2s[mb][nb] = mfma_32k16(xa8[mb], yb8[nb], gW2s[mb][nb]);
                // dH1 = W2 . dZ2: two K = 32 steps, dZ2 in accumulator layout = the B operand
#pragma unroll
                for (int mb = 0; mb < 4; ++mb) acc[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    const bf16x8 db = pack8(dZ[2 * s], dZ[2 * s + 1]);
#pragma unroll
                    for (int mb = 0; mb < 4; ++mb)
                        acc[mb] = mfma_k32(ldbf8(LS + NB_W2B, (((s * 4 + g) * 4 + mb) * 16 + j) * 8), db, acc[mb]);
                }
            } else {
                // split: dW2 on split bf16 32x32x16 MFMAs, x32[b][e] / y32[b][e] over envs 8h+e (dw2_split32);
                // exact: f32 MFMAs, x[s][b] / y[s][b] over env 4s+g (k-step s)
                constexpr bool S2 = SPL;
                float x[4][4], y[4][4];     // exact
                float x32[2][8], y32[2][8];   // split: dw2_split32's operands
                if constexpr (S2) {
#pragma unroll
                    for (int e = 0; e < 8; ++e)
#pragma unroll
                        for (int b = 0; b < 2; ++b) {
                            x32[b][e] = h1t[(8 * h32 + e) * SAS + 32 * b + c32];   // H1[32b + c][env 8h+e]
                            y32[b][e] = dzt[(8 * h32 + e) * SAS + 32 * b + c32];   // dZ2[32b + c][env 8h+e]
                        }
                } else {
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        x[s][b] = h1t[(4 * s + g) * SAS + 16 * b + j];   // H1[16b + j][env 4s+g]
                        y[s][b] = dzt[(4 * s + g) * SAS + 16 * b + j];   // dZ2[16b + j][env 4s+g]
                    }
                }
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    H1[b] = ld4(h1t + j * SAS + 16 * b + 4 * g);   // accumulator layout
                    dZ[b] = ld4(dzt + j * SAS + 16 * b + 4 * g);
                }
                if (CP && (lane >> 4) == t) {
                    act0 = PS[P_SACT + 2 * (lane & 15)];
                    act1 = PS[P_SACT + 2 * (lane & 15) + 1];
                }
                publish(flags + 1, ++tiles);
                STAMP(13);
                // db2 partials and dW2 += H1^T dZ2 over the tile's 16 envs (K = env)
                bf16x8 dpre[2][3];   // split: the dH1 operand pieces, made before the dW2 MFMAs
                if constexpr (S2) {
                    if constexpr (!HLP) {   // HLP: the helper pair's consumer takes dW2 and db2
#pragma unroll
                        for (int b = 0; b < 2; ++b)
                            gb2s[b] += ((y32[b][0] + y32[b][1]) + (y32[b][2] + y32[b][3])) +
                                       ((y32[b][4] + y32[b][5]) + (y32[b][6] + y32[b][7]));
                    }
                    split8(dZ[0], dZ[1], dpre[0]);
                    split8(dZ[2], dZ[3], dpre[1]);
                    if constexpr (!HLP) dw2_split32(x32, y32, gW2s);
                } else if constexpr (!HLP) {
#pragma unroll
                for (int s = 0; s < 4; ++s) {
#pragma unroll
                    for (int b = 0; b < 4; ++b) gb2[b] += y[s][b];
#pragma unroll
                    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
                        for (int nb = 0; nb < 4; ++nb) gW2[mb][nb] = mfma(x[s][mb], y[s][nb], gW2[mb][nb]);
                }
                }
                // dH1 = W2 . dZ2 (A = W2^T image)
#pragma unroll
                for (int mb = 0; mb < 4; ++mb) acc[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
                if constexpr (S2) {
                    // one scheduling region with the dW2 MFMAs: the splits first, then 80 x (one
                    // MFMA, three VALU), so the dH1 splits issue in the bf16 MFMAs' gaps (c4 82.5 ->
                    // 80.7 us per step, c3/c2 -1.5 %; profiles/r03v_cons_sched.txt)
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
#pragma unroll
                        for (int mb = 0; mb < 4; ++mb) {
                            bf16x8 w[3];
                            ld_pieces(LS, NX_W2B, (((s * 4 + g) * 4 + mb) * 16 + j) * 8, w);
                            acc[mb] = mfma_split(w, dpre[s], acc[mb]);
                        }
                    }
                    __builtin_amdgcn_sched_group_barrier(0x002, 40, 0);
#pragma unroll
                    for (int i = 0; i < (HLP ? 48 : 72); ++i) {   // 24 dW2 (32x32x16) + 48 dH1 MFMAs
                        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
                    }
                } else {
                // exact f32, k-step (fb, r) = W2^T row 16fb + 4g + r.  Each fb group of 16 MFMAs is
                // SrcC-fenced and its operands are loaded one group ahead, before the previous
                // group's fence: no load issues while an f32 MFMA of this loop is in flight (the
                // one-step-ahead prefetch let the compiler issue W2^T loads into in-flight SrcC
                // registers 4-5 wait states after the MFMA; see mfma()).
                f32x4 wc[4], wn[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) wc[r] = ld4(LS + N_W2T + (4 * g + r) * HID + 4 * j);
#pragma unroll
                for (int fb = 0; fb < 4; ++fb) {
                    if (fb < 3) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) wn[r] = ld4(LS + N_W2T + (16 * (fb + 1) + 4 * g + r) * HID + 4 * j);
                    }
                    fence_begin<true>(acc);
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int mb = 0; mb < 4; ++mb) acc[mb] = mfma(wc[r][mb], dZ[fb][r], acc[mb]);
                    fence_end<true>(acc);
#pragma unroll
                    for (int r = 0; r < 4; ++r) wc[r] = wn[r];
                }
                }
            }
            STAMP(14);
            float* sa = PS + P_SA;
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[mb][r] *= fmaf(-H1[mb][r], H1[mb][r], 1.0f);
                st4(sa + j * SAS + 16 * mb + 4 * g, acc[mb]);
            }
            wave_sync();
            // dW1 (+ db1 as input row 11) += z^T dZ1; A = student-filtered inputs of env 4s+g
            if constexpr (BS) {   // K = the tile's 16 envs (4g + jj), operands rounded to bf16
                float zz[4];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    zz[jj] = j < 12 ? fminf(fmaxf((xin[jj] - smu) * srs, -5.0f), 5.0f) : 0.0f;
                }
                const s16x4 za = pack4(zz[0], zz[1], zz[2], zz[3]);
#pragma unroll
                for (int nb = 0; nb < 4; ++nb) {
                    const float* c = sa + 16 * nb + j;
                    gW1[nb] = mfma_k16(za, pack4(c[(4 * g) * SAS], c[(4 * g + 1) * SAS], c[(4 * g + 2) * SAS],
                                                 c[(4 * g + 3) * SAS]), gW1[nb]);
                }
            } else {
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const float z = j < 12 ? fminf(fmaxf((xin[s] - smu) * srs, -5.0f), 5.0f) : 0.0f;
#pragma unroll
                    for (int nb = 0; nb < 4; ++nb) gW1[nb] = mfma(z, sa[(4 * s + g) * SAS + 16 * nb + j], gW1[nb]);
                }
            }
            wave_sync();   // sa is rewritten by the next tile
            STAMP(15);
            return true;
        };
        // after the last tile of a group (envs base ...): CP steps the envs
        auto end_group = [&](uint32_t base, uint32_t Ck) {
            const uint32_t i = base + (uint32_t)lane;
            const bool lvalid = lane < gs && i < n32;
            if constexpr (CP) {
                STAMP(4);
                if (a.obs_in) {
                    if (lvalid) met_n += 1.0f;
                } else if (lane < gs) {   // act[] rows: published with the group's tiles
                    rd::State st{};
                    if (lvalid) load_state(a.state, a.n, i, st);
                    met_r += env_step_group(a, Ck, i, lvalid, act0, act1, st, met_n);
                }
                STAMP(5);
            }
        };
        if constexpr (HLP) {
            // helper pair 2 + o: dW2 = H1^T dZ2 and db2 of owner o's tile, read from the owner's
            // slot beside the owner consumer's dH1 / dW1 (the owner's producer never rewrites the
            // slot: one tile per owner in this layout)
            if (helper && og < ngroups) {
                const float* OP = lds + TN + SN + (pair & 1) * PSCR;
                STAMP(20);
                ok = wait_ge(reinterpret_cast<const uint32_t*>(OP + P_FLAGS), 1u, err);
                STAMP(21);
                if (ok) {
                    const float* h1t = OP + P_H1T;
                    const float* dzt = OP + P_DZT;
                    if constexpr (SPL) {   // as the plain layout's consumer (dw2_split32)
                        float x32[2][8], y32[2][8];
#pragma unroll
                        for (int e = 0; e < 8; ++e)
#pragma unroll
                            for (int b = 0; b < 2; ++b) {
                                x32[b][e] = h1t[(8 * h32 + e) * SAS + 32 * b + c32];
                                y32[b][e] = dzt[(8 * h32 + e) * SAS + 32 * b + c32];
                            }
#pragma unroll
                        for (int b = 0; b < 2; ++b)
                            gb2s[b] += ((y32[b][0] + y32[b][1]) + (y32[b][2] + y32[b][3])) +
                                       ((y32[b][4] + y32[b][5]) + (y32[b][6] + y32[b][7]));
                        dw2_split32(x32, y32, gW2s);
                    } else {
                    float x[4][4], y[4][4];
#pragma unroll
                    for (int s = 0; s < 4; ++s)
#pragma unroll
                        for (int b = 0; b < 4; ++b) {
                            x[s][b] = h1t[(4 * s + g) * SAS + 16 * b + j];
                            y[s][b] = dzt[(4 * s + g) * SAS + 16 * b + j];
                        }
#pragma unroll
                        for (int s = 0; s < 4; ++s) {
#pragma unroll
                            for (int b = 0; b < 4; ++b) gb2[b] += y[s][b];
#pragma unroll
                            for (int mb = 0; mb < 4; ++mb) {
                                fence_begin<true>(gW2[mb]);
#pragma unroll
                                for (int nb = 0; nb < 4; ++nb) gW2[mb][nb] = mfma(x[s][mb], y[s][nb], gW2[mb][nb]);
                                fence_end<true>(gW2[mb]);
                            }
                        }
                    }
                }
                STAMP(22);
            }
        }
        uint32_t gi = 0, tcc = 0;   // TC: groups started, teacher tiles published
        for (uint32_t kk = 0;; ++kk) {
        for (uint32_t grp = gfirst; ok && grp < ngroups; grp += gstride, ++gi) {
            const uint32_t base = grp * (uint32_t)gs;
            const int ntile = (int)min((uint32_t)(gs / TILE), (n32 - base + TILE - 1) / TILE);
            if constexpr (TC) {
                if (!(ok = wait_ge(flags + 2, gi + 1, err))) break;
            }
            for (int t = 0; ok && t < ntile; ++t) {
                if constexpr (TC) {
                    // the teacher forward of the next (odd) tile, from the producer's observation rows:
                    // its means go to P_TM, read by the producer at that tile (one tile in flight: the
                    // producer takes them before it publishes the tile this wave consumes next)
                    if (!(t & 1) && t + 1 < ntile) {
                        const float* obt = PS + P_SO + TILE * (t + 1) * SOS;
                        float m0, m1;
                        if constexpr (SPL) {
                            mlp_forward_split(LT, obt, j, g, m0, m1);
                        } else {
                            f32x4 h1[4], h2[4];
                            mlp_forward<true>(LT, obt, j, g, h1, h2, m0, m1);
                        }
                        if (g == 0) {
                            PS[P_TM + 2 * j] = m0;
                            PS[P_TM + 2 * j + 1] = m1;
                        }
                        publish(flags + 3, ++tcc);
                    }
                }
                ok = bwd_tile(t);
            }
            if (!ok) break;
            end_group(base, C + kk);
        }
        if (!KS || !ok || kk + 1 >= (uint32_t)a.ksteps) break;
        }
        // ------------------------------------------------------------ this wave's share
#pragma unroll
        for (int x = 0; x < 4; ++x) gb2[x] = xsum32(xsum16(gb2[x]));   // over the k-groups g
#pragma unroll
        for (int x = 0; x < 2; ++x) gb2s[x] = xsum32(gb2s[x]);          // D32: over the two lane halves
        if constexpr (CP) { met_r = wave_sum(met_r); met_n = wave_sum(met_n); }
        STAMP(6);
        __syncthreads();   // (one of the two barriers every wave meets) weights/scratch are free
        STAMP(9);
        float* R = lds + pair * RPAD;   // rows of RROW floats: W1|b1 rows 0..11, W2 rows 12..75
        if constexpr (D32) {   // 32 x 32 blocks: column lane & 31, row (reg & 3) + 8 (reg >> 2) + 4 h
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        R[(12 + 32 * mb + (r & 3) + 8 * (r >> 2) + 4 * h32) * RROW + 32 * nb + c32] = gW2s[mb][nb][r];
        } else {
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
#pragma unroll
            for (int nb = 0; nb < 4; ++nb)
#pragma unroll
                for (int r = 0; r < 4; ++r) R[(12 + 16 * mb + 4 * g + r) * RROW + 16 * nb + j] = gW2[mb][nb][r];
        }
        if (g < 3) {   // rows 4g + r < 12: W1 rows 0..10 and b1 as row 11
#pragma unroll
            for (int nb = 0; nb < 4; ++nb)
#pragma unroll
                for (int r = 0; r < 4; ++r) R[(4 * g + r) * RROW + 16 * nb + j] = gW1[nb][r];
        }
        if constexpr (D32) {
            if (h32 == 0) {
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) R[RSHIFT + P_B2 + 32 * nb + c32] = gb2s[nb];
            }
        } else if (g == 0) {
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) R[RSHIFT + P_B2 + 16 * nb + j] = gb2[nb];
        }
        if (CP && lane == 0) {   // the producer's region entries past W2 hold the other metrics
            R[RSHIFT + P_TOT] = met_r;
            R[RSHIFT + P_TOT + 3] = met_n;
        }
    }

    // Both roles passed exactly one s_barrier above (a wave-level count on gfx950, so the
    // two call sites pair up); this second one publishes the regions.
    __syncthreads();
    static_assert(RED_COLS % 4 == 0, "a 16-B store stays inside one workspace chunk");
#pragma unroll
    for (int u = 0; u < (P_PAD / 4 + BLOCK - 1) / BLOCK; ++u) {
        const int p4 = threadIdx.x + u * BLOCK;
        if (p4 < P_PAD / 4) {
            const int q = ridx(4 * p4);   // 4 | 64: the four entries stay contiguous
            gst<BS>(reinterpret_cast<f32x4*>(a.ws + ws_index(4 * p4, blockIdx.x, gridDim.x)),
                       sum4(ld4(lds + q), ld4(lds + RPAD + q), ld4(lds + 2 * RPAD + q), ld4(lds + 3 * RPAD + q)));
        }
    }
    STAMP(7);
    RTSTAMP(17);
}


// Sum the rollout's per-workgroup partials (fixed order: deterministic), then TF1 Adam.
__global__ __launch_bounds__(RED_BLOCK) void reduce_adam_kernel(ReduceArgs a) {
    __shared__ float part[RED_ROWS][RED_COLS];
    if (a.adam && a.xerr && __hip_atomic_load(a.xerr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        // the gradient exchange before this update failed (reacher_comm.h): no replica applies
        // a partial sum; the step is reported by the host readers (ctl[13]) and rdd_step
        a.adam = 0;
        a.bump_opt = 0;
        if (blockIdx.x == 0 && threadIdx.x == 0) a.ctl[13] = 1u;
    }
    const uint32_t C = a.ctl[4], S = a.ctl[5];
    const float b1p = __uint_as_float(a.ctl[6]), b2p = __uint_as_float(a.ctl[7]);
    const int col = threadIdx.x & (RED_COLS - 1), row = threadIdx.x / RED_COLS;
    const int p = blockIdx.x * RED_COLS + col;
    // the Adam operands are loaded first, so their round trip overlaps the partial sums
    float m_p = 0.f, v_p = 0.f, w_p = 0.f;
    if (a.adam && row == 0 && p < P_TOT) {
        m_p = a.m[p];
        v_p = a.v[p];
        w_p = a.params[p];
    }
    if (a.reduce) part[row][col] = p < P_PAD ? col_rows(a.ws, a.nblk, p, row) : 0.f;
    __syncthreads();
    if (row == 0 && p < P_PAD) col_finish(a, p, &part[0][col], RED_COLS, m_p, v_p, w_p, S, b1p, b2p);
    if (blockIdx.x == 0 && threadIdx.x == 0) bump_ctl(a, C, S, b1p, b2p, a.ctl[12]);
}

__global__ __launch_bounds__(256) void reset_state_kernel(int64_t n, int64_t env_base, uint64_t seed, float* state) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float d[6];
    rd::philox_draw(seed, (uint64_t)(env_base + i), 0u, d);
    rd::State st;
    rd::env_reset(st, d);
    state[i] = st.q0; state[n + i] = st.q1; state[2 * n + i] = st.v0; state[3 * n + i] = st.v1;
    state[4 * n + i] = st.tx; state[5 * n + i] = st.ty; state[6 * n + i] = st.dx; state[7 * n + i] = st.dy;
}

// rdd_set_env_state's range check: the fused rollout takes its joint trig on the short paths
// (rd_physics.h, kWideRange = false: joint 1 on the hardware within its limit, joint 0 reduced by
// 2 pi below 8192 rad), which an episode's own states never leave; a caller's state outside that
// range (or not finite) raises flag[0]
__global__ __launch_bounds__(256) void check_state_kernel(int64_t n, const float* state, uint32_t* flag) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float q0 = state[i], q1 = state[n + i];
    if (!(fabsf(q0) < rd::kRolloutMaxQ0) || !(fabsf(q1) <= rd::kRolloutMaxQ1))
        __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void init_ctl_kernel(uint32_t* ctl, float b1, float b2) {
    if (threadIdx.x < 2) {
        const int o = 4 * threadIdx.x;   // live words and their snapshot
        ctl[o] = 0u; ctl[o + 1] = 0u; ctl[o + 2] = __float_as_uint(b1); ctl[o + 3] = __float_as_uint(b2);
    }
    if (threadIdx.x >= 8 && threadIdx.x < 16) ctl[threadIdx.x] = threadIdx.x == 12 ? 1u : 0u;
}

// policy query: obs rows -> pdflat of teacher and/or student (one 16-env tile per wave pass)
template <bool BS>
__global__ __launch_bounds__(FBLOCK) void forward_kernel(const float* tnet, const float* snet, const float* obs,
                                                         int64_t n, float* tflat, float* sflat) {
    __shared__ __attribute__((aligned(16))) float lds[NET + NET_S + FWAVES * TILE * SOS];
    load_net(lds, tnet, false, FBLOCK);
    if constexpr (BS) load_net_bf16(lds + NET, snet, FBLOCK);
    else load_net(lds + NET, snet, false, FBLOCK);
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
    float* ob = lds + NET + NET_S + wave * TILE * SOS;
    const int64_t ntiles = (n + TILE - 1) / TILE;
    for (int64_t t = (int64_t)blockIdx.x * FWAVES + wave; t < ntiles; t += (int64_t)gridDim.x * FWAVES) {
        // raw observations of the tile's 16 envs -> scratch rows (component 11 = 1)
        for (int x = lane; x < TILE * SOS; x += 64) {
            const int e = x / SOS, k = x % SOS;
            const int64_t i = t * TILE + e;
            ob[x] = k == OBD ? 1.0f : (i < n ? obs[i * OBD + k] : 0.0f);
        }
        wave_sync();
        const int64_t i = t * TILE + j;
        f32x4 H1[4], H2[4];
        float m0, m1;
        for (int net = 0; net < 2; ++net) {
            float* out = net ? sflat : tflat;
            if (!out) continue;   // wave-uniform
            const float* L = lds + net * NET;
            float ls0 = L[N_LS], ls1 = L[N_LS + 1];
            if (BS && net == 1) {
                mlp_forward_bf16(L, ob, j, g, H1, H2, m0, m1);
                ls0 = L[NB_LS]; ls1 = L[NB_LS + 1];
            } else {
                // BS: beside the bf16 student's forward hipcc issues an LDS load into the SrcC of
                // one of the teacher's in-flight f32 MFMAs (hazards.py LDSRC): fenced (see mfma())
                mlp_forward<BS>(L, ob, j, g, H1, H2, m0, m1);
            }
            if (i < n && g == 0) {
                out[i * 4 + 0] = m0;
                out[i * 4 + 1] = m1;
                out[i * 4 + 2] = ls0;
                out[i * 4 + 3] = ls1;
            }
        }
        wave_sync();
    }
}

int num_cus(int device) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 256;
    return prop.multiProcessorCount;
}

}  // namespace

struct rdd_trainer {
    rdd_config cfg{};
    int device = 0;
    hipStream_t stream = nullptr;
    int grid = 0;
    float* state = nullptr;    // [8][n]
    float* tnet = nullptr;     // [P + 22]
    float* snet = nullptr;     // [P + 22]
    float* timg = nullptr;     // [NET]   teacher LDS image
    float* simg = nullptr;     // [NET_S] student LDS image
    float* m = nullptr;
    float* v = nullptr;
    float* grad = nullptr;     // [P] (own or bound)
    float* own_grad = nullptr;
    float* ws = nullptr;       // partials of up to ws_rows workgroups (ws_index layout)
    float* hist = nullptr;     // [hist_len][4]
    uint32_t* ctl = nullptr;   // [16]: step words, snapshot, [8] hand-off timeout flag
    unsigned long long* dbg = nullptr;   // RD_STAMPS builds only
    int last_grid = 0;                   // workgroups of the last rollout (rows of ws to reduce)
    int ws_rows = 0;                     // rows of ws (the device's CU count, or cfg.grid)
    int gs = GROUP;                      // envs per group of the env rollout
    int accum = 1;                       // rollouts per optimiser step (MSE normalisation)
    rd_comm* comm = nullptr;             // bound RCCL communicator (multi-GPU), not owned

};

namespace {

// Envs per group (one producer/consumer pair steps a group of gs envs, gs/16 tiles at a
// time): 64 fills every lane of the physics and is fastest from one group per pair up
// (measured: c3 = one 64-env group per pair 39.6 us vs 41.9 with 32-env groups); below
// that a pair's tiles run serially while most CUs idle, so small batches use 32- or 16-env
// groups over more pairs (c2, 4,096 envs: 19.1 us per launch vs 35.4 with 64-env groups).
// rdd_config.group_envs = 16|32|64 fixes it (tests: the group size changes only the
// summation order).
int group_envs(int64_t n, int pairs_total, int fixed) {
    if (fixed) return fixed;
    if (n >= (int64_t)GROUP * pairs_total) return 64;
    if (n >= (int64_t)32 * pairs_total) return 32;
    return 16;
}

// LDS image kinds and sizes (floats) of a trainer's teacher and student
int teacher_kind(const rdd_trainer* t) { return t->cfg.f32_split ? IMG_SPLIT : IMG_F32; }
int student_kind(const rdd_trainer* t) {
    return t->cfg.student_dtype == RDD_DTYPE_BF16 ? IMG_BF16 : (t->cfg.f32_split ? IMG_SPLIT : IMG_F32);
}
int image_floats(int kind, bool student) {
    if (kind == IMG_SPLIT) return student ? NETX_S : NETX;
    if (kind == IMG_BF16) return NETB_S;
    return student ? NET_S : NET;
}

// Which wave of a pair steps the envs.  The bf16 student (BASELINE config 5):
// the consumer, after its last tile of a group (the actions travel with each tile's slot):
// this balances the roles, since the producer's forward (f32 teacher + bf16 student) is the
// longer one.  Its MFMAs are all bf16 (XDL: the compiler protects their SrcC) except the
// exact teacher's f32 ones, which are SrcC-fenced.  The f32 student: the producer steps the
// envs it computed the actions for (a consumer-side step there measured c4 -0.8 %, c3 +2.7 %,
// c2 +3.7 % and would need the consumer's f32 MFMAs fenced; profiles/r03h_cp_f32_and_nopack.txt).
int grid_for(int64_t n, int gs, int cap) {
    const int64_t want = ((n + gs - 1) / gs + PAIRS - 1) / PAIRS;   // one group per pair at least
    return (int)(want < cap ? want : cap);
}

ReduceArgs reduce_args(const rdd_trainer* t, int reduce, int adam, int accum) {
    ReduceArgs a;
    a.ws = t->ws;
    a.nblk = t->last_grid;
    a.grad = t->grad;
    a.params = t->snet;
    a.m = t->m;
    a.v = t->v;
    a.ctl = t->ctl;
    a.hist = t->hist;
    a.hist_len = t->cfg.metrics_len;
    a.reduce = reduce;
    a.adam = adam;
    a.accum = accum;
    a.bump_env = reduce;
    a.bump_opt = adam;
    a.lr = t->cfg.lr;
    a.b1 = t->cfg.beta1;
    a.b2 = t->cfg.beta2;
    a.eps = t->cfg.eps;
    a.simg = t->simg;
    a.img_kind = student_kind(t);
    a.xerr = rd_comm_device_err(t->comm);
    return a;
}

int launch_rollout(rdd_trainer* t, const float* obs_in = nullptr, int64_t n_obs = 0, int64_t n_obs_global = 0,
                   const float* tflat_in = nullptr, int ksteps = 1) {
    RolloutArgs a;
    a.ksteps = ksteps;
    a.n = obs_in ? n_obs : t->cfg.n_envs;
    a.obs_in = obs_in;
    a.timg = t->timg;
    a.simg = t->simg;
    a.env_base = t->cfg.env_base;
    a.seed = t->cfg.seed;
    a.state = t->state;
    a.tnet = tflat_in ? tflat_in : t->tnet;   // rows mode: the recorded teacher outputs
    a.snet = t->snet;
    a.ctl = t->ctl;
    a.ws = t->ws;
    a.loss = t->cfg.loss;
    a.act_student = t->cfg.act_with == RDD_ACT_STUDENT;
    a.stagger = t->cfg.stagger;
    a.dbg = t->dbg;
    // MSE averages over the envs of all ranks and over the accum_steps rollouts of one optimiser step
    a.inv_n_global = obs_in ? 1.0f / (float)n_obs_global : 1.0f / ((float)t->cfg.n_envs_global * (float)t->accum);
    int grid = t->grid;   // <= t->ws_rows, the partial rows the workspace holds
    a.gs = t->gs;
    if (obs_in) {
        a.gs = group_envs(n_obs, t->ws_rows * PAIRS, t->cfg.group_envs);
        grid = grid_for(n_obs, a.gs, t->ws_rows);
    }
    const bool bs = t->cfg.student_dtype == RDD_DTYPE_BF16, spl = t->cfg.f32_split != 0;
    // helper pairs (f32 student): every group one 16-env tile and at most two groups per
    // workgroup -- the batch would leave half the pairs idle or hold one tile each, so pairs 2,
    // 3 run the owners' teacher forwards on the other SIMDs instead (c2: DESIGN.md §3)
    const int64_t ngroups = (a.n + a.gs - 1) / a.gs;
    const bool hlp = !bs && !tflat_in && a.gs == TILE && ngroups <= 2 * (int64_t)t->ws_rows &&
                     t->cfg.group_envs == 0 &&   // a fixed group size keeps the plain layout
                     ksteps == 1;                // K env steps per launch: the plain layout
    if (hlp) grid = (int)((ngroups + 1) / 2);
    t->last_grid = grid;
    void (*k)(RolloutArgs) =
        bs ? (spl ? rollout_kernel<true, true, true, MD_TEACHER, false, true>   // TC: DESIGN.md §3 "c5"
                  : rollout_kernel<true, false, true, MD_TEACHER>)
           : hlp ? (spl ? rollout_kernel<false, true, false, MD_HELPER> : rollout_kernel<false, false, false, MD_HELPER>)
                 : (spl ? rollout_kernel<false, true, false, MD_TEACHER> : rollout_kernel<false, false, false, MD_TEACHER>);
    if (ksteps > 1)   // K steps per launch: the producer steps the envs it reads (no CP)
        k = bs ? (spl ? rollout_kernel<true, true, false, MD_TEACHER, true> : rollout_kernel<true, false, false, MD_TEACHER, true>)
               : (spl ? rollout_kernel<false, true, false, MD_TEACHER, true> : rollout_kernel<false, false, false, MD_TEACHER, true>);
    if (tflat_in)   // the teacher is not run: the bf16 student's kernel does not depend on the teacher's mode
        k = bs ? rollout_kernel<true, false, false, MD_ROWS>
               : (spl ? rollout_kernel<false, true, false, MD_ROWS> : rollout_kernel<false, false, false, MD_ROWS>);
    hipLaunchKernelGGL(k, dim3(grid), dim3(BLOCK), 0, t->stream, a);
    RD_HIP(hipGetLastError(), "rollout_kernel launch");
    return RD_OK;
}

// reduce: partials -> grad (accum: +=) and advance the env clock; adam: TF1 Adam and
// advance the optimiser step
int launch_reduce(rdd_trainer* t, int reduce, int adam, int accum = 0) {
    const ReduceArgs a = reduce_args(t, reduce, adam, accum);
    hipLaunchKernelGGL(reduce_adam_kernel, dim3(RED_GRID), dim3(RED_BLOCK), 0, t->stream, a);
    RD_HIP(hipGetLastError(), "reduce_adam_kernel launch");
    return RD_OK;
}

}  // namespace

extern "C" {

int rdd_param_count(void) { return P_TOT; }

int rdd_set_stream(rdd_trainer* t, void* hip_stream) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_set_stream: null handle");
    t->stream = (hipStream_t)hip_stream;
    return RD_OK;
}

int rdd_create(rdd_trainer** out, const rdd_config* cfg, int device, void* hip_stream) {
    if (!out || !cfg) return rd::set_error(RD_EINVAL, "rdd_create: null argument");
    if (cfg->n_envs <= 0 || cfg->n_envs_global < cfg->n_envs || cfg->env_base < 0 ||
        cfg->n_envs > ((int64_t)1 << 31) || (cfg->loss != RDD_LOSS_MSE && cfg->loss != RDD_LOSS_KL) ||
        (cfg->act_with != RDD_ACT_TEACHER && cfg->act_with != RDD_ACT_STUDENT) || !(cfg->lr > 0) ||
        cfg->grid < 0 || cfg->metrics_len < 0 || (cfg->stagger != 0 && cfg->stagger != 1) ||
        (cfg->student_dtype != RDD_DTYPE_F32 && cfg->student_dtype != RDD_DTYPE_BF16) || cfg->accum_steps < 0 ||
        (cfg->f32_split != 0 && cfg->f32_split != 1) ||
        (cfg->group_envs != 0 && cfg->group_envs != 16 && cfg->group_envs != 32 && cfg->group_envs != 64))
        return rd::set_error(RD_EINVAL, "rdd_create: bad config");
    rd::DeviceGuard g(device);
    RD_HIP(g.err, "rdd_create: hipSetDevice");
    rdd_trainer* t = new (std::nothrow) rdd_trainer();
    if (!t) return rd::set_error(RD_EINVAL, "rdd_create: out of host memory");
    t->cfg = *cfg;
    if (t->cfg.metrics_len == 0) t->cfg.metrics_len = 4096;
    t->accum = cfg->accum_steps > 1 ? cfg->accum_steps : 1;
    t->device = device;
    t->stream = (hipStream_t)hip_stream;
    const int cap = cfg->grid > 0 ? cfg->grid : num_cus(device);
    t->ws_rows = cap;
    t->gs = group_envs(cfg->n_envs, cap * PAIRS, cfg->group_envs);
    t->grid = grid_for(cfg->n_envs, t->gs, cap);
    t->last_grid = t->grid;
    const size_t netf = P_TOT + 2 * OBD;
    hipError_t e = hipSuccess;
    auto alloc = [&](void** p, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc(p, bytes);
        if (e == hipSuccess) e = hipMemsetAsync(*p, 0, bytes, t->stream);
    };
    alloc((void**)&t->state, sizeof(float) * 8 * cfg->n_envs);
    alloc((void**)&t->tnet, sizeof(float) * netf);
    alloc((void**)&t->snet, sizeof(float) * netf);
    alloc((void**)&t->timg, sizeof(float) * image_floats(teacher_kind(t), false));
    alloc((void**)&t->simg, sizeof(float) * image_floats(student_kind(t), true));
    alloc((void**)&t->m, sizeof(float) * P_TOT);
    alloc((void**)&t->v, sizeof(float) * P_TOT);
    alloc((void**)&t->own_grad, sizeof(float) * P_TOT);
    t->grad = t->own_grad;
    alloc((void**)&t->ws, sizeof(float) * (size_t)t->ws_rows * P_WS);
    alloc((void**)&t->hist, sizeof(float) * (size_t)t->cfg.metrics_len * N_MET);
    alloc((void**)&t->ctl, sizeof(uint32_t) * 16);
#ifdef RD_STAMPS
    alloc((void**)&t->dbg, sizeof(unsigned long long) * (size_t)t->ws_rows * WAVES * NSTAMP);
#endif
    if (e != hipSuccess) {
        rdd_destroy(t);
        return rd::hip_fail(e, "rdd_create: allocation");
    }
    *out = t;
    return RD_OK;
}

int rdd_destroy(rdd_trainer* t) {
    if (!t) return RD_OK;
    rd::DeviceGuard g(t->device);
    for (void* p : {(void*)t->state, (void*)t->tnet, (void*)t->snet, (void*)t->m, (void*)t->v, (void*)t->own_grad,
                    (void*)t->ws, (void*)t->hist, (void*)t->ctl, (void*)t->dbg, (void*)t->timg, (void*)t->simg})
        if (p) (void)hipFree(p);
    delete t;
    return RD_OK;
}

static int set_net(rdd_trainer* t, float* dst, const float* params, const float* mu, const float* sd,
                   const char* what) {
    if (!t || !params || !mu || !sd) return rd::set_error(RD_EINVAL, "%s: null argument", what);
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, what);
    RD_HIP(hipMemcpyAsync(dst, params, sizeof(float) * P_TOT, hipMemcpyDeviceToDevice, t->stream), what);
    RD_HIP(hipMemcpyAsync(dst + P_TOT, mu, sizeof(float) * OBD, hipMemcpyDeviceToDevice, t->stream), what);
    RD_HIP(hipMemcpyAsync(dst + P_TOT + OBD, sd, sizeof(float) * OBD, hipMemcpyDeviceToDevice, t->stream), what);
    const bool student = dst == t->snet;
    const int kind = student ? student_kind(t) : teacher_kind(t);
    hipLaunchKernelGGL(pack_net_kernel, dim3(1), dim3(256), 0, t->stream, dst, student ? t->simg : t->timg,
                       image_floats(kind, student), student ? 1 : 0, kind);
    RD_HIP(hipGetLastError(), what);
    return RD_OK;
}

int rdd_set_teacher(rdd_trainer* t, const float* p, const float* mu, const float* sd) {
    return set_net(t, t ? t->tnet : nullptr, p, mu, sd, "rdd_set_teacher");
}

int rdd_set_student(rdd_trainer* t, const float* p, const float* mu, const float* sd) {
    return set_net(t, t ? t->snet : nullptr, p, mu, sd, "rdd_set_student");
}

int rdd_get_student(rdd_trainer* t, float* params) {
    if (!t || !params) return rd::set_error(RD_EINVAL, "rdd_get_student: null argument");
    rd::DeviceGuard g(t->device);
    RD_HIP(hipMemcpyAsync(params, t->snet, sizeof(float) * P_TOT, hipMemcpyDeviceToDevice, t->stream),
           "rdd_get_student");
    return RD_OK;
}

int rdd_reset(rdd_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_reset: null handle");
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_reset: hipSetDevice");
    const int64_t n = t->cfg.n_envs;
    hipLaunchKernelGGL(reset_state_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, t->stream, n,
                       t->cfg.env_base, t->cfg.seed, t->state);
    hipLaunchKernelGGL(init_ctl_kernel, dim3(1), dim3(64), 0, t->stream, t->ctl, t->cfg.beta1, t->cfg.beta2);
    RD_HIP(hipMemsetAsync(t->m, 0, sizeof(float) * P_TOT, t->stream), "rdd_reset");
    RD_HIP(hipMemsetAsync(t->v, 0, sizeof(float) * P_TOT, t->stream), "rdd_reset");
    RD_HIP(hipGetLastError(), "rdd_reset: launch");
    return RD_OK;
}

int rdd_rollout(rdd_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_rollout: null handle");
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_rollout: hipSetDevice");
    if (int rc = launch_rollout(t)) return rc;
    return launch_reduce(t, 1, 0);
}

// a bound exchange that failed earlier (reacher_comm.h): no further steps on this trainer
static int comm_ok(const rdd_trainer* t, const char* what) {
    if (rd_comm_failed(t->comm))
        return rd::set_error(RD_ECOMM, "%s: a gradient exchange of this trainer failed (its optimiser step was "
                                       "skipped); destroy the communicator", what);
    return RD_OK;
}

int rdd_rollout_accum(rdd_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_rollout_accum: null handle");
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_rollout_accum: hipSetDevice");
    if (int rc = launch_rollout(t, nullptr, 0, 0, nullptr, t->accum)) return rc;
    return launch_reduce(t, 1, 0);
}

int rdd_apply(rdd_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_apply: null handle");
    if (int rc = comm_ok(t, "rdd_apply")) return rc;
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_apply: hipSetDevice");
    return launch_reduce(t, 0, 1);
}

int rdd_step(rdd_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_step: null handle");
    if (int rc = comm_ok(t, "rdd_step")) return rc;
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_step: hipSetDevice");
    if (int rc = launch_rollout(t)) return rc;
    if (!t->comm) return launch_reduce(t, 1, 1);
    // sharded step: the exchange sits between the reduction and Adam, all on one stream
    if (int rc = launch_reduce(t, 1, 0)) return rc;
    if (int rc = rd_comm_allreduce_f32(t->comm, t->grad, P_TOT, t->stream)) return rc;
    return launch_reduce(t, 0, 1);
}

int rdd_step_accum(rdd_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_step_accum: null handle");
    if (int rc = comm_ok(t, "rdd_step_accum")) return rc;
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_step_accum: hipSetDevice");
    if (int rc = launch_rollout(t, nullptr, 0, 0, nullptr, t->accum)) return rc;
    if (!t->comm) return launch_reduce(t, 1, 1);
    if (int rc = launch_reduce(t, 1, 0)) return rc;
    if (int rc = rd_comm_allreduce_f32(t->comm, t->grad, P_TOT, t->stream)) return rc;
    return launch_reduce(t, 0, 1);
}

int rdd_bind_comm(rdd_trainer* t, rd_comm* comm) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_bind_comm: null handle");
    t->comm = comm;
    return RD_OK;
}

int rdd_allreduce_grad(rdd_trainer* t) {
    if (!t || !t->comm) return rd::set_error(RD_EINVAL, "rdd_allreduce_grad: no communicator bound");
    if (int rc = comm_ok(t, "rdd_allreduce_grad")) return rc;
    return rd_comm_allreduce_f32(t->comm, t->grad, P_TOT, t->stream);
}

int rdd_rollout_obs(rdd_trainer* t, const float* obs, int64_t n, int64_t n_global) {
    if (!t || !obs || n <= 0 || n > ((int64_t)1 << 31) || n_global < n)
        return rd::set_error(RD_EINVAL, "rdd_rollout_obs: bad argument");
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_rollout_obs: hipSetDevice");
    if (int rc = launch_rollout(t, obs, n, n_global)) return rc;
    return launch_reduce(t, 1, 0);
}

int rdd_step_obs(rdd_trainer* t, const float* obs, int64_t n) {
    if (!t || !obs || n <= 0 || n > ((int64_t)1 << 31)) return rd::set_error(RD_EINVAL, "rdd_step_obs: bad argument");
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_step_obs: hipSetDevice");
    if (int rc = launch_rollout(t, obs, n, n)) return rc;
    return launch_reduce(t, 1, 1);
}

static int rows_args(rdd_trainer* t, const float* obs, const float* t_pdflat, int64_t n, int64_t n_global,
                     const char* what) {
    if (!t || !obs || !t_pdflat || n <= 0 || n > ((int64_t)1 << 31) || n_global < n)
        return rd::set_error(RD_EINVAL, "%s: bad argument", what);
    if (((uintptr_t)t_pdflat & 15) != 0) return rd::set_error(RD_EINVAL, "%s: t_pdflat must be 16-byte aligned", what);
    return RD_OK;
}

int rdd_rollout_rows(rdd_trainer* t, const float* obs, const float* t_pdflat, int64_t n, int64_t n_global) {
    if (int rc = rows_args(t, obs, t_pdflat, n, n_global, "rdd_rollout_rows")) return rc;
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_rollout_rows: hipSetDevice");
    if (int rc = launch_rollout(t, obs, n, n_global, t_pdflat)) return rc;
    return launch_reduce(t, 1, 0);
}

int rdd_step_rows(rdd_trainer* t, const float* obs, const float* t_pdflat, int64_t n) {
    if (int rc = rows_args(t, obs, t_pdflat, n, n, "rdd_step_rows")) return rc;
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_step_rows: hipSetDevice");
    if (int rc = launch_rollout(t, obs, n, n, t_pdflat)) return rc;
    return launch_reduce(t, 1, 1);
}

int rdd_launch_stage(rdd_trainer* t, int stage) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_launch_stage: null handle");
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_launch_stage: hipSetDevice");
    switch (stage) {
        case RDD_STAGE_ROLLOUT: return launch_rollout(t);
        case RDD_STAGE_REDUCE: return launch_reduce(t, 1, 0);
        case RDD_STAGE_APPLY: return launch_reduce(t, 0, 1);
        case RDD_STAGE_REDUCE_APPLY: return launch_reduce(t, 1, 1);
        case RDD_STAGE_REDUCE_ACCUM: return launch_reduce(t, 1, 0, 1);
        case RDD_STAGE_REDUCE_ACCUM_APPLY: return launch_reduce(t, 1, 1, 1);
        default: return rd::set_error(RD_EINVAL, "rdd_launch_stage: bad stage %d", stage);
    }
}

float* rdd_grad_buffer(rdd_trainer* t) { return t ? t->grad : nullptr; }

int rdd_bind_grad_buffer(rdd_trainer* t, float* grad) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_bind_grad_buffer: null handle");
    t->grad = grad ? grad : t->own_grad;
    return RD_OK;
}

int rdd_forward(rdd_trainer* t, const float* obs, int64_t n, float* tflat, float* sflat) {
    if (!t || !obs || n <= 0) return rd::set_error(RD_EINVAL, "rdd_forward: bad argument");
    rd::DeviceGuard g(t->device);
    RD_HIP(g.err, "rdd_forward: hipSetDevice");
    const int64_t ntiles = (n + TILE - 1) / TILE;
    int64_t blocks = (ntiles + FWAVES - 1) / FWAVES;
    if (blocks > 2 * num_cus(t->device)) blocks = 2 * num_cus(t->device);
    if (t->cfg.student_dtype == RDD_DTYPE_BF16)
        hipLaunchKernelGGL(forward_kernel<true>, dim3((unsigned)blocks), dim3(FBLOCK), 0, t->stream, t->tnet, t->snet,
                           obs, n, tflat, sflat);
    else
        hipLaunchKernelGGL(forward_kernel<false>, dim3((unsigned)blocks), dim3(FBLOCK), 0, t->stream, t->tnet,
                           t->snet, obs, n, tflat, sflat);
    RD_HIP(hipGetLastError(), "forward_kernel launch");
    return RD_OK;
}

int rdd_get_env_state(rdd_trainer* t, float* state) {
    if (!t || !state) return rd::set_error(RD_EINVAL, "rdd_get_env_state: null argument");
    rd::DeviceGuard g(t->device);
    RD_HIP(hipMemcpyAsync(state, t->state, sizeof(float) * 8 * t->cfg.n_envs, hipMemcpyDeviceToDevice, t->stream),
           "rdd_get_env_state");
    return RD_OK;
}

int rdd_set_env_state(rdd_trainer* t, const float* state) {
    if (!t || !state) return rd::set_error(RD_EINVAL, "rdd_set_env_state: null argument");
    rd::DeviceGuard g(t->device);
    // the caller's angles are checked before they replace the trainer's (ctl[14]: this check's flag)
    const int64_t n = t->cfg.n_envs;
    uint32_t bad = 0;
    RD_HIP(hipMemsetAsync(t->ctl + 14, 0, sizeof(uint32_t), t->stream), "rdd_set_env_state");
    hipLaunchKernelGGL(check_state_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, t->stream, n, state,
                       t->ctl + 14);
    RD_HIP(hipGetLastError(), "rdd_set_env_state: check_state_kernel launch");
    RD_HIP(hipMemcpyAsync(&bad, t->ctl + 14, sizeof(bad), hipMemcpyDeviceToHost, t->stream), "rdd_set_env_state");
    RD_HIP(hipStreamSynchronize(t->stream), "rdd_set_env_state");
    if (bad)
        return rd::set_error(RD_EINVAL,
                             "rdd_set_env_state: a joint angle outside the fused rollout's range (|q0| < %g, |q1| <= %g "
                             "rad, finite); the gym-API env (rd_set_state) takes any state",
                             (double)rd::kRolloutMaxQ0, (double)rd::kRolloutMaxQ1);
    RD_HIP(hipMemcpyAsync(t->state, state, sizeof(float) * 8 * n, hipMemcpyDeviceToDevice, t->stream),
           "rdd_set_env_state");
    return RD_OK;
}

static int read_ctl(rdd_trainer* t, uint32_t (&c)[16], const char* what) {
    rd::DeviceGuard g(t->device);
    RD_HIP(hipMemcpyAsync(c, t->ctl, sizeof(c), hipMemcpyDeviceToHost, t->stream), what);
    RD_HIP(hipStreamSynchronize(t->stream), what);
    if (c[8]) return rd::set_error(RD_EINVAL, "%s: a rollout's producer/consumer hand-off timed out", what);
    if (c[13]) return rd::set_error(RD_ECOMM, "%s: a gradient exchange failed; its optimiser step was skipped", what);
    return RD_OK;
}

int rdd_get_counter(rdd_trainer* t, int64_t* steps) {
    if (!t || !steps) return rd::set_error(RD_EINVAL, "rdd_get_counter: null argument");
    uint32_t c[16];
    if (int rc = read_ctl(t, c, "rdd_get_counter")) return rc;
    *steps = c[0];
    return RD_OK;
}

int rdd_get_counters(rdd_trainer* t, int64_t* env_steps, int64_t* opt_steps) {
    if (!t) return rd::set_error(RD_EINVAL, "rdd_get_counters: null handle");
    uint32_t c[16];
    if (int rc = read_ctl(t, c, "rdd_get_counters")) return rc;
    if (env_steps) *env_steps = c[0];
    if (opt_steps) *opt_steps = c[1];
    return RD_OK;
}

int rdd_read_metrics(rdd_trainer* t, int64_t count, double* out) {
    if (!t || !out || count < 0) return rd::set_error(RD_EINVAL, "rdd_read_metrics: bad argument");
    int64_t steps = 0;   // metrics are kept per optimiser step
    if (int rc = rdd_get_counters(t, nullptr, &steps)) return rc;
    const int64_t H = t->cfg.metrics_len;
    if (count > steps || count > H) return rd::set_error(RD_EINVAL, "rdd_read_metrics: only %lld steps kept",
                                                         (long long)(steps < H ? steps : H));
    float* host = new (std::nothrow) float[(size_t)H * N_MET];
    if (!host) return rd::set_error(RD_EINVAL, "rdd_read_metrics: out of host memory");
    hipError_t e = hipMemcpy(host, t->hist, sizeof(float) * H * N_MET, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        delete[] host;
        return rd::hip_fail(e, "rdd_read_metrics");
    }
    for (int64_t k = 0; k < count; ++k) {
        const int64_t s = (steps - count + k) % H;
        for (int j = 0; j < N_MET; ++j) out[k * N_MET + j] = host[s * N_MET + j];
    }
    delete[] host;
    return RD_OK;
}


#ifdef RD_STAMPS
// Diagnostic build only: copy (and zero) the per-wave stamp sums [grid*8][16] to the host.
int rdd_debug_stamps(rdd_trainer* t, unsigned long long* out, int64_t cap) {
    if (!t || !out || !t->dbg) return rd::set_error(RD_EINVAL, "rdd_debug_stamps: bad argument");
    const int64_t cnt = (int64_t)t->ws_rows * WAVES * NSTAMP;
    if (cap < cnt) return rd::set_error(RD_EINVAL, "rdd_debug_stamps: need %lld", (long long)cnt);
    RD_HIP(hipStreamSynchronize(t->stream), "rdd_debug_stamps");
    RD_HIP(hipMemcpy(out, t->dbg, sizeof(unsigned long long) * cnt, hipMemcpyDeviceToHost), "rdd_debug_stamps");
    RD_HIP(hipMemset(t->dbg, 0, sizeof(unsigned long long) * cnt), "rdd_debug_stamps");
    return (int)cnt;
}
#endif

}  // extern "C"
