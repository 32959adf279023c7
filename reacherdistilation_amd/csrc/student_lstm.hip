// The reference's LSTM student (include/reacher_student_lstm.h): forward over T unrolled
// steps of B windows and one truncated-BPTT distillation step, for gfx950.
//
// Graph (reference student_nn.py:21-49): x_t = [dropout(ob_t), dense32(prev_pdflat_t)];
// TF1 LSTMCell(200) (gates i, j, f, o; forget_bias 1); head 200-64-128-64-32-4 (tanh) -- one
// head PER UNROLLED STEP: the reference builds it with tf.layers.dense inside its Python loop
// over the T steps without reuse, so step t has its own five layers (dense_{5t+1..5t+5}),
// while the LSTMCell object (and the prev-pdflat dense) are shared.
//
// MI355X mapping.  Rows = (t, window) pairs, t-major, so every per-step slice is contiguous.
// All GEMM-shaped work runs on one MFMA GEMM (csrc/rd_gemm.h) with fused epilogues:
//  * the input half of the gate GEMM, [x_t] . Wl[0:43], is ONE GEMM over all T x B rows
//    (bias fused); only the recurrent half h_{t-1} . Wl[43:243] is per step, with the cell
//    fused into its epilogue (lstm_rec_fwd_kernel);
//  * the heads run once over all T x B rows after the recurrence (bias + tanh fused), step t's
//    rows with step t's weights;
//  * backward: each head layer's weight gradient and data gradient (tanh' of the stored
//    activation fused) run as one grouped launch (rdg::gemm2); BPTT is one launch per step,
//    dh_{t-1} = dz_t Wr^T with the cell backward of step t-1 in its epilogue; the LSTM weight
//    gradients ([x | h_prev]^T dz over all T x B rows) are one grouped launch at the end,
//    split-K with a fixed-order reduction when the output tile grid is small;
//  * bias gradients are deterministic two-level column sums; no atomics anywhere.
// Activations of all steps stay resident in HBM (sized at create for max_windows).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>

#include "../../include/reacher_student_lstm.h"
#include "rd_common.h"
#include "rd_gemm.h"
#include "rd_physics.h"

namespace {

constexpr int U = RDL_UNITS;             // 200
constexpr int G4 = 4 * U;                // 800 gates
constexpr int XI = 11 + 32;              // 43 cell inputs
constexpr int XLD = 44;                  // X row stride (16-B rows)
constexpr int H1 = 64, H2 = 128, H3 = 64, H4 = 32;
// head activations A_l are stored [row][H_l + 4] with column H_l = 1, so the next layer's
// weight-gradient GEMM over H_l + 1 rows of A^T yields [dW; db] in the flat [W | b] layout
// (tf.layers.dense order) in one launch, no column-sum pass
constexpr int L1 = H1 + 4, L2 = H2 + 4, L3 = H3 + 4, L4 = H4 + 4;

// flat parameter offsets (variable-creation order): the shared part, then the T heads; OFF_W1 ..
// OFF_B5 are offsets inside a head (head t at OFF_H + t HSZ)
constexpr int OFF_WP = 0;
constexpr int OFF_BP = OFF_WP + 4 * 32;
constexpr int OFF_WL = OFF_BP + 32;
constexpr int OFF_BL = OFF_WL + (XI + U) * G4;
constexpr int OFF_H = OFF_BL + G4;
constexpr int OFF_W1 = 0;
constexpr int OFF_B1 = OFF_W1 + U * H1;
constexpr int OFF_W2 = OFF_B1 + H1;
constexpr int OFF_B2 = OFF_W2 + H1 * H2;
constexpr int OFF_W3 = OFF_B2 + H2;
constexpr int OFF_B3 = OFF_W3 + H2 * H3;
constexpr int OFF_W4 = OFF_B3 + H3;
constexpr int OFF_B4 = OFF_W4 + H3 * H4;
constexpr int OFF_W5 = OFF_B4 + H4;
constexpr int OFF_B5 = OFF_W5 + H4 * 4;
constexpr int HSZ = OFF_B5 + 4;                 // 31,652 floats per head
static_assert(OFF_H == RDL_CELL_PARAMS && HSZ == RDL_HEAD_PARAMS && RDL_PARAMS == OFF_H + 10 * HSZ, "flat layout");
static_assert(OFF_WL % 4 == 0 && OFF_H % 4 == 0 && HSZ % 4 == 0 && OFF_W2 % 4 == 0 && OFF_W3 % 4 == 0 &&
                  OFF_W4 % 4 == 0 && OFF_W5 % 4 == 0 && (OFF_WL + XI * G4) % 4 == 0,
              "16-B aligned weight matrices");
__host__ __device__ constexpr int64_t params_of(int T) { return OFF_H + (int64_t)T * HSZ; }

constexpr int N_MET = 4;
constexpr int LOSS_BLOCK = 256;
constexpr int COLSUM_CHUNK = 512;         // rows per first-level column-sum block

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// X[r] = [dropout(ob[r]) (11) | prev[r] . Wp + bp (32) | 0]; r = t B + b
__global__ __launch_bounds__(256) void inputs_kernel(const float* ob, const float* prev, const float* params,
                                                     float* X, int64_t R, int64_t B, float keep_prob, uint64_t seed,
                                                     int64_t row_base, const uint32_t* ctl, uint32_t* bar) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx == 0) {
        bar[1] = 0u;    // the persistent BPTT's grid-barrier counter
        bar[3] += 1u;   // the persistent forward's granule generation: one per forward call
    }
    if (idx >= R * XLD) return;
    const int64_t r = idx / XLD;
    const int col = (int)(idx % XLD);
    float v = 0.0f;
    if (col < 11) {
        v = ob[r * 11 + col];
        if (keep_prob < 1.0f) {   // tf.nn.dropout (student_nn.py:24)
            const int64_t t = r / B, b = r % B;
            const uint64_t w = (uint64_t)(row_base + b);
            uint32_t o[4];
            rd::philox((uint32_t)w, (uint32_t)(w >> 32), ctl[0], (uint32_t)(4 * t + col / 4), (uint32_t)seed,
                       (uint32_t)(seed >> 32), o);
            v = rd::u01(o[col & 3]) < keep_prob ? v / keep_prob : 0.0f;
        }
    } else if (col < XI) {        // hid_prev_pdflat = dense(prev_pdflat, 32) (student_nn.py:26)
        const int c = col - 11;
        const float* p = prev + r * 4;
        v = params[OFF_BP + c];
#pragma unroll
        for (int a = 0; a < 4; ++a) v = fmaf(p[a], params[OFF_WP + a * 32 + c], v);
    }
    X[idx] = v;
}

// TF1 LSTMCell: z = [i | j | f | o]; c = sig(f + 1) c_prev + sig(i) tanh(j); h = sig(o) tanh(c)
__global__ __launch_bounds__(256) void cell_fwd_kernel(const float* Z, const float* c_prev, float* G, float* c_out,
                                                       float* h_out, int64_t B) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= B * U) return;
    const int64_t b = idx / U;
    const int u = (int)(idx % U);
    const float* z = Z + b * G4;
    const float gi = sigm(z[u]), gj = tanhf(z[U + u]), gf = sigm(z[2 * U + u] + 1.0f), go = sigm(z[3 * U + u]);
    const float c = fmaf(gf, c_prev[idx], gi * gj);
    float* g = G + b * G4;
    g[u] = gi; g[U + u] = gj; g[2 * U + u] = gf; g[3 * U + u] = go;
    c_out[idx] = c;
    h_out[idx] = go * tanhf(c);
}

// One step of the forward recurrence with the cell in the epilogue (replaces the recurrent
// GEMM accumulating into Z + cell_fwd_kernel): a workgroup owns 64 rows x 16 units, i.e. the
// 64 gate columns {i, j, f, o} x those units of Wr, so at the end of the K loop every lane
// holds all four gate pre-activations of its (row, unit) outputs.  4 waves, wave w = rows
// 16w..16w+15 x the 4 gate blocks (one A and four B operands per k-step, 4 MFMAs).  The k
// order and the epilogue's z = (acc + 0) + Zx are the unfused path's, so G, c and h are
// bitwise those of the two-launch form.  Z_s keeps the input half (the backward reuses Z).
constexpr int RF_ROWS = 64, RF_UNITS = 16, RF_TK = 16, RF_LS = 64 + 16;
__global__ __launch_bounds__(256) void lstm_rec_fwd_kernel(const float* __restrict__ Hp, const float* __restrict__ Wr,
                                                           const float* __restrict__ Zx,
                                                           const float* __restrict__ cprev, float* __restrict__ Gs,
                                                           float* __restrict__ cs, float* __restrict__ hs,
                                                           int64_t B) {
    __shared__ __attribute__((aligned(16))) float As[2][RF_TK][RF_LS];   // [k][row]
    __shared__ __attribute__((aligned(16))) float Bs[2][RF_TK][RF_LS];   // [k][16 gate + unit]
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, i = lane & 15, gq = lane >> 4;
    const int64_t m0 = (int64_t)blockIdx.y * RF_ROWS;
    const int u0 = blockIdx.x * RF_UNITS;
    // staging: thread t loads 4 consecutive k of row m0 + t/4 (A) and 4 consecutive units of
    // gate (t%16)/4 at k row t/16 (B, one 16-B load from Wr's row)
    const int64_t am = m0 + (tid >> 2);
    const int ak = 4 * (tid & 3);
    const int bk = tid >> 4, bq = tid & 15, by = bq >> 2, bu = u0 + 4 * (bq & 3);
    auto load_a = [&](int k0) { return rdg::load4<true>(Hp + am * U + k0 + ak, am < B ? min(4, U - (k0 + ak)) : 0); };
    auto load_b = [&](int k0) {
        const int k = k0 + bk;
        return rdg::load4<true>(Wr + (int64_t)k * G4 + by * U + bu, k < U ? min(4, U - bu) : 0);
    };
    auto stage = [&](int buf, rdg::f32x4 a, rdg::f32x4 b) {
#pragma unroll
        for (int e = 0; e < 4; ++e) As[buf][ak + e][tid >> 2] = a[e];
        *reinterpret_cast<rdg::f32x4*>(&Bs[buf][bk][16 * by + 4 * (bq & 3)]) = b;
    };
    rdg::f32x4 acc[4];
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[y] = rdg::f32x4{0.f, 0.f, 0.f, 0.f};
    // load pipeline of rd_gemm.h: tile t+2's loads issue right after tile t+1 is staged, so
    // they stay in flight across the barrier and the next MFMA phase
    constexpr int NT = (U + RF_TK - 1) / RF_TK;
    stage(0, load_a(0), load_b(0));
    rdg::f32x4 na = load_a(RF_TK), nb = load_b(RF_TK);
    __syncthreads();
    for (int kt = 0; kt < NT; ++kt) {
        const int buf = kt & 1;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int kk = 4 * s + gq;
            const float a = As[buf][kk][16 * wave + i];
#pragma unroll
            for (int y = 0; y < 4; ++y)
                acc[y] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Bs[buf][kk][16 * y + i], acc[y], 0, 0, 0);
        }
        if (kt + 1 < NT) {
            stage(buf ^ 1, na, nb);
            if (kt + 2 < NT) {
                na = load_a((kt + 2) * RF_TK);
                nb = load_b((kt + 2) * RF_TK);
            }
        }
        __syncthreads();
    }
    // epilogue: operands first, then TF1 LSTMCell (cell_fwd_kernel's arithmetic)
    const int u = u0 + i;
    float zx[4][4], cpv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + 16 * wave + 4 * gq + r;
        const bool ok = row < B && u < U;
#pragma unroll
        for (int y = 0; y < 4; ++y) zx[y][r] = ok ? Zx[row * G4 + y * U + u] : 0.0f;
        cpv[r] = ok ? cprev[row * U + u] : 0.0f;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + 16 * wave + 4 * gq + r;
        if (row >= B || u >= U) continue;
        const float gi = sigm((acc[0][r] + 0.0f) + zx[0][r]), gj = tanhf((acc[1][r] + 0.0f) + zx[1][r]);
        const float gf = sigm((acc[2][r] + 0.0f) + zx[2][r] + 1.0f), go = sigm((acc[3][r] + 0.0f) + zx[3][r]);
        const float c = fmaf(gf, cpv[r], gi * gj);
        float* g = Gs + row * G4;
        g[u] = gi; g[U + u] = gj; g[2 * U + u] = gf; g[3 * U + u] = go;
        cs[row * U + u] = c;
        hs[row * U + u] = go * tanhf(c);
    }
}

// ---------------------------------------------------------------- persistent recurrence
// Small batches (B <= PR_ROWS windows, e.g. the reference's 20) are launch-latency bound:
// ~10 us per recurrent step whatever the work.  lstm_fwd_persist_kernel runs ALL T steps of
// the forward recurrence in one launch and lstm_bptt_persist_kernel all T steps of BPTT.
// Workgroup w owns units 16w..16w+15 (13 workgroups): its slice of Wr stays in LDS for the
// whole launch (the forward's 64 gate columns, BPTT's 16 rows of Wr^T), its cell states c
// (forward) and dc (BPTT) stay in registers, and between steps the workgroups exchange h
// (forward) or partial dh (BPTT) through global memory (the workgroups sit on different XCDs,
// whose L2s are not coherent), with bounded spins that raise a flag instead of hanging (all 13
// workgroups are co-resident: one per CU of 256).  The forward's h travels as data-tagged
// granules, no grid barrier (round 5: 81 -> 68 us for T = 10 at 20 windows); BPTT keeps the
// write-through payload + agent-scope arrival counter form, since its granule form (52
// 8-byte granules per thread and step instead of 13 16-byte loads) measured slower (76 -> 103 us,
// profiles/r05i_*).  The forward's MFMA sequence and cell arithmetic are
// lstm_rec_fwd_kernel's, so G, c and h are bitwise those of the per-step launches.
constexpr int PR_ROWS = 32, PR_UNITS = 16, PR_K = 208, PR_GRID = (U + PR_UNITS - 1) / PR_UNITS;
constexpr int PR_WS = 80;    // forward Wr slice row stride: [k][16 gate + unit], conflict-free B reads
constexpr int PR_HS = 48;    // A operand row stride: [k][row], conflict-free A reads
constexpr int PR_ZS = 68;    // gate pre-activation exchange [row][64 + pad]
constexpr uint32_t PR_SPIN_LIMIT = 1u << 22;

// BPTT's hand-off between the workgroups of a persistent launch (cdna_hip_programming.md §6
// Guideline 16, the write-through form): the exchanged payload (h, dz) is stored with sc1 buffer stores
// and drained (s_waitcnt vmcnt(0)) before the workgroup's arrival on an agent-scope counter,
// and EVERY load of it is an sc1 buffer load -- no L2 writeback or L1 invalidate fences (a
// release/acquire pair per step measured ~3.5 us).  All other data these kernels read was
// written before the launch.
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pr_rsrc(const float* base, int64_t floats) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, (int)(floats * 4), 0x00020000);
}
__device__ __forceinline__ rdg::f32x4 pr_load4(__amdgpu_buffer_rsrc_t r, int64_t idx) {   // sc1
    return __builtin_bit_cast(rdg::f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(idx * 4), 0, 16));
}
__device__ __forceinline__ void pr_store(__amdgpu_buffer_rsrc_t r, int64_t idx, float x) {   // sc1
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), r, (int)(idx * 4), 0, 16);
}

// grid barrier #k of a launch (target = k * gridDim.x arrivals on *bar); false on timeout
__device__ __forceinline__ bool pr_grid_sync(uint32_t* bar, uint32_t target, uint32_t* err) {
    __shared__ int ok_s;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's sc1 payload stores have landed
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int ok = 1;
        for (uint32_t spins = 0; __hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target;) {
            if (++spins > PR_SPIN_LIMIT) {
                __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        ok_s = ok;
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keeps the payload loads below the poll
    return ok_s != 0;
}

// Data-tagged granules (cdna_hip_programming.md §6 Guideline 16, R2 / MI355X_MICROARCH.md
// "allgather"): each exchanged f32 travels as ONE naturally aligned 8-byte word {tag, value},
// written by one agent-scope (sc1) store and read by agent-scope loads; a consumer re-reads
// its granules until every tag is the one it waits for.  No payload drain, no arrival counter,
// no barrier poll per step: the data is the flag.  Tags = (generation << 8) | phase, the
// generation advanced on the device once per forward call (inputs_kernel, bar[3]; a replayed
// graph advances it too), so a granule left by an earlier call never matches.  Two buffers by
// step parity: a workgroup overwrites parity p only after it read every other workgroup's
// granules of the step between, which those wrote only after reading parity p themselves.
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
__device__ __forceinline__ void gr_store(unsigned long long* p, uint32_t tag, float v) {
    __hip_atomic_store((gu64_t*)(p), ((unsigned long long)tag << 32) | __float_as_uint(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long gr_load(const unsigned long long* p) {
    return __hip_atomic_load((const gu64_t*)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t gr_tag(uint32_t gen, uint32_t phase) { return (gen << 8) | phase; }

// rows [32][NB*U] of a [B][ld] matrix -> S[b*PR_K + k][row] (row stride PR_HS); every 16-B load
// of the thread is issued before its first LDS store.  ld4(row, col) loads 4 floats.
template <int NB, class L>
__device__ __forceinline__ void stage_rows(int B, float (*S)[PR_HS], L&& ld4) {
    constexpr int F4 = U / 4, PER = (NB * PR_ROWS * F4 + 255) / 256;
    rdg::f32x4 v[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int f = threadIdx.x + 256 * j, b = f / (PR_ROWS * F4), r = f - b * (PR_ROWS * F4);
        const int row = r / F4, k4 = r - row * F4;
        v[j] = (b < NB && row < B) ? ld4(row, b * U + 4 * k4) : rdg::f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int f = threadIdx.x + 256 * j, b = f / (PR_ROWS * F4), r = f - b * (PR_ROWS * F4);
        const int row = r / F4, k4 = r - row * F4;
        if (b < NB) {
#pragma unroll
            for (int e = 0; e < 4; ++e) S[b * PR_K + 4 * k4 + e][row] = v[j][e];
        }
    }
}

// bar: [2] timeout flag, [3] granule generation (inputs_kernel).  hx: h granules [2][PR_ROWS][U]
// (step parity).  state0: null (zero state) or [c | h] of [B][U] each; Cs/H rows of step 0 are
// written from it for the backward.
constexpr int GR_SWEEP = (PR_ROWS * U + 255) / 256;   // h granules per thread per step (25 at 32 rows)
__global__ __launch_bounds__(256) void lstm_fwd_persist_kernel(const float* __restrict__ Wr, const float* __restrict__ Z,
                                                               const float* __restrict__ state0, float* __restrict__ G,
                                                               float* __restrict__ Cs, float* __restrict__ H, int B,
                                                               int T, uint32_t* bar, unsigned long long* hx) {
    __shared__ __attribute__((aligned(16))) float Ws[PR_K][PR_WS];
    __shared__ __attribute__((aligned(16))) float Hs[PR_K][PR_HS];
    __shared__ __attribute__((aligned(16))) float Zl[PR_ROWS][PR_ZS];
    __shared__ int fail_s;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, i = lane & 15, gq = lane >> 4;
    const int u0 = blockIdx.x * PR_UNITS;
    const int rb = wave & 1, ch = wave >> 1;   // rows 16 rb.., gate blocks 2 ch, 2 ch + 1
    const uint32_t gen = bar[3];
    if (tid == 0) fail_s = 0;
    {   // Wr slice: rows k of 4 gate blocks x 16 units (four 16-B pieces each), loads batched
        constexpr int PER = (PR_K * 16 + 255) / 256;
        rdg::f32x4 v[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int f = tid + 256 * j, k = f >> 4, y = (f >> 2) & 3, c4 = f & 3, u = u0 + 4 * c4;
            v[j] = (k < U && u < U) ? *reinterpret_cast<const rdg::f32x4*>(Wr + (int64_t)k * G4 + y * U + u)
                                    : rdg::f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int f = tid + 256 * j, k = f >> 4, y = (f >> 2) & 3, c4 = f & 3;
            if (k < PR_K) *reinterpret_cast<rdg::f32x4*>(&Ws[k][16 * y + 4 * c4]) = v[j];
        }
    }
    for (int x = tid; x < (PR_K - U) * PR_HS; x += 256) Hs[U + x / PR_HS][x % PR_HS] = 0.0f;   // k >= U: never written
    // this thread's (row, unit) points of the cell: p = tid, tid + 256 over B x 16
    float cst[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int pt = tid + 256 * q, row = pt >> 4, u = u0 + (pt & 15);
        cst[q] = 0.0f;
        if (row < B && u < U) {
            const int64_t idx = (int64_t)row * U + u;
            const float c0 = state0 ? state0[idx] : 0.0f, h0 = state0 ? state0[(int64_t)B * U + idx] : 0.0f;
            cst[q] = c0;
            Cs[idx] = c0;   // rows of step 0, read by the backward
            H[idx] = h0;
        }
    }
    // the input half of a step's gate pre-activations (written by the Zx GEMM before this
    // launch): loaded one step ahead, before the grid barrier, so that only h crosses it
    float zx[2][4];
    auto load_zx = [&](int s) {
        const float* Zs = Z + (int64_t)s * B * G4;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int pt = tid + 256 * q, row = pt >> 4, u = u0 + (pt & 15);
            const bool ok = row < B && u < U;
#pragma unroll
            for (int y = 0; y < 4; ++y) zx[q][y] = ok ? Zs[(int64_t)row * G4 + y * U + u] : 0.0f;
        }
    };
    load_zx(0);
    for (int s = 0; s < T; ++s) {
        // A operand: h_s [B][U] -> Hs[k][row] (step 0: the initial state, read directly)
        const float* hs = s == 0 ? (state0 ? state0 + (int64_t)B * U : nullptr) : H + (int64_t)s * B * U;
        {
            if (s > 0) {   // h_s: the other workgroups' granules of step s, re-read until every tag matches
                const unsigned long long* src = hx + (int64_t)(s & 1) * PR_ROWS * U;
                const uint32_t want = gr_tag(gen, (uint32_t)s);
                const int nb = B * U;
                for (uint32_t spins = 0;;) {
                    unsigned long long v[GR_SWEEP];
#pragma unroll
                    for (int j = 0; j < GR_SWEEP; ++j) v[j] = gr_load(src + min(tid + 256 * j, nb - 1));
                    bool ok = true;
#pragma unroll
                    for (int j = 0; j < GR_SWEEP; ++j) {
                        const int idx = tid + 256 * j;
                        if (idx < nb) {
                            ok &= (uint32_t)(v[j] >> 32) == want;
                            Hs[idx % U][idx / U] = __uint_as_float((uint32_t)v[j]);
                        }
                    }
                    if (ok) break;
                    if (++spins > PR_SPIN_LIMIT) {
                        __hip_atomic_store(bar + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        fail_s = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            } else if (hs) {
                stage_rows<1>(B, Hs, [&](int row, int c) {
                    return *reinterpret_cast<const rdg::f32x4*>(hs + (int64_t)row * U + c);
                });
            } else {
                for (int x = tid; x < PR_ROWS * U; x += 256) Hs[x % U][x / U] = 0.0f;
            }
        }
        __syncthreads();
        if (fail_s) return;   // (uniform) a peer's granules never arrived: the timeout flag is raised
        // one accumulation chain per gate block and k order as lstm_rec_fwd_kernel (bitwise);
        // the two blocks' chains interleave
        rdg::f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        {
            for (int kt = 0; kt < PR_K / 16; ++kt) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int kk = 16 * kt + 4 * q + gq;
                    const float a = Hs[kk][16 * rb + i];
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Ws[kk][16 * (2 * ch) + i], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Ws[kk][16 * (2 * ch + 1) + i], acc1, 0, 0, 0);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {   // C layout: lane (i, gq) holds rows 4 gq + r, column i
            Zl[16 * rb + 4 * gq + r][16 * (2 * ch) + i] = acc0[r];
            Zl[16 * rb + 4 * gq + r][16 * (2 * ch + 1) + i] = acc1[r];
        }
        __syncthreads();
        // TF1 LSTMCell (lstm_rec_fwd_kernel's arithmetic)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int pt = tid + 256 * q, row = pt >> 4, ul = pt & 15, u = u0 + ul;
            if (row >= B || u >= U) continue;
            const float* zr = Zl[row];
            const float gi = sigm((zr[ul] + 0.0f) + zx[q][0]), gj = tanhf((zr[16 + ul] + 0.0f) + zx[q][1]);
            const float gf = sigm((zr[32 + ul] + 0.0f) + zx[q][2] + 1.0f), go = sigm((zr[48 + ul] + 0.0f) + zx[q][3]);
            const float c = fmaf(gf, cst[q], gi * gj);
            cst[q] = c;
            const int64_t row_g = (int64_t)s * B + row;
            float* g = G + row_g * G4;
            g[u] = gi; g[U + u] = gj; g[2 * U + u] = gf; g[3 * U + u] = go;
            Cs[(row_g + B) * U + u] = c;
            const float h = go * tanhf(c);
            H[(row_g + B) * U + u] = h;   // for the backward (a later launch)
            if (s + 1 < T) gr_store(hx + (int64_t)((s + 1) & 1) * PR_ROWS * U + (int64_t)row * U + u, gr_tag(gen, (uint32_t)(s + 1)), h);
        }
        if (s + 1 < T) load_zx(s + 1);
    }
}

// BPTT of all T steps, split-K over the workgroups: per step s (T-1 .. 0) workgroup w
//  (1) sums dh_next for its 16 units from the 13 partials of step s+1 (fixed order, sc1 loads),
//  (2) runs the cell backward at its (row, unit) points -> dz_s of its 64 gate columns (to dZ
//      for the weight gradients, and to LDS),
//  (3) multiplies those 64 columns by its 64 rows of Wr^T: a partial dh_{s-1} for ALL units,
//      stored sc1 to its slot of a per-step-parity partial buffer, then the grid barrier.
// So a step exchanges 13 x 2 KB per workgroup (the units' partials), not all of dz (64 KB).
constexpr int PB_N = 208;    // units, padded: 13 column blocks of 16
constexpr int PB_PART = PB_N * PR_ROWS;   // floats of one workgroup's partial [unit][row]
__global__ __launch_bounds__(256) void lstm_bptt_persist_kernel(const float* __restrict__ Wr, const float* __restrict__ dHh,
                                                                const float* __restrict__ G, const float* __restrict__ Cs,
                                                                float* __restrict__ dZ, float* __restrict__ part,
                                                                float* __restrict__ dbl, const float* __restrict__ prev,
                                                                float* __restrict__ Q, int B, int T, uint32_t* bar) {
    __shared__ __attribute__((aligned(16))) float Wb[64][PB_N];        // [local gate col y*16+c][unit]
    __shared__ __attribute__((aligned(16))) float As[64][PR_HS];       // dz_s of the local columns: [col][row]
    static_assert(PR_HS >= 40, "As also holds the 5 x 8 row-group sums at the end");
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, i = lane & 15, gq = lane >> 4;
    const int u0 = blockIdx.x * PR_UNITS;
    const int rb = wave & 1, cb0 = (wave >> 1) * 7, ncb = (wave >> 1) ? 6 : 7;   // rows 16 rb.., column blocks
    const __amdgpu_buffer_rsrc_t rP = pr_rsrc(part, (int64_t)2 * PR_GRID * PB_PART);
    {   // Wb[y*16 + c][n] = Wr[n][y*U + u0 + c]: rows n of Wr, 16 consecutive gate columns each
        constexpr int PER = (PB_N * 16 + 255) / 256;
        rdg::f32x4 v[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int f = tid + 256 * j, n = f >> 4, y = (f >> 2) & 3, c4 = f & 3, u = u0 + 4 * c4;
            v[j] = (n < U && u < U) ? *reinterpret_cast<const rdg::f32x4*>(Wr + (int64_t)n * G4 + y * U + u)
                                    : rdg::f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int f = tid + 256 * j, n = f >> 4, y = (f >> 2) & 3, c4 = f & 3;
            if (n < PB_N) {
#pragma unroll
                for (int e = 0; e < 4; ++e) Wb[16 * y + 4 * c4 + e][n] = v[j][e];
            }
        }
    }
    for (int x = tid; x < 64 * PR_HS; x += 256) As[x / PR_HS][x % PR_HS] = 0.0f;   // rows >= B stay 0
    // this thread's points: unit c = tid & 15, rows 4 r4 .. 4 r4 + 3 (threads < 128)
    const int c = tid & 15, r4 = tid >> 4, u = u0 + c;
    const bool act = tid < 128 && u < U;
    float dcs[4] = {0.f, 0.f, 0.f, 0.f};
    float bsum[4] = {0.f, 0.f, 0.f, 0.f};   // dbl: this thread's rows, all steps, per gate
    float qsum[4][4] = {};                    // Q = prev^T dz: [prev component][gate]
    float cg[4][4], cct[4], ccp[4], cdh[4], cpv[4][4];
    auto load_cell = [&](int s) {   // gates, c_t, c_{t-1}, dh from the head: written before the launch
        const int64_t rs = (int64_t)s * B;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 4 * r4 + r;
            const bool ok = act && row < B;
            const int64_t idx = (rs + row) * U + u;
            const float* g = G + (rs + row) * G4;
#pragma unroll
            for (int y = 0; y < 4; ++y) cg[r][y] = ok ? g[y * U + u] : 0.0f;
            cct[r] = ok ? Cs[idx + (int64_t)B * U] : 0.0f;
            ccp[r] = ok ? Cs[idx] : 0.0f;
            cdh[r] = ok ? dHh[idx] : 0.0f;
#pragma unroll
            for (int a = 0; a < 4; ++a) cpv[r][a] = ok ? prev[(rs + row) * 4 + a] : 0.0f;
        }
    };
    load_cell(T - 1);
    uint32_t nsync = 0;
    for (int s = T - 1; s >= 0; --s) {
        float dhn[4] = {0.f, 0.f, 0.f, 0.f};
        if (s < T - 1 && act) {   // (1) dh_next: the 13 partials of step s+1, fixed order
            const int64_t pb = (int64_t)((s + 1) & 1) * PR_GRID * PB_PART + (int64_t)u * PR_ROWS + 4 * r4;
            rdg::f32x4 v[PR_GRID];
#pragma unroll
            for (int w = 0; w < PR_GRID; ++w) v[w] = pr_load4(rP, pb + (int64_t)w * PB_PART);
            rdg::f32x4 acc = v[0];
#pragma unroll
            for (int w = 1; w < PR_GRID; ++w) acc += v[w];
#pragma unroll
            for (int r = 0; r < 4; ++r) dhn[r] = acc[r];
        }
        // (2) TF1 LSTMCell backward (cell_bwd_kernel's arithmetic)
        const int64_t rs = (int64_t)s * B;
        if (act) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 4 * r4 + r;
                if (row >= B) continue;
                const float gi = cg[r][0], gj = cg[r][1], gf = cg[r][2], go = cg[r][3];
                const float dh = s < T - 1 ? cdh[r] + dhn[r] : cdh[r];
                const float tc = tanhf(cct[r]);
                const float dcv = fmaf(dh * go, fmaf(-tc, tc, 1.0f), dcs[r]);
                const float z0 = dcv * gj * gi * (1.0f - gi), z1 = dcv * gi * fmaf(-gj, gj, 1.0f);
                const float z2 = dcv * ccp[r] * gf * (1.0f - gf), z3 = dh * tc * go * (1.0f - go);
                float* dz = dZ + (rs + row) * G4;
                dz[u] = z0; dz[U + u] = z1; dz[2 * U + u] = z2; dz[3 * U + u] = z3;
                As[c][row] = z0; As[16 + c][row] = z1; As[32 + c][row] = z2; As[48 + c][row] = z3;
                bsum[0] += z0; bsum[1] += z1; bsum[2] += z2; bsum[3] += z3;
#pragma unroll
                for (int a = 0; a < 4; ++a) {
                    qsum[a][0] = fmaf(cpv[r][a], z0, qsum[a][0]);
                    qsum[a][1] = fmaf(cpv[r][a], z1, qsum[a][1]);
                    qsum[a][2] = fmaf(cpv[r][a], z2, qsum[a][2]);
                    qsum[a][3] = fmaf(cpv[r][a], z3, qsum[a][3]);
                }
                dcs[r] = dcv * gf;
            }
        }
        if (s == 0) break;
        load_cell(s - 1);
        __syncthreads();
        // (3) partial dh_{s-1}[row][n] over the local columns, for every unit n
        rdg::f32x4 acc[7];
#pragma unroll
        for (int q = 0; q < 7; ++q) acc[q] = rdg::f32x4{0.f, 0.f, 0.f, 0.f};
        {
#pragma unroll
            for (int kq = 0; kq < 16; ++kq) {
                const int kk = 4 * kq + gq;
                const float a = As[kk][16 * rb + i];
#pragma unroll
                for (int q = 0; q < 7; ++q)
                    if (q < ncb) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Wb[kk][16 * (cb0 + q) + i], acc[q], 0, 0, 0);
            }
        }
        const int64_t po = (int64_t)(s & 1) * PR_GRID * PB_PART + (int64_t)blockIdx.x * PB_PART;
#pragma unroll
        for (int q = 0; q < 7; ++q) {   // lane (i, gq): rows 16 rb + 4 gq .. +3 of unit 16 (cb0 + q) + i
            if (q < ncb)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, acc[q]), rP,
                                                       (int)((po + (int64_t)(16 * (cb0 + q) + i) * PR_ROWS + 16 * rb + 4 * gq) * 4),
                                                       0, 16);
        }
        __syncthreads();   // As is rewritten by the next step's cell
        if (!pr_grid_sync(bar + 1, ++nsync * gridDim.x, bar + 2)) return;
    }
    // dbl (the gate bias gradient) and Q = prev^T dz of the local columns: the 8 row groups'
    // sums, in order (As[col][8 j + r4] holds sum j of row group r4)
    __syncthreads();
    if (tid < 128) {
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            As[16 * y + c][r4] = bsum[y];
#pragma unroll
            for (int a = 0; a < 4; ++a) As[16 * y + c][8 * (a + 1) + r4] = qsum[a][y];
        }
    }
    __syncthreads();
    for (int o = tid; o < 64 * 5; o += 256) {
        const int col = o & 63, j = o >> 6, y = col >> 4, uu = u0 + (col & 15);
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) v += As[col][8 * j + k];
        if (uu < U) {
            if (j == 0) dbl[y * U + uu] = v;
            else Q[(j - 1) * G4 + y * U + uu] = v;
        }
    }
}

// dWp = Q . Wl[11:43]^T and dbp = Wl[11:43] . dbl: the input-side dense32 layer's gradients
// (student_nn.py:26) from the BPTT kernel's gate sums, without materialising dP = dZ . Wl^T
// (the same sums in another order: sum over the rows first, then over the 800 gate columns)
__global__ __launch_bounds__(256) void dense32_grad_kernel(const float* __restrict__ P, const float* __restrict__ Q,
                                                           float* __restrict__ g) {
    // block o: 0..127 dWp[a][c] (a = o / 32), 128..159 dbp[c]; a fixed-order tree over 256 threads
    __shared__ float red[256];
    const int o = blockIdx.x, c = o & 31;
    const float* w = P + OFF_WL + (int64_t)(11 + c) * G4;
    const float* q = o < 128 ? Q + (o >> 5) * G4 : g + OFF_BL;
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < (G4 + 255) / 256; ++j) {
        const int k = threadIdx.x + 256 * j;
        if (k < G4) v = fmaf(w[k], q[k], v);
    }
    red[threadIdx.x] = v;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0) g[(o < 128 ? OFF_WP : OFF_BP - 128) + o] = red[0];
}

// ---------------------------------------------------------------- fused head (small batches)
// The head 200-64-128-64-32-4 (student_nn.py:42-46) over a few hundred rows is five launches of
// ~10 us each, none of them busy.  head_fwd_kernel runs all five layers for 16 rows per
// workgroup: activations stay in LDS between layers, weights stream from L2 as the B
// operands, and every layer's output is also stored (A1..A4 for the backward, Y).  Same MFMA
// k order and epilogue (acc + b, tanhf) as the unsplit rd_gemm launches it replaces.
constexpr int HF_ROWS = 16, HF_MAX_ROWS = 1 << 18;
constexpr int64_t HPART_MAX_FLOATS = (int64_t)128 << 20;   // the fused head's partial rows: at most 512 MB (reacher_student_lstm.h)
template <int K, int N, bool TANH, int LI, int LO>
__device__ __forceinline__ void head_layer(const float (*in)[LI], float (*out)[LO], const float* __restrict__ W,
                                           const float* __restrict__ b, float* __restrict__ gout, int ldg,
                                           int64_t row0, int64_t R) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, gq = lane >> 4;
    constexpr int NB = (N + 15) / 16;
#pragma unroll
    for (int it = 0; it < (NB + 3) / 4; ++it) {   // unrolled: every weight load of the layer in flight at once
        const int cb = wave + 4 * it;
        if (cb >= NB) break;
        const int col = 16 * cb + i;
        const bool cv = col < N;
        rdg::f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kq = 0; kq < K / 4; ++kq) {
            const int k = 4 * kq + gq;
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(in[i][k], cv ? W[k * N + col] : 0.0f, acc, 0, 0, 0);
        }
        const float bv = cv ? b[col] : 0.0f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 4 * gq + r;
            float v = acc[r] + bv;
            if (TANH) v = tanhf(v);
            if (cv) {
                out[row][col] = v;
                if (row0 + row < R) gout[(row0 + row) * ldg + col] = v;
            }
        }
    }
    __syncthreads();
}

// rows row0.. of a [R][ld] matrix, columns 0..COLS-1 -> dst[16][LDD] (zero past R): every
// load of the thread issued before its first LDS store (one round trip, not one per element)
template <int COLS, int LDD, int NT = 256>
__device__ __forceinline__ void head_stage(const float* __restrict__ src, int ld, int64_t row0, int64_t R,
                                           float (*dst)[LDD], int tid) {
    constexpr int PER = (HF_ROWS * COLS + NT - 1) / NT;
    float v[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int x = tid + NT * j, row = x / COLS, c = x - row * COLS;
        v[j] = (x < HF_ROWS * COLS && row0 + row < R) ? src[(row0 + row) * ld + c] : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int x = tid + NT * j, row = x / COLS, c = x - row * COLS;
        if (x < HF_ROWS * COLS) dst[row][c] = v[j];
    }
}

// workgroup (t, rb) of the grid T x nb: rows t B + 16 rb .. of step t, with step t's head
__global__ __launch_bounds__(256) void head_fwd_kernel(const float* __restrict__ Hc, const float* __restrict__ P0,
                                                       float* A1, float* A2, float* A3, float* A4, float* Y, int64_t B,
                                                       int nb) {
    __shared__ __attribute__((aligned(16))) float X0[HF_ROWS][U + 4];
    __shared__ __attribute__((aligned(16))) float X1[HF_ROWS][L1];
    __shared__ __attribute__((aligned(16))) float X2[HF_ROWS][L2];
    __shared__ __attribute__((aligned(16))) float X3[HF_ROWS][L3];
    __shared__ __attribute__((aligned(16))) float X4[HF_ROWS][L4];
    __shared__ __attribute__((aligned(16))) float X5[HF_ROWS][8];
    const int ts = blockIdx.x / nb, rb = blockIdx.x - ts * nb;
    const int64_t row0 = (int64_t)ts * B + (int64_t)rb * HF_ROWS, R = (int64_t)(ts + 1) * B;
    const float* P = P0 + OFF_H + (int64_t)ts * HSZ;   // step ts's head
    head_stage<U, U + 4>(Hc, U, row0, R, X0, threadIdx.x);
    __syncthreads();
    head_layer<U, H1, true>(X0, X1, P + OFF_W1, P + OFF_B1, A1, L1, row0, R);
    head_layer<H1, H2, true>(X1, X2, P + OFF_W2, P + OFF_B2, A2, L2, row0, R);
    head_layer<H2, H3, true>(X2, X3, P + OFF_W3, P + OFF_B3, A3, L3, row0, R);
    head_layer<H3, H4, true>(X3, X4, P + OFF_W4, P + OFF_B4, A4, L4, row0, R);
    head_layer<H4, 4, false>(X4, X5, P + OFF_W5, P + OFF_B5, Y, 4, row0, R);
}

// Head backward for the same small batches: per 16-row workgroup the data gradients down the
// head (tanh' of the stored activations fused, as the EPI_DTANH GEMMs), dh_head for BPTT,
// and the five [dW; db] weight-gradient partials over its rows (the stored activations carry
// the ones column; Hc gets one in LDS) as one partial row of the flat [W1 b1 ... W5 b5] range;
// head_wgrad_reduce_kernel sums the rows in a fixed order.  Two launches instead of six.
constexpr int HB_PART = HSZ;   // 31,652 floats: [W1;b1][W2;b2][W3;b3][W4;b4][W5;b5] of one head
// dIn[16][NI] = (dOut[16][KO] . W^T) (* (1 - act^2) when DT); W is [NI][KO] (layer input x output)
// wf(it, kq, cv, col, k): the weight W[col][k] of this lane's column block it, k step kq (zero
// past NI): streamed from L2 (head_dgrad) or held in registers (head_bwd_kernel<true>)
template <int KO, int NI, bool DT, int NW, int LD, int LI, int LA, class WF>
__device__ __forceinline__ void head_dgrad_f(const float (*dout)[LD], float (*din)[LI], const float (*act)[LA], WF wf,
                                             float* gout, int ldg, int64_t row0, int64_t R, int tid) {
    const int wave = tid >> 6, lane = tid & 63, i = lane & 15, gq = lane >> 4;
    constexpr int NB = (NI + 15) / 16;
#pragma unroll
    for (int it = 0; it < (NB + NW - 1) / NW; ++it) {   // unrolled: every weight load of the layer in flight at once
        const int cb = wave + NW * it;
        if (cb >= NB) break;
        const int col = 16 * cb + i;
        const bool cv = col < NI;
        rdg::f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kq = 0; kq < KO / 4; ++kq) {
            const int k = 4 * kq + gq;
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(dout[i][k], wf(it, kq, cv, col, k), acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 4 * gq + r;
            float v = acc[r];
            if (DT) {
                const float a = act[row][col < NI ? col : 0];
                v *= fmaf(-a, a, 1.0f);
            }
            if (cv) {
                if (din) din[row][col] = v;
                if (gout && row0 + row < R) gout[(row0 + row) * ldg + col] = v;
            }
        }
    }
}
template <int KO, int NI, bool DT, int NW = 4, int LD, int LI, int LA>
__device__ __forceinline__ void head_dgrad(const float (*dout)[LD], float (*din)[LI], const float (*act)[LA],
                                           const float* __restrict__ W, float* gout, int ldg, int64_t row0, int64_t R,
                                           int tid) {
    head_dgrad_f<KO, NI, DT, NW>(dout, din, act,
                                 [W](int, int, bool cv, int col, int k) { return cv ? W[col * KO + k] : 0.0f; }, gout,
                                 ldg, row0, R, tid);
}
// this lane's weights of head_dgrad_f's column blocks (it) and k steps (kq), loaded once
template <int KO, int NI, int NW>
struct HeadW {
    static constexpr int NB = (NI + 15) / 16, IT = (NB + NW - 1) / NW;
    float w[IT][KO / 4];
    __device__ __forceinline__ void load(const float* __restrict__ W, int tid) {
        const int wave = tid >> 6, lane = tid & 63, i = lane & 15, gq = lane >> 4;
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int cb = wave + NW * it, col = 16 * cb + i;
            const bool cv = cb < NB && col < NI;
#pragma unroll
            for (int kq = 0; kq < KO / 4; ++kq) w[it][kq] = cv ? W[col * KO + 4 * kq + gq] : 0.0f;
        }
    }
    __device__ __forceinline__ float operator()(int it, int kq, bool, int, int) const { return w[it][kq]; }
};
// part[m][n] = sum over the 16 rows of act[row][m] d[row][n], m < M (the last input row is the
// ones column: the bias gradient), n < N (one tile of rows: head_bwd_kernel<false>)
template <int M, int N, int LA, int LD>
__device__ __forceinline__ void head_wgrad(const float (*act)[LA], const float (*d)[LD], float* __restrict__ part) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, gq = lane >> 4;
    constexpr int MB = (M + 15) / 16, NB = (N + 15) / 16;
    for (int t = wave; t < MB * NB; t += 4) {
        const int m0 = 16 * (t / NB), n0 = 16 * (t % NB);
        const int mc = m0 + i < M ? m0 + i : M - 1, nc = n0 + i < N ? n0 + i : N - 1;
        rdg::f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int k = 4 * s + gq;
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(act[k][mc], d[k][nc], acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + 4 * gq + r, n = n0 + i;
            if (m < M && n < N) part[m * N + n] = acc[r];
        }
    }
}
// acc += sum over the 16 rows of act[row][m] d[row][n], m < M (the last input row is the ones
// column: the bias gradient), n < N: 16x16 output tiles t = wave, wave + 4, ...; the
// accumulators stay in registers over a workgroup's tiles of rows (head_bwd_kernel)
template <int M, int N, int NW = 4>
constexpr int wq() { return (((M + 15) / 16) * ((N + 15) / 16) + NW - 1) / NW; }
template <int M, int N, int NW = 4, int LA, int LD>
__device__ __forceinline__ void head_wgrad_acc(const float (*act)[LA], const float (*d)[LD],
                                               rdg::f32x4 (&acc)[wq<M, N, NW>()], int tid) {
    const int wave = tid >> 6, lane = tid & 63, i = lane & 15, gq = lane >> 4;
    constexpr int MB = (M + 15) / 16, NB = (N + 15) / 16;
#pragma unroll
    for (int q = 0; q < wq<M, N, NW>(); ++q) {
        const int t = wave + NW * q;
        if (t >= MB * NB) break;
        const int m0 = 16 * (t / NB), n0 = 16 * (t % NB);
        const int mc = m0 + i < M ? m0 + i : M - 1, nc = n0 + i < N ? n0 + i : N - 1;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int k = 4 * s + gq;
            acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(act[k][mc], d[k][nc], acc[q], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);   // one tile's LDS operands live at a time
    }
}
// part[m][n] = the accumulated tiles
template <int M, int N, int NW = 4>
__device__ __forceinline__ void head_wgrad_store(const rdg::f32x4 (&acc)[wq<M, N, NW>()], float* __restrict__ part) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, gq = lane >> 4;
    constexpr int MB = (M + 15) / 16, NB = (N + 15) / 16;
#pragma unroll
    for (int q = 0; q < wq<M, N, NW>(); ++q) {
        const int t = wave + NW * q;
        if (t >= MB * NB) break;
        const int m0 = 16 * (t / NB), n0 = 16 * (t % NB);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + 4 * gq + r, n = n0 + i;
            if (m < M && n < N) part[m * N + n] = acc[q][r];
        }
    }
}

// MT: tpb tiles per workgroup with the weight-gradient accumulators in registers over all of them
// (eight waves share them), for large batches; else one tile, four waves, 64 VGPRs
template <bool MT>
__global__ __launch_bounds__(MT ? 512 : 256) void head_bwd_kernel(const float* __restrict__ Hc, const float* __restrict__ P0,
                                                       const float* __restrict__ A1, const float* __restrict__ A2,
                                                       const float* __restrict__ A3, const float* __restrict__ A4,
                                                       const float* __restrict__ dY, float* __restrict__ dHh,
                                                       float* __restrict__ part, int64_t B, int nb, int tpb) {
    __shared__ __attribute__((aligned(16))) float X0[HF_ROWS][U + 4];   // Hc, ones column U
    __shared__ __attribute__((aligned(16))) float X1[HF_ROWS][L1];
    __shared__ __attribute__((aligned(16))) float X2[HF_ROWS][L2];
    __shared__ __attribute__((aligned(16))) float X3[HF_ROWS][L3];
    __shared__ __attribute__((aligned(16))) float X4[HF_ROWS][L4];
    __shared__ __attribute__((aligned(16))) float D5[HF_ROWS][8];
    __shared__ __attribute__((aligned(16))) float D4[HF_ROWS][L4];
    __shared__ __attribute__((aligned(16))) float D3[HF_ROWS][L3];
    __shared__ __attribute__((aligned(16))) float D2[HF_ROWS][L2];
    __shared__ __attribute__((aligned(16))) float D1[HF_ROWS][L1];
    // workgroup (t, rb): rows t B + 16 tpb rb .. of step t, tpb tiles of 16 rows in turn; the
    // weight-gradient accumulators run over all of them and leave one partial row
    const int ts = blockIdx.x / nb, rb = blockIdx.x - ts * nb;
    const int64_t R = (int64_t)(ts + 1) * B;
    const float* P = P0 + OFF_H + (int64_t)ts * HSZ;
    float* pw = part + (int64_t)blockIdx.x * HB_PART;
    constexpr int NW = MT ? 8 : 4, NT = 64 * NW;   // MT: eight waves share the accumulators
    rdg::f32x4 a1[wq<U + 1, H1, NW>()], a2[wq<H1 + 1, H2, NW>()], a3[wq<H2 + 1, H3, NW>()],
        a4[wq<H3 + 1, H4, NW>()], a5[wq<H4 + 1, 4, NW>()];
#define RDL_ZERO(a) _Pragma("unroll") for (auto& x : a) x = rdg::f32x4{0.f, 0.f, 0.f, 0.f};
    RDL_ZERO(a1) RDL_ZERO(a2) RDL_ZERO(a3) RDL_ZERO(a4) RDL_ZERO(a5)
#undef RDL_ZERO
    // MT: this lane's share of step ts's head weights held in registers over all the tiles
    HeadW<4, H4, NW> w5;
    HeadW<H4, H3, NW> w4;
    HeadW<H3, H2, NW> w3;
    HeadW<H2, H1, NW> w2;
    HeadW<H1, U, NW> w1;
    if constexpr (MT) {
        w5.load(P + OFF_W5, threadIdx.x);
        w4.load(P + OFF_W4, threadIdx.x);
        w3.load(P + OFF_W3, threadIdx.x);
        w2.load(P + OFF_W2, threadIdx.x);
        w1.load(P + OFF_W1, threadIdx.x);
    }
    for (int k = 0; k < (MT ? tpb : 1); ++k) {
        const int64_t row0 = (int64_t)ts * B + ((int64_t)rb * tpb + k) * HF_ROWS;
        if (row0 >= R) break;   // workgroup-uniform
        // loop-invariant weights and lane indices: opaque copies keep their loads and address
        // arithmetic inside the loop (hoisted, every layer's operands and addresses would be live
        // at once and spill)
        const float* Pk = P;
        int tid = threadIdx.x;
        asm volatile("" : "+s"(Pk), "+v"(tid));
        // rows past R (the step's last row) are zero (activations and gradients): they add nothing
        head_stage<U, U + 4, NT>(Hc, U, row0, R, X0, tid);
        head_stage<H1 + 1, L1, NT>(A1, L1, row0, R, X1, tid);   // with the ones column
        head_stage<H2 + 1, L2, NT>(A2, L2, row0, R, X2, tid);
        head_stage<H3 + 1, L3, NT>(A3, L3, row0, R, X3, tid);
        head_stage<H4 + 1, L4, NT>(A4, L4, row0, R, X4, tid);
        head_stage<4, 8, NT>(dY, 4, row0, R, D5, tid);
        if (tid < HF_ROWS) X0[tid][U] = row0 + tid < R ? 1.0f : 0.0f;
        __syncthreads();
        if constexpr (MT) {
            head_dgrad_f<4, H4, true, NW>(D5, D4, X4, w5, nullptr, 0, row0, R, tid);
            __syncthreads();
            head_dgrad_f<H4, H3, true, NW>(D4, D3, X3, w4, nullptr, 0, row0, R, tid);
            __syncthreads();
            head_dgrad_f<H3, H2, true, NW>(D3, D2, X2, w3, nullptr, 0, row0, R, tid);
            __syncthreads();
            head_dgrad_f<H2, H1, true, NW>(D2, D1, X1, w2, nullptr, 0, row0, R, tid);
            __syncthreads();
            head_dgrad_f<H1, U, false, NW>(D1, (float(*)[U + 4]) nullptr, X0, w1, dHh, U, row0, R, tid);   // dh_head
        } else {
            head_dgrad<4, H4, true, NW>(D5, D4, X4, Pk + OFF_W5, nullptr, 0, row0, R, tid);
            __syncthreads();
            head_dgrad<H4, H3, true, NW>(D4, D3, X3, Pk + OFF_W4, nullptr, 0, row0, R, tid);
            __syncthreads();
            head_dgrad<H3, H2, true, NW>(D3, D2, X2, Pk + OFF_W3, nullptr, 0, row0, R, tid);
            __syncthreads();
            head_dgrad<H2, H1, true, NW>(D2, D1, X1, Pk + OFF_W2, nullptr, 0, row0, R, tid);
            __syncthreads();
            head_dgrad<H1, U, false, NW>(D1, (float(*)[U + 4]) nullptr, X0, Pk + OFF_W1, dHh, U, row0, R, tid);
        }
        if constexpr (MT) {   // [dW1; db1] .. [dW5; db5] accumulated over the tiles
            head_wgrad_acc<U + 1, H1, NW>(X0, D1, a1, tid);
            head_wgrad_acc<H1 + 1, H2, NW>(X1, D2, a2, tid);
            head_wgrad_acc<H2 + 1, H3, NW>(X2, D3, a3, tid);
            head_wgrad_acc<H3 + 1, H4, NW>(X3, D4, a4, tid);
            head_wgrad_acc<H4 + 1, 4, NW>(X4, D5, a5, tid);
            __syncthreads();   // the next tile restages the LDS rows
        } else {              // one tile: each layer's partial stored at once
            head_wgrad<U + 1, H1>(X0, D1, pw);
            head_wgrad<H1 + 1, H2>(X1, D2, pw + (OFF_W2 - OFF_W1));
            head_wgrad<H2 + 1, H3>(X2, D3, pw + (OFF_W3 - OFF_W1));
            head_wgrad<H3 + 1, H4>(X3, D4, pw + (OFF_W4 - OFF_W1));
            head_wgrad<H4 + 1, 4>(X4, D5, pw + (OFF_W5 - OFF_W1));
        }
    }
    if constexpr (MT) {
        head_wgrad_store<U + 1, H1, NW>(a1, pw);
        head_wgrad_store<H1 + 1, H2, NW>(a2, pw + (OFF_W2 - OFF_W1));
        head_wgrad_store<H2 + 1, H3, NW>(a3, pw + (OFF_W3 - OFF_W1));
        head_wgrad_store<H3 + 1, H4, NW>(a4, pw + (OFF_W4 - OFF_W1));
        head_wgrad_store<H4 + 1, 4, NW>(a5, pw + (OFF_W5 - OFF_W1));
    }
}

// head t's gradient (blockIdx.y = t): grad[OFF_H + t HSZ + p] = sum over step t's nb
// workgroups' partial rows, in row order
__global__ __launch_bounds__(256) void head_wgrad_reduce_kernel(const float* __restrict__ part, int nb,
                                                                float* __restrict__ g) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= HB_PART) return;
    const float* q = part + (int64_t)blockIdx.y * nb * HB_PART + p;
    float a = 0.f, b = 0.f;
    int w = 0;
    for (; w + 1 < nb; w += 2) {
        a += q[(int64_t)w * HB_PART];
        b += q[(int64_t)(w + 1) * HB_PART];
    }
    if (w < nb) a += q[(int64_t)w * HB_PART];
    g[OFF_H + (int64_t)blockIdx.y * HSZ + p] = a + b;
}

// BPTT through one cell (dh = dh_head + dh_next; dc carried in place).  The fused backward
// runs this only for the last step; the others ride in the dh GEMM's epilogue
// (rdg::EPI_LSTM_BWD, the same arithmetic)
__global__ __launch_bounds__(256) void cell_bwd_kernel(const float* dh_head, const float* dh_next, int add_next,
                                                       const float* G, const float* c_t, const float* c_prev,
                                                       float* dc, float* dZ, int64_t B) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= B * U) return;
    const int64_t b = idx / U;
    const int u = (int)(idx % U);
    const float* g = G + b * G4;
    const float gi = g[u], gj = g[U + u], gf = g[2 * U + u], go = g[3 * U + u];
    const float dh = add_next ? dh_head[idx] + dh_next[idx] : dh_head[idx];
    const float tc = tanhf(c_t[idx]);
    const float dcv = fmaf(dh * go, fmaf(-tc, tc, 1.0f), dc[idx]);
    float* dz = dZ + b * G4;
    dz[u] = dcv * gj * gi * (1.0f - gi);
    dz[U + u] = dcv * gi * fmaf(-gj, gj, 1.0f);
    dz[2 * U + u] = dcv * c_prev[idx] * gf * (1.0f - gf);
    dz[3 * U + u] = dh * tc * go * (1.0f - go);
    dc[idx] = dcv * gf;
}

// loss (reference loss.py:3-13 / action-MSE) and dY; per-block partials (fixed-order tree)
__global__ __launch_bounds__(LOSS_BLOCK) void loss_kernel(const float* Y, const float* tgt, float* dY, int64_t R,
                                                          int loss, float inv_n, float* part, uint32_t* ctl, float* hist,
                                                          int hist_len) {
    __shared__ float sl[LOSS_BLOCK], ss[LOSS_BLOCK];
    const int64_t r = (int64_t)blockIdx.x * LOSS_BLOCK + threadIdx.x;
    float lv = 0.f, sq = 0.f;
    if (r < R) {
        const float* o = Y + r * 4;
        const float* t = tgt + r * 4;
        const float e0 = o[0] - t[0], e1 = o[1] - t[1];
        sq = fmaf(e0, e0, e1 * e1);
        float d0, d1, d2 = 0.f, d3 = 0.f;
        if (loss == RDL_LOSS_MSE) {
            d0 = e0 * inv_n;
            d1 = e1 * inv_n;
            lv = 0.5f * inv_n * sq;
        } else {
            const float ivt0 = expf(-2.0f * t[2]), ivt1 = expf(-2.0f * t[3]);
            const float vs0 = expf(2.0f * o[2]), vs1 = expf(2.0f * o[3]);
            lv = ((t[2] - o[2]) + 0.5f * (vs0 + e0 * e0) * ivt0 - 0.5f) +
                 ((t[3] - o[3]) + 0.5f * (vs1 + e1 * e1) * ivt1 - 0.5f);
            d0 = e0 * ivt0;
            d1 = e1 * ivt1;
            d2 = fmaf(vs0, ivt0, -1.0f);
            d3 = fmaf(vs1, ivt1, -1.0f);
        }
        float* d = dY + r * 4;
        d[0] = d0; d[1] = d1; d[2] = d2; d[3] = d3;
    }
    sl[threadIdx.x] = lv;
    ss[threadIdx.x] = sq;
    __syncthreads();
    for (int s = LOSS_BLOCK / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            sl[threadIdx.x] += sl[threadIdx.x + s];
            ss[threadIdx.x] += ss[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = sl[0];
        part[2 * blockIdx.x + 1] = ss[0];
    }
    if (gridDim.x == 1 && hist) {   // one block: metrics_kernel's work here (one launch fewer)
        if (threadIdx.x == 0) {
            float* h = hist + (int64_t)(ctl[0] % (uint32_t)hist_len) * N_MET;
            h[0] = sl[0];
            h[1] = ss[0];
            h[2] = (float)R;
            h[3] = 0.f;
        }
        __syncthreads();   // ctl[0] is read before the snapshot below rewrites nothing it needs
        if (threadIdx.x < 4) ctl[4 + threadIdx.x] = ctl[threadIdx.x];
    }
}

// metrics of this rollout into the ring slot of the current optimiser step; snapshot of the
// step words for the Adam kernel (whose block 0 rewrites them)
__global__ void metrics_kernel(const float* part, int nblk, float rows, uint32_t* ctl, float* hist, int hist_len) {
    __shared__ float sl[256], ss[256];
    float a = 0.f, b = 0.f;
    for (int k = threadIdx.x; k < nblk; k += 256) {
        a += part[2 * k];
        b += part[2 * k + 1];
    }
    sl[threadIdx.x] = a;
    ss[threadIdx.x] = b;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            sl[threadIdx.x] += sl[threadIdx.x + s];
            ss[threadIdx.x] += ss[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        float* h = hist + (int64_t)(ctl[0] % (uint32_t)hist_len) * N_MET;
        h[0] = sl[0];
        h[1] = ss[0];
        h[2] = rows;
        h[3] = 0.f;
    }
    if (threadIdx.x < 4) ctl[4 + threadIdx.x] = ctl[threadIdx.x];
}

// deterministic column sums: out[c] (+ blockIdx.y * ld_out) = sum over rows [y*chunk, ...)
// column `col` of a [rows][ld] buffer = 1
__global__ __launch_bounds__(256) void ones_column_kernel(float* A, int64_t rows, int ld, int col) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r < rows) A[r * ld + col] = 1.0f;
}

__global__ __launch_bounds__(256) void colsum_kernel(const float* src, int64_t M, int N, int64_t ld, int64_t chunk,
                                                     float* out, int64_t ld_out) {
    __shared__ float s[4][64];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63), ph = threadIdx.x >> 6;
    const int64_t r0 = (int64_t)blockIdx.y * chunk, r1 = min(M, r0 + chunk);
    float a = 0.f, b = 0.f;
    if (c < N) {
        int64_t r = r0 + ph;
        for (; r + 4 < r1; r += 8) {   // two chains: loads of 2 rows in flight per step
            a += src[r * ld + c];
            b += src[(r + 4) * ld + c];
        }
        if (r < r1) a += src[r * ld + c];
    }
    s[ph][threadIdx.x & 63] = a + b;
    __syncthreads();
    if (ph == 0 && c < N) out[(int64_t)blockIdx.y * ld_out + c] = (s[0][threadIdx.x] + s[1][threadIdx.x]) +
                                                                 (s[2][threadIdx.x] + s[3][threadIdx.x]);
}

struct AdamArgs {
    const float* grad;
    float* params;
    float* m;
    float* v;
    uint32_t* ctl;
    float lr, b1, b2, eps;
    int64_t n;   // parameters (params_of(T))
};

__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    const uint32_t S = a.ctl[4];
    const float b1p = __uint_as_float(a.ctl[5]), b2p = __uint_as_float(a.ctl[6]);
    if (p < a.n) {   // TF1 ApplyAdam (lstm_train.py:73-79)
        const float g = a.grad[p];
        const float alpha = a.lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
        float m = a.m[p], v = a.v[p];
        m += (g - m) * (1.0f - a.b1);
        v += (g * g - v) * (1.0f - a.b2);
        a.m[p] = m;
        a.v[p] = v;
        a.params[p] -= (m * alpha) / (sqrtf(v) + a.eps);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.ctl[0] = S + 1u;
        a.ctl[1] = __float_as_uint(b1p * a.b1);
        a.ctl[2] = __float_as_uint(b2p * a.b2);
    }
}

__global__ void init_ctl_kernel(uint32_t* ctl, float b1, float b2) {
    if (threadIdx.x < 2) {
        const int o = 4 * threadIdx.x;
        ctl[o] = 0u; ctl[o + 1] = __float_as_uint(b1); ctl[o + 2] = __float_as_uint(b2); ctl[o + 3] = 0u;
    }
}

int cu_count(int device) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 256;
    return prop.multiProcessorCount;
}

constexpr int64_t SPLIT_FLOATS = 16 << 20;  // split-K partials (64 MB)

}  // namespace

struct rdl_trainer {
    rdl_config cfg{};
    int device = 0, cus = 256;
    hipStream_t stream = nullptr;
    int T = 0;
    int64_t np = 0;   // flat parameters: the shared cell part + T heads (params_of(T))
    int64_t Bmax = 0;
    float *params = nullptr, *m = nullptr, *v = nullptr, *grad = nullptr, *own_grad = nullptr;
    float *X = nullptr, *H = nullptr, *Cs = nullptr, *Z = nullptr, *G = nullptr;
    float *A1 = nullptr, *A2 = nullptr, *A3 = nullptr, *A4 = nullptr, *Y = nullptr, *dY = nullptr;
    float *D32 = nullptr, *D64a = nullptr, *D128 = nullptr, *D64b = nullptr, *dHh = nullptr, *dP = nullptr;
    float *dhn = nullptr, *dc = nullptr;
    float *split = nullptr, *colws = nullptr, *lpart = nullptr, *hist = nullptr;
    float* hpart = nullptr;    // fused head backward: one partial row of HB_PART per workgroup (head_nb)
    int64_t colws_floats = 0;
    uint32_t* ctl = nullptr;
    uint32_t* bar = nullptr;   // persistent kernels: [0] forward / [1] BPTT barrier arrivals, [2] timeout flag
    float* bpart = nullptr;                // persistent BPTT: per-step-parity partial dh of every workgroup
    unsigned long long* hx = nullptr;      // persistent forward: per-step-parity h granules
    float* qbuf = nullptr;     // persistent BPTT: Q = prev^T dz [4][800]
    int64_t last_B = 0;   // windows of the last forward pass (rdl_final_state)
};

namespace {

hipError_t mm(rdl_trainer* t, int M, int N, int K, const float* A, int64_t lda, int ta, const float* B, int64_t ldb,
              int tb, float* C, int64_t ldc, const float* bias = nullptr, int epi = rdg::EPI_NONE,
              const float* aux = nullptr, int64_t ldaux = 0, int accum = 0) {
    rdg::GemmArgs g{};
    g.M = M; g.N = N; g.K = K;
    g.A = A; g.lda = lda; g.ta = ta;
    g.B = B; g.ldb = ldb; g.tb = tb;
    g.C = C; g.ldc = ldc;
    g.bias = bias; g.epi = epi; g.aux = aux; g.ldaux = ldaux; g.accum = accum;
    return rdg::gemm(t->stream, g, t->split, SPLIT_FLOATS, t->cus);
}

rdg::GemmArgs ga(int M, int N, int K, const float* A, int64_t lda, int ta, const float* B, int64_t ldb, int tb,
                 float* C, int64_t ldc, int epi = rdg::EPI_NONE, const float* aux = nullptr, int64_t ldaux = 0) {
    rdg::GemmArgs g{};
    g.M = M; g.N = N; g.K = K;
    g.A = A; g.lda = lda; g.ta = ta;
    g.B = B; g.ldb = ldb; g.tb = tb;
    g.C = C; g.ldc = ldc;
    g.epi = epi; g.aux = aux; g.ldaux = ldaux;
    return g;
}

// two independent GEMMs as one grouped launch (rdg::gemm2): a head layer's weight gradient
// beside its data gradient, the two halves of the LSTM weight gradient
hipError_t mm2(rdl_trainer* t, const rdg::GemmArgs& g0, const rdg::GemmArgs& g1) {
    return rdg::gemm2(t->stream, g0, g1, t->split, SPLIT_FLOATS, t->cus);
}

hipError_t colsum(rdl_trainer* t, const float* src, int64_t M, int N, int64_t ld, float* out) {
    const unsigned gx = (unsigned)((N + 63) / 64);
    if (M <= COLSUM_CHUNK) {
        hipLaunchKernelGGL(colsum_kernel, dim3(gx, 1), dim3(256), 0, t->stream, src, M, N, ld, (int64_t)COLSUM_CHUNK,
                           out, (int64_t)0);
        return hipGetLastError();
    }
    const int64_t nch = (M + COLSUM_CHUNK - 1) / COLSUM_CHUNK;
    hipLaunchKernelGGL(colsum_kernel, dim3(gx, (unsigned)nch), dim3(256), 0, t->stream, src, M, N, ld,
                       (int64_t)COLSUM_CHUNK, t->colws, (int64_t)N);
    hipLaunchKernelGGL(colsum_kernel, dim3(gx, 1), dim3(256), 0, t->stream, (const float*)t->colws, nch, N,
                       (int64_t)N, nch, out, (int64_t)0);
    return hipGetLastError();
}

#define RDL_CK(call, what) RD_HIP((call), what)

// the persistent recurrence kernels for batches of at most PR_ROWS windows, and the
// one-launch head for at most HF_MAX_ROWS rows; rdl_config.kernels can select the per-step /
// per-layer launches instead (RDL_KERNELS_*: tests compare the two paths)

// head_bwd_kernel's 16-row tiles per workgroup: one while the T x ceil(B / 16) tiles fill at
// most ~4 workgroups per CU, then up to 8, so the partial rows (HB_PART floats each) and their
// reduce shrink with the batch
int head_tpb(int T, int64_t B) {
    const int64_t tiles = (B + HF_ROWS - 1) / HF_ROWS;
    return (int)std::max<int64_t>(1, std::min<int64_t>(8, (int64_t)T * tiles / 1024));
}
int head_nb(int T, int64_t B) {
    const int64_t tiles = (B + HF_ROWS - 1) / HF_ROWS, tpb = head_tpb(T, B);
    return (int)((tiles + tpb - 1) / tpb);
}

bool fused_head(const rdl_trainer* t, int64_t R) {
    // the partial rows of its T x head_nb workgroups live in hpart (sized at create for
    // max_windows when that fits HPART_MAX_FLOATS); with one head per step, the per-layer path
    // is T x 11 launches, so the fused head now covers up to 16,384 rows
    return !(t->cfg.kernels & RDL_KERNELS_LAYER_HEAD) && t->hpart && R <= HF_MAX_ROWS;
}

bool persistent(const rdl_trainer* t, int64_t B) {
    return !(t->cfg.kernels & RDL_KERNELS_STEP_RECURRENCE) && B <= PR_ROWS;
}

// forward over all T steps of B windows.  out_pdflat: where the head's output goes (the
// internal Y when training).
int run_forward(rdl_trainer* t, const float* ob, const float* prev, const float* state0, int64_t B, float* out_pdflat,
                bool train) {
    const int T = t->T;
    const int64_t R = (int64_t)T * B;
    const float* P = t->params;
    t->last_B = B;
    hipLaunchKernelGGL(inputs_kernel, dim3((unsigned)((R * XLD + 255) / 256)), dim3(256), 0, t->stream, ob, prev, P,
                       t->X, R, B, train ? t->cfg.keep_prob : 1.0f, t->cfg.seed, t->cfg.row_base,
                       (const uint32_t*)t->ctl, t->bar);
    RDL_CK(hipGetLastError(), "rdl inputs_kernel");
    if (persistent(t, B)) {   // Zx, then all T recurrent steps in one launch (it writes the step-0 state rows)
        RDL_CK(mm(t, (int)R, G4, XI, t->X, XLD, 0, P + OFF_WL, G4, 0, t->Z, G4, P + OFF_BL), "rdl gemm Zx");
        hipLaunchKernelGGL(lstm_fwd_persist_kernel, dim3(PR_GRID), dim3(256), 0, t->stream, P + OFF_WL + XI * G4,
                           (const float*)t->Z, state0, t->G, t->Cs, t->H, (int)B, T, t->bar, t->hx);
        RDL_CK(hipGetLastError(), "rdl lstm_fwd_persist_kernel");
    } else {
    if (state0) {
        RDL_CK(hipMemcpyAsync(t->Cs, state0, sizeof(float) * B * U, hipMemcpyDeviceToDevice, t->stream), "rdl state");
        RDL_CK(hipMemcpyAsync(t->H, state0 + B * U, sizeof(float) * B * U, hipMemcpyDeviceToDevice, t->stream),
               "rdl state");
    } else {
        RDL_CK(hipMemsetAsync(t->Cs, 0, sizeof(float) * B * U, t->stream), "rdl state");
        RDL_CK(hipMemsetAsync(t->H, 0, sizeof(float) * B * U, t->stream), "rdl state");
    }
    // input half of the gate pre-activations for all steps: Z = X[:, :43] Wl[0:43] + bl
    RDL_CK(mm(t, (int)R, G4, XI, t->X, XLD, 0, P + OFF_WL, G4, 0, t->Z, G4, P + OFF_BL), "rdl gemm Zx");
    for (int s = 0; s < T; ++s) {
        float* Zs = t->Z + (int64_t)s * B * G4;
        hipLaunchKernelGGL(lstm_rec_fwd_kernel, dim3((U + RF_UNITS - 1) / RF_UNITS, (unsigned)((B + RF_ROWS - 1) / RF_ROWS)),
                           dim3(256), 0, t->stream, (const float*)(t->H + (int64_t)s * B * U), P + OFF_WL + XI * G4,
                           (const float*)Zs, (const float*)(t->Cs + (int64_t)s * B * U), t->G + (int64_t)s * B * G4,
                           t->Cs + (int64_t)(s + 1) * B * U, t->H + (int64_t)(s + 1) * B * U, B);
        RDL_CK(hipGetLastError(), "rdl lstm_rec_fwd_kernel");
    }
    }
    // step t's head over its B rows (student_nn.py:42-46, one head per unrolled step)
    const float* Hc = t->H + B * U;
    if (fused_head(t, R)) {
        const int nb = (int)((B + HF_ROWS - 1) / HF_ROWS);
        hipLaunchKernelGGL(head_fwd_kernel, dim3((unsigned)(T * nb)), dim3(256), 0, t->stream, Hc, P, t->A1, t->A2,
                           t->A3, t->A4, out_pdflat, B, nb);
        RDL_CK(hipGetLastError(), "rdl head_fwd_kernel");
        return RD_OK;
    }
    for (int s = 0; s < T; ++s) {
        const float* Ph = P + OFF_H + (int64_t)s * HSZ;
        const int64_t r0 = (int64_t)s * B;
        const int Bi = (int)B;
        RDL_CK(mm(t, Bi, H1, U, Hc + r0 * U, U, 0, Ph + OFF_W1, H1, 0, t->A1 + r0 * L1, L1, Ph + OFF_B1, rdg::EPI_TANH),
               "rdl head1");
        RDL_CK(mm(t, Bi, H2, H1, t->A1 + r0 * L1, L1, 0, Ph + OFF_W2, H2, 0, t->A2 + r0 * L2, L2, Ph + OFF_B2,
                  rdg::EPI_TANH), "rdl head2");
        RDL_CK(mm(t, Bi, H3, H2, t->A2 + r0 * L2, L2, 0, Ph + OFF_W3, H3, 0, t->A3 + r0 * L3, L3, Ph + OFF_B3,
                  rdg::EPI_TANH), "rdl head3");
        RDL_CK(mm(t, Bi, H4, H3, t->A3 + r0 * L3, L3, 0, Ph + OFF_W4, H4, 0, t->A4 + r0 * L4, L4, Ph + OFF_B4,
                  rdg::EPI_TANH), "rdl head4");
        RDL_CK(mm(t, Bi, 4, H4, t->A4 + r0 * L4, L4, 0, Ph + OFF_W5, 4, 0, out_pdflat + r0 * 4, 4, Ph + OFF_B5),
               "rdl head5");
    }
    return RD_OK;
}

int run_backward(rdl_trainer* t, const float* prev, const float* tgt, int64_t B, int64_t B_global) {
    const int T = t->T;
    const int64_t R = (int64_t)T * B;
    const int Ri = (int)R;
    const float* P = t->params;
    float* g = t->grad;
    const int lblk = (int)((R + LOSS_BLOCK - 1) / LOSS_BLOCK);
    const bool fold = lblk == 1;   // a single loss block writes the metrics itself
    hipLaunchKernelGGL(loss_kernel, dim3(lblk), dim3(LOSS_BLOCK), 0, t->stream, (const float*)t->Y, tgt, t->dY, R,
                       t->cfg.loss, 1.0f / ((float)T * (float)B_global), t->lpart, t->ctl, fold ? t->hist : nullptr,
                       t->cfg.metrics_len);
    RDL_CK(hipGetLastError(), "rdl loss_kernel");
    if (!fold) {
        hipLaunchKernelGGL(metrics_kernel, dim3(1), dim3(256), 0, t->stream, (const float*)t->lpart, lblk, (float)R,
                           t->ctl, t->hist, t->cfg.metrics_len);
        RDL_CK(hipGetLastError(), "rdl metrics_kernel");
    }
    const float* Hc = t->H + B * U;
    if (fused_head(t, R)) {   // the heads' backward as two launches (head_bwd_kernel + fixed-order reduce)
        const int nb = head_nb(T, B), tpb = head_tpb(T, B);
        hipLaunchKernelGGL(tpb > 1 ? head_bwd_kernel<true> : head_bwd_kernel<false>, dim3((unsigned)(T * nb)),
                           dim3(tpb > 1 ? 512 : 256), 0, t->stream, Hc, P,
                           (const float*)t->A1, (const float*)t->A2, (const float*)t->A3, (const float*)t->A4,
                           (const float*)t->dY, t->dHh, t->hpart, B, nb, tpb);
        RDL_CK(hipGetLastError(), "rdl head_bwd_kernel");
        hipLaunchKernelGGL(head_wgrad_reduce_kernel, dim3((HB_PART + 255) / 256, (unsigned)T), dim3(256), 0, t->stream,
                           (const float*)t->hpart, nb, g);
        RDL_CK(hipGetLastError(), "rdl head_wgrad_reduce_kernel");
    } else {
    // step s's head backward over its B rows (weight gradients; data gradients with the tanh
    // derivative fused): per layer, [dW; db] (weight gradient, ones column) beside the data
    // gradient with tanh'
    for (int s = 0; s < T; ++s) {
        const float* Ph = P + OFF_H + (int64_t)s * HSZ;
        float* gh = g + OFF_H + (int64_t)s * HSZ;
        const int64_t r0 = (int64_t)s * B;
        const int Bi = (int)B;
        const float *a1 = t->A1 + r0 * L1, *a2 = t->A2 + r0 * L2, *a3 = t->A3 + r0 * L3, *a4 = t->A4 + r0 * L4;
        const float* dy = t->dY + r0 * 4;
        float *d32 = t->D32 + r0 * H4, *d64a = t->D64a + r0 * H3, *d128 = t->D128 + r0 * H2, *d64b = t->D64b + r0 * H1;
        RDL_CK(mm2(t, ga(H4 + 1, 4, Bi, a4, L4, 1, dy, 4, 0, gh + OFF_W5, 4),
                   ga(Bi, H4, 4, dy, 4, 0, Ph + OFF_W5, 4, 1, d32, H4, rdg::EPI_DTANH, a4, L4)),
               "rdl dW5 db5 | dZ4");
        RDL_CK(mm2(t, ga(H3 + 1, H4, Bi, a3, L3, 1, d32, H4, 0, gh + OFF_W4, H4),
                   ga(Bi, H3, H4, d32, H4, 0, Ph + OFF_W4, H4, 1, d64a, H3, rdg::EPI_DTANH, a3, L3)),
               "rdl dW4 db4 | dZ3");
        RDL_CK(mm2(t, ga(H2 + 1, H3, Bi, a2, L2, 1, d64a, H3, 0, gh + OFF_W3, H3),
                   ga(Bi, H2, H3, d64a, H3, 0, Ph + OFF_W3, H3, 1, d128, H2, rdg::EPI_DTANH, a2, L2)),
               "rdl dW3 db3 | dZ2");
        RDL_CK(mm2(t, ga(H1 + 1, H2, Bi, a1, L1, 1, d128, H2, 0, gh + OFF_W2, H2),
                   ga(Bi, H1, H2, d128, H2, 0, Ph + OFF_W2, H2, 1, d64b, H1, rdg::EPI_DTANH, a1, L1)),
               "rdl dW2 db2 | dZ1");
        RDL_CK(mm2(t, ga(U, H1, Bi, Hc + r0 * U, U, 1, d64b, H1, 0, gh + OFF_W1, H1),
                   ga(Bi, U, H1, d64b, H1, 0, Ph + OFF_W1, H1, 1, t->dHh + r0 * U, U)),
               "rdl dW1 | dHhead");
        RDL_CK(colsum(t, d64b, B, H1, H1, gh + OFF_B1), "rdl db1");
    }
    }
    // BPTT (the gate buffer Z is reused for dz: the forward keeps activations in G)
    float* dZl = t->Z;
    if (persistent(t, B)) {
        hipLaunchKernelGGL(lstm_bptt_persist_kernel, dim3(PR_GRID), dim3(256), 0, t->stream, P + OFF_WL + XI * G4,
                           (const float*)t->dHh, (const float*)t->G, (const float*)t->Cs, dZl, t->bpart, g + OFF_BL,
                           prev, t->qbuf, (int)B, T, t->bar);
        RDL_CK(hipGetLastError(), "rdl lstm_bptt_persist_kernel");
    } else {
    RDL_CK(hipMemsetAsync(t->dc, 0, sizeof(float) * B * U, t->stream), "rdl bptt");
    const unsigned cb = (unsigned)((B * U + 255) / 256);
    // the last step's cell alone; then per step s the GEMM dh_{s-1} = dz_s . Wr^T whose
    // epilogue (or split-K reduce) runs the cell backward of step s-1 -> dz_{s-1}, dc
    hipLaunchKernelGGL(cell_bwd_kernel, dim3(cb), dim3(256), 0, t->stream,
                       (const float*)(t->dHh + (int64_t)(T - 1) * B * U), (const float*)t->dhn, 0,
                       (const float*)(t->G + (int64_t)(T - 1) * B * G4), (const float*)(t->Cs + (int64_t)T * B * U),
                       (const float*)(t->Cs + (int64_t)(T - 1) * B * U), t->dc, dZl + (int64_t)(T - 1) * B * G4, B);
    RDL_CK(hipGetLastError(), "rdl cell_bwd_kernel");
    for (int s = T - 1; s > 0; --s) {
        rdg::GemmArgs g{};
        g.M = (int)B; g.N = U; g.K = G4;
        g.A = dZl + (int64_t)s * B * G4; g.lda = G4; g.ta = 0;
        g.B = P + OFF_WL + XI * G4; g.ldb = G4; g.tb = 1;
        g.C = t->dhn; g.ldc = U;
        g.epi = rdg::EPI_LSTM_BWD;
        g.aux = t->dHh + (int64_t)(s - 1) * B * U; g.ldaux = U;
        g.lg = t->G + (int64_t)(s - 1) * B * G4;
        g.lct = t->Cs + (int64_t)s * B * U;
        g.lcp = t->Cs + (int64_t)(s - 1) * B * U;
        g.lcc = t->dc;
        g.lz = dZl + (int64_t)(s - 1) * B * G4;
        RDL_CK(rdg::gemm(t->stream, g, t->split, SPLIT_FLOATS, t->cus), "rdl gemm dh + cell");
    }
    }
    // LSTM weights: dWl = [x | h_prev]^T dz over all rows; dbl; then dp -> dWp, dbp
    RDL_CK(mm2(t, ga(XI, G4, Ri, t->X, XLD, 1, dZl, G4, 0, g + OFF_WL, G4),
               ga(U, G4, Ri, t->H, U, 1, dZl, G4, 0, g + OFF_WL + XI * G4, G4)),
           "rdl dWl x | h");
    if (!persistent(t, B)) RDL_CK(colsum(t, dZl, R, G4, G4, g + OFF_BL), "rdl dbl");   // else summed in BPTT
    if (persistent(t, B)) {   // from the BPTT kernel's dbl and Q = prev^T dz: one launch
        hipLaunchKernelGGL(dense32_grad_kernel, dim3(160), dim3(256), 0, t->stream, P, (const float*)t->qbuf, g);
        RDL_CK(hipGetLastError(), "rdl dense32_grad_kernel");
    } else {
        RDL_CK(mm(t, Ri, 32, G4, dZl, G4, 0, P + OFF_WL + 11 * G4, G4, 1, t->dP, 32), "rdl dP");
        RDL_CK(mm(t, 4, 32, Ri, prev, 4, 1, t->dP, 32, 0, g + OFF_WP, 32), "rdl dWp");
        RDL_CK(colsum(t, t->dP, R, 32, 32, g + OFF_BP), "rdl dbp");
    }
    return RD_OK;
}

int launch_adam(rdl_trainer* t) {
    AdamArgs a{t->grad, t->params, t->m, t->v, t->ctl, t->cfg.lr, t->cfg.beta1, t->cfg.beta2, t->cfg.eps, t->np};
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)((t->np + 255) / 256)), dim3(256), 0, t->stream, a);
    RD_HIP(hipGetLastError(), "rdl adam_kernel");
    return RD_OK;
}

bool bad_windows(const rdl_trainer* t, int64_t B) { return B <= 0 || B > t->Bmax; }

}  // namespace

extern "C" {

int64_t rdl_param_count(int32_t steps) { return steps > 0 ? params_of(steps) : -1; }

int rdl_create(rdl_trainer** out, const rdl_config* cfg, int device, void* hip_stream) {
    if (!out || !cfg) return rd::set_error(RD_EINVAL, "rdl_create: null argument");
    if ((cfg->loss != RDL_LOSS_MSE && cfg->loss != RDL_LOSS_KL) || !(cfg->lr > 0) || cfg->steps <= 0 ||
        cfg->max_windows <= 0 || (int64_t)cfg->steps * cfg->max_windows > ((int64_t)1 << 22) || cfg->metrics_len < 0 ||
        !(cfg->keep_prob > 0.0f && cfg->keep_prob <= 1.0f) || cfg->row_base < 0 ||
        (cfg->kernels & ~(RDL_KERNELS_STEP_RECURRENCE | RDL_KERNELS_LAYER_HEAD)))
        return rd::set_error(RD_EINVAL, "rdl_create: bad config");
    rd::DeviceGuard dg(device);
    RD_HIP(dg.err, "rdl_create: hipSetDevice");
    rdl_trainer* t = new (std::nothrow) rdl_trainer();
    if (!t) return rd::set_error(RD_EINVAL, "rdl_create: out of host memory");
    t->cfg = *cfg;
    if (t->cfg.metrics_len == 0) t->cfg.metrics_len = 4096;
    t->device = device;
    t->cus = cu_count(device);
    t->stream = (hipStream_t)hip_stream;
    t->T = cfg->steps;
    t->np = params_of(t->T);
    t->Bmax = cfg->max_windows;
    const int64_t R = (int64_t)t->T * t->Bmax, B = t->Bmax;
    const int64_t nch = (R + COLSUM_CHUNK - 1) / COLSUM_CHUNK;
    t->colws_floats = nch * G4;
    hipError_t e = hipSuccess;
    auto alloc = [&](float** p, int64_t floats) {
        if (e == hipSuccess) e = hipMalloc((void**)p, sizeof(float) * (size_t)floats);
        if (e == hipSuccess) e = hipMemsetAsync(*p, 0, sizeof(float) * (size_t)floats, t->stream);
    };
    alloc(&t->params, t->np);
    alloc(&t->m, t->np);
    alloc(&t->v, t->np);
    alloc(&t->own_grad, t->np);
    alloc(&t->X, R * XLD);
    alloc(&t->H, (R + B) * U);
    alloc(&t->Cs, (R + B) * U);
    alloc(&t->Z, R * G4);
    alloc(&t->G, R * G4);
    alloc(&t->A1, R * L1);
    alloc(&t->A2, R * L2);
    alloc(&t->A3, R * L3);
    alloc(&t->A4, R * L4);
    alloc(&t->Y, R * 4);
    alloc(&t->dY, R * 4);
    alloc(&t->D32, R * H4);
    alloc(&t->D64a, R * H3);
    alloc(&t->D128, R * H2);
    alloc(&t->D64b, R * H1);
    alloc(&t->dHh, R * U);
    alloc(&t->dP, R * 32);
    alloc(&t->dhn, B * U);
    alloc(&t->dc, B * U);
    alloc(&t->split, SPLIT_FLOATS);
    int64_t nbmax = 0;   // the most workgroups of any batch up to Bmax (head_nb is not monotone)
    for (int64_t b = HF_ROWS; b < t->Bmax + HF_ROWS; b += HF_ROWS) nbmax = std::max<int64_t>(nbmax, head_nb(t->T, b));
    const int64_t hp = (int64_t)t->T * nbmax * HB_PART;
    if (hp <= HPART_MAX_FLOATS) alloc(&t->hpart, hp);
    alloc(&t->colws, t->colws_floats);
    alloc(&t->lpart, 2 * ((R + LOSS_BLOCK - 1) / LOSS_BLOCK));
    alloc(&t->hist, (int64_t)t->cfg.metrics_len * N_MET);
    if (e == hipSuccess) e = hipMalloc((void**)&t->ctl, sizeof(uint32_t) * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&t->bar, sizeof(uint32_t) * 4);
    alloc(&t->bpart, (int64_t)2 * PR_GRID * PB_PART);
    if (e == hipSuccess) e = hipMalloc((void**)&t->hx, sizeof(unsigned long long) * 2 * PR_ROWS * U);
    if (e == hipSuccess) e = hipMemsetAsync(t->hx, 0, sizeof(unsigned long long) * 2 * PR_ROWS * U, t->stream);
    alloc(&t->qbuf, 4 * G4);
    if (e == hipSuccess) e = hipMemsetAsync(t->bar, 0, sizeof(uint32_t) * 4, t->stream);
    t->grad = t->own_grad;
    if (e != hipSuccess) {
        rdl_destroy(t);
        return rd::hip_fail(e, "rdl_create: allocation");
    }
    {   // the ones columns of the head activations (the head GEMMs write columns 0..H_l-1)
        const unsigned gr = (unsigned)((R + 255) / 256);
        hipLaunchKernelGGL(ones_column_kernel, dim3(gr), dim3(256), 0, t->stream, t->A1, R, L1, H1);
        hipLaunchKernelGGL(ones_column_kernel, dim3(gr), dim3(256), 0, t->stream, t->A2, R, L2, H2);
        hipLaunchKernelGGL(ones_column_kernel, dim3(gr), dim3(256), 0, t->stream, t->A3, R, L3, H3);
        hipLaunchKernelGGL(ones_column_kernel, dim3(gr), dim3(256), 0, t->stream, t->A4, R, L4, H4);
        if ((e = hipGetLastError()) != hipSuccess) {
            rdl_destroy(t);
            return rd::hip_fail(e, "rdl_create: ones columns");
        }
    }
    if (int rc = rdl_reset(t)) {
        rdl_destroy(t);
        return rc;
    }
    *out = t;
    return RD_OK;
}

int rdl_destroy(rdl_trainer* t) {
    if (!t) return RD_OK;
    rd::DeviceGuard dg(t->device);
    float* bufs[] = {t->params, t->m, t->v, t->own_grad, t->X, t->H, t->Cs, t->Z, t->G, t->A1, t->A2, t->A3, t->A4,
                     t->Y, t->dY, t->D32, t->D64a, t->D128, t->D64b, t->dHh, t->dP, t->dhn, t->dc, t->split,
                     t->colws, t->lpart, t->hist, t->bpart, t->qbuf, t->hpart};
    for (float* p : bufs)
        if (p) (void)hipFree(p);
    if (t->hx) (void)hipFree(t->hx);
    if (t->ctl) (void)hipFree(t->ctl);
    if (t->bar) (void)hipFree(t->bar);
    delete t;
    return RD_OK;
}

int rdl_set_stream(rdl_trainer* t, void* hip_stream) {
    if (!t) return rd::set_error(RD_EINVAL, "rdl_set_stream: null handle");
    t->stream = (hipStream_t)hip_stream;
    return RD_OK;
}

int rdl_set_params(rdl_trainer* t, const float* params) {
    if (!t || !params) return rd::set_error(RD_EINVAL, "rdl_set_params: null argument");
    rd::DeviceGuard dg(t->device);
    RD_HIP(hipMemcpyAsync(t->params, params, sizeof(float) * t->np, hipMemcpyDeviceToDevice, t->stream),
           "rdl_set_params");
    return RD_OK;
}

int rdl_get_params(rdl_trainer* t, float* params) {
    if (!t || !params) return rd::set_error(RD_EINVAL, "rdl_get_params: null argument");
    rd::DeviceGuard dg(t->device);
    RD_HIP(hipMemcpyAsync(params, t->params, sizeof(float) * t->np, hipMemcpyDeviceToDevice, t->stream),
           "rdl_get_params");
    return RD_OK;
}

int rdl_get_slots(rdl_trainer* t, float* m, float* v) {
    if (!t || !m || !v) return rd::set_error(RD_EINVAL, "rdl_get_slots: null argument");
    rd::DeviceGuard dg(t->device);
    RD_HIP(hipMemcpyAsync(m, t->m, sizeof(float) * t->np, hipMemcpyDeviceToDevice, t->stream), "rdl_get_slots");
    RD_HIP(hipMemcpyAsync(v, t->v, sizeof(float) * t->np, hipMemcpyDeviceToDevice, t->stream), "rdl_get_slots");
    return RD_OK;
}

int rdl_set_slots(rdl_trainer* t, const float* m, const float* v) {
    if (!t || !m || !v) return rd::set_error(RD_EINVAL, "rdl_set_slots: null argument");
    rd::DeviceGuard dg(t->device);
    RD_HIP(hipMemcpyAsync(t->m, m, sizeof(float) * t->np, hipMemcpyDeviceToDevice, t->stream), "rdl_set_slots");
    RD_HIP(hipMemcpyAsync(t->v, v, sizeof(float) * t->np, hipMemcpyDeviceToDevice, t->stream), "rdl_set_slots");
    return RD_OK;
}

int rdl_reset(rdl_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdl_reset: null handle");
    rd::DeviceGuard dg(t->device);
    RD_HIP(hipMemsetAsync(t->m, 0, sizeof(float) * t->np, t->stream), "rdl_reset");
    RD_HIP(hipMemsetAsync(t->v, 0, sizeof(float) * t->np, t->stream), "rdl_reset");
    hipLaunchKernelGGL(init_ctl_kernel, dim3(1), dim3(64), 0, t->stream, t->ctl, t->cfg.beta1, t->cfg.beta2);
    RD_HIP(hipGetLastError(), "rdl_reset");
    return RD_OK;
}

int rdl_forward(rdl_trainer* t, const float* ob, const float* prev_pdflat, const float* state0, int64_t windows,
                float* pdflat, float* state_out) {
    if (!t || !ob || !prev_pdflat || !pdflat || bad_windows(t, windows))
        return rd::set_error(RD_EINVAL, "rdl_forward: bad argument");
    rd::DeviceGuard dg(t->device);
    RD_HIP(dg.err, "rdl_forward");
    if (int rc = run_forward(t, ob, prev_pdflat, state0, windows, pdflat, false)) return rc;
    if (state_out) {
        const int64_t last = (int64_t)t->T * windows * U;
        RD_HIP(hipMemcpyAsync(state_out, t->Cs + last, sizeof(float) * windows * U, hipMemcpyDeviceToDevice,
                              t->stream), "rdl_forward: state");
        RD_HIP(hipMemcpyAsync(state_out + windows * U, t->H + last, sizeof(float) * windows * U,
                              hipMemcpyDeviceToDevice, t->stream), "rdl_forward: state");
    }
    return RD_OK;
}

int rdl_final_state(rdl_trainer* t, int64_t windows, float* state_out) {
    if (!t || !state_out || windows <= 0 || windows != t->last_B)
        return rd::set_error(RD_EINVAL, "rdl_final_state: no forward pass of %lld windows to read",
                             (long long)windows);
    rd::DeviceGuard dg(t->device);
    RD_HIP(dg.err, "rdl_final_state");
    const int64_t last = (int64_t)t->T * windows * U;   // rows of step T: (c, h) after the last step
    RD_HIP(hipMemcpyAsync(state_out, t->Cs + last, sizeof(float) * windows * U, hipMemcpyDeviceToDevice, t->stream),
           "rdl_final_state");
    RD_HIP(hipMemcpyAsync(state_out + windows * U, t->H + last, sizeof(float) * windows * U, hipMemcpyDeviceToDevice,
                          t->stream), "rdl_final_state");
    return RD_OK;
}

int rdl_rollout(rdl_trainer* t, const float* ob, const float* prev_pdflat, const float* t_pdflat,
                const float* state0, int64_t windows, int64_t windows_global) {
    if (!t || !ob || !prev_pdflat || !t_pdflat || bad_windows(t, windows) || windows_global < windows)
        return rd::set_error(RD_EINVAL, "rdl_rollout: bad argument");
    rd::DeviceGuard dg(t->device);
    RD_HIP(dg.err, "rdl_rollout");
    if (int rc = run_forward(t, ob, prev_pdflat, state0, windows, t->Y, true)) return rc;
    return run_backward(t, prev_pdflat, t_pdflat, windows, windows_global);
}

int rdl_apply(rdl_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdl_apply: null handle");
    rd::DeviceGuard dg(t->device);
    RD_HIP(dg.err, "rdl_apply");
    return launch_adam(t);
}

int rdl_step(rdl_trainer* t, const float* ob, const float* prev_pdflat, const float* t_pdflat, const float* state0,
             int64_t windows) {
    if (int rc = rdl_rollout(t, ob, prev_pdflat, t_pdflat, state0, windows, windows)) return rc;
    return launch_adam(t);
}

float* rdl_grad_buffer(rdl_trainer* t) { return t ? t->grad : nullptr; }

int rdl_bind_grad_buffer(rdl_trainer* t, float* grad) {
    if (!t) return rd::set_error(RD_EINVAL, "rdl_bind_grad_buffer: null handle");
    t->grad = grad ? grad : t->own_grad;
    return RD_OK;
}

int rdl_head_path(const rdl_trainer* t) {
    if (!t) return rd::set_error(RD_EINVAL, "rdl_head_path: null handle");
    return (t->cfg.kernels & RDL_KERNELS_LAYER_HEAD) || !t->hpart ? 0 : 1;
}

int rdl_get_counter(rdl_trainer* t, int64_t* opt_steps) {
    if (!t || !opt_steps) return rd::set_error(RD_EINVAL, "rdl_get_counter: null argument");
    rd::DeviceGuard dg(t->device);
    uint32_t c[8], b[4];
    RD_HIP(hipMemcpyAsync(c, t->ctl, sizeof(c), hipMemcpyDeviceToHost, t->stream), "rdl_get_counter");
    RD_HIP(hipMemcpyAsync(b, t->bar, sizeof(b), hipMemcpyDeviceToHost, t->stream), "rdl_get_counter");
    RD_HIP(hipStreamSynchronize(t->stream), "rdl_get_counter");
    if (b[2])   // a persistent launch gave up at a grid barrier (workgroups not co-resident)
        return rd::set_error(RD_EINVAL, "rdl: a persistent recurrence launch timed out at its grid barrier; "
                                        "the steps since are invalid (rdl_config.kernels = RDL_KERNELS_STEP_RECURRENCE avoids the persistent kernels)");
    *opt_steps = c[0];
    return RD_OK;
}

int rdl_read_metrics(rdl_trainer* t, int64_t count, double* out) {
    if (!t || !out || count < 0) return rd::set_error(RD_EINVAL, "rdl_read_metrics: bad argument");
    int64_t steps = 0;
    if (int rc = rdl_get_counter(t, &steps)) return rc;
    const int64_t Hn = t->cfg.metrics_len;
    if (count > steps || count > Hn)
        return rd::set_error(RD_EINVAL, "rdl_read_metrics: only %lld steps kept", (long long)(steps < Hn ? steps : Hn));
    float* host = new (std::nothrow) float[(size_t)Hn * N_MET];
    if (!host) return rd::set_error(RD_EINVAL, "rdl_read_metrics: out of host memory");
    hipError_t e = hipMemcpy(host, t->hist, sizeof(float) * Hn * N_MET, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        delete[] host;
        return rd::hip_fail(e, "rdl_read_metrics");
    }
    for (int64_t k = 0; k < count; ++k) {
        const int64_t s = (steps - count + k) % Hn;
        for (int j = 0; j < N_MET; ++j) out[k * N_MET + j] = host[s * N_MET + j];
    }
    delete[] host;
    return RD_OK;
}

}  // extern "C"
