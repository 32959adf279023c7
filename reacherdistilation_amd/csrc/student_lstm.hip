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

// X[r] = [dropout(ob[r]) (11) | prev[r] . Wp + bp (32) | 0]; r = t B + b (the persistent forward
// forms its steps' rows itself with the same arithmetic)
__global__ __launch_bounds__(256) void inputs_kernel(const float* ob, const float* prev, const float* params,
                                                     float* X, int64_t R, int64_t B, float keep_prob, uint64_t seed,
                                                     int64_t row_base, const uint32_t* ctl) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
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
// 16w..16w+15 x the 4 gate blocks (one A and four B operands per k-step, 4 MFMAs).  The K sum
// runs as two chains, k < 112 and k >= 112, and the epilogue's z = ((lo + hi) + 0) + Zx: the
// persistent kernel's order (its waves split K there), so both give bitwise the same G, c and
// h.  Z_s keeps the input half (the backward reuses Z).
constexpr int RF_ROWS = 64, RF_UNITS = 16, RF_TK = 16, RF_LS = 64 + 16;
constexpr int LSTM_KH = 112;   // the recurrent K sum as two chains, k < 112 and k >= 112, added (lo + hi)
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
    rdg::f32x4 lo[4], hi[4];   // the two K chains (the persistent kernel's waves kh = 0, 1)
#pragma unroll
    for (int y = 0; y < 4; ++y) lo[y] = hi[y] = rdg::f32x4{0.f, 0.f, 0.f, 0.f};
    auto tile = [&](int buf, rdg::f32x4 (&acc)[4]) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int kk = 4 * s + gq;
            const float a = As[buf][kk][16 * wave + i];
#pragma unroll
            for (int y = 0; y < 4; ++y)
                acc[y] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Bs[buf][kk][16 * y + i], acc[y], 0, 0, 0);
        }
    };
    // load pipeline of rd_gemm.h: tile t+2's loads issue right after tile t+1 is staged, so
    // they stay in flight across the barrier and the next MFMA phase
    constexpr int NT = (U + RF_TK - 1) / RF_TK;
    static_assert(LSTM_KH % RF_TK == 0, "the K split falls on a tile boundary");
    stage(0, load_a(0), load_b(0));
    rdg::f32x4 na = load_a(RF_TK), nb = load_b(RF_TK);
    __syncthreads();
    for (int kt = 0; kt < NT; ++kt) {
        const int buf = kt & 1;
        if (kt < LSTM_KH / RF_TK) tile(buf, lo);
        else tile(buf, hi);
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
        const float gi = sigm(((lo[0][r] + hi[0][r]) + 0.0f) + zx[0][r]), gj = tanhf(((lo[1][r] + hi[1][r]) + 0.0f) + zx[1][r]);
        const float gf = sigm(((lo[2][r] + hi[2][r]) + 0.0f) + zx[2][r] + 1.0f), go = sigm(((lo[3][r] + hi[3][r]) + 0.0f) + zx[3][r]);
        const float c = fmaf(gf, cpv[r], gi * gj);
        float* g = Gs + row * G4;
        g[u] = gi; g[U + u] = gj; g[2 * U + u] = gf; g[3 * U + u] = go;
        cs[row * U + u] = c;
        hs[row * U + u] = go * tanhf(c);
    }
}

// ---------------------------------------------------------------- persistent recurrence
// Small batches (B <= PR_ROWS windows, e.g. the reference's 20) are latency bound: ~10 us per
// recurrent step as separate launches whatever the work.  lstm_fwd_persist_kernel runs ALL T
// steps of the forward recurrence in one launch and lstm_bptt_persist_kernel all T steps of BPTT.
// Workgroup w owns units 4w..4w+3 (50 workgroups, round 5; 13 of 16 units before): its 16 gate
// columns c = 4 y + j (gate y, unit j), its slice of Wr held in REGISTERS as the MFMA B operands
// for the whole launch, its cell points (row, unit) one per thread.  Per step the critical path
// is the h hand-off, one short MFMA chain per wave and one cell evaluation per thread: at 13
// workgroups each SIMD issued 104 f32 MFMAs per step with LDS-fed operands (2.9 us) and a thread
// ran two cells (2.2 us), stamped in profiles/r05l_lstm_stamps.jsonl.  The forward's h travels
// as data-tagged granules, no grid barrier; BPTT keeps the write-through payload + agent-scope
// arrival counter form (its granule form measured slower at 13 workgroups, profiles/r05i_*).
// The forward's K sum is two chains, k < PR_KH and k >= PR_KH, added (lo + hi) -- the per-step
// kernel's order -- so G, c and h are bitwise those of the per-step launches.
constexpr int PR_ROWS = 32, PR_UNITS = 4, PR_GRID = U / PR_UNITS;   // 50 workgroups
constexpr int PR_COLS = 4 * PR_UNITS;   // 16 gate columns per workgroup: c = 4 y + j
constexpr int PR_KH = LSTM_KH;          // K split of the forward's gate sums (lstm_rec_fwd_kernel's)
constexpr int PR_KQ = PR_KH / 4, PR_KQ1 = (U - PR_KH) / 4;   // k steps of the two halves (28, 22: pad k >= U skipped)
constexpr uint32_t PR_SPIN_LIMIT = 1u << 22;
static_assert(U % PR_UNITS == 0 && PR_KH % RF_TK == 0 && PR_KQ1 <= PR_KQ, "persistent LSTM tiling");

// BPTT's hand-off between the workgroups of a persistent launch (cdna_hip_programming.md §6
// Guideline 16, the write-through form): the exchanged payload (partial dh) is stored with sc1
// buffer stores and drained (s_waitcnt vmcnt(0)) before the workgroup's arrival on an agent-scope
// counter, and EVERY load of it is an sc1 buffer load -- no L2 writeback or L1 invalidate fences
// (a release/acquire pair per step measured ~3.5 us).  All other data these kernels read was
// written before the launch.
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pr_rsrc(const float* base, int64_t floats) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, (int)(floats * 4), 0x00020000);
}
__device__ __forceinline__ rdg::f32x4 pr_load4(__amdgpu_buffer_rsrc_t r, int64_t idx) {   // sc1
    return __builtin_bit_cast(rdg::f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(idx * 4), 0, 16));
}

// Data-tagged granules (cdna_hip_programming.md §6 Guideline 16, R2 / MI355X_MICROARCH.md
// "allgather"): each exchanged f32 travels as ONE naturally aligned 8-byte word {tag, value},
// written by one agent-scope (sc1) store and read by agent-scope loads; a consumer re-reads
// its granules until every tag is the one it waits for.  No payload drain, no arrival counter,
// no barrier poll per step: the data is the flag.  Tags = (generation << 12) | phase, the
// generation advanced on the device once per forward call (the forward's last workgroup, bar[3];
// a replayed graph advances it too), so a granule left by an earlier call never matches.  Two buffers by
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
// phase = the unrolled step s + 1 <= T - 1 in its own 12 bits (persistent() admits T < PR_MAX_T),
// the generation in the 20 above: with an 8-bit phase, T >= 258 let step 257 of call g - 1 carry
// step 1's tag of call g
constexpr int PR_PHASE_BITS = 12;
constexpr int PR_MAX_T = 1 << PR_PHASE_BITS;
__device__ __forceinline__ uint32_t gr_tag(uint32_t gen, uint32_t phase) { return (gen << PR_PHASE_BITS) | phase; }

// SrcC fence around MFMA chains (student_mlp.hip's fence_begin / fence_end): every operand is
// in registers before the chains start, the accumulators pass through an empty asm
// (memory clobber) before and after them and are read by a VALU before the closing one, so no
// load issues while one of these f32 MFMAs is in flight -- hipcc otherwise renames a chain's
// accumulators and loads the next operands into registers an in-flight MFMA still reads as SrcC
// (scripts/isa/hazards.py class LDSRC; found in the sixteen-wave head backward, round 5).  Used by
// the head's data gradients and the persistent BPTT's weight-gradient chains.
template <int Q>
__device__ __forceinline__ void fence_begin(rdg::f32x4 (&G)[Q]) {
#pragma unroll
    for (int t = 0; t < Q; ++t) asm volatile("" : "+v"(G[t])::"memory");
}
template <int Q>
__device__ __forceinline__ void fence_end(rdg::f32x4 (&G)[Q]) {
#pragma unroll
    for (int t = 0; t < Q; ++t) G[t][3] = __builtin_amdgcn_fmed3f(G[t][3], G[t][3], G[t][3]);
#pragma unroll
    for (int t = 0; t < Q; ++t) asm volatile("" : "+v"(G[t])::"memory");
}
// bar: [0] the forward's finished-workgroup count, [1] the BPTT's barrier counter, [2] timeout
// flag, [3] granule generation.  The last forward workgroup to finish (every one has read the
// generation by then) resets [0] and [1] and advances [3], so the next call's tags are new.
// hx: h granules [2][PR_ROWS][U] (step parity).  state0: null (zero state) or [c | h] of
// [B][U] each; Cs/H rows of step 0 are written from it for the backward.  Wave (rb, kh): rows
// 16 rb.. x the 16 local columns over K half kh; thread t < 4 B: the cell point (row t / 4,
// unit u0 + t % 4).  The launch also forms the inputs (round 5: no inputs_kernel, no Zx GEMM
// launch): per step s the rows X_s = [dropout(ob) | prev . Wp + bp] (x_value: inputs_kernel's
// arithmetic; workgroup 0 stores them for the weight gradient) and the input half of the gates
// Zx_s = X_s Wl[0:43] + bl of the local columns (the Zx GEMM's MFMA k order and epilogue), so
// G, c and h stay bitwise those of the per-step path.  Zx of step s+1 is formed right after step
// s publishes h, while the granules travel.
constexpr int PR_XQ = (XI + 3) / 4;                    // Zx k steps (11; k = 43 is the zero column)
// FU: units per forward workgroup (FNCB column blocks of 16 gate columns each; grid U / FU).
// Measured at 20 windows (round 5): FU 2 / 4 / 8 (100 / 50 / 25 workgroups) forward 43.7 / 43.0 /
// 51.7 us -- fewer readers of the h granules do not pay for the longer MFMA chains
constexpr int FU = 4, FNCB = (FU + 3) / 4, PR_GRID_F = U / FU;
static_assert(U % FU == 0 && (FU % 4 == 0 || FU < 4) && FU * PR_ROWS <= 256, "forward tiling: a cell point per thread");
__global__ __launch_bounds__(256) void lstm_fwd_persist_kernel(const float* __restrict__ P, const float* __restrict__ ob,
                                                               const float* __restrict__ prev, float* __restrict__ X,
                                                               const float* __restrict__ state0, float* __restrict__ G,
                                                               float* __restrict__ Cs, float* __restrict__ H, int B,
                                                               int T, float keep_prob, uint64_t seed, int64_t row_base,
                                                               const uint32_t* __restrict__ ctl, uint32_t* bar,
                                                               unsigned long long* hx) {
    __shared__ __attribute__((aligned(16))) float Zp[2][PR_ROWS][16 * FNCB + 1];   // the K halves' sums [row][c]
    __shared__ __attribute__((aligned(16))) float Xs[PR_ROWS][XLD];               // X_s rows; zero past B
    __shared__ __attribute__((aligned(16))) float Zx[PR_ROWS][16 * FNCB + 1];     // Zx_s of the local columns
    __shared__ int fail_s;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, i = lane & 15, gq = lane >> 4;
    const int u0 = blockIdx.x * FU;
    const int rb = wave & 1, kh = wave >> 1;
    const int kq0 = kh ? PR_KQ : 0;
    const uint32_t gen = bar[3], step = ctl[0];
    const float* Wr = P + OFF_WL + XI * G4;
    if (tid == 0) fail_s = 0;
    // this lane's B operands over the launch: Wr[k][y U + u0 + 4 cb + j] of column i = 4 y + j of
    // block cb, and (block zcb = wave / 2 of the Zx product) Wl[k][..], k < 43, with its bias
    float bw[FNCB][PR_KQ], bx[PR_XQ];
#pragma unroll
    for (int cb = 0; cb < FNCB; ++cb) {
        const int64_t col = (int64_t)(i >> 2) * U + u0 + 4 * cb + (i & 3);
#pragma unroll
        for (int q = 0; q < PR_KQ; ++q) {
            const int k = 4 * (kq0 + q) + gq;
            bw[cb][q] = (q < PR_KQ1 || kh == 0) ? Wr[(int64_t)k * G4 + col] : 0.0f;
        }
    }
    const int zcb = wave >> 1;   // Zx: waves (rb, zcb) for zcb < FNCB
    const int64_t zcol = (int64_t)(i >> 2) * U + u0 + 4 * (zcb < FNCB ? zcb : 0) + (i & 3);
#pragma unroll
    for (int q = 0; q < PR_XQ; ++q) {
        const int k = 4 * q + gq;
        bx[q] = (zcb < FNCB && k < XI) ? P[OFF_WL + (int64_t)k * G4 + zcol] : 0.0f;
    }
    const float bias = P[OFF_BL + zcol];
    // this thread's column of the dense32 part of X (c = 11 + tid % 32 for every row it forms)
    const int dc = tid & 31;
    float wp[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) wp[a] = P[OFF_WP + a * 32 + dc];
    const float bpc = P[OFF_BP + dc];
    for (int x = tid; x < PR_ROWS * XLD; x += 256) (&Xs[0][0])[x] = 0.0f;
    const bool pt = tid < FU * B;
    const int pr = tid / FU, pj = tid % FU, pu = u0 + pj;
    const int pc = 16 * (pj >> 2) + (pj & 3);   // the point's local column of gate 0 (+ 4 y)
    float cst = 0.0f;
    if (pt) {
        const int64_t idx = (int64_t)pr * U + pu;
        const float c0 = state0 ? state0[idx] : 0.0f, h0 = state0 ? state0[(int64_t)B * U + idx] : 0.0f;
        cst = c0;
        Cs[idx] = c0;   // rows of step 0, read by the backward
        H[idx] = h0;
    }
    // X_s -> Xs (and X, workgroup 0): x_value's arithmetic with one Philox draw per (row, 4
    // columns) of the dropout part and the dense32 part's weights held in registers; then
    // Zx_s = Xs Wl[0:43] + bl on waves 0, 1 -> Zx
    auto inputs = [&](int s) {
        for (int x = tid; x < 3 * B; x += 256) {   // dropout(ob) (student_nn.py:24): columns 4 q .. 4 q + 3 < 11
            const int r = x / 3, q = x - 3 * r;
            const int64_t rg = (int64_t)s * B + r;
            uint32_t o[4] = {0u, 0u, 0u, 0u};
            if (keep_prob < 1.0f) {
                const uint64_t w = (uint64_t)(row_base + r);
                rd::philox((uint32_t)w, (uint32_t)(w >> 32), step, (uint32_t)(4 * s + q), (uint32_t)seed,
                           (uint32_t)(seed >> 32), o);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int c = 4 * q + e;
                if (c < 11) {
                    float v = ob[rg * 11 + c];
                    if (keep_prob < 1.0f) v = rd::u01(o[e]) < keep_prob ? v / keep_prob : 0.0f;
                    Xs[r][c] = v;
                    if (blockIdx.x == 0) X[rg * XLD + c] = v;
                }
            }
        }
        for (int x = tid; x < 32 * B; x += 256) {   // prev . Wp + bp (student_nn.py:26)
            const int r = x >> 5;
            const int64_t rg = (int64_t)s * B + r;
            const float* pv = prev + rg * 4;
            float v = bpc;
#pragma unroll
            for (int a = 0; a < 4; ++a) v = fmaf(pv[a], wp[a], v);
            Xs[r][11 + dc] = v;
            if (blockIdx.x == 0) X[rg * XLD + 11 + dc] = v;
        }
        if (blockIdx.x == 0)
            for (int r = tid; r < B; r += 256) X[((int64_t)s * B + r) * XLD + XI] = 0.0f;
        __syncthreads();   // Xs complete; the previous step's cell has read Zx
        if (zcb < FNCB) {
            float av[PR_XQ];
#pragma unroll
            for (int q = 0; q < PR_XQ; ++q) av[q] = Xs[16 * rb + i][4 * q + gq];
            rdg::f32x4 acc[1] = {{0.f, 0.f, 0.f, 0.f}};
            fence_begin(acc);
#pragma unroll
            for (int q = 0; q < PR_XQ; ++q) acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q], bx[q], acc[0], 0, 0, 0);
            fence_end(acc);
#pragma unroll
            for (int r = 0; r < 4; ++r) Zx[16 * rb + 4 * gq + r][16 * zcb + i] = acc[0][r] + bias;
        }
    };
    __syncthreads();   // Xs zeroed before the staging writes
    inputs(0);
    const int arow = 16 * rb + i;   // this lane's A-operand row (h_s row), k = 4 (kq0 + q) + gq
    const bool av_ok = arow < B;
    for (int s = 0; s < T; ++s) {
        // this wave's A operands: h_s[arow][k] over its K half, straight into registers -- each
        // wave gathers its own quadrant of the other workgroups' granules (re-read until every
        // tag matches) and starts its chain when they are in, no staging, no workgroup barrier
        float av[PR_KQ];
        if (s > 0) {
            const unsigned long long* src = hx + (int64_t)(s & 1) * PR_ROWS * U + (int64_t)(av_ok ? arow : 0) * U + 4 * kq0 + gq;
            const uint32_t want = gr_tag(gen, (uint32_t)s);
            for (uint32_t spins = 0;;) {
                unsigned long long v[PR_KQ];
#pragma unroll
                for (int q = 0; q < PR_KQ1; ++q) v[q] = av_ok ? gr_load(src + 4 * q) : (unsigned long long)want << 32;
                if (kh == 0) {
#pragma unroll
                    for (int q = PR_KQ1; q < PR_KQ; ++q) v[q] = av_ok ? gr_load(src + 4 * q) : (unsigned long long)want << 32;
                }
                bool ok = true;
#pragma unroll
                for (int q = 0; q < PR_KQ; ++q) ok &= (q < PR_KQ1 || kh == 0) ? (uint32_t)(v[q] >> 32) == want : true;
#pragma unroll
                for (int q = 0; q < PR_KQ; ++q) av[q] = (q < PR_KQ1 || kh == 0) ? __uint_as_float((uint32_t)v[q]) : 0.0f;
                if (__all(ok)) break;
                if (++spins > PR_SPIN_LIMIT) {
                    __hip_atomic_store(bar + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    fail_s = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        } else {
            const float* hs = state0 && av_ok ? state0 + (int64_t)B * U + (int64_t)arow * U + 4 * kq0 + gq : nullptr;
#pragma unroll
            for (int q = 0; q < PR_KQ; ++q) av[q] = hs && (q < PR_KQ1 || kh == 0) ? hs[4 * q] : 0.0f;
        }
        // this wave's K half: one accumulation chain per column block in k order (the per-step
        // kernel's lo / hi), the blocks' chains interleaved
        rdg::f32x4 acc[FNCB];
#pragma unroll
        for (int cb = 0; cb < FNCB; ++cb) acc[cb] = rdg::f32x4{0.f, 0.f, 0.f, 0.f};
        fence_begin(acc);
#pragma unroll
        for (int q = 0; q < PR_KQ1; ++q) {
#pragma unroll
            for (int cb = 0; cb < FNCB; ++cb) acc[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q], bw[cb][q], acc[cb], 0, 0, 0);
        }
        if (kh == 0) {
#pragma unroll
            for (int q = PR_KQ1; q < PR_KQ; ++q) {
#pragma unroll
                for (int cb = 0; cb < FNCB; ++cb) acc[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q], bw[cb][q], acc[cb], 0, 0, 0);
            }
        }
        fence_end(acc);
#pragma unroll
        for (int cb = 0; cb < FNCB; ++cb)
#pragma unroll
            for (int r = 0; r < 4; ++r) Zp[kh][16 * rb + 4 * gq + r][16 * cb + i] = acc[cb][r];   // C: rows 4 gq + r, column i
        __syncthreads();
        if (fail_s) break;   // (uniform) a peer's granules never arrived: the timeout flag is raised
        // TF1 LSTMCell (lstm_rec_fwd_kernel's arithmetic) at this thread's point
        if (pt) {
            float z[4];
#pragma unroll
            for (int y = 0; y < 4; ++y) z[y] = ((Zp[0][pr][pc + 4 * y] + Zp[1][pr][pc + 4 * y]) + 0.0f) + Zx[pr][pc + 4 * y];
            const float gi = sigm(z[0]), gj = tanhf(z[1]), gf = sigm(z[2] + 1.0f), go = sigm(z[3]);
            const float c = fmaf(gf, cst, gi * gj);
            cst = c;
            const float h = go * tanhf(c);
            if (s + 1 < T) gr_store(hx + (int64_t)((s + 1) & 1) * PR_ROWS * U + (int64_t)pr * U + pu, gr_tag(gen, (uint32_t)(s + 1)), h);
            const int64_t row_g = (int64_t)s * B + pr;
            float* g = G + row_g * G4 + pu;
            g[0] = gi; g[U] = gj; g[2 * U] = gf; g[3 * U] = go;
            Cs[(row_g + B) * U + pu] = c;
            H[(row_g + B) * U + pu] = h;   // for the backward (a later launch)
        }
        if (s + 1 < T) inputs(s + 1);
    }
    // the last workgroup to finish advances the generation (every workgroup read it at entry)
    __syncthreads();
    if (tid == 0) {
        const uint32_t done = __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (done + 1 == gridDim.x) {
            __hip_atomic_store(bar, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(bar + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(bar + 3, gen + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// BPTT of all T steps, split-K over the workgroups: per step s (T-1 .. 0) workgroup w
//  (1) sums dh_next at its points from the 50 partials of step s+1 (fixed order, sc1 loads),
//  (2) runs the cell backward at its points -> dz_s of its 16 gate columns (to LDS),
//  (3) multiplies those 16 columns by its 16 rows of Wr^T: a partial dh_{s-1} for ALL units,
//      stored sc1 to its slot of a per-step-parity partial buffer, arrives at the grid barrier,
//  (4) while the other workgroups arrive: its 16 columns of dWl += [x_s | h_{s-1}]^T dz_s (the
//      LSTM kernel's weight gradient, 243 x 16 per workgroup, accumulated in registers over the
//      steps: no dz round trip through HBM and no weight-gradient launch, round 5).
constexpr int PB_N = 208;    // units, padded: 13 column blocks of 16
constexpr int PB_PART = PB_N * PR_ROWS;   // floats of one workgroup's partial [unit][row]
constexpr int PB_RED = 4 + 16;            // per point: the dbl sums (4 gates) and Q = prev^T dz (4 x 4)
__global__ __launch_bounds__(256) void lstm_bptt_persist_kernel(const float* __restrict__ Wr, const float* __restrict__ dHh,
                                                                const float* __restrict__ G, const float* __restrict__ Cs,
                                                                const float* __restrict__ X, const float* __restrict__ Hp,
                                                                float* __restrict__ dWl, float* __restrict__ part,
                                                                float* __restrict__ dbl, const float* __restrict__ prev,
                                                                float* __restrict__ Q, int B, int T, uint32_t* bar) {
    __shared__ __attribute__((aligned(16))) float Dz[PR_ROWS][PR_COLS + 1];          // dz_s [row][c]; zero past B
    __shared__ float red[PR_ROWS][PR_UNITS][PB_RED];
    __shared__ int ok_s;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, i = lane & 15, gq = lane >> 4;
    const int u0 = blockIdx.x * PR_UNITS;
    // (4)'s operands and sums: wave w owns dWl rows 16 (w + 4 q) .. +15 (q < 4) x the 16 local
    // columns; xa[q][rq] = A^T[k = 16 (w + 4 q) + i][r = 4 rq + gq], A = [x_s | h_{s-1}] rows of step s
    rdg::f32x4 accw[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) accw[q] = rdg::f32x4{0.f, 0.f, 0.f, 0.f};
    float xa[4][PR_ROWS / 4];
    auto load_a = [&](int s) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = 16 * (wave + 4 * q) + i;
#pragma unroll
            for (int rq = 0; rq < PR_ROWS / 4; ++rq) {
                const int r = 4 * rq + gq;
                const int64_t row = (int64_t)s * B + r;
                // branch-free: every lane loads (a lane without an entry from X[0]) and selects, so
                // the 32 loads stay in flight together (as branches, the no-SLP build waited
                // vmcnt(0) between them: BPTT 45 -> 56 us at 20 windows, profiles/r06e_*)
                const bool in = r < B && k < XI + U;
                const float* src = !in ? X : k < XI ? X + row * XLD + k : Hp + row * U + (k - XI);
                const float v = *src;
                xa[q][rq] = in ? v : 0.0f;
            }
        }
    };
    auto dwl_step = [&]() {   // dz_s is in Dz (rows >= B zero)
        float dv[PR_ROWS / 4];
#pragma unroll
        for (int rq = 0; rq < PR_ROWS / 4; ++rq) dv[rq] = Dz[4 * rq + gq][i];
        const int nrq = (B + 3) >> 2;
        fence_begin(accw);
#pragma unroll
        for (int rq = 0; rq < PR_ROWS / 4; ++rq) {
            if (rq < nrq) {
#pragma unroll
                for (int q = 0; q < 4; ++q) accw[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[q][rq], dv[rq], accw[q], 0, 0, 0);
            }
        }
        fence_end(accw);
    };
    const int rb = wave & 1, cbo = wave >> 1;   // rows 16 rb.., unit blocks cbo, cbo + 2, .. (7 or 6 of 13)
    const __amdgpu_buffer_rsrc_t rP = pr_rsrc(part, (int64_t)2 * PR_GRID * PB_PART);
    // this lane's B operands over the launch: B[k][n] = Wr[n][y U + u0 + j] at k = 4 y + j = 4 q4 + gq
    float bw[7][4];
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        const int n = 16 * (cbo + 2 * q) + i;
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) bw[q][q4] = n < U ? Wr[(int64_t)n * G4 + q4 * U + u0 + gq] : 0.0f;
    }
    for (int x = tid; x < PR_ROWS * (PR_COLS + 1); x += 256) (&Dz[0][0])[x] = 0.0f;
    const bool pt = tid < 4 * B;
    const int pr = tid >> 2, pj = tid & 3, pu = u0 + pj;
    float dcs = 0.f;
    float bsum[4] = {0.f, 0.f, 0.f, 0.f};   // dbl: this point's row, all steps, per gate
    float qsum[4][4] = {};                    // Q = prev^T dz: [prev component][gate]
    float cg[4], cct, ccp, cdh, cpv[4];
    auto load_cell = [&](int s) {   // gates, c_t, c_{t-1}, dh from the head: written before the launch
        // branch-free as load_a: a lane without a point loads row (s, 0) of its unit (valid) and
        // its values are never used (every use is under pt)
        const int64_t rs = (int64_t)s * B + (pt ? pr : 0);
        const float* g = G + rs * G4 + pu;
#pragma unroll
        for (int y = 0; y < 4; ++y) cg[y] = g[y * U];
        cct = Cs[(rs + B) * U + pu];
        ccp = Cs[rs * U + pu];
        cdh = dHh[rs * U + pu];
#pragma unroll
        for (int a = 0; a < 4; ++a) cpv[a] = prev[rs * 4 + a];
    };
    load_cell(T - 1);
    load_a(T - 1);
    __syncthreads();   // Dz zeroed
    uint32_t nsync = 0;
    for (int s = T - 1; s >= 0; --s) {
        float dhn = 0.f;
        if (s < T - 1 && pt) {   // (1) dh_next at the point: the 50 partials of step s+1, summed in workgroup order
            const int64_t pb = (int64_t)((s + 1) & 1) * PR_GRID * PB_PART + (int64_t)pu * PR_ROWS + pr;
            float v[PR_GRID];
#pragma unroll
            for (int w = 0; w < PR_GRID; ++w)
                v[w] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rP, (int)((pb + (int64_t)w * PB_PART) * 4), 0, 16));
            float acc = v[0];
#pragma unroll
            for (int w = 1; w < PR_GRID; ++w) acc += v[w];
            dhn = acc;
        }
        // (2) TF1 LSTMCell backward (cell_bwd_kernel's arithmetic)
        if (pt) {
            const float gi = cg[0], gj = cg[1], gf = cg[2], go = cg[3];
            const float dh = s < T - 1 ? cdh + dhn : cdh;
            const float tc = tanhf(cct);
            const float dcv = fmaf(dh * go, fmaf(-tc, tc, 1.0f), dcs);
            const float z0 = dcv * gj * gi * (1.0f - gi), z1 = dcv * gi * fmaf(-gj, gj, 1.0f);
            const float z2 = dcv * ccp * gf * (1.0f - gf), z3 = dh * tc * go * (1.0f - go);
            Dz[pr][pj] = z0; Dz[pr][4 + pj] = z1; Dz[pr][8 + pj] = z2; Dz[pr][12 + pj] = z3;
            bsum[0] += z0; bsum[1] += z1; bsum[2] += z2; bsum[3] += z3;
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                qsum[a][0] = fmaf(cpv[a], z0, qsum[a][0]);
                qsum[a][1] = fmaf(cpv[a], z1, qsum[a][1]);
                qsum[a][2] = fmaf(cpv[a], z2, qsum[a][2]);
                qsum[a][3] = fmaf(cpv[a], z3, qsum[a][3]);
            }
            dcs = dcv * gf;
        }
        if (s == 0) break;
        load_cell(s - 1);
        __syncthreads();
        // (3) partial dh_{s-1}[row][n] over the 16 local columns, for every unit n
        rdg::f32x4 acc[7];
#pragma unroll
        for (int q = 0; q < 7; ++q) acc[q] = rdg::f32x4{0.f, 0.f, 0.f, 0.f};
        {
            float av[4];
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) av[q4] = Dz[16 * rb + i][4 * q4 + gq];
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
#pragma unroll
                for (int q = 0; q < 6; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q4], bw[q][q4], acc[q], 0, 0, 0);
                if (cbo == 0) acc[6] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q4], bw[6][q4], acc[6], 0, 0, 0);
            }
        }
        const int64_t po = (int64_t)(s & 1) * PR_GRID * PB_PART + (int64_t)blockIdx.x * PB_PART;
#pragma unroll
        for (int q = 0; q < 7; ++q) {   // lane (i, gq): rows 16 rb + 4 gq .. +3 of unit 16 (cbo + 2 q) + i
            if (q < 6 || cbo == 0)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, acc[q]), rP,
                                                       (int)((po + (int64_t)(16 * (cbo + 2 * q) + i) * PR_ROWS + 16 * rb + 4 * gq) * 4),
                                                       0, 16);
        }
        // (4) while the sc1 partial stores drain, then arrive (every wave's stores landed first)
        dwl_step();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(bar + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        load_a(s - 1);
        if (tid == 0) {
            const uint32_t target = ++nsync * gridDim.x;
            int ok = 1;
            for (uint32_t spins = 0; __hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target;) {
                if (++spins > PR_SPIN_LIMIT) {
                    __hip_atomic_store(bar + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            ok_s = ok;
        }
        __syncthreads();   // Dz is rewritten by the next step
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keeps the payload loads below the poll
        if (!ok_s) return;
    }
    __syncthreads();   // dz_0 in Dz
    dwl_step();
#pragma unroll
    for (int q = 0; q < 4; ++q) {   // C: rows k = 16 (w + 4 q) + 4 gq + r, local column i
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int k = 16 * (wave + 4 * q) + 4 * gq + r;
            if (k < XI + U) dWl[(int64_t)k * G4 + (i >> 2) * U + u0 + (i & 3)] = accw[q][r];
        }
    }
    // dbl (the gate bias gradient) and Q = prev^T dz of the local columns: the points' sums, in row order
    __syncthreads();
    if (pt) {
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            red[pr][pj][y] = bsum[y];
#pragma unroll
            for (int a = 0; a < 4; ++a) red[pr][pj][4 + 4 * a + y] = qsum[a][y];
        }
    }
    __syncthreads();
    for (int o = tid; o < PR_UNITS * PB_RED; o += 256) {
        const int jj = o / PB_RED, e = o - jj * PB_RED, uu = u0 + jj;
        float v = 0.f;
        for (int r = 0; r < B; ++r) v += red[r][jj][e];
        if (e < 4) dbl[e * U + uu] = v;
        else Q[((e - 4) >> 2) * G4 + ((e - 4) & 3) * U + uu] = v;
    }
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

// workgroup (t, rb) of the grid T x nb: rows t B + 16 rb .. of step t, with step t's head.
// WL (grids of at most HB_WIDE_GRID workgroups, e.g. the reference's 20 windows): the head's
// 31,652 parameters are copied into LDS first (LDS-DMA, one issue burst beside the row
// staging), so the five layers read their B operands from LDS instead of paying an L2/HBM
// round trip each (round 5); same values, same MFMA order.  Larger grids stream them from L2
// (124 KB of LDS would leave one workgroup per CU).
constexpr int HB_WIDE_GRID = 256;   // at most this many one-tile workgroups: the latency-bound forms
static_assert(HSZ % 4 == 0 && (OFF_H % 4) == 0, "16-B pieces of a head's parameters");
// A head's weights in the head backward's MFMA operand order ("packed"), kept beside the
// parameters (t->wpack, [T][HWP]): written by the Adam kernel with every update and by
// pack_heads_kernel when the parameters are set.  Per layer (W5, W4, W3, W2, W1 of [NI][KO]),
// per column block cb < ceil(NI / 16) and k step kq < KO / 4, 64 floats, lane (i, gq) ->
// W[16 cb + i][4 kq + gq] (zero past NI).  A wave of head_bwd_kernel<false, 16> loads each of its
// B operands with one coalesced 256-B access instead of sixteen 16-B pieces of sixteen lines
// (the [NI][KO] layout read per lane cost the backward 15 us of a 24 us launch at 20 windows,
// profiles/r05p_*).
__host__ __device__ constexpr int hw_size(int KO, int NI) { return ((NI + 15) / 16) * 16 * KO; }
constexpr int HWP_5 = 0, HWP_4 = HWP_5 + hw_size(4, H4), HWP_3 = HWP_4 + hw_size(H4, H3),
              HWP_2 = HWP_3 + hw_size(H3, H2), HWP_1 = HWP_2 + hw_size(H2, H1), HWP = HWP_1 + hw_size(H1, U);
// packed index of head offset o (within one head's HSZ), or -1 for the biases (KO is a power of
// two in every layer: shifts and masks, no divisions)
template <int KO>
__device__ __forceinline__ int hw_at(int base, int rel) {
    const int col = rel / KO, k = rel & (KO - 1);
    return base + (((col >> 4) * (KO / 4) + (k >> 2)) << 6) + ((k & 3) << 4) + (col & 15);
}
__device__ __forceinline__ int hw_index(int o) {
    static_assert((H1 & (H1 - 1)) == 0 && (H2 & (H2 - 1)) == 0 && (H3 & (H3 - 1)) == 0 && (H4 & (H4 - 1)) == 0,
                  "power-of-two layer widths");
    if (o < OFF_B1) return hw_at<H1>(HWP_1, o - OFF_W1);
    if (o >= OFF_W2 && o < OFF_B2) return hw_at<H2>(HWP_2, o - OFF_W2);
    if (o >= OFF_W3 && o < OFF_B3) return hw_at<H3>(HWP_3, o - OFF_W3);
    if (o >= OFF_W4 && o < OFF_B4) return hw_at<H4>(HWP_4, o - OFF_W4);
    if (o >= OFF_W5 && o < OFF_B5) return hw_at<4>(HWP_5, o - OFF_W5);
    return -1;
}
__global__ __launch_bounds__(256) void pack_heads_kernel(const float* __restrict__ P, float* __restrict__ wpack, int T) {
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= (int64_t)T * HSZ) return;
    const int ts = (int)(q / HSZ), o = (int)(q - (int64_t)ts * HSZ);
    const int w = hw_index(o);
    if (w >= 0) wpack[(int64_t)ts * HWP + w] = P[OFF_H + q];
}
// step t's head -> W (16-B LDS-DMA pieces, lane l of a wave's burst to base + 16 l); the caller
// waits (vmcnt) before its barrier
__device__ __forceinline__ void head_params_to_lds(const float* __restrict__ P, float* W) {
    constexpr int V4 = HSZ / 4, PER = (V4 + 255) / 256;
    const int wbase = threadIdx.x & ~63;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int x = threadIdx.x + 256 * u;
        if (x < V4) __builtin_amdgcn_global_load_lds(P + 4 * x, W + 4 * (wbase + 256 * u), 16, 0, 0);
    }
}
// The loss of a training forward (small batches; loss_kernel's per-row arithmetic) at the end
// of head_fwd_kernel: dY of the workgroup's rows and its loss / squared-error sums; the metrics
// (their sum in workgroup order) are formed by grad_finish_kernel after BPTT.
struct HeadLoss {
    const float* tgt;   // null: no loss (inference forward)
    float* dY;
    float* part;        // [grid][2] partial sums
    float inv_n;
    int loss;
};
__device__ __forceinline__ float2 row_loss(const float* o, const float* t, int loss, float inv_n, float* d) {
    const float e0 = o[0] - t[0], e1 = o[1] - t[1];
    const float sq = fmaf(e0, e0, e1 * e1);
    float lv, d0, d1, d2 = 0.f, d3 = 0.f;
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
    d[0] = d0; d[1] = d1; d[2] = d2; d[3] = d3;
    return make_float2(lv, sq);
}
template <bool WL>
__global__ __launch_bounds__(256) void head_fwd_kernel(const float* __restrict__ Hc, const float* __restrict__ P0,
                                                       float* A1, float* A2, float* A3, float* A4, float* Y, int64_t B,
                                                       int nb, HeadLoss hl) {
    __shared__ __attribute__((aligned(16))) float Wl[WL ? HSZ : 4];
    __shared__ __attribute__((aligned(16))) float X0[HF_ROWS][U + 4];
    __shared__ __attribute__((aligned(16))) float X1[HF_ROWS][L1];
    __shared__ __attribute__((aligned(16))) float X2[HF_ROWS][L2];
    __shared__ __attribute__((aligned(16))) float X3[HF_ROWS][L3];
    __shared__ __attribute__((aligned(16))) float X4[HF_ROWS][L4];
    __shared__ __attribute__((aligned(16))) float X5[HF_ROWS][8];
    const int ts = blockIdx.x / nb, rb = blockIdx.x - ts * nb;
    const int64_t row0 = (int64_t)ts * B + (int64_t)rb * HF_ROWS, R = (int64_t)(ts + 1) * B;
    const float* P = P0 + OFF_H + (int64_t)ts * HSZ;
    if constexpr (WL) head_params_to_lds(P, Wl);
    head_stage<U, U + 4>(Hc, U, row0, R, X0, threadIdx.x);
    if constexpr (WL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's pieces of Wl have landed
    __syncthreads();
    const float* W = WL ? (const float*)Wl : P;
    head_layer<U, H1, true>(X0, X1, W + OFF_W1, W + OFF_B1, A1, L1, row0, R);
    head_layer<H1, H2, true>(X1, X2, W + OFF_W2, W + OFF_B2, A2, L2, row0, R);
    head_layer<H2, H3, true>(X2, X3, W + OFF_W3, W + OFF_B3, A3, L3, row0, R);
    head_layer<H3, H4, true>(X3, X4, W + OFF_W4, W + OFF_B4, A4, L4, row0, R);
    head_layer<H4, 4, false>(X4, X5, W + OFF_W5, W + OFF_B5, Y, 4, row0, R);
    if (!hl.tgt) return;   // (uniform) inference forward
    __shared__ float ls[HF_ROWS][2];
    const int tid = threadIdx.x;
    if (tid < HF_ROWS) {   // X5 holds the layer's output rows (head_layer ends with a barrier)
        float2 v = make_float2(0.f, 0.f);
        if (row0 + tid < R) {
            float o[4] = {X5[tid][0], X5[tid][1], X5[tid][2], X5[tid][3]};
            float d[4];
            v = row_loss(o, hl.tgt + (row0 + tid) * 4, hl.loss, hl.inv_n, d);
            *reinterpret_cast<rdg::f32x4*>(hl.dY + (row0 + tid) * 4) = rdg::f32x4{d[0], d[1], d[2], d[3]};
        }
        ls[tid][0] = v.x;
        ls[tid][1] = v.y;
    }
    __syncthreads();
    if (tid == 0) {
        float a = 0.f, b = 0.f;
        for (int r = 0; r < HF_ROWS; ++r) { a += ls[r][0]; b += ls[r][1]; }
        hl.part[2 * blockIdx.x] = a;
        hl.part[2 * blockIdx.x + 1] = b;
    }
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
    constexpr int NB = (NI + 15) / 16, IT = (NB + NW - 1) / NW;
    if constexpr (NW != 16) {   // four waves (mid-size batches: weights streamed per MFMA, 56 VGPRs;
                                // the fenced form below held 167 and ran slower) and MT (weights in
                                // registers already): the round-4 chains, clean in the hazard scan
#pragma unroll
        for (int it = 0; it < IT; ++it) {   // unrolled: every weight load of the layer in flight at once
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
        return;
    }
    // the chains' operands: dout's (shared by every column block) and this lane's weights, all
    // loads issued before the first MFMA; the chains interleave (one accumulator per block)
    float av[KO / 4], bv[IT][KO / 4];
#pragma unroll
    for (int kq = 0; kq < KO / 4; ++kq) av[kq] = dout[i][4 * kq + gq];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int col = 16 * (wave + NW * it) + i;
        const bool cv = wave + NW * it < NB && col < NI;
#pragma unroll
        for (int kq = 0; kq < KO / 4; ++kq) bv[it][kq] = wf(it, kq, cv, col, 4 * kq + gq);
    }
    rdg::f32x4 acc[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) acc[it] = rdg::f32x4{0.f, 0.f, 0.f, 0.f};
    fence_begin(acc);
#pragma unroll
    for (int kq = 0; kq < KO / 4; ++kq) {
#pragma unroll
        for (int it = 0; it < IT; ++it)
            if (wave + NW * it < NB) acc[it] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kq], bv[it][kq], acc[it], 0, 0, 0);
    }
    fence_end(acc);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int cb = wave + NW * it;
        if (cb >= NB) break;
        const int col = 16 * cb + i;
        const bool cv = col < NI;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 4 * gq + r;
            float v = acc[it][r];
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
    // from the packed layout (pack_layer): one coalesced load per operand
    __device__ __forceinline__ void load_packed(const float* __restrict__ Wp, int tid) {
        const int wave = tid >> 6, lane = tid & 63;
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int cb = wave + NW * it;
#pragma unroll
            for (int kq = 0; kq < KO / 4; ++kq) w[it][kq] = cb < NB ? Wp[(cb * (KO / 4) + kq) * 64 + lane] : 0.0f;
        }
    }
    __device__ __forceinline__ float operator()(int it, int kq, bool, int, int) const { return w[it][kq]; }
};
// part[m][n] = sum over the 16 rows of act[row][m] d[row][n], m < M (the last input row is the
// ones column: the bias gradient), n < N (one tile of rows: head_bwd_kernel<false>)
template <int M, int N, int NW, int LA, int LD>
__device__ __forceinline__ void head_wgrad(const float (*act)[LA], const float (*d)[LD], float* __restrict__ part) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, gq = lane >> 4;
    constexpr int MB = (M + 15) / 16, NB = (N + 15) / 16;
    for (int t = wave; t < MB * NB; t += NW) {
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
// (eight waves share them), for large batches; else one tile per workgroup, NWV waves: sixteen
// when the whole grid is one wave of workgroups (e.g. the reference's 20 windows: 20
// workgroups on 256 CUs, latency bound -- round 5), else four
template <bool MT, int NWV>
__global__ __launch_bounds__(64 * NWV) void head_bwd_kernel(const float* __restrict__ Hc, const float* __restrict__ P0,
                                                       const float* __restrict__ A1, const float* __restrict__ A2,
                                                       const float* __restrict__ A3, const float* __restrict__ A4,
                                                       const float* __restrict__ dY, float* __restrict__ dHh,
                                                       float* __restrict__ part, int64_t B, int nb, int tpb,
                                                       const float* __restrict__ wpack) {
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
    constexpr int NW = NWV, NT = 64 * NW;   // MT: eight waves share the accumulators
    static_assert(!MT || NW == 8, "the MT form runs eight waves");
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
    // RW: the weights held in registers -- MT (read once per workgroup over its tiles) and the
    // sixteen-wave form (one column block per wave: every layer's weights in one round trip at
    // entry, beside the row staging, instead of one round trip per layer)
    constexpr bool RW = MT || NW == 16;
    if (RW && wpack) {   // (uniform) the packed copy of this step's head weights
        const float* d = wpack + (int64_t)ts * HWP;
        w5.load_packed(d + HWP_5, threadIdx.x);
        w4.load_packed(d + HWP_4, threadIdx.x);
        w3.load_packed(d + HWP_3, threadIdx.x);
        w2.load_packed(d + HWP_2, threadIdx.x);
        w1.load_packed(d + HWP_1, threadIdx.x);
    } else if constexpr (RW) {
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
        if constexpr (MT) asm volatile("" : "+s"(Pk), "+v"(tid));
        // rows past R (the step's last row) are zero (activations and gradients): they add nothing
        head_stage<U, U + 4, NT>(Hc, U, row0, R, X0, tid);
        head_stage<H1 + 1, L1, NT>(A1, L1, row0, R, X1, tid);   // with the ones column
        head_stage<H2 + 1, L2, NT>(A2, L2, row0, R, X2, tid);
        head_stage<H3 + 1, L3, NT>(A3, L3, row0, R, X3, tid);
        head_stage<H4 + 1, L4, NT>(A4, L4, row0, R, X4, tid);
        head_stage<4, 8, NT>(dY, 4, row0, R, D5, tid);
        if (tid < HF_ROWS) X0[tid][U] = row0 + tid < R ? 1.0f : 0.0f;
        __syncthreads();
        if constexpr (RW) {
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
            head_wgrad<U + 1, H1, NW>(X0, D1, pw);
            head_wgrad<H1 + 1, H2, NW>(X1, D2, pw + (OFF_W2 - OFF_W1));
            head_wgrad<H2 + 1, H3, NW>(X2, D3, pw + (OFF_W3 - OFF_W1));
            head_wgrad<H3 + 1, H4, NW>(X3, D4, pw + (OFF_W4 - OFF_W1));
            head_wgrad<H4 + 1, 4, NW>(X4, D5, pw + (OFF_W5 - OFF_W1));
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

// One launch for the gradient's last pieces (small batches, after BPTT): blocks < T HB_BLK run
// head_wgrad_reduce_kernel's sums, the next 160 (dense) dense32_grad_kernel's dot products.
constexpr int HB_BLK = (HB_PART + 255) / 256;
__device__ __forceinline__ void head_part_sum(const float* __restrict__ part, int nb, float* __restrict__ g, int t, int p) {
    if (p >= HB_PART) return;
    const float* q = part + (int64_t)t * nb * HB_PART + p;
    float a = 0.f, b = 0.f;
    int w = 0;
    for (; w + 1 < nb; w += 2) {
        a += q[(int64_t)w * HB_PART];
        b += q[(int64_t)(w + 1) * HB_PART];
    }
    if (w < nb) a += q[(int64_t)w * HB_PART];
    g[OFF_H + (int64_t)t * HSZ + p] = a + b;
}
// dWp = Q . Wl[11:43]^T and dbp = Wl[11:43] . dbl: the input-side dense32 layer's gradients
// (student_nn.py:26) from the BPTT kernel's gate sums, without materialising dP = dZ . Wl^T
// (the same sums in another order: sum over the rows first, then over the 800 gate columns)
__device__ __forceinline__ void dense32_dot(const float* __restrict__ P, const float* __restrict__ Q, float* __restrict__ g,
                                            int o) {
    // o: 0..127 dWp[a][c] (a = o / 32), 128..159 dbp[c]; a fixed-order tree over 256 threads
    __shared__ float red[256];
    const int c = o & 31;
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
// The last block: the metrics of the step from head_fwd_kernel's loss partials (lpart, nl
// workgroups, summed in workgroup order) into the ring slot, and the step words' snapshot for
// the Adam kernel (loss_kernel's job on the other paths).
__global__ __launch_bounds__(256) void grad_finish_kernel(const float* __restrict__ part, int nb, int T,
                                                          const float* __restrict__ P, const float* __restrict__ Q,
                                                          float* __restrict__ g, const float* __restrict__ lpart, int nl,
                                                          float rows, uint32_t* ctl, float* hist, int hist_len) {
    const int b = blockIdx.x;
    if (b < T * HB_BLK) {
        head_part_sum(part, nb, g, b / HB_BLK, (b % HB_BLK) * 256 + threadIdx.x);
    } else if (b < T * HB_BLK + 160) {
        dense32_dot(P, Q, g, b - T * HB_BLK);   // (uniform per block)
    } else if (threadIdx.x == 0) {
        float a = 0.f, c = 0.f;
        for (int w = 0; w < nl; ++w) {
            a += lpart[2 * w];
            c += lpart[2 * w + 1];
        }
        float* h = hist + (int64_t)(ctl[0] % (uint32_t)hist_len) * N_MET;
        h[0] = a;
        h[1] = c;
        h[2] = rows;
        h[3] = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) ctl[4 + k] = ctl[k];
    }
}

// head t's gradient (blockIdx.y = t): grad[OFF_H + t HSZ + p] = sum over step t's nb
// workgroups' partial rows, in row order
__global__ __launch_bounds__(256) void head_wgrad_reduce_kernel(const float* __restrict__ part, int nb,
                                                                float* __restrict__ g) {
    head_part_sum(part, nb, g, blockIdx.y, blockIdx.x * 256 + threadIdx.x);
}
__global__ __launch_bounds__(256) void dense32_grad_kernel(const float* __restrict__ P, const float* __restrict__ Q,
                                                           float* __restrict__ g) {
    dense32_dot(P, Q, g, blockIdx.x);
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
    float* wpack;   // the heads' weights in the head backward's operand order (hw_index)
    float* m;
    float* v;
    uint32_t* ctl;
    float lr, b1, b2, eps;
    int64_t n;   // parameters (params_of(T))
};

// TF1 ApplyAdam (lstm_train.py:73-79) of parameter p with gradient g; the heads' weights also
// into their packed copy
__device__ __forceinline__ void adam_param(const AdamArgs& a, int p, float g, float b1p, float b2p) {
    {
        const float alpha = a.lr * sqrtf(1.0f - b2p) / (1.0f - b1p);
        float m = a.m[p], v = a.v[p];
        m += (g - m) * (1.0f - a.b1);
        v += (g * g - v) * (1.0f - a.b2);
        a.m[p] = m;
        a.v[p] = v;
        const float w = a.params[p] - (m * alpha) / (sqrtf(v) + a.eps);
        a.params[p] = w;
        if (p >= OFF_H) {
            const int q = p - OFF_H, ts = q / HSZ, x = hw_index(q - ts * HSZ);
            if (x >= 0) a.wpack[(int64_t)ts * HWP + x] = w;
        }
    }
}
__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    const uint32_t S = a.ctl[4];
    const float b1p = __uint_as_float(a.ctl[5]), b2p = __uint_as_float(a.ctl[6]);
    if (p < a.n) adam_param(a, p, a.grad[p], b1p, b2p);
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
    float* wpack = nullptr;    // [T][HWP]: the heads' weights packed by the training forward (small batches)
    int64_t colws_floats = 0;
    uint32_t* ctl = nullptr;
    bool loss_in_head = false;   // the last forward computed the loss (head_fwd_kernel<true>)
    uint32_t* bar = nullptr;   // persistent kernels: [0] forward / [1] BPTT barrier arrivals, [2] timeout flag,
                               // [3] granule generation
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

bool persistent(const rdl_trainer* t, int64_t B) {   // (T < PR_MAX_T: every phase fits its tag field)
    return !(t->cfg.kernels & RDL_KERNELS_STEP_RECURRENCE) && B <= PR_ROWS && t->T < PR_MAX_T;
}

// forward over all T steps of B windows.  out_pdflat: where the head's output goes (the
// internal Y when training).
// tgt (training): the loss rides in the head forward where that runs as one wide-grid launch
// (t->loss_in_head tells run_backward)
int run_forward(rdl_trainer* t, const float* ob, const float* prev, const float* state0, int64_t B, float* out_pdflat,
                bool train, const float* tgt = nullptr, int64_t B_global = 0) {
    const int T = t->T;
    const int64_t R = (int64_t)T * B;
    const float* P = t->params;
    t->last_B = B;
    t->loss_in_head = false;
    const float kp = train ? t->cfg.keep_prob : 1.0f;
    if (persistent(t, B)) {   // X, Zx and all T recurrent steps in one launch (it writes the step-0 state rows)
        hipLaunchKernelGGL(lstm_fwd_persist_kernel, dim3(PR_GRID_F), dim3(256), 0, t->stream, P, ob, prev, t->X, state0,
                           t->G, t->Cs, t->H, (int)B, T, kp, t->cfg.seed, t->cfg.row_base, (const uint32_t*)t->ctl,
                           t->bar, t->hx);
        RDL_CK(hipGetLastError(), "rdl lstm_fwd_persist_kernel");
    } else {
    hipLaunchKernelGGL(inputs_kernel, dim3((unsigned)((R * XLD + 255) / 256)), dim3(256), 0, t->stream, ob, prev, P,
                       t->X, R, B, kp, t->cfg.seed, t->cfg.row_base, (const uint32_t*)t->ctl);
    RDL_CK(hipGetLastError(), "rdl inputs_kernel");
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
        const bool wl = (int64_t)T * nb <= HB_WIDE_GRID;
        HeadLoss hl{};
        if (wl && tgt && persistent(t, B)) {   // grad_finish_kernel forms the metrics
            hl = HeadLoss{tgt, t->dY, t->lpart, 1.0f / ((float)T * (float)B_global), t->cfg.loss};
            t->loss_in_head = true;
        }
        auto* kern = wl ? head_fwd_kernel<true> : head_fwd_kernel<false>;
        hipLaunchKernelGGL(kern, dim3((unsigned)(T * nb)), dim3(256), 0, t->stream, Hc, P, t->A1, t->A2,
                           t->A3, t->A4, out_pdflat, B, nb, hl);
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
    if (!t->loss_in_head) {   // else the head forward formed dY and the metrics
    hipLaunchKernelGGL(loss_kernel, dim3(lblk), dim3(LOSS_BLOCK), 0, t->stream, (const float*)t->Y, tgt, t->dY, R,
                       t->cfg.loss, 1.0f / ((float)T * (float)B_global), t->lpart, t->ctl, fold ? t->hist : nullptr,
                       t->cfg.metrics_len);
    RDL_CK(hipGetLastError(), "rdl loss_kernel");
    if (!fold) {
        hipLaunchKernelGGL(metrics_kernel, dim3(1), dim3(256), 0, t->stream, (const float*)t->lpart, lblk, (float)R,
                           t->ctl, t->hist, t->cfg.metrics_len);
        RDL_CK(hipGetLastError(), "rdl metrics_kernel");
    }
    }
    const float* Hc = t->H + B * U;
    // small batches: the head rows' sums, the dense32 gradient and the metrics as one launch after BPTT
    const bool finish = t->loss_in_head;
    if (fused_head(t, R)) {   // the heads' backward as two launches (head_bwd_kernel + fixed-order reduce)
        const int nb = head_nb(T, B), tpb = head_tpb(T, B);
        const bool wide = tpb == 1 && (int64_t)T * nb <= HB_WIDE_GRID;
        auto* kern = tpb > 1 ? head_bwd_kernel<true, 8> : wide ? head_bwd_kernel<false, 16> : head_bwd_kernel<false, 4>;
        hipLaunchKernelGGL(kern, dim3((unsigned)(T * nb)), dim3(tpb > 1 ? 512 : wide ? 1024 : 256), 0, t->stream, Hc, P,
                           (const float*)t->A1, (const float*)t->A2, (const float*)t->A3, (const float*)t->A4,
                           (const float*)t->dY, t->dHh, t->hpart, B, nb, tpb,
                           wide ? (const float*)t->wpack : nullptr);
        RDL_CK(hipGetLastError(), "rdl head_bwd_kernel");
        if (!finish) {
            hipLaunchKernelGGL(head_wgrad_reduce_kernel, dim3((HB_PART + 255) / 256, (unsigned)T), dim3(256), 0,
                               t->stream, (const float*)t->hpart, nb, g);
            RDL_CK(hipGetLastError(), "rdl head_wgrad_reduce_kernel");
        }
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
                           (const float*)t->dHh, (const float*)t->G, (const float*)t->Cs, (const float*)t->X,
                           (const float*)t->H, g + OFF_WL, t->bpart, g + OFF_BL,
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
    // LSTM weights: dWl = [x | h_prev]^T dz over all rows (in the persistent BPTT for small
    // batches); dbl; then dp -> dWp, dbp
    if (!persistent(t, B))
        RDL_CK(mm2(t, ga(XI, G4, Ri, t->X, XLD, 1, dZl, G4, 0, g + OFF_WL, G4),
                   ga(U, G4, Ri, t->H, U, 1, dZl, G4, 0, g + OFF_WL + XI * G4, G4)),
               "rdl dWl x | h");
    if (!persistent(t, B)) RDL_CK(colsum(t, dZl, R, G4, G4, g + OFF_BL), "rdl dbl");   // else summed in BPTT
    if (finish) {   // the heads' row sums + dWp, dbp from the BPTT kernel's dbl and Q = prev^T dz
        hipLaunchKernelGGL(grad_finish_kernel, dim3((unsigned)(T * HB_BLK + 161)), dim3(256), 0, t->stream,
                           (const float*)t->hpart, head_nb(T, B), T, P, (const float*)t->qbuf, g,
                           (const float*)t->lpart, (int)(T * ((B + HF_ROWS - 1) / HF_ROWS)), (float)R, t->ctl, t->hist,
                           t->cfg.metrics_len);
        RDL_CK(hipGetLastError(), "rdl grad_finish_kernel");
    } else if (persistent(t, B)) {   // from the BPTT kernel's dbl and Q = prev^T dz: one launch
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
    AdamArgs a{t->grad, t->params, t->wpack, t->m, t->v, t->ctl, t->cfg.lr, t->cfg.beta1, t->cfg.beta2, t->cfg.eps, t->np};
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
    alloc(&t->wpack, (int64_t)t->T * HWP);
    alloc(&t->colws, t->colws_floats);
    alloc(&t->lpart, std::max<int64_t>(2 * ((R + LOSS_BLOCK - 1) / LOSS_BLOCK), 2 * HB_WIDE_GRID));
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
                     t->colws, t->lpart, t->hist, t->bpart, t->qbuf, t->hpart, t->wpack};
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
    const int64_t n = (int64_t)t->T * HSZ;
    hipLaunchKernelGGL(pack_heads_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, t->stream,
                       (const float*)t->params, t->wpack, t->T);
    RD_HIP(hipGetLastError(), "rdl_set_params: pack_heads_kernel");
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
    if (int rc = run_forward(t, ob, prev_pdflat, state0, windows, t->Y, true, t_pdflat, windows_global)) return rc;
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
