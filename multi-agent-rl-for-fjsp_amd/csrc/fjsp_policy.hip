// fjsp_policy.hip — fused A2C policy step for gfx950 (one launch per vector step).
//
// Replaces the ~40 PyTorch launches of a2c_vec.VecMultiAgentA2C.policy (reference predict,
// a2c.py:168-252): for every env, the 8 actor MLPs (networks.ActorNetwork: d -> 256 -> 256 ->
// n_a, softmax), the action mask / renormalisation / uniform fallback (a2c.py:204-220), the
// action draw (inverse CDF over the masked probabilities, or argmax) and the centralised
// critic (networks.CentralizedCriticNetwork: 38 -> 256 -> 256 -> 128 -> 1).
//
// Grid (1-D, 512 threads = 8 wavefronts per workgroup, two workgroups per CU: 70 KB of LDS):
//   blocks [0, nc)            the critic on tiles of 32 envs (values wanted)
//   blocks [nc, nc + 8 na)    actor (b - nc) / na on tiles of 64 envs (actions wanted)
// (k_policy_step, the collect's launch, adds the env step of each tile and, by default, runs the
// pickup station's and the AGV's tiles as two 32-env workgroups each: 10 na actor blocks.)
// The hidden activations never leave LDS, as bf16 planes (below) [3][env][k]:
//   actor:  x [3][64][16+8]; on two column tiles h1 in two K halves [3][64][128+8] (rows 0..127,
//           then 128..255: layer 2 is summed over the two halves, so one half-size buffer
//           serves); on one column tile (a 32-env half, or a station tile's <= 32 distinct
//           inputs) the whole h1 [3][32][256+8]
//   critic: x [3][32][48+8]; h1, then h2 [3][32][256+8] (in place across a barrier)
// Every layer with K >= 16 runs on v_mfma_f32_32x32x16_bf16 with f32 operands split into three
// bf16 planes (six plane products per 16-deep block, below).  Actor: each wave owns 32 rows of
// layer 2 x the tile's 64 envs (two 32 x 32 tiles sharing each weight fragment); layer 1 one
// 32 x 32 tile per wave and half.  Critic: one 32-row tile per wave (layer 3: waves 0..3).  The
// actor's 256 -> n_a logits and the critic's 128 -> 1 value are f32 VALU dot products straight
// from the accumulators.  Weights are pre-split and pre-packed per (row tile, 16-deep block,
// plane) in lane order (a2c_vec.pack_policy_weights, include/fjsp.h), so each A fragment is one
// coalesced 1 KB load per wave; B fragments (activations) are 16-byte conflict-free LDS reads.
// Numerics: each product carries <= ~2^-22 relative error (f32's own rounding is 2^-24 per
// operation), sums in f32; the outputs equal PyTorch's f32 policy within 1e-5 (tests) and the
// reference's greedy actions on its trained policy.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../include/fjsp.h"
#include "fjsp_stamps.h"
#include "fjsp_stepdev.h"

namespace {

// diagnostic builds only (-DFJSP_STAMPS, scripts/diag_policy_stamps.py): per workgroup, wave 0's
// phase clock stamps; slots 0 / 10 s_memrealtime at entry / exit, 1..9 s_memtime at entry,
// forced check, inputs, layer 1, h1, layer 2, h2, critic layer 3 or actor logits, exit; 11 HW_ID,
// 12 XCC_ID, 13 role | forced << 8
FJSP_DIAG(__device__ unsigned long long g_pstamps[2048 * 16];)
#ifdef FJSP_STAMPS
#define PST(i, v)                                                                                \
    do {                                                                                         \
        if (tid == 0) g_pstamps[(size_t)blockIdx.x * 16 + (i)] = (unsigned long long)(v);        \
    } while (0)
#else
#define PST(i, v) ((void)0)
#endif

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int TA = 64;                // envs per actor workgroup (two 32-env column tiles)
constexpr int TC = 32;                // envs per critic workgroup
constexpr int NWAVE = 8;
constexpr int NTHR = 64 * NWAVE;
constexpr int HID = 256;
constexpr int NAG = 8;
constexpr int A_DPAD = FJSP_POLICY_ACTOR_DPAD, C_DPAD = FJSP_POLICY_CRITIC_DPAD;
static_assert(A_DPAD % 16 == 0 && C_DPAD % 16 == 0, "inputs come in 16-deep MFMA blocks");

// f32 products on the bf16 matrix cores.  Every f32 operand x is carried as three bf16 planes,
// hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid) (both differences exact in f32), so
// x = hi + mid + lo up to 2^-24 |x|; a . b is the sum of the six plane products of order >= 2^-16
// (hi.hi, hi.mid, mid.hi, mid.mid, hi.lo, lo.hi), the three dropped ones are <= 2^-23 |a b|
// together (with the split residuals <= ~2^-22 |a b|, the order of f32 rounding), and every
// product of two bf16 is exact in the f32 accumulator.  Cost: one 16-deep block of a 32 x 32 tile
// is six v_mfma_f32_32x32x16_bf16 (32 cycles each) against eight v_mfma_f32_32x32x2_f32 (64
// cycles each), 192 against 512 cycles.  Weights are split once per update on the host side
// (a2c_vec.pack_policy_weights), activations when they are written to LDS.
constexpr int NP = 3;                              // bf16 planes per f32 value
// bf16 row strides of the activation planes [env][k] (k + 8: the 16-byte fragment reads of 16
// consecutive lanes hit distinct banks); plane sizes
constexpr int XSA = A_DPAD + 8, XSC = C_DPAD + 8, HSA = HID / 2 + 8, HSC = HID + 8;
constexpr int XPA = TA * XSA, XPC = TC * XSC, HPA = TA * HSA, HPC = TC * HSC;
constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int X_BYTES = cmax(NP * XPA, NP * XPC) * 2;
constexpr int H_BYTES = cmax(cmax(NP * HPA, NP * HPC) * 2, NWAVE * 8 * TA * 4);   // also the logit partials
constexpr int W3_BYTES = 8 * HID * 4;
constexpr int LDS_BYTES = X_BYTES + H_BYTES + W3_BYTES;
// the actor's input planes end here; the station dedup's slot / input words fit in the rest of X
constexpr int ACT_X_BYTES = NP * XPA * 2;
static_assert(A_DPAD * 32 == NTHR, "a half tile's inputs: one per thread");
static_assert(NP * HPC * 2 <= H_BYTES && NWAVE * 8 * TA * 4 <= H_BYTES, "one column tile's whole h1, then the logit partials");
static_assert(ACT_X_BYTES + (64 + 4 + 3 * 64) * 4 <= X_BYTES, "station dedup words beside the actor inputs");
static_assert(2 * LDS_BYTES <= 160 * 1024, "two workgroups per CU");

__constant__ int c_obs_off[NAG] = {0, 7, 20, 23, 26, 29, 32, 35};
__constant__ int c_obs_dim[NAG] = {7, 13, 3, 3, 3, 3, 3, 3};
__constant__ int c_mask_off[NAG] = {0, 3, 11, 14, 17, 20, 23, 26};
__constant__ int c_nact[NAG] = {3, 8, 3, 3, 3, 3, 3, 3};

using fjsp::fmix64;

__device__ __forceinline__ void split3(float v, __bf16& hi, __bf16& mid, __bf16& lo) {
    hi = (__bf16)v;
    const float r = v - (float)hi;
    mid = (__bf16)r;
    lo = (__bf16)(r - (float)mid);
}

// acc += a . b over one 16-deep block, small products first
__device__ __forceinline__ f32x16 mfma6(const bf16x8 a[NP], const bf16x8 b[NP], f32x16 acc) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
}

// Weight blocks of one row tile in flight: a register ring of D + 1 blocks x NP planes.
constexpr int WPD = 1;
template <int KB>
struct WRing {
    static constexpr int D = KB < WPD ? KB : WPD;
    bf16x8 w[D + 1][NP];
};
// W packed [row tiles][KBT][NP][64 lanes][8] bf16, element (t, kb, p, l, j) = plane p of
// W[32 t + (l & 31)][16 kb + 8 (l >> 5) + j] (the A-operand lane order of the 32x32x16 MFMA: one
// coalesced 1 KB load per plane and block).  Blocks kb0 .. kb0 + KB - 1 of row tile rt:
template <int KB, int KBT>
__device__ __forceinline__ const bf16x8* wblocks(const bf16x8* __restrict__ wp, int rt, int kb0, int lane) {
    return wp + ((size_t)rt * KBT + kb0) * NP * 64 + lane;
}
// Issue the ring's first D blocks, ahead of the barrier before the layer.
template <int KB>
__device__ __forceinline__ void wring_start(WRing<KB>& R, const bf16x8* __restrict__ a) {
#pragma unroll
    for (int q = 0; q < WRing<KB>::D; q++)
#pragma unroll
        for (int p = 0; p < NP; p++) R.w[q][p] = a[(q * NP + p) * 64];
}

// acc[c] += W(blocks at a) . act(env columns c0 + 32 c .. + 31), c < NC, over KB 16-deep blocks;
// act = LDS planes [NP][env][ST] (plane size PL), k contiguous from the first block (lane l
// reads its 8 k of column l & 31 as one 16-byte B fragment).  R holds blocks 0..D-1
// (wring_start).  Fully unrolled so that the rings are registers without copies (a rotating copy
// made the compiler wait for each weight load right after issuing it): weight blocks D ahead,
// B fragments one MFMA group ahead, each pinned by a scheduling barrier (the scheduler otherwise
// sinks the loads to their first use).
template <int KB, int ST, int PL, int NC>
__device__ __forceinline__ void mfma_rows(WRing<KB>& R, const bf16x8* __restrict__ a, const __bf16* act, int c0, int lane,
                                          f32x16 acc[NC]) {
    constexpr int D = WRing<KB>::D;
    const __bf16* bq = act + (c0 + (lane & 31)) * ST + 8 * (lane >> 5);
    bf16x8 fb[2][NP];
#pragma unroll
    for (int p = 0; p < NP; p++) fb[0][p] = *reinterpret_cast<const bf16x8*>(bq + p * PL);
#pragma unroll
    for (int kb = 0; kb < KB; kb++) {
        if (kb + D < KB) {
#pragma unroll
            for (int p = 0; p < NP; p++) R.w[(kb + D) % (D + 1)][p] = a[((kb + D) * NP + p) * 64];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < NC; c++) {
            const int g = kb * NC + c;
            if (g + 1 < KB * NC) {
                const int kn = (g + 1) / NC, cn = (g + 1) % NC;
#pragma unroll
                for (int p = 0; p < NP; p++)
                    fb[(g + 1) & 1][p] = *reinterpret_cast<const bf16x8*>(bq + 32 * cn * ST + 16 * kn + p * PL);
            }
            __builtin_amdgcn_sched_barrier(0);
            acc[c] = mfma6(R.w[kb % (D + 1)], fb[g & 1], acc[c]);
        }
    }
}

template <int NC>
__device__ __forceinline__ void zero_acc(f32x16 acc[NC]) {
#pragma unroll
    for (int j = 0; j < NC; j++)
#pragma unroll
        for (int r = 0; r < 16; r++) acc[j][r] = 0.0f;
}

// C/D layout of the 32x32 MFMAs: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5), so
// a lane's 16 rows of a tile at row0 are four runs of 4: row0 + 8 g + 4 (lane >> 5) + i, r = 4 g + i.
// Per-row f32 vectors (biases, the value head) for those rows:
struct Row16 {
    float4 v[4];
    __device__ __forceinline__ float operator[](int r) const {
        const float4& q = v[r >> 2];
        return (r & 3) == 0 ? q.x : (r & 3) == 1 ? q.y : (r & 3) == 2 ? q.z : q.w;
    }
};
__device__ __forceinline__ Row16 load_rows(const float* __restrict__ B, int row0, int lane) {
    Row16 r;
#pragma unroll
    for (int g = 0; g < 4; g++) r.v[g] = *reinterpret_cast<const float4*>(B + row0 + 8 * g + 4 * (lane >> 5));
    return r;
}
__device__ __forceinline__ float relu(float v) { return v > 0.0f ? v : 0.0f; }
// relu(acc + bias) of a tile -> rows k0 .. k0 + 31, env columns col0 .. col0 + 31 of the bf16
// planes [NP][env][ST] (4 consecutive k per store)
template <int ST, int PL>
__device__ __forceinline__ void store_planes(const f32x16& acc, int k0, int col0, const Row16& bias, __bf16* out, int lane) {
    const int col = col0 + (lane & 31);
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const int k = k0 + 8 * g + 4 * (lane >> 5);
        bf16x4 ph, pm, pl;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            __bf16 x0, x1, x2;
            split3(relu(acc[4 * g + i] + bias[4 * g + i]), x0, x1, x2);
            ph[i] = x0;
            pm[i] = x1;
            pl[i] = x2;
        }
        *reinterpret_cast<bf16x4*>(out + col * ST + k) = ph;
        *reinterpret_cast<bf16x4*>(out + PL + col * ST + k) = pm;
        *reinterpret_cast<bf16x4*>(out + 2 * PL + col * ST + k) = pl;
    }
}

// relu(acc + bias) of a tile -> rows (features) row0 .. row0 + 31 of the sample-major f32 matrix
// out [samples][ld] for samples col0 .. col0 + 31 (< n): four 16-byte stores per lane
__device__ __forceinline__ void store_rows_f32(const f32x16& acc, int row0, const Row16& bias, float* __restrict__ out,
                                               int ld, int col0, int n, int lane) {
    const int col = col0 + (lane & 31);
    if (col >= n) return;
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const int r = 4 * g;
        *reinterpret_cast<float4*>(out + (size_t)col * ld + row0 + 8 * g + 4 * (lane >> 5)) =
            make_float4(relu(acc[r] + bias[r]), relu(acc[r + 1] + bias[r + 1]), relu(acc[r + 2] + bias[r + 2]),
                        relu(acc[r + 3] + bias[r + 3]));
    }
}

// The logits' partial sums of this wave's 32 rows of h2 = relu(acc + b2) (rows of the C/D
// layout) for NA actions -> s_part[wave][j][env]: per lane its 16 rows, then the other
// half-wave's 16 (lane ^ 32).  Actions in chunks of up to 4 (all 8 at once spilled at 128 VGPRs).
template <int NA, int NC>
__device__ __forceinline__ void logit_partials(const f32x16 acc[NC], const Row16& b2, const float* s_w3, float* s_part,
                                               int wave, int lane) {
    constexpr int CH = NA < 4 ? NA : 4;
    static_assert(NA % CH == 0, "action chunks");
#pragma unroll
    for (int c = 0; c < NC; c++) {
        float h[16];
#pragma unroll
        for (int r = 0; r < 16; r++) h[r] = relu(acc[c][r] + b2[r]);
#pragma unroll
        for (int j0 = 0; j0 < NA; j0 += CH) {
            float l[CH];
#pragma unroll
            for (int j = 0; j < CH; j++) l[j] = 0.0f;
#pragma unroll
            for (int g = 0; g < 4; g++)
#pragma unroll
                for (int j = 0; j < CH; j++) {
                    const float4 w =
                        *reinterpret_cast<const float4*>(s_w3 + (j0 + j) * HID + 32 * wave + 8 * g + 4 * (lane >> 5));
                    l[j] = fmaf(w.x, h[4 * g], l[j]);
                    l[j] = fmaf(w.y, h[4 * g + 1], l[j]);
                    l[j] = fmaf(w.z, h[4 * g + 2], l[j]);
                    l[j] = fmaf(w.w, h[4 * g + 3], l[j]);
                }
#pragma unroll
            for (int j = 0; j < CH; j++) {
                const float t = l[j] + __shfl_xor(l[j], 32);
                if (lane < 32) s_part[(wave * 8 + j0 + j) * TA + 32 * c + lane] = t;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// The tile's inputs: din feature rows from row off of the [38][n] slab, zero-padded to DPAD, for
// the tile's T envs -> registers (issued first: they overlap the mask check) -> the bf16 planes
// [NP][T][DPAD + 8].  ROWS: the inputs are sample-major rows [n][GROW] instead (the update's
// distinct global states, gathered from k_group_keys' rows), read along each row.
constexpr int XI = cmax(C_DPAD * TC, A_DPAD * TA) / NTHR;
constexpr int GROW = 40;   // floats per sample-major feature row (38 + 2 zeros)
template <int T, int DPAD, bool ROWS>
__device__ __forceinline__ void input_kc(int i, int& k, int& c) {
    k = ROWS ? i % DPAD : i / T;
    c = ROWS ? i / DPAD : i % T;
}
template <int T, int DPAD, bool ROWS = false, int NV = XI>
__device__ __forceinline__ void inputs_load(const float* __restrict__ feats, int n, int e0, int off, int din, int tid,
                                            float v[NV]) {
#pragma unroll
    for (int q = 0; q < NV; q++) {
        int k, c;
        const int i = tid + q * NTHR;
        input_kc<T, DPAD, ROWS>(i, k, c);
        const size_t at = ROWS ? (size_t)(e0 + c) * GROW + off + k : (size_t)(off + k) * n + e0 + c;
        v[q] = (i < DPAD * T && k < din && e0 + c < n) ? feats[at] : 0.0f;
    }
}
template <int T, int DPAD, bool ROWS = false>
__device__ __forceinline__ void inputs_store(const float v[XI], int tid, __bf16* s_x) {
    constexpr int S = DPAD + 8, PL = T * S;
#pragma unroll
    for (int q = 0; q < XI; q++) {
        int k, c;
        const int i = tid + q * NTHR;
        input_kc<T, DPAD, ROWS>(i, k, c);
        if (i < DPAD * T) {
            __bf16 x0, x1, x2;
            split3(v[q], x0, x1, x2);
            s_x[c * S + k] = x0;
            s_x[PL + c * S + k] = x1;
            s_x[2 * PL + c * S + k] = x2;
        }
    }
}

struct PolicyArgs {
    const float* feats;
    const int8_t* masks;
    int n;
    const float* actor_w;
    const float* critic_w;
    const uint64_t* seedp;
    uint32_t gid0, step;
    int deterministic;
    uint8_t* actions;
    float* values;
    float* probs_out;
    int nc, na;   // critic / actor workgroups per role
    int tile0 = 0;   // first 64-env tile of the launch (k_policy_step over an env range)
    int xmap = 0;    // actor workgroup -> (role, tile) order, actor_block
    int dedup = 1;   // the station agents' MLP once per distinct input of a tile (actor_tile)
    int split = 0;   // k_policy_step: the pickup station's and the AGV's tiles as two 32-env workgroups each
};

// Actor workgroup j (after the critic's) -> (role, tile).  Workgroups are dealt to the 8 XCDs
// round-robin (block b -> XCD b mod 8), and each XCD has its own 4 MB L2, while the eight actors'
// split-bf16 weights are 8 x 428 KB + the critic's 667 KB.  xmap 0: role-major (every XCD sees
// every role's tiles, so every L2 pulls all nine networks each launch); 1: role = j mod 8 (one
// actor per XCD; the AGV's tiles all on one XCD); 2: the roles in four pairs, each pair on two
// XCDs with the tiles alternating between them (two actors + the critic per L2, the AGV's tiles
// over 64 CUs); 3: two quads of roles, each with one of the two heavy actors (AGV, pickup
// station) and three stations, each quad on four XCDs with its roles rotating over them round by
// round (four actors + the critic per L2, every XCD one heavy role's share).
__device__ __forceinline__ void actor_block(const PolicyArgs& A, int j, int& role, int& tile) {
    if (A.xmap == 3) {
        constexpr uint32_t QUAD = 0x7650'4321u;   // nibble 4q + i = role i of quad q
        const int x = j & 7, k = j >> 3, q = x >> 2;
        role = (int)((QUAD >> (4 * (4 * q + (((x & 3) + k) & 3)))) & 0xFu);
        tile = k;
    } else if (A.xmap == 1) {
        role = j & 7;
        tile = j >> 3;
    } else if (A.xmap == 2) {
        // pairs (AGV, small machine), (pickup, big machine), (blue 1, blue 2), (red, green)
        constexpr uint32_t PAIR = 0x7654'3021u;   // nibble 2p + s = role s of pair p
        const int x = j & 7, k = j >> 3, p = x & 3, h = x >> 2;
        role = (int)((PAIR >> (4 * (2 * p + ((k + h) & 1)))) & 0xFu);
        tile = k;
    } else {
        role = j / A.na;
        tile = j % A.na;
    }
}

// The critic on a tile of 32 envs: layers 1 and 2 one 32-row tile per wave, layer 3 (128 rows)
// on waves 0..3, the value head from layer 3's accumulators.  SAVE (the A2C update's forward,
// fjsp_a2c_critic_forward): the post-ReLU hidden layers also go to HBM, h1 / h2 [n][256] and
// h3 [n][128] f32, sample-major (what the backward reads).
struct CriticSave {
    float* h1;
    float* h2;
    float* h3;
};
template <bool SAVE, bool ROWS = false>
__device__ __forceinline__ void critic_tile(const PolicyArgs& A, int tile, unsigned char* s_mem, int tid, int lane,
                                            int wave, const CriticSave& sv) {
    __bf16* s_x = reinterpret_cast<__bf16*>(s_mem);              // inputs [NP][TC][XSC]
    __bf16* s_h = reinterpret_cast<__bf16*>(s_mem + X_BYTES);    // h1, then h2 [NP][TC][HSC]
    float* s_part = reinterpret_cast<float*>(s_mem);             // value partials [4][TC] (after layer 1)
    const int n = A.n, e0 = tile * TC;
    const float* wb = A.critic_w;
    const bf16x8* W1 = reinterpret_cast<const bf16x8*>(wb);
    const float* B1 = wb + NP * HID * C_DPAD / 2;
    const bf16x8* W2 = reinterpret_cast<const bf16x8*>(B1 + HID);
    const float* B2 = B1 + HID + NP * HID * HID / 2;
    const bf16x8* W3 = reinterpret_cast<const bf16x8*>(B2 + HID);     // [4 row tiles][16][NP][64][8]
    const float* B3 = B2 + HID + NP * 128 * HID / 2;                  // [128]
    const float* W4 = B3 + 128;                                       // [128]
    const float* B4 = W4 + 128;                                       // [1]
    float xv[XI];
    inputs_load<TC, C_DPAD, ROWS>(A.feats, n, e0, 0, 38, tid, xv);
    WRing<C_DPAD / 16> r1;
    wring_start(r1, wblocks<C_DPAD / 16, C_DPAD / 16>(W1, wave, 0, lane));
    const Row16 b1 = load_rows(B1, 32 * wave, lane);
    inputs_store<TC, C_DPAD, ROWS>(xv, tid, s_x);
    __syncthreads();
    PST(3, __builtin_amdgcn_s_memtime());
    f32x16 a[1];
    zero_acc<1>(a);
    mfma_rows<C_DPAD / 16, XSC, XPC, 1>(r1, wblocks<C_DPAD / 16, C_DPAD / 16>(W1, wave, 0, lane), s_x, 0, lane, a);
    PST(4, __builtin_amdgcn_s_memtime());
    WRing<HID / 16> r2;
    wring_start(r2, wblocks<HID / 16, HID / 16>(W2, wave, 0, lane));
    store_planes<HSC, HPC>(a[0], 32 * wave, 0, b1, s_h, lane);
    if (SAVE) store_rows_f32(a[0], 32 * wave, b1, sv.h1, HID, e0, n, lane);
    const Row16 b2 = load_rows(B2, 32 * wave, lane);
    __syncthreads();
    PST(5, __builtin_amdgcn_s_memtime());
    zero_acc<1>(a);
    mfma_rows<HID / 16, HSC, HPC, 1>(r2, wblocks<HID / 16, HID / 16>(W2, wave, 0, lane), s_h, 0, lane, a);
    PST(6, __builtin_amdgcn_s_memtime());
    const int rt3 = wave & 3;
    WRing<HID / 16> r3;
    wring_start(r3, wblocks<HID / 16, HID / 16>(W3, rt3, 0, lane));
    const Row16 b3 = load_rows(B3, 32 * rt3, lane), w4 = load_rows(W4, 32 * rt3, lane);
    __syncthreads();                               // every wave has read h1
    store_planes<HSC, HPC>(a[0], 32 * wave, 0, b2, s_h, lane);
    if (SAVE) store_rows_f32(a[0], 32 * wave, b2, sv.h2, HID, e0, n, lane);
    __syncthreads();
    PST(7, __builtin_amdgcn_s_memtime());
    if (wave < 4) {
        zero_acc<1>(a);
        mfma_rows<HID / 16, HSC, HPC, 1>(r3, wblocks<HID / 16, HID / 16>(W3, rt3, 0, lane), s_h, 0, lane, a);
        if (SAVE) store_rows_f32(a[0], 32 * rt3, b3, sv.h3, 128, e0, n, lane);
        // the value head: this lane's 16 rows of h3, the other half-wave's (lane ^ 32), then the
        // four row tiles through LDS
        float v = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; r++) v = fmaf(w4[r], relu(a[0][r] + b3[r]), v);
        v += __shfl_xor(v, 32);
        if (lane < 32) s_part[wave * TC + lane] = v;
    }
    PST(8, __builtin_amdgcn_s_memtime());
    __syncthreads();
    if (tid < TC && e0 + tid < n) {
        float val = B4[0];
#pragma unroll
        for (int w = 0; w < 4; w++) val += s_part[w * TC + tid];
        A.values[e0 + tid] = val;
    }
}

// The actor's layers 1-3 on NC 32-env column tiles of s_x (layer 1 per K half of layer 2: one
// 32 x 32 tile per wave and half, so only half of h1 is ever in LDS), leaving the logit partials
// [8 waves][8 actions][TA] in s_part.
template <int NC>
__device__ __forceinline__ void actor_mlp(const PolicyArgs& A, int role, unsigned char* s_mem, int tid, int lane, int wave,
                                          const bf16x8* W1, const float* B1, const bf16x8* W2, const float* B2) {
    __bf16* s_x = reinterpret_cast<__bf16*>(s_mem);
    __bf16* s_h = reinterpret_cast<__bf16*>(s_mem + X_BYTES);
    float* s_part = reinterpret_cast<float*>(s_mem + X_BYTES);
    const float* s_w3 = reinterpret_cast<const float*>(s_mem + X_BYTES + H_BYTES);
    if constexpr (NC == 1) {
        // one column tile: the whole h1 [NP][32][256 + 8] fits the h buffer, so layer 1 runs on
        // all eight waves at once (row tile = wave) and layer 2 sums its 16 blocks in one pass
        // (the same block order as the two halves: bit-identical)
        WRing<1> r1;
        wring_start(r1, wblocks<1, 1>(W1, wave, 0, lane));
        const Row16 b1 = load_rows(B1, 32 * wave, lane);
        __syncthreads();
        PST(3, __builtin_amdgcn_s_memtime());
        f32x16 a1[1];
        zero_acc<1>(a1);
        mfma_rows<1, XSA, XPA, 1>(r1, wblocks<1, 1>(W1, wave, 0, lane), s_x, 0, lane, a1);
        WRing<HID / 16> r2;
        wring_start(r2, wblocks<HID / 16, HID / 16>(W2, wave, 0, lane));
        store_planes<HSC, HPC>(a1[0], 32 * wave, 0, b1, s_h, lane);
        __syncthreads();
        PST(4, __builtin_amdgcn_s_memtime());
        f32x16 acc[1];
        zero_acc<1>(acc);
        mfma_rows<HID / 16, HSC, HPC, 1>(r2, wblocks<HID / 16, HID / 16>(W2, wave, 0, lane), s_h, 0, lane, acc);
        const Row16 b2 = load_rows(B2, 32 * wave, lane);
        __syncthreads();                           // every wave has read h1 (s_part overlays it)
        PST(7, __builtin_amdgcn_s_memtime());
        if (c_nact[role] == 8) logit_partials<8, 1>(acc, b2, s_w3, s_part, wave, lane);
        else logit_partials<3, 1>(acc, b2, s_w3, s_part, wave, lane);
        __syncthreads();
        PST(8, __builtin_amdgcn_s_memtime());
        return;
    }
    const int rt1 = wave & 3, ct1 = wave >> 2;   // layer-1 tile of each half
    const bool l1 = NC == 2 || ct1 == 0;          // with one column tile, waves 4..7 have no layer-1 tile
    WRing<1> r1;
    if (l1) wring_start(r1, wblocks<1, 1>(W1, rt1, 0, lane));
    Row16 b1 = load_rows(B1, 32 * rt1, lane);
    __syncthreads();
    PST(3, __builtin_amdgcn_s_memtime());
    f32x16 acc[NC];
    zero_acc<NC>(acc);
#pragma unroll
    for (int half = 0; half < 2; half++) {
        f32x16 a1[1];
        if (l1) {
            zero_acc<1>(a1);
            mfma_rows<1, XSA, XPA, 1>(r1, wblocks<1, 1>(W1, 4 * half + rt1, 0, lane), s_x, 32 * ct1, lane, a1);
        }
        WRing<HID / 32> r2;
        wring_start(r2, wblocks<HID / 32, HID / 16>(W2, wave, 8 * half, lane));
        if (l1) store_planes<HSA, HPA>(a1[0], 32 * rt1, 32 * ct1, b1, s_h, lane);
        __syncthreads();
        PST(4 + 2 * half, __builtin_amdgcn_s_memtime());
        mfma_rows<HID / 32, HSA, HPA, NC>(r2, wblocks<HID / 32, HID / 16>(W2, wave, 8 * half, lane), s_h, 0, lane, acc);
        if (half == 0) {                           // the second half's layer-1 weights and biases
            if (l1) wring_start(r1, wblocks<1, 1>(W1, 4 + rt1, 0, lane));
            b1 = load_rows(B1, 128 + 32 * rt1, lane);
        }
        __syncthreads();                           // every wave has read this half
        PST(5 + 2 * half, __builtin_amdgcn_s_memtime());
    }
    // layer 3, the logits, straight from the accumulators
    const Row16 b2 = load_rows(B2, 32 * wave, lane);
    if (c_nact[role] == 8) logit_partials<8, NC>(acc, b2, s_w3, s_part, wave, lane);
    else logit_partials<3, NC>(acc, b2, s_w3, s_part, wave, lane);
    __syncthreads();
    PST(8, __builtin_amdgcn_s_memtime());
}

// Actor `role` on a tile of 64 envs.  Layer 1 is computed per K half of layer 2 (rows 0..127,
// then 128..255: one 32 x 32 tile per wave each), each half stored as the bf16 planes of layer
// 2's input and summed into layer 2's accumulators (32 rows x 64 envs per wave), so only half of
// h1 is ever in LDS.
// half >= 0: only the tile's envs 32 half .. 32 half + 31, on one column tile (the split pickup /
// AGV workgroups of k_policy_step, PolicyArgs::split)
__device__ __forceinline__ void actor_tile(const PolicyArgs& A, int role, int tile, unsigned char* s_mem, int tid,
                                           int lane, int wave, int& act_out, int half = -1) {
    __bf16* s_x = reinterpret_cast<__bf16*>(s_mem);                      // inputs [NP][TA][XSA]
    float* s_part = reinterpret_cast<float*>(s_mem + X_BYTES);           // logit partials [8][8][TA] (after layer 2)
    float* s_w3 = reinterpret_cast<float*>(s_mem + X_BYTES + H_BYTES);   // logit weights [8][256]
    const int n = A.n, e0 = tile * TA + (half < 0 ? 0 : 32 * half), ne = half < 0 ? TA : 32;
    const float* wb = A.actor_w + (size_t)role * FJSP_POLICY_ACTOR_FLOATS;
    const bf16x8* W1 = reinterpret_cast<const bf16x8*>(wb);
    const float* B1 = wb + NP * HID * A_DPAD / 2;
    const bf16x8* W2 = reinterpret_cast<const bf16x8*>(B1 + HID);
    const float* B2 = B1 + HID + NP * HID * HID / 2;
    const float* W3 = B2 + HID;                                          // f32 [8][256]
    const float* B3 = W3 + 8 * HID;                                      // [8]
    float xv[XI];
    if (half < 0) inputs_load<TA, A_DPAD>(A.feats, n, e0, c_obs_off[role], c_obs_dim[role], tid, xv);
    else inputs_load<32, A_DPAD, false, 1>(A.feats, n, e0, c_obs_off[role], c_obs_dim[role], tid, xv);
    const float4 w3v = reinterpret_cast<const float4*>(W3)[tid];
    const int na = c_nact[role], mo = c_mask_off[role];
    // a tile in which the agent has exactly one valid action in every env: the draw (and argmax)
    // returns that action whatever the network says, and the masked probabilities are exactly
    // one-hot (p / p, or the uniform fallback over one action) -- skip the MLP.  The station
    // agents are forced in 96-100 % of an A2C collect's samples and whole tiles in 38-100 %
    // (scripts/diag_forced_actions.py)
    uint32_t mbits = 0;   // the env's valid actions (threads < TA)
    int forced = 1;
    if (tid < ne && e0 + tid < n) {
#pragma unroll
        for (int j = 0; j < 8; j++)
            if (j < na && A.masks[(size_t)(mo + j) * n + e0 + tid] != 0) mbits |= 1u << j;
        forced = __builtin_popcount(mbits) == 1;
    }
    if (__syncthreads_and(forced)) {
        PST(13, role | 256);
        PST(9, __builtin_amdgcn_s_memtime());
        PST(10, __builtin_amdgcn_s_memrealtime());
        if (tid < ne && e0 + tid < n) {
            const int e = e0 + tid, only = __builtin_ctz(mbits | 256u);
            A.actions[(size_t)role * n + e] = (uint8_t)only;
            act_out = only;
            if (A.probs_out)
                for (int j = 0; j < 8; j++) A.probs_out[((size_t)role * 8 + j) * n + e] = j == only ? 1.0f : 0.0f;
        }
        return;
    }
    PST(2, __builtin_amdgcn_s_memtime());
    reinterpret_cast<float4*>(s_w3)[tid] = w3v;
    // The station agents (three inputs) see a handful of distinct inputs per tile (<= 7 in every
    // unforced tile of an A2C collect, scripts/diag_tile_distinct.py): their MLP then runs once
    // per distinct input on ONE 32-env column tile (half the matrix-core work) and every env reads
    // its input's logits.  A column's outputs depend only on its input (each MFMA output element
    // sums the same 16-deep blocks in the same order), so the probabilities are bit-identical.
    int ncol = half < 0 ? 2 : 1;
    uint32_t* s_slot = reinterpret_cast<uint32_t*>(s_mem + ACT_X_BYTES);   // [64] slot | leader << 8
    if (role >= 2 && half < 0 && A.dedup) {
        uint32_t* s_feat = s_slot + TA + 4;                                   // [3][64] input bits
        if (wave < 3) s_feat[wave * TA + lane] = __float_as_uint(xv[0]);     // wave w: feature w of env lane
        __syncthreads();
        if (wave == 0) {
            const uint32_t x0 = s_feat[lane], x1 = s_feat[TA + lane], x2 = s_feat[2 * TA + lane];
            uint64_t rem = __ballot(e0 + lane < n);
            uint32_t slot = 0, nu = 0;
            while (rem) {
                const int l = __builtin_ctzll(rem);
                const uint32_t y0 = __shfl(x0, l), y1 = __shfl(x1, l), y2 = __shfl(x2, l);
                const uint64_t same = __ballot(x0 == y0 && x1 == y1 && x2 == y2) & rem;
                if ((same >> lane) & 1u) slot = nu | (lane == l ? 256u : 0u);
                rem &= ~same;
                ++nu;
            }
            s_slot[lane] = slot;
            if (lane == 0) s_slot[TA] = nu;
        }
        __syncthreads();
        if (s_slot[TA] <= 32) ncol = 1;
    }
    if (half >= 0) {
        // the half's 32 envs into columns 0 .. 31 (the 64-column plane layout)
        constexpr int S = A_DPAD + 8;
        const int k = tid / 32, c = tid % 32;   // 16 x 32 inputs: one per thread
        __bf16 x0, x1, x2;
        split3(xv[0], x0, x1, x2);
        s_x[c * S + k] = x0;
        s_x[XPA + c * S + k] = x1;
        s_x[2 * XPA + c * S + k] = x2;
        actor_mlp<1>(A, role, s_mem, tid, lane, wave, W1, B1, W2, B2);
    } else if (ncol == 1) {
        // the distinct inputs (each group's first env) into columns 0 .. nu - 1
        constexpr int S = A_DPAD + 8;
#pragma unroll
        for (int q = 0; q < XI; q++) {
            const int i = tid + q * NTHR, k = i / TA, c = i % TA;
            const uint32_t sl = s_slot[c];
            if (i < A_DPAD * TA && (sl & 256u)) {
                __bf16 x0, x1, x2;
                split3(xv[q], x0, x1, x2);
                const int col = (int)(sl & 255u);
                s_x[col * S + k] = x0;
                s_x[XPA + col * S + k] = x1;
                s_x[2 * XPA + col * S + k] = x2;
            }
        }
        actor_mlp<1>(A, role, s_mem, tid, lane, wave, W1, B1, W2, B2);
    } else {
        inputs_store<TA, A_DPAD>(xv, tid, s_x);
        actor_mlp<2>(A, role, s_mem, tid, lane, wave, W1, B1, W2, B2);
    }
    if (tid < ne && e0 + tid < n) {
        const int e = e0 + tid;
        const int col = ncol == 1 && half < 0 ? (int)(s_slot[tid] & 255u) : tid;   // this env's logit column
        float lg[8], p[8], m[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            float v = 0.0f;
            if (j < na) {
                v = B3[j];
#pragma unroll
                for (int w = 0; w < NWAVE; w++) v += s_part[(w * 8 + j) * TA + col];
            }
            lg[j] = v;
        }
        float mx = -INFINITY;
        // fixed 8-trip loops guarded by na: fully unrolled, the arrays stay in registers
#pragma unroll
        for (int j = 0; j < 8; j++) if (j < na) mx = fmaxf(mx, lg[j]);
        float s = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; j++) { p[j] = j < na ? expf(lg[j] - mx) : 0.0f; s += p[j]; }
        float s2 = 0.0f, ms = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            m[j] = j < na && ((mbits >> j) & 1u) ? 1.0f : 0.0f;
            p[j] = (p[j] / s) * m[j];
            s2 += p[j];
            ms += m[j];
        }
#pragma unroll
        for (int j = 0; j < 8; j++) p[j] = s2 > 0.0f ? p[j] / s2 : m[j] / ms;
        int act = 0;
        if (A.deterministic) {
            float best = p[0];
#pragma unroll
            for (int j = 1; j < 8; j++) if (j < na && p[j] > best) { best = p[j]; act = j; }
        } else {
            const uint64_t seed = *A.seedp;
            // keyed by the env's GLOBAL id: shards of a multi-GPU job draw independent streams
            const uint64_t h = fmix64(seed ^ fmix64(((uint64_t)(A.gid0 + (uint32_t)e) << 32) | A.step) ^
                                      (uint64_t)(role + 1) * 0x9E3779B97F4A7C15ull);
            const float u = (float)(h >> 40) * (1.0f / 16777216.0f);
            float tot = 0.0f, cdf[8];
#pragma unroll
            for (int j = 0; j < 8; j++) { tot += j < na ? p[j] : 0.0f; cdf[j] = tot; }
            const float x = (1.0f - u) * tot;
#pragma unroll
            for (int j = 0; j < 8; j++) act += (j < na && cdf[j] < x) ? 1 : 0;
            if (act >= na) act = na - 1;
        }
        A.actions[(size_t)role * n + e] = (uint8_t)act;
        act_out = act;
        if (A.probs_out)
            for (int j = 0; j < 8; j++) A.probs_out[((size_t)role * 8 + j) * n + e] = j < na ? p[j] : 0.0f;
    }
}

// Packed weights (floats; the bf16 blocks are NP * rows * K / 2 floats), see include/fjsp.h.
__global__ void __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(4, 4))) k_policy(PolicyArgs A) {
    __shared__ __attribute__((aligned(16))) unsigned char s_mem[LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // (critic first or last, the AGV's workgroups first: within 3 %, profiles/r03/experiments)
    const int b = blockIdx.x;
    int role = NAG, tile = 0;
    if (b >= A.nc) actor_block(A, b - A.nc, role, tile);
    PST(0, __builtin_amdgcn_s_memrealtime());
    PST(1, __builtin_amdgcn_s_memtime());
    PST(11, __builtin_amdgcn_s_getreg(4 | (31 << 11)));
    PST(12, __builtin_amdgcn_s_getreg(20 | (31 << 11)));
    PST(13, role);
    int act = 0;
    if (role == NAG) critic_tile<false>(A, b, s_mem, tid, lane, wave, CriticSave{});
    else actor_tile(A, role, tile, s_mem, tid, lane, wave, act);
    PST(9, __builtin_amdgcn_s_memtime());
    PST(10, __builtin_amdgcn_s_memrealtime());
}

// ---- the collect's vector step in one launch: policy + FJSPSimulation.step (a2c.py:284-309)
// The step of a 64-env tile needs only that tile's eight actions (FJSPSimulation.py:144-242), so
// it runs inside the policy launch, in the actor workgroup of the tile that finishes last: no
// wait, no assumption about which workgroups are resident.  Hand-off (MI355X_MICROARCH.md
// § inter-workgroup visibility, "Valid forms" table, first row): each actor workgroup stores its
// role's 64 actions write-through (sc1, 4 envs per dword), its storing wave drains them
// (vmcnt(0)), the workgroup's barrier, then one lane adds 1 to the tile's arrival counter
// (agent-scope atomic); the workgroup whose add returns 7 is the tile's last, resets the counter
// for the next launch, and its wave 0 loads the 8 x 16 action words with sc1 loads (L2-served,
// never an L1 copy) and steps the tile's envs exactly as k_step<canon> does.  Every other load
// of the step (state words, order table, tray-slot arena, MT rows, the reward table) reads bytes
// no other workgroup writes in this launch.
typedef __attribute__((address_space(1))) uint32_t gu32;
struct StepArgs {
    fjsp::DevState S;
    fjsp::Cfg C;
    // the step's outputs (row t of the collect's slabs; the collect's subset of fjsp_out, so that
    // the kernel's arguments fit the SGPRs: any may be NULL)
    double* rewards;
    uint8_t* term;
    uint8_t* trunc;
    uint32_t* status;
    int8_t* next_masks;
    float* feats;
    uint32_t* tile_cnt;    // [na] arrivals per tile (0 between launches)
    uint32_t* tile_act;    // [na][8][16] the tile's actions, 4 envs per dword
    int flags;             // STEP_AUTORESET
};
constexpr int STEP_AUTORESET = 1;   // reset(seed=None) an env whose episode ended

// The tile's state words, [NSTATE][64] u32 after the policy's LDS (STATE_BYTES more per
// workgroup: 2 x 77.5 KB still fit a CU): every actor workgroup of the tile copies them in with
// LDS DMAs at its start, in the shadow of its network, so the one that runs the step reads them
// from LDS instead of waiting a memory round trip after the hand-off.
constexpr int STATE_BYTES = fjsp::NSTATE * 64 * 4;
// ... and the reward table (RLUT_SIZE doubles, the same for every tile) after them, so the step
// tail neither copies it nor waits for it
constexpr int LUT_BYTES = fjsp::RLUT_SIZE * 8;
static_assert(LUT_BYTES % 256 == 0, "the reward table in whole 64-dword DMA pieces");
static_assert(2 * (LDS_BYTES + STATE_BYTES + LUT_BYTES) <= 160 * 1024, "two workgroups per CU");
__device__ __forceinline__ void state_prefetch(const StepArgs& St, int tile, uint32_t* s_state, int lane, int wave) {
    const int e = min(tile * TA + lane, St.S.n - 1);
    for (int i = wave; i < fjsp::NSTATE; i += NWAVE)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(St.S.words + (size_t)i * St.S.n + e),
                                         (__attribute__((address_space(3))) void*)(s_state + i * 64), 4, 0, 0);
    const uint32_t* lut = reinterpret_cast<const uint32_t*>(St.C.lut);
    uint32_t* s_lut = s_state + fjsp::NSTATE * 64;
    for (int i = wave; i < LUT_BYTES / 256; i += NWAVE)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(lut + i * 64 + lane),
                                         (__attribute__((address_space(3))) void*)(s_lut + i * 64), 4, 0, 0);
}

// The step tail's outputs staged in the (then free) policy LDS as rows of the tile's 64 envs, then
// copied out by all eight waves in 16-byte pieces: 24 store instructions for the workgroup
// instead of 108 four- or one-byte stores on the stepping wave (the store issue was ~5 k of the
// tail's ~16 k cycles, scripts/diag_collect_tail.py).  Rows: u32 [69][64] = a2c features 0..37,
// state words 38..67, status 68; f64 [8][64] rewards; u8 [31][64] = masks 0..28, term, trunc.
constexpr int STG_F32 = 0, STG_NF32 = fjsp::NFEAT + fjsp::NSTATE + 1;
constexpr int STG_F64 = STG_F32 + STG_NF32 * 64 * 4;
constexpr int STG_U8 = STG_F64 + NAG * 64 * 8, STG_NU8 = fjsp::NMASK + 2;
static_assert(STG_U8 + STG_NU8 * 64 <= LDS_BYTES - 16 && STG_F64 % 16 == 0 && STG_U8 % 16 == 0, "staging rows");
// observe() into the staging rows (StoreSink's values for the collect's two outputs); one wave
// builds the a2c features, another the masks, from the staged state (the work of the other half
// is dead code in each)
template <bool FEATS, bool MASKS>
struct TileSink {
    uint32_t* rf;   // feature rows
    uint8_t* rm;    // mask rows
    int lane;
    __device__ __forceinline__ void feat(int c, float v) { if (FEATS) rf[c * 64 + lane] = __float_as_uint(v); }
    __device__ __forceinline__ void i32(int f, int v) { feat(fjsp::FEAT_OF_I32[f], (float)v); }
    __device__ __forceinline__ void i8(int f, int v) { feat(fjsp::FEAT_OF_I8[f], (float)(int8_t)v); }
    __device__ __forceinline__ void f32(int f, float v) { feat(fjsp::FEAT_OF_F32[f], v); }
    __device__ __forceinline__ void mask(int f, int v) { if (MASKS) rm[f * 64 + lane] = (uint8_t)(int8_t)v; }
};
// the next observation of a staged tile from its staged post-step state: wave 1 the masks, wave 2
// the features (and the state's status word, which observe() flags on an int8 overflow)
__device__ __forceinline__ void tile_observe(const StepArgs& St, unsigned char* s_mem, const uint32_t* s_state, int lane,
                                             int wave) {
    uint32_t* rf = reinterpret_cast<uint32_t*>(s_mem + STG_F32);
    fjsp::Env E;
    // the mask wave never reads the status word (observe() only ORs flags into it) and does not
    // load it: wave 2 rewrites that staged word below, with no barrier between the two waves
#pragma unroll
    for (int i = 0; i < fjsp::NSTATE; i++) E.w[i] = (wave == 1 && i == 2) ? 0u : rf[(fjsp::NFEAT + i) * 64 + lane];
    fjsp::Cfg C = St.C;
    C.lut = reinterpret_cast<const double*>(s_state + fjsp::NSTATE * 64);
    if (wave == 1) {
        TileSink<false, true> sink{rf, s_mem + STG_U8, lane};
        fjsp::observe(E, C, sink);
    } else {
        TileSink<true, false> sink{rf, s_mem + STG_U8, lane};
        fjsp::observe(E, C, sink);
        rf[(fjsp::NFEAT + 2) * 64 + lane] = E.w[2];
    }
}
static_assert(fjsp::NSTATE > 2, "the status word is state word 2 (fjsp_env.h Env::status)");
__device__ __forceinline__ void tile_copy_out(const StepArgs& St, int tile, const unsigned char* s_mem, int tid) {
    const size_t n = (size_t)St.S.n, e0 = (size_t)tile * TA;
    const uint4* sf = reinterpret_cast<const uint4*>(s_mem + STG_F32);
    for (int c = tid; c < STG_NF32 * 16; c += NTHR) {
        const int row = c >> 4, piece = c & 15;
        uint32_t* dst = row < fjsp::NFEAT ? (St.feats ? reinterpret_cast<uint32_t*>(St.feats) + row * n : nullptr)
                        : row < fjsp::NFEAT + fjsp::NSTATE ? St.S.words + (row - fjsp::NFEAT) * n : St.status;
        if (dst) *reinterpret_cast<uint4*>(dst + e0 + 4 * piece) = sf[c];
    }
    const uint4* sd = reinterpret_cast<const uint4*>(s_mem + STG_F64);
    if (St.rewards) {
        for (int c = tid; c < NAG * 32; c += NTHR)
            *reinterpret_cast<uint4*>(St.rewards + (c >> 5) * n + e0 + 2 * (c & 31)) = sd[c];
    }
    const uint4* sb = reinterpret_cast<const uint4*>(s_mem + STG_U8);
    for (int c = tid; c < STG_NU8 * 4; c += NTHR) {
        const int row = c >> 2, piece = c & 3;
        uint8_t* dst = row < fjsp::NMASK ? (St.next_masks ? reinterpret_cast<uint8_t*>(St.next_masks) + row * n : nullptr)
                       : row == fjsp::NMASK ? St.term : St.trunc;
        if (dst) *reinterpret_cast<uint4*>(dst + e0 + 16 * piece) = sb[c];
    }
}

// STAGED: a full tile whose outputs go through the staging rows (tile_copy_out); else every lane
// stores its own outputs (partial tiles, unaligned outputs).
template <bool STAGED>
__device__ __forceinline__ void tile_step(const PolicyArgs& A, const StepArgs& St, int tile, unsigned char* s_mem,
                                          const uint32_t* s_state, int lane) {
    const double* s_lut = reinterpret_cast<const double*>(s_state + fjsp::NSTATE * 64);
    const int e = tile * TA + lane;
    const bool valid = e < A.n;
    FJSP_DIAG(const int tid = lane;)   // diagnostic builds: the tail's phases into the workgroup's slots 2..6
    fjsp::Env E;
    int act[NAG];
    if (valid) {
#pragma unroll
        for (int i = 0; i < fjsp::NSTATE; i++) E.w[i] = s_state[i * 64 + lane];
        const gu32* ta = (const gu32*)(St.tile_act) + (size_t)tile * NAG * 16 + (lane >> 2);
#pragma unroll
        for (int a = 0; a < NAG; a++)
            act[a] = (int)((__hip_atomic_load(ta + a * 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (8 * (lane & 3))) &
                           0xFFu);
    }
    if (!valid) return;
    PST(2, __builtin_amdgcn_s_memtime());
    fjsp::Cfg C = St.C;
    C.lut = s_lut;
    const fjsp::Tables T = fjsp::tables_of(St.S, e);
    // k_step<canon>'s step_and_emit for the outputs the collect asks for (the observation before
    // the auto-reset is not among them)
    const uint32_t n = (uint32_t)St.S.n, ue = (uint32_t)e;
    uint32_t* rf = reinterpret_cast<uint32_t*>(s_mem + STG_F32);
    double* rd = reinterpret_cast<double*>(s_mem + STG_F64);
    uint8_t* rb = s_mem + STG_U8;
    uint32_t res[NAG];
    const double g8 = fjsp::env_advance<true>(E, T, C, act, nullptr, res);
    PST(3, __builtin_amdgcn_s_memtime());
#pragma unroll
    for (int a = 0; a < NAG; a++) {
        const double r = g8 + fjsp::local_reward(C, a, res[a], act[a]);
        if (STAGED) rd[a * 64 + lane] = r;
        else if (St.rewards) fjsp::st32(St.rewards, (uint32_t)a * n + ue, r);
    }
    const int nord = E.norders();
    const int all_done = E.ncompleted() == nord && nord > 0 && E.next_order() == nord;
    const int truncated = E.step() >= C.max_steps;
    if (STAGED) {
        rb[fjsp::NMASK * 64 + lane] = (uint8_t)all_done;
        rb[(fjsp::NMASK + 1) * 64 + lane] = (uint8_t)truncated;
        rf[(STG_NF32 - 1) * 64 + lane] = E.status();
    } else {
        if (St.term) fjsp::st32(St.term, ue, (uint8_t)all_done);
        if (St.trunc) fjsp::st32(St.trunc, ue, (uint8_t)truncated);
        if (St.status) fjsp::st32(St.status, ue, E.status());
    }
    E.set_step(E.step() + 1);
    PST(4, __builtin_amdgcn_s_memtime());
    if ((St.flags & STEP_AUTORESET) && (all_done || truncated)) E = fjsp::env_reset_cold(E, T, C, St.S, e, nord);
    PST(5, __builtin_amdgcn_s_memtime());
    if (STAGED) {   // the observation: tile_observe on waves 1 and 2
#pragma unroll
        for (int i = 0; i < fjsp::NSTATE; i++) rf[(fjsp::NFEAT + i) * 64 + lane] = E.w[i];
    } else {
        if (St.next_masks || St.feats) {
            fjsp::StoreSink nsink{nullptr, nullptr, nullptr, St.next_masks, 0u, n, ue, St.feats};
            fjsp::observe(E, C, nsink);
        }
        fjsp::env_store(E, St.S.words, St.S.n, e);
    }
    PST(6, __builtin_amdgcn_s_memtime());
}

// STAGED (every tile full, every output and state row 16-byte aligned): the tail's outputs go
// through the staging rows (tile_copy_out)
template <bool STAGED>
__global__ void __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(4, 4))) k_policy_step(PolicyArgs A, StepArgs St) {
    __shared__ __attribute__((aligned(16))) unsigned char s_mem[LDS_BYTES + STATE_BYTES + LUT_BYTES];
    uint32_t* s_state = reinterpret_cast<uint32_t*>(s_mem + LDS_BYTES);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int b = blockIdx.x;
    PST(0, __builtin_amdgcn_s_memrealtime());
    PST(1, __builtin_amdgcn_s_memtime());
    if (b < A.nc) {
        critic_tile<false>(A, 2 * A.tile0 + b, s_mem, tid, lane, wave, CriticSave{});
        return;
    }
    int role, tile, half = -1;
    if (A.split) {
        // role-major with the pickup station's and the AGV's tiles as two 32-env halves each:
        // pickup h0, pickup h1, AGV h0, AGV h1, then the six stations (a tile's blocks share an XCD)
        const int j = b - A.nc, r = j / A.na;
        tile = j % A.na;
        role = r < 4 ? r >> 1 : r - 2;
        half = r < 4 ? (r & 1) : -1;
    } else {
        actor_block(A, b - A.nc, role, tile);
    }
    PST(13, role);
    tile += A.tile0;
    state_prefetch(St, tile, s_state, lane, wave);   // landed by actor_tile's first barrier
    int act = 0;
    actor_tile(A, role, tile, s_mem, tid, lane, wave, act, half);
    if (wave == 0) {
        const uint32_t a = (uint32_t)act & 0xFFu;
        const int l4 = 4 * (lane & 15);
        const uint32_t w = (uint32_t)__shfl(a, l4) | ((uint32_t)__shfl(a, l4 + 1) << 8) |
                           ((uint32_t)__shfl(a, l4 + 2) << 16) | ((uint32_t)__shfl(a, l4 + 3) << 24);
        // the role's 16 action words (4 envs each); a half stores its 8
        if (lane < (half < 0 ? 16 : 8))
            __hip_atomic_store((gu32*)(St.tile_act) + ((size_t)tile * NAG + role) * 16 + 8 * max(half, 0) + lane, w,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // every wave: its action stores (wave 0) and its state DMAs into LDS have landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // every wave is done with s_mem, the action words are drained
    uint32_t* s_last = reinterpret_cast<uint32_t*>(s_mem + LDS_BYTES - 16);
    if (tid == 0) {
        gu32* cnt = (gu32*)(St.tile_cnt) + tile;
        const uint32_t arrivals = NAG + (A.split ? 2u : 0u);
        const uint32_t last = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == arrivals - 1;
        if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *s_last = last;
    }
    __syncthreads();
    if (!*s_last) return;
    PST(14, __builtin_amdgcn_s_memtime());   // diagnostic builds: the tile's step tail
    if (STAGED) {
        if (wave == 0) tile_step<true>(A, St, tile, s_mem, s_state, lane);
        __syncthreads();                      // the step's staging rows are in
        if (wave == 1 || wave == 2) tile_observe(St, s_mem, s_state, lane, wave);
        __syncthreads();                      // the observation's
        tile_copy_out(St, tile, s_mem, tid);
    } else if (wave == 0) {
        tile_step<false>(A, St, tile, s_mem, s_state, lane);
    }
    PST(15, __builtin_amdgcn_s_memtime());
}

// The critic's forward over n samples for the A2C update (values + the saved hidden layers), on
// sample-major input rows [n][GROW].
__global__ void __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(4, 4)))
k_critic_fwd(PolicyArgs A, CriticSave sv) {
    __shared__ __attribute__((aligned(16))) unsigned char s_mem[LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    critic_tile<true, true>(A, (int)blockIdx.x, s_mem, tid, lane, wave, sv);
}

// The critic's backward through layers 3 and 2 for the A2C update (a2c_vec._CriticGrouped): on a
// tile of 32 samples, g2 = (g3 W3) * [h2 > 0] and g1 = (g2 W2) * [h1 > 0], the input gradients of
// the two 256-wide ReLU layers, with W3^T / W2^T packed like the forward's weights and the
// upstream gradient split into bf16 planes in LDS; g2 and g1 go to HBM (the split-K weight
// gradients read them) with per-tile column sums (the bias gradients).  One pass instead of two
// GEMMs and two ReLU / bias-gradient passes.
struct CriticBwd {
    const float* g3;    // [n][128] layer 3's pre-activation gradient (fjsp_a2c_value_head_grad)
    const float* h1;    // [n][256] post-ReLU hidden layers of the forward
    const float* h2;
    const float* w3t;   // P(W3^T [256][128]), NP * 256 * 128 / 2 floats
    const float* w2t;   // P(W2^T [256][256])
    float* g2;          // [n][256]
    float* g1;
    float* bp2;         // [tiles][256] column sums of g2 / g1 per tile
    float* bp1;
    int n;
};
constexpr int GS3 = 128 + 8;   // bf16 stride of the g3 planes [NP][TC][GS3]
static_assert(NP * TC * GS3 * 2 <= H_BYTES && NP * HPC * 2 <= H_BYTES, "backward planes");
// this lane's 16 values of rows row0.. (C/D layout) at sample column col of a sample-major
// [n][ld] f32 matrix (0 past n)
__device__ __forceinline__ void load_tile_rows(const float* __restrict__ m, int ld, int col, int n, int row0, int lane,
                                               float v[16]) {
#pragma unroll
    for (int g = 0; g < 4; g++) {
        float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
        if (col < n) q = *reinterpret_cast<const float4*>(m + (size_t)col * ld + row0 + 8 * g + 4 * (lane >> 5));
        v[4 * g] = q.x; v[4 * g + 1] = q.y; v[4 * g + 2] = q.z; v[4 * g + 3] = q.w;
    }
}
// g = acc * [h > 0] -> HBM (sample-major [n][256]) and, for the tile's 32 samples, the column
// sums into bp[row] (lanes 0 / 32 after a butterfly over each half-wave)
__device__ __forceinline__ void relu_grad_out(f32x16& acc, const float h[16], float* __restrict__ g, float* __restrict__ bp,
                                              int col, int n, int row0, int lane) {
#pragma unroll
    for (int r = 0; r < 16; r++) acc[r] = h[r] > 0.0f ? acc[r] : 0.0f;
    if (col < n) {
#pragma unroll
        for (int q = 0; q < 4; q++)
            *reinterpret_cast<float4*>(g + (size_t)col * HID + row0 + 8 * q + 4 * (lane >> 5)) =
                make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
    }
    float t[16];
#pragma unroll
    for (int r = 0; r < 16; r++) t[r] = acc[r];   // columns past n are 0 (h loaded as 0)
#pragma unroll
    for (int o = 1; o < 32; o <<= 1)
#pragma unroll
        for (int r = 0; r < 16; r++) t[r] += __shfl_xor(t[r], o);
    if ((lane & 31) == 0) {
#pragma unroll
        for (int q = 0; q < 4; q++)
            *reinterpret_cast<float4*>(bp + row0 + 8 * q + 4 * (lane >> 5)) =
                make_float4(t[4 * q], t[4 * q + 1], t[4 * q + 2], t[4 * q + 3]);
    }
}
// a tile's f32 gradient (rows row0.., the C/D layout) -> bf16 planes [NP][TC][ST] (no ReLU, no bias)
template <int ST, int PL>
__device__ __forceinline__ void store_planes_raw(const f32x16& acc, int k0, __bf16* out, int lane) {
    const int col = lane & 31;
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const int k = k0 + 8 * g + 4 * (lane >> 5);
        bf16x4 ph, pm, pl;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            __bf16 x0, x1, x2;
            split3(acc[4 * g + i], x0, x1, x2);
            ph[i] = x0;
            pm[i] = x1;
            pl[i] = x2;
        }
        *reinterpret_cast<bf16x4*>(out + col * ST + k) = ph;
        *reinterpret_cast<bf16x4*>(out + PL + col * ST + k) = pm;
        *reinterpret_cast<bf16x4*>(out + 2 * PL + col * ST + k) = pl;
    }
}
__global__ void __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(4, 4))) k_critic_bwd(CriticBwd B) {
    __shared__ __attribute__((aligned(16))) __bf16 s_g[H_BYTES / 2];   // g3 planes, then g2 planes
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tile = blockIdx.x, e0 = tile * TC, n = B.n;
    const int col = e0 + (lane & 31);
    const bf16x8* W3T = reinterpret_cast<const bf16x8*>(B.w3t);
    const bf16x8* W2T = reinterpret_cast<const bf16x8*>(B.w2t);
    WRing<8> r3;
    wring_start(r3, wblocks<8, 8>(W3T, wave, 0, lane));
    float hv[16];
    load_tile_rows(B.h2, HID, col, n, 32 * wave, lane, hv);
    // g3 [32 samples][128] -> planes: thread t: sample t / 16, 8 consecutive features
    {
        const int sl = tid >> 4, f0 = (tid & 15) * 8, c = e0 + sl;
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = 0.0f;
        if (c < n) {
            const float4 a = *reinterpret_cast<const float4*>(B.g3 + (size_t)c * 128 + f0);
            const float4 b = *reinterpret_cast<const float4*>(B.g3 + (size_t)c * 128 + f0 + 4);
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
        }
        bf16x8 ph, pm, pl;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            __bf16 x0, x1, x2;
            split3(v[i], x0, x1, x2);
            ph[i] = x0;
            pm[i] = x1;
            pl[i] = x2;
        }
        constexpr int PL3 = TC * GS3;
        *reinterpret_cast<bf16x8*>(s_g + sl * GS3 + f0) = ph;
        *reinterpret_cast<bf16x8*>(s_g + PL3 + sl * GS3 + f0) = pm;
        *reinterpret_cast<bf16x8*>(s_g + 2 * PL3 + sl * GS3 + f0) = pl;
    }
    __syncthreads();
    f32x16 a[1];
    zero_acc<1>(a);
    mfma_rows<8, GS3, TC * GS3, 1>(r3, wblocks<8, 8>(W3T, wave, 0, lane), s_g, 0, lane, a);
    WRing<16> r2;
    wring_start(r2, wblocks<16, 16>(W2T, wave, 0, lane));
    relu_grad_out(a[0], hv, B.g2, B.bp2 + (size_t)tile * HID, col, n, 32 * wave, lane);
    load_tile_rows(B.h1, HID, col, n, 32 * wave, lane, hv);
    __syncthreads();                               // every wave has read the g3 planes
    store_planes_raw<HSC, HPC>(a[0], 32 * wave, s_g, lane);
    __syncthreads();
    zero_acc<1>(a);
    mfma_rows<16, HSC, HPC, 1>(r2, wblocks<16, 16>(W2T, wave, 0, lane), s_g, 0, lane, a);
    relu_grad_out(a[0], hv, B.g1, B.bp1 + (size_t)tile * HID, col, n, 32 * wave, lane);
}

// The grouped update's critic in ONE pass per 32-state tile (fjsp_a2c_critic_fused; a2c.py:683-699,
// 713-722 over the batch's distinct global states, networks.py:41-61).  The critic loss of a batch
// whose distinct state u occurs n_u times is sum_u sum_{samples, agents} (V_u - R)^2 / (8 count), a
// quadratic in V_u: loss_u = a_u / 2 V^2 + b_u V + c_u with a_u = 2 n_u / count, b_u = -2 sum R /
// (8 count), c_u = sum R^2 / (8 count) (coef [n][3], f64, summed per group by the caller), so
// dL / dV_u = a_u V_u + b_u is known as soon as the forward has V_u, and the backward runs in the
// same workgroup: forward as critic_tile (x -> h1 -> h2 -> h3 -> V; the ReLU masks of h1 / h2 kept
// as 16 bits per lane, the C/D positions the backward's g1 / g2 tiles use), then gv (f64), g3 =
// gv w4 [h3 > 0] from layer 3's accumulators, g2 = (g3 W3) [h2 > 0] and g1 = (g2 W2) [h1 > 0] on
// the matrix cores (split-bf16, as k_critic_bwd).  Out: h1, h2, g3, g2, g1 (the split-K weight
// gradients' operands), per tile the bias gradients and w4's / b4's gradients, the loss; nothing
// else is written or re-read (the three-kernel path wrote h3, read it back for the value head and
// read h1 / h2 / g3 again for the backward: 8 KB per state against 4.7 KB here).
struct CriticFused {
    const double* coef;   // [n][3]: a, b, c
    const float* w3t;     // P(W3^T [256][128]), as CriticBwd
    const float* w2t;     // P(W2^T [256][256])
    float* h1;            // [n][256] post-ReLU
    float* h2;
    float* g3;            // [n][128] layer 3's pre-activation gradient
    float* g2;            // [n][256] pre-activation gradients of layers 2 / 1
    float* g1;
    float* part;          // [tiles][FPW]: b1 | b2 | b3 grads, w4 grad [128], b4 grad, 3 zeros
    double* loss;         // [tiles]
    float* values;        // [n] or null
};
constexpr int FPW = 2 * HID + 2 * 128 + 4;
// the column (sample) sums of a lane's 16 rows over the tile's 32 columns -> bp[row] (lanes 0 / 32)
__device__ __forceinline__ void col_sums_out(float t[16], float* __restrict__ bp, int row0, int lane) {
#pragma unroll
    for (int o = 1; o < 32; o <<= 1)
#pragma unroll
        for (int r = 0; r < 16; r++) t[r] += __shfl_xor(t[r], o);
    if ((lane & 31) == 0) {
#pragma unroll
        for (int q = 0; q < 4; q++)
            *reinterpret_cast<float4*>(bp + row0 + 8 * q + 4 * (lane >> 5)) =
                make_float4(t[4 * q], t[4 * q + 1], t[4 * q + 2], t[4 * q + 3]);
    }
}
// acc * mask bits -> HBM rows (sample-major [n][ld]) and the per-tile column sums into bp
__device__ __forceinline__ void masked_grad_out(f32x16& acc, uint32_t bits, float* __restrict__ g, int ld,
                                                float* __restrict__ bp, int col, int n, int row0, int lane) {
#pragma unroll
    for (int r = 0; r < 16; r++) acc[r] = (bits >> r) & 1u ? acc[r] : 0.0f;
    if (col < n) {
#pragma unroll
        for (int q = 0; q < 4; q++)
            *reinterpret_cast<float4*>(g + (size_t)col * ld + row0 + 8 * q + 4 * (lane >> 5)) =
                make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
    }
    float t[16];
#pragma unroll
    for (int r = 0; r < 16; r++) t[r] = acc[r];   // columns past n are 0 (their gv is 0)
    col_sums_out(t, bp, row0, lane);
}
__device__ __forceinline__ uint32_t relu_bits(const f32x16& acc, const Row16& bias) {
    uint32_t m = 0;
#pragma unroll
    for (int r = 0; r < 16; r++) m |= (acc[r] + bias[r] > 0.0f ? 1u : 0u) << r;
    return m;
}
__global__ void __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(4, 4)))
k_critic_fused(PolicyArgs A, CriticFused F) {
    __shared__ __attribute__((aligned(16))) unsigned char s_mem[LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tile = blockIdx.x, n = A.n, e0 = tile * TC;
    const int col = e0 + (lane & 31);
    __bf16* s_x = reinterpret_cast<__bf16*>(s_mem);              // inputs [NP][TC][XSC]
    __bf16* s_h = reinterpret_cast<__bf16*>(s_mem + X_BYTES);    // h1, h2, then g3, g2 planes
    float* s_part = reinterpret_cast<float*>(s_mem);             // value partials [4][TC] (after layer 1)
    float* s_gv = reinterpret_cast<float*>(s_mem + X_BYTES + H_BYTES);   // [TC] dL / dV
    float* part = F.part + (size_t)tile * FPW;
    const float* wb = A.critic_w;
    const bf16x8* W1 = reinterpret_cast<const bf16x8*>(wb);
    const float* B1 = wb + NP * HID * C_DPAD / 2;
    const bf16x8* W2 = reinterpret_cast<const bf16x8*>(B1 + HID);
    const float* B2 = B1 + HID + NP * HID * HID / 2;
    const bf16x8* W3 = reinterpret_cast<const bf16x8*>(B2 + HID);
    const float* B3 = B2 + HID + NP * 128 * HID / 2;
    const float* W4 = B3 + 128;
    const float* B4 = W4 + 128;
    const bf16x8* W3T = reinterpret_cast<const bf16x8*>(F.w3t);
    const bf16x8* W2T = reinterpret_cast<const bf16x8*>(F.w2t);
    // ---- forward (critic_tile<SAVE, ROWS> with the ReLU masks kept)
    float xv[XI];
    inputs_load<TC, C_DPAD, true>(A.feats, n, e0, 0, 38, tid, xv);
    WRing<C_DPAD / 16> r1;
    wring_start(r1, wblocks<C_DPAD / 16, C_DPAD / 16>(W1, wave, 0, lane));
    const Row16 b1 = load_rows(B1, 32 * wave, lane);
    inputs_store<TC, C_DPAD, true>(xv, tid, s_x);
    __syncthreads();
    f32x16 a[1];
    zero_acc<1>(a);
    mfma_rows<C_DPAD / 16, XSC, XPC, 1>(r1, wblocks<C_DPAD / 16, C_DPAD / 16>(W1, wave, 0, lane), s_x, 0, lane, a);
    WRing<HID / 16> r2;
    wring_start(r2, wblocks<HID / 16, HID / 16>(W2, wave, 0, lane));
    const uint32_t m1 = relu_bits(a[0], b1);
    store_planes<HSC, HPC>(a[0], 32 * wave, 0, b1, s_h, lane);
    store_rows_f32(a[0], 32 * wave, b1, F.h1, HID, e0, n, lane);
    const Row16 b2 = load_rows(B2, 32 * wave, lane);
    __syncthreads();
    zero_acc<1>(a);
    mfma_rows<HID / 16, HSC, HPC, 1>(r2, wblocks<HID / 16, HID / 16>(W2, wave, 0, lane), s_h, 0, lane, a);
    const int rt3 = wave & 3;
    WRing<HID / 16> r3;
    wring_start(r3, wblocks<HID / 16, HID / 16>(W3, rt3, 0, lane));
    const Row16 b3 = load_rows(B3, 32 * rt3, lane), w4 = load_rows(W4, 32 * rt3, lane);
    const uint32_t m2 = relu_bits(a[0], b2);
    __syncthreads();                               // every wave has read h1
    store_planes<HSC, HPC>(a[0], 32 * wave, 0, b2, s_h, lane);
    store_rows_f32(a[0], 32 * wave, b2, F.h2, HID, e0, n, lane);
    __syncthreads();
    if (wave < 4) {
        zero_acc<1>(a);
        mfma_rows<HID / 16, HSC, HPC, 1>(r3, wblocks<HID / 16, HID / 16>(W3, rt3, 0, lane), s_h, 0, lane, a);
        float v = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; r++) v = fmaf(w4[r], relu(a[0][r] + b3[r]), v);
        v += __shfl_xor(v, 32);
        if (lane < 32) s_part[wave * TC + lane] = v;
    }
    WRing<8> rb3;
    wring_start(rb3, wblocks<8, 8>(W3T, wave, 0, lane));
    __syncthreads();                               // value partials in; layer 3 done with the h2 planes
    // ---- the value, its gradient and the loss (one lane per state)
    if (wave == 0) {
        double lt = 0.0;
        float gv = 0.0f, vg = 0.0f;
        if (lane < TC && e0 + lane < n) {
            float val = B4[0];
#pragma unroll
            for (int w = 0; w < 4; w++) val += s_part[w * TC + lane];
            const double* c = F.coef + (size_t)(e0 + lane) * 3;
            const double v64 = (double)val;
            gv = (float)(c[0] * v64 + c[1]);
            lt = (0.5 * c[0] * v64 + c[1]) * v64 + c[2];
            vg = gv;
            if (F.values) F.values[e0 + lane] = val;
        }
        if (lane < TC) s_gv[lane] = gv;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            lt += __shfl_xor(lt, o);
            vg += __shfl_xor(vg, o);
        }
        if (lane == 0) {
            F.loss[tile] = lt;
            *reinterpret_cast<float4*>(part + 2 * HID + 2 * 128) = make_float4(vg, 0.f, 0.f, 0.f);
        }
    }
    __syncthreads();
    // ---- value head backward (waves 0..3: layer 3's accumulators): g3 = gv w4 [h3 > 0], w4's
    // gradient sum gv h3, b3's sum g3; g3 -> HBM and -> bf16 planes for g2
    constexpr int PL3 = TC * GS3;
    if (wave < 4) {
        const float gv = s_gv[lane & 31];
        float tw[16], tb[16];
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const float h = relu(a[0][r] + b3[r]);
            tw[r] = gv * h;
            a[0][r] = h > 0.0f ? gv * w4[r] : 0.0f;
            tb[r] = a[0][r];
        }
        if (col < n) {
#pragma unroll
            for (int q = 0; q < 4; q++)
                *reinterpret_cast<float4*>(F.g3 + (size_t)col * 128 + 32 * rt3 + 8 * q + 4 * (lane >> 5)) =
                    make_float4(a[0][4 * q], a[0][4 * q + 1], a[0][4 * q + 2], a[0][4 * q + 3]);
        }
        store_planes_raw<GS3, PL3>(a[0], 32 * rt3, s_h, lane);
        col_sums_out(tb, part + 2 * HID, 32 * rt3, lane);
        col_sums_out(tw, part + 2 * HID + 128, 32 * rt3, lane);
    }
    __syncthreads();
    // ---- g2 = (g3 W3) [h2 > 0], g1 = (g2 W2) [h1 > 0] (k_critic_bwd's products)
    zero_acc<1>(a);
    mfma_rows<8, GS3, PL3, 1>(rb3, wblocks<8, 8>(W3T, wave, 0, lane), s_h, 0, lane, a);
    WRing<16> rb2;
    wring_start(rb2, wblocks<16, 16>(W2T, wave, 0, lane));
    masked_grad_out(a[0], m2, F.g2, HID, part + HID, col, n, 32 * wave, lane);
    __syncthreads();                               // every wave has read the g3 planes
    store_planes_raw<HSC, HPC>(a[0], 32 * wave, s_h, lane);
    __syncthreads();
    zero_acc<1>(a);
    mfma_rows<16, HSC, HPC, 1>(rb2, wblocks<16, 16>(W2T, wave, 0, lane), s_h, 0, lane, a);
    masked_grad_out(a[0], m1, F.g1, HID, part, col, n, 32 * wave, lane);
}

// The critic's weight gradients gW = G^T X over the batch's distinct states (r06; the backward of
// networks.CentralizedCriticNetwork's Linear layers, a2c.py:683-699): G f32 [U][M] (k_critic_fused's
// g1 / g2 / g3, sample-major), X f32 [U][nx] (x / h1 / h2) -> gW [M][nx].  The contraction runs over
// the samples, so both MFMA operands need 8 consecutive SAMPLES of one feature per lane while the
// rows hold consecutive features.  Each workgroup owns a contiguous run of 16-sample stages
// (split-K) and its whole [M][NPAD] output in the accumulators of its 8 waves (TM x TN 32 x 32 tiles
// each).  Per stage, waves 0-3 load the G tile and waves 4-7 the X tile (4 samples x 4 features per
// lane, 128-byte row segments; one stage ahead into registers), split them into the three bf16
// planes and write them TRANSPOSED into LDS images [plane][feature][16 samples] (48-byte rows: the
// fragment reads of every ds_read_b128 lane group hit distinct banks); the images are double
// buffered, so the split and the stores of stage s + 1 run beside the MFMAs of stage s with one
// barrier per stage.  Six plane products per 16-deep block (mfma6: f32-level products, as the
// forward).  The per-workgroup partials are summed in a fixed order (k_wgrad_reduce, f64):
// deterministic.  Replaces three split-K hipBLASLt f32 GEMMs with both operands' K strided.
constexpr int WG_KS = 16;                  // samples per stage: one 16-deep block
constexpr int WG_ROW = 24;                 // bf16 per LDS image row (16 samples + 8 of padding)
constexpr int WG_MAXD = 4;                 // the deepest load pipeline of the k_wgrad instances
constexpr int WG_VPM = 2;                  // split VALU per MFMA in the interleave
int g_wgrad_waves = 16;                    // k_wgrad16 (16) or k_wgrad (8 waves): library-wide option "wgrad_waves"
// one stage of F features (F % 4 == 0, F <= 256) -> registers: lane t (0..255 of its wave half)
// holds the 4 x 4 block (samples 4 (t & 3) .., features 4 (t >> 2) ..).  Buffer loads through a
// descriptor over the rows from the workgroup's first stage on; the lane's offsets within a stage
// are fixed for the launch.  Rows past U (outside the descriptor) and features past F (an offset
// outside it) load zeros.  (64-bit per-lane address arithmetic for plain loads, and loads under a
// branch, made the compiler wait for every load in flight at each stage.)
struct WgSrc {
    __amdgpu_buffer_rsrc_t rsrc;
    int voff[4];
};
__device__ __forceinline__ WgSrc wg_src(const float* src, int64_t ld, int F, int64_t r0, int64_t U, int t) {
    WgSrc w;
    const int64_t rem = (U - r0) * ld * 4;
    const int bytes = rem <= 0 ? 0 : rem > 0x7FFFFF00ll ? 0x7FFFFF00 : (int)rem;
    w.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src + r0 * ld), (short)0, bytes, 0x00020000);
    const int sq = t & 3, fq = t >> 2;
#pragma unroll
    for (int i = 0; i < 4; i++) w.voff[i] = 4 * fq < F ? (int)(((4 * sq + i) * ld + 4 * fq) * 4) : 0x7FFFFFF0;
    return w;
}
// off: the stage's byte offset, added in the lane offsets (the descriptor's range check then sees it)
__device__ __forceinline__ void wg_load(const WgSrc& w, int off, float4 (&v)[4]) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const auto r = __builtin_amdgcn_raw_buffer_load_b128(w.rsrc, (int)((unsigned)w.voff[i] + (unsigned)off), 0, 0);
        v[i] = make_float4(__uint_as_float(r[0]), __uint_as_float(r[1]), __uint_as_float(r[2]), __uint_as_float(r[3]));
    }
}
__device__ __forceinline__ float f4c(const float4& v, int c) { return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w; }
// the block's planes into an image [NP][256 rows][WG_ROW]: per feature 4 samples = 8 bytes per
// plane.  Every lane stores (lanes past F store the zeros they loaded: the image rows past F are
// zero), so the stores and the MFMAs share one basic block and interleave
__device__ __forceinline__ void wg_store(const float4 (&v)[4], int t, __bf16* s) {
    constexpr int plane = 256 * WG_ROW;
    const int sq = t & 3, fq = t >> 2;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        bf16x4 ph, pm, pl;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            __bf16 x0, x1, x2;
            split3(f4c(v[i], c), x0, x1, x2);
            ph[i] = x0;
            pm[i] = x1;
            pl[i] = x2;
        }
        const int o = (4 * fq + c) * WG_ROW + 4 * sq;
        *reinterpret_cast<bf16x4*>(s + o) = ph;
        *reinterpret_cast<bf16x4*>(s + plane + o) = pm;
        *reinterpret_cast<bf16x4*>(s + 2 * plane + o) = pl;
    }
}
// D: stages in flight per lane (register sets; the loads of stage j + D are issued when stage j + 1
// is stored, so D - 1 stages of loads wait under the MFMAs; one stage in flight left the kernel
// latency-bound at ~2 TB/s)
template <int M, int NPAD, int TM, int TN, int D>
__global__ void __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_wgrad(const float* __restrict__ g, int64_t ldg, const float* __restrict__ x, int64_t ldx, int nx, int64_t U,
        float* __restrict__ part) {
    static_assert((M / 32 / TM) * (NPAD / 32 / TN) == NWAVE, "one tile group per wave");
    constexpr int PL = 256 * WG_ROW;                     // plane size (bf16): 256 rows, whatever M / nx
    constexpr int BUF = 2 * NP * PL;                     // one stage's two images (G, X)
    __shared__ __attribute__((aligned(16))) __bf16 s_img[2 * BUF];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool ldr_g = wave < 4;                         // this wave's share of the loads: G or X
    const int t = tid & 255;
    constexpr int WN = NPAD / 32 / TN;
    const int mb0 = (wave / WN) * TM, nb0 = (wave % WN) * TN;
    // this workgroup's stages b, b + P, b + 2P, ...: at any time the workgroups stream one window of
    // rows (contiguous runs per workgroup measured the same)
    const int64_t stages = (U + WG_KS - 1) / WG_KS, P = gridDim.x, b = blockIdx.x;
    const int nj = stages > b ? (int)((stages - b + P - 1) / P) : 0;
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] = 0.0f;
    const int64_t ld = ldr_g ? ldg : ldx;
    const int img = ldr_g ? 0 : NP * PL;
    const WgSrc ws = wg_src(ldr_g ? g : x, ld, ldr_g ? M : nx, b * WG_KS, U, t);
    const int sstride = (int)(P * WG_KS * ld * 4);  // bytes from one of this workgroup's stages to the next
    float4 v[D][4];   // register set k holds the stages j = k (mod D)
    if (nj > 0) {
        // loads are unconditional (past the last stage they read zeros): a conditional load's
        // register merge made the compiler wait for it at once
#pragma unroll
        for (int k = 0; k < D; k++) wg_load(ws, k * sstride, v[k]);
        wg_store(v[0], t, s_img + img);
        wg_load(ws, D * sstride, v[0]);
    }
    __syncthreads();
    const int h = lane >> 5, r32 = lane & 31;
    for (int jb = 0; jb < nj; jb += D) {
#pragma unroll
        for (int d = 0; d < D; d++) {
            const int j = jb + d;
            if (j >= nj) break;
            const __bf16* cg = s_img + (j & 1) * BUF;
            const __bf16* cx = cg + NP * PL;
            bf16x8 a[TM][NP];
#pragma unroll
            for (int i = 0; i < TM; i++) {
                const int o = (32 * (mb0 + i) + r32) * WG_ROW + 8 * h;
#pragma unroll
                for (int p = 0; p < NP; p++) a[i][p] = *reinterpret_cast<const bf16x8*>(cg + p * PL + o);
            }
#pragma unroll
            for (int jj = 0; jj < TN; jj++) {
                bf16x8 bb[NP];
                const int o = (32 * (nb0 + jj) + r32) * WG_ROW + 8 * h;
#pragma unroll
                for (int p = 0; p < NP; p++) bb[p] = *reinterpret_cast<const bf16x8*>(cx + p * PL + o);
#pragma unroll
                for (int i = 0; i < TM; i++) acc[i][jj] = mfma6(a[i], bb, acc[i][jj]);
            }
            // stage j + 1 into the other buffer (past the last stage: zeros nobody reads), stage
            // j + 1 + D's loads out, the split and stores interleaved with this stage's MFMAs
            const int k = (d + 1) % D;
            wg_store(v[k], t, s_img + ((j + 1) & 1) * BUF + img);
            wg_load(ws, (j + 1 + D) * sstride, v[k]);
#pragma unroll
            for (int q = 0; q < TM * TN * 6; q++) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);          // one MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, WG_VPM, 0);     // VALU of the split
                if (q % 4 == 3) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);   // an LDS store
            }
            __syncthreads();
        }
    }
    // the partial [M][NPAD] of this workgroup: C/D row (r & 3) + 8 (r >> 2) + 4 h, column lane & 31
    float* pp = part + (size_t)blockIdx.x * M * NPAD;
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++)
                pp[(size_t)(32 * (mb0 + i) + (r & 3) + 8 * (r >> 2) + 4 * h) * NPAD + 32 * (nb0 + j) + r32] = acc[i][j][r];
}
// k_wgrad on 16 waves (the default; 4 per SIMD, 128 registers each): every wave loads (waves 0-7
// the G tile, 8-15 the X tile, 2 samples x 4 features per lane), holds TM x TN accumulator tiles and
// runs its A fragments one row tile at a time; more waves per SIMD hide the loads, the split and
// the stage barrier behind each other's MFMAs (the 8-wave kernel's W2 instance left the matrix
// cores 63 % idle): W2 / W3 / W1 0.35 / 0.215 / 0.157 against 0.40 / 0.24 / 0.18 ms at 540 k
// states, bit-identical (the same products per accumulator in the same order); W2 on 1 x 4 tiles
// per wave (fewer fragment reads and registers): 0.38 against 0.47 ms for 2 x 2 on dense random
// operands, equal (0.35) on the update's half-zero gradients.
__device__ __forceinline__ void wg_load2(const WgSrc& w, int off, float4 (&v)[2]) {
#pragma unroll
    for (int i = 0; i < 2; i++) {
        const auto r = __builtin_amdgcn_raw_buffer_load_b128(w.rsrc, (int)((unsigned)w.voff[i] + (unsigned)off), 0, 0);
        v[i] = make_float4(__uint_as_float(r[0]), __uint_as_float(r[1]), __uint_as_float(r[2]), __uint_as_float(r[3]));
    }
}
__device__ __forceinline__ WgSrc wg_src2(const float* src, int64_t ld, int F, int64_t r0, int64_t U, int t) {
    WgSrc w;
    const int64_t rem = (U - r0) * ld * 4;
    const int bytes = rem <= 0 ? 0 : rem > 0x7FFFFF00ll ? 0x7FFFFF00 : (int)rem;
    w.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src + r0 * ld), (short)0, bytes, 0x00020000);
    const int sp = t & 7, fq = t >> 3;   // samples 2 sp, 2 sp + 1; features 4 fq ..
#pragma unroll
    for (int i = 0; i < 2; i++) w.voff[i] = 4 * fq < F ? (int)(((2 * sp + i) * ld + 4 * fq) * 4) : 0x7FFFFFF0;
    w.voff[2] = w.voff[3] = 0;
    return w;
}
__device__ __forceinline__ void wg_store2(const float4 (&v)[2], int t, __bf16* s) {
    constexpr int plane = 256 * WG_ROW;
    const int sp = t & 7, fq = t >> 3;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        __bf16 h0, m0, l0, h1, m1, l1;
        split3(f4c(v[0], c), h0, m0, l0);
        split3(f4c(v[1], c), h1, m1, l1);
        typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
        const int o = (4 * fq + c) * WG_ROW + 2 * sp;
        *reinterpret_cast<bf16x2*>(s + o) = bf16x2{h0, h1};
        *reinterpret_cast<bf16x2*>(s + plane + o) = bf16x2{m0, m1};
        *reinterpret_cast<bf16x2*>(s + 2 * plane + o) = bf16x2{l0, l1};
    }
}
template <int M, int NPAD, int TM, int TN, int D>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4, 4)))
k_wgrad16(const float* __restrict__ g, int64_t ldg, const float* __restrict__ x, int64_t ldx, int nx, int64_t U,
          float* __restrict__ part) {
    static_assert((M / 32 / TM) * (NPAD / 32 / TN) == 16, "one tile group per wave");
    constexpr int WN = NPAD / 32 / TN;
    constexpr int PL = 256 * WG_ROW, BUF = 2 * NP * PL;
    __shared__ __attribute__((aligned(16))) __bf16 s_img[2 * BUF];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool ldr_g = wave < 8;
    const int t = tid & 511;
    const int mb0 = (wave / WN) * TM, nb0 = (wave % WN) * TN;
    const int64_t stages = (U + WG_KS - 1) / WG_KS, P = gridDim.x, b = blockIdx.x;
    const int nj = stages > b ? (int)((stages - b + P - 1) / P) : 0;
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] = 0.0f;
    const int64_t ld = ldr_g ? ldg : ldx;
    const int img = ldr_g ? 0 : NP * PL;
    const WgSrc ws = wg_src2(ldr_g ? g : x, ld, ldr_g ? M : nx, b * WG_KS, U, t);
    const int sstride = (int)(P * WG_KS * ld * 4);
    float4 v[D][2];
    if (nj > 0) {
#pragma unroll
        for (int k = 0; k < D; k++) wg_load2(ws, k * sstride, v[k]);
        wg_store2(v[0], t, s_img + img);
        wg_load2(ws, D * sstride, v[0]);
    }
    __syncthreads();
    const int h = lane >> 5, r32 = lane & 31;
    for (int jb = 0; jb < nj; jb += D) {
#pragma unroll
        for (int d = 0; d < D; d++) {
            const int j = jb + d;
            if (j >= nj) break;
            const __bf16* cg = s_img + (j & 1) * BUF;
            const __bf16* cx = cg + NP * PL;
#pragma unroll
            for (int i = 0; i < TM; i++) {
                bf16x8 a[NP];
                const int oa = (32 * (mb0 + i) + r32) * WG_ROW + 8 * h;
#pragma unroll
                for (int p = 0; p < NP; p++) a[p] = *reinterpret_cast<const bf16x8*>(cg + p * PL + oa);
#pragma unroll
                for (int jj = 0; jj < TN; jj++) {
                    bf16x8 bb[NP];
                    const int o = (32 * (nb0 + jj) + r32) * WG_ROW + 8 * h;
#pragma unroll
                    for (int p = 0; p < NP; p++) bb[p] = *reinterpret_cast<const bf16x8*>(cx + p * PL + o);
                    acc[i][jj] = mfma6(a, bb, acc[i][jj]);
                }
            }
            const int k = (d + 1) % D;
            wg_store2(v[k], t, s_img + ((j + 1) & 1) * BUF + img);
            wg_load2(ws, (j + 1 + D) * sstride, v[k]);
            __syncthreads();
        }
    }
    float* pp = part + (size_t)blockIdx.x * M * NPAD;
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++)
                pp[(size_t)(32 * (mb0 + i) + (r & 3) + 8 * (r >> 2) + 4 * h) * NPAD + 32 * (nb0 + j) + r32] = acc[i][j][r];
}
// out [M][ldo] (columns < nout) = the sum of the P partials in partial order, in f64
__global__ void __launch_bounds__(256) k_wgrad_reduce(const float* __restrict__ part, int P, int M, int npad, int nout,
                                                      float* __restrict__ out, int64_t ldo) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= M * nout) return;
    const int m = i / nout, c = i - m * nout;
    const float* p = part + (size_t)m * npad + c;
    const size_t stride = (size_t)M * npad;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int q = 0;
    for (; q + 4 <= P; q += 4) {
        s0 += p[(size_t)q * stride];
        s1 += p[(size_t)(q + 1) * stride];
        s2 += p[(size_t)(q + 2) * stride];
        s3 += p[(size_t)(q + 3) * stride];
    }
    for (; q < P; q++) s0 += p[(size_t)q * stride];
    out[(size_t)m * ldo + c] = (float)((s0 + s1) + (s2 + s3));
}

// Keys of the A2C update's grouping of repeated inputs (a2c_vec.row_keys, the same hash): per
// sample s = t * n + e of feats f32 [T][38][n], key a < 8 over actor a's 13 padded input columns
// (its OBS_DIMS[a] a2c features, then zeros), key 8 over all 38; k = fmix64(k * MUL + bits(x_c)
// + c + 1) from k = 0.  One lane per sample, each column a coalesced load.  rows (may be null):
// the sample's 38 features also as a sample-major row [S][GROW] (zero-padded), what the grouping
// check compares and the update's critic reads.
constexpr uint64_t GK_MUL = 0x100000001B3ull * 0x9E37ull + 1ull;
__device__ __forceinline__ uint64_t gk_fmix(uint64_t z) {
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ void __launch_bounds__(256) k_group_keys(const float* __restrict__ feats, int T, int n,
                                                    uint64_t* __restrict__ keys, float* __restrict__ rows) {
    const size_t S = (size_t)T * n;
    const size_t s = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= S) return;
    const size_t t = s / (size_t)n, e = s - t * (size_t)n;
    const float* x = feats + t * 38 * (size_t)n + e;
    constexpr int offs[NAG + 1] = {0, 7, 20, 23, 26, 29, 32, 35, 38};
    uint64_t kc = 0;
    uint64_t ka[NAG];
#pragma unroll
    for (int a = 0; a < NAG; a++) ka[a] = 0;
    float xv[GROW];
#pragma unroll
    for (int c = 0; c < GROW; c++) xv[c] = c < 38 ? x[(size_t)c * n] : 0.0f;
#pragma unroll
    for (int c = 0; c < 38; c++) {
        const uint64_t b = (uint64_t)__float_as_uint(xv[c]);
        kc = gk_fmix(kc * GK_MUL + b + (uint64_t)(c + 1));
#pragma unroll
        for (int a = 0; a < NAG; a++)
            if (c >= offs[a] && c < offs[a + 1]) ka[a] = gk_fmix(ka[a] * GK_MUL + b + (uint64_t)(c - offs[a] + 1));
    }
#pragma unroll
    for (int a = 0; a < NAG; a++) {   // the zero padding up to 13 columns
#pragma unroll
        for (int c = offs[a + 1] - offs[a]; c < 13; c++) ka[a] = gk_fmix(ka[a] * GK_MUL + (uint64_t)(c + 1));
        keys[(size_t)a * S + s] = ka[a];
    }
    keys[(size_t)NAG * S + s] = kc;
    if (rows) {
        float4* r = reinterpret_cast<float4*>(rows + s * GROW);
#pragma unroll
        for (int q = 0; q < GROW / 4; q++) r[q] = make_float4(xv[4 * q], xv[4 * q + 1], xv[4 * q + 2], xv[4 * q + 3]);
    }
}

// Weights into the matrix cores' operand order (a2c_vec.pack_mfma, include/fjsp.h): W f32 [B][R][K]
// (or, transposed, the K x R source [B][K][R] read as its transpose) -> [B][R/32][K/16][3][64][8]
// bf16, element (b, t, kb, p, l, j) = plane p of split3(W[b][32 t + (l & 31)][16 kb + 8 (l >> 5)
// + j]).  One thread per (b, t, kb, l, 4 consecutive j): reads 4 values, writes 4 bf16 of each
// plane.  Replaces ~9 elementwise / stack / permute launches per matrix after every update.
__global__ void __launch_bounds__(256) k_pack_mfma(const float* __restrict__ W, int B, int R, int K, int tr,
                                                   __bf16* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int KB = K / 16, RT = R / 32;
    const int64_t total = (int64_t)B * RT * KB * 64 * 2;
    if (i >= total) return;
    const int q = (int)(i & 1);                       // j half: 4 q .. 4 q + 3
    const int l = (int)((i >> 1) & 63);
    int64_t rest = i >> 7;
    const int kb = (int)(rest % KB);
    rest /= KB;
    const int t = (int)(rest % RT);
    const int b = (int)(rest / RT);
    const int row = 32 * t + (l & 31), k0 = 16 * kb + 8 * (l >> 5) + 4 * q;
    const float* src = W + (size_t)b * R * K;
    bf16x4 ph, pm, pl;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const float v = tr ? src[(size_t)(k0 + j) * R + row] : src[(size_t)row * K + k0 + j];
        __bf16 x0, x1, x2;
        split3(v, x0, x1, x2);
        ph[j] = x0;
        pm[j] = x1;
        pl[j] = x2;
    }
    // [b][t][kb][p][l][j]: plane stride 64 * 8 bf16
    __bf16* o = out + ((((size_t)b * RT + t) * KB + kb) * NP * 64 + l) * 8 + 4 * q;
    *reinterpret_cast<bf16x4*>(o) = ph;
    *reinterpret_cast<bf16x4*>(o + 64 * 8) = pm;
    *reinterpret_cast<bf16x4*>(o + 2 * 64 * 8) = pl;
}

// The shard learner's combiner keys (shard_learner.combine): per (agent a, sample s = t n + e)
// info = the agent's mask bits | action << 8 and the record key fmix64(key_a ^ fmix64(info * MIX +
// 1)) over the actor input key of fjsp_a2c_group_keys (the same wrapping 64-bit arithmetic as
// a2c_vec._fmix64), so that samples with equal (input, mask, action) share a key; bad[block] = 1
// where a mask byte is neither 0 nor 1 (the bits would not carry it).
__global__ void __launch_bounds__(256) k_shard_keys(const uint64_t* __restrict__ keys, const int8_t* __restrict__ masks,
                                                    const uint8_t* __restrict__ actions, int T, int n,
                                                    uint64_t* __restrict__ tk, int32_t* __restrict__ info,
                                                    int32_t* __restrict__ bad) {
    const size_t S = (size_t)T * n;
    const size_t s = (size_t)blockIdx.x * 256 + threadIdx.x;
    int nb = 0;
    if (s < S) {
        const size_t t = s / (size_t)n, e = s - t * (size_t)n;
        uint32_t bits = 0;
        for (int c = 0; c < 29; c++) {
            const int m = masks[(t * 29 + c) * (size_t)n + e];
            bits |= (uint32_t)(m != 0) << c;
            nb |= m != 0 && m != 1;
        }
#pragma unroll
        for (int a = 0; a < NAG; a++) {
            const uint32_t ab = (bits >> c_mask_off[a]) & ((1u << c_nact[a]) - 1u);
            const uint32_t w = ab | ((uint32_t)actions[(t * NAG + a) * (size_t)n + e] << 8);
            info[(size_t)a * S + s] = (int32_t)w;
            tk[(size_t)a * S + s] = gk_fmix(keys[(size_t)a * S + s] ^ gk_fmix((uint64_t)w * 0x9E3779B97F4A7C15ull + 1ull));
        }
    }
    if (__syncthreads_or(nb) && threadIdx.x == 0) bad[blockIdx.x] = 1;
}

// The actor loss head of the grouped A2C update for one (agent, sample): the reference's
// entropy, masked renormalisation / uniform fallback, Categorical log-prob and actor loss
// (a2c.py:204-220, 705-731; a2c_vec.A2CLosses) and its gradient with respect to the sample's
// eight probabilities, which are read from the agent's distinct-input outputs through inv.
// L = sum over agents of -(sum adv_n logp) / count - c (sum entropy) / count; per (a, s):
//   grad[mask_off[a] + j][s] = dL / dp_j for the agent's valid actions j < nact[a] (29 rows: a
//   padded action's probability is an exact 0 out of the softmax, its gradient is never used);
//   sums[a][block] = the workgroup's (adv_n logp, entropy) sums.
__global__ void __launch_bounds__(256) k_actor_head(const float* __restrict__ pu, int umax,
                                                    const int64_t* __restrict__ inv, int T, int n,
                                                    const int8_t* __restrict__ masks,
                                                    const uint8_t* __restrict__ actions,
                                                    const double* __restrict__ advs, const float* __restrict__ adv_mean,
                                                    const float* __restrict__ adv_std, float inv_count, float ent_coef,
                                                    float* __restrict__ grad, double* __restrict__ sums) {
    const int a = blockIdx.y;
    const size_t S = (size_t)T * n;
    const size_t s = (size_t)blockIdx.x * 256 + threadIdx.x;
    double sl = 0.0, se = 0.0;
    if (s < S) {
        const size_t t = s / (size_t)n, e = s - t * (size_t)n;
        const size_t u = (size_t)inv[(size_t)a * S + s];
        const int na = c_nact[a], mo = c_mask_off[a];
        // the rollout slab's layout [T][8][n]: actions u8, GAE advantages f64, normalised here as
        // calc_actor_loss does on FloatTensor(adv) (a2c.py:724-731): (adv - mean) / (std + 1e-8)
        const size_t ta = (t * NAG + (size_t)a) * (size_t)n + e;
        const int act = (int)actions[ta];
        const float adv = adv_std ? ((float)advs[ta] - adv_mean[a]) / (adv_std[a] + 1e-8f) : (float)advs[ta];
        float p[8], m[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            p[j] = pu[((size_t)a * 8 + j) * umax + u];
            m[j] = j < na ? (float)masks[(t * 29 + mo + j) * n + e] : 0.0f;
        }
        // entropy and its gradient
        float ent = 0.0f, g[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const float pe = p[j] + 1e-10f;
            ent += p[j] * logf(pe);
            g[j] = -ent_coef * inv_count * -(logf(pe) + p[j] / pe);
        }
        ent = -ent;
        // masked probabilities: p m / sum(p m), or m / sum(m) when nothing valid is left
        float sr = 0.0f, sm = 0.0f, pm[8];
#pragma unroll
        for (int j = 0; j < 8; j++) { sr += p[j] * m[j]; sm += m[j]; }
#pragma unroll
        for (int j = 0; j < 8; j++) pm[j] = sr > 0.0f ? (p[j] * m[j]) / sr : m[j] / sm;
        float s2 = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; j++) s2 += pm[j];
        float qa = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; j++) qa = j == act ? pm[j] / s2 : qa;
        const float eps = 1.1920928955078125e-07f;
        const float qc = fminf(fmaxf(qa, eps), 1.0f - eps);
        const float logp = logf(qc);
        // d L / d logp = -adv / count; through clamp (inclusive), q = pm / s2, pm = p m / sr
        const float gq = (qa >= eps && qa <= 1.0f - eps) ? (-adv * inv_count) / qc : 0.0f;
        if (sr > 0.0f) {
            float gpm[8], dot = 0.0f;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                gpm[j] = (j == act ? gq / s2 : 0.0f) - gq * qa / s2;   // d q_act / d pm_j
                dot += gpm[j] * (p[j] * m[j]);
            }
#pragma unroll
            for (int j = 0; j < 8; j++) g[j] += m[j] * (gpm[j] / sr - dot / (sr * sr));
        }
#pragma unroll
        for (int j = 0; j < 8; j++)
            if (j < na) grad[(size_t)(mo + j) * S + s] = g[j];   // valid actions only (rows mo..mo+na)
        sl = (double)(adv * logp);
        se = (double)ent;
    }
    // the workgroup's sums, one partial pair per workgroup (no atomics: ~16 000 workgroups per
    // agent adding into one address serialise)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        sl += __shfl_xor(sl, off);
        se += __shfl_xor(se, off);
    }
    __shared__ double s_part[4][2];
    if ((threadIdx.x & 63) == 0) { s_part[threadIdx.x >> 6][0] = sl; s_part[threadIdx.x >> 6][1] = se; }
    __syncthreads();
    if (threadIdx.x < 2) {
        const double v = s_part[0][threadIdx.x] + s_part[1][threadIdx.x] + s_part[2][threadIdx.x] + s_part[3][threadIdx.x];
        sums[((size_t)a * gridDim.x + blockIdx.x) * 2 + threadIdx.x] = v;
    }
}

// The shard learner's actor loss head over an owner's records (shard_learner.owner_losses): a
// record stands for n samples of one agent with equal (input, mask, action) and carries w = the
// f64 sum of their normalised advantages; the samples' loss terms and gradients are linear in the
// advantage and share everything else, so per record: -(w logp) / count - c n entropy / count, and
// grad[j][r] = dL / dp_j of the record (k_actor_head's formulas with adv -> w and the entropy
// weighted by n).  pu [8][umax] = the agent's probabilities per distinct input, inv [R] = each
// record's input group; info [R] = mask bits | action << 8.
__global__ void __launch_bounds__(256) k_record_head(const float* __restrict__ pu, int umax,
                                                     const int64_t* __restrict__ inv, int R, int na,
                                                     const int32_t* __restrict__ info, const double* __restrict__ wsum,
                                                     const int32_t* __restrict__ cnt, float inv_count, float ent_coef,
                                                     float* __restrict__ grad, double* __restrict__ sums) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    double sl = 0.0, se = 0.0;
    if (r < R) {
        const size_t u = (size_t)inv[r];
        const uint32_t w0 = (uint32_t)info[r];
        const int act = (int)((w0 >> 8) & 0xFFu);
        const float adv = (float)wsum[r];
        const float nr = (float)cnt[r];
        float p[8], m[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            p[j] = pu[(size_t)j * umax + u];
            m[j] = j < na ? (float)((w0 >> j) & 1u) : 0.0f;
        }
        float ent = 0.0f, g[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const float pe = p[j] + 1e-10f;
            ent += p[j] * logf(pe);
            g[j] = -ent_coef * inv_count * nr * -(logf(pe) + p[j] / pe);
        }
        ent = -ent;
        float sr = 0.0f, sm = 0.0f, pm[8];
#pragma unroll
        for (int j = 0; j < 8; j++) { sr += p[j] * m[j]; sm += m[j]; }
#pragma unroll
        for (int j = 0; j < 8; j++) pm[j] = sr > 0.0f ? (p[j] * m[j]) / sr : m[j] / sm;
        float s2 = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; j++) s2 += pm[j];
        float qa = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; j++) qa = j == act ? pm[j] / s2 : qa;
        const float eps = 1.1920928955078125e-07f;
        const float qc = fminf(fmaxf(qa, eps), 1.0f - eps);
        const float logp = logf(qc);
        const float gq = (qa >= eps && qa <= 1.0f - eps) ? (-adv * inv_count) / qc : 0.0f;
        if (sr > 0.0f) {
            float gpm[8], dot = 0.0f;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                gpm[j] = (j == act ? gq / s2 : 0.0f) - gq * qa / s2;
                dot += gpm[j] * (p[j] * m[j]);
            }
#pragma unroll
            for (int j = 0; j < 8; j++) g[j] += m[j] * (gpm[j] / sr - dot / (sr * sr));
        }
#pragma unroll
        for (int j = 0; j < 8; j++)
            if (j < na) grad[(size_t)j * R + r] = g[j];
        sl = (double)adv * (double)logp;
        se = (double)nr * (double)ent;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        sl += __shfl_xor(sl, off);
        se += __shfl_xor(se, off);
    }
    __shared__ double s_part[4][2];
    if ((threadIdx.x & 63) == 0) { s_part[threadIdx.x >> 6][0] = sl; s_part[threadIdx.x >> 6][1] = se; }
    __syncthreads();
    if (threadIdx.x < 2)
        sums[(size_t)blockIdx.x * 2 + threadIdx.x] =
            s_part[0][threadIdx.x] + s_part[1][threadIdx.x] + s_part[2][threadIdx.x] + s_part[3][threadIdx.x];
}

// The grouping check of the A2C update (a2c_vec.A2CLosses, replaces the torch gather-and-compare
// of every input with its group's representative): sample s is bad when any of actor a's input
// columns differs bitwise from those of rep_a[a][s], or any of its 38 global-state columns from
// those of rep_c[s] (a hash collision merged two different inputs).  Samples that represent
// their own group are skipped.  The inputs are read from the sample-major rows k_group_keys
// wrote (a representative's features are one 160-byte row, not 38 scattered words of the
// feature-major slab).  bad[block] = 1 if any sample of the workgroup is bad, else 0.
__global__ void __launch_bounds__(256) k_group_verify(const float* __restrict__ rows, int T, int n,
                                                      const int64_t* __restrict__ rep_a,
                                                      const int64_t* __restrict__ rep_c, int32_t* __restrict__ bad) {
    const size_t S = (size_t)T * n;
    const size_t s = (size_t)blockIdx.x * 256 + threadIdx.x;
    int diff = 0;
    if (s < S) {
        constexpr int offs[NAG + 1] = {0, 7, 20, 23, 26, 29, 32, 35, 38};
        const uint4* x = reinterpret_cast<const uint4*>(rows) + s * (GROW / 4);
        uint4 v[GROW / 4];
#pragma unroll
        for (int q = 0; q < GROW / 4; q++) v[q] = x[q];
        auto word = [](const uint4& u, int i) { return i == 0 ? u.x : i == 1 ? u.y : i == 2 ? u.z : u.w; };
        const size_t rc = (size_t)rep_c[s];
        if (rc != s) {
            const uint4* y = reinterpret_cast<const uint4*>(rows) + rc * (GROW / 4);
#pragma unroll
            for (int q = 0; q < GROW / 4; q++) {
                const uint4 w = y[q];
                diff |= (int)((w.x ^ v[q].x) | (w.y ^ v[q].y) | (w.z ^ v[q].z) | (w.w ^ v[q].w)) != 0;
            }
        }
#pragma unroll
        for (int a = 0; a < NAG; a++) {
            const size_t ra = (size_t)rep_a[(size_t)a * S + s];
            if (ra != s) {
                const uint4* y = reinterpret_cast<const uint4*>(rows) + ra * (GROW / 4);
#pragma unroll
                for (int q = offs[a] / 4; q <= (offs[a + 1] - 1) / 4; q++) {
                    const uint4 w = y[q];
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int c = 4 * q + i;
                        if (c >= offs[a] && c < offs[a + 1]) diff |= (int)(word(w, i) != word(v[q], i));
                    }
                }
            }
        }
    }
    diff = __syncthreads_or(diff);
    if (threadIdx.x == 0) bad[blockIdx.x] = diff ? 1 : 0;
}

// ReLU backward fused with the bias gradient of the layer under it (the critic's split-K
// backward, a2c_vec._LinearSplitK): g = gy where y > 0 else 0 for y = relu(x W^T + b) [rows][C],
// and part[block][c] = sum of g[r][c] over the workgroup's RB rows (the caller sums the
// blocks).  One pass over gy and y instead of a threshold pass plus a column reduction.
// 256 threads = (256 / (C / 4)) rows x (C / 4) float4 columns.
template <int C>
__global__ void __launch_bounds__(256) k_relu_bias_grad(const float* __restrict__ gy, const float* __restrict__ y,
                                                        int64_t rows, float* __restrict__ g,
                                                        float* __restrict__ part) {
    constexpr int Q = C / 4, RP = 256 / Q, RB = 128;
    const int q = threadIdx.x % Q, rr = threadIdx.x / Q;
    const int64_t r0 = (int64_t)blockIdx.x * RB;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    auto row = [&](int64_t r) {
        const float4 a = reinterpret_cast<const float4*>(gy + r * C)[q];
        const float4 v = reinterpret_cast<const float4*>(y + r * C)[q];
        const float4 o = make_float4(v.x > 0.f ? a.x : 0.f, v.y > 0.f ? a.y : 0.f, v.z > 0.f ? a.z : 0.f,
                                     v.w > 0.f ? a.w : 0.f);
        reinterpret_cast<float4*>(g + r * C)[q] = o;
        acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
    };
    if (r0 + RB <= rows) {   // a full block: fixed trip count, loads batched by the unroll
#pragma unroll 8
        for (int i = rr; i < RB; i += RP) row(r0 + i);
    } else {
        for (int i = rr; i < RB && r0 + i < rows; i += RP) row(r0 + i);
    }
    __shared__ float4 s_acc[256];
    s_acc[threadIdx.x] = acc;
    __syncthreads();
    if (rr == 0) {
        for (int k = 1; k < RP; k++) {
            const float4 b = s_acc[k * Q + q];
            acc.x += b.x; acc.y += b.y; acc.z += b.z; acc.w += b.w;
        }
        reinterpret_cast<float4*>(part + (size_t)blockIdx.x * C)[q] = acc;
    }
}

// Backward of the critic's last two layers, y = relu(h W3^T + b3) [rows][128], v = y w4 + b4,
// from the value gradient gv [rows] in one pass over y (a2c_vec._ValueHead): g = gv w4 where
// y > 0 else 0 (the gradient into layer 3's pre-activation), and per block of 128 rows the
// partial sums part[block][0..127] = sum g (layer 3's bias gradient), [128..255] = sum gv y
// (w4's gradient), [256] = sum gv (b4's gradient), [257..259] = 0.
__global__ void __launch_bounds__(256) k_value_head_grad(const float* __restrict__ y, const float* __restrict__ gv,
                                                         const float* __restrict__ w4, int64_t rows,
                                                         float* __restrict__ g, float* __restrict__ part) {
    constexpr int C = 128, Q = C / 4, RP = 256 / Q, RB = 128, PW = 2 * C + 4;
    const int q = threadIdx.x % Q, rr = threadIdx.x / Q;
    const int64_t r0 = (int64_t)blockIdx.x * RB;
    const float4 w = reinterpret_cast<const float4*>(w4)[q];
    float4 ab = make_float4(0.f, 0.f, 0.f, 0.f), aw = ab;
    float av = 0.f;
    auto row = [&](int64_t r) {
        const float gr = gv[r];
        const float4 v = reinterpret_cast<const float4*>(y + r * C)[q];
        const float4 o = make_float4(v.x > 0.f ? gr * w.x : 0.f, v.y > 0.f ? gr * w.y : 0.f,
                                     v.z > 0.f ? gr * w.z : 0.f, v.w > 0.f ? gr * w.w : 0.f);
        reinterpret_cast<float4*>(g + r * C)[q] = o;
        ab.x += o.x; ab.y += o.y; ab.z += o.z; ab.w += o.w;
        aw.x += gr * v.x; aw.y += gr * v.y; aw.z += gr * v.z; aw.w += gr * v.w;
        av += gr;
    };
    if (r0 + RB <= rows) {
#pragma unroll 8
        for (int i = rr; i < RB; i += RP) row(r0 + i);
    } else {
        for (int i = rr; i < RB && r0 + i < rows; i += RP) row(r0 + i);
    }
    __shared__ float4 s_b[256], s_w[256];
    __shared__ float s_v[256];
    s_b[threadIdx.x] = ab;
    s_w[threadIdx.x] = aw;
    s_v[threadIdx.x] = q == 0 ? av : 0.f;
    __syncthreads();
    float* out = part + (size_t)blockIdx.x * PW;
    if (rr == 0) {
        for (int k = 1; k < RP; k++) {
            const float4 b = s_b[k * Q + q], c = s_w[k * Q + q];
            ab.x += b.x; ab.y += b.y; ab.z += b.z; ab.w += b.w;
            aw.x += c.x; aw.y += c.y; aw.z += c.z; aw.w += c.w;
        }
        reinterpret_cast<float4*>(out)[q] = ab;
        reinterpret_cast<float4*>(out + C)[q] = aw;
    }
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int k = 0; k < RP; k++) t += s_v[k * Q];
        reinterpret_cast<float4*>(out + 2 * C)[0] = make_float4(t, 0.f, 0.f, 0.f);
    }
}

}  // namespace

int fjsp_internal_fail(const char* msg);

// Library-wide variants of the policy launches, set with fjsp_set_option(NULL or any handle,
// "policy_xmap" | "policy_dedup" | "policy_split", v) (A/B runs and the bit-identity tests; read
// per launch, so a captured graph keeps the variant it was captured with).  Every setting gives
// byte-identical outputs.
//   policy_xmap 0..3: actor_block's workgroup -> XCD order (0, the default: none).  Orders 1-3
//     lay the launch out per XCD and so run without the split below.
//   policy_dedup 0/1: the station agents' MLP once per distinct input of a 64-env tile (1, default)
//     or on every env.
//   policy_split 0/1: k_policy_step's pickup-station and AGV tiles as two 32-env workgroups each
//     (1, default: half the matrix-core chain of the launch's longest workgroups) or one.
static int g_policy_xmap = 0, g_policy_dedup = 1, g_policy_split = 1;
static int policy_xmap() { return g_policy_xmap; }
static int policy_dedup() { return g_policy_dedup; }
static int policy_split() { return g_policy_split; }
extern "C" int fjsp_internal_policy_option(const char* name, int64_t value) {
    if (!strcmp(name, "policy_xmap")) {
        if (value < 0 || value > 3) return fjsp_internal_fail("policy_xmap must be in 0..3");
        g_policy_xmap = (int)value;
        return 0;
    }
    if (!strcmp(name, "policy_dedup")) { g_policy_dedup = value != 0; return 0; }
    if (!strcmp(name, "wgrad_waves")) {
        if (value != 8 && value != 16) return fjsp_internal_fail("wgrad_waves must be 8 or 16");
        g_wgrad_waves = (int)value;
        return 0;
    }
    if (!strcmp(name, "policy_split")) { g_policy_split = value != 0; return 0; }
    return fjsp_internal_fail("unknown option");
}

// fjsp_a2c_policy_step's launch (fjsp_hip.hip holds the handle): k_policy_step on the policy's
// grid, the step's state / config / outputs and the tile hand-off buffers from the handle.
int fjsp_internal_policy_step(const float* feats, const int8_t* masks, int32_t n, const float* actor_w,
                              const float* critic_w, const uint64_t* seed, uint32_t env_gid0, uint32_t step,
                              int32_t deterministic, uint8_t* actions, float* values, const fjsp::DevState& S,
                              const fjsp::Cfg& C, const fjsp_out& out, uint32_t* tile_cnt, uint32_t* tile_act,
                              int32_t autoreset, int32_t env_begin, int32_t env_count, hipStream_t stream) {
    if (out.obs_i32 || out.obs_i8 || out.obs_f32 || out.masks || out.results || out.orders_completed || out.packaged ||
        out.sim_time || out.next_i32 || out.next_i8 || out.next_f32)
        return fjsp_internal_fail("fjsp_a2c_policy_step: outputs limited to rewards, term, trunc, status, next_masks, feats");
    // envs [env_begin, env_begin + env_count): whole 64-env tiles (the caller checks the range)
    PolicyArgs A{feats, masks, n, actor_w, critic_w, seed, env_gid0, step, deterministic, actions, values, nullptr,
                 values ? (env_count + TC - 1) / TC : 0, (env_count + TA - 1) / TA, env_begin / TA, policy_xmap(), policy_dedup()};
    A.split = policy_split() && A.xmap == 0;
    const int actor_blocks = (NAG + (A.split ? 2 : 0)) * A.na;
    // the tiles copy their outputs out in 16-byte pieces when every tile is full and every output
    // row and state row of a tile starts 16-byte aligned (n % 64 == 0, 16-byte aligned bases)
    const uintptr_t bases = (uintptr_t)out.rewards | (uintptr_t)out.term | (uintptr_t)out.trunc | (uintptr_t)out.status |
                            (uintptr_t)out.next_masks | (uintptr_t)out.feats | (uintptr_t)S.words;
    StepArgs St{S, C, out.rewards, out.term, out.trunc, out.status, out.next_masks, out.feats, tile_cnt, tile_act,
                autoreset ? STEP_AUTORESET : 0};
    if (n % TA == 0 && (bases & 15u) == 0)
        hipLaunchKernelGGL(k_policy_step<true>, dim3((unsigned)(A.nc + actor_blocks)), dim3(NTHR), 0, stream, A, St);
    else
        hipLaunchKernelGGL(k_policy_step<false>, dim3((unsigned)(A.nc + actor_blocks)), dim3(NTHR), 0, stream, A, St);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}   // fjsp_hip.hip: sets fjsp_last_error()

extern "C" int fjsp_a2c_actor_head(const float* pu, int32_t umax, const int64_t* inv, int32_t T, int32_t n,
                                   const int8_t* masks, const uint8_t* actions, const double* adv, const float* adv_mean,
                                   const float* adv_std, float inv_count, float ent_coef, float* grad, double* sums,
                                   void* stream) {
    if (T <= 0 || n <= 0 || umax <= 0) return fjsp_internal_fail("fjsp_a2c_actor_head: T, n and umax must be > 0");
    if (!pu || !inv || !masks || !actions || !adv || !grad || !sums || (!adv_mean != !adv_std))
        return fjsp_internal_fail("fjsp_a2c_actor_head: null buffer");
    const size_t S = (size_t)T * (size_t)n;
    hipLaunchKernelGGL(k_actor_head, dim3((unsigned)((S + 255) / 256), NAG), dim3(256), 0, (hipStream_t)stream, pu, umax,
                       inv, T, n, masks, actions, adv, adv_mean, adv_std, inv_count, ent_coef, grad, sums);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}

extern "C" int fjsp_a2c_group_keys(const float* feats, int32_t T, int32_t n, uint64_t* keys, float* rows,
                                   void* stream) {
    if (T <= 0 || n <= 0) return fjsp_internal_fail("fjsp_a2c_group_keys: T and n must be > 0");
    if (!feats || !keys) return fjsp_internal_fail("fjsp_a2c_group_keys: null buffer");
    const size_t S = (size_t)T * (size_t)n;
    if (rows && ((uintptr_t)rows & 15u)) return fjsp_internal_fail("fjsp_a2c_group_keys: rows must be 16-byte aligned");
    hipLaunchKernelGGL(k_group_keys, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, (hipStream_t)stream, feats, T, n,
                       keys, rows);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}

extern "C" int fjsp_a2c_pack_mfma(const float* W, int32_t B, int32_t R, int32_t K, int32_t transposed, float* out,
                                  void* stream) {
    if (B <= 0 || R <= 0 || K <= 0 || R % 32 || K % 16)
        return fjsp_internal_fail("fjsp_a2c_pack_mfma: need B > 0, R a multiple of 32, K a multiple of 16");
    if (!W || !out) return fjsp_internal_fail("fjsp_a2c_pack_mfma: null buffer");
    if ((uintptr_t)out & 7u) return fjsp_internal_fail("fjsp_a2c_pack_mfma: out must be 8-byte aligned");
    const int64_t total = (int64_t)B * (R / 32) * (K / 16) * 128;
    hipLaunchKernelGGL(k_pack_mfma, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, W, B, R, K,
                       transposed, reinterpret_cast<__bf16*>(out));
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}

extern "C" int fjsp_a2c_record_head(const float* pu, int32_t umax, const int64_t* inv, int32_t R, int32_t nact,
                                    const int32_t* info, const double* wsum, const int32_t* cnt, float inv_count,
                                    float ent_coef, float* grad, double* sums, void* stream) {
    if (R <= 0 || umax <= 0 || nact <= 0 || nact > 8)
        return fjsp_internal_fail("fjsp_a2c_record_head: need R > 0, umax > 0, 0 < nact <= 8");
    if (!pu || !inv || !info || !wsum || !cnt || !grad || !sums) return fjsp_internal_fail("fjsp_a2c_record_head: null buffer");
    hipLaunchKernelGGL(k_record_head, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, (hipStream_t)stream, pu, umax, inv, R,
                       nact, info, wsum, cnt, inv_count, ent_coef, grad, sums);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}

extern "C" int fjsp_a2c_shard_keys(const uint64_t* keys, const int8_t* masks, const uint8_t* actions, int32_t T,
                                   int32_t n, uint64_t* tk, int32_t* info, int32_t* bad, void* stream) {
    if (T <= 0 || n <= 0) return fjsp_internal_fail("fjsp_a2c_shard_keys: T and n must be > 0");
    if (!keys || !masks || !actions || !tk || !info || !bad) return fjsp_internal_fail("fjsp_a2c_shard_keys: null buffer");
    const size_t S = (size_t)T * (size_t)n;
    hipLaunchKernelGGL(k_shard_keys, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, (hipStream_t)stream, keys, masks,
                       actions, T, n, tk, info, bad);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}

extern "C" int fjsp_a2c_group_verify(const float* rows, int32_t T, int32_t n, const int64_t* rep_a,
                                     const int64_t* rep_c, int32_t* bad, void* stream) {
    if (T <= 0 || n <= 0) return fjsp_internal_fail("fjsp_a2c_group_verify: T and n must be > 0");
    if (!rows || !rep_a || !rep_c || !bad) return fjsp_internal_fail("fjsp_a2c_group_verify: null buffer");
    if ((uintptr_t)rows & 15u) return fjsp_internal_fail("fjsp_a2c_group_verify: rows must be 16-byte aligned");
    const size_t S = (size_t)T * (size_t)n;
    hipLaunchKernelGGL(k_group_verify, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, (hipStream_t)stream, rows, T,
                       n, rep_a, rep_c, bad);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}

extern "C" int fjsp_a2c_relu_bias_grad(const float* gy, const float* y, int64_t rows, int32_t cols, float* g,
                                       float* part, void* stream) {
    if (rows <= 0) return fjsp_internal_fail("fjsp_a2c_relu_bias_grad: rows must be > 0");
    if (cols != 128 && cols != 256) return fjsp_internal_fail("fjsp_a2c_relu_bias_grad: cols must be 128 or 256");
    if (!gy || !y || !g || !part) return fjsp_internal_fail("fjsp_a2c_relu_bias_grad: null buffer");
    const dim3 grid((unsigned)((rows + 127) / 128));
    if (cols == 256)
        hipLaunchKernelGGL(k_relu_bias_grad<256>, grid, dim3(256), 0, (hipStream_t)stream, gy, y, rows, g, part);
    else
        hipLaunchKernelGGL(k_relu_bias_grad<128>, grid, dim3(256), 0, (hipStream_t)stream, gy, y, rows, g, part);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}

extern "C" int fjsp_a2c_value_head_grad(const float* y, const float* gv, const float* w4, int64_t rows, float* g,
                                        float* part, void* stream) {
    if (rows <= 0) return fjsp_internal_fail("fjsp_a2c_value_head_grad: rows must be > 0");
    if (!y || !gv || !w4 || !g || !part) return fjsp_internal_fail("fjsp_a2c_value_head_grad: null buffer");
    hipLaunchKernelGGL(k_value_head_grad, dim3((unsigned)((rows + 127) / 128)), dim3(256), 0, (hipStream_t)stream, y,
                       gv, w4, rows, g, part);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}

#ifdef FJSP_STAMPS
extern "C" int fjsp_debug_policy_stamps(unsigned long long* out, int32_t clear) {   // out[2048 * 16]
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pstamps), sizeof(unsigned long long) * 2048 * 16) != hipSuccess) return -2;
    if (clear) {
        static unsigned long long z[2048 * 16];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_pstamps), z, sizeof(z)) != hipSuccess) return -2;
    }
    return 0;
}
#endif

extern "C" int fjsp_a2c_critic_forward(const float* x, int32_t n, const float* critic_w, float* h1, float* h2,
                                       float* h3, float* values, void* stream) {
    if (n <= 0) return fjsp_internal_fail("fjsp_a2c_critic_forward: n must be > 0");
    if (!x || !critic_w || !h1 || !h2 || !h3 || !values) return fjsp_internal_fail("fjsp_a2c_critic_forward: null buffer");
    if ((uintptr_t)x & 15u) return fjsp_internal_fail("fjsp_a2c_critic_forward: x must be 16-byte aligned");
    PolicyArgs A{x, nullptr, n, nullptr, critic_w, nullptr, 0u, 0u, 0, nullptr, values, nullptr, (n + TC - 1) / TC, 0};
    hipLaunchKernelGGL(k_critic_fwd, dim3((unsigned)A.nc), dim3(NTHR), 0, (hipStream_t)stream, A, CriticSave{h1, h2, h3});
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}

extern "C" int fjsp_a2c_critic_fused(const float* x, int32_t n, const float* critic_w, const float* w3t,
                                     const float* w2t, const double* coef, float* h1, float* h2, float* g3, float* g2,
                                     float* g1, float* part, double* loss, float* values, void* stream) {
    if (n <= 0) return fjsp_internal_fail("fjsp_a2c_critic_fused: n must be > 0");
    if (!x || !critic_w || !w3t || !w2t || !coef || !h1 || !h2 || !g3 || !g2 || !g1 || !part || !loss)
        return fjsp_internal_fail("fjsp_a2c_critic_fused: null buffer");
    if (((uintptr_t)x | (uintptr_t)h1 | (uintptr_t)h2 | (uintptr_t)g3 | (uintptr_t)g2 | (uintptr_t)g1 | (uintptr_t)part) & 15u)
        return fjsp_internal_fail("fjsp_a2c_critic_fused: x, h1, h2, g3, g2, g1 and part must be 16-byte aligned");
    PolicyArgs A{x, nullptr, n, nullptr, critic_w, nullptr, 0u, 0u, 0, nullptr, values, nullptr, (n + TC - 1) / TC, 0};
    const CriticFused F{coef, w3t, w2t, h1, h2, g3, g2, g1, part, loss, values};
    hipLaunchKernelGGL(k_critic_fused, dim3((unsigned)A.nc), dim3(NTHR), 0, (hipStream_t)stream, A, F);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}

extern "C" int fjsp_a2c_wgrad(const float* g, int32_t m, int64_t ldg, const float* x, int32_t nx, int64_t ldx, int64_t U,
                              float* part, int32_t P, float* out, int32_t nout, int64_t ldo, void* stream) {
    if (U <= 0 || P <= 0) return fjsp_internal_fail("fjsp_a2c_wgrad: U and P must be > 0");
    if (!g || !x || !part || !out) return fjsp_internal_fail("fjsp_a2c_wgrad: null buffer");
    if (((uintptr_t)g | (uintptr_t)x) & 15u || (ldg & 3) || (ldx & 3) || (nx & 3) || ldg < m || ldx < nx)
        return fjsp_internal_fail("fjsp_a2c_wgrad: g and x must be 16-byte aligned rows (ld % 4 == 0, nx % 4 == 0)");
    if (nout <= 0 || nout > nx || ldo < nout) return fjsp_internal_fail("fjsp_a2c_wgrad: 0 < nout <= nx, ldo >= nout");
    // buffer-load offsets are 32-bit: the rows, plus the stages read ahead past the last one
    const int64_t ldm = ldg > ldx ? ldg : ldx;
    if ((U + (int64_t)(WG_MAXD + 1) * P * WG_KS) * ldm * 4 > 0x7FFFFF00ll || (int64_t)P * WG_KS * ldm * 4 > 0x7FFFFFFFll)
        return fjsp_internal_fail("fjsp_a2c_wgrad: U * ld * 4 must stay below 2 GiB (split the batch)");
    const hipStream_t st = (hipStream_t)stream;
    int npad;
    if (m == 256 && nx > 64 && nx <= 256) {
        npad = 256;
        if (g_wgrad_waves == 16)
            hipLaunchKernelGGL((k_wgrad16<256, 256, 1, 4, 1>), dim3((unsigned)P), dim3(1024), 0, st, g, ldg, x, ldx, nx, U, part);
        else
            hipLaunchKernelGGL((k_wgrad<256, 256, 2, 4, 2>), dim3((unsigned)P), dim3(NTHR), 0, st, g, ldg, x, ldx, nx, U, part);
    } else if (m == 128 && nx > 64 && nx <= 256) {
        npad = 256;
        if (g_wgrad_waves == 16)
            hipLaunchKernelGGL((k_wgrad16<128, 256, 1, 2, 2>), dim3((unsigned)P), dim3(1024), 0, st, g, ldg, x, ldx, nx, U, part);
        else
            hipLaunchKernelGGL((k_wgrad<128, 256, 2, 2, 4>), dim3((unsigned)P), dim3(NTHR), 0, st, g, ldg, x, ldx, nx, U, part);
    } else if (m == 256 && nx <= 64) {
        npad = 64;
        if (g_wgrad_waves == 16)
            hipLaunchKernelGGL((k_wgrad16<256, 64, 1, 1, 3>), dim3((unsigned)P), dim3(1024), 0, st, g, ldg, x, ldx, nx, U, part);
        else
            hipLaunchKernelGGL((k_wgrad<256, 64, 1, 2, 4>), dim3((unsigned)P), dim3(NTHR), 0, st, g, ldg, x, ldx, nx, U, part);
    } else {
        return fjsp_internal_fail("fjsp_a2c_wgrad: (m, nx) must be (256, 68..256), (128, 68..256) or (256, 4..64)");
    }
    hipLaunchKernelGGL(k_wgrad_reduce, dim3((unsigned)((m * nout + 255) / 256)), dim3(256), 0, st, part, P, m, npad, nout,
                       out, ldo);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}

extern "C" int fjsp_a2c_critic_backward(const float* g3, const float* h1, const float* h2, int32_t n, const float* w3t,
                                        const float* w2t, float* g2, float* g1, float* bias_part2, float* bias_part1,
                                        void* stream) {
    if (n <= 0) return fjsp_internal_fail("fjsp_a2c_critic_backward: n must be > 0");
    if (!g3 || !h1 || !h2 || !w3t || !w2t || !g2 || !g1 || !bias_part2 || !bias_part1)
        return fjsp_internal_fail("fjsp_a2c_critic_backward: null buffer");
    const CriticBwd B{g3, h1, h2, w3t, w2t, g2, g1, bias_part2, bias_part1, n};
    hipLaunchKernelGGL(k_critic_bwd, dim3((unsigned)((n + TC - 1) / TC)), dim3(NTHR), 0, (hipStream_t)stream, B);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}

extern "C" int fjsp_a2c_policy(const float* feats, const int8_t* masks, int32_t n, const float* actor_w,
                               const float* critic_w, const uint64_t* seed, uint32_t env_gid0, uint32_t step,
                               int32_t deterministic,
                               uint8_t* actions, float* values, float* probs, void* stream) {
    if (n <= 0) return fjsp_internal_fail("fjsp_a2c_policy: n must be > 0");
    if (!feats || (!actions && !values) || (values && !critic_w) || (actions && (!masks || !actor_w || !seed)))
        return fjsp_internal_fail("fjsp_a2c_policy: null buffer");
    // workgroups: the critic on 32-env tiles (values wanted), then each actor on 64-env tiles
    // (actions wanted)
    PolicyArgs A{feats, masks, n, actor_w, critic_w, seed, env_gid0, step, deterministic, actions, values, probs,
                 values ? (n + TC - 1) / TC : 0, actions ? (n + TA - 1) / TA : 0, 0, policy_xmap(), policy_dedup()};
    hipLaunchKernelGGL(k_policy, dim3((unsigned)(A.nc + NAG * A.na)), dim3(NTHR), 0, (hipStream_t)stream, A);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}
