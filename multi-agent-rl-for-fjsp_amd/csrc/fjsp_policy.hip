// fjsp_policy.hip — fused A2C policy step for gfx950 (one launch per vector step).
//
// Replaces the ~40 PyTorch launches of a2c_vec.VecMultiAgentA2C.policy (reference predict,
// a2c.py:168-252): for every env, the 8 actor MLPs (networks.ActorNetwork: d -> 256 -> 256 ->
// n_a, softmax), the action mask / renormalisation / uniform fallback (a2c.py:204-220), the
// action draw (inverse CDF over the masked probabilities, or argmax) and the centralised
// critic (networks.CentralizedCriticNetwork: 38 -> 256 -> 256 -> 128 -> 1).
//
// Grid: blockIdx.y = role (0 critic, 1..8 actor of agent y - 1), blockIdx.x = tile of 64 envs;
// 512 threads = 8 wavefronts.  The hidden activations never leave LDS:
//   x   [40][TILE]  inputs of the tile (feature rows of the kernel-written [38][N] slab)
//   h   [256][TILE] layer 1, then layer 2, then the critic's layer 3 (in place: results stay in
//                   registers across a barrier), so two workgroups fit a CU (74 KB of LDS each)
// Every layer with K >= 16 runs on v_mfma_f32_32x32x2_f32 (exact f32 fma chains): each wave
// owns 32 output rows x the tile's 64 envs = two 32 x 32 tiles sharing one weight fragment (the
// critic's 128-row layer 3: waves 0..3).
// The actor's 256 -> n_a logits and the critic's 128 -> 1 value are VALU dot products.
// MFMA A operands (weights) are pre-packed on the host per (row tile, k-step) in lane order
// (fjsp_pack_policy_weights layout below), so each k-step's A fragment is one coalesced
// 256-byte load; B fragments (activations) are conflict-free LDS reads.
// f32 arithmetic throughout (the reference networks are f32); summation order differs from
// PyTorch's GEMMs only by rounding (tests: 1e-5).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/fjsp.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// 64 envs per workgroup on 8 waves: each weight fragment loaded from L2 feeds two MFMAs (one
// per 32-env column tile), half the weight traffic of 32-env tiles at the same waves per CU
// (two 74 KB workgroups = 16 waves).  The weight loads, one 256-byte A fragment per MFMA with
// 32-env tiles, are what bounds this kernel: 4 SIMDs x 256 B per 16-cycle MFMA = the CU's
// 64 B/clk vector-memory path.
constexpr int TILE = 64;              // envs per workgroup
constexpr int NCOL = TILE / 32;       // 32-column MFMA tiles per row tile
constexpr int NWAVE = 8;
constexpr int NTHR = 64 * NWAVE;
constexpr int HID = 256;
constexpr int NAG = 8;
constexpr int KS2 = HID / 2;   // k-steps of 2 for a 256-wide contraction

__constant__ int c_obs_off[NAG] = {0, 7, 20, 23, 26, 29, 32, 35};
__constant__ int c_obs_dim[NAG] = {7, 13, 3, 3, 3, 3, 3, 3};
__constant__ int c_mask_off[NAG] = {0, 3, 11, 14, 17, 20, 23, 26};
__constant__ int c_nact[NAG] = {3, 8, 3, 3, 3, 3, 3, 3};

__device__ __forceinline__ uint64_t fmix64(uint64_t z) {
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z;
}

// MFMA A operands are packed per row tile t in groups of 4 k-steps: element (t, q, l, j) =
// W[32 t + (l & 31)][2 (4 q + j) + (l >> 5)], so one 16-byte load per lane fetches the A
// fragments of 4 consecutive k-steps (a coalesced 1 KB per wave instruction).
// acc[i][j] += W(row tile rt0 + i) . act(col tile j); act = LDS [K][TILE] (rows = k), KS = K / 2.
template <int NT, int KS>
__device__ __forceinline__ void mfma_rows(const float* __restrict__ wp, int rt0, const float* act, int lane,
                                          f32x16 acc[NT][NCOL]) {
    static_assert(KS % 4 == 0, "k-steps come in groups of 4");
    constexpr int NQ = KS / 4;
    const float4* a[NT];
#pragma unroll
    for (int i = 0; i < NT; i++) a[i] = reinterpret_cast<const float4*>(wp) + (size_t)(rt0 + i) * NQ * 64 + lane;
    const int kr = lane >> 5, cl = lane & 31;
    constexpr int PF = NQ < 2 ? NQ : 2;   // groups in flight (3, 4, 6 in a register ring: no faster, r03)
    float4 buf[PF][NT];
#pragma unroll
    for (int p = 0; p < PF; p++)
#pragma unroll
        for (int i = 0; i < NT; i++) buf[p][i] = a[i][p * 64];
#pragma unroll 2
    for (int q = 0; q < NQ; q++) {
        float4 cur[NT];
#pragma unroll
        for (int i = 0; i < NT; i++) cur[i] = buf[q % PF][i];
        if (q + PF < NQ) {
#pragma unroll
            for (int i = 0; i < NT; i++) buf[q % PF][i] = a[i][(q + PF) * 64];
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int k = 2 * (4 * q + j) + kr;
            float b[NCOL];
#pragma unroll
            for (int c = 0; c < NCOL; c++) b[c] = act[k * TILE + 32 * c + cl];
#pragma unroll
            for (int i = 0; i < NT; i++) {
                const float fa = j == 0 ? cur[i].x : j == 1 ? cur[i].y : j == 2 ? cur[i].z : cur[i].w;
#pragma unroll
                for (int c = 0; c < NCOL; c++) acc[i][c] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa, b[c], acc[i][c], 0, 0, 0);
            }
        }
    }
}

template <int NT>
__device__ __forceinline__ void zero_acc(f32x16 acc[NT][NCOL]) {
#pragma unroll
    for (int i = 0; i < NT; i++)
#pragma unroll
        for (int j = 0; j < NCOL; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] = 0.0f;
}

// relu(acc + bias) -> out LDS [rows][TILE]; C/D layout of the 32x32 f32 MFMA: col = lane & 31,
// row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5).
__device__ __forceinline__ void store_tile(const f32x16& acc, int row0, int col0, const float* __restrict__ bias,
                                           float* out, int lane) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int row = row0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const float v = acc[r] + bias[row];
        out[row * TILE + col0 + (lane & 31)] = v > 0.0f ? v : 0.0f;
    }
}
template <int NT>
__device__ __forceinline__ void store_rows(const f32x16 acc[NT][NCOL], int row0, const float* __restrict__ bias, float* out,
                                           int lane) {
#pragma unroll
    for (int i = 0; i < NT; i++)
#pragma unroll
        for (int j = 0; j < NCOL; j++) store_tile(acc[i][j], row0 + 32 * i, 32 * j, bias, out, lane);
}

// Hidden layers 1 and 2 of a 256-wide MLP on the tile (x in s_x [DPAD][TILE]) -> s_h [256][TILE].
template <int DPAD>
__device__ __forceinline__ void hidden256(const float* __restrict__ W, const float* s_x, float* s_h, int wave, int lane) {
    const float* W1 = W;                         // packed [8][DPAD/8][64][4]
    const float* B1 = W1 + 256 * DPAD;           // [256]
    const float* W2 = B1 + 256;                  // packed [8][32][64][4]
    const float* B2 = W2 + 256 * 256;            // [256]
    f32x16 acc[1][NCOL];
    zero_acc<1>(acc);
    mfma_rows<1, DPAD / 2>(W1, wave, s_x, lane, acc);
    store_rows<1>(acc, 32 * wave, B1, s_h, lane);
    __syncthreads();
    zero_acc<1>(acc);
    mfma_rows<1, 128>(W2, wave, s_h, lane, acc);
    __syncthreads();                             // every wave has read h1
    store_rows<1>(acc, 32 * wave, B2, s_h, lane);
    __syncthreads();
}

__global__ void __launch_bounds__(NTHR, 4) k_policy(const float* __restrict__ feats, const int8_t* __restrict__ masks,
                                                   int n, const float* __restrict__ actor_w,
                                                   const float* __restrict__ critic_w, const uint64_t* __restrict__ seedp,
                                                   uint32_t gid0, uint32_t step, int deterministic, uint8_t* __restrict__ actions,
                                                   float* __restrict__ values, float* __restrict__ probs_out, int role0) {
    __shared__ float s_x[FJSP_POLICY_CRITIC_DPAD * TILE];   // inputs; later the logits [8][TILE]
    __shared__ float s_h[HID * TILE];                        // h1, then h2 (then critic h3)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // the critic (the heaviest role: 848 MFMAs per wave against 544) first: 576 workgroups run
    // on 512 two-per-CU slots, and the ones left for the second round should be the short ones
    // (measured: 83.8 -> 75.0 us per launch at 4 096 envs)
    const int y = (int)blockIdx.y + role0;   // role0 = 1: the actors only (no values wanted)
    const int role = y == 0 ? NAG : y - 1;
    const int e0 = blockIdx.x * TILE;
    const bool critic = role == NAG;
    if (!critic) {
        // a tile in which the agent has exactly one valid action in every env: the draw (and
        // argmax) returns that action whatever the network says, and the masked probabilities
        // are exactly one-hot (p / p, or the uniform fallback over one action) -- skip the MLP.
        // The station agents are forced in 96-100 % of an A2C collect's samples and whole
        // tiles in 38-100 % (scripts/diag_forced_actions.py)
        const int na = c_nact[role], mo = c_mask_off[role];
        int forced = 1, only = 0;
        if (tid < TILE && e0 + tid < n) {
            int cnt = 0;
#pragma unroll
            for (int j = 0; j < 8; j++)
                if (j < na && masks[(size_t)(mo + j) * n + e0 + tid] != 0) { cnt++; only = j; }
            forced = cnt == 1;
        }
        if (__syncthreads_and(forced)) {
            if (tid < TILE && e0 + tid < n) {
                const int e = e0 + tid;
                actions[(size_t)role * n + e] = (uint8_t)only;
                if (probs_out)
                    for (int j = 0; j < 8; j++) probs_out[((size_t)role * 8 + j) * n + e] = j == only ? 1.0f : 0.0f;
            }
            return;
        }
    }
    const int din = critic ? 38 : c_obs_dim[role];
    const int off = critic ? 0 : c_obs_off[role];
    const int dpad = critic ? FJSP_POLICY_CRITIC_DPAD : FJSP_POLICY_ACTOR_DPAD;
    for (int i = tid; i < dpad * TILE; i += NTHR) {
        const int k = i / TILE, c = i % TILE;
        s_x[i] = (k < din && e0 + c < n) ? feats[(size_t)(off + k) * n + e0 + c] : 0.0f;
    }
    __syncthreads();
    if (critic) {
        hidden256<FJSP_POLICY_CRITIC_DPAD>(critic_w, s_x, s_h, wave, lane);
        const float* W3 = critic_w + 256 * FJSP_POLICY_CRITIC_DPAD + 256 + 256 * 256 + 256;   // packed [4][32][64][4]
        const float* B3 = W3 + 128 * HID;                  // [128]
        const float* W4 = B3 + 128;                        // [128]
        const float* B4 = W4 + 128;                        // [1]
        f32x16 acc[1][NCOL];
        if (wave < 4) {                                    // 128 rows = 4 row tiles
            zero_acc<1>(acc);
            mfma_rows<1, 128>(W3, wave, s_h, lane, acc);
        }
        __syncthreads();
        if (wave < 4) store_rows<1>(acc, 32 * wave, B3, s_h, lane);   // h3 [128][TILE]
        __syncthreads();
        if (tid < TILE && e0 + tid < n) {
            float v = B4[0];
            for (int k = 0; k < 128; k++) v = fmaf(W4[k], s_h[k * TILE + tid], v);
            values[e0 + tid] = v;
        }
        return;
    }
    const float* W = actor_w + (size_t)role * FJSP_POLICY_ACTOR_FLOATS;
    hidden256<FJSP_POLICY_ACTOR_DPAD>(W, s_x, s_h, wave, lane);
    // layer 3: logits [8][TILE]; wave -> action row, lane -> env; weights wave-uniform
    const float* W3 = W + 256 * FJSP_POLICY_ACTOR_DPAD + 256 + 256 * 256 + 256;   // [8][256]
    const float* B3 = W3 + 8 * HID;                                                // [8]
    float* s_logit = s_x;
    static_assert(NWAVE == 8 && TILE == 64, "one logit row per wave, one env per lane");
    {
        const int c = lane, r = wave;
        float l = B3[r];
        for (int k = 0; k < HID; k++) l = fmaf(W3[r * HID + k], s_h[k * TILE + c], l);
        s_logit[r * TILE + c] = l;
    }
    __syncthreads();
    if (tid < TILE && e0 + tid < n) {
        const int c = tid, e = e0 + tid;
        const int na = c_nact[role], mo = c_mask_off[role];
        float p[8], m[8];
        float mx = -INFINITY;
        // fixed 8-trip loops guarded by na: fully unrolled, the arrays stay in registers
#pragma unroll
        for (int j = 0; j < 8; j++) if (j < na) mx = fmaxf(mx, s_logit[j * TILE + c]);
        float s = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; j++) { p[j] = j < na ? expf(s_logit[j * TILE + c] - mx) : 0.0f; s += p[j]; }
        float s2 = 0.0f, ms = 0.0f;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            m[j] = j < na ? (float)masks[(size_t)(mo + j) * n + e] : 0.0f;
            p[j] = (p[j] / s) * m[j];
            s2 += p[j];
            ms += m[j];
        }
#pragma unroll
        for (int j = 0; j < 8; j++) p[j] = s2 > 0.0f ? p[j] / s2 : m[j] / ms;
        int act = 0;
        if (deterministic) {
            float best = p[0];
#pragma unroll
            for (int j = 1; j < 8; j++) if (j < na && p[j] > best) { best = p[j]; act = j; }
        } else {
            const uint64_t seed = *seedp;
            // keyed by the env's GLOBAL id: shards of a multi-GPU job draw independent streams
            const uint64_t h = fmix64(seed ^ fmix64(((uint64_t)(gid0 + (uint32_t)e) << 32) | step) ^
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
        actions[(size_t)role * n + e] = (uint8_t)act;
        if (probs_out)
            for (int j = 0; j < 8; j++) probs_out[((size_t)role * 8 + j) * n + e] = j < na ? p[j] : 0.0f;
    }
}

// Keys of the A2C update's grouping of repeated inputs (a2c_vec.row_keys, the same hash): per
// sample s = t * n + e of feats f32 [T][38][n], key a < 8 over actor a's 13 padded input columns
// (its OBS_DIMS[a] a2c features, then zeros), key 8 over all 38; k = fmix64(k * MUL + bits(x_c)
// + c + 1) from k = 0.  One lane per sample, each column a coalesced load.
constexpr uint64_t GK_MUL = 0x100000001B3ull * 0x9E37ull + 1ull;
__device__ __forceinline__ uint64_t gk_fmix(uint64_t z) {
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ void __launch_bounds__(256) k_group_keys(const float* __restrict__ feats, int T, int n,
                                                    uint64_t* __restrict__ keys) {
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
#pragma unroll
    for (int c = 0; c < 38; c++) {
        const uint64_t b = (uint64_t)__float_as_uint(x[(size_t)c * n]);
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
                                                    const int64_t* __restrict__ actions,
                                                    const float* __restrict__ adv_n, float inv_count, float ent_coef,
                                                    float* __restrict__ grad, double* __restrict__ sums) {
    const int a = blockIdx.y;
    const size_t S = (size_t)T * n;
    const size_t s = (size_t)blockIdx.x * 256 + threadIdx.x;
    double sl = 0.0, se = 0.0;
    if (s < S) {
        const size_t t = s / (size_t)n, e = s - t * (size_t)n;
        const size_t u = (size_t)inv[(size_t)a * S + s];
        const int na = c_nact[a], mo = c_mask_off[a];
        const int act = (int)actions[(size_t)a * S + s];
        const float adv = adv_n[(size_t)a * S + s];
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

// The grouping check of the A2C update (a2c_vec.A2CLosses, replaces the torch gather-and-compare
// of every input with its group's representative): sample s is bad when any of actor a's input
// columns differs bitwise from those of rep_a[a][s], or any of its 38 global-state columns from
// those of rep_c[s] (a hash collision merged two different inputs).  Samples that represent
// their own group are skipped.  bad[block] = 1 if any sample of the workgroup is bad, else 0.
__global__ void __launch_bounds__(256) k_group_verify(const float* __restrict__ feats, int T, int n,
                                                      const int64_t* __restrict__ rep_a,
                                                      const int64_t* __restrict__ rep_c, int32_t* __restrict__ bad) {
    const size_t S = (size_t)T * n;
    const size_t s = (size_t)blockIdx.x * 256 + threadIdx.x;
    int diff = 0;
    if (s < S) {
        constexpr int offs[NAG + 1] = {0, 7, 20, 23, 26, 29, 32, 35, 38};
        const size_t t = s / (size_t)n, e = s - t * (size_t)n;
        const uint32_t* x = reinterpret_cast<const uint32_t*>(feats) + t * 38 * (size_t)n + e;
        uint32_t v[38];
#pragma unroll
        for (int c = 0; c < 38; c++) v[c] = x[(size_t)c * n];
        auto col = [&](size_t r) {
            const size_t tr = r / (size_t)n, er = r - tr * (size_t)n;
            return reinterpret_cast<const uint32_t*>(feats) + tr * 38 * (size_t)n + er;
        };
        const size_t rc = (size_t)rep_c[s];
        if (rc != s) {
            const uint32_t* y = col(rc);
#pragma unroll
            for (int c = 0; c < 38; c++) diff |= (int)(y[(size_t)c * n] != v[c]);
        }
#pragma unroll
        for (int a = 0; a < NAG; a++) {
            const size_t ra = (size_t)rep_a[(size_t)a * S + s];
            if (ra != s) {
                const uint32_t* y = col(ra);
#pragma unroll
                for (int c = offs[a]; c < offs[a + 1]; c++) diff |= (int)(y[(size_t)c * n] != v[c]);
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

int fjsp_internal_fail(const char* msg);   // fjsp_hip.hip: sets fjsp_last_error()

extern "C" int fjsp_a2c_actor_head(const float* pu, int32_t umax, const int64_t* inv, int32_t T, int32_t n,
                                   const int8_t* masks, const int64_t* actions, const float* adv_n, float inv_count,
                                   float ent_coef, float* grad, double* sums, void* stream) {
    if (T <= 0 || n <= 0 || umax <= 0) return fjsp_internal_fail("fjsp_a2c_actor_head: T, n and umax must be > 0");
    if (!pu || !inv || !masks || !actions || !adv_n || !grad || !sums)
        return fjsp_internal_fail("fjsp_a2c_actor_head: null buffer");
    const size_t S = (size_t)T * (size_t)n;
    hipLaunchKernelGGL(k_actor_head, dim3((unsigned)((S + 255) / 256), NAG), dim3(256), 0, (hipStream_t)stream, pu, umax,
                       inv, T, n, masks, actions, adv_n, inv_count, ent_coef, grad, sums);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}

extern "C" int fjsp_a2c_group_keys(const float* feats, int32_t T, int32_t n, uint64_t* keys, void* stream) {
    if (T <= 0 || n <= 0) return fjsp_internal_fail("fjsp_a2c_group_keys: T and n must be > 0");
    if (!feats || !keys) return fjsp_internal_fail("fjsp_a2c_group_keys: null buffer");
    const size_t S = (size_t)T * (size_t)n;
    hipLaunchKernelGGL(k_group_keys, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, (hipStream_t)stream, feats, T, n,
                       keys);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}

extern "C" int fjsp_a2c_group_verify(const float* feats, int32_t T, int32_t n, const int64_t* rep_a,
                                     const int64_t* rep_c, int32_t* bad, void* stream) {
    if (T <= 0 || n <= 0) return fjsp_internal_fail("fjsp_a2c_group_verify: T and n must be > 0");
    if (!feats || !rep_a || !rep_c || !bad) return fjsp_internal_fail("fjsp_a2c_group_verify: null buffer");
    const size_t S = (size_t)T * (size_t)n;
    hipLaunchKernelGGL(k_group_verify, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, (hipStream_t)stream, feats, T,
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

extern "C" int fjsp_a2c_policy(const float* feats, const int8_t* masks, int32_t n, const float* actor_w,
                               const float* critic_w, const uint64_t* seed, uint32_t env_gid0, uint32_t step,
                               int32_t deterministic,
                               uint8_t* actions, float* values, float* probs, void* stream) {
    if (n <= 0) return fjsp_internal_fail("fjsp_a2c_policy: n must be > 0");
    if (!feats || (!actions && !values) || (values && !critic_w) || (actions && (!masks || !actor_w || !seed)))
        return fjsp_internal_fail("fjsp_a2c_policy: null buffer");
    // roles: y = 0 the critic, 1..8 the actors; without actions only the critic (values), without
    // values only the actors
    const int role0 = values ? 0 : 1, role1 = actions ? NAG + 1 : 1;
    dim3 grid((n + TILE - 1) / TILE, role1 - role0);
    hipLaunchKernelGGL(k_policy, grid, dim3(NTHR), 0, (hipStream_t)stream, feats, masks, n, actor_w, critic_w, seed, env_gid0,
                       step, deterministic, actions, values, probs, role0);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}
