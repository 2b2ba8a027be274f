// fjsp_stepdev.h — device side of one env step shared by the step kernels (fjsp_hip.hip) and the
// fused policy + step kernel of the A2C collect (fjsp_policy.hip): the HBM state layout
// (DevState), the per-env MT19937 stream and reset, the observation sinks and step_and_emit
// (FJSPSimulation.step, FJSPSimulation.py:144-242, on the fjsp_env.h state machine).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fjsp_env.h"
#include "fjsp_stamps.h"
#include "../../include/fjsp.h"

namespace fjsp {

constexpr int BLOCK = 64;
constexpr int MT_N = 624;

struct DevState {
    uint32_t* words;
    uint32_t* orders;
    uint16_t* scode;
    uint8_t* snext;
    uint16_t* scstep;
    uint32_t* mt;       // [2][n][624] MT rows (live one selected by W3 bit 31)
    uint32_t* nxt;      // [MAX_ORDERS][n] pre-drawn next order tables (W[PGW])
    int n;
};
// Handle words after the state rows ([NWORDS][n] u32 + AUX_WORDS): the fault word (fjsp_faults:
// bit 0 = a bounded hand-off wait gave up) and the bound of those waits (option "spin_cap").
// Not kernel arguments: a pointer or a field more in DevState / Cfg, live through the step loops,
// pushed k_step_ag into SGPR spills (+6 % per step, measured).
// AUX_TEST_STALL: test option "test_stall" (tests/test_gpu_agents.py), see stall_for_test.
constexpr int AUX_WORDS = 4, AUX_FAULT = 0, AUX_SPIN_CAP = 1, AUX_TEST_STALL = 2;
__device__ __forceinline__ uint32_t* aux_words(const DevState& S) { return S.words + (size_t)NWORDS * S.n; }
// Test option "test_stall" = s: the wave that owns a multi-wave workgroup's hand-offs sleeps
// s x 127 x 64 cycles before its first step (called for workgroup 0 only, once per launch), so
// the other waves' bounded waits for its first post give up — the give-up path under test.  One
// scalar load per launch; nothing in the step loops.
__device__ __forceinline__ void stall_for_test(const DevState& S) {
    const uint32_t s = aux_words(S)[AUX_TEST_STALL];
    for (uint32_t i = 0; i < s; i++) __builtin_amdgcn_s_sleep(127);
}

// ---------------------------------------------------------------- load / store of Env
// The register state is the HBM row layout itself (fjsp_env.h, struct Env): 30 coalesced words.
__device__ __forceinline__ void env_load(Env& E, const uint32_t* __restrict__ w, int n, int e) {
#pragma unroll
    for (int i = 0; i < NSTATE; i++) E.w[i] = w[i * n + e];
}
__device__ __forceinline__ void env_store(const Env& E, uint32_t* __restrict__ w, int n, int e) {
#pragma unroll
    for (int i = 0; i < NSTATE; i++) w[i * n + e] = E.w[i];
}
static_assert(NWORDS >= NSTATE, "state buffer rows");

// ---------------------------------------------------------------- MT19937, lazily twisted
// Per-env state: 624 words, env-major (row e = mt + e * 624, 16-byte aligned), so the words a
// lane streams through are contiguous for that lane (lanes of a wave sit at different stream
// positions: a word-major layout would make every load touch 64 rows).
// Cursor word W3: mti (bits 0..9) | g (bits 16..25).  Words [0, g) of the row already hold the
// current block, [g, 624) still the previous one; mti <= g is the next word to consume.
// Word i of a new block is generated on demand with the same in-place recurrence as numpy's
// sequential twist (mt[i+1] is still old, mt[i+397 mod 624] is new iff i >= 227), so the k-th
// draw equals numpy's k-th draw.
// Standard numpy (key, pos): pos == 624 <-> (mti, g) = (0, 0); pos < 624 <-> (pos, 624).
__device__ inline void mt_seed(uint32_t* __restrict__ mt, int e, uint32_t seed) {
    uint4* row = reinterpret_cast<uint4*>(mt + (size_t)e * MT_N);
    uint32_t x = seed;
    for (int q = 0; q < MT_N / 4; q++) {
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int i = 4 * q + j;
            if (i > 0) x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)i;
            v[j] = x;
        }
        row[q] = make_uint4(v[0], v[1], v[2], v[3]);
    }
}

// Batched reader of the lazily twisted stream for resets.  A refill of B words starts at the
// 16-byte aligned word pa = pos & ~3 and loads the words it needs as two runs of B/4 + 1 uint4
// (words [pa, pa+B+4) and [pa+396, pa+B+400), wrapped into the row; 624 is a multiple of 4
// so no uint4 straddles the wrap), regenerates the words at or past g, writes the batch back
// as uint4 (words before g are written back unchanged) and returns the B tempered words in
// registers; the pos - pa words before pos are skipped by the consumer.  cnt = words of the
// batch inside the row (a multiple of 4; a batch never crosses the wrap).
constexpr int MTB = 32;

// the two runs of a refill at pa (mt_batch), as uint4
template <int B>
__device__ __forceinline__ void mt_load(const uint32_t* __restrict__ roww, int pa, uint4 (&va)[(B + 4) / 4],
                                        uint4 (&vc)[(B + 4) / 4]) {
    const uint4* row = reinterpret_cast<const uint4*>(roww);
#pragma unroll
    for (int q = 0; q < (B + 4) / 4; q++) {
        int ia = pa + 4 * q;
        ia = ia >= MT_N ? ia - MT_N : ia;
        int ic = pa + 396 + 4 * q;
        ic = ic >= MT_N ? ic - MT_N : ic;
        ic = ic >= MT_N ? ic - MT_N : ic;
        va[q] = row[ia >> 2];
        vc[q] = row[ic >> 2];
    }
}

// mt_batch on runs already loaded (mt_load at pa = pos & ~3, no store to them since)
template <int B>
__device__ __forceinline__ void mt_batch_loaded(uint32_t* __restrict__ roww, int pos, int& g, uint32_t (&v)[B], int& pa,
                                                int& cnt, const uint4 (&va)[(B + 4) / 4], const uint4 (&vc)[(B + 4) / 4]) {
    uint4* row = reinterpret_cast<uint4*>(roww);
    pa = pos & ~3;
    cnt = (MT_N - pa) < B ? (MT_N - pa) : B;
    uint32_t a[B + 4], c[B + 4];
#pragma unroll
    for (int q = 0; q < (B + 4) / 4; q++) {
        a[4 * q] = va[q].x; a[4 * q + 1] = va[q].y; a[4 * q + 2] = va[q].z; a[4 * q + 3] = va[q].w;
        c[4 * q] = vc[q].x; c[4 * q + 1] = vc[q].y; c[4 * q + 2] = vc[q].z; c[4 * q + 3] = vc[q].w;
    }
    uint32_t w[B];
#pragma unroll
    for (int j = 0; j < B; j++) {
        const uint32_t y = (a[j] & 0x80000000u) | (a[j + 1] & 0x7fffffffu);   // a[cnt] = word 0 at the wrap
        const uint32_t regen = c[j + 1] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);   // word pa + j + 397
        const uint32_t stale = (uint32_t)((pa + j - g) >> 31);   // all ones iff word pa + j < g (already current)
        w[j] = (regen & ~stale) | (a[j] & stale);   // bitwise: no branch per word
        uint32_t t = w[j];
        t ^= t >> 11;
        t ^= (t << 7) & 0x9d2c5680u;
        t ^= (t << 15) & 0xefc60000u;
        t ^= t >> 18;
        v[j] = t;
    }
#pragma unroll
    for (int q = 0; q < B / 4; q++)
        if (4 * q < cnt) row[(pa >> 2) + q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
    if (pa + cnt > g) g = pa + cnt;
}

template <int B>
__device__ __forceinline__ void mt_batch(uint32_t* __restrict__ roww, int pos, int& g, uint32_t (&v)[B], int& pa,
                                         int& cnt) {
    uint4 va[(B + 4) / 4], vc[(B + 4) / 4];
    mt_load<B>(roww, pos & ~3, va, vc);
    mt_batch_loaded<B>(roww, pos, g, v, pa, cnt, va, vc);
}

// generate_order (FJSPSimulation.py:101-131) as a state machine over the stream: per order
// randint(1, 10) then choice(ProductType) then choice(PackagingColor) (:107,111-112) with
// numpy's masked rejection: rng 8 / mask 15 for the product count (field k = 0), rng 2 /
// mask 3 for type and colour (k = 1, 2).
struct OrderDraw {
    int o, k, np, ty;
    uint32_t last;
};

// Consume words [skip, cnt) of one batch (straight-line selects, no per-draw branch) until
// `num_orders` orders are complete; returns the words consumed.  The order word is stored
// every draw, to slot o (overwritten later by order o's own store) or, once the table is
// complete, as the unchanged last order.
template <int B>
__device__ __forceinline__ int draw_orders(const uint32_t (&v)[B], int skip, int cnt, int num_orders, OrderDraw& d,
                                           uint32_t* orders, int stride) {
    int used = 0;
#pragma unroll
    for (int j = 0; j < B; j++) {
        const bool act = j >= skip && j < cnt && d.o < num_orders;
        const uint32_t x = v[j] & (d.k == 0 ? 15u : 3u);
        const bool acc = act && x <= (d.k == 0 ? 8u : 2u);
        const bool emit = acc && d.k == 2;
        d.np = (acc && d.k == 0) ? 1 + (int)x : d.np;
        d.ty = (acc && d.k == 1) ? 1 + (int)x : d.ty;
        const uint32_t ow = ow_make(d.np, d.ty, 1 + (int)x);
        d.last = emit ? ow : d.last;
        orders[(d.o < num_orders ? d.o : num_orders - 1) * stride] = d.last;
        d.o += emit ? 1 : 0;
        d.k = acc ? (d.k == 2 ? 0 : d.k + 1) : d.k;
        used += act ? 1 : 0;
    }
    return used;
}

// MT rows: two per env ([2][N][624]); bit 31 of the cursor word W3 selects the live one (the
// other is the pre-draw wave's working copy, see k_step_pipe).  W[PGW] = the pre-draw record:
// 0, or ready (bit 0) | cursor after the pre-drawn orders (mti bits 1..10, g bits 11..20) |
// row (bit 21) | num_orders (bits 24..30), with the orders in S.nxt.
constexpr int PGW = NSTATE;
static_assert(NWORDS > PGW, "state buffer rows");
__device__ __forceinline__ uint32_t* mt_row(const DevState& S, uint32_t w3, int e) {
    return S.mt + ((size_t)(w3 >> 31) * S.n + e) * MT_N;
}

// FJSPSimulation.reset body after the optional reseed (FJSPSimulation.py:301-320): clear the
// env and draw num_orders orders from the env's live MT row.  clear_pg: drop a pre-drawn
// next table (it was drawn from the stream position this reset consumes).
__device__ __forceinline__ void env_reset(Env& E, const Tables& T, const Cfg& C, const DevState& S, int e,
                                          int num_orders, bool clear_pg = true) {
    env_clear(E, C);
    E.set_norders(num_orders);
    const uint32_t w3 = (uint32_t)E.mti();
    uint32_t* roww = mt_row(S, w3, e);
    int pos = (int)(w3 & 0x3FF), g = (int)((w3 >> 16) & 0x3FF);
    OrderDraw d{0, 0, 0, 0, 0u};
    while (d.o < num_orders) {
        uint32_t v[MTB];
        int pa, cnt;
        mt_batch<MTB>(roww, pos, g, v, pa, cnt);
        pos += draw_orders<MTB>(v, pos - pa, cnt, num_orders, d, T.orders, T.stride);
        if (pos == MT_N) { pos = 0; g = 0; }
    }
    E.set_mti((int)((uint32_t)pos | ((uint32_t)g << 16) | (w3 & 0x80000000u)));
    if (clear_pg) S.words[(size_t)PGW * S.n + e] = 0u;
}

// reset(seed=None) from a pre-drawn table (lane's slots nxt[o * BLOCK]): the same state as
// env_reset, the stream position and live row taken from the pre-draw.
__device__ __forceinline__ void env_reset_predrawn(Env& E, const Tables& T, const Cfg& C, int num_orders,
                                                   uint32_t w3, const uint32_t* nxt) {
    env_clear(E, C);
    E.set_norders(num_orders);
    for (int o = 0; o < num_orders; o++) T.orders[o * T.stride] = nxt[o * BLOCK];
    E.set_mti((int)w3);
}

// Auto-reset inside the step kernels is a cold path (once per ~200 steps), taken in a branch.
// Inlined: a call would need a stack frame in scratch memory (368 B per lane: the by-value
// state and the callee-saved registers), and a kernel that uses scratch pays for its set-up
// on every launch (measured: k_step 12.1 -> 7.9 us per launch in rocprof) and its allocation
// raised every step kernel to 228+ VGPRs (157-233 inlined).
__device__ __forceinline__
Env env_reset_cold(Env E, Tables T, Cfg C, DevState S, int e, int num_orders, bool clear_pg = true) {
    env_reset(E, T, C, S, e, num_orders, clear_pg);
    return E;
}

__device__ __forceinline__ Tables tables_of(const DevState& S, int e) {
    Tables T;
    T.orders = S.orders + e;
    T.scode = S.scode + e;
    T.snext = S.snext + e;
    T.scstep = S.scstep + e;
    T.stride = S.n;
    return T;
}

// Output byte offsets are 32-bit (the host checks every output slab is < 4 GiB), so the
// stores use the SGPR-base + 32-bit VGPR-offset form instead of 64-bit per-lane addresses.
template <class V>
__device__ __forceinline__ void st32(V* base, uint32_t elem, V v) {
    *reinterpret_cast<V*>(reinterpret_cast<char*>(base) + elem * (uint32_t)sizeof(V)) = v;
}
// a2c feature column of each observation field (a2c.py:137-166: agents in order, keys sorted,
// action_mask dropped); checked against spec.a2c_feature_index by fjsp_a2c_layout's test.
constexpr int NFEAT = 38;
constexpr int8_t FEAT_OF_I32[NI32] = {5, 6, 4, 3, 2, 0, 1, 11, 12, 9, 18, 19, 17, 16, 10, 13, 7, 14, 8, 15};
constexpr int8_t FEAT_OF_I8[NI8] = {20, 22, 23, 25, 26, 28, 29, 31, 32, 34, 35, 37};
constexpr int8_t FEAT_OF_F32[NF32] = {21, 24, 27, 30, 33, 36};

// Sink that stores each observation field as soon as it is computed (fjsp_env.h observe()).
struct StoreSink {
    int32_t* pi32; int8_t* pi8; float* pf32; int8_t* pmk;
    uint32_t t, n, e;
    float* pfeat = nullptr;   // optional a2c features [T][38][N]
    __device__ __forceinline__ void feat(int c, float v) { if (pfeat) st32(pfeat, (t * NFEAT + (uint32_t)c) * n + e, v); }
    __device__ __forceinline__ void i32(int f, int v) {
        if (pi32) st32(pi32, (t * NI32 + (uint32_t)f) * n + e, (int32_t)v);
        feat(FEAT_OF_I32[f], (float)v);
    }
    __device__ __forceinline__ void i8(int f, int v) {
        if (pi8) st32(pi8, (t * NI8 + (uint32_t)f) * n + e, (int8_t)v);
        feat(FEAT_OF_I8[f], (float)(int8_t)v);
    }
    __device__ __forceinline__ void f32(int f, float v) {
        if (pf32) st32(pf32, (t * NF32 + (uint32_t)f) * n + e, v);
        feat(FEAT_OF_F32[f], v);
    }
    __device__ __forceinline__ void mask(int f, int v) { if (pmk) st32(pmk, (t * NMASK + (uint32_t)f) * n + e, (int8_t)v); }
};


// fmix64 counter RNG for synthetic actions (oracle_actions spec)
__device__ __forceinline__ uint64_t fmix64(uint64_t z) {
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z;
}

// FULL = false: only obs, masks, rewards, term, trunc and status are written (the other
// fjsp_out pointers are never read, so they take no SGPRs in the hot loop).
template <bool CANON, bool FULL = true>
__device__ __forceinline__ void step_and_emit(Env& E, const Tables& T, const Cfg& C, const DevState& S, int e,
                                              const int* act, const uint8_t* order, int autoreset, const fjsp_out& out,
                                              uint32_t t) {
    const uint32_t n = (uint32_t)S.n, ue = (uint32_t)e;
    uint32_t res[NA];
    const double g8 = env_advance<CANON>(E, T, C, act, order, res);
    if (out.rewards) {
#pragma unroll
        for (int a = 0; a < NA; a++) st32(out.rewards, (t * NA + (uint32_t)a) * n + ue, g8 + local_reward(C, a, res[a], act[a]));
    }
    if (FULL && out.results) {
#pragma unroll
        for (int a = 0; a < NA; a++) st32(out.results, (t * NA + (uint32_t)a) * n + ue, res[a]);
    }
    FJSP_STAMP(E, 3);
    StoreSink sink{out.obs_i32, out.obs_i8, out.obs_f32, out.masks, t, n, ue};
    observe(E, C, sink);
    FJSP_STAMP(E, 4);
    const int nord = E.norders();
    const int all_done = E.ncompleted() == nord && nord > 0 && E.next_order() == nord;
    const int truncated = E.step() >= C.max_steps;
    if (out.term) st32(out.term, t * n + ue, (uint8_t)all_done);
    if (out.trunc) st32(out.trunc, t * n + ue, (uint8_t)truncated);
    if (FULL && out.orders_completed) st32(out.orders_completed, t * n + ue, E.ncompleted());
    if (FULL && out.packaged) st32(out.packaged, t * n + ue, E.total_packaged());
    if (FULL && out.sim_time) st32(out.sim_time, t * n + ue, (double)(E.step() + 1) * (double)C.step_size);
    if (out.status) st32(out.status, t * n + ue, E.status());
    FJSP_STAMP(E, 5);
    E.set_step(E.step() + 1);
    if (autoreset && (all_done || truncated))
        E = env_reset_cold(E, T, C, S, e, nord);   // reset(seed=None) continues the MT stream
    if (FULL && (out.next_i32 || out.next_i8 || out.next_f32 || out.next_masks || out.feats)) {
        StoreSink nsink{out.next_i32, out.next_i8, out.next_f32, out.next_masks, t, n, ue, out.feats};
        observe(E, C, nsink);
    }
    FJSP_STAMP(E, 6);
}

}  // namespace fjsp

// fjsp_policy.hip: the launch of the fused policy + step kernel (fjsp_a2c_policy_step) over the
// envs [env_begin, env_begin + env_count) (env_begin a multiple of 64); tile_cnt [ceil(n / 64)]
// arrival counters (zero between launches), tile_act [ceil(n / 64)][8][16] words.
int fjsp_internal_policy_step(const float* feats, const int8_t* masks, int32_t n, const float* actor_w,
                              const float* critic_w, const uint64_t* seed, uint32_t env_gid0, uint32_t step,
                              int32_t deterministic, uint8_t* actions, float* values, const fjsp::DevState& S,
                              const fjsp::Cfg& C, const fjsp_out& out, uint32_t* tile_cnt, uint32_t* tile_act,
                              int32_t autoreset, int32_t env_begin, int32_t env_count, hipStream_t stream);
