// fjsp_hip.hip — HIP kernels (gfx950) and the C-ABI of libfjsp.so (include/fjsp.h).
//
// Layout in HBM (all SoA, N = number of envs, lane e of a wavefront = env e):
//   words  u32 [NWORDS][N]        packed register state of fjsp::Env (pack/unpack below)
//   orders u32 [64][N]            order table (processed/packaged masks, n, type, colour)
//   scode  u16 [255][N]           tray-slot arena: tray code
//   snext  u8  [255][N]           tray-slot arena: next slot of the FIFO the slot is in
//   scstep u16 [255][N]           tray-slot arena: completion step of an in-flight run
//   mt     u32 [N][624]           per-env MT19937 state (numpy legacy RandomState), env-major
// Kernels: one lane per env, 64-lane workgroups (one wavefront; 4096 envs -> 64 CUs).
//   k_reset      FJSPSimulation.reset (FJSPSimulation.py:286-323)
//   k_step       FJSPSimulation.step  (FJSPSimulation.py:144-242), actions from HBM
//   k_step_many  K fused steps with on-device counter-RNG actions
//   k_gae        transition_memory.py:83-105 (returns + GAE), one lane per (agent, env) column
// Compiled with -ffp-contract=off: rewards and GAE follow Python's unfused fp64 op order.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#include <string>
#include <type_traits>

#include "fjsp_env.h"
#include "fjsp_stamps.h"
#include "fjsp_stepdev.h"
#include "../../include/fjsp.h"

using namespace fjsp;

namespace {

// diagnostic builds only (fjsp_stamps.h)
FJSP_DIAG(__device__ unsigned long long g_stamps[8];
          __device__ unsigned long long g_pgstamps[4];     // pre-draw wave: busy cycles, active steps, busy in active steps, steps
          __device__ unsigned long long g_emitstamps[4];   // emit waves 1, 2: busy cycles, steps
          __device__ unsigned long long g_agstamps[64];)   // k_step_ag per wave [busy, wait] cycles, marks (scripts/diag_ag_stamps.py)

// Bounded wait of one wave for a hand-off flag another wave of its workgroup releases.  The
// waves of a workgroup are co-resident, so a correct kernel always gets there; the bound turns a
// hand-off bug into a flagged launch (ST_SPIN_TIMEOUT on the workgroup's envs, the handle's fault
// word) instead of a device hang.  Once one wait of the workgroup gave up (*abort) the others
// stop waiting too, after at most 256 more sleeps each (so the bound is a multiple of 256
// sleeps, at least 256).  abort and cap live in LDS and are read
// only every 256 sleeps: nothing of the bound stays live in registers across the step loop (a
// cap held in an SGPR through the loop pushed the multi-wave kernels into SGPR spills, +6 %).
__device__ __forceinline__ void spin_until(uint32_t* flag, uint32_t v, uint32_t* abort, const uint32_t* cap) {
    for (uint32_t it = 1; __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != v; it++) {
        if ((it & 255u) == 0u) {
            if (it >= *cap || __hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                __hip_atomic_store(abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                break;
            }
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// Env block of workgroup b of nb.  Workgroups are dealt to the 8 XCDs round-robin (b -> XCD
// b % 8, MI355X_MICROARCH.md), and each XCD has its own L2.  With few envs per workgroup the
// byte fields of 8 consecutive env blocks share one 128-B line of an output row: mapping them to
// one XCD lets its L2 merge the partial lines into whole ones before they go to HBM (dealt
// round-robin, 8 L2s each wrote back a 16-B piece of every line).  Only the speed depends on the
// dispatch order; any b -> block bijection gives the same results.
__device__ __forceinline__ int xcd_block(int b, int nb) {
    return (nb & 7) ? b : (b & 7) * (nb >> 3) + (b >> 3);
}

// The workgroup's give-up flag into the handle's fault word (one lane; a vector atomic).
__device__ __forceinline__ void report_abort(const DevState& S, uint32_t abort) {
    if (abort) __hip_atomic_fetch_or(aux_words(S) + AUX_FAULT, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


__global__ void __launch_bounds__(BLOCK) k_seed(DevState S, const uint32_t* __restrict__ seeds, uint32_t seed_base) {
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= S.n) return;
    mt_seed(S.mt, e, seeds ? seeds[e] : seed_base + (uint32_t)e);
    S.words[3 * S.n + e] = 0;
    S.words[(size_t)PGW * S.n + e] = 0;
}

__global__ void __launch_bounds__(BLOCK) k_reset(DevState S, Cfg C, const uint32_t* __restrict__ seeds,
                                                 const uint8_t* __restrict__ env_mask, int num_orders, fjsp_out out) {
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= S.n) return;
    if (env_mask && !env_mask[e]) return;
    Tables T = tables_of(S, e);
    Env E;
    int mti = (int)S.words[3 * S.n + e];
    if (seeds) { mt_seed(S.mt, e, seeds[e]); mti = 0; }
    E.set_mti(mti);
    env_reset(E, T, C, S, e, num_orders);
    StoreSink sink{out.obs_i32, out.obs_i8, out.obs_f32, out.masks, 0u, (uint32_t)S.n, (uint32_t)e, out.feats};
    observe(E, C, sink);
    env_store(E, S.words, S.n, e);
    if (out.status) out.status[e] = E.status();
}

// fjsp_pack_a2c: features + masks of the current observation (no state change)
__global__ void __launch_bounds__(BLOCK) k_pack(DevState S, Cfg C, float* __restrict__ feats, int8_t* __restrict__ masks) {
    const int e = blockIdx.x * BLOCK + threadIdx.x;
    if (e >= S.n) return;
    Env E;
    env_load(E, S.words, S.n, e);
    StoreSink sink{nullptr, nullptr, nullptr, masks, 0u, (uint32_t)S.n, (uint32_t)e, feats};
    observe(E, C, sink);
}

__device__ __forceinline__ void synth_uniform(uint64_t seed, uint32_t gid, uint32_t step, int* act) {
    const uint64_t h = fmix64(seed ^ fmix64(((uint64_t)gid << 32) | step));
    const int nact[NA] = {3, 8, 3, 3, 3, 3, 3, 3};
#pragma unroll
    for (int a = 0; a < NA; a++) act[a] = (int)((((uint32_t)(h >> (8 * a)) & 0xFFu) * (uint32_t)nact[a]) >> 8);
}

__device__ __forceinline__ void synth_actions(uint64_t seed, uint32_t gid, uint32_t step, int mode, const Env& E,
                                              const Tables& T, const Cfg& C, int* act) {
    if (mode == FJSP_ACTIONS_HEURISTIC) {
        heuristic_actions(E, T, act);
        return;
    }
    if (mode == FJSP_ACTIONS_UNMASKED) {
        synth_uniform(seed, gid, step, act);
        return;
    }
    const uint64_t h = fmix64(seed ^ fmix64(((uint64_t)gid << 32) | step));
    MaskBits mb;
    compute_masks(E, C, mb);
#pragma unroll
    for (int a = 0; a < NA; a++) {
        const uint32_t bits = mb.bits[a];
        const int cnt = __popc(bits);
        int j = (int)((((uint32_t)(h >> (8 * a)) & 0xFFu) * (uint32_t)cnt) >> 8);
        // j-th set bit
        uint32_t b = bits;
        for (int k = 0; k < j; k++) b &= b - 1u;
        act[a] = __ffs(b) - 1;
    }
}

// One full env step + outputs at trajectory index t; handles auto-reset.
// Per-wave LDS staging tile of one step's lean outputs ([F][64] per field block).  The step
// writes it with ds_write (StageSink), then the wave copies each block out as whole 16-byte
// chunks: ~15 global_store_dwordx4 (every instruction 1 KiB contiguous) instead of ~85
// scalar-per-lane stores.  Requires N % 64 == 0 and 16-byte aligned outputs (host-checked).
struct alignas(16) StageTile {
    int32_t i32[NI32 * BLOCK];
    float f32[NF32 * BLOCK];
    double rew[NA * BLOCK];
    uint32_t status[BLOCK];
    int8_t i8[NI8 * BLOCK];
    int8_t mask[NMASK * BLOCK];
    uint8_t term[BLOCK];
    uint8_t trunc[BLOCK];
};
struct StageSink {
    StageTile* tl;
    int lane;
    __device__ __forceinline__ void i32(int f, int v) { tl->i32[f * BLOCK + lane] = v; }
    __device__ __forceinline__ void i8(int f, int v) { tl->i8[f * BLOCK + lane] = (int8_t)v; }
    __device__ __forceinline__ void f32(int f, float v) { tl->f32[f * BLOCK + lane] = v; }
    __device__ __forceinline__ void mask(int f, int v) { tl->mask[f * BLOCK + lane] = (int8_t)v; }
};
// Copy ROWS rows of ROWBYTES from the tile to global rows spaced `gstride` bytes apart.
template <int ROWS, int ROWBYTES>
__device__ __forceinline__ void copy_rows(const void* tile, void* gbase, size_t gstride, int lane) {
    constexpr int CPR = ROWBYTES / 16;
    constexpr int TOTAL = ROWS * CPR;
    const uint8_t* src = (const uint8_t*)tile;
    uint8_t* dst = (uint8_t*)gbase;
#pragma unroll
    for (int c0 = 0; c0 < TOTAL; c0 += BLOCK) {
        const int c = c0 + lane;
        if (c < TOTAL) {
            const int r = c / CPR, off = (c - r * CPR) * 16;
            const uint4 v = *(const uint4*)(src + r * ROWBYTES + off);
            *(uint4*)(dst + (size_t)r * gstride + off) = v;
        }
    }
}
__device__ __forceinline__ void copy_out(const StageTile& tl, const fjsp_out& out, uint32_t t, size_t n, int blk,
                                         int lane) {
    const size_t col = (size_t)blk * BLOCK;
    if (out.obs_i32) copy_rows<NI32, 4 * BLOCK>(tl.i32, out.obs_i32 + (size_t)t * NI32 * n + col, n * 4, lane);
    if (out.obs_f32) copy_rows<NF32, 4 * BLOCK>(tl.f32, out.obs_f32 + (size_t)t * NF32 * n + col, n * 4, lane);
    if (out.rewards) copy_rows<NA, 8 * BLOCK>(tl.rew, out.rewards + (size_t)t * NA * n + col, n * 8, lane);
    if (out.status) copy_rows<1, 4 * BLOCK>(tl.status, out.status + (size_t)t * n + col, n * 4, lane);
    if (out.obs_i8) copy_rows<NI8, BLOCK>(tl.i8, out.obs_i8 + (size_t)t * NI8 * n + col, n, lane);
    if (out.masks) copy_rows<NMASK, BLOCK>(tl.mask, out.masks + (size_t)t * NMASK * n + col, n, lane);
    if (out.term) copy_rows<1, BLOCK>(tl.term, out.term + (size_t)t * n + col, n, lane);
    if (out.trunc) copy_rows<1, BLOCK>(tl.trunc, out.trunc + (size_t)t * n + col, n, lane);
}

// Lean + LDS-staged variant of step_and_emit (obs, masks, rewards, term, trunc, status).
__device__ __forceinline__ void step_and_emit_staged(Env& E, const Tables& T, const Cfg& C, const DevState& S, int e,
                                                     const int* act, int autoreset, const fjsp_out& out, uint32_t t,
                                                     StageTile* tl, int lane) {
    uint32_t res[NA];
    const double g8 = env_advance<true>(E, T, C, act, nullptr, res);
#pragma unroll
    for (int a = 0; a < NA; a++) tl->rew[a * BLOCK + lane] = g8 + local_reward(C, a, res[a], act[a]);
    FJSP_STAMP(E, 3);
    StageSink sink{tl, lane};
    observe(E, C, sink);
    FJSP_STAMP(E, 4);
    const int nord = E.norders();
    const int all_done = E.ncompleted() == nord && nord > 0 && E.next_order() == nord;
    const int truncated = E.step() >= C.max_steps;
    tl->term[lane] = (uint8_t)all_done;
    tl->trunc[lane] = (uint8_t)truncated;
    tl->status[lane] = E.status();
    __syncthreads();
    copy_out(*tl, out, t, (size_t)S.n, blockIdx.x, lane);
    __syncthreads();
    FJSP_STAMP(E, 5);
    E.set_step(E.step() + 1);
    if (autoreset && (all_done || truncated))
        E = env_reset_cold(E, T, C, S, e, nord);   // reset(seed=None) continues the MT stream
    FJSP_STAMP(E, 6);
}

// EPW: envs per workgroup (64, 32 or 16; lanes >= EPW idle; option "step_envs").  Fewer envs per
// wave would shorten the union of the lanes' branches and spread 4 096 envs over all 256 CUs; it
// measured slower (fjsp_step), so 64 stays the default.
template <bool CANON, int EPW>
__global__ void __launch_bounds__(BLOCK) k_step(DevState S, Cfg C, const uint8_t* __restrict__ actions, uint64_t order_packed,
                                                int autoreset, fjsp_out out) {
    FJSP_DIAG(
    const uint64_t t_entry = __builtin_amdgcn_s_memtime();
    )
    __shared__ double s_lut[RLUT_SIZE];
    const int e = blockIdx.x * EPW + threadIdx.x;
    const bool valid = (int)threadIdx.x < EPW && e < S.n;
    // the state and action loads are issued before the reward table's: one HBM round trip
    Env E;
    int act[NA];
    if (valid) {
        env_load(E, S.words, S.n, e);
#pragma unroll
        for (int a = 0; a < NA; a++) act[a] = actions[a * S.n + e];
    }
    for (int i = threadIdx.x; i < RLUT_SIZE; i += BLOCK) s_lut[i] = C.lut[i];
    __syncthreads();
    C.lut = s_lut;
    if (!valid) return;
    FJSP_DIAG(
    const uint64_t t_lut = __builtin_amdgcn_s_memtime();
    )
    Tables T = tables_of(S, e);
    uint8_t order[NA];
#pragma unroll
    for (int i = 0; i < NA; i++) order[i] = (uint8_t)(order_packed >> (8 * i));
    // stamp slots: 0 entry -> LUT -> state + action loads landed, 1 action phase, 2 run,
    // 3 rewards, 4 observe, 5 term / trunc / status, 6 auto-reset + next obs, 7 state store drained
    FJSP_DIAG(
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int i = 0; i < 8; i++) E.st_acc[i] = 0;
    E.st_t0 = __builtin_amdgcn_s_memtime();
    E.st_acc[0] = E.st_t0 - t_entry;
    (void)t_lut;
                     )
    step_and_emit<CANON>(E, T, C, S, e, act, order, autoreset, out, 0);
    env_store(E, S.words, S.n, e);
    FJSP_DIAG(
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    FJSP_STAMP_AT(E, 7);
    if (threadIdx.x == 0)
        for (int i = 0; i < 8; i++) atomicAdd((unsigned long long*)&g_stamps[i], (unsigned long long)E.st_acc[i]);
    )
}

// ---------------------------------------------------------------- step server (fjsp_server_*)
// The one-launch-per-step path pays a launch, a cold chip and a stream synchronisation per step
// (k_step: 6.8 us of kernel time for ONE env, the facade 18.8 us of launch + sync).  The server is
// a persistent k_step: each workgroup keeps its 64 envs' state words in registers and the reward
// table in LDS, and steps them whenever the host bumps a doorbell word in host memory; the host
// waits for every workgroup's done word.  No launch, no stream operation per step; the tables stay
// warm in L2.  Control block: host memory (hipHostMalloc, coherent, mapped), one per handle.
constexpr int SRV_MAX_WG = 256;   // 16 384 envs
struct alignas(64) ServerCtl {
    uint32_t seq;                  // host: the step requested (monotonic)
    uint32_t stop;                 // host: leave now (the state words are written back)
    uint32_t inbox[4];             // host, one-env inline mode: (seq & 0xFFFF) << 16 | two action bytes each
    uint32_t pad[10];
    uint32_t done[SRV_MAX_WG];     // kernel: the last seq each workgroup completed
    uint32_t exited[SRV_MAX_WG];   // kernel: the epoch of the launch that left
};

// Exit conditions every wave reaches: the stop word, or idle_ticks of the 100 MHz clock without a
// new request (the host relaunches well before that: fjsp_server_step's restart_ms); a step itself
// is bounded straight-line code.  Only lane 0 of workgroup 0 polls the host's words (system-scope
// loads over the bus, all of one poll issued together: one bus round trip per poll); it relays
// each request (and a stop) through two device words, relay[0] = the request, relay[1] = stop,
// which the other workgroups' lane 0 poll in L2 (both set by the host before the launch:
// relay[0] = start_seq, relay[1] = 0).  Inline mode (actions == nullptr, one env): the request's
// eight action bytes ride in the doorbell's cache line (ctl->inbox, each word tagged with the
// request's low 16 bits), so the poll that sees the request also has its actions — no second
// round trip to read them.
__global__ void __launch_bounds__(BLOCK) k_step_server(DevState S, Cfg C, ServerCtl* ctl, uint32_t* relay,
                                                       const uint8_t* actions, int autoreset, fjsp_out out,
                                                       uint32_t start_seq, uint32_t epoch, uint64_t idle_ticks) {
    __shared__ double s_lut[RLUT_SIZE];
    const int lane = threadIdx.x;
    const int e = blockIdx.x * BLOCK + lane;
    const bool valid = e < S.n;
    Env E;
    if (valid) env_load(E, S.words, S.n, e);
    for (int i = lane; i < RLUT_SIZE; i += BLOCK) s_lut[i] = C.lut[i];
    __syncthreads();
    C.lut = s_lut;
    const Tables T = tables_of(S, valid ? e : 0);
    uint32_t last = start_seq;
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const bool inline_act = actions == nullptr;
    uint32_t ib[4] = {0u, 0u, 0u, 0u};
    for (;;) {
        uint32_t sq = last, quit = 0;
        if (lane == 0 && blockIdx.x == 0) {
            for (;;) {
                // relaxed loads issued together (the acquire fence below orders what follows)
                sq = __hip_atomic_load(&ctl->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                const uint32_t stop = __hip_atomic_load(&ctl->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                bool got = sq != last;
                if (inline_act) {
#pragma unroll
                    for (int k = 0; k < 4; k++)
                        ib[k] = __hip_atomic_load(&ctl->inbox[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    // the host writes the inbox before seq: every tag = the next request's means
                    // its actions are complete (a poll that saw seq but not yet the inbox polls again)
                    const uint32_t tag = (last + 1u) & 0xFFFFu;
                    got = (ib[0] >> 16) == tag && (ib[1] >> 16) == tag && (ib[2] >> 16) == tag && (ib[3] >> 16) == tag;
                    sq = last + 1u;
                }
                if (got) {
                    __hip_atomic_store(&relay[0], sq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                if (stop || __builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) {
                    __hip_atomic_store(&relay[1], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                    quit = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        } else if (lane == 0) {
            for (;;) {
                sq = __hip_atomic_load(&relay[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                if (sq != last) break;
                // the relay's stop, or this workgroup's own idle bound (a backstop: workgroup 0
                // relays every stop and timeout)
                if (__hip_atomic_load(&relay[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
                    __builtin_amdgcn_s_memrealtime() - t0 > idle_ticks + idle_ticks / 2) {
                    quit = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        sq = (uint32_t)__shfl((int)sq, 0);
        quit = (uint32_t)__shfl((int)quit, 0);
        if (quit) break;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // every lane: the request's actions are visible
        last = sq;
        if (valid) {
            int act[NA];
            if (inline_act) {   // one env: lane 0 of workgroup 0, which polled the inbox
#pragma unroll
                for (int a = 0; a < NA; a++) act[a] = (int)((ib[a >> 1] >> (8 * (a & 1))) & 0xFFu);
            } else {
#pragma unroll
                for (int a = 0; a < NA; a++) act[a] = actions[a * S.n + e];
            }
            step_and_emit<true>(E, T, C, S, e, act, nullptr, autoreset, out, 0);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // this lane's outputs reach host / device memory
        __syncthreads();
        if (lane == 0) __hip_atomic_store(&ctl->done[blockIdx.x], sq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        t0 = __builtin_amdgcn_s_memrealtime();
    }
    if (valid) env_store(E, S.words, S.n, e);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    if (lane == 0) __hip_atomic_store(&ctl->exited[blockIdx.x], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The env's order table and used tray-slot prefix into LDS tables (one lane per env): the
// loads of eight rows are issued together and waited for once (a load-then-store loop per row
// waits out one HBM round trip per row, ~30 us per launch at 30 orders and a few dozen slots).
__device__ __forceinline__ void tables_copy_in(const DevState& S, const Tables& T, int e, int norders, int nslots) {
    const size_t n = (size_t)S.n;
    for (int o0 = 0; o0 < norders; o0 += 8) {
        uint32_t v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = o0 + j < norders ? S.orders[(size_t)(o0 + j) * n + e] : 0u;
#pragma unroll
        for (int j = 0; j < 8; j++)
            if (o0 + j < norders) T.orders[(o0 + j) * T.stride] = v[j];
    }
    for (int q0 = 0; q0 < nslots; q0 += 8) {
        uint32_t c[8], x[8], t[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const bool in = q0 + j < nslots;
            const size_t i = (size_t)(q0 + j) * n + e;
            c[j] = in ? S.scode[i] : 0u;
            x[j] = in ? S.snext[i] : 0u;
            t[j] = in ? S.scstep[i] : 0u;
        }
#pragma unroll
        for (int j = 0; j < 8; j++)
            if (q0 + j < nslots) {
                T.scode[(q0 + j) * T.stride] = (uint16_t)c[j];
                T.snext[(q0 + j) * T.stride] = (uint8_t)x[j];
                T.scstep[(q0 + j) * T.stride] = (uint16_t)t[j];
            }
    }
}

// K fused steps.  LDS = true stages the env's order table and tray-slot arena in LDS for
// the whole launch (one 64-lane workgroup = 64 envs, 97.5 KB of LDS), so the linked-list
// walks and order-word read-modify-writes of the step are ds_* round trips (~100 cycles)
// instead of L2/HBM round trips; only the used prefix is copied in and out.
template <bool LDS, bool FULL, bool STAGED = false>
__global__ void __launch_bounds__(BLOCK) k_step_many(DevState S, Cfg C, int K, uint64_t seed, uint32_t gid0,
                                                     uint32_t step0, int mode, int autoreset, fjsp_out out) {
    struct NoTile { int unused; };
    __shared__ typename std::conditional<STAGED, StageTile, NoTile>::type s_tile;
    __shared__ uint32_t s_orders[LDS ? MAX_ORDERS * BLOCK : 1];
    __shared__ uint16_t s_code[LDS ? MAX_SLOTS * BLOCK : 1];
    __shared__ uint8_t s_next[LDS ? MAX_SLOTS * BLOCK : 1];
    __shared__ uint16_t s_cstep[LDS ? MAX_SLOTS * BLOCK : 1];
    __shared__ double s_lut[RLUT_SIZE];
    const int lane = threadIdx.x;
    for (int i = lane; i < RLUT_SIZE; i += BLOCK) s_lut[i] = C.lut[i];
    __syncthreads();
    C.lut = s_lut;
    const int e = blockIdx.x * BLOCK + lane;
    if (e >= S.n) return;
    Env E;
    env_load(E, S.words, S.n, e);
    Tables T;
    if constexpr (LDS) {
        T.orders = s_orders + lane;
        T.scode = s_code + lane;
        T.snext = s_next + lane;
        T.scstep = s_cstep + lane;
        T.stride = BLOCK;
        tables_copy_in(S, T, e, E.norders(), E.slot_next());
    } else {
        T = tables_of(S, e);
    }
    FJSP_DIAG(
    for (int i = 0; i < 8; i++) E.st_acc[i] = 0;
    E.st_t0 = __builtin_amdgcn_s_memtime();
    )
    for (int k = 0; k < K; k++) {
        int act[NA];
        synth_actions(seed, gid0 + (uint32_t)e, step0 + (uint32_t)k, mode, E, T, C, act);
        FJSP_STAMP(E, 0);
        if constexpr (STAGED)
            step_and_emit_staged(E, T, C, S, e, act, autoreset, out, (uint32_t)k, &s_tile, lane);
        else
            step_and_emit<true, FULL>(E, T, C, S, e, act, nullptr, autoreset, out, (uint32_t)k);
    }
    if constexpr (LDS) {
        for (int o = 0; o < E.norders(); o++) S.orders[(size_t)o * S.n + e] = T.orders[o * BLOCK];
        for (int s = 0; s < E.slot_next(); s++) {
            S.scode[(size_t)s * S.n + e] = T.scode[s * BLOCK];
            S.snext[(size_t)s * S.n + e] = T.snext[s * BLOCK];
            S.scstep[(size_t)s * S.n + e] = T.scstep[s * BLOCK];
        }
    }
    env_store(E, S.words, S.n, e);
    FJSP_DIAG(
    if (lane == 0)
        for (int i = 0; i < 8; i++) atomicAdd((unsigned long long*)&g_stamps[i], (unsigned long long)E.st_acc[i]);
    )
}

// K fused steps, pipelined over 2 or 3 wavefronts per 64-env workgroup (lean outputs only).
// Wave 0 ("sim") advances the env state: actions, action phase, SimPy run, auto-reset; after
// each step it leaves a snapshot of the pre-reset state (the 22 words the observation reads),
// the 8 action-result words and the step's completed orders / packaged products in LDS.  The
// emit wave(s), on other SIMDs of the same CU, turn snapshot k into the outputs of step k
// (rewards, observation, masks, term, trunc, status) while wave 0 already computes step k+1,
// and precompute the next step's actions when they do not depend on the state (uniform
// random mode).  Snapshots and action slots are double-buffered; one workgroup barrier per
// step orders them.
// Output sink of one emit wave: part 0 stores the int32 and float32 observation fields, part 1
// the int8 fields and the masks (the other part's values are dead code and never computed);
// part -1 stores everything.
template <int PART>
struct PartSink {
    StoreSink s;
    __device__ __forceinline__ void i32(int f, int v) { if (PART <= 0) s.i32(f, v); }
    __device__ __forceinline__ void f32(int f, float v) { if (PART <= 0) s.f32(f, v); }
    __device__ __forceinline__ void i8(int f, int v) { if (PART != 0) s.i8(f, v); }
    __device__ __forceinline__ void mask(int f, int v) { if (PART != 0) s.mask(f, v); }
};

// Output sink of one of k_step_ag's four emit waves: only the fields in the compile-time masks
// are computed and stored (observe()'s other values are dead code).
template <uint32_t I32M, uint32_t I8M, uint32_t F32M, uint32_t MKM>
struct FieldSink {
    StoreSink s;
    __device__ __forceinline__ void i32(int f, int v) { if ((I32M >> f) & 1u) s.i32(f, v); }
    __device__ __forceinline__ void f32(int f, float v) { if ((F32M >> f) & 1u) s.f32(f, v); }
    __device__ __forceinline__ void i8(int f, int v) { if ((I8M >> f) & 1u) s.i8(f, v); }
    __device__ __forceinline__ void mask(int f, int v) { if ((MKM >> f) & 1u) s.mask(f, v); }
};

// State words the observation / masks / term / trunc / status read (observe, compute_masks):
// all but the MT cursor (W3), the packaging run lists (W13-16), the machines' next-event steps
// (W19) and the packaging completion counters (W24-25).
constexpr uint32_t SNAP_WORDS = ((1u << NSTATE) - 1u) & ~((1u << 3) | (0xFu << 13) | (1u << 19) | (3u << 24));
// Snapshot slot: 32 words per lane = the 22 observed state words (SNAP_WORDS, in word order),
// the 8 action-result words (action in bits 8..11) and the step's completed orders | packaged
// products << 16, stored lane-major as 8 uint4 per lane (16-byte LDS accesses, conflict-free:
// consecutive lanes 16 bytes apart within each 1 KB row).
constexpr int SNAP_N = 32;
static_assert(__builtin_popcount(SNAP_WORDS) + NA + 1 <= SNAP_N, "snapshot slot");
struct alignas(16) PipeSnap {
    uint4 q[SNAP_N / 4][BLOCK];
};
__device__ __forceinline__ void snap_put(PipeSnap& sp, int lane, const uint32_t* v) {
#pragma unroll
    for (int g = 0; g < SNAP_N / 4; g++) sp.q[g][lane] = make_uint4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
}
__device__ __forceinline__ void snap_get(const PipeSnap& sp, int lane, uint32_t* v) {
#pragma unroll
    for (int g = 0; g < SNAP_N / 4; g++) {
        const uint4 x = sp.q[g][lane];
        v[4 * g] = x.x; v[4 * g + 1] = x.y; v[4 * g + 2] = x.z; v[4 * g + 3] = x.w;
    }
}
constexpr int SNAP_RES = __builtin_popcount(SNAP_WORDS), SNAP_GSTAT = SNAP_RES + NA;

__device__ __forceinline__ uint32_t pack_actions(const int* act, int lo) {
    return (uint32_t)act[lo] | ((uint32_t)act[lo + 1] << 8) | ((uint32_t)act[lo + 2] << 16) | ((uint32_t)act[lo + 3] << 24);
}

// PG: a pre-draw wave (wave 1 + NEMIT, a SIMD of its own) draws each env's next order table
// while the episode runs, so an auto-reset is a table copy instead of ~130 MT draws on the
// sim wave's critical path.  It copies the live MT row to the env's other row (CQ uint4 per
// step), then draws from the copy (PB words per step) into LDS; the sim wave consumes a
// finished table at reset (the other row becomes live) or, if it is not finished, resets
// inline from the live row.  Copies are cooperative (the wave copies one env's row with
// contiguous 1 KB loads); the draw is per lane.  The two waves exchange per-lane mailboxes double-buffered by
// step parity (written in step k, read in step k + 1, the barrier between): the sim wave
// posts its episode counter, num_orders and cursor word, the pre-draw wave whether its table
// is ready for that episode counter and the cursor word after it.  A finished table outlives
// the launch (W[PGW], S.nxt); every other reset path clears it.
constexpr int PG_CR = 1;   // pre-draw work per step: MT rows copied (whole wave) ...
constexpr int PG_PB = 8;   // ... and words drawn per env
constexpr int AG_PB = 4;   // words drawn per env per step in k_step_ag
// The pre-draw wave (k_step_pipe<..., PG>, k_step_ag): see the comment above k_step_pipe.
// s_mb / s_cp / s_nxt are the kernel's LDS mailboxes, row-copy staging and next tables.
// FINAL_MB: the sim side also posts in the final epoch K (k_step_ag resets at the top of an
// epoch), so a table it consumed or abandoned there must not be stored as ready.
// ASYNC (k_step_ag): a row loaded in step k is held in registers and stored in step k + 1, and
// each MT refill is loaded a step ahead: their latency hides behind the barrier instead of
// the step (plain loads; an LDS DMA would be drained by the barrier's fence).  s_cp unused.
template <int CR, int PB, bool FINAL_MB = false, bool ASYNC = false>
__device__ __forceinline__ void predraw_wave(const DevState& S, int K, int lane, int e, bool valid, size_t ebase,
                                             uint32_t (*s_mb)[2][BLOCK], uint4 (*s_cp)[3][BLOCK], uint32_t* s_nxt) {
    const uint32_t n = (uint32_t)S.n;
    // the pre-draw wave: 0 idle, 1 copying the live row, 2 drawing, 3 table ready
    int ph = 0, nord = 0, pos = 0, g = 0;
    uint32_t src = 0, my = 0x100u;   // live row at the start of the pre-draw; episode it is for
    OrderDraw d{0, 0, 0, 0, 0u};
    int ls_prev[CR];       // ASYNC: lanes whose row DMA is in flight (ph == 4) and their source rows
    uint32_t sl_prev[CR];
    bool inflight = false;
    // ASYNC: the runs of the next refill, loaded a step ahead (after the draw that precedes it):
    // the draw waits for loads a step old, not for loads it issues; pf_pa = their refill, -1 none
    uint4 pfa[(PB + 4) / 4], pfc[(PB + 4) / 4];
    int pf_pa = -1;
    // ASYNC: the rows in flight, in registers (plain loads are not waited for at the barrier; an
    // LDS DMA is: the barrier's fence drains it)
    // (three scalars, not an array: an array here stays in scratch memory and each load is
    // waited for at once)
    static_assert(!ASYNC || CR == 1, "one row in flight per step");
    uint4 cp0 = make_uint4(0u, 0u, 0u, 0u), cp1 = cp0, cp2 = cp0;
    if (valid) {
        const uint32_t pg = S.words[(size_t)PGW * n + e];
        if (pg & 1u) {
            ph = 3;
            my = 0;
            nord = (int)((pg >> 24) & 0x7Fu);
            pos = (int)((pg >> 1) & 0x3FFu);
            g = (int)((pg >> 11) & 0x3FFu);
            src = ((pg >> 21) & 1u) ^ (nord > 0 ? 1u : 0u);
        }
    }
    FJSP_DIAG(
    uint64_t pg_busy = 0, pg_act = 0, pg_busy_act = 0, pg_ph[3] = {0, 0, 0};
    )
    for (int k = 0; k <= K; k++) {
        FJSP_DIAG(
        const uint64_t pt0 = __builtin_amdgcn_s_memtime();
        bool pg_active = false;
        )
        if (valid) {
            const uint32_t si = s_mb[0][k & 1][lane];
            if ((si & 0xFFu) != my) {   // a new episode: start over from its stream position
                const uint32_t sw = s_mb[1][k & 1][lane];
                my = si & 0xFFu;
                nord = (int)((si >> 8) & 0x7Fu);
                src = sw >> 31;
                pos = (int)(sw & 0x3FFu);
                g = (int)((sw >> 16) & 0x3FFu);
                d = OrderDraw{0, 0, 0, 0, 0u};
                pf_pa = -1;
                ph = nord > 0 ? 1 : 3;
            }
        }
        // Copy the live rows of up to CR envs that start a pre-draw (the whole wave, one
        // env at a time: contiguous 1 KB loads): loads first, the per-lane draw in the shadow
        // of their latency, then the stores.  Rows copied in step k are first read in k + 1.
        // ASYNC: the runs of the next refill from pos (disjoint from the words stored since)
        auto prefetch = [&](const uint32_t* work) __attribute__((always_inline)) {
            pf_pa = pos & ~3;
            mt_load<PB>(work, pf_pa, pfa, pfc);
        };
        auto draw_step = [&]() __attribute__((always_inline)) {
            if (valid && ph == 2) {
                uint32_t* work = S.mt + ((size_t)(src ^ 1u) * n + e) * MT_N;
                uint32_t v[PB];
                int pa, cnt;
                if (ASYNC && pf_pa == (pos & ~3)) {
                    // the refill after this one first (a refill reads no word this one stores),
                    // then this one on runs loaded a step ago
                    const int pn = pf_pa + PB >= MT_N ? 0 : pf_pa + PB;
                    uint4 pna[(PB + 4) / 4], pnc[(PB + 4) / 4];
                    mt_load<PB>(work, pn, pna, pnc);
                    mt_batch_loaded<PB>(work, pos, g, v, pa, cnt, pfa, pfc);
#pragma unroll
                    for (int q = 0; q < (PB + 4) / 4; q++) { pfa[q] = pna[q]; pfc[q] = pnc[q]; }
                    pf_pa = pn;
                    pos += draw_orders<PB>(v, pos - pa, cnt, nord, d, s_nxt + lane, BLOCK);
                    if (pos == MT_N) { pos = 0; g = 0; }
                    if (d.o >= nord) { ph = 3; pf_pa = -1; }
                } else {
                    mt_batch<PB>(work, pos, g, v, pa, cnt);
                    pos += draw_orders<PB>(v, pos - pa, cnt, nord, d, s_nxt + lane, BLOCK);
                    if (pos == MT_N) { pos = 0; g = 0; }
                    if (d.o >= nord) ph = 3;
                    if (ASYNC) {
                        if (ph == 2) prefetch(work);
                        else pf_pa = -1;
                    }
                }
            }
        };
        FJSP_DIAG(
        const uint64_t pt1 = __builtin_amdgcn_s_memtime();
        )
        const int promote = ph;   // ASYNC: ph == 4 lanes become drawable after this step's draw
        uint64_t need = __ballot(valid && ph == 1);
        FJSP_DIAG(
        pg_active = need != 0 || __ballot(valid && ph == 2) != 0;
        )
        if (ASYNC) {
            // the draw first (its runs were loaded two steps ago), then last step's rows (loaded
            // after that step's prefetches), then this step's row loads: each wait is for loads
            // a step old, never for the ones just issued (vmcnt counts in order)
            draw_step();
            FJSP_DIAG(
            const uint64_t pt2 = __builtin_amdgcn_s_memtime();
            if (pg_active) { pg_ph[0] += pt1 - pt0; pg_ph[1] += pt2 - pt1; }
            )
            if (ASYNC && inflight) {   // last step's row DMAs: store them, the lanes draw from the next step on
                const int pb = (k - 1) & 1;
#pragma unroll
                for (int r = 0; r < CR; r++) {
                    const size_t el = ebase + (size_t)ls_prev[r];
                    uint4* rd = reinterpret_cast<uint4*>(S.mt + ((size_t)(sl_prev[r] ^ 1u) * n + el) * MT_N);
                    rd[lane] = cp0;
                    rd[lane + 64] = cp1;
                    if (lane + 128 < MT_N / 4) rd[lane + 128] = cp2;
                }
                (void)pb;
                inflight = false;
            }

#pragma unroll
            for (int r = 0; r < CR; r++)
                if (promote == 4 && ph == 4 && lane == ls_prev[r]) ph = 2;
            if (valid && promote == 4 && ph == 2)   // rows stored above: their first refill
                prefetch(S.mt + ((size_t)(src ^ 1u) * n + e) * MT_N);
            if (need) {
                const int first = __builtin_ctzll(need);
#pragma unroll
                for (int r = 0; r < CR; r++) {
                    ls_prev[r] = need ? __builtin_ctzll(need) : first;
                    need &= need - 1;
                    sl_prev[r] = (uint32_t)__builtin_amdgcn_readlane((int)src, ls_prev[r]);
                    const size_t el = ebase + (size_t)ls_prev[r];
                    const uint4* rs = reinterpret_cast<const uint4*>(S.mt + ((size_t)sl_prev[r] * n + el) * MT_N);
                    cp0 = rs[lane];
                    cp1 = rs[lane + 64];
                    cp2 = rs[min(lane + 128, MT_N / 4 - 1)];
                    if (lane == ls_prev[r] && ph == 1) ph = 4;
                }
                inflight = true;
            }
        } else if (need) {
            // rows go through LDS by DMA (global_load_lds: no VGPRs held across the draw);
            // slots beyond the envs waiting re-copy the first env's row (identical stores)
            const int first = __builtin_ctzll(need);
            int ls[CR];
#pragma unroll
            for (int r = 0; r < CR; r++) {
                ls[r] = need ? __builtin_ctzll(need) : first;
                need &= need - 1;
                const uint32_t sl = (uint32_t)__builtin_amdgcn_readlane((int)src, ls[r]);
                const size_t el = ebase + (size_t)ls[r];
                const uint4* rs = reinterpret_cast<const uint4*>(S.mt + ((size_t)sl * n + el) * MT_N);
#pragma unroll
                for (int i = 0; i < 3; i++)
                    __builtin_amdgcn_global_load_lds(
                        (__attribute__((address_space(1))) void*)(rs + min(lane + 64 * i, MT_N / 4 - 1)),
                        (__attribute__((address_space(3))) void*)&s_cp[r][i][0], 16, 0, 0);
            }
            draw_step();
            __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the row DMAs have landed
#pragma unroll
            for (int r = 0; r < CR; r++) {
                const uint32_t sl = (uint32_t)__builtin_amdgcn_readlane((int)src, ls[r]);
                const size_t el = ebase + (size_t)ls[r];
                uint4* rd = reinterpret_cast<uint4*>(S.mt + ((size_t)(sl ^ 1u) * n + el) * MT_N);
                rd[lane] = s_cp[r][0][lane];
                rd[lane + 64] = s_cp[r][1][lane];
                if (lane + 128 < MT_N / 4) rd[lane + 128] = s_cp[r][2][lane];
                if (lane == ls[r]) ph = 2;
            }
        } else {
            draw_step();
        }
        if (valid) {
            const uint32_t wrow = nord > 0 ? (src ^ 1u) : src;
            s_mb[2][(k + 1) & 1][lane] = (ph == 3 ? 1u : 0u) | (my << 1) | ((uint32_t)nord << 9);
            s_mb[3][(k + 1) & 1][lane] = (uint32_t)pos | ((uint32_t)g << 16) | (wrow << 31);
        }
        FJSP_DIAG(
        {
            const uint64_t dt = __builtin_amdgcn_s_memtime() - pt0;
            pg_busy += dt;
            if (pg_active) { pg_act += 1; pg_busy_act += dt; }
            (void)pg_ph;
        }
        )
        __syncthreads();
    }
    if (ASYNC) __builtin_amdgcn_s_waitcnt(0x0F70);   // no LDS DMA outlives the workgroup
    FJSP_DIAG(
    if (lane == 0) {
        atomicAdd(&g_pgstamps[0], (unsigned long long)pg_busy);
        atomicAdd(&g_pgstamps[1], (unsigned long long)pg_act);
        atomicAdd(&g_pgstamps[2], (unsigned long long)pg_busy_act);
        atomicAdd(&g_pgstamps[3], (unsigned long long)(K + 1));
        if (ASYNC) { atomicAdd(&g_agstamps[52], (unsigned long long)pg_ph[0]); atomicAdd(&g_agstamps[53], (unsigned long long)pg_ph[1]); }
    }
    )
    if (valid) {
        uint32_t pg = 0;
        if (FINAL_MB && (s_mb[0][(K + 1) & 1][lane] & 0xFFu) != my) ph = 0;   // reset in the final epoch
        if (ph == 3) {
            const uint32_t wrow = nord > 0 ? (src ^ 1u) : src;
            pg = 1u | ((uint32_t)pos << 1) | ((uint32_t)g << 11) | (wrow << 21) | ((uint32_t)nord << 24);
            for (int o = 0; o < nord; o++) S.nxt[(size_t)o * n + e] = s_nxt[o * BLOCK + lane];
        }
        S.words[(size_t)PGW * n + e] = pg;
    }
}

__device__ constexpr fjsp_out kNoOutDev = {};
// The multi-wave kernels' arguments (k_step_pipe, k_step_ag), read per role from the kernarg
// segment through a pointer the compiler cannot see through (`opaque`): a value read once at the
// kernel's entry stays in an SGPR through every role's step loop (the state pointers, the config,
// the output pointers and the action stream: 44 SGPR spills, ~400 v_readlane reloads in r03's
// k_step_ag); read inside the role's branch it lives only there.  (volatile reads of the by-value
// parameters copied them to scratch.)  Same layouts as the parameter lists.
struct PipeArgs {
    DevState S;
    Cfg C;
    int K;
    uint64_t seed;
    uint32_t gid0, step0;
    int mode, autoreset;
    fjsp_out out;
};
struct AgArgs {
    DevState S;
    Cfg C;
    int K;
    uint64_t seed;
    uint32_t gid0, step0;
    int autoreset;
    fjsp_out out;
};
static_assert(sizeof(DevState) == 64 && sizeof(Cfg) == 48 && offsetof(AgArgs, C) == 64 && offsetof(AgArgs, K) == 112 &&
                  offsetof(AgArgs, seed) == 120 && offsetof(AgArgs, gid0) == 128 && offsetof(AgArgs, autoreset) == 136 &&
                  offsetof(AgArgs, out) == 144,
              "AgArgs mirrors k_step_ag's kernel arguments (the kernarg segment's layout)");
static_assert(offsetof(PipeArgs, K) == 112 && offsetof(PipeArgs, seed) == 120 && offsetof(PipeArgs, step0) == 132 &&
                  offsetof(PipeArgs, mode) == 136 && offsetof(PipeArgs, autoreset) == 140 && offsetof(PipeArgs, out) == 144,
              "PipeArgs mirrors k_step_pipe's kernel arguments");
template <class T>
__device__ __forceinline__ const T* opaque(const T* p) {
    asm volatile("" : "+s"(p));
    return p;
}
template <class A>
__device__ __forceinline__ const A* kargs() {
    return opaque((const A*)__builtin_amdgcn_kernarg_segment_ptr());
}
__device__ __forceinline__ const AgArgs* ag_args() { return kargs<AgArgs>(); }
template <class A>
__device__ __forceinline__ Cfg cfg_at(const A* a, const double* lut) {
    Cfg c = a->C;
    c.lut = lut;
    return c;
}
// the outputs a role writes, read in its branch
__device__ __forceinline__ fjsp_out out_at(const fjsp_out& o) {
    fjsp_out r = kNoOutDev;
    r.obs_i32 = o.obs_i32; r.obs_i8 = o.obs_i8; r.obs_f32 = o.obs_f32; r.masks = o.masks;
    r.rewards = o.rewards; r.term = o.term; r.trunc = o.trunc; r.status = o.status;
    return r;
}

// STALL: the test build of the kernel (option "test_stall"): the production instances carry no
// code of it (any code there shifted k_step_ag's register allocation: +1.2 % per step, measured).
template <bool LDS, int NEMIT, bool PG = false, bool STALL = false>
__global__ void __launch_bounds__((1 + NEMIT + PG) * BLOCK) __attribute__((amdgpu_waves_per_eu(1, 2))) k_step_pipe(DevState S, Cfg Ck, int K, uint64_t seed,
                                                              uint32_t gid0, uint32_t step0, int mode, int autoreset,
                                                              fjsp_out out) {
    static_assert(!PG || LDS, "the pre-drawn tables live in LDS");
    // pre-draw work per step (sized so the wave stays off the critical path): rows copied by
    // the whole wave (CR envs, 1 KB per load), words drawn per env
    constexpr int CR = PG_CR, PB = PG_PB;
    __shared__ uint32_t s_orders[LDS ? MAX_ORDERS * BLOCK : 1];
    __shared__ uint32_t s_nxt[PG ? MAX_ORDERS * BLOCK : 1];
    __shared__ uint32_t s_mb[PG ? 4 : 1][2][BLOCK];   // sim: epi | nord << 8, cursor word; pre-draw: ready, cursor
    __shared__ uint4 s_cp[PG ? PG_CR : 1][3][BLOCK];   // MT rows in flight (pre-draw copies)
    // Pickup + AGV ahead (PG, uniform-random actions).  Neither agent's next action depends on
    // anything the packaging agents or the run phase of the current step change, except where
    // a drop at packaging routes the tray (deferred: agv_pack_drop).  So after the machines'
    // actions of step k the sim wave posts the words they read (s_post, then s_postflag = k+1);
    // emit wave 1 runs step k+1's pickup on them (s_pick, s_pickflag = k+1), emit wave 2 step
    // k+1's AGV on both, while the sim wave finishes step k; at the top of step k+1 the sim
    // wave applies both (lanes that just reset run the two agents themselves).
    constexpr int NPOST = 10;   // W0, W4, W5, W6 (loc after the move), W7..W12 (lists 0..5)
    __shared__ uint32_t s_post[PG ? NPOST : 1][BLOCK];
    __shared__ uint32_t s_pick[PG ? 6 : 1][BLOCK];   // next_order, W4, W5, W7, result, flags
    __shared__ uint32_t s_agv[PG ? 12 : 1][BLOCK];   // W5, W6, W7..W12, result, flags, move, pend
    __shared__ uint32_t s_postflag, s_pickflag, s_abort, s_cap;
    __shared__ uint16_t s_code[LDS ? MAX_SLOTS * BLOCK : 1];
    __shared__ uint8_t s_next[LDS ? MAX_SLOTS * BLOCK : 1];
    __shared__ uint16_t s_cstep[LDS ? MAX_SLOTS * BLOCK : 1];
    __shared__ PipeSnap snap[2];
    __shared__ uint32_t s_act[2][2][BLOCK];
    __shared__ double s_lut[RLUT_SIZE];
    for (int i = threadIdx.x; i < RLUT_SIZE; i += (1 + NEMIT + PG) * BLOCK) s_lut[i] = Ck.lut[i];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / BLOCK);
    const int lane = threadIdx.x % BLOCK;
    const int e = blockIdx.x * BLOCK + lane;
    const bool valid = e < S.n;
    const bool pre = mode == FJSP_ACTIONS_UNMASKED;   // actions independent of the state
    const uint32_t n = (uint32_t)S.n, ue = (uint32_t)e;
    if (wave == 1 && pre && K > 0) {
        int act[NA];
        synth_uniform(seed, gid0 + (uint32_t)e, step0, act);
        s_act[0][0][lane] = pack_actions(act, 0);
        s_act[0][1][lane] = pack_actions(act, 4);
    }
    if (threadIdx.x == 0) { s_abort = 0; s_cap = aux_words(S)[AUX_SPIN_CAP]; }
    if constexpr (PG) {   // step-0 mailboxes
        if (threadIdx.x == 0) { s_postflag = 0; s_pickflag = 0; }
        if (wave == 0 && valid) {
            s_mb[0][0][lane] = ((S.words[e] >> 16) & 0xFFu) << 8;   // episode counter 0 | num_orders
            s_mb[1][0][lane] = S.words[3 * n + e];
        }
        if (wave == 1 + NEMIT && valid) {
            const uint32_t pg = S.words[(size_t)PGW * n + e];
            uint32_t r = 0, c = 0;
            if (pg & 1u) {   // a table finished in an earlier launch
                const int no = (int)((pg >> 24) & 0x7Fu);
                for (int o = 0; o < no; o++) s_nxt[o * BLOCK + lane] = S.nxt[(size_t)o * n + e];
                r = 1u | ((uint32_t)no << 9);
                c = ((pg >> 1) & 0x3FFu) | (((pg >> 11) & 0x3FFu) << 16) | (((pg >> 21) & 1u) << 31);
            }
            s_mb[2][0][lane] = r;
            s_mb[3][0][lane] = c;
        }
    }
    __syncthreads();
    if constexpr (STALL) {
        if (wave == 0 && blockIdx.x == 0) stall_for_test(S);
    }
    if (wave == 0) {
        // the config and the action stream read in this branch (kargs)
        const PipeArgs* pa = kargs<PipeArgs>();
        const DevState S = pa->S;
        const Cfg C = cfg_at(pa, s_lut);
        const uint64_t seed = pa->seed;
        const uint32_t gid0 = pa->gid0, step0 = pa->step0;
        const int mode = pa->mode;
        __builtin_amdgcn_s_setprio(3);   // the sim wave is the critical path: win shared issue slots
        Env E;
        if (valid) env_load(E, S.words, S.n, e);
        Tables T = tables_of(S, valid ? e : 0);
        if constexpr (LDS) {   // the env's order table and used slot prefix live in LDS for the launch
            T.orders = s_orders + lane;
            T.scode = s_code + lane;
            T.snext = s_next + lane;
            T.scstep = s_cstep + lane;
            T.stride = BLOCK;
            if (valid) tables_copy_in(S, T, e, E.norders(), E.slot_next());
        }
        FJSP_DIAG(
        for (int i = 0; i < 8; i++) E.st_acc[i] = 0;
        E.st_t0 = __builtin_amdgcn_s_memtime();
        )
        int epi = 0;   // episodes started in this launch (mod 256), the pre-draw tag
        bool fresh = true;   // this step's pickup runs here (first step of the launch / after a reset)
        for (int k = 0; k <= K; k++) {
            if (k < K && valid) {
                int act[NA];
                if (pre) {
                    const uint32_t a0 = s_act[k & 1][0][lane], a1 = s_act[k & 1][1][lane];
#pragma unroll
                    for (int a = 0; a < 4; a++) { act[a] = (a0 >> (8 * a)) & 0xFF; act[4 + a] = (a1 >> (8 * a)) & 0xFF; }
                } else {
                    synth_actions(seed, gid0 + (uint32_t)e, step0 + (uint32_t)k, mode, E, T, C, act);
                }
                FJSP_STAMP(E, 0);
                uint32_t res[NA];
                bool ahead = false;
                int ahead_move = 0;
                if constexpr (PG) {
                    if (pre && !fresh) {   // step k's pickup and AGV ran on the emit waves
                        E.w[0] = (E.w[0] & 0x00FFFFFFu) | (s_pick[0][lane] << 24);
                        E.w[4] = s_pick[1][lane];
                        res[0] = s_pick[4][lane];
#pragma unroll
                        for (int i = 0; i < 8; i++) E.w[5 + i] = s_agv[i][lane];   // W5..W12
                        res[1] = s_agv[8][lane];
                        E.w[2] |= s_pick[5][lane] | s_agv[9][lane];
                        ahead_move = (int)s_agv[10][lane];
                        const uint32_t pend = s_agv[11][lane];
                        if (pend) agv_pack_drop(E, T, C, pend);
                        ahead = true;
                    }
                }
                auto mid = [&](const Env& Em, int mv) {
                    if constexpr (PG) {
                        if (pre) {
                            s_post[0][lane] = Em.w[0];
                            s_post[1][lane] = Em.w[4];
                            s_post[2][lane] = Em.w[5];
                            s_post[3][lane] = mv ? ((Em.w[6] & ~7u) | (uint32_t)mv) : Em.w[6];
#pragma unroll
                            for (int i = 0; i < 6; i++) s_post[4 + i][lane] = Em.w[7 + i];
                            __hip_atomic_store(&s_postflag, (uint32_t)(k + 1), __ATOMIC_RELEASE,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                    }
                };
                const int nc0 = E.ncompleted(), tp0 = E.total_packaged();
                (void)env_advance<true>(E, T, C, act, nullptr, res, mid, ahead, ahead_move);   // g/8: the emit wave
                flag_obs_overflow(E);
                uint32_t v[SNAP_N];
                int j = 0;
#pragma unroll
                for (int i = 0; i < NSTATE; i++)
                    if ((SNAP_WORDS >> i) & 1u) v[j++] = E.w[i];
#pragma unroll
                for (int a = 0; a < NA; a++) v[SNAP_RES + a] = res[a] | ((uint32_t)act[a] << 8);
                v[SNAP_GSTAT] = (uint32_t)(E.ncompleted() - nc0) | ((uint32_t)(E.total_packaged() - tp0) << 16);
#pragma unroll
                for (int i = SNAP_GSTAT + 1; i < SNAP_N; i++) v[i] = 0u;
                snap_put(snap[k & 1], lane, v);
                const int nord = E.norders();
                const int all_done = E.ncompleted() == nord && nord > 0 && E.next_order() == nord;
                const int truncated = E.step() >= C.max_steps;
                FJSP_STAMP(E, 3);
                E.set_step(E.step() + 1);
                fresh = false;
                if (autoreset && (all_done || truncated)) {   // reset(seed=None)
                    fresh = true;
                    if constexpr (PG) {
                        const uint32_t pr = s_mb[2][k & 1][lane];
                        if ((pr & 1u) && ((pr >> 1) & 0xFFu) == (uint32_t)epi && (int)((pr >> 9) & 0x7Fu) == nord)
                            env_reset_predrawn(E, T, C, nord, s_mb[3][k & 1][lane], s_nxt + lane);
                        else
                            E = env_reset_cold(E, T, C, S, e, nord, false);
                        epi = (epi + 1) & 0xFF;
                    } else {
                        E = env_reset_cold(E, T, C, S, e, nord);
                    }
                }
                if constexpr (PG) {
                    s_mb[0][(k + 1) & 1][lane] = (uint32_t)epi | ((uint32_t)E.norders() << 8);
                    s_mb[1][(k + 1) & 1][lane] = E.w[3];
                }
                FJSP_STAMP(E, 6);
            }
            __syncthreads();
        }
        if (valid) {
            if constexpr (LDS) {
                for (int o = 0; o < E.norders(); o++) S.orders[(size_t)o * S.n + e] = T.orders[o * BLOCK];
                for (int q = 0; q < E.slot_next(); q++) {
                    S.scode[(size_t)q * S.n + e] = T.scode[q * BLOCK];
                    S.snext[(size_t)q * S.n + e] = T.snext[q * BLOCK];
                    S.scstep[(size_t)q * S.n + e] = T.scstep[q * BLOCK];
                }
            }
            // every wait happened before the last barrier: a give-up is visible here
            if (s_abort) E.w[2] |= ST_SPIN_TIMEOUT | ST_DIVERGED;
            env_store(E, S.words, S.n, e);
        }
        if (lane == 0) report_abort(S, s_abort);
        FJSP_DIAG(
        if (lane == 0)
            for (int i = 0; i < 8; i++) atomicAdd((unsigned long long*)&g_stamps[i], (unsigned long long)E.st_acc[i]);
        )
    } else if (PG && wave == 1 + NEMIT) {
        predraw_wave<CR, PB>(S, K, lane, e, valid, (size_t)blockIdx.x * BLOCK, s_mb, s_cp, s_nxt);
    } else {
        // NEMIT == 2: two emit waves split the outputs: wave 1 rewards + int32 / float32
        // observation fields (+ the next step's uniform actions), wave 2 int8 fields, masks,
        // term, trunc, status.  NEMIT == 1 (many envs: the CUs are already full): one wave.
        const int part = wave - 1;
        // the config, the outputs and the action stream read in this branch (kargs)
        const PipeArgs* pa = kargs<PipeArgs>();
        const Cfg C = cfg_at(pa, s_lut);
        const fjsp_out out = out_at(pa->out);
        const uint64_t seed = pa->seed;
        const uint32_t gid0 = pa->gid0, step0 = pa->step0;
        FJSP_DIAG(
        uint64_t em_busy = 0;
        )
        for (int k = 0; k <= K; k++) {
            FJSP_DIAG(
            const uint64_t et0 = __builtin_amdgcn_s_memtime();
            )
            // order within a step (PG): wave 1 first draws step k + 1's actions, writes step
            // k - 1's rewards and runs step k + 1's pickup as soon as the sim wave posts (early
            // in step k), then the observation fields; wave 2 writes its fields, then runs step
            // k + 1's AGV (needs that pickup)
            int act_next[NA];
            if (part == 0 && pre && k + 1 < K) {
                synth_uniform(seed, gid0 + (uint32_t)e, step0 + (uint32_t)(k + 1), act_next);
                s_act[(k + 1) & 1][0][lane] = pack_actions(act_next, 0);
                s_act[(k + 1) & 1][1][lane] = pack_actions(act_next, 4);
            }
            const bool have = k > 0 && valid;
            const uint32_t t = (uint32_t)(k - 1);
            uint32_t v[SNAP_N];
            Env E;
            if (have) {
                snap_get(snap[(k - 1) & 1], lane, v);
                int j = 0;
#pragma unroll
                for (int i = 0; i < NSTATE; i++) E.w[i] = ((SNAP_WORDS >> i) & 1u) ? v[j++] : 0u;
            }
            const StoreSink sink{out.obs_i32, out.obs_i8, out.obs_f32, out.masks, t, n, ue};
            if (part == 0 && have && out.rewards) {
                const uint32_t gs = v[SNAP_GSTAT];
                const double g8 = global_reward8(C, (int)(gs & 0xFFFFu), (int)(gs >> 16));
#pragma unroll
                for (int a = 0; a < NA; a++) {
                    const uint32_t r = v[SNAP_RES + a];
                    st32(out.rewards, (t * NA + (uint32_t)a) * n + ue,
                         g8 + C.lut[reward_index(a, r & 0xFFFF00FFu, (int)((r >> 8) & 0xFu))]);
                }
            }
            if constexpr (PG) {   // step k + 1's pickup, once the sim wave has posted its state
                if (part == 0 && pre && k + 1 < K) {
                    spin_until(&s_postflag, (uint32_t)(k + 1), &s_abort, &s_cap);
                    if (valid) {
                        Env Ep;
#pragma unroll
                        for (int i = 0; i < NSTATE; i++) Ep.w[i] = 0u;
                        Ep.w[0] = s_post[0][lane];
                        Ep.w[4] = s_post[1][lane];
                        Ep.w[5] = s_post[2][lane];
                        Ep.w[7 + L_PREADY] = s_post[4 + L_PREADY][lane];
                        const Tables Tp{s_orders + lane, s_code + lane, s_next + lane, s_cstep + lane, BLOCK};
                        const uint32_t r = pickup_execute(Ep, Tp, C, act_next[0]);
                        s_pick[0][lane] = Ep.w[0] >> 24;
                        s_pick[1][lane] = Ep.w[4];
                        s_pick[2][lane] = Ep.w[5];
                        s_pick[3][lane] = Ep.w[7 + L_PREADY];
                        s_pick[4][lane] = r;
                        s_pick[5][lane] = Ep.w[2];
                    }
                    __hip_atomic_store(&s_pickflag, (uint32_t)(k + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            if (have) {
                if (part == 0) {   // int32 / float32 fields (+ everything when NEMIT == 1)
                    PartSink<NEMIT == 1 ? -1 : 0> ps{sink};
                    observe(E, C, ps);
                }
                if (part == NEMIT - 1) {   // int8 fields, masks, term, trunc, status
                    if (NEMIT == 2) {
                        PartSink<1> ps{sink};
                        observe(E, C, ps);
                    }
                    const int nord = E.norders();
                    const int all_done = E.ncompleted() == nord && nord > 0 && E.next_order() == nord;
                    const int truncated = E.step() >= C.max_steps;
                    if (out.term) st32(out.term, t * n + ue, (uint8_t)all_done);
                    if (out.trunc) st32(out.trunc, t * n + ue, (uint8_t)truncated);
                    if (out.status)
                        st32(out.status, t * n + ue, E.status() | (s_abort ? ST_SPIN_TIMEOUT | ST_DIVERGED : 0u));
                }
            }
            if constexpr (PG) {   // step k + 1's AGV, on the posted state and that step's pickup
                if (part == 1 && pre && k + 1 < K) {
                    spin_until(&s_pickflag, (uint32_t)(k + 1), &s_abort, &s_cap);
                    if (valid) {
                        Env Ea;
#pragma unroll
                        for (int i = 0; i < NSTATE; i++) Ea.w[i] = 0u;
                        Ea.w[5] = s_pick[2][lane];
                        Ea.w[6] = s_post[3][lane];
#pragma unroll
                        for (int i = 0; i < 6; i++) Ea.w[7 + i] = s_post[4 + i][lane];
                        Ea.w[7 + L_PREADY] = s_pick[3][lane];
                        const Tables Ta{s_orders + lane, s_code + lane, s_next + lane, s_cstep + lane, BLOCK};
                        const int a1 = (int)((s_act[(k + 1) & 1][0][lane] >> 8) & 0xFFu);
                        int mv = 0;
                        uint32_t pend = 0;
                        const uint32_t r = agv_execute<true>(Ea, Ta, C, a1, &mv, &pend);
#pragma unroll
                        for (int i = 0; i < 8; i++) s_agv[i][lane] = Ea.w[5 + i];
                        s_agv[8][lane] = r;
                        s_agv[9][lane] = Ea.w[2];
                        s_agv[10][lane] = (uint32_t)mv;
                        s_agv[11][lane] = pend;
                    }
                }
            }
            FJSP_DIAG(
            em_busy += __builtin_amdgcn_s_memtime() - et0;
            )
            __syncthreads();
        }
        FJSP_DIAG(
        if (lane == 0 && part < 2) {
            atomicAdd(&g_emitstamps[2 * part], (unsigned long long)em_busy);
            atomicAdd(&g_emitstamps[2 * part + 1], (unsigned long long)(K + 1));
        }
        )
    }
}

// ---------------------------------------------------------------- agent-group pipeline
// k_step_ag: K fused steps (uniform-random actions, LDS tables, auto-reset with pre-drawn
// tables), the env's agents split over the wavefronts of its 64-env workgroup.  Per step the
// chains that stay sequential are  AGV (k) -> machines' actions (k) -> AGV (k+1)  and
// AGV (k) -> pickup station (k+1) -> AGV (k+1); everything else hangs off them:
//   AM owns every state word but the packaging ones.  At the top of step k it auto-resets the
//      env once K has counted step k-1's order completions (FJSPSimulation.reset(seed=None)),
//      applies the pickup and AGV results of step k (computed during step k-1; a lane that just
//      reset, and the first step of a launch, runs those two agents here), runs the machines'
//      actions (MachineAgent.py:99-139), posts the pickup / AGV words and the machine lists
//      (release flag), then the machines' run phase (:151-169) and its half of the snapshot.
//   E3 runs step k+1's pickup station (PickupStationAgent.py:146-248) on P's AGV result of
//      step k, and posts it (release flag).
//   P  runs step k+1's AGV (AGVAgent.py:180-368, a drop at packaging deferred): the half that
//      needs only the AGV's own words (agv_pre: outcome, prefetch of the list front it would
//      pop) at the top of the step, the rest (agv_fin) once AM's post and E3's pickup are in.
//      In the reference's agent order the pickup and the AGV read nothing that the packaging
//      agents or the run phase of step k change.
//   K  owns the packaging words (W1, W13-16, W20-29): at the top of step k the completions due
//      (PackagingAgent.py:143-147, older events than the step's actions), the AGV's drop
//      routed (FJSPSimulation.add_tray_to_packaging, with the in-flight counts before the run),
//      the stations' actions and grants (:91-141) and the order completions
//      (FJSPSimulation.py:245-258) — it needs only P's AGV result of the previous step.
//   E0..E3 turn step k-1's snapshot into the outputs; E0 also draws step k+2's actions.
//   PD pre-draws the next order tables (predraw_wave).
// The order words are shared by AM (processed bits) and K (packaged / complete bits): both OR
// atomically (order_or); P and E3 read the static fields and the bits of the tray the AGV picks
// up, which nothing else changes then.  The tray-slot arena needs no atomics: within a step
// every slot is written by the one wave that owns the list it joins.  Hand-offs inside a step:
// release / acquire flags (AM -> P, E3, K; E3 -> P); everything else crosses the one barrier
// per step.  Result words are 16 bits (result | action << 8).
// Waves w and w + 4 share a SIMD (two waves per SIMD issue VALU at twice one wave's rate): K
// shares AM's (both busy early in the step; AM has the higher priority), P (the critical path
// after AM's post, higher priority) shares the lightest emit wave's, PD and E3 pair up.
// wave of each role: AM, P, E1, E2, K, E0, PD, E3 (waves w and w + 4 share a SIMD): AM+PD, P+E0,
// E1+K, E2+E3 (0.6 % faster than AM+K, E1+PD; other pairings measured within noise)
constexpr int AG_LAYOUT[8] = {0, 1, 2, 3, 6, 5, 4, 7};
constexpr int AG_AM = AG_LAYOUT[0], AG_P = AG_LAYOUT[1], AG_E1 = AG_LAYOUT[2], AG_E2 = AG_LAYOUT[3], AG_K = AG_LAYOUT[4],
              AG_E0 = AG_LAYOUT[5], AG_PD = AG_LAYOUT[6], AG_E3 = AG_LAYOUT[7], AG_WAVES = 8;
// packaging-owned state words (K): W1, W13..W16 (packaging run lists), W20..W29
constexpr uint32_t K_WORDS = (1u << 1) | (0xFu << 13) | (0x3FFu << 20);
// masks per emit wave: pickup [0,3) | the AGV's pickup / drop [9,11) | the AGV's moves [3,9),
// machines [11,17), packaging [17,29)
// (other splits of the fields over the emit waves measured within 1 %)
// station masks (3 per station, from field 11) emitted by E0 instead of E3: E3 arrived last at
// the barrier in 92 % of the steps; 0 / 2 / 4 / 6 stations: 1.212 / 1.183 / 1.186 / 1.210 us per
// step at 16 envs per workgroup (profiles/r02/experiments/e3_masks_to_e0_*.json)
constexpr int AG_E0ST = 2;
constexpr uint32_t AG_E0ST_BITS = ((1u << (3 * AG_E0ST)) - 1u) << 11;
constexpr uint32_t AG_MASKS_E0 = 0x7u | AG_E0ST_BITS, AG_MASKS_E2 = 0x3u << 9,
                   AG_MASKS_E3 = ((0x3Fu << 3) | (0x3FFFFu << 11)) & ~AG_E0ST_BITS;
static_assert((AG_MASKS_E0 | AG_MASKS_E2 | AG_MASKS_E3) == (1u << NMASK) - 1u && !(AG_MASKS_E0 & AG_MASKS_E2) &&
              !(AG_MASKS_E0 & AG_MASKS_E3) && !(AG_MASKS_E2 & AG_MASKS_E3), "mask split");
// snapshot slot words (PipeSnap, 32 per lane): AM writes q[0..3], K q[4..7]
enum : int { SA_W0 = 0, SA_ST, SA_W4, SA_W5, SA_W6, SA_L0, SA_M0 = SA_L0 + 6, SA_M1, SA_R01, SA_R23,
             SK_W1 = 16, SK_P0, SK_N0 = SK_P0 + 4, SK_ST = SK_N0 + 4, SK_G, SK_R45, SK_R67 };
static_assert(SA_R23 < 16 && SK_R67 < 32, "snapshot slot");
// P's results for a step (s_res): next_order, W4, W5..W12, pickup result, AGV result, status, drop
enum : int { RS_NO = 0, RS_W4, RS_W5, RS_R0 = RS_W5 + 8, RS_R1, RS_ST, RS_PEND = 15, RS_N };
static_assert(RS_N <= 16, "s_res slot");
// AM's post 1 (s_p1): W0, W4, W5, W6, W7, W8 after the step's pickup and AGV, the AGV's drop
enum : int { P1_W0 = 0, P1_W4, P1_W5, P1_W6, P1_W7, P1_W8, P1_PEND, P1_N };
__device__ __forceinline__ void q_get(const uint4* q, int ng, uint32_t* v) {   // ng groups, stride BLOCK
#pragma unroll
    for (int g = 0; g < ng; g++) {
        const uint4 x = q[g * BLOCK];
        v[4 * g] = x.x; v[4 * g + 1] = x.y; v[4 * g + 2] = x.z; v[4 * g + 3] = x.w;
    }
}
__device__ __forceinline__ void q_put(uint4* q, int ng, const uint32_t* v) {
#pragma unroll
    for (int g = 0; g < ng; g++) q[g * BLOCK] = make_uint4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
}

__device__ __forceinline__ void snap_put4(PipeSnap& sp, int q0, int lane, const uint32_t* v) {
#pragma unroll
    for (int g = 0; g < 4; g++) sp.q[q0 + g][lane] = make_uint4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
}

// AM's reset decision at the top of step k (end of step k-1), as P and E0 see it: AM's W0 posted
// in step k-1 (next_order, num_orders, step) and K's completed orders after step k-1.
__device__ __forceinline__ bool ag_fresh(int k, bool valid, const uint4 (*s_p1)[2][BLOCK], const uint32_t (*s_kpost)[BLOCK],
                                         int lane, const Cfg& C, int autoreset) {
    if (k == 0) return true;   // the first step of a launch runs the pickup and the AGV on AM
    if (!valid) return false;
    const uint32_t w0a = s_p1[(k - 1) & 1][0][lane].x;   // P1_W0 of step k-1
    const int nord = (int)((w0a >> 16) & 0xFFu);
    const int all_done = (int)(s_kpost[(k - 1) & 1][lane] & 0xFFu) == nord && nord > 0 && (int)(w0a >> 24) == nord;
    return autoreset && (all_done || (int)(w0a & 0xFFFFu) >= C.max_steps);
}

// One emit role's outputs of step t from the step's snapshot (AM's and K's words, SA_* / SK_*):
// E0 rewards and the pickup's masks, E1 int32 and float32 fields, E2 int8 fields, term, trunc,
// status and the AGV's pickup / drop masks, E3 the other masks.
__device__ __forceinline__ void ag_emit(int part, const uint32_t* v, uint32_t t, uint32_t n, uint32_t ue, const Cfg& C,
                                        const fjsp_out& out) {
    Env E;
#pragma unroll
    for (int i = 0; i < NSTATE; i++) E.w[i] = 0u;
    E.w[0] = v[SA_W0]; E.w[2] = v[SA_ST] | v[SK_ST]; E.w[4] = v[SA_W4]; E.w[5] = v[SA_W5];
    E.w[6] = v[SA_W6];
#pragma unroll
    for (int l = 0; l < 6; l++) E.w[7 + l] = v[SA_L0 + l];
    E.w[17] = v[SA_M0]; E.w[18] = v[SA_M1];
    E.w[1] = v[SK_W1];
#pragma unroll
    for (int s = 0; s < 4; s++) { E.w[20 + s] = v[SK_P0 + s]; E.w[26 + s] = v[SK_N0 + s]; }
    const StoreSink sink{out.obs_i32, out.obs_i8, out.obs_f32, out.masks, t, n, ue};
    if (part == 0) {
        if (out.rewards) {
            const uint32_t gs = v[SK_G];
            const double g8 = global_reward8(C, (int)(gs & 0xFFFFu), (int)(gs >> 16));
            const uint32_t rw[4] = {v[SA_R01], v[SA_R23], v[SK_R45], v[SK_R67]};
#pragma unroll
            for (int a = 0; a < NA; a++) {
                const uint32_t r = (rw[a >> 1] >> (16 * (a & 1))) & 0xFFFFu;
                st32(out.rewards, (t * NA + (uint32_t)a) * n + ue,
                     g8 + C.lut[reward_index(a, r & 0xFFu, (int)((r >> 8) & 0xFu))]);
            }
        }
        FieldSink<0u, 0u, 0u, AG_MASKS_E0> ps{sink};
        observe(E, C, ps);
    } else if (part == 1) {
        FieldSink<(1u << NI32) - 1u, 0u, (1u << NF32) - 1u, 0u> ps{sink};
        observe(E, C, ps);
    } else if (part == 3) {
        FieldSink<0u, 0u, 0u, AG_MASKS_E3> ps{sink};
        observe(E, C, ps);
    } else {
        FieldSink<0u, (1u << NI8) - 1u, 0u, AG_MASKS_E2> ps{sink};
        observe(E, C, ps);
        const int nord = E.norders();
        const int all_done = E.ncompleted() == nord && nord > 0 && E.next_order() == nord;
        const int truncated = E.step() >= C.max_steps;
        if (out.term) st32(out.term, t * n + ue, (uint8_t)all_done);
        if (out.trunc) st32(out.trunc, t * n + ue, (uint8_t)truncated);
        if (out.status) st32(out.status, t * n + ue, E.status());
    }
}


// EPW: envs per workgroup (64, 32 or 16; lanes >= EPW idle): fewer envs per CU spread N envs
// over more CUs (every workgroup keeps its 150 KB of LDS, so one workgroup per CU).
template <int EPW, bool STALL = false>   // STALL: the test build (option "test_stall"), see k_step_pipe
__global__ void __launch_bounds__(AG_WAVES * BLOCK) __attribute__((amdgpu_waves_per_eu(1, 2)))
k_step_ag(DevState S, Cfg Ck, int K, uint64_t seed, uint32_t gid0, uint32_t step0, int autoreset, fjsp_out out) {
    static_assert(EPW == 64 || EPW == 32 || EPW == 16, "envs per workgroup");
    FJSP_DIAG(
    const uint64_t t_entry = __builtin_amdgcn_s_memtime();
    )
    // pre-draw work per step: the draw costs more than its loads' latency here (PD shares its
    // SIMD with E0), so four words per step (~33 steps for 30 orders) beat eight (measured)
    constexpr int CR = PG_CR, PB = AG_PB;
    __shared__ uint32_t s_orders[MAX_ORDERS * BLOCK];
    __shared__ uint32_t s_nxt[MAX_ORDERS * BLOCK];
    __shared__ uint32_t s_mb[4][2][BLOCK];   // AM <-> PD mailboxes (predraw_wave)
    __shared__ uint4 s_cp[1][3][BLOCK];   // unused by predraw_wave<ASYNC> (rows travel in registers)
    __shared__ uint16_t s_code[MAX_SLOTS * BLOCK];
    __shared__ uint8_t s_next[MAX_SLOTS * BLOCK];
    __shared__ uint16_t s_cstep[MAX_SLOTS * BLOCK];
    __shared__ PipeSnap snap[2];
    __shared__ uint32_t s_act[3][2][BLOCK];   // step k's actions in slot k % 3 (E0 draws two steps ahead)
    // hand-off slots are lane-major uint4 groups (one 16-byte LDS access per 4 words)
    __shared__ uint4 s_p1[2][2][BLOCK];   // AM post 1 (P1_*), by step parity
    __shared__ uint4 s_p2[BLOCK];         // AM post 2: W9..W12 (machine lists) after the machines' actions
    __shared__ uint4 s_res[2][4][BLOCK];  // P: step k+1's pickup + AGV results (RS_*), by step parity
    __shared__ uint32_t s_kpost[3][BLOCK];      // K after step k: W1 (completed orders) by step parity, final status
    __shared__ uint32_t s_flag1;   // AM posted step k's pickup / AGV words and machine lists (k + 1)
    __shared__ uint32_t s_uflag;   // E3 posted step k+1's pickup (k + 1)
    __shared__ uint32_t s_abort;   // a bounded hand-off wait of this workgroup gave up (spin_until)
    __shared__ uint32_t s_cap;     // its bound (aux word AUX_SPIN_CAP)
    __shared__ uint4 s_pk[BLOCK];   // E3: W0, W4, W5, W7 after step k+1's pickup
    __shared__ uint2 s_pkr[BLOCK];  // E3: its result word, status bits
    __shared__ double s_lut[RLUT_SIZE];
    for (int i = threadIdx.x; i < RLUT_SIZE; i += AG_WAVES * BLOCK) s_lut[i] = Ck.lut[i];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / BLOCK);
    const int lane = threadIdx.x % BLOCK;
    const int blk = xcd_block((int)blockIdx.x, (int)gridDim.x);
    const int e = blk * EPW + lane;
    const bool valid = lane < EPW && e < S.n;
    const uint32_t n = (uint32_t)S.n, ue = (uint32_t)e;
    const Tables TL{s_orders + lane, s_code + lane, s_next + lane, s_cstep + lane, BLOCK};
    FJSP_DIAG(uint64_t ag_busy = 0, ag_wait = 0;   // per step: busy until the barrier; AM: until post 1, K / P: spinning
              uint64_t amt[6] = {0, 0, 0, 0, 0, 0};   // AM: cycles into the step at its phase marks
              uint64_t ag_last = 0;)                   // steps this wave arrived last at the barrier
    if (wave == AG_P) {   // the first two steps' actions
        for (int j = 0; j < 2 && j < K; j++) {
            int act[NA];
            synth_uniform(seed, gid0 + (uint32_t)e, step0 + (uint32_t)j, act);
            s_act[j][0][lane] = pack_actions(act, 0);
            s_act[j][1][lane] = pack_actions(act, 4);
        }
    }
    if (threadIdx.x == 0) { s_flag1 = 0; s_uflag = 0; s_abort = 0; s_cap = aux_words(S)[AUX_SPIN_CAP]; }
    auto ag_spin = [&](uint32_t* flag, uint32_t v) __attribute__((always_inline)) {
        spin_until(flag, v, &s_abort, &s_cap);
    };
    if (valid) {
        // the env's order table, used slot prefix and pre-drawn table live in LDS for the launch
        // (copied in before the first barrier: K's first completions read them), copied by all
        // eight waves, rows r = wave (mod 8), loads batched: a per-lane loop with an LDS store
        // after each load waits out one HBM round trip per row (~30 µs per launch)
        // one round of loads: the state words and, speculatively, every order row, every
        // pre-drawn row and the first 4 slot rows of this wave (all inside the allocations); a
        // row is kept only if the words say it is live.  Slot rows past the first 32 follow in
        // rounds of 8 per wave.
        const uint32_t w0 = S.words[e], w5 = S.words[5 * n + e], pg = S.words[(size_t)PGW * n + e];
        uint32_t ov[MAX_ORDERS / AG_WAVES], pv[MAX_ORDERS / AG_WAVES];
#pragma unroll
        for (int j = 0; j < MAX_ORDERS / AG_WAVES; j++) {
            const size_t o = (size_t)(wave + AG_WAVES * j);
            ov[j] = S.orders[o * n + e];
            pv[j] = S.nxt[o * n + e];
        }
        uint32_t cv[8], xv[8], tv[8];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const size_t q = (size_t)(wave + AG_WAVES * j);
            cv[j] = S.scode[q * n + e];
            xv[j] = S.snext[q * n + e];
            tv[j] = S.scstep[q * n + e];
        }
        const uint32_t nslots = w5 >> 24;
        const uint32_t no = (w0 >> 16) & 0xFFu, npd = (pg & 1u) ? (pg >> 24) & 0x7Fu : 0u;
#pragma unroll
        for (int j = 0; j < MAX_ORDERS / AG_WAVES; j++) {
            const uint32_t o = (uint32_t)(wave + AG_WAVES * j);
            if (o < no) TL.orders[o * BLOCK] = ov[j];
            if (o < npd) s_nxt[o * BLOCK + lane] = pv[j];
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t q = (uint32_t)(wave + AG_WAVES * j);
            if (q < nslots) {
                TL.scode[q * BLOCK] = (uint16_t)cv[j];
                TL.snext[q * BLOCK] = (uint8_t)xv[j];
                TL.scstep[q * BLOCK] = (uint16_t)tv[j];
            }
        }
        for (uint32_t q0 = (uint32_t)wave + 4 * AG_WAVES; q0 < nslots; q0 += 8 * AG_WAVES) {
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t q = q0 + (uint32_t)(AG_WAVES * j);
                cv[j] = q < nslots ? S.scode[(size_t)q * n + e] : 0u;
                xv[j] = q < nslots ? S.snext[(size_t)q * n + e] : 0u;
                tv[j] = q < nslots ? S.scstep[(size_t)q * n + e] : 0u;
            }
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t q = q0 + (uint32_t)(AG_WAVES * j);
                if (q < nslots) {
                    TL.scode[q * BLOCK] = (uint16_t)cv[j];
                    TL.snext[q * BLOCK] = (uint8_t)xv[j];
                    TL.scstep[q * BLOCK] = (uint16_t)tv[j];
                }
            }
        }
        if (wave == AG_AM) {
            s_mb[0][0][lane] = no << 8;   // episode counter 0 | num_orders
            s_mb[1][0][lane] = S.words[3 * n + e];
        }
        if (wave == AG_PD) {   // a table finished in an earlier launch
            s_mb[2][0][lane] = (pg & 1u) ? 1u | (npd << 9) : 0u;
            s_mb[3][0][lane] = (pg & 1u) ? ((pg >> 1) & 0x3FFu) | (((pg >> 11) & 0x3FFu) << 16) | (((pg >> 21) & 1u) << 31) : 0u;
        }
    }
    __syncthreads();
    // [56] launch prologue (entry -> tables in LDS), summed over workgroups
    FJSP_DIAG(
    if (threadIdx.x == 0) atomicAdd(&g_agstamps[56], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_entry));
    )
    if constexpr (STALL) {
        if (wave == AG_AM && blockIdx.x == 0) stall_for_test(S);
    }
    if (wave == AG_AM) {
        const Cfg C = cfg_at(ag_args(), s_lut);
        __builtin_amdgcn_s_setprio(3);   // the machines -> AGV chain is the critical path
        Env E;
        if (valid) env_load(E, S.words, S.n, e);
        int epi = 0;
        bool fresh = true, trunc_prev = false;
        FJSP_DIAG(
        const uint64_t loop_t0 = __builtin_amdgcn_s_memtime();
        )
        for (int k = 0; k <= K; k++) {
            AG_T0();
            AG_MARK(0);
            // the machine queues' front successors as P's AGV of step k saw the queues (AM's own
            // lists: the run phase leaves them alone), read with this step's inputs: the START
            // pops then need no table read after the AGV's drop (machine_execute)
            int pl0 = 0, pl1 = 0, pn0 = NIL, pn1 = NIL;
            if (valid && k < K) {
                pl0 = E.ll(L_M0Q);
                pl1 = E.ll(L_M1Q);
                if (pl0 >= 2) pn0 = TL.snext[E.lh(L_M0Q) * BLOCK];
                if (pl1 >= 2) pn1 = TL.snext[E.lh(L_M1Q) * BLOCK];
            }
            // this step's inputs, read together: K's completion count, the actions, P's results
            uint32_t kc = 0, a0 = 0, a1 = 0, rs[16];
            if (valid) {
                kc = s_kpost[(k - 1) & 1][lane];
                if (k < K) {
                    a0 = s_act[k % 3][0][lane];
                    a1 = s_act[k % 3][1][lane];
                    q_get(&s_res[k & 1][0][lane], 4, rs);
                }
            }
            if (valid) {
                if (k > 0) {   // end of step k - 1: auto-reset once K has counted the completions
                    const int nord = E.norders();
                    const int all_done = (int)(kc & 0xFFu) == nord && nord > 0 && E.next_order() == nord;
                    if (autoreset && (all_done || trunc_prev)) {
                        fresh = true;
                        const uint32_t pr = s_mb[2][k & 1][lane];
                        if ((pr & 1u) && ((pr >> 1) & 0xFFu) == (uint32_t)epi && (int)((pr >> 9) & 0x7Fu) == nord)
                            env_reset_predrawn(E, TL, C, nord, s_mb[3][k & 1][lane], s_nxt + lane);
                        else
                            E = env_reset_cold(E, TL, C, S, e, nord, false);
                        epi = (epi + 1) & 0xFF;
                    }
                }
            }
            AG_MARK(1);
            if (k < K && valid) {
                int act[NA];
#pragma unroll
                for (int a = 0; a < 4; a++) { act[a] = (a0 >> (8 * a)) & 0xFF; act[4 + a] = (a1 >> (8 * a)) & 0xFF; }
                uint32_t r0, r1, pend = 0;
                if (!fresh) {   // step k's pickup and AGV ran on P during step k - 1
                    E.w[0] = (E.w[0] & 0x00FFFFFFu) | (rs[RS_NO] << 24);
                    E.w[4] = rs[RS_W4];
#pragma unroll
                    for (int i = 0; i < 8; i++) E.w[5 + i] = rs[RS_W5 + i];
                    r0 = rs[RS_R0];
                    r1 = rs[RS_R1];
                    E.w[2] |= rs[RS_ST];
                } else {
                    r0 = (pickup_execute(E, TL, C, act[0]) & 0xFFu) | ((uint32_t)act[0] << 8);
                    int mv = 0;
                    r1 = (agv_execute<true>(E, TL, C, act[1], &mv, &pend) & 0xFFu) | ((uint32_t)act[1] << 8);
                    if (mv) E.set_loc(mv);   // the move always lands inside the run
                }
                AG_MARK(2);
                int s0 = -1, s1 = -1;
                const int nk0 = fresh ? -1 : pl0 >= 2 ? pn0 : E.lt(L_M0Q);
                const int nk1 = fresh ? -1 : pl1 >= 2 ? pn1 : E.lt(L_M1Q);
                const uint32_t r2 = (machine_execute<0>(E, TL, act[2], &s0, nk0) & 0xFFu) | ((uint32_t)act[2] << 8);
                const uint32_t r3 = (machine_execute<1>(E, TL, act[3], &s1, nk1) & 0xFFu) | ((uint32_t)act[3] << 8);
                AG_MARK(3);
                {   // the post: pickup / AGV words (P1_*), machine lists
                    const uint32_t p1[8] = {E.w[0], E.w[4], E.w[5], E.w[6], E.w[7], E.w[8], pend, 0u};
                    q_put(&s_p1[k & 1][0][lane], 2, p1);
                    s_p2[lane] = make_uint4(E.w[9], E.w[10], E.w[11], E.w[12]);
                }
                // stored by the lanes that posted, after their post in the same instruction
                // stream (a store by the other lanes could be scheduled first); every workgroup
                // has a valid lane
                __hip_atomic_store(&s_flag1, (uint32_t)(k + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                AG_ACC(ag_wait);
                AG_MARK(4);
                machines_run<true>(E, TL, C, s0, s1);
                AG_MARK(5);
                if (E.ll(L_M0Q) > 127 || E.ll(L_M1Q) > 127) E.flag(ST_OBS_OVERFLOW | ST_DIVERGED);
                const uint32_t v[16] = {E.w[0], E.w[2], E.w[4], E.w[5], E.w[6], E.w[7], E.w[8], E.w[9], E.w[10],
                                        E.w[11], E.w[12], E.w[17], E.w[18], r0 | (r1 << 16), r2 | (r3 << 16), 0u};
                snap_put4(snap[k & 1], 0, lane, v);
                trunc_prev = E.step() >= C.max_steps;
                E.set_step(E.step() + 1);
                fresh = false;
            }
            if (valid) {   // PD's mailbox for the next step (off the way to the post: its release waits for them)
                s_mb[0][(k + 1) & 1][lane] = (uint32_t)epi | ((uint32_t)E.norders() << 8);
                s_mb[1][(k + 1) & 1][lane] = E.w[3];
            }
            AG_ACC(ag_busy);
            AG_BARRIER();
        }
        FJSP_DIAG(
        if (lane == 0) atomicAdd(&g_agstamps[24], (unsigned long long)(__builtin_amdgcn_s_memtime() - loop_t0));
        )
        if (valid) {
            s_act[0][0][lane] = (uint32_t)E.norders();   // for the copy-out by all waves below
            s_act[0][1][lane] = (uint32_t)E.slot_next();
            E.w[2] |= s_kpost[2][lane];
            // every wait happened before the last barrier: a give-up is visible here
            if (s_abort) E.w[2] |= ST_SPIN_TIMEOUT | ST_DIVERGED;
#pragma unroll
            for (int i = 0; i < NSTATE; i++)
                if (!((K_WORDS >> i) & 1u)) S.words[i * n + e] = E.w[i];
        }
    } else if (wave == AG_K) {
        const Cfg C = cfg_at(ag_args(), s_lut);
        __builtin_amdgcn_s_setprio(2);
        Env E;
#pragma unroll
        for (int i = 0; i < NSTATE; i++) E.w[i] = 0u;
        if (valid) {
#pragma unroll
            for (int i = 0; i < NSTATE; i++)
                if ((K_WORDS >> i) & 1u) E.w[i] = S.words[i * n + e];
            E.w[0] = S.words[e] & 0xFFFFu;   // the step counter (AM owns W0)
        }
        bool trunc_prev = false;
        for (int k = 0; k <= K; k++) {
            AG_T0();
            bool fresh = k == 0;
            if (valid && k > 0) {   // the reset AM makes at the top of this step, on the packaging words
                const uint32_t w0a = s_p1[(k - 1) & 1][0][lane].x;   // AM's W0 after step k-1's pickup (P1_W0)
                const int nord = (int)((w0a >> 16) & 0xFFu);
                const int all_done = E.ncompleted() == nord && nord > 0 && (int)(w0a >> 24) == nord;
                if (autoreset && (all_done || trunc_prev)) {   // env_clear of the packaging words
                    fresh = true;
                    E.w[0] = 0u; E.w[1] = 0u; E.w[2] = 0u;
#pragma unroll
                    for (int s = 0; s < 4; s++) {
                        E.w[7 + L_PKG + s] = (uint32_t)NIL | ((uint32_t)NIL << 8);
                        E.w[20 + s] = (uint32_t)NIL << 2;
                        E.w[26 + s] = 0u;
                    }
                    E.w[24] = 0u; E.w[25] = 0u;
                }
            }
            if (k < K) {
                // the AGV's drop of step k: P computed it during step k-1; a lane that just reset
                // carries nothing; the first step of a launch runs its AGV on AM (post 1)
                uint32_t pend = 0;
                if (k == 0) {
                    AG_SPIN_T0();
                    ag_spin(&s_flag1, 1u);
                    AG_SPIN_ACC();
                    if (valid) pend = s_p1[0][1][lane].z;   // P1_PEND
                } else if (valid && !fresh) {
                    pend = s_res[k & 1][RS_PEND / 4][lane].w;   // RS_PEND = 15
                }
                if (valid) {
                    const int step = E.step(), tp0 = E.total_packaged();
                    const uint32_t a1 = s_act[k % 3][1][lane];
                    // completions due this step (NORMAL events older than the step's actions)
                    int done[4], orders_done = 0;
                    const bool due0 = pack_due<0>(E, TL, step), due1 = pack_due<1>(E, TL, step);
                    const bool due2 = pack_due<2>(E, TL, step), due3 = pack_due<3>(E, TL, step);
                    done[0] = pack_complete<0>(E, TL, due0, &orders_done);
                    done[1] = pack_complete<1>(E, TL, due1, &orders_done);
                    done[2] = pack_complete<2>(E, TL, due2, &orders_done);
                    done[3] = pack_complete<3>(E, TL, due3, &orders_done);
                    if (pend) agv_pack_drop(E, TL, C, pend);   // routing reads the in-flight counts before the run
                    int st[4] = {0, 0, 0, 0};
                    uint32_t r[4];
                    r[0] = pack_execute<0>(E, (int)(a1 & 0xFFu), &st[0]);
                    r[1] = pack_execute<1>(E, (int)((a1 >> 8) & 0xFFu), &st[1]);
                    r[2] = pack_execute<2>(E, (int)((a1 >> 16) & 0xFFu), &st[2]);
                    r[3] = pack_execute<3>(E, (int)(a1 >> 24), &st[3]);
                    pack_finish<0>(E, TL, C, st[0], done[0]);
                    pack_finish<1>(E, TL, C, st[1], done[1]);
                    pack_finish<2>(E, TL, C, st[2], done[2]);
                    pack_finish<3>(E, TL, C, st[3], done[3]);
                    E.set_ncompleted(E.ncompleted() + orders_done);
                    if (E.p_queued(0) > 127 || E.p_queued(1) > 127 || E.p_queued(2) > 127 || E.p_queued(3) > 127)
                        E.flag(ST_OBS_OVERFLOW | ST_DIVERGED);
                    s_kpost[k & 1][lane] = E.w[1];
#pragma unroll
                    for (int q = 0; q < 4; q++) r[q] = (r[q] & 0xFFu) | (((a1 >> (8 * q)) & 0xFFu) << 8);
                    const uint32_t v[16] = {E.w[1], E.w[20], E.w[21], E.w[22], E.w[23], E.w[26], E.w[27], E.w[28],
                                            E.w[29], E.w[2],
                                            (uint32_t)orders_done | ((uint32_t)(E.total_packaged() - tp0) << 16),
                                            r[0] | (r[1] << 16), r[2] | (r[3] << 16), 0u, 0u, 0u};
                    snap_put4(snap[k & 1], 4, lane, v);
                    trunc_prev = step >= C.max_steps;
                    E.set_step(step + 1);
                }
            } else if (valid) {
                s_kpost[2][lane] = E.w[2];   // status bits for AM's final store of W2
            }
            AG_ACC(ag_busy);
            AG_BARRIER();
        }
        if (valid) {
#pragma unroll
            for (int i = 0; i < NSTATE; i++)
                if ((K_WORDS >> i) & 1u) S.words[i * n + e] = E.w[i];
        }
    } else if (wave == AG_P) {
        const Cfg C = cfg_at(ag_args(), s_lut);
        __builtin_amdgcn_s_setprio(3);
        // W6..W12 after this wave's last AGV: the next AGV's own words and the list fronts it
        // prefetches, unless AM reset the env (or the launch starts): then AM's post of the step
        uint32_t sa[7] = {0u, 0u, 0u, 0u, 0u, 0u, 0u};
        for (int k = 0; k <= K; k++) {
            AG_T0();
            if (k + 1 < K) {   // step k + 1's AGV: its own half now, the rest on AM's post and E3's pickup
                const int act1 = (int)((s_act[(k + 1) % 3][0][lane] >> 8) & 0xFFu);
                AG_MARK(0);
                const bool fresh = ag_fresh(k, valid, s_p1, s_kpost, lane, C, autoreset);
                AG_SPIN_T0();
                const bool wait_first = __ballot(valid && fresh) != 0;
                if (wait_first) ag_spin(&s_flag1, (uint32_t)(k + 1));
                AG_MARK(1);
                Env Ea;
#pragma unroll
                for (int i = 0; i < NSTATE; i++) Ea.w[i] = 0u;
                AgvPre pre{};
                if (valid) {
                    if (fresh) {
                        uint32_t p1[8];
                        q_get(&s_p1[k & 1][0][lane], 2, p1);
                        const uint4 p2 = s_p2[lane];
                        sa[0] = p1[P1_W6]; sa[1] = p1[P1_W7]; sa[2] = p1[P1_W8];
                        sa[3] = p2.x; sa[4] = p2.y; sa[5] = p2.z; sa[6] = p2.w;
                    }
#pragma unroll
                    for (int i = 0; i < 7; i++) Ea.w[6 + i] = sa[i];
                    pre = agv_pre(Ea, TL, C, act1);
                }
                AG_MARK(2);
                if (!wait_first) ag_spin(&s_flag1, (uint32_t)(k + 1));
                ag_spin(&s_uflag, (uint32_t)(k + 1));
                AG_SPIN_ACC();
                AG_MARK(3);
                if (valid) {
                    const uint4 p2 = s_p2[lane];
                    const uint4 pk = s_pk[lane];        // E3: W0, W4, W5, W7 after step k+1's pickup
                    const uint2 pr = s_pkr[lane];       // E3: pickup result, status bits
                    Ea.w[5] = pk.z; Ea.w[7] = pk.w;
                    Ea.w[9] = p2.x; Ea.w[10] = p2.y; Ea.w[11] = p2.z; Ea.w[12] = p2.w;
                    int mv = 0;
                    uint32_t pend = 0;
                    const uint32_t r1 = (agv_fin(Ea, TL, pre, &mv, &pend) & 0xFFu) | ((uint32_t)act1 << 8);
                    if (mv) Ea.set_loc(mv);
                    AG_MARK(4);
#pragma unroll
                    for (int i = 0; i < 7; i++) sa[i] = Ea.w[6 + i];
                    const uint32_t rs[16] = {pk.x >> 24, pk.y, Ea.w[5], Ea.w[6], Ea.w[7], Ea.w[8], Ea.w[9],
                                             Ea.w[10], Ea.w[11], Ea.w[12], pr.x, r1, pr.y | Ea.w[2], 0u, 0u, pend};
                    q_put(&s_res[(k + 1) & 1][0][lane], 4, rs);
                }
                AG_MARK(5);
            }
            AG_ACC(ag_busy);
            AG_BARRIER();
        }
    } else if (wave == AG_PD) {
        predraw_wave<CR, PB, true, true>(S, K, lane, e, valid, (size_t)blk * EPW, s_mb, s_cp, s_nxt);
    } else {
        // E0: step k+2's actions, rewards, the pickup's masks; E1: int32 and float32 fields; E2:
        // int8 fields, term, trunc, status, the AGV's pickup / drop masks; E3: step k+1's pickup
        // station (for P), the other masks (balanced by measured cycles: scripts/diag_ag_stamps.py;
        // E0 shares P's SIMD)
        const Cfg C = cfg_at(ag_args(), s_lut);
        const int part = wave == AG_E0 ? 0 : wave == AG_E1 ? 1 : wave == AG_E2 ? 2 : 3;
        if (part == 3) __builtin_amdgcn_s_setprio(2);   // E3 runs the pickup station for P first
        const AgArgs* ea = ag_args();   // the outputs and E0's action stream, read in this branch
        fjsp_out eo = kNoOutDev;
        eo.obs_i32 = ea->out.obs_i32; eo.obs_i8 = ea->out.obs_i8; eo.obs_f32 = ea->out.obs_f32; eo.masks = ea->out.masks;
        eo.rewards = ea->out.rewards; eo.term = ea->out.term; eo.trunc = ea->out.trunc; eo.status = ea->out.status;
        const uint64_t eseed = ea->seed;
        const uint32_t egid = ea->gid0 + (uint32_t)e, estep = ea->step0;
        for (int k = 0; k <= K; k++) {
            AG_T0();
            if (part == 3 && k + 1 < K) {   // step k+1's pickup station, from P's AGV result of step k
                const bool fresh = ag_fresh(k, valid, s_p1, s_kpost, lane, C, autoreset);
                if (__ballot(valid && fresh) != 0) ag_spin(&s_flag1, (uint32_t)(k + 1));
                AG_MARK(3);
                if (valid) {
                    Env Ep;
#pragma unroll
                    for (int i = 0; i < NSTATE; i++) Ep.w[i] = 0u;
                    if (fresh) {
                        uint32_t p1[8];
                        q_get(&s_p1[k & 1][0][lane], 2, p1);
                        Ep.w[0] = p1[P1_W0]; Ep.w[4] = p1[P1_W4]; Ep.w[5] = p1[P1_W5]; Ep.w[7] = p1[P1_W7];
                    } else {
                        uint32_t rs[16];
                        q_get(&s_res[k & 1][0][lane], 2, rs);   // RS_NO, RS_W4, RS_W5..: W5, W6, W7
                        Ep.w[0] = (s_p1[(k - 1) & 1][0][lane].x & 0x00FFFFFFu) | (rs[RS_NO] << 24);
                        Ep.w[4] = rs[RS_W4]; Ep.w[5] = rs[RS_W5]; Ep.w[7] = rs[RS_W5 + 2];
                    }
                    const int act0 = (int)(s_act[(k + 1) % 3][0][lane] & 0xFFu);
                    const uint32_t r0 = (pickup_execute(Ep, TL, C, act0) & 0xFFu) | ((uint32_t)act0 << 8);
                    AG_MARK(4);
                    s_pk[lane] = make_uint4(Ep.w[0], Ep.w[4], Ep.w[5], Ep.w[7]);
                    s_pkr[lane] = make_uint2(r0, Ep.w[2]);
                    __hip_atomic_store(&s_uflag, (uint32_t)(k + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            AG_MARK(0);
            if (part == 0 && k + 2 < K) {   // E0 draws step k + 2's actions (uniform random)
                int act[NA];
                synth_uniform(eseed, egid, estep + (uint32_t)(k + 2), act);
                s_act[(k + 2) % 3][0][lane] = pack_actions(act, 0);
                s_act[(k + 2) % 3][1][lane] = pack_actions(act, 4);
            }
            if (k > 0 && valid) {
                const uint32_t t = (uint32_t)(k - 1);
                uint32_t v[SNAP_N];
                snap_get(snap[(k - 1) & 1], lane, v);
                if (part == 2 && s_abort) v[SA_ST] |= ST_SPIN_TIMEOUT | ST_DIVERGED;
                FJSP_DIAG(
                __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the snapshot arrived
                )
                AG_MARK(1);
                ag_emit(part, v, t, n, ue, C, eo);
            }
            AG_MARK(2);
            AG_ACC(ag_busy);
            AG_BARRIER();
        }
    }
    __syncthreads();
    // the state pointers read again for the copy-out (otherwise live in SGPRs through every
    // role's step loop)
    const DevState So = ag_args()->S;
    if (threadIdx.x == 0) report_abort(So, s_abort);
    FJSP_DIAG(
    const uint64_t t_out = __builtin_amdgcn_s_memtime();
    )
    if (valid) {   // the order table and the used slot prefix back to HBM, rows r = wave (mod 8)
        const uint32_t no = s_act[0][0][lane], ns = s_act[0][1][lane];
        for (uint32_t o = (uint32_t)wave; o < no; o += AG_WAVES) So.orders[(size_t)o * n + e] = TL.orders[o * BLOCK];
        for (uint32_t q = (uint32_t)wave; q < ns; q += AG_WAVES) {
            So.scode[(size_t)q * n + e] = TL.scode[q * BLOCK];
            So.snext[(size_t)q * n + e] = TL.snext[q * BLOCK];
            So.scstep[(size_t)q * n + e] = TL.scstep[q * BLOCK];
        }
    }
    FJSP_DIAG(
    // stamp slots by role: AM 0, E0 1, K 2, E1 3, P 4, PD 5, E2 6, E3 7 (scripts/diag_ag_stamps.py):
    // [2 slot] busy, [2 slot + 1] wait, [16] steps, [17] SIMD map, [18..23] AM marks, [24] AM wall,
    // [25 + slot] last arrivals
    const int slot = wave == AG_AM ? 0 : wave == AG_E0 ? 1 : wave == AG_K ? 2 : wave == AG_E1 ? 3 : wave == AG_P ? 4
                   : wave == AG_PD ? 5 : wave == AG_E2 ? 6 : 7;
    if (lane == 0 && blockIdx.x == 0) {   // SIMD of each role (HW_REG_HW_ID bits 5:4)
        const uint32_t hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
        atomicOr(&g_agstamps[17], (unsigned long long)((hw >> 4) & 3u) << (4 * slot));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0 && wave == AG_AM) {   // [57] copy-out drained, [58] entry -> end (AM's wave)
        atomicAdd(&g_agstamps[57], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_out));
        atomicAdd(&g_agstamps[58], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_entry));
    }
    if (lane == 0 && wave != AG_PD) {
        atomicAdd(&g_agstamps[2 * slot], (unsigned long long)ag_busy);
        atomicAdd(&g_agstamps[2 * slot + 1], (unsigned long long)ag_wait);
        atomicAdd(&g_agstamps[25 + slot], (unsigned long long)ag_last);
        if (wave == AG_AM) {
            atomicAdd(&g_agstamps[16], (unsigned long long)(K + 1));
            for (int i = 0; i < 6; i++) atomicAdd(&g_agstamps[18 + i], (unsigned long long)amt[i]);
        }
        if (wave == AG_P)
            for (int i = 0; i < 6; i++) atomicAdd(&g_agstamps[33 + i], (unsigned long long)amt[i]);
        if (wave == AG_E3)   // after the pickup post, the snapshot, the stores, the fresh wait, the pickup
            for (int i = 0; i < 6; i++) atomicAdd(&g_agstamps[40 + i], (unsigned long long)amt[i]);
        if (wave == AG_E2)   // top, the snapshot, the stores
            for (int i = 0; i < 4; i++) atomicAdd(&g_agstamps[46 + i], (unsigned long long)amt[i]);
    }
    )
}

// transition_memory.py:83-105 over a [T][M] rollout buffer; column m = a*N + e, one lane per
// column, the scan in the reference's operation order (backwards over t).  The scan is one
// dependent chain per column and the chip holds only M / 64 waves of them (512 at 8 x 4 096
// columns: 2 per CU), so the loads are software-pipelined: the inputs of GAE_U timesteps go out
// in one batch into registers (buffer A), the next GAE_U (buffer B) are issued before A's scan,
// and so on — two batches of independent loads in flight per wave instead of one dependent
// round trip per timestep.  Only the loads move; the arithmetic is the same sequence per column.
// SHARED: values f32/f64 [T + 1][N] shared by the agents of an env (the critic's value, a2c.py:
// 321-332), boot = row T; else values [T][M] and boot [M].
constexpr int GAE_U = 16;
template <class VT, bool SHARED>
struct GaeChunk {
    double r[GAE_U];
    VT v[GAE_U];
    uint8_t d[GAE_U];
};
// Loads of the GAE_U timesteps t0, t0 - 1, ... (rows below 0 clamped to row 0: never used, and
// no branch around a load — a load under a branch made the compiler drain every load at the join).
template <class VT, bool SHARED>
__device__ __forceinline__ void gae_load(GaeChunk<VT, SHARED>& c, const double* __restrict__ r,
                                         const VT* __restrict__ v, const uint8_t* __restrict__ done, int t0, int N,
                                         int M, int m, int e) {
#pragma unroll
    for (int j = 0; j < GAE_U; j++) {
        const int t = t0 - j > 0 ? t0 - j : 0;
        c.r[j] = __builtin_nontemporal_load(r + (size_t)t * M + m);
        c.v[j] = v[SHARED ? (size_t)t * N + e : (size_t)t * M + m];
        c.d[j] = done[(size_t)t * N + e];
    }
}
// The scan over timesteps t0, t0 - 1, ... down to max(t0 - GAE_U + 1, 0) (FULL: all GAE_U).
template <class VT, bool SHARED, bool FULL>
__device__ __forceinline__ void gae_scan(const GaeChunk<VT, SHARED>& c, int t0, int T, int M, int m, double bootv,
                                         double gamma, double gl, double& nv, double& rr, double& gae,
                                         double* __restrict__ ret, double* __restrict__ adv) {
#pragma unroll
    for (int j = 0; j < GAE_U; j++) {
        const int t = t0 - j;
        if (FULL || t >= 0) {
            if (t == T - 1 || c.d[j]) {   // a trajectory ends at t
                nv = (t == T - 1 && !c.d[j]) ? bootv : 0.0;
                rr = nv;
                gae = 0.0;
            }
            const size_t i = (size_t)t * M + m;
            const double rt = c.r[j];
            const double vt = (double)c.v[j];
            rr = rt + gamma * rr;
            __builtin_nontemporal_store(rr, ret + i);
            const double td = rt + gamma * nv - vt;
            gae = td + gl * gae;
            __builtin_nontemporal_store(gae, adv + i);
            nv = vt;
        }
    }
}
template <class VT, bool SHARED>
__device__ __forceinline__ void gae_scan_any(const GaeChunk<VT, SHARED>& c, int t0, int T, int M, int m, double bootv,
                                             double gamma, double gl, double& nv, double& rr, double& gae,
                                             double* __restrict__ ret, double* __restrict__ adv) {
    if (t0 >= GAE_U - 1) gae_scan<VT, SHARED, true>(c, t0, T, M, m, bootv, gamma, gl, nv, rr, gae, ret, adv);
    else gae_scan<VT, SHARED, false>(c, t0, T, M, m, bootv, gamma, gl, nv, rr, gae, ret, adv);
}
template <class VT, bool SHARED>
__global__ void __launch_bounds__(64) k_gae(const double* __restrict__ r, const VT* __restrict__ v,
                                            const uint8_t* __restrict__ done, const double* __restrict__ boot, int T,
                                            int N, int M, double gamma, double lamb, double* __restrict__ ret,
                                            double* __restrict__ adv) {
    const int m = blockIdx.x * 64 + threadIdx.x;
    if (m >= M) return;
    const int e = m % N;
    const double gl = gamma * lamb;
    const double bootv = SHARED ? (double)v[(size_t)T * N + e] : boot[m];
    double nv = 0.0, rr = 0.0, gae = 0.0;
    GaeChunk<VT, SHARED> A, B;
    int t0 = T - 1;
    gae_load(A, r, v, done, t0, N, M, m, e);
    for (;;) {   // A holds t0.., B is loaded before A's scan, and the other way round
        gae_load(B, r, v, done, t0 - GAE_U, N, M, m, e);
        gae_scan_any(A, t0, T, M, m, bootv, gamma, gl, nv, rr, gae, ret, adv);
        t0 -= GAE_U;
        if (t0 < 0) break;
        gae_load(A, r, v, done, t0 - GAE_U, N, M, m, e);
        gae_scan_any(B, t0, T, M, m, bootv, gamma, gl, nv, rr, gae, ret, adv);
        t0 -= GAE_U;
        if (t0 < 0) break;
    }
}

// The shared-value scan (fjsp_gae_shared, N % 64 == 0) with its loads on a loader wave: per
// workgroup 64 columns (one agent, 64 consecutive envs), a scan wave and a loader wave that keeps
// L chunks of U timesteps in flight into an LDS ring by 16-byte LDS DMAs (r: two timesteps per
// instruction, values four, done flags sixteen: 13 instructions per 16-timestep chunk, waited for
// by a counted vmcnt), so the scan wave issues only its stores and LDS reads.  Same arithmetic
// sequence per column as k_gae.  Measured at 256 x 8 x 4 096: 37.4 us against 42.4 us for
// k_gae<float, true> (scripts/diag_gae.py, profiles/r04/gae_ab.json).
constexpr int GLW_U = 16, GLW_L = 2;
struct GaeSlot {
    double r[GLW_U][64];
    float v[GLW_U][64];
    uint8_t d[GLW_U][64];
};
__device__ __forceinline__ void dma16(const void* g, void* s) {
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)g, (__attribute__((address_space(3))) void*)s,
                                     16, 0, 0);
}
__global__ void __launch_bounds__(128) k_gae_lw(const double* __restrict__ r, const float* __restrict__ v,
                                               const uint8_t* __restrict__ done, int T, int N, int M, double gamma,
                                               double lamb, double* __restrict__ ret, double* __restrict__ adv) {
    constexpr int U = GLW_U, L = GLW_L, S = L + 1, PER = U / 2 + U / 4 + U / 16;
    static_assert(U % 16 == 0 && PER * (L - 1) <= 63, "chunk shape / vmcnt");
    __shared__ GaeSlot slot[S];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int m0 = blockIdx.x * 64, e0 = m0 % N;
    const int nch = (T + U - 1) / U;
    auto issue = [&](int c) __attribute__((always_inline)) {   // chunk c: timesteps T-1-cU down (rows < 0: row 0)
        GaeSlot& s = slot[c % S];
        const int t0 = T - 1 - c * U;
#pragma unroll
        for (int i = 0; i < U / 2; i++) {
            const int t = max(t0 - 2 * i - (lane >> 5), 0);
            dma16(r + (size_t)t * M + m0 + 2 * (lane & 31), &s.r[2 * i][0]);
        }
#pragma unroll
        for (int i = 0; i < U / 4; i++) {
            const int t = max(t0 - 4 * i - (lane >> 4), 0);
            dma16(v + (size_t)t * N + e0 + 4 * (lane & 15), &s.v[4 * i][0]);
        }
#pragma unroll
        for (int i = 0; i < U / 16; i++) {
            const int t = max(t0 - 16 * i - (lane >> 2), 0);
            dma16(done + (size_t)t * N + e0 + 16 * (lane & 3), &s.d[16 * i][0]);
        }
    };
    constexpr int VM = PER * (L - 1);   // vmcnt <= VM: every chunk but the last L - 1 issued has landed
    constexpr int WAIT = (VM & 15) | ((VM >> 4) << 14) | (7 << 4) | (15 << 8);
    if (wave == 1) {
        for (int c = 0; c < L; c++) issue(c);
        __builtin_amdgcn_s_waitcnt(WAIT);
    }
    __syncthreads();
    const int m = m0 + lane;
    const double gl = gamma * lamb;
    const double bootv = (double)v[(size_t)T * N + e0 + lane];
    double nv = 0.0, rr = 0.0, gae = 0.0;
    for (int p = 0; p < nch; p++) {
        if (wave == 1) {
            issue(p + L);                          // into the slot chunk p - 1 held (scanned)
            __builtin_amdgcn_s_waitcnt(WAIT);      // chunk p + 1 has landed
        } else {
            const GaeSlot& s = slot[p % S];
            const int t0 = T - 1 - p * U;
#pragma unroll
            for (int j = 0; j < U; j++) {
                const int t = t0 - j;
                if (t < 0) continue;
                const uint8_t dj = s.d[j][lane];
                if (t == T - 1 || dj) {   // a trajectory ends at t
                    nv = (t == T - 1 && !dj) ? bootv : 0.0;
                    rr = nv;
                    gae = 0.0;
                }
                const size_t i = (size_t)t * M + m;
                const double rt = s.r[j][lane];
                const double vt = (double)s.v[j][lane];
                rr = rt + gamma * rr;
                __builtin_nontemporal_store(rr, ret + i);
                const double td = rt + gamma * nv - vt;
                gae = td + gl * gae;
                __builtin_nontemporal_store(gae, adv + i);
                nv = vt;
            }
        }
        __syncthreads();
    }
    if (wave == 1) __builtin_amdgcn_s_waitcnt(0x0F70);   // no LDS DMA outlives the workgroup
}

}  // namespace

// ================================================================ C-ABI
struct fjsp_handle {
    fjsp_config cfg;
    Cfg dcfg;
    int n;
    int device;
    hipStream_t stream;
    DevState S;
    void* base;
    size_t bytes;
    int has_reset;
    hipEvent_t ev0, ev1;
    int timed;
    double* lut_dev;
    double lut_host[RLUT_SIZE];
    int use_lds;     // fused kernel variant (fjsp_set_option "fused_lds")
    int use_staged;  // LDS-staged wide output stores (fjsp_set_option "staged_stores")
    int timing;      // hipEvent bracketing of step launches (off while graph-capturing)
    int use_pipe;    // two-wave pipelined k_step_many for lean outputs (fjsp_set_option "pipeline")
    int use_pg;      // pre-draw wave in the pipelined kernel (fjsp_set_option "predraw")
    int use_ag;      // agent-group pipeline k_step_ag for uniform-random actions (fjsp_set_option "agents")
    int ag_epw;      // k_step_ag envs per workgroup: 64 / 32 / 16, 0 = auto (fjsp_set_option "ag_envs")
    int step_epw;    // k_step envs per workgroup: 64 / 32 / 16, 0 = 64 (fjsp_set_option "step_envs")
    const char* last_kernel;   // name of the last step kernel launched (fjsp_last_kernel)
    uint32_t env_id_base;      // global id of env 0 (fjsp_set_option "env_id_base")
    // fjsp_a2c_policy_step's tile hand-off: [ntiles] arrival counters (zero between launches),
    // then [ntiles][8][16] action words; outside the state block (not part of a snapshot)
    uint32_t* tiles;
    int ntiles;
    int test_stall;   // option "test_stall" (tests): launch the STALL builds of the multi-wave kernels
    // step server (fjsp_server_*): the persistent k_step_server, its control block in host memory
    ServerCtl* srv;
    uint32_t* srv_relay;      // device words: workgroup 0 relays each request / stop to the others
    hipStream_t srv_stream;   // its own stream: nothing on h->stream queues behind the resident kernel
    hipEvent_t srv_ev;        // h->stream's work before a (re)launch
    int srv_configured, srv_running, srv_autoreset, srv_nwg;
    const uint8_t* srv_actions;
    fjsp_out srv_out;
    uint32_t srv_epoch;
    std::chrono::steady_clock::time_point srv_last;   // the last request (idle relaunch)
};

static thread_local std::string g_err;

// shared with the other translation unit of the library (fjsp_policy.hip)
int fjsp_internal_fail(const char* msg) {
    g_err = msg;
    return -1;
}

static int fail(const char* msg) {
    g_err = msg;
    return -1;
}
static int hip_fail(const char* what, hipError_t e) {
    char buf[256];
    snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
    g_err = buf;
    return -2;
}
#define HIPCHK(x)                                 \
    do {                                          \
        hipError_t _e = (x);                      \
        if (_e != hipSuccess) return hip_fail(#x, _e); \
    } while (0)

// words of the tile hand-off block: counters (padded to 64 words), then the action words
static size_t tile_words(int ntiles) { return (((size_t)ntiles + 63) & ~(size_t)63) + (size_t)ntiles * 8 * 16; }

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

extern "C" {

static int server_stop(fjsp_handle* h) {
    if (!h->srv_running) return 0;
    DeviceGuard g(h->device);
    __atomic_store_n(&h->srv->stop, 1u, __ATOMIC_RELEASE);
    const hipError_t e = hipStreamSynchronize(h->srv_stream);   // bounded: every poll reads stop
    h->srv_running = 0;
    __atomic_store_n(&h->srv->stop, 0u, __ATOMIC_RELEASE);
    if (e != hipSuccess) return hip_fail("step server stop", e);
    return 0;
}
// every other entry point that touches the envs' state stops a resident server first (its state
// words live in the kernel's registers until it leaves)
#define SERVER_QUIESCE(h)                                 \
    do {                                                  \
        if ((h) && (h)->srv_running) {                    \
            if (int rc_ = server_stop(h)) return rc_;     \
        }                                                 \
    } while (0)

int fjsp_abi_version(void) { return FJSP_ABI_VERSION; }
const char* fjsp_last_error(void) { return g_err.c_str(); }

int fjsp_default_config(fjsp_config* c) {
    if (!c) return fail("null config");
    c->num_trays = 1000;
    c->tray_capacity = 5;
    c->mask_tray_capacity = 5;
    c->storage_capacity = 100;
    c->step_size = 10;
    c->max_episode_steps = 200;
    c->agv_speed = 1;
    c->pt_small = 60;
    c->pt_big = 120;
    c->pt_packaging = 30;
    c->packaging_capacity = 20;
    return 0;
}

int fjsp_default_reward_weights(fjsp_reward_weights* w) {
    if (!w) return fail("null weights");
    const double d[NW] = {100.0, 10.0, -0.1, 1.0, 5.0, -1.0, 2.0, -0.1, 10.0, -5.0, 5.0, 1.0, -2.0, 20.0, 2.0, -1.0};
    static_assert(sizeof(fjsp_reward_weights) == sizeof(double) * NW, "reward weight layout");
    memcpy(w, d, sizeof(d));
    return 0;
}

int fjsp_set_reward_weights(fjsp_handle* h, const fjsp_reward_weights* w) {
    if (!h || !w) return fail("null argument");
    SERVER_QUIESCE(h);
    DeviceGuard g(h->device);
    build_reward_lut(reinterpret_cast<const double*>(w), h->cfg.step_size, h->lut_host);
    // stream-ordered: launches queued before this call keep the old table contents
    HIPCHK(hipStreamSynchronize(h->stream));
    HIPCHK(hipMemcpy(h->lut_dev, h->lut_host, sizeof(double) * RLUT_SIZE, hipMemcpyHostToDevice));
    return 0;
}

int fjsp_check_config(const fjsp_config* c) {
    if (!c) return fail("null config");
    if (c->step_size <= 0) return fail("step_size must be > 0");
    if (c->agv_speed <= 0 || 8 >= c->step_size * c->agv_speed)
        return fail("AGV moves must finish inside one step: 8 / agv_speed < step_size");
    if (c->pt_small <= 0 || c->pt_small % c->step_size) return fail("pt_small must be a positive multiple of step_size");
    if (c->pt_big <= 0 || c->pt_big % c->step_size) return fail("pt_big must be a positive multiple of step_size");
    if (c->pt_packaging <= 0 || c->pt_packaging % c->step_size)
        return fail("pt_packaging must be a positive multiple of step_size");
    if (c->tray_capacity < 1 || c->tray_capacity > 7) return fail("tray_capacity must be in 1..7");
    if (c->max_episode_steps < 0 || c->max_episode_steps > 253) return fail("max_episode_steps must be in 0..253");
    if (c->packaging_capacity < 1 || c->packaging_capacity > 255) return fail("packaging_capacity must be in 1..255");
    if (c->storage_capacity < 0 || c->num_trays < 0) return fail("negative capacity");
    return 0;
}

int fjsp_create(const fjsp_config* cfg, int32_t num_envs, int32_t device, void* hip_stream, fjsp_handle** out) {
    if (!out) return fail("null out");
    *out = nullptr;
    fjsp_config c;
    if (cfg) c = *cfg; else fjsp_default_config(&c);
    if (fjsp_check_config(&c)) return -1;
    if (num_envs <= 0) return fail("num_envs must be > 0");
    DeviceGuard g(device);
    fjsp_handle* h = new fjsp_handle();   // value-initialised: every pointer starts null
    h->cfg = c;
    h->n = num_envs;
    h->device = device;
    h->stream = (hipStream_t)hip_stream;
    // kernel-variant defaults (fjsp_set_option changes them per handle; every variant is
    // byte-identical): LDS tables auto (every workgroup a CU), direct stores, the pipelined /
    // pre-draw / agent-group kernels on, k_step_ag's envs per workgroup auto, per-launch events on
    h->use_lds = -1;
    h->use_staged = 0;
    h->timing = 1;
    h->use_pipe = 1;
    h->use_pg = 1;
    h->use_ag = 1;
    h->ag_epw = 0;
    h->step_epw = 0;
    h->dcfg.step_size = c.step_size;
    h->dcfg.max_steps = c.max_episode_steps;
    h->dcfg.tray_cap = c.tray_capacity;
    h->dcfg.mask_tray_cap = c.mask_tray_capacity;
    h->dcfg.storage_cap = c.storage_capacity;
    h->dcfg.pool0 = c.num_trays < 1000 ? c.num_trays : 1000;
    h->dcfg.pkg_cap = c.packaging_capacity;
    h->dcfg.ptk_small = c.pt_small / c.step_size;
    h->dcfg.ptk_big = c.pt_big / c.step_size;
    h->dcfg.ptk_pack = c.pt_packaging / c.step_size;

    const size_t n = (size_t)num_envs;
    const size_t b_words = ((size_t)NWORDS * n + AUX_WORDS) * 4, b_orders = (size_t)MAX_ORDERS * n * 4;
    const size_t b_scode = (size_t)MAX_SLOTS * n * 2, b_snext = (size_t)MAX_SLOTS * n, b_scstep = (size_t)MAX_SLOTS * n * 2;
    const size_t b_mt = (size_t)2 * MT_N * n * 4, b_nxt = (size_t)MAX_ORDERS * n * 4;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    h->bytes = al(b_words) + al(b_orders) + al(b_scode) + al(b_snext) + al(b_scstep) + al(b_nxt) + al(b_mt);
    // every failure below goes through fjsp_destroy, which frees whatever was allocated
    auto bail = [&](const char* what, hipError_t err) { fjsp_destroy(h); return hip_fail(what, err); };
    hipError_t e = hipMalloc(&h->base, h->bytes);
    if (e != hipSuccess) { h->base = nullptr; return bail("hipMalloc(state)", e); }
    char* p = (char*)h->base;
    h->S.words = (uint32_t*)p; p += al(b_words);
    h->S.orders = (uint32_t*)p; p += al(b_orders);
    h->S.scode = (uint16_t*)p; p += al(b_scode);
    h->S.snext = (uint8_t*)p; p += al(b_snext);
    h->S.scstep = (uint16_t*)p; p += al(b_scstep);
    h->S.nxt = (uint32_t*)p; p += al(b_nxt);
    h->S.mt = (uint32_t*)p;
    h->S.n = num_envs;
    e = hipMemsetAsync(h->base, 0, h->bytes, h->stream);
    if (e != hipSuccess) return bail("init", e);
    e = hipEventCreate(&h->ev0);
    if (e != hipSuccess) { h->ev0 = nullptr; return bail("hipEventCreate", e); }
    e = hipEventCreate(&h->ev1);
    if (e != hipSuccess) { h->ev1 = nullptr; return bail("hipEventCreate", e); }
    e = hipMalloc(&h->lut_dev, sizeof(double) * RLUT_SIZE);
    if (e != hipSuccess) { h->lut_dev = nullptr; return bail("hipMalloc(reward table)", e); }
    h->ntiles = (num_envs + 63) / 64;
    e = hipMalloc(&h->tiles, tile_words(h->ntiles) * 4);
    if (e != hipSuccess) { h->tiles = nullptr; return bail("hipMalloc(tile hand-off)", e); }
    e = hipMemsetAsync(h->tiles, 0, tile_words(h->ntiles) * 4, h->stream);
    if (e != hipSuccess) return bail("init", e);
    {
        // the aux words: fault 0, hand-off bound ~0.1 s of sleeps (far beyond any legitimate wait)
        const uint32_t aux[AUX_WORDS] = {0u, 1u << 22, 0u, 0u};
        e = hipMemcpyAsync(h->S.words + (size_t)NWORDS * n, aux, sizeof(aux), hipMemcpyHostToDevice, h->stream);
        if (e != hipSuccess) return bail("aux words", e);
        e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) return bail("aux words", e);
    }
    h->dcfg.lut = h->lut_dev;
    {
        fjsp_reward_weights w;
        fjsp_default_reward_weights(&w);
        build_reward_lut(reinterpret_cast<const double*>(&w), c.step_size, h->lut_host);
        e = hipMemcpy(h->lut_dev, h->lut_host, sizeof(double) * RLUT_SIZE, hipMemcpyHostToDevice);
        if (e != hipSuccess) return bail("reward table", e);
    }
    // default streams: env e behaves like a process that called np.random.seed(e)
    // (fjsp_set_option "env_id_base" re-keys them by global id)
    hipLaunchKernelGGL(k_seed, dim3((h->n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, h->stream, h->S,
                       (const uint32_t*)nullptr, 0u);
    e = hipGetLastError();
    if (e != hipSuccess) return bail("k_seed", e);
    *out = h;
    return 0;
}

int fjsp_destroy(fjsp_handle* h) {
    if (!h) return 0;
    DeviceGuard g(h->device);
    (void)server_stop(h);
    if (h->srv_ev) (void)hipEventDestroy(h->srv_ev);
    if (h->srv_stream) (void)hipStreamDestroy(h->srv_stream);
    if (h->srv) (void)hipHostFree(h->srv);
    if (h->srv_relay) (void)hipFree(h->srv_relay);
    (void)hipStreamSynchronize(h->stream);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    if (h->lut_dev) (void)hipFree(h->lut_dev);
    if (h->tiles) (void)hipFree(h->tiles);
    if (h->base) (void)hipFree(h->base);
    delete h;
    return 0;
}

extern "C" int fjsp_internal_policy_option(const char* name, int64_t value);   // fjsp_policy.hip (not in fjsp.h)

int fjsp_set_option(fjsp_handle* h, const char* name, int64_t value) {
    if (!name) return fail("null argument");
    // library-wide options (h may be null): the A2C policy launches' variants
    if (!strncmp(name, "policy_", 7) || !strcmp(name, "wgrad_waves")) return fjsp_internal_policy_option(name, value);
    if (!h) return fail("null handle (only the policy_* and wgrad_waves options are library-wide)");
    SERVER_QUIESCE(h);
    if (!strcmp(name, "fused_lds")) { h->use_lds = value < 0 ? -1 : value != 0; return 0; }
    if (!strcmp(name, "staged_stores")) { h->use_staged = value != 0; return 0; }
    if (!strcmp(name, "pipeline")) { h->use_pipe = value != 0; return 0; }
    if (!strcmp(name, "predraw")) { h->use_pg = value != 0; return 0; }
    if (!strcmp(name, "agents")) { h->use_ag = value != 0; return 0; }
    if (!strcmp(name, "step_envs")) {
        if (value != 0 && value != 16 && value != 32 && value != 64) return fail("step_envs must be 0, 16, 32 or 64");
        h->step_epw = (int)value;
        return 0;
    }
    if (!strcmp(name, "ag_envs")) {
        if (value != 0 && value != 16 && value != 32 && value != 64) return fail("ag_envs must be 0, 16, 32 or 64");
        h->ag_epw = (int)value;
        return 0;
    }
    if (!strcmp(name, "timing")) { h->timing = value != 0; if (!h->timing) h->timed = 0; return 0; }
    if (!strcmp(name, "spin_cap")) {
        if (value < 256 || value > 0x7FFFFFFFll) return fail("spin_cap must be in 256..2^31-1");
        DeviceGuard g(h->device);
        const uint32_t v = (uint32_t)value;
        HIPCHK(hipStreamSynchronize(h->stream));
        HIPCHK(hipMemcpy(h->S.words + (size_t)NWORDS * h->n + AUX_SPIN_CAP, &v, 4, hipMemcpyHostToDevice));
        return 0;
    }
    if (!strcmp(name, "test_stall")) {   // tests only: see stall_for_test (fjsp_stepdev.h)
        if (value < 0 || value > (1 << 20)) return fail("test_stall must be in 0..2^20");
        DeviceGuard g(h->device);
        const uint32_t v = (uint32_t)value;
        HIPCHK(hipStreamSynchronize(h->stream));
        HIPCHK(hipMemcpy(h->S.words + (size_t)NWORDS * h->n + AUX_TEST_STALL, &v, 4, hipMemcpyHostToDevice));
        h->test_stall = value != 0;
        return 0;
    }
    if (!strcmp(name, "env_id_base")) {
        // the handle is shard [value, value + n) of a larger job: env e's default stream becomes
        // np.random.seed(value + e), as for env value + e of one big handle (stream-ordered)
        if (value < 0 || value > 0xFFFFFFFFll) return fail("env_id_base must be in 0..2^32-1");
        DeviceGuard g(h->device);
        hipLaunchKernelGGL(k_seed, dim3((h->n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, h->stream, h->S,
                           (const uint32_t*)nullptr, (uint32_t)value);
        HIPCHK(hipGetLastError());
        h->env_id_base = (uint32_t)value;
        return 0;
    }
    return fail("unknown option");
}

int fjsp_set_stream(fjsp_handle* h, void* s) {
    if (!h) return fail("null handle");
    h->stream = (hipStream_t)s;
    return 0;
}
int fjsp_num_envs(const fjsp_handle* h) { return h ? h->n : -1; }
int64_t fjsp_state_bytes(const fjsp_handle* h) { return h ? (int64_t)(h->bytes / h->n) : -1; }

static const fjsp_out kNoOut = {};

int fjsp_reset(fjsp_handle* h, const uint32_t* seeds, const uint8_t* env_mask, int32_t num_orders, const fjsp_out* out) {
    if (!h) return fail("null handle");
    SERVER_QUIESCE(h);
    if (num_orders < 0 || num_orders > MAX_ORDERS) return fail("num_orders must be in 0..64");
    DeviceGuard g(h->device);
    dim3 grid((h->n + BLOCK - 1) / BLOCK);
    hipLaunchKernelGGL(k_reset, grid, dim3(BLOCK), 0, h->stream, h->S, h->dcfg, seeds, env_mask, num_orders,
                       out ? *out : kNoOut);
    HIPCHK(hipGetLastError());
    h->has_reset = 1;
    return 0;
}

int fjsp_step(fjsp_handle* h, const uint8_t* actions, const uint8_t* agent_order, int32_t autoreset, const fjsp_out* out) {
    if (!h) return fail("null handle");
    SERVER_QUIESCE(h);
    if (!actions) return fail("null actions");
    if (!h->has_reset) return fail("fjsp_step before fjsp_reset");
    bool canon = true;
    uint64_t packed = 0;
    if (agent_order) {
        unsigned seen = 0;
        for (int i = 0; i < NA; i++) {
            if (agent_order[i] >= NA || (seen >> agent_order[i]) & 1u) return fail("agent_order must be a permutation of 0..7");
            seen |= 1u << agent_order[i];
            canon = canon && agent_order[i] == i;
            packed |= (uint64_t)agent_order[i] << (8 * i);
        }
    }
    DeviceGuard g(h->device);
    // 64 envs per workgroup unless the option says otherwise: at 4 096 envs 16- / 32-env
    // workgroups (all 256 CUs busy) measured slower, 8.58 / 8.32 against 7.61 us per launch
    // (profiles/r06/kstep/ab_step_envs_4096.json): the step is not bound by its lanes' branch union
    const int epw = h->step_epw ? h->step_epw : 64;
    const dim3 grid((h->n + epw - 1) / epw);
    const fjsp_out o = out ? *out : kNoOut;
    if (h->timing) HIPCHK(hipEventRecord(h->ev0, h->stream));
#define FJSP_LAUNCH_STEP(CN)                                                                                      \
    do {                                                                                                           \
        if (epw == 16)                                                                                             \
            hipLaunchKernelGGL((k_step<CN, 16>), grid, dim3(BLOCK), 0, h->stream, h->S, h->dcfg, actions, packed, \
                               autoreset, o);                                                                      \
        else if (epw == 32)                                                                                        \
            hipLaunchKernelGGL((k_step<CN, 32>), grid, dim3(BLOCK), 0, h->stream, h->S, h->dcfg, actions, packed, \
                               autoreset, o);                                                                      \
        else                                                                                                       \
            hipLaunchKernelGGL((k_step<CN, 64>), grid, dim3(BLOCK), 0, h->stream, h->S, h->dcfg, actions, packed, \
                               autoreset, o);                                                                      \
    } while (0)
    if (canon) {
        h->last_kernel = "k_step<canon>";
        FJSP_LAUNCH_STEP(true);
    } else {
        h->last_kernel = "k_step<ordered>";
        FJSP_LAUNCH_STEP(false);
    }
#undef FJSP_LAUNCH_STEP
    HIPCHK(hipGetLastError());
    if (h->timing) {
        HIPCHK(hipEventRecord(h->ev1, h->stream));
        h->timed = 1;
    }
    return 0;
}

// ---- the step server (include/fjsp.h fjsp_server_*)
// The resident kernel leaves after 5 ms without a request (the host relaunches it after 2 ms idle,
// ~30 us): a process-wide hipDeviceSynchronize (torch.cuda.synchronize) issued between steps waits
// for the resident kernel, i.e. at most that long.
static constexpr uint64_t SRV_IDLE_TICKS = 500000ull;     // 5 ms of the 100 MHz clock
static constexpr int SRV_RESTART_US = 2000;
static constexpr int SRV_WAIT_MS = 2000;                  // a request not done by then is an error

static int server_launch(fjsp_handle* h) {
    DeviceGuard g(h->device);
    HIPCHK(hipEventRecord(h->srv_ev, h->stream));            // the state as h->stream leaves it
    HIPCHK(hipStreamWaitEvent(h->srv_stream, h->srv_ev, 0));
    h->srv_epoch++;
    const uint32_t seq = __atomic_load_n(&h->srv->seq, __ATOMIC_ACQUIRE);
    for (int w = 0; w < h->srv_nwg; w++) {
        __atomic_store_n(&h->srv->done[w], seq, __ATOMIC_RELAXED);
        __atomic_store_n(&h->srv->exited[w], 0u, __ATOMIC_RELAXED);
    }
    __atomic_store_n(&h->srv->stop, 0u, __ATOMIC_RELEASE);
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)h->srv_relay, (int)seq, 1, h->srv_stream));
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)(h->srv_relay + 1), 0, 1, h->srv_stream));
    hipLaunchKernelGGL(k_step_server, dim3(h->srv_nwg), dim3(BLOCK), 0, h->srv_stream, h->S, h->dcfg, h->srv,
                       h->srv_relay, h->srv_actions, h->srv_autoreset, h->srv_out, seq, h->srv_epoch, SRV_IDLE_TICKS);
    HIPCHK(hipGetLastError());
    h->srv_running = 1;
    h->srv_last = std::chrono::steady_clock::now();
    h->last_kernel = "k_step_server";
    return 0;
}

int fjsp_server_start(fjsp_handle* h, const uint8_t* actions, int32_t autoreset, const fjsp_out* out) {
    if (!h) return fail("null handle");
    if (!actions && h->n != 1) return fail("fjsp_server_start: null actions (inline mode) needs a one-env handle");
    if (!h->has_reset) return fail("fjsp_server_start before fjsp_reset");
    if (h->n > SRV_MAX_WG * BLOCK) return fail("fjsp_server_start: at most 16384 envs per handle");
    SERVER_QUIESCE(h);
    DeviceGuard g(h->device);
    if (!h->srv) {
        void* p = nullptr;
        HIPCHK(hipHostMalloc(&p, sizeof(ServerCtl), hipHostMallocCoherent | hipHostMallocMapped));
        memset(p, 0, sizeof(ServerCtl));
        h->srv = (ServerCtl*)p;
        HIPCHK(hipMalloc(&h->srv_relay, 64));
        HIPCHK(hipStreamCreateWithFlags(&h->srv_stream, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&h->srv_ev, hipEventDisableTiming));
    }
    h->srv_actions = actions;
    h->srv_out = out ? *out : kNoOut;
    h->srv_autoreset = autoreset != 0;
    h->srv_nwg = (h->n + BLOCK - 1) / BLOCK;
    h->srv_configured = 1;
    return server_launch(h);
}

static int server_request(fjsp_handle* h, const uint8_t* inline_actions);

int fjsp_server_step(fjsp_handle* h) {
    if (!h) return fail("null handle");
    if (!h->srv_configured) return fail("fjsp_server_step before fjsp_server_start");
    if (!h->srv_actions) return fail("fjsp_server_step: the server runs in inline mode (fjsp_server_step_actions)");
    return server_request(h, nullptr);
}

int fjsp_server_step_actions(fjsp_handle* h, const uint8_t* actions) {
    if (!h) return fail("null handle");
    if (!actions) return fail("null actions");
    if (!h->srv_configured) return fail("fjsp_server_step_actions before fjsp_server_start");
    if (h->srv_actions) return fail("fjsp_server_step_actions: the server was started with an actions buffer");
    return server_request(h, actions);
}

static int server_request(fjsp_handle* h, const uint8_t* inline_actions) {
    const auto now = std::chrono::steady_clock::now();
    if (h->srv_running &&
        std::chrono::duration_cast<std::chrono::microseconds>(now - h->srv_last).count() > SRV_RESTART_US) {
        if (int rc = server_stop(h)) return rc;   // idle: relaunch before the kernel's own timeout
    }
    if (!h->srv_running) {
        if (int rc = server_launch(h)) return rc;
    }
    const uint32_t seq = __atomic_load_n(&h->srv->seq, __ATOMIC_RELAXED) + 1u;
    if (inline_actions) {   // the inbox before seq (the kernel accepts a request by the inbox tags)
        const uint32_t tag = (seq & 0xFFFFu) << 16;
        for (int k = 0; k < 4; k++)
            __atomic_store_n(&h->srv->inbox[k], tag | inline_actions[2 * k] | ((uint32_t)inline_actions[2 * k + 1] << 8),
                             __ATOMIC_RELEASE);
    }
    __atomic_store_n(&h->srv->seq, seq, __ATOMIC_RELEASE);   // after the caller's action bytes
    const auto t0 = std::chrono::steady_clock::now();
    for (int w = 0; w < h->srv_nwg; w++) {
        for (uint32_t it = 0; __atomic_load_n(&h->srv->done[w], __ATOMIC_ACQUIRE) != seq; it++) {
            if ((it & 1023u) == 1023u) {
                const bool left = __atomic_load_n(&h->srv->exited[w], __ATOMIC_ACQUIRE) == h->srv_epoch;
                const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                                    std::chrono::steady_clock::now() - t0).count();
                if (left || ms > SRV_WAIT_MS) {
                    (void)server_stop(h);
                    return fail(left ? "step server left before the request" : "step server request timed out");
                }
            }
        }
    }
    h->srv_last = std::chrono::steady_clock::now();
    return 0;
}

int fjsp_server_stop(fjsp_handle* h) {
    if (!h) return fail("null handle");
    return server_stop(h);
}

int fjsp_a2c_policy_step(fjsp_handle* h, const float* feats, const int8_t* masks, const float* actor_w,
                         const float* critic_w, const uint64_t* seed, uint32_t env_gid0, uint32_t step,
                         int32_t deterministic, uint8_t* actions, float* values, int32_t autoreset, const fjsp_out* out,
                         int32_t env_begin, int32_t env_count, void* stream) {
    if (!h) return fail("null handle");
    SERVER_QUIESCE(h);
    if (!h->has_reset) return fail("fjsp_a2c_policy_step before fjsp_reset");
    if (!feats || !masks || !actor_w || !seed || !actions || (values && !critic_w))
        return fail("fjsp_a2c_policy_step: null buffer");
    if (env_begin < 0 || env_count <= 0 || env_begin % 64 || env_begin + env_count > h->n ||
        (env_count % 64 && env_begin + env_count != h->n))
        return fail("fjsp_a2c_policy_step: envs [env_begin, env_begin + env_count) must be whole 64-env tiles of the handle");
    DeviceGuard g(h->device);
    hipStream_t st = stream ? (hipStream_t)stream : h->stream;
    // the handle's one event pair times launches on its own stream only: a collect that runs its
    // env groups on several streams would otherwise report whichever launch recorded last
    const bool timed = h->timing && st == h->stream;
    if (timed) HIPCHK(hipEventRecord(h->ev0, st));
    h->last_kernel = "k_policy_step";
    const size_t cnt_words = ((size_t)h->ntiles + 63) & ~(size_t)63;
    const int rc = fjsp_internal_policy_step(feats, masks, h->n, actor_w, critic_w, seed, env_gid0, step, deterministic,
                                             actions, values, h->S, h->dcfg, out ? *out : kNoOut, h->tiles,
                                             h->tiles + cnt_words, autoreset, env_begin, env_count, st);
    if (rc) return rc;
    if (timed) {
        HIPCHK(hipEventRecord(h->ev1, st));
        h->timed = 1;
    }
    return 0;
}

int fjsp_step_many(fjsp_handle* h, int32_t K, uint64_t action_seed, uint32_t env_gid0, uint32_t step0,
                   int32_t action_mode, int32_t autoreset, const fjsp_out* traj) {
    if (!h) return fail("null handle");
    SERVER_QUIESCE(h);
    if (K < 0) return fail("K must be >= 0");
    if (action_mode != FJSP_ACTIONS_UNMASKED && action_mode != FJSP_ACTIONS_MASKED && action_mode != FJSP_ACTIONS_HEURISTIC)
        return fail("bad action_mode");
    if (!h->has_reset) return fail("fjsp_step_many before fjsp_reset");
    if (K == 0) return 0;
    const fjsp_out o = traj ? *traj : kNoOut;
    // outputs are addressed with 32-bit byte offsets: the largest per-step block is the a2c
    // features (38 x 4 B per env) or the rewards (8 x 8 B)
    const uint64_t row_bytes = o.feats ? 4ull * NFEAT : 64ull;
    if ((uint64_t)K * (uint64_t)h->n * row_bytes >= (1ull << 32)) return fail("K * num_envs too large for one launch");
    DeviceGuard g(h->device);
    dim3 grid((h->n + BLOCK - 1) / BLOCK);
    if (h->timing) HIPCHK(hipEventRecord(h->ev0, h->stream));
    const bool full = o.results || o.orders_completed || o.packaged || o.sim_time || o.next_i32 || o.next_i8 ||
                      o.next_f32 || o.next_masks || o.feats;
    auto launch = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, dim3(BLOCK), 0, h->stream, h->S, h->dcfg, K, action_seed, env_gid0, step0,
                           action_mode, autoreset, o);
    };
    // staged stores need whole 64-env blocks and 16-byte aligned output rows
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15u) == 0; };
    const bool staged = h->use_staged && !full && h->n % BLOCK == 0 && al16(o.obs_i32) && al16(o.obs_i8) &&
                        al16(o.obs_f32) && al16(o.masks) && al16(o.rewards) && al16(o.term) && al16(o.trunc) &&
                        al16(o.status);
    // LDS tables (97.5 KB per 64-env workgroup) pay while every workgroup has a CU of its own
    const bool lds = h->use_lds < 0 ? h->n <= 256 * BLOCK : h->use_lds != 0;
    const bool two_emit = h->n <= 256 * BLOCK;
    // the pre-draw wave pays while the CUs have a free SIMD (and only with auto-reset)
    const bool pg = h->use_pg && lds && two_emit && autoreset;
    // the agent-group pipeline: state-independent (uniform-random) actions, LDS tables, pre-draw;
    // also for 16 384 < N <= 32 768, where its 64-env workgroups run in two rounds and still beat
    // k_step_pipe<1emit> (24 576 envs 3.17 against 3.75, 32 768 3.20-3.59 against 3.87 ms per
    // 1 024-step launch; 49 152: 4.85 against 4.37-4.72; profiles/r04/ag_two_rounds_ab.json)
    const bool ag_wide = h->n > 256 * BLOCK && h->n <= 512 * BLOCK && h->use_lds != 0 && h->use_pg && autoreset;
    const bool ag = h->use_ag && h->use_pipe && !full && !staged && (pg || ag_wide) &&
                    action_mode == FJSP_ACTIONS_UNMASKED;
    h->last_kernel = ag ? "k_step_ag<lds,predraw>"
                   : (h->use_pipe && !full && !staged)
                         ? (lds ? (two_emit ? (pg ? "k_step_pipe<lds,2emit,predraw>" : "k_step_pipe<lds,2emit>")
                                            : "k_step_pipe<lds,1emit>")
                                : (two_emit ? "k_step_pipe<2emit>" : "k_step_pipe<1emit>"))
                   : full ? (lds ? "k_step_many<lds,full>" : "k_step_many<full>")
                   : staged ? (lds ? "k_step_many<lds,staged>" : "k_step_many<staged>")
                   : (lds ? "k_step_many<lds>" : "k_step_many");
    if (ag) {
        // envs per workgroup: auto = the fewest that still give every workgroup a CU of its own
        // for long launches (1.30 -> 1.22 us per step at 4 096 envs); 64 for launches of fewer
        // than 64 steps, whose time is mostly the per-workgroup fixed cost (K = 20: 36.6 against
        // 39.9 us in rocprof)
        int epw = h->ag_epw;
        if (epw == 0) epw = K < 64 ? 64 : h->n <= 256 * 16 ? 16 : h->n <= 256 * 32 ? 32 : 64;
        const dim3 agrid((h->n + epw - 1) / epw);
        auto launch_ag = [&](auto kern) {
            hipLaunchKernelGGL(kern, agrid, dim3(AG_WAVES * BLOCK), 0, h->stream, h->S, h->dcfg, K, action_seed,
                               env_gid0, step0, autoreset, o);
        };
        if (h->test_stall) {
            if (epw == 16) launch_ag(k_step_ag<16, true>);
            else if (epw == 32) launch_ag(k_step_ag<32, true>);
            else launch_ag(k_step_ag<64, true>);
        } else if (epw == 16) launch_ag(k_step_ag<16>);
        else if (epw == 32) launch_ag(k_step_ag<32>);
        else launch_ag(k_step_ag<64>);
    } else if (h->use_pipe && !full && !staged) {
        // a second emit wave pays while the CUs are not full (N <= 16384 at 64 envs per CU)
        const bool two = two_emit;
        auto launch_pipe = [&](auto kern, int waves) {
            hipLaunchKernelGGL(kern, grid, dim3(waves * BLOCK), 0, h->stream, h->S, h->dcfg, K, action_seed, env_gid0,
                               step0, action_mode, autoreset, o);
        };
        if (lds && two && pg && h->test_stall) launch_pipe(k_step_pipe<true, 2, true, true>, 4);
        else if (lds && two && pg) launch_pipe(k_step_pipe<true, 2, true>, 4);
        else if (lds) two ? launch_pipe(k_step_pipe<true, 2>, 3) : launch_pipe(k_step_pipe<true, 1>, 2);
        else two ? launch_pipe(k_step_pipe<false, 2>, 3) : launch_pipe(k_step_pipe<false, 1>, 2);
    } else if (lds) {
        if (full) launch(k_step_many<true, true>);
        else if (staged) launch(k_step_many<true, false, true>);
        else launch(k_step_many<true, false>);
    } else {
        if (full) launch(k_step_many<false, true>);
        else if (staged) launch(k_step_many<false, false, true>);
        else launch(k_step_many<false, false>);
    }
    HIPCHK(hipGetLastError());
    if (h->timing) {
        HIPCHK(hipEventRecord(h->ev1, h->stream));
        h->timed = 1;
    }
    return 0;
}

int fjsp_gae(const double* rewards, const float* values, const uint8_t* done, const double* boot, int32_t T, int32_t N,
             int32_t M, double gamma, double lamb, double* ret, double* adv, void* stream) {
    if (T <= 0 || N <= 0 || M <= 0 || M % N) return fail("bad GAE shape (T > 0, N > 0, M multiple of N)");
    if (!rewards || !values || !done || !boot || !ret || !adv) return fail("null GAE buffer");
    hipLaunchKernelGGL((k_gae<float, false>), dim3((M + 63) / 64), dim3(64), 0, (hipStream_t)stream, rewards, values,
                       done, boot, T, N, M, gamma, lamb, ret, adv);
    HIPCHK(hipGetLastError());
    return 0;
}

int fjsp_gae_f64(const double* rewards, const double* values, const uint8_t* done, const double* boot, int32_t T,
                 int32_t N, int32_t M, double gamma, double lamb, double* ret, double* adv, void* stream) {
    if (T <= 0 || N <= 0 || M <= 0 || M % N) return fail("bad GAE shape (T > 0, N > 0, M multiple of N)");
    if (!rewards || !values || !done || !boot || !ret || !adv) return fail("null GAE buffer");
    hipLaunchKernelGGL((k_gae<double, false>), dim3((M + 63) / 64), dim3(64), 0, (hipStream_t)stream, rewards, values,
                       done, boot, T, N, M, gamma, lamb, ret, adv);
    HIPCHK(hipGetLastError());
    return 0;
}

// The batch statistics the grouped update reads from the GAE outputs (f64 [T][8][N]), in one
// pass: per sample (t, e) the f64 sums over the 8 agents of the f32-rounded return and of its
// square (the critic loss's coefficients, a2c_vec.critic_coef; calc_critic_loss uses
// FloatTensor(returns), a2c.py:713-722), and per agent the f64 sums of the f32-rounded advantage
// and of its square (calc_actor_loss's normalisation, a2c.py:724-731), as per-workgroup partials
// part[t][block][8][2] summed by the caller in a fixed order.  ret / adv may be null (that half
// skipped).
__global__ void __launch_bounds__(256) k_slab_stats(const double* __restrict__ ret, const double* __restrict__ adv,
                                                    int T, int N, double* __restrict__ rsum, double* __restrict__ rsq,
                                                    double* __restrict__ part) {
    const int t = blockIdx.y;
    const int e = blockIdx.x * 256 + threadIdx.x;
    const bool in = e < N;
    if (ret) {
        double s = 0.0, q = 0.0;
        if (in) {
#pragma unroll
            for (int a = 0; a < NA; a++) {
                const double r = (double)(float)ret[((size_t)t * NA + a) * N + e];
                s += r;
                q += r * r;
            }
            rsum[(size_t)t * N + e] = s;
            rsq[(size_t)t * N + e] = q;
        }
    }
    if (adv) {
        __shared__ double s_p[4][NA][2];
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
        for (int a = 0; a < NA; a++) {
            double x = in ? (double)(float)adv[((size_t)t * NA + a) * N + e] : 0.0;
            double x2 = x * x;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                x += __shfl_xor(x, o);
                x2 += __shfl_xor(x2, o);
            }
            if (lane == 0) { s_p[w][a][0] = x; s_p[w][a][1] = x2; }
        }
        __syncthreads();
        if (threadIdx.x < NA * 2) {
            const int a = threadIdx.x >> 1, c = threadIdx.x & 1;
            part[(((size_t)t * gridDim.x + blockIdx.x) * NA + a) * 2 + c] = s_p[0][a][c] + s_p[1][a][c] + s_p[2][a][c] + s_p[3][a][c];
        }
    }
}

int fjsp_a2c_slab_stats(const double* ret, const double* adv, int32_t T, int32_t N, double* rsum, double* rsq,
                        double* part, void* stream) {
    if (T <= 0 || N <= 0) return fail("fjsp_a2c_slab_stats: T and N must be > 0");
    if ((!ret && !adv) || (ret && (!rsum || !rsq)) || (adv && !part)) return fail("fjsp_a2c_slab_stats: null buffer");
    hipLaunchKernelGGL(k_slab_stats, dim3((unsigned)((N + 255) / 256), (unsigned)T), dim3(256), 0, (hipStream_t)stream, ret,
                       adv, T, N, rsum, rsq, part);
    HIPCHK(hipGetLastError());
    return 0;
}

int fjsp_gae_shared(const double* rewards, const float* values, const uint8_t* done, int32_t T, int32_t N,
                    int32_t agents, double gamma, double lamb, double* ret, double* adv, void* stream) {
    if (T <= 0 || N <= 0 || agents <= 0 || (int64_t)agents * N > INT32_MAX)
        return fail("bad GAE shape (T > 0, N > 0, agents > 0)");
    if (!rewards || !values || !done || !ret || !adv) return fail("null GAE buffer");
    const int M = agents * N;
    // the loader-wave scan: 64-column workgroups never straddle two agents, and its 16-byte LDS
    // DMAs need 16-byte aligned rows (a sub-view at an odd offset takes the register scan)
    const bool aligned = (((uintptr_t)rewards | (uintptr_t)values | (uintptr_t)done) & 15u) == 0;
    if (N % 64 == 0 && aligned)
        hipLaunchKernelGGL(k_gae_lw, dim3(M / 64), dim3(128), 0, (hipStream_t)stream, rewards, values, done, T, N, M,
                           gamma, lamb, ret, adv);
    else
        hipLaunchKernelGGL((k_gae<float, true>), dim3((M + 63) / 64), dim3(64), 0, (hipStream_t)stream, rewards,
                           values, done, nullptr, T, N, M, gamma, lamb, ret, adv);
    HIPCHK(hipGetLastError());
    return 0;
}

#ifdef FJSP_STAMPS
// diagnostic build only: accumulated per-phase wave cycles of k_step_many (and reset them)
extern "C" int fjsp_debug_stamps(unsigned long long* out) {
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 8));
    unsigned long long z[8] = {0};
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)));
    return 0;
}
extern "C" int fjsp_debug_agstamps(unsigned long long* out) {   // out[16]: k_step_ag per wave busy / wait, epochs
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_agstamps), sizeof(unsigned long long) * 64));
    unsigned long long z[64] = {0};
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_agstamps), z, sizeof(z)));
    return 0;
}
extern "C" int fjsp_debug_pgstamps(unsigned long long* out) {   // out[8]: pre-draw [4], emit [4]
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pgstamps), sizeof(unsigned long long) * 4));
    HIPCHK(hipMemcpyFromSymbol(out + 4, HIP_SYMBOL(g_emitstamps), sizeof(unsigned long long) * 4));
    unsigned long long z[4] = {0};
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_pgstamps), z, sizeof(z)));
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_emitstamps), z, sizeof(z)));
    return 0;
}
#endif

int fjsp_pack_a2c(fjsp_handle* h, float* feats, int8_t* masks) {
    if (!h) return fail("null handle");
    SERVER_QUIESCE(h);
    if (!h->has_reset) return fail("fjsp_pack_a2c before fjsp_reset");
    if (!feats && !masks) return 0;
    DeviceGuard g(h->device);
    Cfg C = h->dcfg;
    C.lut = h->lut_dev;
    k_pack<<<(h->n + BLOCK - 1) / BLOCK, BLOCK, 0, h->stream>>>(h->S, C, feats, masks);
    HIPCHK(hipGetLastError());
    return 0;
}

int fjsp_a2c_layout(int32_t* out) {
    if (!out) return fail("null argument");
    for (int f = 0; f < NI32; f++) out[FEAT_OF_I32[f]] = f;
    for (int f = 0; f < NI8; f++) out[FEAT_OF_I8[f]] = NI32 + f;
    for (int f = 0; f < NF32; f++) out[FEAT_OF_F32[f]] = NI32 + NI8 + f;
    return 0;
}

int64_t fjsp_snapshot_bytes(const fjsp_handle* h) { return h ? (int64_t)h->bytes : -1; }

int fjsp_snapshot(fjsp_handle* h, void* dst) {
    if (!h || !dst) return fail("null argument");
    SERVER_QUIESCE(h);
    if (!h->has_reset) return fail("fjsp_snapshot before fjsp_reset");
    DeviceGuard g(h->device);
    HIPCHK(hipMemcpyAsync(dst, h->base, h->bytes, hipMemcpyDefault, h->stream));
    return 0;
}

int fjsp_restore(fjsp_handle* h, const void* src) {
    if (!h || !src) return fail("null argument");
    SERVER_QUIESCE(h);
    DeviceGuard g(h->device);
    // everything but the aux words (fault word, spin_cap, test options): those stay the handle's
    const size_t state = (size_t)NWORDS * h->n * 4, rest = (size_t)((char*)h->S.orders - (char*)h->base);
    HIPCHK(hipMemcpyAsync(h->base, src, state, hipMemcpyDefault, h->stream));
    HIPCHK(hipMemcpyAsync((char*)h->base + rest, (const char*)src + rest, h->bytes - rest, hipMemcpyDefault, h->stream));
    h->has_reset = 1;
    return 0;
}

const char* fjsp_last_kernel(const fjsp_handle* h) {
    return (h && h->last_kernel) ? h->last_kernel : "";
}

int fjsp_faults(fjsp_handle* h, uint32_t* out, int32_t clear) {
    if (!h || !out) return fail("null argument");
    SERVER_QUIESCE(h);
    DeviceGuard g(h->device);
    HIPCHK(hipStreamSynchronize(h->stream));
    uint32_t* w = h->S.words + (size_t)NWORDS * h->n + AUX_FAULT;
    HIPCHK(hipMemcpy(out, w, sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (clear) HIPCHK(hipMemset(w, 0, sizeof(uint32_t)));
    return 0;
}

int fjsp_sync(fjsp_handle* h) {
    if (!h) return fail("null handle");
    SERVER_QUIESCE(h);
    DeviceGuard g(h->device);
    HIPCHK(hipStreamSynchronize(h->stream));
    return 0;
}

int fjsp_last_kernel_ms(fjsp_handle* h, float* ms) {
    if (!h || !ms) return fail("null argument");
    if (!h->timed) return fail("no timed launch yet");
    DeviceGuard g(h->device);
    HIPCHK(hipEventSynchronize(h->ev1));
    HIPCHK(hipEventElapsedTime(ms, h->ev0, h->ev1));
    return 0;
}

// MT19937 state exchange in numpy's (key[624], pos) convention (np.random.get_state()[1:3]).
int fjsp_mt_get(fjsp_handle* h, int32_t env, uint32_t* key, int32_t* pos) {
    if (!h || !key || !pos) return fail("null argument");
    SERVER_QUIESCE(h);
    if (env < 0 || env >= h->n) return fail("env index out of range");
    DeviceGuard g(h->device);
    HIPCHK(hipStreamSynchronize(h->stream));
    uint32_t st = 0;
    HIPCHK(hipMemcpy(&st, h->S.words + (size_t)3 * h->n + env, 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(key, h->S.mt + ((size_t)(st >> 31) * h->n + env) * MT_N, 4 * MT_N, hipMemcpyDeviceToHost));
    int mti = (int)(st & 0x3FF), gg = (int)((st >> 16) & 0x3FF);
    if (gg == 0) { *pos = MT_N; return 0; }
    for (int i = gg; i < MT_N; i++) {   // finish the in-place twist of the current block
        const int i1 = (i + 1 == MT_N) ? 0 : i + 1;
        const int im = (i + 397 >= MT_N) ? i + 397 - MT_N : i + 397;
        const uint32_t y = (key[i] & 0x80000000u) | (key[i1] & 0x7fffffffu);
        key[i] = key[im] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    *pos = mti;
    return 0;
}

int fjsp_mt_set(fjsp_handle* h, int32_t env, const uint32_t* key, int32_t pos) {
    if (!h || !key) return fail("null argument");
    SERVER_QUIESCE(h);
    if (env < 0 || env >= h->n) return fail("env index out of range");
    if (pos < 0 || pos > MT_N) return fail("pos must be in 0..624");
    DeviceGuard g(h->device);
    HIPCHK(hipStreamSynchronize(h->stream));
    const uint32_t st = pos >= MT_N ? 0u : ((uint32_t)pos | ((uint32_t)MT_N << 16));
    HIPCHK(hipMemcpy(h->S.mt + (size_t)env * MT_N, key, 4 * MT_N, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(h->S.words + (size_t)3 * h->n + env, &st, 4, hipMemcpyHostToDevice));
    const uint32_t zero = 0;   // a pre-drawn table belongs to the replaced stream
    HIPCHK(hipMemcpy(h->S.words + (size_t)PGW * h->n + env, &zero, 4, hipMemcpyHostToDevice));
    return 0;
}

int fjsp_read_env(fjsp_handle* h, int32_t env, fjsp_env_view* v) {
    if (!h || !v) return fail("null argument");
    SERVER_QUIESCE(h);
    if (env < 0 || env >= h->n) return fail("env index out of range");
    DeviceGuard g(h->device);
    HIPCHK(hipStreamSynchronize(h->stream));
    uint32_t w[NWORDS];
    uint32_t orders[MAX_ORDERS];
    // one strided copy per table (column `env` of the [rows][N] SoA arrays)
    HIPCHK(hipMemcpy2D(w, 4, h->S.words + env, (size_t)h->n * 4, 4, NWORDS, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy2D(orders, 4, h->S.orders + env, (size_t)h->n * 4, 4, MAX_ORDERS, hipMemcpyDeviceToHost));
    memset(v, 0, sizeof(*v));
    v->current_step = (int32_t)(w[0] & 0xFFFF);
    v->num_orders = (int32_t)((w[0] >> 16) & 0xFF);
    v->next_order = (int32_t)(w[0] >> 24);
    v->orders_completed = (int32_t)(w[1] & 0xFF);
    v->total_packaged = (int32_t)(w[1] >> 8);
    v->status = w[2];
    const int loc = (int)(w[6] & 7), carry = (int)((w[6] >> 3) & 0xFF), code = (int)((w[6] >> 11) & 0x1FFF);
    v->agv_row = loc_row(loc);
    v->agv_col = loc_col(loc);
    v->agv_carrying = carry != NIL;
    v->agv_tray_count = carry != NIL ? (code >> 10) & 7 : 0;
    for (int i = 0; i < v->num_orders && i < MAX_ORDERS; i++) {
        const uint32_t o = orders[i];
        const uint32_t n = (o >> 20) & 15, full = (1u << n) - 1u;
        const uint32_t pc = (uint32_t)__builtin_popcount(o & full), kc = (uint32_t)__builtin_popcount((o >> 9) & full);
        v->orders[i] = n | (((o >> 24) & 3) << 4) | (((o >> 26) & 3) << 6) | (pc << 8) | (kc << 12) | (((o >> 18) & 1) << 16);
    }
    return 0;
}

}  // extern "C"
