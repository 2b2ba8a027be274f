// fjsp_env.h — per-env FJSP state machine, written for one wavefront lane per env (gfx950).
//
// This is the MI355X-native restatement of the reference step (FJSPSimulation.py:144-242).
// Instead of a discrete-event heap it uses the closed form of the SimPy schedule the
// reference produces (proven against the oracle's general heap):
//   * all process bodies start at the step boundary T (URGENT Initialize);
//   * machine / packaging completions are multiples of step_size, so a completion due at T
//     fires in the run that follows the action phase at T, before that run's grants;
//   * AGV moves (distance <= 8 < step_size) complete inside the run -> position := target.
// Per-env state: a handful of registers (the Env struct, loaded/stored SoA [field][N]) plus
// three small tables addressed by (index * stride + lane): the order table (u32 per order),
// and a tray-slot arena (code u16, next u8, complete-step u16 per slot) that holds every
// FIFO of the reference (pickup ready trays, storage, machine queues / ready trays and the
// packaging product queues, whose entries are tray-sized runs of one order).
//
// Numerics: rewards in fp64 following RewardModel's Python operation order
// (utils/RewardModel.py:34-110); this file must be compiled with -ffp-contract=off.
#pragma once
#include <stdint.h>

#include "fjsp_stamps.h"

#ifndef FJSP_DEV
#define FJSP_DEV __device__ __forceinline__
#endif
#ifndef FJSP_HD   // small maps the host side of the library uses too
#ifdef __HIP__
#define FJSP_HD __host__ __device__ __forceinline__
#else
#define FJSP_HD FJSP_DEV
#endif
#endif

namespace fjsp {

FJSP_DEV float __uint_as_float_fjsp(uint32_t u) { float f; __builtin_memcpy(&f, &u, 4); return f; }
FJSP_DEV uint32_t __float_as_uint_fjsp(float f) { uint32_t u; __builtin_memcpy(&u, &f, 4); return u; }

constexpr int NA = 8;
constexpr int NI32 = 20, NI8 = 12, NF32 = 6, NMASK = 29;
constexpr int MAX_ORDERS = 64;
constexpr int MAX_SLOTS = 255;   // slot index 255 = NIL
constexpr int NIL = 255;

// lists in the slot arena
enum : int { L_PREADY = 0, L_STORAGE = 1, L_M0Q = 2, L_M0R = 3, L_M1Q = 4, L_M1R = 5, L_PKG = 6, NLIST = 10 };

// locations (enums/LocationType.py values) and coordinates (constants.py:5-11)
enum : int { LOC_PICKUP = 1, LOC_BIG = 2, LOC_SMALL = 3, LOC_STORAGE = 4, LOC_PACK = 5 };
// Small integer maps are 4-bit fields of a constant word (nib): a chain of `x == k ? ...`
// on one variable is turned into a switch by the compiler, i.e. branches on a wavefront.
constexpr uint32_t nibs(int a0, int a1, int a2, int a3, int a4, int a5, int a6 = 0, int a7 = 0) {
    return (uint32_t)a0 | ((uint32_t)a1 << 4) | ((uint32_t)a2 << 8) | ((uint32_t)a3 << 12) | ((uint32_t)a4 << 16) |
           ((uint32_t)a5 << 20) | ((uint32_t)a6 << 24) | ((uint32_t)a7 << 28);
}
FJSP_HD int nib(uint32_t table, int i) { return (int)((table >> (4 * i)) & 0xFu); }
constexpr uint32_t ROW_TAB = nibs(0, 0, 0, 2, 3, 3);   // location -> grid row
constexpr uint32_t COL_TAB = nibs(0, 0, 3, 3, 0, 5);   // location -> grid column
FJSP_HD int loc_row(int l) { return nib(ROW_TAB, l); }
FJSP_HD int loc_col(int l) { return nib(COL_TAB, l); }
// AGV move action a (1..5) -> location (AGVAgent.py:218-224)
constexpr uint32_t MOVE_TAB = nibs(0, LOC_PICKUP, LOC_SMALL, LOC_BIG, LOC_STORAGE, LOC_PACK);
FJSP_DEV int move_loc(int a) { return nib(MOVE_TAB, a & 7); }
FJSP_DEV int iabs(int x) { return x < 0 ? -x : x; }
FJSP_DEV int manhattan(int a, int b) {
    return iabs(loc_row(a) - loc_row(b)) + iabs(loc_col(a) - loc_col(b));
}

// order word: processed mask [0,9) | packaged mask [9,18) | complete bit 18 |
//             n [20,24) | type [24,26) | color [26,28)
FJSP_DEV int ow_n(uint32_t w) { return (w >> 20) & 15; }
FJSP_DEV int ow_type(uint32_t w) { return (w >> 24) & 3; }
FJSP_DEV int ow_color(uint32_t w) { return (w >> 26) & 3; }
FJSP_DEV uint32_t ow_make(int n, int type, int color) {
    return ((uint32_t)n << 20) | ((uint32_t)type << 24) | ((uint32_t)color << 26);
}
// tray code: order [0,6) | start [6,10) | count [10,13)
FJSP_DEV int tc_order(int c) { return c & 63; }
FJSP_DEV int tc_start(int c) { return (c >> 6) & 15; }
FJSP_DEV int tc_count(int c) { return (c >> 10) & 7; }
FJSP_DEV int tc_make(int o, int s, int n) { return o | (s << 6) | (n << 10); }
FJSP_DEV uint32_t tc_range(int c) { return ((1u << tc_count(c)) - 1u) << tc_start(c); }

// RewardModel weights (utils/RewardModel.py:12-32), in fjsp_reward_weights field order.
enum : int { W_ORDER = 0, W_THROUGHPUT, W_TIME, W_PICK_LOAD, W_PICK_TRAY, W_PICK_IDLE, W_AGV_DELIVERY, W_AGV_MOVE,
             W_AGV_PACKAGING, W_AGV_INVALID, W_M_COMPLETE, W_M_START, W_M_IDLE, W_P_COMPLETE, W_P_START, W_P_IDLE,
             NW };

// Reward lookup table (device memory): the local reward of every (agent kind, result bits,
// action == 0) combination, each summed from 0.0 in calculate_local_reward's order on the host,
// plus the global-reward weights.  Layout: [0,16) pickup, [16,48) AGV, [48,64) machine,
// [64,80) packaging, [80] ORDER, [81] THROUGHPUT, [82] TIME * step_size, [96,352) progress.
// [96, 352): (1.0 / n) * 100.0 for n < 256 (PackagingAgent START progress, in fp64).
constexpr int RPROG = 96, RPROG_N = 256;
constexpr int RLUT_SIZE = RPROG + RPROG_N;

struct Cfg {
    int step_size, max_steps, tray_cap, mask_tray_cap, storage_cap, pool0, pkg_cap;
    int ptk_small, ptk_big, ptk_pack;   // processing times in steps
    const double* lut;                  // RLUT_SIZE doubles
};

// Host side: fill the reward table from RewardModel weights (w in fjsp_reward_weights order).
inline void build_reward_lut(const double* w, int step_size, double* lut) {
    for (int i = 0; i < RLUT_SIZE; i++) lut[i] = 0.0;
    for (int idx = 0; idx < 16; idx++) {   // bit0 start/loaded, bit1 completed, bit2 idle flag, bit3 action == 0
        const bool b0 = idx & 1, b1 = idx & 2, idle = (idx & 4) && (idx & 8);
        double p = 0.0, m = 0.0, k = 0.0;
        if (b0) p += w[W_PICK_LOAD];
        if (b1) p += w[W_PICK_TRAY];
        if (idle) p += w[W_PICK_IDLE];
        if (b0) m += w[W_M_START];
        if (b1) m += w[W_M_COMPLETE];
        if (idle) m += w[W_M_IDLE];
        if (b0) k += w[W_P_START];
        if (b1) k += w[W_P_COMPLETE];
        if (idle) k += w[W_P_IDLE];
        lut[idx] = p; lut[48 + idx] = m; lut[64 + idx] = k;
    }
    for (int idx = 0; idx < 32; idx++) {   // bit0 invalid, bit1 moved, bit2 pickup, bit3 drop, bit4 to packaging
        double a = 0.0;
        if (idx & 4) a += w[W_AGV_DELIVERY];
        if (idx & 8) a += w[W_AGV_DELIVERY];
        if (idx & 16) a += w[W_AGV_PACKAGING];
        if (idx & 2) a += w[W_AGV_MOVE];
        if (idx & 1) a += w[W_AGV_INVALID];
        lut[16 + idx] = a;
    }
    lut[80] = w[W_ORDER];
    lut[81] = w[W_THROUGHPUT];
    lut[82] = w[W_TIME] * (double)step_size;   // TIME_PENALTY * time_elapsed (time_elapsed = step_size)
    for (int n = 1; n < RPROG_N; n++) lut[RPROG + n] = (1.0 / (double)n) * 100.0;
}

// status bits (include/fjsp.h)
constexpr uint32_t ST_DIVERGED = 0x1u, ST_OBS_OVERFLOW = 0x2u, ST_PKG_WAIT = 0x4u, ST_TRAY_LOST = 0x8u,
                   ST_PROD_LOST = 0x10u, ST_OVERWRITE = 0x20u, ST_SLOT_OVERFLOW = 0x40u,
                   ST_SPIN_TIMEOUT = 0x80u;   // a wave's wait for another wave's hand-off hit its bound

// Number of packed u32 words of Env in the SoA state buffer.
constexpr int NWORDS = 40;   // rows of the HBM state buffer (30 used)

// Diagnostic phase stamps: fjsp_stamps.h (FJSP_STAMP, FJSP_STAMP_AGENT; nothing in the product build).

// Per-env register state: 30 packed u32 words, bit-identical to the HBM `words` rows, so
// loading / storing an env is a plain copy and the live state costs 30 VGPRs instead of ~95.
// Field names follow the reference objects; every word index below is a compile-time
// constant at each use (list / machine / station indices come from templates or unrolled
// loops), so the words stay in registers.
//   W0  step[0,16) norders[16,24) next_order[24,32)     W1  ncompleted[0,8) total_packaged[8,32)
//   W2  status                                          W3  MT19937 cursor (mti | g << 16)
//   W4  pickup: cur_order[0,8) (0xFF none) cur_idx[8,12) cur_n[12,16) cur_type[16,18)
//       cur_color[18,20) tray_valid[20] tray_count[21,24) tray_start[24,28)
//   W5  tray_order[0,8) pool[8,24) slot_next[24,32)
//   W6  AGV: loc[0,3) carry[3,11) carry_code[11,24) carry_type[24,26) carry_color[26,28) np[28] nk[29]
//   W7+l   list l: head[0,8) tail[8,16) len[16,32)
//   W17+m  machine m: busy[0] cur[1,9) code[9,22) prog[22] k[23,27)     W19 next[0]|next[1] << 16
//   W20+s  packaging s: busy[0] hascur[1] qfirst[2,10) inflight[10,18) queued[18,32)
//   W24/25 completed[0..3] (16 bits each)                W26+s queue length at the last START
constexpr int NSTATE = 30;

struct Env {
    uint32_t w[NSTATE];
    FJSP_DIAG(uint64_t st_acc[8], st_t0;)
    FJSP_DEV uint32_t bf(int i, int o, int b) const { return (w[i] >> o) & ((1u << b) - 1u); }
    FJSP_DEV void sbf(int i, int o, int b, uint32_t v) {
        const uint32_t m = ((1u << b) - 1u) << o;
        w[i] = (w[i] & ~m) | ((v << o) & m);
    }
    // episode
    FJSP_DEV int step() const { return bf(0, 0, 16); }
    FJSP_DEV void set_step(int v) { sbf(0, 0, 16, v); }
    FJSP_DEV int norders() const { return bf(0, 16, 8); }
    FJSP_DEV void set_norders(int v) { sbf(0, 16, 8, v); }
    FJSP_DEV int next_order() const { return w[0] >> 24; }
    FJSP_DEV void set_next_order(int v) { sbf(0, 24, 8, v); }
    FJSP_DEV int ncompleted() const { return bf(1, 0, 8); }
    FJSP_DEV void set_ncompleted(int v) { sbf(1, 0, 8, v); }
    FJSP_DEV int total_packaged() const { return w[1] >> 8; }
    FJSP_DEV void set_total_packaged(int v) { sbf(1, 8, 24, v); }
    FJSP_DEV uint32_t status() const { return w[2]; }
    FJSP_DEV void flag(uint32_t b) { w[2] |= b; }
    FJSP_DEV int mti() const { return (int)w[3]; }
    FJSP_DEV void set_mti(int v) { w[3] = (uint32_t)v; }
    // pickup station (PickupStationAgent.py:88-94)
    FJSP_DEV int cur_order() const { const int v = bf(4, 0, 8); return v == 0xFF ? -1 : v; }
    FJSP_DEV void set_cur_order(int v) { sbf(4, 0, 8, v < 0 ? 0xFFu : (uint32_t)v); }
    FJSP_DEV int cur_idx() const { return bf(4, 8, 4); }
    FJSP_DEV void set_cur_idx(int v) { sbf(4, 8, 4, v); }
    FJSP_DEV int cur_n() const { return bf(4, 12, 4); }
    FJSP_DEV int cur_type() const { return bf(4, 16, 2); }
    FJSP_DEV int cur_color() const { return bf(4, 18, 2); }
    FJSP_DEV void set_cur_info(uint32_t ow) {   // n, type, colour of an order word at once
        sbf(4, 12, 8, ((ow >> 20) & 15u) | (((ow >> 24) & 15u) << 4));
    }
    FJSP_DEV int tray_valid() const { return bf(4, 20, 1); }
    FJSP_DEV void set_tray_valid(int v) { sbf(4, 20, 1, v); }
    FJSP_DEV int tray_count() const { return bf(4, 21, 3); }
    FJSP_DEV void set_tray_count(int v) { sbf(4, 21, 3, v); }
    FJSP_DEV int tray_start() const { return bf(4, 24, 4); }
    FJSP_DEV void set_tray_start(int v) { sbf(4, 24, 4, v); }
    FJSP_DEV int tray_order() const { return bf(5, 0, 8); }
    FJSP_DEV void set_tray_order(int v) { sbf(5, 0, 8, v); }
    FJSP_DEV int pool() const { return bf(5, 8, 16); }
    FJSP_DEV void set_pool(int v) { sbf(5, 8, 16, v); }
    FJSP_DEV int slot_next() const { return w[5] >> 24; }
    FJSP_DEV void set_slot_next(int v) { sbf(5, 24, 8, v); }
    // AGV (AGVAgent.py:41-45): location, carried tray slot (NIL = none), cached tray facts
    FJSP_DEV int loc() const { return bf(6, 0, 3); }
    FJSP_DEV void set_loc(int v) { sbf(6, 0, 3, v); }
    FJSP_DEV int carry() const { return bf(6, 3, 8); }
    FJSP_DEV void set_carry(int v) { sbf(6, 3, 8, v); }
    FJSP_DEV int carry_code() const { return bf(6, 11, 13); }
    FJSP_DEV int carry_type() const { return bf(6, 24, 2); }
    FJSP_DEV int carry_color() const { return bf(6, 26, 2); }
    FJSP_DEV int carry_np() const { return bf(6, 28, 1); }
    FJSP_DEV int carry_nk() const { return bf(6, 29, 1); }
    FJSP_DEV void set_carried(int slot, int code, int type, int color, int np, int nk) {
        w[6] = (w[6] & 7u) | ((uint32_t)slot << 3) | ((uint32_t)code << 11) | ((uint32_t)type << 24) |
               ((uint32_t)color << 26) | ((uint32_t)np << 28) | ((uint32_t)nk << 29);
    }
    // FIFO lists in the slot arena
    FJSP_DEV int lh(int l) const { return bf(7 + l, 0, 8); }
    FJSP_DEV int lt(int l) const { return bf(7 + l, 8, 8); }
    FJSP_DEV int ll(int l) const { return w[7 + l] >> 16; }
    FJSP_DEV void set_list(int l, int h, int t, int n) {
        w[7 + l] = (uint32_t)h | ((uint32_t)t << 8) | ((uint32_t)n << 16);
    }
    // machines (MachineAgent.py:40-47)
    FJSP_DEV int m_busy(int m) const { return bf(17 + m, 0, 1); }
    FJSP_DEV void set_m_busy(int m, int v) { sbf(17 + m, 0, 1, v); }
    FJSP_DEV int m_cur(int m) const { return bf(17 + m, 1, 8); }
    FJSP_DEV void set_m_cur(int m, int v) { sbf(17 + m, 1, 8, v); }
    FJSP_DEV int m_code(int m) const { return bf(17 + m, 9, 13); }
    FJSP_DEV int m_prog(int m) const { return bf(17 + m, 22, 1); }
    FJSP_DEV void set_m_prog(int m, int v) { sbf(17 + m, 22, 1, v); }
    FJSP_DEV int m_k(int m) const { return bf(17 + m, 23, 4); }
    FJSP_DEV void set_m_k(int m, int v) { sbf(17 + m, 23, 4, v); }
    FJSP_DEV int m_next(int m) const { return bf(19, 16 * m, 16); }
    FJSP_DEV void set_m_next(int m, int v) { sbf(19, 16 * m, 16, v); }
    FJSP_DEV void set_m_grant(int m, int slot, int code, int busy) {   // k = 0, progress unchanged
        w[17 + m] = (w[17 + m] & (1u << 22)) | (uint32_t)busy | ((uint32_t)slot << 1) | ((uint32_t)code << 9);
    }
    // packaging (PackagingAgent.py:250-256): qfirst = first queued (not yet granted) run
    FJSP_DEV int p_busy(int s) const { return bf(20 + s, 0, 1); }
    FJSP_DEV void set_p_busy(int s, int v) { sbf(20 + s, 0, 1, v); }
    FJSP_DEV int p_hascur(int s) const { return bf(20 + s, 1, 1); }
    FJSP_DEV int p_qfirst(int s) const { return bf(20 + s, 2, 8); }
    FJSP_DEV void set_p_qfirst(int s, int v) { sbf(20 + s, 2, 8, v); }
    FJSP_DEV int p_inflight(int s) const { return bf(20 + s, 10, 8); }
    FJSP_DEV void set_p_inflight(int s, int v) { sbf(20 + s, 10, 8, v); }
    FJSP_DEV int p_queued(int s) const { return w[20 + s] >> 18; }
    FJSP_DEV void set_p_queued(int s, int v) { sbf(20 + s, 18, 14, v); }
    FJSP_DEV int p_completed(int s) const { return bf(24 + (s >> 1), 16 * (s & 1), 16); }
    FJSP_DEV void set_p_completed(int s, int v) { sbf(24 + (s >> 1), 16 * (s & 1), 16, v); }
    // queue length at the last START (0 = never started); the float progress of the observation
    // is derived from it (pack_progress), so the step itself never computes it
    FJSP_DEV int p_startn(int s) const { return (int)w[26 + s]; }
};

// OR into an order word shared by two waves (k_step_ag: the machines' processed bits and the
// packaging completions update one word from different wavefronts); returns the old word.
#ifdef __HIP__
FJSP_DEV uint32_t order_or(uint32_t* p, uint32_t v) {
    return __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
#else
inline uint32_t order_or(uint32_t* p, uint32_t v) { const uint32_t o = *p; *p = o | v; return o; }
#endif

// ---- table accessors: element i of a per-env table = base[i * stride]
struct Tables {
    uint32_t* orders;   // [MAX_ORDERS]
    uint16_t* scode;    // [MAX_SLOTS] tray code
    uint8_t* snext;     // [MAX_SLOTS] next slot in its list
    uint16_t* scstep;   // [MAX_SLOTS] step at which an in-flight packaging run completes
    int stride;
};

template <int L>
FJSP_DEV void list_push(Env& E, const Tables& T, int s) {
    const int n = E.ll(L);
    T.snext[s * T.stride] = (uint8_t)NIL;
    if (n != 0) T.snext[E.lt(L) * T.stride] = (uint8_t)s;
    E.set_list(L, n == 0 ? s : E.lh(L), s, n + 1);
}
template <int L>
FJSP_DEV int list_pop(Env& E, const Tables& T) {
    const int s = E.lh(L), n = E.ll(L) - 1;
    const int next = T.snext[s * T.stride];
    E.set_list(L, n == 0 ? NIL : next, n == 0 ? NIL : E.lt(L), n);
    return s;
}
// Lists selected at run time (CAND = bitmask of the lists the index can name): the list word
// is picked / written back with a select chain over the candidate registers, so lanes that
// pop or push different lists share ONE memory round trip instead of one branch each.
template <uint32_t CAND>
FJSP_DEV uint32_t lword(const Env& E, int l) {
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < NLIST; i++)
        if ((CAND >> i) & 1u) v = (l == i) ? E.w[7 + i] : v;
    return v;
}
template <uint32_t CAND>
FJSP_DEV void set_lword(Env& E, int l, uint32_t v) {
#pragma unroll
    for (int i = 0; i < NLIST; i++)
        if ((CAND >> i) & 1u) E.w[7 + i] = (l == i) ? v : E.w[7 + i];
}
template <uint32_t CAND>
FJSP_DEV void list_push_dyn(Env& E, const Tables& T, int l, int s) {
    const uint32_t lw = lword<CAND>(E, l);
    const uint32_t n = lw >> 16;
    T.snext[s * T.stride] = (uint8_t)NIL;
    if (n != 0) T.snext[((lw >> 8) & 0xFFu) * T.stride] = (uint8_t)s;
    set_lword<CAND>(E, l, (n == 0 ? (uint32_t)s : (lw & 0xFFu)) | ((uint32_t)s << 8) | ((n + 1) << 16));
}
template <uint32_t CAND>
FJSP_DEV int list_pop_dyn(Env& E, const Tables& T, int l) {   // list must be non-empty
    const uint32_t lw = lword<CAND>(E, l);
    const int s = (int)(lw & 0xFFu);
    const uint32_t n = (lw >> 16) - 1u;
    const uint32_t next = T.snext[s * T.stride];
    set_lword<CAND>(E, l, n == 0 ? ((uint32_t)NIL | ((uint32_t)NIL << 8)) : (next | (lw & 0xFF00u) | (n << 16)));
    return s;
}

// new tray slot holding `code` (bump allocator, reset per episode)
FJSP_DEV int slot_new(Env& E, const Tables& T, int code) {
    const int s = E.slot_next();
    if (s >= MAX_SLOTS) { E.flag(ST_SLOT_OVERFLOW | ST_DIVERGED); return -1; }
    E.set_slot_next(s + 1);
    T.scode[s * T.stride] = (uint16_t)code;
    return s;
}

// ---- reward / result bit layout (oracle/fjsp_oracle.c, RESULT_KEYS in gen_golden.py)
constexpr uint32_t R_EXEC = 0x80u;

// PickupStationAgent.execute_action (PickupStationAgent.py:190-276), predicated like
// agv_execute: LOAD's outcome (start the next order, take an empty tray, load one product,
// hand the tray to ready_trays when the order ends / the tray is full) and SIGNAL are
// conditions; the only memory operations are the next order's word (when an order starts)
// and the single tray push.
FJSP_DEV uint32_t pickup_execute(Env& E, const Tables& T, const Cfg& C, int action) {
    const int co = E.cur_order(), no = E.next_order();
    const bool more = no < E.norders();
    const bool has_orders = more || co >= 0;
    const bool a1 = action == 1;
    // order (PickupStationAgent.py:210-215)
    const bool start = a1 && co < 0 && more;
    if (start) E.set_cur_info(T.orders[no * T.stride]);
    E.set_next_order(no + (start ? 1 : 0));
    const int co1 = start ? no : co;
    const int idx1 = start ? 0 : E.cur_idx();
    const bool ok_order = a1 && co1 >= 0;
    // tray (:217-222)
    const bool tv = E.tray_valid();
    const int pool = E.pool();
    const bool take = ok_order && !tv && pool > 0;
    const bool ok = ok_order && (tv || pool > 0);
    const int cnt = take ? 0 : E.tray_count();
    const int torder = take ? co1 : E.tray_order();
    const int tstart = take ? idx1 : E.tray_start();
    // load one product (:224-262)
    const bool blocked = ok && (cnt >= C.tray_cap || co1 != torder);   // full / :231-235 (unreachable)
    const bool load = ok && !blocked;
    const int cnt2 = cnt + (load ? 1 : 0);
    const int idx2 = idx1 + (load ? 1 : 0);
    const bool finished = load && idx2 >= E.cur_n();
    const bool trayfull = load && !finished && cnt2 >= C.tray_cap;
    // SIGNAL (:264-272)
    const bool sig = action == 2 && tv && E.tray_count() > 0;
    const bool push = (ok && (blocked || finished || trayfull)) || sig;
    // state
    E.set_pool(pool - (take ? 1 : 0));
    E.set_cur_order(finished ? -1 : co1);
    E.set_cur_idx(finished ? 0 : idx2);
    E.set_tray_order(torder);
    E.set_tray_start(tstart);
    E.set_tray_count(cnt2);
    E.set_tray_valid((tv || take) && !push);
    if (push) {
        const int s = slot_new(E, T, tc_make(torder, tstart, cnt2));
        if (s >= 0) list_push<L_PREADY>(E, T, s);
    }
    // result: 1 success, 2 product_loaded, 4 tray_completed, 8 idle_with_orders
    uint32_t r = R_EXEC;
    r |= action == 0 ? (1u | (has_orders ? 8u : 0u)) : 0u;
    r |= load ? 3u : 0u;
    r |= (ok && (blocked || finished || trayfull)) ? 4u : 0u;
    r |= sig ? 1u : 0u;
    return r;
}

// FJSPSimulation.add_tray_to_packaging (FJSPSimulation.py:402-430): first station (dict order
// blue_1, blue_2, red, green) whose colour matches and whose Resource has capacity; -1 = none
// (the products are lost).  PackagingColor RED=1 BLUE=2 GREEN=3.
FJSP_DEV int pkg_station(const Env& E, const Cfg& C, int color) {
    const uint32_t room = (uint32_t)(E.p_inflight(0) < C.pkg_cap) | ((uint32_t)(E.p_inflight(1) < C.pkg_cap) << 1) |
                          ((uint32_t)(E.p_inflight(2) < C.pkg_cap) << 2) | ((uint32_t)(E.p_inflight(3) < C.pkg_cap) << 3);
    // stations of each colour: RED -> {red}, BLUE -> {blue_1, blue_2}, GREEN -> {green}
    const uint32_t cand = (uint32_t)nib(nibs(0, 0x4, 0x3, 0x8, 0, 0), color & 3) & room;
    return __builtin_ffs((int)cand) - 1;   // first in dict order; -1 = none
}

constexpr uint16_t PKG_CONT = 0xFFFF;   // scstep of a run that is not the first of its batch
constexpr uint32_t PICK_LISTS = (1u << L_PREADY) | (1u << L_STORAGE) | (1u << L_M0R) | (1u << L_M1R);
constexpr uint32_t DROP_LISTS = (1u << L_STORAGE) | (1u << L_M0Q) | (1u << L_M1Q) | (0xFu << L_PKG);

// AGVAgent.execute_action / _execute_pickup / _execute_drop (AGVAgent.py:180-368).
// Returns the result word; *move_to receives the target location of a spawned move.
// Written predicated (straight-line): every action's outcome is computed as a condition and the
// state words are updated with selects, so a wavefront whose lanes take all 8 actions executes
// one path instead of the union of 8 branchy ones.  Only the memory operations sit in (two)
// small guarded blocks: the PICKUP pop's loads and the DROP push's stores.
// DEFER (the pipelined kernel's AGV-ahead wave): a drop at packaging is not routed here — the
// station choice needs the Resource counts after the current run phase — but returned in
// *pend (1 | slot << 1 | code << 9 | colour << 22) for agv_pack_drop.
template <bool DEFER = false>
FJSP_DEV uint32_t agv_execute(Env& E, const Tables& T, const Cfg& C, int action, int* move_to,
                              uint32_t* pend = nullptr) {
    const int loc = E.loc();
    const int carry = E.carry();
    const bool has = carry != NIL;
    // 1..5: moves (AGVAgent.py:218-252); distance 0 is a successful no-op
    const bool is_move = (unsigned)(action - 1) < 5u;
    const int ml = move_loc(action);
    const int d = manhattan(loc, ml);
    const bool moved = is_move && d != 0;
    // 6: PICKUP, FIFO front of the list at this location (_execute_pickup :254-293)
    const int src = nib(nibs(0, L_PREADY, L_M1R, L_M0R, L_STORAGE, L_STORAGE), loc);
    const uint32_t lws = lword<PICK_LISTS>(E, src);
    const bool ok6 = action == 6 && !has && loc != LOC_PACK && (lws >> 16) != 0;
    // 7: DROP (_execute_drop :295-368): validity per location as one bit vector indexed by loc
    const int code = E.carry_code(), ty = E.carry_type(), np = E.carry_np(), nk = E.carry_nk();
    const uint32_t cond = ((uint32_t)(tc_count(code) == 0) << LOC_PICKUP) |
                          ((uint32_t)(np && (ty == 1 || ty == 2)) << LOC_SMALL) |
                          ((uint32_t)(np && (ty == 3 || ty == 2)) << LOC_BIG) | (1u << LOC_STORAGE) |
                          ((uint32_t)(nk && !np) << LOC_PACK);
    const bool ok7 = action == 7 && has && ((cond >> loc) & 1u);
    const bool at_pick = loc == LOC_PICKUP, at_store = loc == LOC_STORAGE, at_pack = loc == LOC_PACK;
    const bool store_full = E.ll(L_STORAGE) >= C.storage_cap;
    const int st = DEFER ? -1 : pkg_station(E, C, E.carry_color());
    const int base = nib(nibs(0xF, 0xF, L_M1Q, L_M0Q, L_STORAGE, L_PKG), loc);
    const bool no_dst = base == 0xF || (at_store && store_full) || (at_pack && (DEFER || st < 0));
    const int dst = no_dst ? -1 : base + (at_pack ? st : 0);
    // memory: pop (loads) / push (stores)
    uint32_t next = 0, scode = 0, ow = 0;
    const int ps = (int)(lws & 0xFFu);
    if (ok6) {
        next = T.snext[ps * T.stride];
        scode = T.scode[ps * T.stride];
        ow = T.orders[tc_order((int)scode) * T.stride];
    }
    const bool push = ok7 && dst >= 0;
    const uint32_t lwd = lword<DROP_LISTS>(E, dst);
    if (push) {
        T.snext[carry * T.stride] = (uint8_t)NIL;
        if (at_pack) T.scstep[carry * T.stride] = PKG_CONT;
        if ((lwd >> 16) != 0) T.snext[((lwd >> 8) & 0xFFu) * T.stride] = (uint8_t)carry;
    }
    // list words
    const uint32_t n6 = (lws >> 16) - 1u;
    const uint32_t popped = n6 == 0 ? ((uint32_t)NIL | ((uint32_t)NIL << 8)) : (next | (lws & 0xFF00u) | (n6 << 16));
    const uint32_t nd = lwd >> 16;
    const uint32_t pushed = (nd == 0 ? (uint32_t)carry : (lwd & 0xFFu)) | ((uint32_t)carry << 8) | ((nd + 1) << 16);
#pragma unroll
    for (int i = 0; i < NLIST; i++) {
        if (!(((PICK_LISTS | DROP_LISTS) >> i) & 1u)) continue;
        uint32_t v = E.w[7 + i];
        if ((PICK_LISTS >> i) & 1u) v = (ok6 && src == i) ? popped : v;
        if ((DROP_LISTS >> i) & 1u) v = (push && dst == i) ? pushed : v;
        E.w[7 + i] = v;
    }
    // packaging station: the dropped tray's products join its queue (PackagingAgent.add_tray)
    if (!DEFER) {
        const bool to_st = push && at_pack;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t wk = E.w[20 + k];
            const uint32_t qf = ((wk >> 2) & 0xFFu) == (uint32_t)NIL ? (uint32_t)carry : ((wk >> 2) & 0xFFu);
            const uint32_t nw = (wk & ~(0xFFu << 2) & 0x3FFFFu) | (qf << 2) | (((wk >> 18) + (uint32_t)tc_count(code)) << 18);
            E.w[20 + k] = (to_st && st == k) ? nw : wk;
        }
    } else {
        *pend = (ok7 && at_pack) ? (1u | ((uint32_t)carry << 1) | ((uint32_t)code << 9) | ((uint32_t)E.carry_color() << 22)) : 0u;
    }
    // AGV word: carried tray (pickup) / empty hands (drop)
    const uint32_t rg = tc_range((int)scode);
    const bool full6 = tc_count((int)scode) > 0;
    const uint32_t carried = (E.w[6] & 7u) | ((uint32_t)ps << 3) | (scode << 11) |
                             (full6 ? (((uint32_t)ow_type(ow) << 24) | ((uint32_t)ow_color(ow) << 26) |
                                       ((uint32_t)((ow & rg) != rg) << 28) | ((uint32_t)(((ow >> 9) & rg) != rg) << 29))
                                    : 0u);
    const uint32_t dropped = (E.w[6] & ~(0xFFu << 3)) | ((uint32_t)NIL << 3);
    E.w[6] = ok6 ? carried : ok7 ? dropped : E.w[6];
    // add_empty_tray at the pickup station; lost tray / products flags
    E.set_pool(E.pool() + ((ok7 && at_pick) ? 1 : 0));
    uint32_t fl = (ok7 && at_store && store_full) ? ST_TRAY_LOST : 0u;
    fl |= (!DEFER && ok7 && at_pack && st < 0) ? ST_PROD_LOST : 0u;
    E.w[2] |= fl;
    if (moved) *move_to = ml;
    // result: 1 success, 2 invalid, 4 moved, 8 pickup, 16 drop, 32 to packaging; 16.. distance
    const bool success = action == 0 || is_move || ok6 || ok7;
    uint32_t r = R_EXEC | (success ? 1u : 2u);
    r |= moved ? (4u | ((uint32_t)d << 16)) : 0u;
    r |= ok6 ? 8u : 0u;
    r |= ok7 ? (16u | (at_pack ? 32u : 0u)) : 0u;
    return r;
}

// agv_execute<true> in two halves (k_step_ag's P wave).  agv_pre needs only the AGV's own words
// (W6: location and carried tray, W8: storage) and the list words as they were after the AGV's
// previous step (E): it decides the action's outcome where that does not depend on other agents
// and prefetches the front slot of the list a PICKUP would pop — a list's front does not change
// while it is non-empty (the pickup station and the machines only append; only the AGV pops).
// agv_fin completes the step on the final list words (after the pickup station's action and the
// machines' actions of the previous step).  Together they equal agv_execute<true>.
struct AgvPre {
    int loc, carry, code, src, dst, ml, d, action;
    bool want6, is_move, moved, ok7, at_pick, at_store, at_pack, store_full;
    uint32_t pre_len, pnext, pcode, pow;
};
FJSP_DEV AgvPre agv_pre(const Env& E, const Tables& T, const Cfg& C, int action) {
    AgvPre a;
    a.action = action;
    a.loc = E.loc();
    a.carry = E.carry();
    const bool has = a.carry != NIL;
    a.is_move = (unsigned)(action - 1) < 5u;
    a.ml = move_loc(action);
    a.d = manhattan(a.loc, a.ml);
    a.moved = a.is_move && a.d != 0;
    a.src = nib(nibs(0, L_PREADY, L_M1R, L_M0R, L_STORAGE, L_STORAGE), a.loc);
    a.want6 = action == 6 && !has && a.loc != LOC_PACK;
    a.code = E.carry_code();
    const int ty = E.carry_type(), np = E.carry_np(), nk = E.carry_nk();
    const uint32_t cond = ((uint32_t)(tc_count(a.code) == 0) << LOC_PICKUP) |
                          ((uint32_t)(np && (ty == 1 || ty == 2)) << LOC_SMALL) |
                          ((uint32_t)(np && (ty == 3 || ty == 2)) << LOC_BIG) | (1u << LOC_STORAGE) |
                          ((uint32_t)(nk && !np) << LOC_PACK);
    a.ok7 = action == 7 && has && ((cond >> a.loc) & 1u);
    a.at_pick = a.loc == LOC_PICKUP;
    a.at_store = a.loc == LOC_STORAGE;
    a.at_pack = a.loc == LOC_PACK;
    a.store_full = E.ll(L_STORAGE) >= C.storage_cap;
    const int base = nib(nibs(0xF, 0xF, L_M1Q, L_M0Q, L_STORAGE, L_PKG), a.loc);
    const bool no_dst = base == 0xF || (a.at_store && a.store_full) || a.at_pack;
    a.dst = no_dst ? -1 : base;
    // prefetch the front of the pickup source
    const uint32_t lws = lword<PICK_LISTS>(E, a.src);
    a.pre_len = a.want6 ? (lws >> 16) : 0u;
    a.pnext = 0; a.pcode = 0; a.pow = 0;
    if (a.pre_len != 0) {
        const int ps = (int)(lws & 0xFFu);
        a.pnext = T.snext[ps * T.stride];
        a.pcode = T.scode[ps * T.stride];
        a.pow = T.orders[tc_order((int)a.pcode) * T.stride];
    }
    return a;
}
FJSP_DEV uint32_t agv_fin(Env& E, const Tables& T, const AgvPre& a, int* move_to, uint32_t* pend) {
    const uint32_t lws = lword<PICK_LISTS>(E, a.src);
    const uint32_t len = lws >> 16;
    const bool ok6 = a.want6 && len != 0;
    const int ps = (int)(lws & 0xFFu);
    uint32_t next = a.pnext, scode = a.pcode, ow = a.pow;
    if (ok6 && a.pre_len == 0) {   // the list was empty before: its front is new
        next = T.snext[ps * T.stride];
        scode = T.scode[ps * T.stride];
        ow = T.orders[tc_order((int)scode) * T.stride];
    } else if (ok6 && a.pre_len == 1 && len >= 2) {   // the single front got a successor: the
        next = (lws >> 8) & 0xFFu;                      // tray pushed since (one push per list per
    }                                                   // step: pickup, a machine's SIGNAL), the tail
    const int carry = a.carry;
    const bool push = a.ok7 && a.dst >= 0;
    const uint32_t lwd = lword<DROP_LISTS>(E, a.dst);
    if (push) {
        T.snext[carry * T.stride] = (uint8_t)NIL;
        if ((lwd >> 16) != 0) T.snext[((lwd >> 8) & 0xFFu) * T.stride] = (uint8_t)carry;
    }
    const uint32_t n6 = len - 1u;
    const uint32_t popped = n6 == 0 ? ((uint32_t)NIL | ((uint32_t)NIL << 8)) : (next | (lws & 0xFF00u) | (n6 << 16));
    const uint32_t nd = lwd >> 16;
    const uint32_t pushed = (nd == 0 ? (uint32_t)carry : (lwd & 0xFFu)) | ((uint32_t)carry << 8) | ((nd + 1) << 16);
#pragma unroll
    for (int i = 0; i < NLIST; i++) {
        if (!(((PICK_LISTS | DROP_LISTS) >> i) & 1u)) continue;
        uint32_t v = E.w[7 + i];
        if ((PICK_LISTS >> i) & 1u) v = (ok6 && a.src == i) ? popped : v;
        if ((DROP_LISTS >> i) & 1u) v = (push && a.dst == i) ? pushed : v;
        E.w[7 + i] = v;
    }
    *pend = (a.ok7 && a.at_pack) ? (1u | ((uint32_t)carry << 1) | ((uint32_t)a.code << 9) | ((uint32_t)E.carry_color() << 22)) : 0u;
    const uint32_t rg = tc_range((int)scode);
    const bool full6 = tc_count((int)scode) > 0;
    const uint32_t carried = (E.w[6] & 7u) | ((uint32_t)ps << 3) | (scode << 11) |
                             (full6 ? (((uint32_t)ow_type(ow) << 24) | ((uint32_t)ow_color(ow) << 26) |
                                       ((uint32_t)((ow & rg) != rg) << 28) | ((uint32_t)(((ow >> 9) & rg) != rg) << 29))
                                    : 0u);
    const uint32_t dropped = (E.w[6] & ~(0xFFu << 3)) | ((uint32_t)NIL << 3);
    E.w[6] = ok6 ? carried : a.ok7 ? dropped : E.w[6];
    E.set_pool(E.pool() + ((a.ok7 && a.at_pick) ? 1 : 0));
    E.w[2] |= (a.ok7 && a.at_store && a.store_full) ? ST_TRAY_LOST : 0u;
    if (a.moved) *move_to = a.ml;
    const bool success = a.action == 0 || a.is_move || ok6 || a.ok7;
    uint32_t r = R_EXEC | (success ? 1u : 2u);
    r |= a.moved ? (4u | ((uint32_t)a.d << 16)) : 0u;
    r |= ok6 ? 8u : 0u;
    r |= a.ok7 ? (16u | (a.at_pack ? 32u : 0u)) : 0u;
    return r;
}

// The packaging half of a deferred AGV drop (agv_execute<true>): route the tray to its station
// (FJSPSimulation.add_tray_to_packaging) with the Resource counts as they are now.
FJSP_DEV void agv_pack_drop(Env& E, const Tables& T, const Cfg& C, uint32_t pend) {
    const int carry = (int)((pend >> 1) & 0xFFu), code = (int)((pend >> 9) & 0x1FFFu);
    const int st = pkg_station(E, C, (int)((pend >> 22) & 3u));
    if (st < 0) { E.flag(ST_PROD_LOST); return; }
    const uint32_t lwd = lword<(0xFu << L_PKG)>(E, L_PKG + st);
    T.snext[carry * T.stride] = (uint8_t)NIL;
    T.scstep[carry * T.stride] = PKG_CONT;
    const uint32_t nd = lwd >> 16;
    if (nd != 0) T.snext[((lwd >> 8) & 0xFFu) * T.stride] = (uint8_t)carry;
    set_lword<(0xFu << L_PKG)>(E, L_PKG + st,
                                (nd == 0 ? (uint32_t)carry : (lwd & 0xFFu)) | ((uint32_t)carry << 8) | ((nd + 1) << 16));
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t wk = E.w[20 + k];
        const uint32_t qf = ((wk >> 2) & 0xFFu) == (uint32_t)NIL ? (uint32_t)carry : ((wk >> 2) & 0xFFu);
        const uint32_t nw = (wk & ~(0xFFu << 2) & 0x3FFFFu) | (qf << 2) | (((wk >> 18) + (uint32_t)tc_count(code)) << 18);
        E.w[20 + k] = (st == k) ? nw : wk;
    }
}

// MachineAgent.execute_action (MachineAgent.py:99-139); grant happens in the run.
template <int M>
// next_known >= 0: the queue front's successor, known without reading the table (k_step_ag's
// AM reads it before the AGV's drop: the drop only appends, so a front with a successor keeps
// it, a lone front gets the dropped tray, now the tail, and an empty queue's dropped tray is
// alone); -1: read it.
FJSP_DEV uint32_t machine_execute(Env& E, const Tables& T, int action, int* start_slot, int next_known = -1) {
    constexpr int LQ = M == 0 ? L_M0Q : L_M1Q;
    constexpr int LR = M == 0 ? L_M0R : L_M1R;
    const bool busy = E.m_busy(M);
    const bool idle_q = E.ll(LQ) > 0 && !busy;
    const int cur = E.m_cur(M);
    const bool go = action == 1 && idle_q;            // START: pop the queue front
    const bool sig = action == 2 && !busy && cur != NIL;   // SIGNAL: current tray -> ready_trays
    if (go) {
        if (next_known < 0) {
            *start_slot = list_pop<LQ>(E, T);
        } else {
            const int h = E.lh(LQ), n = E.ll(LQ) - 1;
            E.set_list(LQ, n == 0 ? NIL : next_known, n == 0 ? NIL : E.lt(LQ), n);
            *start_slot = h;
        }
    }
    if (sig) {
        list_push<LR>(E, T, cur);
        E.set_m_cur(M, NIL);
    }
    // 1 success, 2 started, 4 completed, 8 idle_with_queue
    uint32_t r = R_EXEC;
    r |= action == 0 ? (1u | (idle_q ? 8u : 0u)) : 0u;
    r |= go ? 3u : 0u;
    r |= sig ? 5u : 0u;
    return r;
}

// PackagingAgent.execute_action (PackagingAgent.py:301-335)
template <int S>
FJSP_DEV uint32_t pack_execute(Env& E, int action, int* started) {
    const int n = E.p_queued(S);
    const bool busy = E.p_busy(S);
    const bool go = action == 1 && n > 0;
    E.w[26 + S] = go ? (uint32_t)n : E.w[26 + S];   // progress = pack_progress(n), see observe
    *started = go ? 1 : *started;
    // 1 success, 2 started, 4 completed, 8 idle_with_queue; 16.. completed count
    uint32_t r = R_EXEC;
    r |= action == 0 ? (1u | ((n > 0 && !busy) ? 8u : 0u)) : 0u;
    r |= go ? 3u : 0u;
    r |= (action == 2 && !busy && E.p_hascur(S)) ? (4u | ((uint32_t)E.p_completed(S) << 16)) : 0u;
    return r;
}

// ---------------------------------------------------------------- run phase (T, T+step]
// Machines: a product completion due this step (old NORMAL event), then the grant of this
// step's START (MachineAgent.py:151-169).  Both machines' memory reads (the completing
// product's order word, the granted tray's code) are issued together; two completions of
// the same order update its word once.
template <int M>
FJSP_DEV void machine_done(Env& E, const Cfg& C, int step) {
    const int k = E.m_k(M);
    E.set_m_k(M, k + 1);
    if (k + 1 >= tc_count(E.m_code(M))) { E.set_m_busy(M, 0); E.set_m_prog(M, 1); }
    else E.set_m_next(M, step + (M == 0 ? C.ptk_small : C.ptk_big));
}
template <int M>
FJSP_DEV void machine_grant(Env& E, const Cfg& C, int slot, int code, int step) {
    if (E.m_cur(M) != NIL) E.flag(ST_OVERWRITE);
    const int busy = tc_count(code) > 0;   // an empty tray's loop body never runs
    E.set_m_grant(M, slot, code, busy);
    if (busy) E.set_m_next(M, step + (M == 0 ? C.ptk_small : C.ptk_big));
    else E.set_m_prog(M, 1);
}
// AT: the order words are shared with another wave (k_step_ag) -> atomic OR, no read.
template <bool AT = false>
FJSP_DEV void machines_run(Env& E, const Tables& T, const Cfg& C, int s0, int s1) {
    const int step = E.step();
    const bool due0 = E.m_busy(0) && E.m_next(0) == step, due1 = E.m_busy(1) && E.m_next(1) == step;
    const int c0 = E.m_code(0), c1 = E.m_code(1);
    const int o0 = tc_order(c0), o1 = tc_order(c1);
    const int g0 = T.scode[(s0 >= 0 ? s0 : 0) * T.stride];
    const int g1 = T.scode[(s1 >= 0 ? s1 : 0) * T.stride];
    const uint32_t b0 = 1u << (tc_start(c0) + E.m_k(0)), b1 = 1u << (tc_start(c1) + E.m_k(1));
    // product.is_processed = True
    if constexpr (AT) {
        if (due0) order_or(&T.orders[o0 * T.stride], b0);
        if (due1) order_or(&T.orders[o1 * T.stride], b1);
    } else {
        // independent loads (addresses clamped to valid entries when unused)
        const uint32_t w0 = T.orders[(due0 ? o0 : 0) * T.stride];
        const uint32_t w1 = T.orders[(due1 ? o1 : 0) * T.stride];
        if (due0) T.orders[o0 * T.stride] = w0 | b0;
        if (due1) T.orders[o1 * T.stride] = ((due0 && o0 == o1) ? (w0 | b0) : w1) | b1;
    }
    if (due0) machine_done<0>(E, C, step);
    if (s0 >= 0) machine_grant<0>(E, C, s0, g0, step);
    if (due1) machine_done<1>(E, C, step);
    if (s1 >= 0) machine_grant<1>(E, C, s1, g1, step);
}

// Packaging: completions of the batch due this step, then grants of this step's START.
// A batch (every run queued at one START) is a contiguous stretch of the station's list: its
// first run's scstep holds the completion step, the other runs PKG_CONT (written when the AGV
// drops them), so a START is one store and a completion pops runs until the next batch start
// or the first ungranted run (qfirst).
// `due` = the in-flight head run completes now (pack_due: the four stations' head checks are
// issued as one batch of independent loads).
template <int S>
FJSP_DEV bool pack_due(const Env& E, const Tables& T, int step) {
    constexpr int L = L_PKG + S;
    const int h = E.lh(L);
    const bool inflight = E.ll(L) > 0 && h != E.p_qfirst(S);
    const uint16_t cs = T.scstep[(inflight ? h : 0) * T.stride];   // slot 0 always exists
    return inflight && cs == (uint16_t)step;
}
template <int S, bool AT = false>
FJSP_DEV void pack_run(Env& E, const Tables& T, const Cfg& C, int started, bool due, int* orders_done) {
    constexpr int L = L_PKG + S;
    const int step = E.step();
    const int qfirst = E.p_qfirst(S);
    if (started && E.p_inflight(S) + E.p_queued(S) > C.pkg_cap)
        E.flag(ST_PKG_WAIT | ST_DIVERGED);   // Request would wait (users == capacity)
    // completions (PackagingAgent.py:143-147)
    int done = 0;
    while (due) {
        const int s = list_pop<L>(E, T);
        const int code = T.scode[s * T.stride];
        const int o = tc_order(code);
        const uint32_t add = tc_range(code) << 9;
        uint32_t w = (AT ? order_or(&T.orders[o * T.stride], add) : T.orders[o * T.stride]) | add;
        const uint32_t full = (1u << ow_n(w)) - 1u;
        if (!(w & (1u << 18)) && ((w >> 9) & full) == full) {   // _check_order_completions
            w |= 1u << 18;
            *orders_done += 1;
            if (AT) order_or(&T.orders[o * T.stride], 1u << 18);   // only this wave writes the bit
        }
        if (!AT) T.orders[o * T.stride] = w;
        done += tc_count(code);
        // the batch continues while the next run is granted (not qfirst) and not a batch start
        due = E.ll(L) > 0 && E.lh(L) != qfirst && T.scstep[E.lh(L) * T.stride] == PKG_CONT;
    }
    if (done) {
        E.set_p_completed(S, E.p_completed(S) + done);
        E.set_total_packaged(E.total_packaged() + done);
        E.set_p_inflight(S, E.p_inflight(S) - done);
        E.set_p_busy(S, 0);
    }
    // grants: every queued product, in queue order (PackagingAgent.py:136-141)
    if (started) {   // the whole queue [qfirst, tail] is one batch: mark its first run
        T.scstep[qfirst * T.stride] = (uint16_t)(step + C.ptk_pack);
        const int inflight = E.p_inflight(S) + E.p_queued(S);
        // busy = 1, hascur = 1, qfirst = NIL, inflight += queued, queued = 0
        E.w[20 + S] = 3u | ((uint32_t)NIL << 2) | ((uint32_t)(inflight & 0xFF) << 10);
    }
}

// k_step_ag splits pack_run around the action phase.  pack_complete: the completions of the
// station's in-flight batch due at this step (NORMAL events older than the step's actions,
// PackagingAgent.py:143-147) computed BEFORE the AGV's drop and the station's action: the
// completed runs leave the head of the station's list (a drop joins its tail, and the batch
// ends at the first run that is not PKG_CONT either way) and their products are ORed into the
// order table; returns the products packaged.  The counters and the busy flag are left as the
// action phase reads them (routing reads in-flight counts, the action reads busy) and applied
// by pack_finish together with the grants.
template <int S>
FJSP_DEV int pack_complete(Env& E, const Tables& T, bool due, int* orders_done) {
    constexpr int L = L_PKG + S;
    const int qfirst = E.p_qfirst(S);
    int done = 0;
    while (due) {
        const int s = list_pop<L>(E, T);
        const int code = T.scode[s * T.stride];
        const int o = tc_order(code);
        const uint32_t add = tc_range(code) << 9;
        const uint32_t w = order_or(&T.orders[o * T.stride], add) | add;
        const uint32_t full = (1u << ow_n(w)) - 1u;
        if (!(w & (1u << 18)) && ((w >> 9) & full) == full) {   // _check_order_completions
            order_or(&T.orders[o * T.stride], 1u << 18);
            *orders_done += 1;
        }
        done += tc_count(code);
        due = E.ll(L) > 0 && E.lh(L) != qfirst && T.scstep[E.lh(L) * T.stride] == PKG_CONT;
    }
    return done;
}
template <int S>
FJSP_DEV void pack_finish(Env& E, const Tables& T, const Cfg& C, int started, int done) {
    if (started && E.p_inflight(S) + E.p_queued(S) > C.pkg_cap) E.flag(ST_PKG_WAIT | ST_DIVERGED);
    if (done) {
        E.set_p_completed(S, E.p_completed(S) + done);
        E.set_total_packaged(E.total_packaged() + done);
        E.set_p_inflight(S, E.p_inflight(S) - done);
        E.set_p_busy(S, 0);
    }
    if (started) {
        T.scstep[E.p_qfirst(S) * T.stride] = (uint16_t)(E.step() + C.ptk_pack);
        const int inflight = E.p_inflight(S) + E.p_queued(S);
        E.w[20 + S] = 3u | ((uint32_t)NIL << 2) | ((uint32_t)(inflight & 0xFF) << 10);
    }
}

// ---------------------------------------------------------------- observations
// Observations and masks are emitted field by field into a Sink (store-as-you-go keeps the
// 67 output values out of the register file).  Sink API:
//   i32(f, v)  f in [0,20)   i8(f, v)  f in [0,12)   f32(f, v)  f in [0,6)   mask(f, v)  f in [0,29)
struct Obs {
    int32_t i32[NI32];
    int8_t i8[NI8];
    float f32[NF32];
    int8_t mask[NMASK];
};
struct ObsSink {   // materialises an Obs (host harness, tests)
    Obs& o;
    FJSP_DEV void i32(int f, int v) { o.i32[f] = v; }
    FJSP_DEV void i8(int f, int v) { o.i8[f] = (int8_t)v; }
    FJSP_DEV void f32(int f, float v) { o.f32[f] = v; }
    FJSP_DEV void mask(int f, int v) { o.mask[f] = (int8_t)v; }
};
struct MaskBits {  // mask bits per agent (bit i = action i valid), for masked synthetic actions
    uint32_t bits[NA] = {0, 0, 0, 0, 0, 0, 0, 0};
    FJSP_DEV void i32(int, int) {}
    FJSP_DEV void i8(int, int) {}
    FJSP_DEV void f32(int, float) {}
    FJSP_DEV void mask(int f, int v) {
        const int a = f < 3 ? 0 : f < 11 ? 1 : 2 + (f - 11) / 3;
        const int off = f < 3 ? 0 : f < 11 ? 3 : 11 + 3 * (a - 2);
        bits[a] |= (uint32_t)(v != 0) << (f - off);
    }
};

template <class Sink>
FJSP_DEV void compute_masks(const Env& E, const Cfg& C, Sink& m) {
    // pickup (PickupStationAgent.py:144-186)
    const int co = E.cur_order(), more_orders = E.next_order() < E.norders();
    const int tv = E.tray_valid(), tcnt = E.tray_count();
    const int has_order = co >= 0 || more_orders;
    const int has_tray = tv || E.pool() > 0;
    const int not_full = tv ? (tcnt < C.mask_tray_cap) : 1;
    const int prem = co >= 0 ? (E.cur_idx() < E.cur_n()) : more_orders;
    m.mask(0, 1);
    m.mask(1, has_order && has_tray && not_full && prem);
    m.mask(2, tv && tcnt > 0);
    // AGV (AGVAgent.py:79-178); the AGV is never mid-move at a step boundary
    const int loc = E.loc();
    m.mask(3, 1);
    m.mask(4, loc != LOC_PICKUP);
    m.mask(5, loc != LOC_SMALL);
    m.mask(6, loc != LOC_BIG);
    m.mask(7, loc != LOC_STORAGE);
    m.mask(8, loc != LOC_PACK);
    int pick = 0, drop = 0;
    if (E.carry() == NIL) {
        pick = (loc == LOC_PICKUP && E.ll(L_PREADY) > 0) || (loc == LOC_SMALL && E.ll(L_M0R) > 0) ||
               (loc == LOC_BIG && E.ll(L_M1R) > 0) || (loc == LOC_STORAGE && E.ll(L_STORAGE) > 0);
    } else {
        const int ty = E.carry_type(), np = E.carry_np();
        drop = (loc == LOC_PICKUP && tc_count(E.carry_code()) == 0) ||
               (loc == LOC_SMALL && np && (ty == 1 || ty == 2)) || (loc == LOC_BIG && np && (ty == 3 || ty == 2)) ||
               (loc == LOC_PACK && E.carry_nk() && !np) || (loc == LOC_STORAGE);
    }
    m.mask(9, pick);
    m.mask(10, drop);
    // machines (MachineAgent.py:72-97)
    m.mask(11, 1); m.mask(12, E.ll(L_M0Q) > 0 && !E.m_busy(0)); m.mask(13, !E.m_busy(0) && E.m_cur(0) != NIL);
    m.mask(14, 1); m.mask(15, E.ll(L_M1Q) > 0 && !E.m_busy(1)); m.mask(16, !E.m_busy(1) && E.m_cur(1) != NIL);
    // packaging (PackagingAgent.py:64-89)
#pragma unroll
    for (int s = 0; s < 4; s++) {
        const int busy = E.p_busy(s);
        m.mask(17 + 3 * s, 1);
        m.mask(18 + 3 * s, E.p_queued(s) > 0 && !busy && E.p_inflight(s) < C.pkg_cap);
        m.mask(19 + 3 * s, !busy && E.p_hascur(s));
    }
}

// PackagingAgent START: self.processing_progress = (i / len(self.product_queue)) * 100 with
// i == 1, in fp64 then float32 (tabulated for n < 256 in the reward table; exact either way).
FJSP_DEV float pack_progress(const Cfg& C, int n) {
    if (__builtin_expect(n >= RPROG_N, 0)) return (float)((1.0 / (double)n) * 100.0);   // n > packaging_capacity
    return (float)C.lut[RPROG + n];   // lut[RPROG] = 0.0: never started
}

FJSP_DEV int obs_i8_checked(Env& E, int v) {
    if (v > 127) E.flag(ST_OBS_OVERFLOW | ST_DIVERGED);
    return (int)(int8_t)v;
}

template <class Sink>
FJSP_DEV void observe(Env& E, const Cfg& C, Sink& o) {
    // pickup (PickupStationAgent.py:102-142)
    int osz = 0, rem = 0, npt = 0, npc = 0;
    const int co = E.cur_order();
    if (co >= 0) {
        osz = E.cur_n(); rem = osz - E.cur_idx();
        if (rem > 0) { npt = E.cur_type(); npc = E.cur_color(); }
    }
    int tt = 0, tcol = 0, tcnt = 0;
    if (E.tray_valid()) {
        tcnt = E.tray_count();
        if (tcnt > 0 && E.tray_order() == co) {   // a loaded tray always belongs to the current order
            tt = E.cur_type(); tcol = E.cur_color();
        }
    }
    o.i32(0, osz); o.i32(1, rem); o.i32(2, npt); o.i32(3, npc);
    o.i32(4, tt); o.i32(5, tcol); o.i32(6, tcnt);
    // AGV (AGVAgent.py:53-76)
    const int c = E.carry() != NIL, loc = E.loc();
    o.i32(7, loc_row(loc)); o.i32(8, loc_col(loc));
    o.i32(9, c);
    o.i32(10, c ? tc_count(E.carry_code()) : 0);
    o.i32(11, c ? E.carry_type() : 0);
    o.i32(12, c ? E.carry_np() : 0);
    o.i32(13, c ? E.carry_nk() : 0);
    o.i32(14, E.ll(L_PREADY));
    o.i32(15, E.m_busy(0)); o.i32(16, E.m_busy(1));
    o.i32(17, E.ll(L_M0R)); o.i32(18, E.ll(L_M1R));
    o.i32(19, E.ll(L_STORAGE));
    // machines (MachineAgent.py:62-70) and packaging (PackagingAgent.py:54-62)
    o.i8(0, E.m_busy(0)); o.i8(1, obs_i8_checked(E, E.ll(L_M0Q)));
    o.i8(2, E.m_busy(1)); o.i8(3, obs_i8_checked(E, E.ll(L_M1Q)));
    o.f32(0, E.m_prog(0) ? 1.0f : 0.0f);
    o.f32(1, E.m_prog(1) ? 1.0f : 0.0f);
#pragma unroll
    for (int s = 0; s < 4; s++) {
        o.i8(4 + 2 * s, E.p_busy(s));
        o.i8(5 + 2 * s, obs_i8_checked(E, E.p_queued(s)));
        o.f32(2 + s, pack_progress(C, E.p_startn(s)));
    }
    compute_masks(E, C, o);
}

// ---------------------------------------------------------------- heuristic policy
// MultiAgentA2C._get_heuristic_actions (a2c.py:390-537) on the packed state.  The reference
// compares the AGV position with (2,3) small, (0,3) big, (0,0) pickup, (3,5) packaging and
// (1,5) for storage; (1,5) is no location (STORAGE is (3,0), constants.py:9), so the
// "at storage" tests are constant false, exactly as in the reference.  The AGV is never
// mid-move at a step boundary (is_moving branch).
FJSP_DEV int machine_available(const Env& E, int m) {   // not busy and len(tray_queue) < 3
    return !E.m_busy(m) && E.ll(m == 0 ? L_M0Q : L_M1Q) < 3;
}
FJSP_DEV void heuristic_actions(const Env& E, const Tables& T, int* act) {
    const int has_orders = E.next_order() < E.norders() || E.cur_order() >= 0;
    act[0] = has_orders ? 1 : 0;
    const int loc = E.loc();
    int a = 0;
    if (E.carry() != NIL) {
        if (E.carry_np()) {
            const int ty = E.carry_type();
            const int m = (ty == 1 || ty == 2) ? 0 : 1;   // SMALL / MEDIUM -> small machine
            if (machine_available(E, m)) a = loc == (m == 0 ? LOC_SMALL : LOC_BIG) ? 7 : (m == 0 ? 2 : 3);
            else a = 4;                                    // "at storage" is never true
        } else if (E.carry_nk()) {
            a = loc == LOC_PACK ? 7 : 5;
        }
    } else if (E.ll(L_M0R) > 0) {
        a = loc == LOC_SMALL ? 6 : 2;
    } else if (E.ll(L_M1R) > 0) {
        a = loc == LOC_BIG ? 6 : 3;
    } else if (E.ll(L_STORAGE) > 0) {
        // for storage_tray in storage.trays: first tray needing processing whose machine is
        // available -> MOVE_TO_STORAGE (PICKUP needs the impossible (1,5)); else check pickup
        int found = 0;
        int s = E.lh(L_STORAGE);
        for (int i = E.ll(L_STORAGE); i > 0 && !found; i--) {
            const int c = T.scode[s * T.stride];
            const uint32_t w = T.orders[tc_order(c) * T.stride], rg = tc_range(c);
            if ((w & rg) != rg) {
                const int ty = ow_type(w);
                found = machine_available(E, (ty == 1 || ty == 2) ? 0 : 1);
            }
            s = T.snext[s * T.stride];
        }
        a = found ? 4 : (E.ll(L_PREADY) > 0 ? (loc == LOC_PICKUP ? 6 : 1) : 0);
    } else if (E.ll(L_PREADY) > 0) {
        a = loc == LOC_PICKUP ? 6 : 1;
    } else if (E.m_busy(0) || E.m_cur(0) != NIL) {
        a = loc == LOC_SMALL ? 0 : 2;
    } else if (E.m_busy(1) || E.m_cur(1) != NIL) {
        a = loc == LOC_BIG ? 0 : 3;
    } else if (has_orders) {
        a = loc == LOC_PICKUP ? 0 : 1;
    }
    act[1] = a;
#pragma unroll
    for (int m = 0; m < 2; m++) {
        const int idle = !E.m_busy(m);
        act[2 + m] = (E.ll(m == 0 ? L_M0Q : L_M1Q) > 0 && idle) ? 1 : (E.m_cur(m) != NIL && idle) ? 2 : 0;
    }
#pragma unroll
    for (int s = 0; s < 4; s++) act[4 + s] = (E.p_queued(s) > 0 && !E.p_busy(s)) ? 1 : 0;
}

// ---------------------------------------------------------------- reset
// Fresh episode state (FJSPSimulation.reset: new agents, storage, tray pool); the MT cursor
// (W3) is kept.
FJSP_DEV void env_clear(Env& E, const Cfg& C) {
    const uint32_t mt = E.w[3];
#pragma unroll
    for (int i = 0; i < NSTATE; i++) E.w[i] = 0;
    E.w[3] = mt;
    E.w[4] = 0xFFu;                                            // cur_order = none
    E.w[5] = (uint32_t)C.pool0 << 8;                           // tray pool, slot_next = 0
    E.w[6] = (uint32_t)LOC_PICKUP | ((uint32_t)NIL << 3);      // AGV at pickup, carrying nothing
#pragma unroll
    for (int l = 0; l < NLIST; l++) E.w[7 + l] = (uint32_t)NIL | ((uint32_t)NIL << 8);
#pragma unroll
    for (int m = 0; m < 2; m++) E.w[17 + m] = (uint32_t)NIL << 1;
#pragma unroll
    for (int s = 0; s < 4; s++) E.w[20 + s] = (uint32_t)NIL << 2;
}

// ---------------------------------------------------------------- one step
// calculate_local_reward (utils/RewardModel.py:46-97) as one table lookup (build_reward_lut).
FJSP_DEV uint32_t reward_index(int a, uint32_t r, int act) {
    const uint32_t a0 = act == 0;   // actions.get(agent_id, 0) == 0 (absent agents have r == 0)
    const uint32_t f = (r >> 1) & 7u;
    return a == 0 ? (f | (a0 << 3)) : a == 1 ? 16u + ((r >> 1) & 31u) : (a <= 3 ? 48u : 64u) + (f | (a0 << 3));
}
FJSP_DEV double local_reward(const Cfg& C, int a, uint32_t r, int act) { return C.lut[reward_index(a, r, act)]; }

// The int8 observation fields (queue lengths) overflow exactly when observe() would flag it;
// lets a step that does not build the observation itself keep the sticky status bit.
FJSP_DEV void flag_obs_overflow(Env& E) {
    const bool ov = E.ll(L_M0Q) > 127 || E.ll(L_M1Q) > 127 || E.p_queued(0) > 127 || E.p_queued(1) > 127 ||
                    E.p_queued(2) > 127 || E.p_queued(3) > 127;
    if (ov) E.flag(ST_OBS_OVERFLOW | ST_DIVERGED);
}

// calculate_global_reward (utils/RewardModel.py:34-44) / len(self.agents), Python op order.
FJSP_DEV double global_reward8(const Cfg& C, int orders_done, int packaged) {
    double g = C.lut[80] * (double)orders_done;
    g += C.lut[81] * (double)packaged;
    g += C.lut[82];
    return g / 8.0;
}

// Actions in dict order, then env.run in closed form.  actions[a] for agent a (canonical order);
// order = execution order (CANON -> 0..7).  Fills res[8]; returns the shared global reward / 8.
struct NoMid {
    FJSP_DEV void operator()(const Env&, int) const {}
};
// mid(E, move_to) runs right after the machines' actions (the pipelined kernel hands the
// pickup / AGV state to other waves there).  ahead: the pickup station and the AGV already
// acted (on those waves, from the previous step's hand-off); res[0], res[1] hold their results,
// the caller applied their state words and ahead_move is the AGV's move target.
template <bool CANON, class Mid = NoMid>
FJSP_DEV double env_advance(Env& E, const Tables& T, const Cfg& C, const int* act, const uint8_t* order,
                            uint32_t* res, Mid mid = Mid(), bool ahead = false, int ahead_move = 0) {
    int move_to = ahead ? ahead_move : 0, m_start[2] = {-1, -1}, p_started[4] = {0, 0, 0, 0};
    const int products_before = E.total_packaged();
    // 1. actions in dict order (FJSPSimulation.py:172-174)
#pragma unroll
    for (int i = 0; i < NA; i++) {
        const int a = CANON ? i : (int)order[i];
        const int ac = act[a];
        uint32_t r = 0;
        if (ac != 255) {
            switch (a) {
            case 0: r = ahead ? res[0] : pickup_execute(E, T, C, ac); break;
            case 1: r = ahead ? res[1] : agv_execute(E, T, C, ac, &move_to); break;
            case 2: r = machine_execute<0>(E, T, ac, &m_start[0]); break;
            case 3: r = machine_execute<1>(E, T, ac, &m_start[1]); break;
            case 4: r = pack_execute<0>(E, ac, &p_started[0]); break;
            case 5: r = pack_execute<1>(E, ac, &p_started[1]); break;
            case 6: r = pack_execute<2>(E, ac, &p_started[2]); break;
            default: r = pack_execute<3>(E, ac, &p_started[3]); break;
            }
        }
        res[a] = r;
        if (CANON) FJSP_STAMP_AGENT(E, i);
        if (CANON && i == 3) mid(E, move_to);
    }
    FJSP_STAMP(E, 1);
    // 2. env.run(until=now+step_size) in closed form
    if (move_to) E.set_loc(move_to);
    machines_run(E, T, C, m_start[0], m_start[1]);
    int orders_done = 0;
    const int step = E.step();
    const bool due0 = pack_due<0>(E, T, step), due1 = pack_due<1>(E, T, step);
    const bool due2 = pack_due<2>(E, T, step), due3 = pack_due<3>(E, T, step);
    pack_run<0>(E, T, C, p_started[0], due0, &orders_done);
    pack_run<1>(E, T, C, p_started[1], due1, &orders_done);
    pack_run<2>(E, T, C, p_started[2], due2, &orders_done);
    pack_run<3>(E, T, C, p_started[3], due3, &orders_done);
    E.set_ncompleted(E.ncompleted() + orders_done);
    FJSP_STAMP(E, 2);
    // 3. calculate_global_reward; combine_rewards divides it by len(self.agents)
    return global_reward8(C, orders_done, E.total_packaged() - products_before);
}

// One step with rewards (host harness / tests): r_a = g / 8 + local_a (combine_rewards).
template <bool CANON>
FJSP_DEV void env_step(Env& E, const Tables& T, const Cfg& C, const int* act, const uint8_t* order, uint32_t* res,
                       double* rew) {
    const double g8 = env_advance<CANON>(E, T, C, act, order, res);
#pragma unroll
    for (int a = 0; a < NA; a++) rew[a] = g8 + local_reward(C, a, res[a], act[a]);
}

}  // namespace fjsp
