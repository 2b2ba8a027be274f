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

#ifndef FJSP_DEV
#define FJSP_DEV __device__ __forceinline__
#endif

namespace fjsp {

constexpr int NA = 8;
constexpr int NI32 = 20, NI8 = 12, NF32 = 6, NMASK = 29;
constexpr int MAX_ORDERS = 64;
constexpr int MAX_SLOTS = 255;   // slot index 255 = NIL
constexpr int NIL = 255;

// lists in the slot arena
enum : int { L_PREADY = 0, L_STORAGE = 1, L_M0Q = 2, L_M0R = 3, L_M1Q = 4, L_M1R = 5, L_PKG = 6, NLIST = 10 };

// locations (enums/LocationType.py values) and coordinates (constants.py:5-11)
enum : int { LOC_PICKUP = 1, LOC_BIG = 2, LOC_SMALL = 3, LOC_STORAGE = 4, LOC_PACK = 5 };
FJSP_DEV int loc_row(int l) { return (l == LOC_SMALL) ? 2 : (l >= LOC_STORAGE ? 3 : 0); }
FJSP_DEV int loc_col(int l) { return (l == LOC_PICKUP || l == LOC_STORAGE) ? 0 : (l == LOC_PACK ? 5 : 3); }
// AGV move action a (1..5) -> location (AGVAgent.py:218-224)
FJSP_DEV int move_loc(int a) {
    return a == 1 ? LOC_PICKUP : a == 2 ? LOC_SMALL : a == 3 ? LOC_BIG : a == 4 ? LOC_STORAGE : LOC_PACK;
}
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

struct Cfg {
    int step_size, max_steps, tray_cap, mask_tray_cap, storage_cap, pool0, pkg_cap;
    int ptk_small, ptk_big, ptk_pack;   // processing times in steps
    double w[NW];
};

// status bits (include/fjsp.h)
constexpr uint32_t ST_DIVERGED = 0x1u, ST_OBS_OVERFLOW = 0x2u, ST_PKG_WAIT = 0x4u, ST_TRAY_LOST = 0x8u,
                   ST_PROD_LOST = 0x10u, ST_OVERWRITE = 0x20u, ST_SLOT_OVERFLOW = 0x40u;

// Number of packed u32 words of Env in the SoA state buffer.
constexpr int NWORDS = 40;

// Per-env register state.  Field names follow the reference objects.
struct Env {
    int step, norders, next_order, ncompleted, total_packaged, mti;
    uint32_t status;
    // pickup station (PickupStationAgent.py:88-94)
    int cur_order, cur_idx, cur_n, cur_type, cur_color;
    int tray_valid, tray_order, tray_start, tray_count, pool, slot_next;
    // AGV (AGVAgent.py:41-45): location, carried tray slot (NIL = none) and cached tray facts
    int loc, carry, carry_code, carry_type, carry_color, carry_np, carry_nk;
    // FIFO lists in the slot arena
    int lh[NLIST], lt[NLIST], ll[NLIST];
    // machines (MachineAgent.py:40-47): current tray slot/code, busy, progress(0/1),
    // products processed so far, step of the next product completion
    int m_busy[2], m_cur[2], m_code[2], m_prog[2], m_k[2], m_next[2];
    // packaging (PackagingAgent.py:250-256): qfirst = first queued (not yet granted) run
    int p_busy[4], p_hascur[4], p_completed[4], p_qfirst[4], p_inflight[4], p_queued[4];
    float p_prog[4];
};

// ---- table accessors: element i of a per-env table = base[i * stride]
struct Tables {
    uint32_t* orders;   // [MAX_ORDERS]
    uint16_t* scode;    // [MAX_SLOTS] tray code
    uint8_t* snext;     // [MAX_SLOTS] next slot in its list
    uint16_t* scstep;   // [MAX_SLOTS] step at which an in-flight packaging run completes
    int stride;
};

FJSP_DEV void list_push(Env& E, const Tables& T, int L, int s) {
    T.snext[s * T.stride] = (uint8_t)NIL;
    if (E.ll[L] == 0) E.lh[L] = s;
    else T.snext[E.lt[L] * T.stride] = (uint8_t)s;
    E.lt[L] = s;
    E.ll[L] += 1;
}
FJSP_DEV int list_pop(Env& E, const Tables& T, int L) {
    int s = E.lh[L];
    E.lh[L] = T.snext[s * T.stride];
    E.ll[L] -= 1;
    if (E.ll[L] == 0) { E.lh[L] = NIL; E.lt[L] = NIL; }
    return s;
}
// new tray slot holding `code` (bump allocator, reset per episode)
FJSP_DEV int slot_new(Env& E, const Tables& T, int code) {
    if (E.slot_next >= MAX_SLOTS) { E.status |= ST_SLOT_OVERFLOW | ST_DIVERGED; return -1; }
    int s = E.slot_next++;
    T.scode[s * T.stride] = (uint16_t)code;
    return s;
}

// ---- reward / result bit layout (oracle/fjsp_oracle.c, RESULT_KEYS in gen_golden.py)
constexpr uint32_t R_EXEC = 0x80u;

// PickupStationAgent.execute_action (PickupStationAgent.py:190-276)
FJSP_DEV uint32_t pickup_execute(Env& E, const Tables& T, const Cfg& C, int action) {
    uint32_t r = R_EXEC;   // 1 success, 2 product_loaded, 4 tray_completed, 8 idle_with_orders
    auto push_tray = [&]() {
        int s = slot_new(E, T, tc_make(E.tray_order, E.tray_start, E.tray_count));
        if (s >= 0) list_push(E, T, L_PREADY, s);
        E.tray_valid = 0;
    };
    if (action == 0) {
        if (E.next_order < E.norders || E.cur_order >= 0) r |= 8u;
        r |= 1u;
    } else if (action == 1) {
        if (E.cur_order < 0) {
            if (E.next_order < E.norders) {
                E.cur_order = E.next_order++;
                E.cur_idx = 0;
                uint32_t w = T.orders[E.cur_order * T.stride];
                E.cur_n = ow_n(w); E.cur_type = ow_type(w); E.cur_color = ow_color(w);
            } else {
                return r;
            }
        }
        if (!E.tray_valid) {
            if (E.pool > 0) {
                E.pool -= 1;
                E.tray_valid = 1; E.tray_order = E.cur_order; E.tray_start = E.cur_idx; E.tray_count = 0;
            } else {
                return r;
            }
        }
        if (E.tray_count < C.tray_cap) {
            if (E.cur_order != E.tray_order) {   // :231-235 (unreachable with the reference's flow)
                push_tray();
                return r | 4u;
            }
            E.tray_count += 1;
            E.cur_idx += 1;
            r |= 2u | 1u;
            if (E.cur_idx >= E.cur_n) {
                E.cur_order = -1; E.cur_idx = 0;
                push_tray();
                return r | 4u;
            }
            if (E.tray_count >= C.tray_cap) {
                push_tray();
                return r | 4u;
            }
        } else {
            push_tray();
            return r | 4u;
        }
    } else if (action == 2) {
        if (E.tray_valid && E.tray_count > 0) {
            push_tray();
            r |= 1u;
        }
    }
    return r;
}

// FJSPSimulation.add_tray_to_packaging (FJSPSimulation.py:402-430): first station (dict order
// blue_1, blue_2, red, green) whose colour matches and whose Resource has capacity.
FJSP_DEV void add_tray_to_packaging(Env& E, const Tables& T, const Cfg& C, int s, int code) {
    const int color = E.carry_color;
    // PackagingColor RED=1 BLUE=2 GREEN=3; stations 0,1 blue, 2 red, 3 green
    int st = -1;
    if (color == 2) {
        if (E.p_inflight[0] < C.pkg_cap) st = 0;
        else if (E.p_inflight[1] < C.pkg_cap) st = 1;
    } else if (color == 1) {
        if (E.p_inflight[2] < C.pkg_cap) st = 2;
    } else if (color == 3) {
        if (E.p_inflight[3] < C.pkg_cap) st = 3;
    }
    int n = tc_count(code);
    switch (st) {   // constant list indices keep the list registers out of scratch
    case 0: list_push(E, T, L_PKG + 0, s); if (E.p_qfirst[0] == NIL) E.p_qfirst[0] = s; E.p_queued[0] += n; break;
    case 1: list_push(E, T, L_PKG + 1, s); if (E.p_qfirst[1] == NIL) E.p_qfirst[1] = s; E.p_queued[1] += n; break;
    case 2: list_push(E, T, L_PKG + 2, s); if (E.p_qfirst[2] == NIL) E.p_qfirst[2] = s; E.p_queued[2] += n; break;
    case 3: list_push(E, T, L_PKG + 3, s); if (E.p_qfirst[3] == NIL) E.p_qfirst[3] = s; E.p_queued[3] += n; break;
    default: E.status |= ST_PROD_LOST; break;
    }
}

// AGVAgent.execute_action / _execute_pickup / _execute_drop (AGVAgent.py:180-368).
// Returns the result word; *move_to receives the target location of a spawned move.
FJSP_DEV uint32_t agv_execute(Env& E, const Tables& T, const Cfg& C, int action, int* move_to) {
    uint32_t r = R_EXEC;   // 1 success, 2 invalid, 4 moved, 8 pickup, 16 drop, 32 to packaging; 16.. distance
    if (action == 0) return r | 1u;
    if (action >= 1 && action <= 5) {
        int l = move_loc(action);
        int d = manhattan(E.loc, l);
        if (d == 0) return r | 1u;
        *move_to = l;
        return r | 1u | 4u | ((uint32_t)d << 16);
    }
    if (action == 6) {
        if (E.carry != NIL) return r | 2u;
        int s = -1;
        switch (E.loc) {
        case LOC_PICKUP: if (E.ll[L_PREADY]) s = list_pop(E, T, L_PREADY); break;
        case LOC_SMALL: if (E.ll[L_M0R]) s = list_pop(E, T, L_M0R); break;
        case LOC_BIG: if (E.ll[L_M1R]) s = list_pop(E, T, L_M1R); break;
        case LOC_STORAGE: if (E.ll[L_STORAGE]) s = list_pop(E, T, L_STORAGE); break;
        default: return r | 2u;   // PACKAGING
        }
        if (s < 0) return r | 2u;
        int code = T.scode[s * T.stride];
        E.carry = s; E.carry_code = code;
        int n = tc_count(code);
        if (n > 0) {
            uint32_t w = T.orders[tc_order(code) * T.stride];
            uint32_t rg = tc_range(code);
            E.carry_type = ow_type(w);
            E.carry_color = ow_color(w);
            E.carry_np = (w & rg) != rg;
            E.carry_nk = ((w >> 9) & rg) != rg;
        } else {
            E.carry_type = 0; E.carry_color = 0; E.carry_np = 0; E.carry_nk = 0;
        }
        return r | 1u | 8u;
    }
    if (action == 7) {
        if (E.carry == NIL) return r | 2u;
        int s = E.carry, code = E.carry_code, ty = E.carry_type;
        switch (E.loc) {
        case LOC_PICKUP:
            if (tc_count(code) != 0) return r | 2u;
            E.pool += 1;    // add_empty_tray
            break;
        case LOC_SMALL:
            if (!(E.carry_np && (ty == 1 || ty == 2))) return r | 2u;
            list_push(E, T, L_M0Q, s);
            break;
        case LOC_BIG:
            if (!(E.carry_np && (ty == 3 || ty == 2))) return r | 2u;
            list_push(E, T, L_M1Q, s);
            break;
        case LOC_STORAGE:
            if (E.ll[L_STORAGE] < C.storage_cap) list_push(E, T, L_STORAGE, s);
            else E.status |= ST_TRAY_LOST;
            break;
        default:   // PACKAGING
            if (!(E.carry_nk && !E.carry_np)) return r | 2u;
            add_tray_to_packaging(E, T, C, s, code);
            r |= 32u;
            break;
        }
        E.carry = NIL;
        return r | 1u | 16u;
    }
    return r | 2u;
}

// MachineAgent.execute_action (MachineAgent.py:99-139); grant happens in the run.
template <int M>
FJSP_DEV uint32_t machine_execute(Env& E, const Tables& T, int action, int* start_slot) {
    constexpr int LQ = M == 0 ? L_M0Q : L_M1Q;
    constexpr int LR = M == 0 ? L_M0R : L_M1R;
    uint32_t r = R_EXEC;   // 1 success, 2 started, 4 completed, 8 idle_with_queue
    if (action == 0) {
        if (E.ll[LQ] > 0 && !E.m_busy[M]) r |= 8u;
        r |= 1u;
    } else if (action == 1) {
        if (E.ll[LQ] > 0 && !E.m_busy[M]) {
            *start_slot = list_pop(E, T, LQ);
            r |= 2u | 1u;
        }
    } else if (action == 2) {
        if (!E.m_busy[M] && E.m_cur[M] != NIL) {
            list_push(E, T, LR, E.m_cur[M]);
            E.m_cur[M] = NIL;
            r |= 4u | 1u;
        }
    }
    return r;
}

// PackagingAgent.execute_action (PackagingAgent.py:301-335)
template <int S>
FJSP_DEV uint32_t pack_execute(Env& E, int action, int* started) {
    uint32_t r = R_EXEC;   // 1 success, 2 started, 4 completed, 8 idle_with_queue; 16.. completed count
    if (action == 0) {
        if (E.p_queued[S] > 0 && !E.p_busy[S]) r |= 8u;
        r |= 1u;
    } else if (action == 1) {
        int n = E.p_queued[S];
        if (n > 0) {
            *started = 1;
            // self.processing_progress = (i / len(self.product_queue)) * 100 with i == 1
            E.p_prog[S] = (float)((1.0 / (double)n) * 100.0);
            r |= 2u | 1u;
        }
    } else if (action == 2) {
        if (!E.p_busy[S] && E.p_hascur[S]) r |= 4u | ((uint32_t)(E.p_completed[S] & 0xFFFF) << 16);
    }
    return r;
}

// ---------------------------------------------------------------- run phase (T, T+step]
// Machine: completion due this step (old NORMAL event) else grant of a START.
template <int M>
FJSP_DEV void machine_run(Env& E, const Tables& T, const Cfg& C, int start_slot) {
    const int ptk = M == 0 ? C.ptk_small : C.ptk_big;
    if (E.m_busy[M] && E.m_next[M] == E.step) {
        int code = E.m_code[M];
        int o = tc_order(code);
        uint32_t bit = 1u << (tc_start(code) + E.m_k[M]);
        T.orders[o * T.stride] |= bit;          // product.is_processed = True
        E.m_k[M] += 1;
        if (E.m_k[M] >= tc_count(code)) { E.m_busy[M] = 0; E.m_prog[M] = 1; }
        else E.m_next[M] = E.step + ptk;
    }
    if (start_slot >= 0) {   // grant at T: is_busy, current_tray := tray (MachineAgent.py:159-160)
        if (E.m_cur[M] != NIL) E.status |= ST_OVERWRITE;
        int code = T.scode[start_slot * T.stride];
        E.m_cur[M] = start_slot; E.m_code[M] = code; E.m_k[M] = 0;
        if (tc_count(code) > 0) { E.m_busy[M] = 1; E.m_next[M] = E.step + ptk; }
        else { E.m_busy[M] = 0; E.m_prog[M] = 1; }   // empty tray: loop body never runs
    }
}

// Packaging: completions of the batch due this step, then grants of this step's START.
template <int S>
FJSP_DEV void pack_run(Env& E, const Tables& T, const Cfg& C, int started, int* orders_done) {
    constexpr int L = L_PKG + S;
    if (started && E.p_inflight[S] + E.p_queued[S] > C.pkg_cap)
        E.status |= ST_PKG_WAIT | ST_DIVERGED;   // Request would wait (users == capacity)
    // completions (PackagingAgent.py:143-147)
    int done = 0;
    while (E.ll[L] > 0 && E.lh[L] != E.p_qfirst[S] && T.scstep[E.lh[L] * T.stride] == (uint16_t)E.step) {
        int s = list_pop(E, T, L);
        int code = T.scode[s * T.stride];
        int o = tc_order(code);
        uint32_t w = T.orders[o * T.stride] | (tc_range(code) << 9);
        uint32_t full = (1u << ow_n(w)) - 1u;
        if (!(w & (1u << 18)) && ((w >> 9) & full) == full) {   // _check_order_completions
            w |= 1u << 18;
            *orders_done += 1;
        }
        T.orders[o * T.stride] = w;
        done += tc_count(code);
    }
    if (done) {
        E.p_completed[S] += done; E.total_packaged += done; E.p_inflight[S] -= done; E.p_busy[S] = 0;
    }
    // grants: every queued product, in queue order (PackagingAgent.py:136-141)
    if (started) {
        uint16_t cs = (uint16_t)(E.step + C.ptk_pack);
        for (int s = E.p_qfirst[S]; s != NIL; s = T.snext[s * T.stride]) T.scstep[s * T.stride] = cs;
        E.p_qfirst[S] = NIL;
        E.p_inflight[S] += E.p_queued[S];
        E.p_queued[S] = 0;
        E.p_busy[S] = 1;
        E.p_hascur[S] = 1;
    }
}

// ---------------------------------------------------------------- observations
struct Obs {
    int32_t i32[NI32];
    int8_t i8[NI8];
    float f32[NF32];
    int8_t mask[NMASK];
};

FJSP_DEV void compute_masks(const Env& E, const Cfg& C, int8_t* m) {
    // pickup (PickupStationAgent.py:144-186)
    int has_order = E.cur_order >= 0 || E.next_order < E.norders;
    int has_tray = E.tray_valid || E.pool > 0;
    int not_full = E.tray_valid ? (E.tray_count < C.mask_tray_cap) : 1;
    int prem = E.cur_order >= 0 ? (E.cur_idx < E.cur_n) : (E.next_order < E.norders);
    m[0] = 1;
    m[1] = (int8_t)(has_order && has_tray && not_full && prem);
    m[2] = (int8_t)(E.tray_valid && E.tray_count > 0);
    // AGV (AGVAgent.py:79-178); the AGV is never mid-move at a step boundary
    m[3] = 1;
    m[4] = E.loc != LOC_PICKUP;
    m[5] = E.loc != LOC_SMALL;
    m[6] = E.loc != LOC_BIG;
    m[7] = E.loc != LOC_STORAGE;
    m[8] = E.loc != LOC_PACK;
    int pick = 0, drop = 0;
    if (E.carry == NIL) {
        pick = (E.loc == LOC_PICKUP && E.ll[L_PREADY] > 0) || (E.loc == LOC_SMALL && E.ll[L_M0R] > 0) ||
               (E.loc == LOC_BIG && E.ll[L_M1R] > 0) || (E.loc == LOC_STORAGE && E.ll[L_STORAGE] > 0);
    } else {
        int ty = E.carry_type;
        drop = (E.loc == LOC_PICKUP && tc_count(E.carry_code) == 0) ||
               (E.loc == LOC_SMALL && E.carry_np && (ty == 1 || ty == 2)) ||
               (E.loc == LOC_BIG && E.carry_np && (ty == 3 || ty == 2)) ||
               (E.loc == LOC_PACK && E.carry_nk && !E.carry_np) || (E.loc == LOC_STORAGE);
    }
    m[9] = (int8_t)pick;
    m[10] = (int8_t)drop;
    // machines (MachineAgent.py:72-97)
    m[11] = 1; m[12] = E.ll[L_M0Q] > 0 && !E.m_busy[0]; m[13] = !E.m_busy[0] && E.m_cur[0] != NIL;
    m[14] = 1; m[15] = E.ll[L_M1Q] > 0 && !E.m_busy[1]; m[16] = !E.m_busy[1] && E.m_cur[1] != NIL;
    // packaging (PackagingAgent.py:64-89)
#pragma unroll
    for (int s = 0; s < 4; s++) {
        m[17 + 3 * s] = 1;
        m[18 + 3 * s] = E.p_queued[s] > 0 && !E.p_busy[s] && E.p_inflight[s] < C.pkg_cap;
        m[19 + 3 * s] = !E.p_busy[s] && E.p_hascur[s];
    }
}

FJSP_DEV int8_t to_i8(Env& E, int v) {
    if (v > 127) E.status |= ST_OBS_OVERFLOW | ST_DIVERGED;
    return (int8_t)v;
}

FJSP_DEV void observe(Env& E, const Cfg& C, Obs& o) {
    // pickup (PickupStationAgent.py:102-142)
    int osz = 0, rem = 0, npt = 0, npc = 0;
    if (E.cur_order >= 0) {
        osz = E.cur_n; rem = E.cur_n - E.cur_idx;
        if (rem > 0) { npt = E.cur_type; npc = E.cur_color; }
    }
    int tt = 0, tcol = 0, tcnt = 0;
    if (E.tray_valid) {
        tcnt = E.tray_count;
        if (tcnt > 0 && E.tray_order == E.cur_order) {   // a loaded tray always belongs to the current order
            tt = E.cur_type; tcol = E.cur_color;
        }
    }
    o.i32[0] = osz; o.i32[1] = rem; o.i32[2] = npt; o.i32[3] = npc;
    o.i32[4] = tt; o.i32[5] = tcol; o.i32[6] = tcnt;
    // AGV (AGVAgent.py:53-76)
    int c = E.carry != NIL;
    o.i32[7] = loc_row(E.loc); o.i32[8] = loc_col(E.loc);
    o.i32[9] = c;
    o.i32[10] = c ? tc_count(E.carry_code) : 0;
    o.i32[11] = c ? E.carry_type : 0;
    o.i32[12] = c ? E.carry_np : 0;
    o.i32[13] = c ? E.carry_nk : 0;
    o.i32[14] = E.ll[L_PREADY];
    o.i32[15] = E.m_busy[0]; o.i32[16] = E.m_busy[1];
    o.i32[17] = E.ll[L_M0R]; o.i32[18] = E.ll[L_M1R];
    o.i32[19] = E.ll[L_STORAGE];
    // machines (MachineAgent.py:62-70) and packaging (PackagingAgent.py:54-62)
    o.i8[0] = (int8_t)E.m_busy[0]; o.i8[1] = to_i8(E, E.ll[L_M0Q]);
    o.i8[2] = (int8_t)E.m_busy[1]; o.i8[3] = to_i8(E, E.ll[L_M1Q]);
    o.f32[0] = E.m_prog[0] ? 1.0f : 0.0f;
    o.f32[1] = E.m_prog[1] ? 1.0f : 0.0f;
#pragma unroll
    for (int s = 0; s < 4; s++) {
        o.i8[4 + 2 * s] = (int8_t)E.p_busy[s];
        o.i8[5 + 2 * s] = to_i8(E, E.p_queued[s]);
        o.f32[2 + s] = E.p_prog[s];
    }
    compute_masks(E, C, o.mask);
}

// ---------------------------------------------------------------- reset
FJSP_DEV void env_clear(Env& E, const Cfg& C) {
    E.step = 0; E.next_order = 0; E.ncompleted = 0; E.total_packaged = 0; E.status = 0;
    E.cur_order = -1; E.cur_idx = 0; E.cur_n = 0; E.cur_type = 0; E.cur_color = 0;
    E.tray_valid = 0; E.tray_order = 0; E.tray_start = 0; E.tray_count = 0;
    E.pool = C.pool0; E.slot_next = 0;
    E.loc = LOC_PICKUP; E.carry = NIL; E.carry_code = 0; E.carry_type = 0; E.carry_color = 0; E.carry_np = 0; E.carry_nk = 0;
#pragma unroll
    for (int l = 0; l < NLIST; l++) { E.lh[l] = NIL; E.lt[l] = NIL; E.ll[l] = 0; }
#pragma unroll
    for (int m = 0; m < 2; m++) { E.m_busy[m] = 0; E.m_cur[m] = NIL; E.m_code[m] = 0; E.m_prog[m] = 0; E.m_k[m] = 0; E.m_next[m] = 0; }
#pragma unroll
    for (int s = 0; s < 4; s++) {
        E.p_busy[s] = 0; E.p_hascur[s] = 0; E.p_completed[s] = 0; E.p_qfirst[s] = NIL;
        E.p_inflight[s] = 0; E.p_queued[s] = 0; E.p_prog[s] = 0.0f;
    }
}

// ---------------------------------------------------------------- one step
// actions[a] for agent a in canonical order; order = execution order (CANON -> 0..7).
// Returns the number of orders completed this step; fills res[8] and rewards[8].
template <bool CANON>
FJSP_DEV void env_step(Env& E, const Tables& T, const Cfg& C, const int* act, const uint8_t* order,
                       uint32_t* res, double* rew) {
    int move_to = 0, m_start[2] = {-1, -1}, p_started[4] = {0, 0, 0, 0};
    const int products_before = E.total_packaged;
    // 1. actions in dict order (FJSPSimulation.py:172-174)
#pragma unroll
    for (int i = 0; i < NA; i++) {
        const int a = CANON ? i : (int)order[i];
        const int ac = act[a];
        uint32_t r = 0;
        if (ac != 255) {
            switch (a) {
            case 0: r = pickup_execute(E, T, C, ac); break;
            case 1: r = agv_execute(E, T, C, ac, &move_to); break;
            case 2: r = machine_execute<0>(E, T, ac, &m_start[0]); break;
            case 3: r = machine_execute<1>(E, T, ac, &m_start[1]); break;
            case 4: r = pack_execute<0>(E, ac, &p_started[0]); break;
            case 5: r = pack_execute<1>(E, ac, &p_started[1]); break;
            case 6: r = pack_execute<2>(E, ac, &p_started[2]); break;
            default: r = pack_execute<3>(E, ac, &p_started[3]); break;
            }
        }
        res[a] = r;
    }
    // 2. env.run(until=now+step_size) in closed form
    if (move_to) E.loc = move_to;
    machine_run<0>(E, T, C, m_start[0]);
    machine_run<1>(E, T, C, m_start[1]);
    int orders_done = 0;
    pack_run<0>(E, T, C, p_started[0], &orders_done);
    pack_run<1>(E, T, C, p_started[1], &orders_done);
    pack_run<2>(E, T, C, p_started[2], &orders_done);
    pack_run<3>(E, T, C, p_started[3], &orders_done);
    E.ncompleted += orders_done;
    // 3-4. rewards (RewardModel.calculate_global_reward / calculate_local_reward / combine)
    double g = C.w[W_ORDER] * (double)orders_done;
    g += C.w[W_THROUGHPUT] * (double)(E.total_packaged - products_before);
    g += C.w[W_TIME] * (double)C.step_size;
    const double g8 = g / 8.0;   // combine_rewards: global / len(self.agents)
#pragma unroll
    for (int a = 0; a < NA; a++) {
        const uint32_t r = res[a];
        const int a0 = act[a] == 0;   // actions.get(agent_id, 0) == 0 (absent agents: r == 0)
        double loc = 0.0;
        if (a == 0) {
            if (r & 2u) loc += C.w[W_PICK_LOAD];
            if (r & 4u) loc += C.w[W_PICK_TRAY];
            if (a0 && (r & 8u)) loc += C.w[W_PICK_IDLE];
        } else if (a == 1) {
            if (r & 8u) loc += C.w[W_AGV_DELIVERY];
            if (r & 16u) loc += C.w[W_AGV_DELIVERY];
            if (r & 32u) loc += C.w[W_AGV_PACKAGING];
            if (r & 4u) loc += C.w[W_AGV_MOVE];
            if (r & 2u) loc += C.w[W_AGV_INVALID];
        } else if (a <= 3) {
            if (r & 2u) loc += C.w[W_M_START];
            if (r & 4u) loc += C.w[W_M_COMPLETE];
            if (a0 && (r & 8u)) loc += C.w[W_M_IDLE];
        } else {
            if (r & 2u) loc += C.w[W_P_START];
            if (r & 4u) loc += C.w[W_P_COMPLETE];
            if (a0 && (r & 8u)) loc += C.w[W_P_IDLE];
        }
        rew[a] = g8 + loc;
    }
}

}  // namespace fjsp
