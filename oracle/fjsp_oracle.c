/*
 * fjsp_oracle.c — CPU restatement of the reference FJSP simulation. TEST INFRASTRUCTURE.
 *
 * This file is the parity ORACLE.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker / CPU baseline: the product path
 * (multi-agent-rl-for-fjsp_amd/) never links, loads or calls it.
 *
 * It restates, object by object and event by event, the reference's pure-Python
 * simulation (FARIDKH/Multi-agent-RL-for-FJSP @ /root/reference) together with the SimPy-4
 * event-loop semantics it depends on (simpy is a third-party dependency absent from the
 * reference tree; requirements.txt:6 `simpy>=4.0.0`).  It deliberately does NOT use the
 * closed-form per-agent shortcuts of the HIP kernel: it keeps a general (time, priority,
 * eid) event heap, Request/Release resources with put/get queues, processes written as
 * resumable generators, tray objects with product lists, and a literal tray pool, so that
 * parity between it and the kernel is a real cross-check.  It is pinned against golden
 * traces produced by running the reference itself (tests/golden/gen_golden.py).
 *
 * Reference map (file:line in /root/reference):
 *   step ............ FJSPSimulation.py:144-242     reset ........ FJSPSimulation.py:286-323
 *   generate_order .. FJSPSimulation.py:101-131     trays ........ FJSPSimulation.py:89-98
 *   completions ..... FJSPSimulation.py:245-258     pkg routing .. FJSPSimulation.py:402-430
 *   pickup .......... agents/PickupStationAgent.py:102-292
 *   agv ............. agents/AGVAgent.py:53-403
 *   machines ........ agents/MachineAgent.py:62-169 (+Small/BigMachineAgent.py pt 60/120)
 *   packaging ....... agents/PackagingAgent.py:54-153
 *   storage ......... models/Storage.py:16-36      tray props ... models/Tray.py:16-52
 *   rewards ......... utils/RewardModel.py:34-110 (fp64, Python operation order)
 *   GAE / returns ... transition_memory.py:83-105
 *   RNG ............. numpy legacy RandomState: MT19937 init_genrand + masked-rejection
 *                     bounded ints (np.random.seed/randint/choice)
 *   SimPy core ...... Environment.schedule/step/run, Initialize, Timeout, Process._resume,
 *                     Resource/Request/Release
 *
 * Compile with -ffp-contract=off (the reward / GAE arithmetic must match Python's
 * unfused fp64 operation order bit for bit).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

/* fp contraction is disabled by the build flags (-ffp-contract=off) */

/* ---------------------------------------------------------------- configuration */
enum { C_NUM_TRAYS, C_TRAY_CAP, C_MASK_TRAY_CAP, C_STORAGE_CAP, C_STEP, C_MAX_STEPS,
       C_AGV_SPEED, C_PT_SMALL, C_PT_BIG, C_PT_PACK, C_PACK_CAP, C_NCFG };

#define MAX_ORDERS 128
#define MAX_PROD 16           /* products per order: randint(1,10) -> <= 9 */
#define MAX_EVENTS 4096          /* pending heap entries */
#define MAX_EVPOOL 65536         /* events created per episode */
#define MAX_PROCS 16384
#define MAX_TRAYS 4096
#define QCAP 8192

/* status bits (see include/fjsp.h FJSP_STATUS_*) */
#define ST_EXCEPTION    0x1u   /* the reference would raise out of step() */
#define ST_OBS_OVERFLOW 0x2u   /* int8 observation out of range (numpy OverflowError) */
#define ST_PKG_WAIT     0x4u   /* a packaging request had to wait (users == capacity) */
#define ST_TRAY_LOST    0x8u   /* storage full: dropped tray lost (Storage.py:18-22) */
#define ST_PROD_LOST    0x10u  /* no packaging station with capacity (FJSPSimulation.py:426) */
#define ST_OVERWRITE    0x20u  /* machine START overwrote an unsignalled processed tray */
#define ST_ORACLE_LIMIT 0x80000000u

/* ---------------------------------------------------------------- MT19937 (numpy legacy) */
typedef struct { uint32_t mt[624]; int mti; } mt19937;

static void mt_seed(mt19937* s, uint32_t seed) {
    s->mt[0] = seed;
    for (int i = 1; i < 624; i++)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->mti = 624;
}

static uint32_t mt_next(mt19937* s) {
    if (s->mti >= 624) {
        for (int i = 0; i < 624; i++) {
            uint32_t y = (s->mt[i] & 0x80000000u) | (s->mt[(i + 1) % 624] & 0x7fffffffu);
            s->mt[i] = s->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        s->mti = 0;
    }
    uint32_t y = s->mt[s->mti++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

/* numpy random_bounded_uint64_fill, rng <= 0xFFFFFFFF, use_masked=True: one raw 32-bit
 * draw per attempt, rejected while (u & mask) > rng. */
static uint32_t mt_bounded(mt19937* s, uint32_t rng) {
    if (rng == 0) return 0;
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (mt_next(s) & mask)) > rng) {}
    return v;
}

/* ---------------------------------------------------------------- simulation objects */
typedef struct { int n, type, color, complete; double completion_time; } order_t;
typedef struct { int len, order_id, cap; int prod[64]; } tray_t;   /* prod = o*MAX_PROD+k */

typedef struct { int buf[QCAP]; int head, len; } fifo;   /* list used as pop(0)/append */
static void q_clear(fifo* q) { q->head = 0; q->len = 0; }
static int  q_get(fifo* q, int i) { return q->buf[(q->head + i) % QCAP]; }
static int  q_push(fifo* q, int v) { if (q->len >= QCAP) return -1; q->buf[(q->head + q->len) % QCAP] = v; q->len++; return 0; }
static int  q_pop0(fifo* q) { int v = q->buf[q->head]; q->head = (q->head + 1) % QCAP; q->len--; return v; }
/* list.remove(x): first occurrence; returns 0 on success, -1 if absent (ValueError) */
static int q_remove(fifo* q, int v) {
    for (int i = 0; i < q->len; i++) {
        if (q_get(q, i) == v) {
            for (int j = i; j + 1 < q->len; j++)
                q->buf[(q->head + j) % QCAP] = q->buf[(q->head + j + 1) % QCAP];
            q->len--;
            return 0;
        }
    }
    return -1;
}

/* -------- SimPy-4 restatement: events, callbacks, heap, resources, processes */
enum { CB_RESUME = 1, CB_TRIGGER_GET, CB_TRIGGER_PUT, CB_STOP };
enum { EV_PLAIN, EV_TIMEOUT, EV_INIT, EV_PROCESS, EV_REQUEST, EV_RELEASE };

typedef struct { int kind, arg; } cb_t;
typedef struct {
    int kind;
    int triggered, processed, ok, defused;
    int ncb; cb_t cb[4];
    int res;            /* resource index for REQUEST/RELEASE */
    int request;        /* RELEASE: the request event it releases */
    int proc;           /* PROCESS event: its process */
} event_t;

typedef struct { double t; int prio; long eid; int ev; } heap_item;

enum { P_AGV, P_MACHINE, P_PACK };
typedef struct {
    int kind, pc, alive;
    int agent;          /* machine index 0/1 or packaging station 0..3 */
    int tray;           /* machine: the tray being processed */
    int product;        /* packaging: the product */
    int k;              /* machine: product loop index */
    int req;            /* request event */
    int self_ev;        /* the process's own event */
    int tr, tc;         /* AGV target */
} proc_t;

typedef struct { int capacity; fifo users, put_q, get_q; } resource_t;

typedef struct {
    int32_t cfg[C_NCFG];
    mt19937 rng;
    /* SimPy environment */
    double now;
    long next_eid;
    int nheap; heap_item heap[MAX_EVENTS];
    int nevents; event_t ev[MAX_EVPOOL];
    int nprocs; proc_t procs[MAX_PROCS];
    resource_t res[6];      /* 0,1 machines (cap 1); 2..5 packaging (cap 20) */
    int stop_flag;
    /* tracking (FJSPSimulation.py:53-56) */
    int norders; order_t orders[MAX_ORDERS];
    uint8_t processed[MAX_ORDERS * MAX_PROD], packaged[MAX_ORDERS * MAX_PROD];
    int ncompleted, total_packaged, current_step;
    /* trays */
    int ntrays; tray_t trays[MAX_TRAYS];
    /* pickup station (PickupStationAgent.py:88-94) */
    fifo order_queue; int cur_order, cur_idx; fifo trays_at_station; int cur_tray; fifo ps_ready;
    /* AGV (AGVAgent.py:41-45) */
    int pos_r, pos_c, carrying, is_moving;
    /* machines (MachineAgent.py:40-47) */
    struct { fifo queue, ready; int cur_tray, busy; double progress; int pt; } m[2];
    /* packaging (PackagingAgent.py:250-256), order blue_1, blue_2, red, green */
    struct { int color; fifo queue; int cur_product, busy; double progress; int completed; } p[4];
    /* storage (Storage.py:13-15) */
    fifo storage;
    uint32_t status;
    /* scratch for step results */
    uint32_t results[8];
} sim_t;

/* LocationType values / coordinates (constants.py:5-11; enums/LocationType.py) */
enum { LOC_NONE = 0, LOC_PICKUP = 1, LOC_BIG = 2, LOC_SMALL = 3, LOC_STORAGE = 4, LOC_PACK = 5 };
static const int LOC_R[6] = {0, 0, 0, 2, 3, 3};
static const int LOC_C[6] = {0, 0, 3, 3, 0, 5};
/* iteration order of LOCATION_POSITIONS dict: PICKUP, BIG_MACHINE, SMALL_MACHINE, STORAGE, PACKAGING */
static int current_location(const sim_t* s) {
    for (int l = 1; l <= 5; l++) if (s->pos_r == LOC_R[l] && s->pos_c == LOC_C[l]) return l;
    return LOC_NONE;
}
/* AGV move actions 1..5 -> PICKUP, SMALL, BIG, STORAGE, PACKAGING (AGVAgent.py:218-224) */
static const int MOVE_LOC[6] = {0, LOC_PICKUP, LOC_SMALL, LOC_BIG, LOC_STORAGE, LOC_PACK};
/* PackagingColor: RED=1 BLUE=2 GREEN=3; stations blue_1, blue_2, red, green (FJSPSimulation.py:68-73) */
static const int PKG_COLOR[4] = {2, 2, 1, 3};

#define PROD(o, k) ((o) * MAX_PROD + (k))

static void oracle_fail(sim_t* s, uint32_t bit) { s->status |= bit; }

/* ---- tray helpers (models/Tray.py) */
static int tray_needs_processing(const sim_t* s, int t) {
    const tray_t* tr = &s->trays[t];
    for (int i = 0; i < tr->len; i++) if (!s->processed[tr->prod[i]]) return 1;
    return 0;
}
static int tray_needs_packaging(const sim_t* s, int t) {
    const tray_t* tr = &s->trays[t];
    for (int i = 0; i < tr->len; i++) if (!s->packaged[tr->prod[i]]) return 1;
    return 0;
}
static int prod_order(int p) { return p / MAX_PROD; }
/* tray_type as ProductType value of the first product, 0 if empty */
static int tray_type(const sim_t* s, int t) {
    const tray_t* tr = &s->trays[t];
    return tr->len ? s->orders[prod_order(tr->prod[0])].type : 0;
}
static int tray_color(const sim_t* s, int t) {
    const tray_t* tr = &s->trays[t];
    return tr->len ? s->orders[prod_order(tr->prod[0])].color : 0;
}

/* ---- event pool / heap */
static int new_event(sim_t* s, int kind) {
    if (s->nevents >= (int)(sizeof(s->ev) / sizeof(s->ev[0]))) { oracle_fail(s, ST_ORACLE_LIMIT); s->nevents = 0; }
    int e = s->nevents++;
    memset(&s->ev[e], 0, sizeof(event_t));
    s->ev[e].kind = kind;
    return e;
}
static void add_cb(sim_t* s, int e, int kind, int arg) {
    event_t* ev = &s->ev[e];
    if (ev->ncb >= 4) { oracle_fail(s, ST_ORACLE_LIMIT); return; }
    ev->cb[ev->ncb].kind = kind; ev->cb[ev->ncb].arg = arg; ev->ncb++;
}
static int heap_less(const heap_item* a, const heap_item* b) {
    if (a->t != b->t) return a->t < b->t;
    if (a->prio != b->prio) return a->prio < b->prio;
    return a->eid < b->eid;
}
static void schedule(sim_t* s, int e, int prio, double delay) {
    if (s->nheap >= MAX_EVENTS) { oracle_fail(s, ST_ORACLE_LIMIT); return; }
    heap_item it = {s->now + delay, prio, s->next_eid++, e};
    int i = s->nheap++;
    s->heap[i] = it;
    while (i > 0) {
        int p = (i - 1) / 2;
        if (!heap_less(&s->heap[i], &s->heap[p])) break;
        heap_item tmp = s->heap[i]; s->heap[i] = s->heap[p]; s->heap[p] = tmp; i = p;
    }
}
static heap_item heap_pop(sim_t* s) {
    heap_item top = s->heap[0];
    s->heap[0] = s->heap[--s->nheap];
    int i = 0;
    for (;;) {
        int l = 2 * i + 1, r = l + 1, m = i;
        if (l < s->nheap && heap_less(&s->heap[l], &s->heap[m])) m = l;
        if (r < s->nheap && heap_less(&s->heap[r], &s->heap[m])) m = r;
        if (m == i) break;
        heap_item tmp = s->heap[i]; s->heap[i] = s->heap[m]; s->heap[m] = tmp; i = m;
    }
    return top;
}
/* Event.succeed (NORMAL, delay 0) */
static void ev_succeed(sim_t* s, int e) {
    s->ev[e].triggered = 1; s->ev[e].ok = 1;
    schedule(s, e, 1, 0.0);
}

/* ---- resources (Resource/_do_put/_do_get/_trigger_put/_trigger_get) */
static void trigger_put(sim_t* s, int r);
static void trigger_get(sim_t* s, int r);

static void do_put(sim_t* s, int r, int req) {
    resource_t* R = &s->res[r];
    if (R->users.len < R->capacity) {
        q_push(&R->users, req);
        ev_succeed(s, req);
    }
}
static void do_get(sim_t* s, int r, int rel) {
    resource_t* R = &s->res[r];
    q_remove(&R->users, s->ev[rel].request);     /* ValueError swallowed */
    ev_succeed(s, rel);
}
static void trigger_put(sim_t* s, int r) {
    resource_t* R = &s->res[r];
    int idx = 0;
    while (idx < R->put_q.len) {
        int pe = q_get(&R->put_q, idx);
        do_put(s, r, pe);
        if (!s->ev[pe].triggered) idx++;
        else q_remove(&R->put_q, pe);         /* pop(idx) */
        break;                                /* _do_put returns None -> stop */
    }
}
static void trigger_get(sim_t* s, int r) {
    resource_t* R = &s->res[r];
    int idx = 0;
    while (idx < R->get_q.len) {
        int ge = q_get(&R->get_q, idx);
        do_get(s, r, ge);
        if (!s->ev[ge].triggered) idx++;
        else q_remove(&R->get_q, ge);
        break;
    }
}
/* Request(resource): Put.__init__ */
static int make_request(sim_t* s, int r) {
    int e = new_event(s, EV_REQUEST);
    s->ev[e].res = r;
    q_push(&s->res[r].put_q, e);
    add_cb(s, e, CB_TRIGGER_GET, r);
    trigger_put(s, r);
    if (r >= 2 && !s->ev[e].triggered) oracle_fail(s, ST_PKG_WAIT);
    return e;
}
/* Request.__exit__: cancel if untriggered, then Release(resource, request) */
static void request_exit(sim_t* s, int req) {
    int r = s->ev[req].res;
    if (!s->ev[req].triggered) q_remove(&s->res[r].put_q, req);
    int e = new_event(s, EV_RELEASE);
    s->ev[e].res = r; s->ev[e].request = req;
    q_push(&s->res[r].get_q, e);
    add_cb(s, e, CB_TRIGGER_PUT, r);
    trigger_get(s, r);
}

/* ---- processes */
static void proc_resume(sim_t* s, int p, int ev);

static int spawn(sim_t* s, int kind) {
    if (s->nprocs >= MAX_PROCS) { oracle_fail(s, ST_ORACLE_LIMIT); s->nprocs = 0; }
    int p = s->nprocs++;
    memset(&s->procs[p], 0, sizeof(proc_t));
    s->procs[p].kind = kind; s->procs[p].alive = 1;
    s->procs[p].self_ev = new_event(s, EV_PROCESS);
    s->ev[s->procs[p].self_ev].proc = p;
    /* Initialize: URGENT, callbacks=[proc._resume] */
    int init = new_event(s, EV_INIT);
    s->ev[init].triggered = 1; s->ev[init].ok = 1;
    add_cb(s, init, CB_RESUME, p);
    schedule(s, init, 0, 0.0);
    return p;
}
static int make_timeout(sim_t* s, double d) {
    int e = new_event(s, EV_TIMEOUT);
    s->ev[e].triggered = 1; s->ev[e].ok = 1;
    schedule(s, e, 1, d);
    return e;
}
/* process termination: schedule own event ok / failed */
static void proc_end(sim_t* s, int p, int ok) {
    proc_t* P = &s->procs[p];
    P->alive = 0;
    int e = P->self_ev;
    s->ev[e].triggered = 1; s->ev[e].ok = ok;
    schedule(s, e, 1, 0.0);
}

/* Runs the generator body from its program counter until the next yield.  Returns the
 * yielded event, or -1 when the generator finished (ok) / -2 when it raised. */
static int gen_step(sim_t* s, int p) {
    proc_t* P = &s->procs[p];
    switch (P->kind) {
    case P_AGV:   /* AGVAgent._move_process :387-396 */
        if (P->pc == 0) {
            int d = abs(s->pos_r - P->tr) + abs(s->pos_c - P->tc);
            double travel = (double)d / (double)s->cfg[C_AGV_SPEED];
            s->is_moving = 1;
            P->pc = 1;
            return make_timeout(s, travel);
        }
        s->pos_r = P->tr; s->pos_c = P->tc; s->is_moving = 0;
        return -1;
    case P_MACHINE: { /* MachineAgent._simpy_processing_process :151-169 */
        int m = P->agent;
        if (P->pc == 0) {                 /* with resource.request() as req: yield req */
            P->req = make_request(s, m);
            P->pc = 1;
            return P->req;
        }
        if (P->pc == 1) {
            s->m[m].busy = 1;
            s->m[m].cur_tray = P->tray;
            P->k = 0;
            P->pc = 2;
        } else if (P->pc == 2) {          /* resumed after a product timeout */
            s->processed[s->trays[P->tray].prod[P->k]] = 1;
            P->k++;
        }
        if (P->k < s->trays[P->tray].len) {
            return make_timeout(s, (double)s->m[m].pt);
        }
        s->m[m].busy = 0;
        s->m[m].progress = 1.0;
        request_exit(s, P->req);
        return -1;
    }
    case P_PACK: { /* PackagingAgent._simpy_packaging_process :133-147 */
        int st = P->agent;
        if (P->pc == 0) {
            P->req = make_request(s, 2 + st);
            P->pc = 1;
            return P->req;
        }
        if (P->pc == 1) {
            s->p[st].busy = 1;
            s->p[st].cur_product = P->product;
            if (q_remove(&s->p[st].queue, P->product) != 0) {
                /* list.remove -> ValueError inside the with-block: __exit__ releases, the
                 * process fails and env.step() re-raises (reference raises). */
                request_exit(s, P->req);
                oracle_fail(s, ST_EXCEPTION);
                return -2;
            }
            P->pc = 2;
            return make_timeout(s, (double)s->cfg[C_PT_PACK]);
        }
        s->packaged[P->product] = 1;
        s->p[st].completed += 1;
        s->total_packaged += 1;
        s->p[st].busy = 0;
        request_exit(s, P->req);
        return -1;
    }
    }
    return -1;
}

/* Process._resume */
static void proc_resume(sim_t* s, int p, int ev) {
    (void)ev;
    for (;;) {
        int y = gen_step(s, p);
        if (y == -1) { proc_end(s, p, 1); return; }
        if (y == -2) { proc_end(s, p, 0); return; }
        if (!s->ev[y].processed) { add_cb(s, y, CB_RESUME, p); return; }
        /* already processed: continue the loop immediately */
    }
}

/* Environment.step */
static void env_step(sim_t* s) {
    heap_item it = heap_pop(s);
    s->now = it.t;
    event_t* e = &s->ev[it.ev];
    int ncb = e->ncb; cb_t cbs[4];
    memcpy(cbs, e->cb, sizeof(cbs));
    e->processed = 1; e->ncb = 0;
    for (int i = 0; i < ncb; i++) {
        switch (cbs[i].kind) {
        case CB_RESUME: proc_resume(s, cbs[i].arg, it.ev); break;
        case CB_TRIGGER_GET: trigger_get(s, cbs[i].arg); break;
        case CB_TRIGGER_PUT: trigger_put(s, cbs[i].arg); break;
        case CB_STOP: s->stop_flag = 1; return;
        }
    }
    if (!e->ok && !e->defused) oracle_fail(s, ST_EXCEPTION);
}

/* Environment.run(until=now+step) */
static void env_run(sim_t* s, double until) {
    int e = new_event(s, EV_PLAIN);
    s->ev[e].triggered = 1; s->ev[e].ok = 1;
    schedule(s, e, 0, until - s->now);
    add_cb(s, e, CB_STOP, 0);
    s->stop_flag = 0;
    while (!s->stop_flag && s->nheap > 0 && !(s->status & ST_EXCEPTION)) env_step(s);
}

/* ---------------------------------------------------------------- agents */
static int has_capacity(const sim_t* s, int st) {
    return s->res[2 + st].users.len < s->res[2 + st].capacity;
}

/* PickupStationAgent.execute_action :190-276 */
static uint32_t pickup_execute(sim_t* s, int action) {
    uint32_t r = 0x80;   /* bits: 0 success, 1 product_loaded, 2 tray_completed, 3 idle_with_orders */
    if (action == 0) {
        if (s->order_queue.len > 0 || s->cur_order >= 0) r |= 8;
        r |= 1;
    } else if (action == 1) {
        if (s->cur_order < 0) {
            if (s->order_queue.len > 0) { s->cur_order = q_pop0(&s->order_queue); s->cur_idx = 0; }
            else return r;
        }
        if (s->cur_tray < 0) {
            if (s->trays_at_station.len > 0) {
                s->cur_tray = q_pop0(&s->trays_at_station);
                s->trays[s->cur_tray].order_id = s->cur_order;
            } else return r;
        }
        int product = PROD(s->cur_order, s->cur_idx);
        tray_t* T = &s->trays[s->cur_tray];
        if (T->len < T->cap) {                       /* not is_full() */
            if (s->cur_order != T->order_id) {       /* :231-235 (unreachable in practice) */
                q_push(&s->ps_ready, s->cur_tray); s->cur_tray = -1;
                r |= 4;
                return r;
            }
            T->prod[T->len++] = product;
            s->cur_idx += 1;
            r |= 2 | 1;
            if (s->cur_idx >= s->orders[s->cur_order].n) {
                s->cur_order = -1; s->cur_idx = 0;
                q_push(&s->ps_ready, s->cur_tray); s->cur_tray = -1;
                r |= 4;
                return r;
            }
            if (T->len >= T->cap) {
                q_push(&s->ps_ready, s->cur_tray); s->cur_tray = -1;
                r |= 4;
                return r;
            }
        } else {
            q_push(&s->ps_ready, s->cur_tray); s->cur_tray = -1;
            r |= 4;
            return r;
        }
    } else if (action == 2) {
        if (s->cur_tray >= 0 && s->trays[s->cur_tray].len > 0) {
            q_push(&s->ps_ready, s->cur_tray); s->cur_tray = -1;
            r |= 1;
        }
    }
    return r;
}

/* FJSPSimulation.add_tray_to_packaging :402-430 and PackagingAgent.add_tray :127-131 */
static void add_tray_to_packaging(sim_t* s, int t) {
    tray_t* T = &s->trays[t];
    if (T->len == 0) { oracle_fail(s, ST_EXCEPTION); return; }   /* ValueError */
    int color = s->orders[prod_order(T->prod[0])].color;
    int st = -1;
    for (int i = 0; i < 4; i++) if (PKG_COLOR[i] == color && has_capacity(s, i)) { st = i; break; }
    if (st < 0) { oracle_fail(s, ST_PROD_LOST); return; }
    for (int i = 0; i < T->len; i++)
        if (s->orders[prod_order(T->prod[i])].color == PKG_COLOR[st]) q_push(&s->p[st].queue, T->prod[i]);
}

/* AGVAgent.execute_action :180-252, _execute_pickup :254-293, _execute_drop :295-368 */
static uint32_t agv_execute(sim_t* s, int action) {
    /* bits: 0 success, 1 invalid, 2 moved, 3 pickup_success, 4 drop_success,
     * 5 delivered_to_packaging; bits 16.. distance */
    uint32_t r = 0x80;
    if (s->is_moving) return r | 2;
    if (action == 0) return r | 1;
    if (action >= 1 && action <= 5) {
        int loc = MOVE_LOC[action];
        int d = abs(s->pos_r - LOC_R[loc]) + abs(s->pos_c - LOC_C[loc]);
        if (d == 0) return r | 1;
        int p = spawn(s, P_AGV);
        s->procs[p].tr = LOC_R[loc]; s->procs[p].tc = LOC_C[loc];
        return r | 1 | 4 | ((uint32_t)d << 16);
    }
    int cur = current_location(s);
    if (action == 6) {
        if (s->carrying >= 0) return r | 2;
        if (cur == LOC_NONE) return r | 2;
        int t = -1;
        if (cur == LOC_PICKUP) { if (s->ps_ready.len) t = q_pop0(&s->ps_ready); }
        else if (cur == LOC_SMALL) { if (s->m[0].ready.len) t = q_pop0(&s->m[0].ready); }
        else if (cur == LOC_BIG) { if (s->m[1].ready.len) t = q_pop0(&s->m[1].ready); }
        else if (cur == LOC_STORAGE) { if (s->storage.len) t = q_pop0(&s->storage); }
        else if (cur == LOC_PACK) return r | 2;
        if (t >= 0) { s->carrying = t; return r | 1 | 8; }
        return r | 2;
    }
    if (action == 7) {
        if (s->carrying < 0) return r | 2;
        if (cur == LOC_NONE) return r | 2;
        int t = s->carrying;
        int ok = 0;
        if (cur == LOC_PICKUP) {
            if (s->trays[t].len == 0) {
                s->trays[t].order_id = -1;     /* add_empty_tray */
                q_push(&s->trays_at_station, t);
                ok = 1;
            } else return r | 2;
        } else if (cur == LOC_SMALL || cur == LOC_BIG) {
            int m = (cur == LOC_SMALL) ? 0 : 1;
            if (tray_needs_processing(s, t)) {
                int ty = tray_type(s, t);
                int compat = (m == 0) ? (ty == 1 || ty == 2) : (ty == 3 || ty == 2);
                if (compat) { q_push(&s->m[m].queue, t); ok = 1; }
                else return r | 2;
            } else return r | 2;
        } else if (cur == LOC_STORAGE) {
            if (s->storage.len < s->cfg[C_STORAGE_CAP]) q_push(&s->storage, t);
            else oracle_fail(s, ST_TRAY_LOST);
            ok = 1;
        } else if (cur == LOC_PACK) {
            if (tray_needs_packaging(s, t) && !tray_needs_processing(s, t)) {
                add_tray_to_packaging(s, t);
                ok = 1;
                r |= 32;
            } else return r | 2;
        }
        if (ok) { s->carrying = -1; r |= 1 | 16; }
        return r;
    }
    return r | 2;
}

/* MachineAgent.execute_action :99-139 */
static uint32_t machine_execute(sim_t* s, int m, int action) {
    uint32_t r = 0x80;   /* 0 success, 1 started, 2 completed, 3 idle_with_queue */
    if (action == 0) {
        if (s->m[m].queue.len > 0 && !s->m[m].busy) r |= 8;
        r |= 1;
    } else if (action == 1) {
        if (s->m[m].queue.len > 0 && !s->m[m].busy) {
            int t = q_pop0(&s->m[m].queue);
            if (s->m[m].cur_tray >= 0) oracle_fail(s, ST_OVERWRITE);
            int p = spawn(s, P_MACHINE);
            s->procs[p].agent = m; s->procs[p].tray = t;
            r |= 2 | 1;
        }
    } else if (action == 2) {
        if (!s->m[m].busy && s->m[m].cur_tray >= 0) {
            q_push(&s->m[m].ready, s->m[m].cur_tray);
            s->m[m].cur_tray = -1;
            r |= 4 | 1;
        }
    }
    return r;
}

/* PackagingAgent.execute_action :301-335 */
static uint32_t pack_execute(sim_t* s, int st, int action) {
    uint32_t r = 0x80;   /* 0 success, 1 started, 2 completed, 3 idle_with_queue; 16.. completed count */
    if (action == 0) {
        if (s->p[st].queue.len > 0 && !s->p[st].busy) r |= 8;
        r |= 1;
    } else if (action == 1) {
        int n = s->p[st].queue.len;
        for (int i = 0; i < n; i++) {
            int prod = q_get(&s->p[st].queue, i);
            int p = spawn(s, P_PACK);
            s->procs[p].agent = st; s->procs[p].product = prod;
            r |= 2 | 1;
            s->p[st].progress = (1.0 / (double)n) * 100.0;
        }
    } else if (action == 2) {
        if (!s->p[st].busy && s->p[st].cur_product >= 0) {
            r |= 4;
            r |= ((uint32_t)s->p[st].completed & 0xFFFFu) << 16;
        }
    }
    return r;
}

/* ---------------------------------------------------------------- observations */
typedef struct {
    int32_t obs_i32[20];
    int8_t obs_i8[12];
    float obs_f32[6];
    int8_t masks[29];
    uint8_t term, trunc, pad[2];
    double rewards[8];
    double sim_time;
    int32_t orders_completed, packaged;
    uint32_t results[8];
    uint32_t status;
    int32_t current_step;
} oracle_rec;

static int8_t to_i8(sim_t* s, int v) {
    if (v > 127 || v < -128) { oracle_fail(s, ST_OBS_OVERFLOW | ST_EXCEPTION); }
    return (int8_t)v;
}

static void observe(sim_t* s, oracle_rec* o) {
    /* pickup (PickupStationAgent.py:102-186) */
    int order_size = 0, remaining = 0, npt = 0, npc = 0, tt = 0, tc = 0, tcnt = 0;
    if (s->cur_order >= 0) {
        order_size = s->orders[s->cur_order].n;
        remaining = order_size - s->cur_idx;
        if (remaining > 0) { npt = s->orders[s->cur_order].type; npc = s->orders[s->cur_order].color; }
    }
    if (s->cur_tray >= 0) {
        tcnt = s->trays[s->cur_tray].len;
        if (tcnt > 0) { tt = tray_type(s, s->cur_tray); tc = tray_color(s, s->cur_tray); }
    }
    int32_t* I = o->obs_i32;
    I[0] = order_size; I[1] = remaining; I[2] = npt; I[3] = npc; I[4] = tt; I[5] = tc; I[6] = tcnt;
    int has_order = s->cur_order >= 0 || s->order_queue.len > 0;
    int has_tray = s->cur_tray >= 0 || s->trays_at_station.len > 0;
    int not_full = 1;
    if (s->cur_tray >= 0) not_full = s->trays[s->cur_tray].len < s->cfg[C_MASK_TRAY_CAP];
    int prem = 0;
    if (s->cur_order >= 0) prem = s->cur_idx < s->orders[s->cur_order].n;
    else if (s->order_queue.len > 0) prem = 1;
    o->masks[0] = 1;
    o->masks[1] = (has_order && has_tray && not_full && prem);
    o->masks[2] = (s->cur_tray >= 0 && s->trays[s->cur_tray].len > 0);
    /* AGV (AGVAgent.py:53-178) */
    int c = s->carrying;
    I[7] = s->pos_r; I[8] = s->pos_c;
    I[9] = c >= 0;
    I[10] = c >= 0 ? s->trays[c].len : 0;
    I[11] = c >= 0 ? tray_type(s, c) : 0;
    I[12] = c >= 0 && tray_needs_processing(s, c);
    I[13] = c >= 0 && tray_needs_packaging(s, c);
    I[14] = s->ps_ready.len;
    I[15] = s->m[0].busy; I[16] = s->m[1].busy;
    I[17] = s->m[0].ready.len; I[18] = s->m[1].ready.len;
    I[19] = s->storage.len;
    int8_t* M = &o->masks[3];
    memset(M, 0, 8);
    M[0] = 1;
    if (!s->is_moving) {
        int cur = current_location(s);
        for (int a = 1; a <= 5; a++) if (cur != MOVE_LOC[a]) M[a] = 1;
        if (c < 0 && cur != LOC_NONE) {
            if (cur == LOC_PICKUP) M[6] = s->ps_ready.len > 0;
            else if (cur == LOC_SMALL) M[6] = s->m[0].ready.len > 0;
            else if (cur == LOC_BIG) M[6] = s->m[1].ready.len > 0;
            else if (cur == LOC_STORAGE) M[6] = s->storage.len > 0;
        } else if (c >= 0 && cur != LOC_NONE) {
            int ty = tray_type(s, c);
            if (cur == LOC_PICKUP) M[7] = s->trays[c].len == 0;
            else if (cur == LOC_SMALL) M[7] = tray_needs_processing(s, c) && (ty == 1 || ty == 2);
            else if (cur == LOC_BIG) M[7] = tray_needs_processing(s, c) && (ty == 3 || ty == 2);
            else if (cur == LOC_PACK) M[7] = tray_needs_packaging(s, c) && !tray_needs_processing(s, c);
            else if (cur == LOC_STORAGE) M[7] = 1;
        }
    }
    /* machines (MachineAgent.py:62-97) */
    for (int m = 0; m < 2; m++) {
        o->obs_i8[2 * m] = (int8_t)s->m[m].busy;
        o->obs_i8[2 * m + 1] = to_i8(s, s->m[m].queue.len);
        o->obs_f32[m] = (float)s->m[m].progress;
        int8_t* K = &o->masks[11 + 3 * m];
        K[0] = 1;
        K[1] = s->m[m].queue.len > 0 && !s->m[m].busy;
        K[2] = !s->m[m].busy && s->m[m].cur_tray >= 0;
    }
    /* packaging (PackagingAgent.py:54-89) */
    for (int st = 0; st < 4; st++) {
        o->obs_i8[4 + 2 * st] = (int8_t)s->p[st].busy;
        o->obs_i8[4 + 2 * st + 1] = to_i8(s, s->p[st].queue.len);
        o->obs_f32[2 + st] = (float)s->p[st].progress;
        int8_t* K = &o->masks[17 + 3 * st];
        K[0] = 1;
        K[1] = s->p[st].queue.len > 0 && !s->p[st].busy && has_capacity(s, st);
        K[2] = !s->p[st].busy && s->p[st].cur_product >= 0;
    }
}

/* ---------------------------------------------------------------- reset / step */
static void sim_init(sim_t* s) {
    /* FJSPSimulation._init_agents/_init_storage/_init_trays + fresh simpy.Environment */
    s->now = 0.0; s->next_eid = 0; s->nheap = 0; s->nevents = 0; s->nprocs = 0;
    for (int r = 0; r < 6; r++) {
        s->res[r].capacity = r < 2 ? 1 : s->cfg[C_PACK_CAP];
        q_clear(&s->res[r].users); q_clear(&s->res[r].put_q); q_clear(&s->res[r].get_q);
    }
    q_clear(&s->order_queue); s->cur_order = -1; s->cur_idx = 0; q_clear(&s->trays_at_station);
    s->cur_tray = -1; q_clear(&s->ps_ready);
    s->pos_r = 0; s->pos_c = 0; s->carrying = -1; s->is_moving = 0;
    for (int m = 0; m < 2; m++) {
        q_clear(&s->m[m].queue); q_clear(&s->m[m].ready);
        s->m[m].cur_tray = -1; s->m[m].busy = 0; s->m[m].progress = 0.0;
        s->m[m].pt = m == 0 ? s->cfg[C_PT_SMALL] : s->cfg[C_PT_BIG];
    }
    for (int st = 0; st < 4; st++) {
        s->p[st].color = PKG_COLOR[st];
        q_clear(&s->p[st].queue); s->p[st].cur_product = -1; s->p[st].busy = 0;
        s->p[st].progress = 0.0; s->p[st].completed = 0;
    }
    q_clear(&s->storage);
    s->ntrays = s->cfg[C_NUM_TRAYS] < MAX_TRAYS ? s->cfg[C_NUM_TRAYS] : MAX_TRAYS;
    for (int t = 0; t < s->ntrays; t++) {
        s->trays[t].len = 0; s->trays[t].order_id = -1; s->trays[t].cap = s->cfg[C_TRAY_CAP];
    }
    /* available_trays.pop() x min(1000, n): ids n-1, n-2, ... (FJSPSimulation.py:96-98) */
    int give = s->ntrays < 1000 ? s->ntrays : 1000;
    for (int i = 0; i < give; i++) q_push(&s->trays_at_station, s->ntrays - 1 - i);
    s->norders = 0; s->ncompleted = 0; s->current_step = 0; s->total_packaged = 0;
    memset(s->processed, 0, sizeof(s->processed));
    memset(s->packaged, 0, sizeof(s->packaged));
}

void* oracle_create(const int32_t* cfg) {
    sim_t* s = (sim_t*)calloc(1, sizeof(sim_t));
    memcpy(s->cfg, cfg, sizeof(s->cfg));
    mt_seed(&s->rng, 5489u);
    sim_init(s);
    return s;
}
void oracle_destroy(void* h) { free(h); }
void oracle_seed(void* h, uint32_t seed) { mt_seed(&((sim_t*)h)->rng, seed); }

int oracle_reset(void* h, int num_orders, oracle_rec* o) {
    sim_t* s = (sim_t*)h;
    sim_init(s);
    s->status = 0;
    if (num_orders > MAX_ORDERS) { s->status |= ST_ORACLE_LIMIT; num_orders = MAX_ORDERS; }
    for (int i = 0; i < num_orders; i++) {        /* generate_order :101-131 */
        int n = 1 + (int)mt_bounded(&s->rng, 8);  /* randint(1, 10) */
        int ty = 1 + (int)mt_bounded(&s->rng, 2); /* choice(list(ProductType)) */
        int co = 1 + (int)mt_bounded(&s->rng, 2); /* choice(list(PackagingColor)) */
        order_t* O = &s->orders[s->norders];
        O->n = n; O->type = ty; O->color = co; O->complete = 0; O->completion_time = 0;
        q_push(&s->order_queue, s->norders);
        s->norders++;
    }
    if (o) {
        memset(o, 0, sizeof(*o));
        observe(s, o);
        o->status = s->status;
    }
    return (int)s->status;
}

/* FJSPSimulation.step :144-242.  actions[a] for agent a (canonical agent index), 255 = the
 * agent is absent from the action dict; order[] = execution order (dict order). */
int oracle_step(void* h, const uint8_t* actions, const uint8_t* order, oracle_rec* o) {
    static const uint8_t canon[8] = {0, 1, 2, 3, 4, 5, 6, 7};
    sim_t* s = (sim_t*)h;
    if (!order) order = canon;
    if (s->status & ST_EXCEPTION) {   /* the reference raised earlier: nothing is defined */
        if (o) { memset(o, 0, sizeof(*o)); o->status = s->status; }
        return (int)s->status;
    }
    int orders_before = s->ncompleted, products_before = s->total_packaged;
    uint32_t res[8] = {0};
    for (int i = 0; i < 8; i++) {
        int a = order[i];
        int act = actions[a];
        if (act == 255) continue;        /* agent missing from the dict */
        switch (a) {
        case 0: res[a] = pickup_execute(s, act); break;
        case 1: res[a] = agv_execute(s, act); break;
        case 2: case 3: res[a] = machine_execute(s, a - 2, act); break;
        default: res[a] = pack_execute(s, a - 4, act); break;
        }
        if (s->status & ST_EXCEPTION) break;
    }
    if (!(s->status & ST_EXCEPTION)) env_run(s, s->now + (double)s->cfg[C_STEP]);
    /* _check_order_completions :245-258 */
    for (int i = 0; i < s->norders; i++) {
        order_t* O = &s->orders[i];
        if (O->complete) continue;
        int all = 1;
        for (int k = 0; k < O->n; k++) if (!s->packaged[PROD(i, k)]) { all = 0; break; }
        if (all) { O->complete = 1; O->completion_time = s->now; s->ncompleted++; }
    }
    int orders_completed = s->ncompleted - orders_before;
    int products_packaged = s->total_packaged - products_before;
    int time_elapsed = s->cfg[C_STEP];
    /* RewardModel.calculate_global_reward :34-44 */
    double g = 100.0 * (double)orders_completed;
    g += 10.0 * (double)products_packaged;
    g += -0.1 * (double)time_elapsed;
    if (o) memset(o, 0, sizeof(*o));
    for (int a = 0; a < 8; a++) {
        int act = actions[a] == 255 ? 0 : actions[a];   /* actions.get(agent_id, 0) */
        uint32_t r = res[a];
        double loc = 0.0;                                 /* calculate_local_reward :46-97 */
        if (a == 0) {
            if (r & 2) loc += 1.0;
            if (r & 4) loc += 5.0;
            if (act == 0 && (r & 8)) loc += -1.0;
        } else if (a == 1) {
            if (r & 8) loc += 2.0;
            if (r & 16) loc += 2.0;
            if (r & 32) loc += 10.0;
            if (r & 4) loc += -0.1;
            if (r & 2) loc += -5.0;
        } else if (a <= 3) {
            if (r & 2) loc += 1.0;
            if (r & 4) loc += 5.0;
            if (act == 0 && (r & 8)) loc += -2.0;
        } else {
            if (r & 2) loc += 2.0;
            if (r & 4) loc += 20.0;
            if (act == 0 && (r & 8)) loc += -1.0;
        }
        if (o) o->rewards[a] = g / 8.0 + loc;           /* combine_rewards :99-110 */
        s->results[a] = r;
    }
    if (o) observe(s, o);
    int all_done = s->ncompleted == s->norders && s->norders > 0 && s->order_queue.len == 0;
    int truncated = s->current_step >= s->cfg[C_MAX_STEPS];
    if (o) {
        o->term = (uint8_t)all_done; o->trunc = (uint8_t)truncated;
        o->sim_time = s->now; o->orders_completed = s->ncompleted; o->packaged = s->total_packaged;
        memcpy(o->results, res, sizeof(res));
        o->current_step = s->current_step;
        o->status = s->status;
    }
    s->current_step += 1;
    return (int)s->status;
}

/* Order table view (for get_order_progress parity, FJSPSimulation.py:260-284):
 * per order u32 = n | type<<4 | color<<6 | processed_count<<8 | packaged_count<<12 | complete<<16 */
int oracle_orders(void* h, uint32_t* out, int max) {
    sim_t* s = (sim_t*)h;
    int n = s->norders < max ? s->norders : max;
    for (int i = 0; i < n; i++) {
        int pc = 0, kc = 0;
        for (int k = 0; k < s->orders[i].n; k++) { pc += s->processed[PROD(i, k)]; kc += s->packaged[PROD(i, k)]; }
        out[i] = (uint32_t)s->orders[i].n | ((uint32_t)s->orders[i].type << 4) |
                 ((uint32_t)s->orders[i].color << 6) | ((uint32_t)pc << 8) | ((uint32_t)kc << 12) |
                 ((uint32_t)s->orders[i].complete << 16);
    }
    return s->norders;
}

int oracle_record_size(void) { return (int)sizeof(oracle_rec); }
int oracle_current_step(void* h) { return ((sim_t*)h)->current_step; }

/* ---------------------------------------------------------------- synthetic actions */
static uint64_t fmix64(uint64_t z) {
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z;
}
static const int N_ACT[8] = {3, 8, 3, 3, 3, 3, 3, 3};
/* Counter RNG for synthetic actions (spec shared with tests/golden/gen_golden.py and the
 * HIP kernel).  masks: 29 int8 in canonical layout or NULL for unmasked. */
void oracle_actions(uint64_t seed, uint32_t env_gid, uint32_t step, const int8_t* masks, uint8_t* out) {
    static const int MOFF[8] = {0, 3, 11, 14, 17, 20, 23, 26};
    uint64_t h = fmix64(seed ^ fmix64(((uint64_t)env_gid << 32) | step));
    for (int a = 0; a < 8; a++) {
        uint32_t b = (uint32_t)(h >> (8 * a)) & 0xFFu;
        if (!masks) { out[a] = (uint8_t)((b * (uint32_t)N_ACT[a]) >> 8); continue; }
        int cnt = 0;
        for (int i = 0; i < N_ACT[a]; i++) cnt += masks[MOFF[a] + i] != 0;
        int j = (int)((b * (uint32_t)cnt) >> 8);
        for (int i = 0; i < N_ACT[a]; i++) {
            if (masks[MOFF[a] + i]) { if (j == 0) { out[a] = (uint8_t)i; break; } j--; }
        }
    }
}

/* MultiAgentA2C._get_heuristic_actions (a2c.py:390-537), statement by statement.  Tuples
 * the heuristic compares the AGV position with: small (2,3), big (0,3), pickup (0,0),
 * packaging (3,5) and "storage" (1,5) -- the latter is not STORAGE's position (3,0,
 * constants.py:9), so that comparison is always false in the reference and here. */
static int at(const sim_t* s, int r, int c) { return s->pos_r == r && s->pos_c == c; }
static int machine_available(const sim_t* s, int m) { return !s->m[m].busy && s->m[m].queue.len < 3; }
void oracle_heuristic(void* h, uint8_t* out) {
    const sim_t* s = (const sim_t*)h;
    out[0] = (s->order_queue.len > 0 || s->cur_order >= 0) ? 1 : 0;
    int a = 0;
    if (s->is_moving) {
        a = 0;
    } else if (s->carrying >= 0) {
        const int t = s->carrying;
        if (tray_needs_processing(s, t)) {
            const int ty = tray_type(s, t);                      /* 1 SMALL, 2 MEDIUM, 3 BIG */
            const int m = (ty == 1 || ty == 2) ? 0 : 1;
            const int tr = m == 0 ? 2 : 0, move = m == 0 ? 2 : 3;
            if (machine_available(s, m)) a = at(s, tr, 3) ? 7 : move;
            else a = at(s, 1, 5) ? 7 : 4;
        } else if (tray_needs_packaging(s, t)) {
            a = at(s, 3, 5) ? 7 : 5;
        } else {
            a = 0;
        }
    } else if (s->m[0].ready.len > 0) {
        a = at(s, 2, 3) ? 6 : 2;
    } else if (s->m[1].ready.len > 0) {
        a = at(s, 0, 3) ? 6 : 3;
    } else if (s->storage.len > 0) {
        int found = 0;
        for (int i = 0; i < s->storage.len && !found; i++) {
            const int t = q_get((fifo*)&s->storage, i);
            if (!tray_needs_processing(s, t)) continue;
            const int ty = tray_type(s, t);
            const int m = (ty == 1 || ty == 2) ? 0 : 1;
            if (machine_available(s, m)) { a = at(s, 1, 5) ? 6 : 4; found = 1; }
        }
        if (!found) a = s->ps_ready.len > 0 ? (at(s, 0, 0) ? 6 : 1) : 0;   /* for ... else */
    } else if (s->ps_ready.len > 0) {
        a = at(s, 0, 0) ? 6 : 1;
    } else if (s->m[0].busy || s->m[0].cur_tray >= 0) {
        a = at(s, 2, 3) ? 0 : 2;
    } else if (s->m[1].busy || s->m[1].cur_tray >= 0) {
        a = at(s, 0, 3) ? 0 : 3;
    } else if (s->order_queue.len > 0 || s->cur_order >= 0) {
        a = at(s, 0, 0) ? 0 : 1;
    }
    out[1] = (uint8_t)a;
    for (int m = 0; m < 2; m++) {
        if (s->m[m].queue.len > 0 && !s->m[m].busy) out[2 + m] = 1;
        else if (s->m[m].cur_tray >= 0 && !s->m[m].busy) out[2 + m] = 2;
        else out[2 + m] = 0;
    }
    for (int st = 0; st < 4; st++) out[4 + st] = (s->p[st].queue.len > 0 && !s->p[st].busy) ? 1 : 0;
}

/* Rollout of n_envs independent envs (the CPU baseline and the bulk parity driver).
 * Env e: global id gid0+e, seeded seeds[e], `steps` steps, actions from the counter RNG
 * (policy 0 unmasked, 1 masked), from `actions_in` [steps][n_envs][8] (policy 2) or from
 * oracle_heuristic (policy 3);
 * auto-reset with seed=None on term|trunc.  If `rec_out` is non-NULL it receives
 * [steps][n_envs] records (post-step obs); reset obs go to `reset_out` if non-NULL. */
int oracle_rollout(const int32_t* cfg, int n_envs, uint32_t gid0, const uint32_t* seeds,
                   int num_orders, int steps, uint64_t action_seed, int policy,
                   const uint8_t* actions_in, oracle_rec* rec_out, oracle_rec* reset_out,
                   uint64_t* checksum) {
    uint64_t ck = 0;
    sim_t* s = (sim_t*)oracle_create(cfg);
    oracle_rec cur, rec;
    for (int e = 0; e < n_envs; e++) {
        mt_seed(&s->rng, seeds[e]);
        oracle_reset(s, num_orders, &cur);
        for (int t = 0; t < steps; t++) {
            uint8_t act[8];
            if (policy == 2) memcpy(act, actions_in + ((size_t)t * n_envs + e) * 8, 8);
            else if (policy == 3) oracle_heuristic(s, act);
            else oracle_actions(action_seed, gid0 + (uint32_t)e, (uint32_t)t, policy == 1 ? cur.masks : NULL, act);
            oracle_step(s, act, NULL, &rec);
            ck = ck * 0x100000001B3ull + (uint64_t)(rec.rewards[0] * 8.0) + (uint64_t)rec.obs_i32[14];
            if (rec_out) rec_out[(size_t)t * n_envs + e] = rec;
            cur = rec;
            if (rec.term || rec.trunc) {
                oracle_reset(s, num_orders, &cur);
            }
            if (reset_out) reset_out[(size_t)t * n_envs + e] = cur;
        }
    }
    oracle_destroy(s);
    if (checksum) *checksum = ck;
    return 0;
}

/* ---------------------------------------------------------------- GAE / returns */
/* transition_memory.py:83-105, one (agent) column: rewards r[T], values v[T] (as the f32
 * critic outputs), bootstrap next_value per segment.  seg_end[t] != 0 closes a segment;
 * boots[k] is the next_value of the k-th segment. */
void oracle_gae(const double* r, const float* v, const double* boots, const uint8_t* seg_end,
                int T, int stride, double gamma, double lamb, double* ret, double* adv) {
    int start = 0, seg = 0;
    for (int t = 0; t < T; t++) {
        if (!seg_end[t] && t != T - 1) continue;
        int end = t + 1;
        double nv = boots[(size_t)seg * stride];
        double rr = nv;
        for (int i = end - 1; i >= start; i--) {          /* _compute_returns */
            rr = r[(size_t)i * stride] + gamma * rr;
            ret[(size_t)i * stride] = rr;
        }
        double gae = 0.0;
        double next_value = nv;
        for (int i = end - 1; i >= start; i--) {          /* _compute_gae */
            double val = (double)v[(size_t)i * stride];
            double td = r[(size_t)i * stride] + gamma * next_value - val;
            gae = td + gamma * lamb * gae;
            adv[(size_t)i * stride] = gae;
            next_value = val;
        }
        start = end; seg++;
    }
}
