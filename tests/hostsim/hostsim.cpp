// hostsim.cpp — TEST-ONLY host build of the kernel's per-env state machine
// (multi-agent-rl-for-fjsp_amd/csrc/fjsp_env.h) so its closed-form logic can be checked
// against the oracle on CPU in the build container (no GPU there).  The product library
// (libfjsp.so) never contains or loads this; the GPU parity tests are the real proof.
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#define FJSP_DEV inline
#include "../../multi-agent-rl-for-fjsp_amd/csrc/fjsp_env.h"
using namespace fjsp;

struct HS {
    int n; Cfg C;
    Env* E; uint32_t* orders; uint16_t* scode; uint8_t* snext; uint16_t* scstep;
    uint32_t (*mt)[624]; int* mti;
};
static uint32_t mt_next_(uint32_t* s, int& mti) {
    if (mti >= 624) {
        for (int i = 0; i < 624; i++) {
            uint32_t y = (s[i] & 0x80000000u) | (s[(i + 1) % 624] & 0x7fffffffu);
            s[i] = s[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        mti = 0;
    }
    uint32_t y = s[mti++];
    y ^= y >> 11; y ^= (y << 7) & 0x9d2c5680u; y ^= (y << 15) & 0xefc60000u; y ^= y >> 18;
    return y;
}
static int bounded(uint32_t* s, int& mti, uint32_t rng, uint32_t mask) {
    uint32_t v; do { v = mt_next_(s, mti) & mask; } while (v > rng); return (int)v;
}
static Tables tabs(HS* h, int e) { Tables T; T.orders = h->orders + e; T.scode = h->scode + e; T.snext = h->snext + e; T.scstep = h->scstep + e; T.stride = h->n; return T; }

extern "C" {
void* hs_create(const int32_t* c, int n) {
    HS* h = (HS*)calloc(1, sizeof(HS));
    h->n = n;
    // c = oracle cfg order: num_trays, tray_cap, mask_tray_cap, storage_cap, step, max_steps, speed, pt_s, pt_b, pt_p, pkg_cap
    h->C.step_size = c[4]; h->C.max_steps = c[5]; h->C.tray_cap = c[1]; h->C.mask_tray_cap = c[2];
    h->C.storage_cap = c[3]; h->C.pool0 = c[0] < 1000 ? c[0] : 1000; h->C.pkg_cap = c[10];
    h->C.ptk_small = c[7] / c[4]; h->C.ptk_big = c[8] / c[4]; h->C.ptk_pack = c[9] / c[4];
    const double w[NW] = {100.0, 10.0, -0.1, 1.0, 5.0, -1.0, 2.0, -0.1, 10.0, -5.0, 5.0, 1.0, -2.0, 20.0, 2.0, -1.0};
    double* lut = (double*)calloc(RLUT_SIZE, sizeof(double));
    build_reward_lut(w, c[4], lut);
    h->C.lut = lut;
    h->E = (Env*)calloc(n, sizeof(Env));
    h->orders = (uint32_t*)calloc((size_t)MAX_ORDERS * n, 4);
    h->scode = (uint16_t*)calloc((size_t)MAX_SLOTS * n, 2);
    h->snext = (uint8_t*)calloc((size_t)MAX_SLOTS * n, 1);
    h->scstep = (uint16_t*)calloc((size_t)MAX_SLOTS * n, 2);
    h->mt = (uint32_t(*)[624])calloc((size_t)n, sizeof(uint32_t[624]));
    h->mti = (int*)calloc(n, sizeof(int));
    return h;
}
void hs_destroy(void* p) {
    HS* h = (HS*)p; free((void*)h->C.lut); free(h->E); free(h->orders); free(h->scode); free(h->snext); free(h->scstep); free(h->mt); free(h->mti); free(h);
}
static void reset_one(HS* h, int e, int num_orders) {
    Env& E = h->E[e]; Tables T = tabs(h, e);
    env_clear(E, h->C);
    E.set_norders(num_orders);
    for (int o = 0; o < num_orders; o++) {
        int n = 1 + bounded(h->mt[e], h->mti[e], 8, 15);
        int ty = 1 + bounded(h->mt[e], h->mti[e], 2, 3);
        int co = 1 + bounded(h->mt[e], h->mti[e], 2, 3);
        T.orders[o * T.stride] = ow_make(n, ty, co);
    }
}
// out: obs_i32[20], i8[12], f32[6], masks[29] per env (AoS for the harness)
static void obs_out(HS* h, int e, int32_t* i32, int8_t* i8, float* f32, int8_t* mk) {
    Obs o; ObsSink sk{o}; observe(h->E[e], h->C, sk);
    memcpy(i32 + 20 * e, o.i32, 80); memcpy(i8 + 12 * e, o.i8, 12); memcpy(f32 + 6 * e, o.f32, 24); memcpy(mk + 29 * e, o.mask, 29);
}
void hs_reset(void* p, const uint32_t* seeds, int num_orders, int32_t* i32, int8_t* i8, float* f32, int8_t* mk) {
    HS* h = (HS*)p;
    for (int e = 0; e < h->n; e++) {
        if (seeds) {
            uint32_t* s = h->mt[e]; s[0] = seeds[e];
            for (int i = 1; i < 624; i++) s[i] = 1812433253u * (s[i - 1] ^ (s[i - 1] >> 30)) + (uint32_t)i;
            h->mti[e] = 624;
        }
        reset_one(h, e, num_orders);
        obs_out(h, e, i32, i8, f32, mk);
    }
}
// actions [n][8]; outputs AoS per env; autoreset continues the MT stream
void hs_step(void* p, const uint8_t* actions, int autoreset, int32_t* i32, int8_t* i8, float* f32, int8_t* mk,
             double* rew, uint8_t* term, uint8_t* trunc, uint32_t* res, uint32_t* status,
             int32_t* ri32, int8_t* ri8, float* rf32, int8_t* rmk) {
    HS* h = (HS*)p;
    for (int e = 0; e < h->n; e++) {
        Env& E = h->E[e]; Tables T = tabs(h, e);
        int act[8]; for (int a = 0; a < 8; a++) act[a] = actions[8 * e + a];
        env_step<true>(E, T, h->C, act, nullptr, res + 8 * e, rew + 8 * e);
        obs_out(h, e, i32, i8, f32, mk);
        const int nord = E.norders();
        int all_done = E.ncompleted() == nord && nord > 0 && E.next_order() == nord;
        int tr = E.step() >= h->C.max_steps;
        term[e] = (uint8_t)all_done; trunc[e] = (uint8_t)tr; status[e] = E.status();
        E.set_step(E.step() + 1);
        if (autoreset && (all_done || tr)) reset_one(h, e, nord);
        obs_out(h, e, ri32, ri8, rf32, rmk);
    }
}
// heuristic proposals (a2c.py:390-537) for every env: out [n][8]
void hs_heuristic(void* p, uint8_t* out) {
    HS* h = (HS*)p;
    for (int e = 0; e < h->n; e++) {
        int act[8];
        heuristic_actions(h->E[e], tabs(h, e), act);
        for (int a = 0; a < 8; a++) out[8 * e + a] = (uint8_t)act[a];
    }
}
}
