// san_main.cpp — TEST-ONLY sanitizer run of the host build of the kernel's state machine
// (csrc/fjsp_env.h through hostsim.cpp) and of the parity oracle (oracle/fjsp_oracle.c), built
// together with -fsanitize=address,undefined (tests/test_sanitizers.py).  It steps N envs with
// the closed form and with the oracle's event heap side by side (random and masked-random
// actions, auto-reset continuing the MT19937 stream, default and stress configurations) and
// compares every output byte; any sanitizer report aborts the run.
#include <stdio.h>
#include <string.h>

#include "hostsim.cpp"

extern "C" {
void* oracle_create(const int32_t* cfg);
void oracle_destroy(void* h);
void oracle_seed(void* h, uint32_t seed);
int oracle_record_size(void);
void oracle_actions(uint64_t seed, uint32_t env_gid, uint32_t step, const int8_t* masks, uint8_t* out);
}

struct Rec {   // oracle_rec (oracle/fjsp_oracle.c)
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
};
extern "C" int oracle_reset(void* h, int num_orders, Rec* o);
extern "C" int oracle_step(void* h, const uint8_t* actions, const uint8_t* order, Rec* o);

static int run(const int32_t* cfg, int n, int steps, int num_orders, int policy) {
    void* hs = hs_create(cfg, n);
    int32_t* i32 = new int32_t[20 * n]; int8_t* i8 = new int8_t[12 * n]; float* f32 = new float[6 * n];
    int8_t* mk = new int8_t[29 * n]; double* rew = new double[8 * n]; uint8_t* term = new uint8_t[n];
    uint8_t* trunc = new uint8_t[n]; uint32_t* res = new uint32_t[8 * n]; uint32_t* st = new uint32_t[n];
    int32_t* ri32 = new int32_t[20 * n]; int8_t* ri8 = new int8_t[12 * n]; float* rf32 = new float[6 * n];
    int8_t* rmk = new int8_t[29 * n]; uint8_t* acts = new uint8_t[8 * n];
    uint32_t* seeds = new uint32_t[n];
    void** sims = new void*[n];
    for (int e = 0; e < n; e++) seeds[e] = 100u + (uint32_t)e;
    hs_reset(hs, seeds, num_orders, i32, i8, f32, rmk);
    Rec cur;
    for (int e = 0; e < n; e++) {
        sims[e] = oracle_create(cfg);
        oracle_seed(sims[e], seeds[e]);
        oracle_reset(sims[e], num_orders, &cur);
    }
    int bad = 0, ends = 0, skipped = 0;
    for (int t = 0; t < steps; t++) {
        for (int e = 0; e < n; e++) oracle_actions(0, (uint32_t)e, (uint32_t)t, policy ? rmk + 29 * e : nullptr, acts + 8 * e);
        hs_step(hs, acts, 1, i32, i8, f32, mk, rew, term, trunc, res, st, ri32, ri8, rf32, rmk);
        for (int e = 0; e < n; e++) {
            Rec r;
            oracle_step(sims[e], acts + 8 * e, nullptr, &r);
            if ((st[e] & 1u) || (r.status & 0x7u)) {   // a path the closed form flags, not emulates
                skipped++;
            } else if (memcmp(i32 + 20 * e, r.obs_i32, 80) || memcmp(i8 + 12 * e, r.obs_i8, 12) ||
                       memcmp(f32 + 6 * e, r.obs_f32, 24) || memcmp(mk + 29 * e, r.masks, 29) ||
                       memcmp(rew + 8 * e, r.rewards, 64) || term[e] != r.term || trunc[e] != r.trunc) {
                if (bad < 5) fprintf(stderr, "mismatch: policy %d step %d env %d\n", policy, t, e);
                bad++;
            }
            if (r.term || r.trunc) {
                ends++;
                oracle_reset(sims[e], num_orders, &cur);
            }
        }
    }
    printf("policy %d: %d envs x %d steps, %d episode ends, %d flagged, %d mismatches\n", policy, n, steps, ends,
           skipped, bad);
    for (int e = 0; e < n; e++) oracle_destroy(sims[e]);
    hs_destroy(hs);
    delete[] i32; delete[] i8; delete[] f32; delete[] mk; delete[] rew; delete[] term; delete[] trunc; delete[] res;
    delete[] st; delete[] ri32; delete[] ri8; delete[] rf32; delete[] rmk; delete[] acts; delete[] seeds; delete[] sims;
    return bad;
}

int main(int argc, char** argv) {
    if (oracle_record_size() != (int)sizeof(Rec)) { fprintf(stderr, "record layout\n"); return 2; }
    const int n = argc > 1 ? atoi(argv[1]) : 256, steps = argc > 2 ? atoi(argv[2]) : 400;
    // oracle cfg order: num_trays, tray_cap, mask_tray_cap, storage_cap, step, max_steps, speed, pt_s, pt_b, pt_p, pkg_cap
    const int32_t dflt[11] = {1000, 5, 5, 100, 10, 200, 1, 60, 120, 30, 20};
    const int32_t stress[11] = {40, 3, 5, 2, 10, 50, 1, 60, 120, 30, 2};
    int bad = 0;
    bad += run(dflt, n, steps, 30, 0);
    bad += run(dflt, n, steps, 30, 1);
    bad += run(stress, n / 4, steps, 6, 1);
    printf("%s\n", bad ? "FAIL" : "OK");
    return bad ? 1 : 0;
}
