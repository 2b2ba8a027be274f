// Diagnostic cycle stamps of the step kernels: compiled in only by the diagnostic builds
// (scripts/build_diag.sh: -DFJSP_STAMPS, -DFJSP_STAMPS_FINE; read by scripts/diag_stamps.py,
// diag_ag_stamps.py, diag_fixed_cost.py).  The product build expands every macro here to
// nothing, so its code is the same with or without this file.
//
//   FJSP_DIAG(code)           code only in a stamps build (declarations, s_memtime reads, sums)
//   FJSP_STAMP_AT / FJSP_STAMP / FJSP_STAMP_AGENT   per-env phase stamps (Env::st_acc, k_step*)
//   AG_T0 / AG_ACC / AG_MARK / AG_SPIN_T0 / AG_SPIN_ACC / AG_BARRIER   k_step_ag's per-wave
//                             busy / wait cycles, phase marks and last arrivals at the barrier
//                             (they name the k_step_ag locals ag_wait, ag_last, amt, _ag_t0)
#pragma once

#ifdef FJSP_STAMPS

#define FJSP_DIAG(...) __VA_ARGS__

// per-env s_memtime deltas per step phase; -DFJSP_STAMPS_FINE splits the action phase per
// agent: slots 0 synth, 1 pickup, 2 AGV, 3 machines, 4 packaging, 5 run, 6 rewards + observe +
// stores, 7 auto-reset
#define FJSP_STAMP_AT(E, i)                                \
    do {                                                   \
        uint64_t _t = __builtin_amdgcn_s_memtime();        \
        (E).st_acc[i] += _t - (E).st_t0;                   \
        (E).st_t0 = _t;                                    \
    } while (0)
#ifdef FJSP_STAMPS_FINE
#define FJSP_STAMP(E, i)                                                          \
    do {                                                                          \
        constexpr int _m[7] = {0, -1, 5, 6, 6, 6, 7};                             \
        if (_m[i] >= 0) FJSP_STAMP_AT(E, _m[i] >= 0 ? _m[i] : 0);                 \
    } while (0)
#define FJSP_STAMP_AGENT(E, a)                                                    \
    do {                                                                          \
        if ((a) == 0) FJSP_STAMP_AT(E, 1);                                        \
        if ((a) == 1) FJSP_STAMP_AT(E, 2);                                        \
        if ((a) == 3) FJSP_STAMP_AT(E, 3);                                        \
        if ((a) == 7) FJSP_STAMP_AT(E, 4);                                        \
    } while (0)
#else
#define FJSP_STAMP(E, i) FJSP_STAMP_AT(E, i)
#define FJSP_STAMP_AGENT(E, a) ((void)0)
#endif

#define AG_T0() const uint64_t _ag_t0 = __builtin_amdgcn_s_memtime()
#define AG_ACC(v) ((v) += __builtin_amdgcn_s_memtime() - _ag_t0)
#define AG_MARK(i) (amt[i] += __builtin_amdgcn_s_memtime() - _ag_t0)
#define AG_SPIN_T0() const uint64_t _ag_w0 = __builtin_amdgcn_s_memtime()
#define AG_SPIN_ACC() (ag_wait += __builtin_amdgcn_s_memtime() - _ag_w0)
#define AG_BARRIER()                                                        \
    do {                                                                    \
        const uint64_t _b0 = __builtin_amdgcn_s_memtime();                 \
        __syncthreads();                                                    \
        ag_last += (__builtin_amdgcn_s_memtime() - _b0) < 200 ? 1 : 0;     \
    } while (0)

#else

#define FJSP_DIAG(...)
#define FJSP_STAMP_AT(E, i) ((void)0)
#define FJSP_STAMP(E, i) ((void)0)
#define FJSP_STAMP_AGENT(E, a) ((void)0)
#define AG_T0() ((void)0)
#define AG_ACC(v) ((void)0)
#define AG_MARK(i) ((void)0)
#define AG_SPIN_T0() ((void)0)
#define AG_SPIN_ACC() ((void)0)
#define AG_BARRIER() __syncthreads()

#endif
