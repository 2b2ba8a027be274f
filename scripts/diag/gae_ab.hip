// DIAGNOSTIC (A/B of the GAE kernel's load pipelining; not product code): the r03 kernel (one
// dependent round trip per timestep) against the software-pipelined kernel of
// multi-agent-rl-for-fjsp_amd/csrc/fjsp_hip.hip at several batch depths.  scripts/diag_gae.py.
#include <hip/hip_runtime.h>
#include <stdint.h>
namespace {
template <class VT>
__global__ void __launch_bounds__(256) k_gae_r03(const double* __restrict__ r, const VT* __restrict__ v,
                                             const uint8_t* __restrict__ done, const double* __restrict__ boot, int T,
                                             int N, int M, double gamma, double lamb, double* __restrict__ ret,
                                             double* __restrict__ adv) {
    const int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= M) return;
    const int e = m % N;
    const double gl = gamma * lamb;
    double nv = 0.0, rr = 0.0, gae = 0.0;
    for (int t = T - 1; t >= 0; t--) {
        const size_t i = (size_t)t * M + m;
        if (t == T - 1 || done[(size_t)t * N + e]) {
            nv = (t == T - 1 && !done[(size_t)t * N + e]) ? boot[m] : 0.0;
            rr = nv;
            gae = 0.0;
        }
        const double rt = r[i];
        const double vt = (double)v[i];
        rr = rt + gamma * rr;
        ret[i] = rr;
        const double td = rt + gamma * nv - vt;
        gae = td + gl * gae;
        adv[i] = gae;
        nv = vt;
    }
}
template <class VT, bool SHARED, int GAE_U>
struct GaeChunk {
    double r[GAE_U];
    VT v[GAE_U];
    uint8_t d[GAE_U];
};
// Loads of the GAE_U timesteps t0, t0 - 1, ... (rows below 0 clamped to row 0: never used, and
// no branch around a load — a load under a branch made the compiler drain every load at the join).
template <class VT, bool SHARED, int GAE_U>
__device__ __forceinline__ void gae_load(GaeChunk<VT, SHARED, GAE_U>& c, const double* __restrict__ r,
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
template <class VT, bool SHARED, bool FULL, int GAE_U>
__device__ __forceinline__ void gae_scan(const GaeChunk<VT, SHARED, GAE_U>& c, int t0, int T, int M, int m, double bootv,
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
template <class VT, bool SHARED, int GAE_U>
__device__ __forceinline__ void gae_scan_any(const GaeChunk<VT, SHARED, GAE_U>& c, int t0, int T, int M, int m, double bootv,
                                             double gamma, double gl, double& nv, double& rr, double& gae,
                                             double* __restrict__ ret, double* __restrict__ adv) {
    if (t0 >= GAE_U - 1) gae_scan<VT, SHARED, true, GAE_U>(c, t0, T, M, m, bootv, gamma, gl, nv, rr, gae, ret, adv);
    else gae_scan<VT, SHARED, false, GAE_U>(c, t0, T, M, m, bootv, gamma, gl, nv, rr, gae, ret, adv);
}
template <class VT, bool SHARED, int GAE_U>
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
    GaeChunk<VT, SHARED, GAE_U> A, B;
    int t0 = T - 1;
    gae_load<VT, SHARED, GAE_U>(A, r, v, done, t0, N, M, m, e);
    for (;;) {   // A holds t0.., B is loaded before A's scan, and the other way round
        gae_load<VT, SHARED, GAE_U>(B, r, v, done, t0 - GAE_U, N, M, m, e);
        gae_scan_any<VT, SHARED, GAE_U>(A, t0, T, M, m, bootv, gamma, gl, nv, rr, gae, ret, adv);
        t0 -= GAE_U;
        if (t0 < 0) break;
        gae_load<VT, SHARED, GAE_U>(A, r, v, done, t0 - GAE_U, N, M, m, e);
        gae_scan_any<VT, SHARED, GAE_U>(B, t0, T, M, m, bootv, gamma, gl, nv, rr, gae, ret, adv);
        t0 -= GAE_U;
        if (t0 < 0) break;
    }
}

}  // namespace

extern "C" int gae_r03(const double* r, const float* v, const uint8_t* d, const double* boot, int T, int N, int M,
                       double g, double l, double* ret, double* adv, void* s) {
    hipLaunchKernelGGL(k_gae_r03<float>, dim3((M + 255) / 256), dim3(256), 0, (hipStream_t)s, r, v, d, boot, T, N, M, g, l,
                       ret, adv);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
#define GEN(U)                                                                                                        \
    extern "C" int gae_u##U(const double* r, const float* v, const uint8_t* d, const double* boot, int T, int N,      \
                            int M, double g, double l, double* ret, double* adv, void* s) {                           \
        hipLaunchKernelGGL((k_gae<float, false, U>), dim3((M + 63) / 64), dim3(64), 0, (hipStream_t)s, r, v, d, boot, \
                           T, N, M, g, l, ret, adv);                                                                  \
        return hipGetLastError() == hipSuccess ? 0 : -1;                                                              \
    }                                                                                                                 \
    extern "C" int gae_shared_u##U(const double* r, const float* v, const uint8_t* d, int T, int N, int A, double g,  \
                                   double l, double* ret, double* adv, void* s) {                                     \
        const int M = A * N;                                                                                          \
        hipLaunchKernelGGL((k_gae<float, true, U>), dim3((M + 63) / 64), dim3(64), 0, (hipStream_t)s, r, v, d,        \
                           nullptr, T, N, M, g, l, ret, adv);                                                         \
        return hipGetLastError() == hipSuccess ? 0 : -1;                                                              \
    }
GEN(4)
GEN(8)
GEN(16)
GEN(24)
GEN(32)

// ---- variant: a loader wave feeding the scan wave through an LDS ring (LDS DMA, 16 B per lane).
// The scan wave issues only stores; the loader keeps L chunks of U timesteps in flight with a
// counted vmcnt wait, so the loads' latency hides behind L chunk scans.  N % 64 == 0.
namespace {
__device__ __forceinline__ void dma16(const void* g, void* s) {
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)g, (__attribute__((address_space(3))) void*)s,
                                     16, 0, 0);
}
template <int U>
struct GaeSlot {
    double r[U][64];
    float v[U][64];
    uint8_t d[U][64];
};
template <int U, int L>
__global__ void __launch_bounds__(128) k_gae_lw(const double* __restrict__ r, const float* __restrict__ v,
                                               const uint8_t* __restrict__ done, int T, int N, int M, double gamma,
                                               double lamb, double* __restrict__ ret, double* __restrict__ adv) {
    static_assert(U % 16 == 0, "16 timesteps per done DMA");
    constexpr int S = L + 1, PER = U / 2 + U / 4 + U / 16;   // slots, DMA instructions per chunk
    static_assert(PER * (L - 1) <= 63, "vmcnt");
    __shared__ GaeSlot<U> slot[S];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int m0 = blockIdx.x * 64, e0 = m0 % N;
    const int nch = (T + U - 1) / U;
    auto issue = [&](int c) __attribute__((always_inline)) {   // chunk c: timesteps T-1-cU .. down
        GaeSlot<U>& s = slot[c % S];
        const int t0 = T - 1 - c * U;
#pragma unroll
        for (int i = 0; i < U / 2; i++) {
            int t = t0 - 2 * i - (lane >> 5);
            t = t > 0 ? t : 0;
            dma16(r + (size_t)t * M + m0 + 2 * (lane & 31), &s.r[2 * i][0]);
        }
#pragma unroll
        for (int i = 0; i < U / 4; i++) {
            int t = t0 - 4 * i - (lane >> 4);
            t = t > 0 ? t : 0;
            dma16(v + (size_t)t * N + e0 + 4 * (lane & 15), &s.v[4 * i][0]);
        }
#pragma unroll
        for (int i = 0; i < U / 16; i++) {
            int t = t0 - 16 * i - (lane >> 2);
            t = t > 0 ? t : 0;
            dma16(done + (size_t)t * N + e0 + 16 * (lane & 3), &s.d[16 * i][0]);
        }
    };
    // vmcnt <= PER * (L - 1), expcnt / lgkmcnt not waited for
    constexpr int VM = PER * (L - 1);
    constexpr int WAIT_AHEAD = (VM & 15) | ((VM >> 4) << 14) | (7 << 4) | (15 << 8);
    if (wave == 1) {
        for (int c = 0; c < L; c++) issue(c);
        __builtin_amdgcn_s_waitcnt(WAIT_AHEAD);   // chunk 0 landed
    }
    __syncthreads();
    const int m = m0 + lane;
    const double gl = gamma * lamb;
    const double bootv = (double)v[(size_t)T * N + e0 + lane];
    double nv = 0.0, rr = 0.0, gae = 0.0;
    for (int p = 0; p < nch; p++) {
        if (wave == 1) {
            issue(p + L);
            __builtin_amdgcn_s_waitcnt(WAIT_AHEAD);   // chunk p + 1 landed
        } else {
            const GaeSlot<U>& s = slot[p % S];
            const int t0 = T - 1 - p * U;
#pragma unroll
            for (int j = 0; j < U; j++) {
                const int t = t0 - j;
                if (t < 0) continue;
                const uint8_t dj = s.d[j][lane];
                if (t == T - 1 || dj) {
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

#define GENLW(U, L)                                                                                                   \
    extern "C" int gae_shared_lw_u##U##_l##L(const double* r, const float* v, const uint8_t* d, int T, int N, int A,  \
                                             double g, double l, double* ret, double* adv, void* s) {                 \
        if (N % 64) return -2;                                                                                        \
        const int M = A * N;                                                                                          \
        hipLaunchKernelGGL((k_gae_lw<U, L>), dim3(M / 64), dim3(128), 0, (hipStream_t)s, r, v, d, T, N, M, g, l, ret, \
                           adv);                                                                                      \
        return hipGetLastError() == hipSuccess ? 0 : -1;                                                              \
    }
GENLW(16, 2)
GENLW(16, 3)
GENLW(16, 4)
GENLW(32, 2)
