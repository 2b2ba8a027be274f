// fjsp_group.hip — the A2C update's grouping of repeated inputs on the GPU (a2c_vec.RowGroups):
// per row of grouping keys (8 actor rows + the critic's, fjsp_a2c_group_keys) the distinct keys,
// each sample's group, the samples sorted by group (stable: equal keys keep sample order) and each
// group's first sample and run end.  The reference runs every network once per sample
// (a2c.py:647-703 _update over the batch); the grouped update runs it once per distinct input and
// sums the samples' gradients by runs of this order, so the order must be deterministic.
//
// One flat radix sort of all rows (rocPRIM's device radix sort) (the row id in key bits 59..62 above 59 bits of the hash: rows
// stay contiguous), 32-bit sample positions as the payload (the grouping needs no more), then one
// inclusive scan of the run starts, and one pass that scatters each sorted position's sample,
// group and run start.  Replaces torch.sort (64-bit payload), a blocked prefix sum, a binary
// search per group and three gathers / scatters over [R][S].
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <stdint.h>

#include "../../include/fjsp.h"

int fjsp_internal_fail(const char* msg);

namespace {

constexpr uint64_t KEY_MASK = (1ull << 59) - 1;

// flat[i] = row r's key (59 bits) | r << 59, pos[i] = i, for i = r * S + s
__global__ void __launch_bounds__(256) k_group_flat(const uint64_t* __restrict__ keys, int64_t S, int64_t RS,
                                                    uint64_t* __restrict__ flat, uint32_t* __restrict__ pos) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= RS) return;
    const uint64_t r = (uint64_t)(i / S);
    flat[i] = (keys[i] & KEY_MASK) | (r << 59);
    pos[i] = (uint32_t)i;
}

// 1 where a row starts or the sorted key changes (a group's first sorted position)
__global__ void __launch_bounds__(256) k_group_new(const uint64_t* __restrict__ sk, int64_t S, int64_t RS,
                                                   uint32_t* __restrict__ nw) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= RS) return;
    nw[i] = (i % S == 0 || sk[i] != sk[i - 1]) ? 1u : 0u;
}

// groups per row from the inclusive scan G of the run starts: U[r] = G[last of r] - G[first of r] + 1
__global__ void k_group_counts(const uint32_t* __restrict__ G, int32_t R, int64_t S, int64_t* __restrict__ U) {
    const int r = (int)threadIdx.x;
    if (r < R) U[r] = (int64_t)G[(int64_t)(r + 1) * S - 1] - (int64_t)G[(int64_t)r * S] + 1;
}

// starts[r][g] = S for every group slot (padding groups keep it), before k_group_runs
__global__ void __launch_bounds__(256) k_group_fill(int64_t* __restrict__ starts, int64_t n, int64_t S) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) starts[i] = S;
}

// sorted position j of row r (i = r * S + j): its sample p and group g;
// perm[r][j] = p, gsorted[r][j] = g, inv[r][p] = g, and at a group's first position
// starts[r][g] = j, first[r][g] = p
__global__ void __launch_bounds__(256) k_group_runs(const uint32_t* __restrict__ spos, const uint32_t* __restrict__ G,
                                                    int64_t S, int64_t RS, int64_t umax, int64_t* __restrict__ perm,
                                                    int64_t* __restrict__ inv, int64_t* __restrict__ starts,
                                                    int64_t* __restrict__ first, int32_t* __restrict__ gsorted) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= RS) return;
    const int64_t r = i / S, j = i - r * S;
    const int64_t g = (int64_t)G[i] - (int64_t)G[r * S];
    const int64_t p = (int64_t)spos[i] - r * S;
    perm[i] = p;
    gsorted[i] = (int32_t)g;
    inv[r * S + p] = g;
    if ((j == 0 || G[i] != G[i - 1]) && g < umax) {   // g < umax: a caller's umax below a count stays in bounds
        starts[r * umax + g] = j;
        first[r * umax + g] = p;
    }
}

// per group slot: ends (the next group's start, S for the last and the padding), a padding
// group's representative (the row's last sorted sample, as a gather of perm at S - 1)
__global__ void __launch_bounds__(256) k_group_ends(const int64_t* __restrict__ starts, const int64_t* __restrict__ perm,
                                                    int32_t R, int64_t S, int64_t umax, int64_t* __restrict__ first,
                                                    int64_t* __restrict__ ends) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)R * umax) return;
    const int64_t r = i / umax, g = i - r * umax;
    ends[i] = g + 1 < umax ? starts[i + 1] : S;
    if (starts[i] == S) first[i] = perm[r * S + S - 1];
}

// rep[r][s] = first[r][inv[r][s]]: each sample's group representative
__global__ void __launch_bounds__(256) k_group_rep(const int64_t* __restrict__ inv, const int64_t* __restrict__ first,
                                                   int64_t S, int64_t RS, int64_t umax, int64_t* __restrict__ rep) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= RS) return;
    const int64_t r = i / S, g = inv[i];
    rep[i] = g < umax ? first[r * umax + g] : -1;
}

// Run sums: out[j][g] = sum over the sorted positions of group g of row a = rowmap[j] of
// vals[j][perm[a][pos]] (* scale[j], in f32, as the gradient is scaled before the sum), summed in
// f64, stored as f32.  The backward of a per-group gather (each group's samples' gradients
// summed: a2c_vec._GatherRuns, _ActorHead): deterministic, one pass over the values.
// k_run_chunks: a workgroup takes RS_CH sorted positions of one row, forms their f64 prefix sums
// (per thread 4, then a block scan of the thread totals in a fixed order), and each run of one
// group inside the chunk is the difference of the prefixes at its two ends (the group ids of a
// row's sorted positions rise by one per run, so run k of the chunk is group g0 + k).  A run that
// crosses a chunk end leaves its chunk part (cont / first_part, last_part / last_g); k_run_carry
// adds those over chunks with the same construction one level up (prefix sums and a prefix max
// of the run-start chunks, one workgroup per row).
constexpr int RS_CH = 1024, RS_T = 256;

// inclusive scan of v over the RS_T threads of a workgroup (Kogge-Stone, fixed order); sc: LDS
template <class T, class Op>
__device__ __forceinline__ T block_scan(T v, T* sc, Op op) {
    const int t = (int)threadIdx.x;
    sc[t] = v;
    __syncthreads();
#pragma unroll
    for (int d = 1; d < RS_T; d <<= 1) {
        const T o = t >= d ? sc[t - d] : v;
        __syncthreads();
        if (t >= d) v = op(o, v);
        sc[t] = v;
        __syncthreads();
    }
    return v;
}

__global__ void __launch_bounds__(RS_T) k_run_chunks(const float* __restrict__ vals, const int32_t* __restrict__ rowmap,
                                                   const float* __restrict__ scale, const int64_t* __restrict__ perm,
                                                   const int32_t* __restrict__ gsorted, int64_t S, int64_t umax,
                                                   int64_t nch, float* __restrict__ out, double* __restrict__ first_part,
                                                   uint8_t* __restrict__ cont, double* __restrict__ last_part,
                                                   int32_t* __restrict__ last_g) {
    __shared__ double s_sc[RS_T];
    __shared__ double s_lo[RS_CH], s_hi[RS_CH];   // per run k: the prefix before its first / at its last position
    const int64_t c = blockIdx.x;
    const int j = (int)blockIdx.y, t = (int)threadIdx.x;
    const int64_t a = rowmap[j];
    const float sc = scale ? scale[j] : 1.0f;
    const int64_t pos0 = c * RS_CH, pend = pos0 + RS_CH < S ? pos0 + RS_CH : S;   // [pos0, pend)
    const int32_t* gs = gsorted + a * S;
    const int64_t* pm = perm + a * S;
    const float* vr = vals + (int64_t)j * S;
    int32_t g[4];
    double pre[4];
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int64_t p = pos0 + 4 * t + i;
        g[i] = p < pend ? gs[p] : -1;
        acc += p < pend ? (double)(vr[pm[p]] * sc) : 0.0;
        pre[i] = acc;
    }
    const double incl = block_scan(acc, s_sc, [](double x, double y) { return x + y; });
    const double off = incl - acc;   // the prefix before this thread's positions
    const int32_t g0 = gs[pos0];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int64_t p = pos0 + 4 * t + i;
        if (p >= pend) break;
        const int k = g[i] - g0;
        if (p == pos0 || gs[p - 1] != g[i]) s_lo[k] = i == 0 ? off : off + pre[i - 1];
        if (p + 1 == pend || gs[p + 1] != g[i]) s_hi[k] = off + pre[i];
    }
    __syncthreads();
    const int32_t glast = gs[pend - 1];
    const int m = glast - g0 + 1;
    const int32_t prev_g = pos0 > 0 ? gs[pos0 - 1] : -2;
    const int32_t next_g = pend < S ? gs[pend] : -2;
    const int64_t jc = (int64_t)j * nch + c;
    for (int k = t; k < m; k += RS_T) {
        const double sum = s_hi[k] - s_lo[k];
        const bool from_prev = k == 0 && prev_g == g0, into_next = k == m - 1 && next_g == glast;
        if (from_prev) {
            first_part[jc] = sum;
            cont[jc] = into_next ? 2 : 1;   // 2: the run covers the whole chunk and goes on
        } else if (into_next) {
            last_part[jc] = sum;
            last_g[jc] = g0 + k;
        } else if (g0 + k < umax) {
            out[(int64_t)j * umax + g0 + k] = (float)sum;
        }
    }
}

// Per row (one workgroup): over its chunks, Q = inclusive prefix sums of the continuation parts
// (first_part where cont != 0) and M = the last chunk <= c where a crossing run starts; a chunk e
// whose first run ends there (cont == 1) completes the run that started in chunk M[e - 1]:
// last_part[M] + Q[e] - Q[M].  Q is kept in qbuf [J][nch] for the lookups.
__global__ void __launch_bounds__(RS_T) k_run_carry(int64_t nch, int64_t umax, const double* __restrict__ first_part,
                                                  const uint8_t* __restrict__ cont, const double* __restrict__ last_part,
                                                  const int32_t* __restrict__ last_g, double* __restrict__ qbuf,
                                                  float* __restrict__ out) {
    __shared__ double s_sc[RS_T];
    __shared__ int64_t s_mx[RS_T];
    const int64_t j = blockIdx.x, base = j * nch;
    const int t = (int)threadIdx.x;
    double qcarry = 0.0;
    int64_t mcarry = -1;
    for (int64_t c0 = 0; c0 < nch; c0 += RS_CH) {
        double q[4], acc = 0.0;
        int64_t mx[4], m = -1;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int64_t c = c0 + 4 * t + i;
            const bool in = c < nch;
            acc += in && cont[base + c] ? first_part[base + c] : 0.0;
            q[i] = acc;
            if (in && last_g[base + c] >= 0) m = c;
            mx[i] = m;
        }
        const double qi = block_scan(acc, s_sc, [](double x, double y) { return x + y; });
        (void)block_scan(m, s_mx, [](int64_t x, int64_t y) { return x > y ? x : y; });   // s_mx: inclusive maxima
        const double qoff = qcarry + (qi - acc);
        // the running max before this thread: the inclusive max of the thread before it
        const int64_t mprev_t = t > 0 ? s_mx[t - 1] : -1;
        const int64_t moff = mprev_t > mcarry ? mprev_t : mcarry;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int64_t c = c0 + 4 * t + i;
            if (c < nch) qbuf[base + c] = qoff + q[i];
        }
        __syncthreads();   // this tile's Q is visible to the workgroup
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int64_t c = c0 + 4 * t + i;
            if (c >= nch || cont[base + c] != 1) continue;
            int64_t st = i == 0 ? moff : (mx[i - 1] > moff ? mx[i - 1] : moff);   // last start chunk < c
            if (st < 0) continue;   // cannot happen: a continued run started in an earlier chunk
            const double s = last_part[base + st] + (qoff + q[i]) - qbuf[base + st];
            if (last_g[base + st] < umax) out[j * umax + last_g[base + st]] = (float)s;
        }
        qcarry += s_sc[RS_T - 1];
        mcarry = s_mx[RS_T - 1] > mcarry ? s_mx[RS_T - 1] : mcarry;
        __syncthreads();
    }
}

// ---- the low-cardinality rows (lowcard mask): a stable counting sort instead of the radix sort.
// The station agents' rows of the A2C grouping hold <= ~30 distinct keys per 10^6 samples; a
// radix sort pays 8 passes over them (8 bits per pass of 63 key bits).  Per such row: the distinct
// keys in a 256-slot open-addressing table (LC_CAP = 64 at most, else the row is reported as
// overflowing: counts[r] = -1, and the caller groups again without the mask), their ranks in key
// order, per 1 024-sample chunk the samples of each rank (one wave per chunk), one exclusive scan
// over (row, rank, chunk), and a stable scatter: a wave takes its chunk's samples in order, 64 at
// a time, and each sample's position is its rank's running offset + the lanes before it with the
// same rank (six ballots).  The output is the radix sort's exactly: per row the (row-tagged) keys
// ascending, equal keys in sample order.
constexpr int LC_CAP = 64, LC_SLOTS = 256, LC_CH = 1024;
struct RowList {   // row ids, by value in the kernel arguments
    int32_t r[16];
};
constexpr uint64_t LC_EMPTY = ~0ull;   // never a masked key (bit 63 is clear)

__device__ __forceinline__ int lc_hash(uint64_t k) { return (int)((k * 0x9E3779B97F4A7C15ull) >> 56); }

// insert k into a 256-slot table (LDS or global); returns true if it was new; *over on overflow
template <bool SHARED>
__device__ __forceinline__ bool lc_insert(uint64_t* tbl, uint64_t k, bool* full) {
    int h = lc_hash(k);
    for (int probe = 0; probe < LC_SLOTS; probe++, h = (h + 1) & (LC_SLOTS - 1)) {
        uint64_t cur = tbl[h];
        if (cur == k) return false;
        if (cur == LC_EMPTY) {
            const uint64_t old = SHARED ? atomicCAS((unsigned long long*)&tbl[h], (unsigned long long)LC_EMPTY,
                                                    (unsigned long long)k)
                                        : atomicCAS((unsigned long long*)&tbl[h], (unsigned long long)LC_EMPTY,
                                                    (unsigned long long)k);
            if (old == LC_EMPTY) return true;
            if (old == k) return false;
        }
    }
    *full = true;
    return false;
}

__device__ __forceinline__ int lc_find(const uint64_t* tbl, uint64_t k) {   // slot of a key known to be there
    int h = lc_hash(k);
    for (int probe = 0; probe < LC_SLOTS; probe++, h = (h + 1) & (LC_SLOTS - 1))
        if (tbl[h] == k) return h;
    return -1;
}

// grid (chunks, low rows), 256 threads: the chunk's distinct keys, then into the row's global table
// (gtbl [nl][256], gcnt [nl], over [nl]; rows[i] = the i-th low row)
__global__ void __launch_bounds__(256) k_lc_distinct(const uint64_t* __restrict__ keys, RowList rows,
                                                     int64_t S, uint64_t* __restrict__ gtbl, uint32_t* __restrict__ gcnt,
                                                     uint32_t* __restrict__ over) {
    __shared__ uint64_t t[LC_SLOTS];
    __shared__ uint32_t n;
    __shared__ bool full;
    const int li = (int)blockIdx.y, tid = (int)threadIdx.x;
    const int64_t r = rows.r[li], c0 = (int64_t)blockIdx.x * LC_CH;
    t[tid] = LC_EMPTY;
    if (tid == 0) { n = 0; full = false; }
    __syncthreads();
    for (int i = tid; i < LC_CH; i += 256) {
        const int64_t s = c0 + i;
        if (s >= S) break;
        const uint64_t k = keys[r * S + s] & KEY_MASK;
        bool f = false;
        if (lc_insert<true>(t, k, &f)) atomicAdd(&n, 1u);
        if (f) full = true;
    }
    __syncthreads();
    if (full || n > (uint32_t)LC_CAP) {
        if (tid == 0) atomicOr(&over[li], 1u);
        return;
    }
    const uint64_t k = t[tid];
    if (k != LC_EMPTY) {
        bool f = false;
        if (lc_insert<false>(gtbl + (int64_t)li * LC_SLOTS, k, &f)) {
            if (atomicAdd(&gcnt[li], 1u) + 1u > (uint32_t)LC_CAP) atomicOr(&over[li], 1u);
        }
        if (f) atomicOr(&over[li], 1u);
    }
}

// one workgroup of 256 per low row: rank of every used slot in ascending key order (grank [nl][256])
__global__ void __launch_bounds__(256) k_lc_rank(const uint64_t* __restrict__ gtbl, const uint32_t* __restrict__ over,
                                                 uint8_t* __restrict__ grank) {
    __shared__ uint64_t t[LC_SLOTS];
    const int li = (int)blockIdx.x, tid = (int)threadIdx.x;
    if (over[li]) return;
    const uint64_t k = gtbl[(int64_t)li * LC_SLOTS + tid];
    t[tid] = k;
    __syncthreads();
    int rank = 0;
    for (int j = 0; j < LC_SLOTS; j++) rank += (t[j] != LC_EMPTY && t[j] < k) ? 1 : 0;
    grank[(int64_t)li * LC_SLOTS + tid] = k == LC_EMPTY ? (uint8_t)255 : (uint8_t)rank;
}

// one wave per (chunk, low row): samples per rank, hist [nl][LC_CAP][nch]
// (an overflowed row counts its chunk's samples as rank 0, so every row's counts still sum to S and
// the scan's offsets of the other rows stay in their rows; its samples are not scattered)
__global__ void __launch_bounds__(64) k_lc_hist(const uint64_t* __restrict__ keys, RowList rows,
                                                int64_t S, int64_t nch, const uint64_t* __restrict__ gtbl,
                                                const uint8_t* __restrict__ grank, const uint32_t* __restrict__ over,
                                                uint32_t* __restrict__ hist) {
    __shared__ uint64_t t[LC_SLOTS];
    __shared__ uint8_t rk[LC_SLOTS];
    __shared__ uint32_t h[LC_CAP];
    const int li = (int)blockIdx.y, lane = (int)threadIdx.x;
    const int64_t r = rows.r[li], c = blockIdx.x;
    if (over[li]) {
        const int64_t len = S - c * LC_CH < LC_CH ? S - c * LC_CH : LC_CH;
        hist[((int64_t)li * LC_CAP + lane) * nch + c] = lane == 0 ? (uint32_t)len : 0u;
        return;
    }
    for (int j = lane; j < LC_SLOTS; j += 64) {
        t[j] = gtbl[(int64_t)li * LC_SLOTS + j];
        rk[j] = grank[(int64_t)li * LC_SLOTS + j];
    }
    h[lane] = 0;
    __syncthreads();
    for (int i = lane; i < LC_CH; i += 64) {
        const int64_t s = c * LC_CH + i;
        if (s >= S) break;
        const int q = rk[lc_find(t, keys[r * S + s] & KEY_MASK)];
        atomicAdd(&h[q], 1u);
    }
    __syncthreads();
    hist[((int64_t)li * LC_CAP + lane) * nch + c] = h[lane];
}

// one wave per (chunk, low row): the stable scatter into the row's part of sorted / spos
__global__ void __launch_bounds__(64) k_lc_scatter(const uint64_t* __restrict__ keys, RowList rows,
                                                   int64_t S, int64_t nch, const uint64_t* __restrict__ gtbl,
                                                   const uint8_t* __restrict__ grank, const uint32_t* __restrict__ over,
                                                   const uint32_t* __restrict__ offs, uint64_t* __restrict__ sorted,
                                                   uint32_t* __restrict__ spos) {
    __shared__ uint64_t t[LC_SLOTS];
    __shared__ uint8_t rk[LC_SLOTS];
    __shared__ uint32_t base[LC_CAP];
    const int li = (int)blockIdx.y, lane = (int)threadIdx.x;
    if (over[li]) return;
    const int64_t r = rows.r[li], c = blockIdx.x;
    for (int j = lane; j < LC_SLOTS; j += 64) {
        t[j] = gtbl[(int64_t)li * LC_SLOTS + j];
        rk[j] = grank[(int64_t)li * LC_SLOTS + j];
    }
    // offs: the exclusive scan over [nl][LC_CAP][nch]; row li's samples start at li * S there
    base[lane] = offs[((int64_t)li * LC_CAP + lane) * nch + c] - (uint32_t)(li * S);
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int i0 = 0; i0 < LC_CH; i0 += 64) {
        const int64_t s = c * LC_CH + i0 + lane;
        const bool ok = s < S;
        uint64_t k = 0;
        int q = 0;
        if (ok) {
            k = keys[r * S + s] & KEY_MASK;
            q = rk[lc_find(t, k)];
        }
        uint64_t peers = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 6; b++) {
            const uint64_t m = __ballot((q >> b) & 1);
            peers &= ((q >> b) & 1) ? m : ~m;
        }
        const uint32_t my = base[q] + (uint32_t)__popcll(peers & lt);
        __builtin_amdgcn_wave_barrier();
        if (ok && (peers >> lane) == 1ull) base[q] += (uint32_t)__popcll(peers);   // the group's last lane
        __builtin_amdgcn_wave_barrier();
        if (ok) {
            const int64_t d = r * S + my;
            sorted[d] = k | ((uint64_t)r << 59);
            spos[d] = (uint32_t)(r * S + s);
        }
    }
}

// flat / pos for the high-cardinality rows only, compacted (hrows[i] = the i-th such row)
__global__ void __launch_bounds__(256) k_group_flat_rows(const uint64_t* __restrict__ keys, RowList hrows,
                                                         int64_t S, int64_t HS, uint64_t* __restrict__ flat,
                                                         uint32_t* __restrict__ pos) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= HS) return;
    const int64_t hi = i / S, s = i - hi * S;
    const uint64_t r = (uint64_t)hrows.r[hi];
    flat[i] = (keys[r * S + s] & KEY_MASK) | (r << 59);
    pos[i] = (uint32_t)(r * S + s);
}

// counts[r] = -1 for a low row that overflowed LC_CAP (the caller groups again without the mask)
__global__ void k_lc_flag(RowList rows, int32_t nl, const uint32_t* __restrict__ over, int64_t* __restrict__ counts) {
    const int i = (int)threadIdx.x;
    if (i < nl && over[i]) counts[rows.r[i]] = -1;
}

int launch_error() {
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        fjsp_internal_fail(hipGetErrorString(err));
        return -2;
    }
    return 0;
}

unsigned blocks(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

extern "C" int fjsp_a2c_group_temp_bytes(int64_t count, uint64_t* bytes) {
    if (count <= 0 || count >= (1ll << 31)) return fjsp_internal_fail("fjsp_a2c_group_temp_bytes: count must be in (0, 2^31)");
    if (!bytes) return fjsp_internal_fail("fjsp_a2c_group_temp_bytes: null pointer");
    size_t a = 0, b = 0, c = 0;
    if (rocprim::radix_sort_pairs(nullptr, a, (const uint64_t*)nullptr, (uint64_t*)nullptr, (const uint32_t*)nullptr,
                                  (uint32_t*)nullptr, (uint32_t)count, 0u, 63u) != hipSuccess ||
        rocprim::inclusive_scan(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)count,
                                rocprim::plus<uint32_t>()) != hipSuccess ||
        rocprim::exclusive_scan(nullptr, c, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)count,
                                rocprim::plus<uint32_t>()) != hipSuccess)
        return fjsp_internal_fail("fjsp_a2c_group_temp_bytes: rocprim size query failed");
    a = a > b ? a : b;
    *bytes = (uint64_t)(a > c ? a : c);
    return 0;
}

extern "C" int fjsp_a2c_group_sort(const uint64_t* keys, int32_t R, int64_t S, uint32_t lowcard, void* temp,
                                   uint64_t temp_bytes, uint64_t* flat, uint64_t* sorted, uint32_t* pos, uint32_t* spos,
                                   uint32_t* runs, uint32_t* scan, int64_t* counts, void* stream) {
    const int64_t RS = (int64_t)R * S;
    if (R <= 0 || R > 16 || S <= 0 || RS >= (1ll << 31))
        return fjsp_internal_fail("fjsp_a2c_group_sort: need 0 < R <= 16, S > 0, R * S < 2^31");
    if (!keys || !temp || !flat || !sorted || !pos || !spos || !runs || !scan || !counts)
        return fjsp_internal_fail("fjsp_a2c_group_sort: null buffer");
    uint64_t need = 0;
    if (int rc = fjsp_a2c_group_temp_bytes(RS, &need)) return rc;
    if (temp_bytes < need) return fjsp_internal_fail("fjsp_a2c_group_sort: temp buffer too small");
    const hipStream_t st = (hipStream_t)stream;
    // the counting path's rows, and its scratch: the per-(row, rank, chunk) counts and their scan
    // in runs / scan (free until the run starts), the tables at the end of pos (the radix sort's
    // input uses only its first (R - nl) * S words)
    RowList lrl{}, hrl{};
    int32_t* lrows = lrl.r;
    int32_t* hrows = hrl.r;
    int nl = 0, nh = 0;
    for (int r = 0; r < R; r++) {
        if ((lowcard >> r) & 1u) lrows[nl++] = r;
        else hrows[nh++] = r;
    }
    const int64_t nch = (S + LC_CH - 1) / LC_CH;
    const size_t tbl_bytes = (size_t)nl * LC_SLOTS * 8 + 32 * 4 + (size_t)nl * LC_SLOTS + 64;
    if (nl > 0 && ((int64_t)nl * LC_CAP * nch > RS || tbl_bytes > (size_t)nl * (size_t)S * 4)) {
        for (int i = 0; i < nl; i++) hrows[nh++] = lrows[i];   // too small for the scratch: radix sort them all
        nl = 0;
        for (int a = 0; a < nh; a++)   // keep ascending row order
            for (int b = a + 1; b < nh; b++)
                if (hrows[b] < hrows[a]) { const int32_t x = hrows[a]; hrows[a] = hrows[b]; hrows[b] = x; }
    }
    size_t tb = (size_t)temp_bytes;
    if (nl == 0) {
        hipLaunchKernelGGL(k_group_flat, dim3(blocks(RS)), dim3(256), 0, st, keys, S, RS, flat, pos);
        if (int rc = launch_error()) return rc;
        // stable LSD radix sort over the 63 key bits (row id 59..62 above 59 hash bits)
        if (rocprim::radix_sort_pairs(temp, tb, flat, sorted, pos, spos, (uint32_t)RS, 0u, 63u, st) != hipSuccess)
            return fjsp_internal_fail("fjsp_a2c_group_sort: radix sort failed");
    } else {
        // small device arrays (row lists, tables) at the end of pos
        char* ex = (char*)(pos + RS) - tbl_bytes;
        ex = (char*)(((uintptr_t)ex) & ~(uintptr_t)63);
        uint64_t* gtbl = (uint64_t*)ex;
        uint32_t* gcnt = (uint32_t*)(gtbl + (size_t)nl * LC_SLOTS);   // [16] counts, then [16] overflow flags
        uint32_t* over = gcnt + 16;
        uint8_t* grank = (uint8_t*)(over + 16);
        if (hipMemsetAsync(gtbl, 0xFF, (size_t)nl * LC_SLOTS * 8, st) != hipSuccess ||
            hipMemsetAsync(gcnt, 0, 32 * 4, st) != hipSuccess)
            return fjsp_internal_fail("fjsp_a2c_group_sort: scratch set-up failed");
        if (nh > 0) {
            const int64_t HS = (int64_t)nh * S;
            hipLaunchKernelGGL(k_group_flat_rows, dim3(blocks(HS)), dim3(256), 0, st, keys, hrl, S, HS, flat, pos);
            if (int rc = launch_error()) return rc;
            if (rocprim::radix_sort_pairs(temp, tb, flat, sorted, pos, spos, (uint32_t)HS, 0u, 63u, st) != hipSuccess)
                return fjsp_internal_fail("fjsp_a2c_group_sort: radix sort failed");
            // the i-th high row's sorted block to its own row (last first: blocks only move up)
            for (int i = nh - 1; i >= 0; i--) {
                if (hrows[i] == i) continue;
                if (hipMemcpyAsync(sorted + (int64_t)hrows[i] * S, sorted + (int64_t)i * S, 8 * (size_t)S,
                                   hipMemcpyDeviceToDevice, st) != hipSuccess ||
                    hipMemcpyAsync(spos + (int64_t)hrows[i] * S, spos + (int64_t)i * S, 4 * (size_t)S,
                                   hipMemcpyDeviceToDevice, st) != hipSuccess)
                    return fjsp_internal_fail("fjsp_a2c_group_sort: block move failed");
            }
        }
        hipLaunchKernelGGL(k_lc_distinct, dim3((unsigned)nch, (unsigned)nl), dim3(256), 0, st, keys, lrl, S, gtbl, gcnt,
                           over);
        if (int rc = launch_error()) return rc;
        hipLaunchKernelGGL(k_lc_rank, dim3((unsigned)nl), dim3(256), 0, st, gtbl, over, grank);
        if (int rc = launch_error()) return rc;
        hipLaunchKernelGGL(k_lc_hist, dim3((unsigned)nch, (unsigned)nl), dim3(64), 0, st, keys, lrl, S, nch, gtbl, grank,
                           over, runs);
        if (int rc = launch_error()) return rc;
        const size_t nhist = (size_t)nl * LC_CAP * (size_t)nch;
        tb = (size_t)temp_bytes;
        if (rocprim::exclusive_scan(temp, tb, runs, scan, 0u, nhist, rocprim::plus<uint32_t>(), st) != hipSuccess)
            return fjsp_internal_fail("fjsp_a2c_group_sort: count scan failed");
        hipLaunchKernelGGL(k_lc_scatter, dim3((unsigned)nch, (unsigned)nl), dim3(64), 0, st, keys, lrl, S, nch, gtbl,
                           grank, over, scan, sorted, spos);
        if (int rc = launch_error()) return rc;
        // k_lc_flag below reads over after the counts
        hipLaunchKernelGGL(k_group_new, dim3(blocks(RS)), dim3(256), 0, st, sorted, S, RS, runs);
        if (int rc = launch_error()) return rc;
        tb = (size_t)temp_bytes;
        if (rocprim::inclusive_scan(temp, tb, runs, scan, (size_t)RS, rocprim::plus<uint32_t>(), st) != hipSuccess)
            return fjsp_internal_fail("fjsp_a2c_group_sort: scan failed");
        hipLaunchKernelGGL(k_group_counts, dim3(1), dim3(64), 0, st, scan, R, S, counts);
        if (int rc = launch_error()) return rc;
        hipLaunchKernelGGL(k_lc_flag, dim3(1), dim3(64), 0, st, lrl, nl, over, counts);
        return launch_error();
    }
    hipLaunchKernelGGL(k_group_new, dim3(blocks(RS)), dim3(256), 0, st, sorted, S, RS, runs);
    if (int rc = launch_error()) return rc;
    tb = (size_t)temp_bytes;
    if (rocprim::inclusive_scan(temp, tb, runs, scan, (size_t)RS, rocprim::plus<uint32_t>(), st) != hipSuccess)
        return fjsp_internal_fail("fjsp_a2c_group_sort: scan failed");
    hipLaunchKernelGGL(k_group_counts, dim3(1), dim3(64), 0, st, scan, R, S, counts);
    return launch_error();
}

extern "C" int fjsp_a2c_group_runs(const uint32_t* spos, const uint32_t* scan, int32_t R, int64_t S, int64_t umax,
                                   int64_t* starts, int64_t* perm, int64_t* inv, int64_t* rep, int64_t* first,
                                   int64_t* ends, int32_t* gsorted, void* stream) {
    const int64_t RS = (int64_t)R * S;
    if (R <= 0 || R > 16 || S <= 0 || umax <= 0 || RS >= (1ll << 31))
        return fjsp_internal_fail("fjsp_a2c_group_runs: need 0 < R <= 16, S > 0, umax > 0, R * S < 2^31");
    if (!spos || !scan || !starts || !perm || !inv || !rep || !first || !ends || !gsorted)
        return fjsp_internal_fail("fjsp_a2c_group_runs: null buffer");
    const hipStream_t st = (hipStream_t)stream;
    const int64_t RU = (int64_t)R * umax;
    hipLaunchKernelGGL(k_group_fill, dim3(blocks(RU)), dim3(256), 0, st, starts, RU, S);
    if (int rc = launch_error()) return rc;
    hipLaunchKernelGGL(k_group_runs, dim3(blocks(RS)), dim3(256), 0, st, spos, scan, S, RS, umax, perm, inv, starts, first,
                       gsorted);
    if (int rc = launch_error()) return rc;
    hipLaunchKernelGGL(k_group_ends, dim3(blocks(RU)), dim3(256), 0, st, starts, perm, R, S, umax, first, ends);
    if (int rc = launch_error()) return rc;
    hipLaunchKernelGGL(k_group_rep, dim3(blocks(RS)), dim3(256), 0, st, inv, first, S, RS, umax, rep);
    return launch_error();
}

extern "C" int fjsp_a2c_run_sums_bytes(int32_t J, int64_t S, uint64_t* bytes) {
    if (J <= 0 || S <= 0 || !bytes) return fjsp_internal_fail("fjsp_a2c_run_sums_bytes: need J > 0, S > 0");
    const int64_t n = (int64_t)J * ((S + RS_CH - 1) / RS_CH);
    *bytes = (uint64_t)n * (8 + 8 + 8 + 4 + 1) + 64;
    return 0;
}

extern "C" int fjsp_a2c_run_sums(const float* vals, int32_t J, const int32_t* rowmap, const float* scale,
                                 const int64_t* perm, const int32_t* gsorted, int64_t S, int64_t umax, void* temp,
                                 uint64_t temp_bytes, float* out, void* stream) {
    if (J <= 0 || J > 65535 || S <= 0 || umax <= 0) return fjsp_internal_fail("fjsp_a2c_run_sums: need 0 < J < 65536, S > 0, umax > 0");
    if (!vals || !rowmap || !perm || !gsorted || !temp || !out) return fjsp_internal_fail("fjsp_a2c_run_sums: null buffer");
    uint64_t need = 0;
    if (int rc = fjsp_a2c_run_sums_bytes(J, S, &need)) return rc;
    if (temp_bytes < need) return fjsp_internal_fail("fjsp_a2c_run_sums: temp buffer too small");
    const hipStream_t st = (hipStream_t)stream;
    const int64_t nch = (S + RS_CH - 1) / RS_CH, n = (int64_t)J * nch;
    double* first_part = (double*)temp;
    double* last_part = first_part + n;
    double* qbuf = last_part + n;
    int32_t* last_g = (int32_t*)(qbuf + n);
    uint8_t* cont = (uint8_t*)(last_g + n);
    if (hipMemsetAsync(out, 0, sizeof(float) * (size_t)J * (size_t)umax, st) != hipSuccess ||
        hipMemsetAsync(last_g, 0xFF, sizeof(int32_t) * (size_t)n, st) != hipSuccess ||
        hipMemsetAsync(cont, 0, (size_t)n, st) != hipSuccess)
        return fjsp_internal_fail("fjsp_a2c_run_sums: memset failed");
    hipLaunchKernelGGL(k_run_chunks, dim3((unsigned)nch, (unsigned)J), dim3(RS_T), 0, st, vals, rowmap, scale, perm, gsorted, S,
                       umax, nch, out, first_part, cont, last_part, last_g);
    if (int rc = launch_error()) return rc;
    if (nch > 1) {
        hipLaunchKernelGGL(k_run_carry, dim3((unsigned)J), dim3(RS_T), 0, st, nch, umax, first_part, cont, last_part, last_g,
                           qbuf, out);
        if (int rc = launch_error()) return rc;
    }
    return 0;
}
