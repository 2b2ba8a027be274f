// fjsp_group.hip — the A2C update's grouping of repeated inputs on the GPU (a2c_vec.RowGroups):
// per row of grouping keys (8 actor rows + the critic's, fjsp_a2c_group_keys) the distinct keys,
// each sample's group, the samples sorted by group (stable: equal keys keep sample order) and each
// group's first sample and run end.  The reference runs every network once per sample
// (a2c.py:647-703 _update over the batch); the grouped update runs it once per distinct input and
// sums the samples' gradients by runs of this order, so the order must be deterministic.
//
// One flat radix sort of all rows (the row id in key bits 59..62 above 59 bits of the hash: rows
// stay contiguous), 32-bit sample positions as the payload (the grouping needs no more), then one
// inclusive scan of the run starts, and one pass that scatters each sorted position's sample,
// group and run start.  Replaces torch.sort (64-bit payload), a blocked prefix sum, a binary
// search per group and three gathers / scatters over [R][S].
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
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
    if (j == 0 || G[i] != G[i - 1]) {
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
    const int64_t r = i / S;
    rep[i] = first[r * umax + inv[i]];
}

// Run sums: out[j][g] = sum over the sorted positions of group g of row a = rowmap[j] of
// vals[j][perm[a][pos]] (* scale[j], in f32, as the gradient is scaled before the sum), summed in
// f64 in sorted order, stored as f32.  The backward of a per-group gather (each group's samples'
// gradients summed: a2c_vec._GatherRuns, _ActorHead): deterministic, one pass.  Each workgroup
// takes RS_CH sorted positions of one row: per thread 4 positions reduced by runs (a run wholly
// inside them is final), then each run start walks the following threads' head partials; a run
// that crosses the chunk's ends leaves its partial sums to k_run_carry, which adds them chunk by
// chunk from the chunk where the run starts.
constexpr int RS_CH = 1024, RS_T = 256;
__global__ void __launch_bounds__(RS_T) k_run_chunks(const float* __restrict__ vals, const int32_t* __restrict__ rowmap,
                                                   const float* __restrict__ scale, const int64_t* __restrict__ perm,
                                                   const int32_t* __restrict__ gsorted, int64_t S, int64_t umax,
                                                   int64_t nch, float* __restrict__ out, double* __restrict__ first_part,
                                                   uint8_t* __restrict__ whole, double* __restrict__ last_part,
                                                   int32_t* __restrict__ last_g) {
    __shared__ int32_t s_hg[RS_T], s_tg[RS_T];
    __shared__ double s_hs[RS_T], s_ts[RS_T];
    __shared__ uint8_t s_single[RS_T];
    const int64_t c = blockIdx.x;
    const int j = (int)blockIdx.y, t = (int)threadIdx.x;
    const int64_t a = rowmap[j];
    const float sc = scale ? scale[j] : 1.0f;
    const int64_t pos0 = c * RS_CH;
    const int32_t* gs = gsorted + a * S;
    const int64_t* pm = perm + a * S;
    const float* vr = vals + (int64_t)j * S;
    int32_t g[4];
    double v[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int64_t p = pos0 + 4 * t + i;
        g[i] = p < S ? gs[p] : -1;
        v[i] = p < S ? (double)(vr[pm[p]] * sc) : 0.0;
    }
    // runs of this thread's 4 positions: interior runs are final, head and tail go to LDS
    int32_t hg = g[0], tg = g[0];
    double hs = v[0], ts = v[0];
    bool single = true;
#pragma unroll
    for (int i = 1; i < 4; i++) {
        if (g[i] == tg) {
            ts += v[i];
        } else {
            if (single) {
                hs = ts;
                single = false;
            } else if (tg >= 0) {
                out[(int64_t)j * umax + tg] = (float)ts;   // an interior run: all of its positions are here
            }
            tg = g[i];
            ts = v[i];
        }
    }
    if (single) hs = ts;
    s_hg[t] = hg;
    s_hs[t] = hs;
    s_tg[t] = tg;
    s_ts[t] = ts;
    s_single[t] = single ? 1 : 0;
    __syncthreads();
    const int32_t prev_g = pos0 > 0 ? gs[pos0 - 1] : -2;
    const int32_t next_g = pos0 + RS_CH < S ? gs[pos0 + RS_CH] : -2;
    // a run starting at (thread t0's head or tail) with group gg and partial s: walk forward
    auto finish = [&](int t0, int32_t gg, double s, bool at_chunk_start) {
        int u = t0;
        bool cont = true;
        while (cont && u + 1 < RS_T && s_hg[u + 1] == gg) {
            u++;
            s += s_hs[u];
            cont = s_single[u] != 0;
        }
        const bool to_end = cont && u + 1 == RS_T;
        const bool from_prev = at_chunk_start && prev_g == gg;
        const bool into_next = to_end && next_g == gg;
        const int64_t k = (int64_t)j * nch + c;
        if (from_prev) {
            first_part[k] = s;
            whole[k] = into_next ? 1 : 0;
        } else if (into_next) {
            last_part[k] = s;
            last_g[k] = gg;
        } else {
            out[(int64_t)j * umax + gg] = (float)s;
        }
    };
    if (hg >= 0 && (t == 0 || hg != s_tg[t - 1])) {   // the head run starts here
        if (single) finish(t, hg, hs, t == 0);
        else {
            const bool from_prev = t == 0 && prev_g == hg;
            const int64_t k = (int64_t)j * nch + c;
            if (from_prev) {
                first_part[k] = hs;
                whole[k] = 0;
            } else {
                out[(int64_t)j * umax + hg] = (float)hs;   // ends inside this thread
            }
        }
    }
    if (!single && tg >= 0) finish(t, tg, ts, false);   // the tail run starts inside this thread
}

// runs that cross chunk ends: from the chunk where one starts, its partial + the first partials
// of the following chunks while they lie wholly inside the run
__global__ void __launch_bounds__(256) k_run_carry(int J, int64_t nch, int64_t umax, const double* __restrict__ first_part,
                                                   const uint8_t* __restrict__ whole, const double* __restrict__ last_part,
                                                   const int32_t* __restrict__ last_g, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)J * nch) return;
    const int32_t gg = last_g[i];
    if (gg < 0) return;
    const int64_t j = i / nch;
    int64_t c = i - j * nch;
    double s = last_part[i];
    while (++c < nch) {
        const int64_t k = j * nch + c;
        s += first_part[k];
        if (!whole[k]) break;
    }
    out[j * umax + gg] = (float)s;
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
    size_t a = 0, b = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, a, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                           (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)count, 0, 63) != hipSuccess ||
        hipcub::DeviceScan::InclusiveSum(nullptr, b, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)count) !=
            hipSuccess)
        return fjsp_internal_fail("fjsp_a2c_group_temp_bytes: hipcub size query failed");
    *bytes = (uint64_t)(a > b ? a : b);
    return 0;
}

extern "C" int fjsp_a2c_group_sort(const uint64_t* keys, int32_t R, int64_t S, void* temp, uint64_t temp_bytes,
                                   uint64_t* flat, uint64_t* sorted, uint32_t* pos, uint32_t* spos, uint32_t* runs,
                                   uint32_t* scan, int64_t* counts, void* stream) {
    const int64_t RS = (int64_t)R * S;
    if (R <= 0 || R > 16 || S <= 0 || RS >= (1ll << 31))
        return fjsp_internal_fail("fjsp_a2c_group_sort: need 0 < R <= 16, S > 0, R * S < 2^31");
    if (!keys || !temp || !flat || !sorted || !pos || !spos || !runs || !scan || !counts)
        return fjsp_internal_fail("fjsp_a2c_group_sort: null buffer");
    uint64_t need = 0;
    if (int rc = fjsp_a2c_group_temp_bytes(RS, &need)) return rc;
    if (temp_bytes < need) return fjsp_internal_fail("fjsp_a2c_group_sort: temp buffer too small");
    const hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_group_flat, dim3(blocks(RS)), dim3(256), 0, st, keys, S, RS, flat, pos);
    if (int rc = launch_error()) return rc;
    size_t tb = (size_t)temp_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(temp, tb, flat, sorted, pos, spos, (int)RS, 0, 63, st) != hipSuccess)
        return fjsp_internal_fail("fjsp_a2c_group_sort: radix sort failed");
    hipLaunchKernelGGL(k_group_new, dim3(blocks(RS)), dim3(256), 0, st, sorted, S, RS, runs);
    if (int rc = launch_error()) return rc;
    tb = (size_t)temp_bytes;
    if (hipcub::DeviceScan::InclusiveSum(temp, tb, runs, scan, (int)RS, st) != hipSuccess)
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
    *bytes = (uint64_t)n * (8 + 1 + 8 + 4) + 64;
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
    char* p = (char*)temp;
    double* first_part = (double*)p;
    double* last_part = first_part + n;
    int32_t* last_g = (int32_t*)(last_part + n);
    uint8_t* whole = (uint8_t*)(last_g + n);
    if (hipMemsetAsync(out, 0, sizeof(float) * (size_t)J * (size_t)umax, st) != hipSuccess ||
        hipMemsetAsync(last_g, 0xFF, sizeof(int32_t) * (size_t)n, st) != hipSuccess)
        return fjsp_internal_fail("fjsp_a2c_run_sums: memset failed");
    hipLaunchKernelGGL(k_run_chunks, dim3((unsigned)nch, (unsigned)J), dim3(RS_T), 0, st, vals, rowmap, scale, perm, gsorted, S,
                       umax, nch, out, first_part, whole, last_part, last_g);
    if (int rc = launch_error()) return rc;
    hipLaunchKernelGGL(k_run_carry, dim3(blocks(n)), dim3(256), 0, st, J, nch, umax, first_part, whole, last_part, last_g, out);
    return launch_error();
}
