// rl_sort.h -- stable LSD radix sort of (slot, request-index) pairs, gfx950.
//
// Groups a batch's requests by state-table slot while keeping arrival order
// inside each group (stable), which is what lets the replay kernels apply the
// reference's per-key atomic scripts in `seq` order.  One-sweep design:
//   * the digit histograms of every pass come from the probe kernel (fused),
//   * each pass is ONE kernel: a 4096-element tile is ranked wave-locally
//     (8 ballots per element match the 8-bit digit across the 64 lanes, LDS
//     digit counters per wave, 2 barriers per tile), the tile's per-digit
//     offsets come from a decoupled look-back over earlier tiles, then keys and
//     values are staged in LDS in output order (digit-major) and written by
//     consecutive threads, so each digit's run leaves as full-line stores.
// Look-back words pack {2-bit flag, 30-bit count} in one 32-bit word, stored
// and loaded with relaxed agent-scope atomics (global_store/load sc1): the
// word is its own granule, so no fence is needed (MI355X_MICROARCH.md,
// "R2's granule needs no ordering").  Tile ids are taken from an atomic
// counter, so a tile only ever waits on tiles that have already started.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_semantics.h"

namespace rl {

constexpr int SORT_BLOCK = 256;
#ifndef RL_SORT_ITEMS
#define RL_SORT_ITEMS 16
#endif
constexpr int SORT_ITEMS = RL_SORT_ITEMS;   // keys per thread; a tile is SORT_BLOCK x SORT_ITEMS
constexpr int SORT_TILE = SORT_BLOCK * SORT_ITEMS;
constexpr int SORT_WAVES = SORT_BLOCK / 64;
constexpr int RADIX = 256;
constexpr uint32_t LB_AGG = 1u << 30;
constexpr uint32_t LB_INC = 2u << 30;
constexpr uint32_t LB_VAL = (1u << 30) - 1;
constexpr uint32_t LB_SPIN_LIMIT = 1u << 24;

__device__ inline uint32_t ld_agent(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void st_agent(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ inline uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t t = __shfl_up(v, off, 64);
        if (lane >= off) v += t;
    }
    return v;
}

// exclusive scan of one value per thread across a 256-thread block
__device__ inline uint32_t block_excl_scan_256(uint32_t v, uint32_t* s_tmp /*[4]*/) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc = wave_incl_scan(v, lane);
    if (lane == 63) s_tmp[wave] = inc;
    __syncthreads();
    uint32_t pre = 0;
    for (int w = 0; w < wave; w++) pre += s_tmp[w];
    return pre + inc - v;
}

// One stable pass over the 8-bit digit at `shift`.  Blocks take tiles from
// an atomic counter until every tile is done (a grid smaller than the tile
// count is persistent; a tile only ever waits on tiles already taken).
// skip (nullable): a device flag that turns the pass into a no-op.
// mdev (nullable): the batch size in device memory, at most m (the grid is
// sized for m; tiles past the device size exit at once).
// rin / rout (FIRST only, nullable): records of `rw` 16-byte words in input
// order, moved along with the keys -- rout[pos] = rin[idx] -- and the value written is the
// output position itself, so later passes carry each element's position in
// this pass's output (where its record now is).
// plan (nullable, the MSD pass of the grouping sort): the block of tile 0
// writes plan[0] = 1 when no digit of this pass holds more than plan_cap
// elements (every bucket then fits k_sort_local) and plan[1] = 1 otherwise,
// and plan[0] to plan_host (nullable) too.
template <bool FIRST>
__global__ __launch_bounds__(SORT_BLOCK) void k_sort_pass(
    const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin, uint32_t* __restrict__ kout,
    uint32_t* __restrict__ vout, uint32_t m, int shift, const uint32_t* __restrict__ ghist,
    uint32_t* status, uint32_t* tile_ctr, uint32_t* eflags, const uint32_t* skip = nullptr,
    uint32_t* plan = nullptr, uint32_t plan_cap = 0, uint32_t* plan_host = nullptr, const uint32_t* mdev = nullptr,
    const uint4* __restrict__ rin = nullptr, uint4* __restrict__ rout = nullptr, int rw = 1) {
    if (skip && *skip) return;
    if (mdev) m = min(m, *mdev);   // a batch sized on the device (the routed path): m is its bound
    __shared__ uint32_t s_wcnt[SORT_WAVES][RADIX];
    __shared__ uint32_t s_goff[RADIX];
    __shared__ uint32_t s_tstart[RADIX];
    __shared__ uint32_t s_key[SORT_TILE], s_src[SORT_TILE];
    __shared__ uint32_t s_tmp[SORT_WAVES];
    __shared__ uint32_t s_tile;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t ntiles = (m + SORT_TILE - 1) / SORT_TILE;
    for (;;) {
    if (tid == 0) s_tile = atomicAdd(tile_ctr, 1u);
#pragma unroll
    for (int w = 0; w < SORT_WAVES; w++) s_wcnt[w][tid] = 0;
    __syncthreads();
    const uint32_t tile = s_tile;
    if (tile >= ntiles) return;   // block-uniform
    const uint32_t base = tile * SORT_TILE + wave * (64 * SORT_ITEMS);

    uint32_t key[SORT_ITEMS], val[SORT_ITEMS], rank[SORT_ITEMS];
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; j++) {
        uint32_t idx = base + j * 64 + lane;
        bool ok = idx < m;
        key[j] = ok ? kin[idx] : 0xffffffffu;
        val[j] = FIRST ? idx : (ok ? vin[idx] : 0u);
    }
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; j++) {
        uint32_t idx = base + j * 64 + lane;
        bool ok = idx < m;
        uint32_t d = (key[j] >> shift) & (RADIX - 1);
        uint64_t peers = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            uint32_t bit = (d >> b) & 1u;
            uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        if (ok) {
            uint32_t below = __popcll(peers & lt);
            uint32_t cur = s_wcnt[wave][d];
            rank[j] = cur + below;
            if (below == 0) s_wcnt[wave][d] = cur + (uint32_t)__popcll(peers);
        }
    }
    __syncthreads();
    // per digit: exclusive prefix over the waves of this tile, tile total
    uint32_t tot = 0;
#pragma unroll
    for (int w = 0; w < SORT_WAVES; w++) {
        uint32_t c = s_wcnt[w][tid];
        s_wcnt[w][tid] = tot;
        tot += c;
    }
    // decoupled look-back for digit `tid`
    uint32_t* st = status + (size_t)tile * RADIX;
    uint32_t excl = 0;
    if (tile == 0) {
        st_agent(&st[tid], LB_INC | tot);
    } else {
        st_agent(&st[tid], LB_AGG | tot);
        int64_t pt = (int64_t)tile - 1;
        uint32_t spins = 0;
        while (pt >= 0) {
            uint32_t s = ld_agent(&status[(size_t)pt * RADIX + tid]);
            uint32_t flag = s & ~LB_VAL;
            if (flag == 0) {
                if (++spins > LB_SPIN_LIMIT) { atomicOr(eflags, EF_LOOKBACK); break; }
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            excl += s & LB_VAL;
            if (flag == LB_INC) break;
            pt--;
        }
        st_agent(&st[tid], LB_INC | (excl + tot));
    }
    const uint32_t gh = ghist[tid];
    if (plan && tile == 0) {
        // the largest bucket of this digit (block max of the histogram)
        uint32_t mx = gh;
        for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, off));
        __syncthreads();
        if (lane == 0) s_tmp[wave] = mx;
        __syncthreads();
        if (tid == 0) {
            for (int w = 1; w < SORT_WAVES; w++) mx = max(mx, s_tmp[w]);
            plan[0] = mx <= plan_cap ? 1u : 0u;
            plan[1] = mx <= plan_cap ? 0u : 1u;
            if (plan_host) plan_host[0] = plan[0];   // mapped host word: the engine's next prediction
        }
        __syncthreads();
    }
    uint32_t g = block_excl_scan_256(gh, s_tmp);
    s_goff[tid] = g + excl;
    __syncthreads();   // s_tmp is reused by the next scan
    s_tstart[tid] = block_excl_scan_256(tot, s_tmp);   // the digit's first position in the tile
    __syncthreads();
    // the tile in output order in LDS, then written out with consecutive
    // threads on consecutive positions of each digit's run: every run of a
    // bucket is one stretch of full lines instead of one scattered element
    // per lane (and records are read from the tile's L2-resident input range)
#pragma unroll
    for (int j = 0; j < SORT_ITEMS; j++) {
        uint32_t idx = base + j * 64 + lane;
        if (idx < m) {
            uint32_t d = (key[j] >> shift) & (RADIX - 1);
            uint32_t li = s_tstart[d] + s_wcnt[wave][d] + rank[j];
            s_key[li] = key[j];
            s_src[li] = FIRST ? idx : val[j];
        }
    }
    __syncthreads();
    const uint32_t t0 = tile * SORT_TILE;
    const uint32_t nt = m - t0 < (uint32_t)SORT_TILE ? m - t0 : (uint32_t)SORT_TILE;
    for (uint32_t t = tid; t < nt; t += SORT_BLOCK) {
        const uint32_t k = s_key[t];
        const uint32_t d = (k >> shift) & (RADIX - 1);
        const uint32_t pos = s_goff[d] + (t - s_tstart[d]);
        const uint32_t src = s_src[t];
        kout[pos] = k;
        if (FIRST && rout) {
            vout[pos] = pos;
            for (int w = 0; w < rw; w++) rout[(size_t)pos * rw + w] = rin[(size_t)src * rw + w];
        } else {
            vout[pos] = src;   // FIRST: the input index
        }
    }
    __syncthreads();   // s_tile, s_wcnt, s_goff, s_tstart, s_key, s_src, s_tmp are rewritten by the next tile
    }
}

}  // namespace rl
